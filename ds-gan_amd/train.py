"""Training loop with the reference's semantics (DSGAN/train.py:47-185) on the MI355X build.

Same order of work per iteration: set_input -> optimize_parameters -> get_img_tir / get_img_gen
/ get_img_label -> SSIM + PSNR of image 0 (device-side, util/metrics.py) -> every
``output_freq`` iterations the loss line and ``result.csv``; per epoch ``each_epoch.csv``,
``save_networks(epoch)`` and ``update_learning_rate()``.  The seed is 20 (:48).  Image dumps
(cv2) and the visualizer/HTML are out of scope (SURVEY.md §8 out-of-scope list).

    python ds-gan_amd/train.py --dataroot DATA --out RESULTS [reference TrainOptions flags...]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        ds-gan_amd/train.py --dataroot DATA --out RESULTS --batchSize 128 [...]

Multi-GPU replaces the reference's single-process nn.DataParallel (DSGAN/models/networks.py:
74-77) with one process per GPU: under torchrun (WORLD_SIZE > 1) every rank joins the RCCL
process group and drives cuda:LOCAL_RANK; ``--batchSize`` stays the GLOBAL batch, of which each
rank trains its DataParallel-style chunk (data/__init__.py); the printed / CSV losses are the
global-batch values (an all-reduce of the per-rank means at logging time); only rank 0 writes
checkpoints and CSV files, behind a barrier.
"""
import argparse
import csv
import math
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def setup_seed(seed):
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)
    random.seed(seed)


def init_distributed():
    """(rank, world, local_rank); joins the RCCL process group when launched by torchrun."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1:
        return 0, 1, None
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return dist.get_rank(), world, local


def global_losses(losses, n_local, n_global):
    """Per-rank batch means -> the global-batch means the reference logs (weights n_rank/n)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return losses
    dev = torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([v * n_local / n_global for v in losses.values()], dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return type(losses)(zip(losses.keys(), t.tolist()))


class NonfiniteMonitor:
    """Reports the optimizer steps that the bf16 non-finite guard or the fp16 loss scaler skipped
    (``Pix2PixModel.nonfinite_report``), so that a network that stops learning shows in the log.

    ``poll()`` runs at logging time.  It returns the text appended to the loss line: empty while no
    step was ever skipped, else the running counts, e.g. ``skipped G 3/400 D 0/400``.  When every
    step of one network since the previous poll was skipped, and there were at least
    ``abort_window`` of them, the network is no longer training: ``poll()`` raises RuntimeError."""

    def __init__(self, model, abort_window=50):
        self.model = model
        self.abort_window = int(abort_window)
        self.last = {}

    def poll(self):
        rep = self.model.nonfinite_report() if hasattr(self.model, "nonfinite_report") else {}
        dead = []
        for net, (skipped, calls) in rep.items():
            s0, c0 = self.last.get(net, (0, 0))
            if calls - c0 >= self.abort_window and skipped - s0 == calls - c0:
                dead.append("%s skipped all of its last %d optimizer steps" % (net, calls - c0))
        self.last = dict(rep)
        if dead:
            raise RuntimeError("non-finite gradients: " + "; ".join(dead) + " (--nonfinite_guard)")
        if not any(s for s, _ in rep.values()):
            return ""
        return "skipped " + " ".join("%s %d/%d" % (k, s, c) for k, (s, c) in rep.items()) + " "


def main(argv=None, output_freq=100):
    from data import CreateDataLoader
    from models import create_model
    from options.train_options import TrainOptions
    from util.metrics import TrainMetrics

    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--out", default=os.path.abspath(os.path.join("..", "resext50_vision1")))
    ap.add_argument("--dataroot", default="/root/dataset/256x256")
    known, rest = ap.parse_known_args(argv)
    rank, world, local = init_distributed()
    setup_seed(20)
    out = known.out
    if rank == 0:
        os.makedirs(out, exist_ok=True)
    opt = TrainOptions().parse(known.dataroot, out, rest)   # parse() sets checkpoints_dir = out/checkpoints
    if world > 1:
        opt.gpu_ids = [local]   # one process per GPU: this rank's device
    dataset = CreateDataLoader(opt, "train").load_data()
    print("#training images = %d" % len(dataset))
    model = create_model(opt)
    model.setup(opt)
    metrics = TrainMetrics(model.device)
    guard = NonfiniteMonitor(model)
    history = []
    for epoch in range(opt.epoch_count, opt.niter + opt.niter_decay + 1):
        metrics.reset()
        epoch_start_time = time.time()
        epoch_iter, i = 0, -1
        for i, data in enumerate(dataset):
            iter_start_time = time.time()
            epoch_iter += opt.batchSize
            model.set_input(data)
            model.optimize_parameters()
            model.get_img_tir(data)
            with torch.no_grad():   # the reference runs this forward with autograd on; output is identical
                model.get_img_gen(data)
            model.get_img_label(data)
            # the reference scores image 0 of the GLOBAL batch only (DSGAN/train.py:110-124); under
            # DDP that image is rank 0's fake_B[0] (Tensor.chunk order), so rank 0's accumulators
            # are exactly the reference's metric and no cross-rank reduction is needed
            metrics.update(model.fake_B[0], model.real_B[0])
            if (i + 1) % output_freq == 0:
                losses = global_losses(model.get_current_losses(), int(model.real_A.shape[0]),
                                       int(data.get("global_batch", model.real_A.shape[0])))
                skipped = guard.poll()   # every rank: a network that stopped learning ends every rank
                if rank != 0:
                    continue
                ssim_avg, psnr_avg = metrics.averages()
                t = (time.time() - iter_start_time) / opt.batchSize
                message = "(epoch: %d, iters: %d, time: %.3f) " % (epoch, epoch_iter, t)
                message += "".join("%s: %.3f " % (k, v) for k, v in losses.items())
                print(message + "ssim: %.4f psnr: %.3f" % (ssim_avg, psnr_avg) + (" " + skipped if skipped else ""))
                with open(os.path.join(out, "result.csv"), "a", newline="") as f:
                    csv.writer(f).writerow([epoch, "".join("%s: %.3f " % (k, v) for k, v in losses.items()) + "  ",
                                            ssim_avg, psnr_avg])
        ssim_avg, psnr_avg = metrics.averages()
        history.append((epoch, ssim_avg, psnr_avg))
        if rank == 0:
            with open(os.path.join(out, "each_epoch.csv"), "a", newline="") as f:
                csv.writer(f).writerow([epoch, "train", ssim_avg, psnr_avg])
            print("saving the model at the end of epoch %d, iters %d" % (epoch, i + 1))
            model.save_networks(epoch)
            print("End of epoch %d / %d \t Time Taken: %d sec" % (epoch, opt.niter + opt.niter_decay,
                                                                    time.time() - epoch_start_time))
        if world > 1:
            dist.barrier()
        model.update_learning_rate()
    return model, history


if __name__ == "__main__":
    main()
