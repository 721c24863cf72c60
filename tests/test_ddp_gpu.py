"""Data-parallel equivalence on the one-GPU box: two ranks share cuda:0 and
exchange gradients over gloo (RCCL refuses two ranks on one device); each trains one image of a
batch of two through the product path -- Pix2PixModel.optimize_parameters with the D all-reduce
before optimizer_D.step and the G buckets all-reduced during backward_G (dsgan_hip.dist) -- and
the result must equal ONE process training the whole batch (the reference's nn.DataParallel,
DSGAN/models/networks.py:74-77, computes every loss on the gathered global batch):

  * the averaged flat G and D gradients equal the single-process gradients (TV is a batch SUM,
    DSGAN/models/pix2pix_model.py:189-191: the per-rank TV coefficient carries the world size);
  * the post-step D (and G) parameters are identical on both ranks and equal the single run's --
    the G step reads the updated D, so an exchange that landed after optimizer_D.step would show.
fp32 mode, pool_size 0, "fanin" weight recipe.  Gradients are compared PER TENSOR with the bars of
test_model_gpu.py::test_full_step_fp32_vs_oracle (2e-3 of the tensor's norm, or 8x its measured
fp32 conditioning): the batch sum of every weight-grad is split differently across the two runs,
so they differ at fp32 reassociation level, but a bucket that fired before one of its tensors'
grads landed would leave that tensor at half its value.

``test_one_rank_rccl_exchange_is_bitwise_neutral`` runs the RCCL ("nccl") branch itself on the
one GPU: a 1-rank group with the D all-reduce (ReduceOp.AVG) and the G buckets (async, started
from the autograd thread during backward_G) forced on must give bitwise the flat gradients and
post-step parameters of the same step without any exchange -- a bucket launched on RCCL's stream
before its weight-grad kernels finished, or an optimizer step that did not wait for it, changes
bits.  The same holds with the step replayed from its HIP graphs, the exchanges captured into the
second graph (the multi-GPU bench and train loop run that way).
"""
import os
import random

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model(precision="fp32", batch=2):
    import dsgan_hip
    from oracle import dsgan_cpu as O
    from oracle.recipe import make_params
    from options.train_options import default_train_opt
    from models import create_model
    dsgan_hip.require_gpu()
    random.seed(20)
    torch.manual_seed(20)
    m = create_model(default_train_opt(gpu_ids=[0], pool_size=0, precision=precision, batchSize=batch))
    with torch.no_grad():
        for net, pr in ((m.netG, make_params(O.g_param_spec(), "fanin", 1000)),
                        (m.netD, make_params(O.d_param_spec(), "fanin", 5000)),
                        (m.vgg, make_params(O.vgg_param_spec(True), "vgg", 7000))):
            for k, v in net.state_dict().items():
                v.copy_(pr[k])
    return m


def _grads_and_params(m):
    torch.cuda.synchronize()
    return {"tG": {k: p.grad.detach().cpu().clone() for k, p in m.netG.named_parameters()},
            "tD": {k: p.grad.detach().cpu().clone() for k, p in m.netD.named_parameters()},
            "gG": torch.cat([p.grad.detach().flatten() for p in m.netG.parameters()]).cpu(),
            "gD": torch.cat([p.grad.detach().flatten() for p in m.netD.parameters()]).cpu(),
            "pG": torch.cat([p.detach().flatten() for p in m.netG.parameters()]).cpu(),
            "pD": torch.cat([p.detach().flatten() for p in m.netD.parameters()]).cpu(),
            "loss_G": float(m.loss_G), "loss_D": float(m.loss_D)}


def _worker(rank, world, port, out_dir, precision="fp32", size=64, per_rank=1):
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.recipe import synth_pair
    m = _model(precision, world * per_rank)
    assert m.g_buckets is not None and len(m.g_buckets.buckets) >= 3
    A, B = synth_pair(world * per_rank, size, seed=4)
    sl = slice(rank * per_rank, (rank + 1) * per_rank)
    m.set_input({"A": A[sl].cuda(), "B": B[sl].cuda(), "A_paths": ["a"] * per_rank, "B_paths": ["b"] * per_rank})
    m.optimize_parameters()
    res = _grads_and_params(m)
    torch.save(res, os.path.join(out_dir, "rank%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()


def _rel(a, b):
    return ((a.double() - b.double()).norm() / max(b.double().norm().item(), 1e-30)).item()


def _two_ranks(tmp_path, precision="fp32", size=64, per_rank=1):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = 33500 + random.randint(0, 2000)
    ps = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), precision, size, per_rank)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    return (torch.load(tmp_path / "rank0.pt", weights_only=True), torch.load(tmp_path / "rank1.pt", weights_only=True))


@pytest.mark.parametrize("prec", ["bf16", "fp32"])
def test_two_ranks_equal_one_process_256(tmp_path, prec):
    """the same equivalence in the bench's mode -- bf16 MFMA operands, the
    stacked batch-2N D pass (pix2pix_model.D_BATCH), the bf16 non-finite guard -- at 256^2 with two
    images per rank.  Both ranks must end bitwise equal.  Against one process training all four
    images the gradients agree only to bf16 level, not fp32 reassociation: the split-K plans of the
    D convs follow the batch (2N = 4 per rank, 8 in one process), so their fp32 sums reassociate and
    some 16-bit activations round one ulp (2^-8) apart (measured: D loss 1.2e-5, flat D grad 1.7e-2
    relative).  So the exchange is judged against a control: the averaged gradient must be far
    closer to the one-process gradient than rank 0's own shard gradient (one process on its two
    images, what a missing exchange would leave) is -- a lost, doubled or unscaled exchange fails."""
    from oracle.recipe import synth_pair
    from models import pix2pix_model as PM
    assert PM.D_BATCH
    r0, r1 = _two_ranks(tmp_path, prec, 256, 2)
    A, B = synth_pair(4, 256, seed=4)

    def one_process(sl, n):
        m = _model(prec, n)
        assert m.d_batch
        m.set_input({"A": A[sl].cuda(), "B": B[sl].cuda(), "A_paths": ["a"] * n, "B_paths": ["b"] * n})
        m.optimize_parameters()
        return _grads_and_params(m)
    one = one_process(slice(0, 4), 4)
    local = one_process(slice(0, 2), 2)     # rank 0's shard alone: the no-exchange control
    for k in ("gG", "gD", "pG", "pD"):
        assert torch.equal(r0[k], r1[k]), k
    assert abs(0.5 * (r0["loss_D"] + r1["loss_D"]) - one["loss_D"]) <= 1e-4 * abs(one["loss_D"])
    assert torch.isfinite(r0["gG"]).all() and torch.isfinite(r0["gD"]).all()
    for k in ("gD", "gG"):
        e, c = _rel(r0[k], one[k]), _rel(local[k], one[k])
        print("%s DDP %s: rel vs one process %.3g, control (rank 0 shard alone) %.3g" % (prec, k, e, c))
        assert e < 0.1 and e < 0.25 * c, (k, e, c)


def test_two_ranks_equal_one_process(tmp_path):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = 33500 + random.randint(0, 2000)
    ps = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)

    from oracle.recipe import synth_pair
    m = _model()
    A, B = synth_pair(2, 64, seed=4)
    m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": ["a"] * 2, "B_paths": ["b"] * 2})
    m.optimize_parameters()
    one = _grads_and_params(m)

    # identical exchanges on both ranks: bitwise equal gradients and parameters
    for k in ("gG", "gD", "pG", "pD"):
        assert torch.equal(r0[k], r1[k]), k
    # the mean of the per-rank losses is the global-batch loss
    assert abs(0.5 * (r0["loss_D"] + r1["loss_D"]) - one["loss_D"]) <= 1e-5 * abs(one["loss_D"])
    # averaged gradients == one process on the whole batch, per tensor (fp32 reassociation level)
    assert _rel(r0["gD"], one["gD"]) < 2e-5, _rel(r0["gD"], one["gD"])
    assert _rel(r0["gG"], one["gG"]) < 1e-3, _rel(r0["gG"], one["gG"])
    from oracle import dsgan_cpu as O
    from oracle.recipe import make_params
    from test_model_gpu import fp32_sensitivity
    sens, _ = fp32_sensitivity(make_params(O.g_param_spec(), "fanin", 1000), make_params(O.d_param_spec(), "fanin", 5000),
                               A, B)
    for tag in ("G", "D"):
        for k, g1 in one["t" + tag].items():
            g2 = r0["t" + tag][k]
            err = (g2.double() - g1.double()).norm().item()
            bar = max(2e-3 * g1.double().norm().item(), 8 * sens[(tag, k)]) + 1e-6
            assert err <= bar, (tag, k, err, bar)
    # post-step parameters: the D step used the exchanged gradient (Adam's first step is
    # lr * sign(g): equal wherever |g| is above fp32 noise)
    big = one["gD"].abs() > 1e-6
    assert (r0["pD"][big] - one["pD"][big]).abs().max().item() < 1e-6
    bigG = one["gG"].abs() > 1e-5
    frac = ((r0["pG"][bigG] - one["pG"][bigG]).abs() > 1e-6).double().mean().item()
    assert frac < 1e-3, frac


def _nccl_worker(port, out_dir):
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    from oracle.recipe import synth_pair
    from dsgan_hip import dist as hdist
    res = {}
    for mode in ("plain", "exchange", "exchange_graph", "plain2"):
        m = _model("bf16")
        m.cuda_graph = mode == "exchange_graph"
        if mode.startswith("exchange"):
            m.exchange = True
            # small buckets: several async RCCL all-reduces start during backward_G
            m.g_buckets = hdist.GradBuckets(m.flatG.grad, m.flatG.layout, bucket_mb=4)
            assert len(m.g_buckets.buckets) >= 8
        for it in range(4):   # graph mode: eager warm-up, capture + replay, two replays
            A, B = synth_pair(2, 64, seed=40 + it)
            m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": ["a"] * 2, "B_paths": ["b"] * 2})
            m.optimize_parameters()
            if mode.startswith("exchange"):
                assert m.g_buckets.pending is None
        if mode == "exchange_graph":   # the exchanges were captured: the step replayed from its graphs
            assert m.cuda_graph and len(m._graphs) == 1
        torch.cuda.synchronize()
        res[mode] = {"gG": m.flatG.grad.detach().cpu().clone(), "gD": m.flatD.grad.detach().cpu().clone(),
                     "pG": m.flatG.data.detach().cpu().clone(), "pD": m.flatD.data.detach().cpu().clone()}
    torch.save(res, os.path.join(out_dir, "nccl.pt"))
    dist.destroy_process_group()


def test_one_rank_rccl_exchange_is_bitwise_neutral(tmp_path):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = 36000 + random.randint(0, 2000)
    p = ctx.Process(target=_nccl_worker, args=(port, str(tmp_path)))
    p.start()
    p.join(timeout=240)
    assert p.exitcode == 0, p.exitcode
    r = torch.load(tmp_path / "nccl.pt", weights_only=True)
    for k in ("gG", "gD", "pG", "pD"):
        assert torch.equal(r["plain"][k], r["plain2"][k]), ("step not deterministic", k)
        assert torch.equal(r["plain"][k], r["exchange"][k]), k
        assert torch.equal(r["plain"][k], r["exchange_graph"][k]), ("graph replay with captured RCCL exchanges", k)
