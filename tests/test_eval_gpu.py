"""Evaluation / inference path: the HIP ms_ssim (DSGAN/MS_SSIM.py:153-225)
against the golden vector and the CPU oracle, and the ``--model test`` generator-only model
loading a checkpoint written by the training model.

Tolerance: ms_ssim is a product of five fp32 plane means; |HIP - oracle| <= 2e-5 absolute
(the oracle itself matches the reference to 1e-6, tests/test_oracle.py)."""
import os
import tempfile

import pytest
import torch

from oracle import dsgan_cpu as O
from oracle.recipe import make_params, synth_pair

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _f3_pair():
    # the exact generator sequence of tests/test_oracle.py::test_ssim_msssim
    g = torch.Generator().manual_seed(3)
    X = torch.rand(2, 3, 64, 64, generator=g)
    _ = (X + 0.2 * torch.randn(2, 3, 64, 64, generator=g)).clamp(0, 1)
    X2 = torch.rand(1, 3, 176, 176, generator=g)
    Y2 = (X2 + 0.2 * torch.randn(1, 3, 176, 176, generator=g)).clamp(0, 1)
    return X2, Y2


def test_ms_ssim_golden(golden):
    import MS_SSIM as M
    X2, Y2 = _f3_pair()
    v = M.ms_ssim(X2.to(DEV), Y2.to(DEV), data_range=1.0).item()
    assert abs(v - float(golden["F3_msssim"])) < 2e-5, (v, float(golden["F3_msssim"]))


@pytest.mark.parametrize("shape", [(2, 3, 176, 176), (2, 3, 181, 199), (1, 1, 256, 256)])
def test_ms_ssim_vs_oracle(shape):
    import MS_SSIM as M
    g = torch.Generator().manual_seed(shape[2] + shape[3])
    X = torch.rand(shape, generator=g)
    Y = (X + 0.15 * torch.randn(shape, generator=g)).clamp(0, 1)
    got = M.ms_ssim(X.to(DEV), Y.to(DEV), data_range=1.0, size_average=False).cpu()
    for n in range(shape[0]):
        ref = float(O.ms_ssim(X[n:n + 1], Y[n:n + 1]))
        assert abs(got[n].item() - ref) < 2e-5, (n, got[n].item(), ref)
    mean = M.ms_ssim(X.to(DEV), Y.to(DEV), data_range=1.0).item()
    assert abs(mean - float(O.ms_ssim(X, Y))) < 2e-5
    # the (t+1)/2 affine form the quality metric uses on generator outputs in [-1, 1]
    from dsgan_hip import functional as HF
    v = HF.ms_ssim_affine((2 * X - 1).to(DEV), (2 * Y - 1).to(DEV), 0.5, 0.5).item()
    assert abs(v - mean) < 2e-5


def test_ms_ssim_rejects_small_images():
    import MS_SSIM as M
    x = torch.rand(1, 3, 150, 150, device=DEV)
    with pytest.raises(AssertionError):
        M.ms_ssim(x, x, data_range=1.0)


def test_test_model_loads_training_checkpoint():
    """save_networks of the training model -> ``--model test`` -> identical generator output."""
    import dsgan_hip
    from models import create_model
    from options.test_options import default_test_opt
    from options.train_options import default_train_opt
    dsgan_hip.require_gpu()
    with tempfile.TemporaryDirectory() as d:
        opt = default_train_opt(gpu_ids=[0], pool_size=0, precision="fp32", checkpoints_dir=d)
        m = create_model(opt)
        gp = make_params(O.g_param_spec(), "fanin", 1000)
        with torch.no_grad():
            for k, v in m.netG.state_dict().items():
                v.copy_(gp[k])
        A, _ = synth_pair(2, 64, seed=11)
        with torch.no_grad():
            ref = m.netG(A.to(DEV)).cpu()
        m.save_networks("7")
        # a reference-style DataParallel checkpoint name/prefix loads too
        sd = torch.load(os.path.join(d, opt.name, "7_useSE_net_G.pth"), weights_only=True)
        torch.save({"module." + k: v for k, v in sd.items()}, os.path.join(d, opt.name, "8_net_G.pth"))
        for epoch in ("7", "8"):
            topt = default_test_opt(gpu_ids=[0], precision="fp32", checkpoints_dir=d, which_epoch=epoch,
                                    name=opt.name)
            t = create_model(topt)
            assert type(t).__name__ == "TestModel"
            t.setup(topt)
            t.set_input({"A": A, "A_paths": ["a", "b"]})
            t.test()
            assert torch.equal(t.fake_B.cpu(), ref), epoch


@pytest.mark.parametrize("gray", [False, True])
def test_data_loader_gpu_transforms_bit_exact(tmp_path, gray):
    """CreateDataLoader batches (uint8 upload + dsgan_u8_to_image) == the reference's torch CPU
    transforms: ToTensor (/255), crop, Normalize(0.5, 0.5), flip, RGB->gray (aligned_dataset.py:52-82)."""
    import random
    import numpy as np
    from PIL import Image
    from data import CreateDataLoader
    from options.train_options import default_train_opt
    rng = np.random.default_rng(1)
    d = tmp_path / "train_all"
    d.mkdir()
    for i in range(4):
        for side in ("a", "b"):
            Image.fromarray(rng.integers(0, 256, (40, 48, 3), dtype=np.uint8)).save(str(d / ("%s_%d.png" % (side, i))))
    opt = default_train_opt(gpu_ids=[0], dataroot=str(tmp_path), phase="train_all", loadSize_w=48, fineSize_w=32,
                            loadSize_h=40, fineSize_h=24, batchSize=2, nThreads=0, serial_batches=True,
                            input_nc=1 if gray else 3)
    loader = CreateDataLoader(opt, "train").load_data()
    random.seed(9)
    batches = list(loader)
    assert len(batches) == 2
    random.seed(9)
    for bi, data in enumerate(batches):
        for j in range(2):
            k = 2 * bi + j
            wo, ho = random.randint(0, 48 - 32 - 1), random.randint(0, 40 - 24 - 1)
            flip = random.random() < 0.5
            for side, key, g in (("a", "A", gray), ("b", "B", False)):
                img = np.asarray(Image.open(str(d / ("%s_%d.png" % (side, k)))).convert("RGB"))
                t = torch.from_numpy(img.copy()).permute(2, 0, 1).contiguous().float().div(255)
                t = t[:, ho:ho + 24, wo:wo + 32]
                m = torch.tensor([0.5, 0.5, 0.5])[:, None, None]
                t = t.sub(m).div(m)
                if flip:
                    t = t.index_select(2, torch.arange(31, -1, -1))
                if g:
                    t = (t[0] * 0.299 + t[1] * 0.587 + t[2] * 0.114).unsqueeze(0)
                got = data[key][j].cpu()
                assert got.shape == t.shape and torch.equal(got, t), (k, key)


def test_train_loop_metrics_vs_oracle(tmp_path):
    """ds-gan_amd/train.py end to end on a 4-pair 64x64 dataset (batch 2, one epoch): the
    device-side SSIM/PSNR of train.py:110-124 equal the oracle's skimage restatement on the same
    generator outputs (parity unpinned against skimage itself, which is absent here)."""
    import numpy as np
    from PIL import Image
    import train as T
    rng = np.random.default_rng(2)
    d = tmp_path / "data" / "train_all"
    d.mkdir(parents=True)
    for i in range(4):
        for side in ("a", "b"):
            Image.fromarray(rng.integers(0, 256, (64, 64, 3), dtype=np.uint8)).save(str(d / ("%s_%d.png" % (side, i))))
    model, hist = T.main(["--dataroot", str(tmp_path / "data"), "--out", str(tmp_path / "out"), "--gpu_ids", "0",
                          "--batchSize", "2", "--nThreads", "0", "--niter", "1", "--niter_decay", "0",
                          "--loadSize_w", "64", "--fineSize_w", "64", "--loadSize_h", "64", "--fineSize_h", "64",
                          "--pool_size", "0"], output_freq=1)
    assert len(hist) == 1
    # recompute the last iteration's metrics from the tensors the model holds
    from util.metrics import TrainMetrics
    m = TrainMetrics(model.device)
    m.update(model.fake_B[0], model.real_B[0])
    s, p = m.averages()
    lab, res = O.to_u8_hwc(model.real_B[0]), O.to_u8_hwc(model.fake_B[0])
    assert abs(s - O.sk_ssim(lab, res)) < 1e-5, (s, O.sk_ssim(lab, res))
    assert abs(p - O.cal_psnr(lab, res)) < 1e-4, (p, O.cal_psnr(lab, res))
    assert os.path.exists(tmp_path / "out" / "each_epoch.csv")
    assert os.path.exists(tmp_path / "out" / "checkpoints" / model.opt.name / "1_useSE_net_G.pth")


def test_nonfinite_skips_are_logged():
    """a step the bf16 non-finite guard skips shows in train.py's loss line.  One batch
    with a NaN pixel makes both networks' gradients non-finite: that step is skipped (graph replay
    included), the steps around it apply, and NonfiniteMonitor reports the counts."""
    import train as T
    from options.train_options import default_train_opt
    from models import create_model
    torch.manual_seed(20)
    model = create_model(default_train_opt(gpu_ids=[0], precision="bf16", batchSize=1, pool_size=0))
    assert model.scaler_G is not None and model.scaler_D is not None   # the guard is on by default in bf16
    mon = T.NonfiniteMonitor(model, abort_window=3)
    A, B = synth_pair(1, 64, seed=4)
    bad = A.clone()
    bad[0, 0, 5, 7] = float("nan")
    for i, a in enumerate((A, A, bad, A)):
        model.set_input({"A": a.to(DEV), "B": B.to(DEV), "A_paths": [""], "B_paths": [""]})
        model.optimize_parameters()
        if i == 1:
            assert mon.poll() == ""      # nothing skipped yet: the line is unchanged
    assert model.nonfinite_report() == {"G": (1, 4), "D": (1, 4)}
    assert mon.poll() == "skipped G 1/4 D 1/4 "
    assert all(torch.isfinite(p).all() for p in (model.flatG.data, model.flatD.data))
