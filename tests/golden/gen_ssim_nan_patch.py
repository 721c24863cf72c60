"""Generates tests/golden/ssim_nan_patch.npz: the 16x16 input patches (real, fake in [-1, 1]) around
the SSIM output pixels whose backward coefficients were NaN in round 5's configs[4] run.

Run on the GPU box against a library built with round 5's losses.hip (the SSIM coefficient maps as
S * (1 / A1), S * (1 / A2)):
    bash tools/ab_lib.sh fead3f5 var_libs/old_ssim.so losses.hip
    DSGAN_HIP_LIB=$PWD/var_libs/old_ssim.so python tests/golden/gen_ssim_nan_patch.py [out.npz]
It replays the configs[4] quality leg (fp16, 512^2, batch 8, the reference init, pool 0, D_BATCH on)
for three steps, forms step 4's fake_B, runs the SSIM forward of (real_B, fake_B) and finds the output
pixels whose coefficient maps are not finite.  The SSIM of one output pixel reads only its 11 x 11
input window, in the same order at any tile offset, so a patch holding that window reproduces the
pixel's arithmetic: tests/test_ops_gpu.py::test_ssim_bwd_on_round5_nan_patches checks the current
kernel's input-grad there (finite, vs float64 autograd of the reference's formula).  Inputs only; the
expected values are computed by the test from oracle/dsgan_cpu.py.
"""
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import dsgan_cpu as O  # noqa: E402
from oracle.recipe import make_params, synth_pair  # noqa: E402

PATCH, OFF, MAX_PATCHES = 16, 2, 16


def main():
    import dsgan_hip
    from dsgan_hip import _lib, functional as HF
    from options.train_options import default_train_opt
    from models import create_model
    dsgan_hip.require_gpu()
    random.seed(20)
    torch.manual_seed(20)
    m = create_model(default_train_opt(gpu_ids=[0], pool_size=0, precision="fp16", batchSize=8, cuda_graph=0))
    with torch.no_grad():
        for net, pr in ((m.netG, make_params(O.g_param_spec(), "ref", 1000)),
                        (m.netD, make_params(O.d_param_spec(), "ref", 5000)),
                        (m.vgg, make_params(O.vgg_param_spec(True), "vgg", 7000))):
            for k, v in net.state_dict().items():
                v.copy_(pr[k])
    m.d_batch = True
    for i in range(4):
        A, B = synth_pair(8, 512, seed=100 + i)
        m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * 8, "B_paths": [""] * 8})
        if i < 3:
            m.optimize_parameters()
    with torch.no_grad():
        m.forward()
    real = ((m.real_B.float()) * 1).contiguous()
    fake = m.fake_B.detach().float().contiguous()
    N, C, H, W = real.shape
    Ho, Wo = H - 10, W - 10
    coef = torch.empty((3, N * C, Ho, Wo), device=real.device, dtype=torch.float32)
    s = torch.empty((), device=real.device, dtype=torch.float32)
    part = torch.empty(_lib.load().dsgan_ssim_parts(N * C, H, W), device=real.device, dtype=torch.float32)
    _lib.call("dsgan_ssim_fwd", _lib.ptr(real), _lib.ptr(fake), 0.5, 0.5, N * C, H, W, _lib.ptr(HF.gauss_win(real.device)),
              1e-4, 9e-4, _lib.ptr(coef), _lib.ptr(s), _lib.ptr(part), _lib.stream())
    torch.cuda.synchronize()
    bad = (~torch.isfinite(coef)).any(0).nonzero().tolist()
    print("non-finite coefficient pixels: %d" % len(bad), flush=True)
    rs, fs, where = [], [], []
    for p, oh, ow in bad:
        h0, w0 = min(max(oh - OFF, 0), H - PATCH), min(max(ow - OFF, 0), W - PATCH)
        if any(q == p and abs(a - h0) < PATCH and abs(b - w0) < PATCH for q, a, b in where):
            continue
        where.append((p, h0, w0))
        rs.append(real.view(N * C, H, W)[p, h0:h0 + PATCH, w0:w0 + PATCH].cpu().numpy())
        fs.append(fake.view(N * C, H, W)[p, h0:h0 + PATCH, w0:w0 + PATCH].cpu().numpy())
        if len(where) == MAX_PATCHES:
            break
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "ssim_nan_patch.npz")
    np.savez_compressed(out, real=np.stack(rs)[:, None], fake=np.stack(fs)[:, None], where=np.array(where, np.int32))
    print("wrote %s: %d patches at (plane, h0, w0) %s" % (out, len(where), where), flush=True)


if __name__ == "__main__":
    main()
