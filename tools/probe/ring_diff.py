"""Where the persistent ring (planner knob 11) differs from the one-tile ring kernel: per output tensor,
the count of differing elements, the max |diff| and the (image, channel-tile, pixel-tile) positions."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch  # noqa: E402
import dsgan_hip  # noqa: E402
from dsgan_hip import _lib, functional as HF  # noqa: E402
from dsgan_hip._lib import call, ptr, stream  # noqa: E402

lib = _lib.load()
for half in ("bf16", "fp16"):
    dsgan_hip.set_precision(half)
    hd = torch.bfloat16 if half == "bf16" else torch.float16
    for (M, K, HW, NB) in [(512, 256, 128 * 128, 4), (768, 128, 64 * 64, 25)]:
        g0 = torch.Generator(device="cuda").manual_seed(M + K + NB)
        w = (torch.randn(M, K, device="cuda", generator=g0) / K ** 0.5).to(hd)
        bias = torch.randn(M, device="cuda", generator=g0)
        x = torch.randn(NB, K, HW, device="cuda", generator=g0).to(hd)
        outs = []
        for pers in (0, 1):
            lib.dsgan_pw_tune(9, 1)
            lib.dsgan_pw_tune(11, pers)
            y = torch.full((NB, M, HW), float("nan"), device="cuda", dtype=hd)
            gp = torch.full((NB, M, HW), float("nan"), device="cuda", dtype=hd)
            ws = torch.empty(max(1, lib.dsgan_pw_fd_workspace(0, M, K, HW, NB)), device="cuda")
            call("dsgan_pw_fwd_io_ws", ptr(w), 1, ptr(x), K * HW, 1, ptr(y), M * HW, 1, ptr(gp), M * HW, 1, ptr(bias),
                 M, K, HW, NB, 1, 0, 0.2, *HF.wsa(ws), stream())
            torch.cuda.synchronize()
            outs.append((y.float(), gp.float()))
        lib.dsgan_pw_tune(11, 0)
        for name, a, b in (("y", outs[0][0], outs[1][0]), ("gp", outs[0][1], outs[1][1])):
            d = (a != b) & ~(torch.isnan(a) & torch.isnan(b))
            n = int(d.sum())
            print(half, (M, K, HW, NB), name, "differ:", n, "of", d.numel(), "nan ref/got:",
                  int(torch.isnan(a).sum()), int(torch.isnan(b).sum()), flush=True)
            if n:
                idx = d.nonzero()
                print("   max|diff|", float((a - b)[d].abs().max()), "first", idx[:5].tolist(),
                      "img", sorted(set(idx[:, 0].tolist()))[:8], "mtiles", sorted(set((idx[:, 1] // 256).tolist()))[:8],
                      "ptiles", sorted(set((idx[:, 2] // 256).tolist()))[:8], flush=True)
                import collections
                cm = collections.Counter((idx[:, 1] % 256).tolist())
                pm = collections.Counter((idx[:, 2] % 256).tolist())
                print("   channel-in-tile", sorted(cm.items())[:40], flush=True)
                print("   pixel-in-tile", sorted(pm.items())[:64], flush=True)
                z = torch.einsum("mk,nkp->nmp", w.float(), x.float()) + bias[None, :, None]
                for t in idx[:6].tolist():
                    zz = float(z[t[0], t[1], t[2]])
                    print("   at", t, "ref", float(a[t[0], t[1], t[2]]), "got", float(b[t[0], t[1], t[2]]), "z", zz,
                          "gelu", float(torch.nn.functional.gelu(torch.tensor(zz))), flush=True)
