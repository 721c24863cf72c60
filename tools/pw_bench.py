"""In-process A/B of the pointwise GEMM launches of one bench step (B=16, 256^2) under planner knob
settings (dsgan_pw_tune), interleaved rounds, median per case (cdna_hip_programming.md §5.4 rule 24).

usage: python tools/pw_bench.py [--arm "0=1,2=256"] [--arm "0=0"] [--only SUBSTR] [--rounds 5]
Each --arm is a list key=value knob settings applied before timing (default: the built-in plan and
split-K off).  Cases follow the launch table (tools/launch_table.py, profiles/r03/launches_*.txt).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]

import torch  # noqa: E402

import dsgan_hip  # noqa: E402
from dsgan_hip import _lib  # noqa: E402
from dsgan_hip._lib import call, ptr, stream  # noqa: E402
from dsgan_hip import functional as HF  # noqa: E402

B = 16
GELU = 1


def cases(arms):
    """(name, flops, bytes, fn) -- each fn allocates nothing inside the timed call.  Scratch is sized
    for the largest plan over every arm's knob settings (a split plan differs per arm)."""
    out = []
    hd = torch.bfloat16
    lib = _lib.load()

    def most(q):
        base = {k: lib.dsgan_pw_tune(k, -1) for k in range(12)}
        n = 0
        for kv in arms:
            for k, v in kv.items():
                lib.dsgan_pw_tune(k, v)
            n = max(n, q())
        for k, v in base.items():
            lib.dsgan_pw_tune(k, v)
        return n

    def ws_fd(mode, M, K, P):
        n = most(lambda: lib.dsgan_pw_fd_workspace(mode, M, K, P, B))
        return torch.empty(max(n, 1), device="cuda")

    # unfused MLP blocks: (C, C4, P-out, HW)
    for C, C4, Pc, H in [(512, 2048, 256, 64), (1024, 4096, 512, 32), (512, 2048, 1024, 16), (256, 1024, 512, 32)]:
        HW = H * H
        h = torch.randn(B, C, HW, device="cuda").to(hd)
        w1 = (torch.randn(C4, C, device="cuda") / C ** 0.5).to(hd)
        b1 = torch.randn(C4, device="cuda")
        w2 = (torch.randn(Pc, C4, device="cuda") / C4 ** 0.5).to(hd)
        b2 = torch.randn(Pc, device="cuda")
        g = torch.empty(B, C4, HW, device="cuda", dtype=hd)
        gp = torch.empty_like(g)
        out_ = torch.randn(B, Pc, HW, device="cuda")
        dy = torch.randn(B, Pc, HW, device="cuda")
        dz = torch.empty_like(g)
        dh = torch.empty(B, C, HW, device="cuda")
        wsa, wsb, wsc, wsd = ws_fd(0, C4, C, HW), ws_fd(0, Pc, C4, HW), ws_fd(1, C4, Pc, HW), ws_fd(1, C, C4, HW)
        wg1 = torch.zeros(C4, C, device="cuda")
        wg2 = torch.zeros(Pc, C4, device="cuda")
        gb1, gb2 = torch.zeros(C4, device="cuda"), torch.zeros(Pc, device="cuda")
        wsw2 = torch.empty(max(1, most(lambda: lib.dsgan_pw_wgrad_workspace(Pc, C4, HW, B))), device="cuda")
        wsw1 = torch.empty(max(1, most(lambda: lib.dsgan_pw_wgrad_workspace(C4, C, HW, B))), device="cuda")
        tag = "C%d@%d" % (C, H)
        f1 = 2.0 * B * HW * C4 * C
        f2 = 2.0 * B * HW * C4 * Pc
        out += [
            ("fwd1-gp " + tag, f1, B * HW * (C * 2 + C4 * 4),
             lambda h=h, w1=w1, b1=b1, g=g, gp=gp, C=C, C4=C4, HW=HW, ws=wsa: call(
                 "dsgan_pw_fwd_io_ws", ptr(w1), 1, ptr(h), C * HW, 1, ptr(g), C4 * HW, 1, ptr(gp), C4 * HW, 1, ptr(b1),
                 C4, C, HW, B, GELU, 0, 0.2, ptr(ws), ws.numel(), stream())),
            ("fwd2-acc " + tag, f2, B * HW * (C4 * 2 + Pc * 8),
             lambda g=g, w2=w2, b2=b2, o=out_, C4=C4, Pc=Pc, HW=HW, ws=wsb: call(
                 "dsgan_pw_fwd_io_ws", ptr(w2), 1, ptr(g), C4 * HW, 1, ptr(o), Pc * HW, 0, None, 0, 0, ptr(b2),
                 Pc, C4, HW, B, 0, 1, 0.2, ptr(ws), ws.numel(), stream())),
            ("dgrad2-gp " + tag, f2, B * HW * (Pc * 4 + C4 * 4),
             lambda w2=w2, dy=dy, dz=dz, gp=gp, C4=C4, Pc=Pc, HW=HW, ws=wsc: call(
                 "dsgan_pw_dgrad_io_ws", ptr(w2), 1, ptr(dy), Pc * HW, 0, ptr(dz), C4 * HW, 1, ptr(gp), C4 * HW,
                 C4, Pc, HW, B, 0, ptr(ws), ws.numel(), stream())),
            ("dgrad1 " + tag, f1, B * HW * (C4 * 2 + C * 4),
             lambda w1=w1, dz=dz, dh=dh, C=C, C4=C4, HW=HW, ws=wsd: call(
                 "dsgan_pw_dgrad_io_ws", ptr(w1), 1, ptr(dz), C4 * HW, 1, ptr(dh), C * HW, 0, None, 0, C, C4,
                 HW, B, 0, ptr(ws), ws.numel(), stream())),
            ("wgrad2 " + tag, f2, B * HW * (Pc * 4 + C4 * 2),
             lambda dy=dy, g=g, wg2=wg2, gb2=gb2, C4=C4, Pc=Pc, HW=HW, ws=wsw2: call(
                 "dsgan_pw_wgrad_mixed", ptr(dy), Pc * HW, 0, ptr(g), C4 * HW, 1, ptr(wg2), ptr(gb2), Pc, C4, HW, B,
                 ptr(ws), ws.numel(), stream())),
            ("wgrad1 " + tag, f1, B * HW * (C4 * 2 + C * 2),
             lambda dz=dz, h=h, wg1=wg1, gb1=gb1, C=C, C4=C4, HW=HW, ws=wsw1: call(
                 "dsgan_pw_wgrad_mixed", ptr(dz), C4 * HW, 1, ptr(h), C * HW, 1, ptr(wg1), ptr(gb1), C4, C, HW, B,
                 ptr(ws), ws.numel(), stream())),
        ]
    # fp32 generic path (downSkip / shortcut 1x1s): (mode, M, K, H)
    for mode, M, K, H in [(1, 64, 1024, 16), (1, 128, 1024, 16), (1, 256, 1024, 16), (1, 512, 1024, 16),
                          (0, 1024, 256, 32), (0, 256, 512, 64), (1, 512, 256, 64), (0, 1024, 64, 16),
                          (0, 64, 128, 256), (1, 128, 64, 256)]:
        HW = H * H
        w = torch.randn(M, K, device="cuda") if mode == 0 else torch.randn(K, M, device="cuda")
        x = torch.randn(B, K, HW, device="cuda")
        y = torch.empty(B, M, HW, device="cuda")
        ws = ws_fd(mode, M, K, HW)
        out.append(("%s-f32 M%d K%d @%d" % ("fwd" if mode == 0 else "dgrad", M, K, H), 2.0 * B * HW * M * K,
                    B * HW * (K + M) * 4,
                    lambda mode=mode, w=w, x=x, y=y, M=M, K=K, HW=HW, ws=ws: call(
                        "dsgan_pw_gemm", mode, ptr(w), 0, ptr(x), K * HW, ptr(y), M * HW, None, None, 0, None, 0,
                        M, B * HW, K, HW, B, 0, 0, 0, 0, 0.2, ptr(ws), ws.numel(), stream())))
    return out


def timeit(fn, it):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arm", action="append", default=None)
    ap.add_argument("--only", default=None)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--it", type=int, default=10)
    a = ap.parse_args()
    dsgan_hip.require_gpu()
    HF.set_precision("bf16")
    lib = _lib.load()
    arms = a.arm or ["", "0=0"]
    base = {k: lib.dsgan_pw_tune(k, -1) for k in range(12)}
    parsed = []
    for s in arms:
        kv = dict(base)
        for t in filter(None, s.split(",")):
            k, v = t.split("=")
            kv[int(k)] = int(v)
        parsed.append(kv)
    cs = [c for c in cases(parsed) if not a.only or a.only in c[0]]
    res = {(c[0], i): [] for c in cs for i in range(len(parsed))}
    for _ in range(a.rounds):
        for i, kv in enumerate(parsed):
            for k, v in kv.items():
                lib.dsgan_pw_tune(k, v)
            for name, fl, by, fn in cs:
                res[(name, i)].append(timeit(fn, a.it))
    for k, v in base.items():
        lib.dsgan_pw_tune(k, v)
    print("arms: " + " | ".join("[%d] %s" % (i, s or "built-in") for i, s in enumerate(arms)))
    tot = [0.0] * len(parsed)
    for name, fl, by, fn in cs:
        row = []
        for i in range(len(parsed)):
            t = sorted(res[(name, i)])[len(res[(name, i)]) // 2]
            tot[i] += t
            row.append("%8.1f us %6.0f TF/s %6.0f GB/s" % (t, fl / t / 1e6, by / t / 1e3))
        print("%-24s %s" % (name, " | ".join(row)), flush=True)
    print("%-24s %s" % ("total", " | ".join("%8.1f us" % t for t in tot)))


if __name__ == "__main__":
    main()
