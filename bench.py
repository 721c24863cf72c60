"""DS-GAN G+D train-step throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]            # N=1 default
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A "step" is one Pix2PixModel.optimize_parameters (DSGAN/models/pix2pix_model.py:201-217):
G forward, D update (2 D passes + backward + Adam), G update (D pass, L1, VGG16 x2, TV, SSIM,
G backward + Adam), with the RCCL gradient all-reduces when N > 1.  Workload = BASELINE
config 2 per GPU: 256x256 pairs, batch 16 per GPU, bf16 MFMA operands (fp32 accumulate and
fp32 master weights/activations), synthetic inputs resident in HBM, weak scaling.

Printed JSON (rank 0): value = image-pairs/s over all ranks; "roofline" for the dominant kernel
family (the implicit-GEMM MFMA kernel: algorithmic conv FLOPs / HIP-event time of its
launches in the timed region, vs the dense bf16 MFMA peak); "cpu_baseline" = the CPU oracle
(oracle/dsgan_cpu.py, a port of the reference step) timed on this host's cores.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "256×256 paired imgs/sec (G+D step) at 1/2/4/8 MI355X; MS-SSIM Δ vs ref"
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3


def cpu_baseline(threads):
    """Bounded sample of the same step on the CPU oracle: 1 warmup + 6 timed steps at 256^2, B=2
    (~10-20 s of CPU work)."""
    from oracle import dsgan_cpu as O
    from oracle.recipe import make_params, synth_pair
    torch.set_num_threads(threads)
    gp = make_params(O.g_param_spec(), "ref", 1000)
    dp = make_params(O.d_param_spec(), "ref", 5000)
    vp = make_params(O.vgg_param_spec(False), "vgg", 7000)
    st = O.OracleStep(gp, dp, vp, pool_size=50)
    A, B = synth_pair(2, 256, seed=0)
    st.step(A, B)
    t0 = time.time()
    steps = 6
    for _ in range(steps):
        st.step(A, B)
    dt = time.time() - t0
    return dict(value=round(2 * steps / dt, 4), unit="img/s", cores=threads, kind="port",
                sample="oracle/dsgan_cpu.py OracleStep, fp32, 256x256, batch 2, %d timed steps after 1 warmup (%.1f s)" % (steps, dt))


PMC_TRAFFIC = os.path.join(REPO, "profiles", "r01", "pmc_traffic.json")


def pmc_traffic(family):
    """HBM bytes per launch of a kernel family, from the committed rocprofv3 --pmc passes over
    this same bench command (tools/gpu_pmc.sh -> tools/pmc_traffic.py; FETCH_SIZE doubled per
    the gfx950 correction, + WRITE_SIZE).  None when that family was not profiled."""
    try:
        with open(PMC_TRAFFIC) as f:
            fams = json.load(f)["families"]
        return fams[family]["traffic_bytes_per_launch"] if family in fams else None
    except (OSError, ValueError, KeyError):
        return None


def quality(steps=10, batch=2, size=256, threads=16):
    """'MS-SSIM Δ vs ref' of the BASELINE metric.  The GPU model (bench precision) and the CPU
    oracle (oracle/dsgan_cpu.py, the reference step restated in fp32 -- the checker, never the
    thing measured) train `steps` steps from identical weights (the reference's own N(0, 0.02)
    init recipe) on identical synthetic 256^2 pairs (pool_size 0).  Δ = |MS-SSIM(fake_gpu, real_B)
    - MS-SSIM(fake_ref, real_B)| on the last step's fake_B, DSGAN/MS_SSIM.py:153 with data_range 1."""
    import random
    from oracle import dsgan_cpu as O
    from oracle.recipe import make_params, synth_pair
    from options.train_options import default_train_opt
    from models import create_model
    from dsgan_hip import functional as HF
    torch.set_num_threads(threads)
    prec = HF.get_precision()
    random.seed(20)
    torch.manual_seed(20)
    model = create_model(default_train_opt(gpu_ids=[torch.cuda.current_device()], pool_size=0, precision=prec,
                                           batchSize=batch))
    gp = make_params(O.g_param_spec(), "ref", 1000)
    dp = make_params(O.d_param_spec(), "ref", 5000)
    with torch.no_grad():
        for net, pr in ((model.netG, gp), (model.netD, dp), (model.vgg, make_params(O.vgg_param_spec(True), "vgg", 7000))):
            for k, v in net.state_dict().items():
                v.copy_(pr[k])
    ref = O.OracleStep(gp, dp, make_params(O.vgg_param_spec(False), "vgg", 7000), pool_size=0)
    t0 = time.time()
    for i in range(steps):
        A, B = synth_pair(batch, size, seed=100 + i)
        model.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * batch, "B_paths": [""] * batch})
        model.optimize_parameters()
        ref.step(A, B)
    fg = model.fake_B.detach().float().cpu()
    fo = ref.fake_B
    tgt = (B + 1) / 2
    m_gpu = O.ms_ssim((fg + 1) / 2, tgt).item()
    m_ref = O.ms_ssim((fo + 1) / 2, tgt).item()
    HF.set_precision(prec)
    return {"msssim_delta": round(abs(m_gpu - m_ref), 6), "msssim_gpu": round(m_gpu, 6), "msssim_ref": round(m_ref, 6),
            "msssim_gpu_vs_ref": round(O.ms_ssim(((fg + 1) / 2).clamp(0, 1), ((fo + 1) / 2).clamp(0, 1)).item(), 6),
            "steps": steps, "batch": batch, "size": size, "init": "reference N(0,0.02) recipe", "precision": prec,
            "ref": "oracle/dsgan_cpu.py fp32 (%d threads)" % threads, "seconds": round(time.time() - t0, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16, help="per-GPU batch (BASELINE config 2: 16)")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-quality", action="store_true", help="skip the MS-SSIM delta leg")
    ap.add_argument("--cpu-threads", type=int, default=16)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))

    import dsgan_hip
    from dsgan_hip import functional as HF
    from options.train_options import default_train_opt
    from models import create_model
    from oracle.recipe import synth_pair

    dsgan_hip.require_gpu()
    torch.manual_seed(20)
    opt = default_train_opt(gpu_ids=[local], precision=args.precision, batchSize=args.batch)
    model = create_model(opt)
    A, B = synth_pair(args.batch, args.size, seed=rank)
    data = {"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * args.batch, "B_paths": [""] * args.batch}
    model.set_input(data)

    for _ in range(args.warmup):
        model.optimize_parameters()
    torch.cuda.synchronize()

    HF.IGEMM_TIMER.rec = []
    HF.IGEMM_TIMER.on = True
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        model.optimize_parameters()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    HF.IGEMM_TIMER.on = False
    if world > 1:
        t = torch.tensor([dt], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    ig = HF.IGEMM_TIMER.summary()

    fams = HF.IGEMM_TIMER.families()
    if rank == 0:
        imgs = args.batch * args.steps * world
        peak = PEAK_BF16_TFLOPS if args.precision == "bf16" else PEAK_F32_TFLOPS
        ach = ig["flops"] / (ig["total_ms"] * 1e-3) / 1e12 if ig["total_ms"] > 0 else 0.0
        # dominant kernel: the contraction family with the most time in the timed steps
        dom, (dn, dms, dfl) = max(fams.items(), key=lambda kv: kv[1][1])
        dach = dfl / (dms * 1e-3) / 1e12 if dms > 0 else 0.0
        out = {
            "metric": METRIC,
            "value": round(imgs / dt, 3),
            "unit": "img/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (u8-uniform TIR/RGB pairs normalised as aligned_dataset.py; seeded random-init weights)",
            "config": {"workload": "DS-GAN optimize_parameters, MixConvNeXtML G + PatchGAN D + VGG16 perceptual + SSIM/L1/TV",
                       "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                       "image": [args.size, args.size], "parallelism": "dp%d" % world,
                       "baseline_config": ("configs[1]: 256x256, batch 16, bf16, 1xMI355X"
                                           if (args.size, args.batch) == (256, 16) else
                                           "configs[4] shape: 512x512, batch 8/GPU (bf16 for the named fp16)"
                                           if (args.size, args.batch) == (512, 8) else
                                           "off-baseline shape %dx%d, batch %d" % (args.size, args.size, args.batch))},
            "roofline": {"bound": "mfma", "kernel": dom,
                         "achieved": round(dach, 2), "peak": peak, "unit": "TFLOP/s",
                         "frac": round(dach / peak, 4), "traffic": pmc_traffic(dom),
                         "traffic_unit": "HBM bytes per launch (rocprofv3 PMC, profiles/r01/pmc_traffic.json)",
                         "traffic_gbs": (round(pmc_traffic(dom) / (dms / max(1, dn) * 1e-3) / 1e9, 1)
                                         if pmc_traffic(dom) and dms > 0 else None),
                         "launches_per_step": round(dn / args.steps, 2),
                         "kernel_ms_per_step": round(dms / args.steps, 3),
                         "avg_launch_us": round(dms / max(1, dn) * 1e3, 1),
                         "gflop_per_launch": round(dfl / max(1, dn) / 1e9, 3),
                         "all_contractions": {"achieved": round(ach, 2), "frac": round(ach / peak, 4),
                                              "ms_per_step": round(ig["total_ms"] / args.steps, 3),
                                              "gflop_per_step": round(ig["flops"] / args.steps / 1e9, 1),
                                              "launches_per_step": ig["launches"] // max(1, args.steps)},
                         "families": {k: {"ms_per_step": round(v[1] / args.steps, 3),
                                          "tflops": round(v[2] / (v[1] * 1e-3) / 1e12, 1) if v[1] > 0 else 0.0}
                                      for k, v in sorted(fams.items(), key=lambda kv: -kv[1][1])}},
        }
        if not args.no_cpu_baseline and world == 1:
            try:
                out["cpu_baseline"] = cpu_baseline(args.cpu_threads)
            except Exception as e:  # reported, never fatal to the GPU measurement
                out["cpu_baseline"] = {"error": repr(e)}
        if not args.no_quality and world == 1:
            try:
                out["quality"] = quality(threads=args.cpu_threads)
            except Exception as e:
                out["quality"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
