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
family: its algorithmic FLOPs and bytes per launch (every operand read / written once, in its
stored dtype) over the HIP-event time of its launches in the timed region, bound = the resource
that work needs longest at peak (dense bf16 MFMA 2.5 PF/s, HBM 8 TB/s), plus the PMC traffic
and MFMA-busy of the same command from the committed rocprofv3 summaries under profiles/;
"quality" (MS-SSIM Δ vs the fp32 oracle after 10 steps at the bench batch) and "cpu_baseline"
(the oracle, a port of the reference step, timed on this host's cores over steps 3-7 of that
same 10-step run) at N=1 only.
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


PEAK_HBM_GBS = 8000.0       # MI355X HBM3E (MI355X_MICROARCH.md)
STEP_GFLOP_PER_IMG = 367.02  # algorithmic GFLOP per 256x256 image pair of one G+D step


def host_cpu():
    """The host's CPU as BASELINE.md §3 asks for it: model name, physical cores of the CPUs this
    process may run on (sched affinity, SMT siblings counted once), and the cgroup CPU quota; the
    baseline uses every physical core it is allowed (min of the two)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    cpus = sorted(os.sched_getaffinity(0))
    phys = set()
    for c in cpus:
        try:
            base = "/sys/devices/system/cpu/cpu%d/topology/" % c
            with open(base + "physical_package_id") as f1, open(base + "core_id") as f2:
                phys.add((f1.read().strip(), f2.read().strip()))
        except OSError:
            phys.add(("?", str(c)))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    threads = len(phys) if quota is None else min(len(phys), quota)
    return {"cpu_model": model, "logical_cpus_allowed": len(cpus), "physical_cores_allowed": len(phys),
            "cgroup_cpu_quota": quota, "threads": threads}


def reference_legs(steps=10, batch=16, size=256, threads=None, timed=(2, 7)):
    """The two legs of the metric that need the reference's arithmetic, on ONE shared run:

    * quality -- 'MS-SSIM Δ vs ref': the GPU model (bench precision) and the CPU oracle
      (oracle/dsgan_cpu.py, the reference step restated in fp32 -- the checker, never the thing
      measured) train `steps` steps from identical weights (the reference's own N(0, 0.02) init
      recipe) on identical synthetic pairs at the bench batch (pool_size 0).  Δ =
      |MS-SSIM(fake_gpu, real_B) - MS-SSIM(fake_ref, real_B)| on the last step's fake_B,
      DSGAN/MS_SSIM.py:153 with data_range 1.
    * cpu_baseline -- the oracle's steps [timed[0], timed[1]) of that same run (BASELINE.md §3:
      2 warm-up + 5 timed steps, fp32), clamped to the steps run, on every physical core the
      process may use (``host_cpu``; ``threads`` overrides).
    Each leg reports its own error instead of hiding the other."""
    import random
    from oracle import dsgan_cpu as O
    from oracle.recipe import make_params, synth_pair
    from options.train_options import default_train_opt
    from models import create_model
    from dsgan_hip import functional as HF
    host = host_cpu()
    if threads is None:
        threads = host["threads"]
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
    cpu_s = []
    for i in range(steps):
        A, B = synth_pair(batch, size, seed=100 + i)
        model.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * batch, "B_paths": [""] * batch})
        model.optimize_parameters()
        tc = time.perf_counter()
        ref.step(A, B)
        cpu_s.append(time.perf_counter() - tc)
        print("[bench] reference leg step %d/%d: oracle %.1f s" % (i + 1, steps, cpu_s[-1]), file=sys.stderr, flush=True)
    HF.set_precision(prec)
    try:
        fg = model.fake_B.detach().float().cpu()
        fo = ref.fake_B
        tgt = (B + 1) / 2
        m_gpu = O.ms_ssim((fg + 1) / 2, tgt).item()
        m_ref = O.ms_ssim((fo + 1) / 2, tgt).item()
        quality = {"msssim_delta": round(abs(m_gpu - m_ref), 6), "msssim_gpu": round(m_gpu, 6),
                   "msssim_ref": round(m_ref, 6),
                   "msssim_gpu_vs_ref": round(O.ms_ssim(((fg + 1) / 2).clamp(0, 1), ((fo + 1) / 2).clamp(0, 1)).item(), 6),
                   "steps": steps, "batch": batch, "size": size, "init": "reference N(0,0.02) recipe",
                   "precision": prec, "ref": "oracle/dsgan_cpu.py fp32 (%d threads)" % threads,
                   "seconds": round(time.time() - t0, 1)}
    except Exception as e:  # noqa: BLE001 -- reported in the line, never fatal
        quality = {"error": repr(e)}
    try:
        b = min(timed[1], steps)
        a = min(timed[0], max(0, b - 1))
        ts = sum(cpu_s[a:b])
        cpu = dict(value=round(batch * (b - a) / ts, 4), unit="img/s", cores=threads, kind="port",
                   cpu_model=host["cpu_model"], physical_cores_allowed=host["physical_cores_allowed"],
                   logical_cpus_allowed=host["logical_cpus_allowed"], cgroup_cpu_quota=host["cgroup_cpu_quota"],
                   sample="oracle/dsgan_cpu.py OracleStep (a port of the reference step), fp32, %dx%d, batch %d: "
                          "steps %d-%d of the quality leg's %d (%d warm-up + %d timed, %.1f s), %d host threads "
                          "(every physical core this job may use)"
                          % (size, size, batch, a + 1, b, steps, a, b - a, ts, threads))
    except Exception as e:  # noqa: BLE001
        cpu = {"error": repr(e)}
    return quality, cpu


def _profile_json(name):
    """A committed rocprofv3 summary over this same bench command (the newest round that has it)."""
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):
        path = os.path.join(REPO, "profiles", rnd, name)
        try:
            with open(path) as f:
                return json.load(f)["families"], "profiles/%s/%s" % (rnd, name)
        except (OSError, ValueError, KeyError):
            continue
    return {}, None


def rocprof_family_avg_us(csv_path, family):
    """(average us, calls) of every kernel whose name contains ``family`` in a rocprofv3 --stats
    style CSV (tools/prof_stats.py): the figure the line's ``avg_launch_us`` must agree with."""
    import csv
    calls, ns = 0, 0.0
    with open(csv_path, newline="") as f:
        for row in csv.DictReader(f):
            if family in row["Name"]:
                calls += int(row["Calls"])
                ns += float(row["TotalDurationNs"])
    return (ns / calls / 1e3 if calls else None), calls


def roofline_block(ig, fams, timing_steps, peak, roof_src, pmc_t=None, pmc_t_src=None, pmc_m=None, pmc_m_src=None,
                   pw_ms=None):
    """The line's ``roofline`` object from the kernel timer's records.

    ``ig`` = KernelTimer.summary() and ``fams`` = KernelTimer.families() over the launches of
    ``timing_steps`` whole steps: the timed region's steps when the timer read them, or the eager
    steps timed after it when events recorded by graph nodes are unreadable.  Every per-step
    figure divides by ``timing_steps`` -- never by the bench's --steps, which the timer may not
    have seen.  The dominant kernel is the contraction family with the most time; its bound is
    whichever resource its algorithmic work needs longest at peak.

    ``pw_ms`` = per-launch ms of the pointwise GEMM kernels alone (``KernelTimer.pw_kernel_ms``: the
    library's events around the GEMM kernel launch, without the split-K finishing pass the C-ABI
    call may add).  When the dominant family is ``pwgemm_kernel`` and those cover the same launches,
    ``achieved`` / ``frac`` / ``avg_launch_us`` are the kernel's own (the figure rocprofv3 reports);
    the C-ABI bracket stays beside it as ``bracket_avg_launch_us``."""
    pmc_t, pmc_m = pmc_t or {}, pmc_m or {}
    ts = max(1, int(timing_steps))
    ach = ig["flops"] / (ig["total_ms"] * 1e-3) / 1e12 if ig["total_ms"] > 0 else 0.0
    dom, (dn, dms, dfl, dby) = max(fams.items(), key=lambda kv: kv[1][1])
    bracket_ms = dms
    kernel_only = bool(dom == "pwgemm_kernel" and pw_ms and len(pw_ms) == dn)
    if kernel_only:
        dms = float(sum(pw_ms))
    t_avg = dms / max(1, dn) * 1e-3
    fl_l, by_l = dfl / max(1, dn), dby / max(1, dn)
    mfma_ach, hbm_ach = fl_l / t_avg / 1e12, by_l / t_avg / 1e9
    hbm_bound = by_l / (PEAK_HBM_GBS * 1e9) > fl_l / (peak * 1e12)
    traffic = pmc_t.get(dom, {}).get("traffic_bytes_per_launch")
    return {"bound": "hbm" if hbm_bound else "mfma", "kernel": dom, "timing": roof_src, "timing_steps": ts,
            "achieved": round(hbm_ach if hbm_bound else mfma_ach, 2), "peak": PEAK_HBM_GBS if hbm_bound else peak,
            "unit": "GB/s" if hbm_bound else "TFLOP/s",
            "frac": round(hbm_ach / PEAK_HBM_GBS if hbm_bound else mfma_ach / peak, 4),
            "traffic": traffic,
            "traffic_unit": "HBM bytes per launch, rocprofv3 PMC (FETCH_SIZE x2 + WRITE_SIZE) over this command: %s" % pmc_t_src,
            "algorithmic_bytes_per_launch": round(by_l), "algorithmic_gflop_per_launch": round(fl_l / 1e9, 3),
            "waste_ratio": round(traffic / by_l, 3) if traffic and by_l else None,
            "mfma": {"achieved_tflops": round(mfma_ach, 2), "frac": round(mfma_ach / peak, 4),
                     "pmc_mfma_busy": pmc_m.get(dom, {}).get("mfma_busy"), "pmc_source": pmc_m_src},
            "hbm": {"achieved_gbs": round(hbm_ach, 1), "frac": round(hbm_ach / PEAK_HBM_GBS, 4)},
            "launches_per_step": round(dn / ts, 2), "kernel_ms_per_step": round(dms / ts, 3),
            "avg_launch_us": round(dms / max(1, dn) * 1e3, 1),
            "avg_launch_timing": ("kernel-only events around the GEMM kernel launch (dsgan_ktimer)" if kernel_only else
                                  "HIP events around the C-ABI call (kernel-only events unavailable: %s)"
                                  % ("not the pointwise family" if dom != "pwgemm_kernel" else
                                     "unreadable" if pw_ms is None else
                                     "%d kernel pairs for %d calls" % (len(pw_ms), dn))),
            "bracket_avg_launch_us": round(bracket_ms / max(1, dn) * 1e3, 1),
            "all_contractions": {"achieved": round(ach, 2), "frac": round(ach / peak, 4),
                                 "ms_per_step": round(ig["total_ms"] / ts, 3),
                                 "gflop_per_step": round(ig["flops"] / ts / 1e9, 1),
                                 "launches_per_step": round(ig["launches"] / ts, 2)},
            "families": {k: {"ms_per_step": round(v[1] / ts, 3), "launches_per_step": round(v[0] / ts, 2),
                             "tflops": round(v[2] / (v[1] * 1e-3) / 1e12, 1) if v[1] > 0 else 0.0,
                             "gbs": round(v[3] / (v[1] * 1e-3) / 1e9, 1) if v[1] > 0 else 0.0}
                         for k, v in sorted(fams.items(), key=lambda kv: -kv[1][1])}}


EAGER_TIMING_STEPS = 2   # eager steps timed after the region when graph-node events are unreadable


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16, help="per-GPU batch (BASELINE config 2: 16)")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp16", "fp32"],
                    help="MFMA operand type (fp32 accumulation); configs[4] names fp16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-quality", action="store_true", help="skip the MS-SSIM delta leg")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="oracle threads for cpu_baseline (default: every physical core the job may use)")
    ap.add_argument("--quality-steps", type=int, default=10, help="steps of the shared quality / cpu_baseline leg")
    ap.add_argument("--no-train-equiv", action="store_true",
                    help="skip the train.py-equivalent iteration leg (profiling runs)")
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

    graphed = bool(getattr(model, "cuda_graph", False))
    nwarm = max(args.warmup, 2) if graphed else args.warmup   # eager step + capture, both untimed
    for w in range(nwarm):
        if graphed and w == 1:
            # the per-launch HIP events of the roofline leg are recorded INSIDE the captured graphs
            # (the capture happens in this call): every replay re-records them, and the leg reads the
            # last timed replay's
            HF.IGEMM_TIMER.reset()
            HF.IGEMM_TIMER.on = True
        model.optimize_parameters()
    torch.cuda.synchronize()

    if not graphed:
        HF.IGEMM_TIMER.reset()
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
    roof_src = "HIP events inside the captured graphs, last timed replay" if graphed else "HIP events, timed steps"
    # the graph's event nodes are re-recorded by every replay, so a readable record covers ONE step
    timing_steps = 1 if graphed else args.steps
    try:
        ig = HF.IGEMM_TIMER.summary()
        if ig["launches"] == 0:
            raise RuntimeError("no timer records")
    except Exception:   # noqa: BLE001 -- events recorded by graph nodes unreadable: time eager steps
        torch.cuda.synchronize()
        HF.IGEMM_TIMER.reset()
        HF.IGEMM_TIMER.on = True
        model.cuda_graph = False
        for _ in range(EAGER_TIMING_STEPS):
            model.optimize_parameters()
        model.cuda_graph = graphed
        HF.IGEMM_TIMER.on = False
        ig = HF.IGEMM_TIMER.summary()
        timing_steps = EAGER_TIMING_STEPS
        roof_src = ("HIP events of %d eager steps after the timed region (graph-node events unreadable)"
                    % EAGER_TIMING_STEPS)

    # train.py-equivalent iteration (DSGAN/train.py:106-124): the step plus the post-step
    # get_img_tir / get_img_gen forward / get_img_label and the per-iteration SSIM + PSNR of image 0
    # (device-side, util/metrics.py) -- timed separately, never part of `value`
    n_tp, dt_tp = 0, None
    if not args.no_train_equiv:
        from util.metrics import TrainMetrics
        metrics = TrainMetrics(model.device)
        n_tp = max(1, args.steps)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(n_tp):
            model.set_input(data)
            model.optimize_parameters()
            model.get_img_tir(data)
            with torch.no_grad():
                model.get_img_gen(data)
            model.get_img_label(data)
            metrics.update(model.fake_B[0], model.real_B[0])
        torch.cuda.synchronize()
        dt_tp = time.perf_counter() - t1
        if world > 1:
            t = torch.tensor([dt_tp], device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt_tp = t.item()

    fams = HF.IGEMM_TIMER.families()
    pw_ms = HF.IGEMM_TIMER.pw_kernel_ms()   # the pointwise GEMM kernels alone (no split-K finishing pass)
    if rank == 0:
        imgs = args.batch * args.steps * world
        peak = PEAK_F32_TFLOPS if args.precision == "fp32" else PEAK_BF16_TFLOPS   # dense fp16 = bf16 rate
        pmc_t, pmc_t_src = _profile_json("pmc_traffic.json")
        pmc_m, pmc_m_src = _profile_json("mfma_pmc.json")
        roof = roofline_block(ig, fams, timing_steps, peak, roof_src, pmc_t, pmc_t_src, pmc_m, pmc_m_src, pw_ms=pw_ms)
        out = {
            "metric": METRIC,
            "value": round(imgs / dt, 3),
            "unit": "img/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": nwarm,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (u8-uniform TIR/RGB pairs normalised as aligned_dataset.py; seeded random-init weights)",
            "config": {"workload": "DS-GAN optimize_parameters, MixConvNeXtML G + PatchGAN D + VGG16 perceptual + SSIM/L1/TV",
                       "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                       "image": [args.size, args.size], "parallelism": "dp%d" % world,
                       "hip_graphs": graphed,
                       "baseline_config": ("configs[1]: 256x256, batch 16, bf16, 1xMI355X"
                                           if (args.size, args.batch, world) == (256, 16, 1) else
                                           "configs[2]: 256x256, batch 16/GPU, %dxMI355X, grad all-reduce over RCCL" % world
                                           if (args.size, args.batch) == (256, 16) else
                                           "configs[3] shape: 256x256, batch 32/GPU (VGG16 perceptual + SSIM; "
                                           "--ssim_loss ms_ssim is the MS-SSIM opt-in)"
                                           if (args.size, args.batch) == (256, 32) else
                                           ("configs[4]: 512x512 upsampled, batch 8/GPU, fp16 MFMA operands (%dxMI355X)" % world
                                            if args.precision == "fp16" else
                                            "configs[4] shape (512x512, batch 8/GPU) in %s (configs[4] names fp16: "
                                            "--precision fp16)" % args.precision)
                                           if (args.size, args.batch) == (512, 8) else
                                           "off-baseline shape %dx%d, batch %d" % (args.size, args.size, args.batch))},
            "roofline": roof,
            # the whole step against the dense MFMA peak: SURVEY.md section 8(d)'s algorithmic work per
            # image pair (367.02 GFLOP at 256^2: G fwd+bwd 244.5, D 13.0, VGG16 2 fwd + 1 data-grad 109.5)
            "step_roofline": {"gflop_per_img": STEP_GFLOP_PER_IMG if args.size == 256 else None,
                              "achieved_tflops": round(STEP_GFLOP_PER_IMG * imgs / dt / 1e3, 1) if args.size == 256 else None,
                              "peak_tflops": peak,
                              "frac": round(STEP_GFLOP_PER_IMG * imgs / dt / 1e3 / peak, 4) if args.size == 256 else None,
                              "counted_conv_gflop_per_img": round(ig["flops"] / timing_steps / 1e9 / args.batch, 2),
                              "source": "SURVEY.md 8(d); counted = the conv launches IGEMM_TIMER saw"},
        }
        if dt_tp:
            out["train_py_equiv"] = {
                "iters_per_s": round(n_tp / dt_tp, 3), "img_per_s": round(args.batch * world * n_tp / dt_tp, 3),
                "ms_per_iter": round(dt_tp / n_tp * 1e3, 3), "iters": n_tp,
                "what": "DSGAN/train.py:106-124 iteration: set_input + optimize_parameters + get_img_tir + "
                        "get_img_gen (forward) + get_img_label + per-iteration SSIM/PSNR of image 0"}
        if world == 1 and not (args.no_cpu_baseline and args.no_quality):
            try:
                q, cpu = reference_legs(steps=args.quality_steps, batch=args.batch, size=args.size,
                                        threads=args.cpu_threads)
                if not args.no_quality:
                    out["quality"] = q
                if not args.no_cpu_baseline:
                    out["cpu_baseline"] = cpu
            except Exception as e:  # reported, never fatal to the GPU measurement
                for leg, skip in (("quality", args.no_quality), ("cpu_baseline", args.no_cpu_baseline)):
                    if not skip:
                        out[leg] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
