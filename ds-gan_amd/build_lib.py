"""Build libdsgan_hip.so in-tree: hipcc --offload-arch=gfx950, one object per source, then link.

    python ds-gan_amd/build_lib.py [-j N] [--force] [--measure]

The library lands at ds-gan_amd/dsgan_hip/libdsgan_hip.so (git-ignored, but it travels to the
GPU box with the gpurun snapshot).  Objects are rebuilt only when a source or header is newer.
--measure builds the measurement variant (-DDSG_MEASURE: the pricing branches of planner knob 10,
e.g. epilogues that drop their stores) as libdsgan_hip_measure.so from its own objects; tools load
it with DSGAN_HIP_LIB=.../libdsgan_hip_measure.so.  The product library never carries them.
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "dsgan_hip")
OBJ_DIR = os.path.join(HERE, "build", "obj")
LIB = os.path.join(OUT_DIR, "libdsgan_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-fPIC", "-std=c++17", "--offload-arch=" + ARCH, "-Wno-unused-result", "-I" + CSRC]


# per-source extra flags
EXTRA = {"dwconv.hip": ["-fno-slp-vectorize"], "mlp.hip": ["-fno-slp-vectorize"], "thin3.hip": ["-fno-slp-vectorize"]}
# The pointwise GEMM units: their epilogue loops (8 accumulator blocks, every epilogue option) must
# unroll fully -- the accumulators and the prefetched gp registers are indexed by the loop counters --
# and LLVM's default budget for a #pragma unroll (16K instructions) refused them once the 16-byte
# stores carried their hazard pad (pw_impl.h pw_st128): "loop not unrolled", the arrays went to
# scratch and the gp-multiplied data-grad ran 8x slower.
for _f in ("pw_fwd_bf16.hip", "pw_fwd_f16.hip", "pw_dgrad_bf16.hip", "pw_dgrad_f16.hip", "pw_wgrad_bf16.hip",
           "pw_wgrad_f16.hip", "pwgemm.hip"):
    EXTRA[_f] = ["-mllvm", "-pragma-unroll-threshold=200000", "-Werror=pass-failed"]


def _includes(path, seen=None):
    """The csrc headers a source pulls in (transitively, quoted includes only)."""
    seen = set() if seen is None else seen
    import re
    with open(path) as f:
        for m in re.finditer(r'^\s*#\s*include\s+"([^"]+)"', f.read(), re.M):
            h = os.path.join(CSRC, m.group(1))
            if os.path.exists(h) and h not in seen:
                seen.add(h)
                _includes(h, seen)
    return seen


def _newer(src, obj, headers):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or any(os.path.getmtime(h) > t for h in headers)


def _compile(src, obj, defs=()):
    cmd = [HIPCC] + FLAGS + list(defs) + EXTRA.get(os.path.basename(src), []) + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("compile failed: %s\n%s\n%s" % (" ".join(cmd), r.stdout, r.stderr))
    return obj


def build(jobs=8, force=False, verbose=True, measure=False):
    obj_dir = OBJ_DIR + ("_measure" if measure else "")
    lib = LIB.replace(".so", "_measure.so") if measure else LIB
    defs = ["-DDSG_MEASURE"] if measure else []
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(OUT_DIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(obj_dir, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(s, o, _includes(s)):
            todo.append((s, o))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            futs = [ex.submit(_compile, s, o, defs) for s, o in todo]
            for f in cf.as_completed(futs):
                o = f.result()
                if verbose:
                    print("  built", os.path.relpath(o, HERE), flush=True)
    if todo or not os.path.exists(lib) or any(os.path.getmtime(o) > os.path.getmtime(lib) for o in objs):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s\n%s" % (r.stdout, r.stderr))
        if verbose:
            print("  linked", os.path.relpath(lib, HERE), flush=True)
    return lib


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--measure", action="store_true", help="the DSG_MEASURE variant (libdsgan_hip_measure.so)")
    a = ap.parse_args()
    build(a.j, a.force, measure=a.measure)
