"""Check that templating a kernel source on the 16-bit operand type left the bf16 code unchanged:
compile the committed (git HEAD) and the working-tree version of one csrc file device-only to
assembly and compare every bf16 kernel's instruction stream (labels normalised).

    python tools/isa_same.py mlp.hip [extra hipcc flags...]
"""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "ds-gan_amd", "csrc")


def kernels(path):
    txt = open(path).read()
    out = {}
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)^\s*s_endpgm", txt, re.S | re.M):
        body = [ln.strip() for ln in m.group(2).split("\n")]
        body = [re.sub(r"\.L(BB\d+_\d+|post_getpc\d+)", "L", ln) for ln in body if ln and not ln.startswith((".", ";"))]
        out[m.group(1)] = body
    return out


def demangle(names):
    return subprocess.run(["c++filt"] + list(names), capture_output=True, text=True).stdout.split("\n")


def main():
    src, extra = sys.argv[1], sys.argv[2:]
    tmp = tempfile.mkdtemp()
    old = os.path.join(tmp, "old")
    os.makedirs(old)
    for f in os.listdir(CSRC):
        if f.endswith((".h", ".hip")):
            r = subprocess.run(["git", "-C", REPO, "show", "HEAD:ds-gan_amd/csrc/" + f], capture_output=True)
            if r.returncode == 0:
                open(os.path.join(old, f), "wb").write(r.stdout)
    cc = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S"] + extra
    subprocess.run(cc + ["-I" + old, os.path.join(old, src), "-o", os.path.join(tmp, "old.s")], check=True,
                   capture_output=True)
    subprocess.run(cc + ["-I" + CSRC, os.path.join(CSRC, src), "-o", os.path.join(tmp, "new.s")], check=True,
                   capture_output=True)
    o, n = kernels(os.path.join(tmp, "old.s")), kernels(os.path.join(tmp, "new.s"))
    # mangled names: a leading T16 template argument is "DF16b" (__bf16) / "DF16_" (_Float16); the
    # other parameters' mangling changes with it, so new bf16 kernels are matched by their bodies
    old_bodies = {tuple(v): k for k, v in o.items()}
    nd = n
    same = diff = 0
    for k, v in nd.items():
        if "IDF16_" in k:
            continue
        if tuple(v) in old_bodies:
            same += 1
        else:
            diff += 1
            print("DIFF (%d instr, no identical old kernel): %s" % (len(v), k[:120]))
    nf16 = sum(1 for k in nd if "IDF16_" in k)
    print("%s: %d bf16 kernels identical, %d differ; %d fp16 instantiations" % (src, same, diff, nf16))
    return 1 if diff else 0


if __name__ == "__main__":
    sys.exit(main())
