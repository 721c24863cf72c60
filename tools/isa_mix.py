"""Static instruction mix of one kernel's loop bodies from an llvm-objdump listing: per basic block
between a backward branch target and the branch, the count of MFMA / VALU / LDS / VMEM / SALU /
waitcnt instructions -- the VALU-per-MFMA ratio of the hot loop without a GPU run.

    python tools/isa_mix.py listing.s <kernel-symbol-substring>
"""
import re
import sys


def kernel_lines(path, sub):
    out, on = [], False
    for line in open(path):
        m = re.match(r"^[0-9a-f]+ <(.*)>:$", line.strip())
        if m:
            on = sub in m.group(1)
            if on:
                out = []
            elif out:
                break
            continue
        if on and line.strip():
            out.append(line)
    return out


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("ds_read", "ds_write", "ds_bpermute", "ds_swizzle")):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    lines = kernel_lines(sys.argv[1], sys.argv[2])
    addrs = []
    for ln in lines:
        m = re.search(r"//\s*([0-9A-F]+):", ln)
        op = ln.split()[0]
        tgt = re.search(r"<[^+>]*\+0x([0-9a-f]+)>", ln)
        addrs.append((int(m.group(1), 16) if m else None, op, tgt))
    base = addrs[0][0] if addrs and addrs[0][0] is not None else 0
    tot = {}
    for a, op, _ in addrs:
        c = classify(op)
        tot[c] = tot.get(c, 0) + 1
    print("whole kernel:", tot)
    # loops: backward branches
    for i, (a, op, tgt) in enumerate(addrs):
        if op.startswith("s_cbranch") or op.startswith("s_branch"):
            if tgt and a is not None:
                t = base + int(tgt.group(1), 16)
                if t < a:
                    body = [o for (aa, o, _) in addrs if aa is not None and t <= aa <= a]
                    mix = {}
                    for o in body:
                        c = classify(o)
                        mix[c] = mix.get(c, 0) + 1
                    r = mix.get("valu", 0) / max(1, mix.get("mfma", 0))
                    print("loop %x..%x (%d instr): %s  valu/mfma %.1f" % (t - base, a - base, len(body), mix, r))


if __name__ == "__main__":
    main()
