"""Instruction mix of the hottest (longest backward-branch) loop of each kernel in a device-only
.s file: python tools/loop_mix.py file.s [name-regex]"""
import re
import sys


def main():
    txt = open(sys.argv[1]).read()
    flt = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)^\s*s_endpgm", txt, re.S | re.M):
        name, body = m.group(1), m.group(2)
        if not flt.search(name):
            continue
        lines = [ln.strip() for ln in body.split("\n")]
        lines = [ln for ln in lines if ln and not ln.startswith(";") and not (ln.startswith(".") and not ln.endswith(":"))]
        labels = {ln[:-1]: i for i, ln in enumerate(lines) if ln.endswith(":")}
        loops = []
        for i, ln in enumerate(lines):
            mm = re.match(r"s_cbranch_\w+\s+(\.LBB\S+)", ln) or re.match(r"s_branch\s+(\.LBB\S+)", ln)
            if mm and mm.group(1) in labels and labels[mm.group(1)] < i:
                loops.append((labels[mm.group(1)], i))
        if not loops:
            continue
        # the innermost loop holding MFMAs (the K loop), else the longest loop
        mf = [lp for lp in loops if any("mfma" in ln for ln in lines[lp[0]:lp[1]])]
        a, b = min(mf, key=lambda x: x[1] - x[0]) if mf else max(loops, key=lambda x: x[1] - x[0])
        cnt = {}
        for ln in lines[a:b]:
            op = ln.split()[0]
            k = ("mfma" if "mfma" in op else "ds_read" if op.startswith("ds_read") else "ds_write" if op.startswith("ds_write")
                 else "vmem_ld" if op.startswith(("buffer_load", "global_load")) else "vmem_st" if op.startswith(("buffer_store", "global_store"))
                 else "waitcnt" if op.startswith("s_waitcnt") else "salu" if op.startswith("s_") else "valu" if op.startswith("v_") else "other")
            cnt[k] = cnt.get(k, 0) + 1
        per = cnt.get("valu", 0) / max(1, cnt.get("mfma", 0))
        print("%-90s len %4d valu/mfma %.1f %s" % (name[:90], b - a, per, dict(sorted(cnt.items()))))


if __name__ == "__main__":
    main()
