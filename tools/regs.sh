#!/bin/bash
# Register / spill / occupancy table of every kernel in one HIP source (device-only compile).
# usage: tools/regs.sh ds-gan_amd/csrc/<file>.hip [grep-filter]
src=$1; flt=${2:-.}
# the per-file flags of ds-gan_amd/build_lib.py (EXTRA)
case "$(basename "$src")" in dwconv.hip|mlp.hip|thin3.hip) set -- "$1" "$flt" "$3 -fno-slp-vectorize";; esac
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I"$(dirname "$src")" --cuda-device-only -c "$src" \
  -o /tmp/regs_$$.o -Rpass-analysis=kernel-resource-usage $3 2>&1 |
python3 -c '
import re, sys, subprocess
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m: continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}; rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1); cur[k.strip()] = v.strip()
names = subprocess.run(["c++filt"] + [r["name"] for r in rows], capture_output=True, text=True).stdout.split("\n")
for r, n in zip(rows, names):
    if re.search(sys.argv[1], n):
        print("V%-4s A%-4s spill%-4s scr%-5s LDS%-6s occ%s  %s" % (r.get("VGPRs"), r.get("AGPRs"), r.get("VGPRs Spill"), r.get("ScratchSize [bytes/lane]"), r.get("LDS Size [bytes/block]"), r.get("Occupancy [waves/SIMD]"), n[:110]))
' "$flt"
rm -f /tmp/regs_$$.o
