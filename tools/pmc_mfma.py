"""Per-kernel-family PMC counters from rocprofv3 --pmc result databases (one DB per pass), with
the derived MFMA utilisation.
usage: pmc_mfma.py OUT_JSON DB [DB ...]

Derived per family (per launch averages; MI355X_MICROARCH.md § rocprofv3 PMC slots and
§ Per-instruction cycle constants):
  * clock_ghz      = GRBM_GUI_ACTIVE / 8 XCDs / duration   (GRBM counts per XCD, summed)
  * mfma_busy      = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the share of
                     all SIMD-cycles of the launch in which the matrix pipe was busy
  * mfma_cyc_per_inst = SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_MFMA (32 for 32x32x16 bf16)
  * issue split    = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
  * lds_conflict   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
"""
import collections
import json
import os
import re
import sqlite3
import sys


def fam(name):
    if os.environ.get("PMC_BY") == "name":   # one row per template instance
        m = re.search(r"dsg::(\w+?_kernel<[^(]*>)", name)
        return m.group(1) if m else (name if name.startswith("_ZN3dsg") else None)
    m = re.search(r"dsg::(\w+?_kernel|\w+)(<|\()", name)
    if m:
        return m.group(1)
    # names c++filt leaves mangled (16-bit float template arguments, DF16b / DF16_)
    m = re.match(r"_ZN3dsg(\d+)", name)
    return name[m.end():m.end() + int(m.group(1))] if m else None


def main():
    out_path, dbs = sys.argv[1], sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0.0, 0.0]))
    for db in dbs:
        c = sqlite3.connect(db)
        for name, cn, v, d in c.execute("select kernel_name, counter_name, value, duration from counters_collection"):
            f = fam(name)
            if f is None:
                continue
            a = acc[f][cn]
            a[0] += 1
            a[1] += v
            a[2] += d
    res = {}
    for f, cs in acc.items():
        r = {}
        for cn, (n, v, d) in cs.items():
            r[cn] = v / n
            r.setdefault("launches", n)
            r.setdefault("dur_us", d / n / 1e3)
        g = r.get("GRBM_GUI_ACTIVE")
        if g:
            cyc = g / 8.0
            r["clock_ghz"] = cyc / (r["dur_us"] * 1e3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in r:
                r["mfma_busy"] = r["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cyc)
        if r.get("SQ_INSTS_MFMA") and r.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            r["mfma_cyc_per_inst"] = r["SQ_VALU_MFMA_BUSY_CYCLES"] / r["SQ_INSTS_MFMA"]
        w = r.get("SQ_WAVE_CYCLES")
        if w:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in r:
                    r[k.lower().replace("sq_", "") + "_frac"] = r[k] / w
        if "SQ_ACTIVE_INST_VALU" in r and g:   # quad-cycles summed over waves -> share of SIMD-cycles
            r["valu_busy"] = 4.0 * r["SQ_ACTIVE_INST_VALU"] / (1024.0 * g / 8.0)
        if "SQ_VALU_MFMA_COEXEC_CYCLES" in r and g:
            r["coexec"] = r["SQ_VALU_MFMA_COEXEC_CYCLES"] / (1024.0 * g / 8.0)
        if r.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_conflict_frac"] = r.get("SQ_LDS_BANK_CONFLICT", 0.0) / r["SQ_LDS_IDX_ACTIVE"]
        res[f] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in sorted(r.items())}
    json.dump({"source": "rocprofv3 --pmc passes over `bench.py --steps 3 --warmup 1` (tools/gpu_mfma_pmc.sh)",
               "families": res}, open(out_path, "w"), indent=1)
    order = sorted(res, key=lambda f: -res[f]["dur_us"] * res[f]["launches"])
    for f in order[:20]:
        r = res[f]
        print("%-26s n=%4d %8.1fus clk=%s mfma_busy=%s cyc/mfma=%s wait=%s inst=%s lds_cf=%s valu=%s coexec=%s" % (
            f, r["launches"], r["dur_us"], r.get("clock_ghz"), r.get("mfma_busy"), r.get("mfma_cyc_per_inst"),
            r.get("wait_any_frac"), r.get("wait_inst_any_frac"), r.get("lds_conflict_frac"), r.get("valu_busy"),
            r.get("coexec")))


if __name__ == "__main__":
    main()
