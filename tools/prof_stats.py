"""Per-kernel summary (rocprofv3 --stats style CSV) from a rocprofv3 results .db.
usage: prof_stats.py RESULTS_DB [OUT_CSV] [--steps K]   (per-step ms column when --steps given)"""
import csv, sqlite3, sys

db = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 0
c = sqlite3.connect(db)
rows = list(c.execute(
    "select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
    "from kernels group by name order by sum(end-start) desc"))
tot = sum(r[2] for r in rows)
hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"]
recs = [[r[0], r[1], r[2], round(r[3], 1), round(100.0 * r[2] / tot, 2), r[4], r[5]] for r in rows]
if out:
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(hdr)
        w.writerows(recs)
for r in recs[:40]:
    extra = "  %.3f ms/step" % (r[2] / 1e6 / steps) if steps else ""
    print("%6.2f%% %9.3f ms %6d  %s%s" % (r[4], r[2] / 1e6, r[1], r[0][:90], extra))
print("total %.3f ms" % (tot / 1e6))
