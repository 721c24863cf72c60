"""Per-dispatch rows of the last step from a rocprofv3 results .db (every column of the kernels
table, in launch order) -- which launch of a kernel family is slow, with its grid.
usage: prof_dispatch.py RESULTS_DB OUT_CSV [--last N]"""
import csv
import sqlite3
import sys

db, out = sys.argv[1], sys.argv[2]
last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 800
c = sqlite3.connect(db)
cur = c.execute("select * from kernels order by start")
cols = [d[0] for d in cur.description]
rows = cur.fetchall()[-last:]
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(cols + ["dur_us"])
    si, ei = cols.index("start"), cols.index("end")
    for r in rows:
        w.writerow(list(r) + [round((r[ei] - r[si]) / 1e3, 2)])
print("columns:", ",".join(cols))
