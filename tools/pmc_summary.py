"""Per-kernel PMC counter averages from rocprofv3 --pmc result databases.
usage: pmc_summary.py DB [DB ...] [--filter substr]"""
import re, sqlite3, sys, collections
args = [a for a in sys.argv[1:] if not a.startswith("--")]
flt = sys.argv[sys.argv.index("--filter") + 1] if "--filter" in sys.argv else "dsg::"
out = collections.defaultdict(dict)
for db in args:
    if db == flt:
        continue
    c = sqlite3.connect(db)
    for name, cn, v, d, n in c.execute("select kernel_name, counter_name, avg(value), avg(duration), count(*) "
                                        "from counters_collection group by kernel_name, counter_name"):
        if flt not in name:
            continue
        short = re.sub(r"\(.*", "", name).replace("void ", "")[:70]
        out[short][cn] = v
        out[short]["dur_us"] = d / 1e3
for k, d in out.items():
    print(k)
    for cn in sorted(d):
        print("   %-28s %16.1f" % (cn, d[cn]))
