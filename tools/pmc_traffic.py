"""HBM traffic per launch, per kernel family, from two rocprofv3 --pmc passes over the same
bench command (FETCH_SIZE in one, WRITE_SIZE in the other; MI355X_MICROARCH.md § HBM: the two
cannot share a pass, and on gfx950 FETCH_SIZE counts half the bytes of 16-byte-per-lane
streaming reads, so it is doubled here; both counters are in KiB).
usage: pmc_traffic.py FETCH_DB WRITE_DB OUT_JSON"""
import json, re, sqlite3, sys, collections


def fam(name):
    m = re.search(r"dsg::(\w+?_kernel|\w+)(<|\()", name)
    if m:
        return m.group(1)
    # names c++filt leaves mangled (16-bit float template arguments, DF16b / DF16_)
    m = re.match(r"_ZN3dsg(\d+)", name)
    return name[m.end():m.end() + int(m.group(1))] if m else None


def per_family(db, counter):
    c = sqlite3.connect(db)
    acc = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for name, v, d in c.execute("select kernel_name, value, duration from counters_collection where counter_name=?",
                                (counter,)):
        f = fam(name)
        if f is None:
            continue
        a = acc[f]; a[0] += 1; a[1] += v; a[2] += d
    return acc


fe, wr = per_family(sys.argv[1], "FETCH_SIZE"), per_family(sys.argv[2], "WRITE_SIZE")
out = {}
for f in sorted(set(fe) & set(wr)):
    n, kb_f, d = fe[f]
    n2, kb_w, _ = wr[f]
    fetch = 2.0 * kb_f * 1024 / n
    write = kb_w * 1024 / n2
    out[f] = {"launches": n, "fetch_bytes_per_launch": round(fetch), "write_bytes_per_launch": round(write),
              "traffic_bytes_per_launch": round(fetch + write), "avg_profiled_us": round(d / n / 1e3, 1)}
json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over `bench.py --steps 3 --warmup 1` "
                     "(FETCH_SIZE x2, gfx950 correction)", "families": out}, open(sys.argv[3], "w"), indent=1)
for f, v in sorted(out.items(), key=lambda kv: -kv[1]["traffic_bytes_per_launch"] * kv[1]["launches"])[:15]:
    print("%-28s %5d launches  %8.1f MB/launch  (%.1f us)" % (f, v["launches"], v["traffic_bytes_per_launch"] / 1e6,
                                                              v["avg_profiled_us"]))
