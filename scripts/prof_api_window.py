"""HIP runtime API time inside a roctx region of a rocprofv3 database (--hip-runtime-trace --marker-trace):
which API calls the host spends the region's idle time in (code-object loads, allocations, synchronising copies).

usage: prof_api_window.py DB REGION_SUBSTRING [INDEX]   (INDEX: which matching region, default 0 = the first)"""
import re
import sqlite3
import sys
from collections import defaultdict


def main(db, sub, index="0"):
    c = sqlite3.connect(db)
    views = [r[0] for r in c.execute("select name from sqlite_master where type in ('view','table')")]
    cols = lambda v: [r[1] for r in c.execute(f"pragma table_info('{v}')")]
    rv = next(v for v in ("regions", "markers", "region") if v in views)
    av = next((v for v in ("regions_and_samples", "hip_api", "api") if v in views), None)
    rc = cols(rv)
    textcols = [x for x in rc if x not in ("start", "end")]
    # the roctx message column: the text column whose values contain the region substring
    msg = None
    for x in textcols:
        try:
            if c.execute(f"select count(*) from {rv} where {x} like ?", (f"%{sub}%",)).fetchone()[0]:
                msg = x
                break
        except sqlite3.Error:
            continue
    if msg is None:
        print("no region", sub, "; region columns:", rc)
        print(list(c.execute(f"select * from {rv} limit 5")))
        return
    api_name = "name" if "name" in rc else msg
    sel = list(c.execute(f"select {msg}, start, end from {rv} where {msg} like ? order by start", (f"%{sub}%",)))
    regs = list(c.execute(f"select {api_name}, start, end from {rv} order by start"))
    name, t0, t1 = sel[int(index)]
    # every region row in the window whose name is not a roctx message is an API call
    api = defaultdict(lambda: [0, 0, 0])
    for n, s, e in regs:
        if s >= t0 and e <= t1 and n and not n.startswith("{") and not n.startswith("roctx"):
            k = re.sub(r"\(.*$", "", n)[:60]
            api[k][0] += 1
            api[k][1] += e - s
            api[k][2] = max(api[k][2], e - s)
    print(f"# HIP API inside `{name}` ({(t1 - t0) / 1e6:.1f} ms)\n")
    print("| API | calls | total ms | max ms |\n|---|---:|---:|---:|")
    for k, (n, t, m) in sorted(api.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"| `{k}` | {n} | {t / 1e6:.3f} | {m / 1e6:.3f} |")


if __name__ == "__main__":
    main(*sys.argv[1:])
