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
    rn = next(x for x in ("name", "message") if x in rc)
    probe = list(c.execute(f"select * from {rv} limit 500"))
    for i, x in enumerate(rc):
        vals = {r[i] for r in probe if isinstance(r[i], str)}
        if len(vals) > 1 and any(" " in v for v in vals):
            rn = x
            break
    regs = list(c.execute(f"select {rn}, start, end from {rv} order by start"))
    sel = [r for r in regs if sub in (r[0] or "")]
    if not sel:
        print("no region", sub)
        return
    name, t0, t1 = sel[int(index)]
    # every region row in the window whose name is not a roctx message is an API call
    api = defaultdict(lambda: [0, 0, 0])
    for n, s, e in regs:
        if s >= t0 and e <= t1 and n and not n.startswith("{"):
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
