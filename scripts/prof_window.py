"""Kernel busy time inside roctx regions of a rocprofv3 rocpd database (--kernel-trace --marker-trace).

usage: prof_window.py DB REGION_SUBSTRING [OUT]
For the LAST region whose name contains REGION_SUBSTRING: wall span, summed kernel time, kernel count, the top
kernels in the window, and the nested regions' totals (where host time goes between kernels)."""
import re
import sqlite3
import sys
from collections import defaultdict


def cols(c, view):
    return [r[1] for r in c.execute(f"pragma table_info('{view}')")]


def main(db, sub, out=None):
    c = sqlite3.connect(db)
    views = [r[0] for r in c.execute("select name from sqlite_master where type in ('view','table')")]
    lines = []
    kv = next((v for v in ("kernels", "kernel") if v in views), None)
    rv = next((v for v in ("regions", "markers", "region") if v in views), None)
    if kv is None or rv is None:
        print("views:", views)
        for v in views:
            if re.search("kernel|region|marker", v):
                print(v, cols(c, v))
        return
    kc, rc = cols(c, kv), cols(c, rv)
    ks = [x for x in ("start", "start_ns", "begin") if x in kc][0]
    ke = [x for x in ("end", "end_ns", "stop") if x in kc][0]
    kn = [x for x in ("name", "kernel_name", "display_name") if x in kc][0]
    rs = [x for x in ("start", "start_ns", "begin") if x in rc][0]
    re_ = [x for x in ("end", "end_ns", "stop") if x in rc][0]
    rn = [x for x in ("name", "display_name", "message") if x in rc][0]
    # roctx ranges: the message may live in another column (name = "roctxThreadRangeA"); pick the first text
    # column whose values vary
    textcols = [x for x in rc if x not in (rs, re_)]
    probe = list(c.execute(f"select * from {rv} limit 200"))
    for i, x in enumerate(rc):
        vals = {r[i] for r in probe if isinstance(r[i], str)}
        if x in textcols and len(vals) > 1 and any(" " in v for v in vals):
            rn = x
            break
    else:
        print("region columns:", rc)
        for r in probe[:3]:
            print(r)
    # with API tracing the first rows are HIP calls: take the text column that actually holds the region name
    for x in textcols:
        try:
            if c.execute(f"select count(*) from {rv} where {x} like ?", (f"%{sub}%",)).fetchone()[0]:
                rn = x
                break
        except sqlite3.Error:
            continue
    regs = list(c.execute(f"select {rn}, {rs}, {re_} from {rv} order by {rs}"))
    sel = [r for r in regs if sub in (r[0] or "")]
    if not sel:
        print("no region matching", sub, "; names:", sorted({r[0] for r in regs})[:50])
        return
    import os
    name, t0, t1 = sel[int(os.environ.get("PML_WIN_INDEX", "-1"))]     # which matching region (default: the last)
    ks_ = list(c.execute(f"select {kn}, {ks}, {ke} from {kv} where {ks} >= ? and {ke} <= ? order by {ks}", (t0, t1)))
    busy = sum(e - s for _, s, e in ks_)
    lines.append(f"# window `{name}`: wall {(t1 - t0) / 1e6:.3f} ms, kernels {len(ks_)}, kernel time "
                 f"{busy / 1e6:.3f} ms ({100 * busy / max(t1 - t0, 1):.1f} % busy)")
    agg = defaultdict(lambda: [0, 0])
    for n, s, e in ks_:
        k = re.sub(r"\(.*$", "", n)[:90]
        agg[k][0] += 1
        agg[k][1] += e - s
    lines += ["", "| kernel | calls | total ms |", "|---|---:|---:|"]
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        lines.append(f"| `{k}` | {n} | {t / 1e6:.3f} |")
    inner = defaultdict(lambda: [0, 0])
    for n, s, e in regs:
        if s >= t0 and e <= t1 and (s, e) != (t0, t1):
            inner[n][0] += 1
            inner[n][1] += e - s
    lines += ["", "| nested region | count | total ms |", "|---|---:|---:|"]
    for k, (n, t) in sorted(inner.items(), key=lambda kv: -kv[1][1])[:25]:
        lines.append(f"| {k} | {n} | {t / 1e6:.3f} |")
    # idle gaps between kernels (GPU waiting for the host): grouped by the kernel pair around the gap and by the
    # innermost nested region containing the gap
    gaps = defaultdict(lambda: [0, 0])
    greg = defaultdict(lambda: [0, 0])
    nested = sorted(((n, s, e) for n, s, e in regs if s >= t0 and e <= t1 and (s, e) != (t0, t1)),
                    key=lambda r: r[2] - r[1])
    end_prev, name_prev = t0, "<window start>"
    short = lambda n: re.sub(r"<.*$", "", re.sub(r"\(.*$", "", n))[:48]
    for n, s, e in ks_ + [("<window end>", t1, t1)]:
        if s - end_prev > 5000:
            g = s - end_prev
            key = f"{short(name_prev)} -> {short(n)}"
            gaps[key][0] += 1
            gaps[key][1] += g
            mid = (s + end_prev) // 2
            r = next((rn_ for rn_, rs_, re2 in nested if rs_ <= mid <= re2), "(top level)")
            greg[r][0] += 1
            greg[r][1] += g
        if e > end_prev:
            end_prev, name_prev = e, n
    idle = sum(t for _, t in gaps.values())
    lines += ["", f"Idle gaps > 5 us: {sum(c for c, _ in gaps.values())}, {idle / 1e6:.3f} ms", "",
              "| previous kernel -> next kernel | gaps | idle ms |", "|---|---:|---:|"]
    for k, (n, t) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:20]:
        lines.append(f"| `{k}` | {n} | {t / 1e6:.3f} |")
    lines += ["", "| innermost region of the gap | gaps | idle ms |", "|---|---:|---:|"]
    for k, (n, t) in sorted(greg.items(), key=lambda kv: -kv[1][1])[:15]:
        lines.append(f"| {k} | {n} | {t / 1e6:.3f} |")
    # timeline: every kernel of the window in start order (offset from the window start, duration, the queue /
    # stream column when the database has one) -- the critical path of windows with side-stream work
    qcol = next((x for x in ("stream_id", "queue_id", "stream", "queue") if x in kc), None)
    if os.environ.get("PML_WIN_TIMELINE", "1") == "0":
        tl = []
    elif qcol is not None:
        tl = list(c.execute(f"select {kn}, {ks}, {ke}, {qcol} from {kv} where {ks} >= ? and {ke} <= ? order by {ks}",
                            (t0, t1)))
    else:
        tl = [(n, s, e, "-") for n, s, e in ks_]
    lines += ["", f"Timeline ({qcol or 'no queue column'}):", "", "| start ms | dur ms | queue | kernel |",
              "|---:|---:|---|---|"]
    for n, s, e, q in tl:
        lines.append(f"| {(s - t0) / 1e6:.3f} | {(e - s) / 1e6:.3f} | {q} | `{short(n)}` |")
    text = "\n".join(lines)
    print(text)
    if out:
        open(out, "w").write(text + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
