"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite) into a markdown table of the top kernels."""
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name) if not name.startswith("void at::") else name
    m = re.match(r"void ([\w:]+)(<[^(]*?>)?", name)
    base = m.group(1) if m else name[:80]
    tmpl = (m.group(2) or "") if m else ""
    if base.startswith(("seg_", "reduce_", "re_", "tl_")):
        return base + tmpl
    return base + ("<…>" if tmpl else "")


def main(db, out, title, top=20):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    agg = {}
    for name, calls, tot, avg, pct in rows:
        k = short(name)
        a = agg.setdefault(k, [0, 0.0, 0.0])
        a[0] += calls
        a[1] += tot
        a[2] += pct
    lines = [f"# {title}", "", "Durations from the rocpd `top_kernels` view (microseconds).", "", "| kernel | calls | total ms | avg us | % GPU time |", "|---|---:|---:|---:|---:|"]
    for k, (calls, tot, pct) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        lines.append(f"| `{k}` | {calls} | {tot / 1e3:.2f} | {tot / calls:.1f} | {pct:.1f} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "rocprofv3 kernel summary",
         int(sys.argv[4]) if len(sys.argv) > 4 else 20)
