"""Summarise rocprofv3 --pmc CSV passes: mean counter value per kernel (selected kernels) across passes."""
import csv
import glob
import re
import sys
from collections import defaultdict


def main(root, pattern="tl_|seg_|segdot", out=None):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"]
                if not re.search(pattern, name):
                    continue
                short = re.sub(r"\(.*", "", name).replace("void ", "")
                acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    lines = []
    for k in sorted(acc):
        lines.append(f"## {k}")
        for c in sorted(acc[k]):
            v = acc[k][c]
            lines.append(f"  {c:45s} mean {sum(v) / len(v):16.1f}  (n={len(v)})")
    text = "\n".join(lines)
    print(text)
    if out:
        open(out, "w").write(text + "\n")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3] or []), out=sys.argv[3] if len(sys.argv) > 3 else None)
