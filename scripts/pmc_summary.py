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
    # mean dispatch duration from the kernel traces of the same runs (effective clock = GRBM_GUI_ACTIVE / 8 / time)
    for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", "")
                if not re.search(pattern, name) or "Start_Timestamp" not in r:
                    continue
                short = re.sub(r"\(.*", "", name).replace("void ", "")
                acc[short]["duration_us"].append((float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3)
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
