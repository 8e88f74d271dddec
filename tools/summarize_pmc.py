"""Per-kernel summary of rocprofv3 --pmc counter_collection CSVs (mean value per dispatch and total)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n.split("::")[-1][:60] if "::" in n else n[:60]


def main(d):
    for path in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        agg = defaultdict(lambda: [0.0, 0])
        with open(path) as f:
            for r in csv.DictReader(f):
                key = (short(r.get("Kernel_Name", "?")), r.get("Counter_Name", "?"))
                agg[key][0] += float(r.get("Counter_Value", 0) or 0)
                agg[key][1] += 1
        print(f"== {os.path.basename(path)}")
        for (k, c), (tot, n) in sorted(agg.items(), key=lambda kv: (-kv[1][0] if 'SIZE' in kv[0][1] else 0, kv[0])):
            print(f"  {k:60s} {c:32s} dispatches={n:6d} mean={tot / max(1, n):16.4f} total={tot:18.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
