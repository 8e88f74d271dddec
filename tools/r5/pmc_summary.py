#!/usr/bin/env python3
"""Per-kernel sums of rocprofv3 PMC counters (counter_collection.csv files under a directory).
usage: pmc_summary.py DIR [kernel-substring ...]"""
import collections
import csv
import glob
import os
import re
import sys


def short(n):
    n = n.replace("void ", "").replace("sml::(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n)


root = sys.argv[1]
keep = sys.argv[2:]
files = sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True))
for f in files:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = short(r.get("Kernel_Name", "?"))
        if keep and not any(s in k for s in keep):
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    print(f"== {os.path.relpath(f, root)}")
    for k, cs in sorted(acc.items(), key=lambda x: -max(x[1].values())):
        nd = max(1, len(disp[k]))
        print(f"  {k}  dispatches={nd}")
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} total {v:16.4g}  per-dispatch {v / nd:14.4g}")
