#!/usr/bin/env python3
"""Per-iteration timeline of a rocprofv3 kernel trace of bench.py.

Splits the dispatch stream at each ``root_init_kernel`` (one per tree), and for the last complete iterations reports the wall span,
the summed kernel busy time, the idle gaps between dispatches and the busy
time / call count per kernel family.

usage: python tools/trace_timeline.py gpurun_out/<dir>/prof/bench_kernel_trace.csv [--iters 3]
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"::([A-Za-z_0-9]+_kernel)", name)
    if m:
        t = re.search(r"_kernel<([^>]*)>", name)
        return m.group(1) + (f"<{t.group(1)}>" if t else "")
    return name.split("(")[0][-60:]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    rows = []
    with open(args.trace) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2].startswith("root_init_kernel")]
    if len(starts) < 2:
        raise SystemExit("need >= 2 root_init_kernel dispatches")
    spans = list(zip(starts[:-1], starts[1:]))[-args.iters:]
    for a, b in spans:
        it = rows[a:b]
        wall = rows[b][0] - it[0][0]
        busy = sum(e - s for s, e, _, _ in it)
        gaps = [it[i + 1][0] - it[i][1] for i in range(len(it) - 1)] + [rows[b][0] - it[-1][1]]
        fam = defaultdict(lambda: [0, 0, 0])
        for s, e, n, blocks in it:
            fam[n][0] += e - s
            fam[n][1] += 1
            fam[n][2] += blocks
        print(f"iteration: wall {wall / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us, "
              f"gaps {sum(gaps) / 1e3:.1f} us over {len(it)} dispatches "
              f"(median gap {sorted(gaps)[len(gaps) // 2] / 1e3:.2f} us)")
        for n, (t, c, bl) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
            print(f"  {n:40s} {t / 1e3:8.1f} us  {c:4d} calls  {t / 1e3 / c:7.2f} us/call  avg grid {bl / c:8.0f}")


if __name__ == "__main__":
    main()
