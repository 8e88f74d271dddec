#!/bin/bash
# Round-5 pass 54: VW estimator fit timeline (kernels + host-to-device copies) for one fit after warm-up.
OUT=${1:-gpurun_out/r5p54}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/prof" -o vw -- python3 tools/bench_vw.py --steps 1 --warmup 1 > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 1; }
k=$(find "$OUT/prof" -name '*kernel_trace.csv' -print -quit)
m=$(find "$OUT/prof" -name '*memory_copy_trace.csv' -print -quit)
python3 - "$k" "$m" > "$OUT/timeline.txt" <<'PY'
import csv, sys
ks = list(csv.DictReader(open(sys.argv[1])))
ms = list(csv.DictReader(open(sys.argv[2]))) if sys.argv[2] else []
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:50]) for r in ks]
ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", r.get("Direction", "") + " " + r.get("Size", "")) for r in ms]
ev.sort()
# the last fit: events after the largest gap > 20 ms
starts = [e[0] for e in ev]
cut = 0
for i in range(1, len(ev)):
    if ev[i][0] - ev[i - 1][1] > 20_000_000:
        cut = i
ev = ev[cut:]
t0 = ev[0][0]
tot = {}
for s, e, kind, name in ev:
    key = (kind, name.split("(")[0])
    d = tot.setdefault(key, [0, 0.0])
    d[0] += 1
    d[1] += (e - s) / 1e3
span = (max(e for _, e, _, _ in ev) - t0) / 1e3
print(f"last fit span {span:.1f} us, {len(ev)} events")
for (kind, name), (n, us) in sorted(tot.items(), key=lambda x: -x[1][1])[:20]:
    print(f"{kind} {us:10.1f} us {n:6d}  {name}")
# busy union of kernels and of copies
def union(kind):
    iv = sorted((s, e) for s, e, k, _ in ev if k == kind)
    busy, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None: busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None: busy += cur_e - cur_s
    return busy / 1e3
print(f"kernel busy {union('K'):.1f} us, copy busy {union('C'):.1f} us")
# coarse timeline: 2 ms buckets, kernel / copy busy time and the dominant kernel name per bucket
B = 2000_000
nb = int((max(e for _, e, _, _ in ev) - t0) // B) + 1
rows = [[0.0, 0.0, {}] for _ in range(nb)]
for s, e, kind, name in ev:
    b = int((s - t0) // B)
    d = (e - s) / 1e3
    rows[b][0 if kind == "K" else 1] += d
    if kind == "K":
        nm = name.split("(")[0][-40:]
        rows[b][2][nm] = rows[b][2].get(nm, 0.0) + d
for i, (k, c, names) in enumerate(rows):
    top = max(names.items(), key=lambda x: x[1])[0] if names else ""
    print(f"{i * 2:4d} ms  kernels {k:7.0f} us  copies {c:7.0f} us  {top}")
PY
cat "$OUT/timeline.txt"
rm -rf "$OUT/prof"
