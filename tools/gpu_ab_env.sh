#!/bin/bash
# Same-box A/B of engine env knobs on the headline bench: tools/gpu_ab_env.sh OUT "VAR=a VAR2=b" "VAR=c" ...
# One bench.py run per setting (plus a repeat of the first), each under its own time limit.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
out="gpurun_out/$1"; shift
mkdir -p "$out"
export PYTHONUNBUFFERED=1
i=0
for setting in "$@" "$1"; do
  i=$((i + 1))
  echo "== $i: $setting" | tee -a "$out/summary.txt"
  env $setting timeout -k 10 240 python bench.py --steps 5 --warmup 2 > "$out/run_$i.log" 2>&1 || exit $?
  python - "$out/run_$i.log" >> "$out/summary.txt" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line); c = d["config"]
        print("  ms_per_fit %.2f  iteration_ms %.3f  phases %s" % (d["ms_per_step"], c["iteration_ms"], c["fit_phases_ms"]))
PY
  tail -1 "$out/summary.txt"
done
