#!/bin/bash
# Same-box A/B of the GBDT extension against a saved baseline build (ab_base/_gbdt*.so, not tracked):
# GBDT GPU tests on the new build, then bench new / base / new. Each GPU step has its own time limit.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
out="gpurun_out/${1:-ab_so}"
mkdir -p "$out"
export PYTHONUNBUFFERED=1
so=$(ls synapseml_amd/_gbdt.cpython-*.so)
cp "$so" /tmp/new_gbdt.so
timeout -k 10 400 python -u -m pytest tests/test_gbdt_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/pytest_gbdt_gpu.log" 2>&1 || { tail -30 "$out/pytest_gbdt_gpu.log"; exit 1; }
tail -2 "$out/pytest_gbdt_gpu.log"
run() {
  timeout -k 10 240 python bench.py --steps 5 --warmup 2 > "$out/bench_$1.log" 2>&1 || exit $?
  python - "$out/bench_$1.log" "$1" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line); c = d["config"]
        print("%-6s ms_per_fit %.2f  iteration_ms %.3f  %s" % (sys.argv[2], d["ms_per_step"], c["iteration_ms"], c["fit_phases_ms"]))
PY
}
run new1
cp ab_base/_gbdt.cpython-*.so "$so"
run base
cp /tmp/new_gbdt.so "$so"
run new2
