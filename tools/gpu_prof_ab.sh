#!/bin/bash
# rocprofv3 kernel stats of the bench for the current GBDT extension and the saved baseline (ab_base/).
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
out="$ROOT/gpurun_out/${1:-prof_ab}"
mkdir -p "$out"
so=$(ls "$ROOT"/synapseml_amd/_gbdt.cpython-*.so)
cp "$so" /tmp/new_gbdt.so
cd /tmp && export TMPDIR=/tmp
prof() {
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$1" -o bench \
    -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 > "$out/$1_stdout.log" 2>&1 || exit $?
  echo "$1 rc=0"
}
prof new
cp "$ROOT"/ab_base/_gbdt.cpython-*.so "$so"
prof base
cp /tmp/new_gbdt.so "$so"
cd "$ROOT" && bash tools/gpu_ab_env.sh ab_minrows_rot "SML_HIST_MIN_ROWS=1024" "SML_HIST_MIN_ROWS=2048" "SML_HIST_MIN_ROWS=4096"
