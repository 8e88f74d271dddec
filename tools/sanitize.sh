#!/bin/bash
# Host-code sanitizer runs of the native GBDT engine: ASan+UBSan and TSan builds of
# tests/native/gbdt_host_test.cpp against the CPU backend. GPU sanitizers are not available on this pool.
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/build/sanitize"
mkdir -p "$OUT"
SRC="config.cpp dataset.cpp tree.cpp objective.cpp backend_cpu.cpp booster.cpp"
FILES=""
for f in $SRC; do FILES="$FILES $ROOT/csrc/gbdt/$f"; done
FILES="$FILES $ROOT/tests/native/gpu_stub.cpp $ROOT/tests/native/gbdt_host_test.cpp"
COMMON="-std=c++17 -O1 -g -fno-omit-frame-pointer -I$ROOT/csrc/gbdt -fopenmp"
g++ $COMMON -fsanitize=address,undefined -fno-sanitize-recover=undefined $FILES -o "$OUT/gbdt_asan"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/gbdt_asan"
if [ "${SKIP_TSAN:-0}" != "1" ]; then
  # OpenMP runtime internals are not TSan-instrumented: single-threaded pass for the engine's own code
  g++ $COMMON -fsanitize=thread $FILES -o "$OUT/gbdt_tsan"
  OMP_NUM_THREADS=1 TSAN_OPTIONS=halt_on_error=1 "$OUT/gbdt_tsan"
fi
echo "sanitizers clean"
