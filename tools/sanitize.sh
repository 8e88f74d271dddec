#!/bin/bash
# Host-code sanitizer runs (GPU sanitizers are not available on this pool):
#   ASan + UBSan  GBDT engine (CPU backend), VW learner core and image kernels, each with its native host test
#   TSan          GBDT engine with 4 OpenMP threads plus 4 std::threads pushing / predicting concurrently;
#                 built with clang + LLVM libomp and the Archer OMPT tool, which makes OpenMP's barriers and
#                 locks visible to TSan (so no OMP_NUM_THREADS=1 crutch and no race suppressions)
# SKIP_TSAN=1 runs the ASan/UBSan part only; ONLY=gbdt|vw|image|tsan runs one part.
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/build/sanitize"
mkdir -p "$OUT"
ONLY="${ONLY:-all}"
GB=""
for f in config.cpp dataset.cpp tree.cpp objective.cpp backend_cpu.cpp booster.cpp; do GB="$GB $ROOT/csrc/gbdt/$f"; done
GB="$GB $ROOT/tests/native/gpu_stub.cpp $ROOT/tests/native/gbdt_host_test.cpp"
COMMON="-std=c++17 -O1 -g -fno-omit-frame-pointer"
ASAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined"
export ASAN_OPTIONS=detect_leaks=1:abort_on_error=1:strict_string_checks=1:detect_stack_use_after_return=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
if [ "$ONLY" = all ] || [ "$ONLY" = gbdt ]; then
  g++ $COMMON $ASAN -fopenmp -I"$ROOT/csrc/gbdt" $GB -o "$OUT/gbdt_asan"
  OMP_NUM_THREADS=4 "$OUT/gbdt_asan"
fi
if [ "$ONLY" = all ] || [ "$ONLY" = vw ]; then
  g++ $COMMON $ASAN -I"$ROOT/csrc/vw" "$ROOT/csrc/vw/vw_core.cpp" "$ROOT/tests/native/vw_host_test.cpp" -o "$OUT/vw_asan"
  "$OUT/vw_asan"
fi
if [ "$ONLY" = all ] || [ "$ONLY" = image ]; then
  g++ $COMMON $ASAN -fopenmp -I"$ROOT/csrc/image" "$ROOT/csrc/image/image_ops.cpp" \
    "$ROOT/csrc/image/jpeg_decode.cpp" "$ROOT/tests/native/image_host_test.cpp" -o "$OUT/image_asan"
  OMP_NUM_THREADS=4 "$OUT/image_asan"
fi
if [ "${SKIP_TSAN:-0}" != "1" ] && { [ "$ONLY" = all ] || [ "$ONLY" = tsan ]; }; then
  LLVM=/opt/rocm/llvm
  "$LLVM/bin/clang++" $COMMON -fsanitize=thread -fopenmp -I"$ROOT/csrc/gbdt" $GB -o "$OUT/gbdt_tsan" \
    -Wl,-rpath,"$LLVM/lib"
  OMP_NUM_THREADS=4 OMP_TOOL_LIBRARIES="$LLVM/lib/libarcher.so" TSAN_OPTIONS="halt_on_error=1:exitcode=66:ignore_noninstrumented_modules=1" \
    "$OUT/gbdt_tsan"
fi
echo "sanitizers clean"
