#!/bin/bash
# Round-6 pass 44: the strip stem's bf16x6 (3-plane) fp32 form and the other stem tests.
OUT=${1:-gpurun_out/r6p44}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_conv_mfma.py -m gpu -x -q -k "stem" --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" "$OUT/pytest.log" | head -30; exit $rc; }
exit 0
