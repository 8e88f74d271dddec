#!/bin/bash
# Round-6 pass 41: the full check on the final kernels (GPU suite in one process, smoke, headline bench), then
# the conv-form env A/B (pass40).
bash tools/r6/full_gpu.sh gpurun_out/r6p41 || exit 1
bash tools/r6/pass40.sh gpurun_out/r6p41/ab
