#!/bin/bash
# trunk filter gradients on the side stream at batch 32 too (SIDE_WGRAD_MIN_BATCH 32 vs 128 in ab/base_tree)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/host_time.py --batch 32 > gpurun_out/host32_new.log 2>&1 && echo new && cat gpurun_out/host32_new.log &&
bash tools/gpu_b32_ab2.sh
