#!/bin/bash
# BERT weight gradients deferred to the end of the encoder backward (side stream, beside the trunk's
# backward): encoder / DP tests, then bench A/B vs ab/base_tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mmbt_gpu.py tests/test_dp_gpu.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/t_defer.log 2>&1 && tail -1 gpurun_out/t_defer.log &&
bash tools/gpu_b32_ab.sh && tail -1 gpurun_out/ab_new_256.log | cut -c 1-2000
