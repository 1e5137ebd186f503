#!/bin/bash
# side-stream filter gradients (batch >= 128): trunk / DP tests, then bench A/B vs ab/base_tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py tests/test_dp_gpu.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/t_side.log 2>&1 && tail -1 gpurun_out/t_side.log &&
bash tools/gpu_b32_ab.sh
