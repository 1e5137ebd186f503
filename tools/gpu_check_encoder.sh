#!/bin/bash
# encoder / DP / uncertainty GPU tests after a host-side change
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mmbt_gpu.py tests/test_dp_gpu.py tests/test_uncertainty_gpu.py tests/test_robustness_gpu.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/t_enc.log 2>&1 && tail -1 gpurun_out/t_enc.log
