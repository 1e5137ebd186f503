#!/bin/bash
# round 6: parity with the late flush as the default (MMU_WGRAD_INTERLEAVE=2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_mmbt_gpu.py tests/test_graph_gpu.py tests/test_dp_gpu.py tests/test_dp_full_gpu.py tests/test_uncertainty_gpu.py tests/test_robustness_gpu.py -m gpu -q \
  --timeout 300 --timeout-method thread > gpurun_out/r6fl_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r6fl_tests.log | head -20; tail -5 gpurun_out/r6fl_tests.log; exit 1; }
tail -1 gpurun_out/r6fl_tests.log
