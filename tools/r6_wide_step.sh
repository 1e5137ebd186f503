#!/bin/bash
# round 6: 256x384 tiling + split tail in the full step -- model tests, then a same-box step A/B
# (flag run = MMU_GEMM_WIDE=0, the round-5 tiling)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6ws
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_mmbt_gpu.py tests/test_uncertainty_gpu.py -m gpu -q \
  --timeout 300 --timeout-method thread -k "gemm or full_t508c-full-bf16 or small or member" \
  > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" ${o}_tests.log | head -20; tail -5 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/env_ab2.sh r6ws_ab MMU_GEMM_WIDE=0 || exit 1
echo done
