#!/bin/bash
# round 6: split-K reduce + table in one pass, batched colsum reductions: tests, then tree A/Bs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6k
timeout -k 10 600 python -u -m pytest tests/test_resnet_gpu.py tests/test_kernels_gpu.py tests/test_mmbt_gpu.py -m gpu -q \
  --timeout 300 --timeout-method thread -k "colsum or bnb or stats or parts or embed or small_t16 or full_t508c-full-bf16 or model_grads or bottleneck or dbias or layer_backward or encoder" \
  > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" ${o}_tests.log | head -20; tail -5 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/tree_ab.sh r6k_ab32 --global-batch 32 || exit 1
bash tools/tree_ab.sh r6k_ab || exit 1
bash tools/env_ab2.sh r6k_route3 MMU_ROUTE_FUSED=3 || exit 1
bash tools/env_ab2.sh r6k_route3_32 MMU_ROUTE_FUSED=3 --global-batch 32 || exit 1
echo done
