#!/bin/bash
# round 6: the identity block's skip gradient read through bn3's mask in conv1's dX epilogue
# (res_mask) -- tests, then a same-box A/B of MMU_SKIP_MASKED (0 = the materialised dSkip)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6m
timeout -k 10 600 python -u -m pytest tests/test_resnet_gpu.py tests/test_mmbt_gpu.py tests/test_dp_gpu.py -m gpu -q \
  --timeout 300 --timeout-method thread -k "gated or bnb or resnet or small_t16 or full_t508c-full-bf16 or model_grads or bottleneck or sync" \
  > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" ${o}_tests.log | head -20; tail -5 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/env_ab2.sh r6m_ab MMU_SKIP_MASKED=0 || exit 1
bash tools/env_ab2.sh r6m_ab32 MMU_SKIP_MASKED=0 --global-batch 32 || exit 1
echo done
