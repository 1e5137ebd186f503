#!/bin/bash
# round 6: BatchNorm backward reduction from the next conv's data-gradient epilogue
# (STORE_BNB / ADD_RES_BNB / mmu_conv3x3_implicit_bnb): kernel / model tests, then a same-box
# step A/B of MMU_BN_BWD_FUSION (0 = the BatchNorms' own reduction pass), batch 256 and 32
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6g
timeout -k 10 900 python -u -m pytest tests/test_resnet_gpu.py tests/test_mmbt_gpu.py tests/test_dp_gpu.py -m gpu -v -s \
  --timeout 300 --timeout-method thread -k "bnb or stats or parts or resnet or small_t16 or full_t508c-full-bf16 or model_grads or bottleneck or momentum or sync" \
  > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" ${o}_tests.log | head -20; tail -5 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/env_ab2.sh r6g_ab MMU_BN_BWD_FUSION=0 || exit 1
bash tools/env_ab2.sh r6g_ab32 MMU_BN_BWD_FUSION=0 --global-batch 32 || exit 1
echo done
