#!/bin/bash
# round 6: the encoder hands the pooler only the [CLS] rows -- parity tests, then a same-box step
# A/B (flag = MMU_CLS_ONLY=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6cls
timeout -k 10 800 python -u -m pytest tests/test_mmbt_gpu.py tests/test_graph_gpu.py tests/test_robustness_gpu.py tests/test_uncertainty_gpu.py tests/test_dp_gpu.py tests/test_native_abi.py -m gpu -q \
  --timeout 300 --timeout-method thread > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" ${o}_tests.log | head -20; tail -5 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/env_ab2.sh r6cls_ab MMU_CLS_ONLY=0 || exit 1
