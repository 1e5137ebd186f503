#!/bin/bash
# round 6: the encoder's deferred weight-gradient work issued item by item from the trunk's
# BatchNorm backwards (MMU_WGRAD_INTERLEAVE=1) -- parity with it on, then same-box step A/Bs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6il
MMU_WGRAD_INTERLEAVE=1 timeout -k 10 600 python -u -m pytest tests/test_mmbt_gpu.py tests/test_graph_gpu.py tests/test_dp_gpu.py -m gpu -q \
  --timeout 300 --timeout-method thread -k "small or full_t508c-full-bf16 or graph or two_ranks" \
  > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" ${o}_tests.log | head -20; tail -5 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/env_ab2.sh r6il_ab32 MMU_WGRAD_INTERLEAVE=1 --global-batch 32 || exit 1
bash tools/env_ab2.sh r6il_ab MMU_WGRAD_INTERLEAVE=1 || exit 1
