#!/bin/bash
# round 6: the split-K tabulating reduce at 64 x 64 blocks -- tests, then tree A/Bs at batch 32 / 256
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6l
timeout -k 10 600 python -u -m pytest tests/test_resnet_gpu.py tests/test_kernels_gpu.py -m gpu -q \
  --timeout 300 --timeout-method thread -k "colsum or bnb or stats or parts" \
  > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" ${o}_tests.log | head -20; tail -5 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/tree_ab.sh r6l_ab32 --global-batch 32 || exit 1
bash tools/tree_ab.sh r6l_ab || exit 1
echo done
