#!/bin/bash
# round 6: downsample blocks -- conv1's dX epilogue adds the downsample conv's dX (and writes the
# previous bn3's backward reduction): tests, then a same-box step A/B (flag = MMU_DS_SINK=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6ds
timeout -k 10 700 python -u -m pytest tests/test_resnet_gpu.py tests/test_mmbt_gpu.py tests/test_dp_gpu.py tests/test_graph_gpu.py -m gpu -q \
  --timeout 300 --timeout-method thread > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" ${o}_tests.log | head -20; tail -5 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/env_ab2.sh r6ds_ab MMU_DS_SINK=0 || exit 1
bash tools/env_ab2.sh r6ds_ab32 MMU_DS_SINK=0 --global-batch 32 || exit 1
