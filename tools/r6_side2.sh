#!/bin/bash
# round 6: the trunk's filter gradients on a second side stream (MMU_TRUNK_SIDE2=1) instead of behind the
# encoder's weight gradients on the first -- parity subset, then a same-box step A/B at batch 256
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
MMU_TRUNK_SIDE2=1 timeout -k 10 600 python -u -m pytest tests/test_mmbt_gpu.py tests/test_resnet_gpu.py -m gpu -q --timeout 300 --timeout-method thread \
  -k "full_t508c-full-bf16 or bottleneck or resnet" > gpurun_out/r6s2_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r6s2_tests.log | head; tail -3 gpurun_out/r6s2_tests.log; exit 1; }
tail -1 gpurun_out/r6s2_tests.log
bash tools/env_ab2.sh r6s2_ab MMU_TRUNK_SIDE2=1 || exit 1
