#!/bin/bash
# round 6: the split-K BERT weight gradients on the 256x384 tile -- tests, product A/B, step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6wg
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "wide or splitk or weight_grad" > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" ${o}_tests.log | head; tail -20 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
for v in 0 1 0 1; do echo "== wide_wgrad=$v"; MMU_GEMM_WIDE_WGRAD=$v timeout -k 10 200 python -u tools/gemm_bench.py --no-ref --cases "wgrad" 2>&1 | grep -v amdgpu.ids || exit 1; done > ${o}_times.txt 2>&1
cat ${o}_times.txt
bash tools/env_ab2.sh r6wg_ab MMU_GEMM_WIDE_WGRAD=0 || exit 1
