#!/bin/bash
# round 6: GEMM column sums as partial rows (no float atomics) -- tests, dZ product A/B, step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6cs
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm" > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" ${o}_tests.log | head; tail -20 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
for v in 0 1 0 1; do echo "== cs_part=$v"; MMU_GEMM_CS_PART=$v timeout -k 10 200 python -u tools/gemm_bench.py --no-ref --cases "bwd dZ   B=W2" 2>&1 | grep -v amdgpu.ids || exit 1; done > ${o}_dz.txt 2>&1
cat ${o}_dz.txt
bash tools/env_ab2.sh r6cs_ab MMU_GEMM_CS_PART=0 || exit 1
