#!/bin/bash
# round 6: batch 32's N = 768 BERT products (M = 16416: 195 tiles of 256^2 for 256 CUs) on 128^2 tiles
# (MMU_GEMM_SMALL_BELOW=256) -- product A/B, then the batch-32 step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CASES="fwd o    drop,fwd ffn2,bwd dA   B=W1,bwd dX   B=Wqkv,bwd dO   B=Wo"
for v in 0 256 0 256; do echo "== small_below=$v"; MMU_GEMM_SMALL_BELOW=$v timeout -k 10 200 python -u tools/gemm_bench.py --no-ref --rows 16416 --cases "$CASES" 2>&1 | grep -v amdgpu.ids || exit 1; done > gpurun_out/r6s32.txt 2>&1
cat gpurun_out/r6s32.txt
bash tools/env_ab2.sh r6s32_ab MMU_GEMM_SMALL_BELOW=256 --global-batch 32 || exit 1
