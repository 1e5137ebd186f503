#!/bin/bash
# round 6: the 256x384 tile at batch 32 too (MMU_GEMM_WIDE_MIN_TILES=256: FFN1 520 wide tiles + split
# tail, QKV 390) -- product A/B at M = 16416, then the batch-32 step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1024 256 1024 256; do echo "== wide_min=$v"; MMU_GEMM_WIDE_MIN_TILES=$v timeout -k 10 200 python -u tools/gemm_bench.py --no-ref --rows 16416 --cases "fwd qkv,fwd ffn1 gelu" 2>&1 | grep -v amdgpu.ids || exit 1; done > gpurun_out/r6w32.txt 2>&1
cat gpurun_out/r6w32.txt
bash tools/env_ab2.sh r6w32_ab MMU_GEMM_WIDE_MIN_TILES=256 --global-batch 32 || exit 1
