#!/bin/bash
# round 6: A/B of s_setprio 1 for waves 4-7 of the 8-wave GEMM tiles, and of the dZ group height
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CASES="fwd qkv,fwd ffn1 gelu,fwd ffn2,fwd o    drop,bwd dZ   B=W2,bwd dA   B=W1,bwd dX   B=Wqkv,wgrad W1"
for v in 0 1 0 1; do echo "== prio=$v"; MMU_GEMM_PRIO=$v timeout -k 10 200 python -u tools/gemm_bench.py --no-ref --cases "$CASES" 2>&1 | grep -v amdgpu.ids || exit 1; done > gpurun_out/r6prio.txt 2>&1
for g in 1 2 4 8 2 4; do echo "== dz_group=$g"; MMU_GEMM_DZ_GROUP=$g timeout -k 10 200 python -u tools/gemm_bench.py --no-ref --cases "bwd dZ   B=W2^T kmaj," 2>&1 | grep -v amdgpu.ids || exit 1; done >> gpurun_out/r6prio.txt 2>&1
cat gpurun_out/r6prio.txt
