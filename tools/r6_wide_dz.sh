#!/bin/bash
# round 6: the dGELU product (dZ) on the wide tile -- with / without the bias-gradient column sums
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for v in 1 2 1 2; do echo "== wide=$v"; MMU_GEMM_WIDE=$v timeout -k 10 200 python -u tools/gemm_bench.py --no-ref --cases "bwd dZ   B=W2,fwd ffn1 gelu" 2>&1 | grep -v amdgpu.ids || exit 1; done > gpurun_out/r6w_dz.txt 2>&1
cat gpurun_out/r6w_dz.txt
