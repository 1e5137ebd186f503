#!/bin/bash
# round 6: the trunk's BatchNorm-reduction data gradients -- 256^2 tiles (base) vs 128^2 tiles for K <= 256 / 512
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for v in none 256 512 none 256 512; do echo "== smallk=$v"; if [ $v = none ]; then timeout -k 10 200 python -u tools/bnb_bench.py; else MMU_GEMM_SMALLK_BNB=$v timeout -k 10 200 python -u tools/bnb_bench.py; fi 2>&1 | grep -v amdgpu.ids || exit 1; done > gpurun_out/r6bnb.txt 2>&1
cat gpurun_out/r6bnb.txt
