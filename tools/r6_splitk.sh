#!/bin/bash
# round 6: split-K slice count of the weight gradients -- ~640 workgroups (base) vs one round
# (MMU_SPLITK_ROUND=1); same-box step A/B at batch 32 (graph) and 256, plus the BERT wgrad shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1 0 1; do echo "== round=$v rows=16416"; MMU_SPLITK_ROUND=$v timeout -k 10 200 python -u tools/gemm_bench.py --no-ref --rows 16416 --cases "wgrad" 2>&1 | grep -v amdgpu.ids || exit 1; done > gpurun_out/r6sk_wgrad.txt 2>&1
for v in 0 1; do echo "== round=$v rows=131328"; MMU_SPLITK_ROUND=$v timeout -k 10 200 python -u tools/gemm_bench.py --no-ref --cases "wgrad" 2>&1 | grep -v amdgpu.ids || exit 1; done >> gpurun_out/r6sk_wgrad.txt 2>&1
cat gpurun_out/r6sk_wgrad.txt
bash tools/env_ab2.sh r6sk_ab32 MMU_SPLITK_ROUND=1 --global-batch 32 || exit 1
bash tools/env_ab2.sh r6sk_ab MMU_SPLITK_ROUND=1 || exit 1
