#!/bin/bash
# round 6: the split-K workspace caps the weight gradients' slice count (W1: 64 MiB -> 7 slices of
# 18.8 K tokens: ~300-us workgroups that hold every CU the trunk backward's chain kernels wait for);
# step A/B with 256 MiB / 1 GiB workspaces (more, shorter slices)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 64 256 1024; do echo "== ws_mb=$v"; MMU_SPLITK_WS_MB=$v timeout -k 10 200 python -u tools/gemm_bench.py --no-ref --cases "wgrad" 2>&1 | grep -v amdgpu.ids || exit 1; done > gpurun_out/r6skw.txt 2>&1
cat gpurun_out/r6skw.txt
bash tools/env_ab2.sh r6skw_ab256 MMU_SPLITK_WS_MB=256 || exit 1
bash tools/env_ab2.sh r6skw_ab1g MMU_SPLITK_WS_MB=1024 || exit 1
