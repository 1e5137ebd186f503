#!/bin/bash
# round 6: batch-32 graph step with the interleaved BERT weight gradients, also with the trunk's
# filter gradients on the side stream (MMU_SIDE_WGRAD_MIN_BATCH=1); kernel trace of the latter
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export MMU_WGRAD_INTERLEAVE=1
bash tools/env_ab2.sh r6il2_ab32 MMU_SIDE_WGRAD_MIN_BATCH=1 --global-batch 32 || exit 1
MMU_SIDE_WGRAD_MIN_BATCH=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6il2_prof32 -o run -- python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --global-batch 32 > gpurun_out/r6il2_prof32.log 2>&1 || { tail -5 gpurun_out/r6il2_prof32.log; exit 1; }
echo done
