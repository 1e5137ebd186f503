#!/bin/bash
# round 6 final tree: the N = 2 bench path on one GPU (gloo, both ranks on cuda:0) -- the launcher,
# the DP hooks and the JSON line the driver's SCALE run reads
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
MMU_BENCH_BACKEND=gloo MMU_BENCH_ONE_DEVICE=1 timeout -k 10 600 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r6_n2_rehearsal.log 2>&1 || { tail -20 gpurun_out/r6_n2_rehearsal.log; exit 1; }
tail -1 gpurun_out/r6_n2_rehearsal.log | cut -c1-400
