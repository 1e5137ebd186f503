#!/bin/bash
# round 6: HIP-graph replay of the batch-256 step (bench.py --graph on) against eager launches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --graph off > gpurun_out/r6g256_eager_$i.log 2>&1 || exit 1
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --graph on > gpurun_out/r6g256_graph_$i.log 2>&1 || exit 1
done
for f in gpurun_out/r6g256_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
