#!/bin/bash
# round 6: a high-priority main stream (bench.py --main-priority high) against the side stream's weight
# gradients -- alternated step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6ps_base_$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --main-priority high > gpurun_out/r6ps_high_$i.log 2>&1 || exit 1
done
for f in gpurun_out/r6ps_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
