#!/bin/bash
# round 6 final tree: the other workloads' bench lines (BASELINE config 3 uncertainty, config 5 FLAVA,
# encoders, ViLT)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in uncertainty flava encoders vilt vilt_train; do
  timeout -k 10 400 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6_bench_$w.log 2>&1 || { echo "$w failed"; tail -5 gpurun_out/r6_bench_$w.log; exit 1; }
  echo "$w $(grep -o '"value": [0-9.]*' gpurun_out/r6_bench_$w.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_bench_$w.log)"
done
