#!/bin/bash
# round 6 final: the driver-style bench line, then a rocprofv3 --stats pass of the same command
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --steps 20 --warmup 3 > gpurun_out/r6_bench_final.log 2>&1 || { tail -5 gpurun_out/r6_bench_final.log; exit 1; }
tail -1 gpurun_out/r6_bench_final.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6_stats -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6_stats.log 2>&1 || { tail -5 gpurun_out/r6_stats.log; exit 1; }
tail -1 gpurun_out/r6_stats.log
rm -f gpurun_out/r6_stats/run_kernel_trace.csv
ls gpurun_out/r6_stats
