#!/bin/bash
# Same-box A/B of a library environment switch (e.g. MMU_GEMM_SK): bench.py alternating
# VAR=0 / VAR=1, 2 x 2 runs of 10 steps (BENCH_ARGS passed through), each run under its own limit.
#   tools/env_ab.sh <name> <VAR>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
name=$1; var=$2
mkdir -p gpurun_out
for i in 1 2; do
  for v in 0 1; do
    env "$var=$v" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $BENCH_ARGS \
      > gpurun_out/${name}_${var}${v}_$i.log 2>&1 || exit 1
  done
done
for f in gpurun_out/${name}_${var}*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
