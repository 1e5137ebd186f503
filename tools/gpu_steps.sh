#!/bin/bash
# One GPU call's steps (run from the repo root on the GPU box): each step under its own time
# limit, stopping at the first failure.  Usage: tools/gpu_steps.sh <name> <pytest -k expr> [bench A/B flag]
#   <name>:   output prefix under gpurun_out/
#   pytest:   "-" to skip; else the -k expression over the GPU tests (files in $FILES)
#   A/B flag: a bench.py flag alternated against the default, 2 x 2 runs of 10 steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
name=$1; expr=$2; flag=$3
FILES=${FILES:-tests}
mkdir -p gpurun_out
if [ "$expr" != "-" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread -s $FILES \
    -m gpu -k "$expr" > gpurun_out/${name}_tests.log 2>&1
  rc=$?
  tail -5 gpurun_out/${name}_tests.log
  [ $rc -eq 0 ] || { echo "TESTS rc=$rc"; exit $rc; }
fi
if [ -n "$flag" ]; then
  for i in 1 2; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $BENCH_ARGS > gpurun_out/${name}_ab_base_$i.log 2>&1 || exit 1
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $BENCH_ARGS $flag > gpurun_out/${name}_ab_flag_$i.log 2>&1 || exit 1
  done
  for f in gpurun_out/${name}_ab_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
fi
