#!/bin/bash
# same-box A/B of the working tree against ab/base_tree (tools/ab_tree.sh): 2 x (base, new) bench
# runs of 10 steps.  Usage: bash tools/tree_ab.sh <name> [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
name=$1; shift
root=$(pwd)
mkdir -p gpurun_out
for i in 1 2; do
  (cd ab/base_tree && timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@") > gpurun_out/${name}_base_$i.log 2>&1 || { tail -5 gpurun_out/${name}_base_$i.log; exit 1; }
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/${name}_new_$i.log 2>&1 || { tail -5 gpurun_out/${name}_new_$i.log; exit 1; }
done
for f in gpurun_out/${name}_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
