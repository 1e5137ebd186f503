#!/bin/bash
# same-box A/B of an environment switch on bench.py: 2 x (base, VAR=VAL), 10 steps each.
# Usage: bash tools/env_ab2.sh <name> VAR=VAL [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
name=$1; kv=$2; shift 2
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/${name}_base_$i.log 2>&1 || { tail -5 gpurun_out/${name}_base_$i.log; exit 1; }
  env $kv timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/${name}_flag_$i.log 2>&1 || { tail -5 gpurun_out/${name}_flag_$i.log; exit 1; }
done
for f in gpurun_out/${name}_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
