#!/bin/bash
# batch-32 bench A/B with longer runs (30 steps, four alternations): ab/base_tree vs the working tree
set -o pipefail
mkdir -p gpurun_out
root=$(pwd)
for t in base new base new base new base new; do
  dir=$root; [ $t = base ] && dir=$root/ab/base_tree
  (cd $dir && timeout -k 10 300 python3 bench.py --global-batch 32 --steps 30 --warmup 6 --no-cpu-baseline) > gpurun_out/ab2_${t}.log 2>&1 || { tail -5 gpurun_out/ab2_${t}.log; exit 1; }
  echo "$t B=32 $(tail -1 gpurun_out/ab2_${t}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
