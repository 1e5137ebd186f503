# same-box A/B of the uncertainty workload: ab/r2_tree (round-2 final), ab/base_tree (HEAD), working tree; twice
set -o pipefail
mkdir -p gpurun_out
root=$(pwd)
for rep in 1 2; do
  for t in r2 base new; do
    dir=$root; [ $t != new ] && dir=$root/ab/${t}_tree
    (cd $dir && timeout -k 10 300 python3 bench.py --workload uncertainty --steps 3 --warmup 1 --no-cpu-baseline) > gpurun_out/uab_${t}_$rep.log 2>&1 || { tail -5 gpurun_out/uab_${t}_$rep.log; exit 1; }
    echo "$t rep $rep $(tail -1 gpurun_out/uab_${t}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["fused_block_roofline"]["ms_per_layer"])')"
  done
done
