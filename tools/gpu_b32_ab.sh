# bench A/B at per-rank batch 32 (three alternations) and 256 (two): ab/base_tree (a full HEAD snapshot,
# tools/ab_tree.sh) vs the working tree; then the ResNet GPU tests on the working tree
set -o pipefail
mkdir -p gpurun_out
root=$(pwd)
for b in 32 256; do
  reps="base new base new base new"; [ $b = 256 ] && reps="base new base new"
  for t in $reps; do
    dir=$root; [ $t = base ] && dir=$root/ab/base_tree
    (cd $dir && timeout -k 10 300 python3 bench.py --global-batch $b --steps 10 --warmup 4 --no-cpu-baseline) > gpurun_out/ab_${t}_$b.log 2>&1 || { tail -5 gpurun_out/ab_${t}_$b.log; exit 1; }
    echo "$t B=$b $(tail -1 gpurun_out/ab_${t}_$b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done


