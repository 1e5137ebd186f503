# kernel traces of one bench step, ab/base_tree vs working tree, at per-rank batch 256 and 32
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
root=$(pwd)
for b in 256 32; do
  for t in base new; do
    dir=$root; [ $t = base ] && dir=$root/ab/base_tree
    rm -rf $root/gpurun_out/prof_${t}_$b
    (cd $dir && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $root/gpurun_out/prof_${t}_$b -o run -- python3 bench.py --global-batch $b --steps 3 --warmup 2 --no-cpu-baseline) > gpurun_out/prof_${t}_$b.log 2>&1 || { tail -5 gpurun_out/prof_${t}_$b.log; exit 1; }
    python3 tools/prof_summary.py gpurun_out/prof_${t}_$b/run_kernel_trace.csv > gpurun_out/prof_${t}_$b.md 2>&1
    echo "$t B=$b"; head -8 gpurun_out/prof_${t}_$b.md | tail -6
  done
done
