# GEMM last-tile-row skip (waves whose rows lie past M skip MFMAs and their A DMA): every GPU
# test on the working tree, then same-box alternating bench A/Bs against ab/base_tree (HEAD)
# at per-rank batch 32 and 256; each step under its own time limit
set -o pipefail
mkdir -p gpurun_out
root=$(pwd)
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_gpu_tail.log 2>&1 || { tail -40 gpurun_out/t_gpu_tail.log; exit 1; }
tail -1 gpurun_out/t_gpu_tail.log
for t in base new base new base new; do
  dir=$root; [ $t = base ] && dir=$root/ab/base_tree
  (cd $dir && timeout -k 10 300 python3 bench.py --global-batch 32 --steps 30 --warmup 6 --no-cpu-baseline) > gpurun_out/tail_${t}.log 2>&1 || { tail -5 gpurun_out/tail_${t}.log; exit 1; }
  echo "$t B=32 $(tail -1 gpurun_out/tail_${t}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
for t in base new base new; do
  dir=$root; [ $t = base ] && dir=$root/ab/base_tree
  (cd $dir && timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline) > gpurun_out/tail256_${t}.log 2>&1 || { tail -5 gpurun_out/tail256_${t}.log; exit 1; }
  echo "$t B=256 $(tail -1 gpurun_out/tail256_${t}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["avg_launch_ms"])')"
done
