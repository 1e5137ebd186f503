# BatchNorm 8 K-element block floor: every GPU test on the working tree, smoke(), then
# alternating batch-32 and batch-256 bench A/Bs against ab/base_tree (HEAD); each step timed
set -o pipefail
mkdir -p gpurun_out
root=$(pwd)
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_gpu_bn8k.log 2>&1 || { tail -40 gpurun_out/t_gpu_bn8k.log; exit 1; }
tail -1 gpurun_out/t_gpu_bn8k.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_bn8k.log 2>&1 || { tail -20 gpurun_out/smoke_bn8k.log; exit 1; }
tail -1 gpurun_out/smoke_bn8k.log
for t in base new base new base new; do
  dir=$root; [ $t = base ] && dir=$root/ab/base_tree
  (cd $dir && timeout -k 10 300 python3 bench.py --global-batch 32 --steps 30 --warmup 6 --no-cpu-baseline) > gpurun_out/bn8k_${t}.log 2>&1 || { tail -5 gpurun_out/bn8k_${t}.log; exit 1; }
  echo "$t B=32 $(tail -1 gpurun_out/bn8k_${t}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
timeout -k 10 400 python3 bench.py > gpurun_out/bench_bn8k.log 2>&1 || { tail -5 gpurun_out/bench_bn8k.log; exit 1; }
tail -1 gpurun_out/bench_bn8k.log | cut -c1-300
