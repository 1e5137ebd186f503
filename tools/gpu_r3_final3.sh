# round-3 record on the working tree (HEAD + the batch-32 1x1 filter-gradient routing): every GPU
# test, smoke(), the train-step bench (per-rank batch 256 with the CPU baseline), a batch-32 A/B
# of the routing change against ab/base_tree (HEAD), then a kernel trace of the bench; each step
# under its own time limit
set -o pipefail
mkdir -p gpurun_out
root=$(pwd)
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_gpu_final3.log 2>&1 || { tail -40 gpurun_out/t_gpu_final3.log; exit 1; }
tail -1 gpurun_out/t_gpu_final3.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final3.log 2>&1 || { tail -20 gpurun_out/smoke_final3.log; exit 1; }
tail -1 gpurun_out/smoke_final3.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_final3.log 2>&1 || { tail -5 gpurun_out/bench_final3.log; exit 1; }
tail -1 gpurun_out/bench_final3.log | cut -c1-300
for t in base new base new base new; do
  dir=$root; [ $t = base ] && dir=$root/ab/base_tree
  (cd $dir && timeout -k 10 300 python3 bench.py --global-batch 32 --steps 30 --warmup 6 --no-cpu-baseline) > gpurun_out/ab3_${t}.log 2>&1 || { tail -5 gpurun_out/ab3_${t}.log; exit 1; }
  echo "$t B=32 $(tail -1 gpurun_out/ab3_${t}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final3 -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/prof_final3.log 2>&1 || { tail -20 gpurun_out/prof_final3.log; exit 1; }
tail -1 gpurun_out/prof_final3.log | cut -c1-200
