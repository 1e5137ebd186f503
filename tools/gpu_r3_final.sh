# round-3 record on one MI355X: every GPU test, smoke(), then the bench lines (train step with the
# CPU baseline, uncertainty, FLAVA, per-rank batch 32); each step under its own time limit
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_gpu_final.log 2>&1 || { tail -40 gpurun_out/t_gpu_final.log; exit 1; }
tail -1 gpurun_out/t_gpu_final.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -2 gpurun_out/smoke_final.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_final.log 2>&1 || { tail -5 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log | cut -c1-400
timeout -k 10 300 python3 bench.py --workload uncertainty --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_unc_final.log 2>&1 || { tail -5 gpurun_out/bench_unc_final.log; exit 1; }
timeout -k 10 300 python3 bench.py --workload flava --no-cpu-baseline > gpurun_out/bench_flava_final.log 2>&1 || { tail -5 gpurun_out/bench_flava_final.log; exit 1; }
timeout -k 10 300 python3 bench.py --global-batch 32 --steps 10 --warmup 4 --no-cpu-baseline > gpurun_out/bench_b32_final.log 2>&1 || { tail -5 gpurun_out/bench_b32_final.log; exit 1; }
for f in bench_unc_final bench_flava_final bench_b32_final; do tail -1 gpurun_out/$f.log | cut -c1-200; done
