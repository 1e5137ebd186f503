# round-3 record after the strided convs and the side-stream filter gradients: every GPU test,
# smoke(), the train-step bench lines (per-rank batch 256 with the CPU baseline, and 32), then a
# kernel trace of the bench for the step profile; each step under its own time limit
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_gpu_final2.log 2>&1 || { tail -40 gpurun_out/t_gpu_final2.log; exit 1; }
tail -1 gpurun_out/t_gpu_final2.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final2.log 2>&1 || { tail -20 gpurun_out/smoke_final2.log; exit 1; }
tail -1 gpurun_out/smoke_final2.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_final2.log 2>&1 || { tail -5 gpurun_out/bench_final2.log; exit 1; }
tail -1 gpurun_out/bench_final2.log | cut -c1-300
timeout -k 10 300 python3 bench.py --global-batch 32 --steps 10 --warmup 4 --no-cpu-baseline > gpurun_out/bench_b32_final2.log 2>&1 || { tail -5 gpurun_out/bench_b32_final2.log; exit 1; }
tail -1 gpurun_out/bench_b32_final2.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final2 -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/prof_final2.log 2>&1 || { tail -20 gpurun_out/prof_final2.log; exit 1; }
tail -1 gpurun_out/prof_final2.log | cut -c1-200
