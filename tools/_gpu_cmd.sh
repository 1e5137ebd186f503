set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -2 gpurun_out/t_gpu.log
timeout -k 10 400 python -u bench.py --workload uncertainty --steps 3 --warmup 1 > gpurun_out/bench_unc.log 2>&1 || { tail -30 gpurun_out/bench_unc.log; exit 1; }
tail -1 gpurun_out/bench_unc.log
