set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { grep -E "Error|FAILED|err|assert" gpurun_out/t_gpu.log | head -30; exit 1; }
tail -1 gpurun_out/t_gpu.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench_pool.log 2>&1 || { tail -20 gpurun_out/bench_pool.log; exit 1; }
tail -1 gpurun_out/bench_pool.log | cut -c1-300
