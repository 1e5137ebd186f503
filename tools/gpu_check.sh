set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { grep -E "Error|FAILED|assert" gpurun_out/t_gpu.log | head -30; exit 1; }
tail -1 gpurun_out/t_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
