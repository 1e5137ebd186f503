set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { grep -E "Error|FAILED|err" gpurun_out/t_gpu.log | head -30; exit 1; }
tail -2 gpurun_out/t_gpu.log
