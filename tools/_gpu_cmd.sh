set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t_resnet.log 2>&1 || { grep -E "Error|FAILED|err|assert" gpurun_out/t_resnet.log | head -30; exit 1; }
tail -1 gpurun_out/t_resnet.log
