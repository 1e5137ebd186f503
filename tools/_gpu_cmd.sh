set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_flava_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_flava.log 2>&1
rc=$?; tail -25 gpurun_out/t_flava.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/t_gpu.log; exit $rc
