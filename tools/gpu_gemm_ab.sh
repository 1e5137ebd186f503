# GEMM A/B on one MI355X: GEMM parity tests (default and with the variant env), then
# tools/gemm_bench.py over an env switch.   usage: bash tools/gpu_gemm_ab.sh VAR VALS [tag] [testenv]
set -o pipefail
mkdir -p gpurun_out
var=$1; vals=$2; tag=${3:-ab}; tenv=${4:-}
timeout -k 10 300 env $tenv python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k gemm --timeout 120 --timeout-method thread > gpurun_out/t_gemm.log 2>&1 || { grep -E "Error|FAILED|assert" gpurun_out/t_gemm.log | head -30; exit 1; }
tail -1 gpurun_out/t_gemm.log
timeout -k 10 300 python -u tools/gemm_bench.py --var $var --vals $vals > gpurun_out/gemm_$tag.txt 2>&1 || { tail -20 gpurun_out/gemm_$tag.txt; exit 1; }
cat gpurun_out/gemm_$tag.txt
