# FLAVA encoder parity, split-K A/B at B=32, PMC passes on attention / LN / BN kernels
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_flava_encoders_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_flavaenc.log 2>&1 || { tail -30 gpurun_out/t_flavaenc.log; exit 1; }
tail -1 gpurun_out/t_flavaenc.log
bash tools/gpu_r3_pmc2.sh || exit 1
