# BatchNorm ReLU-mask check on one MI355X: BN / ResNet GPU tests, BN kernel timings, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_resnet_gpu.py tests/test_mmbt_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_bn.log 2>&1 || { grep -E "Error|FAILED|assert" gpurun_out/t_bn.log | head -30; exit 1; }
tail -1 gpurun_out/t_bn.log
timeout -k 10 200 python -u tools/bn_bench.py > gpurun_out/bn_bench.txt 2>&1 || { tail -20 gpurun_out/bn_bench.txt; exit 1; }
cat gpurun_out/bn_bench.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_bn.log 2>&1 || { tail -20 gpurun_out/bench_bn.log; exit 1; }
tail -1 gpurun_out/bench_bn.log
