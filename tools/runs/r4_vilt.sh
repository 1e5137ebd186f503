# round 4: ViLT on the HIP kernels vs transformers (tests/test_vilt_gpu.py), then the encoder
# bench lines (FLAVA encoders = config 5's producer; ViLT classification)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_vilt_gpu.py tests/test_flava_encoders_gpu.py -s -v --timeout 300 --timeout-method thread > gpurun_out/r4_vilt_tests.log 2>&1; rc=$?
grep -E "^\[|PASSED|FAILED|Error|passed|failed" gpurun_out/r4_vilt_tests.log | head -30
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 bench.py --workload encoders --steps 5 --warmup 2 > gpurun_out/r4_bench_encoders.log 2>&1 || { tail -5 gpurun_out/r4_bench_encoders.log; exit 1; }
tail -1 gpurun_out/r4_bench_encoders.log
timeout -k 10 400 python3 bench.py --workload vilt --steps 5 --warmup 2 > gpurun_out/r4_bench_vilt.log 2>&1 || { tail -5 gpurun_out/r4_bench_vilt.log; exit 1; }
tail -1 gpurun_out/r4_bench_vilt.log
