# round 4, first lease: the product-precision parity tests (printing their measured errors),
# the whole GPU suite, smoke(), the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_mmbt_gpu.py tests/test_dp_gpu.py -s -x -v --timeout 300 --timeout-method thread -k "train_step or bnfit or single_device" > gpurun_out/r4_parity.log 2>&1; rc=$?
grep -E "^\[|PASSED|FAILED|Error" gpurun_out/r4_parity.log | head -40
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r4_gpu_tests.log 2>&1; rc2=$?
tail -1 gpurun_out/r4_gpu_tests.log; grep FAILED gpurun_out/r4_gpu_tests.log | head
[ $rc2 -le 1 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { tail -20 gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/r4_bench_v1.log 2>&1 || { tail -5 gpurun_out/r4_bench_v1.log; exit 1; }
tail -1 gpurun_out/r4_bench_v1.log | cut -c1-400
