set -o pipefail
for v in 3 4; do
MMU_ATTN_FWD=$v timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/t_attn$v.log 2>&1
rc=$?; tail -2 gpurun_out/t_attn$v.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python tools/attn_bench.py --var MMU_ATTN_FWD --vals 1,2,3,4 > gpurun_out/attn_v2c.txt 2>&1
