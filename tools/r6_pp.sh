#!/bin/bash
# round 6: ping-pong GEMM schedule (gemm_pp_kernel) -- GEMM tests with it, then per-shape
# timings of both schedules on one box (MMU_GEMM_PP=0: the 2-phase big kernel)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6i
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "gemm" > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" ${o}_tests.log | head -20; tail -5 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
for i in 1 2; do
MMU_GEMM_PP=0 timeout -k 10 200 python -u tools/gemm_bench.py --no-ref > ${o}_gemm_off_$i.log 2>&1 || { tail -5 ${o}_gemm_off_$i.log; exit 1; }
MMU_GEMM_PP=1 timeout -k 10 200 python -u tools/gemm_bench.py --no-ref > ${o}_gemm_on_$i.log 2>&1 || { tail -5 ${o}_gemm_on_$i.log; exit 1; }
done
paste ${o}_gemm_off_1.log ${o}_gemm_on_1.log | grep -v amdgpu.ids
echo done
