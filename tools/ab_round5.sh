#!/bin/bash
# Round-5 A/B batch (one GPU call): the GEMM + attention parity tests under the new defaults,
# then the stream-K GEMM tail (MMU_GEMM_SK 0/1: tools/gemm_bench.py, bench.py at batch 256 and
# 32) and the attention keep words ahead of the forward (MMU_ATTN_KEEPIN 0/2/3: attn_bench).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
MMU_GEMM_SK=1 MMU_ATTN_KEEPIN=2 timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "gemm or attention" > gpurun_out/r5ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5ab_tests.log; [ $rc -eq 0 ] || { echo "TESTS rc=$rc"; exit $rc; }
for i in 1 2; do
  for v in 0 2 3; do
    MMU_ATTN_KEEPIN=$v timeout -k 10 200 python tools/attn_bench.py > gpurun_out/r5ab_attn_k${v}_$i.log 2>&1 || exit 1
  done
done
for v in 0 1; do MMU_GEMM_SK=$v timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/r5ab_gb_sk$v.log 2>&1 || exit 1; done
tools/env_ab.sh r5ab_sk MMU_GEMM_SK || exit 1
BENCH_ARGS="--global-batch 32" tools/env_ab.sh r5ab_sk32 MMU_GEMM_SK || exit 1
