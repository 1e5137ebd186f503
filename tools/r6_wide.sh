#!/bin/bash
# round 6: 256x384 GEMM tiling + split tail rows -- parity tests, then a same-box A/B on the BERT
# shapes (MMU_GEMM_WIDE / MMU_GEMM_TAIL alternated, tools/gemm_bench.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6w2
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm" > ${o}_tests.log 2>&1 || { echo "tests failed"; tail -40 ${o}_tests.log; exit 1; }
tail -3 ${o}_tests.log
CASES=${CASES:-"fwd qkv,fwd ffn1 gelu,fwd ffn2,fwd o    drop,bwd dZ   B=W2,bwd dA   B=W1,bwd dX   B=Wqkv,bwd dO   B=Wo"}
for v in ${VARIANTS:-0:0 1:1 0:1 0:0 1:1 0:1}; do
  wd=${v%%:*}; tl=${v##*:}
  echo "== wide=$wd tail=$tl" >> ${o}_times.txt
  MMU_GEMM_WIDE=$wd MMU_GEMM_TAIL=$tl timeout -k 10 240 python -u tools/gemm_bench.py --no-ref --cases "$CASES" 2>&1 \
    | grep -v amdgpu.ids >> ${o}_times.txt || { echo "gemm_bench failed $v"; tail -5 ${o}_times.txt; exit 1; }
done
cat ${o}_times.txt
