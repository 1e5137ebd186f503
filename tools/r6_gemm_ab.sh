#!/bin/bash
# round 6 GEMM A/B: epilogue store policy (MMU_GEMM_STORE_POL 0 = plain, 16 = sc1) x tile-order
# group height (MMU_GEMM_GROUP_M), alternated on one box (tools/gemm_bench.py), then FETCH_SIZE /
# WRITE_SIZE per variant from rocprofv3 PMC passes over the same cases
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r6g
mkdir -p gpurun_out
CASES=${CASES:-"fwd qkv,fwd ffn1 gelu,fwd ffn1 bias only,fwd ffn2,fwd o    drop,bwd dZ   B=W2,bwd dA   B=W1,bwd dX   B=Wqkv"}
VARIANTS=${VARIANTS:-"0:0 16:0 0:0 16:0 16:4 16:16 0:16"}
for v in $VARIANTS; do
  pol=${v%%:*}; gm=${v##*:}
  echo "== pol=$pol group_m=$gm" >> ${o}_times.txt
  MMU_GEMM_STORE_POL=$pol MMU_GEMM_GROUP_M=$gm timeout -k 10 240 python -u tools/gemm_bench.py --no-ref \
    --cases "$CASES" >> ${o}_times.txt 2>&1 || { echo "gemm_bench failed pol=$pol gm=$gm"; tail -5 ${o}_times.txt; exit 1; }
done
cat ${o}_times.txt
if [ -n "$PMC" ]; then
  for v in 0:0 16:0; do
    pol=${v%%:*}; gm=${v##*:}
    for c in FETCH_SIZE WRITE_SIZE; do
      MMU_GEMM_STORE_POL=$pol MMU_GEMM_GROUP_M=$gm timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace --output-format csv \
        -d gpurun_out/r6g_pmc_${pol}_${gm}_$c -o run -- python tools/gemm_bench.py --no-ref --iters 2 \
        --cases "$CASES" > gpurun_out/r6g_pmc_${pol}_${gm}_$c.log 2>&1 || { echo "pmc failed $v $c"; exit 1; }
    done
  done
fi
