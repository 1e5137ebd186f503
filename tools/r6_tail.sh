#!/bin/bash
# round 6: what the partial last round of tiles costs -- the BERT GEMMs at M = 256 x 513 / 32 x 513
# token rows against M rounded down to whole 256-row tiles (131072 / 16384)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 131328 131072 16416 16384; do
  timeout -k 10 200 python -u tools/gemm_bench.py --no-ref --rows $r > gpurun_out/r6j_rows_$r.log 2>&1 || { tail -5 gpurun_out/r6j_rows_$r.log; exit 1; }
done
paste gpurun_out/r6j_rows_131328.log gpurun_out/r6j_rows_131072.log | grep -v amdgpu | cut -c1-200
paste gpurun_out/r6j_rows_16416.log gpurun_out/r6j_rows_16384.log | grep -v amdgpu | cut -c1-200
