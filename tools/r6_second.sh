#!/bin/bash
# round 6, second GPU call: the batch-4 fixture (with / without the stream residue), the sync-BN
# routing diagnostic, then the GEMM store-policy x group-height A/B (+ PMC traffic passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6b
timeout -k 10 600 python -u -m pytest tests/test_mmbt_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread \
  -k "t508c_b4" > ${o}_b4.log 2>&1; echo "b4 rc=$?"
MMU_STREAM_RESIDUE=0 timeout -k 10 600 python -u -m pytest tests/test_mmbt_gpu.py -m gpu -v -s --timeout 300 \
  --timeout-method thread -k "t508c_b4" > ${o}_b4_nores.log 2>&1; echo "b4 nores rc=$?"
timeout -k 10 600 python -u -m pytest tests/test_dp_gpu.py -m gpu -v -s --timeout 400 --timeout-method thread \
  -k "gap_is_conv_routing" > ${o}_syncbn.log 2>&1; echo "syncbn rc=$?"
grep -hE "^\[" ${o}_b4.log ${o}_b4_nores.log ${o}_syncbn.log | cut -c1-300
PMC=1 bash tools/r6_gemm_ab.sh
