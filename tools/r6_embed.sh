#!/bin/bash
# round 6: embedding backward rewrite -- its kernel test and the model tests that cover it, then
# a same-box step A/B against the previous tree (ab/base_tree), alternating, 10 steps each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6e
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_mmbt_gpu.py -m gpu -v -s --timeout 300 \
  --timeout-method thread -k "embed or small_t16 or full_t508c-full-bf16 or side_stream or checkpoint" > ${o}_tests.log 2>&1 \
  || { grep -E "FAILED|Error|assert" ${o}_tests.log | head -20; tail -5 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
for i in 1 2; do
  (cd ab/base_tree && timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline) > ${o}_base_$i.log 2>&1 || { tail -5 ${o}_base_$i.log; exit 1; }
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > ${o}_new_$i.log 2>&1 || { tail -5 ${o}_new_$i.log; exit 1; }
done
for f in ${o}_base_*.log ${o}_new_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
