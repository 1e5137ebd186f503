#!/bin/bash
# round 6: attention changes -- the attention GPU tests, then a same-box A/B of tools/attn_bench.py
# (ab/base.so = the previous tree, alternating)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/${TAG:-r6c}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread \
  -k "attention" > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" ${o}_tests.log | head -20; tail -5 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
for i in 1 2; do
  echo "== base $i" >> ${o}_ab.txt
  MMU_LIB_PATH=ab/base.so timeout -k 10 300 python -u tools/attn_bench.py >> ${o}_ab.txt 2>&1 || exit 1
  echo "== new $i" >> ${o}_ab.txt
  timeout -k 10 300 python -u tools/attn_bench.py >> ${o}_ab.txt 2>&1 || exit 1
done
grep -v amdgpu.ids ${o}_ab.txt
