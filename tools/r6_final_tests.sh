#!/bin/bash
# round 6 final: the whole GPU suite on the final tree (second half from the batch-4 bnfit test on)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${SEL:-} > gpurun_out/r6_gpu_tests_final2.log 2>&1
rc=$?
tail -3 gpurun_out/r6_gpu_tests_final2.log
exit $rc
