#!/bin/bash
# round 6 final: the whole GPU suite on the final tree, in one process (SEL: extra pytest args)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/r6_gpu_tests_final${TAG:-}.log
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${SEL:-} > $out 2>&1
rc=$?
tail -3 $out
exit $rc
