#!/bin/bash
# round 6: conv routing with the BatchNorm passes fused into the conv epilogues (MMU_ROUTE_FUSED
# 1: every eligible 1x1 forward + the 128-channel 3x3 forward on mmu; 2: + the 64-channel 3x3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6g
MMU_ROUTE_FUSED=2 timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "bottleneck or block" > ${o}_route_tests.log 2>&1 || { tail -5 ${o}_route_tests.log; exit 1; }
tail -1 ${o}_route_tests.log
bash tools/env_ab2.sh r6g_route1 MMU_ROUTE_FUSED=1 || exit 1
bash tools/env_ab2.sh r6g_route2 MMU_ROUTE_FUSED=2 || exit 1
echo done
