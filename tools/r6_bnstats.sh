#!/bin/bash
# round 6: BatchNorm statistics from the conv epilogues + the embedding backward rewrite:
# kernel / model tests, then a same-box step A/B of MMU_BN_STATS_FUSION (0 = the BatchNorms'
# own statistics pass), batch 256 and batch 32, plus one kernel trace of the new tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6f
timeout -k 10 900 python -u -m pytest tests/test_resnet_gpu.py tests/test_kernels_gpu.py tests/test_mmbt_gpu.py -m gpu -v -s \
  --timeout 300 --timeout-method thread -k "stats or parts or embed or resnet or small_t16 or full_t508c-full-bf16 or model_grads or bottleneck or momentum" \
  > ${o}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" ${o}_tests.log | head -20; tail -5 ${o}_tests.log; exit 1; }
tail -1 ${o}_tests.log
bash tools/env_ab2.sh r6f_ab MMU_BN_STATS_FUSION=0 || exit 1
bash tools/env_ab2.sh r6f_ab32 MMU_BN_STATS_FUSION=0 --global-batch 32 || exit 1
cd /tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6f_prof -o run -- python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline > ${o}_prof.log 2>&1 || { tail -5 ${o}_prof.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/r6f_prof/run_kernel_trace.csv --md gpurun_out/r6f_step_profile.md > /dev/null 2>&1 || true
echo done
