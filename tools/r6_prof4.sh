#!/bin/bash
# round 6: kernel traces of the current tree, batch 256 (eager) and batch 32 (graph replay)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6g_prof256 -o run -- python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline > gpurun_out/r6g_prof256.log 2>&1 || { tail -5 gpurun_out/r6g_prof256.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/r6g_prof256/run_kernel_trace.csv --md gpurun_out/r6g_step_profile_b256.md > /dev/null 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6g_prof32 -o run -- python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --global-batch 32 > gpurun_out/r6g_prof32.log 2>&1 || { tail -5 gpurun_out/r6g_prof32.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/r6g_prof32/run_kernel_trace.csv --md gpurun_out/r6g_step_profile_b32.md > /dev/null 2>&1 || true
true
ls gpurun_out/r6g_prof32
echo done
