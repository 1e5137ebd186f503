#!/bin/bash
# round 6 final: the graph-replay tests, then the driver-style bench line + rocprofv3 --stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_graph_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r6_graph_final.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r6_graph_final.log | head; tail -3 gpurun_out/r6_graph_final.log; exit 1; }
tail -1 gpurun_out/r6_graph_final.log
bash tools/r6_final_bench.sh
