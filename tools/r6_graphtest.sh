#!/bin/bash
# round 6: the full-model graph replay test, with and without the downsample sink (prints d, d_ee)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for v in 0 1 0 1; do
  echo "== MMU_DS_SINK=$v"
  MMU_DS_SINK=$v timeout -k 10 300 python -u -m pytest -q -s --timeout 280 --timeout-method thread tests/test_graph_gpu.py -k "replay_equals_eager_steps and True" 2>&1 | grep -E "\[graph|passed|failed"
done > gpurun_out/r6_graphtest.txt 2>&1
cat gpurun_out/r6_graphtest.txt
