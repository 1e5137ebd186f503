#!/bin/bash
# round 6 final: PMC passes over one bench step (tools/pmc_bench.sh) -> per-kernel summary + GEMM traffic
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/pmc_bench.sh r6last || exit 1
rm -rf gpurun_out/pmc_r6last/p*/run_kernel_trace.csv
ls gpurun_out/ | grep pmc_r6last
