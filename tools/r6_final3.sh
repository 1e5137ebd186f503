#!/bin/bash
# round 6 final tree: bench line + rocprofv3 --stats, then the batch-256 / 32 step traces
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/r6_final_bench.sh || exit 1
bash tools/r6_prof4.sh || exit 1
