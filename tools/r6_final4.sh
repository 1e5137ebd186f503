#!/bin/bash
# round 6 final tree (last): the whole GPU suite, then the bench line + rocprofv3 --stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=_last bash tools/r6_final_tests.sh || exit 1
bash tools/r6_final_bench.sh || exit 1
