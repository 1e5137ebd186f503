#!/bin/bash
# round 6: trunk filter gradients on the side stream at batch 32 (HIP-graph replay) -- flag run
# MMU_SIDE_WGRAD_MIN_BATCH=1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/env_ab2.sh r6sd_ab32 MMU_SIDE_WGRAD_MIN_BATCH=1 --global-batch 32 || exit 1
