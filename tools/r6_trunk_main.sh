#!/bin/bash
# round 6: the trunk's filter gradients on the main stream at batch 256 (MMU_SIDE_WGRAD_MIN_BATCH=100000),
# now that the encoder's weight gradients start at the first trunk BatchNorm backward
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/env_ab2.sh r6tm_ab MMU_SIDE_WGRAD_MIN_BATCH=100000 || exit 1
