#!/bin/bash
# round 6: the deferred BERT weight gradients issued at the first trunk BatchNorm backward, behind the
# embedding / image-projection backward (MMU_WGRAD_INTERLEAVE=2) -- step A/B, batch 256 and 32
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash tools/env_ab2.sh r6fl_ab MMU_WGRAD_INTERLEAVE=2 || exit 1
bash tools/env_ab2.sh r6fl_ab32 MMU_WGRAD_INTERLEAVE=2 --global-batch 32 || exit 1
