#!/bin/bash
# round 6: fewer weight-gradient slices than one round (40 / 48 MiB split-K workspace: W1 / W2 4-5
# slices, ~55-70 % of the CUs), leaving CUs to the trunk backward's chain; step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/env_ab2.sh r6skw_ab40 MMU_SPLITK_WS_MB=40 || exit 1
bash tools/env_ab2.sh r6skw_ab48 MMU_SPLITK_WS_MB=48 || exit 1
