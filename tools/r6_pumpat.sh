#!/bin/bash
# round 6: the encoder's weight gradients issued at the 4th / 10th trunk BatchNorm backward instead of the
# 1st (MMU_WGRAD_PUMP_AT): the latency-bound layer4 chain then runs without them
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/env_ab2.sh r6pa4_ab MMU_WGRAD_PUMP_AT=4 || exit 1
bash tools/env_ab2.sh r6pa10_ab MMU_WGRAD_PUMP_AT=10 || exit 1
