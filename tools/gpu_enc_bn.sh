#!/bin/bash
# encoder / DP / uncertainty GPU tests after the deferral change, the BN block-reduce A/B, and a
# longer batch-32 bench A/B (base_tree = the commit before the BN change, deferral in both)
set -o pipefail
bash tools/gpu_check_encoder.sh && bash tools/gpu_bn_ab.sh && bash tools/gpu_b32_ab2.sh
