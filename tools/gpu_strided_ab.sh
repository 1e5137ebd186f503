#!/bin/bash
# strided conv routing: parity tests, the per-shape A/B, then bench A/B vs ab/base_tree (HEAD)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/t_strided.log 2>&1 && tail -1 gpurun_out/t_strided.log &&
timeout -k 10 240 python -u tools/conv_strided_bench.py --batch 256 > gpurun_out/strided_256.log 2>&1 && cat gpurun_out/strided_256.log &&
bash tools/gpu_b32_ab.sh
