#!/bin/bash
# strided conv kernels: parity tests, then the per-shape A/B vs MIOpen at batch 256 and 32
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "strided or conv3x3 or model_grads" > gpurun_out/t_strided.log 2>&1 && tail -3 gpurun_out/t_strided.log &&
timeout -k 10 240 python -u tools/conv_strided_bench.py --batch 256 > gpurun_out/strided_256.log 2>&1 && cat gpurun_out/strided_256.log &&
timeout -k 10 240 python -u tools/conv_strided_bench.py --batch 32 > gpurun_out/strided_32.log 2>&1 && cat gpurun_out/strided_32.log
