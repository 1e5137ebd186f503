#!/bin/bash
# strided conv kernels after the split-K change: per-shape A/B at batch 256 and 32, then bench B=32 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "strided or wgrad" > gpurun_out/t_strided.log 2>&1 && tail -1 gpurun_out/t_strided.log &&
timeout -k 10 240 python -u tools/conv_strided_bench.py --batch 256 > gpurun_out/strided_256.log 2>&1 && cat gpurun_out/strided_256.log &&
timeout -k 10 240 python -u tools/conv_strided_bench.py --batch 32 > gpurun_out/strided_32.log 2>&1 && cat gpurun_out/strided_32.log
