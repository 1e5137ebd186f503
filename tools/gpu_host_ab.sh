#!/bin/bash
# host-overhead trims: GPU tests, then host enqueue time (new vs ab/base_tree), then the batch-32 bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_resnet_gpu.py tests/test_mmbt_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_host.log 2>&1 && tail -1 gpurun_out/t_host.log &&
timeout -k 10 300 python3 -u tools/host_time.py --batch 32 > gpurun_out/host32_new.log 2>&1 && echo new && cat gpurun_out/host32_new.log &&
(cd ab/base_tree && timeout -k 10 300 python3 -u tools/host_time.py --batch 32) > gpurun_out/host32_base.log 2>&1 && echo base && cat gpurun_out/host32_base.log &&
bash tools/gpu_b32_ab2.sh
