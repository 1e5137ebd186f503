#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py tests/test_mmbt_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_hp.log 2>&1 && tail -1 gpurun_out/t_hp.log &&
timeout -k 10 300 python3 -u tools/host_profile.py --batch 32 > gpurun_out/host_prof32.log 2>&1 &&
timeout -k 10 300 python3 -u tools/host_time.py --batch 32 > gpurun_out/host32.log 2>&1 && cat gpurun_out/host32.log
