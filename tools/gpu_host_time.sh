#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/host_time.py --batch 32 > gpurun_out/host32.log 2>&1 && cat gpurun_out/host32.log &&
timeout -k 10 300 python3 -u tools/host_time.py --batch 256 --steps 6 > gpurun_out/host256.log 2>&1 && cat gpurun_out/host256.log
