set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u tools/conv1x1_bench.py --batch 256 > gpurun_out/conv1x1_b256.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv1x1_bench.py --batch 32 > gpurun_out/conv1x1_b32.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b256 -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_b256.log 2>&1
