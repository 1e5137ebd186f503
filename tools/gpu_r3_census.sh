set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_bench_ab.sh || exit 1
timeout -k 10 300 python3 tools/conv_census.py --batch 256 > gpurun_out/census_256.log 2>&1 || { tail -5 gpurun_out/census_256.log; exit 1; }
timeout -k 10 300 python3 tools/conv_census.py --batch 32 > gpurun_out/census_32.log 2>&1 || { tail -5 gpurun_out/census_32.log; exit 1; }
tail -1 gpurun_out/census_256.log; tail -1 gpurun_out/census_32.log
