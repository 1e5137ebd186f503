# kernel trace of the per-rank B=32 step (working tree), then the conv census at 256 and 32
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b32n -o run -- python3 bench.py --global-batch 32 --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/prof_b32n.log 2>&1 || { tail -20 gpurun_out/prof_b32n.log; exit 1; }
grep metric gpurun_out/prof_b32n.log | cut -c1-200
timeout -k 10 300 python3 tools/conv_census.py --batch 256 > gpurun_out/census_256.log 2>&1 || { tail -5 gpurun_out/census_256.log; exit 1; }
timeout -k 10 300 python3 tools/conv_census.py --batch 32 > gpurun_out/census_32.log 2>&1 || { tail -5 gpurun_out/census_32.log; exit 1; }
tail -1 gpurun_out/census_256.log; tail -1 gpurun_out/census_32.log
