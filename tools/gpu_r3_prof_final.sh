# kernel trace of the final round-3 tree's default bench (per-rank batch 256)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final5 -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/prof_final5.log 2>&1 || { tail -20 gpurun_out/prof_final5.log; exit 1; }
tail -1 gpurun_out/prof_final5.log | cut -c1-200
