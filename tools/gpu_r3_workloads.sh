# Round-3 HEAD re-check of the other bench workloads (FLAVA train step, ensemble x MC-dropout
# eval) and a kernel trace of the per-rank batch-32 step (config 4's share at N = 8)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --workload flava --steps 20 --warmup 5 > gpurun_out/bench_flava_r3.log 2>&1 || { tail -20 gpurun_out/bench_flava_r3.log; exit 1; }
tail -1 gpurun_out/bench_flava_r3.log | cut -c1-250
timeout -k 10 400 python3 -u bench.py --workload uncertainty --steps 5 --warmup 2 > gpurun_out/bench_unc_r3.log 2>&1 || { tail -20 gpurun_out/bench_unc_r3.log; exit 1; }
tail -1 gpurun_out/bench_unc_r3.log | cut -c1-250
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b32_r3 -o run -- python3 bench.py --global-batch 32 --steps 8 --warmup 4 --no-cpu-baseline > gpurun_out/prof_b32_r3.log 2>&1 || { tail -20 gpurun_out/prof_b32_r3.log; exit 1; }
tail -1 gpurun_out/prof_b32_r3.log | cut -c1-200
