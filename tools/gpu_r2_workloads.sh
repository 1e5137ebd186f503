# Round-2 re-check of the two other bench workloads (FLAVA train step, ensemble x MC-dropout eval).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --workload flava --steps 20 --warmup 5 > gpurun_out/bench_flava.log 2>&1 || { tail -20 gpurun_out/bench_flava.log; exit 1; }
tail -1 gpurun_out/bench_flava.log
timeout -k 10 400 python -u bench.py --workload uncertainty --steps 5 --warmup 2 > gpurun_out/bench_unc.log 2>&1 || { tail -20 gpurun_out/bench_unc.log; exit 1; }
tail -1 gpurun_out/bench_unc.log
