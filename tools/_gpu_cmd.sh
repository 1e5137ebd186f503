set -o pipefail
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log
timeout -k 10 400 python -u bench.py --workload uncertainty --steps 3 --warmup 1 > gpurun_out/bench_unc_final.log 2>&1 || { tail -20 gpurun_out/bench_unc_final.log; exit 1; }
tail -1 gpurun_out/bench_unc_final.log
