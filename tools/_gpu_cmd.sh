set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { grep -E "Error|FAILED|err" gpurun_out/t_gpu.log | head -30; exit 1; }
tail -1 gpurun_out/t_gpu.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v15 -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_v15.log 2>&1 || { tail -20 gpurun_out/prof_v15.log; exit 1; }
grep '"metric"' gpurun_out/prof_v15.log | cut -c1-200
