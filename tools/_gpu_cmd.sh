set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v16 -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_v16.log 2>&1 || { tail -20 gpurun_out/prof_v16.log; exit 1; }
grep '"metric"' gpurun_out/prof_v16.log | cut -c1-200
find gpurun_out/prof_v16 -name "*stats*" | head
