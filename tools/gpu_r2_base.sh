# Round-2 check on a fresh MI355X: GPU tests, smoke, bench, rocprofv3 kernel stats of the bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { grep -E "Error|FAILED|assert" gpurun_out/t_gpu.log | head -30; exit 1; }
tail -1 gpurun_out/t_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
tail -1 gpurun_out/prof.log
