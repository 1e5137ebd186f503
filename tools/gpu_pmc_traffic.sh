# two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) over a short bench.py run, each its own run
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_f.log 2>&1 || { echo "fetch pass rc=$?"; tail -5 gpurun_out/pmc_f.log; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_w.log 2>&1 || { echo "write pass rc=$?"; tail -5 gpurun_out/pmc_w.log; exit 1; }
ls gpurun_out/pmc_f gpurun_out/pmc_w
