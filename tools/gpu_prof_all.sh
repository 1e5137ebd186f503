# rocprofv3 kernel stats of the three bench workloads (mmbt train step, uncertainty, flava)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mmbt -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/prof_mmbt.log 2>&1 || { tail -20 gpurun_out/prof_mmbt.log; exit 1; }
tail -1 gpurun_out/prof_mmbt.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_unc -o run -- python3 bench.py --workload uncertainty --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_unc.log 2>&1 || { tail -20 gpurun_out/prof_unc.log; exit 1; }
tail -1 gpurun_out/prof_unc.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_flava -o run -- python3 bench.py --workload flava --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_flava.log 2>&1 || { tail -20 gpurun_out/prof_flava.log; exit 1; }
tail -1 gpurun_out/prof_flava.log
