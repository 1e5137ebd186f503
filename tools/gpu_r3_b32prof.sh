# attention A/B (base = HEAD) + kernel-trace profile of the per-rank B=32 step
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_attn_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b32 -o run -- python3 bench.py --global-batch 32 --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/prof_b32.log 2>&1 || { tail -20 gpurun_out/prof_b32.log; exit 1; }
tail -1 gpurun_out/prof_b32.log | cut -c1-300
