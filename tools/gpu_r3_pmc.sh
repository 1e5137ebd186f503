# PMC passes on the hot kernels + a per-rank B=32 bench line
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 700 bash tools/pmc_passes.sh gpurun_out/pmc attn_fwd attn_bwd gemm_w1 gemm_qkv gemm_dz gemm_wgrad || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt 2>&1
timeout -k 10 300 python3 bench.py --global-batch 32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_b32.log 2>&1 || { tail -20 gpurun_out/bench_b32.log; exit 1; }
tail -1 gpurun_out/bench_b32.log | cut -c1-400
