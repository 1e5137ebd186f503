# round-3 profile: step kernel stats of the bench + PMC passes on the hot kernels
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mmbt -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/prof_mmbt.log 2>&1 || { tail -20 gpurun_out/prof_mmbt.log; exit 1; }
tail -1 gpurun_out/prof_mmbt.log | cut -c1-300
timeout -k 10 600 bash tools/pmc_passes.sh gpurun_out/pmc attn_fwd attn_bwd gemm_w1 gemm_qkv gemm_dz gemm_wgrad || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt 2>&1
tail -60 gpurun_out/pmc_summary.txt
