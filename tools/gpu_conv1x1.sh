# 1x1 conv products, MIOpen vs mmu_gemm, at per-rank batch 32 and 256 (the _mmu_1x1 routing rule)
set -o pipefail
mkdir -p gpurun_out
for b in 32 256; do
  timeout -k 10 300 python3 tools/conv1x1_bench.py --batch $b > gpurun_out/conv1x1_b$b.log 2>&1 || { tail -5 gpurun_out/conv1x1_b$b.log; exit 1; }
done
cat gpurun_out/conv1x1_b32.log gpurun_out/conv1x1_b256.log
