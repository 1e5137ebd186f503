# BatchNorm grid sizing sweep: tools/bn_bench.py per-step BN time at batch 32 and 256 with the
# library in the tree (target 1024 blocks, >= 4096 elements per block) and ab/bn_* variants
# (>= 8192 / >= 16384 elements per block, target 512 blocks), alternating, same box
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in base m8k m16k t512; do
    lib=""; [ $v != base ] && lib=$(pwd)/ab/bn_$v/libmmu_hip.so
    for b in 32 256; do
      MMU_LIB_PATH=$lib timeout -k 10 120 python3 tools/bn_bench.py --batch $b > gpurun_out/bng_${v}_${b}.log 2>&1 || { tail -5 gpurun_out/bng_${v}_${b}.log; exit 1; }
      echo "$v B=$b $(tail -1 gpurun_out/bng_${v}_${b}.log)"
    done
  done
done
