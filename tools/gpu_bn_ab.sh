# one-launch BatchNorm: GPU tests, then the trunk BN shapes timed with the in-tree library, the
# ab/varA library (if present) and the ab/base_tree library (three-launch kernels), batch 32 / 256
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -k batchnorm -x -v --timeout 120 --timeout-method thread > gpurun_out/t_bn.log 2>&1 || { tail -30 gpurun_out/t_bn.log; exit 1; }
tail -2 gpurun_out/t_bn.log
for b in 32 256; do
  for t in new varA base_tree; do
    lib=; [ $t != new ] && lib=$(pwd)/ab/$t/multi-modal-uncertainty_amd/src/libmmu_hip.so
    [ -n "$lib" ] && [ ! -f "$lib" ] && continue
    MMU_LIB_PATH=$lib timeout -k 10 200 python3 tools/bn_bench.py --batch $b > gpurun_out/bn_${t}_$b.log 2>&1 || { tail -5 gpurun_out/bn_${t}_$b.log; exit 1; }
    echo "$t B=$b $(tail -1 gpurun_out/bn_${t}_$b.log)"
  done
done
