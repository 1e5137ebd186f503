# short-K split-K for f32 weight gradients: conv1x1 products (mmu dW column) with the in-tree library vs
# ab/base_tree, at per-rank batch 32 and 256, then the bench at batch 32 / 256 (alternated)
set -o pipefail
mkdir -p gpurun_out
base=$(pwd)/ab/base_tree/multi-modal-uncertainty_amd/src/libmmu_hip.so
for b in 32 256; do
  timeout -k 10 300 python3 tools/conv1x1_bench.py --batch $b > gpurun_out/wg_new_$b.log 2>&1 || { tail -5 gpurun_out/wg_new_$b.log; exit 1; }
  MMU_LIB_PATH=$base timeout -k 10 300 python3 tools/conv1x1_bench.py --batch $b > gpurun_out/wg_base_$b.log 2>&1 || { tail -5 gpurun_out/wg_base_$b.log; exit 1; }
done
for b in 32 256; do
  for t in base new base new; do
    lib=; [ $t = base ] && lib=$base
    MMU_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --global-batch $b --steps 10 --warmup 4 --no-cpu-baseline > gpurun_out/wgb_${t}_$b.log 2>&1 || { tail -5 gpurun_out/wgb_${t}_$b.log; exit 1; }
    echo "$t B=$b $(tail -1 gpurun_out/wgb_${t}_$b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
timeout -k 10 300 python3 -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_wg.log 2>&1 || { tail -20 gpurun_out/t_wg.log; exit 1; }
tail -1 gpurun_out/t_wg.log
