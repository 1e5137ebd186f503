set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { grep -E "Error|FAILED|err" gpurun_out/t_gpu.log | head -30; exit 1; }
tail -1 gpurun_out/t_gpu.log
for i in 1 2; do
for lib in ab/head.so multi-modal-uncertainty_amd/src/libmmu_hip.so; do
echo "== $lib" >> gpurun_out/attn_delta_ab.txt
MMU_LIB_PATH=$lib timeout -k 10 200 python -u tools/attn_bench.py --iters 10 >> gpurun_out/attn_delta_ab.txt 2>&1 || exit 1
done; done
grep -v amdgpu.ids gpurun_out/attn_delta_ab.txt
