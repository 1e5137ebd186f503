set -o pipefail
for i in 1 2; do
for lib in ab/head.so multi-modal-uncertainty_amd/src/libmmu_hip.so; do
echo "== $lib" >> gpurun_out/attn_ab.txt
MMU_LIB_PATH=$lib timeout -k 10 200 python -u tools/attn_bench.py --iters 10 >> gpurun_out/attn_ab.txt 2>&1 || exit 1
done; done
