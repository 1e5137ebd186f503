# same-box A/B of the attention kernels: ab/base_tree (HEAD) library vs the working tree, alternated,
# then the attention GPU parity tests on the working-tree library
set -o pipefail
mkdir -p gpurun_out
base=$(pwd)/ab/base_tree/multi-modal-uncertainty_amd/src/libmmu_hip.so
for i in 1 2; do
  MMU_LIB_PATH=$base timeout -k 10 120 python3 tools/attn_bench.py --iters 10 > gpurun_out/attn_base_$i.log 2>&1 || { tail -5 gpurun_out/attn_base_$i.log; exit 1; }
  echo "base $i"; grep p= gpurun_out/attn_base_$i.log
  timeout -k 10 120 python3 tools/attn_bench.py --iters 10 > gpurun_out/attn_new_$i.log 2>&1 || { tail -5 gpurun_out/attn_new_$i.log; exit 1; }
  echo "new $i"; grep p= gpurun_out/attn_new_$i.log
done
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -k "attn or attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1 || { tail -20 gpurun_out/t_attn.log; exit 1; }
tail -1 gpurun_out/t_attn.log
