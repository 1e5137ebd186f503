# round 4: product-precision parity with the torch-bf16 noise comparator; DP f32/bf16 bucket
# parity; attention A/B (HEAD lib vs scalar softmax math vs scalar + dQ at 3 waves/SIMD)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests/test_mmbt_gpu.py tests/test_dp_gpu.py -s -v --timeout 400 --timeout-method thread -k "train_step or bnfit or single_device" > gpurun_out/r4_parity2.log 2>&1
grep -E "^\[|PASSED|FAILED|Error" gpurun_out/r4_parity2.log | head -40
for v in base scalar scalar_dq3 base scalar scalar_dq3; do
  lib=""; [ $v != base ] && lib=ab/$v.so
  MMU_LIB_PATH=$lib timeout -k 10 120 python3 tools/attn_bench.py > gpurun_out/r4_attn_$v.log 2>&1 || { tail -5 gpurun_out/r4_attn_$v.log; exit 1; }
  echo "== $v"; cat gpurun_out/r4_attn_$v.log
done
