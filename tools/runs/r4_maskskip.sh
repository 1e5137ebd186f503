# round 4: attention forward skips the key-mask accumulator init on unmasked tiles (ab/maskskip.so):
# attention parity, then same-box A/B against the committed library (attn_bench, train-step bench)
set -o pipefail
mkdir -p gpurun_out
MMU_LIB_PATH=ab/w3.so timeout -k 10 600 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_flava_gpu.py tests/test_mmbt_gpu.py -x -q --timeout 300 --timeout-method thread -k "attention or forward_variants or seqattn or flava_encoders or dropout" > gpurun_out/r4_maskskip_tests.log 2>&1 || { tail -30 gpurun_out/r4_maskskip_tests.log; exit 1; }
tail -1 gpurun_out/r4_maskskip_tests.log
for v in base maskskip w3 base maskskip w3; do
  lib=""; [ $v != base ] && lib=ab/$v.so
  MMU_LIB_PATH=$lib timeout -k 10 120 python3 tools/attn_bench.py > gpurun_out/r4_attn2_$v.log 2>&1 || { tail -5 gpurun_out/r4_attn2_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/r4_attn2_$v.log
done
for v in base maskskip w3 base maskskip w3; do
  lib=""; [ $v != base ] && lib=ab/$v.so
  MMU_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/r4_bench2_$v.log 2>&1 || { tail -5 gpurun_out/r4_bench2_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r4_bench2_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
