# round 4: persistent big-tile GEMM (ab/persist.so) -- GEMM / conv parity, then same-box A/B
# against the committed tree's library (GEMM shapes, then the train-step bench)
set -o pipefail
mkdir -p gpurun_out
MMU_LIB_PATH=ab/persist.so timeout -k 10 600 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_resnet_gpu.py -x -q --timeout 300 --timeout-method thread -k "gemm or conv or bottleneck or model_grads" > gpurun_out/r4_persist_tests.log 2>&1 || { tail -30 gpurun_out/r4_persist_tests.log; exit 1; }
tail -1 gpurun_out/r4_persist_tests.log
for v in base persist; do
  lib=""; [ $v != base ] && lib=ab/$v.so
  MMU_LIB_PATH=$lib timeout -k 10 300 python3 tools/gemm_bench.py --vals 0 --iters 6 > gpurun_out/r4_gemm_$v.log 2>&1 || { tail -5 gpurun_out/r4_gemm_$v.log; exit 1; }
done
paste -d'|' <(cut -c1-70 gpurun_out/r4_gemm_base.log) <(cut -c43-60 gpurun_out/r4_gemm_persist.log)
for v in base persist base persist; do
  lib=""; [ $v != base ] && lib=ab/$v.so
  MMU_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/r4_bench_$v.log 2>&1 || { tail -5 gpurun_out/r4_bench_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r4_bench_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["achieved"], d["roofline"]["frac"])')"
done
