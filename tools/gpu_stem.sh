# stem conv: parity test, kernel timings vs MIOpen, then the full-tree bench A/B (tools/gpu_b32_ab.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_resnet_gpu.py -k stem_conv -x -v --timeout 200 --timeout-method thread > gpurun_out/t_stem.log 2>&1 || { tail -40 gpurun_out/t_stem.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/t_stem.log
for b in 256 32; do
  timeout -k 10 200 python3 tools/stem_bench.py --batch $b > gpurun_out/stem_$b.log 2>&1 || { tail -5 gpurun_out/stem_$b.log; exit 1; }
  grep -v amdgpu gpurun_out/stem_$b.log
done
bash tools/gpu_b32_ab.sh
