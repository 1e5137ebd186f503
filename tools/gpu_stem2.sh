# stem conv: parity, timings vs MIOpen, PMC passes on both stem kernels
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_resnet_gpu.py -k stem_conv -x -q --timeout 200 --timeout-method thread > gpurun_out/t_stem.log 2>&1 || { tail -40 gpurun_out/t_stem.log; exit 1; }
tail -1 gpurun_out/t_stem.log
for b in 256 32; do
  timeout -k 10 200 python3 tools/stem_bench.py --batch $b > gpurun_out/stem_$b.log 2>&1 || { tail -5 gpurun_out/stem_$b.log; exit 1; }
  grep -v amdgpu gpurun_out/stem_$b.log
done
rm -rf gpurun_out/pmc_stem
bash tools/pmc_passes.sh gpurun_out/pmc_stem stem_fwd stem_wgrad > gpurun_out/pmc_stem.log 2>&1 || { tail -5 gpurun_out/pmc_stem.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_stem --raw > gpurun_out/pmc_stem_summary.txt
head -3 gpurun_out/pmc_stem_summary.txt
grep -A18 "stem_fwd_kernel" gpurun_out/pmc_stem_summary.txt | head -20
