set -o pipefail
for cfg in "1 65536" "1024 4096" "2048 4096" "512 8192"; do
set -- $cfg
for b in 32 256; do
echo "== target=$1 min=$2 batch=$b" >> gpurun_out/bn_ab.txt
MMU_BN_TARGET=$1 MMU_BN_MIN=$2 timeout -k 10 120 python -u tools/bn_bench.py --batch $b >> gpurun_out/bn_ab.txt 2>&1 || exit 1
done; done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --global-batch 32 --no-cpu-baseline > gpurun_out/bench_b32.log 2>&1 || exit 1
MMU_GEMM_TAIL=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --global-batch 32 --no-cpu-baseline > gpurun_out/bench_b32_tail.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_b256.log 2>&1 || exit 1
for f in bench_b32 bench_b32_tail bench_b256; do grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log; done
