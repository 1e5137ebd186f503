set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in 0 1; do
    MMU_CONV_SPLITK=$v timeout -k 10 300 python3 bench.py --global-batch 32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sk_${v}_$i.log 2>&1 || { tail -5 gpurun_out/sk_${v}_$i.log; exit 1; }
    echo "splitk=$v run $i $(tail -1 gpurun_out/sk_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
(cd ab/base_tree && timeout -k 10 300 python3 bench.py --global-batch 32 --steps 10 --warmup 3 --no-cpu-baseline) > gpurun_out/sk_base.log 2>&1 || { tail -5 gpurun_out/sk_base.log; exit 1; }
echo "base $(tail -1 gpurun_out/sk_base.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
