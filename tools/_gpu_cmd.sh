set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m pytest tests/test_flava_gpu.py -x -q --timeout 200 --timeout-method thread -k train_entry > gpurun_out/t_flava_train.log 2>&1
rc=$?; tail -5 gpurun_out/t_flava_train.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload flava --steps 10 --warmup 3 > gpurun_out/bench_flava.log 2>&1
rc=$?; tail -1 gpurun_out/bench_flava.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_flava -o run -- python3 bench.py --workload flava --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/prof_flava.log 2>&1
