#!/bin/bash
# round 6, first GPU call: box facts, the whole GPU suite (-s: parity prints), the residue-off
# parity arm, bench N=1 (driver form), batch 32 (graph auto), and the --gpus 2 self-launch rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r6a
{ echo "nproc $(nproc)"; python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())";
  cat /sys/fs/cgroup/cpu.max 2>&1; echo "OMP=$OMP_NUM_THREADS"; } > ${o}_box.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > ${o}_tests.log 2>&1 \
  || { grep -E "Error|FAILED|assert" ${o}_tests.log | head -30; exit 1; }
tail -1 ${o}_tests.log
MMU_STREAM_RESIDUE=0 timeout -k 10 600 python -u -m pytest tests/test_mmbt_gpu.py -m gpu -v -s --timeout 300 \
  --timeout-method thread -k "full_t508c or small_b8" > ${o}_nores_tests.log 2>&1; echo "nores rc=$?"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > ${o}_smoke.log 2>&1 || { tail -20 ${o}_smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > ${o}_bench.log 2>&1 || { tail -20 ${o}_bench.log; exit 1; }
tail -1 ${o}_bench.log
timeout -k 10 300 python -u bench.py --global-batch 32 --steps 20 --warmup 3 --no-cpu-baseline > ${o}_b32.log 2>&1 || { tail -20 ${o}_b32.log; exit 1; }
tail -1 ${o}_b32.log
MMU_BENCH_BACKEND=gloo MMU_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -u bench.py --gpus 2 --global-batch 32 --steps 2 \
  --warmup 1 --no-cpu-baseline > ${o}_n2.log 2>&1 || { tail -20 ${o}_n2.log; exit 1; }
tail -1 ${o}_n2.log
