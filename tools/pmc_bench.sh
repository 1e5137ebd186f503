#!/bin/bash
# PMC counters for every kernel of the real train step: 4 rocprofv3 passes (the
# tools/pmc_passes.sh counter sets, one run each under its own kill timeout) over a 1-step
# bench.py run, then the per-kernel summary and the GEMM HBM traffic file bench.py reports.
# Usage: bash tools/pmc_bench.sh OUTTAG   (writes gpurun_out/pmc_<OUTTAG>/, _summary.txt, _gemm_traffic.json)
set -o pipefail
tag=${1:-bench}
out=gpurun_out/pmc_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY"
PB="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
i=0
for P in "$PA" "$PB" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $out/p$i -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $out/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $out/p$i.log; exit 1; }
  echo "pass $i done"
done
python3 tools/pmc_summary.py $out > gpurun_out/pmc_${tag}_summary.txt
python3 tools/pmc_traffic.py $out/p3/run_counter_collection.csv $out/p4/run_counter_collection.csv --out gpurun_out/pmc_${tag}_gemm_traffic.json
