#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass, each under its own kill timeout) over
# tools/kprof.py kernels.  Usage: bash tools/pmc_passes.sh OUTDIR kernel [kernel ...]
set -o pipefail
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY"
PB="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
for k in "$@"; do
  i=0
  for P in "$PA" "$PB"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $out/${k}_p$i -o run -- python3 tools/kprof.py $k > $out/${k}_p$i.log 2>&1 || { echo "pass $k p$i failed rc=$?"; exit 1; }
  done
done
echo done
