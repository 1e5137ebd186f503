#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass, each under its own kill timeout) over
# tools/kprof.py kernels.  Usage: bash tools/pmc_passes.sh OUTDIR kernel [kernel ...]
# Passes: A/B = SQ instruction / cycle counters (<= 8 SQ each), C = FETCH_SIZE (3 TCC),
# D = WRITE_SIZE (2 TCC): HBM-side bytes per dispatch (gfx950: KiB units, see pmc_summary.py).
set -o pipefail
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY"
PB="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
PC="FETCH_SIZE"
PD="WRITE_SIZE"
for k in "$@"; do
  i=0
  for P in "$PA" "$PB" "$PC" "$PD"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $out/${k}_p$i -o run -- python3 tools/kprof.py $k > $out/${k}_p$i.log 2>&1 || { echo "pass $k p$i failed rc=$?"; exit 1; }
  done
done
echo done
