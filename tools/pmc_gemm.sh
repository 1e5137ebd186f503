# SQ + TCC counter passes over single GEMM kernels (tools/kprof.py); each pass its own run.
set -o pipefail
out=gpurun_out/pmc_gemm
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY"
PB="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
PC="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
for k in "$@"; do
  i=0
  for P in "$PA" "$PB" "$PC"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $out/${k}_p$i -o run -- python3 tools/kprof.py $k > $out/${k}_p$i.log 2>&1 || { echo "pass $k p$i failed rc=$?"; tail -5 $out/${k}_p$i.log; exit 1; }
  done
done
python3 tools/pmc_summary.py $out
