# split-K A/B at B=32, then PMC passes (SQ instruction / cycle counters, FETCH / WRITE bytes)
# on the attention, LayerNorm and BatchNorm kernels of the current tree
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_r3_splitk_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 700 bash tools/pmc_passes.sh gpurun_out/pmc2 attn_fwd attn_bwd ln_fwd ln_bwd bn_fwd bn_bwd || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc2 > gpurun_out/pmc2_summary.txt 2>&1
tail -3 gpurun_out/pmc2_summary.txt
