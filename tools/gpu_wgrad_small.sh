#!/bin/bash
# short-K 1x1 filter gradients at batch 32: timings, then a kernel trace of the mmu calls
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wgs_prof -o wgs -- python3 -u tools/wgrad_small.py --iters 5 > gpurun_out/wgs_prof.log 2>&1 &&
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/wgs_prof/**/*kernel_stats.csv", recursive=True)
for row in csv.DictReader(open(f[0])):
    if "gemm" in row["Name"] or "splitk" in row["Name"]:
        print(row["Name"][:90], row["Calls"], row["AverageNs"])
PY
