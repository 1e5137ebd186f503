"""HBM traffic per launch of the BERT-layer GEMMs from two rocprofv3 PMC passes of bench.py.

Collect (separate passes: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass; no trace
domains beside --kernel-trace):
  rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- python bench.py ...
  rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- python bench.py ...
Then:
  python tools/pmc_traffic.py gpurun_out/pmc_f/run_counter_collection.csv gpurun_out/pmc_w/run_counter_collection.csv \
      --out profiles/r1_gemm_traffic.json

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes of a wide
coalesced read (128-B requests tallied at 64 B), so bytes = (2 * FETCH_SIZE + WRITE_SIZE) KiB.
bench.py reports the per-launch figure as roofline.traffic.
"""
import argparse
import csv
import json
import re
from collections import defaultdict

GEMM = re.compile(r"mmu::gemm_(big|small|pipe|wide)_kernel")


def per_dispatch(path, counter):
    """per-dispatch counter sums of the BERT-layer GEMM launches: big-tile mmu_gemm kernels
    dispatched between an embedding forward and the next embedding backward (the encoder
    of one step: the ResNet trunk runs before the one and after the other)"""
    vals = defaultdict(float)
    names = {}
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    inside = False
    for r in rows:
        n = r["Kernel_Name"]
        if "embed_fwd" in n:
            inside = True
        elif "embed_bwd" in n:
            inside = False
        if not inside or not GEMM.search(n) or "gemm_small" in n:
            continue
        d = r["Dispatch_Id"]
        vals[d] += float(r["Counter_Value"])
        names[d] = n
    return vals, names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    f, fn = per_dispatch(a.fetch_csv, "FETCH_SIZE")
    w, wn = per_dispatch(a.write_csv, "WRITE_SIZE")
    gf = [v for d, v in f.items() if GEMM.search(fn[d])]
    gw = [v for d, v in w.items() if GEMM.search(wn[d])]
    if not gf or not gw:
        raise SystemExit("no GEMM dispatches with counters found")
    fk = sum(gf) / len(gf)
    wk = sum(gw) / len(gw)
    per_kernel = defaultdict(lambda: [0, 0.0, 0, 0.0])
    for d, v in f.items():
        if GEMM.search(fn[d]):
            k = per_kernel[fn[d]]
            k[0] += 1
            k[1] += v
    for d, v in w.items():
        if GEMM.search(wn[d]):
            k = per_kernel[wn[d]]
            k[2] += 1
            k[3] += v
    res = {
        "kernel": "mmu_gemm (all BERT-layer GEMMs, fwd + bwd)",
        "launches_fetch_pass": len(gf), "launches_write_pass": len(gw),
        "fetch_size_kib_avg": fk, "write_size_kib_avg": wk,
        "traffic_bytes_per_launch": (2.0 * fk + wk) * 1024.0,
        "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB (gfx950 FETCH_SIZE counts half of wide reads)",
        "per_kernel": {n: {"launches": v[0], "fetch_kib_avg": v[1] / max(v[0], 1), "write_kib_avg": v[3] / max(v[2], 1),
                           "bytes_per_launch": (2.0 * v[1] / max(v[0], 1) + v[3] / max(v[2], 1)) * 1024.0}
                       for n, v in per_kernel.items()},
    }
    js = json.dumps(res, indent=1)
    print(js)
    if a.out:
        open(a.out, "w").write(js + "\n")


if __name__ == "__main__":
    main()
