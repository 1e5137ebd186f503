"""Summarise a rocprofv3 --kernel-trace CSV for ONE steady-state training step.

The step window is the span between the last two launches of the fused BertAdam
update kernel (one per optimizer step), so MIOpen's first-call solver search and
the warm-up never enter the numbers.

  python tools/prof_summary.py gpurun_out/prof1/run_kernel_trace.csv [--md out.md]
  python tools/prof_summary.py gpurun_out/prof1/run_results.db [--md out.md]
"""
import argparse
import csv
import re
from collections import defaultdict

CATS = [
    ("mmu GEMM (BERT layers + ResNet 1x1 / 3x3 convs)", r"mmu::gemm_|gemm_(small|big)_kernel|mmu::splitk"),
    ("mmu attention", r"mmu::attn_|mmu::seqattn_"),
    ("mmu LayerNorm", r"mmu::ln_|ln_fwd_kernel|ln_fwd2_kernel|ln_fwd32_kernel|ln_bwd_kernel|ln_bwd_res"),
    ("mmu stem conv (7x7 / 2)", r"mmu::stem_|stem_(fwd|wgrad)"),
    ("mmu embed / pool", r"mmu::embed|mmu::row_pool|embed_fwd_kernel|embed_bwd"),
    ("mmu BertAdam", r"mmu::adam"),
    ("mmu BatchNorm (ResNet)", r"mmu::bn_|bn_(stats|apply|bwd)"),
    ("mmu colsum", r"mmu::colsum"),
    ("ResNet conv (MIOpen / CK)", r"conv|igemm|gtcx|ck::tensor_operation"),
    ("ResNet batch-norm (MIOpen)", r"BatchNorm"),
    ("torch elementwise / reduce", r"at::native|elementwise|reduce_kernel"),
    ("GEMM library (hipBLASLt/rocBLAS)", r"Cijk|rocblas|hipblas"),
    ("copies / fills", r"rocclr"),
]


def category(name):
    for cat, pat in CATS:
        if re.search(pat, name):
            return cat
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--md", default=None)
    ap.add_argument("--marker", default="adam_update_kernel",
                    help="a kernel launched once per step (FLAVA / torch AdamW: nll_loss_forward)")
    a = ap.parse_args()
    if a.trace.endswith(".db"):  # rocprofv3's default rocpd (sqlite) output
        import sqlite3
        cur = sqlite3.connect(a.trace).execute("select name, start, end from kernels")
        rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e} for n, s, e in cur]
    else:
        rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(adam) < 2:
        raise SystemExit("need >= 2 optimizer steps in the trace")
    lo, hi = adam[-2] + 1, adam[-1] + 1
    win = rows[lo:hi]
    t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
    wall = (t1 - t0) / 1e6
    per_kernel = defaultdict(lambda: [0, 0.0])
    per_cat = defaultdict(lambda: [0, 0.0])
    for r in win:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        k = r["Kernel_Name"]
        per_kernel[k][0] += 1
        per_kernel[k][1] += d
        c = category(k)
        per_cat[c][0] += 1
        per_cat[c][1] += d
    busy = sum(v[1] for v in per_cat.values())
    lines = [f"# One steady-state training step (between the last two `{a.marker}` launches)", "",
             f"step wall (first dispatch start -> last end): {wall:.2f} ms; summed kernel time {busy:.2f} ms; "
             f"dispatches {len(win)}", "", "| category | launches | ms | % of kernel time |", "|---|---|---|---|"]
    for c, (n, ms) in sorted(per_cat.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"| {c} | {n} | {ms:.2f} | {100 * ms / busy:.1f} |")
    # the launches bench.py's roofline times with HIP events: the big-tile GEMMs between the
    # embedding forward and the embedding backward (the encoder of the step)
    inside, bert = False, []
    for r in win:
        k = r["Kernel_Name"]
        if "embed_fwd" in k:
            inside = True
        elif "embed_bwd" in k:
            inside = False
        elif inside and re.search(r"gemm_(big|wide)_kernel", k):
            bert.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    if bert:
        lines += ["", f"BERT-layer GEMM launches (big-tile `mmu_gemm` between embed_fwd and embed_bwd; what "
                      f"bench.py's roofline times with HIP events): {len(bert)} launches, mean "
                      f"{sum(bert) / len(bert):.1f} us, total {sum(bert) / 1e3:.2f} ms"]
    lines += ["", "| kernel | launches | total ms | avg us |", "|---|---|---|---|"]
    for k, (n, ms) in sorted(per_kernel.items(), key=lambda kv: -kv[1][1])[:40]:
        lines.append(f"| `{k[:120]}` | {n} | {ms:.2f} | {1000 * ms / n:.1f} |")
    out = "\n".join(lines)
    print(out)
    if a.md:
        with open(a.md, "w") as f:
            f.write(out + "\n")


if __name__ == "__main__":
    main()
