"""Summarise rocprofv3 PMC csv files written by tools/pmc_passes.sh: per kernel name,
counter values averaged over dispatches (mmu kernels only), then the derived figures
DESIGN §3 cites, per dispatch:

  dur_us      mean kernel duration from the passes' own kernel traces (profiled: a few %
              slower than un-profiled runs); with the counter means, hbm_GBps is the
              aggregate over every dispatch of that kernel (all shapes)
  hbm_GBps    HBM-side bytes / dur, bytes = (2 * FETCH_SIZE + WRITE_SIZE) KiB * 1024
              (gfx950: FETCH_SIZE counts half the bytes of 16-B streaming reads;
              /opt/skills/guides/MI355X_MICROARCH.md "HBM")
  mfma_util   SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs): the fraction of
              SIMD-cycles with the matrix core busy (GRBM_GUI_ACTIVE sums the 8 XCDs)
  valu_per_mfma, lds_conflict_per_lds, wait_frac (SQ_WAIT_ANY / SQ_WAVE_CYCLES)

  python tools/pmc_summary.py gpurun_out/pmc [--raw]
"""
import csv
import glob
import sys
from collections import defaultdict


def _mmu(name):
    return "mmu::" in name or "_ZN3mmu" in name


def main():
    root = sys.argv[1]
    raw = "--raw" in sys.argv
    acc = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            if not _mmu(r["Kernel_Name"]):
                continue
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (d, c), v in per.items():
            acc[names[d][:70]][c].append(v)
    for f in sorted(glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            if _mmu(r["Kernel_Name"]):
                durs[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    print(f"{'kernel':70s} {'dur_us':>8s} {'hbm_GBps':>9s} {'mfma_util':>9s} {'valu/mfma':>9s} "
          f"{'lds_cfl':>7s} {'wait':>5s}")
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = durs.get(k, [])
        dur = sum(d) / len(d) if d else float("nan")  # mean: counters are means over the same dispatches
        byt = (2 * m.get("FETCH_SIZE", float("nan")) + m.get("WRITE_SIZE", float("nan"))) * 1024
        cyc = m.get("GRBM_GUI_ACTIVE", float("nan")) / 8
        util = m.get("SQ_VALU_MFMA_BUSY_CYCLES", float("nan")) / (cyc * 1024) if cyc else float("nan")
        mf = m.get("SQ_INSTS_MFMA", 0)
        vpm = m.get("SQ_INSTS_VALU", float("nan")) / mf if mf else float("nan")
        lds = m.get("SQ_INSTS_LDS", 0)
        cfl = m.get("SQ_LDS_BANK_CONFLICT", float("nan")) / lds if lds else float("nan")
        wc = m.get("SQ_WAVE_CYCLES", 0)
        wt = m.get("SQ_WAIT_ANY", float("nan")) / wc if wc else float("nan")
        print(f"{k:70s} {dur:8.1f} {byt / (dur * 1e3):9.0f} {util:9.3f} {vpm:9.1f} {cfl:7.3f} {wt:5.2f}")
        if raw:
            for c, v in sorted(cs.items()):
                print(f"   {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")


if __name__ == "__main__":
    main()
