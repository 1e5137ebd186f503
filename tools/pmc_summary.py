"""Summarise rocprofv3 PMC csv files written by tools/pmc_passes.sh: per kernel name,
counter values averaged over dispatches (mmu kernels only)."""
import csv
import glob
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            if "mmu::" not in r["Kernel_Name"]:
                continue
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (d, c), v in per.items():
            acc[names[d][:70]][c].append(v)
    for k, cs in acc.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")


if __name__ == "__main__":
    main()
