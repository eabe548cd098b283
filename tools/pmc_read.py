"""Summarise rocprofv3 --pmc counter CSVs of gemm kernels: python tools/pmc_read.py DIR [DIR...]
Prints, per directory, the mean per dispatch of every counter of kernels named gemm*."""
import csv
import glob
import os
import sys
from collections import defaultdict

MATCH = os.environ.get("PMC_MATCH", "gemm")  # kernel-name substrings, '|'-separated (hipBLASLt: Cijk)


def _hit(name):
    return any(m in name for m in MATCH.split("|"))


def read(d):
    vals = defaultdict(list)
    durs = []
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if not _hit(r.get("Kernel_Name", "")):
                continue
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if _hit(r.get("Kernel_Name", "")):
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    return {k: sum(v) / len(v) for k, v in vals.items()}, (sum(durs) / len(durs) if durs else 0.0)


if __name__ == "__main__":
    for d in sys.argv[1:]:
        c, us = read(d)
        print(d, f"mean {us:.1f} us")
        for k in sorted(c):
            print(f"  {k:28s} {c[k]:.4g}")
