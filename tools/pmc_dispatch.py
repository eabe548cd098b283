"""Per-dispatch counter values of kernels whose name contains a substring, in dispatch order
(rocprofv3 --pmc CSVs): python tools/pmc_dispatch.py DIR [substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "gemm"
    rows = defaultdict(dict)
    names = {}
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if sub not in r.get("Kernel_Name", ""):
                continue
            k = int(r["Dispatch_Id"])
            rows[k][r["Counter_Name"]] = rows[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[k] = r["Kernel_Name"][:60]
    for k in sorted(rows):
        print(k, names[k], {c: round(v / 1e6, 2) for c, v in sorted(rows[k].items())})


if __name__ == "__main__":
    main()
