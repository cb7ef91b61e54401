"""Average rocprofv3 PMC counters per kernel (development tool).

usage: python scripts/pmc_summary.py DIR   (a rocprofv3 -d DIR output tree)
Each counter is averaged over the dispatches that recorded it.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0]
                c = r["Counter_Name"]
                acc[k][c] += float(r["Counter_Value"])
                disp[k][c].add((f, r["Dispatch_Id"]))
    for k in sorted(acc):
        vals = "  ".join(f"{c}={v / len(disp[k][c]):.4g}" for c, v in sorted(acc[k].items()))
        print(f"{k}: {vals}")


if __name__ == "__main__":
    main(sys.argv[1])
