"""HBM traffic per launch of every kernel, from rocprofv3 FETCH_SIZE and
WRITE_SIZE passes (scripts/gpu_check.sh pmc) -> profiles/pmc_traffic.json,
which bench.py reads for roofline.traffic.

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE counts
TCC_EA0_RDREQ x 64 B while the requests of wide reads are 128 B, so it reports
half the bytes of a wide streaming read; it is doubled here.  WRITE_SIZE is
exact for 16-byte-per-lane stores.  Both are in KiB.

usage: python scripts/pmc_traffic.py OUTDIR [n] [alphabet]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(d, n=1 << 20, alphabet="A"):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
                k = k.split("::")[-1]
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kernels = {}
    for k, c in acc.items():
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        fetch = 2 * 1024 * sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
        write = 1024 * sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
        kernels[k] = {"fetch_bytes": round(fetch), "write_bytes": round(write),
                      "hbm_bytes_per_launch": round(fetch + write)}
    out = {"n": n, "alphabet": alphabet, "source": os.path.relpath(d, ROOT),
           "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); KiB -> bytes",
           "kernels": kernels}
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], *(int(sys.argv[2]),) if len(sys.argv) > 2 else ())
