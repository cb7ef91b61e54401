#!/usr/bin/env python3
"""Development: the trace events inside one decode_host call of
host_outlier_trace.py (copies and kernels, ms from the call's start).
  python3 dev/scripts/host_call_timeline.py OUT CALL [CALL ...]"""
import glob
import json
import sqlite3
import sys


def main():
    out = sys.argv[1]
    meta = json.load(open(out + "/calls.json"))
    db = sqlite3.connect(glob.glob(out + "/**/*results.db", recursive=True)[0])
    ev = []
    for s, e, name, size in db.execute("select start, end, name, size from memory_copies"):
        ev.append((s, e, "H2D" if "HOST_TO" in name else name, size))
    for s, e, name in db.execute("select start, end, name from kernels"):
        ev.append((s, e, name.split("(")[0][-24:], 0))
    ev.sort()
    for k in map(int, sys.argv[2:]):
        c = meta["calls"][k]
        print("call", k, (c[1] - c[0]) / 1e6, "ms")
        for x in ev:
            if x[0] >= c[0] and x[1] <= c[1]:
                print(f"  +{(x[0] - c[0]) / 1e6:7.3f} .. +{(x[1] - c[0]) / 1e6:7.3f}  {x[2]:24s} {x[3] / 1e6:8.2f}MB")


if __name__ == "__main__":
    main()
