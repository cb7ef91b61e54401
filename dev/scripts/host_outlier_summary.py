#!/usr/bin/env python3
"""Development: per decode_host call of host_outlier_trace.py, what the
trace shows inside it (copies, kernels, the biggest idle gap of the GPU).
  python3 dev/scripts/host_outlier_summary.py OUT   (OUT/calls.json, OUT/**/run_results.db)"""
import glob
import json
import os
import sqlite3
import sys


def main():
    out = sys.argv[1]
    meta = json.load(open(os.path.join(out, "calls.json")))
    db = sqlite3.connect(glob.glob(os.path.join(out, "**", "*results.db"), recursive=True)[0])
    ev = []
    for s, e, name, size, tid in db.execute("select start, end, name, size, tid from memory_copies"):
        ev.append((s, e, "H2D" if "HOST_TO_DEVICE" in name else "D2H" if "DEVICE_TO_HOST" in name else name,
                   size, tid))
    for s, e, name, tid in db.execute("select start, end, name, tid from kernels"):
        ev.append((s, e, name.split("(")[0].replace("__amd_rocclr_", "rocclr:")[:28], 0, tid))
    ev.sort()
    t_min = min(x[0] for x in ev)
    off = 0  # trace clock vs CLOCK_MONOTONIC: try both
    calls = meta["calls"]
    def inside(c, o):
        return [x for x in ev if x[0] >= c[0] + o and x[1] <= c[1] + o]
    hits0 = sum(len(inside(c, 0)) for c in calls)
    hits1 = sum(len(inside(c, meta["boottime_minus_monotonic_ns"])) for c in calls)
    off = 0 if hits0 >= hits1 else meta["boottime_minus_monotonic_ns"]
    print("clock:", "monotonic" if off == 0 else "boottime", "events matched", max(hits0, hits1), "of", len(ev))
    for k, c in enumerate(calls):
        xs = inside(c, off)
        wall = (c[1] - c[0]) / 1e6
        if not xs:
            print(f"call {k}: {wall:.2f} ms, no events")
            continue
        first = (xs[0][0] - c[0] - off) / 1e6
        last = (c[1] + off - max(x[1] for x in xs)) / 1e6
        # busy union and biggest gap
        gaps = []
        end = xs[0][1]
        for x in xs[1:]:
            if x[0] > end:
                gaps.append(((x[0] - end) / 1e6, (end - c[0] - off) / 1e6, x[2]))
            end = max(end, x[1])
        gaps.sort(reverse=True)
        h2d = sum(x[3] for x in xs if x[2] == "H2D") / 1e6
        d2h = sum(x[3] for x in xs if x[2] == "D2H") / 1e6
        print(f"call {k}: wall {wall:.2f} ms  first event +{first:.2f}  idle after last {last:.2f}  "
              f"events {len(xs)}  H2D {h2d:.0f} MB D2H {d2h:.0f} MB  gaps(ms, at, next) "
              + ", ".join(f"{g:.2f}@{a:.2f}->{nm}" for g, a, nm in gaps[:3]))


if __name__ == "__main__":
    main()
