#!/usr/bin/env python3
"""Development: timeline of one host-memory decode (the last single-context
call of dev/scripts/host_path_trace.py) from a rocprofv3 memory-copy +
kernel trace: per copy and kernel, start / end relative to the call's first
event (us), direction or name, bytes if known; and the overlap of H2D, D2H
and kernels.  Usage: host_trace_summary.py TRACE_DIR"""
import csv
import os
import sys


def load(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    d = sys.argv[1]
    cp = load(os.path.join(d, "run_memory_copy_trace.csv"))
    kt = load(os.path.join(d, "run_kernel_trace.csv"))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
           "H2D" if "HOST_TO_DEVICE" in r["Direction"] else "D2H" if "DEVICE_TO_HOST" in r["Direction"] else r["Direction"],
           r.get("Stream_Id")) for r in cp]
    ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K:" + r["Kernel_Name"][:40], r.get("Queue_Id")) for r in kt]
    ev.sort()
    # calls: a qh_k_dec_reserve launch starts each slice; group by gaps > 200 us
    groups, cur = [], []
    for e in ev:
        if cur and e[0] - max(x[1] for x in cur) > 200_000:
            groups.append(cur)
            cur = []
        cur.append(e)
    groups.append(cur)
    # the single-context calls are the 6 groups after setup; take the 5th
    cand = [g for g in groups if any("dense_pack" in x[2] for x in g)]
    g = cand[5] if len(cand) > 5 else cand[-1]
    t0 = g[0][0]
    span = (max(x[1] for x in g) - t0) / 1e3
    print(f"call: {len(g)} events, {span:.1f} us")
    for s, e, name, q in g:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {name}  q/stream={q}")
    def busy(pred):
        iv = sorted((s, e) for s, e, n, _ in g if pred(n))
        tot, ce = 0, None
        for s, e in iv:
            if ce is None or s > ce:
                tot += e - s
                ce = e
            elif e > ce:
                tot += e - ce
                ce = e
        return tot / 1e3
    print("busy us: H2D %.1f  D2H %.1f  kernels %.1f" % (busy(lambda n: n == "H2D"), busy(lambda n: n == "D2H"),
                                                          busy(lambda n: n.startswith("K:"))))


if __name__ == "__main__":
    main()
