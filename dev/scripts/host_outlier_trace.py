#!/usr/bin/env python3
"""Development: bench.py's host-memory leg (config 3) with every
decode_host call's start / end on CLOCK_MONOTONIC, for a rocprofv3
--memory-copy-trace --kernel-trace run whose copies and kernels
host_outlier_summary.py then places per call:
  rocprofv3 --memory-copy-trace --kernel-trace -d OUT -o run -- \\
      python3 dev/scripts/host_outlier_trace.py OUT/calls.json"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from nghttp3_amd import HuffmanBatchCodec, synth
    from nghttp3_amd import qpack_huffman as q
    dev = torch.device("cuda", 0)
    codec = HuffmanBatchCodec(device=0)
    src, spans, total = codec.synth(0x5EED0003, 1 << 20, 8, 256, synth.ALPHABET_A)
    n = spans.shape[0]
    ln = spans[:, 1] & 0xFFFFFFFF
    enc = torch.empty(int(((ln * 30 + 7) // 8).sum().item()), dtype=torch.uint8, device=dev)
    eout = torch.empty((n, 2), dtype=torch.int64, device=dev)
    codec.encode_dev(src, spans, enc, eout)
    torch.cuda.synchronize()
    eb = int((eout[:, 1] & 0xFFFFFFFF).sum().item())
    calls = []
    inner = codec.decode_host

    def traced(*a, **k):
        t0 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
        r = inner(*a, **k)
        calls.append([t0, time.clock_gettime_ns(time.CLOCK_MONOTONIC), a[2] is not None])
        return r

    codec.decode_host = traced
    legs = []
    for _ in range(int(os.environ.get("QH_TRACE_LEGS", "1"))):
        r = bench.leg_host_path(torch, codec, q, enc, eout, eb, total, n, dev)
        legs.append({"pinned_ms_each": r["pinned"]["ms_each"], "pageable_ms_each": r["pageable"]["ms_each"]})
        print(json.dumps(legs[-1]), flush=True)
    with open(sys.argv[1], "w") as f:
        json.dump({"calls": calls, "legs": legs,
                   "boottime_minus_monotonic_ns": time.clock_gettime_ns(time.CLOCK_BOOTTIME)
                   - time.clock_gettime_ns(time.CLOCK_MONOTONIC)}, f)


if __name__ == "__main__":
    main()
