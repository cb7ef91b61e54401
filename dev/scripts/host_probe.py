#!/usr/bin/env python3
"""The host-memory decode leg of bench.py (pinned and pageable, with its
copy-engine probe) on config 3, for the library QHUFF_LIB points at.
Development tool, one GPU."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    node = os.environ.get("QH_PROBE_NODE")  # (bind the leg to this NUMA node instead of the GPU's)
    if node is not None:
        def forced(torch_, dev_, _n=int(node)):
            cpus = set()
            for part in open(f"/sys/devices/system/node/node{_n}/cpulist").read().strip().split(","):
                lo, _, hi = part.partition("-")
                cpus.update(range(int(lo), int(hi or lo) + 1))
            return _n, cpus
        bench._gpu_numa = forced
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
    # (QH_PRE: bench legs run first, to find which one changes the host leg)
    pre = os.environ.get("QH_PRE", "").split("+")
    if "cold" in pre or "dec" in pre:
        from nghttp3_amd.qpack_huffman import decode_slot_size
        cap = int(decode_slot_size((eout[:, 1] & 0xFFFFFFFF).cpu().numpy()).sum())
        dec = torch.empty(cap + 64, dtype=torch.uint8, device=dev)
        dout = torch.empty((n, 2), dtype=torch.int64, device=dev)
        for _ in range(20):
            codec.decode_dev(enc, eout, dec, dout)
        if "cold" in pre:
            bench.leg_cold(torch, codec, src, spans, enc, eout, dec, dout, total, dev)
        if "dense" in pre:
            for _ in range(20):
                codec.decode_dev(enc, eout, dec, dout, dense=True)
    if "two" in pre:
        c2 = HuffmanBatchCodec(device=0, stream=torch.cuda.Stream(dev))
        e2, o2 = torch.empty_like(enc), torch.empty_like(eout)
        c2.encode_dev(src, spans, e2, o2)
        torch.cuda.synchronize()
        del c2, e2, o2
    if "events" in pre:
        codec.enable_timing(True)
        for _ in range(5):
            codec.encode_dev(src, spans, enc, eout)
        codec.kernel_times()
        codec.enable_timing(False)
    torch.cuda.synchronize()
    r = bench.leg_host_path(torch, codec, q, enc, eout, eb, total, n, dev)
    print(json.dumps({"lib": os.environ.get("QHUFF_LIB", "default"), "node": r["gpu_numa_node"],
                      "gpu_node": bench._gpu_numa.__wrapped__ if hasattr(bench._gpu_numa, "__wrapped__") else None,
                      "probe_both_ms": r["probe"]["both_ms"],
                      "pinned": r["pinned"], "pageable_ms": r["pageable"]["ms"]}))


if __name__ == "__main__":
    main()
