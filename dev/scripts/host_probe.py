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
    r = bench.leg_host_path(torch, codec, q, enc, eout, eb, total, n, dev)
    print(json.dumps({"lib": os.environ.get("QHUFF_LIB", "default"), "probe_both_ms": r["probe"]["both_ms"],
                      "pinned": r["pinned"], "pageable_ms": r["pageable"]["ms"]}))


if __name__ == "__main__":
    main()
