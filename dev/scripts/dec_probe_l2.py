#!/usr/bin/env python3
"""Development probe: the window decoder on config 3's encoded strings, and
on the same number of spans that all point into the first K encoded strings
(input always L2-resident), to price the input side of the decode."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from nghttp3_amd import HuffmanBatchCodec, synth
    from nghttp3_amd import qpack_huffman as q
    c = HuffmanBatchCodec(device=0)
    n = 1 << 20
    src, spans, total = c.synth(0x5EED0003, n, 8, 256, synth.ALPHABET_A)
    ln = spans[:, 1] & 0xFFFFFFFF
    enc = torch.empty(int(((ln * 30 + 7) // 8).sum().item()), dtype=torch.uint8, device="cuda")
    eout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    c.encode_dev(src, spans, enc, eout)
    torch.cuda.synchronize()
    for k in (0, 4096, 65536):
        e2 = eout.clone()
        if k:
            e2[:, 0] = eout[torch.arange(n, device="cuda") % k, 0]
            e2[:, 1] = eout[torch.arange(n, device="cuda") % k, 1]
        elen = e2[:, 1] & 0xFFFFFFFF
        cap = int(q.decode_slot_size(elen).sum().item())
        dec = torch.empty(cap, dtype=torch.uint8, device="cuda")
        dout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
        c.decode_dev(enc, e2, dec, dout)
        c.enable_timing(True)
        for _ in range(5):
            c.decode_dev(enc, e2, dec, dout)
        kt = c.kernel_times()
        c.enable_timing(False)
        us = {a: round(ms / max(cnt, 1) * 1e3, 1) for a, (cnt, ms) in kt.items()}
        ok = bool(((dout[:, 1] >> 32) == 0).all())
        print(json.dumps({"input_strings": k or n, "plain": int((dout[:, 1] & 0xFFFFFFFF).sum().item()),
                          "kernels_us": us, "ok": ok}), flush=True)


if __name__ == "__main__":
    main()
