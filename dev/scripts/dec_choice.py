#!/usr/bin/env python3
"""Development: whole-decode time (all of its kernels, HIP events around
decode_dev) of decoder variants (QHUFF_DECODER names of the loaded library)
on config 3 (alphabet A), the same shape in alphabet U, and rank 0's config-5
shard (2^21 Zipf strings); bit-exactness checked.  One JSON line each."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from nghttp3_amd import HuffmanBatchCodec, synth
    from nghttp3_amd import qpack_huffman as q
    kinds = (sys.argv[1] if len(sys.argv) > 1 else "peek11s,sorted11").split(",")
    if "peek11s_fixed" not in kinds:
        kinds.append("peek11s_fixed")
    base = HuffmanBatchCodec(0)
    cases = []
    for name, alph in (("c3_A", synth.ALPHABET_A), ("c3_U", synth.ALPHABET_U)):
        src, spans, total = base.synth(0x5EED0003, 1 << 20, 8, 256, alph)
        cases.append((name, src, spans, total))
    zl = synth.zipf_lengths(0x5EED0005, 1 << 21, 1, 4096, 1.2)
    spans, total = base.spans_to_device(zl)
    cases.append(("c5_shard", base.synth_fill(0x5EED0005, 0, total, synth.ALPHABET_A), spans, total))
    for name, src, spans, total in cases:
        n = spans.shape[0]
        ln = spans[:, 1] & 0xFFFFFFFF
        enc = torch.empty(int(((ln * 30 + 7) // 8).sum().item()), dtype=torch.uint8, device="cuda")
        eout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
        base.encode_dev(src, spans, enc, eout)
        torch.cuda.synchronize()
        cap = int(q.decode_slot_size(eout[:, 1] & 0xFFFFFFFF).sum().item())
        dec = torch.empty(cap, dtype=torch.uint8, device="cuda")
        dout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
        for kind in kinds:
            os.environ["QHUFF_DECODER"] = kind
            c = HuffmanBatchCodec(0)
            c.decode_dev(enc, eout, dec, dout)
            torch.cuda.synchronize()
            ok = bool(((dout[:, 1] & 0xFFFFFFFF) == ln).all()) and bool(((dout[:, 1] >> 32) == 0).all())
            i = torch.randint(0, n, (4096,), device="cuda")
            ok = ok and all(bool((dec[int(dout[j, 0]):int(dout[j, 0]) + int(ln[j])] ==
                                  src[int(spans[j, 0]):int(spans[j, 0]) + int(ln[j])]).all()) for j in i[:64].tolist())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            e0.record()
            for _ in range(reps):
                c.decode_dev(enc, eout, dec, dout)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            print(json.dumps({"case": name, "decoder": kind, "us": round(us, 1),
                              "GiBps": round(total / us / 1e3 / 1.073741824, 1), "ok": ok}), flush=True)
            c.close()
        del enc, dec, dout, eout


if __name__ == "__main__":
    main()
