#!/usr/bin/env python3
"""Development: whole-encode time (every kernel, HIP events around
encode_dev) of the encoders (windows, fused, waves) of the loaded library
(QHUFF_LIB) on config 3 (alphabet A), the same shape in alphabet U, and
rank 0's config-5 shard (2^21 Zipf strings); bytes checked against the
first encoder's."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from nghttp3_amd import HuffmanBatchCodec, synth
    kinds = (sys.argv[1] if len(sys.argv) > 1 else "windows,fused").split(",")
    lib = os.path.basename(os.environ.get("QHUFF_LIB", "libqhuff.so"))
    c = HuffmanBatchCodec(0)
    cases = []
    for name, alph in (("c3_A", synth.ALPHABET_A), ("c3_U", synth.ALPHABET_U)):
        src, spans, total = c.synth(0x5EED0003, 1 << 20, 8, 256, alph)
        cases.append((name, src, spans, total))
    zl = synth.zipf_lengths(0x5EED0005, 1 << 21, 1, 4096, 1.2)
    spans, total = c.spans_to_device(zl)
    cases.append(("c5_shard", c.synth_fill(0x5EED0005, 0, total, synth.ALPHABET_A), spans, total))
    for name, src, spans, total in cases:
        n = spans.shape[0]
        ln = spans[:, 1] & 0xFFFFFFFF
        bound = int(((ln * 30 + 7) // 8).sum().item()) + 64
        ref = None
        for kind in kinds:
            c.set_encoder(kind)
            enc = torch.zeros(bound, dtype=torch.uint8, device="cuda")
            eout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
            c.encode_dev(src, spans, enc, eout)
            torch.cuda.synchronize()
            e = int((eout[:, 1] & 0xFFFFFFFF).sum().item())
            if ref is None:
                ref = (enc[:e].clone(), eout.clone())
                ok = True
            else:
                ok = bool(torch.equal(enc[:e], ref[0][:e])) and bool(torch.equal(eout, ref[1]))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            e0.record()
            for _ in range(reps):
                c.encode_dev(src, spans, enc, eout)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            print(json.dumps({"lib": lib, "case": name, "encoder": kind, "us": round(us, 1),
                              "GiBps": round(total / us / 1e3 / 1.073741824, 1), "same_bytes": ok}), flush=True)
            del enc, eout
        c.set_encoder("windows")


if __name__ == "__main__":
    main()
