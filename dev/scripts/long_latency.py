#!/usr/bin/env python3
"""Decode time of a few long strings (the wave-per-string path of the sorted
decoder against the lane path), and of rank 0's config-5 shard at several
thresholds (development tool, one GPU).  QHUFF_LONG_MIN is read at context
creation, so each setting gets its own context."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(lmin, src, spans, total, label, reps=5, decoder="sorted"):
    import torch
    from nghttp3_amd import HuffmanBatchCodec
    from nghttp3_amd.qpack_huffman import decode_slot_size
    os.environ["QHUFF_LONG_MIN"] = str(lmin)
    c = HuffmanBatchCodec(device=0)
    c.set_decoder(decoder)
    n = spans.shape[0]
    ln = spans[:, 1] & 0xFFFFFFFF
    enc = torch.zeros(int(((ln * 30 + 7) // 8).sum().item()) + 64, dtype=torch.uint8, device="cuda")
    eout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    c.encode_dev(src, spans, enc, eout)
    cap = int(decode_slot_size(eout[:, 1] & 0xFFFFFFFF).sum().item())
    dec = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    dout = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    c.decode_dev(enc, eout, dec, dout)
    st = c.stats()
    ok = st["n_errors"] == 0 and st["out_bytes"] == total
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        c.decode_dev(enc, eout, dec, dout)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    print(json.dumps({"case": label, "decoder": decoder, "long_min": lmin, "strings": n, "plain_bytes": total, "decode_us": round(us, 1),
                      "GiBps": round(total / (us * 1e-6) / 2**30, 1), "ok": ok}), flush=True)
    c.close()


def sections(reps=10):
    """qh_decode_sections_batch (device form, framing sync included) on one
    field section holding one value of 40,960 encoded bytes (the largest
    nghttp3 accepts), and on 64 such sections."""
    import time
    import numpy as np
    import torch
    from nghttp3_amd import qpack, synth
    text = synth.fill(0x5EED0411, 80000, synth.ALPHABET_A).tobytes()
    lo, hi = 0, len(text)
    while lo < hi:  # the longest value whose representation fits the limit
        mid = (lo + hi + 1) // 2
        if len(qpack.write_indexed_name(0x50, 5, 4, text[:mid])) <= 1 + 3 + 40960:
            lo = mid
        else:
            hi = mid - 1
    sec = b"\x00\x00" + qpack.write_indexed_name(0x50, 5, 4, text[:lo])
    d = qpack.FieldSectionDecoder(0, dtable0=True)
    for nsec in (1, 64):
        data = sec * nsec
        blocks = np.zeros((nsec, 2), dtype=np.int64)
        blocks[:, 0] = np.arange(nsec) * len(sec)
        blocks[:, 1] = len(sec)
        src = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).cuda()
        blk = torch.from_numpy(blocks).cuda()
        g = d.decode_blocks_dev(src, blk)
        torch.cuda.synchronize()
        ok = bool((g["status"][:nsec] == 0).all()) and int((g["strs"][:1, 1] & 0xFFFFFFFF).item()) == lo
        t0 = time.perf_counter()
        for _ in range(reps):
            g = d.decode_blocks_dev(src, blk, g)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) * 1e6 / reps
        print(json.dumps({"case": f"sections: {nsec} x one value of {len(sec) - 7} encoded B "
                                  f"({lo} B decoded)", "us": round(us, 1), "ok": ok}), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "sections":
        return sections()
    import numpy as np
    import torch
    from nghttp3_amd import HuffmanBatchCodec, synth
    base = HuffmanBatchCodec(device=0)
    for nstr, ln in ((1, 65536), (64, 65536), (1024, 8192)):
        spans, total = base.spans_to_device(np.full(nstr, ln, dtype=np.int64))
        src = base.synth_fill(0x5EED0007, 0, total, synth.ALPHABET_A)
        for lmin in (4096, 0):
            run(lmin, src, spans, total, f"{nstr} x {ln} B")
        run(4096, src, spans, total, f"{nstr} x {ln} B", decoder="windows")
    zl = synth.zipf_lengths(0x5EED0005, 2097152, 1, 4096, 1.2)
    spans, total = base.spans_to_device(zl)
    src = base.synth_fill(0x5EED0005, 0, total, synth.ALPHABET_A)
    for lmin in (0, 4096, 2048):
        run(lmin, src, spans, total, "config-5 shard")


if __name__ == "__main__":
    main()
