#!/usr/bin/env python3
"""Time every decoder variant (QHUFF_DECODER) on a BASELINE-shaped batch and
check each against the plaintext (development tool, one GPU).  Loads the
development build (make dev -> nghttp3_amd/lib/libqhuff_dev.so), which holds
every variant; the product library ships peek11s and wring11x16r2 only.

Usage: python scripts/dec_variants.py [--n N] [--alphabet A|U] [--reps R]
         [--kinds fsm,peek11,...]
Prints one JSON line per variant: kernel avg us (HIP events), plaintext
GiB/s of the kernel alone, bit_exact.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
_DEV = os.path.join(ROOT, "nghttp3_amd", "lib", "libqhuff_dev.so")
if os.path.exists(_DEV):  # (else the product library: its kPeekVariants entries)
    os.environ.setdefault("QHUFF_LIB", _DEV)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--lo", type=int, default=8)
    ap.add_argument("--hi", type=int, default=256)
    ap.add_argument("--alphabet", default="A")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--kinds", default="wring11x16r2,peek11s")
    ap.add_argument("--zipf", action="store_true", help="config 5 lengths (Zipf 1..4096)")
    args = ap.parse_args()
    import torch
    from nghttp3_amd import HuffmanBatchCodec, synth
    from nghttp3_amd import qpack_huffman as q

    alph = synth.ALPHABET_A if args.alphabet == "A" else synth.ALPHABET_U
    base = HuffmanBatchCodec(device=0)
    if args.zipf:
        zl = synth.zipf_lengths(0x5EED0005, args.n, 1, 4096, 1.2)
        spans, total = base.spans_to_device(zl)
        src = base.synth_fill(0x5EED0005, 0, total, alph)
    else:
        src, spans, total = base.synth(0x5EED0003, args.n, args.lo, args.hi, alph)
    n = args.n
    ln = spans[:, 1] & 0xFFFFFFFF
    bound = int(((ln * 30 + 7) // 8).sum().item())
    enc = torch.empty(bound, dtype=torch.uint8, device="cuda")
    eout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    base.encode_dev(src, spans, enc, eout)
    torch.cuda.synchronize()
    elen = eout[:, 1] & 0xFFFFFFFF
    cap = int(q.decode_slot_size(elen).sum().item())
    ebytes = int(elen.sum().item())
    dec = torch.empty(cap, dtype=torch.uint8, device="cuda")
    dout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    rep_p = torch.repeat_interleave(spans[:, 0], ln)
    pos = torch.arange(total, device="cuda", dtype=torch.int64) - rep_p
    for kind in args.kinds.split(","):
        os.environ["QHUFF_DECODER"] = kind
        c = HuffmanBatchCodec(device=0)
        dec.fill_(0)
        c.decode_dev(enc, eout, dec, dout)
        c.enable_timing(True)
        for _ in range(args.reps):
            c.decode_dev(enc, eout, dec, dout)
        kt = c.kernel_times()
        c.enable_timing(False)
        st = c.stats()
        ok = st["n_errors"] == 0 and bool(((dout[:, 1] & 0xFFFFFFFF) == ln).all())
        if ok:
            rep_d = torch.repeat_interleave(dout[:, 0], ln)
            ok = bool((dec[rep_d + pos] == src[:total]).all())
        ks = {k: round(ms / max(cnt, 1) * 1e3, 2) for k, (cnt, ms) in kt.items()}
        main_us = max(ks.values())
        print(json.dumps({"kind": kind, "alphabet": args.alphabet, "zipf": args.zipf, "n": n, "kernels_us": ks,
                          "plain_GiBps": round(total / (main_us * 1e-6) / 2**30, 1),
                          "algo_GBps": round((total + ebytes + 32 * n) / (main_us * 1e-6) / 1e9, 1),
                          "bit_exact": ok}), flush=True)
        c.close()


if __name__ == "__main__":
    main()
