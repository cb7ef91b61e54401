#!/usr/bin/env python3
"""Time the shipped encoders (windows, waves, fused) on a BASELINE-shaped batch and
check their bytes agree (development tool, one GPU).
Usage: python scripts/enc_variants.py [--n N] [--alphabet A|U] [--zipf]"""
import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--alphabet", default="A")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--zipf", action="store_true")
    ap.add_argument("--only", default="", help="comma-separated encoders (default: all)")
    args = ap.parse_args()
    import torch
    from nghttp3_amd import HuffmanBatchCodec, synth
    alph = synth.ALPHABET_A if args.alphabet == "A" else synth.ALPHABET_U
    c = HuffmanBatchCodec(device=0)
    if args.zipf:
        zl = synth.zipf_lengths(0x5EED0005, args.n, 1, 4096, 1.2)
        spans, total = c.spans_to_device(zl)
        src = c.synth_fill(0x5EED0005, 0, total, alph)
    else:
        src, spans, total = c.synth(0x5EED0003, args.n, 8, 256, alph)
    n = spans.shape[0]
    ln = spans[:, 1] & 0xFFFFFFFF
    bound = int(((ln * 30 + 7) // 8).sum().item())
    ref = None
    kinds = [k for k in ("windows", "waves", "fused") if not args.only or k in args.only.split(",")]
    for kind in kinds:
        c.set_encoder(kind)
        enc = torch.zeros(bound, dtype=torch.uint8, device="cuda")
        eout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
        c.encode_dev(src, spans, enc, eout)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            c.encode_dev(src, spans, enc, eout)
        e1.record()
        torch.cuda.synchronize()
        wall_us = e0.elapsed_time(e1) * 1e3 / args.reps
        c.enable_timing(True)
        for _ in range(args.reps):
            c.encode_dev(src, spans, enc, eout)
        kt = c.kernel_times()
        c.enable_timing(False)
        torch.cuda.synchronize()
        eb = int((eout[:, 1] & 0xFFFFFFFF).sum().item())
        got = (enc[:eb].clone(), eout.clone())
        same = True if ref is None else bool(torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]))
        ref = ref or got
        ks = {k: round(ms / max(cnt, 1) * 1e3, 2) for k, (cnt, ms) in kt.items()}
        print(json.dumps({"encoder": kind, "alphabet": args.alphabet, "zipf": args.zipf, "n": n,
                          "kernels_us": ks, "sum_us": round(sum(ks.values()), 2), "wall_us": round(wall_us, 2),
                          "plain_GiBps": round(total / (sum(ks.values()) * 1e-6) / 2**30, 1),
                          "same_as_windows": same,
                          "sha": hashlib.sha256(got[0].cpu().numpy().tobytes() + got[1].cpu().numpy().tobytes())
                          .hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
