#!/usr/bin/env python3
"""Time the region codes pass (qh_k_enc_region) of the library QHUFF_LIB points
at, on config 3's batch, and print its kernel times and stats (a QH_RG_PROBE
build counts streamed rounds / lane-path strings in lane_steps / wave_steps).
Development tool, one GPU.  Usage: QHUFF_LIB=... python dev/scripts/region_probe.py [--alphabet A|U] [--zipf]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--alphabet", default="A")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--zipf", action="store_true")
    ap.add_argument("--encoder", default="region")
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
    c.set_encoder(args.encoder)
    enc = torch.zeros(bound, dtype=torch.uint8, device="cuda")
    eout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    c.encode_dev(src, spans, enc, eout)
    st = c.stats()
    c.enable_timing(True)
    for _ in range(args.reps):
        c.encode_dev(src, spans, enc, eout)
    kt = c.kernel_times()
    c.enable_timing(False)
    torch.cuda.synchronize()
    ks = {k: round(ms / max(cnt, 1) * 1e3, 2) for k, (cnt, ms) in kt.items()}
    print(json.dumps({"lib": os.environ.get("QHUFF_LIB", "default"), "alphabet": args.alphabet,
                      "zipf": args.zipf, "kernels_us": ks, "stats": st}))


if __name__ == "__main__":
    main()
