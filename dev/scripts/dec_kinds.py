#!/usr/bin/env python3
"""Time the shipped decoders (windows, waves, sorted) on config 3 (2^20
strings 8-256 B) or rank 0's config-5 shard (Zipf lengths 1-4096) and check
that their outputs agree (development tool, one GPU).
Usage: python scripts/dec_kinds.py [--zipf] [--alphabet A|U] [--only K,..]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--alphabet", default="A")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--zipf", action="store_true")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import torch
    from nghttp3_amd import HuffmanBatchCodec, synth
    from nghttp3_amd.qpack_huffman import decode_slot_size
    alph = synth.ALPHABET_A if args.alphabet == "A" else synth.ALPHABET_U
    c = HuffmanBatchCodec(device=0)
    if args.zipf:
        n = args.n or 2097152
        zl = synth.zipf_lengths(0x5EED0005, n, 1, 4096, 1.2)
        spans, total = c.spans_to_device(zl)
        src = c.synth_fill(0x5EED0005, 0, total, alph)
    else:
        src, spans, total = c.synth(0x5EED0003, args.n or (1 << 20), 8, 256, alph)
    n = spans.shape[0]
    ln = spans[:, 1] & 0xFFFFFFFF
    enc = torch.zeros(int(((ln * 30 + 7) // 8).sum().item()) + 64, dtype=torch.uint8, device="cuda")
    eout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    c.encode_dev(src, spans, enc, eout)
    elen = eout[:, 1] & 0xFFFFFFFF
    ebytes = int(elen.sum().item())
    cap = int(decode_slot_size(elen).sum().item())
    dec = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    dout = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    kinds = [k for k in ("windows", "waves", "sorted") if not args.only or k in args.only.split(",")]
    for kind in kinds:
        c.set_decoder(kind)
        dec.zero_()
        c.decode_dev(enc, eout, dec, dout)
        st = c.stats()
        alf = round(st["lane_steps"] / (64 * st["wave_steps"]), 4) if st.get("wave_steps") else None
        ok = st["n_errors"] == 0 and st["out_bytes"] == total and \
            bool(((dout[:, 1] & 0xFFFFFFFF) == ln).all())
        # spot-check the bytes of a strided subset
        idx = torch.arange(0, n, 97, device="cuda")
        l = ln[idx]
        pos = torch.arange(int(l.sum().item()), device="cuda") - \
            torch.repeat_interleave(torch.cumsum(l, 0) - l, l)
        ok = ok and bool((dec[torch.repeat_interleave(dout[idx, 0], l) + pos] ==
                          src[torch.repeat_interleave(spans[idx, 0], l) + pos]).all())
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            c.decode_dev(enc, eout, dec, dout)
        e1.record()
        torch.cuda.synchronize()
        wall_us = e0.elapsed_time(e1) * 1e3 / args.reps
        c.enable_timing(True)
        for _ in range(args.reps):
            c.decode_dev(enc, eout, dec, dout)
        kt = c.kernel_times()
        c.enable_timing(False)
        ks = {k: round(ms / max(cnt, 1) * 1e3, 2) for k, (cnt, ms) in kt.items()}
        dk = ks.get("qh_k_dec_peek", 0.0)
        print(json.dumps({"decoder": kind, "alphabet": args.alphabet, "zipf": args.zipf, "n": n,
                          "kernels_us": ks, "sum_us": round(sum(ks.values()), 2), "wall_us": round(wall_us, 2),
                          "wall_GiBps": round(total / (wall_us * 1e-6) / 2**30, 1),
                          "plain_GiBps": round(total / (sum(ks.values()) * 1e-6) / 2**30, 1),
                          "decoder_frac": round((ebytes + total + 32 * n) / (dk * 1e-6) / 8e12, 4) if dk else None,
                          "active_lane_frac": alf, "lane_steps": st.get("lane_steps"), "ok": ok}), flush=True)


if __name__ == "__main__":
    main()
