#!/usr/bin/env python3
"""Lock-step iteration counts of the window decoders (development tool).

Runs the instrumented build (make stamps: QH_STEP_COUNTS=1) on bench.py's
config-3 batch (and alphabet U, and rank 0's config-5 shard) and writes
gpurun_out/<tag>/decoder_steps.json (copied to profiles/<tag>/): per workload and decoder, lane_steps
(iterations run by lanes, 16 table lookups each), wave_steps (per window,
each wave's longest lane) and the active-lane fraction.  bench.py reads it
for roofline.secondary (the decoder's LDS lookups per launch).
Usage: QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so python scripts/decoder_steps.py TAG"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    tag = sys.argv[1]
    import torch
    from nghttp3_amd import HuffmanBatchCodec, _lib, synth
    from nghttp3_amd.qpack_huffman import decode_slot_size
    assert "stamps" in _lib.LIB_PATH, "set QHUFF_LIB to the stamps build"
    c = HuffmanBatchCodec(device=0)
    res = {"lib": "libqhuff_stamps.so (QH_STEP_COUNTS=1)", "workloads": {}}
    for name in ("config3_A", "config3_U", "config5_rank0_of_8"):
        if name.startswith("config5"):
            zl = synth.zipf_lengths(0x5EED0005, 2097152, 1, 4096, 1.2)
            spans, total = c.spans_to_device(zl)
            src = c.synth_fill(0x5EED0005, 0, total, synth.ALPHABET_A)
        else:
            alph = synth.ALPHABET_A if name.endswith("A") else synth.ALPHABET_U
            src, spans, total = c.synth(0x5EED0003, 1 << 20, 8, 256, alph)
        n = spans.shape[0]
        ln = spans[:, 1] & 0xFFFFFFFF
        enc = torch.zeros(int(((ln * 30 + 7) // 8).sum().item()) + 64, dtype=torch.uint8, device="cuda")
        eout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
        c.encode_dev(src, spans, enc, eout)
        cap = int(decode_slot_size(eout[:, 1] & 0xFFFFFFFF).sum().item())
        dec = torch.zeros(cap, dtype=torch.uint8, device="cuda")
        dout = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
        w = {"strings": n, "plain_bytes": total}
        for kind in ("sorted", "windows"):
            c.set_decoder(kind)
            c.decode_dev(enc, eout, dec, dout)
            st = c.stats()
            w[kind] = {"lane_steps": st["lane_steps"], "wave_steps": st["wave_steps"],
                       "lookups": 16 * st["lane_steps"],
                       "active_lane_frac": round(st["lane_steps"] / (64 * st["wave_steps"]), 4),
                       "ok": st["n_errors"] == 0 and st["out_bytes"] == total}
        res["workloads"][name] = w
        print(name, json.dumps(w), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out", tag), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", tag, "decoder_steps.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
