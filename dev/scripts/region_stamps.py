#!/usr/bin/env python3
"""Phase timers of qh_k_enc_region (a QH_STAMPS build: QHUFF_LIB=<it>): cycles
per round of wave 0 of every workgroup, by phase.  Development tool."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
NAMES = {0: "window setup", 1: "DMA wait", 2: "chunk read + gap word", 3: "lookups + scan",
         4: "quads / ORs / pads", 5: "copy-out", 6: "carry", 7: "window tail", 8: "window switch",
         10: "(between windows)", 11: "rounds", 12: "block life (realtime)", 13: "block life (cycles)"}


def main():
    import torch
    from nghttp3_amd import HuffmanBatchCodec, synth, _lib
    c = HuffmanBatchCodec(device=0)
    src, spans, total = c.synth(0x5EED0003, 1 << 20, 8, 256, synth.ALPHABET_A)
    n = spans.shape[0]
    ln = spans[:, 1] & 0xFFFFFFFF
    enc = torch.zeros(int(((ln * 30 + 7) // 8).sum().item()), dtype=torch.uint8, device="cuda")
    eout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    c.set_encoder("region")
    c.encode_dev(src, spans, enc, eout)
    torch.cuda.synchronize()
    lib = _lib.load()
    lib.qh_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    out = (ctypes.c_uint64 * 16)()
    lib.qh_debug_stamps(out, 1)
    c.encode_dev(src, spans, enc, eout)
    torch.cuda.synchronize()
    lib.qh_debug_stamps(out, 1)
    v = list(out)
    rounds = max(v[11], 1)
    rep = {NAMES.get(k, str(k)): round(v[k] / rounds, 1) for k in range(11) if v[k]}
    rep["rounds (wave 0s)"] = v[11]
    rep["block life us (mean)"] = round(v[12] / 100.0 / max(1, 1), 1)
    print(json.dumps({"cycles_per_round": rep, "raw": v}))


if __name__ == "__main__":
    main()
