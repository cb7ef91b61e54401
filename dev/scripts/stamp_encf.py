"""Per-phase cycle breakdown of the fused encoder (development tool).

QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so python scripts/stamp_encf.py
Wave 0 of every workgroup adds s_memtime deltas per phase (qh_k_encf)."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nghttp3_amd import HuffmanBatchCodec, _lib, synth  # noqa: E402

PHASES = {0: "head (tile, strings, scan)", 1: "chunks (load, lookups, scan)",
          2: "aggregate + stage zero", 3: "look-back", 4: "out records", 5: "staging",
          6: "copy-out", 11: "look-back: waits for one record", 15: "windows read (count)",
          12: "block life (realtime)", 13: "block life (clocks)"}


def main():
    lib = _lib.load()
    assert "stamps" in _lib.LIB_PATH, "set QHUFF_LIB to the stamps build"
    lib.qh_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    buf = (ctypes.c_uint64 * 16)()
    n = int(os.environ.get("N", 1 << 20))
    c = HuffmanBatchCodec(0)
    c.set_encoder("fused")
    src, spans, total = c.synth(0x5EED0003, n, 8, 256, synth.ALPHABET_A)
    enc = torch.empty(total * 4 + 64, dtype=torch.uint8, device="cuda")
    eout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    c.encode_dev(src, spans, enc, eout)
    c.sync()
    lib.qh_debug_stamps(buf, 1)
    reps = 5
    for _ in range(reps):
        c.encode_dev(src, spans, enc, eout)
    c.sync()
    lib.qh_debug_stamps(buf, 1)
    v = list(buf)
    tiles = max(v[10], 1)
    out = {PHASES[k]: round(v[k] / tiles, 2) for k in PHASES if k < 12 or k == 15}
    out["tiles (wave 0 count)"] = v[10]
    out["cycles per tile, all phases"] = round((sum(v[k] for k in range(7)) + v[11]) / tiles)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
