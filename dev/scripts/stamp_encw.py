"""Per-phase cycle breakdown of the fused encoder qh_k_encw (development).

QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so python scripts/stamp_encw.py
Wave 0 of every workgroup adds s_memtime deltas per phase."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nghttp3_amd import HuffmanBatchCodec, _lib, synth  # noqa: E402

PHASES = {0: "ticket + strings", 1: "count pass", 2: "hlen + publish", 3: "look-back",
          4: "records + stage zero (per window) / copy-out tail", 5: "codes: find + loads",
          6: "codes: lookups, scan, position", 11: "codes: ORs", 15: "codes: copy-out + zero"}


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
    for _ in range(5):
        c.encode_dev(src, spans, enc, eout)
    c.sync()
    lib.qh_debug_stamps(buf, 1)
    v = list(buf)
    wins = max(v[10], 1)
    out = {PHASES[k]: round(v[k] / wins) for k in PHASES}
    out["windows (wave 0 count)"] = v[10]
    out["cycles per window, all phases"] = round(sum(v[k] for k in PHASES) / wins)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
