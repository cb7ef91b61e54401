#!/usr/bin/env python3
"""Per-phase wave cycles of the pair decoder (development tool).

Run with QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so (make stamps) and
QHUFF_DECODER=<pair variant>.  Every wave of qh_k_dec_pairs adds its
s_memtime deltas per phase (qh_pair_dec.inc PrSt); prints each phase's
share of the waves' summed cycles, cycles per iteration and per group.
Env: N (strings, default 2^20), ALPH (A or U), REPS.
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nghttp3_amd import HuffmanBatchCodec, _lib  # noqa: E402
from nghttp3_amd.qpack_huffman import decode_slot_size  # noqa: E402
from nghttp3_amd.synth import ALPHABET_A, ALPHABET_U  # noqa: E402

PHASES = {0: "queue+waits", 1: "build", 2: "group load", 3: "str start", 4: "iter top", 5: "lookups",
          6: "flushes", 7: "careful", 8: "string ends", 12: "top vmcnt wait", 13: "lane idle at end"}


def main():
    lib = _lib.load()
    assert "stamps" in _lib.LIB_PATH, "set QHUFF_LIB to the stamps build"
    lib.qh_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    buf = (ctypes.c_uint64 * 16)()

    def read():
        assert lib.qh_debug_stamps(buf, 1) == 0
        return list(buf)

    n = int(os.environ.get("N", 1 << 20))
    codec = HuffmanBatchCodec(0)
    dev = torch.device("cuda", 0)
    alph = ALPHABET_U if os.environ.get("ALPH") == "U" else ALPHABET_A
    src, spans, total = codec.synth(0x5EED0003, n, 8, 256, alph)
    enc = torch.empty(total * 4 + 64, dtype=torch.uint8, device=dev)
    eout = torch.empty((n, 2), dtype=torch.int64, device=dev)
    dout = torch.empty((n, 2), dtype=torch.int64, device=dev)
    codec.encode_dev(src, spans, enc, eout)
    codec.sync()
    cap = int(decode_slot_size((eout[:, 1] & 0xFFFFFFFF).cpu().numpy()).sum())
    dec = torch.empty(cap + 64, dtype=torch.uint8, device=dev)
    codec.decode_dev(enc, eout, dec, dout)
    codec.sync()
    read()
    reps = int(os.environ.get("REPS", 3))
    for _ in range(reps):
        codec.decode_dev(enc, eout, dec, dout)
    codec.sync()
    a = [v / reps for v in read()]
    tot = sum(a[k] for k in PHASES)
    out = {"kind": os.environ.get("QHUFF_DECODER"), "alphabet": os.environ.get("ALPH", "A"),
           "share": {PHASES[k]: round(a[k] / tot, 3) for k in PHASES},
           "iterations": a[9], "groups": a[10], "careful_lane_entries": a[11],
           "cyc_per_iter": {PHASES[k]: round(a[k] / max(a[9], 1), 1) for k in (4, 12, 5, 6, 7, 8)},
           "cyc_per_group": {PHASES[k]: round(a[k] / max(a[10], 1), 1) for k in (0, 1, 2, 3, 13)},
           "recent_waits_per_iter": round(a[14] / max(a[9], 1), 3),
           "lane_efficiency": round(a[15] / max(a[9], 1) / 64, 3),
           "iters_per_group": round(a[9] / max(a[10], 1), 2),
           "careful_per_lane_iter": round(a[11] / max(a[9], 1) / 64, 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
