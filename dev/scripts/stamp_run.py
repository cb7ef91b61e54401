"""Per-phase cycle breakdown of the tile kernels (development tool).

Run with QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so (built by
`make stamps`).  Prints, per kernel, the wave-0 cycles per tile and per
round for each phase slot (see QH_ST(k) in the kernels).
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nghttp3_amd import HuffmanBatchCodec, _lib  # noqa: E402
from nghttp3_amd.qpack_huffman import decode_slot_size  # noqa: E402
from nghttp3_amd.synth import ALPHABET_A, ALPHABET_U  # noqa: E402

# kernel -> (phase slots, rounds slot, tiles slot, extra counter slot)
LAYOUT = {
    "dec_lanes": ({0: "window", 1: "decode"}, 10, 10, None),
    "dec_peek": ({0: "window setup", 1: "window decode (all)", 2: "str start", 3: "iter top",
                  4: "iter body", 5: "careful", 6: "str end"}, 11, 10, None),
    "enc_lens": ({0: "head", 2: "dma wait", 3: "lookups", 4: "scan", 5: "ends", 6: "tail"},
                 10, 10, 11),
    "enc_lanes": ({0: "setup", 1: "encode", 2: "copy-out"}, 10, 10, None),
    "encs": ({0: "front setup", 1: "count loop", 2: "count tail", 3: "look-back", 4: "lookups+ends",
              5: "byte chain", 6: "flush", 10: "merge"}, 11, 11, None),
}


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
    src, spans, total = codec.synth(0x5EED0003, n, 8, 256,
                                    ALPHABET_U if os.environ.get("ALPH") == "U" else ALPHABET_A)
    enc = torch.empty(total * 4 + 64, dtype=torch.uint8, device=dev)
    eout = torch.empty((n, 2), dtype=torch.int64, device=dev)
    dout = torch.empty((n, 2), dtype=torch.int64, device=dev)
    hlen = torch.empty(n, dtype=torch.int32, device=dev)
    codec.encode_dev(src, spans, enc, eout)
    codec.sync()
    cap = int(decode_slot_size((eout[:, 1] & 0xFFFFFFFF).cpu().numpy()).sum())
    dec = torch.empty(cap + 64, dtype=torch.uint8, device=dev)
    codec.decode_dev(enc, eout, dec, dout)
    codec.sync()
    read()
    reps = int(os.environ.get("REPS", 5))
    runs = {
        "dec_lanes": lambda: codec.decode_dev(enc, eout, dec, dout),
        "dec_peek": lambda: codec.decode_dev(enc, eout, dec, dout),
        "enc_lens": lambda: codec.encode_count_dev(src, spans, hlen),
        "enc_lanes": lambda: codec.encode_dev(src, spans, enc, eout),
        "encs": lambda: codec.encode_dev(src, spans, enc, eout),
    }
    only = os.environ.get("KERNELS")
    for kern, fn in runs.items():
        if only and kern not in only.split(","):
            continue
        if kern == "encs":
            codec.set_encoder("fused")
        for _ in range(reps):
            fn()
        codec.sync()
        st = read()
        phases, rs, ts, xs = LAYOUT[kern]
        rounds, tiles = max(st[rs], 1), max(st[ts], 1)
        extra = f" counter/round={st[xs] / rounds:.2f}" if xs is not None else ""
        print(f"{kern}: windows/launch={tiles / reps:.0f} rounds/launch={rounds / reps:.0f}{extra}")
        tot = sum(st[k] for k in phases)
        for k, nm in phases.items():
            print(f"  {nm:11s} {st[k] / tiles:9.0f} cyc/tile {st[k] / rounds:8.0f} cyc/round"
                  f"  {100 * st[k] / max(tot, 1):5.1f}%")
        print(f"  wave0 cycles/launch {tot / reps:.3e}")
        if st[8] and reps == 1:
            t0 = (~st[7]) & ((1 << 64) - 1)
            print(f"  starts: first..last {(st[8] - t0) / 100:.1f} us after the first; "
                  f"last end {(st[9] - t0) / 100:.1f} us after the first start")
        if st[12]:
            print(f"  block lifetime: {st[12] / reps * 10 / 1000:.0f} us-blocks/launch (realtime), "
                  f"memtime/realtime = {st[13] / st[12] * 100:.0f} MHz, longest block {st[14] / 100:.1f} us")


if __name__ == "__main__":
    main()
