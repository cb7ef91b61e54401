"""Phase breakdown of qh_k_dec_run (development tool): wave 0 of every block
accumulates s_memtime deltas per phase.  Run with
QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so QHUFF_DECODER=run."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nghttp3_amd import HuffmanBatchCodec, _lib  # noqa: E402
from nghttp3_amd.qpack_huffman import decode_slot_size  # noqa: E402
from nghttp3_amd.synth import ALPHABET_A  # noqa: E402

NAMES = {7: "task-loop", 0: "task-start", 1: "fast", 2: "generic", 3: "last-store", 8: "tail"}


def main():
    lib = _lib.load()
    lib.qh_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    buf = (ctypes.c_uint64 * 16)()
    n = 1 << 20
    codec = HuffmanBatchCodec(0)
    src, spans, total = codec.synth(0x5EED0003, n, 8, 256, ALPHABET_A)
    enc = torch.empty(total * 4 + 64, dtype=torch.uint8, device="cuda")
    eout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    dout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    codec.encode_dev(src, spans, enc, eout)
    codec.sync()
    cap = int(decode_slot_size((eout[:, 1] & 0xFFFFFFFF).cpu().numpy()).sum())
    dec = torch.empty(cap + 64, dtype=torch.uint8, device="cuda")
    codec.decode_dev(enc, eout, dec, dout)
    codec.sync()
    lib.qh_debug_stamps(buf, 1)
    reps = 5
    for _ in range(reps):
        codec.decode_dev(enc, eout, dec, dout)
    codec.sync()
    lib.qh_debug_stamps(buf, 1)
    st = list(buf)
    tot = sum(st[k] for k in NAMES)
    print(f"tasks(wave0s)={st[10] / reps:.0f} bodies={st[11] / reps:.0f} generic={st[12] / reps:.0f}")
    print(f"waves={st[15] / reps:.0f} mean life={st[13] / max(st[15], 1):.4g} cyc "
          f"max life (last launch)={st[14]:.4g} cyc")
    for k, nm in NAMES.items():
        print(f"  {nm:11s} {st[k] / reps:12.4g} cyc  {100 * st[k] / max(tot, 1):5.1f}%  "
              f"per task {st[k] / max(st[10], 1):9.0f}")




def clock():
    lib = _lib.load()
    lib.qh_debug_clock.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]
    buf = (ctypes.c_uint64 * 3)()
    lib.qh_debug_clock(buf, 1 << 22)
    print(f"clock: memtime={buf[0]} realtime={buf[1]} -> {buf[0] / buf[1] * 100:.0f} MHz")


if __name__ == "__main__":
    clock()
    main()
    clock()
