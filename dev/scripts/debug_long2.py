#!/usr/bin/env python3
"""Development: qh_debug_long's segment trace against the Python model
(tests/test_long_model.py) on a few strings, NW = 1, 4, 16."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import torch
    import oracle
    import test_long_model as M
    from nghttp3_amd import HuffmanBatchCodec, synth, _lib
    M._TABLE = M._codes()
    lib = _lib.load()
    lib.qh_debug_long.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int,
                                                          ctypes.c_void_p, ctypes.c_void_p]
    c = HuffmanBatchCodec(0)
    rng = np.random.default_rng(1)
    for n, kind in ((5000, "txt"), (49000, "txt"), (3000, "bin")):
        v = synth.fill(7, n, synth.ALPHABET_A).tobytes() if kind == "txt" else rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        enc = oracle.encode(v)
        tr = []
        st, dec = M.long_decode_model(enc, tr)
        lanes0 = tr.pop(0)
        print(kind, n, "enc", len(enc), "model", st, dec == v, "segments", len(tr), flush=True)
        for nw in (1, 4, 16):
            d_src = torch.from_numpy(np.frombuffer(enc, np.uint8).copy()).cuda()
            d_dst = torch.zeros(len(enc) * 2 + 64, dtype=torch.uint8, device="cuda")
            res = torch.zeros(2, dtype=torch.int32, device="cuda")
            trace = torch.full((8192 + 8 * 512,), -1, dtype=torch.int32, device="cuda")
            _lib.check(lib.qh_debug_long(c._ctx, d_src.data_ptr(), len(enc), d_dst.data_ptr(), nw,
                                         res.data_ptr(), trace.data_ptr()), "qh_debug_long")
            torch.cuda.synchronize()
            r = res.cpu().tolist()
            ta = trace.cpu().numpy()
            t = ta[:4 * len(tr)].reshape(-1, 4)
            tl = ta[4096:4096 + 512].reshape(64, 8)
            for j in range(64):
                if tuple(int(x) for x in tl[j]) != lanes0[j]:
                    print("    lane", j, "gpu", tuple(int(x) for x in tl[j]), "model", lanes0[j])
            got = bytes(d_dst[:r[0]].cpu().numpy())
            first = next((k for k in range(len(tr)) if tuple(int(x) for x in t[k]) != tr[k]), None)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                lib.qh_debug_long(c._ctx, d_src.data_ptr(), len(enc), d_dst.data_ptr(), nw, res.data_ptr(), None)
            e1.record()
            torch.cuda.synchronize()
            print("  us per string (no trace):", round(e0.elapsed_time(e1) * 1e3 / 5, 1))
            print("  nw", nw, "res", r, "bytes ok", got == v, "first diverging segment", first,
                  "" if first is None else (tuple(int(x) for x in t[first]), tr[first]), flush=True)


if __name__ == "__main__":
    main()
