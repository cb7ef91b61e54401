"""TEST INFRASTRUCTURE ONLY: ctypes binding of the C oracle (qh_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker / CPU baseline.  It restates
nghttp3's lib/nghttp3_qpack_huffman.c; see qh_oracle.h for how it is pinned
(table digests vs lib/nghttp3_qpack_huffman_data.c, RFC 7541 Appendix C
vectors, the reference's tests/nghttp3_qpack_test.c:856-899).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libqh_oracle.so")
QPACK_FATAL = -108

_lib = None


class DecodeCtx(ctypes.Structure):
    _fields_ = [("fstate", ctypes.c_uint16), ("flags", ctypes.c_uint8)]


def build():
    src = os.path.join(_HERE, "qh_oracle.c")
    cmd = ["gcc", "-std=c11", "-O2", "-mavx2", "-fPIC", "-shared", "-pthread", "-Wall",
           "-o", LIB_PATH, src]
    subprocess.check_call(cmd)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = ctypes.CDLL(LIB_PATH)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.qho_tables.argtypes = [vp, vp]
    lib.qho_encode_count.argtypes = [vp, sz]
    lib.qho_encode_count.restype = sz
    lib.qho_encode.argtypes = [vp, vp, sz]
    lib.qho_encode.restype = vp
    lib.qho_decode_context_init.argtypes = [ctypes.POINTER(DecodeCtx)]
    lib.qho_decode.argtypes = [ctypes.POINTER(DecodeCtx), vp, vp, sz, ctypes.c_int]
    lib.qho_decode.restype = ctypes.c_ssize_t
    lib.qho_decode_failure_state.argtypes = [ctypes.POINTER(DecodeCtx)]
    lib.qho_decode_failure_state.restype = ctypes.c_int
    lib.qho_encode_batch.argtypes = [vp, vp, vp, sz, vp, vp, vp]
    lib.qho_encode_batch.restype = ctypes.c_uint64
    lib.qho_decode_batch.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp]
    lib.qho_decode_batch.restype = ctypes.c_uint64
    lib.qho_bench_roundtrip.argtypes = [vp, vp, vp, sz, ctypes.c_int, vp, ctypes.c_int,
                                        ctypes.c_double,
                                        ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_int)]
    lib.qho_bench_roundtrip.restype = ctypes.c_int
    _lib = lib
    return lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def tables():
    """(sym uint32[257,2], fsm uint32[257,16]) as the oracle builds them."""
    sym = np.zeros((257, 2), dtype=np.uint32)
    fsm = np.zeros((257, 16), dtype=np.uint32)
    load().qho_tables(_p(sym), _p(fsm))
    return sym, fsm


def encode_count(s: bytes) -> int:
    a = np.frombuffer(bytes(s), dtype=np.uint8) if s else np.zeros(1, np.uint8)
    return int(load().qho_encode_count(_p(a), len(s)))


def encode(s: bytes) -> bytes:
    a = np.frombuffer(bytes(s), dtype=np.uint8) if s else np.zeros(1, np.uint8)
    out = np.zeros(encode_count(s) + 8, dtype=np.uint8)
    end = load().qho_encode(_p(out), _p(a), len(s))
    return out[: end - out.ctypes.data].tobytes()


def new_ctx() -> DecodeCtx:
    c = DecodeCtx()
    load().qho_decode_context_init(ctypes.byref(c))
    return c


def decode(ctx: DecodeCtx, s: bytes, fin: bool):
    """bytes, or the negative error (-108) as the reference returns it."""
    a = np.frombuffer(bytes(s), dtype=np.uint8) if s else np.zeros(1, np.uint8)
    out = np.zeros(2 * len(s) + 8, dtype=np.uint8)  # <= 2 symbols per byte
    rv = load().qho_decode(ctypes.byref(ctx), _p(out), _p(a), len(s), 1 if fin else 0)
    return int(rv) if rv < 0 else out[:rv].tobytes()


def failure_state(ctx: DecodeCtx) -> bool:
    return bool(load().qho_decode_failure_state(ctypes.byref(ctx)))


def decode_one(s: bytes):
    """Whole-string decode as the batch API defines it: (status, bytes)."""
    c = new_ctx()
    r = decode(c, s, True)
    if isinstance(r, int) or failure_state(c):
        return QPACK_FATAL, b""
    return 0, r


def encode_batch(plain, off, ln):
    """Dense encodings of packed strings: (enc uint8, enc_off u64, enc_len u32)."""
    plain = np.ascontiguousarray(plain, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(ln, dtype=np.uint32)
    n = ln.size
    cap = int((ln.astype(np.uint64) * 30 + 7).sum() // 8) + 16
    enc = np.zeros(cap, dtype=np.uint8)
    eoff = np.zeros(max(n, 1), dtype=np.uint64)
    elen = np.zeros(max(n, 1), dtype=np.uint32)
    total = load().qho_encode_batch(_p(plain), _p(off), _p(ln), n, _p(enc), _p(eoff), _p(elen))
    return enc[:total], eoff[:n], elen[:n]


def decode_batch(enc, off, ln):
    """Slot-layout decode (include/qhuff.h): (dst, slot_off, out_len, status)."""
    enc = np.ascontiguousarray(enc, dtype=np.uint8)
    if enc.size == 0:
        enc = np.zeros(1, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(ln, dtype=np.uint32)
    n = ln.size
    cap = int((((ln.astype(np.uint64) * 8 // 5) + 15) // 16 * 16).sum()) + 16
    dst = np.zeros(cap, dtype=np.uint8)
    slot = np.zeros(max(n, 1), dtype=np.uint64)
    olen = np.zeros(max(n, 1), dtype=np.uint32)
    st = np.zeros(max(n, 1), dtype=np.int32)
    load().qho_decode_batch(_p(enc), _p(off), _p(ln), n, _p(dst), _p(slot), _p(olen), _p(st))
    return dst, slot[:n], olen[:n], st[:n]


def bench_roundtrip(plain, off, ln, nthreads: int, reps: int, cpus=None,
                    min_seconds: float = 0.05):
    """CPU baseline: a pool of `nthreads` threads (thread t pinned to cpus[t]
    when given), `reps` barrier-to-barrier encode and decode passes, each
    long enough that a thread works >= min_seconds.  Returns per-rep
    seconds per round over the strings (encode list, decode list), ok, and
    the (encode, decode) repetitions per pass."""
    plain = np.ascontiguousarray(plain, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(ln, dtype=np.uint32)
    e = (ctypes.c_double * max(reps, 1))()
    d = (ctypes.c_double * max(reps, 1))()
    inner = (ctypes.c_int * 2)()
    cp = None
    if cpus is not None:
        cpa = np.ascontiguousarray(list(cpus)[:nthreads], dtype=np.int32)
        assert cpa.size == nthreads
        cp = _p(cpa)
    rv = load().qho_bench_roundtrip(_p(plain), _p(off), _p(ln), ln.size, nthreads, cp, reps,
                                    float(min_seconds), e, d, inner)
    return list(e)[:reps], list(d)[:reps], rv == 0, (inner[0], inner[1])
