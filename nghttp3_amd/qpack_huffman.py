"""Python host interface of the QPACK Huffman engine.

Two layers, mirroring include/qhuff.h:

* The reference's own codec interface (lib/nghttp3_qpack_huffman.h:42-115)
  with the same names, argument meaning and error values:
  ``huffman_encode_count``, ``huffman_encode``,
  ``huffman_decode_context_init``, ``huffman_decode``,
  ``huffman_decode_failure_state``, ``huffman_estimate_decode_length``.
  These call the library's exact-signature drop-ins (the streaming path).

* ``HuffmanBatchCodec``: whole-string batches through the HIP kernels
  (qh_decode_batch / qh_encode_count_batch / qh_encode_batch).  Device
  tensors go in and out without copies; host arrays are staged by the
  library (PCIe-inclusive path).  There is no host fallback.

Span layout (16 B per string, include/qhuff.h qh_span_in / qh_span_out):
as a torch int64 tensor of shape [n, 2]: column 0 = off, column 1 = len in
the low 32 bits and flags / status in the high 32 bits.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import (QH_ERR_NOMEM, QH_ERR_QPACK_FATAL, QH_WHERE_DEVICE,
                   QH_WHERE_HOST, QhError,
                   nghttp3_qpack_huffman_decode_context)

NGHTTP3_ERR_QPACK_FATAL = QH_ERR_QPACK_FATAL

SPAN_IN_DTYPE = np.dtype([("off", "<u8"), ("len", "<u4"), ("flags", "<u4")])
SPAN_OUT_DTYPE = np.dtype([("off", "<u8"), ("len", "<u4"), ("status", "<i4")])


def _buf(data):
    """(ctypes pointer, length, keepalive) for bytes-like input."""
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data, dtype=np.uint8)
    else:
        a = np.frombuffer(bytes(data), dtype=np.uint8)
    return a.ctypes.data_as(ctypes.c_void_p), a.size, a


# ---------------------------------------------------------------------------
# reference interface (streaming path)
# ---------------------------------------------------------------------------

HuffmanDecodeContext = nghttp3_qpack_huffman_decode_context


def huffman_estimate_decode_length(n: int) -> int:
    """lib/nghttp3_qpack_huffman.h:113-115"""
    return n * 8 // 5


def decode_slot_size(n):
    """Bytes a string of n encoded bytes owns in the batch decode output:
    estimate_decode_length + 16, rounded up to 64 (include/qhuff.h).  Works
    on ints and on numpy / torch integer arrays."""
    return (n * 8 // 5 + 16 + 63) // 64 * 64


def huffman_encode_count(src) -> int:
    """lib/nghttp3_qpack_huffman.c:34-43"""
    p, n, _keep = _buf(src)
    return int(_lib.load().nghttp3_qpack_huffman_encode_count(p, n))


def huffman_encode(src) -> bytes:
    """lib/nghttp3_qpack_huffman.c:45-78; returns the encoded bytes."""
    lib = _lib.load()
    p, n, _keep = _buf(src)
    cap = lib.nghttp3_qpack_huffman_encode_count(p, n)
    out = (ctypes.c_uint8 * max(cap, 1))()
    end = lib.nghttp3_qpack_huffman_encode(ctypes.addressof(out), p, n)
    written = end - ctypes.addressof(out)
    assert written == cap
    return bytes(out[:written])


def huffman_decode_context_init(ctx: HuffmanDecodeContext) -> None:
    """lib/nghttp3_qpack_huffman.c:80-85"""
    _lib.load().nghttp3_qpack_huffman_decode_context_init(ctypes.byref(ctx))


def huffman_decode(ctx: HuffmanDecodeContext, src, fin: bool):
    """lib/nghttp3_qpack_huffman.c:87-124.

    Returns the decoded bytes of this chunk, or the negative error code
    NGHTTP3_ERR_QPACK_FATAL (-108) exactly where the reference returns it.
    """
    lib = _lib.load()
    p, n, _keep = _buf(src)
    # A chunk can complete a code begun in an earlier chunk, so its output is
    # bounded by 2 symbols per input byte, not by estimate_decode_length(n).
    out = (ctypes.c_uint8 * (2 * n + 1))()
    rv = lib.nghttp3_qpack_huffman_decode(ctypes.byref(ctx), ctypes.addressof(out), p, n,
                                          1 if fin else 0)
    if rv < 0:
        return int(rv)
    return bytes(out[:rv])


def huffman_decode_failure_state(ctx: HuffmanDecodeContext) -> bool:
    """lib/nghttp3_qpack_huffman.c:126-129"""
    return bool(_lib.load().nghttp3_qpack_huffman_decode_failure_state(ctypes.byref(ctx)))


# ---------------------------------------------------------------------------
# batch interface (HIP kernels)
# ---------------------------------------------------------------------------

def pack_strings(strings):
    """Pack a list of bytes into (src uint8 array, spans SPAN_IN_DTYPE array)."""
    lens = np.fromiter((len(s) for s in strings), dtype=np.uint64, count=len(strings))
    spans = np.zeros(len(strings), dtype=SPAN_IN_DTYPE)
    if len(strings):
        spans["off"][1:] = np.cumsum(lens)[:-1]
    spans["len"] = lens.astype(np.uint32)
    src = np.frombuffer(b"".join(bytes(s) for s in strings), dtype=np.uint8)
    if src.size == 0:
        src = np.zeros(1, dtype=np.uint8)
    return src, spans


def _torch():
    import torch
    return torch


class HuffmanBatchCodec:
    """A qh_ctx bound to one HIP device and stream.

    ``stream``: a torch.cuda.Stream, a raw hipStream_t integer (0 = the
    default stream), or None for torch's current stream on ``device`` (so
    torch's synchronisation and events cover the kernels).
    """

    def __init__(self, device: int = 0, stream=None):
        self._lib = _lib.load()
        if stream is None:
            torch = _torch()
            handle = torch.cuda.current_stream(device).cuda_stream
        elif isinstance(stream, int):
            handle = stream
        else:
            handle = stream.cuda_stream
        ctx = ctypes.c_void_p()
        _lib.check(self._lib.qh_ctx_new(ctypes.byref(ctx), device,
                                        ctypes.c_void_p(handle) if handle else None),
                   "qh_ctx_new")
        self._ctx = ctx
        self.device = device

    def close(self):
        if getattr(self, "_ctx", None):
            self._lib.qh_ctx_del(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- context utilities --------------------------------------------------
    def set_decoder(self, kind: str):
        """'windows' (default), 'sorted' (batch-wide length-class schedule:
        skewed lengths, binary text) or 'waves' (include/qhuff.h
        QH_DECODER_*); results are identical."""
        k = {"windows": _lib.QH_DECODER_WINDOWS, "waves": _lib.QH_DECODER_WAVES,
             "sorted": _lib.QH_DECODER_SORTED}[kind]
        _lib.check(self._lib.qh_ctx_set_decoder(self._ctx, k), "qh_ctx_set_decoder")

    def set_encoder(self, kind: str):
        """'auto' (default: chosen per batch on the device), 'windows'
        (strings of similar length), 'waves' or 'fused' (one pass: long,
        skewed or binary strings); results are identical."""
        k = {"windows": _lib.QH_ENCODER_WINDOWS, "waves": _lib.QH_ENCODER_WAVES,
             "fused": _lib.QH_ENCODER_FUSED, "auto": _lib.QH_ENCODER_AUTO,
             "region": _lib.QH_ENCODER_REGION}[kind]
        _lib.check(self._lib.qh_ctx_set_encoder(self._ctx, k), "qh_ctx_set_encoder")

    def set_option(self, option: str, value: int):
        """Tuning options (include/qhuff.h QH_OPT_*; results are identical):
        'long_min' (the sorted decoder's workgroup-per-string threshold, in
        encoded bytes; 0 = off) and 'lens_lane_pass' (1: every string's
        encoded length counted a lane per string)."""
        k = {"long_min": _lib.QH_OPT_LONG_MIN, "lens_lane_pass": _lib.QH_OPT_LENS_LANE_PASS}[option]
        _lib.check(self._lib.qh_ctx_set_option(self._ctx, k, int(value)), "qh_ctx_set_option")

    def sync(self):
        _lib.check(self._lib.qh_ctx_sync(self._ctx), "qh_ctx_sync")

    def stats(self) -> dict:
        st = _lib.qh_batch_stats()
        _lib.check(self._lib.qh_ctx_last_stats(self._ctx, ctypes.byref(st)), "qh_ctx_last_stats")
        return {k: int(getattr(st, k)) for k, _ in st._fields_}

    def enable_timing(self, on: bool = True):
        _lib.check(self._lib.qh_ctx_enable_timing(self._ctx, 1 if on else 0), "qh_ctx_enable_timing")

    def kernel_times(self) -> dict:
        cap = 16
        names = (ctypes.c_char_p * cap)()
        counts = (ctypes.c_uint64 * cap)()
        ms = (ctypes.c_double * cap)()
        m = _lib.check(self._lib.qh_ctx_kernel_times(self._ctx, names, counts, ms, cap),
                       "qh_ctx_kernel_times")
        return {names[i].decode(): (int(counts[i]), float(ms[i])) for i in range(m)}

    # -- device-resident batches (torch tensors on this device) -------------
    @staticmethod
    def _ptr(t):
        return ctypes.c_void_p(t.data_ptr())

    def decode_dev(self, src, spans, dst, out, dense: bool = False):
        """src: uint8 [>=extent], spans: int64 [n,2], dst: uint8 [cap],
        out: int64 [n,2].  Asynchronous on the context stream.  dense: the
        decoded strings packed back to back (QH_WHERE_DEVICE_DENSE) instead
        of the slot layout."""
        n = spans.shape[0]
        _lib.check(self._lib.qh_decode_batch(self._ctx, self._ptr(src), self._ptr(spans), n,
                                             self._ptr(dst), dst.numel(), self._ptr(out),
                                             _lib.QH_WHERE_DEVICE_DENSE if dense else QH_WHERE_DEVICE),
                   "qh_decode_batch")

    def encode_count_dev(self, src, spans, hlen):
        n = spans.shape[0]
        _lib.check(self._lib.qh_encode_count_batch(self._ctx, self._ptr(src), self._ptr(spans), n,
                                                   self._ptr(hlen), QH_WHERE_DEVICE),
                   "qh_encode_count_batch")

    def encode_dev(self, src, spans, dst, out):
        n = spans.shape[0]
        _lib.check(self._lib.qh_encode_batch(self._ctx, self._ptr(src), self._ptr(spans), n,
                                             self._ptr(dst), dst.numel(), self._ptr(out),
                                             QH_WHERE_DEVICE), "qh_encode_batch")

    def synth(self, seed: int, n: int, lo: int, hi: int, alphabet: bytes):
        """Generate a packed synthetic batch on the device.
        Returns (src uint8 tensor, spans int64 [n,2] tensor, total bytes)."""
        torch = _torch()
        dev = torch.device("cuda", self.device)
        spans = torch.empty((n, 2), dtype=torch.int64, device=dev)
        total = torch.zeros(1, dtype=torch.int64, device=dev)
        _lib.check(self._lib.qh_synth_spans(self._ctx, seed, n, lo, hi, 0, 0.0,
                                            self._ptr(spans), self._ptr(total)), "qh_synth_spans")
        self.sync()
        nbytes = int(total.item())
        return self.synth_fill(seed, 0, nbytes, alphabet), spans, nbytes

    def synth_fill(self, seed: int, first: int, nbytes: int, alphabet: bytes):
        """Bytes [first, first + nbytes) of the packed synthetic stream of
        `seed` (nghttp3_amd/synth.py fill) as a uint8 tensor on the device."""
        torch = _torch()
        src = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=torch.device("cuda", self.device))
        a = np.frombuffer(bytes(alphabet), dtype=np.uint8)
        _lib.check(self._lib.qh_synth_fill(self._ctx, seed, first, self._ptr(src), nbytes,
                                           a.ctypes.data_as(ctypes.c_void_p), a.size), "qh_synth_fill")
        return src

    def spans_to_device(self, lengths):
        """Packed spans (off = exclusive prefix of `lengths`) as an int64
        [n, 2] tensor on the device, and the total bytes."""
        torch = _torch()
        ln = np.ascontiguousarray(lengths, dtype=np.int64)
        off = np.zeros(ln.size, dtype=np.int64)
        if ln.size:
            off[1:] = np.cumsum(ln)[:-1]
        sp = np.stack([off, ln], axis=1) if ln.size else np.zeros((0, 2), dtype=np.int64)
        return torch.from_numpy(np.ascontiguousarray(sp)).to(torch.device("cuda", self.device)), \
            int(ln.sum())

    # -- host batches (library stages H2D / D2H) ----------------------------
    def decode_host(self, src, spans, dst=None, out=None):
        """Decode packed host strings; returns (dst uint8, out SPAN_OUT_DTYPE).

        `dst` / `out` may be caller-provided (e.g. numpy views of pinned
        torch tensors: the copies are then direct DMA)."""
        src = np.ascontiguousarray(src, dtype=np.uint8)
        spans = np.ascontiguousarray(spans, dtype=SPAN_IN_DTYPE)
        n = spans.size
        cap = int(self._lib.qh_decode_dst_size(spans.ctypes.data_as(ctypes.c_void_p), n))
        if dst is None:
            dst = np.zeros(max(cap, 1), dtype=np.uint8)
        assert dst.dtype == np.uint8 and dst.flags.c_contiguous and dst.size >= cap
        if out is None:
            out = np.zeros(n, dtype=SPAN_OUT_DTYPE)
        assert out.dtype == SPAN_OUT_DTYPE and out.size >= n
        _lib.check(self._lib.qh_decode_batch(self._ctx, src.ctypes.data_as(ctypes.c_void_p),
                                             spans.ctypes.data_as(ctypes.c_void_p), n,
                                             dst.ctypes.data_as(ctypes.c_void_p), cap,
                                             out.ctypes.data_as(ctypes.c_void_p), QH_WHERE_HOST),
                   "qh_decode_batch")
        return dst, out

    @staticmethod
    def decode_host_multi(codecs, src, spans, dst=None, out=None):
        """qh_decode_batch_multi: one host batch over several contexts (one
        host thread and H2D / decode / D2H pipeline each); returns (dst,
        out) with out["off"] global (strings in order, packed per range)."""
        lib = _lib.load()
        src = np.ascontiguousarray(src, dtype=np.uint8)
        spans = np.ascontiguousarray(spans, dtype=SPAN_IN_DTYPE)
        n = spans.size
        cap = int(lib.qh_decode_dst_size(spans.ctypes.data_as(ctypes.c_void_p), n))
        if dst is None:
            dst = np.zeros(max(cap, 1), dtype=np.uint8)
        assert dst.dtype == np.uint8 and dst.flags.c_contiguous and dst.size >= cap
        if out is None:
            out = np.zeros(n, dtype=SPAN_OUT_DTYPE)
        ctxs = (ctypes.c_void_p * len(codecs))(*[c._ctx.value for c in codecs])
        _lib.check(lib.qh_decode_batch_multi(ctxs, len(codecs), src.ctypes.data_as(ctypes.c_void_p),
                                             spans.ctypes.data_as(ctypes.c_void_p), n,
                                             dst.ctypes.data_as(ctypes.c_void_p), cap,
                                             out.ctypes.data_as(ctypes.c_void_p)),
                   "qh_decode_batch_multi")
        return dst, out

    def encode_count_host(self, src, spans):
        src = np.ascontiguousarray(src, dtype=np.uint8)
        spans = np.ascontiguousarray(spans, dtype=SPAN_IN_DTYPE)
        hlen = np.zeros(max(spans.size, 1), dtype=np.uint32)
        _lib.check(self._lib.qh_encode_count_batch(self._ctx, src.ctypes.data_as(ctypes.c_void_p),
                                                   spans.ctypes.data_as(ctypes.c_void_p), spans.size,
                                                   hlen.ctypes.data_as(ctypes.c_void_p), QH_WHERE_HOST),
                   "qh_encode_count_batch")
        return hlen[:spans.size]

    def encode_host(self, src, spans):
        """Encode packed host strings; returns (dst uint8, out SPAN_OUT_DTYPE)."""
        src = np.ascontiguousarray(src, dtype=np.uint8)
        spans = np.ascontiguousarray(spans, dtype=SPAN_IN_DTYPE)
        n = spans.size
        cap = int(self._lib.qh_encode_dst_bound(spans.ctypes.data_as(ctypes.c_void_p), n))
        dst = np.zeros(max(cap, 1), dtype=np.uint8)
        out = np.zeros(n, dtype=SPAN_OUT_DTYPE)
        _lib.check(self._lib.qh_encode_batch(self._ctx, src.ctypes.data_as(ctypes.c_void_p),
                                             spans.ctypes.data_as(ctypes.c_void_p), n,
                                             dst.ctypes.data_as(ctypes.c_void_p), cap,
                                             out.ctypes.data_as(ctypes.c_void_p), QH_WHERE_HOST),
                   "qh_encode_batch")
        return dst, out


def unpack_out(out):
    """Split an int64 [n,2] out tensor/array into (off, len, status) numpy."""
    a = out.cpu().numpy() if hasattr(out, "cpu") else np.asarray(out)
    if a.dtype == SPAN_OUT_DTYPE:
        return a["off"].astype(np.int64), a["len"].astype(np.int64), a["status"].astype(np.int64)
    a = a.astype(np.int64).reshape(-1, 2)
    return a[:, 0], a[:, 1] & 0xFFFFFFFF, a[:, 1] >> 32


__all__ = [
    "NGHTTP3_ERR_QPACK_FATAL", "QH_ERR_NOMEM", "QhError", "HuffmanDecodeContext",
    "huffman_estimate_decode_length", "decode_slot_size", "huffman_encode_count", "huffman_encode",
    "huffman_decode_context_init", "huffman_decode", "huffman_decode_failure_state",
    "HuffmanBatchCodec", "pack_strings", "unpack_out", "SPAN_IN_DTYPE", "SPAN_OUT_DTYPE",
]
