"""QPACK field-line framing around the batch Huffman engine (SURVEY.md
section 8(f) rows 1-2), over the C-ABI of nghttp3_amd/csrc/qh_qpack.c.

* ``scan_field_section`` / ``scan_blocks`` / ``scan_encoder_stream`` --
  the framing of nghttp3_qpack_decoder_read_request
  (lib/nghttp3_qpack.c:3347-3800) and nghttp3_qpack_decoder_read_encoder
  (:2815-3150), returning field lines and (off, len, flags) string spans.
* ``write_indexed`` / ``write_indexed_name`` / ``write_literal`` -- the
  representation writers (qpack.c:1851-2069) with the reference's
  Huffman-iff-shorter choice.
* ``FieldSectionDecoder`` -- whole header blocks in, decoded strings out:
  host-side scan, then every Huffman string of the batch in one
  ``qh_decode_batch`` call on the GPU.

Error values are the reference's: -401 DECOMPRESSION_FAILED, -402
ENCODER_STREAM_ERROR, -109 HEADER_TOO_LARGE (nghttp3.h:224-259).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .qpack_huffman import SPAN_IN_DTYPE, SPAN_OUT_DTYPE, HuffmanBatchCodec

QH_ERR_QPACK_HEADER_TOO_LARGE = -109
QH_ERR_QPACK_DECOMPRESSION_FAILED = -401
QH_ERR_QPACK_ENCODER_STREAM_ERROR = -402

SPAN_HUFFMAN, SPAN_NAME = 0x1, 0x2
(FL_INDEXED, FL_INDEXED_PB, FL_INDEXED_NAME, FL_INDEXED_NAME_PB, FL_LITERAL,
 ES_INSERT_INDEXED, ES_INSERT, ES_SET_DTABLE_CAP, ES_DUPLICATE) = range(1, 10)
FL_DYNAMIC, FL_NEVER = 0x1, 0x2

FIELD_LINE_DTYPE = np.dtype([("index", "<u8"), ("opcode", "u1"), ("flags", "u1"),
                             ("reserved", "<u2"), ("name", "<i4"), ("value", "<i4"),
                             ("reserved2", "<u4")])
assert FIELD_LINE_DTYPE.itemsize == 24


PREFIX_DTYPE = np.dtype([("ricnt", "<u8"), ("delta_base", "<u8"), ("sign", "<u4"),
                         ("reserved", "<u4")])


class qh_section_prefix(ctypes.Structure):
    _fields_ = [("ricnt", ctypes.c_uint64), ("delta_base", ctypes.c_uint64),
                ("sign", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


SECTIONS_DTABLE0 = 0x1


class qh_sections(ctypes.Structure):
    """include/qhuff.h qh_sections (outputs of qh_decode_sections_batch)."""
    _fields_ = [("lines", ctypes.c_void_p), ("lines_cap", ctypes.c_size_t),
                ("spans", ctypes.c_void_p), ("spans_cap", ctypes.c_size_t),
                ("strs", ctypes.c_void_p), ("verdict", ctypes.c_void_p),
                ("token", ctypes.c_void_p), ("line_start", ctypes.c_void_p),
                ("span_start", ctypes.c_void_p), ("status", ctypes.c_void_p),
                ("prefixes", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("dst_cap", ctypes.c_uint64),
                ("nlines", ctypes.c_uint64), ("nspans", ctypes.c_uint64),
                ("nhuff", ctypes.c_uint64), ("dst_need", ctypes.c_uint64)]


_L = None


def _load():
    global _L
    if _L is None:
        lib = _lib.load()
        c = ctypes
        vp, sz, u64, u8, i32 = c.c_void_p, c.c_size_t, c.c_uint64, c.c_uint8, c.c_int
        lib.qh_qpack_scan_field_section.argtypes = [vp, sz, u64, c.POINTER(qh_section_prefix), vp, sz,
                                                    c.POINTER(sz), vp, sz, c.POINTER(sz)]
        lib.qh_qpack_scan_field_section.restype = i32
        lib.qh_qpack_scan_blocks.argtypes = [vp, vp, sz, vp, sz, vp, sz, vp, vp, vp]
        lib.qh_qpack_scan_blocks.restype = i32
        lib.qh_qpack_scan_encoder_stream.argtypes = [vp, sz, u64, vp, sz, c.POINTER(sz), vp, sz,
                                                     c.POINTER(sz)]
        lib.qh_qpack_scan_encoder_stream.restype = c.c_ssize_t
        lib.qh_qpack_put_varint_len.argtypes = [u64, sz]
        lib.qh_qpack_put_varint_len.restype = sz
        lib.qh_qpack_put_varint.argtypes = [vp, u64, sz]
        lib.qh_qpack_put_varint.restype = vp
        lib.qh_qpack_write_indexed.argtypes = [vp, u8, u64, sz]
        lib.qh_qpack_write_indexed.restype = sz
        lib.qh_qpack_write_indexed_name.argtypes = [vp, u8, u64, sz, vp, sz]
        lib.qh_qpack_write_indexed_name.restype = sz
        lib.qh_qpack_write_literal.argtypes = [vp, u8, sz, vp, sz, vp, sz]
        lib.qh_qpack_write_literal.restype = sz
        lib.qh_qpack_literal_bound.argtypes = [sz, sz]
        lib.qh_qpack_literal_bound.restype = sz
        lib.qh_qpack_write_sections.argtypes = [vp, vp, vp, vp, sz, vp, vp, sz, vp]
        lib.qh_qpack_write_sections.restype = i32
        lib.nghttp3_check_header_name.argtypes = [vp, sz]
        lib.nghttp3_check_header_name.restype = i32
        lib.nghttp3_check_header_value.argtypes = [vp, sz]
        lib.nghttp3_check_header_value.restype = i32
        lib.qh_check_fields_batch.argtypes = [vp, vp, vp, sz, vp, i32]
        lib.qh_check_fields_batch.restype = i32
        lib.qh_scan_blocks_batch.argtypes = [vp, vp, vp, sz, vp, sz, vp, sz, vp, vp, vp, vp, sz,
                                             c.POINTER(c.c_uint64), i32]
        lib.qh_scan_blocks_batch.restype = i32
        lib.qh_qpack_lookup_token.argtypes = [vp, sz]
        lib.qh_qpack_lookup_token.restype = c.c_int32
        lib.qh_lookup_tokens_batch.argtypes = [vp, vp, vp, sz, vp, i32]
        lib.qh_lookup_tokens_batch.restype = i32
        lib.qh_decode_sections_batch.argtypes = [vp, vp, vp, sz, c.c_uint32, c.POINTER(qh_sections),
                                                 i32]
        lib.qh_decode_sections_batch.restype = i32
        lib.qh_qpack_static_entry.argtypes = [sz, c.POINTER(vp), c.POINTER(sz), c.POINTER(vp),
                                              c.POINTER(sz)]
        lib.qh_qpack_static_entry.restype = i32
        lib.qh_qpack_plan_fields.argtypes = [vp, vp, sz, vp, vp]
        lib.qh_qpack_plan_fields.restype = i32
        lib.qh_encode_sections_batch.argtypes = [vp, vp, vp, sz, vp, vp, sz, vp, vp, u64, vp,
                                                 c.POINTER(u64), i32]
        lib.qh_encode_sections_batch.restype = i32
        _L = lib
    return _L


def _u8(data):
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) \
        else np.ascontiguousarray(data, dtype=np.uint8)
    if a.size == 0:
        a = np.zeros(1, dtype=np.uint8)[:0]
    return a


def _vp(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def scan_field_section(buf, base_off: int = 0):
    """One complete field section -> (status, (ricnt, sign, delta_base) or
    None, lines FIELD_LINE_DTYPE, spans SPAN_IN_DTYPE).  On an error there
    are no lines and the spans are the strings read before it."""
    lib = _load()
    src = _u8(buf)
    cap = src.size + 1  # every line and string takes at least one byte
    lines = np.zeros(cap, dtype=FIELD_LINE_DTYPE)
    spans = np.zeros(cap, dtype=SPAN_IN_DTYPE)
    pf = qh_section_prefix()
    nl, ns = ctypes.c_size_t(0), ctypes.c_size_t(0)
    rv = lib.qh_qpack_scan_field_section(_vp(src), src.size, base_off, ctypes.byref(pf), _vp(lines),
                                         cap, ctypes.byref(nl), _vp(spans), cap, ctypes.byref(ns))
    if rv != 0:
        return rv, None, lines[:0], spans[:ns.value]
    return 0, (pf.ricnt, pf.sign, pf.delta_base), lines[:nl.value], spans[:ns.value]


def scan_blocks(src, blocks):
    """Batch of field sections (blocks: SPAN_IN_DTYPE into src) ->
    (lines, spans, line_start, span_start, status)."""
    lib = _load()
    src = _u8(src)
    blocks = np.ascontiguousarray(blocks, dtype=SPAN_IN_DTYPE)
    nb = blocks.size
    cap = int(blocks["len"].sum(dtype=np.uint64)) + 1
    lines = np.zeros(cap, dtype=FIELD_LINE_DTYPE)
    spans = np.zeros(cap, dtype=SPAN_IN_DTYPE)
    ls = np.zeros(nb + 1, dtype=np.uint32)
    ss = np.zeros(nb + 1, dtype=np.uint32)
    st = np.zeros(max(nb, 1), dtype=np.int32)
    _lib.check(lib.qh_qpack_scan_blocks(_vp(src), _vp(blocks), nb, _vp(lines), cap, _vp(spans), cap,
                                        _vp(ls), _vp(ss), _vp(st)), "qh_qpack_scan_blocks")
    return lines[:ls[nb]], spans[:ss[nb]], ls, ss, st[:nb]


def scan_blocks_dev(codec: HuffmanBatchCodec, src, blocks, lines, spans, line_start, span_start,
                    status, huff=None):
    """GPU framing (qh_scan_blocks_batch) over torch tensors in HBM: src
    uint8, blocks int64 [n,2] (SPAN_IN layout), lines uint8 [cap*24], spans
    int64 [cap,2], line_start / span_start int32 [n+1], status int32 [n],
    optional huff int64 [cap,2] (the Huffman spans alone).  Returns the
    totals (lines, spans, Huffman spans)."""
    lib = _load()
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
    tot = (ctypes.c_uint64 * 3)()
    _lib.check(lib.qh_scan_blocks_batch(codec._ctx, p(src), p(blocks), blocks.shape[0], p(lines),
                                        lines.numel() // FIELD_LINE_DTYPE.itemsize, p(spans),
                                        spans.shape[0], p(line_start), p(span_start), p(status),
                                        p(huff), 0 if huff is None else huff.shape[0], tot,
                                        _lib.QH_WHERE_DEVICE), "qh_scan_blocks_batch")
    return tot[0], tot[1], tot[2]


def scan_encoder_stream(buf, base_off: int = 0):
    """-> (consumed bytes or negative error, instructions, spans)."""
    lib = _load()
    src = _u8(buf)
    cap = src.size + 1
    lines = np.zeros(cap, dtype=FIELD_LINE_DTYPE)
    spans = np.zeros(cap, dtype=SPAN_IN_DTYPE)
    nl, ns = ctypes.c_size_t(0), ctypes.c_size_t(0)
    rv = lib.qh_qpack_scan_encoder_stream(_vp(src), src.size, base_off, _vp(lines), cap,
                                          ctypes.byref(nl), _vp(spans), cap, ctypes.byref(ns))
    return rv, lines[:nl.value], spans[:ns.value]


def put_varint(n: int, prefix: int, fb: int = 0) -> bytes:
    lib = _load()
    buf = (ctypes.c_uint8 * 16)(fb)
    end = lib.qh_qpack_put_varint(buf, n, prefix)
    k = end - ctypes.addressof(buf)
    assert k == lib.qh_qpack_put_varint_len(n, prefix)
    return bytes(buf[:k])


def _write(fn, *args, bound):
    buf = np.zeros(bound, dtype=np.uint8)
    n = fn(_vp(buf), *args)
    return buf[:n].tobytes()


def write_indexed(fb: int, idx: int, prefix: int) -> bytes:
    return _write(_load().qh_qpack_write_indexed, fb, idx, prefix, bound=16)


def write_indexed_name(fb: int, nameidx: int, prefix: int, value: bytes) -> bytes:
    """qpack_encoder_write_indexed_name (qpack.c:1851-1896)."""
    lib = _load()
    v = _u8(value)
    return _write(lib.qh_qpack_write_indexed_name, fb, nameidx, prefix, _vp(v), v.size,
                  bound=lib.qh_qpack_literal_bound(0, v.size))


def write_literal(fb: int, prefix: int, name: bytes, value: bytes) -> bytes:
    """qpack_encoder_write_literal (qpack.c:1944-2006)."""
    lib = _load()
    nm, v = _u8(name), _u8(value)
    return _write(lib.qh_qpack_write_literal, fb, prefix, _vp(nm), nm.size, _vp(v), v.size,
                  bound=lib.qh_qpack_literal_bound(nm.size, v.size))


def write_sections(plain, strs, lines, line_start):
    """Batch writer (qh_qpack_write_sections): -> (dst uint8, sections
    SPAN_IN_DTYPE), every section with a zero prefix."""
    lib = _load()
    plain = _u8(plain)
    strs = np.ascontiguousarray(strs, dtype=SPAN_IN_DTYPE)
    lines = np.ascontiguousarray(lines, dtype=FIELD_LINE_DTYPE)
    line_start = np.ascontiguousarray(line_start, dtype=np.uint32)
    nsec = line_start.size - 1
    cap = int(strs["len"].sum(dtype=np.uint64)) + 20 * lines.size + 20 * nsec + 1
    dst = np.zeros(cap, dtype=np.uint8)
    sections = np.zeros(max(nsec, 1), dtype=SPAN_IN_DTYPE)
    _lib.check(lib.qh_qpack_write_sections(_vp(plain), _vp(strs), _vp(lines), _vp(line_start), nsec,
                                           None, _vp(dst), cap, _vp(sections)),
               "qh_qpack_write_sections")
    end = int(sections["off"][nsec - 1] + sections["len"][nsec - 1]) if nsec else 0
    return dst[:end], sections[:nsec]


def synth_field_sections(seed: int, nblocks: int, fields=(4, 20), namelen=(4, 24),
                         valuelen=(1, 128), alphabet: bytes | None = None):
    """Deterministic synthetic header blocks at dynamic table 0 (config 4's
    shape; the qifs corpus itself is not available offline): per block a
    uniform number of field lines, 30% indexed static, 40% static name
    reference + value, 30% literal name + value; names and values are
    alphabet-A text (nghttp3_amd/synth.py).  Returns (src, blocks, plain,
    strs, lines, line_start)."""
    from . import synth
    alphabet = alphabet or synth.ALPHABET_A
    rng = np.random.default_rng(seed)
    nf = rng.integers(fields[0], fields[1] + 1, nblocks)
    nl = int(nf.sum())
    op = rng.choice(np.array([FL_INDEXED, FL_INDEXED_NAME, FL_LITERAL], dtype=np.uint8),
                    p=[0.3, 0.4, 0.3], size=nl)
    has_name = op == FL_LITERAL
    has_value = op != FL_INDEXED
    nlen = rng.integers(namelen[0], namelen[1] + 1, nl) * has_name
    vlen = rng.integers(valuelen[0], valuelen[1] + 1, nl) * has_value
    # strings in line order: name (if any) then value (if any)
    per = np.stack([nlen, vlen], axis=1).reshape(-1)
    present = np.stack([has_name, has_value], axis=1).reshape(-1)
    slen = per[present].astype(np.uint32)
    sidx = np.cumsum(present) - 1
    strs = np.zeros(slen.size, dtype=SPAN_IN_DTYPE)
    strs["len"] = slen
    if slen.size:
        strs["off"][1:] = np.cumsum(slen.astype(np.uint64))[:-1]
    plain = synth.fill(seed, int(slen.sum(dtype=np.uint64)), alphabet)
    lines = np.zeros(nl, dtype=FIELD_LINE_DTYPE)
    lines["opcode"] = op
    lines["index"] = rng.integers(0, 99, nl) * (op != FL_LITERAL)
    lines["name"] = np.where(has_name, sidx.reshape(-1, 2)[:, 0], -1)
    lines["value"] = np.where(has_value, sidx.reshape(-1, 2)[:, 1], -1)
    line_start = np.zeros(nblocks + 1, dtype=np.uint32)
    line_start[1:] = np.cumsum(nf)
    src, blocks = write_sections(plain, strs, lines, line_start)
    return src, blocks, plain, strs, lines, line_start


def check_header_name(name) -> int:
    """nghttp3_check_header_name (lib/nghttp3_http.c:691-709)."""
    a = _u8(name)
    return _load().nghttp3_check_header_name(_vp(a), a.size)


def check_header_value(value) -> int:
    """nghttp3_check_header_value (lib/nghttp3_http.c:798-838)."""
    a = _u8(value)
    return _load().nghttp3_check_header_value(_vp(a), a.size)


def check_fields_host(codec: HuffmanBatchCodec, src, spans):
    """Batch validation of host strings on the GPU (qh_check_fields_batch):
    spans' QH_SPAN_NAME flag selects the name check.  -> int8 verdicts."""
    lib = _load()
    src = _u8(src)
    spans = np.ascontiguousarray(spans, dtype=SPAN_IN_DTYPE)
    v = np.zeros(max(spans.size, 1), dtype=np.int8)
    _lib.check(lib.qh_check_fields_batch(codec._ctx, _vp(src), _vp(spans), spans.size, _vp(v),
                                         _lib.QH_WHERE_HOST), "qh_check_fields_batch")
    return v[:spans.size]


def check_fields_dev(codec: HuffmanBatchCodec, src, spans, verdict):
    """Device-resident form: src uint8, spans int64 [n,2] (SPAN_IN layout),
    verdict int8 [n] torch tensors; asynchronous on the codec stream."""
    lib = _load()
    _lib.check(lib.qh_check_fields_batch(codec._ctx, ctypes.c_void_p(src.data_ptr()),
                                         ctypes.c_void_p(spans.data_ptr()), spans.shape[0],
                                         ctypes.c_void_p(verdict.data_ptr()), _lib.QH_WHERE_DEVICE),
               "qh_check_fields_batch")


def lookup_token(name) -> int:
    """qpack_lookup_token (lib/nghttp3_qpack.c:342): token or -1."""
    a = _u8(name)
    return _load().qh_qpack_lookup_token(_vp(a), a.size)


def lookup_tokens_host(codec: HuffmanBatchCodec, src, spans):
    """Batch token lookup on the GPU over host strings -> int32 tokens."""
    lib = _load()
    src = _u8(src)
    spans = np.ascontiguousarray(spans, dtype=SPAN_IN_DTYPE)
    t = np.zeros(max(spans.size, 1), dtype=np.int32)
    _lib.check(lib.qh_lookup_tokens_batch(codec._ctx, _vp(src), _vp(spans), spans.size, _vp(t),
                                          _lib.QH_WHERE_HOST), "qh_lookup_tokens_batch")
    return t[:spans.size]


def lookup_tokens_dev(codec: HuffmanBatchCodec, src, spans, token):
    """Device-resident form (torch tensors: uint8 src, int64 [n,2] spans,
    int32 [n] tokens); asynchronous on the codec stream."""
    lib = _load()
    _lib.check(lib.qh_lookup_tokens_batch(codec._ctx, ctypes.c_void_p(src.data_ptr()),
                                          ctypes.c_void_p(spans.data_ptr()), spans.shape[0],
                                          ctypes.c_void_p(token.data_ptr()), _lib.QH_WHERE_DEVICE),
               "qh_lookup_tokens_batch")


class FieldSectionDecoder:
    """Whole header blocks -> every string of every block, decoded, checked
    and (names) tokenised, through one qh_decode_sections_batch call: GPU
    framing, the batch Huffman decoder, a failed Huffman string failing its
    block with -401 as read_request does (qpack.c:3604-3609, :3693-3698),
    the field name / value check and token lookup of every string.

    ``decode_blocks`` takes host arrays (the library stages them);
    ``decode_blocks_dev`` takes tensors already in HBM.  ``dtable0`` decodes
    as a decoder whose dynamic table capacity is 0 (config 4)."""

    def __init__(self, device: int = 0, codec: HuffmanBatchCodec | None = None,
                 dtable0: bool = False):
        self.codec = codec or HuffmanBatchCodec(device)
        self.opts = SECTIONS_DTABLE0 if dtable0 else 0

    def decode_blocks_dev(self, src, blocks, bufs=None):
        """src uint8 and blocks int64 [n,2] (SPAN_IN layout) torch tensors in
        HBM.  Returns a dict of torch tensors (lines, spans, strs, verdict,
        tokens, line_start, span_start, status, dst) plus the totals
        (nlines, nspans, nhuff, dst_need); `bufs` (a previous result)
        reuses its allocations.  Asynchronous after the framing sync."""
        import torch
        dev = src.device
        n = blocks.shape[0]
        b = bufs or {}
        cap = int(src.numel()) + 1  # every line and string takes >= 1 byte
        if b.get("cap", -1) < cap or b.get("n", -1) < n:
            b = {"cap": cap, "n": n,
                 "lines": torch.empty(cap * FIELD_LINE_DTYPE.itemsize, dtype=torch.uint8, device=dev),
                 "spans": torch.empty((cap, 2), dtype=torch.int64, device=dev),
                 "strs": torch.empty((cap, 2), dtype=torch.int64, device=dev),
                 "verdict": torch.empty(cap, dtype=torch.int8, device=dev),
                 "tokens": torch.empty(cap, dtype=torch.int32, device=dev),
                 "line_start": torch.empty(n + 1, dtype=torch.int32, device=dev),
                 "span_start": torch.empty(n + 1, dtype=torch.int32, device=dev),
                 "status": torch.empty(max(n, 1), dtype=torch.int32, device=dev),
                 "dst": torch.empty(64, dtype=torch.uint8, device=dev)}
        lib = _load()
        p = lambda t: t.data_ptr()
        for _ in range(2):  # a second try only when dst was too small
            st = qh_sections(p(b["lines"]), cap, p(b["spans"]), cap, p(b["strs"]), p(b["verdict"]),
                             p(b["tokens"]), p(b["line_start"]), p(b["span_start"]), p(b["status"]),
                             None, p(b["dst"]), b["dst"].numel(), 0, 0, 0, 0)
            rv = lib.qh_decode_sections_batch(self.codec._ctx, ctypes.c_void_p(src.data_ptr()),
                                              ctypes.c_void_p(blocks.data_ptr()), n, self.opts,
                                              ctypes.byref(st), _lib.QH_WHERE_DEVICE)
            if rv == _lib.QH_ERR_NOMEM and st.dst_need > b["dst"].numel():
                b["dst"] = torch.empty(int(st.dst_need), dtype=torch.uint8, device=dev)
                continue
            _lib.check(rv, "qh_decode_sections_batch")
            break
        b.update({"nlines": st.nlines, "nspans": st.nspans, "nhuff": st.nhuff,
                  "dst_need": st.dst_need})
        return b

    def decode_blocks(self, src, blocks):
        """Host arrays in and out: -> dict with lines, spans, strs
        (SPAN_OUT_DTYPE: Huffman strings in dst, raw strings in src),
        huffman (bool per span), verdict, tokens, line_start, span_start,
        status, dst."""
        lib = _load()
        src = _u8(src)
        if src.size == 0:
            src = np.zeros(1, dtype=np.uint8)
        blocks = np.ascontiguousarray(blocks, dtype=SPAN_IN_DTYPE)
        n = blocks.size
        cap = int(blocks["len"].sum(dtype=np.uint64)) + 1
        lines = np.zeros(cap, dtype=FIELD_LINE_DTYPE)
        spans = np.zeros(cap, dtype=SPAN_IN_DTYPE)
        strs = np.zeros(cap, dtype=SPAN_OUT_DTYPE)
        verdict = np.zeros(cap, dtype=np.int8)
        tokens = np.zeros(cap, dtype=np.int32)
        ls = np.zeros(n + 1, dtype=np.uint32)
        ss = np.zeros(n + 1, dtype=np.uint32)
        status = np.zeros(max(n, 1), dtype=np.int32)
        prefixes = np.zeros(max(n, 1), dtype=PREFIX_DTYPE)
        dst = np.zeros(64, dtype=np.uint8)
        for _ in range(2):
            st = qh_sections(lines.ctypes.data, cap, spans.ctypes.data, cap, strs.ctypes.data,
                             verdict.ctypes.data, tokens.ctypes.data, ls.ctypes.data, ss.ctypes.data,
                             status.ctypes.data, prefixes.ctypes.data, dst.ctypes.data, dst.size,
                             0, 0, 0, 0)
            rv = lib.qh_decode_sections_batch(self.codec._ctx, _vp(src), _vp(blocks), n, self.opts,
                                              ctypes.byref(st), _lib.QH_WHERE_HOST)
            if rv == _lib.QH_ERR_NOMEM and st.dst_need > dst.size:
                dst = np.zeros(int(st.dst_need), dtype=np.uint8)
                continue
            _lib.check(rv, "qh_decode_sections_batch")
            break
        ns = int(st.nspans)
        spans = spans[:ns]
        return {"lines": lines[:st.nlines], "spans": spans, "strs": strs[:ns],
                "huffman": (spans["flags"] & SPAN_HUFFMAN) != 0, "verdict": verdict[:ns],
                "tokens": tokens[:ns], "line_start": ls, "span_start": ss, "status": status[:n],
                "prefixes": prefixes[:n], "dst": dst}


def static_entry(idx: int):
    """qh_qpack_static_entry: (name, value) of static table entry idx."""
    lib = _load()
    n, v = ctypes.c_void_p(), ctypes.c_void_p()
    nl, vl = ctypes.c_size_t(), ctypes.c_size_t()
    _lib.check(lib.qh_qpack_static_entry(idx, ctypes.byref(n), ctypes.byref(nl), ctypes.byref(v),
                                         ctypes.byref(vl)), "qh_qpack_static_entry")
    return ctypes.string_at(n, nl.value), ctypes.string_at(v, vl.value) if vl.value else b""


def plan_fields(plain, strs, never=None):
    """qh_qpack_plan_fields: fields (strs[2i], strs[2i+1]) of plain -> the
    field lines the reference encoder writes at dynamic table capacity 0."""
    lib = _load()
    plain = _u8(plain)
    if plain.size == 0:
        plain = np.zeros(1, dtype=np.uint8)
    strs = np.ascontiguousarray(strs, dtype=SPAN_IN_DTYPE)
    nf = strs.size // 2
    lines = np.zeros(max(nf, 1), dtype=FIELD_LINE_DTYPE)
    nv = None if never is None else np.ascontiguousarray(never, dtype=np.uint8)
    _lib.check(lib.qh_qpack_plan_fields(_vp(plain), _vp(strs), nf, None if nv is None else _vp(nv),
                                        _vp(lines)), "qh_qpack_plan_fields")
    return lines[:nf]


class FieldSectionEncoder:
    """Whole field sections out of one qh_encode_sections_batch call: the
    count kernels, Huffman iff shorter, the encode kernels over the picked
    strings, then the representation writer kernel (byte for byte
    qh_qpack_write_sections)."""

    def __init__(self, device: int = 0, codec: HuffmanBatchCodec | None = None):
        self.codec = codec or HuffmanBatchCodec(device)

    def encode_sections(self, plain, strs, lines, line_start, prefixes=None):
        """Host arrays -> (dst uint8, sections SPAN_IN_DTYPE)."""
        lib = _load()
        plain = _u8(plain)
        if plain.size == 0:
            plain = np.zeros(1, dtype=np.uint8)
        strs = np.ascontiguousarray(strs, dtype=SPAN_IN_DTYPE)
        lines = np.ascontiguousarray(lines, dtype=FIELD_LINE_DTYPE)
        if lines.size == 0:
            lines = np.zeros(1, dtype=FIELD_LINE_DTYPE)[:0]
        line_start = np.ascontiguousarray(line_start, dtype=np.uint32)
        nsec = line_start.size - 1
        pf = None if prefixes is None else np.ascontiguousarray(prefixes, dtype=PREFIX_DTYPE)
        sections = np.zeros(max(nsec, 1), dtype=SPAN_IN_DTYPE)
        need = ctypes.c_uint64(0)
        dst = np.zeros(64, dtype=np.uint8)
        for _ in range(2):
            rv = lib.qh_encode_sections_batch(
                self.codec._ctx, _vp(plain), _vp(strs), strs.size, _vp(lines), _vp(line_start),
                nsec, None if pf is None else _vp(pf), _vp(dst), dst.size, _vp(sections),
                ctypes.byref(need), _lib.QH_WHERE_HOST)
            if rv == _lib.QH_ERR_NOMEM and need.value > dst.size:
                dst = np.zeros(int(need.value), dtype=np.uint8)
                continue
            _lib.check(rv, "qh_encode_sections_batch")
            break
        return dst[:need.value], sections[:nsec]

    def encode_sections_dev(self, plain, strs, lines, line_start, dst, sections, prefixes=None):
        """Device-resident form over torch tensors (plain uint8, strs int64
        [n,2], lines uint8 [nlines*24], line_start int32 [nsec+1], dst uint8,
        sections int64 [nsec,2], prefixes optional).  Returns dst_need;
        raises on QH_ERR_NOMEM."""
        lib = _load()
        p = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())
        need = ctypes.c_uint64(0)
        rv = lib.qh_encode_sections_batch(self.codec._ctx, p(plain), p(strs), strs.shape[0], p(lines),
                                          p(line_start), line_start.shape[0] - 1, p(prefixes), p(dst),
                                          dst.numel(), p(sections), ctypes.byref(need),
                                          _lib.QH_WHERE_DEVICE)
        _lib.check(rv, "qh_encode_sections_batch")
        return need.value
