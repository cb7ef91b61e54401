"""TEST INFRASTRUCTURE ONLY: pure-Python restatement of the reference's QPACK
CLI (examples/qpack.cc, qpack_encode.cc, qpack_decode.cc) and of the parts
of lib/nghttp3_qpack.c it exercises, as the checker of the QIF driver
(nghttp3_amd/csrc/qh_qif.cc, config 1).

* ``parse_qif`` -- qpack_encode.cc:149-183: blocks of "name<TAB>value"
  lines separated by an empty line, leading spaces of the value dropped,
  at most 1024 fields per block, the first empty block ends the input.
* ``encode_qif`` -- qpack_encode.cc:109-218 with the encoder at dynamic
  table capacity 0 (-s 0): every block is one field section with prefix
  00 00 (write_field_section_prefix :2424-2460 with ricnt 0, base 0) and
  the representations nghttp3_qpack_encoder_encode_nv :1455-1628 picks
  when nothing can be inserted (lookup_stable :1630-1660 over the static
  table in token_stable order, decide_indexing_mode's NEVER cases
  :1307-1321); the encoder stream stays empty, so only request-stream
  records (stream ids 1, 2, ...) are written (:194-197, :97-107).
* ``decode_wire`` -- qpack_decode.cc:192-296 over the qpack-05 records
  (u64 stream id, u32 length, big endian; stream 0 = encoder stream), with
  the decoder's dynamic table: read_encoder :2815-3150 (set capacity
  :2895-2910 -> set_max_dtable_capacity :3159-3185, rel2abs :3952-3969,
  the inserts :3187-3306 with the capacity checks, eviction in
  context_dtable_add :2071-2127), read_request :3347-3805 (ricnt
  reconstruction :3915-3950, base :3419-3429, blocking :3431-3436,
  brel2abs / pbrel2abs :3971-4017, validate_index :2787-2798, emit
  :4020-4136), blocked streams released in Required-Insert-Count order
  (qpack_decode.cc:154-174, qpack_decode.h:52-59), write_header :179-190.

The static table is read from tests/golden/static_table.json (the
reference's stable[] and token_stable[] parsed as text by
tests/golden/gen_static.py); the Huffman strings go through the oracle
codec.  Pinned by the reference's corpus file: decoding
netbsd-hq.out.256.100.1 at -s 256 gives the 18-block, 217-line QIF
(SURVEY.md section 8c).
"""
from __future__ import annotations

import heapq
import json
import os

from . import decode_one
from . import qpack_frame as qf

ENTRY_OVERHEAD = 32  # NGHTTP3_QPACK_ENTRY_OVERHEAD
MAX_FIELDS = 1024   # qpack_encode.cc:142

_HERE = os.path.dirname(os.path.abspath(__file__))
_STATIC = None


class QifError(Exception):
    pass


def static_table():
    """-> (entries [(name, value)], token_stable [absidx, ...] grouped by
    name in the reference's order, {name: [absidx, ...]})."""
    global _STATIC
    if _STATIC is None:
        path = os.path.join(_HERE, "..", "tests", "golden", "static_table.json")
        d = json.load(open(path))
        ents = [(e["name"].encode(), e["value"].encode()) for e in d["stable"]]
        by_name = {}
        for e in d["token_stable"]:
            by_name.setdefault(ents[e["absidx"]][0], []).append(e["absidx"])
        _STATIC = (ents, [e["absidx"] for e in d["token_stable"]], by_name)
    return _STATIC


def parse_qif(text: bytes):
    """-> list of blocks, each a list of (name, value) bytes pairs."""
    lines = text.split(b"\n")
    if lines and lines[-1] == b"":  # getline: no empty line after the last '\n'
        lines.pop()
    blocks, cur, k = [], [], 0
    while True:
        cur = []
        while k < len(lines):
            line = lines[k]
            k += 1
            if line == b"":
                break
            if len(cur) == MAX_FIELDS:
                raise QifError("too many headers")
            d = line.find(b"\t")
            if d < 0:
                raise QifError("no TAB")
            cur.append((line[:d], line[d + 1:].lstrip(b" ")))
        if not cur:
            return blocks
        blocks.append(cur)


def plan_field(name: bytes, value: bytes, never: bool = False):
    """encode_nv at capacity 0 -> (opcode, static index or 0)."""
    ents, _, by_name = static_table()
    idxs = by_name.get(name)
    if idxs is None:
        return qf.FL_LITERAL, 0
    mode_never = never or name == b"authorization" or (name == b"cookie" and len(value) < 20)
    if not mode_never:
        for i in idxs:
            if ents[i][1] == value:
                return qf.FL_INDEXED, i
    return qf.FL_INDEXED_NAME, idxs[0]


def encode_section(fields) -> bytes:
    out = b"\x00\x00"
    for name, value in fields:
        op, idx = plan_field(name, value)
        if op == qf.FL_INDEXED:
            out += qf.write_indexed(0xC0, idx, 6)
        elif op == qf.FL_INDEXED_NAME:
            out += qf.write_indexed_name(0x50, idx, 4, value)
        else:
            out += qf.write_literal(0x20, 3, name, value)
    return out


def encode_qif(text: bytes) -> bytes:
    out = bytearray()
    for sid, fields in enumerate(parse_qif(text), start=1):
        payload = encode_section(fields)
        out += sid.to_bytes(8, "big") + len(payload).to_bytes(4, "big") + payload
    return bytes(out)


class _Decoder:
    def __init__(self, max_dtable: int):
        self.hard_max = max_dtable
        self.cap = max_dtable  # Decoder::init sets it to the maximum
        self.size = 0
        self.table = []  # newest first: table[0] has absidx next_absidx - 1
        self.next_absidx = 0

    def _add(self, name, value, code):
        space = len(name) + len(value) + ENTRY_OVERHEAD
        if space > self.cap:
            raise QifError(code)
        while self.size + space > self.cap:
            n, v = self.table.pop()
            self.size -= len(n) + len(v) + ENTRY_OVERHEAD
        self.table.insert(0, (name, value))
        self.size += space
        self.next_absidx += 1

    def _get(self, absidx):
        return self.table[self.next_absidx - absidx - 1]

    def _valid_dyn(self, absidx):
        return absidx < self.next_absidx and self.next_absidx - absidx - 1 < len(self.table)

    def read_encoder(self, buf: bytes):
        rv, ins, spans = qf.scan_encoder_stream(buf)
        if rv < 0 or rv != len(buf):
            raise QifError(qf.ENCODER_STREAM_ERROR if rv >= 0 else rv)
        strs = [_string(buf, s) for s in spans]
        ents = static_table()[0]
        for op, fl, index, name, value in ins:
            if op == qf.ES_SET_DTABLE_CAP:
                if index > self.hard_max:
                    raise QifError(qf.ENCODER_STREAM_ERROR)
                self.cap = index
                while self.size > self.cap:
                    n, v = self.table.pop()
                    self.size -= len(n) + len(v) + ENTRY_OVERHEAD
                continue
            if op == qf.ES_INSERT:
                self._add(strs[name], strs[value], qf.ENCODER_STREAM_ERROR)
                continue
            # rel2abs
            if fl & qf.DYNAMIC:
                if self.next_absidx < index + 1:
                    raise QifError(qf.ENCODER_STREAM_ERROR)
                absidx = self.next_absidx - index - 1
                if not self._valid_dyn(absidx):
                    raise QifError(qf.ENCODER_STREAM_ERROR)
                ent = self._get(absidx)
            else:
                if index >= len(ents):
                    raise QifError(qf.ENCODER_STREAM_ERROR)
                ent = ents[index]
            if op == qf.ES_DUPLICATE:
                self._add(ent[0], ent[1], qf.ENCODER_STREAM_ERROR)
            else:
                self._add(ent[0], strs[value], qf.ENCODER_STREAM_ERROR)

    def ricnt(self, encricnt):
        if encricnt == 0:
            return 0
        max_ents = self.hard_max // ENTRY_OVERHEAD
        full = 2 * max_ents
        if encricnt > full:
            raise QifError(qf.DECOMPRESSION_FAILED)
        mx = self.next_absidx + max_ents
        r = mx // full * full + encricnt - 1
        if r > mx:
            if r <= full:
                raise QifError(qf.DECOMPRESSION_FAILED)
            r -= full
        if r == 0:
            raise QifError(qf.DECOMPRESSION_FAILED)
        return r

    def emit(self, buf, ricnt, base, lines, strs):
        ents = static_table()[0]
        out = []
        bad = qf.DECOMPRESSION_FAILED
        for op, fl, index, name, value in lines:
            dyn = bool(fl & qf.DYNAMIC)
            if op in (qf.FL_INDEXED, qf.FL_INDEXED_NAME):
                if dyn:
                    if base < index + 1:
                        raise QifError(bad)
                    absidx = base - index - 1
                    if absidx >= ricnt or not self._valid_dyn(absidx):
                        raise QifError(bad)
                    ent = self._get(absidx)
                else:
                    if index >= len(ents):
                        raise QifError(bad)
                    ent = ents[index]
            elif op in (qf.FL_INDEXED_PB, qf.FL_INDEXED_NAME_PB):
                absidx = index + base
                if absidx >= ricnt or not self._valid_dyn(absidx):
                    raise QifError(bad)
                ent = self._get(absidx)
            else:
                ent = None
            if op in (qf.FL_INDEXED, qf.FL_INDEXED_PB):
                out.append(ent)
            elif op == qf.FL_LITERAL:
                out.append((strs[name], strs[value]))
            else:
                out.append((ent[0], strs[value]))
        return out


def _string(buf, span):
    off, n, fl = span
    raw = bytes(buf[off:off + n])
    if fl & qf.SPAN_HUFFMAN:
        st, out = decode_one(raw)
        if st != 0:
            raise QifError(qf.DECOMPRESSION_FAILED)
        return out
    return raw


def _write_header(out: bytearray, headers):
    for n, v in headers:
        out += n + b"\t" + v + b"\n"
    out += b"\n"


def decode_wire(data: bytes, max_dtable: int = 0, max_blocked: int = 0) -> bytes:
    """The QIF qpack_decode writes for `data` (raises QifError on an error)."""
    dec = _Decoder(max_dtable)
    out = bytearray()
    blocked = []  # heap of (ricnt, seq, buf, base, lines, strs)
    seq = 0
    for sid, off, n in qf.read_qif_out(data):
        buf = data[off:off + n]
        if sid == 0:
            dec.read_encoder(buf)
            while blocked and blocked[0][0] <= dec.next_absidx:
                ric, _, b, base, lines, strs = heapq.heappop(blocked)
                _write_header(out, dec.emit(b, ric, base, lines, strs))
            continue
        st, prefix, lines, spans = qf.scan_field_section(buf)
        strs = [_string(buf, s) for s in spans]
        if st != 0:
            raise QifError(st)
        encricnt, sign, dbase = prefix
        ric = dec.ricnt(encricnt)
        if sign:
            if ric <= dbase:
                raise QifError(qf.DECOMPRESSION_FAILED)
            base = ric - dbase - 1
        else:
            base = ric + dbase
        if ric > dec.next_absidx:
            if len(blocked) >= max_blocked:
                raise QifError("too many blocked streams")
            heapq.heappush(blocked, (ric, seq, buf, base, lines, strs))
            seq += 1
            continue
        _write_header(out, dec.emit(buf, ric, base, lines, strs))
    if blocked:
        raise QifError("streams still blocked")
    return bytes(out)
