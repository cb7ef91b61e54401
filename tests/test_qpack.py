"""QPACK field-line framing: the C scanners
and writers of nghttp3_amd/csrc/qh_qpack.c against the Python restatement
oracle/qpack_frame.py, both pinned by the reference's fuzz corpus file
tests/golden/netbsd-hq.out.256.100.1 (fuzz/corpus/fuzz_qpackdecoder/):

* the compiled reference CLI decoded it into an 18-block, 217-line QIF
  (SURVEY.md section 8c): 199 field lines plus one blank line per block;
* every byte of it was written by the reference encoder, so re-writing each
  field section and the encoder stream from the scanned lines and the
  decoded strings must reproduce it byte for byte (put_varint,
  Huffman-iff-shorter, first bytes and prefixes, qpack.c:1851-2069).

The GPU leg (decode of the scanned Huffman spans through qh_decode_batch)
is in tests/test_gpu.py.
"""
import os
import random

import numpy as np
import pytest

import oracle
from oracle import qpack_frame as ref
from nghttp3_amd import qpack
from nghttp3_amd.qpack_huffman import SPAN_IN_DTYPE

from conftest import GOLDEN

CORPUS = os.path.join(GOLDEN, "netbsd-hq.out.256.100.1")


@pytest.fixture(scope="module")
def netbsd():
    data = open(CORPUS, "rb").read()
    return data, ref.read_qif_out(data)


def _tuples(lines, spans):
    lt = [(int(l["opcode"]), int(l["flags"]), int(l["index"]), int(l["name"]), int(l["value"]))
          for l in lines]
    st = [(int(s["off"]), int(s["len"]), int(s["flags"])) for s in spans]
    return lt, st


def _string(data, span):
    off, n, fl = span
    raw = data[off:off + n]
    if fl & ref.SPAN_HUFFMAN:
        st, out = oracle.decode_one(raw)
        assert st == 0
        return out
    return raw


def _rewrite_section(data, prefix, lines, spans):
    """Re-encode a field section with the oracle writers."""
    ricnt, sign, dbase = prefix
    out = ref.put_varint(ricnt, 8) + ref.put_varint(dbase, 7, 0x80 if sign else 0)
    for op, fl, idx, name, value in lines:
        never = bool(fl & ref.NEVER)
        dyn = bool(fl & ref.DYNAMIC)
        if op == ref.FL_INDEXED:
            out += ref.write_indexed(0x80 if dyn else 0xC0, idx, 6)
        elif op == ref.FL_INDEXED_PB:
            out += ref.write_indexed(0x10, idx, 4)
        elif op == ref.FL_INDEXED_NAME:
            fb = 0x40 | (0x20 if never else 0) | (0 if dyn else 0x10)
            out += ref.write_indexed_name(fb, idx, 4, _string(data, spans[value]))
        elif op == ref.FL_INDEXED_NAME_PB:
            out += ref.write_indexed_name(0x08 if never else 0, idx, 3, _string(data, spans[value]))
        else:
            out += ref.write_literal(0x20 | (0x10 if never else 0), 3, _string(data, spans[name]),
                                     _string(data, spans[value]))
    return out


def test_netbsd_corpus_shape_matches_reference_cli(netbsd):
    data, recs = netbsd
    blocks = [r for r in recs if r[0] != 0]
    assert len(blocks) == 18
    nlines = 0
    for sid, off, n in blocks:
        st, prefix, lines, spans = ref.scan_field_section(data[off:off + n], off)
        assert st == 0
        nlines += len(lines)
    # the QIF the CLI wrote holds one line per field plus one blank line
    # closing each block: 199 + 18 = 217
    assert nlines + len(blocks) == 217
    assert nlines == 199


def test_c_scanner_matches_oracle_on_netbsd(netbsd):
    data, recs = netbsd
    for sid, off, n in recs:
        if sid == 0:
            rv, ins, sp = qpack.scan_encoder_stream(data[off:off + n], off)
            rrv, rins, rsp = ref.scan_encoder_stream(data[off:off + n], off)
            assert rv == rrv == n
            assert _tuples(ins, sp) == (rins, rsp)
            continue
        st, prefix, lines, spans = qpack.scan_field_section(data[off:off + n], off)
        rst, rprefix, rlines, rspans = ref.scan_field_section(data[off:off + n], off)
        assert st == rst == 0 and prefix == rprefix
        assert _tuples(lines, spans) == (rlines, rspans)


def test_netbsd_strings_all_decode(netbsd):
    data, recs = netbsd
    nh = 0
    for sid, off, n in recs:
        if sid == 0:
            _, _, spans = ref.scan_encoder_stream(data[off:off + n], off)
        else:
            _, _, _, spans = ref.scan_field_section(data[off:off + n], off)
        for s in spans:
            txt = _string(data, s)
            assert all(0x20 <= c < 0x7F for c in txt), txt
            nh += bool(s[2] & ref.SPAN_HUFFMAN)
    assert nh > 0


def test_oracle_writers_reproduce_netbsd_byte_for_byte(netbsd):
    data, recs = netbsd
    for sid, off, n in recs:
        blk = data[off:off + n]
        if sid != 0:
            st, prefix, lines, spans = ref.scan_field_section(blk, off)
            assert _rewrite_section(data, prefix, lines, spans) == blk
        else:
            rv, ins, spans = ref.scan_encoder_stream(blk, off)
            out = b""
            for op, fl, idx, name, value in ins:
                if op == ref.ES_INSERT_INDEXED:
                    out += ref.write_indexed_name(0x80 if fl & ref.DYNAMIC else 0xC0, idx, 6,
                                                  _string(data, spans[value]))
                elif op == ref.ES_INSERT:
                    out += ref.write_literal(0x40, 5, _string(data, spans[name]),
                                             _string(data, spans[value]))
                elif op == ref.ES_SET_DTABLE_CAP:
                    out += ref.write_indexed(0x20, idx, 5)
                else:
                    out += ref.write_indexed(0x00, idx, 5)
            assert out == blk


def _random_field(rng):
    alpha = b"abcdefghijklmnopqrstuvwxyz0123456789-_/.:;=%ABCXYZ"
    val = bytes(rng.choice(alpha) for _ in range(rng.choice([0, 1, 3, 7, 30, 127, 128, 300])))
    if rng.random() < 0.2:
        val = bytes(rng.randrange(256) for _ in range(rng.randrange(40)))
    name = bytes(rng.choice(alpha[:36]) for _ in range(rng.choice([1, 4, 6, 12, 31, 40])))
    return name, val


def test_c_writers_match_oracle_writers():
    rng = random.Random(0x5EED0F1)
    for _ in range(400):
        name, val = _random_field(rng)
        never = 0x20 if rng.random() < 0.2 else 0
        idx = rng.choice([0, 14, 15, 16, 98, 127, 128, 10000, (1 << 62) - 1])
        assert qpack.write_indexed_name(0x50 | never, idx, 4, val) == \
            ref.write_indexed_name(0x50 | never, idx, 4, val)
        assert qpack.write_literal(0x20, 3, name, val) == ref.write_literal(0x20, 3, name, val)
        assert qpack.write_literal(0x40, 5, name, val) == ref.write_literal(0x40, 5, name, val)
        assert qpack.write_indexed(0xC0, idx, 6) == ref.write_indexed(0xC0, idx, 6)
        for p in (3, 4, 5, 6, 7, 8):
            assert qpack.put_varint(idx, p) == ref.put_varint(idx, p)


def _synth_section(rng, nfields):
    out = ref.put_varint(0, 8) + ref.put_varint(0, 7)
    for _ in range(nfields):
        name, val = _random_field(rng)
        r = rng.random()
        if r < 0.3:
            out += ref.write_indexed(0xC0, rng.randrange(99), 6)
        elif r < 0.65:
            out += ref.write_indexed_name(0x50, rng.randrange(99), 4, val)
        else:
            out += ref.write_literal(0x20, 3, name, val)
    return out


def test_c_scanner_matches_oracle_on_synthetic_sections_and_errors():
    rng = random.Random(0x5EED0F2)
    cases = []
    for _ in range(60):
        sec = _synth_section(rng, rng.randrange(0, 20))
        cases.append(sec)
        # every truncation of the section (fin on an unfinished line)
        for cut in sorted(set(rng.randrange(len(sec) + 1) for _ in range(6))):
            cases.append(sec[:cut])
        # random byte flips
        b = bytearray(sec)
        b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
        cases.append(bytes(b))
    cases += [
        b"", b"\x00", b"\xff", b"\x00\x00",
        b"\x00\x00" + b"\x2f" + b"\xff" * 12,              # name length overflow
        b"\x00\x00\x27\xfa\x01" + b"a" * 257,               # raw name of 257 > 256
        b"\x00\x00\x2f\xe2\x00" + b"\x00" * 240,            # Huffman name est > 256
        b"\x00\x00\x50\x7f\x81\x80\x04" + b"a" * 10,        # value 65536+1... truncated
        b"\x00\x00\xd1", b"\x00\x00\x10", b"\x00\x00\x00\x00",
    ]
    cases += [b"\x00\x00" + ref.write_indexed(0xC0, rng.randrange(99, 300), 6) for _ in range(4)]
    for sec in cases:
        st, prefix, lines, spans = qpack.scan_field_section(sec, 7)
        rst, rprefix, rlines, rspans = ref.scan_field_section(sec, 7)
        assert st == rst, sec
        assert prefix == rprefix
        assert _tuples(lines, spans) == (rlines, rspans)


def test_table_free_index_checks_match_oracle():
    """Checks brel2abs / pbrel2abs / validate_index / the sign rule make
    whatever the dynamic table holds (qpack.c:3414-3418, :3971-4017,
    :2787-2798)."""
    bad = qpack.QH_ERR_QPACK_DECOMPRESSION_FAILED
    v = ref.write_indexed_name(0x50, 3, 4, b"abc")
    cases = {
        b"\x00\x00" + ref.write_indexed(0xC0, 98, 6): 0,        # last static entry
        b"\x00\x00" + ref.write_indexed(0xC0, 99, 6): bad,      # past the static table
        b"\x00\x00" + ref.write_indexed_name(0x50, 99, 4, b"x"): bad,
        b"\x00\x00" + ref.write_indexed_name(0x50, 200, 4, b"x"): bad,
        b"\x00\x00" + ref.write_indexed(0x80, 0, 6): bad,       # dynamic, ricnt 0
        b"\x00\x00" + ref.write_indexed(0x10, 0, 4): bad,       # post-base, ricnt 0
        b"\x00\x00" + ref.write_indexed_name(0x40, 0, 4, b"x"): bad,
        b"\x00\x00" + ref.write_indexed_name(0x00, 0, 3, b"x"): bad,
        b"\x00\x80" + v: bad,                                     # sign with ricnt 0
        b"\x02\x80" + v: 0,                                       # needs table state
        b"\x02\x00" + ref.write_indexed(0x80, 0, 6): 0,         # dynamic, ricnt > 0
        b"\x00\x00" + v + ref.write_indexed(0xC0, 120, 6): bad,  # after a good line
    }
    for sec, want in cases.items():
        st, _, lines, spans = qpack.scan_field_section(sec)
        rst, _, rlines, rspans = ref.scan_field_section(sec)
        assert st == rst == want, sec
        assert _tuples(lines, spans) == (rlines, rspans)
    # the failed block keeps the string read before the error (its value)
    st, _, lines, spans = qpack.scan_field_section(b"\x00\x00" + v + ref.write_indexed(0xC0, 120, 6))
    assert st == bad and lines.size == 0 and spans.size == 1
    # capacity 0 (config 4): any Required Insert Count but 0 fails
    assert ref.scan_field_section(b"\x02\x00" + v, dtable0=True)[0] == bad
    assert ref.scan_field_section(b"\x00\x00" + v, dtable0=True)[0] == 0
    # encoder stream: a static name reference must be < 99 (rel2abs)
    es = ref.write_indexed_name(0xC0, 99, 6, b"v")
    assert qpack.scan_encoder_stream(es)[0] == ref.scan_encoder_stream(es)[0] == \
        qpack.QH_ERR_QPACK_ENCODER_STREAM_ERROR
    es = ref.write_indexed_name(0xC0, 98, 6, b"v")
    assert qpack.scan_encoder_stream(es)[0] == ref.scan_encoder_stream(es)[0] == len(es)


def test_decode_field_section_error_order():
    """A Huffman string that fails before a framing error decides the block
    (-401, qpack.c:3604-3609), as the streaming reference meets it first."""
    bad_h = b"\x81\x00"          # H=1, 1 byte, zero padding: -108
    too_big = ref.put_varint(65537, 7) + b"a" * 65537
    sec = b"\x00\x00\x50" + bad_h + b"\x50" + too_big
    assert ref.scan_field_section(sec)[0] == qpack.QH_ERR_QPACK_HEADER_TOO_LARGE
    st, lines, spans, strings = ref.decode_field_section(sec)
    assert st == qpack.QH_ERR_QPACK_DECOMPRESSION_FAILED and strings == [None]
    sec = b"\x00\x00\x50\x03abc\x50" + too_big
    assert ref.decode_field_section(sec)[0] == qpack.QH_ERR_QPACK_HEADER_TOO_LARGE


def test_value_too_large_is_header_too_large():
    sec = b"\x00\x00\x50" + ref.put_varint(65537, 7) + b"a" * 65537
    assert qpack.scan_field_section(sec)[0] == qpack.QH_ERR_QPACK_HEADER_TOO_LARGE
    sec = b"\x00\x00\x50" + ref.put_varint(65536, 7) + b"a" * 65536
    assert qpack.scan_field_section(sec)[0] == 0
    # Huffman: 41944 * 8 // 5 = 67110 > 65536
    sec = b"\x00\x00\x50" + ref.put_varint(41944, 7, 0x80) + b"\xff" * 41944
    assert qpack.scan_field_section(sec)[0] == qpack.QH_ERR_QPACK_HEADER_TOO_LARGE


def test_encoder_stream_partial_and_errors():
    rng = random.Random(0x5EED0F3)
    es = b""
    for _ in range(40):
        name, val = _random_field(rng)
        es += rng.choice([
            ref.write_literal(0x40, 5, name, val),
            ref.write_indexed_name(0xC0, rng.randrange(99), 6, val),
            ref.write_indexed(0x20, rng.randrange(5000), 5),
            ref.write_indexed(0x00, rng.randrange(50), 5),
        ])
    for cut in list(range(0, len(es), max(1, len(es) // 50))) + [len(es)]:
        c = qpack.scan_encoder_stream(es[:cut], 3)
        r = ref.scan_encoder_stream(es[:cut], 3)
        assert c[0] == r[0]
        assert _tuples(c[1], c[2]) == (r[1], r[2])
    for bad in [b"\x3f" + b"\xff" * 12, b"\x5f" + b"\xff" * 12, b"\x7f\x82\x01"]:
        c = qpack.scan_encoder_stream(bad)
        r = ref.scan_encoder_stream(bad)
        assert c[0] == r[0] < 0
    assert qpack.scan_encoder_stream(b"\x7f\x82\x01")[0] == qpack.QH_ERR_QPACK_HEADER_TOO_LARGE
    assert qpack.scan_encoder_stream(b"\x3f" + b"\xff" * 12)[0] == \
        qpack.QH_ERR_QPACK_ENCODER_STREAM_ERROR


def test_scan_blocks_matches_per_section_scan():
    rng = random.Random(0x5EED0F4)
    secs = [_synth_section(rng, rng.randrange(0, 15)) for _ in range(100)]
    secs[5] = secs[5][:-1] if secs[5][2:] else b""       # a bad block
    secs[17] = b"\x00\x00\x2f" + b"\xff" * 12              # another
    src = b"".join(secs)
    blocks = np.zeros(len(secs), dtype=SPAN_IN_DTYPE)
    blocks["len"] = [len(s) for s in secs]
    blocks["off"][1:] = np.cumsum(blocks["len"].astype(np.uint64))[:-1]
    lines, spans, ls, ss, status = qpack.scan_blocks(src, blocks)
    for i, sec in enumerate(secs):
        rst, _, rlines, rspans = ref.scan_field_section(sec, int(blocks["off"][i]))
        assert status[i] == rst
        lt, st = _tuples(lines[ls[i]:ls[i + 1]], spans[ss[i]:ss[i + 1]])
        # span indices are batch-global in scan_blocks
        rlines = [(o, f, x, n + ss[i] if n >= 0 else -1, v + ss[i] if v >= 0 else -1)
                  for o, f, x, n, v in rlines]
        assert (lt, st) == (rlines, rspans)
    assert status[17] == qpack.QH_ERR_QPACK_DECOMPRESSION_FAILED


def test_section_writer_matches_oracle_and_round_trips():
    src, blocks, plain, strs, lines, ls = qpack.synth_field_sections(0x5EED0004, 300)
    pb = bytes(plain)
    for b in range(300):
        sec = bytes(src[blocks["off"][b]:blocks["off"][b] + blocks["len"][b]])
        # oracle writers over the same lines
        exp = ref.put_varint(0, 8) + ref.put_varint(0, 7)
        for l in lines[ls[b]:ls[b + 1]]:
            op, idx = int(l["opcode"]), int(l["index"])
            s = lambda k: pb[int(strs["off"][k]):int(strs["off"][k]) + int(strs["len"][k])]
            if op == ref.FL_INDEXED:
                exp += ref.write_indexed(0xC0, idx, 6)
            elif op == ref.FL_INDEXED_NAME:
                exp += ref.write_indexed_name(0x50, idx, 4, s(int(l["value"])))
            else:
                exp += ref.write_literal(0x20, 3, s(int(l["name"])), s(int(l["value"])))
        assert sec == exp
        # scanning it back gives the same lines, and the strings decode back
        st, prefix, rlines, rspans = ref.scan_field_section(sec)
        assert st == 0 and prefix == (0, 0, 0)
        assert [r[0] for r in rlines] == list(lines["opcode"][ls[b]:ls[b + 1]])
        got = [_string(sec, sp) for sp in rspans]
        want = [s(int(k)) for l in lines[ls[b]:ls[b + 1]] for k in (l["name"], l["value"]) if k >= 0]
        assert got == want
    # the whole batch through the C batch scanner
    lines2, spans2, ls2, ss2, status = qpack.scan_blocks(src, blocks)
    assert (status == 0).all()
    assert (ls2 == ls).all()
    assert (lines2["opcode"] == lines["opcode"]).all() and (lines2["index"] == lines["index"]).all()
    assert (spans2["flags"] & qpack.SPAN_NAME != 0).sum() == (lines["name"] >= 0).sum()
