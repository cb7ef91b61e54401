"""The QIF driver (config 1; nghttp3_amd/csrc/qh_qif.cc, the counterpart of
examples/qpack.cc, qpack_encode.cc, qpack_decode.cc) and the encoder-side
library pieces it uses, on the CPU:

* the static table (qh_qpack_static_entry) against the reference's
  stable[] / token_stable[] as parsed into tests/golden/static_table.json;
* qh_qpack_plan_fields against the oracle's restatement of encode_nv at
  dynamic table capacity 0 (oracle/qpack_qif.py);
* the oracle's CLI restatement against the reference's corpus file: 18
  blocks, 217 QIF lines (tests/golden/netbsd.qif);
* the driver in --scalar mode (the library's scalar drop-ins, no GPU):
  decode of the corpus at -s 256 -m 100, blocked streams, config-1 encode
  byte for byte against the oracle, round trips, and the reference CLI's
  failures.
The GPU mode of the same driver is tested in tests/test_gpu_qif.py.
"""
import json
import os
import random
import subprocess

import numpy as np
import pytest

import oracle
from oracle import qpack_frame as qf
from oracle import qpack_qif as oq
from nghttp3_amd import qif, qpack
from nghttp3_amd.qpack_huffman import SPAN_IN_DTYPE

from conftest import GOLDEN

CORPUS = os.path.join(GOLDEN, "netbsd-hq.out.256.100.1")
NETBSD_QIF = os.path.join(GOLDEN, "netbsd.qif")


def test_static_table_matches_reference():
    d = json.load(open(os.path.join(GOLDEN, "static_table.json")))
    assert len(d["stable"]) == 99
    for i, e in enumerate(d["stable"]):
        assert qpack.static_entry(i) == (e["name"].encode(), e["value"].encode()), i
    tokens = json.load(open(os.path.join(GOLDEN, "tokens.json")))["tokens"]
    # token_stable: sorted by (token, index); token t's entries start at t
    order = [(tokens[d["stable"][e["absidx"]]["name"]], e["absidx"]) for e in d["token_stable"]]
    assert order == sorted(order)
    for k, (t, _) in enumerate(order):
        if k == 0 or order[k - 1][0] != t:
            assert t == k


def _plan_c(fields, never=None):
    plain = b"".join(n + v for n, v in fields)
    strs = np.zeros(2 * len(fields), dtype=SPAN_IN_DTYPE)
    o = 0
    for i, (n, v) in enumerate(fields):
        strs[2 * i] = (o, len(n), 0)
        strs[2 * i + 1] = (o + len(n), len(v), 0)
        o += len(n) + len(v)
    return qpack.plan_fields(plain, strs, never)


def test_plan_fields_matches_oracle():
    ents = oq.static_table()[0]
    rng = random.Random(0x5EED0F2)
    fields = list(ents)  # every entry: name and value match
    fields += [(n, v + b"x") for n, v in ents]  # name only
    fields += [(b"authorization", b""), (b"authorization", b"Basic x"),
               (b"cookie", b""), (b"cookie", b"a" * 19), (b"cookie", b"a" * 20),
               (b"x-custom", b""), (b"host", b"example.com"), (b":path", b"/"),
               (b"content-length", b"0"), (b"Content-Length", b"0"), (b"", b"")]
    alpha = b"abcdefghijklmnopqrstuvwxyz-:"
    for _ in range(300):
        n = rng.choice([e[0] for e in ents] + [bytes(rng.choice(alpha) for _ in range(rng.randrange(1, 12)))])
        v = rng.choice([b"", b"0", b"/", b"gzip", b"GET", b"200", b"*", b"no-cache"])
        fields.append((n, v))
    for never in (None, [1] * len(fields)):
        lines = _plan_c(fields, never)
        for i, (n, v) in enumerate(fields):
            op, idx = oq.plan_field(n, v, never=bool(never))
            l = lines[i]
            assert (int(l["opcode"]), int(l["index"])) == (op, idx), (n, v, never)
            assert int(l["flags"]) == (qf.NEVER if never else 0)
            assert int(l["name"]) == (2 * i if op == qf.FL_LITERAL else -1)
            assert int(l["value"]) == (-1 if op == qf.FL_INDEXED else 2 * i + 1)


def test_oracle_decodes_corpus_to_217_line_qif():
    data = open(CORPUS, "rb").read()
    out = oq.decode_wire(data, 256, 100)
    assert out == open(NETBSD_QIF, "rb").read()
    assert out.count(b"\n") == 217
    blocks = oq.parse_qif(out)
    assert len(blocks) == 18 and sum(map(len, blocks)) == 199


def test_config1_qif_shape():
    t = qif.synth_config1()
    blocks = oq.parse_qif(t)
    assert sum(map(len, blocks)) == 1024
    assert all(any(n == b"cookie" for n, _ in b) for b in blocks[:-1])
    assert oq.decode_wire(oq.encode_qif(t)) == t
    assert qif.synth_config1() == t  # deterministic


def _run(tmp_path, args, data, name="in"):
    src = tmp_path / name
    src.write_bytes(data)
    dst = tmp_path / (name + ".out")
    r = qif.run(args[:-1] + [args[-1], str(src), str(dst)])
    return r, (dst.read_bytes() if dst.exists() else None)


def test_driver_scalar_decodes_corpus(tmp_path):
    r, out = _run(tmp_path, ["--scalar", "-s", "256", "-m", "100", "decode"],
                  open(CORPUS, "rb").read())
    assert r.returncode == 0, r.stderr
    assert out == open(NETBSD_QIF, "rb").read()


def test_driver_scalar_carries_partial_encoder_instructions(tmp_path):
    """Every encoder-stream record cut in two records at its middle byte (an
    instruction split across them): the decoder keeps the partial
    instruction until the next encoder-stream record completes it, as the
    reference's read_encoder does; the QIF is the corpus's."""
    import struct
    data = open(CORPUS, "rb").read()
    recs = qf.read_qif_out(data)
    out = []
    nsplit = 0
    for sid, off, n in recs:
        body = data[off:off + n]
        if sid == 0 and n >= 2:
            h = n // 2
            out.append(struct.pack(">QI", 0, h) + body[:h])
            out.append(struct.pack(">QI", 0, n - h) + body[h:])
            nsplit += 1
        else:
            out.append(data[off - 12:off + n])
    assert nsplit > 0
    r, got = _run(tmp_path, ["--scalar", "-s", "256", "-m", "100", "decode"], b"".join(out))
    assert r.returncode == 0, r.stderr
    assert got == open(NETBSD_QIF, "rb").read()


def test_driver_scalar_blocks_before_decoding(tmp_path):
    """A request record with a bad Huffman string, moved ahead of the
    encoder-stream record before it: the reference decoder reads the
    section prefix, blocks the stream (Required Insert Count > inserts so
    far) and only decodes the representations when it is unblocked, so at
    -m 0 the error is the blocking one, and at -m 100 the Huffman one
    (DECOMPRESSION_FAILED) once the inserts arrive."""
    data = open(CORPUS, "rb").read()
    recs = qf.read_qif_out(data)
    raw = [bytearray(data[off - 12:off + n]) for _, off, n in recs]
    sids = [sid for sid, _, _ in recs]
    for k in range(1, len(raw)):
        if sids[k] != 0 and sids[k - 1] == 0:
            st, _, _, spans = qf.scan_field_section(bytes(raw[k][12:]), 0)
            hs = [sp for sp in spans if sp[2] & qf.SPAN_HUFFMAN]
            if st == 0 and hs:
                o, n, _ = hs[0]
                raw[k][12 + o + n - 1] = 0x00  # zero padding: an invalid string
                raw[k - 1], raw[k] = raw[k], raw[k - 1]
                break
    else:
        pytest.fail("no request record after an encoder-stream record")
    wire = b"".join(bytes(x) for x in raw)
    r, _ = _run(tmp_path, ["--scalar", "-s", "256", "-m", "0", "decode"], wire, "m0")
    assert r.returncode != 0 and "blocked" in r.stderr and "DECOMPRESSION" not in r.stderr
    r, _ = _run(tmp_path, ["--scalar", "-s", "256", "-m", "100", "decode"], wire, "m100")
    assert r.returncode != 0 and "ERR_QPACK_DECOMPRESSION_FAILED" in r.stderr


def test_driver_scalar_releases_blocked_streams(tmp_path):
    """Each request record moved before the encoder-stream record that
    precedes it: the decoder blocks it (Required Insert Count > inserts so
    far) and emits it once the inserts arrive; the QIF is the same."""
    data = open(CORPUS, "rb").read()
    recs = qf.read_qif_out(data)
    raw = [data[off - 12:off + n] for _, off, n in recs]
    sids = [sid for sid, _, _ in recs]
    moved = list(raw)
    for k in range(1, len(raw)):
        if sids[k] != 0 and sids[k - 1] == 0:
            moved[k - 1], moved[k] = moved[k], moved[k - 1]
    wire = b"".join(moved)
    want = oq.decode_wire(wire, 256, 100)
    assert want.count(b"\n") == 217
    r, out = _run(tmp_path, ["--scalar", "-s", "256", "-m", "100", "decode"], wire)
    assert r.returncode == 0, r.stderr
    assert out == want
    r, _ = _run(tmp_path, ["--scalar", "-s", "256", "-m", "0", "decode"], wire, "m0")
    assert r.returncode != 0 and "blocked" in r.stderr


def test_driver_scalar_encodes_config1_like_oracle(tmp_path):
    t = qif.synth_config1()
    r, out = _run(tmp_path, ["--scalar", "encode"], t)
    assert r.returncode == 0, r.stderr
    assert out == oq.encode_qif(t)
    assert "compressed" in r.stderr
    r, back = _run(tmp_path, ["--scalar", "decode"], out, "wire")
    assert r.returncode == 0, r.stderr
    assert back == t


def test_driver_scalar_encodes_netbsd_qif(tmp_path):
    t = open(NETBSD_QIF, "rb").read()
    r, out = _run(tmp_path, ["--scalar", "-s", "0", "encode"], t)
    assert r.returncode == 0, r.stderr
    assert out == oq.encode_qif(t)
    r, back = _run(tmp_path, ["--scalar", "decode"], out, "wire")
    assert back == t


@pytest.mark.parametrize("case", ["truncated_header", "truncated_payload", "bad_huffman",
                                  "dtable0_ref", "no_tab", "too_many"])
def test_driver_scalar_failures(tmp_path, case):
    data = open(CORPUS, "rb").read()
    if case == "truncated_header":
        args, inp = ["decode"], data[:5]
    elif case == "truncated_payload":
        args, inp = ["-s", "256", "-m", "100", "decode"], data[:-3]
    elif case == "bad_huffman":
        sec = b"\x00\x00" + b"\x5f\x1d" + b"\x82" + b"\xff\xff"  # H-bit value: EOS bits
        args, inp = ["decode"], (1).to_bytes(8, "big") + len(sec).to_bytes(4, "big") + sec
    elif case == "dtable0_ref":  # the corpus needs the dynamic table
        args, inp = ["decode"], data
    elif case == "no_tab":
        args, inp = ["encode"], b":method GET\n\n"
    else:
        args, inp = ["encode"], b"".join(b"a\tb\n" for _ in range(1025)) + b"\n"
    r, _ = _run(tmp_path, ["--scalar"] + args, inp)
    assert r.returncode != 0


def test_driver_rejects_dynamic_table_encoding(tmp_path):
    r, _ = _run(tmp_path, ["--scalar", "-s", "256", "encode"], b"a\tb\n\n")
    assert r.returncode != 0 and "-s 0" in r.stderr


# The reference CLI's own summary line for this corpus at -s 0 (BASELINE.md,
# "CLI-reported compression": examples/qpack_encode.cc:209-216 printed it in
# the survey's run of the compiled reference): encoded bytes of the
# netbsd QIF's 18 sections, all on the request stream, nothing on the
# encoder stream.
REFERENCE_NETBSD_S0_LINE = "5376 -> 2934 (r:2934 + e:0) 45.42% compressed"


def test_driver_scalar_netbsd_summary_matches_reference_cli(tmp_path):
    r, out = _run(tmp_path, ["--scalar", "-s", "0", "encode"], open(NETBSD_QIF, "rb").read())
    assert r.returncode == 0, r.stderr
    assert r.stderr.strip().splitlines()[-1] == REFERENCE_NETBSD_S0_LINE
    assert len(out) == 2934 + 12 * 18  # request records: 12-byte header each


def _rec(sid, body):
    return sid.to_bytes(8, "big") + len(body).to_bytes(4, "big") + body


# An insert with a literal name "a" whose Huffman value (20 bytes) is cut by
# the end of its encoder-stream record after 6 bytes; a request (Required
# Insert Count 0, :method GET) that needs no insert.
_REQ = b"\x00\x00\xd1"


def _cut_insert(bad):
    value = bytearray(oracle.encode(b"a" * 32))
    assert len(value) == 20
    if bad:
        value[1:5] = b"\xff\xff\xff\xff"  # EOS in the bytes that arrive first
    head = b"\x41a" + bytes([0x80 | len(value)])
    return head + bytes(value[:6]), bytes(value[6:])


def test_driver_scalar_cut_huffman_string_fails_where_it_arrives(tmp_path):
    """The reference decodes a cut Huffman string's bytes as they arrive
    (qpack.c:2737-2763, fin = 0) and fails the encoder-stream record where
    the EOS code first appears (ENCODER_STREAM_ERROR, :2992-2997, :3083-3088),
    so the request after that record is never emitted; a cut at the end of
    the file with bad bytes fails too, a clean one stays pending (exit 0)."""
    p1, p2 = _cut_insert(True)
    wire = _rec(0, p1) + _rec(4, _REQ) + _rec(0, p2)
    r, out = _run(tmp_path, ["--scalar", "-s", "256", "-m", "100", "decode"], wire, "mid")
    assert r.returncode != 0 and "ENCODER_STREAM_ERROR" in r.stderr, r.stderr
    assert out == b""
    r, out = _run(tmp_path, ["--scalar", "-s", "256", "-m", "100", "decode"], _rec(0, p1), "end")
    assert r.returncode != 0 and "ENCODER_STREAM_ERROR" in r.stderr
    # the same cut with clean bytes: the request is emitted, the insert
    # completes in the third record; at the end of the file it stays pending
    q1, q2 = _cut_insert(False)
    r, out = _run(tmp_path, ["--scalar", "-s", "256", "-m", "100", "decode"],
                  _rec(0, q1) + _rec(4, _REQ) + _rec(0, q2), "clean")
    assert r.returncode == 0, r.stderr
    assert out == b":method\tGET\n\n"
    r, out = _run(tmp_path, ["--scalar", "-s", "256", "-m", "100", "decode"], _rec(0, q1), "pend")
    assert r.returncode == 0, r.stderr


def test_driver_scalar_framing_error_keeps_earlier_output(tmp_path):
    """A truncated last record: the records before it are decoded and
    written first, then the framing error ends the run (the reference CLI
    reads record by record, qpack_decode.cc:229-247)."""
    data = open(CORPUS, "rb").read()
    recs = qf.read_qif_out(data)
    _, off, n = recs[-1]
    head = data[:off - 12]
    want = oq.decode_wire(head, 256, 100)
    assert want.count(b"\n\n") >= 10
    for cut, msg in ((data[:-3], "Insufficient input"), (head + data[off - 12:off - 5], "Could not read")):
        r, out = _run(tmp_path, ["--scalar", "-s", "256", "-m", "100", "decode"], cut, "t%d" % len(cut))
        assert r.returncode != 0 and msg in r.stderr, r.stderr
        assert out == want
