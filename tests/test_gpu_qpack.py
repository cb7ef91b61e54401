"""GPU parity for QPACK field sections:
qh_decode_sections_batch (GPU framing -> batch Huffman decode -> per-block
fold, validation, tokens) against the oracle directly: per block the status
of oracle/qpack_frame.decode_field_section (read_request restated, with a
corrupted string failing exactly its own block with -401 as
qpack.c:3604-3609, :3693-3698 do), per string the oracle's decoded bytes,
oracle/http_check's verdict and the reference's token."""
import os

import numpy as np
import pytest

import oracle
from oracle import qpack_frame as ref
from nghttp3_amd import qpack
from nghttp3_amd.qpack_huffman import SPAN_IN_DTYPE

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dec():
    return qpack.FieldSectionDecoder(0)


@pytest.fixture(scope="module")
def dec0(dec):
    """Decoder at dynamic table capacity 0 (config 4), same context."""
    return qpack.FieldSectionDecoder(codec=dec.codec, dtable0=True)


@pytest.fixture(scope="module")
def refdata():
    from conftest import load_json
    d = load_json("http_chars.json")
    return d["VALID_HD_NAME_CHARS"], d["VALID_HD_VALUE_CHARS"], load_json("tokens.json")["tokens"]


def _blocks_of(lens):
    blocks = np.zeros(len(lens), dtype=SPAN_IN_DTYPE)
    blocks["len"] = lens
    if len(lens):
        blocks["off"][1:] = np.cumsum(blocks["len"].astype(np.uint64))[:-1]
    return blocks


def _check_against_oracle(src, blocks, res, refdata, dtable0, strs_dst=None, src_bytes=None):
    """Per block and per string, the C pipeline's result equals the oracle's
    restatement of read_request (oracle/qpack_frame.decode_field_section:
    framing + Huffman in stream order), oracle/http_check and the
    reference's token table."""
    from oracle import http_check
    names, values, tokens = refdata
    data = bytes(src) if src_bytes is None else src_bytes
    dst = res["dst"] if strs_dst is None else strs_dst
    ss, st = res["span_start"], res["status"]
    nbad = 0
    for b in range(blocks.size):
        off, n = int(blocks["off"][b]), int(blocks["len"][b])
        rst, rlines, rspans, rstrings = ref.decode_field_section(data[off:off + n], off, dtable0)
        assert int(st[b]) == rst, (b, int(st[b]), rst)
        nbad += rst != 0
        k0, k1 = int(ss[b]), int(ss[b + 1])
        assert k1 - k0 == len(rspans), b
        # lines: the oracle's for a clean block; none when the framing failed;
        # all of them when only a Huffman string failed (-401 after a clean
        # framing keeps its lines: include/qhuff.h qh_decode_sections_batch)
        fst, _, flines, _ = ref.scan_field_section(data[off:off + n], off, dtable0)
        l0, l1 = int(res["line_start"][b]), int(res["line_start"][b + 1])
        got_lines = [(int(x["opcode"]), int(x["flags"]), int(x["index"]),
                      int(x["name"]) - k0 if int(x["name"]) >= 0 else -1,
                      int(x["value"]) - k0 if int(x["value"]) >= 0 else -1)
                     for x in res["lines"][l0:l1]]
        assert got_lines == (flines if fst == 0 else []), b
        if rst == 0:
            assert got_lines == rlines, b
        got_spans = [(int(x["off"]), int(x["len"]), int(x["flags"])) for x in res["spans"][k0:k1]]
        assert got_spans == rspans, b
        for j, k in enumerate(range(k0, k1)):
            o = res["strs"][k]
            want = rstrings[j]
            is_name = bool(rspans[j][2] & ref.SPAN_NAME)
            if want is None:
                assert int(o["status"]) == -108 and res["verdict"][k] == 0 and res["tokens"][k] == -1
                continue
            assert int(o["status"]) == 0, (b, j, len(want), rspans[j], "binary" if max(want or b"\0") > 126 else "text")
            buf = dst if rspans[j][2] & ref.SPAN_HUFFMAN else src
            got = bytes(buf[int(o["off"]):int(o["off"]) + int(o["len"])])
            assert got == want, (b, j)
            vw = http_check.check_header_name(want, names) if is_name else \
                http_check.check_header_value(want, values)
            assert res["verdict"][k] == vw, (b, j, want)
            tw = http_check.lookup_token(want, tokens) if is_name else -1
            assert res["tokens"][k] == tw, (b, j, want)
    return nbad


def test_netbsd_blocks_decode_on_gpu(dec, refdata):
    data = open(os.path.join(GOLDEN, "netbsd-hq.out.256.100.1"), "rb").read()
    recs = [r for r in ref.read_qif_out(data) if r[0] != 0]
    blocks = np.zeros(len(recs), dtype=SPAN_IN_DTYPE)
    blocks["off"] = [r[1] for r in recs]
    blocks["len"] = [r[2] for r in recs]
    src = np.frombuffer(data, dtype=np.uint8)
    res = dec.decode_blocks(src, blocks)
    assert (res["status"] == 0).all()
    assert res["lines"].size == 199
    assert res["huffman"].sum() > 0
    assert _check_against_oracle(src, blocks, res, refdata, False) == 0


def _corrupted_corpus(seed, nblocks):
    """Synthetic config-4 blocks with every kind of bad input the reference
    rejects, block by block: zero padding / EOS / over-long padding in
    Huffman strings, a Huffman failure before a HEADER_TOO_LARGE, static
    index >= 99, dynamic references and a negative Delta Base at Required
    Insert Count 0, a non-zero Required Insert Count (capacity 0),
    truncation, integer overflow."""
    src, blocks, *_ = qpack.synth_field_sections(seed, nblocks)
    secs = [bytes(src[int(o):int(o) + int(n)]) for o, n in zip(blocks["off"], blocks["len"])]
    rng = np.random.default_rng(seed)
    kinds = []
    for b in rng.choice(nblocks, nblocks // 8, replace=False):
        sec = bytearray(secs[b])
        _, _, _, spans = ref.scan_field_section(bytes(sec))
        hs = [sp for sp in spans if sp[2] & ref.SPAN_HUFFMAN]
        kind = int(rng.integers(0, 10))
        if kind == 0 and hs:       # last byte -> zero padding
            o, n, _ = hs[int(rng.integers(len(hs)))]
            sec[o + n - 1] = 0x00
        elif kind == 1 and hs:     # EOS inside
            o, n, _ = hs[int(rng.integers(len(hs)))]
            if n >= 4:
                sec[o:o + 4] = b"\xff\xff\xff\xff"
        elif kind == 2 and hs:     # padding of 8+ ones
            o, n, _ = hs[int(rng.integers(len(hs)))]
            sec[o + n - 1] = 0xFF
            if n >= 2:
                sec[o + n - 2] = 0xFF
        elif kind == 3:            # bad Huffman string, then a too-large value
            sec += b"\x50\x81\x00\x50" + ref.put_varint(65537, 7) + b"a" * 65537
        elif kind == 4:            # static index past the table
            sec += ref.write_indexed(0xC0, int(rng.integers(99, 5000)), 6)
        elif kind == 5:            # dynamic reference at ricnt 0
            sec += ref.write_indexed(0x80, 0, 6)
        elif kind == 6:            # negative Delta Base at ricnt 0
            sec[1] |= 0x80
        elif kind == 7:            # Required Insert Count 1 (capacity 0 rejects)
            sec[0] = 0x01
        elif kind == 8:            # truncated
            sec = sec[:max(0, len(sec) - int(rng.integers(1, 4)))]
        else:                      # integer overflow in a length
            sec += b"\x2f" + b"\xff" * 12
        secs[b] = bytes(sec)
        kinds.append(kind)
    data = b"".join(secs)
    return np.frombuffer(data, dtype=np.uint8).copy(), _blocks_of([len(x) for x in secs]), kinds


@pytest.mark.parametrize("dtable0", [False, True])
def test_sections_pipeline_matches_oracle_on_corrupted_blocks(dec, dec0, refdata, dtable0):
    """qh_decode_sections_batch, host and device forms, against the oracle
    per block (status) and per string (bytes, verdict, token)."""
    import torch
    d = dec0 if dtable0 else dec
    src, blocks, kinds = _corrupted_corpus(0x5EED0004 + dtable0, 3000)
    res = d.decode_blocks(src, blocks)
    nbad = _check_against_oracle(src, blocks, res, refdata, dtable0)
    assert nbad >= len(kinds) // 2
    # the device-resident form gives the same tensors
    g = d.decode_blocks_dev(torch.from_numpy(src).cuda(),
                            torch.from_numpy(blocks.view(np.int64).reshape(-1, 2).copy()).cuda())
    torch.cuda.synchronize()
    ns = int(g["nspans"])
    assert ns == res["spans"].size and int(g["nlines"]) == res["lines"].size
    gres = {"spans": g["spans"][:ns].cpu().numpy().view(SPAN_IN_DTYPE).reshape(-1),
            "strs": g["strs"][:ns].cpu().numpy().view(qpack.SPAN_OUT_DTYPE).reshape(-1),
            "verdict": g["verdict"][:ns].cpu().numpy(), "tokens": g["tokens"][:ns].cpu().numpy(),
            "span_start": g["span_start"][:blocks.size + 1].cpu().numpy().view(np.uint32),
            "line_start": g["line_start"][:blocks.size + 1].cpu().numpy().view(np.uint32),
            "lines": g["lines"][:int(g["nlines"]) * 24].cpu().numpy().view(qpack.FIELD_LINE_DTYPE),
            "status": g["status"][:blocks.size].cpu().numpy(), "dst": g["dst"].cpu().numpy()}
    assert (gres["status"] == res["status"]).all()
    _check_against_oracle(src, blocks, gres, refdata, dtable0)
    lines = g["lines"][:int(g["nlines"]) * 24].cpu().numpy().view(qpack.FIELD_LINE_DTYPE)
    assert lines.tobytes() == res["lines"].tobytes()


@pytest.mark.parametrize("nblocks", [1, 2, 2047, 2048, 2049, 4097])
def test_sections_pipeline_at_scan_tile_edges(dec0, refdata, nblocks):
    """Framing's four per-block counts go through one segmented scan launch
    (qh_k_scan_seg, 2048 entries per tile, one segment per count) whose
    totals come back in one copy: block counts around the tile size give
    the oracle's results, host and device forms alike."""
    import torch
    src, blocks, kinds = _corrupted_corpus(0x5EED00E0 + nblocks, nblocks)
    res = dec0.decode_blocks(src, blocks)
    _check_against_oracle(src, blocks, res, refdata, True)
    g = dec0.decode_blocks_dev(torch.from_numpy(src).cuda(),
                               torch.from_numpy(blocks.view(np.int64).reshape(-1, 2).copy()).cuda())
    torch.cuda.synchronize()
    assert int(g["nspans"]) == res["spans"].size and int(g["nlines"]) == res["lines"].size
    assert (g["status"][:nblocks].cpu().numpy() == res["status"]).all()
    assert (g["span_start"][:nblocks + 1].cpu().numpy().view(np.uint32) == res["span_start"]).all()
    lines = g["lines"][:int(g["nlines"]) * 24].cpu().numpy().view(qpack.FIELD_LINE_DTYPE)
    assert lines.tobytes() == res["lines"].tobytes()


def test_sections_device_growing_batches(refdata):
    """The device form queues its write pass before it reads framing's
    totals, into scratch laid out for the most spans seen so far: a fresh
    context fed batches that grow (the write runs again after the sync) and
    shrink gives the oracle's results every time."""
    import torch
    d = qpack.FieldSectionDecoder(0, dtable0=True)
    for nblocks in (3, 2049, 10, 4097, 700):
        src, blocks, _ = _corrupted_corpus(0x5EED00F0 + nblocks, nblocks)
        g = d.decode_blocks_dev(torch.from_numpy(src).cuda(),
                                torch.from_numpy(blocks.view(np.int64).reshape(-1, 2).copy()).cuda())
        torch.cuda.synchronize()
        ns = int(g["nspans"])
        gres = {"spans": g["spans"][:ns].cpu().numpy().view(SPAN_IN_DTYPE).reshape(-1),
                "strs": g["strs"][:ns].cpu().numpy().view(qpack.SPAN_OUT_DTYPE).reshape(-1),
                "verdict": g["verdict"][:ns].cpu().numpy(), "tokens": g["tokens"][:ns].cpu().numpy(),
                "span_start": g["span_start"][:nblocks + 1].cpu().numpy().view(np.uint32),
                "line_start": g["line_start"][:nblocks + 1].cpu().numpy().view(np.uint32),
                "lines": g["lines"][:int(g["nlines"]) * 24].cpu().numpy().view(qpack.FIELD_LINE_DTYPE),
                "status": g["status"][:nblocks].cpu().numpy(), "dst": g["dst"].cpu().numpy()}
        _check_against_oracle(src, blocks, gres, refdata, True)


def test_sections_pipeline_clean_blocks_give_the_writer_plaintext(dec0):
    src, blocks, plain, strs, lines, ls = qpack.synth_field_sections(0x5EED000A, 3000)
    res = dec0.decode_blocks(src, blocks)
    assert (res["status"] == 0).all()
    assert res["lines"].size == lines.size
    pb = bytes(plain)
    ks = [int(k) for l in lines for k in (l["name"], l["value"]) if k >= 0]
    assert len(ks) == res["spans"].size
    for j, k in enumerate(ks):
        o = res["strs"][j]
        buf = res["dst"] if res["huffman"][j] else src
        assert bytes(buf[int(o["off"]):int(o["off"]) + int(o["len"])]) == \
            pb[int(strs["off"][k]):int(strs["off"][k]) + int(strs["len"][k])]


def _check_cases():
    from test_http_check import cases
    return cases(0x5EED0F6, 4000)


def test_config4_full_corpus_matches_oracle_digests(dec0):
    """Config 4 at size: all 65,536 blocks through qh_decode_sections_batch
    on the device (capacity 0), against the oracle's digests of every
    decoded string, verdict and token (tests/golden/gen_golden.py)."""
    import hashlib
    import torch
    from conftest import load_json
    d = load_json("digests.json")["configs"]["c4_blocks"]
    src, blocks, *_ = qpack.synth_field_sections(d["seed"], d["nblocks"])
    assert hashlib.sha256(src.tobytes()).hexdigest() == d["blocks_sha256"]
    d_src = torch.from_numpy(np.ascontiguousarray(src)).cuda()
    g = dec0.decode_blocks_dev(d_src, torch.from_numpy(blocks.view(np.int64).reshape(-1, 2).copy()).cuda())
    torch.cuda.synchronize()
    ns = int(g["nspans"])
    assert ns == d["strings"] and int(g["nlines"]) == d["field_lines"]
    assert bool((g["status"][:blocks.size] == 0).all())
    strs = g["strs"][:ns]
    assert bool(((strs[:, 1] >> 32) == 0).all())
    ln = strs[:, 1] & 0xFFFFFFFF
    tot = int(ln.sum().item())
    assert tot == d["string_bytes"]
    huff = ((g["spans"][:ns, 1] >> 32) & qpack.SPAN_HUFFMAN) != 0
    pos = torch.arange(tot, device="cuda", dtype=torch.int64) - \
        torch.repeat_interleave(torch.cumsum(ln, 0) - ln, ln)
    at = torch.repeat_interleave(strs[:, 0], ln) + pos
    hb = torch.repeat_interleave(huff, ln)
    got = torch.where(hb, g["dst"][at.clamp(max=g["dst"].numel() - 1)], d_src[at.clamp(max=d_src.numel() - 1)])
    assert hashlib.sha256(got.cpu().numpy().tobytes()).hexdigest() == d["strings_sha256"]
    assert hashlib.sha256(g["verdict"][:ns].cpu().numpy().tobytes()).hexdigest() == d["verdict_sha256"]
    assert hashlib.sha256(g["tokens"][:ns].cpu().numpy().tobytes()).hexdigest() == d["token_sha256"]


def test_check_fields_batch_host_and_device_match_scalar(dec, refdata):
    import torch
    from oracle import http_check
    names, values, _ = refdata
    strs = _check_cases()
    flags = [qpack.SPAN_NAME if i % 2 else 0 for i in range(len(strs))]
    # unaligned, back-to-back packing
    src = np.frombuffer(b"\x01" * 3 + b"".join(strs), dtype=np.uint8)
    spans = np.zeros(len(strs), dtype=SPAN_IN_DTYPE)
    spans["len"] = [len(x) for x in strs]
    spans["off"] = 3 + np.concatenate([[0], np.cumsum(spans["len"].astype(np.uint64))[:-1]])
    spans["flags"] = flags
    want = np.array([qpack.check_header_name(x) if f else qpack.check_header_value(x)
                     for x, f in zip(strs, flags)], dtype=np.int8)
    # the reference's rules (oracle/http_check over the reference's tables)
    ref_v = np.array([http_check.check_header_name(x, names) if f else
                      http_check.check_header_value(x, values) for x, f in zip(strs, flags)], dtype=np.int8)
    assert (want == ref_v).all()
    got = qpack.check_fields_host(dec.codec, src, spans)
    assert (got == want).all()
    # device-resident, padded buffer
    d_src = torch.zeros(src.size + 64, dtype=torch.uint8, device="cuda")
    d_src[:src.size] = torch.from_numpy(src.copy()).cuda()
    d_sp = torch.from_numpy(spans.view(np.int64).reshape(-1, 2).copy()).cuda()
    d_v = torch.full((len(strs),), -7, dtype=torch.int8, device="cuda")
    qpack.check_fields_dev(dec.codec, d_src, d_sp, d_v)
    torch.cuda.synchronize()
    assert (d_v.cpu().numpy() == want).all()


def test_lookup_tokens_batch_host_and_device_match_scalar(dec):
    import torch
    from conftest import load_json
    from oracle import http_check
    from test_http_check import token_cases
    tokens = load_json("tokens.json")["tokens"]
    names = token_cases(tokens, 0x5EED0F8)
    src = np.frombuffer(b"\x00" * 5 + b"".join(names), dtype=np.uint8)
    spans = np.zeros(len(names), dtype=SPAN_IN_DTYPE)
    spans["len"] = [len(x) for x in names]
    spans["off"] = 5 + np.concatenate([[0], np.cumsum(spans["len"].astype(np.uint64))[:-1]])
    want = np.array([qpack.lookup_token(x) for x in names], dtype=np.int32)
    assert (want == np.array([http_check.lookup_token(x, tokens) for x in names])).all()
    assert (want >= 0).sum() >= 61  # every token name, plus random hits
    assert (qpack.lookup_tokens_host(dec.codec, src, spans) == want).all()
    d_src = torch.from_numpy(src.copy()).cuda()
    d_sp = torch.from_numpy(spans.view(np.int64).reshape(-1, 2).copy()).cuda()
    d_t = torch.full((len(names),), -7, dtype=torch.int32, device="cuda")
    qpack.lookup_tokens_dev(dec.codec, d_src, d_sp, d_t)
    torch.cuda.synchronize()
    assert (d_t.cpu().numpy() == want).all()


def _gpu_scan(dec, src, blocks):
    import torch
    n = blocks.size
    cap = int(blocks["len"].sum(dtype=np.uint64)) + 1
    d_src = torch.from_numpy(np.ascontiguousarray(src)).cuda()
    d_blk = torch.from_numpy(blocks.view(np.int64).reshape(-1, 2).copy()).cuda()
    d_lines = torch.zeros(cap * qpack.FIELD_LINE_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    d_spans = torch.zeros((cap, 2), dtype=torch.int64, device="cuda")
    d_ls = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
    d_ss = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
    d_st = torch.full((max(n, 1),), 7, dtype=torch.int32, device="cuda")
    d_h = torch.zeros((cap, 2), dtype=torch.int64, device="cuda")
    tot = qpack.scan_blocks_dev(dec.codec, d_src, d_blk, d_lines, d_spans, d_ls, d_ss, d_st, d_h)
    torch.cuda.synchronize()
    sp = d_spans.cpu().numpy().view(SPAN_IN_DTYPE).reshape(-1)[:tot[1]]
    hsp = d_h.cpu().numpy().view(SPAN_IN_DTYPE).reshape(-1)[:tot[2]]
    assert hsp.tobytes() == sp[(sp["flags"] & qpack.SPAN_HUFFMAN) != 0].tobytes()
    ls = d_ls.cpu().numpy().view(np.uint32)
    ss = d_ss.cpu().numpy().view(np.uint32)
    lines = d_lines.cpu().numpy().view(qpack.FIELD_LINE_DTYPE)[:ls[n]]
    spans = d_spans.cpu().numpy().view(SPAN_IN_DTYPE).reshape(-1)[:ss[n]]
    return lines, spans, ls, ss, d_st.cpu().numpy()[:n]


def _same_scan(a, b):
    for x, y in zip(a, b):
        assert x.shape == y.shape
        assert x.tobytes() == y.tobytes()


def test_gpu_framing_matches_host_scan_on_netbsd_and_synthetic(dec):
    data = open(os.path.join(GOLDEN, "netbsd-hq.out.256.100.1"), "rb").read()
    recs = [r for r in ref.read_qif_out(data) if r[0] != 0]
    blocks = np.zeros(len(recs), dtype=SPAN_IN_DTYPE)
    blocks["off"] = [r[1] for r in recs]
    blocks["len"] = [r[2] for r in recs]
    src = np.frombuffer(data, dtype=np.uint8)
    _same_scan(_gpu_scan(dec, src, blocks), qpack.scan_blocks(src, blocks))
    # synthetic batch with failing blocks (truncations, overflow, too large)
    src, blocks, *_ = qpack.synth_field_sections(0x5EED0009, 5000)
    src = src.copy()
    blocks = blocks.copy()
    blocks["len"][10] -= 1   # fails unless the block ends in a 1-byte indexed line
    blocks["len"][11] = 1
    src[blocks["off"][12] + 2] = 0x2F
    src[blocks["off"][12] + 3:blocks["off"][12] + 16] = 0xFF
    _same_scan(_gpu_scan(dec, src, blocks), qpack.scan_blocks(src, blocks))
    st = _gpu_scan(dec, src, blocks)[4]
    assert (st[[11, 12]] == qpack.QH_ERR_QPACK_DECOMPRESSION_FAILED).all() and (st[:10] == 0).all()
    # blocks larger than the count pass's per-block slice (32 lines / 64
    # strings) are parsed again in the write pass: mixed with small ones
    src, blocks, *_ = qpack.synth_field_sections(0x5EED000A, 600, fields=(1, 120))
    src = src.copy()
    blocks = blocks.copy()
    blocks["len"][7] -= 1  # a big block that fails
    got = _gpu_scan(dec, src, blocks)
    _same_scan(got, qpack.scan_blocks(src, blocks))
    nl = np.diff(got[2].astype(np.int64))
    assert (nl > 32).sum() > 100 and (nl <= 32).sum() > 100


def _max_huffman_text(limit_enc, seed):
    """Alphabet-A text whose Huffman encoding is exactly limit_enc bytes
    (or the longest one under it)."""
    from nghttp3_amd import synth
    text = synth.fill(seed, limit_enc * 2, synth.ALPHABET_A).tobytes()
    lo, hi = 0, len(text)
    while lo < hi:  # longest prefix whose encoding fits
        mid = (lo + hi + 1) // 2
        if oracle.encode_count(text[:mid]) <= limit_enc:
            lo = mid
        else:
            hi = mid - 1
    return text[:lo]


def _long_value_sections(seed, nblocks, corrupt=True):
    """Field sections whose values nghttp3 decodes through the same
    qpack_read_huffman_string as short ones (qpack.c:2737-2763) up to
    NGHTTP3_QPACK_MAX_VALUELEN (qpack.h:50; a Huffman value counts as
    len * 8 / 5, so 40,960 encoded bytes is the largest, read_string
    qpack.c:3661-3674): Zipf-like lengths of 129 B to 64 KiB, alphabet-A
    text, binary (all 256 byte values, always Huffman-coded as a foreign
    encoder may do), and text with 5% binary bytes; values at the limit and
    one byte past it (-109); literal names; and, when `corrupt`, long strings
    with EOS inside, zero padding, padding of 8 ones, or the last byte cut."""
    from nghttp3_amd import synth
    rng = np.random.default_rng(seed)
    at_limit = _max_huffman_text(40960, seed)
    secs, kinds = [], []
    for b in range(nblocks):
        sec = bytearray(b"\x00\x00")
        for f in range(int(rng.integers(1, 4))):
            kind = int(rng.integers(0, 3))
            if b % 17 == 3 and f == 0:
                v = at_limit
            else:
                n = int(np.exp(rng.uniform(np.log(129), np.log(65536))))
                # (under the limit: ~0.82 encoded bytes per text byte, ~0.93
                # with 5% binary bytes, ~2.9 per binary byte)
                n = min(n, (48000, 14000, 40000)[kind])
                v = synth.fill(int(rng.integers(1 << 62)), n, synth.ALPHABET_A).tobytes()
                if kind == 1:
                    v = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
                elif kind == 2:
                    a = np.frombuffer(v, np.uint8).copy()
                    k = rng.choice(n, max(1, n // 20), replace=False)
                    a[k] = rng.integers(0, 256, k.size)
                    v = a.tobytes()
            enc = bytearray(oracle.encode(v))
            ck = -1
            if corrupt and rng.random() < 0.15 and len(enc) > 8:
                ck = int(rng.integers(0, 4))
                if ck == 0:    # EOS in the middle
                    m = len(enc) // 2
                    enc[m:m + 4] = b"\xff\xff\xff\xff"
                elif ck == 1:  # zero padding
                    enc[-1] = 0x00
                elif ck == 2:  # padding of 8 more ones
                    enc += b"\xff"
                else:          # the last code cut
                    del enc[-1]
            kinds.append(ck)
            if rng.random() < 0.25:  # literal name (Huffman), then the value
                name = synth.fill(int(rng.integers(1 << 62)), int(rng.integers(1, 25)),
                                  synth.ALPHABET_A).tobytes().lower()
                ne = oracle.encode(name)
                sec += ref.put_varint(len(ne), 3, 0x28) + ne
            else:            # static name reference
                sec += ref.put_varint(int(rng.integers(0, 99)), 4, 0x50)
            sec += ref.put_varint(len(enc), 7, 0x80) + bytes(enc)
        if b % 29 == 5:  # a value one encoded byte past the limit: -109
            over = oracle.encode(at_limit + b"a" * 8)
            sec += ref.put_varint(0, 4, 0x50) + ref.put_varint(len(over), 7, 0x80) + over
        secs.append(bytes(sec))
    data = b"".join(secs)
    return np.frombuffer(data, dtype=np.uint8).copy(), _blocks_of([len(x) for x in secs]), kinds


def _dev_result(g, nblocks):
    ns = int(g["nspans"])
    return {"spans": g["spans"][:ns].cpu().numpy().view(SPAN_IN_DTYPE).reshape(-1),
            "strs": g["strs"][:ns].cpu().numpy().view(qpack.SPAN_OUT_DTYPE).reshape(-1),
            "verdict": g["verdict"][:ns].cpu().numpy(), "tokens": g["tokens"][:ns].cpu().numpy(),
            "span_start": g["span_start"][:nblocks + 1].cpu().numpy().view(np.uint32),
            "line_start": g["line_start"][:nblocks + 1].cpu().numpy().view(np.uint32),
            "lines": g["lines"][:int(g["nlines"]) * 24].cpu().numpy().view(qpack.FIELD_LINE_DTYPE),
            "status": g["status"][:nblocks].cpu().numpy(), "dst": g["dst"].cpu().numpy()}


@pytest.mark.parametrize("dtable0", [False, True])
def test_sections_long_and_binary_values_match_oracle(dec, dec0, refdata, dtable0):
    """qh_decode_sections_batch on the strings nghttp3 accepts beyond short
    header text: values of 129 B to the 64 KiB limit (the fused-check
    decoder hands every string of >= 4 KiB to qh_k_dec_long_list, a
    workgroup per string), binary and mixed text (long codes on the lanes'
    careful path), corrupted long strings; host and device forms against
    oracle/qpack_frame.decode_field_section per block and per string."""
    import torch
    d = dec0 if dtable0 else dec
    src, blocks, kinds = _long_value_sections(0x5EED0410 + dtable0, 240)
    res = d.decode_blocks(src, blocks)
    lens = res["spans"]["len"]
    assert (lens >= 4096).sum() >= 100 and (lens >= 30000).sum() >= 10
    assert sum(k >= 0 for k in kinds) >= 40
    nbad = _check_against_oracle(src, blocks, res, refdata, dtable0)
    assert nbad >= 40
    assert (res["status"] == qpack.QH_ERR_QPACK_HEADER_TOO_LARGE).sum() >= 5
    g = d.decode_blocks_dev(torch.from_numpy(src).cuda(),
                            torch.from_numpy(blocks.view(np.int64).reshape(-1, 2).copy()).cuda())
    torch.cuda.synchronize()
    gres = _dev_result(g, blocks.size)
    assert (gres["status"] == res["status"]).all()
    _check_against_oracle(src, blocks, gres, refdata, dtable0)


def test_sections_one_value_at_the_limit(dec0, refdata):
    """One field section holding one value of 40,960 encoded bytes (the
    largest nghttp3 accepts), clean and with EOS in its last segment."""
    v = _max_huffman_text(40960, 0x5EED0411)
    enc = bytearray(oracle.encode(v))
    assert len(enc) == 40960
    for bad in (False, True):
        e = bytearray(enc)
        if bad:
            e[-40:-36] = b"\xff\xff\xff\xff"
        sec = b"\x00\x00" + ref.put_varint(5, 4, 0x50) + ref.put_varint(len(e), 7, 0x80) + bytes(e)
        src = np.frombuffer(sec, np.uint8).copy()
        blocks = _blocks_of([len(sec)])
        res = dec0.decode_blocks(src, blocks)
        assert _check_against_oracle(src, blocks, res, refdata, True) == int(bad)
        if not bad:
            o = res["strs"][0]
            assert bytes(res["dst"][int(o["off"]):int(o["off"]) + int(o["len"])]) == v


@pytest.mark.parametrize("decoder", ["sorted", "waves"])
def test_sections_long_values_other_decoders(refdata, decoder):
    """The same long-value sections through the sorted decoder (its long
    records, a workgroup each) and the waves decoder."""
    d = qpack.FieldSectionDecoder(0, dtable0=True)
    try:
        d.codec.set_decoder(decoder)
        src, blocks, _ = _long_value_sections(0x5EED0412, 60)
        res = d.decode_blocks(src, blocks)
        _check_against_oracle(src, blocks, res, refdata, True)
    finally:
        d.codec.close()
