"""GPU parity for QPACK field sections:
header blocks are framed on the host by nghttp3_amd/csrc/qh_qpack.c and
every Huffman string of the batch is decoded by the HIP kernels through
qh_decode_batch; the decoded strings must equal the oracle's (bit-exact),
and a corrupted string must fail exactly its own block with -401, as
nghttp3_qpack_decoder_read_request does (qpack.c:3604-3609, :3693-3698)."""
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


def _check_strings(src, res):
    spans, dst, out, huff = res["spans"], res["dst"], res["out"], res["huffman"]
    hs = spans[huff]
    for k in range(hs.size):
        raw = bytes(src[hs["off"][k]:hs["off"][k] + hs["len"][k]])
        st, want = oracle.decode_one(raw)
        assert int(out["status"][k]) == st
        if st == 0:
            got = bytes(dst[out["off"][k]:out["off"][k] + out["len"][k]])
            assert got == want


def test_netbsd_blocks_decode_on_gpu(dec):
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
    _check_strings(src, res)


def test_synthetic_sections_decode_on_gpu_with_corruption(dec):
    src, blocks, plain, strs, lines, ls = qpack.synth_field_sections(0x5EED0004, 4096)
    src = src.copy()
    ref_res = qpack.scan_blocks(src, blocks)
    spans = ref_res[1]
    hidx = np.nonzero(spans["flags"] & qpack.SPAN_HUFFMAN)[0]
    # corrupt the last byte of a few Huffman strings into zero padding
    rng = np.random.default_rng(7)
    victims = rng.choice(hidx, 16, replace=False)
    for v in victims:
        src[spans["off"][v] + spans["len"][v] - 1] = 0x00
    res = dec.decode_blocks(src, blocks)
    _check_strings(src, res)
    bad_blocks = set(np.searchsorted(ref_res[3], victims, side="right") - 1)
    for b in range(blocks.size):
        # a zeroed final byte is always invalid padding unless the string is
        # still accepted (oracle decides); compare against the oracle's view
        s0, s1 = ref_res[3][b], ref_res[3][b + 1]
        want = 0
        for k in range(s0, s1):
            if spans["flags"][k] & qpack.SPAN_HUFFMAN:
                raw = bytes(src[spans["off"][k]:spans["off"][k] + spans["len"][k]])
                if oracle.decode_one(raw)[0] != 0:
                    want = qpack.QH_ERR_QPACK_DECOMPRESSION_FAILED
        assert res["status"][b] == want, b
    assert any(res["status"][b] != 0 for b in bad_blocks)
    # clean blocks: every string equals the plaintext the writer was given
    ok = res["status"] == 0
    pb = bytes(plain)
    for b in np.nonzero(ok)[0][:512]:
        ks = [int(k) for l in lines[ls[b]:ls[b + 1]] for k in (l["name"], l["value"]) if k >= 0]
        for j, k in enumerate(range(ref_res[3][b], ref_res[3][b + 1])):
            want = pb[strs["off"][ks[j]]:strs["off"][ks[j]] + strs["len"][ks[j]]]
            if spans["flags"][k] & qpack.SPAN_HUFFMAN:
                pos = int(np.searchsorted(hidx, k))
                got = bytes(res["dst"][res["out"]["off"][pos]:res["out"]["off"][pos] + res["out"]["len"][pos]])
            else:
                got = bytes(src[spans["off"][k]:spans["off"][k] + spans["len"][k]])
            assert got == want


def _check_cases():
    from test_http_check import cases
    return cases(0x5EED0F6, 4000)


def test_check_fields_batch_host_and_device_match_scalar(dec):
    import torch
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


def test_decode_blocks_validates_every_string(dec):
    src, blocks, plain, strs, lines, ls = qpack.synth_field_sections(0x5EED0007, 512)
    src = src.copy()
    res = dec.decode_blocks(src, blocks)
    assert (res["status"] == 0).all()
    # synthetic names / values are alphabet A: upper-case letters make names
    # invalid (nghttp3 rejects upper case), values are all valid
    pb = bytes(plain)
    names = (res["spans"]["flags"] & qpack.SPAN_NAME) != 0
    ks = [int(k) for l in lines for k in (l["name"], l["value"]) if k >= 0]
    for j, k in enumerate(ks):
        s = pb[strs["off"][k]:strs["off"][k] + strs["len"][k]]
        want = qpack.check_header_name(s) if names[j] else qpack.check_header_value(s)
        assert res["verdict"][j] == want


def test_lookup_tokens_batch_host_and_device_match_scalar(dec):
    import torch
    from conftest import load_json
    from test_http_check import token_cases
    names = token_cases(load_json("tokens.json")["tokens"], 0x5EED0F8)
    src = np.frombuffer(b"\x00" * 5 + b"".join(names), dtype=np.uint8)
    spans = np.zeros(len(names), dtype=SPAN_IN_DTYPE)
    spans["len"] = [len(x) for x in names]
    spans["off"] = 5 + np.concatenate([[0], np.cumsum(spans["len"].astype(np.uint64))[:-1]])
    want = np.array([qpack.lookup_token(x) for x in names], dtype=np.int32)
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


def test_device_pipeline_matches_staged_path(dec):
    import torch
    src, blocks, plain, strs, lines, ls = qpack.synth_field_sections(0x5EED000A, 3000)
    res = dec.decode_blocks(src, blocks)
    d = dec.decode_blocks_dev(torch.from_numpy(np.ascontiguousarray(src)).cuda(),
                              torch.from_numpy(blocks.view(np.int64).reshape(-1, 2).copy()).cuda())
    torch.cuda.synchronize()
    assert (d["status"][:blocks.size].cpu().numpy() == res["status"]).all()
    assert d["nspans"] == res["spans"].size
    nh = d["nhuff"]
    assert nh == res["huffman"].sum()
    out = d["out"][:nh].cpu().numpy()
    dst = d["dst"].cpu().numpy()
    ho = res["out"]
    for k in range(ho.size):
        a = bytes(res["dst"][ho["off"][k]:ho["off"][k] + ho["len"][k]])
        b = bytes(dst[out[k, 0]:out[k, 0] + (out[k, 1] & 0xFFFFFFFF)])
        assert a == b
    assert (d["verdict"][:nh].cpu().numpy() == res["verdict"][res["huffman"]]).all()
    sel = d["name_sel"].cpu().numpy()
    names = [bytes(dst[o:o + (l & 0xFFFFFFFF)]) for o, l in out[sel]]
    assert (d["tokens"][:nh].cpu().numpy()[sel] == [qpack.lookup_token(x) for x in names]).all()
