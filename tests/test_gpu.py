"""GPU parity: the HIP batch path (qh_decode_batch / qh_encode_count_batch /
qh_encode_batch through the C ABI) against the oracle and the committed
fixtures.  Integer/byte work, so every comparison is bit-exact."""
import hashlib

import os

import numpy as np
import pytest

import oracle
from conftest import strings_of
from nghttp3_amd import qpack_huffman as q
from nghttp3_amd import synth

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def torch_mod():
    import torch
    return torch


def to_dev(a, dtype=None):
    torch = torch_mod()
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.view(dtype)
    return t.cuda()


def spans_dev(off, ln):
    sp = np.zeros((len(ln), 2), dtype=np.int64)
    sp[:, 0] = np.asarray(off, dtype=np.int64)
    sp[:, 1] = np.asarray(ln, dtype=np.int64)
    return to_dev(sp)


def assert_disjoint(o, l, cap):
    """Output spans lie inside [0, cap) and do not overlap (any order)."""
    o = np.asarray(o, dtype=np.int64)
    l = np.asarray(l, dtype=np.int64)
    assert (o >= 0).all() and (o + l <= cap).all()
    idx = np.argsort(o, kind="stable")
    so, sl = o[idx], l[idx]
    assert (so[1:] >= so[:-1] + sl[:-1]).all()


def decode_dev(codec, enc, off, ln, cap=None):
    torch = torch_mod()
    n = len(ln)
    slots = int(q.decode_slot_size(np.asarray(ln, dtype=np.int64)).sum())
    cap = slots if cap is None else cap
    src = to_dev(enc if len(enc) else np.zeros(1, np.uint8))
    dst = torch.zeros(max(cap, 1), dtype=torch.uint8, device="cuda")
    out = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    codec.decode_dev(src, spans_dev(off, ln), dst[:cap] if cap else dst[:0], out)
    o, l, s = q.unpack_out(out)
    return dst.cpu().numpy(), o, l, s


def encode_dev(codec, plain, off, ln):
    torch = torch_mod()
    n = len(ln)
    bound = int(((np.asarray(ln, dtype=np.int64) * 30 + 7) // 8).sum())
    src = to_dev(plain if len(plain) else np.zeros(1, np.uint8))
    dst = torch.zeros(max(bound, 1), dtype=torch.uint8, device="cuda")
    out = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    codec.encode_dev(src, spans_dev(off, ln), dst, out)
    o, l, s = q.unpack_out(out)
    return dst.cpu().numpy(), o, l, s


def test_kat(codec, kat):
    strs = [bytes.fromhex(v["huffman_hex"]) for v in kat]
    src, sp = q.pack_strings(strs)
    dst, o, l, s = decode_dev(codec, src, sp["off"], sp["len"])
    for i, v in enumerate(kat):
        assert s[i] == 0
        assert dst[o[i]:o[i] + l[i]].tobytes() == v["plain"].encode()
    plains = [v["plain"].encode() for v in kat]
    src, sp = q.pack_strings(plains)
    enc, o, l, s = encode_dev(codec, src, sp["off"], sp["len"])
    for i, v in enumerate(kat):
        assert enc[o[i]:o[i] + l[i]].tobytes().hex() == v["huffman_hex"]


def test_corpus_decode(codec, corpus):
    enc, eoff, elen = corpus["enc"], corpus["enc_off"], corpus["enc_len"]
    want_dst, want_slot, want_len, want_st = oracle.decode_batch(enc, eoff, elen)
    dst, o, l, s = decode_dev(codec, enc, eoff, elen)
    assert (s == 0).all()
    assert (l == want_len.astype(np.int64)).all()
    assert_disjoint(o, l, int(q.decode_slot_size(elen.astype(np.int64)).sum()))
    plain, off, ln = corpus["plain"], corpus["off"], corpus["len"]
    for i in range(len(ln)):
        assert dst[o[i]:o[i] + l[i]].tobytes() == plain[off[i]:off[i] + ln[i]].tobytes(), i


@pytest.mark.parametrize("kind", ["good", "corrupted"])
def test_dense_device_output(codec, corpus, kind):
    """QH_WHERE_DEVICE_DENSE: the decoded strings packed back to back in HBM
    (out[i].off = the decoded bytes of the successful strings before i),
    the same bytes, lengths and statuses as the oracle, on the corpus and on
    the corrupted strings (failed strings take no bytes)."""
    torch = torch_mod()
    if kind == "good":
        enc, eoff, elen = corpus["enc"], corpus["enc_off"], corpus["enc_len"]
    else:
        enc, eoff, elen = corpus["bad"], corpus["bad_off"], corpus["bad_len"]
    want_dst, want_slot, want_len, want_st = oracle.decode_batch(enc, eoff, elen)
    n = len(elen)
    cap = int(q.decode_slot_size(elen.astype(np.int64)).sum())
    dst = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    out = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    codec.decode_dev(to_dev(enc), spans_dev(eoff, elen), dst, out, dense=True)
    o, l, s = q.unpack_out(out)
    d = dst.cpu().numpy()
    assert (s == want_st.astype(np.int64)).all()
    ok = s == 0
    assert (l[ok] == want_len[ok].astype(np.int64)).all()
    lens = np.where(ok, l, 0)
    assert (o == np.concatenate([[0], np.cumsum(lens)[:-1]])).all()
    for i in np.nonzero(ok)[0]:
        w = want_dst[int(want_slot[i]):int(want_slot[i]) + int(want_len[i])]
        assert d[o[i]:o[i] + l[i]].tobytes() == w.tobytes(), i


def test_dense_device_output_cap_and_sorted(codec, corpus):
    """QH_WHERE_DEVICE_DENSE with dst_cap cut to half the decoded bytes:
    strings that fit keep their packed place and bytes, the first that does
    not and every later one get QH_ERR_NOMEM (nothing written past dst_cap);
    and with the sorted decoder the packed output is the window decoder's."""
    torch = torch_mod()
    enc, eoff, elen = corpus["enc"], corpus["enc_off"], corpus["enc_len"]
    want_dst, want_slot, want_len, want_st = oracle.decode_batch(enc, eoff, elen)
    n = len(elen)
    total = int(want_len.astype(np.int64).sum())
    cap = total // 2
    dst = torch.full((cap + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    out = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    codec.decode_dev(to_dev(enc), spans_dev(eoff, elen), dst[:cap], out, dense=True)
    o, l, s = q.unpack_out(out)
    d = dst.cpu().numpy()
    assert (d[cap:] == 0xAB).all()
    # (the slot-layout decode runs in a scratch of dst_cap bytes: the strings
    # whose slots end within it succeed -- a prefix of the batch -- and pack
    # into dst; every later one is QH_ERR_NOMEM)
    k = int(np.argmax(s != 0)) if (s != 0).any() else n
    assert 0 < k < n and (s[:k] == 0).all() and (s[k:] == q.QH_ERR_NOMEM).all()
    lens = want_len[:k].astype(np.int64)
    assert (l[:k] == lens).all() and (o[:k] == np.concatenate([[0], np.cumsum(lens)[:-1]])).all()
    assert int(lens.sum()) <= cap
    for j in range(0, k, max(1, k // 500)):
        ws = int(want_slot[j])
        assert d[o[j]:o[j] + l[j]].tobytes() == want_dst[ws:ws + int(want_len[j])].tobytes(), j
    # the sorted decoder, full cap: the same packed bytes and spans
    full = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
    out_w = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    codec.decode_dev(to_dev(enc), spans_dev(eoff, elen), full, out_w, dense=True)
    ref = (full[:total].cpu().numpy().copy(), out_w.cpu().numpy().copy())
    codec.set_decoder("sorted")
    try:
        full.zero_()
        codec.decode_dev(to_dev(enc), spans_dev(eoff, elen), full, out_w, dense=True)
        assert (full[:total].cpu().numpy() == ref[0]).all() and (out_w.cpu().numpy() == ref[1]).all()
    finally:
        codec.set_decoder("windows")


def test_corpus_encode(codec, corpus):
    plain, off, ln = corpus["plain"], corpus["off"], corpus["len"]
    enc, o, l, s = encode_dev(codec, plain, off, ln)
    assert (s == 0).all()
    assert (l == corpus["enc_len"].astype(np.int64)).all()
    assert (o == corpus["enc_off"].astype(np.int64)).all()
    total = int(corpus["enc_len"].astype(np.int64).sum())
    assert (enc[:total] == corpus["enc"]).all()


def test_stats_describe_the_last_op(corpus):
    """qh_ctx_last_stats after each op of a sequence on one context reports
    that op alone: the stats are double-buffered and an op's first kernel
    zeroes the buffer the next op uses (no memset command), so nothing of an
    earlier op may leak into a later one, in any order of ops."""
    from nghttp3_amd import HuffmanBatchCodec
    c = HuffmanBatchCodec(device=0)
    try:
        bad, boff, blen = corpus["bad"], corpus["bad_off"], corpus["bad_len"]
        nbad = int((corpus["bad_status"] != 0).sum())
        bad_out = int(corpus["bad_out_len"].astype(np.int64)[corpus["bad_status"] == 0].sum())
        enc, eoff, elen = corpus["enc"], corpus["enc_off"], corpus["enc_len"]
        plain, off, ln = corpus["plain"], corpus["off"], corpus["len"]
        ptotal, etotal = int(ln.astype(np.int64).sum()), int(elen.astype(np.int64).sum())
        for rep in range(3):
            _, _, _, s = decode_dev(c, bad, boff, blen)
            st = c.stats()
            assert st["n"] == len(blen) and st["n_errors"] == nbad and st["out_bytes"] == bad_out, (rep, st)
            _, _, _, s = encode_dev(c, plain, off, ln)
            st = c.stats()
            assert st["n"] == len(ln) and st["n_errors"] == 0 and st["out_bytes"] == etotal, (rep, st)
            _, _, _, s = decode_dev(c, enc, eoff, elen)
            st = c.stats()
            assert st["n"] == len(elen) and st["n_errors"] == 0 and st["out_bytes"] == ptotal, (rep, st)
            _, _, _, s = decode_dev(c, enc, eoff, elen)  # the same op twice in a row
            st = c.stats()
            assert st["n_errors"] == 0 and st["out_bytes"] == ptotal and st["in_bytes"] == etotal, (rep, st)
            _, _, _, s = encode_dev(c, plain, off, ln)
            _, _, _, s = encode_dev(c, plain, off, ln)
            st = c.stats()
            assert st["n_errors"] == 0 and st["out_bytes"] == etotal, (rep, st)
    finally:
        c.close()


def test_corpus_encode_count(codec, corpus):
    torch = torch_mod()
    plain, off, ln = corpus["plain"], corpus["off"], corpus["len"]
    hlen = torch.zeros(len(ln), dtype=torch.int32, device="cuda")
    codec.encode_count_dev(to_dev(plain), spans_dev(off, ln), hlen)
    assert (hlen.cpu().numpy().astype(np.int64) == corpus["enc_len"].astype(np.int64)).all()


def test_corrupted_statuses(codec, corpus):
    bad, boff, blen = corpus["bad"], corpus["bad_off"], corpus["bad_len"]
    dst, o, l, s = decode_dev(codec, bad, boff, blen)
    assert (s == corpus["bad_status"].astype(np.int64)).all()
    assert (l == corpus["bad_out_len"].astype(np.int64)).all()
    bo = corpus["bad_out"]
    pos = 0
    for i in range(len(blen)):
        n = int(corpus["bad_out_len"][i])
        if s[i] == 0:
            assert dst[o[i]:o[i] + n].tobytes() == bo[pos:pos + n].tobytes()
        pos += n


def test_error_fixture(codec, errors):
    strs = [bytes.fromhex(c["hex"]) for c in errors["whole"]]
    src, sp = q.pack_strings(strs)
    dst, o, l, s = decode_dev(codec, src, sp["off"], sp["len"])
    for i, c in enumerate(errors["whole"]):
        assert s[i] == c["status"], c
        if c["status"] == 0:
            assert dst[o[i]:o[i] + l[i]].tobytes().hex() == c["out_hex"]


def test_empty_batch_and_empty_strings(codec):
    torch = torch_mod()
    src = torch.zeros(16, dtype=torch.uint8, device="cuda")
    sp = torch.zeros((0, 2), dtype=torch.int64, device="cuda")
    out = torch.zeros((0, 2), dtype=torch.int64, device="cuda")
    codec.decode_dev(src, sp, src, out)
    codec.encode_dev(src, sp, src, out)
    codec.sync()
    dst, o, l, s = decode_dev(codec, np.zeros(4, np.uint8), [0, 1, 2], [0, 0, 0])
    assert (s == 0).all() and (l == 0).all()


def test_unordered_overlapping_spans(codec, corpus):
    # spans need not be packed or monotone: reverse order, duplicates, gaps.
    enc, eoff, elen = corpus["enc"], corpus["enc_off"], corpus["enc_len"]
    rng = np.random.default_rng(11)
    idx = rng.permutation(len(elen))[:1500]
    idx = np.concatenate([idx, idx[:100]])
    dst, o, l, s = decode_dev(codec, enc, eoff[idx], elen[idx])
    plain, off, ln = corpus["plain"], corpus["off"], corpus["len"]
    for j, i in enumerate(idx):
        assert s[j] == 0
        assert dst[o[j]:o[j] + l[j]].tobytes() == plain[off[i]:off[i] + ln[i]].tobytes()


def test_dst_cap_too_small(codec, corpus):
    # Strings whose group of output does not fit get QH_ERR_NOMEM and write
    # nothing; every other string is decoded correctly inside dst_cap.
    enc, eoff, elen = corpus["enc"], corpus["enc_off"], corpus["enc_len"]
    plain, off, ln = corpus["plain"], corpus["off"], corpus["len"]
    n = 3000
    slots = q.decode_slot_size(elen[:n].astype(np.int64))
    cap = int(slots.sum()) // 3
    dst, o, l, s = decode_dev(codec, enc, eoff[:n], elen[:n], cap=cap)
    assert set(np.unique(s)) <= {0, q.QH_ERR_NOMEM}
    assert (s == 0).any() and (s == q.QH_ERR_NOMEM).any()
    ok = s == 0
    assert_disjoint(o[ok], l[ok], cap)
    for i in np.nonzero(ok)[0]:
        assert dst[o[i]:o[i] + l[i]].tobytes() == plain[off[i]:off[i] + ln[i]].tobytes()


def test_host_path_matches(codec, corpus):
    enc, eoff, elen = corpus["enc"], corpus["enc_off"], corpus["enc_len"]
    sp = np.zeros(len(elen), dtype=q.SPAN_IN_DTYPE)
    sp["off"], sp["len"] = eoff, elen
    dst, out = codec.decode_host(enc, sp)
    want_dst, want_slot, want_len, want_st = oracle.decode_batch(enc, eoff, elen)
    assert (out["status"] == 0).all() and (out["len"] == want_len).all()
    plain, off, ln = corpus["plain"], corpus["off"], corpus["len"]
    for i in range(0, len(ln), 7):
        o, n_ = int(out["off"][i]), int(out["len"][i])
        assert dst[o:o + n_].tobytes() == plain[off[i]:off[i] + ln[i]].tobytes()
    psp = np.zeros(len(ln), dtype=q.SPAN_IN_DTYPE)
    psp["off"], psp["len"] = off, ln
    e2, eout = codec.encode_host(plain, psp)
    total = int(corpus["enc_len"].astype(np.int64).sum())
    assert (e2[:total] == corpus["enc"]).all()
    st = codec.stats()
    assert st["n"] == len(ln) and st["out_bytes"] == total
    assert (codec.encode_count_host(plain, psp) == corpus["enc_len"]).all()


def test_host_path_full_size_packed_and_pipelined(codec, digests):
    """Host-memory decode of config 3 at size (2^20 strings: eight slices on
    the copy / compute streams): out[i].off is the packed offset, and the
    packed bytes are the plaintext; with a dst_cap of half the plaintext
    the strings past it get QH_ERR_NOMEM and the rest still decode."""
    torch = torch_mod()
    d = digests["c3_A"]
    src, spans, total = codec.synth(d["seed"], d["n"], d["lo"], d["hi"], synth.ALPHABET_A)
    ln = spans[:, 1] & 0xFFFFFFFF
    enc = torch.zeros(int(((ln * 30 + 7) // 8).sum().item()), dtype=torch.uint8, device="cuda")
    eout = torch.zeros((d["n"], 2), dtype=torch.int64, device="cuda")
    codec.encode_dev(src, spans, enc, eout)
    torch.cuda.synchronize()
    e_h = enc[:d["enc_bytes"]].cpu().numpy()
    eo = eout.cpu().numpy()
    sp = np.zeros(d["n"], dtype=q.SPAN_IN_DTYPE)
    sp["off"], sp["len"] = eo[:, 0], eo[:, 1] & 0xFFFFFFFF
    plain = src[:total].cpu().numpy()
    lens = (spans[:, 1] & 0xFFFFFFFF).cpu().numpy()
    dst, out = codec.decode_host(e_h, sp)
    assert (out["status"] == 0).all() and (out["len"] == lens).all()
    assert (out["off"][1:] == np.cumsum(lens)[:-1]).all() and out["off"][0] == 0
    assert dst[:total].tobytes() == plain.tobytes()
    st = codec.stats()
    assert st["n_errors"] == 0 and st["out_bytes"] == total
    half = total // 2
    small = np.zeros(half, dtype=np.uint8)
    out2 = np.zeros(d["n"], dtype=q.SPAN_OUT_DTYPE)
    import ctypes
    from nghttp3_amd import _lib
    rv = codec._lib.qh_decode_batch(codec._ctx, e_h.ctypes.data_as(ctypes.c_void_p),
                                    sp.ctypes.data_as(ctypes.c_void_p), d["n"],
                                    small.ctypes.data_as(ctypes.c_void_p), half,
                                    out2.ctypes.data_as(ctypes.c_void_p), _lib.QH_WHERE_HOST)
    assert rv == 0
    ok = out2["status"] == 0
    assert set(np.unique(out2["status"])) <= {0, q.QH_ERR_NOMEM} and ok.any() and (~ok).any()
    k = int(np.argmin(ok))  # the first string that did not fit; none after it fits
    assert ok[:k].all() and not ok[k:].any()
    end = int(out2["off"][k - 1] + out2["len"][k - 1])
    assert end <= half and small[:end].tobytes() == plain[:end].tobytes()


@pytest.mark.parametrize("nctx", [2, 4])
def test_host_path_multi_context(codec, corpus, digests, nctx):
    """qh_decode_batch_multi: one host batch over nctx contexts on device 0
    (each with its own stream, host thread and H2D / decode / D2H pipeline;
    on a node, one context per GPU): config 3 at size, strings in global
    order, each range packed from its base (the estimate of the ranges before
    it), every string's bytes the plaintext; the corpus's corrupted strings
    give the oracle's statuses."""
    torch = torch_mod()
    from nghttp3_amd import HuffmanBatchCodec
    d = digests["c3_A"]
    src, spans, total = codec.synth(d["seed"], d["n"], d["lo"], d["hi"], synth.ALPHABET_A)
    ln = spans[:, 1] & 0xFFFFFFFF
    enc = torch.zeros(int(((ln * 30 + 7) // 8).sum().item()), dtype=torch.uint8, device="cuda")
    eout = torch.zeros((d["n"], 2), dtype=torch.int64, device="cuda")
    codec.encode_dev(src, spans, enc, eout)
    torch.cuda.synchronize()
    e_h = enc[:d["enc_bytes"]].cpu().numpy()
    eo = eout.cpu().numpy()
    sp = np.zeros(d["n"], dtype=q.SPAN_IN_DTYPE)
    sp["off"], sp["len"] = eo[:, 0], eo[:, 1] & 0xFFFFFFFF
    plain = src[:total].cpu().numpy()
    lens = ln.cpu().numpy()
    streams = [torch.cuda.Stream() for _ in range(nctx)]
    codecs = [HuffmanBatchCodec(0, stream=st) for st in streams]
    try:
        dst, out = HuffmanBatchCodec.decode_host_multi(codecs, e_h, sp)
        assert (out["status"] == 0).all() and (out["len"] == lens).all()
        assert (np.diff(out["off"].astype(np.int64)) >= out["len"][:-1].astype(np.int64)).all()
        starts = np.cumsum(lens) - lens
        gaps = out["off"].astype(np.int64) - starts  # constant within a range
        assert len(np.unique(gaps)) == nctx and gaps[0] == 0
        got = np.concatenate([dst[o:o + n_] for o, n_ in
                              zip(out["off"].astype(np.int64), lens.astype(np.int64))])
        assert got.tobytes() == plain.tobytes()
        # corrupted strings: the oracle's statuses, good strings' bytes
        bad, boff, blen = corpus["bad"], corpus["bad_off"], corpus["bad_len"]
        bsp = np.zeros(len(blen), dtype=q.SPAN_IN_DTYPE)
        bsp["off"], bsp["len"] = boff, blen
        dst2, out2 = HuffmanBatchCodec.decode_host_multi(codecs, bad, bsp)
        assert (out2["status"] == corpus["bad_status"]).all()
        assert (out2["len"] == corpus["bad_out_len"]).all()
    finally:
        for c in codecs:
            c.close()


def test_host_path_multi_device(codec, digests):
    """qh_decode_batch_multi with one context per GPU (devices 0 .. k-1, k <=
    8): each range's H2D, decode and D2H on its own GPU and link, its host
    thread making that device current.  Skips on a box with fewer than two
    GPUs (the driver's node has eight)."""
    torch = torch_mod()
    ndev = torch.cuda.device_count()
    if ndev < 2:
        pytest.skip("one GPU on this box")
    from nghttp3_amd import HuffmanBatchCodec
    d = digests["c3_A"]
    src, spans, total = codec.synth(d["seed"], d["n"], d["lo"], d["hi"], synth.ALPHABET_A)
    ln = spans[:, 1] & 0xFFFFFFFF
    enc = torch.zeros(int(((ln * 30 + 7) // 8).sum().item()), dtype=torch.uint8, device="cuda")
    eout = torch.zeros((d["n"], 2), dtype=torch.int64, device="cuda")
    codec.encode_dev(src, spans, enc, eout)
    torch.cuda.synchronize()
    e_h = enc[:d["enc_bytes"]].cpu().numpy()
    eo = eout.cpu().numpy()
    sp = np.zeros(d["n"], dtype=q.SPAN_IN_DTYPE)
    sp["off"], sp["len"] = eo[:, 0], eo[:, 1] & 0xFFFFFFFF
    plain = src[:total].cpu().numpy()
    lens = ln.cpu().numpy()
    k = min(ndev, 8)
    codecs = [HuffmanBatchCodec(i, stream=torch.cuda.Stream(device=i)) for i in range(k)]
    try:
        dst, out = HuffmanBatchCodec.decode_host_multi(codecs, e_h, sp)
        assert (out["status"] == 0).all() and (out["len"] == lens).all()
        got = np.concatenate([dst[o:o + n_] for o, n_ in
                              zip(out["off"].astype(np.int64), lens.astype(np.int64))])
        assert got.tobytes() == plain.tobytes()
    finally:
        for c in codecs:
            c.close()


def test_host_path_from_fresh_threads(codec, digests):
    """The host path's returner thread makes the context's device current
    itself (hipSetDevice(c->device) in decode_host_impl): decode_host called
    from a Python thread that never touched the GPU, and
    qh_decode_batch_multi over one context from another, both give the
    plaintext back -- the single-GPU run of the paths
    test_host_path_multi_device covers on a multi-GPU node."""
    import threading
    torch = torch_mod()
    from nghttp3_amd import HuffmanBatchCodec
    d = digests["c3_A"]
    n = 1 << 18  # two slices' worth and more (kHostSliceMin = 2^17)
    src, spans, total = codec.synth(d["seed"], n, d["lo"], d["hi"], synth.ALPHABET_A)
    ln = spans[:, 1] & 0xFFFFFFFF
    enc = torch.zeros(int(((ln * 30 + 7) // 8).sum().item()), dtype=torch.uint8, device="cuda")
    eout = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    codec.encode_dev(src, spans, enc, eout)
    torch.cuda.synchronize()
    eo = eout.cpu().numpy()
    sp = np.zeros(n, dtype=q.SPAN_IN_DTYPE)
    sp["off"], sp["len"] = eo[:, 0], eo[:, 1] & 0xFFFFFFFF
    e_h = enc[:int(sp["len"].sum())].cpu().numpy()
    plain = src[:total].cpu().numpy()
    lens = ln.cpu().numpy()
    res = {}

    def single():
        res["single"] = codec.decode_host(e_h, sp)

    def multi():
        res["multi"] = HuffmanBatchCodec.decode_host_multi([codec], e_h, sp)

    for fn in (single, multi):
        t = threading.Thread(target=fn)
        t.start()
        t.join(timeout=120)
        assert not t.is_alive()
    for key in ("single", "multi"):
        dst, out = res[key]
        assert (out["status"] == 0).all() and (out["len"] == lens).all(), key
        got = np.concatenate([dst[o:o + n_] for o, n_ in
                              zip(out["off"].astype(np.int64), lens.astype(np.int64))])
        assert got.tobytes() == plain.tobytes(), key


def test_host_path_multi_refuses_a_context_twice(codec, corpus):
    """One thread per context: the same context twice in the list is refused
    (QH_ERR_INVALID_ARGUMENT) before any work starts."""
    from nghttp3_amd import HuffmanBatchCodec
    enc, eoff, elen = corpus["enc"], corpus["enc_off"], corpus["enc_len"]
    sp = np.zeros(len(elen), dtype=q.SPAN_IN_DTYPE)
    sp["off"], sp["len"] = eoff, elen
    with pytest.raises(Exception) as ei:
        HuffmanBatchCodec.decode_host_multi([codec, codec], enc, sp)
    assert "-101" in str(ei.value) or "INVALID" in str(ei.value).upper()


def test_host_path_pinned_buffers(codec, corpus, digests):
    """Host-memory decode into pinned dst / out (direct DMA; in development
    builds with QHUFF_HOST_ZC=1 the device-to-host leg as shader stores into
    the caller's buffers, qh_k_copy16): config 3 at size gives the same
    packed bytes and spans as the pageable (staged-copy) path and writes
    nothing past them; a dst_cap of half the plaintext cuts at a string and
    is respected; the corpus's corrupted strings give the oracle's
    statuses."""
    torch = torch_mod()
    d = digests["c3_A"]
    src, spans, total = codec.synth(d["seed"], d["n"], d["lo"], d["hi"], synth.ALPHABET_A)
    ln = spans[:, 1] & 0xFFFFFFFF
    enc = torch.zeros(int(((ln * 30 + 7) // 8).sum().item()), dtype=torch.uint8, device="cuda")
    eout = torch.zeros((d["n"], 2), dtype=torch.int64, device="cuda")
    codec.encode_dev(src, spans, enc, eout)
    torch.cuda.synchronize()
    e_h = enc[:d["enc_bytes"]].cpu().numpy()
    eo = eout.cpu().numpy()
    sp = np.zeros(d["n"], dtype=q.SPAN_IN_DTYPE)
    sp["off"], sp["len"] = eo[:, 0], eo[:, 1] & 0xFFFFFFFF
    plain = src[:total].cpu().numpy()
    cap = int(q.decode_slot_size(sp["len"].astype(np.int64)).sum())
    pd = torch.full((cap,), 0xAB, dtype=torch.uint8).pin_memory()
    po = torch.zeros(d["n"] * 2, dtype=torch.int64).pin_memory()
    dst, out = codec.decode_host(e_h, sp, pd.numpy(), po.numpy().view(q.SPAN_OUT_DTYPE))
    dst_p, out_p = codec.decode_host(e_h, sp)  # pageable: the staged copies
    assert (out == out_p).all() and (out["status"] == 0).all()
    assert dst[:total].tobytes() == plain.tobytes() == dst_p[:total].tobytes()
    assert (dst[total:] == 0xAB).all()  # nothing written past the packed bytes
    half = total // 2
    ph = torch.full((half + 64,), 0xCD, dtype=torch.uint8).pin_memory()
    po2 = torch.zeros(d["n"] * 2, dtype=torch.int64).pin_memory()
    out2 = po2.numpy().view(q.SPAN_OUT_DTYPE)
    import ctypes
    from nghttp3_amd import _lib
    rv = codec._lib.qh_decode_batch(codec._ctx, e_h.ctypes.data_as(ctypes.c_void_p),
                                    sp.ctypes.data_as(ctypes.c_void_p), d["n"],
                                    ctypes.c_void_p(ph.data_ptr()), half,
                                    out2.ctypes.data_as(ctypes.c_void_p), _lib.QH_WHERE_HOST)
    assert rv == 0
    ok = out2["status"] == 0
    k = int(np.argmin(ok))
    assert ok[:k].all() and not ok[k:].any() and k > 0
    end = int(out2["off"][k - 1] + out2["len"][k - 1])
    small = ph.numpy()
    assert end <= half and small[:end].tobytes() == plain[:end].tobytes()
    assert (small[half:] == 0xCD).all()  # dst_cap is respected
    bad, boff, blen = corpus["bad"], corpus["bad_off"], corpus["bad_len"]
    bsp = np.zeros(len(blen), dtype=q.SPAN_IN_DTYPE)
    bsp["off"], bsp["len"] = boff, blen
    bcap = int(q.decode_slot_size(blen.astype(np.int64)).sum())
    pb = torch.zeros(bcap, dtype=torch.uint8).pin_memory()
    pbo = torch.zeros(len(blen) * 2, dtype=torch.int64).pin_memory()
    _, bout = codec.decode_host(bad, bsp, pb.numpy(), pbo.numpy().view(q.SPAN_OUT_DTYPE))
    assert (bout["status"] == corpus["bad_status"]).all()
    assert (bout["len"] == corpus["bad_out_len"].astype(np.int64)).all()


def test_synth_device_matches_host(codec):
    src, spans, total = codec.synth(0x1234, 5000, 1, 300, synth.ALPHABET_A)
    plain, off, ln = synth.batch(0x1234, 5000, 1, 300, synth.ALPHABET_A)
    sp = spans.cpu().numpy()
    assert total == plain.size
    assert (sp[:, 0] == off.astype(np.int64)).all()
    assert ((sp[:, 1] & 0xFFFFFFFF) == ln.astype(np.int64)).all()
    assert (src.cpu().numpy()[:total] == plain).all()


@pytest.mark.parametrize("name,decoder", [("c2_A", "windows"), ("c2_U", "windows"),
                                          ("c3_A", "windows"), ("c3_A", "waves"),
                                          ("c2_U", "waves"), ("c3_A", "fused"),
                                          ("c2_U", "fused"), ("c3_A", "sorted"),
                                          ("c2_U", "sorted"), ("c2_A", "region"),
                                          ("c3_A", "region"), ("c2_U", "region")])
def test_full_size_config(codec, digests, name, decoder):
    """BASELINE configs at full size (2^20 strings): synth digest, encode
    digest vs the oracle's, then decode round trip (size-independent), with
    either shipped decoder ("fused": the fused encoder, window decoder;
    "sorted": the window encoder, the sorted decoder)."""
    codec.set_decoder(decoder if decoder not in ("fused", "region") else "windows")
    codec.set_encoder(decoder if decoder != "sorted" else "windows")
    try:
        _full_size_config(codec, digests, name)
    finally:
        codec.set_decoder("windows")
        codec.set_encoder("windows")


def _full_size_config(codec, digests, name):
    torch = torch_mod()
    d = digests[name]
    alph = synth.ALPHABET_A if d["alphabet"] == "A" else synth.ALPHABET_U
    src, spans, total = codec.synth(d["seed"], d["n"], d["lo"], d["hi"], alph)
    assert total == d["plain_bytes"]
    assert sha(src[:total].cpu().numpy()) == d["plain_sha256"]
    n = d["n"]
    ln = spans[:, 1] & 0xFFFFFFFF
    bound = int(((ln * 30 + 7) // 8).sum().item())
    enc = torch.zeros(bound, dtype=torch.uint8, device="cuda")
    eout = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    codec.encode_dev(src, spans, enc, eout)
    st = codec.stats()
    assert st["n_errors"] == 0 and st["out_bytes"] == d["enc_bytes"]
    elen = (eout[:, 1] & 0xFFFFFFFF).to(torch.int32)
    assert sha(elen.cpu().numpy().astype(np.uint32)) == d["enc_len_sha256"]
    assert sha(enc[:d["enc_bytes"]].cpu().numpy()) == d["enc_sha256"]
    # decode what we encoded: encode's out spans are valid decode in spans
    cap = int(q.decode_slot_size(elen.to(torch.int64)).sum().item())
    dec = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    dout = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    codec.decode_dev(enc, eout, dec, dout)
    st = codec.stats()
    assert st["n_errors"] == 0 and st["out_bytes"] == total
    dlen = dout[:, 1] & 0xFFFFFFFF
    assert bool((dlen == ln).all())
    assert bool(((dout[:, 1] >> 32) == 0).all())
    # gather decoded bytes in string order and compare with the plaintext
    doff = dout[:, 0]
    poff = spans[:, 0]
    rep_d = torch.repeat_interleave(doff, ln)
    rep_p = torch.repeat_interleave(poff, ln)
    pos = torch.arange(total, device="cuda", dtype=torch.int64) - rep_p
    assert bool((dec[rep_d + pos] == src[:total]).all())


_ENV_PROBE = r"""
import hashlib, json, sys
import torch
from nghttp3_amd import HuffmanBatchCodec, synth
d = json.loads(sys.argv[1])
c = HuffmanBatchCodec(device=0)
src, spans, total = c.synth(d["seed"], d["n"], d["lo"], d["hi"], synth.ALPHABET_A)
ln = spans[:, 1] & 0xFFFFFFFF
enc = torch.zeros(int(((ln * 30 + 7) // 8).sum().item()), dtype=torch.uint8, device="cuda")
eout = torch.zeros((d["n"], 2), dtype=torch.int64, device="cuda")
c.encode_dev(src, spans, enc, eout)
elen = eout[:, 1] & 0xFFFFFFFF
cap = int(((elen * 8 // 5 + 16 + 63) // 64 * 64).sum().item())
dec = torch.zeros(cap, dtype=torch.uint8, device="cuda")
dout = torch.zeros((d["n"], 2), dtype=torch.int64, device="cuda")
c.decode_dev(enc, eout, dec, dout)
st = c.stats()
dlen = dout[:, 1] & 0xFFFFFFFF
rep_d = torch.repeat_interleave(dout[:, 0], ln)
pos = torch.arange(total, device="cuda", dtype=torch.int64) - torch.repeat_interleave(spans[:, 0], ln)
print(json.dumps({
    "enc_sha256": hashlib.sha256(enc[:d["enc_bytes"]].cpu().numpy().tobytes()).hexdigest(),
    "dec_ok": bool((dlen == ln).all()) and bool((dec[rep_d + pos] == src[:total]).all()),
    "errors": int(st["n_errors"])}))
"""


def test_results_ignore_environment(digests):
    """The product library reads no development knob from the environment
    (QHUFF_DEBUG bits used to skip or misplace the decoder's
    stores with every status 0): a fresh process with every former knob set
    to a hostile value still encodes config 3 to the oracle's digest and
    decodes it back bit-exact (the reference codec is pure,
    huffman.c:87-124)."""
    import json
    import subprocess
    import sys
    d = digests["c3_A"]
    env = dict(os.environ)
    env.update({"QHUFF_DEBUG": "0x1F", "QHUFF_DECODER": "bogus", "QHUFF_CODES": "fused",
                "QHUFF_LONG_MIN": "1", "QHUFF_PLAN_SKEW": "nan", "QHUFF_PLAN_SKEW_LONG": "-1",
                "QHUFF_BPC": "64", "QHUFF_ENC_BPC": "64", "QHUFF_ENC_THREADS": "128",
                "QHUFF_SEG": "1", "QHUFF_LENS_WIN64": "1", "QHUFF_HOST_MAPPED_ENDS": "1"})
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _ENV_PROBE, json.dumps(d)], env=env, cwd=root,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "not a decoder" not in r.stderr  # (QHUFF_DECODER is not even read)
    got = json.loads(r.stdout.strip().splitlines()[-1])
    assert got == {"enc_sha256": d["enc_sha256"], "dec_ok": True, "errors": 0}


def test_window_decoder_plan_mixed_blocks(codec, corpus):
    """The window decoder's per-block plan (qh_k_dec_plan): a batch whose
    first half has 8-256 B lengths (blocks decoded from their windows of
    consecutive strings) and second half Zipf lengths to 4 KiB with some
    strings of 4-40 KB (blocks that sort themselves by length class), plus
    the corpus's corrupted strings spread through both halves: every
    string's status and bytes are the oracle's, and the output layout is
    the slot layout (out[i].off = the sum of the slots before string i)."""
    torch = torch_mod()
    rng = np.random.default_rng(0x5EED0420)
    n_half = 1 << 18  # (> 256 strings per block of the 1,024-block cut: the plan sorts only those)
    ln = np.concatenate([synth.lengths(0x5EED0421, n_half, 8, 256),
                         synth.zipf_lengths(0x5EED0422, n_half, 1, 4096, 1.2)]).astype(np.uint32)
    ln[n_half + rng.choice(n_half, 40, replace=False)] = rng.integers(5000, 40000, 40)
    plain = synth.fill(0x5EED0423, int(ln.sum(dtype=np.uint64)), synth.ALPHABET_A)
    off = np.concatenate([[0], np.cumsum(ln.astype(np.uint64))[:-1]]).astype(np.uint64)
    enc, eoff, elen = oracle.encode_batch(plain, off, ln)
    # corrupted strings in place of some encodings, in both halves
    bad, boff, blen = corpus["bad"], corpus["bad_off"], corpus["bad_len"]
    pos = np.sort(rng.choice(2 * n_half, len(blen), replace=False))
    strs = [enc[int(o):int(o) + int(l)].tobytes() for o, l in zip(eoff, elen)]
    for k, i in enumerate(pos):
        strs[i] = bad[int(boff[k]):int(boff[k]) + int(blen[k])].tobytes()
    src, sp = q.pack_strings(strs)
    want_dst, want_slot, want_len, want_st = oracle.decode_batch(src, sp["off"], sp["len"])
    d_src = torch.from_numpy(src.copy()).cuda()
    d_sp = torch.from_numpy(sp.view(np.int64).reshape(-1, 2).copy()).cuda()
    cap = int(q.decode_slot_size(sp["len"].astype(np.int64)).sum())
    d_dst = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    d_out = torch.zeros((len(strs), 2), dtype=torch.int64, device="cuda")
    codec.decode_dev(d_src, d_sp, d_dst, d_out)
    o, l, st = q.unpack_out(d_out)
    assert (st == want_st).all() and (l == want_len).all()
    slots = q.decode_slot_size(sp["len"].astype(np.int64))
    assert (o == np.concatenate([[0], np.cumsum(slots)[:-1]])).all()
    dst = d_dst.cpu().numpy()
    check = np.zeros(len(strs), dtype=bool)
    check[::7] = True
    check[pos] = True
    check[np.nonzero(sp["len"] >= 4096)[0]] = True
    for i in np.nonzero(check & (st == 0))[0]:
        assert dst[o[i]:o[i] + l[i]].tobytes() == want_dst[int(want_slot[i]):int(want_slot[i]) + int(l[i])].tobytes(), i


@pytest.mark.parametrize("decoder", ["windows", "waves", "sorted", "region"])
def test_config5_rank_shard_full_size(codec, digests, decoder):
    """Config 5 at size: rank 0's shard of 16M Zipf strings split by bytes
    over 8 GPUs (2.1M strings, 438 MB, lengths 1..4096), as bench.py cuts
    it: the device generator from the global byte offset, encode digests vs
    the oracle's, then the decode round trip (chunked compare)."""
    codec.set_decoder(decoder if decoder != "region" else "sorted")
    # the shipped kernel pairs for skewed lengths ("region": the region codes
    # pass over the Zipf shard's packed strings, the sorted decoder)
    codec.set_encoder({"windows": "windows", "waves": "waves", "sorted": "fused",
                       "region": "region"}[decoder])
    try:
        _config5_rank_shard(codec, digests)
    finally:
        codec.set_decoder("windows")
        codec.set_encoder("windows")


def _config5_rank_shard(codec, digests):
    from nghttp3_amd import shard
    torch = torch_mod()
    d = digests["c5_r0of8"]
    ln_all = synth.zipf_lengths(d["seed"], d["n_total"], d["lo"], d["hi"], d["s"])
    b, e = shard.split_by_bytes(ln_all, d["world"])[d["rank"]]
    assert (b, e) == (d["begin"], d["end"])
    my = ln_all[b:e]
    assert sha(my) == d["len_sha256"]
    first = int(ln_all[:b].sum(dtype=np.uint64))
    spans, total = codec.spans_to_device(my)
    src = codec.synth_fill(d["seed"], first, total, synth.ALPHABET_A)
    assert total == d["plain_bytes"] and sha(src[:total].cpu().numpy()) == d["plain_sha256"]
    n = e - b
    enc = torch.zeros(int((my.astype(np.int64) * 30 + 7).sum() // 8) + 64, dtype=torch.uint8,
                      device="cuda")
    eout = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    codec.encode_dev(src, spans, enc, eout)
    st = codec.stats()
    assert st["n_errors"] == 0 and st["out_bytes"] == d["enc_bytes"]
    elen = eout[:, 1] & 0xFFFFFFFF
    assert sha(elen.cpu().numpy().astype(np.uint32)) == d["enc_len_sha256"]
    assert sha(enc[:d["enc_bytes"]].cpu().numpy()) == d["enc_sha256"]
    cap = int(q.decode_slot_size(elen).sum().item())
    dec = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    dout = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    codec.decode_dev(enc, eout, dec, dout)
    st = codec.stats()
    assert st["n_errors"] == 0 and st["out_bytes"] == total
    ln = spans[:, 1]
    assert bool(((dout[:, 1] & 0xFFFFFFFF) == ln).all()) and bool(((dout[:, 1] >> 32) == 0).all())
    for i0 in range(0, n, 1 << 19):
        i1 = min(n, i0 + (1 << 19))
        l = ln[i0:i1]
        t = int(l.sum().item())
        pos = torch.arange(t, device="cuda", dtype=torch.int64) - \
            torch.repeat_interleave(torch.cumsum(l, 0) - l, l)
        assert bool((dec[torch.repeat_interleave(dout[i0:i1, 0], l) + pos] ==
                     src[torch.repeat_interleave(spans[i0:i1, 0], l) + pos]).all())


def test_encode_unordered_spans(codec, corpus):
    # spans in any order: same bytes, dense output in span order
    plain, off, ln = corpus["plain"], corpus["off"], corpus["len"]
    rng = np.random.default_rng(5)
    idx = rng.permutation(len(ln))[:2000]
    enc, o, l, s = encode_dev(codec, plain, off[idx], ln[idx])
    assert (s == 0).all()
    for j, i in enumerate(idx):
        want = oracle.encode(plain[off[i]:off[i] + ln[i]].tobytes())
        assert enc[o[j]:o[j] + l[j]].tobytes() == want


def test_encode_gapped_spans(codec, corpus):
    # spans with gaps between strings (header-block framing bytes)
    plain, off, ln = corpus["plain"], corpus["off"], corpus["len"]
    rng = np.random.default_rng(6)
    gaps = rng.integers(0, 9, len(ln))
    buf = bytearray()
    offs = []
    for i in range(len(ln)):
        buf += bytes(rng.integers(0, 256, gaps[i]).astype(np.uint8))
        offs.append(len(buf))
        buf += plain[off[i]:off[i] + ln[i]].tobytes()
    src = np.frombuffer(bytes(buf), dtype=np.uint8)
    enc, o, l, s = encode_dev(codec, src, np.array(offs), ln)
    assert (s == 0).all()
    total = int(corpus["enc_len"].astype(np.int64).sum())
    assert (l == corpus["enc_len"].astype(np.int64)).all()
    assert (enc[:total] == corpus["enc"]).all()


def test_encode_overlapping_spans(codec, corpus):
    # heavily overlapping spans (each string starts 3 bytes after the last)
    # and windows mixing near and far spans: lengths and codes per string
    plain = corpus["plain"]
    rng = np.random.default_rng(8)
    n = 3000
    off = np.arange(n, dtype=np.int64) * 3
    ln = rng.integers(0, 400, n).astype(np.int64)
    far = rng.random(n) < 0.02
    off[far] = rng.integers(0, plain.size - 400, int(far.sum()))
    enc, o, l, s = encode_dev(codec, plain, off, ln)
    assert (s == 0).all()
    for j in range(n):
        want = oracle.encode(plain[off[j]:off[j] + ln[j]].tobytes())
        assert enc[o[j]:o[j] + l[j]].tobytes() == want, j


def _mixed_strings(rng, big_len):
    """Empty, short, long and one stage-sized string (codes > 24 KiB, so the
    encoder's direct-to-HBM path runs); alphabet A and uniform bytes."""
    a = np.frombuffer(synth.ALPHABET_A, dtype=np.uint8)
    strs = []
    for i in range(700):
        k = int(rng.integers(0, 5))
        n = [0, int(rng.integers(1, 16)), int(rng.integers(16, 300)),
             int(rng.integers(300, 5000)), int(rng.integers(1, 64))][k]
        if i % 3:
            strs.append(bytes(rng.choice(a, n)))
        else:
            strs.append(bytes(rng.integers(0, 256, n).astype(np.uint8)))
    strs[350] = bytes(rng.choice(a, big_len))
    return strs


def test_mixed_lengths_roundtrip(codec):
    rng = np.random.default_rng(21)
    strs = _mixed_strings(rng, 40000)
    ln = np.array([len(x) for x in strs], dtype=np.int64)
    off = np.concatenate([[0], np.cumsum(ln)[:-1]])
    plain = np.frombuffer(b"".join(strs), dtype=np.uint8)
    enc, o, l, s = encode_dev(codec, plain, off, ln)
    assert (s == 0).all()
    want = [oracle.encode(x) for x in strs]
    assert (l == np.array([len(w) for w in want])).all()
    assert (o == np.concatenate([[0], np.cumsum(l)[:-1]])).all()  # dense
    for j in range(len(strs)):
        assert enc[o[j]:o[j] + l[j]].tobytes() == want[j], j
    dst, do, dl, ds = decode_dev(codec, enc, o, l)
    assert (ds == 0).all() and (dl == ln).all()
    assert_disjoint(do, dl, int(q.decode_slot_size(l).sum()))
    for j in range(len(strs)):
        assert dst[do[j]:do[j] + dl[j]].tobytes() == strs[j], j


def test_encode_dst_cap_too_small(codec, corpus):
    # strings whose encoding would pass dst_cap get NOMEM; nothing is written
    # at or past dst_cap; the others are exact
    torch = torch_mod()
    plain, off, ln = corpus["plain"], corpus["off"], corpus["len"]
    n = 3000
    want_len = corpus["enc_len"][:n].astype(np.int64)
    cap = int(want_len.sum()) // 2
    src = to_dev(plain)
    dst = torch.full((cap + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    out = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    codec.encode_dev(src, spans_dev(off[:n], ln[:n]), dst[:cap], out)
    o, l, s = q.unpack_out(out)
    d = dst.cpu().numpy()
    assert (d[cap:] == 0xA5).all()
    assert set(np.unique(s)) <= {0, q.QH_ERR_NOMEM}
    ok = s == 0
    assert ok.any() and (~ok).any()
    assert (o[ok] + l[ok] <= cap).all()
    for j in np.nonzero(ok)[0]:
        want = oracle.encode(plain[off[j]:off[j] + ln[j]].tobytes())
        assert d[o[j]:o[j] + l[j]].tobytes() == want


# The two shipped decoders (qh_ctx_set_decoder); the development variants
# (make dev) are timed by dev/scripts/dec_variants.py, not shipped.
DECODERS = ["windows", "waves", "sorted"]
# (development: QHUFF_LIB=nghttp3_amd/lib/libqhuff_dev.so QH_TEST_DEV_DECODERS=
# peek11su,... adds those variants of the development build to these tests)
DECODERS += ["dev:" + k for k in os.environ.get("QH_TEST_DEV_DECODERS", "").split(",") if k]


def codec_of(kind):
    from nghttp3_amd import HuffmanBatchCodec
    if kind.startswith("dev:"):
        old = os.environ.get("QHUFF_DECODER")
        os.environ["QHUFF_DECODER"] = kind[4:]
        try:
            return HuffmanBatchCodec(device=0)
        finally:
            if old is None:
                del os.environ["QHUFF_DECODER"]
            else:
                os.environ["QHUFF_DECODER"] = old
    c = HuffmanBatchCodec(device=0)
    c.set_decoder(kind)
    return c


@pytest.mark.parametrize("kind", DECODERS)
def test_decoder_variants(kind, corpus, errors, kat, codec):
    """Both decoders (the window decoder: sorted 256-string windows, W-bit
    peek table in lock-step; the wave decoder: per-wave sorted chunks, input
    through LDS rings)
    give the oracle's bytes and statuses: golden corpus, corrupted strings,
    the reference's error verdicts, RFC vectors, and mixed lengths 0-5000 B
    over alphabet A and all 256 byte values (long codes, EOS-prefix ends)."""
    c = codec_of(kind)
    try:
        bad, boff, blen = corpus["bad"], corpus["bad_off"], corpus["bad_len"]
        dst, o, l, s = decode_dev(c, bad, boff, blen)
        assert (s == corpus["bad_status"]).all()
        assert (l == corpus["bad_out_len"].astype(np.int64)).all()
        bolen = corpus["bad_out_len"].astype(np.int64)
        ooff = np.concatenate([[0], np.cumsum(bolen)])
        for i in np.nonzero(s == 0)[0]:
            assert dst[o[i]:o[i] + l[i]].tobytes() == corpus["bad_out"][ooff[i]:ooff[i + 1]].tobytes()
        enc, eoff, elen = corpus["enc"], corpus["enc_off"], corpus["enc_len"]
        dst, o, l, s = decode_dev(c, enc, eoff, elen)
        assert (s == 0).all()
        assert_disjoint(o, l, int(q.decode_slot_size(elen.astype(np.int64)).sum()))
        plain, off, ln = corpus["plain"], corpus["off"], corpus["len"]
        for i in range(len(ln)):
            assert dst[o[i]:o[i] + l[i]].tobytes() == plain[off[i]:off[i] + ln[i]].tobytes()
        strs = [bytes.fromhex(x["hex"]) for x in errors["whole"]]
        src, sp = q.pack_strings(strs)
        dst, o, l, s = decode_dev(c, src, sp["off"], sp["len"])
        for i, x in enumerate(errors["whole"]):
            assert s[i] == x["status"], x
            if x["status"] == 0:
                assert dst[o[i]:o[i] + l[i]].tobytes().hex() == x["out_hex"]
        src, sp = q.pack_strings([bytes.fromhex(v["huffman_hex"]) for v in kat])
        dst, o, l, s = decode_dev(c, src, sp["off"], sp["len"])
        for i, v in enumerate(kat):
            assert s[i] == 0 and dst[o[i]:o[i] + l[i]].tobytes() == v["plain"].encode()
        rng = np.random.default_rng(77)
        strs = _mixed_strings(rng, 9000)
        encs = [oracle.encode(x) for x in strs]
        src, sp = q.pack_strings(encs)
        dst, o, l, s = decode_dev(c, src, sp["off"], sp["len"])
        assert (s == 0).all()
        for j in range(len(strs)):
            assert dst[o[j]:o[j] + l[j]].tobytes() == strs[j], j
        # random bytes as Huffman input: statuses and outputs as the oracle
        rb = [bytes(rng.integers(0, 256, int(rng.integers(0, 200))).astype(np.uint8))
              for _ in range(3000)]
        rb += [e[:-1] for e in encs[:300] if len(e) > 1]  # truncated strings
        src, sp = q.pack_strings(rb)
        want_dst, want_slot, want_len, want_st = oracle.decode_batch(src, sp["off"], sp["len"])
        dst, o, l, s = decode_dev(c, src, sp["off"], sp["len"])
        assert (s == want_st.astype(np.int64)).all()
        assert (l == want_len.astype(np.int64)).all()
        for j in np.nonzero(s == 0)[0]:
            ws = int(want_slot[j])
            assert dst[o[j]:o[j] + l[j]].tobytes() == want_dst[ws:ws + int(want_len[j])].tobytes()
    finally:
        c.close()


def _long_mode_batch(rng):
    """Strings that drive the window decoder's long iterations (pkv::kLongCodes, qh_dec_common.inc):
    binary text, binary then header text and back, errors met inside long
    iterations (an EOS code mid-string, a cut last code, bad padding), and
    header text sharing windows with them."""
    A = np.frombuffer(synth.ALPHABET_A, dtype=np.uint8)
    def txt(alpha, n):
        return bytes(alpha[rng.integers(0, len(alpha), n)]) if alpha is not None else \
            bytes(rng.integers(0, 256, n).astype(np.uint8))
    plain = []
    for i in range(6000):
        k = i % 6
        n = int(rng.integers(0, 400))
        if k == 0:
            plain.append(txt(None, n))                          # binary
        elif k == 1:
            plain.append(txt(None, n) + txt(A, n))              # binary, then text
        elif k == 2:
            plain.append(txt(A, n // 4) + txt(None, n) + txt(A, 20))
        else:
            plain.append(txt(A, n))                             # text in the same windows
    encs = [oracle.encode(x) for x in plain]
    out = []
    eos = bytes([0xFF, 0xFF, 0xFF, 0xFC])  # 30 ones then 00: an EOS code
    for i, e in enumerate(encs):
        k = i % 7
        if k == 3 and len(e) > 8:
            j = int(rng.integers(1, len(e) - 4))
            e = e[:j] + eos + e[j:]                            # EOS mid-string
        elif k == 4 and len(e) > 1:
            e = e[:-int(rng.integers(1, min(len(e), 5)))]      # cut inside the last codes
        elif k == 5 and len(e) > 1:
            e = e[:-1] + bytes([e[-1] & 0xFE])                 # padding with a zero bit
        elif k == 6 and len(e) > 2:
            j = int(rng.integers(0, len(e)))
            e = e[:j] + bytes([e[j] ^ (1 << int(rng.integers(0, 8)))]) + e[j + 1:]
        out.append(e)
    return out


@pytest.mark.parametrize("kind", DECODERS)
def test_long_code_mode_matches_oracle(kind):
    """Binary-heavy strings (the long-code iterations of the window decoder,
    the careful path of both) with errors inside them: statuses, lengths and
    bytes as the oracle's decode of lib/nghttp3_qpack_huffman.c."""
    c = codec_of(kind)
    try:
        strs = _long_mode_batch(np.random.default_rng(4242))
        src, sp = q.pack_strings(strs)
        want_dst, want_slot, want_len, want_st = oracle.decode_batch(src, sp["off"], sp["len"])
        assert (want_st != 0).sum() > 1000 and (want_st == 0).sum() > 3000
        dst, o, l, s = decode_dev(c, src, sp["off"], sp["len"])
        assert (s == want_st.astype(np.int64)).all()
        assert (l == want_len.astype(np.int64)).all()
        for j in np.nonzero(s == 0)[0]:
            ws = int(want_slot[j])
            assert dst[o[j]:o[j] + l[j]].tobytes() == want_dst[ws:ws + int(want_len[j])].tobytes(), j
    finally:
        c.close()


def _long_strings(rng, n_ok, alphabet, lo, hi):
    """n_ok strings of lo..hi plaintext bytes over `alphabet`, oracle-encoded,
    plus corrupted copies of some of them (a bit flipped, EOS appended,
    the last byte dropped, padding zeroed)."""
    alph = np.frombuffer(alphabet, dtype=np.uint8)
    plains = [bytes(alph[rng.integers(0, alph.size, int(rng.integers(lo, hi + 1)))]) for _ in range(n_ok)]
    src, sp = q.pack_strings(plains)
    enc, eoff, elen = oracle.encode_batch(src, sp["off"], sp["len"])
    strs = [bytes(enc[int(o):int(o) + int(l)]) for o, l in zip(eoff, elen)]
    bad = []
    for k, e in enumerate(strs[: n_ok // 2]):
        b = bytearray(e)
        kind = k % 4
        if kind == 0:
            b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
        elif kind == 1:
            b += b"\xff\xff\xff\xfc"  # EOS (30 ones) and more
        elif kind == 2:
            b = b[:-1] + b"\x00"
        else:
            b[-1] &= 0xF0
        bad.append(bytes(b))
    return strs + bad


@pytest.mark.parametrize("decoder", ["sorted", "windows"])
@pytest.mark.parametrize("alphabet", ["A", "U"])
def test_long_strings_wave_per_string(alphabet, decoder):
    """The wave-per-string path (qh_peek_dec.inc pk_long_string: lanes
    start at 16-byte boundaries and resynchronise) on strings of 4-40 KB --
    the sorted decoder's longest class, the window decoder's deferred
    strings -- and on strings of 200-3000 B with the sorted decoder's
    threshold lowered (qh_ctx_set_option QH_OPT_LONG_MIN) so that both paths run in one batch:
    statuses, lengths and bytes as the oracle's."""
    from nghttp3_amd import HuffmanBatchCodec
    rng = np.random.default_rng(0x10A9 + (alphabet == "U"))
    alph = synth.ALPHABET_A if alphabet == "A" else synth.ALPHABET_U
    cases = [(None, _long_strings(rng, 96, alph, 4096, 40000)),
             ("300", _long_strings(rng, 600, alph, 200, 3000) + _long_strings(rng, 40, alph, 1, 64))]
    for long_min, strs in cases:
        c = HuffmanBatchCodec(device=0)
        if long_min is not None:
            c.set_option("long_min", int(long_min))
        try:
            c.set_decoder(decoder)
            order = rng.permutation(len(strs))
            strs = [strs[i] for i in order]
            src, sp = q.pack_strings(strs)
            want_dst, want_slot, want_len, want_st = oracle.decode_batch(src, sp["off"], sp["len"])
            assert (want_st != 0).sum() > 10 and (want_st == 0).sum() > 40
            dst, o, l, s = decode_dev(c, src, sp["off"], sp["len"])
            assert (s == want_st.astype(np.int64)).all()
            assert (l == want_len.astype(np.int64)).all()
            for j in np.nonzero(s == 0)[0]:
                ws = int(want_slot[j])
                assert dst[o[j]:o[j] + l[j]].tobytes() == want_dst[ws:ws + int(want_len[j])].tobytes(), j
        finally:
            c.close()


@pytest.mark.parametrize("mode", ["default", "lane"])
def test_encode_length_passes(mode, corpus, digests):
    """The encoder's passes: streaming lengths + lane-per-string codes
    (default), and every window's lengths counted a lane per string inside
    the length kernel (QH_OPT_LENS_LANE_PASS, the scattered-window path) -- corpus
    lengths/codes, counts, overlapping and scattered spans, and the
    full-size c2_U digest."""
    import os
    from nghttp3_amd import HuffmanBatchCodec
    c = HuffmanBatchCodec(device=0)
    if mode == "lane":
        c.set_option("lens_lane_pass", 1)
    try:
        torch = torch_mod()
        test_corpus_encode(c, corpus)
        test_corpus_encode_count(c, corpus)
        test_encode_overlapping_spans(c, corpus)
        test_encode_unordered_spans(c, corpus)
        test_encode_gapped_spans(c, corpus)
        d = digests["c2_U"]
        src, spans, total = c.synth(d["seed"], d["n"], d["lo"], d["hi"], synth.ALPHABET_U)
        ln = spans[:, 1] & 0xFFFFFFFF
        enc = torch.zeros(int(((ln * 30 + 7) // 8).sum().item()), dtype=torch.uint8,
                          device="cuda")
        eout = torch.zeros((d["n"], 2), dtype=torch.int64, device="cuda")
        for _ in range(2):  # (the second call: the double-buffered stats and totals)
            c.encode_dev(src, spans, enc, eout)
            st = c.stats()
            assert st["n_errors"] == 0 and st["out_bytes"] == d["enc_bytes"]
            elen = (eout[:, 1] & 0xFFFFFFFF).to(torch.int32)
            assert sha(elen.cpu().numpy().astype(np.uint32)) == d["enc_len_sha256"]
            assert sha(enc[:d["enc_bytes"]].cpu().numpy()) == d["enc_sha256"]
    finally:
        c.close()


@pytest.mark.parametrize("alphabet", ["A", "U"])
def test_zipf_lengths_roundtrip(codec, alphabet):
    """Config-5 shape at reduced size: Zipf(s = 1.2) lengths 1..4096 (long
    strings span many decoder iterations and length-pass rounds), packed;
    encode against the oracle's batch encoder, then decode back."""
    rng = np.random.default_rng(55)
    n = 12000
    ranks = np.arange(1, 4097, dtype=np.float64)
    p = ranks ** -1.2
    p /= p.sum()
    ln = rng.choice(np.arange(1, 4097), size=n, p=p).astype(np.int64)
    a = np.frombuffer(synth.ALPHABET_A if alphabet == "A" else synth.ALPHABET_U, dtype=np.uint8)
    plain = a[rng.integers(0, len(a), int(ln.sum()))]
    off = np.concatenate([[0], np.cumsum(ln)[:-1]])
    want_enc, want_off, want_len = oracle.encode_batch(plain, off, ln)[:3]
    enc, o, l, s = encode_dev(codec, plain, off, ln)
    assert (s == 0).all()
    assert (l == np.asarray(want_len, dtype=np.int64)).all()
    total = int(l.sum())
    assert (enc[:total] == np.asarray(want_enc)[:total]).all()
    dst, do, dl, ds = decode_dev(codec, enc[:total], o, l)
    assert (ds == 0).all() and (dl == ln).all()
    for j in range(0, n, 37):
        assert dst[do[j]:do[j] + dl[j]].tobytes() == plain[off[j]:off[j] + ln[j]].tobytes(), j


# The shipped encoders (qh_ctx_set_encoder): the window encoder (a sorted
# 256-string window per workgroup, LDS stage, coalesced copy-out), the wave
# encoder (per-wave sorted chunks, LDS rings, per-lane 16-byte output
# chunks), the fused one-pass encoder, and the default that picks one of
# the window and fused encoders per batch on the device (QH_ENCODER_AUTO:
# the text cases here take the window path, Zipf, mixed and binary the
# fused one).
ENCODERS = ["windows", "waves", "fused", "auto", "region"]


@pytest.mark.parametrize("kind", ENCODERS)
def test_encoder_variants(kind, corpus, kat, digests):
    """Both encoders give the oracle's bytes: RFC vectors, the golden corpus,
    unordered / gapped / overlapping spans, mixed lengths 0-40000 B over
    alphabet A and all 256 byte values, Zipf lengths, dst_cap refusals, an
    output buffer at every alignment mod 16, and the full-size c2_U digest."""
    from nghttp3_amd import HuffmanBatchCodec
    torch = torch_mod()
    c = HuffmanBatchCodec(device=0)
    c.set_encoder(kind)
    try:
        plains = [v["plain"].encode() for v in kat]
        src, sp = q.pack_strings(plains)
        enc, o, l, s = encode_dev(c, src, sp["off"], sp["len"])
        for i, v in enumerate(kat):
            assert enc[o[i]:o[i] + l[i]].tobytes().hex() == v["huffman_hex"]
        test_corpus_encode(c, corpus)
        test_encode_unordered_spans(c, corpus)
        test_encode_gapped_spans(c, corpus)
        test_encode_overlapping_spans(c, corpus)
        test_mixed_lengths_roundtrip(c)
        test_encode_dst_cap_too_small(c, corpus)
        test_zipf_lengths_roundtrip(c, "U")
        # dst at every alignment: strings' first / last output chunks are
        # written bytewise where they share a dword with a neighbour
        plain, off, ln = corpus["plain"], corpus["off"], corpus["len"]
        n = 2000
        want_len = corpus["enc_len"][:n].astype(np.int64)
        total = int(want_len.sum())
        srcd, spd = to_dev(plain), spans_dev(off[:n], ln[:n])
        for a in range(16):
            buf = torch.full((total + 64,), 0x5A, dtype=torch.uint8, device="cuda")
            out = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
            c.encode_dev(srcd, spd, buf[a:a + total], out)
            d = buf.cpu().numpy()
            assert (d[:a] == 0x5A).all() and (d[a + total:] == 0x5A).all(), a
            assert (d[a:a + total] == corpus["enc"][:total]).all(), a
        d = digests["c2_U"]
        srcu, spans, _ = c.synth(d["seed"], d["n"], d["lo"], d["hi"], synth.ALPHABET_U)
        lnu = spans[:, 1] & 0xFFFFFFFF
        encu = torch.zeros(int(((lnu * 30 + 7) // 8).sum().item()), dtype=torch.uint8,
                           device="cuda")
        eout = torch.zeros((d["n"], 2), dtype=torch.int64, device="cuda")
        c.encode_dev(srcu, spans, encu, eout)
        st = c.stats()
        assert st["n_errors"] == 0 and st["out_bytes"] == d["enc_bytes"]
        assert sha(encu[:d["enc_bytes"]].cpu().numpy()) == d["enc_sha256"]
    finally:
        c.close()


@pytest.mark.gpu
def test_cu_masked_stream_fallbacks(corpus):
    """A context on a stream whose CU mask leaves out most of the chip
    (hipExtStreamCreateWithCUMask, 96 of 256 CUs: some XCDs get no wave)
    takes the one-ticket-counter forms of the fused encoder and the framing
    count (qh_api.inc stream_all_cus): their results equal the full-chip
    context's."""
    import ctypes
    from nghttp3_amd import HuffmanBatchCodec, qpack
    torch = torch_mod()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_uint32)]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    mask = (ctypes.c_uint32 * 8)(0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0, 0, 0, 0, 0)
    stream = ctypes.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(stream), 8, mask) == 0
    # the library's test (stream_all_cus): the stream's mask, as HIP reports it,
    # must not cover every CU
    hip.hipExtStreamGetCUMask.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    got_mask = (ctypes.c_uint32 * 8)()
    assert hip.hipExtStreamGetCUMask(stream, 8, got_mask) == 0
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    assert 0 < sum(bin(x).count("1") for x in got_mask) < ncu
    full = HuffmanBatchCodec(device=0)
    part = HuffmanBatchCodec(device=0, stream=stream.value)
    try:
        # the fused encoder: corpus strings and a 300k-string synthetic batch
        n = len(corpus["len"])
        srcd = to_dev(corpus["plain"])
        spd = spans_dev(corpus["off"], corpus["len"])
        cases = [(srcd, spd, n)]
        s2, sp2, _ = full.synth(0x5EED00C0, 300000, 1, 300, synth.ALPHABET_A)
        cases.append((s2, sp2, 300000))
        for src, sp, m in cases:
            ln = (sp[:, 1] & 0xFFFFFFFF).cpu().numpy().astype(np.int64)
            bound = int(((ln * 30 + 7) // 8).sum()) + 16
            res = []
            for c in (full, part):
                c.set_encoder("fused")
                dst = torch.zeros(bound, dtype=torch.uint8, device="cuda")
                out = torch.zeros((m, 2), dtype=torch.int64, device="cuda")
                torch.cuda.synchronize()
                c.encode_dev(src, sp, dst, out)
                c.sync()
                torch.cuda.synchronize()
                res.append((dst.cpu().numpy(), out.cpu().numpy()))
            assert np.array_equal(res[0][1], res[1][1])
            assert np.array_equal(res[0][0], res[1][0])
            o, l, s = q.unpack_out(torch.from_numpy(res[1][1]))
            assert (s == 0).all()
        # framing (qh_k_frame_count's tickets) through the sections decoder
        src, blocks, *_ = qpack.synth_field_sections(0x5EED0004, 20000)
        d_src = torch.from_numpy(np.ascontiguousarray(src)).cuda()
        d_blk = torch.from_numpy(blocks.view(np.int64).reshape(-1, 2).copy()).cuda()
        got = []
        for c in (full, part):
            torch.cuda.synchronize()
            b = qpack.FieldSectionDecoder(codec=c, dtable0=True).decode_blocks_dev(d_src, d_blk)
            c.sync()
            torch.cuda.synchronize()
            ns, nl = int(b["nspans"]), int(b["nlines"])
            got.append((b["strs"][:ns].cpu().numpy().tobytes(), b["spans"][:ns].cpu().numpy().tobytes(),
                        b["lines"][:nl * 24].cpu().numpy().tobytes(), b["verdict"][:ns].cpu().numpy().tobytes(),
                        b["status"][:20000].cpu().numpy().tobytes(), ns, nl))
        assert got[0][5] > 0 and got[0] == got[1]
        # the host-memory decode: on the full-chip context its pipeline runs
        # on the context's own streams, on the CU-masked one it stays on the
        # caller's stream (decode_host_impl); both give the corpus back
        enc, eoff, elen = corpus["enc"], corpus["enc_off"], corpus["enc_len"]
        sp_h = np.zeros(len(elen), dtype=q.SPAN_IN_DTYPE)
        sp_h["off"], sp_h["len"] = eoff, elen
        outs = []
        for c in (full, part):
            dst_h, out_h = c.decode_host(enc, sp_h)
            assert (out_h["status"] == 0).all() and (out_h["len"] == corpus["len"]).all()
            outs.append(b"".join(dst_h[o:o + n_].tobytes() for o, n_ in
                                 zip(out_h["off"].astype(np.int64), out_h["len"].astype(np.int64))))
        want = b"".join(corpus["plain"][o:o + n_].tobytes() for o, n_ in
                        zip(corpus["off"].astype(np.int64), corpus["len"].astype(np.int64)))
        assert outs[0] == outs[1] == want
    finally:
        part.close()
        full.close()
        hip.hipStreamDestroy(stream)
