"""The oracle against the reference's own pins: RFC 7541 vectors, the
verdicts of lib/nghttp3_qpack_huffman.c, and tests/nghttp3_qpack_test.c:856-899."""
import numpy as np
import pytest

import oracle
from nghttp3_amd import synth


def test_rfc7541_kat(kat):
    for v in kat:
        plain, h = v["plain"].encode(), v["huffman_hex"]
        assert oracle.encode_count(plain) == len(h) // 2
        assert oracle.encode(plain).hex() == h
        assert oracle.decode_one(bytes.fromhex(h)) == (0, plain)


def test_error_verdicts(errors):
    for case in errors["whole"]:
        c = oracle.new_ctx()
        r = oracle.decode(c, bytes.fromhex(case["hex"]), True)
        got = r if isinstance(r, int) else len(r)
        assert got == case["ret"], case
        assert oracle.failure_state(c) == case["failure_state"], case
        assert oracle.decode_one(bytes.fromhex(case["hex"]))[0] == case["status"]


def test_failure_state_streaming(errors):
    # tests/nghttp3_qpack_test.c:883-899: {FF FF FF} fin=0 -> 0 bytes, no
    # failure; one more FF (EOS complete) -> 0 bytes, failure state 0x100.
    s = errors["stream"]
    c = oracle.new_ctx()
    for chunk, fin, ret, fail in zip(s["chunks"], s["fin"], s["ret"], s["failure_state"]):
        r = oracle.decode(c, bytes.fromhex(chunk), bool(fin))
        assert (r if isinstance(r, int) else len(r)) == ret
        assert oracle.failure_state(c) == fail
    assert c.fstate == 0x100


def test_random_roundtrip_like_reference():
    # tests/nghttp3_qpack_test.c:856-881 encodes 100,000 random 100-byte
    # strings and decodes them with fin=1.  glibc rand() is not portable, so
    # the bytes come from splitmix64 (all 256 values).
    n = 100_000
    plain = synth.fill(1000000007, n * 100, synth.ALPHABET_U)
    off = np.arange(n, dtype=np.uint64) * 100
    ln = np.full(n, 100, dtype=np.uint32)
    enc, eoff, elen = oracle.encode_batch(plain, off, ln)
    dst, slot, olen, st = oracle.decode_batch(enc, eoff, elen)
    assert (st == 0).all() and (olen == 100).all()
    dec = dst.reshape(-1)[(slot[:, None] + np.arange(100, dtype=np.uint64)).reshape(-1).astype(np.int64)]
    assert (dec == plain).all()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_streaming_split_points_equal_one_shot(corpus, seed):
    # decoding in k chunks (fin only on the last) == one shot.
    rng = np.random.default_rng(seed)
    enc, eoff, elen = corpus["enc"], corpus["enc_off"], corpus["enc_len"]
    for i in rng.integers(0, elen.size, 300):
        e = enc[int(eoff[i]):int(eoff[i]) + int(elen[i])].tobytes()
        want = oracle.decode_one(e)
        k = int(rng.integers(1, 6))
        cuts = sorted(int(x) for x in rng.integers(0, len(e) + 1, k - 1))
        parts = [e[a:b] for a, b in zip([0] + cuts, cuts + [len(e)])]
        c = oracle.new_ctx()
        got = b""
        status = 0
        for j, part in enumerate(parts):
            r = oracle.decode(c, part, j == len(parts) - 1)
            if isinstance(r, int) or oracle.failure_state(c):
                status = -108
                break
            got += r
        assert (status, got if status == 0 else b"") == want


def test_corpus_roundtrip(corpus):
    plain, off, ln = corpus["plain"], corpus["off"], corpus["len"]
    enc, eoff, elen = oracle.encode_batch(plain, off, ln)
    assert (enc == corpus["enc"]).all() and (elen == corpus["enc_len"]).all()
    dst, slot, olen, st = oracle.decode_batch(enc, eoff, elen)
    assert (st == 0).all() and (olen == ln).all()
    for i in range(0, ln.size, 37):
        a = dst[int(slot[i]):int(slot[i]) + int(olen[i])]
        b = plain[int(off[i]):int(off[i]) + int(ln[i])]
        assert (a == b).all()


def test_corrupted_corpus_statuses(corpus):
    bad, boff, blen = corpus["bad"], corpus["bad_off"], corpus["bad_len"]
    dst, slot, olen, st = oracle.decode_batch(bad, boff, blen)
    assert (st == corpus["bad_status"]).all()
    assert (olen == corpus["bad_out_len"]).all()


def test_cpu_baseline_pool_verifies_and_calibrates(corpus):
    """The bench's CPU leg: pinned pool, barrier-to-barrier passes, passes
    repeated until a thread works >= min_seconds, verification untimed."""
    import os
    plain, off, ln = corpus["plain"], corpus["off"], corpus["len"]
    cpus = sorted(os.sched_getaffinity(0))[:2]
    e, d, ok, inner = oracle.bench_roundtrip(plain, off, ln, len(cpus), 3, cpus=cpus,
                                             min_seconds=0.01)
    assert ok and len(e) == len(d) == 3
    assert all(x > 0 for x in e + d) and min(inner) >= 1
