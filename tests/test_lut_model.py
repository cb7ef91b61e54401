"""CPU model of the batch decoder's symbol-level algorithm (qh_lane_dec.inc).

The HIP decoder reads 12-bit windows from a multi-symbol table
(gen_tables.lut12) and decodes codes longer than 12 bits, and the last bits
of a string, canonically (gen_tables.canonical_slow).  `lut_decode` below is
the same algorithm step for step (word appends, loop bounds, tail and padding
rule) in Python; these tests pin it to the oracle (the reference's nibble FSM,
lib/nghttp3_qpack_huffman.c:87-129) on the golden corpus, the corrupted
strings and the error fixtures, so a table or algorithm error shows up here on
the CPU before any GPU run.
"""
import numpy as np
import pytest

import oracle
from nghttp3_amd.tools import gen_tables as G

MASK64 = (1 << 64) - 1
LUT = G.lut12()
LENGTHS, LIM, FA, RANK, LSYM = G.canonical_slow()
FIRST_LONG = LENGTHS.index(13)


def _slow(w, k0):
    """Canonical decode of the code at the top of the 32-bit window w."""
    k = k0 + sum(1 for j in range(k0, len(LENGTHS) - 1) if w >= LIM[j])
    n = LENGTHS[k]
    return LSYM[RANK[k] + ((w - FA[k]) >> (32 - n))], n


def lut_decode(data):
    """(status, bytes): 0 and the decoded string, or -108 (QPACK fatal)."""
    rem = 8 * len(data)
    bb = nb = 0
    out = bytearray()
    nwords = (len(data) + 3) // 4
    padded = data + b"\0" * (4 * nwords - len(data))
    for wi in range(nwords):
        bb |= int.from_bytes(padded[4 * wi:4 * wi + 4], "big") << (32 - nb)
        nb += 32
        while nb >= 32 and rem >= 32:
            e = LUT[bb >> (64 - G.LUT_BITS)]
            if (e >> 8) & 0xFF == 0:  # code longer than 12 bits
                sym, n = _slow(bb >> 32, FIRST_LONG)
                if sym == G.EOS:
                    return -108, b""
                out.append(sym)
            else:
                out.append((e >> 16) & 0xFF)
                if (e >> 8) & 0xFF == 2:
                    out.append(e >> 24)
                n = e & 63
            bb = (bb << n) & MASK64
            nb -= n
            rem -= n
    while rem > 0:  # fewer than 32 bits left: canonical, one code at a time
        sym, n = _slow(bb >> 32, 0)
        if n > rem:
            break
        if sym == G.EOS:
            return -108, b""
        out.append(sym)
        bb = (bb << n) & MASK64
        rem -= n
    # padding: at most 7 bits, all ones (huffman.c:119-121 ACCEPTED states)
    if rem > 7 or (rem and (bb >> (64 - rem)) != (1 << rem) - 1):
        return -108, b""
    return 0, bytes(out)


def test_lut_covers_short_codes():
    codes = G.canonical_codes()
    for s, (n, c) in enumerate(codes):
        if n <= G.LUT_BITS:
            for tail in range(1 << (G.LUT_BITS - n)):
                e = LUT[(c << (G.LUT_BITS - n)) | tail]
                assert (e >> 16) & 0xFF == s and e & 63 >= n
    long_windows = [i for i, e in enumerate(LUT) if (e >> 8) & 0xFF == 0]
    assert long_windows == [0xFFC, 0xFFD, 0xFFE, 0xFFF]


def test_slow_path_every_code():
    for s, (n, c) in enumerate(G.canonical_codes()):
        for pad in (0, (1 << (32 - n)) - 1):
            assert _slow((c << (32 - n)) | pad, 0) == (s, n)
            if n > G.LUT_BITS:
                assert _slow((c << (32 - n)) | pad, FIRST_LONG) == (s, n)


def test_model_matches_oracle_corpus(corpus):
    enc, eoff, elen = corpus["enc"], corpus["enc_off"], corpus["enc_len"]
    plain, off, ln = corpus["plain"], corpus["off"], corpus["len"]
    for i in range(0, len(elen), 3):
        st, out = lut_decode(enc[eoff[i]:eoff[i] + elen[i]].tobytes())
        assert st == 0
        assert out == plain[off[i]:off[i] + ln[i]].tobytes()


def test_model_matches_oracle_corrupted(corpus):
    bad, boff, blen = corpus["bad"], corpus["bad_off"], corpus["bad_len"]
    bst, bout, bolen = corpus["bad_status"], corpus["bad_out"], corpus["bad_out_len"]
    ooff = np.concatenate([[0], np.cumsum(bolen.astype(np.int64))])
    for i in range(len(blen)):
        st, out = lut_decode(bad[boff[i]:boff[i] + blen[i]].tobytes())
        assert st == bst[i], i
        if st == 0:
            assert out == bout[ooff[i]:ooff[i + 1]].tobytes()


def test_model_error_fixtures(errors):
    for c in errors["whole"]:
        st, out = lut_decode(bytes.fromhex(c["hex"]))
        assert st == c["status"], c
        if st == 0:
            assert out.hex() == c["out_hex"]


def test_model_random_bytes():
    rng = np.random.default_rng(7)
    for _ in range(400):
        data = rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes()
        want = oracle.decode_one(data)
        assert lut_decode(data) == (want[0], want[1] if want[0] == 0 else b"")


@pytest.mark.parametrize("sym", [0, 1, 0x7F, 0xFE, 0xFF])
def test_model_long_codes(sym):
    s = bytes([sym]) * 9
    enc = oracle.encode(s)
    assert lut_decode(enc) == (0, s)
