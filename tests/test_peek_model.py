"""CPU model of the peek decoder (qh_peek_dec.inc), pinned to the oracle.

The HIP kernel looks the top W bits of a lane's 64-bit bit buffer up in a
2^W-entry table (one whole code of <= W bits per lookup), appends one 32-bit
word per group of 4 lookups when <= 32 bits are buffered, feeds 1-bits past
the end of the string, and sends escapes (codes > W bits, too few buffered
bits, the end of the string) to a careful path: refill, then the
end-of-string decision or canonical symbols (the first always, then while the
next code is not a short one, up to 16).  `peek_decode` is that
algorithm step for step; the tests compare it with the oracle (the
reference's nibble FSM, lib/nghttp3_qpack_huffman.c:87-129) on the golden
corpus, the corrupted strings, the error fixtures and random bytes, for every
window the kernel is built with.
"""
import numpy as np
import pytest

import oracle
from nghttp3_amd.tools import gen_tables as G

MASK64 = (1 << 64) - 1
ESC = 0xFF
LENGTHS, LIM, FA, RANK, LSYM = G.canonical_slow()


def peek_table(w):
    """entry = len | sym << 8 for codes of <= w bits, else ESC
    (qh_peek_dec.inc build_peek_table)."""
    tab = [ESC] * (1 << w)
    for sym, (nbits, code) in enumerate(G.sym_table()):
        if nbits > w:
            continue
        head = code >> (32 - w)
        for k in range(1 << (w - nbits)):
            tab[head | k] = nbits | (sym << 8)
    return tab


def _canonical(w32):
    k = sum(1 for j in range(len(LENGTHS) - 1) if w32 >= LIM[j])
    n = LENGTHS[k]
    return LSYM[RANK[k] + ((w32 - FA[k]) >> (32 - n))], n


def peek_decode(data, w, tab):
    """(status, bytes) as the kernel computes them."""
    total = 8 * len(data)
    nwords = (len(data) + 3) // 4
    padded = data + b"\xff" * (4 * nwords - len(data))
    words = [int.from_bytes(padded[4 * i:4 * i + 4], "big") for i in range(nwords)]
    st = {"bb": 0, "nb": 0, "refills": 0}

    def refill():
        if st["nb"] <= 32:
            i = st["refills"]
            word = words[i] if i < nwords else 0xFFFFFFFF
            st["bb"] |= word << (32 - st["nb"])
            st["nb"] += 32
            st["refills"] += 1

    out = bytearray()
    while True:
        for k in range(16):
            if k % 4 == 0:
                refill()
            e = tab[st["bb"] >> (64 - w)]
            if st["nb"] - (e & 0xFF) >= 0:
                n = e & 63
                st["bb"] = (st["bb"] << n) & MASK64
                st["nb"] -= n
                out.append(e >> 8)
                continue
            kc = 0  # careful path: canonical symbols while long codes follow
            while True:
                refill()
                sleft = total - (st["refills"] * 32 - st["nb"])
                if sleft <= 0:
                    return (0, bytes(out)) if sleft == 0 else (-108, b"")
                if sleft <= 7 and (st["bb"] >> (64 - sleft)) == (1 << sleft) - 1:
                    return 0, bytes(out)
                if kc:
                    e2 = tab[st["bb"] >> (64 - w)]
                    if e2 != ESC and st["nb"] - (e2 & 0xFF) >= 0:
                        break
                sym, n = _canonical(st["bb"] >> 32)
                if n > sleft or sym == G.EOS:
                    return -108, b""
                st["bb"] = (st["bb"] << n) & MASK64
                st["nb"] -= n
                out.append(sym)
                kc += 1
                if kc == 16:
                    break
            break


@pytest.fixture(scope="module", params=[10, 11, 12])
def window(request):
    return request.param, peek_table(request.param)


def _check(strs, window):
    w, tab = window
    for s in strs:
        want = oracle.decode_one(s)
        got = peek_decode(s, w, tab)
        if want[0] == 0:
            assert got == (0, want[1]), s.hex()
        else:
            assert got[0] == -108, s.hex()


def test_peek_table_covers_short_codes(window):
    w, tab = window
    for sym, (nbits, code) in enumerate(G.sym_table()):
        if nbits <= w:
            assert tab[code >> (32 - w)] == nbits | (sym << 8)
    assert tab[(1 << w) - 1] == ESC  # all ones: never a short code


def test_peek_model_corpus(window, corpus):
    enc, off, ln = corpus["enc"], corpus["enc_off"], corpus["enc_len"]
    _check([enc[o:o + n].tobytes() for o, n in zip(off[:600], ln[:600])], window)


def test_peek_model_corrupted(window, corpus):
    bad, off, ln = corpus["bad"], corpus["bad_off"], corpus["bad_len"]
    _check([bad[o:o + n].tobytes() for o, n in zip(off, ln)], window)


def test_peek_model_errors(window, errors):
    _check([bytes.fromhex(c["hex"]) for c in errors["whole"]], window)


def test_peek_model_random(window):
    rng = np.random.default_rng(5)
    _check([bytes(rng.integers(0, 256, int(rng.integers(0, 40))).astype(np.uint8))
            for _ in range(1500)], window)
