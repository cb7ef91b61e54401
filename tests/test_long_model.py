"""Step-for-step Python restatement of the long-string decoder
(nghttp3_amd/csrc/qh_long_dec.inc: long_walk, the per-lane speculative walk
with its start mask, resolve, the segment chain), pinned to the oracle
(oracle/qh_oracle.c, huffman.c:87-124) on text, binary and corrupted
strings.  CPU only: it checks the algorithm, the GPU tests check the
kernel."""
import numpy as np
import pytest

import oracle

SEG = 64 * 128


def _codes():
    sym, _ = oracle.tables()
    table = {}
    for s in range(257):
        n, code = int(sym[s][0]), int(sym[s][1])
        table[(n, code >> (32 - n))] = s
    return table


_TABLE = None


class Bits:
    def __init__(self, enc: bytes):
        self.nbits = 8 * len(enc)
        # ones past the string (the decoder's padding feed)
        self.v = int.from_bytes(enc + b"\xff" * 16, "big")
        self.tot = 8 * (len(enc) + 16)

    def get(self, pos, n):
        return (self.v >> (self.tot - pos - n)) & ((1 << n) - 1)


def _code_at(b: Bits, pos):
    """utab_lookup: (length, symbol) of the code at pos; symbol 256 = EOS."""
    for n in range(5, 31):
        s = _TABLE.get((n, b.get(pos, n)))
        if s is not None:
            return n, s
    raise AssertionError("no code")


def long_walk(b, base, s, lim, mask, rec, sync):
    """-> (stop position, symbols, err, synced); mask: set of recorded starts."""
    syms = []
    pos = s
    while pos < lim:
        if sync and pos in mask:
            return pos, syms, False, True
        if rec:
            mask.add(pos)
        sleft = b.nbits - pos
        if sleft <= 7 and b.get(pos, sleft) == (1 << sleft) - 1:
            return b.nbits, syms, False, False
        cn, sym = _code_at(b, pos)
        if sym == 256 or cn > sleft:
            return pos, syms, True, False
        syms.append(sym)
        pos += cn
    return pos, syms, False, False


def long_decode_model(enc: bytes, trace=None):
    """-> (status, decoded bytes) as long_string_coop computes them; trace
    (a list) receives per segment (first-code start, decoded bytes, error so
    far, next start) as qh_debug_long reports them."""
    b = Bits(enc)
    nbits = b.nbits
    nseg = (nbits + SEG - 1) // SEG
    p0, out, bad = 0, bytearray(), False
    for k in range(nseg):
        lanes = []
        for lane in range(64):
            base = k * SEG + 128 * lane
            act = base < nbits
            lim = min(base + 128, nbits)
            mask = set()
            es, spec, ers, _ = long_walk(b, base, base, lim, mask, True, False) if act \
                else (base, [], False, False)
            lanes.append(dict(act=act, base=base, lim=lim, mask=mask, es=es, spec=spec, ers=ers,
                              sc=base, head=[], c=0, e=es, er=ers))

        def resolve(with0):
            while True:
                prev = [L["e"] for L in lanes]
                changed = False
                for j, L in enumerate(lanes):
                    t = p0 if j == 0 else prev[j - 1]
                    if not (L["act"] and (j > 0 or with0) and t != L["sc"]):
                        continue
                    changed = True
                    at, head, er2, sy = long_walk(b, L["base"], t, L["lim"], L["mask"], False, True)
                    L["sc"], L["head"] = t, head
                    if sy:
                        L["c"] = sum(1 for x in L["mask"] if x < at)
                        L["e"], L["er"] = L["es"], L["ers"]
                    else:
                        L["c"] = len(L["spec"])
                        L["e"], L["er"] = at, er2
                if not changed:
                    return

        resolve(False)
        resolve(True)
        if trace is not None and k == 0:
            trace.append([(L["sc"], len(L["head"]), L["c"], len(L["spec"]), L["e"], int(L["er"]),
                           int(L["ers"]), L["es"]) for L in lanes])
        T = 0
        for L in lanes:
            if L["act"]:
                seg = bytes(L["head"]) + bytes(L["spec"][L["c"]:])
                out += seg
                T += len(seg)
                bad = bad or L["er"]
        if trace is not None:
            trace.append((p0, T, int(bad), lanes[63]["e"]))
        p0 = lanes[63]["e"]
    return (-108, b"") if bad else (0, bytes(out))


@pytest.fixture(scope="module", autouse=True)
def table():
    global _TABLE
    _TABLE = _codes()


def _cases():
    from nghttp3_amd import synth
    rng = np.random.default_rng(0x5EED0413)
    out = []
    for n in (1, 700, 1025, 2048, 5000):
        out.append(synth.fill(int(rng.integers(1 << 62)), n, synth.ALPHABET_A).tobytes())
        out.append(rng.integers(0, 256, n // 3 + 1, dtype=np.uint8).tobytes())
        a = np.frombuffer(synth.fill(int(rng.integers(1 << 62)), n, synth.ALPHABET_A).tobytes(), np.uint8).copy()
        k = rng.choice(n, max(1, n // 20), replace=False)
        a[k] = rng.integers(0, 256, k.size)
        out.append(a.tobytes())
    return out


def test_model_matches_oracle_on_good_strings():
    for s in _cases():
        enc = oracle.encode(s)
        assert long_decode_model(enc) == (0, s)


def test_model_matches_oracle_on_corrupted_strings():
    rng = np.random.default_rng(0x5EED0414)
    for s in _cases():
        enc = oracle.encode(s)
        if len(enc) < 8:
            continue
        for kind in range(5):
            e = bytearray(enc)
            if kind == 0:
                m = int(rng.integers(0, len(e) - 4))
                e[m:m + 4] = b"\xff\xff\xff\xff"
            elif kind == 1:
                e[-1] = 0
            elif kind == 2:
                e += b"\xff"
            elif kind == 3:
                del e[-1]
            else:
                e[int(rng.integers(len(e)))] ^= 1 << int(rng.integers(8))
            st, dec = oracle.decode_one(bytes(e))
            assert long_decode_model(bytes(e)) == (st, dec if st == 0 else b""), kind
