#!/usr/bin/env python3
"""Generate the QPACK Huffman code table and 4-bit decode FSM for the engine.

Product-side generator (not the oracle).  It rebuilds, from the RFC 7541
Appendix B code *lengths* alone, the two tables that nghttp3 ships as
generated C data:

* ``huffman_sym_table[257]``  -- lib/nghttp3_qpack_huffman_data.c:30-96
  ({u32 nbits, u32 code}, code MSB-aligned in 32 bits: the reference's
  mkhufftbl.py:444 shifts ``k << (32 - nbits)``).
* ``qpack_huffman_decode_table[257][16]`` -- lib/nghttp3_qpack_huffman_data.c:98-4982
  ({u16 fstate, u8 flags, u8 sym}); flags per lib/nghttp3_qpack_huffman.h:51,54.

Construction (our own, not a transliteration of mkhufftbl.py):

1. RFC 7541's code is canonical (codes assigned in (length, symbol) order),
   so the 257 lengths determine every code word.
2. A binary trie is built from the code words.  Internal nodes are numbered
   in depth-first pre-order, 0-branch first; that numbering is the state id
   the reference FSM uses (huffman.h:56-63: 256 internal nodes, 0 = root).
3. A node is "accepting" when its path from the root is all ones and at
   most 7 bits long (a legal EOS-prefix padding, RFC 7541 5.2).
4. For each state and each nibble the 4 bits are walked; reaching a leaf
   emits its symbol and restarts at the root; reaching EOS sends the FSM
   to the absorbing failure state 256 with no flags.

Usage: ``python gen_tables.py [OUT_HEADER]`` (default: ../csrc/qh_tables.h).
"""
from __future__ import annotations

import os
import sys

# RFC 7541 Appendix B: code length in bits of each symbol 0..255 and EOS (256).
RFC7541_CODE_LENGTHS = (
    13, 23, 28, 28, 28, 28, 28, 28, 28, 24, 30, 28, 28, 30, 28, 28,
    28, 28, 28, 28, 28, 28, 30, 28, 28, 28, 28, 28, 28, 28, 28, 28,
    6, 10, 10, 12, 13, 6, 8, 11, 10, 10, 8, 11, 8, 6, 6, 6,
    5, 5, 5, 6, 6, 6, 6, 6, 6, 6, 7, 8, 15, 6, 12, 10,
    13, 6, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7,
    7, 7, 7, 7, 7, 7, 7, 7, 8, 7, 8, 13, 19, 13, 14, 6,
    15, 5, 6, 5, 6, 5, 6, 6, 6, 5, 7, 7, 6, 6, 6, 5,
    6, 7, 6, 5, 5, 6, 7, 7, 7, 7, 7, 15, 11, 14, 13, 28,
    20, 22, 20, 20, 22, 22, 22, 23, 22, 23, 23, 23, 23, 23, 24, 23,
    24, 24, 22, 23, 24, 23, 23, 23, 23, 21, 22, 23, 22, 23, 23, 24,
    22, 21, 20, 22, 22, 23, 23, 21, 23, 22, 22, 24, 21, 22, 23, 23,
    21, 21, 22, 21, 23, 22, 23, 23, 20, 22, 22, 22, 23, 22, 22, 23,
    26, 26, 20, 19, 22, 23, 22, 25, 26, 26, 26, 27, 27, 26, 24, 25,
    19, 21, 26, 27, 27, 26, 27, 24, 21, 21, 26, 26, 28, 27, 27, 27,
    20, 24, 20, 21, 22, 21, 21, 23, 22, 22, 25, 25, 24, 24, 26, 23,
    26, 27, 26, 26, 27, 27, 27, 27, 27, 28, 27, 27, 27, 27, 27, 26,
    30,
)

EOS = 256
FAIL_STATE = 256
FLAG_ACCEPTED = 0x01  # lib/nghttp3_qpack_huffman.h:51
FLAG_SYM = 0x02  # lib/nghttp3_qpack_huffman.h:54


def canonical_codes(lengths=RFC7541_CODE_LENGTHS):
    """Return [(nbits, code_lsb_aligned)] for the 257 symbols."""
    order = sorted(range(len(lengths)), key=lambda s: (lengths[s], s))
    codes = [None] * len(lengths)
    code = 0
    prev = lengths[order[0]]
    for rank, s in enumerate(order):
        if rank:
            code = (code + 1) << (lengths[s] - prev)
        prev = lengths[s]
        codes[s] = (lengths[s], code)
    return codes


def sym_table():
    """[(nbits, code MSB-aligned in 32 bits)] exactly as huffman_sym_table[]."""
    return [(n, (c << (32 - n)) & 0xFFFFFFFF) for n, c in canonical_codes()]


class _Trie:
    """Flat trie: child[node][bit] -> node, leaf[node] -> symbol or -1."""

    def __init__(self):
        self.child = [[-1, -1]]
        self.leaf = [-1]

    def insert(self, sym, nbits, code):
        node = 0
        for i in range(nbits - 1, -1, -1):
            b = (code >> i) & 1
            if self.child[node][b] < 0:
                self.child[node][b] = len(self.child)
                self.child.append([-1, -1])
                self.leaf.append(-1)
            node = self.child[node][b]
        self.leaf[node] = sym


def decode_fsm():
    """Return the 257 x 16 decode table as rows of (fstate, flags, sym)."""
    trie = _Trie()
    for s, (n, c) in enumerate(canonical_codes()):
        trie.insert(s, n, c)

    # Pre-order numbering of internal nodes (0-branch first) with an explicit
    # stack; remember each internal node's path to decide acceptance.
    state_of = {}
    accepting = {}
    stack = [(0, 0, 1)]  # (node, depth, path_is_all_ones)
    while stack:
        node, depth, ones = stack.pop()
        if trie.leaf[node] >= 0:
            continue
        state_of[node] = len(state_of)
        accepting[node] = bool(ones) and depth <= 7
        left, right = trie.child[node]
        # push right first so the 0-branch is numbered first
        stack.append((right, depth + 1, ones))
        stack.append((left, depth + 1, 0))
    assert len(state_of) == 256, len(state_of)

    node_of = {v: k for k, v in state_of.items()}
    rows = []
    for st in range(256):
        start = node_of[st]
        row = []
        for nib in range(16):
            node = start
            sym = None
            failed = False
            ended_on_leaf = False
            for i in (3, 2, 1, 0):
                node = trie.child[node][(nib >> i) & 1]
                ended_on_leaf = False
                if trie.leaf[node] >= 0:
                    leaf_sym = trie.leaf[node]
                    if leaf_sym == EOS:
                        failed = True
                    else:
                        assert sym is None  # shortest code is 5 bits > 4
                        sym = leaf_sym
                    node = 0
                    ended_on_leaf = True
            if failed:
                row.append((FAIL_STATE, 0, 0))
                continue
            flags = 0
            if sym is not None:
                flags |= FLAG_SYM
            if ended_on_leaf or accepting[node]:
                flags |= FLAG_ACCEPTED
            target = 0 if ended_on_leaf else state_of[node]
            row.append((target, flags, sym if sym is not None else 0))
        rows.append(row)
    rows.append([(FAIL_STATE, 0, 0)] * 16)
    return rows


def packed_fsm():
    """Rows as little-endian u32 words: fstate | flags << 16 | sym << 24.

    This is the in-memory image of nghttp3_qpack_huffman_decode_node
    ({u16 fstate, u8 flags, u8 sym}) on a little-endian host.
    """
    return [[f | (fl << 16) | (s << 24) for f, fl, s in row] for row in decode_fsm()]


# ---------------------------------------------------------------------------
# Symbol-level decode tables (the batch decoder, qh_lane_dec.inc).  They are a
# different *layout* of the same code: canonical_codes() is their only input,
# and tests/test_lut_model.py checks a model of the decoder that uses them
# against the oracle.
# ---------------------------------------------------------------------------

LUT_BITS = 12


def lut12():
    """4096 words indexed by the next 12 bits of input (MSB first).

    word = consumed | nsym << 8 | sym1 << 16 | sym2 << 24, where the window
    starts with sym1's code and, if it also fits, sym2's code (consumed = the
    bits of both).  nsym = 0 (word 0) marks the 4 windows that start a code
    longer than 12 bits (all such codes begin with ten 1-bits)."""
    dec = {}
    for s, (n, c) in enumerate(canonical_codes()):
        if n <= LUT_BITS:
            dec[(n, c)] = s

    def first(bits, avail):  # bits: `avail`-bit integer, MSB first
        for n in range(1, avail + 1):
            s = dec.get((n, bits >> (avail - n)))
            if s is not None:
                return s, n
        return None

    out = []
    for i in range(1 << LUT_BITS):
        r1 = first(i, LUT_BITS)
        if r1 is None:
            out.append(0)
            continue
        s1, n1 = r1
        rest = LUT_BITS - n1
        r2 = first(i & ((1 << rest) - 1), rest) if rest else None
        if r2 is None:
            out.append(n1 | 1 << 8 | s1 << 16)
        else:
            s2, n2 = r2
            out.append((n1 + n2) | 2 << 8 | s1 << 16 | s2 << 24)
    return out


def canonical_slow():
    """Canonical decoding of any code from a left-aligned 32-bit window w.

    Returns (lengths, lim, first_aligned, rank, lsym): for the k-th present
    code length L = lengths[k], lim[k] = (last code of length L + 1) <<
    (32 - L) (exclusive upper bound of those codes, left-aligned; the last
    one is 2**32), first_aligned[k] = first code << (32 - L), rank[k] = number
    of symbols with shorter codes, and lsym = symbols in canonical order.
    Decoding: k = #{j : w >= lim[j]}; L = lengths[k];
    sym = lsym[rank[k] + ((w - first_aligned[k]) >> (32 - L))]."""
    codes = canonical_codes()
    lengths = sorted(set(n for n, _ in codes))
    lsym = sorted(range(len(codes)), key=lambda s: (codes[s][0], s))
    lim, fa, rank = [], [], []
    r = 0
    for L in lengths:
        syms = [s for s in lsym if codes[s][0] == L]
        cs = [codes[s][1] for s in syms]
        assert cs == list(range(cs[0], cs[0] + len(cs)))
        fa.append(cs[0] << (32 - L))
        lim.append((cs[-1] + 1) << (32 - L))
        rank.append(r)
        r += len(syms)
    return lengths, lim, fa, rank, lsym


def render_header():
    out = []
    w = out.append
    w("/* Generated by nghttp3_amd/tools/gen_tables.py -- do not edit.")
    w(" *")
    w(" * QPACK (RFC 9204) / HPACK (RFC 7541 Appendix B) Huffman tables as")
    w(" * X-macro lists, expanded by the users into whatever layout they need:")
    w(" *   QH_SYM_LIST(X)    X(nbits, code) for symbols 0..256 (256 = EOS);")
    w(" *                     code is MSB-aligned in 32 bits.")
    w(" *   QH_FSM_ROWS(R, X) R(X(word) ... 16 words) for each of the 257 FSM")
    w(" *                     states; word = fstate | flags << 16 | sym << 24")
    w(" *                     (the little-endian image of {u16 fstate,")
    w(" *                     u8 flags, u8 sym}).")
    w(" * Contents equal nghttp3's lib/nghttp3_qpack_huffman_data.c:30-96 and")
    w(" * :98-4982; tests/test_tables.py pins them to the reference.")
    w(" */")
    w("#ifndef QH_TABLES_H")
    w("#define QH_TABLES_H")
    w("")
    w("#define QH_NSYM 257")
    w("#define QH_NSTATE 257")
    w("#define QH_FAIL_STATE 256")
    w("#define QH_FLAG_ACCEPTED 0x01u")
    w("#define QH_FLAG_SYM 0x02u")
    w("")
    w("#define QH_SYM_LIST(X) \\")
    syms = sym_table()
    for i in range(0, len(syms), 4):
        w("  " + " ".join("X(%d, 0x%08Xu)" % e for e in syms[i:i + 4]) + " \\")
    w("")
    w("")
    w("#define QH_FSM_ROWS(R, X) \\")
    for st, row in enumerate(packed_fsm()):
        items = ["X(0x%08Xu)" % x for x in row]
        w("  R(" + " ".join(items[:8]) + " \\")
        w("    " + " ".join(items[8:]) + ") \\")
    w("")
    w("")
    w("/* Symbol-level decode tables (gen_tables.py lut12 / canonical_slow):")
    w(" *   QH_LUT12_LIST(X)  X(word) for the 4096 12-bit windows;")
    w(" *   QH_SLOW_LIST(X)   X(lim, first_aligned, length, rank) per present")
    w(" *                     code length, shortest first (lim of the last = 0,")
    w(" *                     i.e. 2**32 truncated: never compared);")
    w(" *   QH_LSYM_LIST(X)   X(sym) for the 257 symbols in canonical order. */")
    w("#define QH_LUT12_BITS %d" % LUT_BITS)
    w("#define QH_LUT12_LIST(X) \\")
    lut = lut12()
    for i in range(0, len(lut), 8):
        w("  " + " ".join("X(0x%08Xu)" % x for x in lut[i:i + 8]) + " \\")
    w("")
    lengths, lim, fa, rank, lsym = canonical_slow()
    w("#define QH_SLOW_NLEN %d" % len(lengths))
    w("#define QH_SLOW_LIST(X) \\")
    for k in range(len(lengths)):
        w("  X(0x%08Xu, 0x%08Xu, %d, %d) \\" % (lim[k] & 0xFFFFFFFF, fa[k], lengths[k], rank[k]))
    w("")
    w("#define QH_LSYM_LIST(X) \\")
    for i in range(0, len(lsym), 16):
        w("  " + " ".join("X(%d)" % x for x in lsym[i:i + 16]) + " \\")
    w("")
    w("")
    w("#endif /* QH_TABLES_H */")
    return "\n".join(out) + "\n"


def main(argv):
    here = os.path.dirname(os.path.abspath(__file__))
    dest = argv[1] if len(argv) > 1 else os.path.join(here, "..", "csrc", "qh_tables.h")
    text = render_header()
    with open(dest, "w") as f:
        f.write(text)
    print("wrote", os.path.normpath(dest))


if __name__ == "__main__":
    main(sys.argv)
