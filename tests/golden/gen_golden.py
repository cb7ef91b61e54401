#!/usr/bin/env python3
"""Regenerate the committed fixtures under tests/golden/.

Run in the build container (needs /root/reference for tables.json only):

    python tests/golden/gen_golden.py

Fixtures (all data, no reference source text):

* tables.json  -- SHA-256 of the reference's generated tables
  (lib/nghttp3_qpack_huffman_data.c:30-96 and :98-4982, parsed from the
  reference file as text) in a canonical binary form: sym = uint32 LE
  [257][2] {nbits, code}; fsm = uint32 LE [257][16] words
  fstate | flags << 16 | sym << 24.
* kat.json     -- RFC 7541 Appendix C.4 / C.6 Huffman known answers
  (published vectors; the survey also reproduced them with the compiled
  reference).
* errors.json  -- invalid / edge encodings with the verdict
  nghttp3_qpack_huffman_decode(fin=1) + failure_state give, and the
  streaming case of tests/nghttp3_qpack_test.c:883-899.  Produced by the
  oracle (pinned by the two fixtures above).
* corpus.npz   -- ~4k mixed strings (edge lengths, alphabets A / U / digits,
  all 256 byte values) with oracle encodings, plus corrupted encodings with
  their statuses.  np.savez, no pickled objects.
* digests.json -- SHA-256 of the plaintext and of the dense oracle encodings
  of the full-size synthetic configs, for size-independent
  parity on the GPU box.
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from nghttp3_amd import synth  # noqa: E402

REF_DATA = "/root/reference/lib/nghttp3_qpack_huffman_data.c"


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def reference_tables():
    """Parse the reference's generated table file (as text)."""
    txt = open(REF_DATA).read()
    sym_txt = txt.split("huffman_sym_table[] = {")[1].split("};")[0]
    sym = np.array([(int(a), int(b, 16)) for a, b in
                    re.findall(r"\{(\d+),\s*0x([0-9A-Fa-f]+)U\}", sym_txt)], dtype=np.uint32)
    fsm_txt = txt.split("qpack_huffman_decode_table[][16] = {")[1]
    ent = re.findall(r"\{0x([0-9A-Fa-f]+),\s*0x([0-9A-Fa-f]+),\s*0x([0-9A-Fa-f]+)\}", fsm_txt)
    fsm = np.array([int(a, 16) | (int(b, 16) << 16) | (int(c, 16) << 24) for a, b, c in ent],
                   dtype=np.uint32).reshape(257, 16)
    assert sym.shape == (257, 2) and fsm.shape == (257, 16)
    return sym, fsm


# RFC 7541 Appendix C.4 (requests) and C.6 (responses), Huffman-coded literals.
RFC7541_KAT = [
    ("www.example.com", "f1e3c2e5f23a6ba0ab90f4ff"),
    ("no-cache", "a8eb10649cbf"),
    ("custom-key", "25a849e95ba97d7f"),
    ("custom-value", "25a849e95bb8e8b4bf"),
    ("302", "6402"),
    ("307", "640eff"),
    ("private", "aec3771a4b"),
    ("Mon, 21 Oct 2013 20:13:21 GMT", "d07abe941054d444a8200595040b8166e082a62d1bff"),
    ("Mon, 21 Oct 2013 20:13:22 GMT", "d07abe941054d444a8200595040b8166e084a62d1bff"),
    ("https://www.example.com", "9d29ad171863c78f0b97c8e9ae82ae43d3"),
    ("gzip", "9bd9ab"),
    ("foo=ASDJKHQKBZXOQWEOPIUAXQWEOIU; max-age=3600; version=1",
     "94e7821dd7f2e6c7b335dfdfcd5b3960d5af27087f3672c1ab270fb5291f9587316065c003ed4ee5b1063d5007"),
    ("", ""),
]


def gen_tables(out):
    if not os.path.exists(REF_DATA):
        print("reference absent: keeping existing tables.json")
        return
    sym, fsm = reference_tables()
    osym, ofsm = oracle.tables()
    assert (sym == osym).all() and (fsm == ofsm).all(), "oracle tables differ from reference"
    json.dump({"source": "lib/nghttp3_qpack_huffman_data.c:30-96,98-4982 (parsed as text)",
               "layout": "sym uint32le[257][2]{nbits,code}; fsm uint32le[257][16] "
                         "fstate|flags<<16|sym<<24",
               "sym_sha256": sha(sym), "fsm_sha256": sha(fsm)}, out, indent=1)


def gen_kat(out):
    for s, h in RFC7541_KAT:
        assert oracle.encode(s.encode()).hex() == h, s
        st, d = oracle.decode_one(bytes.fromhex(h))
        assert st == 0 and d == s.encode()
    json.dump({"source": "RFC 7541 Appendix C.4 and C.6",
               "vectors": [{"plain": s, "huffman_hex": h} for s, h in RFC7541_KAT]}, out, indent=1)


def gen_errors(out):
    cases = []
    # whole-string cases (fin = 1)
    whole = ["ffffffff", "1fff", "00", "fe", "ff", "fffe", "ffff", "fffffffc", "3fffffff",
             "7f", "f8", "07", "1f", "9bd9", "9bd9ab", "9bd9abff", "a8eb10649cbf00",
             "a8eb10649cbf", "25a849e95ba97d7fff"]
    for h in whole:
        c = oracle.new_ctx()
        r = oracle.decode(c, bytes.fromhex(h), True)
        cases.append({"hex": h, "ret": r if isinstance(r, int) else len(r),
                      "out_hex": "" if isinstance(r, int) else r.hex(),
                      "failure_state": oracle.failure_state(c),
                      "status": oracle.decode_one(bytes.fromhex(h))[0]})
    # streaming: tests/nghttp3_qpack_test.c:883-899
    c = oracle.new_ctx()
    r1 = oracle.decode(c, bytes.fromhex("ffffff"), False)
    f1 = oracle.failure_state(c)
    r2 = oracle.decode(c, bytes.fromhex("ff"), False)
    f2 = oracle.failure_state(c)
    stream = {"chunks": ["ffffff", "ff"], "fin": [0, 0],
              "ret": [len(r1) if not isinstance(r1, int) else r1,
                      len(r2) if not isinstance(r2, int) else r2],
              "failure_state": [f1, f2], "fstate_after": c.fstate}
    assert stream["ret"] == [0, 0] and stream["failure_state"] == [False, True]
    assert c.fstate == 0x100
    json.dump({"source": "oracle (restates lib/nghttp3_qpack_huffman.c:87-129); streaming case "
                         "mirrors tests/nghttp3_qpack_test.c:883-899",
               "whole": cases, "stream": stream}, out, indent=1)


def corpus_strings(rng):
    strs = []
    # edge lengths around the 16-byte fetch width and the 4-byte store width
    for n in list(range(0, 40)) + [63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 1000, 4096, 5000]:
        for alph in (synth.ALPHABET_A, synth.ALPHABET_U, b"0123456789"):
            a = np.frombuffer(alph, dtype=np.uint8)
            strs.append(a[rng.integers(0, a.size, n)].tobytes())
    # every byte value, singles and runs
    for b in range(256):
        strs.append(bytes([b]))
        strs.append(bytes([b]) * 7)
    strs.append(bytes(range(256)))
    strs.append(bytes(range(255, -1, -1)))
    # random mix
    while len(strs) < 4096:
        n = int(rng.integers(0, 300))
        alph = [synth.ALPHABET_A, synth.ALPHABET_U, b"abc"][int(rng.integers(0, 3))]
        a = np.frombuffer(alph, dtype=np.uint8)
        strs.append(a[rng.integers(0, a.size, n)].tobytes())
    return strs


def corrupt(enc: bytes, kind: int, rng) -> bytes:
    if not enc:
        return b"\x00"
    b = bytearray(enc)
    if kind == 0:      # EOS injected (30 ones) in the middle
        i = int(rng.integers(0, len(b)))
        b[i:i] = b"\xff\xff\xff\xff"
    elif kind == 1:    # zero padding: clear the last byte's low bits
        b[-1] &= 0x00
    elif kind == 2:    # truncation
        b = b[: max(0, len(b) - 1 - int(rng.integers(0, 3)))]
    elif kind == 3:    # > 7 bits of padding
        b += b"\xff"
    else:              # random bit flips
        for _ in range(3):
            i = int(rng.integers(0, len(b)))
            b[i] ^= 1 << int(rng.integers(0, 8))
    return bytes(b)


def gen_corpus(path):
    rng = np.random.default_rng(0x5EED00C0)
    strs = corpus_strings(rng)
    plain = np.frombuffer(b"".join(strs) or b"\0", dtype=np.uint8)
    ln = np.array([len(s) for s in strs], dtype=np.uint32)
    off = np.zeros(len(strs), dtype=np.uint64)
    off[1:] = np.cumsum(ln.astype(np.uint64))[:-1]
    enc, eoff, elen = oracle.encode_batch(plain, off, ln)
    # corrupted encodings
    bad = []
    for i in range(1024):
        s = strs[int(rng.integers(0, len(strs)))]
        bad.append(corrupt(oracle.encode(s), i % 5, rng))
    bad_cat = np.frombuffer(b"".join(bad) or b"\0", dtype=np.uint8)
    bad_len = np.array([len(x) for x in bad], dtype=np.uint32)
    bad_off = np.zeros(len(bad), dtype=np.uint64)
    bad_off[1:] = np.cumsum(bad_len.astype(np.uint64))[:-1]
    bad_status = np.array([oracle.decode_one(x)[0] for x in bad], dtype=np.int32)
    bad_out = [oracle.decode_one(x)[1] for x in bad]
    bad_out_len = np.array([len(x) for x in bad_out], dtype=np.uint32)
    np.savez_compressed(path, plain=plain, off=off, len=ln, enc=enc, enc_off=eoff, enc_len=elen,
                        bad=bad_cat, bad_off=bad_off, bad_len=bad_len, bad_status=bad_status,
                        bad_out=np.frombuffer(b"".join(bad_out) or b"\0", dtype=np.uint8),
                        bad_out_len=bad_out_len)
    print("corpus:", len(strs), "strings,", int((bad_status != 0).sum()), "of 1024 corrupted fail")


# full-size synthetic configs; config 5 is generated per shard
FULL_CONFIGS = {
    "c2_A": dict(seed=synth.SEEDS[2], n=1 << 20, lo=8, hi=256, alphabet="A"),
    "c2_U": dict(seed=synth.SEEDS[2], n=1 << 20, lo=8, hi=256, alphabet="U"),
    "c3_A": dict(seed=synth.SEEDS[3], n=1 << 20, lo=8, hi=256, alphabet="A"),
}


def alphabet(name):
    return {"A": synth.ALPHABET_A, "U": synth.ALPHABET_U}[name]


def gen_digests(out):
    res = {}
    for name, cfg in FULL_CONFIGS.items():
        plain, off, ln = synth.batch(cfg["seed"], cfg["n"], cfg["lo"], cfg["hi"],
                                     alphabet(cfg["alphabet"]))
        enc, eoff, elen = oracle.encode_batch(plain, off, ln)
        res[name] = dict(cfg, plain_bytes=int(plain.size), enc_bytes=int(enc.size),
                         plain_sha256=sha(plain), len_sha256=sha(ln),
                         enc_sha256=sha(enc), enc_len_sha256=sha(elen))
        print(name, res[name]["plain_bytes"], res[name]["enc_bytes"])
    json.dump({"source": "oracle encodings of nghttp3_amd.synth batches", "configs": res},
              out, indent=1)


# config 5 (16M Zipf strings over 8 GPUs): one rank's shard, as bench.py
# cuts it; config 4: the whole 65,536-block corpus through the oracle
C5 = dict(seed=synth.SEEDS[5], n_total=16 << 20, lo=1, hi=4096, s=1.2, world=8, rank=0,
          alphabet="A")
C4 = dict(seed=synth.SEEDS[4], nblocks=65536, dtable0=True)


def gen_c5_shard():
    from nghttp3_amd import shard
    c = C5
    ln = synth.zipf_lengths(c["seed"], c["n_total"], c["lo"], c["hi"], c["s"])
    b, e = shard.split_by_bytes(ln, c["world"])[c["rank"]]
    first = int(ln[:b].sum(dtype=np.uint64))
    my = ln[b:e]
    plain = synth.fill(c["seed"], int(my.sum(dtype=np.uint64)), alphabet(c["alphabet"]), first=first)
    off = np.zeros(my.size, dtype=np.uint64)
    off[1:] = np.cumsum(my.astype(np.uint64))[:-1]
    enc, eoff, elen = oracle.encode_batch(plain, off, my)
    r = dict(c, begin=int(b), end=int(e), first=first, plain_bytes=int(plain.size),
             enc_bytes=int(enc.size), len_sha256=sha(my), plain_sha256=sha(plain),
             enc_sha256=sha(enc), enc_len_sha256=sha(elen))
    print("c5 shard", r["end"] - r["begin"], r["plain_bytes"], r["enc_bytes"])
    return r


def gen_c4_blocks():
    """Block bytes from the product writer (pinned by the oracle writers in
    tests/test_qpack.py); expected outputs from the oracle: every string
    decoded in span order (oracle/qpack_frame.decode_field_section), its
    verdict (oracle/http_check with the reference's tables) and a name's
    token (the reference's enum)."""
    from oracle import http_check, qpack_frame
    from nghttp3_amd import qpack
    chars = json.load(open(os.path.join(HERE, "http_chars.json")))
    tokens = json.load(open(os.path.join(HERE, "tokens.json")))["tokens"]
    src, blocks, plain, strs, lines, ls = qpack.synth_field_sections(C4["seed"], C4["nblocks"])
    data = bytes(src)
    out, verdict, token = [], [], []
    nlines = 0
    for b in range(blocks.size):
        o, n = int(blocks["off"][b]), int(blocks["len"][b])
        st, rl, rs, rstr = qpack_frame.decode_field_section(data[o:o + n], o, C4["dtable0"])
        assert st == 0
        nlines += len(rl)
        for (so, sn, fl), v in zip(rs, rstr):
            out.append(v)
            if fl & qpack_frame.SPAN_NAME:
                verdict.append(http_check.check_header_name(v, chars["VALID_HD_NAME_CHARS"]))
                token.append(http_check.lookup_token(v, tokens))
            else:
                verdict.append(http_check.check_header_value(v, chars["VALID_HD_VALUE_CHARS"]))
                token.append(-1)
    strings = b"".join(out)
    r = dict(C4, block_bytes=int(src.size), blocks_sha256=sha(src), field_lines=nlines,
             strings=len(out), string_bytes=len(strings),
             strings_sha256=hashlib.sha256(strings).hexdigest(),
             verdict_sha256=sha(np.array(verdict, dtype=np.int8)),
             token_sha256=sha(np.array(token, dtype=np.int32)))
    print("c4", r["strings"], r["string_bytes"], r["field_lines"])
    return r


def update_digests(keys):
    path = os.path.join(HERE, "digests.json")
    d = json.load(open(path))
    if "c5_r0of8" in keys:
        d["configs"]["c5_r0of8"] = gen_c5_shard()
    if "c4_blocks" in keys:
        d["configs"]["c4_blocks"] = gen_c4_blocks()
    d["source"] = "oracle outputs of nghttp3_amd.synth batches (gen_golden.py)"
    with open(path, "w") as f:
        json.dump(d, f, indent=1)


def main():
    with open(os.path.join(HERE, "tables.json.new"), "w") as f:
        gen_tables(f)
    if os.path.getsize(os.path.join(HERE, "tables.json.new")):
        os.replace(os.path.join(HERE, "tables.json.new"), os.path.join(HERE, "tables.json"))
    else:
        os.remove(os.path.join(HERE, "tables.json.new"))
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        gen_kat(f)
    with open(os.path.join(HERE, "errors.json"), "w") as f:
        gen_errors(f)
    gen_corpus(os.path.join(HERE, "corpus.npz"))
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        gen_digests(f)


if __name__ == "__main__":
    if len(sys.argv) > 1:  # e.g. gen_golden.py c5_r0of8 c4_blocks: just those digests
        update_digests(sys.argv[1:])
    else:
        main()
