"""Field name / value validation: the
scalar drop-ins nghttp3_check_header_name / _value in libqhuff
(csrc/qh_http.c) against oracle/http_check.py driven by the reference's own
character tables (tests/golden/http_chars.json).  The GPU batch form is in
tests/test_gpu_qpack.py."""
import random

import pytest

from oracle import http_check as ref
from nghttp3_amd import qpack

from conftest import load_json


@pytest.fixture(scope="module")
def chars():
    d = load_json("http_chars.json")
    return d["VALID_HD_NAME_CHARS"], d["VALID_HD_VALUE_CHARS"]


def cases(seed=0x5EED0F5, n=3000):
    rng = random.Random(seed)
    out = [b"", b":", b"::", b":a", b"a", b"A", b" ", b"\t", b"a ", b" a", b"\ta", b"a\t",
           b"\x7f", b"\x80", b"\xff", b"\x00", b"x" * 31 + b"\x7f", b"x" * 32 + b"\x01",
           b"x" * 64, b":authority", b"Content-Type", b"content-type", b"a b"]
    out += [bytes([c]) for c in range(256)]
    out += [b"ab" + bytes([c]) + b"cd" for c in range(256)]
    for _ in range(n):
        k = rng.choice([1, 2, 5, 15, 16, 17, 31, 32, 33, 63, 100, 300])
        pool = rng.choice([b"abcxyz019-_.!~", b"abcXYZ :;\t", bytes(range(256)), b"a"])
        s = bytes(rng.choice(pool) for _ in range(k))
        if rng.random() < 0.2:
            s = b":" + s
        out.append(s)
    return out


def test_tables_match_the_rules_the_kernel_uses(chars):
    names, values = chars
    for c in range(256):
        assert qpack.check_header_name(bytes([c])) == (1 if names[c] == 1 else 0) or c == ord(":")
        v = qpack.check_header_value(b"a" + bytes([c]) + b"a")
        assert v == (1 if values[c] else 0)


def test_scalar_checks_match_oracle(chars):
    names, values = chars
    for s in cases():
        assert qpack.check_header_name(s) == ref.check_header_name(s, names), s
        assert qpack.check_header_value(s) == ref.check_header_value(s, values), s


def token_cases(tokens, seed=0x5EED0F7):
    rng = random.Random(seed)
    out = [b"", b":", b"x" * 33, b"x" * 32]
    for k in tokens:
        b = k.encode()
        out += [b, b.upper(), b[:-1], b + b"x", b"x" + b[1:], b[:-1] + b"x", b[:1] + b"Z" + b[2:]]
    for _ in range(2000):
        out.append(bytes(rng.choice(b"abcdeghilmnoprstuvwxy-:") for _ in range(rng.randrange(1, 34))))
    return out


def test_lookup_token_matches_reference_enum():
    tokens = load_json("tokens.json")["tokens"]
    assert len(tokens) == 61
    for name, tok in tokens.items():
        assert qpack.lookup_token(name.encode()) == tok
    for s in token_cases(tokens):
        assert qpack.lookup_token(s) == ref.lookup_token(s, tokens), s
