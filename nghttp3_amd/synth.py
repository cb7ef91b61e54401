"""Deterministic synthetic workloads (BASELINE.md "Inputs per config").

Bit-exact host restatement of the device generator in
nghttp3_amd/csrc/qh_device.hip (qh_k_synth_lens / qh_k_synth_fill):

* splitmix64, counter form: draw(seed, k) = mix(seed + (k + 1) * golden).
* string i has length lo + draw(seed ^ LEN_STREAM, i) % (hi - lo + 1);
  strings are packed back to back (off = exclusive prefix sum of lengths);
* byte k of the packed buffer is alphabet[draw(seed ^ BYTE_STREAM, k) % |A|].
"""
from __future__ import annotations

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
LEN_STREAM = 0x4C454E47544853
BYTE_STREAM = 0x4259544553

# Alphabet "A": 76 header-like characters.
ALPHABET_A = (b"abcdefghijklmnopqrstuvwxyz"
              b"ABCDEFGHIJKLMNOPQRSTUVWXYZ"
              b"0123456789"
              b"-_./:;=,?&%+* ")
assert len(ALPHABET_A) == 76
# Alphabet "U": every byte value (stress: long codes, E/D ~ 2.3).
ALPHABET_U = bytes(range(256))

SEEDS = {1: 0x5EED0001, 2: 0x5EED0002, 3: 0x5EED0003, 4: 0x5EED0004, 5: 0x5EED0005}


def _mix(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def draws(seed: int, start: int, count: int) -> np.ndarray:
    k = np.arange(start + 1, start + count + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return _mix(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + k * GOLDEN)


def lengths(seed: int, n: int, lo: int, hi: int) -> np.ndarray:
    r = draws(seed ^ LEN_STREAM, 0, n)
    return (np.uint64(lo) + r % np.uint64(hi - lo + 1)).astype(np.uint32)


def fill(seed: int, nbytes: int, alphabet: bytes, chunk: int = 1 << 24, first: int = 0) -> np.ndarray:
    """Bytes [first, first + nbytes) of the packed stream (qh_synth_fill)."""
    a = np.frombuffer(bytes(alphabet), dtype=np.uint8)
    out = np.empty(nbytes, dtype=np.uint8)
    for s in range(0, nbytes, chunk):
        m = min(chunk, nbytes - s)
        out[s:s + m] = a[(draws(seed ^ BYTE_STREAM, first + s, m) % np.uint64(a.size)).astype(np.int64)]
    return out


def zipf_lengths(seed: int, n: int, lo: int, hi: int, s: float) -> np.ndarray:
    """Config 5's lengths: P(len = k) proportional to k^-s over [lo, hi]
    (s = 1.2 over 1..4096, mean ~209 B), by inverse
    CDF of the 53-bit uniform draw(seed ^ LEN_STREAM, i) / 2^53 (float64,
    sequential cumsum: the same on every host)."""
    k = np.arange(lo, hi + 1, dtype=np.float64)
    w = k ** -float(s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    u = (draws(seed ^ LEN_STREAM, 0, n) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
    idx = np.searchsorted(cdf, u, side="right")
    return (lo + np.minimum(idx, hi - lo)).astype(np.uint32)


def batch(seed: int, n: int, lo: int, hi: int, alphabet: bytes):
    """Returns (plain uint8 array, off uint64 array, len uint32 array)."""
    ln = lengths(seed, n, lo, hi)
    off = np.zeros(n, dtype=np.uint64)
    if n:
        off[1:] = np.cumsum(ln.astype(np.uint64))[:-1]
    total = int(ln.astype(np.uint64).sum())
    return fill(seed, total, alphabet), off, ln
