"""Synthetic workload generator: host restatement pinned by committed digests
(the device generator is checked against the same digests in test_gpu.py)."""
import hashlib

import numpy as np

from nghttp3_amd import synth


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_splitmix64_known_values():
    # splitmix64 seeded with 0: first outputs (published reference values)
    assert [int(x) for x in synth.draws(0, 0, 3)] == [
        0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4, 0x06C45D188009454F]


def test_lengths_in_range():
    ln = synth.lengths(synth.SEEDS[2], 100_000, 8, 256)
    assert ln.min() == 8 and ln.max() == 256
    assert abs(ln.mean() - 132) < 1


def test_full_config_digests(digests):
    for name in ("c2_A", "c3_A"):
        d = digests[name]
        alph = synth.ALPHABET_A if d["alphabet"] == "A" else synth.ALPHABET_U
        plain, off, ln = synth.batch(d["seed"], d["n"], d["lo"], d["hi"], alph)
        assert plain.size == d["plain_bytes"]
        assert sha(ln) == d["len_sha256"]
        assert sha(plain) == d["plain_sha256"]
