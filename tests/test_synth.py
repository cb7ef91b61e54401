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


def test_rank_shards_of_one_batch_tile_it():
    """bench.py's split: N x n strings of one seed, cut by bytes; rank r
    generates its bytes alone from the global byte offset (qh_synth_fill's
    `first`), and the shards concatenate to the whole batch."""
    from nghttp3_amd import shard
    world, n = 4, 5000
    ln = synth.lengths(synth.SEEDS[3], world * n, 8, 256)
    plain = synth.fill(synth.SEEDS[3], int(ln.sum(dtype=np.uint64)), synth.ALPHABET_A)
    parts = []
    for r, (b, e) in enumerate(shard.split_by_bytes(ln, world)):
        first = int(ln[:b].sum(dtype=np.uint64))
        m = int(ln[b:e].sum(dtype=np.uint64))
        parts.append(synth.fill(synth.SEEDS[3], m, synth.ALPHABET_A, first=first))
        assert abs(m - plain.size / world) <= 256
    assert np.concatenate(parts).tobytes() == plain.tobytes()


def test_zipf_lengths_config5_shape():
    ln = synth.zipf_lengths(synth.SEEDS[5], 1 << 20, 1, 4096, 1.2)
    assert ln.min() >= 1 and ln.max() <= 4096
    assert 195 < ln.mean() < 225  # mean ~209 B
    assert (ln == 1).mean() > 0.2  # rank 1 is the most likely length
    again = synth.zipf_lengths(synth.SEEDS[5], 1000, 1, 4096, 1.2)
    assert (again == ln[:1000]).all()
