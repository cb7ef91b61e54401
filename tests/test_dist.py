"""World-size-2 gloo run of the sharded path (CPU): each rank takes its
byte-balanced contiguous shard of one batch, encodes/decodes it alone (the
oracle stands in for the device here), and only the report crosses ranks.
The reduced report must equal the single-process result."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from nghttp3_amd import shard, synth


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        plain, off, ln = synth.batch(synth.SEEDS[4], 20000, 1, 400, synth.ALPHABET_A)
        b, e = shard.split_by_bytes(ln, world)[rank]
        enc, eoff, elen = oracle.encode_batch(plain, off[b:e], ln[b:e])
        dst, slot, olen, st = oracle.decode_batch(enc, eoff, elen)
        local = {"strings": e - b, "plain_bytes": int(ln[b:e].sum()), "enc_bytes": int(enc.size),
                 "errors": int((st != 0).sum()) + int((olen != ln[b:e]).sum()),
                 "time_max": float(rank + 1)}
        rep = shard.reduce_report(local, dist)
        base = shard.output_offsets(int(enc.size), dist)
        q.put((rank, b, e, base, rep, enc.tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_roundtrip_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import oracle
    plain, off, ln = synth.batch(synth.SEEDS[4], 20000, 1, 400, synth.ALPHABET_A)
    enc, eoff, elen = oracle.encode_batch(plain, off, ln)
    # shards tile the batch, in order, with near-equal bytes
    assert res[0][1] == 0 and res[-1][2] == len(ln)
    assert all(res[i][2] == res[i + 1][1] for i in range(world - 1))
    sizes = [int(ln[b:e].sum()) for _, b, e, *_ in res]
    assert max(sizes) - min(sizes) <= 2 * 400  # one string either side of a cut
    # global output offsets come from the all-gather; shards concatenate
    assert [r[3] for r in res] == [0] + list(np.cumsum([len(r[5]) for r in res])[:-1])
    assert b"".join(r[5] for r in res) == enc.tobytes()
    rep = res[0][4]
    assert rep == res[1][4]
    assert rep["strings"] == len(ln) and rep["plain_bytes"] == int(ln.sum())
    assert rep["enc_bytes"] == enc.size and rep["errors"] == 0 and rep["time_max"] == world


def test_split_by_bytes_edges():
    assert shard.split_by_bytes([], 4) == [(0, 0)] * 4
    assert shard.split_by_bytes([5], 3) == [(0, 0), (0, 0), (0, 1)] or \
        sum(e - b for b, e in shard.split_by_bytes([5], 3)) == 1
    r = shard.split_by_bytes([1] * 10, 3)
    assert r[0][0] == 0 and r[-1][1] == 10
    assert sum(e - b for b, e in r) == 10


def block_worker(rank, world, port, q):
    """Config 4 at world size 2: each rank frames its block range alone."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nghttp3_amd import qpack
        src, blocks, *_ = qpack.synth_field_sections(0x5EED0004, 3001)
        lo, hi = shard.block_range_by_bytes(rank, world, blocks["len"])
        lines, spans, ls, ss, st = qpack.scan_blocks(src, blocks[lo:hi])
        local = {"blocks": hi - lo, "lines": int(lines.size), "spans": int(spans.size),
                 "errors": int((st != 0).sum()), "time_max": float(rank + 1)}
        rep = shard.reduce_report(local, dist)
        q.put((rank, lo, hi, rep, spans.tobytes()))
    finally:
        dist.destroy_process_group()


def test_sharded_blocks_gloo():
    from nghttp3_amd import qpack
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=block_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    src, blocks, *_ = qpack.synth_field_sections(0x5EED0004, 3001)
    lines, spans, ls, ss, st = qpack.scan_blocks(src, blocks)
    assert res[0][1] == 0 and res[0][2] == res[1][1] and res[1][2] == blocks.size
    assert b"".join(r[4] for r in res) == spans.tobytes()
    rep = res[0][3]
    assert rep == res[1][3]
    assert rep["blocks"] == blocks.size and rep["lines"] == lines.size
    assert rep["spans"] == spans.size and rep["errors"] == 0 and rep["time_max"] == world


def test_block_range_by_bytes_never_empty():
    """A block bigger than a rank's byte share would leave a later rank no
    block under the byte cut; the split then falls back to the count cut, so
    every rank of a world <= nblocks has at least one block and the ranges
    tile [0, nblocks) (my["off"][0] on an empty range)."""
    lens = np.array([10_000] + [10] * 7, dtype=np.uint64)
    for world in range(1, 9):
        rs = [shard.block_range_by_bytes(r, world, lens) for r in range(world)]
        assert rs[0][0] == 0 and rs[-1][1] == lens.size
        assert all(lo < hi for lo, hi in rs), (world, rs)
        assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
    # balanced blocks keep the byte cut
    even = np.full(64, 100, dtype=np.uint64)
    assert [shard.block_range_by_bytes(r, 4, even) for r in range(4)] == \
        [(0, 16), (16, 32), (32, 48), (48, 64)]
