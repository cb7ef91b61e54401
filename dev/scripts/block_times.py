"""Per-block start/lifetime/placement of one launch (development tool; the
stamps build).  Usage: QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so
python scripts/block_times.py [enc_lens|enc|dec]"""
import ctypes
import os
import sys
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nghttp3_amd import HuffmanBatchCodec, _lib  # noqa: E402
from nghttp3_amd.qpack_huffman import decode_slot_size  # noqa: E402
from nghttp3_amd.synth import ALPHABET_A  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "enc_lens"
    lib = _lib.load()
    n = 1 << 20
    codec = HuffmanBatchCodec(0)
    src, spans, total = codec.synth(0x5EED0003, n, 8, 256, ALPHABET_A)
    enc = torch.empty(total * 4 + 64, dtype=torch.uint8, device="cuda")
    eout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    hlen = torch.empty(n, dtype=torch.int32, device="cuda")
    codec.encode_dev(src, spans, enc, eout)
    codec.sync()
    cap = int(decode_slot_size((eout[:, 1] & 0xFFFFFFFF).cpu().numpy()).sum())
    dec = torch.empty(cap + 64, dtype=torch.uint8, device="cuda")
    dout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    run = {"enc_lens": lambda: codec.encode_count_dev(src, spans, hlen),
           "enc": lambda: codec.encode_dev(src, spans, enc, eout),  # (the codes pass's blocks: it runs last)
           "dec": lambda: codec.decode_dev(enc, eout, dec, dout)}[which]
    for _ in range(3):
        run()
    codec.sync()
    buf = (ctypes.c_uint64 * (8192 * 4))()
    lib.qh_debug_blocks.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    assert lib.qh_debug_blocks(buf, 8192) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 4).astype(np.int64)
    a = a[a[:, 1] > 0]
    t0 = a[:, 0].min()
    st = (a[:, 0] - t0) / 100.0
    life = a[:, 1] / 100.0
    hw = a[:, 2] & 0xFFFFFFFF
    xcd = (a[:, 2] >> 32) & 7  # (XCC_ID, recorded by the stamps build since round 6)
    # HW_ID (gfx9): wave 3:0, simd 5:4, pipe 7:6, cu 11:8, sh 12, se 15:13
    cu = (hw >> 8) & 15
    se = (hw >> 13) & 7
    sh = (hw >> 12) & 1
    print(f"{which}: blocks {len(a)}  start max {st.max():.1f} us  life mean {life.mean():.1f} "
          f"p50 {np.median(life):.1f} p90 {np.percentile(life, 90):.1f} max {life.max():.1f} us  "
          f"end max {(st + life).max():.1f} us")
    bx = np.arange(len(a))
    # shader clock per block: s_memtime ticks / realtime (100 MHz) ticks
    mhz = a[:, 3] / np.maximum(a[:, 1], 1) * 100.0
    print("  clock MHz by blockIdx%8: " + "  ".join(
        f"{k}:{np.mean(mhz[bx % 8 == k]):.0f}" for k in range(8)))
    print("  clock MHz by xcd: " + "  ".join(f"{k}:{np.mean(mhz[xcd == k]):.0f}" for k in range(8)))
    print("  blockIdx%8 == xcd for", int((bx % 8 == xcd).sum()), "of", len(a), "blocks")
    for name, key in (("xcd", xcd), ("blockIdx%8", bx % 8), ("se", se), ("sh", sh)):
        g = defaultdict(list)
        for k, v in zip(key, life):
            g[int(k)].append(v)
        print(f"  by {name}: " + "  ".join(f"{k}:{np.mean(v):.1f}/{np.max(v):.1f}"
                                           for k, v in sorted(g.items())))
    # blocks per CU (se, sh, cu)
    cnt = defaultdict(int)
    cl = defaultdict(list)
    for s_, h_, c_, v in zip(se, sh, cu, life):
        cnt[(s_, h_, c_)] += 1
        cl[(s_, h_, c_)].append(v)
    hist = defaultdict(int)
    for v in cnt.values():
        hist[v] += 1
    print("  blocks per (se,sh,cu) slot:", dict(sorted(hist.items())), " distinct slots", len(cnt))
    slow = sorted(cl.items(), key=lambda kv: -np.mean(kv[1]))[:5]
    print("  slowest slots:", [(k, len(v), round(float(np.mean(v)), 1)) for k, v in slow])
    dec = [f"{np.mean(life[(bx >= len(a) * k // 16) & (bx < len(a) * (k + 1) // 16)]):.0f}" for k in range(16)]
    print("  life by blockIdx sixteenths:", " ".join(dec))
    order = np.argsort(-life)[:10]
    print("  slowest blocks:", [(int(bx[i]), round(float(life[i]), 1), round(float(st[i]), 1)) for i in order])


if __name__ == "__main__":
    main()
