import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import oracle
from nghttp3_amd import HuffmanBatchCodec, synth
codec = HuffmanBatchCodec(0)
n = 1 << 20
def run(seed, alph, reps=2):
    src, spans, total = codec.synth(seed, n, 8, 256, alph)
    plain = src[:total].cpu().numpy(); sp = spans.cpu().numpy()
    off = sp[:, 0].astype(np.uint64); ln = (sp[:, 1] & 0xFFFFFFFF).astype(np.uint32)
    enc_ref, eoff_ref, elen_ref = oracle.encode_batch(plain, off, ln)
    bound = int(((ln.astype(np.int64) * 30 + 7) // 8).sum())
    for rep in range(reps):
        enc = torch.zeros(bound, dtype=torch.uint8, device="cuda")
        eout = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
        torch.cuda.synchronize(); t0 = time.perf_counter()
        codec.encode_dev(src, spans, enc, eout)
        torch.cuda.synchronize(); t1 = time.perf_counter()
        e = enc.cpu().numpy()
        bad = np.nonzero(e[:enc_ref.size] != enc_ref)[0]
        print(hex(seed), "rep", rep, "ms %.3f" % ((t1 - t0) * 1e3), "nbad", bad.size)
        if bad.size:
            eo = eoff_ref.astype(np.int64)
            strs = np.unique(np.searchsorted(eo, bad, side="right") - 1)
            w = (off.astype(np.int64) - int(off[0])) + 16 * np.arange(n)
            tiles = w // 8192
            print("  bad strings", strs.size, "first", strs[:8])
            for s in strs[:6]:
                t = tiles[s]; first = np.searchsorted(tiles, t)
                tile_base = int(off[first])
                print("   s", s, "tile", t, "str-in-tile", s - first, "byte-in-tile", int(off[s]) - tile_base,
                      "end-in-tile", int(off[s]) + int(ln[s]) - tile_base, "len", ln[s], "enc", eo[s], elen_ref[s])
                print("    got ", e[eo[s]:eo[s] + elen_ref[s]].tobytes().hex()[:80])
                print("    want", enc_ref[eo[s]:eo[s] + elen_ref[s]].tobytes().hex()[:80])
run(0x5EED0002, synth.ALPHABET_U)
run(0x5EED0003, synth.ALPHABET_A, 3)
