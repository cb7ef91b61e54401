import sys, os, hashlib
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import oracle
from nghttp3_amd import HuffmanBatchCodec, synth
codec = HuffmanBatchCodec(0)
seed = int(sys.argv[1], 0) if len(sys.argv) > 1 else 0x5EED0003
n = 1 << 20
src, spans, total = codec.synth(seed, n, 8, 256, synth.ALPHABET_A)
plain = src[:total].cpu().numpy(); sp = spans.cpu().numpy()
off = sp[:, 0].astype(np.uint64); ln = (sp[:, 1] & 0xFFFFFFFF).astype(np.uint32)
enc_ref, eoff_ref, elen_ref = oracle.encode_batch(plain, off, ln)
bound = int(((ln.astype(np.int64) * 30 + 7) // 8).sum())
for rep in range(3):
    enc = torch.zeros(bound, dtype=torch.uint8, device="cuda")
    eout = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    codec.encode_dev(src, spans, enc, eout)
    e = enc.cpu().numpy(); eo = eout.cpu().numpy()
    o = eo[:, 0]; l = eo[:, 1] & 0xFFFFFFFF; st = eo[:, 1] >> 32
    print("rep", rep, "len ok", bool((l == elen_ref).all()), "off ok", bool((o == eoff_ref.astype(np.int64)).all()),
          "status ok", bool((st == 0).all()), "bytes ok", bool((e[:enc_ref.size] == enc_ref).all()))
    bad = np.nonzero(e[:enc_ref.size] != enc_ref)[0]
    if bad.size:
        b0 = bad[0]
        s = int(np.searchsorted(eoff_ref.astype(np.int64), b0, side="right") - 1)
        print("  first bad byte", b0, "n bad bytes", bad.size, "string", s, "enc off", eoff_ref[s], "len", elen_ref[s],
              "plain off", off[s], "plain len", ln[s])
        print("  got ", e[eoff_ref[s]:eoff_ref[s] + elen_ref[s] + 4].tobytes().hex())
        print("  want", enc_ref[eoff_ref[s]:eoff_ref[s] + elen_ref[s] + 4].tobytes().hex())
        strs = np.unique(np.searchsorted(eoff_ref.astype(np.int64), bad, side="right") - 1)
        print("  bad strings", strs.size, strs[:20])
        # tile position of first bad string: weight
        w = (off[strs[:10]] - off[0]) + 16 * strs[:10]
        print("  tile", w // 8192, "w mod", w % 8192, "byte-in-tile?")
