import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import oracle
from nghttp3_amd import HuffmanBatchCodec, pack_strings, unpack_out, synth
codec = HuffmanBatchCodec(0)
for n in (9, 300, 2047, 2048, 2049, 4096):
    plain, off, ln = synth.batch(0x5EED0002, n, 0, 300, synth.ALPHABET_A)
    strs = [plain[int(o):int(o) + int(k)].tobytes() for o, k in zip(off, ln)]
    encs = [oracle.encode(s) for s in strs]
    src, sp = pack_strings(encs)
    d_src = torch.from_numpy(src.copy()).cuda()
    d_sp = torch.from_numpy(sp.view(np.int64).reshape(-1, 2).copy()).cuda()
    cap = int((((sp["len"].astype(np.int64) * 8 // 5) + 15) // 16 * 16).sum())
    d_dst = torch.zeros(cap + 64, dtype=torch.uint8, device="cuda")
    d_out = torch.zeros((len(strs), 2), dtype=torch.int64, device="cuda")
    codec.decode_dev(d_src, d_sp, d_dst[:cap], d_out)
    o, l, s = unpack_out(d_out)
    dst = d_dst.cpu().numpy()
    bad = [i for i, x in enumerate(strs) if s[i] != 0 or dst[o[i]:o[i]+l[i]].tobytes() != x]
    print("n", n, "bad", len(bad), bad[:10])
    for i in bad[:3]:
        print("  ", i, "enclen", len(encs[i]), "len", l[i], "want", len(strs[i]), "st", s[i], "off", o[i],
              "got", dst[o[i]:o[i]+l[i]].tobytes()[:40], "want", strs[i][:40])
    print("  stats", codec.stats())
