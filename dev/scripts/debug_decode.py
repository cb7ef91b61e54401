import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import oracle
from nghttp3_amd import HuffmanBatchCodec, pack_strings, unpack_out
codec = HuffmanBatchCodec(0)
strs = [b"", b"a", b"ab", b"abc", b"0123456789abcdef", b"x" * 17, b"hello world", b"\x00", b"\xff" * 3]
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
for i, x in enumerate(strs):
    print(i, encs[i].hex(), "off", o[i], "len", l[i], "st", s[i], "got", dst[o[i]:o[i]+l[i]].tobytes(), "want", x)
print("dst head", dst[:48].tobytes())
print(codec.stats())
