import os, sys
os.environ["QHUFF_SEG"] = "1"; os.environ["QHUFF_SEG_DBG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from nghttp3_amd import HuffmanBatchCodec, synth
c = HuffmanBatchCodec(device=0)
n = 4096
src, spans, total = c.synth(0x5EED0000 + n, n, 8, 256, synth.ALPHABET_A)
ln = spans[:, 1] & 0xFFFFFFFF
bound = int(((ln * 30 + 7) // 8).sum().item()) + 64
c.set_encoder("fused")
enc = torch.full((bound,), 0xA5, dtype=torch.uint8, device="cuda")
eout = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
c.encode_dev(src, spans, enc, eout)
torch.cuda.synchronize()
