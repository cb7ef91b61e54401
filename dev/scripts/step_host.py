#!/usr/bin/env python3
"""Where a bench step's time goes beyond the kernels (development tool, one
GPU): host enqueue time of K round-trip steps, their wall time, and the same
with the per-kernel events on; encoder choice from argv (auto|windows)."""
import sys, os, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from nghttp3_amd import HuffmanBatchCodec, synth, qpack_huffman as q

kind = sys.argv[1] if len(sys.argv) > 1 else "auto"
c = HuffmanBatchCodec(device=0)
if kind != "auto":
    c.set_encoder(kind)
src, spans, total = c.synth(0x5EED0003, 1 << 20, 8, 256, synth.ALPHABET_A)
n = spans.shape[0]
ln = spans[:, 1] & 0xFFFFFFFF
enc = torch.empty(int(((ln * 30 + 7) // 8).sum().item()), dtype=torch.uint8, device="cuda")
eout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
c.encode_dev(src, spans, enc, eout)
torch.cuda.synchronize()
cap = int(q.decode_slot_size(eout[:, 1] & 0xFFFFFFFF).sum().item())
dec = torch.empty(cap, dtype=torch.uint8, device="cuda")
dout = torch.empty((n, 2), dtype=torch.int64, device="cuda")

def step():
    c.encode_dev(src, spans, enc, eout)
    c.decode_dev(enc, eout, dec, dout)

for _ in range(5):
    step()
torch.cuda.synchronize()
for K in (20, 100):
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"kind": kind, "K": K, "enqueue_us_per_step": round((t1 - t0) / K * 1e6, 1),
                      "wall_us_per_step": round((t2 - t0) / K * 1e6, 1),
                      "GiBps": round(total * K / (t2 - t0) / 2**30, 1)}), flush=True)
# host cost of each call alone
for name, f in (("encode", lambda: c.encode_dev(src, spans, enc, eout)), ("decode", lambda: c.decode_dev(enc, eout, dec, dout))):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        f()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"call": name, "enqueue_us": round((t1 - t0) / 50 * 1e6, 1), "wall_us": round((t2 - t0) / 50 * 1e6, 1)}), flush=True)
