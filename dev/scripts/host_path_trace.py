#!/usr/bin/env python3
"""Development: the host-memory decode of config 3 (pinned buffers, 2^20
strings) a few times, for a rocprofv3 --memory-copy-trace --kernel-trace run
of its copies and kernels:
  rocprofv3 --memory-copy-trace --kernel-trace --stats -d OUT -o run -- \\
      python3 dev/scripts/host_path_trace.py
Prints the wall time per decode (and of the 2-context form)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch
    from nghttp3_amd import HuffmanBatchCodec, synth
    from nghttp3_amd import qpack_huffman as q
    codec = HuffmanBatchCodec(0)
    src, spans, total = codec.synth(0x5EED0003, 1 << 20, 8, 256, synth.ALPHABET_A)
    ln = spans[:, 1] & 0xFFFFFFFF
    enc = torch.zeros(int(((ln * 30 + 7) // 8).sum().item()), dtype=torch.uint8, device="cuda")
    eout = torch.zeros((1 << 20, 2), dtype=torch.int64, device="cuda")
    codec.encode_dev(src, spans, enc, eout)
    torch.cuda.synchronize()
    eo = eout.cpu().numpy()
    eb = int((eo[:, 1] & 0xFFFFFFFF).sum())
    e_t = torch.empty(eb, dtype=torch.uint8, pin_memory=True)
    e_t.copy_(enc[:eb])
    sp_t = torch.zeros(eo.shape[0] * 2, dtype=torch.int64, pin_memory=True)
    spn = sp_t.numpy().view(q.SPAN_IN_DTYPE)
    spn["off"], spn["len"] = eo[:, 0], eo[:, 1] & 0xFFFFFFFF
    cap = int(q.decode_slot_size(spn["len"].astype(np.int64)).sum())
    d_t = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
    o_t = torch.empty(eo.shape[0] * 2, dtype=torch.int64, pin_memory=True)
    e_h, d_h, o_h = e_t.numpy(), d_t.numpy(), o_t.numpy().view(q.SPAN_OUT_DTYPE)
    res = {}
    codec.decode_host(e_h, spn, d_h, o_h)
    ts = []
    for _ in range(5):
        a = time.perf_counter()
        codec.decode_host(e_h, spn, d_h, o_h)
        ts.append(time.perf_counter() - a)
    res["one_ctx_ms"] = [round(t * 1e3, 3) for t in ts]
    cs = [HuffmanBatchCodec(0, stream=torch.cuda.Stream()) for _ in range(2)]
    HuffmanBatchCodec.decode_host_multi(cs, e_h, spn, d_h, o_h)
    ts = []
    for _ in range(5):
        a = time.perf_counter()
        HuffmanBatchCodec.decode_host_multi(cs, e_h, spn, d_h, o_h)
        ts.append(time.perf_counter() - a)
    res["two_ctx_ms"] = [round(t * 1e3, 3) for t in ts]
    res["GiBps_one_two"] = [round(total / min(res[k]) * 1e3 / 2**30, 2) for k in ("one_ctx_ms", "two_ctx_ms")]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
