"""Sequential vs two-stream pipelined encode+decode round trips (development
measurement): encode of batch i+1 on stream A while batch i decodes on
stream B; enc buffers alternate."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from nghttp3_amd import HuffmanBatchCodec, synth  # noqa: E402
from nghttp3_amd import qpack_huffman as q  # noqa: E402


def main():
    n, steps = 1 << 20, 20
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    ce = HuffmanBatchCodec(0, stream=sa)
    cd = HuffmanBatchCodec(0, stream=sb)
    src, spans, total = ce.synth(0x5EED0003, n, 8, 256, synth.ALPHABET_A)
    torch.cuda.synchronize()
    ln = spans[:, 1] & 0xFFFFFFFF
    bound = int(((ln * 30 + 7) // 8).sum().item())
    enc = [torch.empty(bound, dtype=torch.uint8, device="cuda") for _ in range(2)]
    eout = [torch.empty((n, 2), dtype=torch.int64, device="cuda") for _ in range(2)]
    dout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    ce.encode_dev(src, spans, enc[0], eout[0])
    ce.sync()
    cap = int(q.decode_slot_size(eout[0][:, 1] & 0xFFFFFFFF).sum().item())
    dec = torch.empty(cap, dtype=torch.uint8, device="cuda")
    ev_enc = [torch.cuda.Event() for _ in range(2)]
    ev_dec = [torch.cuda.Event() for _ in range(2)]

    def seq(k):
        for i in range(k):
            ce.encode_dev(src, spans, enc[0], eout[0])
            ev_enc[0].record(sa)
            sb.wait_event(ev_enc[0])
            cd.decode_dev(enc[0], eout[0], dec, dout)
            ev_dec[0].record(sb)
            sa.wait_event(ev_dec[0])

    def pipe(k):
        for i in range(k):
            b = i & 1
            if i >= 2:
                sa.wait_event(ev_dec[b])  # decode i-2 is done with enc[b]
            ce.encode_dev(src, spans, enc[b], eout[b])
            ev_enc[b].record(sa)
            sb.wait_event(ev_enc[b])
            cd.decode_dev(enc[b], eout[b], dec, dout)
            ev_dec[b].record(sb)

    for name, fn in (("sequential", seq), ("pipelined", pipe), ("sequential", seq), ("pipelined", pipe)):
        fn(3)
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn(steps)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / steps
        print(f"{name}: {dt * 1e3:.3f} ms/step  {total / dt / 2**30:.1f} GiB/s", flush=True)
    # check the last decode
    ok = bool(((dout[:, 1] & 0xFFFFFFFF) == ln).all()) and bool(((dout[:, 1] >> 32) == 0).all())
    print("last decode lengths ok:", ok)


if __name__ == "__main__":
    main()
