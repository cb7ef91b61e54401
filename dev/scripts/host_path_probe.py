"""PCIe probe for the host-memory decode path (development tool): raw pinned
H2D / D2H / both-direction copy rates next to decode_host's time."""
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
    c = HuffmanBatchCodec(0)
    res = {}
    nb = 128 << 20
    h1 = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    h2 = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    d1 = torch.empty(nb, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(nb, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def t(fn, reps=5):
        fn(); torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - a) / reps

    res["h2d_GBps"] = nb / t(lambda: d1.copy_(h1, non_blocking=True)) / 1e9
    res["d2h_GBps"] = nb / t(lambda: h2.copy_(d2, non_blocking=True)) / 1e9

    def both():
        with torch.cuda.stream(s1):
            d1.copy_(h1, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
    res["both_GBps_each"] = nb / t(both) / 1e9
    if hasattr(c._lib, "qh_debug_copy16"):  # development build: zero-copy kernel copies
        import ctypes
        lib = c._lib
        lib.qh_debug_copy16.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_uint64, ctypes.c_void_p]

        def kcopy(dst, src, st):
            assert lib.qh_debug_copy16(c._ctx, dst.data_ptr(), src.data_ptr(), nb, st.cuda_stream) == 0
        res["kernel_d2h_GBps"] = nb / t(lambda: kcopy(h2, d2, s2)) / 1e9
        res["kernel_h2d_GBps"] = nb / t(lambda: kcopy(d1, h1, s1)) / 1e9

        def sdma_h2d_kernel_d2h():
            with torch.cuda.stream(s1):
                d1.copy_(h1, non_blocking=True)
            kcopy(h2, d2, s2)
        res["sdma_h2d_with_kernel_d2h_GBps_each"] = nb / t(sdma_h2d_kernel_d2h) / 1e9

        def kernels_both():
            kcopy(d1, h1, s1)
            kcopy(h2, d2, s2)
        res["kernel_both_GBps_each"] = nb / t(kernels_both) / 1e9
        assert torch.equal(h2[:4096].cpu(), d2[:4096].cpu()) and torch.equal(d1[-4096:].cpu(), h1[-4096:])
    src, spans, total = c.synth(0x5EED0003, 1 << 20, 8, 256, synth.ALPHABET_A)
    ln = spans[:, 1] & 0xFFFFFFFF
    enc = torch.zeros(int(((ln * 30 + 7) // 8).sum().item()), dtype=torch.uint8, device="cuda")
    eout = torch.zeros((1 << 20, 2), dtype=torch.int64, device="cuda")
    c.encode_dev(src, spans, enc, eout)
    torch.cuda.synchronize()
    eo = eout.cpu().numpy()
    eb = int((eo[:, 1] & 0xFFFFFFFF).sum())
    e_t = torch.empty(eb, dtype=torch.uint8, pin_memory=True)
    e_t.copy_(enc[:eb])
    sp_t = torch.zeros((1 << 20) * 2, dtype=torch.int64, pin_memory=True)
    spn = sp_t.numpy().view(q.SPAN_IN_DTYPE)
    spn["off"], spn["len"] = eo[:, 0], eo[:, 1] & 0xFFFFFFFF
    cap = int(q.decode_slot_size(eo[:, 1] & 0xFFFFFFFF).sum())
    d_t = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
    o_t = torch.empty((1 << 20) * 2, dtype=torch.int64, pin_memory=True)
    e_h, d_h, o_h = e_t.numpy(), d_t.numpy(), o_t.numpy().view(q.SPAN_OUT_DTYPE)
    c.decode_host(e_h, spn, d_h, o_h)
    a = time.perf_counter()
    for _ in range(5):
        c.decode_host(e_h, spn, d_h, o_h)
    td = (time.perf_counter() - a) / 5
    res["decode_host_ms"] = td * 1e3
    res["decode_host_GiBps"] = total / td / 2**30
    res["h2d_bytes"] = eb + 16 * (1 << 20)
    res["d2h_bytes"] = total + 16 * (1 << 20)
    a = time.perf_counter()
    for _ in range(5):
        lo = spn["off"].min(); hi = (spn["off"] + spn["len"]).max()
    res["numpy_span_pass_ms"] = (time.perf_counter() - a) / 5 * 1e3
    print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in res.items()}))


if __name__ == "__main__":
    main()
