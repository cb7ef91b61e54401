#!/usr/bin/env python3
"""Development: config 3 (2^20 strings 8-256 B, alphabet A, or ALPH=U) through
the length pass (encode_count_dev) and the window encoder (encode_dev) with the
library QHUFF_LIB names: per-kernel HIP-event times (ablation builds give
wrong lengths; the check against the product digest says which)."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from nghttp3_amd import HuffmanBatchCodec
    from nghttp3_amd.synth import ALPHABET_A, ALPHABET_U
    n = 1 << 20
    codec = HuffmanBatchCodec(0)
    codec.set_encoder("windows")
    src, spans, total = codec.synth(0x5EED0003, n, 8, 256,
                                    ALPHABET_U if os.environ.get("ALPH") == "U" else ALPHABET_A)
    hlen = torch.empty(n, dtype=torch.int32, device="cuda")
    enc = torch.empty(total * 4 + 64, dtype=torch.uint8, device="cuda")
    eout = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    out = {"lib": os.path.basename(os.environ.get("QHUFF_LIB", "libqhuff.so"))}
    for name, fn in (("count", lambda: codec.encode_count_dev(src, spans, hlen)),
                     ("encode", lambda: codec.encode_dev(src, spans, enc, eout))):
        for _ in range(3):
            fn()
        codec.sync()
        codec.enable_timing(True)
        for _ in range(10):
            fn()
        codec.sync()
        out[name] = {k: round(ms / max(c, 1) * 1e3, 2) for k, (c, ms) in codec.kernel_times().items()}
        codec.enable_timing(False)
    out["hlen_digest"] = hashlib.sha256(hlen.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
