"""Compare the fused encoder with the window encoder on a small batch and
print the first differing string (development tool, one GPU)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nghttp3_amd import HuffmanBatchCodec, synth  # noqa: E402


def main():
    n = int(os.environ.get("N", 3000))
    c = HuffmanBatchCodec(0)
    src, spans, total = c.synth(0x5EED0003, n, 8, 256, synth.ALPHABET_A)
    ln = spans[:, 1] & 0xFFFFFFFF
    cap = int(((ln * 30 + 7) // 8).sum().item()) + 64
    res = {}
    for kind in ("windows", "fused"):
        c.set_encoder(kind)
        enc = torch.full((cap,), 0xA5, dtype=torch.uint8, device="cuda")
        out = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
        c.encode_dev(src, spans, enc, out)
        torch.cuda.synchronize()
        res[kind] = (enc.cpu().numpy(), out.cpu().numpy())
    (ew, ow), (ef, of) = res["windows"], res["fused"]
    print("offsets equal:", (ow[:, 0] == of[:, 0]).all(), "lens equal:", ((ow[:, 1] & 0xFFFFFFFF) == (of[:, 1] & 0xFFFFFFFF)).all())
    lens = (ln.cpu().numpy()).astype(np.int64)
    bad = 0
    for i in range(n):
        o, l = ow[i, 0], ow[i, 1] & 0xFFFFFFFF
        o2 = of[i, 0]
        a, b = ew[o:o + l], ef[o2:o2 + l]
        if o != o2 or not (a == b).all():
            d = np.nonzero(a != b)[0]
            print("string", i, "window", i // 64, "lane", i % 64, "plain len", lens[i], "enc len", l,
                  "off", o, o2, "first diff byte", d[:8], "n diff", d.size)
            print("  want", a[:24].tobytes().hex())
            print("  got ", b[:24].tobytes().hex())
            bad += 1
            if bad > 6:
                break
    print("bad strings:", bad)


if __name__ == "__main__":
    main()
