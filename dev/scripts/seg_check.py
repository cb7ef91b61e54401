#!/usr/bin/env python3
"""Development: the segment encoder (QHUFF_SEG=1, QH_ENCODER_FUSED) against
the window encoder on small and full-size batches: first mismatching
string, its window and bytes."""
import os
import sys

os.environ["QHUFF_SEG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch
    from nghttp3_amd import HuffmanBatchCodec, synth
    c = HuffmanBatchCodec(device=0)
    cases = [(1, 8, 256, "A"), (5, 1, 40, "A"), (130, 8, 256, "A"), (1000, 0, 64, "A"), (4096, 8, 256, "A"),
             (4096, 8, 256, "U"), (70000, 1, 600, "A"), (1 << 20, 8, 256, "A"), (1 << 20, 8, 256, "U")]
    if len(sys.argv) > 1:
        cases = cases[:int(sys.argv[1])]
    bad = 0
    for (n, lo, hi, al) in cases:
        alph = synth.ALPHABET_A if al == "A" else synth.ALPHABET_U
        src, spans, total = c.synth(0x5EED0000 + n, n, lo, hi, alph)
        ln = spans[:, 1] & 0xFFFFFFFF
        bound = int(((ln * 30 + 7) // 8).sum().item()) + 64
        res = {}
        for kind in ("windows", "fused"):
            c.set_encoder(kind)
            enc = torch.full((bound,), 0xA5, dtype=torch.uint8, device="cuda")
            eout = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
            c.encode_dev(src, spans, enc, eout)
            torch.cuda.synchronize()
            res[kind] = (enc.cpu().numpy(), eout.cpu().numpy())
        (ew, ow), (ef, of) = res["windows"], res["fused"]
        eb = int((ow[:, 1] & 0xFFFFFFFF).sum())
        ok_o = np.array_equal(ow, of)
        ok_b = np.array_equal(ew[:eb], ef[:eb])
        tail_ok = bool((ef[eb:eb + 32] == 0xA5).all())
        print(f"n={n} lens {lo}-{hi} {al}: spans {'ok' if ok_o else 'BAD'} bytes {'ok' if ok_b else 'BAD'} "
              f"tail {'ok' if tail_ok else 'BAD'} ({eb} bytes)", flush=True)
        if not ok_o:
            i = int(np.nonzero((ow != of).any(axis=1))[0][0])
            print(f"  first span mismatch string {i} (window {i // 128}, lane {i % 64}): "
                  f"windows {ow[i, 0]} {ow[i, 1] & 0xFFFFFFFF} st {ow[i, 1] >> 32}  "
                  f"fused {of[i, 0]} {of[i, 1] & 0xFFFFFFFF} st {of[i, 1] >> 32}; len {int(ln[i])}")
            bad += 1
        elif not ok_b:
            j = int(np.nonzero(ew[:eb] != ef[:eb])[0][0])
            i = int(np.searchsorted(ow[:, 0], j, side="right") - 1)
            nmis = int((ew[:eb] != ef[:eb]).sum())
            w0 = (i // 128) * 128
            w1 = min(w0 + 128, n)
            sp = spans.cpu().numpy()
            offs, lns = sp[w0:w1, 0], sp[w0:w1, 1] & 0xFFFFFFFF
            reg = src[int(offs[0]):int(offs[-1] + lns[-1])].cpu().numpy()
            np.savez(os.path.join(os.environ.get("SEG_DUMP", "/tmp"), f"seg_fail_{n}_{al}.npz"), region=reg,
                     lens=lns, off0=int(offs[0]), src_ptr_mod16=int(src.data_ptr() + int(offs[0])) % 16,
                     B=int(ow[w0, 0]), want=ew[int(ow[w0, 0]):int(ow[w1 - 1, 0] + (ow[w1 - 1, 1] & 0xFFFFFFFF))],
                     got=ef[int(ow[w0, 0]):int(ow[w1 - 1, 0] + (ow[w1 - 1, 1] & 0xFFFFFFFF))])
            print(f"  first byte mismatch at {j} (string {i}, window {i // 128}, offset {j - ow[i, 0]} of "
                  f"{ow[i, 1] & 0xFFFFFFFF}; {nmis} bytes differ): windows {ew[j:j + 8].tolist()} "
                  f"fused {ef[j:j + 8].tolist()}")
            bad += 1
        elif not tail_ok:
            bad += 1
    print("ALL OK" if bad == 0 else f"{bad} BAD", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
