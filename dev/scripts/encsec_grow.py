#!/usr/bin/env python3
"""Development: the growing-batches encoder test step by step with prints
(a fresh context, batches of 3, 2049, 10, 4097, 64 sections)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch
    from nghttp3_amd import qpack
    enc = qpack.FieldSectionEncoder(0)
    for nsec in (3, 2049, 10, 4097, 64):
        src, blocks, plain, strs, lines, line_start = qpack.synth_field_sections(0x5EED0C6 + nsec, nsec)
        t_plain = torch.from_numpy(plain.copy()).cuda()
        t_strs = torch.from_numpy(strs.view(np.int64).reshape(-1, 2).copy()).cuda()
        t_lines = torch.from_numpy(lines.view(np.uint8).copy()).cuda()
        t_ls = torch.from_numpy(line_start.view(np.int32).copy()).cuda()
        t_dst = torch.zeros(src.size + 64, dtype=torch.uint8, device="cuda")
        t_sec = torch.zeros((nsec, 2), dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        print("call", nsec, "strings", strs.size, "lines", lines.size, flush=True)
        a = time.time()
        need = enc.encode_sections_dev(t_plain, t_strs, t_lines, t_ls, t_dst, t_sec)
        print(" returned", need, round(time.time() - a, 3), flush=True)
        torch.cuda.synchronize()
        ok = t_dst[:need].cpu().numpy().tobytes() == src.tobytes()
        print(" synced", round(time.time() - a, 3), "ok", ok, need == src.size, flush=True)


if __name__ == "__main__":
    main()
