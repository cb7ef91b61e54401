#!/usr/bin/env python3
"""Development: config 4 through qh_decode_sections_batch and
qh_encode_sections_batch on the device, five calls each 2 ms apart, for a
rocprofv3 --kernel-trace --memory-copy-trace run; with an argument (the
trace directory) prints the timeline of the 4th call of each pipeline
(kernel / copy start and end from the call's first event, us, and the gaps
between them)."""
import csv
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run():
    import numpy as np
    import torch
    from nghttp3_amd import HuffmanBatchCodec, qpack
    src, blocks, plain, strs, lines, ls = qpack.synth_field_sections(0x5EED0004, 65536)
    d_src = torch.from_numpy(np.ascontiguousarray(src)).cuda()
    d_blk = torch.from_numpy(blocks.view(np.int64).reshape(-1, 2).copy()).cuda()
    codec = HuffmanBatchCodec(0)
    fsd = qpack.FieldSectionDecoder(codec=codec, dtable0=True)
    b = fsd.decode_blocks_dev(d_src, d_blk)
    fse = qpack.FieldSectionEncoder(codec=codec)
    e_plain = torch.from_numpy(np.ascontiguousarray(plain)).cuda()
    e_strs = torch.from_numpy(strs.view(np.int64).reshape(-1, 2).copy()).cuda()
    e_lines = torch.from_numpy(np.ascontiguousarray(lines).view(np.uint8).copy()).cuda()
    e_ls = torch.from_numpy(ls.astype(np.int32)).cuda()
    e_dst = torch.empty(src.size + 64, dtype=torch.uint8, device="cuda")
    e_sec = torch.empty((blocks.size, 2), dtype=torch.int64, device="cuda")
    fse.encode_sections_dev(e_plain, e_strs, e_lines, e_ls, e_dst, e_sec)
    torch.cuda.synchronize()
    res = {}
    for name, fn in (("decode", lambda: fsd.decode_blocks_dev(d_src, d_blk, b)),
                     ("encode", lambda: fse.encode_sections_dev(e_plain, e_strs, e_lines, e_ls, e_dst, e_sec))):
        ts = []
        for _ in range(5):
            time.sleep(0.003)
            a = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(round((time.perf_counter() - a) * 1e3, 4))
        res[name + "_ms"] = ts
    print(json.dumps(res), flush=True)


def summary(d):
    rows = []
    for name in ("run_kernel_trace.csv", "run_memory_copy_trace.csv"):
        p = os.path.join(d, name)
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            lab = ("K:" + r["Kernel_Name"].split("(")[0].replace("void ", "")[:44]) if "Kernel_Name" in r else r["Direction"]
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), lab))
    rows.sort()
    groups, cur = [], []
    for e in rows:
        if cur and e[0] - max(x[1] for x in cur) > 1_000_000:
            groups.append(cur)
            cur = []
        cur.append(e)
    groups.append(cur)
    # groups: setup, 5 decode calls, 5 encode calls: print the 4th of each
    for g in (groups[-7], groups[-2]):
        t0 = g[0][0]
        prev = t0
        for s, e, lab in g:
            print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  gap {(s - prev) / 1e3:6.1f}  {lab}")
            prev = max(prev, e)
        print(f"call {(max(x[1] for x in g) - t0) / 1e3:.1f} us, {len(g)} events")


if __name__ == "__main__":
    if len(sys.argv) > 1:
        summary(sys.argv[1])
    else:
        run()
