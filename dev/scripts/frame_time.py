#!/usr/bin/env python3
"""Development: config 4 (65,536 synthetic blocks) through
qh_decode_sections_batch on the device with the library QHUFF_LIB names:
pipeline time and per-kernel HIP-event times, and a check that the results
match the product library's digest of the decoded strings."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import hashlib
    import numpy as np
    import torch
    from nghttp3_amd import HuffmanBatchCodec, qpack
    src, blocks, *_ = qpack.synth_field_sections(0x5EED0004, 65536)
    d_src = torch.from_numpy(np.ascontiguousarray(src)).cuda()
    d_blk = torch.from_numpy(blocks.view(np.int64).reshape(-1, 2).copy()).cuda()
    codec = HuffmanBatchCodec(0)
    fsd = qpack.FieldSectionDecoder(codec=codec, dtable0=True)
    b = fsd.decode_blocks_dev(d_src, d_blk)
    torch.cuda.synchronize()
    ns = int(b["nspans"])
    dig = hashlib.sha256(b["strs"][:ns].cpu().numpy().tobytes() + b["spans"][:ns].cpu().numpy().tobytes() +
                         b["lines"][:int(b["nlines"]) * 24].cpu().numpy().tobytes()).hexdigest()[:16]
    reps = 20
    torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(reps):
        fsd.decode_blocks_dev(d_src, d_blk, b)
    torch.cuda.synchronize()
    t = (time.perf_counter() - a) / reps
    codec.enable_timing(True)
    for _ in range(5):
        fsd.decode_blocks_dev(d_src, d_blk, b)
    kt = {k: round(ms / max(c, 1) * 1e3, 2) for k, (c, ms) in codec.kernel_times().items()}
    print(json.dumps({"lib": os.path.basename(os.environ.get("QHUFF_LIB", "libqhuff.so")),
                      "pipeline_ms": round(t * 1e3, 4), "kernels_us": kt, "digest": dig}), flush=True)


if __name__ == "__main__":
    main()
