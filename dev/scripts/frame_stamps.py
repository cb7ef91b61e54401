#!/usr/bin/env python3
"""Development: phase timers of qh_k_frame_count on config 4 (65,536
blocks), from the stamps build (make frst -> libqhuff_frst.so, QHUFF_LIB):
s_memtime cycles per wave in stage (DMA + wait), parse, look-back, stores."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("QHUFF_LIB", os.path.join(ROOT, "nghttp3_amd", "lib", "libqhuff_frst.so"))


def main():
    import numpy as np
    import torch
    from nghttp3_amd import HuffmanBatchCodec, qpack, _lib
    lib = _lib.load()
    lib.qh_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    src, blocks, *_ = qpack.synth_field_sections(0x5EED0004, 65536)
    d_src = torch.from_numpy(np.ascontiguousarray(src)).cuda()
    d_blk = torch.from_numpy(blocks.view(np.int64).reshape(-1, 2).copy()).cuda()
    codec = HuffmanBatchCodec(0)
    fsd = qpack.FieldSectionDecoder(codec=codec, dtable0=True)
    b = fsd.decode_blocks_dev(d_src, d_blk)
    torch.cuda.synchronize()
    st = (ctypes.c_uint64 * 16)()
    reps = 5
    lib.qh_debug_stamps(st, 1)
    for _ in range(reps):
        fsd.decode_blocks_dev(d_src, d_blk, b)
    torch.cuda.synchronize()
    lib.qh_debug_stamps(st, 1)
    waves = reps * 65536 // 64
    names = ["stage", "parse", "lookback", "stores"]
    print(json.dumps({"cycles_per_wave": {names[k]: round(st[k] / waves) for k in range(4)}}), flush=True)


if __name__ == "__main__":
    main()
