#!/usr/bin/env python3
"""Development: the long-value section strings through qh_decode_batch
(device, each decoder) against the oracle, reporting the failing strings'
lengths and kinds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import oracle
    from oracle import qpack_frame as ref
    from nghttp3_amd import HuffmanBatchCodec, pack_strings
    from test_gpu_qpack import _long_value_sections
    src, blocks, kinds = _long_value_sections(0x5EED0410, 240)
    encs = []
    for o, n in zip(blocks["off"], blocks["len"]):
        sec = bytes(src[int(o):int(o) + int(n)])
        _, _, _, spans = ref.scan_field_section(sec)
        for so, sn, fl in spans:
            if fl & ref.SPAN_HUFFMAN:
                encs.append(sec[so:so + sn])
    for dec in ("windows", "sorted", "waves"):
        c = HuffmanBatchCodec(0)
        c.set_decoder(dec)
        es, sp = pack_strings(encs)
        dst, out = c.decode_host(es, sp)
        bad = []
        for i, e in enumerate(encs):
            st, want = oracle.decode_one(e)
            got = bytes(dst[int(out["off"][i]):int(out["off"][i]) + int(out["len"][i])]) if out["status"][i] == 0 else b""
            if int(out["status"][i]) != st or (st == 0 and got != want):
                bad.append((i, len(e), st, int(out["status"][i]), "bin" if want and max(want) > 126 else "txt",
                            len(want), len(got), next((k for k in range(min(len(want), len(got))) if want[k] != got[k]), None)))
        print(dec, len(encs), "strings,", len(bad), "bad", bad[:12], flush=True)
        c.close()


if __name__ == "__main__":
    main()
