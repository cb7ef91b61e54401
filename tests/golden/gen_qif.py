#!/usr/bin/env python3
"""Regenerate tests/golden/netbsd.qif: the QIF the reference CLI writes for
its fuzz corpus file netbsd-hq.out.256.100.1 (`qpack decode -s 256 -m 100`),
computed by the oracle's restatement of the CLI (oracle/qpack_qif.py).  The
survey's run of the compiled reference produced an 18-block, 217-line QIF
from it; tests/test_qif.py checks the shape."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import qpack_qif  # noqa: E402


def main():
    data = open(os.path.join(HERE, "netbsd-hq.out.256.100.1"), "rb").read()
    qif = qpack_qif.decode_wire(data, 256, 100)
    open(os.path.join(HERE, "netbsd.qif"), "wb").write(qif)
    print(qif.count(b"\n"), "lines")


if __name__ == "__main__":
    main()
