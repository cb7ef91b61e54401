"""QIF inputs for the driver (config 1): the interop corpus is not available
offline, so config 1 is a 1,024-field QIF
synthesised deterministically from the netbsd QIF (tests/golden/netbsd.qif,
the reference corpus file decoded): its blocks are repeated in order, each
copy's :path value gets a "?q=" query of 8-40 draws and every block gains a
cookie field of 20-80 draws, until the QIF holds exactly 1,024 fields.
Draws are splitmix64 (nghttp3_amd/synth.py) over the alphabet A without
its space (a QIF value loses its leading spaces).

The driver itself is nghttp3_amd/lib/qpack (csrc/qh_qif.cc); ``run`` calls
it as a child process.
"""
from __future__ import annotations

import os
import subprocess

from . import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NETBSD_QIF = os.path.join(ROOT, "tests", "golden", "netbsd.qif")
DRIVER = os.path.join(ROOT, "nghttp3_amd", "lib", "qpack")
CONFIG1_SEED = 0x5EED0001


def blocks_of(text: bytes):
    out, cur = [], []
    for line in text.split(b"\n"):
        if line == b"":
            if cur:
                out.append(cur)
            cur = []
        else:
            cur.append(line)
    if cur:
        out.append(cur)
    return out


def synth_config1(netbsd: bytes | None = None, seed: int = CONFIG1_SEED,
                  nfields: int = 1024) -> bytes:
    """-> QIF text of exactly nfields fields."""
    if netbsd is None:
        netbsd = open(NETBSD_QIF, "rb").read()
    base = blocks_of(netbsd)
    alpha = synth.ALPHABET_A.replace(b" ", b"")  # (QIF drops a value's leading spaces)
    pos = 0

    def take(k):
        nonlocal pos
        d = synth.draws(seed, pos, k)
        pos += k
        return d

    def text(lo, hi):
        n = lo + int(take(1)[0] % (hi - lo + 1))
        return bytes(alpha[int(x % len(alpha))] for x in take(n))

    out, total, b = [], 0, 0
    while total < nfields:
        lines = []
        for line in base[b % len(base)]:
            if line.startswith(b":path\t"):
                line = line + b"?q=" + text(8, 40)
            lines.append(line)
        lines.append(b"cookie\t" + text(20, 80))
        lines = lines[:nfields - total]
        total += len(lines)
        out.append(b"\n".join(lines) + b"\n\n")
        b += 1
    return b"".join(out)


def run(args, timeout=120):
    """The driver as a child process -> CompletedProcess (text stderr)."""
    return subprocess.run([DRIVER] + list(args), capture_output=True, text=True,
                          timeout=timeout)
