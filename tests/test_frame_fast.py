"""The GPU framing count pass's fast parse (nghttp3_amd/csrc/qh_frame_fast.h,
compiled here for the host) gives scan_section's counts, prefixes and line
starts for every block it answers for (tests/c/frame_fast_check.cc), on the
config-4 synthetic corpus and on a copy with random byte flips; it answers
for every clean block.  CPU only: the GPU tests check the kernel."""
import os
import subprocess

import numpy as np

from nghttp3_amd import qpack

from conftest import ROOT


def _build(tmp_path):
    exe = tmp_path / "frame_fast_check"
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                           "-I", os.path.join(ROOT, "nghttp3_amd", "csrc"),
                           os.path.join(ROOT, "tests", "c", "frame_fast_check.cc"), "-o", str(exe)])
    return exe


def _run(exe, tmp_path, src, blocks):
    s, b = tmp_path / "src.bin", tmp_path / "blk.bin"
    np.ascontiguousarray(src).tofile(s)
    pairs = np.zeros((blocks.size, 2), dtype=np.uint64)
    pairs[:, 0] = blocks["off"]
    pairs[:, 1] = blocks["len"]
    pairs.tofile(b)
    out = subprocess.run([str(exe), str(s), str(b)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return [int(x) for x in out.stdout.split()]


def test_fast_parse_matches_scan_section(tmp_path):
    exe = _build(tmp_path)
    src, blocks, *_ = qpack.synth_field_sections(0x5EED00F4, 20000)
    n, fast, mism, clean_fb = _run(exe, tmp_path, src, blocks)
    assert n == 20000 and fast == n and mism == 0 and clean_fb == 0
    # random byte flips: every block still answered for is answered right,
    # and every block scan_section accepts is answered for
    bad = np.array(src, copy=True)
    rng = np.random.default_rng(0x5EED00F5)
    k = rng.choice(bad.size, 8000, replace=False)
    bad[k] = rng.integers(0, 256, k.size)
    n, fast, mism, clean_fb = _run(exe, tmp_path, bad, blocks)
    assert mism == 0 and clean_fb == 0 and fast < n
