"""GPU legs of the encoder-side batch entries and the QIF driver:

* qh_encode_sections_batch (FieldSectionEncoder): byte for byte the host
  writer qh_qpack_write_sections on config-4-shaped sections, host and
  device memory, with and without prefixes;
* a C program (tests/c/sections_roundtrip.c) decodes the corpus file's 18
  field sections with qh_decode_sections_batch and re-encodes them with
  qh_encode_sections_batch: the reference encoder's bytes come back;
* the driver (nghttp3_amd/lib/qpack) in its GPU mode: the corpus decodes
  to the 217-line QIF, config 1 encodes to the oracle's bytes and round
  trips.
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import qpack_qif as oq
from nghttp3_amd import qif, qpack

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu

CORPUS = os.path.join(GOLDEN, "netbsd-hq.out.256.100.1")


@pytest.fixture(scope="module")
def enc(codec):
    return qpack.FieldSectionEncoder(codec=codec)


def test_encode_sections_matches_host_writer(enc):
    src, blocks, plain, strs, lines, line_start = qpack.synth_field_sections(0x5EED0C4, 3000)
    dst, secs = enc.encode_sections(plain, strs, lines, line_start)
    assert dst.tobytes() == src.tobytes()
    assert (secs["off"] == blocks["off"]).all() and (secs["len"] == blocks["len"]).all()
    # prefixes: arbitrary values, written as encoded
    n = line_start.size - 1
    pf = np.zeros(n, dtype=qpack.PREFIX_DTYPE)
    rng = np.random.default_rng(5)
    pf["ricnt"] = rng.integers(0, 1 << 20, n)
    pf["delta_base"] = rng.integers(0, 300, n)
    pf["sign"] = rng.integers(0, 2, n)
    dst2, secs2 = enc.encode_sections(plain, strs, lines, line_start, pf)
    for b in range(0, n, 97):
        sec = dst2[secs2["off"][b]:secs2["off"][b] + secs2["len"][b]].tobytes()
        head = qpack.put_varint(int(pf["ricnt"][b]), 8) + \
            qpack.put_varint(int(pf["delta_base"][b]), 7, 0x80 if pf["sign"][b] else 0)
        body = src[blocks["off"][b] + 2:blocks["off"][b] + blocks["len"][b]].tobytes()
        assert sec == head + body


@pytest.mark.parametrize("nsec", [1, 3, 4, 5, 63, 64, 65, 2047, 2048, 2049, 4097])
def test_encode_sections_at_scan_tile_edges(enc, nsec):
    """Section sizes (16 lanes per section, qh_k_encsec_size) go through one
    scan launch whose total comes back with the picked-string bytes in one
    copy (qh_k_scan_seg): section counts around a size wave's, a block's and
    the scan's 2048-entry tile edges still give the host writer's bytes."""
    src, blocks, plain, strs, lines, line_start = qpack.synth_field_sections(0x5EED0E0 + nsec, nsec)
    dst, secs = enc.encode_sections(plain, strs, lines, line_start)
    assert dst.tobytes() == src.tobytes()
    assert (secs["off"] == blocks["off"]).all() and (secs["len"] == blocks["len"]).all()


@pytest.mark.parametrize("bad", ["opcode", "value"])
def test_encode_sections_rejects_a_bad_line(enc, bad):
    """One unknown opcode or missing value string anywhere in the batch:
    QH_ERR_INVALID_ARGUMENT (the size pass's error word), as the host writer
    rejects it; the batch without it still encodes."""
    from nghttp3_amd import _lib
    src, blocks, plain, strs, lines, line_start = qpack.synth_field_sections(0x5EED0BD, 300)
    lines = lines.copy()
    with_value = np.flatnonzero(lines["value"] >= 0)
    k = int(with_value[len(with_value) // 3])
    if bad == "opcode":
        lines["opcode"][k] = 99
    else:
        lines["value"][k] = -1
    with pytest.raises(_lib.QhError) as ei:
        enc.encode_sections(plain, strs, lines, line_start)
    assert ei.value.code == _lib.QH_ERR_INVALID_ARGUMENT
    lines0 = qpack.synth_field_sections(0x5EED0BD, 300)[4]
    dst, _ = enc.encode_sections(plain, strs, lines0, line_start)
    assert dst.tobytes() == src.tobytes()


def test_encode_sections_device_resident(enc):
    import torch
    src, blocks, plain, strs, lines, line_start = qpack.synth_field_sections(0x5EED0C5, 2000)
    t_plain = torch.from_numpy(plain.copy()).cuda()
    t_strs = torch.from_numpy(strs.view(np.int64).reshape(-1, 2).copy()).cuda()
    t_lines = torch.from_numpy(lines.view(np.uint8).copy()).cuda()
    t_ls = torch.from_numpy(line_start.view(np.int32).copy()).cuda()
    n = line_start.size - 1
    t_dst = torch.zeros(src.size + 64, dtype=torch.uint8, device="cuda")
    t_sec = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    need = enc.encode_sections_dev(t_plain, t_strs, t_lines, t_ls, t_dst, t_sec)
    torch.cuda.synchronize()
    assert need == src.size
    assert t_dst[:need].cpu().numpy().tobytes() == src.tobytes()
    small = torch.zeros(16, dtype=torch.uint8, device="cuda")
    with pytest.raises(Exception):
        enc.encode_sections_dev(t_plain, t_strs, t_lines, t_ls, small, t_sec)


def test_encode_sections_device_resident_growing_batches():
    """The device form queues the picked strings' codes before it reads the
    totals, into scratch sized by earlier calls, and sizes its per-line
    offsets by the most lines seen so far: a fresh context fed batches that
    grow and shrink (each growth re-runs the size pass and the codes after
    the sync) writes the host writer's bytes every time."""
    import torch
    enc = qpack.FieldSectionEncoder(0)
    for nsec in (3, 2049, 10, 4097, 64):
        src, blocks, plain, strs, lines, line_start = qpack.synth_field_sections(0x5EED0C6 + nsec, nsec)
        t_plain = torch.from_numpy(plain.copy()).cuda()
        t_strs = torch.from_numpy(strs.view(np.int64).reshape(-1, 2).copy()).cuda()
        t_lines = torch.from_numpy(lines.view(np.uint8).copy()).cuda()
        t_ls = torch.from_numpy(line_start.view(np.int32).copy()).cuda()
        t_dst = torch.zeros(src.size + 64, dtype=torch.uint8, device="cuda")
        t_sec = torch.zeros((nsec, 2), dtype=torch.int64, device="cuda")
        need = enc.encode_sections_dev(t_plain, t_strs, t_lines, t_ls, t_dst, t_sec)
        torch.cuda.synchronize()
        assert need == src.size, nsec
        # (array_equal: a failing bytes comparison of this size makes pytest
        # diff megabytes)
        assert np.array_equal(t_dst[:need].cpu().numpy(), src), nsec
        sec = t_sec.cpu().numpy()
        assert (sec[:, 0] == blocks["off"].astype(np.int64)).all(), nsec


def test_c_program_decodes_and_reencodes_corpus_sections(tmp_path):
    exe = tmp_path / "sections_roundtrip"
    libdir = os.path.join(ROOT, "nghttp3_amd", "lib")
    subprocess.check_call(["gcc", "-std=c11", "-O1", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "c", "sections_roundtrip.c"),
                           "-L" + libdir, "-lqhuff", "-Wl,-rpath," + libdir,
                           "-Wl,-rpath-link,/opt/rocm/lib", "-o", str(exe)])
    out = subprocess.run([str(exe), CORPUS], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    words = out.stdout.split()
    assert words[0] == "ok" and int(words[1]) == 18 and int(words[2]) == 199
    assert int(words[3]) > 0


def _run(tmp_path, args, data, name="in"):
    src = tmp_path / name
    src.write_bytes(data)
    dst = tmp_path / (name + ".out")
    r = qif.run(args[:-1] + [args[-1], str(src), str(dst)])
    return r, (dst.read_bytes() if dst.exists() else None)


def test_driver_gpu_decodes_corpus(tmp_path):
    r, out = _run(tmp_path, ["-s", "256", "-m", "100", "decode"], open(CORPUS, "rb").read())
    assert r.returncode == 0, r.stderr
    assert out == open(os.path.join(GOLDEN, "netbsd.qif"), "rb").read()
    assert out.count(b"\n") == 217


def test_driver_gpu_config1_round_trip(tmp_path):
    t = qif.synth_config1()
    r, wire = _run(tmp_path, ["--time", "3", "encode"], t)
    assert r.returncode == 0, r.stderr
    assert wire == oq.encode_qif(t)
    r, back = _run(tmp_path, ["--time", "3", "decode"], wire, "wire")
    assert r.returncode == 0, r.stderr
    assert back == t
    assert '"path": "gpu"' in r.stderr


def test_driver_gpu_netbsd_summary_matches_reference_cli(tmp_path):
    """The GPU path prints the reference CLI's summary line for the corpus QIF
    at -s 0 (examples/qpack_encode.cc:209-216) and writes the
    scalar path's bytes."""
    from test_qif import REFERENCE_NETBSD_S0_LINE
    data = open(os.path.join(GOLDEN, "netbsd.qif"), "rb").read()
    r, out = _run(tmp_path, ["-s", "0", "encode"], data)
    assert r.returncode == 0, r.stderr
    assert REFERENCE_NETBSD_S0_LINE in r.stderr.strip().splitlines()
    r2, out2 = _run(tmp_path, ["--scalar", "-s", "0", "encode"], data, "scalar")
    assert r2.returncode == 0 and out == out2
