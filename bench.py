#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: "GiB/s device-resident QPACK Huffman
encode+decode, 1M strings; bit-exact".

One step = one round trip of the hot path over one batch already resident in
HBM: qh_encode_batch (encode_count -> scan -> encode) of the rank's strings,
then qh_decode_batch of the encoded strings.  The batch is config 3
(BASELINE configs[2]): 2^20 strings per GPU, 8-256 B, alphabet A, seed
0x5EED0003.  With N GPUs the job is ONE batch of N x 2^20 strings, split
into contiguous string ranges of equal bytes (nghttp3_amd/shard.py
split_by_bytes); each rank generates and processes
its own range (no string data crosses xGMI), and one all-gather of a u64
places every rank's encoded output in the global layout (output_offsets).
value = plaintext bytes of all ranks x steps / max-over-ranks wall time of
the timed region (barrier + synchronize on both sides), GiB/s.  The decoded
output is checked against the input after the timed region (bit-exact), and
per-kernel HIP-event times from a second pass give the roofline of the
dominant kernel.

`extra` also carries (never the value): config 5 (16M Zipf-length strings
1..4096 B, split by bytes over the ranks), config 4 (65,536 header blocks at
dynamic table 0 through qh_decode_sections_batch, split by block), alphabet
U, the PCIe-inclusive host path, and the CPU baseline of BASELINE.md (the
oracle restatement of lib/nghttp3_qpack_huffman.c, -O2 -mavx2, at T = 1 and
T = all cores, median of 5; rank 0 at N = 1).

`python bench.py --gpus N` starts its N ranks itself (torch.distributed.run,
before any GPU call) unless it already runs under a launcher (WORLD_SIZE).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak, MI355X_MICROARCH.md chip table
GIB = float(1 << 30)
METRIC = "GiB/s device-resident QPACK Huffman encode+decode, 1M strings; bit-exact"
SEED5, SEED4 = 0x5EED0005, 0x5EED0004


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # (200 steps: the timed region's fixed cost -- the first launch after the
    # synchronize and the closing synchronize, ~0.3 ms -- is 4.5% of 20
    # round trips and 0.5% of 200; dev/scripts/step_host.py)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    # (no option may be a prefix of a torch.distributed.run option: --n, --lo ...)
    ap.add_argument("--strings", type=int, default=1 << 20, help="strings per GPU (config 3)")
    ap.add_argument("--min-len", type=int, default=8)
    ap.add_argument("--max-len", type=int, default=256)
    ap.add_argument("--alphabet", choices=["A", "U"], default="A")
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EED0003)
    ap.add_argument("--c5-strings", type=int, default=16 << 20, help="config 5: strings in all")
    ap.add_argument("--c4-blocks", type=int, default=65536, help="config 4: header blocks in all")
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--cpu-t1-strings", type=int, default=1 << 18)
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL over xGMI; gloo only to rehearse ranks on one device")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank on device 0 (multi-rank rehearsal on a 1-GPU box)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the same-run counter passes (rocprofv3 FETCH_SIZE / WRITE_SIZE) and the LDS-chain probe")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the config 4 / config 5 / alphabet-U legs in extra")
    ap.add_argument("--profile-only", action="store_true",
                    help="just run warmup+steps (for rocprofv3), minimal reporting")
    return ap.parse_args()


def spawn(args) -> int:
    """N ranks on this node, one per GPU, before anything touches the GPU."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


class Dist:
    """Barrier and small reductions over the ranks (RCCL, or gloo on CPU
    tensors for the rehearsal mode)."""

    def __init__(self, torch, world, backend, dev):
        self.torch, self.world = torch, world
        self.dist = None
        self.cdev = dev if backend == "nccl" else "cpu"
        if world > 1:
            import torch.distributed as dist
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=dev)
            else:
                dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def _red(self, x, op):
        t = self.torch.tensor([float(x)], dtype=self.torch.float64, device=self.cdev)
        if self.dist:
            self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x):
        return self._red(x, self.dist.ReduceOp.MAX if self.dist else None)

    def sum(self, x):
        return self._red(x, self.dist.ReduceOp.SUM if self.dist else None)

    def offsets(self, local):
        from nghttp3_amd import shard
        return shard.output_offsets(local, self.dist, self.cdev)

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


CHAIN_JSON = os.path.join(ROOT, "profiles", "r03", "lds_chain.json")
LDS_B32_TBPS = 75.0  # ds_read_b32 aggregate, every CU streaming (MI355X_MICROARCH.md LDS section)


def lds_secondary(kernel, avg_us, plain, chain=None):
    """The decoder's second ceiling: its algorithmic table lookups per
    launch -- one per decoded symbol, the plaintext bytes of this run's batch
    (huffman.c:87-124 makes two per byte of input instead) -- over its time,
    against the measured rate of dependent LDS lookup chains
    (dev/ubench/lds_chain.hip at its best occupancy: a property of the chip,
    like the HBM peak) and the guide's ds_read_b32 aggregate."""
    if kernel != "qh_k_dec_peek":
        return None
    src = "this run (dev/ubench/lds_chain)"
    if chain is None:
        try:
            chain = json.load(open(CHAIN_JSON))
            src = "profiles/r03/lds_chain.json"
        except Exception:
            return None
    rate = plain / (avg_us * 1e-6)
    agg = LDS_B32_TBPS * 1e12 / 4
    return {"unit": "lookups/s", "lookups_per_launch": int(plain), "achieved": round(rate, -6),
            "chained_rate": chain["chained_lookups_per_s_best"],
            "frac_of_chained_rate": round(rate / chain["chained_lookups_per_s_best"], 4),
            "ds_read_b32_aggregate": agg, "frac_of_aggregate": round(rate / agg, 4),
            "source": "lookups: decoded symbols of this run; chained rate: " + src}


def leg_counters(args, kernel="qh_k_dec_peek", coalesced=None):
    """Same-run evidence for the roofline: two rocprofv3 counter passes over a
    profile-only child of this bench (config 3, the same batch and library:
    FETCH_SIZE alone, then WRITE_SIZE alone -- gfx950 collects one TCC group
    per pass), each under its own time limit, from /tmp (MI355X_MICROARCH.md
    HBM section: FETCH_SIZE counts 64-byte requests where wide reads are 128
    bytes, so it is doubled; both in KiB), and the dependent-LDS-lookup
    ceiling from dev/ubench/lds_chain on this box.  The child is a process of
    its own (rocprofv3 -- python3 ...), started before nothing but a fork.

    FETCH_SIZE is calibrated per access pattern (dev/ubench/rd_gran.hip,
    profiles/r05/rd_gran_fetch.txt: 256 MiB read once): coalesced 16-byte
    lane loads report 0.50 of the bytes (the guide's x2), but per-lane
    16-byte loads walking separate regions -- the decoder's input DMAs and
    string-start loads -- report 1.06 of them (each 64-byte request counted
    whole).  So with `coalesced` = the kernel's bytes read by coalesced loads
    (the decoder's spans, 16 N), fetch = raw + coalesced / 2; without it, the
    guide's x2."""
    import csv
    import glob
    import shutil
    import tempfile
    out = {"kernel": kernel}
    chain = None
    exe = os.path.join(ROOT, "dev", "ubench", "lds_chain")
    if os.path.exists(exe):
        try:
            r = subprocess.run([exe], capture_output=True, text=True, timeout=90)
            js = [l for l in r.stdout.splitlines() if l.startswith("{")]
            if r.returncode == 0 and js:
                chain = json.loads(js[-1])
        except Exception as e:  # (reported, not fatal)
            out["lds_chain_error"] = str(e)[:200]
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    vals = {}
    tmp = tempfile.mkdtemp(prefix="qh_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(tmp, ctr)
        cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "run", "--",
               sys.executable, os.path.abspath(__file__), "--profile-only", "--steps", "3", "--warmup", "1",
               "--strings", str(args.strings), "--min-len", str(args.min_len), "--max-len", str(args.max_len),
               "--alphabet", args.alphabet, "--seed", hex(args.seed)]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd="/tmp", env=env)
        except subprocess.TimeoutExpired:
            out["error"] = f"{ctr} pass timed out"
            break
        xs = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "")
                    if kernel in name and row.get("Counter_Name") == ctr:
                        xs.append(float(row["Counter_Value"]))
        if r.returncode != 0 or not xs:
            out["error"] = f"{ctr} pass rc={r.returncode}, {len(xs)} rows: " + r.stderr[-300:]
            break
        vals[ctr] = sum(xs) / len(xs)
        out[ctr.lower() + "_launches"] = len(xs)
    shutil.rmtree(tmp, ignore_errors=True)
    if len(vals) == 2:
        raw = 1024 * vals["FETCH_SIZE"]
        out["fetch_raw_bytes"] = round(raw)
        if coalesced is not None:
            out["fetch_bytes"] = round(raw + coalesced / 2)
            out["correction"] = (f"FETCH_SIZE calibrated per pattern (dev/ubench/rd_gran): per-lane 16-byte loads "
                                 f"x1, the {coalesced} bytes of coalesced span loads x2; KiB -> bytes")
        else:
            out["fetch_bytes"] = round(2 * raw)
            out["correction"] = "FETCH_SIZE x2 (guide: coalesced wide reads; this kernel uncalibrated); KiB -> bytes"
        out["write_bytes"] = round(1024 * vals["WRITE_SIZE"])
        out["hbm_bytes_per_launch"] = out["fetch_bytes"] + out["write_bytes"]
    return out, chain


def _cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except Exception:
        pass
    return None


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch

    from nghttp3_amd import HuffmanBatchCodec, shard, synth
    from nghttp3_amd import qpack_huffman as q

    devno = 0 if args.one_device else local_rank
    torch.cuda.set_device(devno)
    dev = torch.device("cuda", devno)
    D = Dist(torch, world, args.dist_backend, dev)
    codec = HuffmanBatchCodec(device=devno)  # on torch's current stream
    alphabet = synth.ALPHABET_A if args.alphabet == "A" else synth.ALPHABET_U

    def timed(fn, reps):
        """Max-over-ranks seconds per call of fn (barrier + sync both sides)."""
        D.barrier()
        torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        D.barrier()
        return D.max((time.perf_counter() - a) / reps)

    def roundtrip_ok(src, spans, dec, dout, chunk=1 << 20):
        """Decoded strings == the input strings, in chunks of strings."""
        n = spans.shape[0]
        ln_all = spans[:, 1] & 0xFFFFFFFF
        if not bool(((dout[:, 1] >> 32) == 0).all()) or not bool(((dout[:, 1] & 0xFFFFFFFF) == ln_all).all()):
            return False
        for i0 in range(0, n, chunk):
            i1 = min(n, i0 + chunk)
            ln = ln_all[i0:i1]
            tot = int(ln.sum().item())
            if tot == 0:
                continue
            starts = torch.repeat_interleave(torch.cumsum(ln, 0) - ln, ln)
            pos = torch.arange(tot, device=dev, dtype=torch.int64) - starts
            if not bool((dec[torch.repeat_interleave(dout[i0:i1, 0], ln) + pos] ==
                         src[torch.repeat_interleave(spans[i0:i1, 0], ln) + pos]).all()):
                return False
        return True

    def buffers(src, spans):
        n = spans.shape[0]
        ln = spans[:, 1] & 0xFFFFFFFF
        enc = torch.empty(max(int(((ln * 30 + 7) // 8).sum().item()), 1), dtype=torch.uint8, device=dev)
        eout = torch.empty((n, 2), dtype=torch.int64, device=dev)
        codec.encode_dev(src, spans, enc, eout)
        torch.cuda.synchronize()
        elen = eout[:, 1] & 0xFFFFFFFF
        cap = int(q.decode_slot_size(elen).sum().item())
        dec = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
        dout = torch.empty((n, 2), dtype=torch.int64, device=dev)
        return enc, eout, int(elen.sum().item()), dec, dout

    # ---- config 3: one global batch of world x n strings, split by bytes ----
    lens_all = synth.lengths(args.seed, args.strings * world, args.min_len, args.max_len)
    b0, b1 = shard.split_by_bytes(lens_all, world)[rank]
    first = int(lens_all[:b0].sum(dtype=np.uint64))
    my_ln = lens_all[b0:b1]
    spans, total = codec.spans_to_device(my_ln)
    src = codec.synth_fill(args.seed, first, total, alphabet)
    n = spans.shape[0]
    enc, eout, enc_bytes, dec, dout = buffers(src, spans)

    def step():
        codec.encode_dev(src, spans, enc, eout)
        codec.decode_dev(enc, eout, dec, dout)

    for _ in range(args.warmup):
        step()
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    D.barrier()
    elapsed_max = D.max(time.perf_counter() - t0)

    if args.profile_only:
        if rank == 0:
            print(json.dumps({"profile_only": True, "ms_per_step": 1e3 * elapsed_max / args.steps}))
        D.close()
        return

    bad = D.sum(0.0 if roundtrip_ok(src, spans, dec, dout) else 1.0)
    enc_global_off = D.offsets(enc_bytes)  # this shard's place in the global encoded layout

    # ---- per-kernel HIP-event times over a second pass ----
    codec.enable_timing(True)
    for _ in range(args.steps):
        step()
    ktimes = codec.kernel_times()
    codec.enable_timing(False)
    t_dec = timed(lambda: codec.decode_dev(enc, eout, dec, dout), args.steps)
    t_enc = timed(lambda: codec.encode_dev(src, spans, enc, eout), args.steps)
    cold = None if args.no_configs else leg_cold(torch, codec, src, spans, enc, eout, dec, dout, total, dev)
    # packed device output (QH_WHERE_DEVICE_DENSE: the slot decode, then a
    # packing pass), reported beside the slot layout
    t_dense = timed(lambda: codec.decode_dev(enc, eout, dec, dout, dense=True), args.steps)
    dense_ok = D.sum(0.0 if roundtrip_ok(src, spans, dec, dout) else 1.0) == 0
    total_all = D.sum(float(total))

    # ---- two batches in flight (reported beside the value, never as it): a
    # second context on its own HIP stream with its own output buffers, the
    # round trips alternating between the two contexts, so step i's decode
    # can run beside step i + 1's encode and each kernel's tail overlaps the
    # other stream's work.  Every step is still a whole encode + decode. ----
    two_ctx = None
    if not args.no_configs:
        codec2 = HuffmanBatchCodec(device=devno, stream=torch.cuda.Stream(dev))
        enc2 = torch.empty_like(enc)
        eout2 = torch.empty_like(eout)
        dec2 = torch.empty_like(dec)
        dout2 = torch.empty_like(dout)
        pair = ((codec, enc, eout, dec, dout), (codec2, enc2, eout2, dec2, dout2))

        def step2(i):
            cx, e_, eo_, d_, do_ = pair[i & 1]
            cx.encode_dev(src, spans, e_, eo_)
            cx.decode_dev(e_, eo_, d_, do_)

        for i in range(2 * args.warmup):
            step2(i)
        t2 = timed(lambda: [step2(i) for i in range(args.steps)], 1) / args.steps
        ok2 = roundtrip_ok(src, spans, dec, dout) and roundtrip_ok(src, spans, dec2, dout2)
        two_ctx = {"GiBps": round(total_all / t2 / GIB, 2), "ms_per_step": round(t2 * 1e3, 4),
                   "vs_value": round(elapsed_max / args.steps / t2, 3),
                   "bit_exact": D.sum(0.0 if ok2 else 1.0) == 0,
                   "how": "two contexts (own stream and buffers each), round trips alternating"}
        del codec2, enc2, eout2, dec2, dout2, pair
    value = total_all * args.steps / elapsed_max / GIB

    def kernel_table(ktimes, n, plain, encb):
        algo = {  # algorithmic HBM bytes per launch
            "qh_k_dec_peek": encb + plain + 32 * n,          # E + D + 16 B span in + 16 B out
            "qh_k_dec_reserve": 16 * n,                      # spans in
            "qh_k_enc_lens_stream": plain + 16 * n + 8 * n,  # D + spans in + len/status out
            "qh_k_enc_lanes": plain + encb + 16 * n + 8 * n + 16 * n,  # D + E + spans
            "qh_k_encw": plain + encb + 16 * n + 16 * n,     # D + E + spans in + out
            "qh_k_sched_count": 16 * n,                      # spans in
            "qh_k_sched_scatter": 16 * n + 24 * n,           # spans in, records out
        }
        kern = {}
        for name, (cnt, ms) in ktimes.items():
            avg_ms = ms / max(cnt, 1)
            gbps = algo.get(name, 0) / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
            kern[name] = {"launches": cnt, "avg_us": round(avg_ms * 1e3, 2),
                          "algo_bytes": algo.get(name), "achieved_GBps": round(gbps, 1)}
        return kern

    kern = kernel_table(ktimes, n, total, enc_bytes)
    dom = max(kern, key=lambda k: kern[k]["avg_us"] * kern[k]["launches"]) if kern else None
    traffic = None
    counters, chain = None, None
    if rank == 0 and world == 1 and dom and not args.no_pmc:
        counters, chain = leg_counters(args, dom, 16 * n if dom == "qh_k_dec_peek" else None)
        traffic = counters.get("hbm_bytes_per_launch")
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if traffic is None and dom and os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            entry = pmc.get("kernels", {}).get(dom)
            if entry and pmc.get("n") == n and pmc.get("alphabet") == args.alphabet:
                traffic = entry.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    roofline = None
    if dom:
        ach = kern[dom]["achieved_GBps"]
        roofline = {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBPS,
                    "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": traffic,
                    "algo_bytes_per_launch": kern[dom]["algo_bytes"],
                    "avg_us": kern[dom]["avg_us"],
                    "traffic_source": ("this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes "
                                       "(extra.counters)" if counters and counters.get("hbm_bytes_per_launch")
                                       else "profiles/pmc_traffic.json" if traffic else None)}
        if traffic:
            roofline["traffic_over_algo"] = round(traffic / max(kern[dom]["algo_bytes"] or 1, 1), 3)
        sec = lds_secondary(dom, kern[dom]["avg_us"], total, chain)
        if sec:
            roofline["secondary"] = sec
            if sec["frac_of_chained_rate"] > roofline["frac"]:
                roofline["bound"] = "lds-chain"
        # neither ceiling near: the kernel waits on latency (dependent
        # lookups, scattered requests), not on a throughput limit
        if max(roofline["frac"], sec["frac_of_chained_rate"] if sec else 0.0) < 0.5:
            roofline["bound"] = "latency"

    # ---- config 5: 16M Zipf strings (s = 1.2, 1..4096 B), split by bytes ----
    config5 = None
    if not args.no_configs and args.c5_strings:
        ln5 = synth.zipf_lengths(SEED5, args.c5_strings, 1, 4096, 1.2)
        c0, c1 = shard.split_by_bytes(ln5, world)[rank]
        f5 = int(ln5[:c0].sum(dtype=np.uint64))
        sp5, tot5 = codec.spans_to_device(ln5[c0:c1])
        src5 = codec.synth_fill(SEED5, f5, tot5, synth.ALPHABET_A)
        enc5, eout5, eb5, dec5, dout5 = buffers(src5, sp5)
        # the shipped decoder (QH_DECODER_SORTED: the length-class schedule)
        # and the one-pass encoder (QH_ENCODER_FUSED); the wave decoder's and
        # the window encoder's times on the same batch are reported beside
        # them, and their bytes must agree
        codec.set_decoder("waves")
        td5_alt = timed(lambda: codec.decode_dev(enc5, eout5, dec5, dout5), 3)
        ok5_alt = roundtrip_ok(src5, sp5, dec5, dout5)
        codec.set_decoder("sorted")
        dec5.zero_()
        codec.decode_dev(enc5, eout5, dec5, dout5)
        ok5 = roundtrip_ok(src5, sp5, dec5, dout5) and ok5_alt
        codec.set_encoder("windows")
        te5_alt = timed(lambda: codec.encode_dev(src5, sp5, enc5, eout5), 3)
        enc5_alt, eout5_alt = enc5[:eb5].clone(), eout5.clone()
        codec.set_encoder("fused")
        enc5.zero_()
        codec.encode_dev(src5, sp5, enc5, eout5)
        ok5 = ok5 and bool(torch.equal(enc5[:eb5], enc5_alt)) and bool(torch.equal(eout5, eout5_alt))
        del enc5_alt, eout5_alt
        te5 = timed(lambda: codec.encode_dev(src5, sp5, enc5, eout5), 5)
        td5 = timed(lambda: codec.decode_dev(enc5, eout5, dec5, dout5), 5)
        # the library defaults on the same batch (QH_ENCODER_AUTO, the
        # window decoder with its per-block plan)
        codec.set_encoder("auto")
        codec.set_decoder("windows")
        te5_def = timed(lambda: codec.encode_dev(src5, sp5, enc5, eout5), 3)
        td5_def = timed(lambda: codec.decode_dev(enc5, eout5, dec5, dout5), 3)
        codec.set_decoder("sorted")
        codec.enable_timing(True)
        for _ in range(3):
            codec.decode_dev(enc5, eout5, dec5, dout5)
        k5 = kernel_table(codec.kernel_times(), sp5.shape[0], tot5, eb5)
        codec.enable_timing(False)
        codec.set_encoder("auto")
        codec.set_decoder("windows")
        d5 = k5.get("qh_k_dec_peek", {})
        p5, e5 = D.sum(float(tot5)), D.sum(float(eb5))
        dec_gbps_min = D.max(-d5.get("achieved_GBps", 0.0))
        config5 = {"strings": args.c5_strings, "plain_bytes": int(p5), "enc_bytes": int(e5),
                   "lengths": "Zipf s=1.2 over 1..4096 B (synth.zipf_lengths, seed 0x5EED0005), "
                              "mean %.1f B" % float(ln5.mean()),
                   "shards": world, "strings_rank0": int(c1 - c0) if rank == 0 else None,
                   "encode_GiBps": round(p5 / te5 / GIB, 2), "decode_GiBps": round(p5 / td5 / GIB, 2),
                   "decoder": "sorted (QH_DECODER_SORTED: length-class schedule + qh_k_dec_peek windows)",
                   "decode_GiBps_wave_decoder": round(p5 / D.max(td5_alt) / GIB, 2),
                   "encoder": "fused (qh_k_encw: lengths and codes in one pass over the plaintext)",
                   "encode_GiBps_window_encoder": round(p5 / D.max(te5_alt) / GIB, 2),
                   "encode_GiBps_default_auto": round(p5 / D.max(te5_def) / GIB, 2),
                   "decode_GiBps_default_windows_plan": round(p5 / D.max(td5_def) / GIB, 2),
                   "decode_kernels_us_rank0": {k: v["avg_us"] for k, v in k5.items()},
                   "round_trip_GiBps": round(p5 / (te5 + td5) / GIB, 2),
                   "decode_kernel_us_rank0": d5.get("avg_us"),
                   "decode_kernel_GBps_min_rank": round(-dec_gbps_min, 1),
                   "decode_kernel_frac_min_rank": round(-dec_gbps_min / HBM_PEAK_GBPS, 4),
                   "bit_exact": D.sum(0.0 if ok5 else 1.0) == 0}
        del src5, sp5, enc5, eout5, dec5, dout5

    # ---- config 4: 65,536 header blocks at dynamic table 0, split by block ----
    config4 = None
    if not args.no_configs and args.c4_blocks:
        config4 = leg_config4(args, torch, dev, codec, D, rank, world, timed)

    # ---- config 1: the QIF driver on the 1,024-field QIF (rank 0, N = 1) ----
    config1 = None
    if rank == 0 and world == 1 and not args.no_configs:
        config1 = leg_config1()

    # ---- alphabet U (config 3 shape), rank 0 alone ----
    configU = None
    if rank == 0 and world == 1 and not args.no_configs:
        u_src, u_spans, u_total = codec.synth(args.seed, args.strings, args.min_len, args.max_len, synth.ALPHABET_U)
        u_enc, u_eout, u_eb, u_dec, u_dout = buffers(u_src, u_spans)
        codec.set_encoder("windows")
        tue_win = timed(lambda: codec.encode_dev(u_src, u_spans, u_enc, u_eout), 3)
        codec.set_encoder("auto")
        tue_def = timed(lambda: codec.encode_dev(u_src, u_spans, u_enc, u_eout), 3)
        codec.set_encoder("fused")  # (binary text: the one-pass encoder, the sorted decoder)
        codec.set_decoder("sorted")
        u_enc.zero_()
        codec.encode_dev(u_src, u_spans, u_enc, u_eout)
        codec.decode_dev(u_enc, u_eout, u_dec, u_dout)
        u_ok = roundtrip_ok(u_src, u_spans, u_dec, u_dout)
        tue = timed(lambda: codec.encode_dev(u_src, u_spans, u_enc, u_eout), 5)
        tud = timed(lambda: codec.decode_dev(u_enc, u_eout, u_dec, u_dout), 5)
        codec.set_decoder("windows")
        tud_win = timed(lambda: codec.decode_dev(u_enc, u_eout, u_dec, u_dout), 3)
        codec.set_encoder("auto")
        configU = {"strings": args.strings, "plain_bytes": u_total, "enc_bytes": u_eb,
                   "encode_GiBps": round(u_total / tue / GIB, 2), "encoder": "fused",
                   "encode_GiBps_window_encoder": round(u_total / tue_win / GIB, 2),
                   "encode_GiBps_default_auto": round(u_total / tue_def / GIB, 2),
                   "decode_GiBps": round(u_total / tud / GIB, 2), "decoder": "sorted",
                   "decode_GiBps_window_decoder": round(u_total / tud_win / GIB, 2),
                   "decode_GiBps_default_windows_plan": round(u_total / tud_win / GIB, 2),
                   "round_trip_GiBps": round(u_total / (tue + tud) / GIB, 2), "bit_exact": u_ok}
        del u_src, u_spans, u_enc, u_eout, u_dec, u_dout

    # ---- PCIe-inclusive host path (reported, never the value) ----
    host_path = None
    if world == 1 and not args.no_host_path:
        host_path = leg_host_path(torch, codec, q, enc, eout, enc_bytes, total, n, dev)
    elif not args.no_host_path:
        # every rank its shard from host memory, over its own link
        host_path = leg_host_path_ranks(torch, codec, q, src, enc, eout, enc_bytes, total, n, dev, D, rank, world)

    # ---- CPU baseline (rank 0, N = 1) ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = leg_cpu(args, src, spans, total, n)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed_max / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64, nghttp3_amd/synth.py)",
            "config": {"workload": "config 3: Huffman encode+decode round trip, 2^20 strings "
                                   f"{args.min_len}-{args.max_len} B per GPU, alphabet {args.alphabet}; one "
                                   "batch of N x 2^20 strings split by bytes over the N GPUs",
                       "strings_per_gpu": args.strings, "strings_rank0": n, "plain_bytes_rank0": total,
                       "enc_bytes_rank0": enc_bytes, "plain_bytes_all": int(total_all),
                       "seed": hex(args.seed), "parallelism": f"shard{world}",
                       "dist_backend": args.dist_backend if world > 1 else None},
            "bit_exact": bad == 0,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "extra": {"decode_GiBps": round(total_all / t_dec / GIB, 2),
                      "encode_GiBps": round(total_all / t_enc / GIB, 2),
                      "decode_dense_GiBps": round(total_all / t_dense / GIB, 2),
                      "decode_dense_bit_exact": dense_ok,
                      "decode_cold_GiBps": cold and cold["decode_cold_GiBps"],
                      "encode_cold_GiBps": cold and cold["encode_cold_GiBps"],
                      "cold_input": cold,
                      "two_batches_in_flight": two_ctx,
                      "enc_global_offset_rank0": enc_global_off,
                      "kernels": kern, "host_path": host_path, "counters": counters,
                      "config5_zipf": config5, "config4_qpack_blocks": config4,
                      "config1_qif": config1,
                      "config3_alphabet_U": configU},
        }
        print(json.dumps(line), flush=True)
    D.close()


def leg_cold(torch, codec, src, spans, enc, eout, dec, dout, total, dev, reps=9):
    """The decoder and the encoder on a cold input: in
    deployment the decoder's input arrives by H2D from a QUIC stream buffer,
    not from an encoder that just wrote it on the same GPU.  Before each
    timed call a 1 GiB scrub buffer is read and written (4x the 256 MiB
    Infinity Cache, 32x the 8 x 4 MiB L2), outside the timed region; HIP
    events on the codec's stream bracket the one call.  The same per-call
    measurement without the scrub is reported beside it (warm: the round
    trip's situation, the encoded bytes still cached from the encode)."""
    scrub = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def one(fn, cold):
        if cold:
            scrub.add_(1)
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) * 1e-3

    out = {}
    for name, fn in (("decode", lambda: codec.decode_dev(enc, eout, dec, dout)),
                     ("encode", lambda: codec.encode_dev(src, spans, enc, eout))):
        fn()  # (a warm-up call, and the encoder's AUTO history)
        ts = {c: sorted(one(fn, c) for _ in range(reps)) for c in (False, True)}
        out[name + "_cold_GiBps"] = round(total / ts[True][reps // 2] / GIB, 2)
        out[name + "_warm_GiBps_same_method"] = round(total / ts[False][reps // 2] / GIB, 2)
        out[name + "_cold_us"] = round(ts[True][reps // 2] * 1e6, 1)
        out[name + "_warm_us"] = round(ts[False][reps // 2] * 1e6, 1)
    out["how"] = ("median of %d single calls, HIP events on the codec stream; cold: a 1 GiB "
                  "read+write scrub before each call, outside the events" % reps)
    del scrub
    return out


def leg_config4(args, torch, dev, codec, D, rank, world, timed):
    """Config 4: synthetic header blocks at dynamic table 0 (the qifs corpus
    is absent offline), split by contiguous block range over the ranks, each
    rank running qh_decode_sections_batch on its blocks in HBM: GPU framing,
    every Huffman string decoded, Huffman failures folded into -401, every
    string validated and every name's token looked up."""
    from nghttp3_amd import qpack as qp
    from nghttp3_amd import shard
    nb_all = args.c4_blocks
    q_src, q_blocks, q_plain, q_strs, q_lines, q_ls = qp.synth_field_sections(SEED4, nb_all)
    lo, hi = shard.block_range_by_bytes(rank, world, q_blocks["len"])
    my = q_blocks[lo:hi].copy()
    base = int(my["off"][0])
    q_host = np.ascontiguousarray(q_src[base:int(my["off"][-1] + my["len"][-1])])
    my["off"] -= base
    d_src = torch.from_numpy(q_host).to(dev)
    d_blk = torch.from_numpy(my.view(np.int64).reshape(-1, 2).copy()).to(dev)
    fsd = qp.FieldSectionDecoder(codec=codec, dtable0=True)
    bufs = fsd.decode_blocks_dev(d_src, d_blk)
    torch.cuda.synchronize()
    t_pipe = timed(lambda: fsd.decode_blocks_dev(d_src, d_blk, bufs), args.steps)
    codec.enable_timing(True)
    for _ in range(3):
        fsd.decode_blocks_dev(d_src, d_blk, bufs)
    kt = {k: round(ms / max(c, 1) * 1e3, 2) for k, (c, ms) in codec.kernel_times().items()}
    codec.enable_timing(False)
    # bit-exact: every string (Huffman ones from dst, raw ones in place) in
    # span order equals the plaintext the writer was given
    ns = int(bufs["nspans"])
    s_lo = int(np.count_nonzero(q_lines["name"][:q_ls[lo]] >= 0)
               + np.count_nonzero(q_lines["value"][:q_ls[lo]] >= 0))
    sel = q_strs[s_lo:s_lo + ns]
    strs = bufs["strs"][:ns]
    huff = ((bufs["spans"][:ns, 1] >> 32) & qp.SPAN_HUFFMAN) != 0
    ln = strs[:, 1] & 0xFFFFFFFF
    want_ln = torch.from_numpy(sel["len"].astype(np.int64)).to(dev)
    ok = bool((bufs["status"][:hi - lo] == 0).all()) and bool(((strs[:, 1] >> 32) == 0).all()) and \
        bool(torch.equal(ln, want_ln))
    h_plain = int(ln[huff].sum().item())
    plain_all = int(ln.sum().item())
    if ok and plain_all:
        starts = torch.repeat_interleave(torch.cumsum(ln, 0) - ln, ln)
        pos = torch.arange(plain_all, device=dev, dtype=torch.int64) - starts
        at = torch.repeat_interleave(strs[:, 0], ln) + pos
        from_dst = torch.repeat_interleave(huff, ln)
        got = torch.where(from_dst, bufs["dst"][at.clamp(max=bufs["dst"].numel() - 1)],
                          d_src[at.clamp(max=d_src.numel() - 1)])
        p0 = int(sel["off"][0])
        want = torch.from_numpy(np.ascontiguousarray(q_plain[p0:p0 + plain_all])).to(dev)
        ok = bool(torch.equal(got, want))
        del starts, pos, at, from_dst, got, want
    valid = int(bufs["verdict"][:ns].to(torch.int64).sum().item())
    # encoder side: this rank's sections written back from their lines and
    # plaintext strings (qh_encode_sections_batch on the device)
    fse = qp.FieldSectionEncoder(codec=codec)
    e_plain = torch.from_numpy(np.ascontiguousarray(q_plain)).to(dev)
    e_strs = torch.from_numpy(q_strs.view(np.int64).reshape(-1, 2).copy()).to(dev)
    l0, l1 = int(q_ls[lo]), int(q_ls[hi])
    e_lines = torch.from_numpy(np.ascontiguousarray(q_lines[l0:l1]).view(np.uint8).copy()).to(dev)
    e_ls = torch.from_numpy((q_ls[lo:hi + 1] - q_ls[lo]).astype(np.int32)).to(dev)
    e_dst = torch.empty(q_host.size + 64, dtype=torch.uint8, device=dev)
    e_sec = torch.empty((hi - lo, 2), dtype=torch.int64, device=dev)
    need = fse.encode_sections_dev(e_plain, e_strs, e_lines, e_ls, e_dst, e_sec)
    torch.cuda.synchronize()
    enc_ok = need == q_host.size and bool(torch.equal(e_dst[:need], d_src))
    t_enc = timed(lambda: fse.encode_sections_dev(e_plain, e_strs, e_lines, e_ls, e_dst, e_sec),
                  args.steps)
    codec.enable_timing(True)
    for _ in range(3):
        fse.encode_sections_dev(e_plain, e_strs, e_lines, e_ls, e_dst, e_sec)
    kts = codec.kernel_times().items()
    kt_enc = {k: round(ms / max(c, 1) * 1e3, 2) for k, (c, ms) in kts}
    kt_enc_call = {k: round(ms / 3 * 1e3, 2) for k, (c, ms) in kts}  # (per call: every launch)
    codec.enable_timing(False)
    del e_plain, e_strs, e_lines, e_ls, e_dst, e_sec
    # host-memory form (the library stages H2D / D2H): this rank's blocks
    reps = 3
    fsd.decode_blocks(q_host, my)
    a = time.perf_counter()
    for _ in range(reps):
        fsd.decode_blocks(q_host, my)
    t_host = D.max((time.perf_counter() - a) / reps)
    blk_all = D.sum(float(q_host.size))
    h_all = D.sum(float(h_plain))
    s_all = D.sum(float(plain_all))
    return {"blocks": nb_all, "field_lines": int(q_lines.size), "block_bytes": int(blk_all),
            "string_bytes": int(s_all), "huffman_plain_bytes": int(h_all), "shards": world,
            "gpu_pipeline_ms": round(t_pipe * 1e3, 4),
            "gpu_pipeline_blocks_per_s": round(nb_all / t_pipe, 1),
            "gpu_pipeline_huffman_GiBps": round(h_all / t_pipe / GIB, 2),
            "gpu_pipeline_block_GBps": round(blk_all / t_pipe / 1e9, 2),
            "valid_strings_rank0": valid,
            "kernel_avg_us_rank0": kt,
            "host_path_ms": round(t_host * 1e3, 3),
            "host_path_blocks_per_s": round(nb_all / t_host, 1),
            "bit_exact": D.sum(0.0 if ok else 1.0) == 0,
            "encoder_gpu_ms": round(t_enc * 1e3, 4),
            "encoder_gpu_blocks_per_s": round(nb_all / t_enc, 1),
            "encoder_gpu_string_GiBps": round(s_all / t_enc / GIB, 2),
            "encoder_kernel_avg_us_rank0": kt_enc,
            "encoder_kernel_us_per_call_rank0": kt_enc_call,
            "encoder_bit_exact": D.sum(0.0 if enc_ok else 1.0) == 0,
            "encoder_pipeline": "qh_encode_sections_batch: count -> pick (Huffman iff shorter) -> "
                                "section sizes -> scan -> (sync) -> codes of the picked strings (their lengths from the count) -> write",
            "pipeline": "qh_decode_sections_batch: frame count -> scans -> (sync) -> frame write -> "
                        "decode -> post (fold -401, check, tokens)",
            "shape": "synthetic (nghttp3_amd/qpack.py synth_field_sections): 4-20 lines per "
                     "block, 30% indexed static, 40% static name ref, 30% literal name; "
                     "names 4-24 B, values 1-128 B, alphabet A; dtable 0"}


def leg_config1():
    """Config 1: the driver (nghttp3_amd/lib/qpack, a child process) encodes
    the 1,024-field QIF and decodes it back, on the GPU batch path and on the
    scalar drop-ins; each batch part timed over 20 repetitions (median), the
    round trip checked byte for byte."""
    import tempfile
    from nghttp3_amd import qif
    text = qif.synth_config1()
    res = {"fields": 1024, "qif_bytes": len(text),
           "source": "nghttp3_amd/qif.py synth_config1 (netbsd QIF, :path queries, cookies; seed 0x5EED0001)"}
    with tempfile.TemporaryDirectory() as d:
        src, wire, back = (os.path.join(d, x) for x in ("c1.qif", "c1.out", "c1.back"))
        open(src, "wb").write(text)
        for path in ("gpu", "scalar"):
            flag = [] if path == "gpu" else ["--scalar"]
            r1 = qif.run(flag + ["--time", "20", "encode", src, wire])
            r2 = qif.run(flag + ["--time", "20", "decode", wire, back])
            if r1.returncode or r2.returncode:
                res[path] = {"error": (r1.stderr + r2.stderr)[-400:]}
                continue
            je = json.loads(r1.stderr.strip().splitlines()[-1])
            jd = json.loads(r2.stderr.strip().splitlines()[-1])
            ok = open(back, "rb").read() == text
            res[path] = {"encode_batch_ms": je["batch_ms"], "encode_plan_ms": je["plan_ms"],
                         "decode_frame_ms": jd["frame_ms"], "decode_batch_ms": jd["batch_ms"],
                         "decode_replay_ms": jd["replay_ms"], "wire_bytes": je["out_bytes"],
                         "round_trip_identical": ok}
    return res


def _gpu_numa(torch, dev):
    """The GPU's NUMA node and that node's CPUs (sysfs), or (None, None)."""
    try:
        pr = torch.cuda.get_device_properties(dev)
        bdf = "%04x:%02x:%02x.0" % (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id)
        node = int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read().strip())
        if node < 0:
            return None, None
        cpus = set()
        for part in open(f"/sys/devices/system/node/node{node}/cpulist").read().strip().split(","):
            lo, _, hi = part.partition("-")
            cpus.update(range(int(lo), int(hi or lo) + 1))
        return node, cpus
    except Exception:
        return None, None


def _page_node(t):
    """NUMA node of the page holding a host tensor's first byte (move_pages),
    or None."""
    try:
        import ctypes
        libc = ctypes.CDLL(None, use_errno=True)
        pages = (ctypes.c_void_p * 1)(t.data_ptr())
        status = (ctypes.c_int * 1)(-1)
        rc = libc.syscall(279, 0, 1, pages, None, status, 0)  # SYS_move_pages (x86_64), query only
        return int(status[0]) if rc == 0 and status[0] >= 0 else None
    except Exception:
        return None


def leg_host_path(torch, codec, q, enc, eout, enc_bytes, total, n, dev):
    """Decode from host memory: H2D of spans and encoded bytes, kernels, D2H
    of results (pageable and pinned buffers), beside a copy-engine probe of
    the same byte counts in the same run (H2D alone, D2H alone, both at once
    on two streams).  The host buffers are allocated with this process bound
    to the GPU's NUMA node's CPUs (first touch places them there); the node of
    each pinned buffer's pages is recorded."""
    node, cpus = _gpu_numa(torch, dev)
    try:
        aff0 = os.sched_getaffinity(0)
    except Exception:
        aff0 = None
    if cpus and aff0 and cpus & aff0:
        os.sched_setaffinity(0, cpus & aff0)
    eo = eout.cpu().numpy()
    cap_h = int(q.decode_slot_size(eo[:, 1] & 0xFFFFFFFF).sum())
    in_bytes, out_bytes = enc_bytes + 16 * n, total + 16 * n
    out = {"gpu_numa_node": node, "bound_cpus": len(cpus & aff0) if cpus and aff0 else None,
           "bytes_in": in_bytes, "bytes_out": out_bytes}
    # copy-engine probe: the path's byte counts, pinned, 3 reps each
    h_in = torch.empty(in_bytes, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(out_bytes, dtype=torch.uint8, pin_memory=True)
    h_in.fill_(1)
    h_out.fill_(1)
    d_in = torch.empty(in_bytes, dtype=torch.uint8, device=dev)
    d_out = torch.empty(out_bytes, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def probe(h2d, d2h, reps=5):
        """The fastest of reps single transfers (the copy engines' best for
        these byte counts: an enqueue that blocks the host until its copy is
        done serialises the two directions in some reps)."""
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            a = time.perf_counter()
            if h2d:
                with torch.cuda.stream(s1):
                    d_in.copy_(h_in, non_blocking=True)
            if d2h:
                with torch.cuda.stream(s2):
                    h_out.copy_(d_out, non_blocking=True)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - a)
        return min(ts)

    probe(True, True, 1)
    t_h2d, t_d2h, t_both = probe(True, False), probe(False, True), probe(True, True)
    out["probe"] = {"h2d_GBps": round(in_bytes / t_h2d / 1e9, 2), "d2h_GBps": round(out_bytes / t_d2h / 1e9, 2),
                    "both_ms": round(t_both * 1e3, 3),
                    "both_GBps_each": [round(in_bytes / t_both / 1e9, 2), round(out_bytes / t_both / 1e9, 2)],
                    "pinned_page_node": [_page_node(h_in), _page_node(h_out)]}
    del h_in, h_out, d_in, d_out
    for kind in ("pageable", "pinned"):
        pin = kind == "pinned"
        e_t = torch.empty(enc_bytes, dtype=torch.uint8, pin_memory=pin)
        e_t.copy_(enc[:enc_bytes])
        sp_t = torch.zeros(n * 2, dtype=torch.int64, pin_memory=pin)
        spn = sp_t.numpy().view(q.SPAN_IN_DTYPE)
        spn["off"], spn["len"] = eo[:, 0], eo[:, 1] & 0xFFFFFFFF
        d_t = torch.empty(max(cap_h, 1), dtype=torch.uint8, pin_memory=pin)
        o_t = torch.empty(n * 2, dtype=torch.int64, pin_memory=pin)
        e_h, d_h, o_h = e_t.numpy(), d_t.numpy(), o_t.numpy().view(q.SPAN_OUT_DTYPE)
        for _ in range(2):  # warm the staging buffers and the host pages
            codec.decode_host(e_h, spn, d_h, o_h)
        # the median of 5 calls; Python's garbage collector held off while
        # they run (a collection inside a call is the harness's pause, not
        # the library's)
        reps = 5

        def med_ms(fn):
            import gc
            ts, thr = [], []
            gc.collect()
            gc.disable()
            try:
                for _ in range(reps):
                    t0 = _cpu_throttled_ms()
                    a = time.perf_counter()
                    fn()
                    ts.append(time.perf_counter() - a)
                    t1 = _cpu_throttled_ms()
                    thr.append(round(t1 - t0, 2) if t0 is not None and t1 is not None else None)
            finally:
                gc.enable()
            return sorted(ts)[reps // 2], [round(t * 1e3, 2) for t in ts], thr

        t_host, ts_host, thr_host = med_ms(lambda: codec.decode_host(e_h, spn, d_h, o_h))
        # (cpu_throttled_ms_each: time the cgroup's CPU quota held the
        # process's threads back during each call)
        out[kind] = {"decode_GiBps_incl_h2d_d2h": round(total / t_host / GIB, 2),
                     "ms": round(t_host * 1e3, 2), "ms_each": ts_host,
                     "cpu_throttled_ms_each": thr_host}
        if pin:
            out[kind]["page_node"] = [_page_node(e_t), _page_node(d_t)]
            # the bound: both directions at once, the probe's time for these bytes
            out[kind]["frac_of_probe_both"] = round(t_both / t_host, 3)
            # the same batch fanned out over 2 contexts of this GPU
            # (qh_decode_batch_multi: own streams, host threads, pipelines;
            # on a node, one context per GPU and link)
            from nghttp3_amd import HuffmanBatchCodec
            cs = [HuffmanBatchCodec(dev.index or 0, stream=torch.cuda.Stream(dev)) for _ in range(2)]
            HuffmanBatchCodec.decode_host_multi(cs, e_h, spn, d_h, o_h)  # warm
            t_m, ts_m, _ = med_ms(lambda: HuffmanBatchCodec.decode_host_multi(cs, e_h, spn, d_h, o_h))
            out["pinned_2ctx_one_gpu"] = {"decode_GiBps_incl_h2d_d2h": round(total / t_m / GIB, 2),
                                          "ms": round(t_m * 1e3, 2), "ms_each": ts_m,
                                          "frac_of_probe_both": round(t_both / t_m, 3)}
            for c_ in cs:
                c_.close()
        del e_t, sp_t, d_t, o_t
    if aff0:
        os.sched_setaffinity(0, aff0)
    return out


def leg_host_path_ranks(torch, codec, q, src, enc, eout, enc_bytes, total, n, dev, D, rank, world):
    """The north-star path at N > 1: each rank decodes its shard of the
    config-3 batch from pinned host memory through qh_decode_batch(...,
    QH_WHERE_HOST) -- its own H2D of spans and encoded bytes, its own D2H of
    the packed decoded bytes, on its own GPU's link (SURVEY.md section
    8(e)).  Each call is bracketed by barriers and timed as the max over
    ranks; the median of 5 calls after a warm one.  Aggregate = plaintext of
    all ranks / that time.  Bit-exact: the packed host output equals the
    shard's plaintext, which synth lays out back to back in string order."""
    node, cpus = _gpu_numa(torch, dev)
    try:
        aff0 = os.sched_getaffinity(0)
    except Exception:
        aff0 = None
    if cpus and aff0 and cpus & aff0:
        os.sched_setaffinity(0, cpus & aff0)
    eo = eout.cpu().numpy()
    cap_h = int(q.decode_slot_size(eo[:, 1] & 0xFFFFFFFF).sum())
    e_t = torch.empty(enc_bytes, dtype=torch.uint8, pin_memory=True)
    e_t.copy_(enc[:enc_bytes])
    sp_t = torch.zeros(n * 2, dtype=torch.int64, pin_memory=True)
    spn = sp_t.numpy().view(q.SPAN_IN_DTYPE)
    spn["off"], spn["len"] = eo[:, 0], eo[:, 1] & 0xFFFFFFFF
    d_t = torch.empty(max(cap_h, 1), dtype=torch.uint8, pin_memory=True)
    o_t = torch.empty(n * 2, dtype=torch.int64, pin_memory=True)
    e_h, d_h, o_h = e_t.numpy(), d_t.numpy(), o_t.numpy().view(q.SPAN_OUT_DTYPE)
    codec.decode_host(e_h, spn, d_h, o_h)  # warm the staging buffers
    ts = []
    for _ in range(5):
        D.barrier()
        a = time.perf_counter()
        codec.decode_host(e_h, spn, d_h, o_h)
        t = time.perf_counter() - a
        ts.append((D.max(t), t))
    ts.sort()
    t_max, t_mine = ts[2]
    ok = bool((o_h["status"] == 0).all()) and int(o_h["len"].astype(np.int64).sum()) == total and \
        bool(np.array_equal(d_h[:total], src[:total].cpu().numpy()))
    bad = D.sum(0.0 if ok else 1.0)
    total_all = D.sum(float(total))
    if aff0:
        os.sched_setaffinity(0, aff0)
    out = {"ranks": world, "form": "each rank: its shard, pinned host buffers, own H2D/D2H (qh_decode_batch, "
                                   "QH_WHERE_HOST)",
           "plain_bytes_all": int(total_all), "ms_max_over_ranks": round(t_max * 1e3, 2),
           "decode_GiBps_incl_h2d_d2h_all": round(total_all / t_max / GIB, 2),
           "ms_each_max_over_ranks": [round(x[0] * 1e3, 2) for x in ts],
           "ms_rank0": round(t_mine * 1e3, 2) if rank == 0 else None,
           "gpu_numa_node_rank0": node if rank == 0 else None,
           "bit_exact": bad == 0}
    del e_t, sp_t, d_t, o_t
    return out


def _cg_paths():
    """This process's cgroup directories that may hold its CPU controller."""
    paths = []
    try:
        for line in open("/proc/self/cgroup"):
            hid, ctl, path = line.rstrip("\n").split(":", 2)
            if hid == "0":
                paths.append(("v2", "/sys/fs/cgroup" + path))
            elif "cpu" in ctl.split(","):
                paths.append(("v1", "/sys/fs/cgroup/" + ctl + path))
                paths.append(("v1", "/sys/fs/cgroup/cpu,cpuacct" + path))
                paths.append(("v1", "/sys/fs/cgroup/cpu" + path))
    except OSError:
        pass
    paths += [("v2", "/sys/fs/cgroup"), ("v1", "/sys/fs/cgroup/cpu"), ("v1", "/sys/fs/cgroup/cpu,cpuacct")]
    return paths


def _cpu_throttled_ms():
    """Milliseconds the cgroup's CPU quota has held this process's threads
    back so far (cpu.stat throttled_usec / throttled_time); None if unknown."""
    for kind, d in _cg_paths():
        try:
            for line in open(os.path.join(d, "cpu.stat")):
                k, v = line.split()[:2]
                if k == "throttled_usec":
                    return int(v) / 1e3
                if k == "throttled_time":  # (v1: ns)
                    return int(v) / 1e6
        except (OSError, ValueError):
            continue
    return None


def _cpu_quota():
    """CPUs' worth of time the cgroup grants this process (cgroup v2 cpu.max
    or v1 cfs quota / period), rounded up; None when unlimited / unknown."""
    import math
    for kind, d in _cg_paths():
        try:
            if kind == "v2":
                q, per = open(os.path.join(d, "cpu.max")).read().split()[:2]
                if q != "max":
                    return max(1, math.ceil(int(q) / int(per)))
            else:
                q = int(open(os.path.join(d, "cpu.cfs_quota_us")).read())
                per = int(open(os.path.join(d, "cpu.cfs_period_us")).read())
                if q > 0:
                    return max(1, math.ceil(q / per))
        except (OSError, ValueError):
            continue
    return None


def leg_cpu(args, src, spans, total, n):
    """BASELINE.md CPU protocol: the oracle restatement (same nibble FSM and
    64-bit accumulator as lib/nghttp3_qpack_huffman.c:34-124, -O2 -mavx2)
    round-trips the same strings at T = 1 (a bounded sample) and T = all
    CPUs of this process's affinity (the whole batch).  The thread pool is
    created once, thread t pinned to the t-th CPU of the affinity list and
    owning a contiguous shard; each encode / decode pass starts and ends at
    a barrier and repeats the shard until a thread has worked >= 50 ms;
    verification runs after the timed passes.  min / median / max over
    `cpu_reps` passes; value = the median round trip."""
    import oracle
    plain = src[:total].cpu().numpy()
    sp = spans.cpu().numpy()
    off = sp[:, 0].astype(np.uint64)
    lens = (sp[:, 1] & 0xFFFFFFFF).astype(np.uint32)
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except Exception:
        cpus = list(range(os.cpu_count() or 1))
    # the CPU time this process may use: a cgroup quota (the GPU box grants a
    # share of its cores) caps the useful thread count below the affinity
    # list; more threads than that only time-slice and add barrier waits
    quota = _cpu_quota()
    nthr = max(1, min(len(cpus), quota)) if quota else len(cpus)
    reps = args.cpu_reps

    def run(k, threads):
        e, d, ok, inner = oracle.bench_roundtrip(plain, off[:k], lens[:k], threads, reps,
                                                 cpus=cpus[:threads], min_seconds=0.05)
        b = float(lens[:k].astype(np.uint64).sum())
        rt = sorted(b / (x + y) / GIB for x, y in zip(e, d))
        de = sorted(b / x / GIB for x in d)
        en = sorted(b / x / GIB for x in e)
        r4 = lambda v: round(v, 4)
        return {"round_trip_GiBps": r4(rt[len(rt) // 2]),
                "round_trip_min_med_max": [r4(rt[0]), r4(rt[len(rt) // 2]), r4(rt[-1])],
                "decode_GiBps": r4(de[len(de) // 2]),
                "decode_min_med_max": [r4(de[0]), r4(de[len(de) // 2]), r4(de[-1])],
                "encode_GiBps": r4(en[len(en) // 2]),
                "encode_min_med_max": [r4(en[0]), r4(en[len(en) // 2]), r4(en[-1])],
                "passes_per_rep": list(inner),
                "strings": int(k), "plain_bytes": int(b), "ok": ok}

    k1 = min(n, args.cpu_t1_strings)
    t1 = run(k1, 1)
    tall = run(n, nthr)
    return {"value": tall["round_trip_GiBps"], "unit": "GiB/s", "cores": nthr,
            "kind": "port",
            "sample": f"T={nthr} pinned threads (affinity {len(cpus)} CPUs, cgroup CPU quota "
                      f"{quota or 'none'}): all {n} strings of the rank-0 batch; "
                      f"T=1: the first {k1} strings; {reps} barrier-to-barrier encode and decode "
                      "passes of >= 50 ms per thread each, verification outside the timed "
                      "passes, median (min/med/max in t1/tall); oracle/qh_oracle.c -O2 -mavx2 "
                      "(restatement of lib/nghttp3_qpack_huffman.c)",
            "t1": t1, "tall": tall, "cpu_model": _cpu_model(), "cpu_quota": quota,
            "affinity_cpus": len(cpus),
            "equivalence": "restatement-vs-reference speed ratio not measurable: the reference "
                           "needs a generated header absent here (DESIGN.md section 1)"}


if __name__ == "__main__":
    main()
