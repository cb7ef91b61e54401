"""bench.py's multi-rank path on the GPU box: `--gpus 2` starts its own two
ranks (torch.distributed.run, before any GPU call), splits one batch by
bytes, and reports a max-over-ranks time.  With one GPU on the test box the
two ranks share device 0 and talk over gloo (--one-device); the driver's
8-GPU run uses RCCL with one rank per GPU."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def test_bench_two_ranks_rehearsal():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--one-device", "--strings", "65536", "--steps", "2", "--warmup", "1",
           "--c5-strings", "200000", "--c4-blocks", "2000", "--no-cpu-baseline"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["bit_exact"] is True
    assert rec["config"]["plain_bytes_all"] > rec["config"]["plain_bytes_rank0"]
    ex = rec["extra"]
    assert ex["config5_zipf"]["bit_exact"] is True and ex["config5_zipf"]["shards"] == 2
    assert ex["config4_qpack_blocks"]["bit_exact"] is True
    assert ex["enc_global_offset_rank0"] == 0
    # the north-star path at N > 1: every rank its shard from pinned host
    # memory, timed as the max over ranks, aggregate over all ranks' bytes
    hp = ex["host_path"]
    assert hp["ranks"] == 2 and hp["bit_exact"] is True
    assert hp["plain_bytes_all"] == rec["config"]["plain_bytes_all"]
    assert hp["decode_GiBps_incl_h2d_d2h_all"] > 0 and hp["ms_rank0"] > 0
    assert hp["ms_max_over_ranks"] >= hp["ms_rank0"] - 1e-6
