"""GPU: bench.py's N > 1 path, run as two ranks sharing the one GPU of the box over gloo (MQ_BENCH_SHARE_GPU=1,
MQ_BENCH_BACKEND=gloo; RCCL refuses two ranks on one device).  This is the code the driver's multi-GPU scaling run
executes per rank: the frame shard, the keypoint all-gather, the max-over-ranks timing, the per-rank fields of the
line and the clip lift split by individual over the ranks (step 4's exchanges on the gloo side group).  Checks: one
JSON line from rank 0 only, n_gpus 2, both ranks' timings, the all-gather's size for one frame of 4 individuals x 8
views x 17 joints per rank, and `value` equal to the units of both ranks over the slowest rank's time."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_sharing_the_gpu():
    env = dict(os.environ, MQ_BENCH_SHARE_GPU="1", MQ_BENCH_BACKEND="gloo")
    steps = 3
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2", "--steps", str(steps),
           "--warmup", "1", "--no-cpu-baseline", "--no-extras", "--no-config5"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints, rank 1 does not
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == steps and d["scaling"] == "weak"
    assert [rk["rank"] for rk in d["ranks"]] == [0, 1]
    slowest = max(rk["steps_ms"] + rk["gather_ms"] for rk in d["ranks"])
    assert all(rk["gather_ms"] >= 0 for rk in d["ranks"]) and d["gather_ms_max"] >= 0
    # per rank and step: 8 views x 4 individuals x 17 joints x (x, y, score) in float32 = 6,528 B
    assert d["gather_bytes_per_rank"] == steps * 8 * 4 * 17 * 3 * 4
    # value: 4 individuals x 1 frame per step on each of the 2 ranks, over the timed region's length (the slowest
    # rank's, barriers included), which covers every rank's steps and all-gather
    units = 2 * 4 * steps
    total_ms = d["ms_per_step"] * steps
    assert d["value"] == pytest.approx(units / (total_ms / 1e3), rel=2e-3)
    assert total_ms >= slowest * (1 - 2e-3)
    assert d["cpu_baseline"] is None
    cl = d["clip_lift"]
    assert cl["clips"] == 2 and cl["finite_3d_fraction"] > 0.9
