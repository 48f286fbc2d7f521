"""GPU: bench.py's one-line JSON contract (the driver parses it): a short run with the small ViT, no CPU
baseline and no extra legs, in a child process (the bench initialises its own HIP context)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_prints_one_contract_line():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--model", "tiny", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--no-lift", "--no-config5", "--no-extras"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["dtype"] == "bf16"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # value is individuals x frames / s of the timed steps
    per_step = d["value"] * d["ms_per_step"] * 1e-3
    assert abs(per_step - round(per_step)) < 0.05 * per_step
    assert "workload" in d["config"]
    rl = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rl, k
    assert rl["bound"] in ("hbm", "mfma") and rl["peak"] > 0
    assert abs(rl["frac"] - rl["achieved"] / rl["peak"]) < 1e-3
