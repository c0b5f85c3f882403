"""GPU: the one JSON line `python bench.py` prints (the driver's contract) -- a short run of the default
configuration, checked for every field the contract names and their relations: value = rollouts per second of the
timed steps (N / ms_per_step), the workload BASELINE's metric is quoted on, the roofline of the step's launch
(achieved = the algorithmic bytes of one launch over its event-timed duration, frac = achieved / peak) and the CPU
baseline's fields."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_default_line_contract():
    args = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "50", "--warmup", "5", "--latency-steps", "50",
            "--device-steps", "50", "--other-steps", "0", "--targets", "0", "--extras", "0", "--cpu-seconds", "0.5"]
    p = subprocess.run(args, cwd=ROOT, capture_output=True, text=True, timeout=200)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[-2000:]  # one line on stdout (native banners go to stderr)
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["metric"] == "SRBD rollouts/sec + p50 MPC-step ms at N=10k H=12; 1/2/4/8 GPU"
    assert d["unit"] == "rollouts/s" and d["higher_is_better"] is True and d["vs_baseline"] is None
    assert (d["n_gpus"], d["steps"], d["warmup"]) == (1, 50, 5)
    assert d["scaling"] == "weak" and d["dtype"] == "f32" and "synthetic" in d["data"]
    c = d["config"]
    assert c["workload"] == "go2_trot_flat_mppi_n10000_h12_zo" and c["num_samples"] == 10000 and c["horizon"] == 12
    assert (c["method"], c["parametrization"]) == ("mppi", "zero_order")
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert abs(d["value"] - c["num_samples"] / (d["ms_per_step"] * 1e-3)) <= 1e-3 * d["value"]
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert r["algorithmic_bytes_per_launch"] == c["num_samples"] * r["bytes_per_rollout"] == 5_800_000
    assert abs(r["achieved"] - r["algorithmic_bytes_per_launch"] / (r["kernel_us"] * 1e3)) <= 0.01 * r["achieved"]
    assert abs(r["frac"] - r["achieved"] / r["peak"]) <= 1e-4
    assert r["traffic"] is None or r["traffic"] > 0
    assert 0 < r["kernel_us"] * 1e-3 < d["ms_per_step"]  # the launch fits inside the host step it is part of
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["kind"] == "port" and cb["unit"] == "rollouts/s" and cb["value"] > 0 and cb["cores"] >= 1
