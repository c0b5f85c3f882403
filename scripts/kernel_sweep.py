#!/usr/bin/env python3
"""Per-kernel timing sweep over workload sizes and rollout variants (hipEvents; run on the GPU box).

Prints one JSON line per (workload, N, variant): kernel microseconds, device step time, and the
rollout kernel's algorithmic HBM rate (N * (4P + 4) bytes / kernel time).
`--cost-terms` runs the same sweep with the opt-in cost terms on (srbd_set_cost_terms).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quadruped-pympc-tamols_amd"))
from quadruped_pympc_amd import _lib  # noqa: E402
from quadruped_pympc_amd.synthetic import CONFIGS, Workload, inputs  # noqa: E402


TERMS = "--cost-terms" in sys.argv


def run(w, mode, steps=2000):
    os.environ["SRBD_ROLLOUT"] = mode
    cfg = _lib.make_config(num_samples=w.num_samples, horizon=w.horizon, method=w.method,
                           parametrization=w.parametrization, num_splines=w.num_splines, mass=w.mass,
                           inertia=w.inertia, dts=np.full(w.horizon, 0.02, np.float32))
    ctx = _lib.Context(cfg)
    if TERMS:
        ctx.set_cost_terms((0.1, 0.1, 0.001), 0.01, 5.0)
    s, r, c = inputs(w, 0)
    sig = np.full(ctx.P, 3.0, np.float32) if w.method == "cem_mppi" else None
    best = np.zeros(ctx.P, np.float32)
    for k in range(5):
        best, sig2, _, _ = ctx.step(s, r, c, best, sigma=sig, counter=k)
    import time
    lat = []
    for k in range(300):
        t0 = time.perf_counter()
        best, sig2, _, _ = ctx.step(s, r, c, best, sigma=sig, counter=100 + k)
        lat.append(time.perf_counter() - t0)
    ctx.bench_device_steps(200)
    ms = ctx.bench_device_steps(steps)
    kern = ctx.time_kernels(200)
    phases = ctx.merge_phases(50)
    ctx.close()
    P = ctx.P
    gbs = w.num_samples * (4 * P + 4) / (kern["rollout_us"] * 1e-6) / 1e9
    return dict(workload=w.name, N=w.num_samples, mode=mode, cost_terms=TERMS, step_us=round(1e3 * ms / steps, 3),
                p50_host_us=round(1e6 * float(np.percentile(lat, 50)), 1),
                rollouts_per_s=round(w.num_samples * steps / (ms * 1e-3), 1),
                **{k: round(v, 3) for k, v in kern.items()}, rollout_gbs=round(gbs, 1), merge_phases_us=phases)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    keys = [a for a in args if a.startswith("c")] or ["c2", "c3"]
    sizes = [int(a) for a in args if not a.startswith("c")] or [10000, 65536]
    for key in keys:
        w0 = CONFIGS[key]
        for n in sizes:
            w = Workload(w0.name, w0.robot, w0.gait, w0.method, w0.parametrization, n, w0.horizon, w0.num_splines)
            for mode in os.environ.get("SWEEP_MODES", "thread,quad").split(","):
                print(json.dumps(run(w, mode)), flush=True)


if __name__ == "__main__":
    main()
