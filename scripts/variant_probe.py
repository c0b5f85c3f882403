#!/usr/bin/env python3
"""Kernel and device-chain timings of one library variant (SRBD_LIB_PATH) over workloads (GPU box).

Usage: SRBD_LIB_PATH=... variant_probe.py NAME cfg[,cfg...]   -> one JSON line per workload
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quadruped-pympc-tamols_amd"))
from quadruped_pympc_amd import _lib  # noqa: E402
from quadruped_pympc_amd.synthetic import CONFIGS, inputs  # noqa: E402


def run(name, key, steps=300):
    w = CONFIGS[key]
    cfg = _lib.make_config(num_samples=w.num_samples, horizon=w.horizon, method=w.method,
                           parametrization=w.parametrization, num_splines=w.num_splines, mass=w.mass,
                           inertia=w.inertia, dts=np.full(w.horizon, 0.02, np.float32))
    ctx = _lib.Context(cfg)
    s, r, c = inputs(w, 0)
    sig = np.full(ctx.P, 3.0, np.float32) if w.method == "cem_mppi" else None
    best = np.zeros(ctx.P, np.float32)
    for k in range(5):
        best, _, _, _ = ctx.step(s, r, c, best, sigma=sig, counter=k)
    lat = []
    for k in range(steps):
        t0 = time.perf_counter()
        best, _, _, _ = ctx.step(s, r, c, best, sigma=sig, counter=100 + k)
        lat.append(time.perf_counter() - t0)
    ctx.bench_device_steps(50)
    ms = ctx.bench_device_steps(steps)
    kern = ctx.time_kernels(100)
    ctx.close()
    P = ctx.P
    us = kern.get("fused_rollout_us") or kern["rollout_us"]
    return dict(variant=name, workload=key, N=w.num_samples, chain_us=round(1e3 * ms / steps, 2),
                host_p50_us=round(1e6 * float(np.percentile(lat, 50)), 1),
                kernels_us={k: round(v, 2) for k, v in kern.items()},
                rollout_frac=round(w.num_samples * (4 * P + 4) / (kern["rollout_us"] * 1e-6) / 8e12, 4),
                launch_frac=round(w.num_samples * (4 * P + 4) / (us * 1e-6) / 8e12, 4))


if __name__ == "__main__":
    name = sys.argv[1]
    for key in sys.argv[2].split(","):
        print(json.dumps(run(name, key)), flush=True)
