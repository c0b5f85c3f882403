#!/usr/bin/env python3
"""Gait-adaptive vs plain sampling MPC at C2 (N=10 000, H=12, MPPI, zero-order) on one GPU:
device-resident chain us/step, host-driven srbd_step p50, and the rollout launch (hipEvents).
Measurement tool."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "quadruped-pympc-tamols_amd")]

import numpy as np  # noqa: E402

from bench import make_cfg  # noqa: E402
from quadruped_pympc_amd import _lib  # noqa: E402
from quadruped_pympc_amd.synthetic import CONFIGS, inputs  # noqa: E402


def measure(ga: bool, n: int):
    w = CONFIGS["c2"]
    ctx = _lib.Context(make_cfg(w, n, 0, 1, 0))
    if ga:
        ctx.set_gait((0.1, 0.6, 0.6, 0.1), 0.02, 0.65, np.array([1.4, 2.0, 2.4], np.float32), None)
    s, r, c = inputs(w, 0)
    best = np.zeros(ctx.P, np.float32)
    for k in range(20):
        best, _, res, _ = ctx.step(s, r, c, best, seed=42, counter=k)
    ctx.bench_device_steps(50)
    ms = ctx.bench_device_steps(2000)
    lat = []
    for k in range(500):
        t0 = time.perf_counter()
        best, _, res, _ = ctx.step(s, r, c, best, seed=42, counter=100 + k)
        lat.append(time.perf_counter() - t0)
    kern = ctx.time_kernels(100)
    ctx.close()
    return {"ga": ga, "N": n, "device_us_per_step": round(1e3 * ms / 2000, 2),
            "host_p50_us": round(1e6 * float(np.percentile(lat, 50)), 2),
            "rollout_us": round(kern["rollout_us"], 2), "merge_us": round(kern["merge_us"], 2)}


if __name__ == "__main__":
    for n in (10000, 65536):
        for ga in (False, True):
            print(json.dumps(measure(ga, n)), flush=True)
