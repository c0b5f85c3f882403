#!/usr/bin/env python3
"""Armed vs unarmed host-to-host srbd_step (measurement tool, GPU box): C2 steps timed from C
(srbd_bench_host_steps), interleaved blocks of each mode; prints one JSON line per mode."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quadruped-pympc-tamols_amd"))
from quadruped_pympc_amd import _lib  # noqa: E402
from quadruped_pympc_amd.synthetic import CONFIGS, inputs  # noqa: E402

key = sys.argv[1] if len(sys.argv) > 1 else "c2"
w = CONFIGS[key]
cfg = _lib.make_config(num_samples=w.num_samples, horizon=w.horizon, method=w.method, parametrization=w.parametrization,
                       num_splines=w.num_splines, mass=w.mass, inertia=w.inertia,
                       dts=np.full(w.horizon, 0.02, np.float32))
ctx = _lib.Context(cfg)
sets = [inputs(w, k) for k in range(8)]
st = np.stack([s[0] for s in sets]).astype(np.float32)
rf = np.stack([s[1] for s in sets]).astype(np.float32)
ct = np.stack([s[2] for s in sets]).astype(np.float32)
sig = np.full(ctx.P, 3.0, np.float32) if w.method == "cem_mppi" else None
best = np.zeros(ctx.P, np.float32)
res = {0: [], 1: []}
k = 0
for rep in range(6):
    for mode in (0, 1):
        ctx.set_armed(bool(mode), 0)
        lat, best, sig = ctx.bench_host_steps(st, rf, ct, best, sig, 42, k, 1000)
        k += 1000
        res[mode].append(lat[50:])
ctx.close()
for mode in (0, 1):
    a = np.concatenate(res[mode])
    print(json.dumps({"workload": w.name, "armed": bool(mode), "mean_us": round(float(a.mean()), 2),
                      "p50_us": round(float(np.percentile(a, 50)), 2), "p99_us": round(float(np.percentile(a, 99)), 2),
                      "steps": int(a.size)}), flush=True)
