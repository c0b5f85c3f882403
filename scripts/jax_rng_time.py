#!/usr/bin/env python3
"""RNG kernel times on the reference's jax.random stream (GPU box): per config, the standalone draw launch and the
rollout launch with the next step's draws fused, by events (srbd_time_kernels).  Usage: jax_rng_time.py [cfg ...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quadruped-pympc-tamols_amd"))
from quadruped_pympc_amd import _lib  # noqa: E402
from quadruped_pympc_amd.synthetic import CONFIGS, inputs  # noqa: E402

for key in sys.argv[1:] or ["c2", "ns", "c5"]:
    w = CONFIGS[key]
    cfg = _lib.make_config(num_samples=w.num_samples, horizon=w.horizon, method=w.method,
                           parametrization=w.parametrization, num_splines=w.num_splines, mass=w.mass,
                           inertia=w.inertia, dts=np.full(w.horizon, w.dt, np.float32), sigma_mppi=w.sigma)
    out = {"workload": w.name}
    for rng in os.environ.get("RNGS", "philox,jax").split(","):
        ctx = _lib.Context(cfg)
        if rng != "philox":
            ctx.set_rng(rng)
        s, r, c = inputs(w, 0)
        sig = np.full(ctx.P, w.sigma, np.float32) if w.method == "cem_mppi" else None
        ctx.step(s, r, c, np.zeros(ctx.P, np.float32), sigma=sig, seed=42, counter=0)
        k = ctx.time_kernels(50)
        out[rng] = {n: round(v, 2) for n, v in k.items() if n in ("rng_us", "rollout_us", "fused_rollout_us")}
        ctx.close()
    print(json.dumps(out), flush=True)
