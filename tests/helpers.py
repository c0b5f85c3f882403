"""Shared test helpers: oracle + product setups for one workload (tests only)."""
from __future__ import annotations

import numpy as np

from oracle.srbd_oracle import PARAM_CODES, SamplingMPCOracle
from quadruped_pympc_amd.synthetic import CONFIGS, Workload, inputs

f32 = np.float32


def make_case(wkey="c2", *, N=1024, method=None, par=None, H=None, S=2, seed=0, k=2, best_scale=1.0,
              dts=None):
    w0 = CONFIGS[wkey]
    w = Workload(w0.name, w0.robot, w0.gait, method or w0.method, par or w0.parametrization, N, H or w0.horizon, S)
    orc = SamplingMPCOracle(mass=w.mass, inertia=w.inertia, horizon=w.horizon, num_samples=N, method=w.method,
                            parametrization=w.parametrization, num_splines=S)
    if dts is not None:
        orc.robot.dts = np.asarray(dts, f32)
    state, ref, contact = inputs(w, k)
    rng = np.random.default_rng(seed)
    t = N // 3
    Z = rng.standard_normal((max(N - 1, 0), orc.P)).astype(f32)
    U = rng.uniform(-10, 10, (max(N - 1 - 2 * t, 0), orc.P)).astype(f32)
    sigma = np.full(orc.P, 3.0, f32) if w.method == "cem_mppi" else None
    noise = orc.assemble_noise(Z, sigma=sigma, U=U)
    best = (best_scale * rng.standard_normal(orc.P)).astype(f32)
    return dict(w=w, orc=orc, state=state.astype(f32), ref=ref.astype(f32), contact=contact.astype(f32),
                noise=noise, best=best, sigma=sigma, dts=orc.robot.dts)


def product_cfg(case, use_graph=True, rank=0, world_size=1):
    from quadruped_pympc_amd import _lib

    w = case["w"]
    return _lib.make_config(num_samples=w.num_samples, horizon=w.horizon, method=w.method,
                            parametrization=w.parametrization, num_splines=w.num_splines, mass=w.mass,
                            inertia=w.inertia, dts=case["dts"], use_graph=use_graph, rank=rank,
                            world_size=world_size)
