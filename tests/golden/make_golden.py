#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run from the repo root).

The reference ships no golden vectors and cannot run here (JAX and gym_quadruped are absent:
ordinary ModuleNotFoundError), so these fixtures are produced by the CPU oracle
restatements (oracle/*.py) on fixed-seed synthetic inputs.  They pin the oracle against drift
(tests/test_golden.py) and give the GPU path fixed input/output pairs that do not need the
oracle at run time (tests/test_gpu_golden.py).  Every fixture stores its inputs with its
outputs.  Parity with the reference itself stays unpinned.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "quadruped-pympc-tamols_amd")]

from oracle.pgg_oracle import PGGOracle  # noqa: E402
from oracle.srbd_ga_oracle import GA_DUTY, GaitAdaptiveOracle, freq_set  # noqa: E402
from oracle.srbd_oracle import SamplingMPCOracle, prepare_state_and_reference  # noqa: E402
from oracle.tamols_oracle import TamolsOracle, synthetic_patch  # noqa: E402
from quadruped_pympc_amd.config import HIP_HEIGHTS, simulation_params  # noqa: E402
from quadruped_pympc_amd.helpers.terrain import TERRAINS  # noqa: E402
from quadruped_pympc_amd.synthetic import CONFIGS, inputs  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
f32 = np.float32

# name: (workload, method, parametrization, H, N, nonuniform dts)
SRBD_CASES = {
    "c1_rs_zo_h10": ("c1", "random_sampling", "zero_order", 10, 128, False),
    "c2_mppi_zo_h12": ("c2", "mppi", "zero_order", 12, 192, False),
    "c3_cem_cubic_h16": ("c3", "cem_mppi", "cubic_spline", 16, 160, False),
    "c2_mppi_linear_h12": ("c2", "mppi", "linear_spline", 12, 128, False),
    "c5_mppi_zo_h12_nonuniform": ("c5", "mppi", "zero_order", 12, 128, True),
}


def srbd_fixture(name, wkey, method, par, H, N, nonuniform):
    w = CONFIGS[wkey]
    o = SamplingMPCOracle(mass=w.mass, inertia=w.inertia, horizon=H, num_samples=N, method=method,
                          parametrization=par, use_nonuniform=nonuniform)
    rng = np.random.default_rng(sum(map(ord, name)))
    state, ref, contact = inputs(w, 3)
    contact = contact[:, :H]
    t = N // 3
    sigma = rng.uniform(0.5, 3.0, o.P).astype(f32) if method == "cem_mppi" else None
    noise = o.assemble_noise(rng.standard_normal((N - 1, o.P)).astype(f32), sigma=sigma,
                             U=rng.uniform(-10, 10, (N - 1 - 2 * t, o.P)).astype(f32))
    best = rng.standard_normal(o.P).astype(f32)
    out = o.compute_control(state.astype(f32), ref.astype(f32), contact.astype(f32), best, noise)
    np.savez_compressed(
        os.path.join(OUT, f"srbd_{name}.npz"),
        # inputs
        method=method, parametrization=par, horizon=H, num_samples=N, num_splines=2, mass=w.mass,
        inertia=w.inertia, dts=o.robot.dts, state=state.astype(f32), ref=ref.astype(f32),
        contact=contact.astype(f32), best_in=best, sigma_in=sigma if sigma is not None else np.zeros(0, f32),
        noise=noise,
        # outputs
        costs=out["costs"], best=out["best"], grf=out["grf"], pred=out["pred"], best_index=out["best_index"],
        best_cost=out["best_cost"], sigma=out.get("sigma", np.zeros(0, f32)))


# gait-adaptive: name: (workload, method, parametrization, H, N, leg phases)
GA_CASES = {
    "c2_mppi_zo_h12": ("c2", "mppi", "zero_order", 12, 160, (0.1, 0.6, 0.6, 0.1)),
    "c2_rs_linear_h12": ("c2", "random_sampling", "linear_spline", 12, 128, (0.64, 0.99, 1.0, 0.3)),
}


def ga_fixture(name, wkey, method, par, H, N, timing):
    w = CONFIGS[wkey]
    o = GaitAdaptiveOracle(pgg_dt=0.02, mass=w.mass, inertia=w.inertia, horizon=H, num_samples=N, method=method,
                           parametrization=par)
    rng = np.random.default_rng(sum(map(ord, name)))
    state, ref, contact = inputs(w, 4)
    contact = contact[:, :H]
    t = N // 3
    noise = o.assemble_noise(rng.standard_normal((N - 1, o.P)).astype(f32),
                             U=rng.uniform(-10, 10, (N - 1 - 2 * t, o.P)).astype(f32))
    fs = freq_set(o.method, (1.4, 2.0, 2.4), 1.65, 1)
    freqs = rng.choice(fs, N).astype(f32)
    best = rng.standard_normal(o.P).astype(f32)
    out = o.compute_control_ga(state.astype(f32), ref.astype(f32), contact.astype(f32), best, noise, freqs, timing)
    np.savez_compressed(
        os.path.join(OUT, f"ga_{name}.npz"),
        method=method, parametrization=par, horizon=H, num_samples=N, num_splines=2, mass=w.mass,
        inertia=w.inertia, dts=o.robot.dts, state=state.astype(f32), ref=ref.astype(f32),
        contact=contact.astype(f32), best_in=best, noise=noise, timing=np.asarray(timing, f32), pgg_dt=0.02,
        duty=GA_DUTY, freq_set=fs, freqs=freqs,
        costs=out["costs"], best=out["best"], grf=out["grf"], pred=out["pred"], best_index=out["best_index"],
        best_cost=out["best_cost"], best_freq=out["best_freq"])


def prepare_fixture():
    rng = np.random.default_rng(11)
    rows = []
    for _ in range(16):
        sc = {k: rng.standard_normal(3) for k in ("position", "linear_velocity", "orientation", "angular_velocity",
                                                  "foot_FL", "foot_FR", "foot_RL", "foot_RR")}
        rs = {k: rng.standard_normal(3) for k in ("ref_position", "ref_linear_velocity", "ref_orientation",
                                                  "ref_angular_velocity")}
        for n in ("FL", "FR", "RL", "RR"):
            rs["ref_foot_" + n] = rng.standard_normal((1, 3))
        cur, prev = rng.integers(0, 2, 4), rng.integers(0, 2, 4)
        best = rng.standard_normal(144).astype(f32)
        s, r, b = prepare_state_and_reference(sc, rs, cur, prev, best, 36)
        flat_sc = np.concatenate([sc[k] for k in ("position", "linear_velocity", "orientation", "angular_velocity",
                                                  "foot_FL", "foot_FR", "foot_RL", "foot_RR")])
        flat_rs = np.concatenate([rs[k].reshape(3) for k in ("ref_position", "ref_linear_velocity", "ref_orientation",
                                                             "ref_angular_velocity", "ref_foot_FL", "ref_foot_FR",
                                                             "ref_foot_RL", "ref_foot_RR")])
        rows.append((flat_sc, flat_rs, cur, prev, best, s, r, b))
    cols = list(zip(*rows))
    np.savez_compressed(os.path.join(OUT, "prepare_state.npz"), state_in=np.stack(cols[0]), ref_in=np.stack(cols[1]),
                        current_contact=np.stack(cols[2]), previous_contact=np.stack(cols[3]),
                        best_in=np.stack(cols[4]), state=np.stack(cols[5]), ref=np.stack(cols[6]),
                        best=np.stack(cols[7]))


def pgg_fixture():
    out = {}
    for gait, (duty, freq) in {0: (0.65, 1.4), 1: (0.7, 1.4), 2: (0.65, 1.8), 5: (0.8, 0.5)}.items():
        g = PGGOracle(duty, freq, gait, 12)
        seqs = []
        for _ in range(60):
            for _ in range(5):
                g.run(0.002, freq)
            seqs.append(g.compute_contact_sequence([0.01, 0.02], [2, 12]))
        out[f"gait{gait}"] = np.stack(seqs)
        out[f"gait{gait}_params"] = np.array([duty, freq])
    np.savez_compressed(os.path.join(OUT, "pgg_sequences.npz"), **out)


def tamols_fixture():
    params = dict(simulation_params["tamols_params"])
    params["h_des"] = HIP_HEIGHTS["go2"]
    orc = TamolsOracle(params, "go2")
    out = {}
    for name, yaw in (("flat", 0.0), ("stepping_stones_medium", 0.3)):
        rng = np.random.default_rng(len(name))
        feet = np.array([[0.62, 0.13, 0.0], [0.62, -0.13, 0.0], [0.24, 0.13, 0.0], [0.24, -0.13, 0.0]])
        seeds = feet + [0.12, 0, 0] + rng.uniform(-0.03, 0.03, (4, 3)) * [1, 1, 0]
        hips = feet + [0, 0, 0.30]
        hms = np.stack([synthetic_patch(s[:2], yaw, TERRAINS[name]) for s in seeds])
        vel = np.array([0.4, 0.05, 0.0])
        base = feet.mean(0) + [0, 0, 0.3]
        contact = np.array([0, 1, 1, 0])
        fh, boxes, valid, scores = orc.compute(hms, seeds, hips, vel, base, contact, feet)
        out.update({f"{name}_heightmaps": hms, f"{name}_seeds": seeds, f"{name}_hips": hips, f"{name}_vel": vel,
                    f"{name}_base": base, f"{name}_contact": contact, f"{name}_feet": feet,
                    f"{name}_footholds": fh, f"{name}_boxes": boxes, f"{name}_valid": valid,
                    f"{name}_scores": scores})
    np.savez_compressed(os.path.join(OUT, "tamols_go2.npz"), **out)


def main():
    for name, spec in SRBD_CASES.items():
        srbd_fixture(name, *spec)
    for name, spec in GA_CASES.items():
        ga_fixture(name, *spec)
    prepare_fixture()
    pgg_fixture()
    tamols_fixture()
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
