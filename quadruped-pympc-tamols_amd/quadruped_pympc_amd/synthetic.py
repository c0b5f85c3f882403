"""Synthetic MPC workloads of the BASELINE.json configurations.

No datasets or simulators exist offline, so every benchmark and parity case is
fed from here: fixed-seed robot states, a forward-walking reference, and the
contact sequence of the configured gait from the periodic gait generator,
advanced 5 simulation steps (dt 0.002 s) per MPC step as in the reference loop
(quadruped_pympc_wrapper.py:134, mpc_frequency 100).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .config import HIP_HEIGHTS, NOMINAL_FEET, ROBOTS
from .helpers.periodic_gait_generator import BOUNDING, PACE, TROT, PeriodicGaitGenerator

GAITS = {"trot": (TROT, 1.4, 0.65), "pace": (PACE, 1.4, 0.7), "bound": (BOUNDING, 1.8, 0.65)}


@dataclass
class Workload:
    name: str
    robot: str
    gait: str
    method: str
    parametrization: str
    num_samples: int
    horizon: int
    num_splines: int = 2
    terrain: str = "flat"
    sigma: float = 3.0
    dt: float = 0.02

    @property
    def mass(self):
        return ROBOTS[self.robot][0]

    @property
    def inertia(self):
        return np.asarray(ROBOTS[self.robot][1], dtype=np.float32)

    def num_params(self):
        if self.parametrization == "linear_spline":
            return 4 * 3 * (self.num_splines + 1)
        if self.parametrization == "cubic_spline":
            return 4 * 12 * self.num_splines
        return 4 * 3 * self.horizon


# BASELINE.json "configs", in order
CONFIGS = {
    "c1": Workload("go2_trot_flat_rs_n128_h10_zo", "go2", "trot", "random_sampling", "zero_order", 128, 10),
    "c2": Workload("go2_trot_flat_mppi_n10000_h12_zo", "go2", "trot", "mppi", "zero_order", 10000, 12),
    "c3": Workload("aliengo_pace_cem_n65536_h16_cubic2", "aliengo", "pace", "cem_mppi", "cubic_spline", 65536, 16),
    "c4": Workload("go2_stones_tamols_mppi_n10000_h12_zo", "go2", "trot", "mppi", "zero_order", 10000, 12,
                   terrain="stepping_stones_medium"),
    "c5": Workload("hyqreal1_bound_mppi_n524288_h12_zo", "hyqreal1", "bound", "mppi", "zero_order", 524288, 12),
    # BASELINE.json north_star's target shape: MPPI, zero-order, N = 65 536, H = 12 on one MI355X
    "ns": Workload("go2_trot_flat_mppi_n65536_h12_zo", "go2", "trot", "mppi", "zero_order", 65536, 12),
}


def robot_state(robot: str, k: int = 0) -> np.ndarray:
    """24-vector [p, v, rpy, omega, feet FL FR RL RR] from default_rng(1234 + k)."""
    rng = np.random.default_rng(1234 + k)
    z = HIP_HEIGHTS[robot] + 0.05
    fx, fy = NOMINAL_FEET[robot]
    s = np.zeros(24)
    s[0:3] = (0.0, 0.0, z)
    s[3:6] = rng.uniform(-0.2, 0.2, 3)
    s[6:9] = rng.uniform(-0.05, 0.05, 3)
    s[9:12] = rng.uniform(-0.3, 0.3, 3)
    s[12:24] = [fx, fy, 0.0, fx, -fy, 0.0, -fx, fy, 0.0, -fx, -fy, 0.0]
    return s


def reference(robot: str, state: np.ndarray) -> np.ndarray:
    r = np.zeros(24)
    r[2] = HIP_HEIGHTS[robot] + 0.05
    r[3] = 0.5
    r[12:24] = state[12:24]
    return r


def contact_sequences(gait: str, horizon: int, steps: int, mpc_dt: float = 0.02, sim_dt: float = 0.002,
                      sim_per_mpc: int = 5) -> list:
    gtype, freq, duty = GAITS[gait]
    pgg = PeriodicGaitGenerator(duty, freq, gtype, horizon)
    out = []
    for _ in range(steps):
        for _ in range(sim_per_mpc):
            pgg.run(sim_dt, pgg.step_freq)
        out.append(pgg.compute_contact_sequence([mpc_dt], [horizon]))
    return out


def inputs(w: Workload, k: int = 0):
    """(state24, ref24, contact (4, H)) for MPC step k."""
    s = robot_state(w.robot, k)
    return s, reference(w.robot, s), contact_sequences(w.gait, w.horizon, k + 1)[-1]


C4_LEGS = ("FL", "FR", "RL", "RR")


def c4_inputs(k: int = 0, horizon: int = 12):
    """C4 (Go2 trot on stepping_stones_medium) MPC step k: the state dict (base over the first stones, feet on
    them), the reference footholds TAMOLS adapts (seeds, (4, 3): a stride ahead of the feet), the hips (4, 3),
    the base reference dict and the trot contact sequence (4, H) -- the inputs of helpers/foothold_pipeline.py."""
    feet = np.array([[1.22, 0.13, 0.05], [1.22, -0.13, 0.05], [0.84, 0.13, 0.05], [0.84, -0.13, 0.05]])
    base = np.array([1.03 + 0.004 * k, 0.0, 0.35])
    state = {"position": base, "linear_velocity": np.array([0.5, 0.02, 0.0]),
             "orientation": np.array([0.01, -0.02, 0.05]), "angular_velocity": np.array([0.0, 0.1, -0.05])}
    state.update({"foot_" + n: feet[i].copy() for i, n in enumerate(C4_LEGS)})
    seeds = feet + np.array([0.12 + 0.002 * k, 0.01, 0.0])
    hips = feet + np.array([0.0, 0.0, 0.3])
    ref_base = {"ref_position": np.array([0.0, 0.0, 0.32]), "ref_linear_velocity": np.array([0.5, 0.0, 0.0]),
                "ref_orientation": np.zeros(3), "ref_angular_velocity": np.zeros(3)}
    cs = contact_sequences("trot", horizon, k + 3)[-1].astype(np.float64)
    return state, seeds, hips, ref_base, cs


def c4_config():
    """A config module for C4 (the mirror's, switched to Go2, MPPI zero-order N = 10 000 H = 12, TAMOLS h_des at
    the Go2 hip height, no solution shift)."""
    import copy
    import types

    from . import config as base
    from .config import HIP_HEIGHTS

    w = CONFIGS["c4"]
    cfg = types.SimpleNamespace(**{k: copy.deepcopy(getattr(base, k)) for k in
                                   ("robot", "mass", "inertia", "hip_height", "gravity_constant", "mpc_params",
                                    "simulation_params")})
    cfg.robot, cfg.mass, cfg.inertia = w.robot, ROBOTS[w.robot][0], np.array(ROBOTS[w.robot][1])
    cfg.hip_height = HIP_HEIGHTS[w.robot]
    cfg.mpc_params.update(horizon=w.horizon, sampling_method=w.method, control_parametrization=w.parametrization,
                          num_parallel_computations=w.num_samples, sigma_mppi=w.sigma, grf_max=cfg.mass * 9.81,
                          device_id=0, shift_solution=False)
    cfg.simulation_params["tamols_params"]["h_des"] = cfg.hip_height
    return cfg
