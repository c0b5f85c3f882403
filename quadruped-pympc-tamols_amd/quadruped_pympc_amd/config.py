"""Configuration mirror of ``quadruped_pympc/config.py`` (reference).

Same module-level names and dict keys (``robot``, ``mass``, ``inertia``,
``gravity_constant``, ``hip_height``, ``mpc_params``, ``simulation_params``) so
code written against the reference reads them unchanged.  Differences:

* it does not import ``gym_quadruped`` (absent here); ``hip_height`` comes from
  ``HIP_HEIGHTS`` below (go1/go2 0.25 and aliengo 0.30 are quoted by the
  reference's own comment at config.py:230; the other robots' values are
  estimates, used only as the TAMOLS ``h_des`` whose weight is 0 by default and
  as ``ref_z``);
* ``mpc_params['type']`` defaults to ``'sampling'`` (the only controller this
  package provides; gradient/acados controllers are out of scope);
* optional keys ``device_id`` (HIP ordinal, or ``'auto'``: replica i -> GPU i mod G, see
  ``runtime.py``) and ``num_elite`` (CEM elite size,
  reference hard-codes 10) and ``use_hip_graph``.

Use :func:`set_robot` to switch robot (the reference edits ``robot`` in-file).
"""
from __future__ import annotations

import numpy as np

# config.py:19-66
ROBOTS = {
    "go1": (12.019, [[1.58460467e-01, 1.21660000e-04, -1.55444692e-02],
                     [1.21660000e-04, 4.68645637e-01, -3.12000000e-05],
                     [-1.55444692e-02, -3.12000000e-05, 5.24474661e-01]]),
    "go2": (15.019, [[1.58460467e-01, 1.21660000e-04, -1.55444692e-02],
                     [1.21660000e-04, 4.68645637e-01, -3.12000000e-05],
                     [-1.55444692e-02, -3.12000000e-05, 5.24474661e-01]]),
    "aliengo": (24.637, [[0.2310941359705289, -0.0014987128245817424, -0.021400468992761768],
                         [-0.0014987128245817424, 1.4485084687476608, 0.0004641447134275615],
                         [-0.021400468992761768, 0.0004641447134275615, 1.503217877350808]]),
    "b2": (83.49, [[0.2310941359705289, -0.0014987128245817424, -0.021400468992761768],
                   [-0.0014987128245817424, 1.4485084687476608, 0.0004641447134275615],
                   [-0.021400468992761768, 0.0004641447134275615, 1.503217877350808]]),
    "hyqreal1": (108.40, [[4.55031444e+00, 2.75249434e-03, -5.11957307e-01],
                          [2.75249434e-03, 2.02411774e+01, -7.38560592e-04],
                          [-5.11957307e-01, -7.38560592e-04, 2.14269772e+01]]),
    "hyqreal2": (126.69, [[4.55031444e+00, 2.75249434e-03, -5.11957307e-01],
                          [2.75249434e-03, 2.02411774e+01, -7.38560592e-04],
                          [-5.11957307e-01, -7.38560592e-04, 2.14269772e+01]]),
    "mini_cheetah": (12.5, [[1.58460467e-01, 1.21660000e-04, -1.55444692e-02],
                            [1.21660000e-04, 4.68645637e-01, -3.12000000e-05],
                            [-1.55444692e-02, -3.12000000e-05, 5.24474661e-01]]),
    "spot": (50.34, [[0.2310941359705289, -0.0014987128245817424, -0.021400468992761768],
                     [-0.0014987128245817424, 1.4485084687476608, 0.0004641447134275615],
                     [-0.021400468992761768, 0.0004641447134275615, 1.503217877350808]]),
}
HIP_HEIGHTS = {"go1": 0.25, "go2": 0.25, "aliengo": 0.30, "b2": 0.45, "hyqreal1": 0.50, "hyqreal2": 0.50,
               "mini_cheetah": 0.225, "spot": 0.45}
# nominal feet offsets used by the synthetic benchmark inputs
NOMINAL_FEET = {"go1": (0.19, 0.13), "go2": (0.19, 0.13), "aliengo": (0.19, 0.13), "b2": (0.34, 0.23),
                "hyqreal1": (0.342, 0.234), "hyqreal2": (0.342, 0.234), "mini_cheetah": (0.19, 0.13),
                "spot": (0.30, 0.17)}

robot = "aliengo"
mass, _inertia = ROBOTS[robot]
inertia = np.array(_inertia)
hip_height = HIP_HEIGHTS[robot]
gravity_constant = 9.81

mpc_params = {
    "type": "sampling",
    "verbose": False,
    "horizon": 12,
    "dt": 0.02,
    "grf_max": mass * gravity_constant,
    "grf_min": 0,
    "mu": 0.5,
    "use_nonuniform_discretization": False,
    "horizon_fine_grained": 2,
    "dt_fine_grained": 0.01,
    "optimize_step_freq": False,
    "step_freq_available": [1.4, 2.0, 2.4],
    # sampling-based MPC (config.py:177-189)
    "sampling_method": "random_sampling",
    "control_parametrization": "cubic_spline",
    "num_splines": 2,
    "num_parallel_computations": 10000,
    "num_sampling_iterations": 1,
    "device": "gpu",
    "sigma_cem_mppi": 3,
    "sigma_mppi": 3,
    "sigma_random_sampling": [0.2, 3, 10],
    "shift_solution": False,
    # extensions (this package)
    "device_id": "auto",
    "num_elite": 10,
    "use_hip_graph": True,
}

simulation_params = {
    "step_height": 0.3 * hip_height,
    "visual_foothold_adaptation": "tamols",
    # config.py:209-243
    "tamols_params": {
        "search_radius": 0.32,
        "search_resolution": 0.04,
        "patch_size": 3,
        "gradient_delta": 0.04,
        "weight_edge_avoidance": 10.0,
        "weight_roughness": 10,
        "weight_deviation": 2,
        "weight_kinematic": 2.0,
        "weight_nominal_kinematic": 0.0,
        "weight_reference_tracking": 10.0,
        "weight_stability": 20.0,
        "stability_margin": 0.06,
        "stability_hard": False,
        "stability_soft": True,
        "estimated_swing_time": 0.25,
        "h_des": hip_height,
        "l_min": {"go1": 0.15, "go2": 0.15, "aliengo": 0.1, "b2": 0.25, "hyqreal1": 0.25, "hyqreal2": 0.25,
                  "mini_cheetah": 0.12, "spot": 0.20},
        "l_max": {"go1": 0.45, "go2": 0.45, "aliengo": 0.55, "b2": 0.75, "hyqreal1": 0.75, "hyqreal2": 0.75,
                  "mini_cheetah": 0.40, "spot": 0.60},
        "slope_threshold": 0.7,
        "constraint_box_dx": 0.05,
        "constraint_box_dy": 0.05,
    },
    "dt": 0.002,
    "gait": "trot",
    # GaitType values: TROT 0, PACE 1, BOUNDING 2, CIRCULARCRAWL 3, BFDIAGONALCRAWL 4,
    # BACKDIAGONALCRAWL 5, FRONTDIAGONALCRAWL 6, FULL_STANCE 7 (helpers/quadruped_utils.py:12-22)
    "gait_params": {
        "trot": {"step_freq": 1.4, "duty_factor": 0.65, "type": 0},
        "crawl": {"step_freq": 0.5, "duty_factor": 0.8, "type": 5},
        "pace": {"step_freq": 1.4, "duty_factor": 0.7, "type": 1},
        "bound": {"step_freq": 1.8, "duty_factor": 0.65, "type": 2},
        "full_stance": {"step_freq": 2, "duty_factor": 0.65, "type": 7},
    },
    "ref_z": hip_height,
    "mpc_frequency": 100,
    "use_inertia_recomputation": True,
    "scene": "flat",
}


def set_robot(name: str) -> None:
    """Switch the robot-dependent module attributes (the reference edits ``robot`` in-file)."""
    global robot, mass, inertia, hip_height
    if name not in ROBOTS:
        raise ValueError(f"unknown robot {name!r}")
    robot = name
    mass = ROBOTS[name][0]
    inertia = np.array(ROBOTS[name][1])
    hip_height = HIP_HEIGHTS[name]
    mpc_params["grf_max"] = mass * gravity_constant
    simulation_params["step_height"] = 0.3 * hip_height
    simulation_params["ref_z"] = hip_height
    simulation_params["tamols_params"]["h_des"] = hip_height
