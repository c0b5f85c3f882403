"""GPU: SRBDControllerInterface.compute_control in one library call (srbd_interface_step through _srbd_fast)
against the Python sequence (srbd_controller_interface.py:113-180: prepare_state_and_reference, with_newkey,
with_newsigma, jitted_compute_control, the GRF mask), bit for bit.

Two interfaces of the same configuration are driven with the same PGG contact sequences over >= 12 MPC steps
(trot: legs lift off and touch down, so prepare_state zeroes warm starts and substitutes swing feet), one through
the one-call path, one with SRBD_INTERFACE_FAST=0.  Every returned value, and every controller attribute the next
call reads (warm start, key, call count, CEM sigma, previous contact), must be equal.
"""
import copy
import types

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LEGS = ("FL", "FR", "RL", "RR")


@pytest.fixture(scope="module")
def lib():
    from quadruped_pympc_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X")
    if _lib.fast is None:
        pytest.fail("_srbd_fast is not built (make -C quadruped-pympc-tamols_amd)")
    return _lib


def _cfg(**mp):
    from quadruped_pympc_amd import config as base

    c = types.SimpleNamespace(**{k: copy.deepcopy(getattr(base, k)) for k in
                                 ("robot", "mass", "inertia", "hip_height", "gravity_constant", "mpc_params",
                                  "simulation_params")})
    c.mpc_params.update(device_id=0, grf_max=c.mass * 9.81, **mp)
    return c


def _dicts(k):
    rng = np.random.default_rng(100 + k)
    sc = {"position": np.array([0.0, 0.0, 0.3]) + 0.01 * rng.standard_normal(3),
          "linear_velocity": 0.1 * rng.standard_normal(3), "orientation": 0.05 * rng.standard_normal(3),
          "angular_velocity": 0.1 * rng.standard_normal(3)}
    feet = np.array([[0.19, 0.14, 0.0], [0.19, -0.14, 0.0], [-0.19, 0.14, 0.0], [-0.19, -0.14, 0.0]])
    for i, n in enumerate(LEGS):
        sc["foot_" + n] = feet[i] + 0.01 * rng.standard_normal(3)
    rs = {"ref_position": np.array([0.0, 0.0, 0.3]), "ref_linear_velocity": np.array([0.4, 0.0, 0.0]),
          "ref_orientation": np.zeros(3), "ref_angular_velocity": np.zeros(3)}
    for i, n in enumerate(LEGS):
        rs["ref_foot_" + n] = (feet[i] + np.array([0.05, 0.0, 0.0]) + 0.01 * rng.standard_normal(3)).reshape(1, 3)
    return sc, rs


@pytest.mark.parametrize("method,par,rng,iters,n,H", [
    ("mppi", "zero_order", "jax", 1, 10000, 12),            # C2 through the plugin API, the drop-in's default stream
    ("mppi", "zero_order", "philox", 2, 10000, 12),
    ("random_sampling", "zero_order", "jax_legacy", 1, 3001, 10),
    ("cem_mppi", "cubic_spline", "jax", 2, 4096, 16),        # sigma reset at iteration 0 of every call
    ("mppi", "linear_spline", "philox", 1, 2048, 12),
])
def test_one_call_equals_python_sequence(lib, monkeypatch, method, par, rng, iters, n, H):
    from quadruped_pympc_amd.helpers.periodic_gait_generator import PeriodicGaitGenerator
    from quadruped_pympc_amd.interfaces.srbd_controller_interface import SRBDControllerInterface

    mp = dict(sampling_method=method, control_parametrization=par, num_parallel_computations=n, horizon=H,
              num_sampling_iterations=iters, rng="jax" if rng == "jax_legacy" else rng,
              jax_threefry_partitionable=rng != "jax_legacy")
    fast, slow = SRBDControllerInterface(_cfg(**mp)), SRBDControllerInterface(_cfg(**mp))
    slow._fast_env = False  # as SRBD_INTERFACE_FAST=0 at its creation
    pgg = PeriodicGaitGenerator(0.65, 1.4, 0, H)
    dts, lens = np.array([0.02]), np.array([H])
    lifts = 0
    try:
        for k in range(14):
            for _ in range(5):
                pgg.run(0.002, pgg.step_freq)
            cs = pgg.compute_contact_sequence(dts, lens)
            sc, rs = _dicts(k)
            prev = np.array(slow.previous_contact_mpc, dtype=float)
            lifts += int(np.sum((prev == 1) & (cs[:, 0] == 0)))
            a = fast.compute_control(sc, rs, cs, None, pgg.phase_signal, pgg.step_freq, 0)
            monkeypatch.setenv("SRBD_INTERFACE_FAST", "0")
            b = slow.compute_control(sc, rs, cs, None, pgg.phase_signal, pgg.step_freq, 0)
            monkeypatch.delenv("SRBD_INTERFACE_FAST")
            for n_ in LEGS:
                assert a[0][n_].dtype == b[0][n_].dtype
                np.testing.assert_array_equal(a[0][n_], b[0][n_], err_msg=f"step {k} grf {n_}")
                np.testing.assert_array_equal(a[1][n_], b[1][n_], err_msg=f"step {k} foothold {n_}")
            assert a[2:5] == b[2:5] == (None, None, None) and a[5] == b[5]
            assert a[6].dtype == b[6].dtype
            np.testing.assert_array_equal(a[6], b[6], err_msg=f"step {k} predicted state")
            ca, cb = fast.controller, slow.controller
            np.testing.assert_array_equal(ca.best_control_parameters, cb.best_control_parameters)
            assert ca.best_control_parameters.dtype == cb.best_control_parameters.dtype
            np.testing.assert_array_equal(ca.master_key, cb.master_key)
            assert ca.master_key.dtype == cb.master_key.dtype and ca._calls == cb._calls
            np.testing.assert_array_equal(fast.previous_contact_mpc, slow.previous_contact_mpc)
            if method == "cem_mppi":
                np.testing.assert_array_equal(ca.sigma_cem_mppi, cb.sigma_cem_mppi)
            assert ca.last_result.best_index == cb.last_result.best_index
            assert ca.context.step_id == cb.context.step_id
        assert fast._fast is not None and slow._fast is None  # each ran the path it was meant to
        assert lifts > 0  # the warm-start zeroing of prepare_state was exercised
    finally:
        fast.controller.close()
        slow.controller.close()


def test_one_call_falls_back_on_other_inputs(lib):
    """Inputs the glue does not take (lists, float32 dict entries) run the Python sequence, with the same result as
    the float64 arrays through the one call."""
    from quadruped_pympc_amd.interfaces.srbd_controller_interface import SRBDControllerInterface

    mp = dict(sampling_method="mppi", control_parametrization="zero_order", num_parallel_computations=2048,
              horizon=12, num_sampling_iterations=1, rng="philox")
    a, b = SRBDControllerInterface(_cfg(**mp)), SRBDControllerInterface(_cfg(**mp))
    try:
        cs = np.ones((4, 12))
        cs[1, :6] = 0
        sc, rs = _dicts(0)
        sc_list = {k: list(v) for k, v in sc.items()}
        ra = a.compute_control(sc, rs, cs, None, None, 1.4, 0)
        rb = b.compute_control(sc_list, rs, cs, None, None, 1.4, 0)
        for n in LEGS:
            np.testing.assert_array_equal(ra[0][n], rb[0][n])
        np.testing.assert_array_equal(ra[6], rb[6])
        np.testing.assert_array_equal(a.controller.master_key, b.controller.master_key)
    finally:
        a.controller.close()
        b.controller.close()
