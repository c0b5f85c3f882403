"""CPU tests of the opt-in cost terms' oracle (oracle/srbd_oracle.py extra_cost; include/srbd_mpc.h
srbd_set_cost_terms).  The terms are a build extension (the reference's sampling cost has none,
SURVEY App. B #6), so these pin the definitions themselves: zero weights reproduce the reference's
cost exactly, every term is non-negative and scales with its weight, GRF smoothing vanishes for
forces constant over the horizon, and the cone term vanishes when no force needed clipping."""
import numpy as np
import pytest

from helpers import f32, make_case
from oracle.srbd_oracle import extra_cost

TERMS = {"r_force": (0.1, 0.1, 0.001), "w_smooth": 0.01, "w_cone": 5.0}


@pytest.mark.parametrize("par", ["zero_order", "linear_spline", "cubic_spline"])
def test_zero_weights_are_the_reference_cost(par):
    case = make_case("c2", N=200, method="mppi", par=par, H=12 if par != "cubic_spline" else 16, seed=2)
    o = case["orc"]
    params = (case["best"][None, :] + case["noise"]).astype(f32)
    a = o.rollout_costs(case["state"], case["ref"], params, case["contact"])
    b = o.rollout_costs(case["state"], case["ref"], params, case["contact"],
                        cost_terms={"r_force": (0, 0, 0), "w_smooth": 0, "w_cone": 0})
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("key", ["r_force", "w_smooth", "w_cone"])
def test_each_term_is_nonnegative_and_scales(key):
    case = make_case("c2", N=300, method="mppi", seed=5)
    o = case["orc"]
    params = (case["best"][None, :] + case["noise"]).astype(f32)
    base = o.rollout_costs(case["state"], case["ref"], params, case["contact"]).astype(np.float64)
    one = {"r_force": (0, 0, 0), "w_smooth": 0.0, "w_cone": 0.0}
    one[key] = TERMS[key]
    c1 = o.rollout_costs(case["state"], case["ref"], params, case["contact"], cost_terms=one).astype(np.float64)
    two = dict(one)
    two[key] = tuple(2 * np.asarray(TERMS[key])) if key == "r_force" else 2 * TERMS[key]
    c2 = o.rollout_costs(case["state"], case["ref"], params, case["contact"], cost_terms=two).astype(np.float64)
    assert np.all(c1 >= base - 1e-3 * np.abs(base))
    d1, d2 = c1 - base, c2 - base
    assert np.all(d1[1:] > 0) or key == "w_cone"
    np.testing.assert_allclose(d2, 2 * d1, rtol=2e-3, atol=1e-2 * np.abs(base).max() * 1e-5 + 1e-2)


def test_smoothing_zero_for_constant_forces_and_cone_zero_inside():
    N = 7
    rng = np.random.default_rng(0)
    F = rng.uniform(-5, 5, (N, 12)).astype(f32)
    F[:, 2::3] = np.abs(F[:, 2::3]) + 20  # fz > 0, |fx|, |fy| <= 5 < mu fz
    pre = np.stack([F[:, 3 * l + q] for l in range(4) for q in (0, 1)], -1)  # nothing clipped
    cs = np.ones(4, f32)
    e = extra_cost(F, pre, cs, f32(36.8), F.copy(), f32(0.5), {"w_smooth": 1.0, "w_cone": 1.0})
    np.testing.assert_array_equal(e, np.zeros(N, f32))
    pre2 = pre.copy()
    pre2[:, 0] = F[:, 2] * 0.5 + 3.0  # leg 0 x exceeded the cone by 3 before the clip
    e2 = extra_cost(F, pre2, cs, f32(36.8), F.copy(), f32(0.5), {"w_cone": 2.0})
    np.testing.assert_allclose(e2, 2.0 * 9.0, rtol=1e-5)


def test_swing_legs_have_no_gravity_reference():
    """u_z = f_z - fref only for stance legs: a flight step (every leg in swing, fref = inf) stays finite."""
    N = 4
    F = np.zeros((N, 12), f32)
    pre = np.zeros((N, 8), f32)
    e = extra_cost(F, pre, np.zeros(4, f32), f32(np.inf), None, f32(0.5), {"r_force": (0.1, 0.1, 0.001)})
    np.testing.assert_array_equal(e, np.zeros(N, f32))


def test_ga_oracle_terms():
    """The gait-adaptive oracle adds the same terms: zero weights are its plain cost, nonzero add."""
    from oracle.srbd_ga_oracle import GaitAdaptiveOracle, freq_set

    case = make_case("c2", N=64, method="mppi", seed=3)
    w = case["w"]
    o = GaitAdaptiveOracle(pgg_dt=0.02, mass=w.mass, inertia=w.inertia, horizon=w.horizon,
                           num_samples=w.num_samples, method=w.method, parametrization=w.parametrization,
                           num_splines=w.num_splines)
    fs = freq_set(o.method, (1.4, 2.0, 2.4), 1.65, 1)
    freqs = np.random.default_rng(1).choice(fs, o.N).astype(f32)
    params = (case["best"][None, :] + case["noise"]).astype(f32)
    timing = (0.1, 0.6, 0.6, 0.1)
    a = o.rollout_costs_ga(case["state"], case["ref"], params, timing, freqs)
    b = o.rollout_costs_ga(case["state"], case["ref"], params, timing, freqs,
                           cost_terms={"r_force": (0, 0, 0), "w_smooth": 0, "w_cone": 0})
    c = o.rollout_costs_ga(case["state"], case["ref"], params, timing, freqs, cost_terms=TERMS)
    np.testing.assert_array_equal(a, b)
    assert np.all(c[1:] > a[1:])
