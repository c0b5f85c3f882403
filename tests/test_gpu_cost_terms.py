"""GPU parity of the opt-in cost terms (srbd_set_cost_terms) against oracle/srbd_oracle.py extra_cost.

Tolerances as tests/test_gpu_parity.py: per-sample costs rtol 2e-5 / atol 1e-3.  The thread and
four-lane rollouts form the terms in the same order, so they agree bit for bit; zero weights leave
the reference's cost bit for bit unchanged.
"""
import numpy as np
import pytest

from helpers import f32, make_case, product_cfg

pytestmark = pytest.mark.gpu

TERMS = {"r_force": (0.1, 0.1, 0.001), "w_smooth": 0.01, "w_cone": 5.0}
CASES = [("mppi", "zero_order", 12), ("random_sampling", "zero_order", 10), ("mppi", "linear_spline", 12),
         ("cem_mppi", "cubic_spline", 16), ("mppi", "zero_order", 7)]


@pytest.fixture(scope="module")
def lib():
    from quadruped_pympc_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X")
    return _lib


def gpu_costs(lib, case, terms, monkeypatch=None, mode=None):
    if monkeypatch is not None and mode is not None:
        monkeypatch.setenv("SRBD_ROLLOUT", mode)
    ctx = lib.Context(product_cfg(case))
    try:
        if terms is not None:
            ctx.set_cost_terms(terms["r_force"], terms["w_smooth"], terms["w_cone"])
        _, _, res, costs = ctx.step(case["state"], case["ref"], case["contact"], case["best"], sigma=case["sigma"],
                                    noise=case["noise"], seed=1, counter=2, want_costs=True)
    finally:
        ctx.close()
    return costs, res


@pytest.mark.parametrize("method,par,H", CASES)
def test_cost_terms_match_oracle(lib, method, par, H):
    case = make_case("c2", N=1500, method=method, par=par, H=H, seed=13)
    o = case["orc"]
    params = (case["best"][None, :] + case["noise"]).astype(f32)
    ref = o.saturate(o.rollout_costs(case["state"], case["ref"], params, case["contact"], cost_terms=TERMS))
    costs, _ = gpu_costs(lib, case, TERMS)
    np.testing.assert_allclose(costs, ref, rtol=2e-5, atol=1e-3)
    plain = o.saturate(o.rollout_costs(case["state"], case["ref"], params, case["contact"]))
    assert np.mean(ref > plain) > 0.9  # the terms are in the cost


@pytest.mark.parametrize("method,par,H", CASES[:4])
def test_cost_terms_rollout_variants_bitwise(lib, monkeypatch, method, par, H):
    case = make_case("c2", N=1000, method=method, par=par, H=H, seed=4)
    a, ra = gpu_costs(lib, case, TERMS, monkeypatch, "thread")
    b, rb = gpu_costs(lib, case, TERMS, monkeypatch, "quad")
    np.testing.assert_array_equal(a, b)
    assert ra.best_index == rb.best_index


def test_zero_weights_leave_the_reference_cost(lib):
    case = make_case("c2", N=800, method="mppi", seed=6)
    a, _ = gpu_costs(lib, case, None)
    b, _ = gpu_costs(lib, case, {"r_force": (0.0, 0.0, 0.0), "w_smooth": 0.0, "w_cone": 0.0})
    np.testing.assert_array_equal(a, b)


def test_invalid_weights_rejected(lib):
    case = make_case("c2", N=64, method="mppi", seed=1)
    ctx = lib.Context(product_cfg(case))
    try:
        with pytest.raises(RuntimeError):
            ctx.set_cost_terms((0.1, -1.0, 0.0), 0.0, 0.0)
        with pytest.raises(RuntimeError):
            ctx.set_cost_terms((0.1, 0.1, 0.1), float("nan"), 0.0)
    finally:
        ctx.close()


def test_gait_adaptive_cost_terms_match_oracle(lib):
    from oracle.srbd_ga_oracle import GA_DUTY, GaitAdaptiveOracle, freq_set

    case = make_case("c2", N=900, method="mppi", seed=8)
    w = case["w"]
    o = GaitAdaptiveOracle(pgg_dt=0.02, mass=w.mass, inertia=w.inertia, horizon=w.horizon,
                           num_samples=w.num_samples, method=w.method, parametrization=w.parametrization,
                           num_splines=w.num_splines)
    fs = freq_set(o.method, (1.4, 2.0, 2.4), 1.65, 1)
    freqs = np.random.default_rng(2).choice(fs, o.N).astype(f32)
    timing = (0.1, 0.6, 0.6, 0.1)
    ctx = lib.Context(product_cfg(case))
    try:
        ctx.set_cost_terms(TERMS["r_force"], TERMS["w_smooth"], TERMS["w_cone"])
        ctx.set_gait(timing, 0.02, GA_DUTY, fs, freqs)
        _, _, _, costs = ctx.step(case["state"], case["ref"], case["contact"], case["best"], noise=case["noise"],
                                  seed=1, counter=2, want_costs=True)
    finally:
        ctx.close()
    params = (case["best"][None, :] + case["noise"]).astype(f32)
    ref = o.saturate(o.rollout_costs_ga(case["state"], case["ref"], params, timing, freqs, cost_terms=TERMS))
    np.testing.assert_allclose(costs, ref, rtol=2e-5, atol=1e-3)


def test_cost_terms_toggle_with_graphs(lib):
    """Setting or clearing the terms on a context whose step graph is already captured re-captures it:
    the next step prices the new cost (oracle), and clearing restores the plain cost bit for bit."""
    case = make_case("c2", N=1200, method="mppi", seed=17)
    o = case["orc"]
    params = (case["best"][None, :] + case["noise"]).astype(f32)
    ctx = lib.Context(product_cfg(case, use_graph=True))
    try:
        def step():
            return ctx.step(case["state"], case["ref"], case["contact"], case["best"], noise=case["noise"], seed=1,
                            counter=2, want_costs=True)[3]
        plain = step()
        plain2 = step()  # graph replay
        ctx.set_cost_terms(TERMS["r_force"], TERMS["w_smooth"], TERMS["w_cone"])
        with_terms = step()
        ctx.set_cost_terms((0.0, 0.0, 0.0), 0.0, 0.0)
        cleared = step()
    finally:
        ctx.close()
    np.testing.assert_array_equal(plain, plain2)
    ref = o.saturate(o.rollout_costs(case["state"], case["ref"], params, case["contact"], cost_terms=TERMS))
    np.testing.assert_allclose(with_terms, ref, rtol=2e-5, atol=1e-3)
    np.testing.assert_array_equal(cleared, plain)
