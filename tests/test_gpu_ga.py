"""GPU parity of the gait-adaptive sampling MPC against oracle/srbd_ga_oracle.py.

Tolerances as tests/test_gpu_parity.py: per-sample costs rtol 2e-5 / atol 1e-3; the oracle's
reduction fed with the GPU's costs reproduces the GPU step (params rtol 1e-5 / atol 1e-4, GRFs
rtol 1e-5 / atol 1e-3); the best step frequency is the injected frequency of the best row
(exact).  Device-drawn frequencies are reproduced exactly with the oracle's Philox4x32-10.
"""
import numpy as np
import pytest

from helpers import f32, make_case, product_cfg
from oracle import c_oracle as co
from oracle.srbd_ga_oracle import GA_DUTY, GaitAdaptiveOracle, freq_set, pgg_jax_contact_sequences

pytestmark = pytest.mark.gpu

COST_RTOL, COST_ATOL = 2e-5, 1e-3
AVAIL = (1.4, 2.0, 2.4)
TIMINGS = [(0.1, 0.6, 0.6, 0.1), (0.0, 0.5, 0.5, 0.0), (0.64, 0.99, 1.0, 0.3)]


@pytest.fixture(scope="module")
def lib():
    from quadruped_pympc_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X")
    return _lib


def ga_oracle(case):
    w = case["w"]
    return GaitAdaptiveOracle(pgg_dt=0.02, mass=w.mass, inertia=w.inertia, horizon=w.horizon,
                              num_samples=w.num_samples, method=w.method, parametrization=w.parametrization,
                              num_splines=w.num_splines)


def device_freqs(fs, N, seed, counter):
    """The library's device draw (rollout_ga_kernel / ga_sample_freq): Philox4x32-10 on counter
    (row, 0x10000, counter lo, counter hi), key = seed; index = hi32(c0 * n)."""
    out = np.empty(N, f32)
    key = (seed & 0xFFFFFFFF, seed >> 32)
    for r in range(N):
        c0 = co.philox((r, 0x10000, counter & 0xFFFFFFFF, counter >> 32), key)[0]
        out[r] = fs[(int(c0) * len(fs)) >> 32]
    return out


def run(lib, case, timing, fs, freqs, seed=42, counter=3, noise=True):
    ctx = lib.Context(product_cfg(case))
    try:
        ctx.set_gait(timing, 0.02, GA_DUTY, fs, freqs)
        best, _, res, costs = ctx.step(case["state"], case["ref"], case["contact"], case["best"],
                                       noise=case["noise"] if noise else None, seed=seed, counter=counter,
                                       want_costs=True)
    finally:
        ctx.close()
    return best, res, costs


@pytest.mark.parametrize("par,H", [("zero_order", 12), ("linear_spline", 12), ("cubic_spline", 16),
                                   ("zero_order", 10)])
@pytest.mark.parametrize("method", ["mppi", "random_sampling"])
@pytest.mark.parametrize("ti", [0, 2])
def test_ga_step_matches_oracle(lib, par, H, method, ti):
    case = make_case("c2", N=1500, method=method, par=par, H=H, seed=7 + ti)
    o = ga_oracle(case)
    rng = np.random.default_rng(ti)
    fs = freq_set(o.method, AVAIL, 1.65, 1)
    freqs = rng.choice(fs, o.N).astype(f32)
    best, res, costs = run(lib, case, TIMINGS[ti], fs, freqs)
    params = (case["best"][None, :] + case["noise"]).astype(f32)
    ref_costs = o.saturate(o.rollout_costs_ga(case["state"], case["ref"], params, TIMINGS[ti], freqs))
    np.testing.assert_allclose(costs, ref_costs, rtol=COST_RTOL, atol=COST_ATOL)
    r = o.reduce(case["state"], case["contact"], case["best"], case["noise"], costs)
    assert res.best_index == r["best_index"]
    np.testing.assert_allclose(best, r["best"], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(np.array(res.grf, f32), r["grf"], rtol=1e-5, atol=1e-3)
    assert res.best_freq == freqs[res.best_index]


def test_ga_contact_sequences_reach_the_kernel(lib):
    """Legs in swing for the whole horizon contribute no force: with every leg in swing the GA cost
    is the free-fall cost plus the frequency term, for any parameters."""
    case = make_case("c2", N=300, method="mppi", seed=3)
    o = ga_oracle(case)
    timing = (0.7, 0.7, 0.7, 0.7)  # t in (0.65, 1): swing until the restart at t >= 1
    freqs = np.full(o.N, 0.5, f32)  # 0.7 + 12 * 0.01 < 1: no restart within the horizon
    assert pgg_jax_contact_sequences(timing, freqs[:1], 12, 0.02).sum() == 0
    _, _, costs = run(lib, case, timing, np.array([0.5], f32), freqs)
    assert np.all(costs == costs[0])
    params = (case["best"][None, :] + case["noise"]).astype(f32)
    ref_costs = o.saturate(o.rollout_costs_ga(case["state"], case["ref"], params, timing, freqs))
    np.testing.assert_allclose(costs, ref_costs, rtol=COST_RTOL, atol=COST_ATOL)


@pytest.mark.parametrize("method", ["mppi", "random_sampling"])
def test_ga_device_frequency_draw(lib, method):
    case = make_case("c2", N=700, method=method, seed=9)
    o = ga_oracle(case)
    fs = freq_set(o.method, AVAIL, 1.65, 1)
    seed, counter = 42 + (1 << 33), 5 + (1 << 32)
    freqs = device_freqs(fs, o.N, seed, counter)
    assert len(set(freqs.tolist())) == len(fs)
    _, res, costs = run(lib, case, TIMINGS[0], fs, None, seed=seed, counter=counter)
    params = (case["best"][None, :] + case["noise"]).astype(f32)
    ref_costs = o.saturate(o.rollout_costs_ga(case["state"], case["ref"], params, TIMINGS[0], freqs))
    np.testing.assert_allclose(costs, ref_costs, rtol=COST_RTOL, atol=COST_ATOL)
    assert res.best_freq == freqs[res.best_index]


def test_ga_clear_returns_to_plain_path(lib):
    case = make_case("c2", N=500, method="mppi", seed=4)
    ctx = lib.Context(product_cfg(case))
    try:
        b0, _, r0, c0 = ctx.step(case["state"], case["ref"], case["contact"], case["best"], noise=case["noise"],
                                 want_costs=True)
        ctx.set_gait(TIMINGS[0], 0.02, GA_DUTY, np.array(AVAIL, f32), None)
        _, _, r1, c1 = ctx.step(case["state"], case["ref"], case["contact"], case["best"], noise=case["noise"],
                                want_costs=True)
        assert not np.array_equal(c0, c1) and r1.best_freq in np.array(AVAIL, f32)
        ctx.clear_gait()
        b2, _, r2, c2 = ctx.step(case["state"], case["ref"], case["contact"], case["best"], noise=case["noise"],
                                 want_costs=True)
        np.testing.assert_array_equal(c0, c2)
        np.testing.assert_array_equal(b0, b2)
        assert r2.best_freq == 0.0
    finally:
        ctx.close()


def test_ga_cem_rejected(lib):
    case = make_case("c3", N=256, method="cem_mppi", seed=1)
    ctx = lib.Context(product_cfg(case))
    try:
        with pytest.raises(RuntimeError, match="gait-adaptive CEM"):
            ctx.set_gait(TIMINGS[0], 0.02, GA_DUTY, np.array(AVAIL, f32), None)
    finally:
        ctx.close()


def test_ga_device_chain_runs(lib):
    """Device-resident chain (graphs recaptured after set_gait) keeps producing finite outputs."""
    case = make_case("c2", N=2000, method="mppi", seed=2)
    ctx = lib.Context(product_cfg(case))
    try:
        ctx.set_gait(TIMINGS[1], 0.02, GA_DUTY, np.array(AVAIL, f32), None)
        ctx.step(case["state"], case["ref"], case["contact"], case["best"])
        ms = ctx.bench_device_steps(9)
        assert ms > 0
        best, _, res, _ = ctx.step(case["state"], case["ref"], case["contact"], case["best"], counter=77)
        assert np.all(np.isfinite(best)) and res.best_freq in np.array(AVAIL, f32)
    finally:
        ctx.close()


def test_interface_gait_adaptive_mppi(lib):
    """SRBDControllerInterface with optimize_step_freq selects the gait-adaptive Sampling_MPC and
    returns a sampled best step frequency (srbd_controller_interface.py:77-81, :150-168)."""
    from quadruped_pympc_amd.interfaces.srbd_controller_interface import SRBDControllerInterface
    from test_host_logic import cfg_module, dicts

    cfg = cfg_module(optimize_step_freq=True, sampling_method="mppi", control_parametrization="zero_order",
                     num_parallel_computations=2000)
    itf = SRBDControllerInterface(cfg)
    sc, rs = dicts(np.random.default_rng(4))
    contact = np.ones((4, 12))
    out = itf.compute_control(sc, rs, contact, None, np.array([0.1, 0.6, 0.6, 0.1]), 1.65, 1)
    assert out[5] in np.array(cfg.mpc_params["step_freq_available"], f32)
    itf.controller.close()


@pytest.mark.parametrize("par,H", [("zero_order", 12), ("linear_spline", 12), ("cubic_spline", 16),
                                   ("zero_order", 10)])
@pytest.mark.parametrize("method", ["mppi", "random_sampling"])
@pytest.mark.parametrize("device_freqs", [False, True])
def test_ga_rollout_variants_bitwise(lib, monkeypatch, par, H, method, device_freqs):
    """rollout_ga_quad_kernel (four lanes per sample) gives rollout_ga_kernel's costs bit for bit."""
    case = make_case("c2", N=1000, method=method, par=par, H=H, seed=21)
    o = ga_oracle(case)
    fs = freq_set(o.method, AVAIL, 1.65, 1)
    freqs = None if device_freqs else np.random.default_rng(5).choice(fs, o.N).astype(f32)
    out = {}
    for mode in ("thread", "quad"):
        monkeypatch.setenv("SRBD_ROLLOUT", mode)
        _, res, costs = run(lib, case, TIMINGS[1], fs, freqs)
        out[mode] = (costs, res.best_index, res.best_freq)
    np.testing.assert_array_equal(out["thread"][0], out["quad"][0])
    assert out["thread"][1:] == out["quad"][1:]
