"""Known-answer tests pinning the CPU oracles (SURVEY 8(c) "analytic known-answer tests").

The reference ships no tests or golden vectors and cannot run here (JAX absent), so the
oracle's parity with the reference is unpinned; these tests pin it to the physics and to the
reference's stated semantics, and pin the numpy and C restatements to each other.
"""
import numpy as np
import pytest

from oracle import c_oracle as co
from oracle.srbd_oracle import (CentroidalModel, SamplingMPCOracle, calculate_inverse, num_params_single_leg,
                                prepare_state_and_reference)
from quadruped_pympc_amd.config import ROBOTS
from quadruped_pympc_amd.synthetic import CONFIGS, inputs

f32 = np.float32


@pytest.mark.parametrize("robot", sorted(ROBOTS))
def test_calculate_inverse_matches_numpy(robot):
    I = np.asarray(ROBOTS[robot][1], dtype=f32)
    np.testing.assert_allclose(calculate_inverse(I), np.linalg.inv(I.astype(np.float64)), rtol=2e-6, atol=1e-7)


def model(robot="go2", H=12):
    m, I = ROBOTS[robot]
    return CentroidalModel(m, I, 0.02, H)


def test_free_fall():
    """No contact: v_z -= 9.81 dt after one Euler step; the position uses the old velocity (unchanged)."""
    m = model()
    x = np.zeros((1, 24), f32)
    x[0, 2] = 0.3
    x[0, 12:] = [0.19, 0.13, 0, 0.19, -0.13, 0, -0.19, 0.13, 0, -0.19, -0.13, 0]
    out = m.integrate(x, np.ones((1, 12), f32) * 7, np.zeros(4, f32), 0)
    assert out[0, 5] == f32(f32(-9.81) * f32(0.02))
    np.testing.assert_array_equal(out[0, 0:3], x[0, 0:3])
    np.testing.assert_array_equal(out[0, 12:], x[0, 12:])


def test_static_stance_equilibrium():
    """Feet symmetric about the CoM, f_i = (0, 0, mg/4), level base: zero linear and angular acceleration."""
    m = model()
    x = np.zeros((1, 24), f32)
    x[0, 12:] = [0.19, 0.13, -0.3, 0.19, -0.13, -0.3, -0.19, 0.13, -0.3, -0.19, -0.13, -0.3]
    F = np.zeros((1, 12), f32)
    F[0, 2::3] = f32(m.mass * 9.81 / 4)
    d = m.fd(x, F, np.ones(4, f32))
    np.testing.assert_allclose(d[0, 3:6], 0, atol=1e-5)
    np.testing.assert_allclose(d[0, 9:12], 0, atol=1e-5)


def case(method="mppi", par="zero_order", N=64, H=12, S=2, seed=0, key="c2"):
    w = CONFIGS[key]
    o = SamplingMPCOracle(mass=w.mass, inertia=w.inertia, horizon=H, num_samples=N, method=method,
                          parametrization=par, num_splines=S)
    s, r, c = inputs(w, 1)
    rng = np.random.default_rng(seed)
    t = N // 3
    noise = o.assemble_noise(rng.standard_normal((N - 1, o.P)).astype(f32), sigma=np.full(o.P, 3, f32),
                             U=rng.uniform(-10, 10, (N - 1 - 2 * t, o.P)).astype(f32))
    return o, s.astype(f32), r.astype(f32), c[:, :H].astype(f32), noise, rng.standard_normal(o.P).astype(f32)


@pytest.mark.parametrize("method", ["mppi", "cem_mppi", "random_sampling"])
def test_zero_noise_keeps_parameters(method):
    """N = 1: only the warm-start row exists; the update is exactly zero."""
    o, s, r, c, _, best = case(method, N=1)
    out = o.compute_control(s, r, c, best, np.zeros((1, o.P), f32))
    np.testing.assert_array_equal(out["best"], best)
    assert out["best_index"] == 0


def test_no_stance_gives_zero_forces():
    """n_stance = 0: inf reference force, neutralised by the compare-select clip (App. A.3)."""
    o, s, r, c, noise, best = case()
    out = o.compute_control(s, r, np.zeros_like(c), best, noise)
    assert np.all(out["grf"] == 0)
    assert np.isfinite(out["costs"]).all()


def test_cubic_spline_identities():
    o, *_ = case(par="cubic_spline", H=16)
    p = np.tile(np.arange(o.PL, dtype=f32), (2, 1))
    fx, fy, fz = o.spline(p, 0.0, 1)
    np.testing.assert_array_equal([fx[0], fy[0], fz[0]], [1, 5, 9])
    const = np.full((1, o.PL), 2.5, f32)
    for n in range(16):
        vals = o.spline(const, n, 16)
        np.testing.assert_allclose([v[0] for v in vals], 2.5, rtol=1e-6)


def test_linear_spline_identities():
    o, *_ = case(par="linear_spline", H=12)
    p = np.tile(np.arange(o.PL, dtype=f32), (1, 1))
    fx, fy, fz = o.spline(p, 0.0, 1)
    np.testing.assert_array_equal([fx[0], fy[0], fz[0]], [0, 3, 6])
    fx, _, _ = o.spline(p, 3, 12)  # halfway through chunk 0 of 6 steps: lerp(p0, p1, 0.5)
    assert fx[0] == f32(0.5)


def test_params_per_leg():
    assert num_params_single_leg(0, 12, 2) == 36
    assert num_params_single_leg(1, 12, 2) == 9
    assert num_params_single_leg(2, 16, 2) == 24


@pytest.mark.parametrize("par,H,key", [("zero_order", 12, "c2"), ("linear_spline", 12, "c2"),
                                       ("cubic_spline", 16, "c3"), ("zero_order", 10, "c1")])
def test_numpy_and_c_oracles_agree(par, H, key):
    o, s, r, c, noise, best = case("mppi", par, N=1500, H=H, key=key, seed=3)
    a = o.rollout_costs(s, r, best[None] + noise, c)
    w = CONFIGS[key]
    cfg = co.make_cfg(N=1500, H=H, method=1, param_kind=o.param_kind, mass=w.mass, inertia=w.inertia)
    b = co.rollout_costs(cfg, s, r, c, best, noise)
    np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-4)
    assert np.mean(a == b) > 0.95  # the two restatements agree bit for bit on almost every sample


def test_c_oracle_full_step_matches_numpy():
    o, s, r, c, noise, best = case("mppi", N=800, seed=5)
    ref = o.compute_control(s, r, c, best, noise)
    w = CONFIGS["c2"]
    cfg = co.make_cfg(N=800, H=12, method=1, param_kind=0, mass=w.mass, inertia=w.inertia)
    nb, _, grf, pred, bc, bi, costs = co.step(cfg, s, r, c, best, noise=noise)
    assert bi == ref["best_index"]
    np.testing.assert_allclose(nb, ref["best"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(grf, ref["grf"], rtol=1e-5, atol=1e-4)


def test_random_sampling_blocks_share_draws():
    """Rows t+1..2t reuse rows 1..t's standard normals scaled 3/0.2 = 15x (App. B #3)."""
    o, *_ = case("random_sampling", N=31)
    rng = np.random.default_rng(0)
    Z = rng.standard_normal((30, o.P)).astype(f32)
    U = rng.uniform(-10, 10, (30 - 20, o.P)).astype(f32)
    n = o.assemble_noise(Z, U=U)
    t = 10
    np.testing.assert_allclose(n[1 + t:1 + 2 * t], f32(3) * Z[:t])
    np.testing.assert_allclose(n[1:1 + t], f32(0.2) * Z[:t])
    assert np.all(np.abs(n[1 + 2 * t:]) <= 10)


def test_saturation():
    c = np.array([1.0, np.nan, np.inf, -np.inf, 5.0], f32)
    np.testing.assert_array_equal(SamplingMPCOracle.saturate(c), [1, 1e6, 1e6, 1e6, 5])


def test_cem_sigma_bounds():
    o, s, r, c, noise, best = case("cem_mppi", N=300, seed=9)
    out = o.compute_control(s, r, c, best, noise)
    assert out["sigma"].shape == (o.P,)
    assert np.all(out["sigma"] >= f32(0.2)) and np.all(out["sigma"] <= 5)
    idx = out["elite"]
    assert list(idx) == sorted(range(300), key=lambda k: (out["costs"][k], k))[:10]


def test_prepare_state_and_reference():
    sc = {k: np.arange(3, dtype=float) + i for i, k in enumerate(
        ["position", "linear_velocity", "orientation", "angular_velocity", "foot_FL", "foot_FR", "foot_RL", "foot_RR"])}
    rs = {k: np.full(3, 10.0 + i) for i, k in enumerate(
        ["ref_position", "ref_linear_velocity", "ref_orientation", "ref_angular_velocity", "ref_foot_FL", "ref_foot_FR",
         "ref_foot_RL", "ref_foot_RR"])}
    best = np.ones(144, f32)
    s, r, b = prepare_state_and_reference(sc, rs, np.array([1, 0, 1, 0]), np.array([1, 1, 1, 1]), best, 36)
    np.testing.assert_array_equal(s[15:18], rs["ref_foot_FR"])  # swing foot <- reference foot
    np.testing.assert_array_equal(s[12:15], sc["foot_FL"])
    assert np.all(b[36:72] == 0) and np.all(b[108:144] == 0) and np.all(b[:36] == 1)  # lift-off zeroing
