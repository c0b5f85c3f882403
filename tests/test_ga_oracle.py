"""Known-answer tests pinning the gait-adaptive oracle (oracle/srbd_ga_oracle.py), CPU only.

The reference (centroidal_nmpc_jax_gait_adaptive.py, periodic_gait_generator_jax.py) cannot run
here (JAX absent): parity unpinned.  These tests pin the vectorised restatement to a literal
per-sample scalar restatement of the same reference lines, and to the base oracle where the two
reference files coincide (an all-stance contact sequence).
"""
import numpy as np
import pytest

from oracle.srbd_ga_oracle import GA_DUTY, GaitAdaptiveOracle, freq_set, pgg_jax_contact_sequences
from oracle.srbd_oracle import CUBIC_SPLINE, LINEAR_SPLINE, MPPI, RANDOM_SAMPLING, ZERO_ORDER, CEM_MPPI, \
    SamplingMPCOracle
from quadruped_pympc_amd.synthetic import CONFIGS, inputs

f32 = np.float32


def scalar_pgg(timing, f, H, dt, duty=GA_DUTY):
    """periodic_gait_generator_jax.py:68-89, 136-151 written out with scalars."""
    t = [f32(v) for v in timing]
    seq = np.zeros((4, H), f32)
    for n in range(H):
        for leg in range(4):
            t[leg] = f32(0) if t[leg] >= f32(1.0) else t[leg]
            t[leg] = f32(t[leg] + f32(f32(dt) * f32(f)))
            seq[leg, n] = 1.0 if t[leg] < f32(duty) else 0.0
    return seq


@pytest.mark.parametrize("timing", [(0, 0.5, 0.5, 0), (0.64, 0.66, 0.99, 1.0), (0.3, 0.1, 0.9, 0.6)])
def test_pgg_jax_restatement_matches_scalar_loop(timing):
    freqs = np.array([0.5, 1.3, 1.4, 2.0, 2.4, 3.7], f32)
    cs = pgg_jax_contact_sequences(timing, freqs, 16, 0.02)
    for i, f in enumerate(freqs):
        np.testing.assert_array_equal(cs[i], scalar_pgg(timing, f, 16, 0.02))


def ga_case(par="zero_order", method="mppi", N=48, H=12, S=2, seed=0):
    w = CONFIGS["c2"]
    kw = dict(mass=w.mass, inertia=w.inertia, horizon=H, num_samples=N, method=method, parametrization=par,
              num_splines=S)
    return GaitAdaptiveOracle(pgg_dt=0.02, **kw), SamplingMPCOracle(**kw), w


def test_all_stance_reduces_to_base_zero_order_plus_frequency_cost():
    """t = 0 and f = 1 keep every leg in stance over H = 12 (t <= 0.24 < 0.65): the counter n_ is
    the step n, so the GA rollout is the base rollout with an all-ones contact plus (f-1.3)*100*(f-1.3)."""
    ga, base, w = ga_case()
    s, r, _ = inputs(w, 1)
    rng = np.random.default_rng(3)
    params = (3 * rng.standard_normal((ga.N, ga.P))).astype(f32)
    freqs = np.full(ga.N, 1.0, f32)
    got = ga.rollout_costs_ga(s, r, params, (0, 0, 0, 0), freqs)
    ref = base.rollout_costs(s, r, params, np.ones((4, ga.horizon), f32))
    d = f32(f32(1.0) - f32(1.3))
    np.testing.assert_array_equal(got, (ref + f32(f32(d * f32(100)) * d)).astype(f32))


def test_zero_order_negative_index_wraps():
    """A leg that has not touched down yet has n_ = -1: jnp indexing wraps params[-1] to the leg's
    last parameter (GA:274-277 under jnp's negative-index rule)."""
    ga, _, _ = ga_case(N=2)
    p = np.arange(2 * ga.PL, dtype=f32).reshape(2, ga.PL)
    fx, fy, fz = ga.spline_vec(p, np.array([-1, 4], np.int32), np.array([1, 6], f32))
    H = ga.horizon
    np.testing.assert_array_equal(fx, [p[0, ga.PL - 1], p[1, 4]])
    np.testing.assert_array_equal(fy, [p[0, H - 1], p[1, 4 + H]])
    np.testing.assert_array_equal(fz, [p[0, 2 * H - 1], p[1, 4 + 2 * H]])


def scalar_decode(kind, H, S, p, step, hl):
    """GA:190-278 for one leg, scalars (step: int counter, hl: float32 horizon_leg)."""
    PL = len(p)

    def at(j):
        return p[j + PL if j < 0 else j]

    if kind == ZERO_ORDER:
        return at(step), at(step + H), at(step + 2 * H)
    cb = np.linspace(0, H, S + 1).astype(f32)
    index = max([k if f32(step) >= cb[k] else 0 for k in range(S + 1)])
    tau = f32(f32(step) / f32(f32(hl) / f32(S)))
    q = f32(f32(tau - f32(index)) / f32(1.0))
    if kind == LINEAR_SPLINE:
        sh = S + 1
        omq = f32(f32(1) - q)
        return tuple(f32(f32(omq * at(index + o)) + f32(q * at(index + o + 1))) for o in (0, sh, 2 * sh))
    a = f32(f32(f32(f32(f32(2) * q) * q) * q) - f32(f32(f32(3) * q) * q)) + f32(1)
    b = f32(f32(f32(f32(q * q) * q) - f32(f32(f32(2) * q) * q)) + q)
    c = f32(f32(f32(f32(-f32(2)) * q) * q) * q) + f32(f32(f32(3) * q) * q)
    d = f32(f32(f32(q * q) * q) - f32(q * q))
    s = 10 * index
    out = []
    for o in (0, 4, 8):
        p0, p1, p2, p3 = at(s + o), at(s + o + 1), at(s + o + 2), at(s + o + 3)
        phi = f32(f32(0.5) * f32(f32(p2 - p1) + f32(p1 - p0)))
        phin = f32(f32(0.5) * f32(f32(p3 - p2) + f32(p2 - p1)))
        out.append(f32(f32(f32(f32(a * p1) + f32(b * phi)) + f32(c * p2)) + f32(d * phin)))
    return tuple(out)


@pytest.mark.parametrize("par,S", [("zero_order", 2), ("linear_spline", 2), ("linear_spline", 3),
                                   ("cubic_spline", 2)])
def test_vectorised_decode_matches_scalar(par, S):
    ga, _, _ = ga_case(par=par, S=S, N=40)
    rng = np.random.default_rng(11)
    p = rng.standard_normal((40, ga.PL)).astype(f32)
    steps = rng.integers(-1, ga.horizon, 40).astype(np.int32)
    hl = rng.integers(1, ga.horizon + 2, 40).astype(f32)
    fx, fy, fz = ga.spline_vec(p, steps, hl)
    for i in range(40):
        e = scalar_decode(ga.param_kind, ga.horizon, S, p[i], int(steps[i]), hl[i])
        np.testing.assert_array_equal([fx[i], fy[i], fz[i]], e)


def test_freq_sets():
    avail = [1.4, 2.0, 2.4]
    np.testing.assert_array_equal(freq_set(RANDOM_SAMPLING, avail, 1.65, 1), np.array(avail, f32))
    np.testing.assert_array_equal(freq_set(RANDOM_SAMPLING, avail, 1.65, 0), np.full(3, f32(1.65)))
    np.testing.assert_array_equal(freq_set(MPPI, avail, 1.65, 0), np.array(avail, f32))
    np.testing.assert_array_equal(freq_set(CEM_MPPI, avail, 1.65, 1),
                                  np.array([1.65, f32(f32(0.2) + f32(1.65)), f32(f32(0.4) + f32(1.65))], f32))


@pytest.mark.parametrize("method", ["mppi", "random_sampling"])
def test_compute_control_ga_best_freq_is_the_argmin_rows(method):
    ga, _, w = ga_case(method=method, par="linear_spline", N=30)
    s, r, c = inputs(w, 2)
    rng = np.random.default_rng(5)
    noise = np.zeros((30, ga.P), f32)
    noise[1:] = 2 * rng.standard_normal((29, ga.P))
    freqs = rng.choice(np.array([1.4, 2.0, 2.4], f32), 30)
    out = ga.compute_control_ga(s, r, c, np.zeros(ga.P, f32), noise, freqs, (0.1, 0.6, 0.6, 0.1))
    assert out["best_freq"] == freqs[out["best_index"]]
    assert out["best_index"] == int(np.argmin(out["costs"]))
