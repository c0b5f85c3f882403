"""Host steps at unfused sizes (N > 65 536, the thread rollout; the draws are made by rng_kernel ahead of
each step's rollout, nothing is prefetched) on one long-lived context.

Every output must equal, bit for bit, a fresh context's first step with the same inputs, whatever the call
sequence: counters that follow on, jumps and repeats, another seed, injected noise in between, and other
entry points (device-resident steps, a checkpoint restore) between host steps.  (Round 3 measured three
placements of the next step's draws for these sizes -- a low-priority side stream after the rollout, the
side stream at once, extra blocks of the merge launch -- against this ordering: C5 on one GPU 208.9 / 217 /
202.0 us vs 201.0 us per host step, so none was kept)
Reference: centroidal_nmpc_jax.py:806-812 (the draws), :828-836 (MPPI update), :1075-1081 (CEM sigma).
"""
import numpy as np
import pytest

from helpers import f32, make_case, product_cfg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from quadruped_pympc_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X")
    return _lib


def _fresh(lib, case, best, sigma, seed, counter):
    ctx = lib.Context(product_cfg(case))
    try:
        b, s, res, costs = ctx.step(case["state"], case["ref"], case["contact"], best, sigma=sigma, seed=seed,
                                    counter=counter, want_costs=True)
    finally:
        ctx.close()
    return b, s, res, costs


def _same(a, b):
    ba, sa, ra, ca = a
    bb, sb, rb, cb = b
    np.testing.assert_array_equal(ba, bb)
    if sa is not None:
        np.testing.assert_array_equal(sa, sb)
    np.testing.assert_array_equal(np.array(ra.grf, f32), np.array(rb.grf, f32))
    np.testing.assert_array_equal(np.array(ra.predicted_state, f32), np.array(rb.predicted_state, f32))
    assert ra.best_index == rb.best_index
    np.testing.assert_array_equal(ca, cb)


@pytest.mark.parametrize("method", ["mppi", "cem_mppi", "random_sampling"])
def test_unfused_steps_match_fresh_contexts(lib, method):
    N = 70000  # above the fuse limit (65 536): the thread rollout, draws made ahead of each rollout
    case = make_case("c2", N=N, method=method)
    sigma = case["sigma"]
    ctx = lib.Context(product_cfg(case))
    try:
        # (seed, counter, injected noise?)
        calls = [(42, 5, False), (42, 6, False), (42, 7, False), (42, 12, False), (42, 12, False),
                 (7, 13, False), (7, 14, True), (7, 15, False), (7, 16, False)]
        best = case["best"].copy()
        for seed, ctr, inj in calls:
            if inj:
                got = ctx.step(case["state"], case["ref"], case["contact"], best, sigma=sigma, noise=case["noise"],
                               seed=seed, counter=ctr, want_costs=True)
                continue
            got = ctx.step(case["state"], case["ref"], case["contact"], best, sigma=sigma, seed=seed, counter=ctr,
                           want_costs=True)
            _same(got, _fresh(lib, case, best, sigma, seed, ctr))
            best = got[0]  # carried warm start: each call's inputs differ
            if sigma is not None:
                sigma = got[1]
    finally:
        ctx.close()


def test_unfused_steps_around_other_entry_points(lib):
    """Device-resident steps and a checkpoint restore between host steps leave the following host steps
    equal to fresh contexts."""
    N = 70000
    case = make_case("c2", N=N, method="mppi")
    ctx = lib.Context(product_cfg(case))
    try:
        best = case["best"].copy()
        a = ctx.step(case["state"], case["ref"], case["contact"], best, seed=42, counter=1)
        st = ctx.get_state()
        ctx.bench_device_steps(3)  # device-resident chain on the same noise buffers
        ctx.set_state(*st)
        for ctr in (2, 3):
            got = ctx.step(case["state"], case["ref"], case["contact"], a[0], seed=42, counter=ctr, want_costs=True)
            _same(got, _fresh(lib, case, a[0], None, 42, ctr))
            a = got
    finally:
        ctx.close()
