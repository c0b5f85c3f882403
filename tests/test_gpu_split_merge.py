"""GPU: the column-split merge's in-launch hand-off across successive launches.

CEM merges split their columns over blocks that meet through SplitXchg (srbd_core.h): epoch-tagged 8-byte words
(the slices' root sums, the tail block's top-K keys) that a long-lived context reuses launch after launch, the tail
block advancing the epoch.  Successive steps on one context (parameters and sigma carried, device draws) must equal
the same steps each run on a fresh context, whose hand-off area starts zeroed -- bit for bit.
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


@pytest.mark.parametrize("N,par,H", [(4096, "cubic_spline", 16), (65536, "cubic_spline", 16),
                                     (20000, "zero_order", 12)])
def test_split_merge_successive_steps(lib, N, par, H):
    case = make_case("c3", N=N, method="cem_mppi", par=par, H=H, seed=N % 89)
    steps = 6
    ctx = lib.Context(product_cfg(case))
    try:
        best, sig = case["best"].copy(), case["sigma"].copy()
        chain = []
        for k in range(steps):
            best, sig, res, _ = ctx.step(case["state"], case["ref"], case["contact"], best, sigma=sig, seed=11,
                                         counter=k)
            chain.append((best.copy(), sig.copy(), np.array(res.grf, f32), np.array(res.predicted_state, f32),
                          res.best_index))
    finally:
        ctx.close()
    best, sig = case["best"].copy(), case["sigma"].copy()
    for k in range(steps):
        fresh = lib.Context(product_cfg(case))
        try:
            best, sig, res, _ = fresh.step(case["state"], case["ref"], case["contact"], best, sigma=sig, seed=11,
                                           counter=k)
        finally:
            fresh.close()
        want = chain[k]
        assert res.best_index == want[4], k
        np.testing.assert_array_equal(best, want[0], err_msg=f"step {k}")
        np.testing.assert_array_equal(sig, want[1], err_msg=f"step {k}")
        np.testing.assert_array_equal(np.array(res.grf, f32), want[2], err_msg=f"step {k}")
        np.testing.assert_array_equal(np.array(res.predicted_state, f32), want[3], err_msg=f"step {k}")
        assert np.all(np.isfinite(sig)) and np.all(sig >= 0.2) and np.all(sig <= 5.0)
