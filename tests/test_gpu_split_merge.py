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


def _finish_step(lib, ctx, case, best, sig, counter):
    """srbd_step_local (rank record) + srbd_step_finish on a one-rank context: the split merge runs in the finish."""
    import ctypes as C

    torch = pytest.importorskip("torch")
    rec = torch.zeros(ctx.record_floats(), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    st = np.ascontiguousarray
    b, s = best.copy(), sig.copy()
    rc = lib.lib.srbd_step_local(ctx.h, lib.fptr(st(case["state"])), lib.fptr(st(case["ref"])),
                                 lib.fptr(st(case["contact"])), case["contact"].shape[1], lib.fptr(b), lib.fptr(s),
                                 None, 11, counter, rec.data_ptr())
    assert rc == 0, lib.last_error(ctx.h)
    res = lib.SrbdResult()
    rc = lib.lib.srbd_step_finish(ctx.h, rec.data_ptr(), 1, lib.fptr(b), lib.fptr(s), C.byref(res), None)
    torch.cuda.synchronize()
    if rc != 0:
        raise RuntimeError(lib.last_error(ctx.h))
    return b, s, res


@pytest.mark.parametrize("path", ["step", "finish"])
def test_split_handoff_timeout_recovers(lib, path):
    """a column-split hand-off that times out (srbd_debug_split_drop: slice 1 withholds the weights' sum,
    so the tail block's bounded 2 s wait expires) fails the call -- srbd_step, or srbd_step_finish on the sharded
    path -- and resets the hand-off state; the next step on the same context equals a fresh context's bit for bit
    (status 0, not the timed-out launch's late words)."""
    case = make_case("c3", N=4096, method="cem_mppi", par="cubic_spline", H=16, seed=23)

    def run(ctx, best, sig, k):
        if path == "step":
            b, s, res, _ = ctx.step(case["state"], case["ref"], case["contact"], best, sigma=sig, seed=11, counter=k)
            return b, s, res
        return _finish_step(lib, ctx, case, best, sig, k)

    ctx = lib.Context(product_cfg(case))
    try:
        b1, s1, _ = run(ctx, case["best"].copy(), case["sigma"].copy(), 0)
        ctx.debug_split_drop()
        with pytest.raises(RuntimeError, match="hand-off timed out"):
            run(ctx, b1, s1, 1)
        b2, s2, r2 = run(ctx, b1, s1, 1)
        b3, s3, r3 = run(ctx, b2, s2, 2)
    finally:
        ctx.close()
    fresh = lib.Context(product_cfg(case))
    try:
        fb2, fs2, fr2 = run(fresh, b1, s1, 1)
        fb3, fs3, fr3 = run(fresh, fb2, fs2, 2)
    finally:
        fresh.close()
    for got, want in (((b2, s2, r2), (fb2, fs2, fr2)), ((b3, s3, r3), (fb3, fs3, fr3))):
        np.testing.assert_array_equal(got[0], want[0])
        np.testing.assert_array_equal(got[1], want[1])
        np.testing.assert_array_equal(np.array(got[2].grf, f32), np.array(want[2].grf, f32))
        assert got[2].status == 0 and got[2].best_index == want[2].best_index
