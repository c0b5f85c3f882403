"""GPU: the fixed reduction tree (srbd_core.h tree_shape) makes a step's result independent of the world size.

Each world size W in {2, 3, 5, 8} runs as W contexts of one GPU: srbd_step_local writes every rank's buffer
(its exchange-level node records), srbd_step_finish folds the gathered buffers to the root.  The merged step
must equal the unsharded srbd_step bit for bit -- parameters, sigma (CEM), GRFs, predicted state, winner --
whatever the rollout form, the in-launch level-1 fold (N > 16 384) or the level the ranks exchange at.
"""
import ctypes as C

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


def unsharded(lib, case):
    cx = lib.Context(product_cfg(case))
    try:
        b, s, res, _ = cx.step(case["state"], case["ref"], case["contact"], case["best"], sigma=case["sigma"],
                               noise=case["noise"])
        return b, s, np.array(res.grf, f32), np.array(res.predicted_state, f32), res.best_index
    finally:
        cx.close()


def sharded(lib, case, W):
    import torch

    ctxs = [lib.Context(product_cfg(case, rank=r, world_size=W)) for r in range(W)]
    try:
        rec_f = ctxs[0].record_floats()
        assert all(cx.record_floats() == rec_f for cx in ctxs)
        assert sum(cx.n_local for cx in ctxs) == case["noise"].shape[0]
        recs = torch.zeros((W, rec_f), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        st = np.ascontiguousarray
        cem = case["sigma"] is not None and ctxs[0].cfg.method == lib.CEM_MPPI
        sig = st(case["sigma"]) if cem else None
        for r, cx in enumerate(ctxs):
            rows = st(case["noise"][cx.row0:cx.row0 + cx.n_local])
            rc = lib.lib.srbd_step_local(cx.h, lib.fptr(st(case["state"])), lib.fptr(st(case["ref"])),
                                         lib.fptr(st(case["contact"])), case["contact"].shape[1],
                                         lib.fptr(st(case["best"])), lib.fptr(sig), lib.fptr(rows), 42, 1,
                                         recs[r].data_ptr())
            assert rc == 0, lib.last_error(cx.h)
        torch.cuda.synchronize()
        outs = []
        for cx in ctxs:
            best = case["best"].copy()
            sg = sig.copy() if cem else None
            res = lib.SrbdResult()
            rc = lib.lib.srbd_step_finish(cx.h, recs.data_ptr(), W, lib.fptr(best), lib.fptr(sg), C.byref(res), None)
            assert rc == 0, lib.last_error(cx.h)
            outs.append((best, sg, np.array(res.grf, f32), np.array(res.predicted_state, f32), res.best_index))
        return outs
    finally:
        for cx in ctxs:
            cx.close()


@pytest.mark.parametrize("wkey,N,method,par,H", [
    ("c2", 5000, "mppi", "zero_order", 12),           # 79 leaves: ranks exchange leaves or level-1 nodes
    ("c2", 70001, "mppi", "zero_order", 12),          # 1094 leaves, 3 levels: level-1 fold in the rollout launch
    ("c3", 65536, "cem_mppi", "cubic_spline", 16),    # CEM: elite rows through the rank buffers
    ("c1", 20000, "random_sampling", "linear_spline", 12),
])
def test_sharded_step_is_world_invariant(lib, wkey, N, method, par, H):
    case = make_case(wkey, N=N, method=method, par=par, H=H, seed=N % 97)
    want = unsharded(lib, case)
    for W in (2, 3, 5, 8):
        for got in sharded(lib, case, W):
            assert got[4] == want[4], (W, got[4], want[4])
            np.testing.assert_array_equal(got[0], want[0], err_msg=f"W={W}")
            if method == "cem_mppi":
                np.testing.assert_array_equal(got[1], want[1], err_msg=f"W={W}")
            np.testing.assert_array_equal(got[2], want[2], err_msg=f"W={W}")
            np.testing.assert_array_equal(got[3], want[3], err_msg=f"W={W}")


def test_too_many_ranks_is_an_error(lib):
    case = make_case("c2", N=300, method="mppi")  # 5 leaves
    with pytest.raises((RuntimeError, ValueError), match="too few rows"):
        lib.Context(product_cfg(case, rank=0, world_size=8))
