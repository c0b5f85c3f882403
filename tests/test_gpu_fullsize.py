"""Full-size GPU parity: the BASELINE.json shapes against the OpenMP C oracle (tests/ only use the oracle).

Covers the shapes the small cases do not reach:
  * C2 exactly (MPPI, zero-order, H=12, N=10 000 -> 157 four-lane block records, one merge block);
  * the north-star target shape (MPPI, zero-order, H=12, N=65 536 -> 1024 block records, split merge);
  * the one-thread-per-sample rollout (zero-order above 65 536 rows) at N=262 144 for MPPI, random
    sampling and CEM (1024 records of 256 rows);
  * the two-level merge tree (> 1024 block records): C5's N=524 288 on one context (2048 records),
    and linear-spline MPPI at N=100 000 (1563 four-lane records);
  * C5 sharded 8 ways (8 contexts of one GPU, rank records merged by srbd_step_finish) against the
    unsharded C5 step.
Noise is injected (parity mode), so both sides roll out identical perturbations.  Costs: rtol 2e-5,
atol 1e-3 against the C oracle (same float order, -ffp-contract=off).  Reduction: the numpy oracle's
reduce() fed with the GPU's costs reproduces the GPU (params rtol 1e-5 / atol 1e-4, GRFs rtol 1e-5 /
atol 1e-3).  End to end: the oracle's reduce() on the C oracle's own costs matches the GPU's GRFs
(rtol 1e-4, atol 5e-3 N) unless the argmin is a near tie (GPU's pick within the cost tolerance of the
oracle's minimum).
"""
import ctypes as C

import numpy as np
import pytest

from helpers import f32, make_case, product_cfg

pytestmark = pytest.mark.gpu

COST_RTOL, COST_ATOL = 2e-5, 1e-3


@pytest.fixture(scope="module")
def lib():
    from quadruped_pympc_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X")
    return _lib


def gpu_step(lib, case):
    ctx = lib.Context(product_cfg(case))
    try:
        best, sigma, res, costs = ctx.step(case["state"], case["ref"], case["contact"], case["best"],
                                           sigma=case["sigma"], noise=case["noise"], seed=42, counter=1,
                                           want_costs=True)
    finally:
        ctx.close()
    return dict(best=best, sigma=sigma, grf=np.array(res.grf, f32), pred=np.array(res.predicted_state, f32),
                best_cost=res.best_cost, best_index=res.best_index, costs=costs)


def c_oracle_costs(case):
    from oracle import c_oracle as co

    o = case["orc"]
    cfg = co.make_cfg(N=case["w"].num_samples, H=o.horizon, method=o.method, param_kind=o.param_kind,
                      num_splines=case["w"].num_splines, mass=case["w"].mass, inertia=case["w"].inertia)
    c = co.rollout_costs(cfg, case["state"], case["ref"], case["contact"], case["best"], case["noise"])
    return o.saturate(c)


def check_full(case, g):
    o = case["orc"]
    c = c_oracle_costs(case)
    np.testing.assert_allclose(g["costs"], c, rtol=COST_RTOL, atol=COST_ATOL)
    # reduction fed with the GPU's costs reproduces the GPU step
    r = o.reduce(case["state"], case["contact"], case["best"], case["noise"], g["costs"])
    assert r["best_index"] == g["best_index"]
    np.testing.assert_allclose(g["best"], r["best"], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(g["grf"], r["grf"], rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(g["pred"], r["pred"], rtol=1e-5, atol=1e-5)
    if "sigma" in r:
        np.testing.assert_allclose(g["sigma"], r["sigma"], rtol=1e-5, atol=1e-5)
    # end to end: the oracle's own costs through the oracle's reduction
    e = o.reduce(case["state"], case["contact"], case["best"], case["noise"], c)
    try:
        np.testing.assert_allclose(g["grf"], e["grf"], rtol=1e-4, atol=5e-3)
        np.testing.assert_allclose(g["best"], e["best"], rtol=1e-4, atol=1e-3)
    except AssertionError:
        assert g["costs"][g["best_index"]] <= c.min() * (1 + COST_RTOL) + COST_ATOL
    return c


FULL = [
    # id, workload, N, method, parametrization, H
    ("c2_exact", "c2", 10000, "mppi", "zero_order", 12),
    ("north_star_65536", "c2", 65536, "mppi", "zero_order", 12),
    ("thread_mppi_262144", "c2", 262144, "mppi", "zero_order", 12),
    ("thread_rs_262144", "c2", 262144, "random_sampling", "zero_order", 12),
    ("thread_cem_262144", "c2", 262144, "cem_mppi", "zero_order", 12),
    ("tree_linear_100000", "c2", 100000, "mppi", "linear_spline", 12),
    ("c5_tree_524288", "c5", 524288, "mppi", "zero_order", 12),
]


@pytest.mark.parametrize("wkey,N,method,par,H", [f[1:] for f in FULL], ids=[f[0] for f in FULL])
def test_full_size_against_c_oracle(lib, wkey, N, method, par, H):
    case = make_case(wkey, N=N, method=method, par=par, H=H, seed=N % 1000 + len(method))
    g = gpu_step(lib, case)
    check_full(case, g)


def test_c5_sharded_8_ranks_on_one_gpu(lib):
    """C5 (HyQReal bound, MPPI, N=524 288, H=12) split over 8 contexts (65 536 rows each, four-lane
    rollout), rank buffers merged by srbd_step_finish on every rank: identical outputs on all 8 ranks,
    bit-equal to the unsharded step (the fixed reduction tree), costs equal to the C oracle's."""
    torch = pytest.importorskip("torch")
    case = make_case("c5", N=524288, seed=77)
    full = gpu_step(lib, case)
    W = 8
    ctxs = [lib.Context(product_cfg(case, rank=r, world_size=W)) for r in range(W)]
    try:
        rec_f = ctxs[0].record_floats()
        recs = torch.zeros((W, rec_f), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        st = np.ascontiguousarray
        for r, cx in enumerate(ctxs):
            assert cx.n_local == 65536
            rows = st(case["noise"][cx.row0:cx.row0 + cx.n_local])
            rc = lib.lib.srbd_step_local(cx.h, lib.fptr(st(case["state"])), lib.fptr(st(case["ref"])),
                                         lib.fptr(st(case["contact"])), case["contact"].shape[1],
                                         lib.fptr(st(case["best"])), None, lib.fptr(rows), 42, 1,
                                         recs[r].data_ptr())
            assert rc == 0, lib.last_error(cx.h)
        torch.cuda.synchronize()
        outs = []
        costs = []
        for cx in ctxs:
            best = case["best"].copy()
            res = lib.SrbdResult()
            cl = np.empty(cx.n_local, f32)
            rc = lib.lib.srbd_step_finish(cx.h, recs.data_ptr(), W, lib.fptr(best), None, C.byref(res),
                                          lib.fptr(cl))
            assert rc == 0, lib.last_error(cx.h)
            outs.append((best, np.array(res.grf, f32), res.best_index))
            costs.append(cl)
    finally:
        for cx in ctxs:
            cx.close()
    for best, grf, bi in outs[1:]:  # every rank merged the same records in the same order
        np.testing.assert_array_equal(best, outs[0][0])
        np.testing.assert_array_equal(grf, outs[0][1])
        assert bi == outs[0][2]
    best, grf, bi = outs[0]  # the unsharded step folds the same reduction tree: the same bits
    assert bi == full["best_index"]
    np.testing.assert_array_equal(best, full["best"])
    np.testing.assert_array_equal(grf, full["grf"])
    np.testing.assert_array_equal(np.concatenate(costs), full["costs"])  # same rows, same rollout math
    np.testing.assert_allclose(full["costs"], c_oracle_costs(case), rtol=COST_RTOL, atol=COST_ATOL)
