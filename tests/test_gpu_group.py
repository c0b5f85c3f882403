"""In-launch group reduction of the rollout's block records (GroupArgs, srbd_device.h group_reduce).

The rollout blocks of a group publish their records write-through and the group's last arriver merges
them into one record (rescaled sums in block order, K smallest keys), so the merge reads one record per
group.  Checked against the ungrouped step (SRBD_GROUP_SIZE=1, read per context): costs bit for bit (the
grouping does not touch the rollout), the same best row, parameters / GRFs to float rounding of the extra
rescaling level; and against the oracle's reduction of the GPU's costs (tests/test_gpu_parity.py
tolerances).  Ragged last groups, every method, the gait-adaptive rollout, graph replays and the
device-resident chain.
"""
import zlib

import numpy as np
import pytest

from helpers import f32, make_case, product_cfg
from test_gpu_parity import check_reduction, lib, run_gpu  # noqa: F401  (lib: module fixture)

pytestmark = pytest.mark.gpu


def run_grouped(lib, monkeypatch, case, gsize, **kw):
    monkeypatch.setenv("SRBD_GROUP_SIZE", str(gsize))
    try:
        return run_gpu(lib, case, **kw)
    finally:
        monkeypatch.delenv("SRBD_GROUP_SIZE")


@pytest.mark.parametrize("method,par,N,gsize", [
    ("mppi", "zero_order", 9000, 4),        # 141 blocks: 36 groups, the last of 1 block
    ("mppi", "zero_order", 9000, 7),        # ragged: 21 groups of 7 + 1 of 1
    ("mppi", "cubic_spline", 6000, 5),
    ("random_sampling", "zero_order", 9000, 6),
    ("cem_mppi", "zero_order", 8000, 8),    # K = 10: the group's top-K merge
    ("mppi", "zero_order", 65536, 32),      # the north-star shape's default grouping, explicitly
])
def test_grouped_equals_ungrouped(lib, monkeypatch, method, par, N, gsize):
    case = make_case("c2", N=N, method=method, par=par, seed=zlib.crc32(f"g{method}{par}{N}".encode()))
    a = run_grouped(lib, monkeypatch, case, 1, noise=False, seed=5, counter=3)
    b = run_grouped(lib, monkeypatch, case, gsize, noise=False, seed=5, counter=3)
    np.testing.assert_array_equal(a["costs"], b["costs"])
    assert a["best_index"] == b["best_index"]
    np.testing.assert_allclose(b["best"], a["best"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(b["grf"], a["grf"], rtol=1e-5, atol=1e-4)
    if method == "cem_mppi":
        np.testing.assert_array_equal(a["sigma"], b["sigma"])  # same elite rows, same sigma arithmetic


@pytest.mark.parametrize("method", ["mppi", "cem_mppi", "random_sampling"])
def test_grouped_against_oracle(lib, monkeypatch, method):
    case = make_case("c2", N=7000, method=method, seed=17)
    g = run_grouped(lib, monkeypatch, case, 9)
    check_reduction(case, g)


def test_grouped_chain_and_graph_replays(lib, monkeypatch):
    """Counters are reset by each group's last arriver: many launches in a row on one context (host steps,
    then the device-resident hipGraph chain) keep matching an ungrouped context fed the same inputs."""
    case = make_case("c2", N=12000, seed=3)
    monkeypatch.setenv("SRBD_GROUP_SIZE", "6")
    cg = lib.Context(product_cfg(case))
    monkeypatch.setenv("SRBD_GROUP_SIZE", "1")
    cu = lib.Context(product_cfg(case))
    monkeypatch.delenv("SRBD_GROUP_SIZE")
    try:
        best = case["best"].copy()
        for k in range(6):
            bg, _, rg, cgc = cg.step(case["state"], case["ref"], case["contact"], best, seed=2, counter=k,
                                     want_costs=True)
            bu, _, ru, cuc = cu.step(case["state"], case["ref"], case["contact"], best, seed=2, counter=k,
                                     want_costs=True)
            np.testing.assert_array_equal(cgc, cuc)
            assert rg.best_index == ru.best_index
            np.testing.assert_allclose(bg, bu, rtol=1e-5, atol=1e-5)
            best = bg
        for ctx in (cg, cu):  # device-resident chain (graph replays of the grouped launch), then a host step
            ctx.bench_device_steps(25)
            ctx.set_state(best, None, 2, 100)
        bg, _, rg, cgc = cg.step(case["state"], case["ref"], case["contact"], best, seed=2, counter=200,
                                 want_costs=True)
        bu, _, ru, cuc = cu.step(case["state"], case["ref"], case["contact"], best, seed=2, counter=200,
                                 want_costs=True)
        np.testing.assert_array_equal(cgc, cuc)
        np.testing.assert_allclose(bg, bu, rtol=1e-5, atol=1e-5)
    finally:
        cg.close()
        cu.close()


def test_grouped_gait_adaptive(lib, monkeypatch):
    case = make_case("c2", N=9000, seed=8)
    res = {}
    for gs in (1, 5):
        monkeypatch.setenv("SRBD_GROUP_SIZE", str(gs))
        ctx = lib.Context(product_cfg(case))
        ctx.set_gait(np.array([0.1, 0.6, 0.6, 0.1], f32), 0.02, 0.65, np.array([1.3, 1.65, 2.0], f32))
        best, _, r, costs = ctx.step(case["state"], case["ref"], case["contact"], case["best"], seed=4, counter=2,
                                     want_costs=True)
        res[gs] = (best, r.best_index, r.best_freq, costs)
        ctx.close()
    monkeypatch.delenv("SRBD_GROUP_SIZE")
    np.testing.assert_array_equal(res[1][3], res[5][3])
    assert res[1][1] == res[5][1] and res[1][2] == res[5][2]
    np.testing.assert_allclose(res[5][0], res[1][0], rtol=1e-5, atol=1e-5)
