"""The host step's two launch-saving forms against the split path on the same GPU (CPU-free, bit for bit).

srbd_step passes the step input by value to the rollout launch (StepInputK; zero-order H 10 / 12, MPPI / random
sampling), whose block 0 writes the device StepInput, and at grouped shapes (N >= 32 768, four lanes per sample)
the rollout launch's last group arriver merges the group records and publishes the outputs (final merge), so
no upload and no merge kernel run.  srbd_step_local + srbd_step_finish on a one-rank context run the other
forms: the one-block upload kernel, the plain rollout, the merge into a rank record, and the merge of that
record.  A one-rank finish rescales by exp(0) = 1, so both give the same bits: costs, parameters, GRFs,
prediction, best row and cost.  Device-resident chains started after either form read the device StepInput it
wrote and must agree too.
"""
import ctypes as C
import zlib

import numpy as np
import pytest

from helpers import f32, make_case, product_cfg
from test_gpu_parity import check_reduction, lib, run_gpu  # noqa: F401  (lib: module fixture)

pytestmark = pytest.mark.gpu

KEYS = ("costs", "best", "grf", "pred")


def split_step(lib, case, noise=True, seed=42, counter=1, ctx=None):
    """srbd_step_local (uploaded input, plain rollout, merge into a rank record) + srbd_step_finish."""
    torch = pytest.importorskip("torch")
    own = ctx is None
    cx = ctx or lib.Context(product_cfg(case))
    try:
        rec = torch.zeros(cx.record_floats(), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        st = np.ascontiguousarray
        rows = st(case["noise"]) if noise else None
        rc = lib.lib.srbd_step_local(cx.h, lib.fptr(st(case["state"])), lib.fptr(st(case["ref"])),
                                     lib.fptr(st(case["contact"])), case["contact"].shape[1],
                                     lib.fptr(st(case["best"])), None, lib.fptr(rows), seed, counter, rec.data_ptr())
        assert rc == 0, lib.last_error(cx.h)
        best = case["best"].copy()
        res = lib.SrbdResult()
        costs = np.empty(cx.n_local, f32)
        rc = lib.lib.srbd_step_finish(cx.h, rec.data_ptr(), 1, lib.fptr(best), None, C.byref(res), lib.fptr(costs))
        assert rc == 0, lib.last_error(cx.h)
        torch.cuda.synchronize()
    finally:
        if own:
            cx.close()
    return dict(best=best, grf=np.array(res.grf, f32), pred=np.array(res.predicted_state, f32),
                best_cost=res.best_cost, best_index=res.best_index, costs=costs)


@pytest.mark.parametrize("method,N,H,noise,rollout", [
    ("mppi", 10000, 12, False, None),           # C2: the headline host step (input by value)
    ("mppi", 10000, 12, True, None),            # injected noise
    ("random_sampling", 3001, 10, False, None),
    ("mppi", 65536, 12, False, None),           # input by value + the in-launch final merge
    ("mppi", 65536, 12, True, None),
    ("random_sampling", 40000, 12, False, None),
    ("mppi", 33000, 10, True, None),            # ragged groups, H 10
    ("mppi", 10000, 12, False, "thread"),       # thread-per-sample rollout
    ("random_sampling", 2999, 10, True, "thread"),
    ("mppi", 131072, 12, False, None),          # past the four-lane range: the thread form by default
])
def test_host_step_equals_split_path(lib, monkeypatch, method, N, H, noise, rollout):
    case = make_case("c2", N=N, method=method, H=H, seed=zlib.crc32(f"sp{method}{N}{H}".encode()))
    if rollout:
        monkeypatch.setenv("SRBD_ROLLOUT", rollout)
    try:
        a = run_gpu(lib, case, noise=noise, seed=11, counter=7)
        b = split_step(lib, case, noise=noise, seed=11, counter=7)
    finally:
        if rollout:
            monkeypatch.delenv("SRBD_ROLLOUT")
    for k in KEYS:
        np.testing.assert_array_equal(a[k], b[k])
    assert a["best_index"] == b["best_index"] and a["best_cost"] == b["best_cost"]
    if noise:
        check_reduction(case, a)


@pytest.mark.parametrize("N", [10000, 65536, 131072])
def test_device_chains_after_either_form(lib, N):
    """A device-resident chain starts from the device StepInput the last host step wrote (the KS launch's block 0,
    or the upload kernel): host steps and chains interleaved, every output and checkpoint equal bit for bit, and
    the arrival counters of the grouped / final-merge launches reset launch after launch."""
    case = make_case("c2", N=N, seed=31)
    ca, cb = lib.Context(product_cfg(case)), lib.Context(product_cfg(case))
    try:
        best = case["best"].copy()
        for k in range(8):
            st = case["state"].copy()
            st[0] += 0.01 * k  # a different input every call
            c = dict(case, state=st, best=best)
            a = ca.step(st, case["ref"], case["contact"], best, seed=5, counter=k, want_costs=True)
            b = split_step(lib, c, noise=False, seed=5, counter=k, ctx=cb)
            np.testing.assert_array_equal(a[0], b["best"])
            np.testing.assert_array_equal(a[3], b["costs"])
            assert a[2].best_index == b["best_index"]
            if k in (2, 5):
                ca.bench_device_steps(9)
                cb.bench_device_steps(9)
                sa, sb = ca.get_state(), cb.get_state()
                np.testing.assert_array_equal(sa[0], sb[0])
                assert sa[2:] == sb[2:] == (5, k + 9)
            best = a[0]
    finally:
        ca.close()
        cb.close()


@pytest.mark.parametrize("method,N", [("mppi", 40000), ("random_sampling", 33000), ("mppi", 65536)])
def test_grouped_step_against_oracle(lib, method, N):
    """Grouped block records (N >= 32 768: the last arriver of each group merges its records, the final merge the
    groups) against the oracle's reduction of the GPU's costs (tests/test_gpu_parity.py tolerances)."""
    case = make_case("c2", N=N, method=method, seed=17)
    check_reduction(case, run_gpu(lib, case))


def test_grouped_gait_adaptive_against_oracle(lib):
    """Gait-adaptive rollout at a grouped shape (its launch keeps the merge kernel)."""
    from oracle.srbd_ga_oracle import GaitAdaptiveOracle

    case = make_case("c2", N=40000, seed=8)
    w = case["w"]
    o = GaitAdaptiveOracle(pgg_dt=0.02, mass=w.mass, inertia=w.inertia, horizon=w.horizon, num_samples=w.num_samples,
                           method=w.method, parametrization=w.parametrization, num_splines=w.num_splines)
    fs = np.array([1.3, 1.65, 2.0], f32)
    freqs = np.random.default_rng(2).choice(fs, w.num_samples).astype(f32)
    ctx = lib.Context(product_cfg(case))
    try:
        ctx.set_gait(np.array([0.1, 0.6, 0.6, 0.1], f32), 0.02, 0.65, fs, freqs)
        best, _, r, costs = ctx.step(case["state"], case["ref"], case["contact"], case["best"], noise=case["noise"],
                                     seed=4, counter=2, want_costs=True)
    finally:
        ctx.close()
    ref = o.reduce(case["state"], case["contact"], case["best"], case["noise"], costs)
    assert r.best_index == ref["best_index"]
    np.testing.assert_allclose(best, ref["best"], rtol=1e-5, atol=1e-4)
    assert r.best_freq == freqs[r.best_index]


@pytest.mark.parametrize("method,N,H,noise", [
    ("mppi", 8257, 12, False),             # 130 leaves: the fewest level-1 nodes (5) that fold in the launch
    ("mppi", 10000, 12, False),            # C2
    ("mppi", 10000, 12, True),
    ("random_sampling", 10000, 12, False),
    ("mppi", 32832, 10, True),             # 17 nodes: both register batches of the root
    ("random_sampling", 40000, 12, True),
    ("mppi", 65536, 12, False),            # 32 nodes (north-star)
])
def test_fast_tail_equals_two_stage(lib, monkeypatch, method, N, H, noise):
    """fast_tail (the level-1 fold and the root merge with one arrival count, tagged node-record hand-off) against
    the two-stage in-launch final merge (SRBD_FAST_TAIL=0: folds, a second count, merge_body) over six successive
    host steps on each context -- the tagged words are rewritten launch after launch -- bit for bit."""
    case = make_case("c2", N=N, method=method, H=H, seed=zlib.crc32(f"ft{method}{N}{H}".encode()))
    monkeypatch.setenv("SRBD_FAST_TAIL", "0")
    slow = lib.Context(product_cfg(case))
    monkeypatch.delenv("SRBD_FAST_TAIL")
    fast = lib.Context(product_cfg(case))
    try:
        bf, bs = case["best"].copy(), case["best"].copy()
        for k in range(6):
            st = case["state"].copy()
            st[1] += 0.005 * k
            nz = case["noise"] if noise else None
            a = fast.step(st, case["ref"], case["contact"], bf, noise=nz, seed=3, counter=k, want_costs=k == 0)
            b = slow.step(st, case["ref"], case["contact"], bs, noise=nz, seed=3, counter=k, want_costs=k == 0)
            np.testing.assert_array_equal(a[0], b[0])
            np.testing.assert_array_equal(np.array(a[2].grf), np.array(b[2].grf))
            np.testing.assert_array_equal(np.array(a[2].predicted_state), np.array(b[2].predicted_state))
            assert (a[2].best_index, a[2].best_cost, a[2].best_freq, a[2].status) == \
                   (b[2].best_index, b[2].best_cost, b[2].best_freq, b[2].status)
            if k == 0:
                np.testing.assert_array_equal(a[3], b[3])
            bf, bs = a[0], b[0]
        assert fast.time_launch(3, 2)[1] & 16 and not slow.time_launch(3, 2)[1] & 16  # the tails the steps ran
    finally:
        fast.close()
        slow.close()
