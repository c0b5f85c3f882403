"""Host steps with the step input as the rollout's kernel argument (StepInputK, srbd_kernels.hip KS).

Zero-order shapes (H 10 / 12, MPPI / random sampling), four-lane and thread-per-sample rollouts: srbd_step passes the step input by value
to the rollout launch, whose block 0 writes the device StepInput for the merge and later readers, and runs
no upload kernel.  Every output must equal the uploaded input's (SRBD_KS=0, read per context) bit for bit:
device draws and injected noise, with and without the in-launch final merge, H 10; and sequences of host
steps interleaved with device-resident chains and state reads, which read the device copy block 0 wrote.
"""
import zlib

import numpy as np
import pytest

from helpers import make_case, product_cfg
from test_gpu_parity import check_reduction, lib, run_gpu  # noqa: F401  (lib: module fixture)

pytestmark = pytest.mark.gpu

KEYS = ("costs", "best", "grf", "pred")


def both(lib, monkeypatch, case, rollout=None, **kw):
    out = {}
    if rollout:
        monkeypatch.setenv("SRBD_ROLLOUT", rollout)
    for ks in ("0", "1"):
        monkeypatch.setenv("SRBD_KS", ks)
        try:
            out[ks] = run_gpu(lib, case, **kw)
        finally:
            monkeypatch.delenv("SRBD_KS")
    if rollout:
        monkeypatch.delenv("SRBD_ROLLOUT")
    return out["0"], out["1"]


@pytest.mark.parametrize("method,N,H,noise,rollout", [
    ("mppi", 10000, 12, False, None),           # C2: the headline host step
    ("mppi", 10000, 12, True, None),            # injected noise
    ("random_sampling", 3001, 10, False, None),
    ("mppi", 65536, 12, False, None),           # with the in-launch final merge
    ("mppi", 40000, 10, True, None),
    ("mppi", 10000, 12, False, "thread"),       # thread-per-sample rollout
    ("random_sampling", 2999, 10, True, "thread"),
    ("mppi", 131072, 12, False, None),          # past the four-lane range: thread form by default
])
def test_ks_bitwise(lib, monkeypatch, method, N, H, noise, rollout):
    case = make_case("c2", N=N, method=method, H=H, seed=zlib.crc32(f"ks{method}{N}{H}".encode()))
    a, b = both(lib, monkeypatch, case, rollout=rollout, noise=noise, seed=11, counter=7)
    for k in KEYS:
        np.testing.assert_array_equal(a[k], b[k])
    assert a["best_index"] == b["best_index"] and a["best_cost"] == b["best_cost"]
    if noise:
        check_reduction(case, b)


@pytest.mark.parametrize("N", [10000, 65536, 131072])
def test_ks_sequence_with_device_chains(lib, monkeypatch, N):
    case = make_case("c2", N=N, seed=31)
    ctxs = {}
    for ks in ("0", "1"):
        monkeypatch.setenv("SRBD_KS", ks)
        ctxs[ks] = lib.Context(product_cfg(case))
    monkeypatch.delenv("SRBD_KS")
    try:
        outs = {}
        for ks, ctx in ctxs.items():
            best = case["best"].copy()
            seq = []
            for k in range(10):
                st = case["state"].copy()
                st[0] += 0.01 * k  # a different input every call
                best, _, r, costs = ctx.step(st, case["ref"], case["contact"], best, seed=5, counter=k,
                                             want_costs=True)
                seq.append((best.copy(), np.array(r.grf), r.best_index, costs))
                if k in (3, 7):  # the device chain starts from the device StepInput the last host step left
                    ctx.bench_device_steps(8)
                    b2, _, seed, ctr = ctx.get_state()
                    seq.append((np.asarray(b2), seed, ctr))
            outs[ks] = seq
        for x, y in zip(outs["0"], outs["1"]):
            for u, v in zip(x, y):
                np.testing.assert_array_equal(np.asarray(u), np.asarray(v))
    finally:
        for ctx in ctxs.values():
            ctx.close()
