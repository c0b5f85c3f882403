"""In-launch final merge (rollout_quad_kernel -> final_merge, srbd_kernels.hip).

Zero-order host steps with grouped block records (N >= 32 768 at the default grouping, or any N with
SRBD_GROUP_SIZE): the rollout launch's last group arriver merges the group records and publishes the step's
outputs itself, with no merge launch.  It runs merge_kernel's staged body with the 512-thread kernel's record
groups, so every output must equal the separate merge's (SRBD_FINAL_MERGE=0, read per context) bit for bit:
device draws and injected noise, MPPI and random sampling, ragged groups, H 10 and 12, many launches in a row
(the done-counter resets), and host steps interleaved with device-resident chains (whose final merge writes
the warm start back into the step input and advances the RNG counter after the launch's draw blocks).
"""
import zlib

import numpy as np
import pytest

from helpers import make_case, product_cfg
from test_gpu_parity import check_reduction, lib, run_gpu  # noqa: F401  (lib: module fixture)

pytestmark = pytest.mark.gpu

KEYS = ("costs", "best", "grf", "pred")


def both(lib, monkeypatch, case, gsize=None, **kw):
    out = {}
    for fm in ("0", "1"):
        monkeypatch.setenv("SRBD_FINAL_MERGE", fm)
        if gsize:
            monkeypatch.setenv("SRBD_GROUP_SIZE", str(gsize))
        try:
            out[fm] = run_gpu(lib, case, **kw)
        finally:
            monkeypatch.delenv("SRBD_FINAL_MERGE")
            if gsize:
                monkeypatch.delenv("SRBD_GROUP_SIZE")
    return out["0"], out["1"]


@pytest.mark.parametrize("method,N,H,gsize,noise", [
    ("mppi", 65536, 12, None, False),           # the north-star shape, default grouping (32 groups)
    ("mppi", 65536, 12, None, True),            # injected noise
    ("random_sampling", 40000, 12, None, False),
    ("mppi", 9000, 12, 4, False),               # 141 blocks: 36 groups, the last of 1 block
    ("mppi", 9000, 10, 7, False),               # H 10, ragged
    ("mppi", 33000, 12, None, False),           # ragged default grouping
])
def test_final_merge_bitwise(lib, monkeypatch, method, N, H, gsize, noise):
    case = make_case("c2", N=N, method=method, H=H, seed=zlib.crc32(f"fm{method}{N}{H}".encode()))
    a, b = both(lib, monkeypatch, case, gsize, noise=noise, seed=7, counter=5)
    for k in KEYS:
        np.testing.assert_array_equal(a[k], b[k])
    assert a["best_index"] == b["best_index"] and a["best_cost"] == b["best_cost"]
    if noise:  # the oracle's reduction of the GPU's costs (injected noise: the oracle has the draws)
        check_reduction(case, b)


def test_final_merge_sequence_with_device_chains(lib, monkeypatch):
    """Host steps and device-resident chains on one context (both with the in-launch final merge), against a
    context with it off: the done counters reset every launch, the chain's warm start and RNG counter come back
    the same (the counter advanced only after the launch's draw blocks have read it), bit for bit."""
    case = make_case("c2", N=65536, seed=21)
    ctxs = {}
    for fm in ("0", "1"):
        monkeypatch.setenv("SRBD_FINAL_MERGE", fm)
        ctxs[fm] = lib.Context(product_cfg(case))
    monkeypatch.delenv("SRBD_FINAL_MERGE")
    try:
        outs = {}
        for fm, ctx in ctxs.items():
            best = case["best"].copy()
            seq = []
            for k in range(12):
                best, _, r, costs = ctx.step(case["state"], case["ref"], case["contact"], best, seed=3, counter=k,
                                             want_costs=True)
                seq.append((best.copy(), np.array(r.grf), r.best_index, costs))
                if k in (4, 8):  # device chains (their final merge writes the warm start and the counter back)
                    ctx.bench_device_steps(10)
                    b2, _, seed2, ctr2 = ctx.get_state()
                    seq.append((np.asarray(b2), seed2, ctr2))
                    ctx.set_state(best, None, 3, 100 + k)
            outs[fm] = seq
        for x, y in zip(outs["0"], outs["1"]):
            for u, v in zip(x, y):
                np.testing.assert_array_equal(np.asarray(u), np.asarray(v))
    finally:
        for ctx in ctxs.values():
            ctx.close()
