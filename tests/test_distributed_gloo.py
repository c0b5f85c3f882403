"""World-size-2 (and 3) gloo tests of the row-sharded path's exchange and merge, on CPU.

Each rank builds its partial record from its own rows (srbd_make_record_host; on the GPU the
rollout kernel's block epilogue + merge produce the same record), the records are all-gathered
in rank order through quadruped_pympc_amd.sharded.RecordExchange, and every rank merges them
(srbd_finish_host).  The merged step must equal the oracle's unsharded step and be identical
on all ranks.  Oracle costs stand in for the GPU rollout here (no device in this container).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, method, N, outdir):
    for p in (os.path.join(ROOT, "quadruped-pympc-tamols_amd"), ROOT):
        sys.path.insert(0, p)
    from oracle.srbd_oracle import SamplingMPCOracle
    from quadruped_pympc_amd import _lib
    from quadruped_pympc_amd.sharded import RecordExchange, shard_rows
    from quadruped_pympc_amd.synthetic import CONFIGS, inputs

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    f32 = np.float32
    w = CONFIGS["c2"]
    o = SamplingMPCOracle(mass=w.mass, inertia=w.inertia, horizon=12, num_samples=N, method=method)
    s, r, c = (a.astype(f32) for a in inputs(w, 3))
    rng = np.random.default_rng(99)  # same seed on every rank: the shared problem
    t = N // 3
    sigma = rng.uniform(0.3, 3, o.P).astype(f32)
    noise = o.assemble_noise(rng.standard_normal((N - 1, o.P)).astype(f32), sigma=sigma,
                             U=rng.uniform(-10, 10, (N - 1 - 2 * t, o.P)).astype(f32))
    best = rng.standard_normal(o.P).astype(f32)
    costs = o.saturate(o.rollout_costs(s, r, best[None] + noise, c))

    cfg = _lib.make_config(num_samples=N, horizon=12, method=method, parametrization="zero_order", mass=w.mass,
                           inertia=w.inertia, dts=np.full(12, 0.02), rank=rank, world_size=world)
    a, n = shard_rows(N, rank, world)
    ex = RecordExchange(_lib.record_floats_host(cfg), world, "cpu")
    ex.local.numpy()[:] = _lib.make_record_host(cfg, rank, world, costs[a:a + n], noise[a:a + n])
    g = ex().numpy()
    nb, ns, res = _lib.finish_host(cfg, g, s, c, best, sigma if method == "cem_mppi" else None)
    ref = o.reduce(s, c, best, noise, costs)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), best=nb, grf=np.array(res.grf), idx=res.best_index,
             pred=np.array(res.predicted_state), sigma=ns if ns is not None else np.zeros(1, f32),
             ref_best=ref["best"], ref_grf=ref["grf"], ref_idx=ref["best_index"], ref_pred=ref["pred"],
             ref_sigma=ref.get("sigma", np.zeros(1, f32)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,method,N", [(2, "mppi", 1001), (2, "cem_mppi", 600), (2, "random_sampling", 450),
                                            (3, "mppi", 1000),
                                            # the driver's 8-GPU node: eight ranks, the exchange level and the
                                            # host tree at the widest world bench.py --gpus runs
                                            (8, "mppi", 4160), (8, "cem_mppi", 2048)])
def test_sharded_merge_gloo(tmp_path, world, method, N):
    mp.start_processes(worker, args=(world, free_port(), method, N, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    outs = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    for o in outs[1:]:  # every rank merges to the same bits
        for k in ("best", "grf", "pred", "sigma", "idx"):
            np.testing.assert_array_equal(o[k], outs[0][k])
    o = outs[0]
    assert int(o["idx"]) == int(o["ref_idx"])
    np.testing.assert_allclose(o["best"], o["ref_best"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(o["grf"], o["ref_grf"], rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(o["pred"], o["ref_pred"], rtol=1e-5, atol=1e-5)
    if method == "cem_mppi":
        np.testing.assert_allclose(o["sigma"], o["ref_sigma"], rtol=1e-5, atol=1e-6)


def test_shard_rows_cover_problem():
    from quadruped_pympc_amd.sharded import shard_rows

    for N in (1, 7, 300, 10000, 65537, 524288):
        for W in (1, 2, 3, 8):
            if W > (N + 63) // 64:  # fewer 64-row leaves than ranks: no whole-node shard for every rank
                with pytest.raises(ValueError):
                    shard_rows(N, W - 1, W)
                continue
            spans = [shard_rows(N, r, W) for r in range(W)]
            assert spans[0][0] == 0
            assert sum(n for _, n in spans) == N
            for (a, n), (b, _) in zip(spans, spans[1:]):
                assert a + n == b
                assert a % 64 == 0 and n > 0  # whole leaves (tree nodes)


def test_shard_rows_balanced():
    """The exchange level is the highest one whose largest rank share is within 1/8 of the best any level allows
    (srbd_core.h tree_shape): no rank is left with a sliver when N sits just past a node boundary."""
    from quadruped_pympc_amd.sharded import shard_rows

    # the fixed cases: C5 on 8 GPUs keeps one level-2 node per rank; 70 001 / 100 000 rows over 2 ranks drop to
    # level 1 (at level 2: 65 536 + 4 465 and 65 536 + 34 464 rows)
    assert [shard_rows(524288, r, 8) for r in range(8)] == [(65536 * r, 65536) for r in range(8)]
    assert [shard_rows(70001, r, 2) for r in range(2)] == [(0, 36864), (36864, 33137)]
    assert [shard_rows(100000, r, 2) for r in range(2)] == [(0, 51200), (51200, 48800)]
    for N in (4097, 10000, 65537, 70001, 100000, 131073, 300000, 524288, 524289):
        for W in (2, 3, 5, 8):
            spans = [shard_rows(N, r, W) for r in range(W)]
            big = max(n for _, n in spans)
            ideal = -(-N // W)
            # within 1/8 of the largest share whole 64-row leaves allow, or that share itself
            assert 8 * big <= 9 * max(ideal, 64 * -(-(-(-N // 64)) // W)), (N, W, spans)
