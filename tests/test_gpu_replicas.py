"""Replica processes on the GPU (SURVEY 8(e) replica mode; batched_simulations.py:40-58 starts one
multiprocessing.Process per environment, each constructing its own controller).  Fresh spawned
processes build the zero-argument Sampling_MPC() (device_id 'auto' from the config), resolve their
ordinal when the HIP context is created and run one MPC step; the parent never touches the GPU in
this test.  One GPU on the box: every replica lands on ordinal 0 (i mod 1); the resolution source is
reported (multiprocessing identity, or SRBD_REPLICA_INDEX when a launcher sets it).
"""
import multiprocessing as mp

import pytest

pytestmark = pytest.mark.gpu


def _replica(q, replica_env):
    import os

    import numpy as np

    if replica_env is not None:
        os.environ["SRBD_REPLICA_INDEX"] = replica_env
    os.environ.pop("LOCAL_RANK", None)
    try:
        from quadruped_pympc_amd import _lib, runtime
        from quadruped_pympc_amd.controllers.sampling.centroidal_nmpc_hip import Sampling_MPC
        from quadruped_pympc_amd.synthetic import CONFIGS, Workload, inputs

        mpc = Sampling_MPC()  # the reference's zero-argument constructor (config mirror, device_id 'auto')
        w0 = CONFIGS["c2"]
        w = Workload(w0.name, w0.robot, w0.gait, "mppi", "zero_order", 1024, mpc.horizon)
        state, ref, contact = inputs(w, 1)
        out = mpc.compute_control_mppi(state.astype(np.float32), ref.astype(np.float32),
                                       contact[:, :mpc.horizon].astype(np.float32), mpc.best_control_parameters,
                                       mpc.master_key)
        grf = np.asarray(out[0], np.float32)
        q.put({"device_id": int(mpc.device_id), "source": runtime.replica_source()[1],
               "index": runtime.replica_source()[0], "gpus": _lib.device_count(),
               "finite": bool(np.isfinite(grf).all()), "n": int(mpc.num_parallel_computations)})
        mpc.close()
    except Exception as e:  # reported to the parent
        q.put({"error": repr(e)})


def test_spawned_replicas_resolve_and_step():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    specs = [None, None, "5"]
    procs = [ctx.Process(target=_replica, args=(q, s)) for s in specs]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for g in got:
        assert "error" not in g, g
        assert g["finite"] and 0 <= g["device_id"] < g["gpus"]
        assert g["device_id"] == g["index"] % g["gpus"]
    srcs = sorted(g["source"] for g in got)
    assert srcs == ["SRBD_REPLICA_INDEX", "multiprocessing identity", "multiprocessing identity"], srcs
    explicit = [g for g in got if g["source"] == "SRBD_REPLICA_INDEX"][0]
    assert explicit["index"] == 5
