"""The sharded driver (quadruped_pympc_amd.sharded) over a real RCCL group on one GPU.

World size 1 (the box has one GPU; RCCL refuses two ranks on one device), both transports: the
library's own RCCL communicator (ncclAllGather issued from C++ on the context stream) and
torch.distributed.all_gather_into_tensor on a torch stream shared with the library.  The
result must equal the unsharded srbd_step on the same noise bit for bit (the fixed reduction tree), also on
device draws, and the device-resident chain must run.  At N = 65 536 (grouped zero-order MPPI) the xGMI host
step folds, exchanges and merges inside the rollout launch (final merger, GroupArgs::xa).  Multi-rank merging is covered on CPU with gloo
(tests/test_distributed_gloo.py) and on this GPU with several contexts
(test_gpu_parity.py::test_sharded_records_on_one_gpu).
"""
import socket

import numpy as np
import pytest

from helpers import make_case, product_cfg

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("transport", ["auto", "xgmi", "rccl", "torch"])
def test_sharded_driver_world1_matches_step(transport):
    import torch
    import torch.distributed as dist

    from quadruped_pympc_amd import _lib
    from quadruped_pympc_amd.sharded import ShardedSamplingMPC

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        for wkey, N, method in (("c2", 3000, "mppi"), ("c2", 3000, "cem_mppi"), ("c2", 3000, "random_sampling"),
                                ("c2", 65536, "mppi"), ("c5", 65536, "mppi")):
            case = make_case(wkey, N=N, method=method, seed=17)
            ref = _lib.Context(product_cfg(case))
            b0, s0, r0, _ = ref.step(case["state"], case["ref"], case["contact"], case["best"], sigma=case["sigma"],
                                     noise=case["noise"])
            bd, _, rd, _ = ref.step(case["state"], case["ref"], case["contact"], case["best"], sigma=case["sigma"],
                                    seed=42, counter=5)
            ref.close()
            mpc = ShardedSamplingMPC(product_cfg(case), 0, 1, 0, transport=transport)
            if transport == "auto":
                assert mpc.transport == "xgmi"
            b1, s1, r1 = mpc.step(case["state"], case["ref"], case["contact"], case["best"], sigma=case["sigma"],
                                  noise_local=case["noise"])
            assert r1.best_index == r0.best_index
            np.testing.assert_array_equal(b1, b0)
            np.testing.assert_array_equal(np.array(r1.grf), np.array(r0.grf))
            if method == "cem_mppi":
                np.testing.assert_array_equal(s1, s0)
            # device draws: the same bits as the unsharded step keyed alike
            b2, _, r2 = mpc.step(case["state"], case["ref"], case["contact"], case["best"], sigma=case["sigma"],
                                 seed=42, counter=5)
            assert r2.best_index == rd.best_index
            np.testing.assert_array_equal(b2, bd)
            # device-resident chain on the torch stream
            assert mpc.device_steps(4) > 0
            torch.cuda.synchronize()
            # after a device chain, a host step still reproduces the unsharded step
            b3, s3, r3 = mpc.step(case["state"], case["ref"], case["contact"], case["best"], sigma=case["sigma"],
                                  noise_local=case["noise"])
            assert r3.best_index == r0.best_index
            np.testing.assert_array_equal(b3, b0)
            mpc.close()
    finally:
        dist.destroy_process_group()
