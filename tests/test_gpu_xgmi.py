"""xGMI mailbox exchange (merge_xchg_kernel) with W ranks as W contexts on one GPU.

The box has one GPU, so the peers' mailboxes are connected in-process (srbd_xgmi_connect_local:
the same kernel, device pointers instead of IPC-mapped ones).  The scenarios run in one worker
process (tests/xgmi_worker.py, see its docstring for why): the merged step must equal the unsharded
step bit for bit (the fixed reduction tree) and be bit-identical on every rank, across host steps and the
replayed device chain; a rank whose peer never arrives must fail after the bounded wait.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def worker_results():
    # one hardware queue per rank stream (8 ranks in the C5 case; HIP's default is 4 queues)
    env = dict(os.environ, GPU_MAX_HW_QUEUES="16")
    p = subprocess.run([sys.executable, os.path.join(HERE, "xgmi_worker.py")], capture_output=True, text=True,
                       timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("case", ["mppi", "cem_mppi", "random_sampling", "mppi_w3", "mppi_ga_w3", "c5_w8", "c5_weak_w2",
                                  "bench_w2", "timeout"])
def test_xgmi_exchange_in_process(worker_results, case):
    assert worker_results[case] == "ok", worker_results[case]
