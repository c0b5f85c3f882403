#!/usr/bin/env python3
"""Per-step cost of the sharded driver on one GPU (RCCL group of one rank): host-driven loop of
ShardedSamplingMPC.device_step vs the library's own device chain.  Measurement tool."""
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "quadruped-pympc-tamols_amd")]

import numpy as np  # noqa: E402

from bench import make_cfg  # noqa: E402
from quadruped_pympc_amd.sharded import ShardedSamplingMPC  # noqa: E402
from quadruped_pympc_amd.synthetic import CONFIGS, inputs  # noqa: E402


def main():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    w = CONFIGS["c2"]
    transport = sys.argv[1] if len(sys.argv) > 1 else "rccl"
    mpc = ShardedSamplingMPC(make_cfg(w, w.num_samples, 0, 1, 0), 0, 1, 0, transport=transport)
    s, r, c = inputs(w, 0)
    best = np.zeros(mpc.P, np.float32)
    for k in range(20):
        best, _, _ = mpc.step(s, r, c, best, seed=42, counter=k)
    res = {}
    res["transport"] = transport
    mpc.device_steps(50)
    torch.cuda.synchronize()
    n = 2000
    t0 = time.perf_counter()
    mpc.device_steps(n)
    torch.cuda.synchronize()
    res["device_chain_us_per_step"] = round(1e6 * (time.perf_counter() - t0) / n, 2)
    lat = []
    for k in range(300):
        t0 = time.perf_counter()
        best, _, _ = mpc.step(s, r, c, best, seed=42, counter=1000 + k)
        lat.append(time.perf_counter() - t0)
    res["host_step_p50_us"] = round(1e6 * float(np.percentile(lat, 50)), 2)
    mpc.close()
    dist.destroy_process_group()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
