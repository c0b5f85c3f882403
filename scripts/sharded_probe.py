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
from quadruped_pympc_amd import _lib  # noqa: E402
from quadruped_pympc_amd.sharded import ShardedSamplingMPC  # noqa: E402
from quadruped_pympc_amd.synthetic import CONFIGS, inputs  # noqa: E402


def local_pair(steps=2000):
    """W=2 ranks as two contexts on this one GPU, connected in-process, device chains run from two
    threads: the exchange protocol's per-step cost (both ranks share the GPU's CUs)."""
    import ctypes as C
    import threading

    from quadruped_pympc_amd import _lib

    w = CONFIGS["c2"]
    ctxs = [_lib.Context(make_cfg(_lib, w, 2 * w.num_samples, r, 2, 0)) for r in range(2)]
    for cx in ctxs:
        cx.check(_lib.lib.srbd_xgmi_export(cx.h, (C.c_uint8 * 64)()), "export")
    arr = (C.c_void_p * 2)(*[cx.h.value for cx in ctxs])
    assert _lib.lib.srbd_xgmi_connect_local(arr, 2) == 0
    ms = [0.0, 0.0]
    st, ref, con = inputs(w, 0)

    def host(i):
        b = np.zeros(ctxs[i].P, np.float32)
        ctxs[i].step_sharded(st, ref, con, b, seed=42, counter=0)

    hs = [threading.Thread(target=host, args=(i,)) for i in range(2)]
    for t in hs:
        t.start()
    for t in hs:
        t.join()

    def run(i, n):
        v = C.c_float(0)
        ctxs[i].check(_lib.lib.srbd_sharded_device_steps(ctxs[i].h, n, C.byref(v)), "steps")
        ms[i] = v.value

    for n in (50, steps):
        ts = [threading.Thread(target=run, args=(i, n)) for i in range(2)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        wall = time.perf_counter() - t0
    for cx in ctxs:
        cx.close()
    print(json.dumps({"transport": "xgmi_local_w2", "rows_per_rank": w.num_samples,
                      "device_chain_us_per_step": round(1e6 * wall / steps, 2),
                      "event_ms_per_rank": [round(m, 3) for m in ms]}))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "local2":
        return local_pair()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    w = CONFIGS[os.environ.get("SHARD_CFG", "c2")]  # e.g. SHARD_CFG=ns: the 8-rank C5 per-rank shape
    transport = sys.argv[1] if len(sys.argv) > 1 else "rccl"
    mpc = ShardedSamplingMPC(make_cfg(_lib, w, w.num_samples, 0, 1, 0), 0, 1, 0, transport=transport)
    s, r, c = inputs(w, 0)
    best = np.zeros(mpc.P, np.float32)
    for k in range(20):
        best, _, _ = mpc.step(s, r, c, best, seed=42, counter=k)
    res = {}
    res["transport"] = transport
    res["workload"] = w.name
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
