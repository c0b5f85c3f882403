#!/usr/bin/env python3
"""Floor costs of the host-driven MPC step on this box (HIP runtime via torch), in microseconds.

Prints p50 of: sync on an idle stream, one tiny kernel + sync, pinned 4 KB H2D + sync,
pinned 4 KB D2H + sync, H2D + kernel + D2H + sync, and the same through a captured graph.
"""
import json
import time

import numpy as np
import torch


def p50(fn, n=2000, warm=50):
    for _ in range(warm):
        fn()
    t = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return round(1e6 * float(np.percentile(t, 50)), 2)


def main():
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    hin = torch.zeros(1100, dtype=torch.float32).pin_memory()
    hout = torch.zeros(800, dtype=torch.float32).pin_memory()
    din = torch.zeros(1100, dtype=torch.float32, device=dev)
    dout = torch.zeros(800, dtype=torch.float32, device=dev)
    res = {}
    with torch.cuda.stream(s):
        res["sync_idle"] = p50(lambda: s.synchronize())
        res["kernel_sync"] = p50(lambda: (dout.add_(1.0), s.synchronize()))
        res["h2d_sync"] = p50(lambda: (din.copy_(hin, non_blocking=True), s.synchronize()))
        res["d2h_sync"] = p50(lambda: (hout.copy_(dout, non_blocking=True), s.synchronize()))

        def chain():
            din.copy_(hin, non_blocking=True)
            dout.add_(din[:800])
            hout.copy_(dout, non_blocking=True)
            s.synchronize()

        res["h2d_kernel_d2h_sync"] = p50(chain)
        g = torch.cuda.CUDAGraph()
        chain_nosync = lambda: (din.copy_(hin, non_blocking=True), dout.add_(din[:800]),  # noqa: E731
                                hout.copy_(dout, non_blocking=True))
        chain_nosync()
        s.synchronize()
        with torch.cuda.graph(g, stream=s):
            chain_nosync()
        res["graph_h2d_kernel_d2h_sync"] = p50(lambda: (g.replay(), s.synchronize()))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
