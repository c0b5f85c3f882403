#!/usr/bin/env python3
"""Phase stamps of one merge launch (probe build; measurement tool, GPU box).

merge_body's stamps (blocks 0 and 1; b1_ = block 1, a column split's first slice): 0 entry, 7 first record chunk
loaded, 6 records staged, 1 beta, 2 tree sums done, 3 top-K done, 4 outputs assembled, 5 published; marks 16 + i:
0 beta scan, 1 tail prep, 2 barrier, 3 / 4 level 0 keys / sums, 6 / 7 level 1 keys / sums, 5 tree levels, 8 end;
block_topk_nodes 25..29: selected nodes, candidate table, ranked, key lists loaded, done.  Prints one JSON line per workload: median over 30 launches of each stamp relative to entry (us).
Usage: python scripts/merge_phases.py c2 [N]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "quadruped-pympc-tamols_amd")
os.environ["SRBD_LIB_PATH"] = os.path.join(PKG, "quadruped_pympc_amd", "libsrbd_hip_probe.so")
sys.path.insert(0, PKG)
from quadruped_pympc_amd import _lib  # noqa: E402
from quadruped_pympc_amd.synthetic import CONFIGS, inputs  # noqa: E402

NAMES = {0: "entry", 7: "chunk0", 6: "staged", 1: "beta", 2: "sums", 3: "topk", 4: "outputs", 5: "published",
         16: "m_beta_scan", 17: "m_tail_prep", 18: "m_barrier", 19: "m_l0_keys", 20: "m_l0_sums", 22: "m_l1_keys",
         23: "m_l1_sums", 21: "m_levels", 24: "m_end", 25: "k_nodes", 26: "k_table", 27: "k_ranked", 28: "k_lists", 29: "k_done"}


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    w = CONFIGS[name]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else w.num_samples
    lib = _lib.lib
    lib.srbd_probe_merge_phases.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    cfg = _lib.make_config(num_samples=n, horizon=w.horizon, method=w.method, parametrization=w.parametrization,
                           num_splines=w.num_splines, mass=w.mass, inertia=w.inertia,
                           dts=np.full(w.horizon, w.dt, np.float32), sigma_mppi=w.sigma)
    ctx = _lib.Context(cfg)
    s, r, c = inputs(w, 0)
    best = np.zeros(ctx.P, np.float32)
    sig = np.full(ctx.P, w.sigma, np.float32) if w.method == "cem_mppi" else None
    for k in range(5):
        best, _, _, _ = ctx.step(s, r, c, best, sigma=sig, counter=k)
    rows = []
    for rep in range(30):
        buf = np.zeros(64, np.uint64)
        assert lib.srbd_probe_merge_phases(ctx.h, buf.ctypes.data_as(C.POINTER(C.c_uint64))) == 0
        b0 = buf[:32].astype(np.int64)
        b1 = buf[32:].astype(np.int64)
        r = {v: (b0[k] - b0[0]) / 100.0 if b0[k] else None for k, v in NAMES.items() if k != 0}
        if b1[0]:  # block 1 (a column-split merge's first slice), relative to block 0's entry
            r.update({"b1_" + v: (b1[k] - b0[0]) / 100.0 if b1[k] else None for k, v in NAMES.items()})
        rows.append(r)
    ctx.close()
    out = {"workload": name, "n": n}
    for k in rows[0]:
        vals = [r[k] for r in rows[5:] if r.get(k) is not None]
        out[k] = round(float(np.median(vals)), 2) if vals else None
    print(json.dumps(out))


if __name__ == "__main__":
    main()
