#!/usr/bin/env python3
"""Timeline of one rollout launch from per-block s_memrealtime stamps (measurement tool; GPU box).

Needs the probe build (`make -C quadruped-pympc-tamols_amd probe`).  Stamps, thread 0 of each block,
after draining its memory operations: 0 entry, 2 horizon done (the prefetch is not stamped: its loads overlap the horizon), 3 block
min/top-K done, 4 weighted sums done, 5 exit (RNG blocks: 0 entry, 5 exit).  Prints one JSON line per
workload: percentiles (us, relative to the earliest block entry) of each stamp over rollout blocks and
of the RNG blocks' entry/exit, plus the mean of each phase.
Usage: python scripts/rollout_timeline.py [c2|c3|...] [N] [mode=quad|thread]
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

NS = 6


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    w = CONFIGS[name]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else w.num_samples
    if len(sys.argv) > 3:
        os.environ["SRBD_ROLLOUT"] = sys.argv[3]
    lib = _lib.lib
    lib.srbd_probe_rstamps.argtypes = [C.POINTER(C.c_uint64), C.c_int]
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
    for rep in range(20):
        lib.srbd_probe_rstamps_clear()
        ctx.time_kernels(1)  # last rollout launch: the fused one when fusion applies
        buf = np.zeros(8192 * NS, np.uint64)
        assert lib.srbd_probe_rstamps(buf.ctypes.data_as(C.POINTER(C.c_uint64)), buf.size) == 0
        st = buf.reshape(-1, NS).astype(np.int64)
        used = st[:, 0] > 0
        st = st[used]
        if not len(st):  # no stamps (e.g. the launch timed was not a rollout of this build): skip the repetition
            continue
        roll = st[:, 2] > 0
        t0 = st[:, 0].min()
        rel = (st - t0) / 100.0  # 100 MHz ticks -> us
        rows.append((rel, roll))
    ctx.close()
    out = {"workload": name, "n": n, "mode": os.environ.get("SRBD_ROLLOUT", "default")}
    if not rows:
        out["error"] = "no block stamps recorded"
        print(json.dumps(out))
        return
    rel, roll = rows[-1]
    out["blocks_rollout"] = int(roll.sum())
    out["blocks_rng"] = int((~roll).sum())
    def pct(x):
        return [round(float(np.percentile(x, q)), 2) for q in (0, 50, 90, 100)]
    agg = {}
    for rel, roll in rows[5:]:
        R = rel[roll]
        G = rel[~roll]
        for i in range(NS):
            if i == 1:  # stamp 1 is not recorded (the prefetch overlaps the horizon)
                continue
            agg.setdefault(f"roll_s{i}", []).append(pct(R[:, i]))
        for i, j, nm in ((0, 2, "prefetch_horizon"), (2, 3, "min"), (3, 4, "wsum"), (4, 5, "tail")):
            agg.setdefault(f"phase_{nm}", []).append(float(np.mean(R[:, j] - R[:, i])))
        if len(G):
            agg.setdefault("rng_entry", []).append(pct(G[:, 0]))
            agg.setdefault("rng_exit", []).append(pct(G[:, 5]))
            agg.setdefault("rng_dur", []).append(float(np.mean(G[:, 5] - G[:, 0])))
    for k, v in agg.items():
        out[k] = np.round(np.median(np.array(v), axis=0), 2).tolist()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
