#!/usr/bin/env python3
"""Tail of one host-step launch (rollout + level-1 folds + in-launch final merge) from s_memrealtime stamps
(measurement tool; GPU box, probe build: `make -C quadruped-pympc-tamols_amd probe`).

Relative to the earliest block entry (us): the last rollout block's leaf sums done (RSTAMP 4), then for the
block that ran the final merge: its leaf sums done, its level-1 fold marks (entry, own stores drained, last of
its group, group's leaf records staged), final_merge marks (entry, group record stores drained, last group,
group records staged) and its merge_body stamps (beta, sums, outputs, published), and its exit (RSTAMP 5).
Prints one JSON line per workload: medians over 20 steps.
Usage: python scripts/step_tail.py [c2|ns|...] [N]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "quadruped-pympc-tamols_amd")
os.environ["SRBD_LIB_PATH"] = os.path.join(PKG, "quadruped_pympc_amd", os.environ.get("SRBD_PROBE_SO", "libsrbd_hip_probe.so"))
sys.path.insert(0, PKG)
from quadruped_pympc_amd import _lib  # noqa: E402
from quadruped_pympc_amd.synthetic import CONFIGS, inputs  # noqa: E402

NS = 6
NB = 8192


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    w = CONFIGS[name]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else w.num_samples
    lib = _lib.lib
    lib.srbd_probe_rstamps.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    lib.srbd_probe_fstamps.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    cfg = _lib.make_config(num_samples=n, horizon=w.horizon, method=w.method, parametrization=w.parametrization,
                           num_splines=w.num_splines, mass=w.mass, inertia=w.inertia,
                           dts=np.full(w.horizon, w.dt, np.float32), sigma_mppi=w.sigma)
    ctx = _lib.Context(cfg)
    s, r, c = inputs(w, 0)
    best = np.zeros(ctx.P, np.float32)
    rows = []
    for k in range(25):
        lib.srbd_probe_rstamps_clear()
        lib.srbd_probe_fstamps_clear()
        best, _, _, _ = ctx.step(s, r, c, best, counter=k)
        rs = np.zeros(NB * NS, np.uint64)
        fs = np.zeros(64 + NB * 8, np.uint64)
        assert lib.srbd_probe_rstamps(rs.ctypes.data_as(C.POINTER(C.c_uint64)), rs.size) == 0
        assert lib.srbd_probe_fstamps(fs.ctypes.data_as(C.POINTER(C.c_uint64)), NB * 8) == 0
        st = rs.reshape(-1, NS).astype(np.int64)
        if fs[0] == 0:
            continue  # no final merge in this launch
        b = int(fs[0]) - 1
        roll = st[:, 2] > 0
        t0 = st[st[:, 0] > 0, 0].min()
        us = lambda t: round((int(t) - t0) / 100.0, 2) if t else None  # noqa: E731
        lst = fs[64:].reshape(-1, 8)
        fast = fs[32] == 0 and fs[13] != 0  # fast_tail: its own marks, no merge_body stamps
        row = {"last_leaf_sums": us(st[roll, 4].max()), "fm_block_leaf_sums": us(st[b, 4]),
               "fold_entry": us(lst[b, 0]), "fold_drained": us(lst[b, 1]), "fold_last": us(lst[b, 2]),
               "fold_staged": us(lst[b, 3]), "fold_headers": us(lst[b, 4]), "fold_sums": us(lst[b, 5])}
        if fast:
            for i, nm in ((1, "ft_own_fold"), (2, "ft_words_issued"), (3, "ft_headers_in"), (4, "ft_root_key"),
                          (5, "ft_wsum"), (6, "ft_batch_a_in"), (7, "ft_batch_b_poll"), (8, "ft_batch_b_in"),
                          (9, "ft_root_sums"), (10, "ft_best_stored"), (11, "ft_barrier"), (12, "ft_outputs"),
                          (13, "ft_published")):
                row[nm] = us(fs[i])
        else:
            row.update({"fm_entry": us(fs[1]), "fm_drained": us(fs[2]), "fm_last": us(fs[3]), "fm_staged": us(fs[4])})
            for i, nm in ((0, "m_entry"), (6, "m_staged"), (16, "m_beta_scan"), (17, "m_tail_prep"), (18, "m_barrier"),
                          (1, "m_beta"), (20, "m_l0_sums"), (21, "m_levels"), (2, "m_sums"), (3, "m_topk"),
                          (4, "m_outputs"), (5, "m_published")):
                row[nm] = us(fs[32 + i])
        row["fm_block_exit"] = us(st[b, 5])
        row["launch_end"] = us(st[st[:, 0] > 0, 5].max())
        rows.append(row)
    ctx.close()
    out = {"workload": name, "n": n, "steps": len(rows)}
    for key in rows[0]:
        v = [x[key] for x in rows[5:] if x[key] is not None]
        out[key] = round(float(np.median(v)), 2) if v else None
    print(json.dumps(out))


if __name__ == "__main__":
    main()
