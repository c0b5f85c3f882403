#!/usr/bin/env python3
"""TAMOLS call anatomy on the GPU (measurement tool): phase stamps of the fused launch
(srbd_tamols_phases) and the host-to-host latency of srbd_tamols_run_terrain at C4."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "quadruped-pympc-tamols_amd"), ROOT]

import numpy as np  # noqa: E402

from quadruped_pympc_amd import _lib, config  # noqa: E402
from quadruped_pympc_amd.helpers.terrain import GpuTerrain  # noqa: E402
from quadruped_pympc_amd.helpers.visual_foothold_adaptation import TamolsSearch, tamols_params_struct  # noqa: E402

ter = GpuTerrain.stepping_stones()
srch = TamolsSearch(0)
params = dict(config.simulation_params["tamols_params"])
params["h_des"] = 0.25
ps = tamols_params_struct(params, "go2")
feet = np.array([[1.22, 0.13, 0.05], [1.22, -0.13, 0.05], [0.84, 0.13, 0.05], [0.84, -0.13, 0.05]])
hips = feet + np.array([0.0, 0.0, 0.3])
contact = np.array([0, 1, 1, 0], np.int32)
kw = dict(forward_vel=np.array([0.5, 0.0, 0.0]), base_position=np.array([1.03, 0.0, 0.35]), current_contact=contact,
          current_feet_pos=feet, want_scores=False, want_heightmaps=False)
_lib.lib.srbd_tamols_phases(srch.h, 1, None)
acc = np.zeros(5)
sub = np.zeros(3)
skew = np.zeros(4)  # block starts: last, median; last slice counted; last leg's end (us from the first start)
n = 200
for k in range(n + 10):
    srch.run_terrain(ter, 0.0, feet + np.array([0.12, 0.01, 0.0]), hips, ps, **kw)
    if k >= 10:
        out = np.zeros(5, np.float32)
        _lib.lib.srbd_tamols_phases(srch.h, 1, _lib.fptr(out))
        acc += out
        raw = np.zeros(4 * 64 * 8, np.uint64)  # block 0 of leg 0: start, staged, walked, patch done
        _lib.lib.srbd_tamols_phases_raw(srch.h, raw.ctypes.data)
        st = raw.reshape(4 * 64, 8).astype(np.float64)
        st = st[st[:, 0] > 0]  # the blocks of this call's legs (16 per leg, or one on a lattice patch)
        t0b = st[:, 0].min()
        skew += np.array([st[:, 0].max() - t0b, np.median(st[:, 0]) - t0b, st[:, 4].max() - t0b,
                          st[:, 5].max() - t0b]) * 0.01
        s0 = raw[:8].astype(np.float64)
        if s0[6] and s0[7]:
            sub += np.array([s0[6] - s0[0], s0[7] - s0[6], s0[1] - s0[7]]) * 0.01
_lib.lib.srbd_tamols_phases(srch.h, 0, None)
lat = []
for k in range(2010):
    t0 = time.perf_counter()
    srch.run_terrain(ter, 0.0, feet + np.array([0.12 + 0.001 * (k % 7), 0.01, 0.0]), hips, ps, **kw)
    lat.append(time.perf_counter() - t0)
lat = np.array(lat[10:]) * 1e6
print(json.dumps({"phases_us": dict(zip(("patch", "queries", "scores", "argmin_count", "span"),
                                        np.round(acc / n, 3).tolist())),
                  "patch_split_us": dict(zip(("stage_scene", "walk", "combine"), np.round(sub / n, 3).tolist())),
                  "starts_us": dict(zip(("last_start", "median_start", "last_counted", "last_leg_end"),
                                        np.round(skew / n, 3).tolist())),
                  "p50_us": round(float(np.percentile(lat, 50)), 2), "p99_us": round(float(np.percentile(lat, 99)), 2)}))
