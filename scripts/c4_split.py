#!/usr/bin/env python3
"""Wall-clock split of the C4 per-MPC-step pipeline on the GPU box (no profiler): the raycast + TAMOLS launch
(srbd_tamols_run_terrain) and the MPPI step (srbd_step) -- or the one-call srbd_foothold_mpc_step -- timed inside the
step by wrapping the C entry points;
the rest is host Python.  Usage: c4_split.py [steps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quadruped-pympc-tamols_amd"))

import numpy as np  # noqa: E402

from quadruped_pympc_amd import _lib  # noqa: E402
from quadruped_pympc_amd.helpers.foothold_pipeline import TamolsMpcStep  # noqa: E402
from quadruped_pympc_amd.helpers.legs_attr import LegsAttr  # noqa: E402
from quadruped_pympc_amd.helpers.terrain import GpuTerrain  # noqa: E402
from quadruped_pympc_amd.synthetic import c4_config, c4_inputs  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
acc = {}


class Timed:
    """Forwards to a ctypes function, adding its wall time to acc[name]."""

    def __init__(self, name, fn):
        self.name, self.fn = name, fn

    def __call__(self, *a):
        t0 = time.perf_counter()
        r = self.fn(*a)
        acc[self.name] = acc.get(self.name, 0.0) + time.perf_counter() - t0
        return r


for name in ("srbd_tamols_run_terrain", "srbd_step", "srbd_prepare_state", "srbd_foothold_mpc_step"):
    setattr(_lib.lib, name, Timed(name, getattr(_lib.lib, name)))

ter = GpuTerrain.stepping_stones()
pipe = TamolsMpcStep(ter, c4_config())
ins = [c4_inputs(k) for k in range(16)]
total = 0.0
for k in range(steps + 50):
    if k == 50:
        acc.clear()
        total = 0.0
    state, seeds, hips, ref_base, cs = ins[k % len(ins)]
    t0 = time.perf_counter()
    pipe.step(state, LegsAttr(*seeds), LegsAttr(*hips), ref_base, cs, state["linear_velocity"],
              state["orientation"], state["angular_velocity"], np.zeros(4), 1.4)
    total += time.perf_counter() - t0
out = {k: round(v / steps * 1e6, 2) for k, v in acc.items()}
out["step_us"] = round(total / steps * 1e6, 2)
out["host_python_us"] = round(out["step_us"] - sum(v for k, v in out.items() if k != "step_us"), 2)
print(json.dumps(out))
pipe.close()
ter.close()
