"""Where _fused_outputs' time goes in a C4 step (one-call path): the method re-stated with perf_counter marks,
p50 per section (us), over 3000 steps on the GPU box."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "quadruped-pympc-tamols_amd"))
import numpy as np  # noqa: E402

from quadruped_pympc_amd import _lib  # noqa: E402
from quadruped_pympc_amd.helpers import foothold_pipeline as fp  # noqa: E402
from quadruped_pympc_amd.helpers.legs_attr import LegsAttr  # noqa: E402
from quadruped_pympc_amd.helpers.terrain import GpuTerrain  # noqa: E402
from quadruped_pympc_amd.synthetic import c4_config, c4_inputs  # noqa: E402

LEGS = fp.LEGS
M = {}
pc = time.perf_counter


def mark(t, k):
    t2 = pc()
    M.setdefault(k, []).append(t2 - t)
    return t2


def outputs(self, rc, res, current_contact, made, seeds, ref_base):
    t = pc()
    iface, ctrl, vfa, io, a = self.iface, self.iface.controller, self.vfa, self._io, self._io_np
    ctx = ctrl.context
    t = mark(t, "attrs")
    hm = self._io_hm.copy()
    t = mark(t, "hm_copy")
    hms = self.heightmaps
    hms.FL._data, hms.FR._data, hms.RL._data, hms.RR._data = hm
    hms.FL.pending = hms.FR.pending = hms.RL.pending = hms.RR.pending = None
    t = mark(t, "hm_set")
    fh = a["footholds"].reshape(4, 3).copy()
    f0, f1, f2, f3 = fh
    t = mark(t, "fh")
    valid = io.valid
    constraints = vfa.footholds_constraints
    if valid[0] or valid[1] or valid[2] or valid[3]:
        boxes = a["boxes"].reshape(4, 2, 3).copy()
        for i, b in enumerate(boxes):
            if valid[i]:
                constraints[LEGS[i]] = [b[0], b[1]]
    t = mark(t, "boxes")
    vfa.last_scores = self._io_scores.copy()
    t = mark(t, "scores")
    vfa.footholds_adaptation, vfa.initialized = LegsAttr(f0, f1, f2, f3), True
    self._ref_state, self._ref_src = None, (ref_base, fh, LegsAttr(*constraints))
    self.last_constraints = constraints
    t = mark(t, "legsattrs")
    iface.previous_contact_mpc = current_contact
    ctrl.best_control_parameters = made[2]
    ctx.step_id += 1
    ctrl.last_result = res
    g, pred = made[0], made[1]
    t = mark(t, "ctrl")
    r = LegsAttr(*g), LegsAttr(f0, f1, f2, f3), None, None, None, 1.4, pred
    mark(t, "ret")
    return r


fp.TamolsMpcStep._fused_outputs = outputs
ter = GpuTerrain.stepping_stones()
pipe = fp.TamolsMpcStep(ter, c4_config())
ins = [c4_inputs(k) for k in range(16)]
for k in range(3020):
    state, seeds, hips, ref_base, cs = ins[k % 16]
    pipe.step(state, LegsAttr(*seeds), LegsAttr(*hips), ref_base, cs, state["linear_velocity"],
              state["orientation"], state["angular_velocity"], np.zeros(4), 1.4)
pipe.close()
ter.close()
print(json.dumps({k: round(float(np.median(v[20:])) * 1e6, 3) for k, v in M.items()}))
