"""Python costs around the C4 step's one C call (measurement tool, GPU box): the pieces TamolsMpcStep.step runs per
call, each timed alone in a loop on a live pipeline (us per call).  One JSON line."""
import ctypes as C
import json
import os
import sys
import timeit

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "quadruped-pympc-tamols_amd"))
import numpy as np  # noqa: E402

from quadruped_pympc_amd import _lib  # noqa: E402
from quadruped_pympc_amd.helpers.foothold_pipeline import TamolsMpcStep  # noqa: E402
from quadruped_pympc_amd.helpers.legs_attr import LegsAttr  # noqa: E402
from quadruped_pympc_amd.helpers.terrain import GpuTerrain  # noqa: E402
from quadruped_pympc_amd.synthetic import c4_config, c4_inputs  # noqa: E402

ter = GpuTerrain.stepping_stones()
pipe = TamolsMpcStep(ter, c4_config())
state, seeds, hips, ref_base, cs = c4_inputs(0)
args = (state, LegsAttr(*seeds), LegsAttr(*hips), ref_base, cs, state["linear_velocity"], state["orientation"],
        state["angular_velocity"], np.zeros(4), 1.4)
for _ in range(30):
    pipe.step(*args)
ctrl, vfa = pipe.controller, pipe.vfa
n = 20000
parts = {
    "_fusable": lambda: pipe._fusable(),
    "asarray+shape": lambda: (np.asarray(cs).ndim == 2 and cs.shape[0] == 4 and cs.shape[1] >= ctrl.horizon),
    "_fused_io": lambda: pipe._fused_io(),
    "SrbdResult()": lambda: _lib.SrbdResult(),
    "arg gathering": lambda: (vfa.search.h.value, pipe.heightmaps.FL.terrain.h.value, C.addressof(vfa._params()),
                              ctrl.context.h.value, C.addressof(pipe._io), ctrl.num_control_parameters_single_leg,
                              _lib.RNG_CODES[ctrl.rng]),
    "LegsAttr x2": lambda: (LegsAttr(*seeds), LegsAttr(*hips)),
    "whole step": lambda: pipe.step(*args),
}
out = {k: round(timeit.timeit(f, number=n if k != "whole step" else 2000) / (n if k != "whole step" else 2000) * 1e6, 3)
       for k, f in parts.items()}
pipe.close()
ter.close()
print(json.dumps(out))
