"""Where the Python time of a C4 step (TamolsMpcStep.step, one-call path) goes: per-method p50 (us)."""
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

T = {}


def wrap(owner, name, key):
    f = getattr(owner, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        T.setdefault(key, []).append(time.perf_counter() - t0)
        return r
    setattr(owner, name, g)


wrap(fp.TamolsMpcStep, "_fusable", "fusable")
wrap(fp.TamolsMpcStep, "_fused_outputs", "fused_outputs")
wrap(fp.TamolsMpcStep, "_step_fused", "step_fused")
wrap(_lib.fast, "foothold_step", "c_call")
wrap(fp.VisualFootholdAdaptation, "update_footholds_adaptation", "vfa_update")
wrap(fp.VisualFootholdAdaptation, "reset", "vfa_reset")
ter = GpuTerrain.stepping_stones()
pipe = fp.TamolsMpcStep(ter, c4_config())
ins = [c4_inputs(k) for k in range(16)]
outer = []
for k in range(3020):
    state, seeds, hips, ref_base, cs = ins[k % 16]
    t0 = time.perf_counter()
    pipe.step(state, LegsAttr(*seeds), LegsAttr(*hips), ref_base, cs, state["linear_velocity"],
              state["orientation"], state["angular_velocity"], np.zeros(4), 1.4)
    outer.append(time.perf_counter() - t0)
pipe.close()
ter.close()
out = {"step": round(float(np.median(outer[20:])) * 1e6, 2)}
out.update({k: round(float(np.median(v[20:])) * 1e6, 2) for k, v in T.items()})
print(json.dumps(out))
