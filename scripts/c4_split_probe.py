"""C4 per-MPC-step time split: the whole TamolsMpcStep.step (Python) vs its one C call (_srbd_fast.foothold_step,
srbd_foothold_mpc_step inside), chained on the device or sequential (SRBD_FOOTHOLD_CHAIN=0); one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "quadruped-pympc-tamols_amd"))
import numpy as np  # noqa: E402

from quadruped_pympc_amd import _lib  # noqa: E402
from quadruped_pympc_amd.helpers.foothold_pipeline import TamolsMpcStep  # noqa: E402
from quadruped_pympc_amd.helpers.legs_attr import LegsAttr  # noqa: E402
from quadruped_pympc_amd.helpers.terrain import GpuTerrain  # noqa: E402
from quadruped_pympc_amd.synthetic import c4_config, c4_inputs  # noqa: E402

inner = []
real = _lib.fast.foothold_step


def timed(*a):
    t0 = time.perf_counter()
    r = real(*a)
    inner.append(time.perf_counter() - t0)
    return r


_lib.fast.foothold_step = timed
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
out = {}
ter = GpuTerrain.stepping_stones()
for mode in ("1", "0", "1"):
    os.environ["SRBD_FOOTHOLD_CHAIN"] = mode
    pipe = TamolsMpcStep(ter, c4_config())
    ins = [c4_inputs(k) for k in range(16)]
    outer = []
    inner.clear()
    for k in range(steps + 20):
        state, seeds, hips, ref_base, cs = ins[k % 16]
        t0 = time.perf_counter()
        pipe.step(state, LegsAttr(*seeds), LegsAttr(*hips), ref_base, cs, state["linear_velocity"],
                  state["orientation"], state["angular_velocity"], np.zeros(4), 1.4)
        outer.append(time.perf_counter() - t0)
    pipe.close()
    o, i = np.array(outer[20:]) * 1e6, np.array(inner[20:]) * 1e6
    out.setdefault("chain" if mode == "1" else "sequential", []).append(
        {"step_p50_us": round(float(np.median(o)), 2), "c_call_p50_us": round(float(np.median(i)), 2),
         "python_p50_us": round(float(np.median(o - i)), 2)})
ter.close()
print(json.dumps(out))
