"""C4 chained step with and without the per-step scores / patches copied to the host (measurement tool): the same
TamolsMpcStep.step loop as c4_split_probe.py, the second run with the foothold io's score and heightmap pointers
cleared (the kernel then stores neither and skips the system release), the objects the glue would build replaced
by placeholders.  One JSON line: step / C-call p50 per setting."""
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
fill = {"on": False}
dummy_hm = tuple(np.zeros((13, 7, 1, 3)) for _ in range(4))
dummy_sc = np.zeros((4, 91))


def timed(*a):
    t0 = time.perf_counter()
    r = real(*a)
    inner.append(time.perf_counter() - t0)
    if fill["on"] and r is not None and len(r) > 11:
        r = r[:10] + (dummy_hm, dummy_sc)
    return r


_lib.fast.foothold_step = timed
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
out = {}
ter = GpuTerrain.stepping_stones()
os.environ["SRBD_FOOTHOLD_CHAIN"] = "1"
for mode in ("outputs", "no_outputs", "outputs", "no_outputs"):
    pipe = TamolsMpcStep(ter, c4_config())
    fill["on"] = mode == "no_outputs"
    if fill["on"]:
        io = pipe._fused_io()
        io.scores = None
        io.heightmaps = None
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
    out.setdefault(mode, []).append({"step_p50_us": round(float(np.median(o)), 2),
                                     "c_call_p50_us": round(float(np.median(i)), 2)})
ter.close()
print(json.dumps(out))
