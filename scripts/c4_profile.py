#!/usr/bin/env python3
"""cProfile of the C4 per-MPC-step pipeline (helpers/foothold_pipeline.py TamolsMpcStep.step) on the GPU box: where
the Python time between the two launches (raycast + TAMOLS, the MPPI step) goes.  Usage: c4_profile.py [steps]"""
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quadruped-pympc-tamols_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from quadruped_pympc_amd.helpers.foothold_pipeline import TamolsMpcStep  # noqa: E402
from quadruped_pympc_amd.helpers.legs_attr import LegsAttr  # noqa: E402
from quadruped_pympc_amd.helpers.terrain import GpuTerrain  # noqa: E402
from quadruped_pympc_amd.synthetic import c4_config, c4_inputs  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
ter = GpuTerrain.stepping_stones()
pipe = TamolsMpcStep(ter, c4_config())
ins = [c4_inputs(k) for k in range(16)]


def run(n):
    for k in range(n):
        state, seeds, hips, ref_base, cs = ins[k % len(ins)]
        pipe.step(state, LegsAttr(*seeds), LegsAttr(*hips), ref_base, cs, state["linear_velocity"],
                  state["orientation"], state["angular_velocity"], np.zeros(4), 1.4)


run(20)
pr = cProfile.Profile()
pr.enable()
run(steps)
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(35)
print(s.getvalue())
pipe.close()
ter.close()
