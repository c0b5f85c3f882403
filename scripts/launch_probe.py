#!/usr/bin/env python3
"""One kind of launch, alone, back to back (srbd_time_launch) -- for rocprofv3 PMC / SQ passes whose per-kernel
averages must describe exactly that launch (measurement tool, GPU box).

Usage: launch_probe.py CONFIG WHICH [ITERS] [RNG]
  CONFIG: c1..c5 / ns (quadruped_pympc_amd.synthetic.CONFIGS);  WHICH: step (the rollout launch exactly as
  srbd_step issues it), step_merge, fused (the plain rollout + next-step draws), rollout (plain, no draws), rng
One srbd_step runs first (it stages the inputs); prints one JSON line (average us, form bits).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quadruped-pympc-tamols_amd"))
sys.path.insert(0, ROOT)
from quadruped_pympc_amd import _lib  # noqa: E402
from quadruped_pympc_amd.synthetic import CONFIGS  # noqa: E402

import bench  # noqa: E402

WHICH = {"rng": _lib.TL_RNG, "rollout": _lib.TL_ROLLOUT, "fused": _lib.TL_ROLLOUT_FUSED, "step": _lib.TL_STEP_ROLLOUT,
         "step_merge": _lib.TL_STEP_MERGE}


def main():
    cfg_key, which = sys.argv[1], sys.argv[2]
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    rng = sys.argv[4] if len(sys.argv) > 4 else "philox"
    w = CONFIGS[cfg_key]
    ctx = _lib.Context(bench.make_cfg(_lib, w, w.num_samples, 0, 1, 0))
    if rng != "philox":
        ctx.set_rng(rng)
    s, r, c = bench.step_inputs(w, 1)[0]
    sigma = np.full(ctx.P, 3.0, np.float32) if w.method == "cem_mppi" else None
    keys = bench.KeyChain(_lib, rng)
    ctx.step(s, r, c, np.zeros(ctx.P, np.float32), sigma=sigma, seed=keys.at(0), counter=0)
    us, form = ctx.time_launch(WHICH[which], iters)
    ctx.close()
    print(json.dumps({"workload": w.name, "launch": which, "iters": iters, "us": round(us, 3), "form": form,
                      "rng": rng}))


if __name__ == "__main__":
    main()
