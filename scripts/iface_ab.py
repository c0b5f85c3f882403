"""Plugin-API step A/B (measurement tool, GPU box): bench.py's interface_latency at C2 with the current
SRBDControllerInterface._fast_step and with the previous form of its eligibility checks (an os.environ lookup, a
function-level import and a set intersection with the controller's dict per call), interleaved.  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "quadruped-pympc-tamols_amd"))
import bench  # noqa: E402
from quadruped_pympc_amd import _lib  # noqa: E402
from quadruped_pympc_amd.interfaces import srbd_controller_interface as sci  # noqa: E402
from quadruped_pympc_amd.synthetic import CONFIGS  # noqa: E402

new_fast_step = sci.SRBDControllerInterface._fast_step
PATCHABLE = frozenset(("prepare_state_and_reference", "with_newkey", "with_newsigma", "shift_solution"))


def old_fast_step(self):
    ctrl = self.controller
    if _lib.fast is None or self._cfg.mpc_params["shift_solution"] or os.environ.get("SRBD_INTERFACE_FAST") == "0":
        return None
    from quadruped_pympc_amd.controllers.sampling import centroidal_nmpc_hip

    if type(ctrl) is not centroidal_nmpc_hip.Sampling_MPC:
        return None
    jcc = ctrl.jitted_compute_control
    if getattr(jcc, "__self__", None) is not ctrl or jcc.__func__ is not sci._OWN_COMPUTE.get(ctrl.sampling_method) \
            or PATCHABLE.intersection(ctrl.__dict__):
        return None
    fs = self._fast
    if fs is None or fs.ctrl is not ctrl or fs.ctx is not ctrl._ctx:
        fs = self._fast = sci._FastStep(self, ctrl)
    return fs


steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
res = {"old": [], "new": []}
for _ in range(3):
    for name, fn in (("old", old_fast_step), ("new", new_fast_step)):
        sci.SRBDControllerInterface._fast_step = fn
        res[name].append(bench.interface_latency(CONFIGS["c2"], steps)["p50_ms"] * 1e3)
print(json.dumps({k: [round(v, 2) for v in vs] for k, vs in res.items()}))
