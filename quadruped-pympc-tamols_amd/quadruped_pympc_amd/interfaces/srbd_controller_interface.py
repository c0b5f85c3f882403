"""``SRBDControllerInterface`` for the MI355X sampling MPC.

Mirror of ``quadruped_pympc/interfaces/srbd_controller_interface.py`` (:7-240),
``type == 'sampling'`` branch (:118-180, :225-240): the same per-call sequence
(prepare_state_and_reference -> per sampling iteration: with_newkey [+ sigma reset
for CEM] -> jitted_compute_control -> reassign best_control_parameters) and the same
7-tuple return.  Gradient (acados) controllers are out of scope and raise.

With the plain ``Sampling_MPC`` and no solution shift, the whole sequence is one library call
(``srbd_interface_step``: prepare_state, the key splits, CEM's sigma reset, the device steps and the GRF
mask, in the same order), its arguments gathered and its results built by the ``_srbd_fast`` glue;
the controller's attributes end as the Python sequence leaves them (``tests/test_gpu_interface_step.py``
pins the two bit for bit).  ``SRBD_INTERFACE_FAST=0`` when an interface is created makes it run the Python
sequence.
"""
from __future__ import annotations

import os

import numpy as np

from .. import _lib
from ..runtime import active_config
from ..helpers.legs_attr import LegsAttr


class SRBDControllerInterface:
    """This is an interface for a controller that uses the SRBD method to optimize the gait"""

    def __init__(self, config_module=None):
        cfg = active_config(config_module)  # the reference's quadruped_pympc.config when installed
        self._cfg = cfg
        self.type = cfg.mpc_params["type"]
        self.mpc_dt = cfg.mpc_params["dt"]
        self.horizon = cfg.mpc_params["horizon"]
        self.optimize_step_freq = cfg.mpc_params["optimize_step_freq"]
        self.step_freq_available = cfg.mpc_params["step_freq_available"]
        self.previous_contact_mpc = np.array([1, 1, 1, 1])
        if self.type != "sampling":
            raise NotImplementedError(f"controller type {self.type!r}: only 'sampling' is provided (MI355X HIP)")
        if self.optimize_step_freq:  # srbd_controller_interface.py:77-81
            from ..controllers.sampling.centroidal_nmpc_hip_gait_adaptive import Sampling_MPC
        else:
            from ..controllers.sampling.centroidal_nmpc_hip import Sampling_MPC

        self.controller = Sampling_MPC(cfg)
        self._fast = None  # _FastStep of the one-call path, made on the first eligible call
        # read once: os.environ lookups cost ~1 us, a fifth of the Python around the one call
        self._fast_env = os.environ.get("SRBD_INTERFACE_FAST") != "0"

    def __getstate__(self):  # a copy makes its own one-call staging (it caches raw addresses)
        d = dict(self.__dict__)
        d["_fast"] = None
        return d

    def __setstate__(self, d):
        d.setdefault("_fast_env", True)
        self.__dict__.update(d)

    def _fast_step(self):
        """The one-call path when it makes exactly the Python sequence's calls: the glue is built, the plain
        Sampling_MPC (not the gait-adaptive one), no solution shift."""
        ctrl = self.controller
        if not self._fast_env or _lib.fast is None or self._cfg.mpc_params["shift_solution"]:
            return None
        if type(ctrl) is not _SAMPLING_MPC:
            return None
        # the controller's own methods, not instance-level replacements of the ones the sequence calls (four
        # lookups: a set intersection with the instance dict cost 1 us)
        d = ctrl.__dict__
        if "prepare_state_and_reference" in d or "with_newkey" in d or "with_newsigma" in d or "shift_solution" in d:
            return None
        jcc = ctrl.jitted_compute_control
        if getattr(jcc, "__self__", None) is not ctrl or jcc.__func__ is not _OWN_COMPUTE.get(ctrl.sampling_method):
            return None
        fs = self._fast
        if fs is None or fs.ctrl is not ctrl or fs.ctx is not ctrl._ctx:
            fs = self._fast = _FastStep(self, ctrl)
        return fs

    def compute_control(self, state_current: dict, ref_state: dict, contact_sequence: np.ndarray, inertia: np.ndarray,
                        pgg_phase_signal: np.ndarray, pgg_step_freq: float, optimize_swing: int,
                        external_wrenches: np.ndarray = np.zeros((6,))):
        fs = self._fast_step()
        if fs is not None:
            out = fs.step(state_current, ref_state, contact_sequence)
            if out is not None:
                return out
        current_contact = np.array([contact_sequence[0][0], contact_sequence[1][0], contact_sequence[2][0],
                                    contact_sequence[3][0]])
        state_current_jax, reference_state_jax = self.controller.prepare_state_and_reference(
            state_current, ref_state, current_contact, self.previous_contact_mpc)
        self.previous_contact_mpc = current_contact

        for iter_sampling in range(self.controller.num_sampling_iterations):
            self.controller = self.controller.with_newkey()
            if self.controller.sampling_method == "cem_mppi":
                if iter_sampling == 0:
                    self.controller = self.controller.with_newsigma(self._cfg.mpc_params["sigma_cem_mppi"])
                (nmpc_GRFs, nmpc_footholds, nmpc_predicted_state, self.controller.best_control_parameters, best_cost,
                 best_sample_freq, costs, sigma_cem_mppi) = self.controller.jitted_compute_control(
                    state_current_jax, reference_state_jax, contact_sequence,
                    self.controller.best_control_parameters, self.controller.master_key,
                    self.controller.sigma_cem_mppi)
                self.controller = self.controller.with_newsigma(sigma_cem_mppi)
            else:
                (nmpc_GRFs, nmpc_footholds, nmpc_predicted_state, self.controller.best_control_parameters, best_cost,
                 best_sample_freq, costs) = self.controller.jitted_compute_control(
                    state_current_jax, reference_state_jax, contact_sequence,
                    self.controller.best_control_parameters, self.controller.master_key, pgg_phase_signal,
                    pgg_step_freq, optimize_swing)

        nmpc_footholds = LegsAttr(FL=ref_state["ref_foot_FL"][0], FR=ref_state["ref_foot_FR"][0],
                                  RL=ref_state["ref_foot_RL"][0], RR=ref_state["ref_foot_RR"][0])
        # leg l's GRFs times current_contact[l] (SCI:175-178), the four products in one array operation (the same
        # dtype promotion and values as four array x scalar products)
        g = np.asarray(nmpc_GRFs).reshape(4, 3) * current_contact[:, None]
        nmpc_GRFs = LegsAttr(FL=g[0], FR=g[1], RL=g[2], RR=g[3])
        return nmpc_GRFs, nmpc_footholds, None, None, None, best_sample_freq, nmpc_predicted_state


def _own_compute():
    from ..controllers.sampling.centroidal_nmpc_hip import Sampling_MPC as S

    return S, {"random_sampling": S.compute_control_random_sampling, "mppi": S.compute_control_mppi,
               "cem_mppi": S.compute_control_cem_mppi}


_SAMPLING_MPC, _OWN_COMPUTE = _own_compute()


class _FastStep:
    """compute_control's sampling branch in one library call (srbd_interface_step through _lib.fast)."""

    def __init__(self, iface: SRBDControllerInterface, ctrl):
        self.iface, self.ctrl = iface, ctrl
        ctx = ctrl.context  # created here if the controller has not stepped yet
        self.ctx, self.h = ctx, ctx.h.value
        self.cem = ctrl.sampling_method == "cem_mppi"
        self.io = io = _lib.InterfaceIO()
        io.horizon = ctrl.horizon
        io.rng = _lib.RNG_CODES[ctrl.rng]
        io.cem = 1 if self.cem else 0
        self.io_addr = _lib.C.addressof(io)
        self.best_buf = np.zeros(ctrl.num_control_parameters, np.float32)
        self.sigma_buf = np.zeros(ctrl.num_control_parameters, np.float32) if self.cem else None
        self.res = _lib.SrbdResult()
        self.res_addr = _lib.C.addressof(self.res)
        self.freq = 1.65 if self.cem else 1.4  # best_sample_freq of compute_control_{cem_mppi, mppi, rs}
        self.jax = ctrl.rng != "philox"

    def step(self, state_current, ref_state, contact_sequence):
        ctrl, iface = self.ctrl, self.iface
        mp = iface._cfg.mpc_params
        r = _lib.fast.interface_step(self.h, self.io_addr, state_current, ref_state, contact_sequence,
                                     ctrl.best_control_parameters, iface.previous_contact_mpc, ctrl.master_key,
                                     ctrl._calls, ctrl.num_sampling_iterations,
                                     mp["sigma_cem_mppi"] if self.cem else None, self.best_buf, self.sigma_buf,
                                     self.res_addr)
        if r is None:  # an input form the glue does not take: the Python sequence
            return None
        f32_contact = contact_sequence.dtype == np.float32
        if len(r) == 3:
            self._failed(*r, f32_contact)
        grf, pred, best, sigma, key, calls, cur, fh = r
        if f32_contact:  # as the Python sequence's float32 current_contact gives (the float64 product is exact)
            cur, grf = cur.astype(np.float32), grf.astype(np.float32)
        iface.previous_contact_mpc = cur
        ctrl.best_control_parameters = best
        ctrl.master_key = key
        if self.jax:
            ctrl._calls = calls
        if self.cem:
            ctrl.sigma_cem_mppi = sigma
        ctrl.last_result = _lib.SrbdResult.from_buffer_copy(self.res)
        self.ctx.step_id += ctrl.num_sampling_iterations
        return LegsAttr(*grf), LegsAttr(*fh), None, None, None, self.freq, pred

    def _failed(self, rc, stage, cur, f32_contact):
        """A call of the chain failed: leave the objects as the Python sequence leaves them, then raise as it does."""
        ctrl, io = self.ctrl, self.io
        if stage >= 1:  # prepare_state ran; `stage - 1` steps completed, the failing one's key split had run
            self.iface.previous_contact_mpc = cur.astype(np.float32) if f32_contact else cur
            ctrl.best_control_parameters = self.best_buf.copy()
            if self.jax:
                k = int(io.key[0])
                ctrl.master_key = np.array([k >> 32, k & 0xFFFFFFFF], np.uint32)
                ctrl._calls = int(io.key[1])
            else:
                ctrl.master_key = np.array([io.key[0], io.key[1]], np.uint64)
            if self.cem:
                ctrl.sigma_cem_mppi = self.sigma_buf.copy() if stage >= 2 else self.iface._cfg.mpc_params[
                    "sigma_cem_mppi"]
            self.ctx.step_id += stage - 1
        what = "srbd_prepare_state" if stage == 0 else "srbd_step"
        raise RuntimeError(f"{what} failed ({rc}): {_lib.last_error(self.ctx.h)}")
