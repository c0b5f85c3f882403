"""One MPC step of the reference's terrain-aware sampling loop (BASELINE configs[3], C4: TAMOLS foothold search +
MPPI N = 10 000 on stepping stones), as ``WBInterface.update_state_and_reference`` and
``SRBDControllerInterface.compute_control`` chain it (wb_interface.py:230-291, srbd_controller_interface.py:113-180):

1. the four legs' heightmaps are updated around the reference footholds at the base yaw (wb_interface.py:233-234);
2. ``VisualFootholdAdaptation.compute_adaptation`` runs TAMOLS on them (:235-240) -- with ``GpuHeightMap`` patches of
   one ``GpuTerrain`` the raycasts and the search are one launch (``srbd_tamols_run_terrain``);
3. ``get_footholds_adapted`` gives the adapted footholds and their constraint boxes (:245);
4. they become ``ref_state``'s ``ref_foot_*`` beside the base reference (:268-285);
5. ``SRBDControllerInterface.compute_control``: ``prepare_state_and_reference`` (swing feet replaced by their
   reference footholds, the warm start of legs that just lifted off zeroed; C++) and one sampling step per iteration
   (``srbd_step`` on the GPU).

What the reference computes around this (the foothold reference generator, the swing / apex bookkeeping that decides
WHEN to adapt, terrain slope estimation, the whole-body controller) is outside the sampling hot path and
stays the caller's: ``step`` takes the reference footholds, hips and base reference as inputs and adapts on every
call (the per-step cost C4 names).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .. import _lib
from ..controllers.sampling import centroidal_nmpc_hip
from ..interfaces.srbd_controller_interface import SRBDControllerInterface
from ..runtime import active_config
from .legs_attr import LegsAttr
from .terrain import GpuHeightMap, GpuTerrain
from .visual_foothold_adaptation import VisualFootholdAdaptation

LEGS = ("FL", "FR", "RL", "RR")


class TamolsMpcStep:
    """Heightmaps over a device-resident terrain, the TAMOLS adaptation and the sampling controller of one robot."""

    def __init__(self, terrain: GpuTerrain, config_module=None, num_rows=13, num_cols=7, dist_x=0.04, dist_y=0.04):
        cfg = active_config(config_module)
        self.cfg = cfg
        self.heightmaps = LegsAttr(*[GpuHeightMap(terrain, num_rows, num_cols, dist_x, dist_y) for _ in LEGS])
        self.vfa = VisualFootholdAdaptation(LEGS, "tamols", cfg)
        self.iface = SRBDControllerInterface(cfg)
        self._ref_state = None
        self._ref_src = None  # (ref_base, the 4 foothold rows, constraints) of a fused step, made into a dict on demand
        self.last_constraints = None
        self.fused = True  # srbd_foothold_mpc_step when the configuration allows (see _fusable)
        self._io = None

    @property
    def controller(self):
        return self.iface.controller

    @property
    def last_ref_state(self):
        """The ref_state the last step gave compute_control (wb_interface.py:268-285)."""
        if self._ref_src is not None:
            ref_base, rows, constraints = self._ref_src
            ref_state = dict(ref_base)
            for i, n in enumerate(LEGS):
                ref_state["ref_foot_" + n] = rows[i][None]  # (1, 3), as wb_interface.py:268-285 shapes it
                ref_state["ref_foot_constraints_" + n] = constraints[n]
            self._ref_state, self._ref_src = ref_state, None
        return self._ref_state

    def _fusable(self):
        """One host call (srbd_foothold_mpc_step) makes exactly the Python chain's calls when: the plain sampling
        controller (not the gait-adaptive one), MPPI or random sampling (no sigma), one sampling iteration, no
        solution shift, TAMOLS adaptation, and the four maps over one terrain with one patch geometry."""
        ctrl = self.iface.controller
        if not self.fused or type(ctrl) is not centroidal_nmpc_hip.Sampling_MPC:
            return False
        if ctrl.sampling_method == "cem_mppi" or ctrl.num_sampling_iterations != 1:
            return False
        if self.cfg.mpc_params["shift_solution"] or self.vfa.adaptation_strategy != "tamols":
            return False
        g = self.heightmaps.FL
        geo = (g.terrain, g.num_rows, g.num_cols, g.dist_x, g.dist_y, g.ray_z)
        return all(isinstance(m, GpuHeightMap) and (m.terrain, m.num_rows, m.num_cols, m.dist_x, m.dist_y, m.ray_z)
                   == geo for m in self.heightmaps)

    def _fused_io(self):
        io = self._io
        if io is None:
            g = self.heightmaps.FL
            io = self._io = _lib.FootholdIO()
            io.rows, io.cols, io.dist_x, io.dist_y, io.ray_z = g.num_rows, g.num_cols, g.dist_x, g.dist_y, g.ray_z
            self._io_np = {k: np.ctypeslib.as_array(getattr(io, k)) for k in
                           ("state_in", "ref_base", "seeds", "hips", "forward_vel", "current_contact",
                            "previous_contact", "footholds", "boxes", "seed_heights", "valid")}
            self._io_scores = np.zeros((4, g.num_rows * g.num_cols))
            # the patches are not copied out: the maps stay pending around the seeds and raycast on access (the same
            # values); the scores only when vfa.keep_scores (without either, the TAMOLS launch stores nothing to the
            # host but its outputs and needs no system release before them: C4 step -2 us)
            io.heightmaps = None
            self._io_ref = C.byref(io)
        io.scores = self._io_scores.ctypes.data if self.vfa.keep_scores else None
        return io

    def _step_fused(self, state_current, ref_feet_pos, hip_pos, ref_base, contact_sequence, base_lin_vel,
                    base_ori_euler_xyz):
        """step() through srbd_foothold_mpc_step; the Python objects it would have updated are updated the same
        way (the heightmaps' patches, VFA's footholds / constraints / scores, the interface's previous contact,
        the controller's warm start, key and last result)."""
        iface, ctrl, vfa = self.iface, self.iface.controller, self.vfa
        io = self._fused_io()
        a = self._io_np
        ctx = ctrl.context
        if _lib.fast is not None:  # the staging, the key split and the call in C (_srbd_fast)
            res = _lib.SrbdResult()
            r = _lib.fast.foothold_step(vfa.search.h.value, self.heightmaps.FL.terrain.h.value,
                                        C.addressof(vfa._params()), ctx.h.value, C.addressof(io), state_current,
                                        ref_base, ref_feet_pos, hip_pos, base_lin_vel, base_ori_euler_xyz,
                                        contact_sequence, ctrl.best_control_parameters, iface.previous_contact_mpc,
                                        ctrl.master_key, ctrl._calls, ctx._best, ctx._contact, C.addressof(res),
                                        ctrl.num_control_parameters_single_leg, _lib.RNG_CODES[ctrl.rng])
            if r is not None:
                rc, stage, current_contact, key, calls = r[:5]
                if stage >= 2:  # compute_control's with_newkey ran
                    ctrl.master_key = key
                    if ctrl.rng != "philox":
                        ctrl._calls = calls
                return self._fused_outputs(rc, res, current_contact, None if rc else r[5:], a["seeds"], ref_base)
        np.concatenate([state_current[k] for k in ("position", "linear_velocity", "orientation", "angular_velocity",
                                                   "foot_FL", "foot_FR", "foot_RL", "foot_RR")], out=a["state_in"])
        np.concatenate([ref_base[k] for k in ("ref_position", "ref_linear_velocity", "ref_orientation",
                                              "ref_angular_velocity")], out=a["ref_base"])
        seeds, hips = a["seeds"], a["hips"]
        seeds[0:3], seeds[3:6], seeds[6:9], seeds[9:12] = ref_feet_pos.FL, ref_feet_pos.FR, ref_feet_pos.RL, \
            ref_feet_pos.RR
        hips[0:3], hips[3:6], hips[6:9], hips[9:12] = hip_pos.FL, hip_pos.FR, hip_pos.RL, hip_pos.RR
        a["forward_vel"][:] = np.asarray(base_lin_vel, dtype=np.float64).reshape(-1)[:3]
        current_contact = np.array([contact_sequence[0][0], contact_sequence[1][0], contact_sequence[2][0],
                                    contact_sequence[3][0]])
        a["current_contact"][:] = current_contact
        a["previous_contact"][:] = iface.previous_contact_mpc
        io.yaw = float(base_ori_euler_xyz[2])
        H = ctx.cfg.horizon
        ctx._contact[...] = np.asarray(contact_sequence)[:, :H]
        ctx._best[...] = np.reshape(ctrl.best_control_parameters, ctx.P)
        key0 = (ctrl.master_key, ctrl._calls)
        ctrl = ctrl.with_newkey()
        seed, counter = ctrl._key_args(ctrl.master_key)
        res = _lib.SrbdResult()
        rc = _lib.lib.srbd_foothold_mpc_step(vfa.search.h, self.heightmaps.FL.terrain.h, C.byref(vfa._params()),
                                             ctx.h, self._io_ref, ctx._a_contact, H, ctx._a_best,
                                             ctrl.num_control_parameters_single_leg, seed, counter, C.byref(res))
        if io.stage < 2:  # compute_control's with_newkey had not run
            ctrl.master_key, ctrl._calls = key0
        return self._fused_outputs(rc, res, current_contact, None, seeds, ref_base)

    def _fused_outputs(self, rc, res, current_contact, made, seeds, ref_base):
        """The objects' state after srbd_foothold_mpc_step, as the Python chain leaves it -- also when a call of the
        chain failed (io.stage: the calls that completed), so an error leaves them as compute_adaptation /
        compute_control would -- and the step's 7-tuple.  made: the objects the C glue built for a completed step (GRF
        rows, predicted state, warm start, foothold rows, constraint boxes, patches, scores), or None."""
        iface, ctrl, vfa, io, a = self.iface, self.iface.controller, self.vfa, self._io, self._io_np
        ctx = ctrl.context
        if made is not None:  # rc == 0, every call completed
            grows, pred, best, frows, boxes, pending, scores = made
            maps = self.heightmaps
            maps.FL._data = maps.FR._data = maps.RL._data = maps.RR._data = None
            maps.FL.pending, maps.FR.pending, maps.RL.pending, maps.RR.pending = pending
            constraints = vfa.footholds_constraints
            for i, b in enumerate(boxes):
                if b is not None:
                    constraints[LEGS[i]] = b
            vfa.last_scores = scores
            footholds = LegsAttr(*frows)
            vfa.footholds_adaptation, vfa.initialized = footholds, True
            self._ref_state, self._ref_src = None, (ref_base, frows, LegsAttr(*constraints))
            self.last_constraints = constraints
            iface.previous_contact_mpc = current_contact
            ctrl.best_control_parameters = best
            ctx.step_id += 1
            ctrl.last_result = res
            return LegsAttr(*grows), LegsAttr(*frows), None, None, None, 1.4, pred
        if io.stage >= 1:  # (compute_adaptation's reset, then its results: initialized again)
            for i, m in enumerate(self.heightmaps):  # pending around the seeds (raycast on access)
                m._data, m.pending = None, (seeds[3 * i:3 * i + 3].copy(), io.yaw)
            fh = a["footholds"].reshape(4, 3).copy()
            f0, f1, f2, f3 = fh
            valid = io.valid
            constraints = vfa.footholds_constraints
            if valid[0] or valid[1] or valid[2] or valid[3]:
                boxes = a["boxes"].reshape(4, 2, 3).copy()  # one copy; each leg's box corners are views of it
                for i, b in enumerate(boxes):
                    if valid[i]:
                        constraints[LEGS[i]] = [b[0], b[1]]
            vfa.last_scores = self._io_scores.copy() if vfa.keep_scores else None
            vfa.footholds_adaptation, vfa.initialized = LegsAttr(f0, f1, f2, f3), True
            self._ref_state, self._ref_src = None, (ref_base, (f0, f1, f2, f3), LegsAttr(*constraints))
            self.last_constraints = constraints
        else:  # the patches stay pending around the seeds (update_height_map ran, the search did not)
            vfa.reset()
            for i, m in enumerate(self.heightmaps):
                m._data, m.pending = None, (seeds[3 * i:3 * i + 3].copy(), io.yaw)
        if io.stage >= 2:
            iface.previous_contact_mpc = current_contact
            ctrl.best_control_parameters = ctx._best.copy()
        if rc != _lib.OK:
            what = "srbd_tamols_run_terrain" if io.stage == 0 else "srbd_prepare_state" if io.stage == 1 else "srbd_step"
            msg = _lib.lib.srbd_tamols_last_error(vfa.search.h) if io.stage == 0 else _lib.last_error(ctx.h)
            raise RuntimeError(f"srbd_foothold_mpc_step: {what} failed ({rc}): "
                               f"{msg.decode() if isinstance(msg, bytes) else msg}")
        ctx.step_id += 1
        ctrl.last_result = res
        g = np.array(res.grf, dtype=np.float32).reshape(4, 3) * current_contact[:, None]  # as compute_control
        pred = np.array(res.predicted_state, dtype=np.float32)
        return LegsAttr(*g), LegsAttr(f0, f1, f2, f3), None, None, None, 1.4, pred

    def step(self, state_current: dict, ref_feet_pos: LegsAttr, hip_pos: LegsAttr, ref_base: dict,
             contact_sequence: np.ndarray, base_lin_vel: np.ndarray, base_ori_euler_xyz: np.ndarray,
             base_ang_vel: np.ndarray, pgg_phase_signal: np.ndarray, pgg_step_freq: float, optimize_swing: int = 0):
        """ref_base: ``ref_position``, ``ref_linear_velocity``, ``ref_orientation``, ``ref_angular_velocity``.
        Returns ``compute_control``'s 7-tuple; the ref_state it was given is kept in ``last_ref_state``."""
        cs = np.asarray(contact_sequence)
        if self._fusable() and cs.ndim == 2 and cs.shape[0] == 4 and cs.shape[1] >= self.controller.horizon:
            return self._step_fused(state_current, ref_feet_pos, hip_pos, ref_base, contact_sequence, base_lin_vel,
                                    base_ori_euler_xyz)
        feet = LegsAttr(*[np.asarray(state_current["foot_" + n], dtype=np.float64) for n in LEGS])
        current_contact = np.array([contact_sequence[i][0] for i in range(4)])
        seeds = LegsAttr(*[np.array(ref_feet_pos[n], dtype=np.float64) for n in LEGS])
        for n in LEGS:  # wb_interface.py:233-234
            self.heightmaps[n].update_height_map(seeds[n], yaw=base_ori_euler_xyz[2])
        self.vfa.reset()  # adapt on every call (the reference gates this on the swing apex)
        self.vfa.compute_adaptation(LEGS, seeds, hip_pos, self.heightmaps, base_lin_vel, base_ori_euler_xyz,
                                    base_ang_vel, base_position=state_current["position"],
                                    current_contact=current_contact, current_feet_pos=feet)
        adapted, constraints = self.vfa.get_footholds_adapted(seeds)
        ref_state = dict(ref_base)  # wb_interface.py:268-285
        for n in LEGS:
            ref_state["ref_foot_" + n] = np.asarray(adapted[n], dtype=np.float64).reshape((1, 3))
            ref_state["ref_foot_constraints_" + n] = constraints[n]
        self._ref_state, self._ref_src = ref_state, None
        self.last_constraints = constraints
        return self.iface.compute_control(state_current, ref_state, contact_sequence, self.cfg.inertia,
                                          pgg_phase_signal, pgg_step_freq, optimize_swing)

    def close(self):
        self.controller.close()
        if self.vfa._search is not None:
            self.vfa._search.close()
