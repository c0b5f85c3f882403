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

import numpy as np

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
        self.last_ref_state = None
        self.last_constraints = None

    @property
    def controller(self):
        return self.iface.controller

    def step(self, state_current: dict, ref_feet_pos: LegsAttr, hip_pos: LegsAttr, ref_base: dict,
             contact_sequence: np.ndarray, base_lin_vel: np.ndarray, base_ori_euler_xyz: np.ndarray,
             base_ang_vel: np.ndarray, pgg_phase_signal: np.ndarray, pgg_step_freq: float, optimize_swing: int = 0):
        """ref_base: ``ref_position``, ``ref_linear_velocity``, ``ref_orientation``, ``ref_angular_velocity``.
        Returns ``compute_control``'s 7-tuple; the ref_state it was given is kept in ``last_ref_state``."""
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
        self.last_ref_state = ref_state
        self.last_constraints = constraints
        return self.iface.compute_control(state_current, ref_state, contact_sequence, self.cfg.inertia,
                                          pgg_phase_signal, pgg_step_freq, optimize_swing)

    def close(self):
        self.controller.close()
        if self.vfa._search is not None:
            self.vfa._search.close()
