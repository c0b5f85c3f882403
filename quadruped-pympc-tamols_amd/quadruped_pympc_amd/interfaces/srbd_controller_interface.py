"""``SRBDControllerInterface`` for the MI355X sampling MPC.

Mirror of ``quadruped_pympc/interfaces/srbd_controller_interface.py`` (:7-240),
``type == 'sampling'`` branch (:118-180, :225-240): the same per-call sequence
(prepare_state_and_reference -> per sampling iteration: with_newkey [+ sigma reset
for CEM] -> jitted_compute_control -> reassign best_control_parameters) and the same
7-tuple return.  Gradient (acados) controllers are out of scope and raise.
"""
from __future__ import annotations

import numpy as np

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

    def compute_control(self, state_current: dict, ref_state: dict, contact_sequence: np.ndarray, inertia: np.ndarray,
                        pgg_phase_signal: np.ndarray, pgg_step_freq: float, optimize_swing: int,
                        external_wrenches: np.ndarray = np.zeros((6,))):
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
