"""MI355X gait-adaptive sampling MPC with the reference's interface.

Drop-in for ``quadruped_pympc/controllers/sampling/centroidal_nmpc_jax_gait_adaptive.py``
(``Sampling_MPC``, :22-1134), which ``SRBDControllerInterface`` selects when
``mpc_params['optimize_step_freq']`` is set (srbd_controller_interface.py:77-81).  Same
constructor, attributes and methods as the base class (``centroidal_nmpc_hip.Sampling_MPC``);
the compute calls take ``(..., key, timing, nominal_step_frequency, optimize_swing)`` and return
``best_step_frequency`` in place of the base file's constant (GA:705, :861).

Per compute call the host forms the candidate set ``jax.random.choice`` draws from (GA:687-692
random sampling, :834-838 MPPI) and hands it with the leg phases (``timing``) to
``srbd_set_gait``; every sample then draws its step frequency on the device and rolls out with
its own contact sequence from the JAX periodic gait generator (see include/srbd_mpc.h).  There is
no CPU path.  ``step_frequencies=`` injects the per-sample frequencies exactly (with ``noise=``,
the parity mode).

CEM: the reference's gait-adaptive CEM cannot be called through its own interface (6 positional
arguments passed where 9 are required, and 7 values returned where 8 are unpacked; SURVEY App. B
#2), so it is not provided: ``compute_control_cem_mppi`` raises ``NotImplementedError``.
"""
from __future__ import annotations

import numpy as np

from .centroidal_nmpc_hip import Sampling_MPC as _BaseSamplingMPC

f32 = np.float32

PGG_DUTY_FACTOR = 0.65  # GA:179 PeriodicGaitGeneratorJax(duty_factor=0.65, step_freq=1.65, mpc_dt=self.dt)


class Sampling_MPC(_BaseSamplingMPC):
    """Sampling MPC that also samples the step frequency (MI355X HIP backend)."""

    def __init__(self, config_module=None):
        super().__init__(config_module)
        self.step_freq_delta = np.asarray(self._cfg.mpc_params["step_freq_available"], dtype=f32)  # GA:182
        if self.step_freq_delta.shape[0] > 8:
            raise ValueError("step_freq_available: at most 8 candidates (SRBD_MAX_FREQS)")

    def _freq_set(self, nominal_step_frequency, optimize_swing):
        """The array jax.random.choice draws from, float32 (x64 off)."""
        if self.sampling_method == "random_sampling":  # GA:688
            return np.where(bool(optimize_swing), self.step_freq_delta, f32(nominal_step_frequency)).astype(f32)
        return self.step_freq_delta  # MPPI, GA:835

    def _run_ga(self, state, reference, contact_sequence, best_control_parameters, key, timing,
                nominal_step_frequency, optimize_swing, noise, step_frequencies):
        fs = self._freq_set(nominal_step_frequency, optimize_swing)
        self.context.set_gait(np.asarray(timing, dtype=f32), self.dt, PGG_DUTY_FACTOR, fs, step_frequencies)
        grf, fh, pred, best, cost, _, costs, _ = self._run(state, reference, contact_sequence,
                                                           best_control_parameters, key, None, noise)
        return grf, fh, pred, best, cost, f32(self.last_result.best_freq), costs

    def compute_control_random_sampling(self, state, reference, contact_sequence, best_control_parameters, key,
                                        timing, nominal_step_frequency, optimize_swing, *, noise=None,
                                        step_frequencies=None):
        """centroidal_nmpc_jax_gait_adaptive.py:630-806."""
        return self._run_ga(state, reference, contact_sequence, best_control_parameters, key, timing,
                            nominal_step_frequency, optimize_swing, noise, step_frequencies)

    def compute_control_mppi(self, state, reference, contact_sequence, best_control_parameters, key, timing,
                             nominal_step_frequency, optimize_swing, *, noise=None, step_frequencies=None):
        """centroidal_nmpc_jax_gait_adaptive.py:808-962."""
        return self._run_ga(state, reference, contact_sequence, best_control_parameters, key, timing,
                            nominal_step_frequency, optimize_swing, noise, step_frequencies)

    def compute_control_cem_mppi(self, *args, **kwargs):
        """centroidal_nmpc_jax_gait_adaptive.py:964-1131 -- not provided (module docstring)."""
        raise NotImplementedError(
            "gait-adaptive CEM-MPPI: the reference's branch is broken as wired (SURVEY App. B #2); "
            "use sampling_method 'mppi' or 'random_sampling' with optimize_step_freq")
