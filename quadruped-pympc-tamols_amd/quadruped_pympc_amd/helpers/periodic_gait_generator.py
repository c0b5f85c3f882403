"""Periodic gait generator: the producer of the (4, H) ``contact_sequence`` the sampling MPC consumes.

Behaviour of ``quadruped_pympc/helpers/periodic_gait_generator.py`` (reference):
phase offsets per gait (:22-46), the per-leg phase/duty-factor contact rule with
its start-up ``init`` hold (:48-76), and the look-ahead sequence
(:93-118, full stance returns 2H ones).  Vectorised over the four legs.
"""
from __future__ import annotations

import numpy as np

TROT, PACE, BOUNDING, CIRCULARCRAWL, BFDIAGONALCRAWL, BACKDIAGONALCRAWL, FRONTDIAGONALCRAWL, FULL_STANCE = range(8)

PHASE_OFFSETS = {
    TROT: (0.5, 1.0, 1.0, 0.5),
    PACE: (0.8, 0.3, 0.8, 0.3),
    BOUNDING: (0.5, 0.5, 0.0, 0.0),
    CIRCULARCRAWL: (0.0, 0.25, 0.75, 0.5),
    BFDIAGONALCRAWL: (0.0, 0.25, 0.5, 0.75),
    BACKDIAGONALCRAWL: (0.0, 0.5, 0.75, 0.25),
    FRONTDIAGONALCRAWL: (0.5, 1.0, 0.75, 1.25),
}


class PeriodicGaitGenerator:
    def __init__(self, duty_factor, step_freq, gait_type, horizon):
        self.duty_factor = duty_factor
        self.step_freq = step_freq
        self.horizon = horizon
        self.gait_type = int(getattr(gait_type, "value", gait_type))
        self.previous_gait_type = self.gait_type
        self.reset()

    def reset(self):
        self.phase_offset = list(PHASE_OFFSETS.get(self.gait_type, (0.0, 0.5, 0.5, 0.0)))
        self._phase_signal = np.asarray(self.phase_offset, dtype=np.float64).copy()
        self._init = np.zeros(4, dtype=bool)
        self.n_contact = 4
        self.time_before_switch_freq = 0

    def run(self, dt, new_step_freq):
        ph = (self._phase_signal + dt * new_step_freq) % 1.0
        off = np.asarray(self.phase_offset)
        holding = self._init & (ph <= off)
        releasing = self._init & ~(ph <= off)
        contact = np.where(self._init, 1.0, (ph < self.duty_factor).astype(np.float64))
        ph = np.where(releasing, 0.0, ph)
        self._init = holding
        self._phase_signal = ph
        return contact

    def set_phase_signal(self, phase_signal, init=None):
        assert len(phase_signal) == 4
        self._phase_signal = np.asarray(phase_signal, dtype=np.float64).copy()
        self._init = np.zeros(4, dtype=bool) if init is None else np.asarray(init, dtype=bool).copy()

    @property
    def phase_signal(self):
        return np.array(self._phase_signal)

    def compute_contact_sequence(self, contact_sequence_dts, contact_sequence_lenghts):
        if self.gait_type == FULL_STANCE:
            self.reset()
            return np.ones((4, self.horizon * 2))
        t0, i0 = self._phase_signal.copy(), self._init.copy()
        seq = np.zeros((4, self.horizon))
        seq[:, 0] = self.run(0.0, self.step_freq)
        j = 0
        for i in range(1, self.horizon):
            if i >= contact_sequence_lenghts[j]:
                j += 1
            seq[:, i] = self.run(contact_sequence_dts[j], self.step_freq)
        self.set_phase_signal(t0, i0)
        return seq

    def set_full_stance(self):
        self.gait_type = FULL_STANCE
        self.reset()

    def restore_previous_gait(self):
        self.gait_type = self.previous_gait_type
        self.reset()
