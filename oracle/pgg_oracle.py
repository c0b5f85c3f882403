"""Scalar restatement of the reference's PeriodicGaitGenerator (TEST INFRASTRUCTURE ONLY).

Row a16 of SURVEY 8(a): the producer of the (4, H) contact_sequence the sampling MPC consumes.
Follows quadruped_pympc/helpers/periodic_gait_generator.py: phase offsets per gait (:22-40),
reset (:41-46), the per-leg loop of run() (:48-76), set_phase_signal (:78-88) and
compute_contact_sequence (:93-118), leg by leg in plain Python like the reference.
Only tests/ may import this module; the product's generator is C++ (srbd_pgg_* in
include/srbd_host.h, quadruped-pympc-tamols_amd/csrc/srbd_host.cpp) behind
quadruped_pympc_amd/helpers/periodic_gait_generator.py.
"""
import numpy as np

# GaitType values, quadruped_pympc/helpers/quadruped_utils.py:12-22
TROT, PACE, BOUNDING, CIRCULARCRAWL, BFDIAGONALCRAWL, BACKDIAGONALCRAWL, FRONTDIAGONALCRAWL, FULL_STANCE = range(8)


class PGGOracle:
    def __init__(self, duty_factor, step_freq, gait_type, horizon):
        self.duty_factor = duty_factor
        self.step_freq = step_freq
        self.horizon = horizon
        self.gait_type = gait_type
        self.reset()

    def reset(self):
        offsets = {TROT: [0.5, 1.0, 1.0, 0.5], PACE: [0.8, 0.3, 0.8, 0.3], BOUNDING: [0.5, 0.5, 0.0, 0.0],
                   CIRCULARCRAWL: [0.0, 0.25, 0.75, 0.5], BFDIAGONALCRAWL: [0.0, 0.25, 0.5, 0.75],
                   BACKDIAGONALCRAWL: [0.0, 0.5, 0.75, 0.25], FRONTDIAGONALCRAWL: [0.5, 1.0, 0.75, 1.25]}
        self.phase_offset = offsets.get(self.gait_type, [0.0, 0.5, 0.5, 0.0])
        self.phase = [float(v) for v in self.phase_offset]
        self.init = [False] * 4

    def run(self, dt, freq):
        contact = [0.0] * 4
        for leg in range(4):
            self.phase[leg] = (self.phase[leg] + dt * freq) % 1.0
            if self.init[leg]:
                contact[leg] = 1.0
                if not self.phase[leg] <= self.phase_offset[leg]:
                    self.init[leg] = False
                    self.phase[leg] = 0.0
            else:
                contact[leg] = 1.0 if self.phase[leg] < self.duty_factor else 0.0
        return contact

    def compute_contact_sequence(self, dts, lengths):
        if self.gait_type == FULL_STANCE:
            self.reset()
            return np.ones((4, 2 * self.horizon))
        saved_phase, saved_init = list(self.phase), list(self.init)
        seq = np.zeros((4, self.horizon))
        seq[:, 0] = self.run(0.0, self.step_freq)
        j = 0
        for i in range(1, self.horizon):
            if i >= lengths[j]:
                j += 1
            seq[:, i] = self.run(dts[j], self.step_freq)
        self.phase, self.init = saved_phase, saved_init
        return seq
