"""Periodic gait generator: the producer of the (4, H) ``contact_sequence`` the sampling MPC consumes.

Mirror of ``quadruped_pympc/helpers/periodic_gait_generator.py`` (reference): the same
constructor, attributes and methods (phase offsets per gait :22-46, ``run`` :48-76,
``set_phase_signal`` :78-87, ``compute_contact_sequence`` :93-118, full stance -> 2H ones).
The state lives in a ``srbd_pgg`` struct and every method runs in ``libsrbd_hip.so``'s C++
host producers (``include/srbd_host.h``), so the 100 Hz loop pays one
ctypes call per sequence instead of H NumPy passes.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .. import _lib

TROT, PACE, BOUNDING, CIRCULARCRAWL, BFDIAGONALCRAWL, BACKDIAGONALCRAWL, FRONTDIAGONALCRAWL, FULL_STANCE = range(8)


def _check(rc, what):
    if rc < 0:
        raise ValueError(f"{what} failed ({rc})")
    return rc


def _check_lengths(lens, n_dts, horizon, gait_type):
    """Raise IndexError where the reference's loop (PGG:111-115) would read contact_sequence_lenghts past its end
    (the library reads lens[j] for j < n_dts only, so a shorter lengths array is walked here first)."""
    if len(lens) >= n_dts or gait_type == FULL_STANCE:
        return
    j = 0
    for i in range(1, horizon):
        if j >= len(lens):
            raise IndexError("compute_contact_sequence: contact_sequence_lenghts too short")
        if i >= lens[j]:
            j += 1
        if j >= n_dts:
            return  # dts[j] past the end: the library reports it


class PeriodicGaitGenerator:
    def __init__(self, duty_factor, step_freq, gait_type, horizon):
        self._g = _lib.SrbdPgg()
        self._gp = C.byref(self._g)
        _check(_lib.lib.srbd_pgg_init(self._gp, int(getattr(gait_type, "value", gait_type)), float(duty_factor),
                                      float(step_freq), int(horizon)), "srbd_pgg_init")
        self.start_and_stop_activated = False
        self.time_before_switch_freq = 0
        self._seq_key = None  # (dts, lens) bytes of the cached sequence-call arguments
        self._out = np.empty(8 * _lib.MAX_HORIZON)
        self._out_p = _lib.dptr(self._out)
        self._addr = C.addressof(self._g)

    # plain attributes of the reference, backed by the C struct
    duty_factor = property(lambda s: s._g.duty_factor, lambda s, v: setattr(s._g, "duty_factor", float(v)))
    step_freq = property(lambda s: s._g.step_freq, lambda s, v: setattr(s._g, "step_freq", float(v)))
    horizon = property(lambda s: s._g.horizon, lambda s, v: setattr(s._g, "horizon", int(v)))
    gait_type = property(lambda s: s._g.gait_type, lambda s, v: setattr(s._g, "gait_type", int(getattr(v, "value", v))))
    previous_gait_type = property(lambda s: s._g.previous_gait_type,
                                  lambda s, v: setattr(s._g, "previous_gait_type", int(getattr(v, "value", v))))
    n_contact = 4

    @property
    def phase_offset(self):
        return list(self._g.phase_offset)

    @property
    def _init(self):
        return np.array(self._g.init, dtype=bool)

    def reset(self):
        _lib.lib.srbd_pgg_reset(self._gp)
        self.time_before_switch_freq = 0

    def run(self, dt, new_step_freq):
        out = np.zeros(4)
        _lib.lib.srbd_pgg_run(self._gp, float(dt), float(new_step_freq), _lib.dptr(out))
        return out

    def set_phase_signal(self, phase_signal, init=None):
        assert len(phase_signal) == 4
        ph = np.ascontiguousarray(phase_signal, dtype=np.float64)
        ini = None if init is None else np.ascontiguousarray(init, dtype=np.int32)
        _lib.lib.srbd_pgg_set_phase_signal(self._gp, _lib.dptr(ph), _lib.iptr(ini))

    @property
    def phase_signal(self):
        return np.array(self._g.phase_signal)

    def compute_contact_sequence(self, contact_sequence_dts, contact_sequence_lenghts):
        if _lib.fast is not None:  # the same C call, its arguments and result array handled in C (_srbd_fast)
            return _lib.fast.pgg_contact_sequence(self._addr, contact_sequence_dts, contact_sequence_lenghts)
        key = (np.asarray(contact_sequence_dts, dtype=np.float64).tobytes(),
               np.asarray(contact_sequence_lenghts, dtype=np.int32).tobytes())
        _check_lengths(np.frombuffer(key[1], dtype=np.int32), len(key[0]) // 8, self._g.horizon, self._g.gait_type)
        if key != self._seq_key:  # the 100 Hz caller passes the same arrays every step
            self._dts = np.frombuffer(key[0], dtype=np.float64).copy()
            self._lens = np.frombuffer(key[1], dtype=np.int32).copy()
            self._dts_p, self._lens_p = _lib.dptr(self._dts), _lib.iptr(self._lens)
            self._seq_key = key
        H = self._g.horizon
        cols = _check(_lib.lib.srbd_pgg_contact_sequence(self._gp, self._dts_p, self._lens_p, len(self._dts),
                                                         self._out_p, min(self._out.size, 8 * H)),
                      "compute_contact_sequence")
        return self._out[:4 * cols].reshape(4, cols).copy()  # row-major 4 x cols

    def set_full_stance(self):
        self.gait_type = FULL_STANCE
        self.reset()

    def restore_previous_gait(self):
        self.gait_type = self.previous_gait_type
        self.reset()
