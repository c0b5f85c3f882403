"""MPC -> whole-body-controller shared-memory transport (single-writer seqlock).

Mirror of the real-robot wire format of ``ros2/run_controller.py`` (reference): 75 float64
(GRF 12, footholds 12, joint pos / vel / acc 12 each, predicted state 12, best step
frequency, MPC loop time, monotonic stamp; :50-83) guarded by a 64-bit sequence number
that is odd while the writer packs and even when stable (writer :343-358, reader :565-580).
Here the sequence word sits at the head of the same segment (8 bytes, then the payload),
so one shared-memory name connects the processes; publish / read run in
``libsrbd_hip.so`` (``srbd_shm_publish`` / ``srbd_shm_read``, include/srbd_host.h) with
atomic word copies, so a reader never returns a torn message.

The reference packs ``nmpc_joints_pos`` into the three joint slots whenever a predicted state
exists; the sampling controller returns ``None`` joints, which that assignment cannot store.
Missing joints are written as zeros here.
"""
from __future__ import annotations

import ctypes as C
import time
from multiprocessing import shared_memory

import numpy as np

from .. import _lib
from .legs_attr import LegsAttr

N_DBL = _lib.SHM_DOUBLES
IDX_GRF, IDX_FH, IDX_JP, IDX_JV, IDX_JA, IDX_PRED = (slice(0, 12), slice(12, 24), slice(24, 36), slice(36, 48),
                                                      slice(48, 60), slice(60, 72))
IDX_BSF, IDX_LAST, IDX_STAMP = 72, 73, 74
SEGMENT_BYTES = 8 + 8 * N_DBL


def legsattr_to12(legs) -> np.ndarray:
    if isinstance(legs, LegsAttr):
        return np.concatenate([np.asarray(legs.FL).reshape(-1), np.asarray(legs.FR).reshape(-1),
                               np.asarray(legs.RL).reshape(-1), np.asarray(legs.RR).reshape(-1)], axis=0)
    return np.asarray(legs, dtype=np.float64).reshape(-1)[:12]


def vec12_to_legsattr(vec12) -> LegsAttr:
    v = np.asarray(vec12).reshape(4, 3)
    return LegsAttr(FL=v[0].copy(), FR=v[1].copy(), RL=v[2].copy(), RR=v[3].copy())


def _fill(dst, src):
    a = np.zeros(12) if src is None else legsattr_to12(src)
    for i in range(12):
        dst[i] = float(a[i])


class _Segment:
    def __init__(self, name: str | None, create: bool):
        self.shm = shared_memory.SharedMemory(name=name, create=create, size=SEGMENT_BYTES if create else 0)
        if create:
            self.shm.buf[:SEGMENT_BYTES] = bytes(SEGMENT_BYTES)
        self._anchor = C.c_char.from_buffer(self.shm.buf)  # holds the buffer export while we use raw pointers
        base = C.addressof(self._anchor)
        self.seq_ptr = C.c_void_p(base)
        self.payload_ptr = C.c_void_p(base + 8)
        self.name = self.shm.name

    def close(self):
        self.seq_ptr = self.payload_ptr = None
        self._anchor = None
        self.shm.close()


class MpcShmWriter(_Segment):
    """The MPC process side: ``publish`` one result per MPC step."""

    def __init__(self, name: str | None = None, create: bool = True):
        super().__init__(name, create)
        self._msg = _lib.ShmMsg()

    def publish(self, grf, footholds, predicted_state, best_sample_freq, last_mpc_loop_time, joints_pos=None,
                joints_vel=None, joints_acc=None, stamp: float | None = None) -> None:
        m = self._msg
        _fill(m.grf, grf)
        _fill(m.footholds, footholds)
        _fill(m.joints_pos, joints_pos)
        _fill(m.joints_vel, joints_vel)
        _fill(m.joints_acc, joints_acc)
        pred = np.asarray(predicted_state, dtype=np.float64).reshape(-1)[:12]
        for i in range(12):
            m.pred[i] = float(pred[i])
        m.best_freq = float(best_sample_freq)
        m.loop_time = float(last_mpc_loop_time)
        m.stamp = float(time.monotonic() if stamp is None else stamp)
        _lib.check(_lib.lib.srbd_shm_publish(self.seq_ptr, self.payload_ptr, C.byref(m)), what="srbd_shm_publish")

    def unlink(self):
        self.shm.unlink()


class MpcShmReader(_Segment):
    """The WBC side: ``read`` returns the latest stable message, or None while the writer is active."""

    def __init__(self, name: str):
        super().__init__(name, create=False)
        self._msg = _lib.ShmMsg()
        self.seq = 0

    def read_raw(self) -> np.ndarray | None:
        seq = C.c_uint64(0)
        rc = _lib.lib.srbd_shm_read(self.seq_ptr, self.payload_ptr, C.byref(self._msg), C.byref(seq))
        if rc < 0:
            raise RuntimeError(f"srbd_shm_read failed ({rc})")
        if rc == 0:
            return None
        self.seq = int(seq.value)
        m = self._msg
        out = np.empty(N_DBL)
        out[IDX_GRF], out[IDX_FH] = m.grf, m.footholds
        out[IDX_JP], out[IDX_JV], out[IDX_JA] = m.joints_pos, m.joints_vel, m.joints_acc
        out[IDX_PRED] = m.pred
        out[IDX_BSF], out[IDX_LAST], out[IDX_STAMP] = m.best_freq, m.loop_time, m.stamp
        return out

    def read(self) -> dict | None:
        tmp = self.read_raw()
        if tmp is None:
            return None
        return {"nmpc_GRFs": vec12_to_legsattr(tmp[IDX_GRF]), "nmpc_footholds": vec12_to_legsattr(tmp[IDX_FH]),
                "nmpc_joints_pos": vec12_to_legsattr(tmp[IDX_JP]), "nmpc_joints_vel": vec12_to_legsattr(tmp[IDX_JV]),
                "nmpc_joints_acc": vec12_to_legsattr(tmp[IDX_JA]), "nmpc_predicted_state": tmp[IDX_PRED].copy(),
                "best_sample_freq": float(tmp[IDX_BSF]), "last_mpc_loop_time": float(tmp[IDX_LAST]),
                "last_mpc_update_mono": float(tmp[IDX_STAMP])}
