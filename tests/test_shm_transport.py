"""CPU tests of the MPC -> WBC shared-memory seqlock (include/srbd_host.h srbd_shm_*,
helpers/mpc_shm.py), the wire format of ros2/run_controller.py:50-83 / :343-358 / :565-580."""
import ctypes as C
import multiprocessing as mp

import numpy as np
import pytest

from quadruped_pympc_amd import _lib
from quadruped_pympc_amd.helpers.legs_attr import LegsAttr
from quadruped_pympc_amd.helpers.mpc_shm import (IDX_BSF, IDX_FH, IDX_GRF, IDX_JP, IDX_LAST, IDX_PRED, IDX_STAMP,
                                                 N_DBL, MpcShmReader, MpcShmWriter)


def test_layout_constants_match_reference():
    assert N_DBL == 75 and (IDX_BSF, IDX_LAST, IDX_STAMP) == (72, 73, 74)
    assert C.sizeof(_lib.ShmMsg) == 8 * 75


def test_roundtrip_and_sequence():
    w = MpcShmWriter()
    r = MpcShmReader(w.name)
    try:
        assert r.read_raw() is not None and r.seq == 0  # zero-initialised, stable
        grf = LegsAttr(FL=np.array([1.0, 2, 3]), FR=np.array([4.0, 5, 6]), RL=np.array([7.0, 8, 9]),
                       RR=np.array([10.0, 11, 12]))
        fh = np.arange(12) * 0.5
        pred = np.arange(24) + 100.0
        w.publish(grf, fh, pred, 1.4, 0.003, stamp=42.0)
        msg = r.read()
        assert r.seq == 2
        np.testing.assert_array_equal(msg["nmpc_GRFs"].FR, [4, 5, 6])
        np.testing.assert_array_equal(np.concatenate([msg["nmpc_footholds"].FL, msg["nmpc_footholds"].RR[-1:]]),
                                      [0, 0.5, 1.0, 5.5])
        np.testing.assert_array_equal(msg["nmpc_predicted_state"], pred[:12])
        np.testing.assert_array_equal(msg["nmpc_joints_pos"].FL, [0, 0, 0])  # sampling MPC: no joints -> zeros
        assert (msg["best_sample_freq"], msg["last_mpc_loop_time"], msg["last_mpc_update_mono"]) == (1.4, 0.003, 42.0)
        w.publish(np.ones(12), np.ones(12), np.ones(12), 2.0, 0.0, joints_pos=np.full(12, 3.0))
        raw = r.read_raw()
        assert r.seq == 4 and raw[IDX_GRF].sum() == 12 and raw[IDX_JP].sum() == 36 and raw[IDX_BSF] == 2.0
    finally:
        r.close()
        w.close()
        w.unlink()


def test_writer_in_progress_is_not_read():
    w = MpcShmWriter()
    r = MpcShmReader(w.name)
    try:
        w.publish(np.ones(12), np.zeros(12), np.zeros(12), 1.0, 0.0)
        seq = C.c_uint64.from_address(w.seq_ptr.value)
        seq.value = 3  # odd: a writer is packing
        assert r.read_raw() is None
        w.publish(np.full(12, 2.0), np.zeros(12), np.zeros(12), 1.0, 0.0)  # (3 | 1) + 1
        assert seq.value == 4 and r.read_raw()[IDX_FH].sum() == 0 and r.seq == 4
        del seq
    finally:
        r.close()
        w.close()
        w.unlink()


def _writer(name, n):
    w = MpcShmWriter(name, create=False)
    for k in range(1, n + 1):
        v = np.full(12, float(k))
        w.publish(v, v, v, float(k), float(k), joints_pos=v, joints_vel=v, joints_acc=v, stamp=float(k))
    w.close()


def test_concurrent_reader_never_sees_a_torn_message():
    """One writer process publishes messages whose 75 words all equal k; the reader must only ever
    return whole messages, in non-decreasing k."""
    w = MpcShmWriter()
    r = MpcShmReader(w.name)
    n = 20000
    p = mp.get_context("fork").Process(target=_writer, args=(w.name, n))
    try:
        p.start()
        last, ok, busy = 0.0, 0, 0
        while True:
            raw = r.read_raw()
            alive = p.is_alive()
            if raw is None:
                busy += 1
            else:
                k = raw[0]
                assert np.all(raw == k), raw
                assert k >= last
                last, ok = k, ok + 1
            if not alive and raw is not None and last == n:
                break
            if not alive and raw is not None and r.seq == 2 * n:
                break
        p.join(timeout=30)
        assert p.exitcode == 0
        assert last == n and r.seq == 2 * n and ok > 10
    finally:
        if p.is_alive():
            p.kill()
        r.close()
        w.close()
        w.unlink()


def test_bad_arguments():
    m = _lib.ShmMsg()
    assert _lib.lib.srbd_shm_publish(None, None, C.byref(m)) == _lib.E_INVALID
    assert _lib.lib.srbd_shm_read(None, None, C.byref(m), None) == _lib.E_INVALID
