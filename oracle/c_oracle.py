"""ctypes wrapper of oracle/libsrbd_oracle.so (TEST INFRASTRUCTURE ONLY; see srbd_oracle.c)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libsrbd_oracle.so")
MAXH = 64


class OracleCfg(C.Structure):
    _fields_ = [("N", C.c_int32), ("H", C.c_int32), ("method", C.c_int32), ("param_kind", C.c_int32),
                ("num_splines", C.c_int32), ("_pad", C.c_int32), ("mass", C.c_float), ("mg", C.c_float),
                ("grf_min", C.c_float), ("grf_max", C.c_float), ("mu", C.c_float), ("inertia", C.c_float * 9),
                ("dts", C.c_float * MAXH), ("sigma_mppi", C.c_float), ("sigma_rs", C.c_float * 3)]


def _load():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", HERE, "libsrbd_oracle.so"], check=True)
    lib = C.CDLL(LIB)
    FP = C.POINTER(C.c_float)
    lib.srbd_oracle_rollout_costs.argtypes = [C.POINTER(OracleCfg), FP, FP, FP, C.c_int, FP, FP, C.c_int, FP, C.c_int]
    lib.srbd_oracle_final.argtypes = [C.POINTER(OracleCfg), FP, FP, C.c_int, FP, FP, FP]
    lib.srbd_oracle_philox.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    lib.srbd_oracle_gen_noise.argtypes = [C.POINTER(OracleCfg), C.c_uint64, C.c_uint64, FP, FP]
    lib.srbd_oracle_step.argtypes = [C.POINTER(OracleCfg), FP, FP, FP, C.c_int, FP, FP, C.c_int, C.c_uint64,
                                     C.c_uint64, FP, FP, FP, FP, FP, C.POINTER(C.c_int32), C.c_int]
    return lib


lib = _load()


def _fp(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_float))


def make_cfg(*, N, H, method, param_kind, num_splines=2, mass, inertia, dt=0.02, dts=None, mu=0.5, grf_min=0.0,
             grf_max=None, sigma_mppi=3.0, sigma_rs=(0.2, 3.0, 10.0)):
    c = OracleCfg()
    c.N, c.H, c.method, c.param_kind, c.num_splines = N, H, method, param_kind, num_splines
    c.mass = float(np.float32(mass))
    c.mg = float(np.float32(mass * 9.81))
    c.grf_min = float(np.float32(grf_min))
    c.grf_max = float(np.float32(grf_max if grf_max is not None else mass * 9.81))
    c.mu = float(np.float32(mu))
    for i, v in enumerate(np.asarray(inertia, dtype=np.float32).reshape(9)):
        c.inertia[i] = float(v)
    d = np.full(H, dt, np.float32) if dts is None else np.asarray(dts, np.float32)
    for i in range(H):
        c.dts[i] = float(d[i])
    c.sigma_mppi = float(np.float32(sigma_mppi))
    for i in range(3):
        c.sigma_rs[i] = float(np.float32(sigma_rs[i]))
    return c


def num_params(c):
    if c.param_kind == 1:
        return 12 * (c.num_splines + 1)
    if c.param_kind == 2:
        return 48 * c.num_splines
    return 12 * c.H


def rollout_costs(c, state, ref, contact, best, noise, nthreads=0):
    state = np.ascontiguousarray(state, np.float32)
    ref = np.ascontiguousarray(ref, np.float32)
    contact = np.ascontiguousarray(contact, np.float32)
    best = np.ascontiguousarray(best, np.float32)
    noise = np.ascontiguousarray(noise, np.float32)
    costs = np.empty(noise.shape[0], np.float32)
    rc = lib.srbd_oracle_rollout_costs(C.byref(c), _fp(state), _fp(ref), _fp(contact), contact.shape[1], _fp(best),
                                       _fp(noise), noise.shape[0], _fp(costs), nthreads)
    assert rc == 0
    return costs


def philox(ctr, key):
    ci = (C.c_uint32 * 4)(*ctr)
    ki = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib.srbd_oracle_philox(ci, ki, o)
    return list(o)


def gen_noise(c, seed, counter, sigma=None):
    P = num_params(c)
    out = np.empty((c.N, P), np.float32)
    s = None if sigma is None else np.ascontiguousarray(np.broadcast_to(sigma, (P,)), np.float32)
    lib.srbd_oracle_gen_noise(C.byref(c), C.c_uint64(seed), C.c_uint64(counter), _fp(s), _fp(out))
    return out


def step(c, state, ref, contact, best, sigma=None, noise=None, seed=42, counter=0, nthreads=0):
    """Full CPU step; returns (best, sigma, grf, pred, best_cost, best_idx, costs)."""
    P = num_params(c)
    state = np.ascontiguousarray(state, np.float32)
    ref = np.ascontiguousarray(ref, np.float32)
    contact = np.ascontiguousarray(contact, np.float32)
    best = np.array(best, np.float32)
    sig = None if sigma is None else np.array(np.broadcast_to(sigma, (P,)), np.float32)
    gen = 1 if noise is None else 0
    nz = np.empty((c.N, P), np.float32) if noise is None else np.ascontiguousarray(noise, np.float32)
    costs = np.empty(c.N, np.float32)
    grf = np.empty(12, np.float32)
    pred = np.empty(24, np.float32)
    bc = np.empty(1, np.float32)
    bi = C.c_int32(0)
    rc = lib.srbd_oracle_step(C.byref(c), _fp(state), _fp(ref), _fp(contact), contact.shape[1], _fp(best), _fp(sig),
                              gen, C.c_uint64(seed), C.c_uint64(counter), _fp(nz), _fp(costs), _fp(grf), _fp(pred),
                              _fp(bc), C.byref(bi), nthreads)
    assert rc == 0
    return best, sig, grf, pred, float(bc[0]), int(bi.value), costs
