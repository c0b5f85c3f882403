"""MI355X sampling MPC with the reference's ``Sampling_MPC`` interface.

Drop-in for ``quadruped_pympc/controllers/sampling/centroidal_nmpc_jax.py``
(``Sampling_MPC``, :20-1097): same constructor (reads ``config.mpc_params``),
attributes (``num_sampling_iterations``, ``sampling_method``,
``best_control_parameters``, ``master_key``, ``sigma_cem_mppi`` ...), methods
(``prepare_state_and_reference``, ``with_newkey``, ``with_newsigma``,
``shift_solution``, ``reset``) and ``jitted_compute_control`` call shapes and
return tuples, so ``SRBDControllerInterface.compute_control``
(srbd_controller_interface.py:113-180) drives it unchanged.

Every compute call goes through ``libsrbd_hip.so`` (hand-written CDNA4 kernels):
device RNG, fused rollout + cost + block softmax partials, and one merge kernel
that produces the GRFs, the predicted state and the updated parameters.  The
HIP context is created on the first compute call (so construction is fork- and
thread-safe, like the reference's lazy XLA compile); there is no CPU fallback.

Noise streams (``mpc_params['rng']``, not a reference key):

* ``'jax'`` (default): the reference's own ``jax.random`` stream, drawn on the device
  (``include/srbd_mpc.h`` ``srbd_set_rng``).  ``master_key`` is ``jax.random.PRNGKey(42)``
  as ``np.uint32[2]`` and ``with_newkey`` is ``split(master_key)[0]``, as in the
  reference (centroidal_nmpc_jax.py:167, :498-501), so the same key gives the same
  noise.  ``mpc_params['jax_threefry_partitionable']`` (default True, JAX >= 0.5)
  selects the counter layout of older JAX releases when False.
* ``'philox'``: this library's Philox4x32-10 stream; ``master_key`` is
  ``np.uint64[2] = (seed, counter)`` and ``with_newkey`` advances the counter.

Pass ``noise=`` (the (N, P) ``additional_random_parameters``) to any compute call to
inject the sampled perturbations exactly.  ``costs`` (unused by every reference
caller) is returned as a lazy array that copies from the device on first access.
"""
from __future__ import annotations

import copy
import ctypes as C
import sys
import warnings

import numpy as np

from ... import _lib
from ...runtime import active_config, resolve_device_id

f32 = np.float32


class LazyCosts:
    """Saturated per-sample costs of one step, fetched from the device on first use."""

    def __init__(self, ctx: "_lib.Context", step_id: int):
        self._ctx, self._step_id, self._data = ctx, step_id, None

    def _get(self) -> np.ndarray:
        if self._data is None:
            if self._ctx.step_id != self._step_id:
                raise RuntimeError("costs of an older step: materialise them before the next compute call")
            self._data = self._ctx.copy_costs()
        return self._data

    def __array__(self, dtype=None, copy=None):
        a = self._get()
        return a if dtype is None else a.astype(dtype)

    def __len__(self):
        return self._ctx.n_local

    def __getitem__(self, i):
        return self._get()[i]

    @property
    def shape(self):
        return (self._ctx.n_local,)


_STATE_KEYS = ("position", "linear_velocity", "orientation", "angular_velocity",
               "foot_FL", "foot_FR", "foot_RL", "foot_RR")
_REF_KEYS = ("ref_position", "ref_linear_velocity", "ref_orientation", "ref_angular_velocity")
_REF_FEET = ("ref_foot_FL", "ref_foot_FR", "ref_foot_RL", "ref_foot_RR")


def _store(dst: np.ndarray, src) -> None:
    """dst[...] = src flattened to dst's size (a plain slice store when the shapes already match)."""
    if getattr(src, "shape", None) == dst.shape:
        dst[:] = src
    else:
        dst[...] = np.reshape(src, dst.shape)


class _PrepBufs:
    """srbd_prepare_state staging: state_in | ref_in | cur | prev (f64), best (f32), state | ref out (f64)."""

    def __init__(self, num_params: int):
        self.f64 = np.zeros(24 + 24 + 4 + 4, np.float64)
        self.state_in, self.ref_in = self.f64[0:24], self.f64[24:48]
        self.cur, self.prev = self.f64[48:52], self.f64[52:56]
        self.best = np.zeros(num_params, f32)
        self.out = np.zeros((2, 24), np.float64)
        a, o = self.f64.ctypes.data, self.out.ctypes.data
        self.addr = tuple(C.cast(a + 8 * k, _lib._DP) for k in (0, 24, 48, 52))
        self.a_best = self.best.ctypes.data_as(_lib._FP)
        self.addr_out = (C.cast(o, _lib._DP), C.cast(o + 24 * 8, _lib._DP))


class Sampling_MPC:
    """This is a small class that implements a sampling based control law (MI355X HIP backend)."""

    def __init__(self, config_module=None):
        cfg = active_config(config_module)  # the reference's quadruped_pympc.config when installed
        mp = cfg.mpc_params
        self._cfg = cfg
        device = mp["device"]
        self.num_parallel_computations = mp["num_parallel_computations"]
        self.sampling_method = mp["sampling_method"]
        self.control_parametrization = mp["control_parametrization"]
        self.num_sampling_iterations = mp["num_sampling_iterations"]
        self.dt = mp["dt"]
        self.horizon = mp["horizon"]
        self.state_dim = 24
        self.control_dim = 24
        self.reference_dim = self.state_dim
        self.max_sampling_forces_x = 10
        self.max_sampling_forces_y = 10
        self.max_sampling_forces_z = 30
        if device != "gpu":
            raise RuntimeError("Sampling_MPC (HIP) runs on the GPU only; mpc_params['device'] must be 'gpu'")
        # ordinal or 'auto' (default): replica process i -> GPU i mod G, resolved at context creation
        self.device_id = mp.get("device_id", "auto")

        # centroidal_nmpc_jax.py:52-93
        if self.control_parametrization == "linear_spline":
            self.num_spline = mp["num_splines"]
            self.num_control_parameters_single_leg = (self.num_spline + 1) * 3
        elif self.control_parametrization == "cubic_spline":
            self.num_spline = mp["num_splines"]
            self.num_control_parameters_single_leg = 4 * 3 * self.num_spline
        else:
            self.num_spline = mp.get("num_splines", 2)
            self.num_control_parameters_single_leg = self.horizon * 3
        self.num_control_parameters = self.num_control_parameters_single_leg * 4

        # centroidal_nmpc_jax.py:96-110
        if self.sampling_method == "random_sampling":
            self.compute_control = self.compute_control_random_sampling
            self.sigma_random_sampling = mp["sigma_random_sampling"]
        elif self.sampling_method == "mppi":
            self.compute_control = self.compute_control_mppi
            self.sigma_mppi = mp["sigma_mppi"]
        elif self.sampling_method == "cem_mppi":
            self.compute_control = self.compute_control_cem_mppi
            self.sigma_cem_mppi = np.ones(self.num_control_parameters, dtype=f32) * mp["sigma_cem_mppi"]
        else:
            print("Error: sampling method not recognized")
            sys.exit(1)
        self.jitted_compute_control = self.compute_control

        # model constants (centroidal_model_jax.py:37-56)
        self.mass = cfg.mass
        self.inertia = np.asarray(cfg.inertia, dtype=f32)
        if mp["use_nonuniform_discretization"]:
            hf = mp["horizon_fine_grained"]
            self.dts = np.concatenate([np.full(hf, mp["dt_fine_grained"], dtype=f32),
                                       np.full(self.horizon - hf, self.dt, dtype=f32)])
        else:
            self.dts = np.full(self.horizon, self.dt, dtype=f32)

        # centroidal_nmpc_jax.py:118-130
        self.Q = np.zeros(self.state_dim, dtype=f32)
        self.Q[2] = 1500
        self.Q[3:6] = 200
        self.Q[6:8] = 500
        self.Q[9:11] = 20
        self.Q[11] = 50
        self.mu = mp["mu"]
        self.f_z_max = mp["grf_max"]
        self.f_z_min = mp["grf_min"]

        self.best_control_parameters = np.zeros((self.num_control_parameters,), dtype=f32)
        rng = mp.get("rng", "jax")
        if rng == "jax" and not mp.get("jax_threefry_partitionable", True):
            rng = "jax_legacy"
        if rng not in _lib.RNG_CODES:
            raise ValueError(f"mpc_params['rng'] must be one of {sorted(_lib.RNG_CODES)}")
        self.rng = rng
        if rng == "philox":
            self.master_key = np.array([42, 0], dtype=np.uint64)
        else:
            self.master_key = _lib.jax_prng_key(42)  # jax.random.PRNGKey(42), centroidal_nmpc_jax.py:167
        self._calls = 0  # numbers the device steps (the draws made ahead are keyed by the next key and call)
        self._ctx = None

    # ------------------------------------------------------------------ copies
    # host staging whose raw addresses are cached (with_newkey's key buffer, prepare_state's arguments) and the
    # device context: a copy (copy.deepcopy, pickle) makes its own on first use instead of sharing the original's
    _TRANSIENT = ("_ctx", "_split_buf", "_split_addr", "_ps")

    def __getstate__(self):
        d = {k: v for k, v in self.__dict__.items() if k not in self._TRANSIENT}
        d["_ctx"] = None
        return d

    def __setstate__(self, d):
        self.__dict__.update(d)

    # ------------------------------------------------------------------ device
    def _srbd_config(self) -> "_lib.SrbdConfig":
        mp = self._cfg.mpc_params
        self.device_id = resolve_device_id(self.device_id)
        return _lib.make_config(
            num_samples=self.num_parallel_computations, horizon=self.horizon, method=self.sampling_method,
            parametrization=self.control_parametrization, num_splines=self.num_spline,
            num_elite=mp.get("num_elite", 10), device_id=self.device_id, use_graph=mp.get("use_hip_graph", True),
            mass=self.mass, inertia=self.inertia, dts=self.dts, grf_min=self.f_z_min, grf_max=self.f_z_max,
            mu=self.mu, q_diag=self.Q, sigma_mppi=mp["sigma_mppi"], sigma_random_sampling=mp["sigma_random_sampling"],
        )

    @property
    def context(self) -> "_lib.Context":
        if self._ctx is None:
            self._ctx = _lib.Context(self._srbd_config())
            # optional extension (not in the reference): mpc_params['cost_terms'] = {'r_force': (rx, ry, rz),
            # 'w_smooth': w, 'w_cone': w}; absent or zero = the reference's cost (include/srbd_mpc.h)
            terms = self._cfg.mpc_params.get("cost_terms")
            if terms:
                self._ctx.set_cost_terms(terms.get("r_force", (0.0, 0.0, 0.0)), terms.get("w_smooth", 0.0),
                                         terms.get("w_cone", 0.0))
            # optional (not in the reference): mpc_params['armed_steps'] = True queues each step's successor
            # ahead of its input (srbd_set_armed; outputs unchanged, launch latency off the call) -- for a
            # controller process that owns its GPU queue; 'armed_deadline_us' bounds the wait (default 50 ms)
            if self._cfg.mpc_params.get("armed_steps", False):
                self._ctx.set_armed(True, int(self._cfg.mpc_params.get("armed_deadline_us", 0)))
            if self.rng != "philox":
                self._ctx.set_rng(self.rng)
        return self._ctx

    def _key_args(self, key):
        """(seed, counter) of srbd_step for a compute call's `key`."""
        if self.rng == "philox":
            key = np.asarray(key, dtype=np.uint64).reshape(-1)
            return int(key[0]), (int(key[1]) if key.shape[0] > 1 else 0)
        self._calls += 1
        return _lib.pack_key(np.asarray(key, dtype=np.uint32)), self._calls

    def _run(self, state, reference, contact_sequence, best_control_parameters, key, sigma, noise):
        ctx = self.context
        seed, counter = self._key_args(key)
        # (the contact rows are cast to float32 as Context stages them)
        best, new_sigma, res, _ = ctx.step(state, reference, contact_sequence, best_control_parameters, sigma=sigma,
                                           noise=noise, seed=seed, counter=counter)
        self.last_result = res
        grf = np.array(res.grf, dtype=f32)
        pred = np.array(res.predicted_state, dtype=f32)
        costs = LazyCosts(ctx, ctx.step_id)
        return grf, np.zeros(12, dtype=np.int32), pred, best, f32(res.best_cost), new_sigma, costs, int(res.best_index)

    # ------------------------------------------------------------------ controls
    def compute_control_random_sampling(self, state, reference, contact_sequence, best_control_parameters, key,
                                        timing=None, nominal_step_frequency=None, optimize_swing=None, *, noise=None):
        """centroidal_nmpc_jax.py:629-787."""
        grf, fh, pred, best, cost, _, costs, _ = self._run(state, reference, contact_sequence,
                                                           best_control_parameters, key, None, noise)
        return grf, fh, pred, best, cost, 1.4, costs

    def compute_control_mppi(self, state, reference, contact_sequence, best_control_parameters, key, timing=None,
                             nominal_step_frequency=None, optimize_swing=None, *, noise=None):
        """centroidal_nmpc_jax.py:789-932."""
        grf, fh, pred, best, cost, _, costs, _ = self._run(state, reference, contact_sequence,
                                                           best_control_parameters, key, None, noise)
        return grf, fh, pred, best, cost, 1.4, costs

    def compute_control_cem_mppi(self, state, reference, contact_sequence, best_control_parameters, key, sigma,
                                 timing=None, nominal_step_frequency=None, *, noise=None):
        """centroidal_nmpc_jax.py:934-1094 (sigma: scalar or (P,))."""
        grf, fh, pred, best, cost, new_sigma, costs, _ = self._run(state, reference, contact_sequence,
                                                                   best_control_parameters, key, sigma, noise)
        return grf, fh, pred, best, cost, 1.65, costs, new_sigma

    # ------------------------------------------------------------------ keys / sigma (:498-511)
    def with_newkey(self):
        if self.rng == "philox":
            self.master_key = np.array([self.master_key[0], self.master_key[1] + np.uint64(1)], dtype=np.uint64)
        else:  # newkey, subkey = jax.random.split(master_key); master_key = newkey
            kb = getattr(self, "_split_buf", None)
            if kb is None:  # key (2) | split(key, 2) (2 x 2), address taken once (srbd_jax_split, _lib.jax_split)
                kb = self._split_buf = np.zeros(6, np.uint32)
                self._split_addr = kb.ctypes.data
            _store(kb[0:2], np.asarray(self.master_key, dtype=np.uint32))
            _lib.check(_lib.lib.srbd_jax_split(self._split_addr, 2, 1 if self.rng == "jax" else 0,
                                               self._split_addr + 8), None, "srbd_jax_split")
            self.master_key = kb[2:4].copy()
        return self

    def get_key(self):
        return self.master_key

    def with_newsigma(self, sigma):
        self.sigma_cem_mppi = sigma
        return self

    def get_sigma(self):
        return self.sigma_cem_mppi

    # ------------------------------------------------------------------ host-side helpers
    def spline_host(self, parameters, step, horizon_leg):
        """Host evaluation of the leg spline (centroidal_nmpc_jax.py:181-268), float32."""
        p = np.asarray(parameters, dtype=f32)
        if self.control_parametrization == "zero_order":
            i = int(np.int16(step))
            return p[i], p[i + self.horizon], p[i + 2 * self.horizon]
        S = self.num_spline
        cb = np.linspace(0, self.horizon, S + 1).astype(f32)
        index = int(np.max(np.where(f32(step) >= cb, np.arange(S + 1), 0)))
        q = f32(f32(f32(step) / f32(horizon_leg / S)) - f32(index))
        if self.control_parametrization == "linear_spline":
            sh = S + 1
            return tuple((f32(1) - q) * p[index + a * sh] + q * p[index + a * sh + 1] for a in range(3))
        s = 10 * index
        a = f32(2) * q * q * q - f32(3) * q * q + f32(1)
        b = q * q * q - f32(2) * q * q + q
        c = f32(-2) * q * q * q + f32(3) * q * q
        d = q * q * q - q * q
        out = []
        for o in (0, 4, 8):
            p0, p1, p2, p3 = p[s + o], p[s + o + 1], p[s + o + 2], p[s + o + 3]
            phi = f32(0.5) * ((p2 - p1) + (p1 - p0))
            phin = f32(0.5) * ((p3 - p2) + (p2 - p1))
            out.append(a * p1 + b * phi + c * p2 + d * phin)
        return tuple(out)

    def shift_solution(self, best_control_parameters, step):
        """centroidal_nmpc_jax.py:513-561: leg-wise control[0], [2], [4] <- spline(control, step, H)."""
        best = np.array(best_control_parameters, dtype=f32)
        PL = self.num_control_parameters_single_leg
        for leg in range(4):
            ctrl = copy.deepcopy(best[leg * PL:(leg + 1) * PL])
            fx, fy, fz = self.spline_host(ctrl, step, self.horizon)
            ctrl[0], ctrl[2], ctrl[4] = fx, fy, fz
            best[leg * PL:(leg + 1) * PL] = ctrl
        return best

    def prepare_state_and_reference(self, state_current, reference_state, current_contact, previous_contact,
                                    mpc_frequency=100):
        """centroidal_nmpc_jax.py:563-627."""
        if self._cfg.mpc_params["shift_solution"]:
            self.best_control_parameters = self.shift_solution(self.best_control_parameters, 1.0 / mpc_frequency)
        ps = self._prep_bufs()
        # list comprehensions over fixed key tuples: ~half the cost of the generator + tuple forms (per-step path)
        np.concatenate([state_current[k] for k in _STATE_KEYS], out=ps.state_in)
        np.concatenate([reference_state[k] for k in _REF_KEYS] + [reference_state[k].reshape((3,)) for k in _REF_FEET],
                       out=ps.ref_in)
        # swing-foot substitution and lift-off zeroing in the C++ host producer (include/srbd_host.h)
        _store(ps.cur, current_contact)
        _store(ps.prev, previous_contact)
        _store(ps.best, self.best_control_parameters)
        _lib.check(_lib.lib.srbd_prepare_state(*ps.addr, self.num_control_parameters_single_leg, ps.a_best,
                                               *ps.addr_out), what="srbd_prepare_state")
        self.best_control_parameters = ps.best.copy()
        state, ref = ps.out[0].copy(), ps.out[1].copy()
        return state, ref

    def _prep_bufs(self):
        """Persistent staging of srbd_prepare_state's arguments, addresses taken once (the call is on the
        per-MPC-step path; a ctypes pointer conversion costs about as much as the C call)."""
        ps = getattr(self, "_ps", None)
        if ps is None:
            ps = self._ps = _PrepBufs(self.num_control_parameters)
        return ps

    def reset(self):
        print("Resetting the controller")

    # ------------------------------------------------------------------ checkpoint (not in the reference)
    def get_state(self) -> dict:
        """Checkpoint of the controller's evolving state, as plain numpy arrays (``np.savez``-able):
        the warm start ``best_control_parameters``, the RNG key ``master_key`` and, for CEM,
        ``sigma_cem_mppi`` -- everything the next compute call depends on besides its arguments --
        plus, once a context exists and has stepped, the device-resident chain state (``device_*``,
        ``srbd_get_state``).  ``set_state`` of it makes the following calls replay bit for bit."""
        st = {"best_control_parameters": np.array(self.best_control_parameters, dtype=f32).reshape(-1),
              "master_key": np.array(self.master_key).reshape(-1)}  # uint32[2] (JAX key) or uint64[2] (Philox)
        if self.sampling_method == "cem_mppi":
            st["sigma_cem_mppi"] = np.array(np.broadcast_to(np.asarray(self.sigma_cem_mppi, dtype=f32),
                                                            (self.num_control_parameters,)), dtype=f32)
        if self._ctx is not None and self._ctx.step_id > 0:
            best, sigma, seed, ctr = self._ctx.get_state()
            st["device_best"] = best
            if sigma is not None:
                st["device_sigma"] = sigma
            st["device_key"] = np.array([seed, ctr], dtype=np.uint64)
        return st

    def set_state(self, st: dict) -> "Sampling_MPC":
        """Restore a ``get_state`` checkpoint.  The host part (warm start, key, sigma) always; the device part
        (``device_*``: what the next device-resident step starts from) only into a context that has run a
        step, since srbd_set_state needs that step's state/reference inputs.  A fresh controller drops the
        device part with a RuntimeWarning: its compute calls start from the host part anyway."""
        self.best_control_parameters = np.array(st["best_control_parameters"], dtype=f32).reshape(-1)
        want = np.uint64 if self.rng == "philox" else np.uint32  # (seed, counter) / a JAX key
        key = np.asarray(st["master_key"])
        if key.dtype != want or key.size != 2:
            raise ValueError(f"set_state: master_key {key.dtype}[{key.size}] does not fit rng={self.rng!r} "
                             f"(expects {np.dtype(want).name}[2]); the checkpoint was taken with another stream")
        self.master_key = key.astype(want).reshape(-1)
        if "sigma_cem_mppi" in st:
            self.sigma_cem_mppi = np.array(st["sigma_cem_mppi"], dtype=f32)
        if "device_best" in st:
            if self._ctx is not None and self._ctx.step_id > 0:
                key = np.asarray(st["device_key"], dtype=np.uint64)
                self._ctx.set_state(st["device_best"], st.get("device_sigma"), int(key[0]), int(key[1]))
            else:
                warnings.warn("set_state: no stepped context yet, the checkpoint's device-resident part "
                              "(device_best/device_sigma/device_key) is not restored", RuntimeWarning, stacklevel=2)
        return self

    def close(self):
        if self._ctx is not None:
            self._ctx.close()
            self._ctx = None
