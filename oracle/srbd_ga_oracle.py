"""CPU oracle (numpy float32) for the gait-adaptive sampling MPC.

TEST INFRASTRUCTURE ONLY (same rules as ``srbd_oracle.py``: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it).

Restates, vectorised over samples (paths relative to the reference repository root):

* ``quadruped_pympc/helpers/periodic_gait_generator_jax.py``  (PGGJ)
  ``PeriodicGaitGeneratorJax.run`` (:68-89) and ``compute_contact_sequence`` (:136-151);
* ``quadruped_pympc/controllers/sampling/centroidal_nmpc_jax_gait_adaptive.py``  (GA)
  ``compute_rollout`` (:326-501), the per-method step-frequency sets (:687-692, :834-838,
  :994-999) and ``best_step_frequency`` (:705, :861, :1022).

Everything else (spline shapes, clip, dynamics, Q, reductions, final GRFs) is the base
``Sampling_MPC`` (``srbd_oracle.py``): the GA file is a copy of NMPC with these changes (diff of
the two files).  Float32 op by op, JAX x64-off evaluation order.

PARITY STATUS: **parity unpinned** (as ``srbd_oracle.py``: JAX absent; the frequency draw
``jax.random.choice`` uses threefry, not reproducible).  Pinned by known-answer tests
(``tests/test_ga_oracle.py``): an all-stance sequence reduces the GA rollout to the base
zero-order rollout plus the frequency term, the PGG restatement against a scalar loop, and the
negative-index wrap of a leg that has not touched down yet.
"""
from __future__ import annotations

import numpy as np

from .srbd_oracle import extra_cost, CUBIC_SPLINE, LINEAR_SPLINE, MAX_SAMPLING_FORCES_X, MAX_SAMPLING_FORCES_Y, \
    MAX_SAMPLING_FORCES_Z, MPPI, CEM_MPPI, RANDOM_SAMPLING, ZERO_ORDER, SamplingMPCOracle

f32 = np.float32

GA_DUTY = 0.65          # GA:179  PeriodicGaitGeneratorJax(duty_factor=0.65, ...)
GA_FREQ_CENTER = 1.3    # GA:500
GA_FREQ_WEIGHT = 100
CEM_FREQ_INCREMENTS = (0.0, 0.2, 0.4)  # GA:995


def pgg_jax_contact_sequences(timing, freqs, horizon, mpc_dt, duty=GA_DUTY):
    """PGGJ:136-151 with run (:68-89), one sequence per sample.

    timing: (4,) leg phases (the caller's ``pgg_phase_signal``, f32 under x64-off jit);
    freqs: (N,) f32 step frequencies.  Returns (N, 4, H) f32 of 0/1.
    Per step: restart (t >= 1 -> 0, :73-76), advance t += mpc_dt * f (:79-82; the product first),
    contact = t < duty (:84-87).
    """
    freqs = np.asarray(freqs, dtype=f32)
    N = freqs.shape[0]
    t = np.broadcast_to(np.asarray(timing, dtype=f32), (N, 4)).copy()
    inc = (f32(mpc_dt) * freqs).astype(f32)
    cs = np.zeros((N, 4, horizon), dtype=f32)
    for n in range(horizon):
        t = np.where(t >= f32(1.0), f32(0.0), t).astype(f32)
        t = (t + inc[:, None]).astype(f32)
        cs[:, :, n] = np.where(t < f32(duty), f32(1.0), f32(0.0))
    return cs


def freq_set(method, step_freq_available, nominal_step_frequency, optimize_swing):
    """Candidate step frequencies jax.random.choice draws from, per method (f32, x64 off)."""
    if method == RANDOM_SAMPLING:  # GA:688
        avail = np.asarray(step_freq_available, dtype=f32)
        return np.where(bool(optimize_swing), avail, f32(nominal_step_frequency)).astype(f32)
    if method == MPPI:  # GA:835 (optimize_swing and the nominal frequency are not used)
        return np.asarray(step_freq_available, dtype=f32)
    # CEM, GA:995-999: choice([0, 0.2, 0.4]) * optimize_swing + nominal
    inc = np.asarray(CEM_FREQ_INCREMENTS, dtype=f32)
    return ((inc * f32(optimize_swing)).astype(f32) + f32(nominal_step_frequency)).astype(f32)


class GaitAdaptiveOracle(SamplingMPCOracle):
    """Restates the GA ``Sampling_MPC`` (GA:22-1134) for RS and MPPI."""

    def __init__(self, *, pgg_dt=None, **kw):
        super().__init__(**kw)
        self.pgg_dt = float(pgg_dt) if pgg_dt is not None else float(self.robot.dts[-1])  # mpc_params['dt']

    # ------------------------------------------------------------ decode
    def _chunk_index_vec(self, step):
        cb = np.linspace(0, self.horizon, self.num_spline + 1).astype(f32)  # GA:196 / :219
        st = step.astype(f32)[:, None]
        return np.max(np.where(st >= cb[None, :], np.arange(self.num_spline + 1)[None, :], 0), axis=1)

    def spline_vec(self, p, step, horizon_leg):
        """Per-sample decode (GA:190-278): p (N, PL), step (N,) int32 counter, horizon_leg (N,) f32."""
        N = p.shape[0]
        rows = np.arange(N)

        def at(j):  # jnp dynamic index: a negative index wraps (index + PL)
            j = np.asarray(j)
            return p[rows, np.where(j < 0, j + self.PL, j)]

        if self.param_kind == ZERO_ORDER:  # GA:269-278, index = int16(step)
            H = self.horizon
            idx = step.astype(np.int16).astype(np.int64)
            return at(idx), at(idx + H), at(idx + 2 * H)
        index = self._chunk_index_vec(step)
        seg = (horizon_leg / f32(self.num_spline)).astype(f32)          # horizon_leg / S
        tau = (step.astype(f32) / seg).astype(f32)
        tau = (tau - (1 * index).astype(f32)).astype(f32)
        q = (tau / f32(1.0)).astype(f32)
        if self.param_kind == LINEAR_SPLINE:  # GA:190-210
            sh = self.num_spline + 1
            omq = (f32(1) - q).astype(f32)
            fx = omq * at(index) + q * at(index + 1)
            fy = omq * at(index + sh) + q * at(index + sh + 1)
            fz = omq * at(index + 2 * sh) + q * at(index + 2 * sh + 1)
            return fx.astype(f32), fy.astype(f32), fz.astype(f32)
        s = 10 * index  # GA:228, cubic (quirk: 10, App. B #4)
        two, three, half = f32(2), f32(3), f32(0.5)
        a = two * q * q * q - three * q * q + f32(1)
        b = (q * q * q - two * q * q + q) * f32(1.0)
        c = -two * q * q * q + three * q * q
        d = (q * q * q - q * q) * f32(1.0)

        def axis(o):
            p0, p1, p2, p3 = at(s + o), at(s + o + 1), at(s + o + 2), at(s + o + 3)
            phi = half * (((p2 - p1) / f32(1.0)) + ((p1 - p0) / f32(1.0)))
            phin = half * (((p3 - p2) / f32(1.0)) + ((p2 - p1) / f32(1.0)))
            return (a * p1 + b * phi + c * p2 + d * phin).astype(f32)

        return axis(0), axis(4), axis(8)

    # ------------------------------------------------------------ rollout
    def rollout_costs_ga(self, state, reference, params, timing, freqs, cost_terms=None):
        """vmap(compute_rollout) of GA:326-501.  Returns unsaturated costs (N,) f32.
        cost_terms: the build's opt-in terms (srbd_oracle.extra_cost), None for the reference's cost."""
        params = np.asarray(params, dtype=f32)
        freqs = np.asarray(freqs, dtype=f32)
        N, PL = params.shape[0], self.PL
        cs = pgg_jax_contact_sequences(timing, freqs, self.horizon, self.pgg_dt)
        hl = (np.sum(cs, axis=2, dtype=f32) + f32(1)).astype(f32)      # GA:345-348
        n_ = np.full((N, 4), -1, dtype=np.int32)                         # GA:339
        x = np.broadcast_to(np.asarray(state, dtype=f32), (N, 24)).copy()
        ref = np.asarray(reference, dtype=f32)
        cost = np.zeros(N, dtype=f32)
        rx = f32(MAX_SAMPLING_FORCES_Z / MAX_SAMPLING_FORCES_X)
        ry = f32(MAX_SAMPLING_FORCES_Z / MAX_SAMPLING_FORCES_Y)
        Fprev = None
        with np.errstate(over="ignore", invalid="ignore", divide="ignore"):
            for n in range(self.horizon):
                c = cs[:, :, n]
                n_ = n_ + c.astype(np.int32)                             # GA:353-356
                fx, fy, fz = [], [], []
                for leg in range(4):
                    a, b, z = self.spline_vec(params[:, leg * PL:(leg + 1) * PL], n_[:, leg], hl[:, leg])
                    fx.append(a)
                    fy.append(b)
                    fz.append(z)
                ns = ((c[:, 0] + c[:, 1]) + c[:, 2]) + c[:, 3]           # GA:382-384
                fref = (f32(self.robot.mass * 9.81) / ns).astype(f32)   # GA:385
                for leg in range(4):                                      # GA:387-407
                    fz[leg] = (fref + fz[leg]).astype(f32)
                    fx[leg] = (fx[leg] * c[:, leg] / rx).astype(f32)
                    fy[leg] = (fy[leg] * c[:, leg] / ry).astype(f32)
                    fz[leg] = (fz[leg] * c[:, leg]).astype(f32)
                pre = np.stack([v for leg in range(4) for v in (fx[leg], fy[leg])], -1).astype(f32)
                fx, fy, fz = self.enforce_force_constraints(fx, fy, fz)   # GA:410-414
                F = np.stack([v for leg in range(4) for v in (fx[leg], fy[leg], fz[leg])], -1).astype(f32)
                x = self.robot.integrate(x, F, c, n)                     # GA:447-451
                e = (x - ref).astype(f32)
                qe = e * self.Q
                acc = qe[:, 0] * e[:, 0]
                for i in range(1, 24):
                    acc = acc + qe[:, i] * e[:, i]
                cost = (cost + acc).astype(f32)
                if cost_terms:
                    cost = (cost + extra_cost(F, pre, c, fref, Fprev, f32(self.mu), cost_terms)).astype(f32)
                Fprev = F
            d = (freqs - f32(GA_FREQ_CENTER)).astype(f32)                 # GA:500
            cost = (cost + ((d * f32(GA_FREQ_WEIGHT)).astype(f32) * d)).astype(f32)
        return cost

    def compute_control_ga(self, state, reference, contact, best, noise, freqs, timing):
        """compute_control_{random_sampling,mppi} of GA:630-962 with the draws given.

        noise: (N, P) additional_random_parameters (row 0 zero); freqs: (N,) step_frequencies_vec.
        The final GRFs / prediction use the caller's contact sequence (GA:720-796), as in NMPC.
        """
        if self.method == CEM_MPPI:
            raise NotImplementedError("gait-adaptive CEM: see DESIGN.md (reference branch broken, App. B #2)")
        noise = np.asarray(noise, dtype=f32)
        best = np.asarray(best, dtype=f32)
        freqs = np.asarray(freqs, dtype=f32)
        params = (best[None, :] + noise).astype(f32)
        costs = self.saturate(self.rollout_costs_ga(state, reference, params, timing, freqs))
        out = self.reduce(state, contact, best, noise, costs)
        out["best_freq"] = freqs[out["best_index"]]
        return out
