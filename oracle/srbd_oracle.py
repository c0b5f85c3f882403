"""CPU oracle (numpy float32) for the sampling SRBD MPC hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker.  The product path (``quadruped_pympc_amd``) never imports it.

This is a line-by-line restatement, vectorised over samples, of the reference's
JAX code.  Every function cites the reference file:line it follows
(paths relative to the reference repository root):

* ``quadruped_pympc/controllers/sampling/centroidal_model_jax.py``  (CMJ)
* ``quadruped_pympc/controllers/sampling/centroidal_nmpc_jax.py``   (NMPC)
* ``quadruped_pympc/interfaces/srbd_controller_interface.py``       (SCI)

Arithmetic is float32 throughout, op-by-op in the reference's evaluation order
(JAX with x64 disabled: Python floats become f32 "weak" scalars).

PARITY STATUS: **parity unpinned** against the reference itself.  The
reference is pure JAX; ``jax`` (and ``gym_quadruped``) are not installed in
this image (an ordinary ModuleNotFoundError, no network), the reference ships
no tests, fixtures or golden vectors, and JAX's threefry bit stream and XLA's
reduction order are therefore unavailable.  The oracle is instead pinned by
analytic known-answer tests (``tests/test_oracle_kat.py``: free fall, static
stance, cofactor inverse vs ``numpy.linalg.inv``, zero-noise MPPI, n_stance=0,
spline identities) and by agreement with the independent C restatement
``oracle/srbd_oracle.c``.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32

# Method / parametrisation codes (mirrors include/srbd_mpc.h)
RANDOM_SAMPLING, MPPI, CEM_MPPI = 0, 1, 2
ZERO_ORDER, LINEAR_SPLINE, CUBIC_SPLINE = 0, 1, 2

METHOD_CODES = {"random_sampling": RANDOM_SAMPLING, "mppi": MPPI, "cem_mppi": CEM_MPPI}
PARAM_CODES = {"zero_order": ZERO_ORDER, "linear_spline": LINEAR_SPLINE, "cubic_spline": CUBIC_SPLINE}

# NMPC:39-41
MAX_SAMPLING_FORCES_X = 10
MAX_SAMPLING_FORCES_Y = 10
MAX_SAMPLING_FORCES_Z = 30


def num_params_single_leg(param_kind: int, horizon: int, num_splines: int) -> int:
    """NMPC:52-93."""
    if param_kind == LINEAR_SPLINE:
        return (num_splines + 1) * 3
    if param_kind == CUBIC_SPLINE:
        return 4 * 3 * num_splines
    return horizon * 3


def q_diag() -> np.ndarray:
    """NMPC:118-130 (Q is diagonal; R is unused by the rollout, NMPC:453-484)."""
    q = np.zeros(24, dtype=f32)
    q[2] = 1500
    q[3] = q[4] = q[5] = 200
    q[6] = q[7] = 500
    q[9] = q[10] = 20
    q[11] = 50
    return q


def calculate_inverse(A: np.ndarray) -> np.ndarray:
    """Cofactor 3x3 inverse, CMJ:67-91.  A: (..., 3, 3) float32."""
    A = np.asarray(A, dtype=f32)
    a11, a12, a13 = A[..., 0, 0], A[..., 0, 1], A[..., 0, 2]
    a21, a22, a23 = A[..., 1, 0], A[..., 1, 1], A[..., 1, 2]
    a31, a32, a33 = A[..., 2, 0], A[..., 2, 1], A[..., 2, 2]
    DET = a11 * (a33 * a22 - a32 * a23) - a21 * (a33 * a12 - a32 * a13) + a31 * (a23 * a12 - a22 * a13)
    M = np.stack(
        [
            np.stack([(a33 * a22 - a32 * a23), -(a33 * a12 - a32 * a13), (a23 * a12 - a22 * a13)], -1),
            np.stack([-(a33 * a21 - a31 * a23), (a33 * a11 - a31 * a13), -(a23 * a11 - a21 * a13)], -1),
            np.stack([(a32 * a21 - a31 * a22), -(a32 * a11 - a31 * a12), (a22 * a11 - a21 * a12)], -1),
        ],
        -2,
    )
    return (M / DET[..., None, None]).astype(f32)


def _matvec3(M, v):
    """jnp.dot(M(3x3), v(3)) with left-to-right accumulation; vectorised over leading dims."""
    return np.stack(
        [M[..., i, 0] * v[..., 0] + M[..., i, 1] * v[..., 1] + M[..., i, 2] * v[..., 2] for i in range(3)], -1
    ).astype(f32)


def _skew_dot(v, f):
    """jnp.dot(skew(v), f), skew rows [0,-v2,v1],[v2,0,-v0],[-v1,v0,0] (CMJ:100-101)."""
    z = f32(0)
    r0 = z * f[..., 0] + (-v[..., 2]) * f[..., 1] + v[..., 1] * f[..., 2]
    r1 = v[..., 2] * f[..., 0] + z * f[..., 1] + (-v[..., 0]) * f[..., 2]
    r2 = (-v[..., 1]) * f[..., 0] + v[..., 0] * f[..., 1] + z * f[..., 2]
    return np.stack([r0, r1, r2], -1).astype(f32)


class CentroidalModel:
    """Restates ``Centroidal_Model_JAX`` (CMJ:19-174)."""

    def __init__(self, mass, inertia, dt, horizon, use_nonuniform=False, horizon_fine=2, dt_fine=0.01):
        self.mass = float(mass)
        self.inertia = np.asarray(inertia, dtype=f32).reshape(3, 3)  # jnp.array(config.inertia) -> f32
        # CMJ:42-53
        if use_nonuniform:
            self.dts = np.concatenate(
                [np.full(horizon_fine, dt_fine, dtype=f32), np.full(horizon - horizon_fine, dt, dtype=f32)]
            )
        else:
            self.dts = np.full(horizon, dt, dtype=f32)
        self.inertia_inv = calculate_inverse(self.inertia)  # CMJ:56

    def fd(self, x: np.ndarray, f: np.ndarray, c: np.ndarray) -> np.ndarray:
        """CMJ:93-162.  x: (N,24) f32 state; f: (N,12) f32 foot forces (inputs[12:]); c: (4,) f32
        contact flags shared by all samples, or (N,4) per sample (gait-adaptive rollouts)."""
        x = np.asarray(x, dtype=f32)
        f = np.asarray(f, dtype=f32)
        c = np.asarray(c, dtype=f32)
        if c.ndim == 2:
            c = [c[:, i:i + 1] for i in range(4)]
        feet = [x[:, 12 + 3 * i: 15 + 3 * i] for i in range(4)]
        forces = [f[:, 3 * i: 3 * i + 3] for i in range(4)]
        com = x[:, 0:3]
        lin_vel = x[:, 3:6]
        temp = forces[0] * c[0] + forces[1] * c[1] + forces[2] * c[2] + forces[3] * c[3]
        gravity = np.array([0, 0, -9.81], dtype=f32)
        inv_m = f32(1) / f32(self.mass)
        lin_acc = inv_m * temp + gravity

        w = x[:, 9:12]
        roll, pitch, yaw = x[:, 6], x[:, 7], x[:, 8]
        sr, cr = np.sin(roll), np.cos(roll)
        sp, cp = np.sin(pitch), np.cos(pitch)
        sy, cy = np.sin(yaw), np.cos(yaw)
        one = np.ones_like(roll)
        zero = np.zeros_like(roll)
        conj = np.stack(
            [
                np.stack([one, zero, -sp], -1),
                np.stack([zero, cr, cp * sr], -1),
                np.stack([zero, -sr, cp * cr], -1),
            ],
            -2,
        )
        temp2 = _skew_dot(feet[0] - com, forces[0]) * c[0]
        temp2 = temp2 + _skew_dot(feet[1] - com, forces[1]) * c[1]
        temp2 = temp2 + _skew_dot(feet[2] - com, forces[2]) * c[2]
        temp2 = temp2 + _skew_dot(feet[3] - com, forces[3]) * c[3]

        euler_rates = _matvec3(calculate_inverse(conj), w)

        R = np.stack(
            [
                np.stack([cp * cy, cp * sy, -sp], -1),
                np.stack([sr * sp * cy - cr * sy, sr * sp * sy + cr * cy, sr * cp], -1),
                np.stack([cr * sp * cy + sr * sy, cr * sp * sy - sr * cy, cr * cp], -1),
            ],
            -2,
        )
        Iw = _matvec3(self.inertia, w)
        wxIw = _skew_dot(w, Iw)
        ang_acc = -_matvec3(self.inertia_inv, wxIw) + _matvec3(self.inertia_inv, _matvec3(R, temp2))
        return np.concatenate([lin_vel, lin_acc, euler_rates, ang_acc], -1).astype(f32)

    def integrate(self, x, f, c, n):
        """CMJ:164-174 (explicit Euler, feet unchanged)."""
        x = np.asarray(x, dtype=f32)
        d = self.fd(x, f, c)
        new = x[:, 0:12] + d * self.dts[n]
        return np.concatenate([new, x[:, 12:]], -1).astype(f32)


class SamplingMPCOracle:
    """Restates ``Sampling_MPC`` (NMPC:20-1097) for one configuration."""

    def __init__(
        self,
        *,
        mass,
        inertia,
        horizon=12,
        dt=0.02,
        num_samples=10000,
        method="mppi",
        parametrization="zero_order",
        num_splines=2,
        mu=0.5,
        grf_min=0.0,
        grf_max=None,
        sigma_mppi=3.0,
        sigma_cem_mppi=3.0,
        sigma_random_sampling=(0.2, 3.0, 10.0),
        use_nonuniform=False,
        horizon_fine=2,
        dt_fine=0.01,
    ):
        self.method = METHOD_CODES[method] if isinstance(method, str) else int(method)
        self.param_kind = PARAM_CODES[parametrization] if isinstance(parametrization, str) else int(parametrization)
        self.horizon = int(horizon)
        self.num_spline = int(num_splines)
        self.N = int(num_samples)
        self.PL = num_params_single_leg(self.param_kind, self.horizon, self.num_spline)
        self.P = 4 * self.PL
        self.mu = mu
        self.f_z_min = grf_min
        self.f_z_max = grf_max if grf_max is not None else mass * 9.81  # config.py:90
        self.sigma_mppi = sigma_mppi
        self.sigma_cem_mppi = sigma_cem_mppi
        self.sigma_random_sampling = list(sigma_random_sampling)
        self.robot = CentroidalModel(mass, inertia, dt, horizon, use_nonuniform, horizon_fine, dt_fine)
        self.Q = q_diag()

    # ---------------------------------------------------------------- splines
    def _chunk_index(self, step):
        # NMPC:187-189 / 210-212
        cb = np.linspace(0, self.horizon, self.num_spline + 1).astype(f32)
        return int(np.max(np.where(f32(step) >= cb, np.arange(self.num_spline + 1), 0)))

    def _tau(self, step, horizon_leg):
        # NMPC:191-192: step / (horizon_leg / S) - index ; int32 step / weak float -> f32
        index = self._chunk_index(step)
        tau = f32(step) / f32(horizon_leg / self.num_spline)
        tau = f32(tau - f32(1 * index))
        return index, f32(tau / f32(1.0))

    def spline(self, params, step, horizon_leg):
        """params: (N, PL) f32.  Returns fx, fy, fz (N,) f32."""
        p = np.asarray(params, dtype=f32)
        if self.param_kind == ZERO_ORDER:  # NMPC:259-268
            idx = int(np.int16(step))
            H = self.horizon
            return p[:, idx], p[:, idx + H], p[:, idx + 2 * H]
        index, q = self._tau(step, horizon_leg)
        if self.param_kind == LINEAR_SPLINE:  # NMPC:181-201
            shift = self.num_spline + 1
            omq = f32(1) - q
            fx = omq * p[:, index] + q * p[:, index + 1]
            fy = omq * p[:, index + shift] + q * p[:, index + shift + 1]
            fz = omq * p[:, index + 2 * shift] + q * p[:, index + 2 * shift + 1]
            return fx, fy, fz
        # cubic, NMPC:204-257 (quirk: start = 10 * index)
        s = 10 * index
        two, three, half = f32(2), f32(3), f32(0.5)
        a = two * q * q * q - three * q * q + f32(1)
        b = (q * q * q - two * q * q + q) * f32(1.0)
        c = -two * q * q * q + three * q * q
        d = (q * q * q - q * q) * f32(1.0)

        def axis(o):
            p0, p1, p2, p3 = p[:, s + o], p[:, s + o + 1], p[:, s + o + 2], p[:, s + o + 3]
            phi = half * (((p2 - p1) / f32(1.0)) + ((p1 - p0) / f32(1.0)))
            phin = half * (((p3 - p2) / f32(1.0)) + ((p2 - p1) / f32(1.0)))
            return a * p1 + b * phi + c * p2 + d * phin

        return axis(0), axis(4), axis(8)

    # --------------------------------------------------------- constraints
    def enforce_force_constraints(self, fx, fy, fz):
        """NMPC:270-314, ``where(a > b, a, b)`` form (NaN -> bound).  fx,fy,fz: lists of 4 arrays."""
        fz_min, fz_max = f32(self.f_z_min), f32(self.f_z_max)
        mu, nmu = f32(self.mu), f32(-self.mu)
        ox, oy, oz = [], [], []
        for i in range(4):
            z = np.where(fz[i] > fz_min, fz[i], fz_min).astype(f32)
            z = np.where(z < fz_max, z, fz_max).astype(f32)
            lo, hi = nmu * z, mu * z
            x = np.where(fx[i] > lo, fx[i], lo).astype(f32)
            x = np.where(x < hi, x, hi).astype(f32)
            y = np.where(fy[i] > lo, fy[i], lo).astype(f32)
            y = np.where(y < hi, y, hi).astype(f32)
            ox.append(x)
            oy.append(y)
            oz.append(z)
        return ox, oy, oz

    def _forces_at(self, params, contact, n, step, horizon_leg, with_pre=False):
        """Decode + gravity compensation + contact mask + clip (NMPC:364-420 and :706-750).
        with_pre: also the masked x / y before the clip (N, 8) and fref (the opt-in cone term)."""
        PL = self.PL
        fx, fy, fz = [], [], []
        for leg in range(4):
            a, b, c = self.spline(params[:, leg * PL:(leg + 1) * PL], step, horizon_leg)
            fx.append(a)
            fy.append(b)
            fz.append(c)
        cs = [f32(contact[leg][n]) for leg in range(4)]
        ns = f32(f32(cs[0] + cs[1]) + cs[2]) + cs[3]
        with np.errstate(divide="ignore", invalid="ignore"):
            fref = f32(self.robot.mass * 9.81) / ns
            rx = f32(MAX_SAMPLING_FORCES_Z / MAX_SAMPLING_FORCES_X)
            ry = f32(MAX_SAMPLING_FORCES_Z / MAX_SAMPLING_FORCES_Y)
            for leg in range(4):
                fz[leg] = fref + fz[leg]
                fx[leg] = fx[leg] * cs[leg] / rx
                fy[leg] = fy[leg] * cs[leg] / ry
                fz[leg] = fz[leg] * cs[leg]
            pre = np.stack([v for leg in range(4) for v in (fx[leg], fy[leg])], -1).astype(f32)
            fx, fy, fz = self.enforce_force_constraints(fx, fy, fz)
        F = np.stack([v for leg in range(4) for v in (fx[leg], fy[leg], fz[leg])], -1).astype(f32)
        if with_pre:
            return F, np.array(cs, dtype=f32), pre, f32(fref)
        return F, np.array(cs, dtype=f32)

    # ------------------------------------------------------------- rollout
    def rollout_costs(self, state, reference, params, contact, cost_terms=None):
        """vmap(compute_rollout), NMPC:316-496.  params (N,P) f32 -> costs (N,) f32 (unsaturated).
        cost_terms: None, or dict(r_force, w_smooth, w_cone) of the build's opt-in terms (extra_cost)."""
        params = np.asarray(params, dtype=f32)
        N = params.shape[0]
        x = np.broadcast_to(np.asarray(state, dtype=f32), (N, 24)).copy()
        ref = np.asarray(reference, dtype=f32)
        cost = np.zeros(N, dtype=f32)
        Fprev = None
        with np.errstate(over="ignore", invalid="ignore", divide="ignore"):
            for n in range(self.horizon):
                F, cs, pre, fref = self._forces_at(params, contact, n, n, self.horizon, with_pre=True)
                x = self.robot.integrate(x, F, cs, n)
                e = (x - ref).astype(f32)
                # e^T Q e with diagonal Q, accumulated i = 0..23
                qe = e * self.Q
                acc = qe[:, 0] * e[:, 0]
                for i in range(1, 24):
                    acc = acc + qe[:, i] * e[:, i]
                cost = cost + acc
                if cost_terms:
                    cost = (cost + extra_cost(F, pre, cs, fref, Fprev, f32(self.mu), cost_terms)).astype(f32)
                Fprev = F
        return cost.astype(f32)

    @staticmethod
    def saturate(costs):
        """NMPC:686-687."""
        c = np.where(np.isnan(costs), f32(1000000), costs)
        c = np.where(np.isinf(c), f32(1000000), c)
        return c.astype(f32)

    def final_grf_and_prediction(self, state, contact, best):
        """NMPC:695-784 (step 0.0, horizon_leg 1) -> (GRFs(12), predicted_state(24))."""
        best = np.asarray(best, dtype=f32)[None, :]
        F, cs = self._forces_at(best, contact, 0, 0.0, 1)
        pred = self.robot.integrate(np.asarray(state, dtype=f32)[None, :], F, cs, 0)
        return F[0], pred[0]

    # -------------------------------------------------------------- noise
    def assemble_noise(self, Z, sigma=None, U=None):
        """Build ``additional_random_parameters`` (N,P) from standard draws.

        Z: (N-1, P) standard normals for MPPI/CEM (NMPC:806-812, :951-958), or for
        random sampling (NMPC:647-677) Z (t, P) normals and U (N-1-2t, P) uniform in
        [-s2, s2]; t = int(N/3).  Row 0 is always zero.  Rows t+1..2t reuse Z (same
        key and shape in the reference, App. B #3).
        """
        N, P = self.N, self.P
        out = np.zeros((N, P), dtype=f32)
        if self.method == MPPI:
            out[1:] = f32(self.sigma_mppi) * np.asarray(Z, dtype=f32)
        elif self.method == CEM_MPPI:
            out[1:] = np.asarray(Z, dtype=f32) * np.asarray(sigma, dtype=f32)
        else:
            t = int(N / 3)
            s0, s1 = self.sigma_random_sampling[0], self.sigma_random_sampling[1]
            out[1:1 + t] = f32(s0) * np.asarray(Z[:t], dtype=f32)
            out[1 + t:1 + 2 * t] = f32(s1) * np.asarray(Z[:t], dtype=f32)
            out[1 + 2 * t:N] = np.asarray(U, dtype=f32)
        return out

    # ------------------------------------------------------------ control
    def compute_control(self, state, reference, contact, best, noise, sigma=None):
        """compute_control_{random_sampling|mppi|cem_mppi}, NMPC:629-1094.

        noise: (N, P) = additional_random_parameters (row 0 zero).
        Returns dict(grf, pred, best, best_cost, best_index, costs[, sigma]).
        """
        noise = np.asarray(noise, dtype=f32)
        best = np.asarray(best, dtype=f32)
        params = (best[None, :] + noise).astype(f32)
        costs = self.saturate(self.rollout_costs(state, reference, params, contact))
        return self.reduce(state, contact, best, noise, costs)

    def reduce(self, state, contact, best, noise, costs):
        """Everything after the rollout, fed with a given (saturated) cost vector."""
        noise = np.asarray(noise, dtype=f32)
        best = np.asarray(best, dtype=f32)
        costs = np.asarray(costs, dtype=f32)
        best_index = int(np.nanargmin(costs))  # first index on ties
        best_cost = costs[best_index]
        out = dict(best_index=best_index, best_cost=best_cost, costs=costs)
        if self.method == RANDOM_SAMPLING:  # NMPC:692
            new_best = (best + noise[best_index]).astype(f32)
        else:  # NMPC:828-836 / :974-982
            beta = best_cost
            with np.errstate(over="ignore", under="ignore"):
                exp_costs = np.exp(f32(-1.0) * (costs - beta)).astype(f32)
            denom = np.sum(exp_costs, dtype=f32)
            weights = (exp_costs / denom).astype(f32)
            upd = np.sum(weights[:, None] * noise, axis=0, dtype=f32)
            new_best = (best + upd).astype(f32)
        out["best"] = new_best
        grf, pred = self.final_grf_and_prediction(state, contact, new_best)
        out["grf"], out["pred"] = grf, pred
        if self.method == CEM_MPPI:  # NMPC:1075-1081
            idx = np.argsort(costs, kind="stable")[:10]
            elite = noise[idx]
            mean = (np.sum(elite, axis=0, dtype=f32) / f32(elite.shape[0])).astype(f32)
            d = (elite - mean).astype(f32)
            var = (np.sum(d * d, axis=0, dtype=f32) / f32(elite.shape[0] - 1)).astype(f32)
            s = np.sqrt((var + f32(1e-8)).astype(f32)).astype(f32)
            s = np.where(s > 5, f32(5), s)
            s = np.where(s < f32(0.2), f32(0.2), s).astype(f32)
            out["sigma"] = s
            out["elite"] = idx
        return out


def extra_cost(F, pre, cs, fref, Fprev, mu, terms):
    """The build's opt-in cost terms of one step (include/srbd_mpc.h srbd_set_cost_terms; not in the
    reference, whose R input cost is commented out at NMPC:453-484).  F (N,12) clipped forces, pre (N,8)
    masked x / y before the clip, cs (4,) or (N,4) contact, fref the gravity share, Fprev the previous
    step's F (None at n = 0).  Returns (N,) f32: per component, leg by leg, r_q u^2 + w_smooth d^2 +
    w_cone v^2 (kernel order: srbd_core.h extra_cost_step)."""
    r = np.asarray(terms.get("r_force", (0.0, 0.0, 0.0)), dtype=f32)
    ws, wc = f32(terms.get("w_smooth", 0.0)), f32(terms.get("w_cone", 0.0))
    cs = np.asarray(cs, dtype=f32)
    N = F.shape[0]
    total = np.zeros(N, dtype=f32)
    for q in range(3):
        e = np.zeros(N, dtype=f32)
        for leg in range(4):
            f = F[:, 3 * leg + q]
            c = cs[..., leg]
            if q == 2:
                u = (f - np.where(c != 0, fref, f32(0))).astype(f32)
            else:
                u = f
            term = ((u * r[q]).astype(f32) * u).astype(f32)
            if Fprev is not None:
                d = (f - Fprev[:, 3 * leg + q]).astype(f32)
                term = (term + (d * ws).astype(f32) * d).astype(f32)
            if q < 2:
                v = (np.abs(pre[:, 2 * leg + q]) - (mu * F[:, 3 * leg + 2]).astype(f32)).astype(f32)
                v = np.where(v > 0, v, f32(0)).astype(f32)
                term = (term + (v * wc).astype(f32) * v).astype(f32)
            e = (e + term).astype(f32)
        total = (total + e).astype(f32)
    return total


def prepare_state_and_reference(state_current, reference_state, current_contact, previous_contact, best, PL):
    """NMPC:563-627 (shift_solution off, config.py:188).  Returns (state24 f64, ref24 f64, best f32)."""
    s = np.concatenate(
        (
            state_current["position"], state_current["linear_velocity"], state_current["orientation"],
            state_current["angular_velocity"], state_current["foot_FL"], state_current["foot_FR"],
            state_current["foot_RL"], state_current["foot_RR"],
        )
    ).reshape((24,))
    for leg, name in enumerate(("FL", "FR", "RL", "RR")):
        if current_contact[leg] == 0.0:
            s[12 + 3 * leg: 15 + 3 * leg] = reference_state["ref_foot_" + name].reshape((3,))
    r = np.concatenate(
        (
            reference_state["ref_position"], reference_state["ref_linear_velocity"],
            reference_state["ref_orientation"], reference_state["ref_angular_velocity"],
            reference_state["ref_foot_FL"].reshape((3,)), reference_state["ref_foot_FR"].reshape((3,)),
            reference_state["ref_foot_RL"].reshape((3,)), reference_state["ref_foot_RR"].reshape((3,)),
        )
    ).reshape((24,))
    best = np.array(best, dtype=f32)
    for leg in range(4):
        if previous_contact[leg] == 1 and current_contact[leg] == 0:
            best[leg * PL:(leg + 1) * PL] = 0.0
    return s, r, best
