/*
 * CPU oracle (plain C, float32) for the sampling SRBD MPC hot path.
 *
 * TEST INFRASTRUCTURE ONLY: built to oracle/libsrbd_oracle.so and used by tests/
 * (as the checker), __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 * The product library (libsrbd_hip.so) never links or calls it.
 *
 * A second, independent restatement (scalar, one sample per loop iteration,
 * OpenMP over samples) of the reference's JAX sampling controller, in the
 * reference's float32 evaluation order.  Compile with -ffp-contract=off.
 * Cited files (relative to the reference repository root):
 *   CMJ  = quadruped_pympc/controllers/sampling/centroidal_model_jax.py
 *   NMPC = quadruped_pympc/controllers/sampling/centroidal_nmpc_jax.py
 *
 * PARITY STATUS: parity unpinned against the reference itself (JAX absent,
 * no reference fixtures); pinned by the analytic KATs in tests/ and by
 * agreement with oracle/srbd_oracle.py.
 *
 * RNG: the product's device RNG is Philox4x32-10 (Random123) + Box-Muller; it is
 * restated here (srbd_oracle_philox / srbd_oracle_gen_noise).  Philox is pinned
 * against the Random123 known-answer vectors and rocRAND (tests/test_philox_kat.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_MAXH 64
#define OR_MAXP 768

typedef struct oracle_cfg {
    int32_t N, H, method, param_kind, num_splines, _pad;
    float mass;            /* config mass (f32) */
    float mg;              /* f32(mass * 9.81) computed in double then rounded (NMPC:380) */
    float grf_min, grf_max, mu;
    float inertia[9];
    float dts[OR_MAXH];
    float sigma_mppi;
    float sigma_rs[3];
} oracle_cfg;

static int num_params_leg(const oracle_cfg* c) {
    if (c->param_kind == 1) return (c->num_splines + 1) * 3;
    if (c->param_kind == 2) return 12 * c->num_splines;
    return 3 * c->H;
}

/* CMJ:67-91 */
static void inv3(const float A[9], float out[9]) {
    float a11 = A[0], a12 = A[1], a13 = A[2], a21 = A[3], a22 = A[4], a23 = A[5], a31 = A[6], a32 = A[7], a33 = A[8];
    float DET = a11 * (a33 * a22 - a32 * a23) - a21 * (a33 * a12 - a32 * a13) + a31 * (a23 * a12 - a22 * a13);
    float M[9] = {(a33 * a22 - a32 * a23), -(a33 * a12 - a32 * a13), (a23 * a12 - a22 * a13),
                  -(a33 * a21 - a31 * a23), (a33 * a11 - a31 * a13), -(a23 * a11 - a21 * a13),
                  (a32 * a21 - a31 * a22), -(a32 * a11 - a31 * a12), (a22 * a11 - a21 * a12)};
    for (int i = 0; i < 9; ++i) out[i] = M[i] / DET;
}

static void mv3(const float M[9], const float v[3], float o[3]) {
    for (int i = 0; i < 3; ++i) o[i] = M[3 * i] * v[0] + M[3 * i + 1] * v[1] + M[3 * i + 2] * v[2];
}

static void skew_dot(const float v[3], const float f[3], float o[3]) {
    o[0] = 0.0f * f[0] + (-v[2]) * f[1] + v[1] * f[2];
    o[1] = v[2] * f[0] + 0.0f * f[1] + (-v[0]) * f[2];
    o[2] = (-v[1]) * f[0] + v[0] * f[1] + 0.0f * f[2];
}

/* CMJ:93-174: x (24) updated in place, f (12) foot forces, c (4) contact, dt */
static void integrate(const oracle_cfg* cfg, const float Iinv[9], float x[24], const float f[12], const float c[4],
                      float dt) {
    float temp[3], lin_acc[3], temp2[3] = {0, 0, 0}, er[3], aa[3];
    float inv_m = 1.0f / cfg->mass;
    for (int k = 0; k < 3; ++k)
        temp[k] = f[k] * c[0] + f[3 + k] * c[1] + f[6 + k] * c[2] + f[9 + k] * c[3];
    const float g[3] = {0.0f, 0.0f, -9.81f};
    for (int k = 0; k < 3; ++k) lin_acc[k] = inv_m * temp[k] + g[k];
    float roll = x[6], pitch = x[7], yaw = x[8];
    float sr = sinf(roll), cr = cosf(roll), sp = sinf(pitch), cp = cosf(pitch), sy = sinf(yaw), cy = cosf(yaw);
    float conj[9] = {1.0f, 0.0f, -sp, 0.0f, cr, cp * sr, 0.0f, -sr, cp * cr};
    for (int i = 0; i < 4; ++i) {
        float v[3] = {x[12 + 3 * i] - x[0], x[13 + 3 * i] - x[1], x[14 + 3 * i] - x[2]}, t[3];
        skew_dot(v, f + 3 * i, t);
        if (i == 0) {
            for (int k = 0; k < 3; ++k) temp2[k] = t[k] * c[0];
        } else {
            for (int k = 0; k < 3; ++k) temp2[k] = temp2[k] + t[k] * c[i];
        }
    }
    float Cinv[9];
    inv3(conj, Cinv);
    mv3(Cinv, x + 9, er);
    float R[9] = {cp * cy, cp * sy, -sp,
                  sr * sp * cy - cr * sy, sr * sp * sy + cr * cy, sr * cp,
                  cr * sp * cy + sr * sy, cr * sp * sy - sr * cy, cr * cp};
    float Iw[3], wxIw[3], a1[3], Rt[3], a2[3];
    mv3(cfg->inertia, x + 9, Iw);
    skew_dot(x + 9, Iw, wxIw);
    mv3(Iinv, wxIw, a1);
    mv3(R, temp2, Rt);
    mv3(Iinv, Rt, a2);
    for (int k = 0; k < 3; ++k) aa[k] = -a1[k] + a2[k];
    float d[12] = {x[3], x[4], x[5], lin_acc[0], lin_acc[1], lin_acc[2], er[0], er[1], er[2], aa[0], aa[1], aa[2]};
    for (int k = 0; k < 12; ++k) x[k] = x[k] + d[k] * dt;
}

/* Per-step spline coefficients (NMPC:181-268). */
typedef struct step_coef {
    int idx;
    float q, omq, a, b, c, d;
} step_coef;

static step_coef make_coef(const oracle_cfg* cfg, float step, int horizon_leg) {
    step_coef s;
    memset(&s, 0, sizeof(s));
    if (cfg->param_kind == 0) {
        s.idx = (int)(int16_t)step;
        return s;
    }
    int S = cfg->num_splines, idx = 0;
    for (int i = 0; i <= S; ++i) {
        float cb = (float)((double)cfg->H * (double)i / (double)S); /* linspace(0,H,S+1) */
        if (step >= cb) idx = i;
    }
    float tau = step / (float)((double)horizon_leg / (double)S);
    tau = tau - (float)idx;
    float q = tau / 1.0f;
    s.idx = idx;
    s.q = q;
    s.omq = 1.0f - q;
    s.a = 2.0f * q * q * q - 3.0f * q * q + 1.0f;
    s.b = (q * q * q - 2.0f * q * q + q) * 1.0f;
    s.c = -2.0f * q * q * q + 3.0f * q * q;
    s.d = (q * q * q - q * q) * 1.0f;
    return s;
}

static void decode_leg(const oracle_cfg* cfg, const float* p, const step_coef* sc, float n_step, float out[3]) {
    int H = cfg->H;
    if (cfg->param_kind == 0) {
        int i = sc->idx;
        out[0] = p[i];
        out[1] = p[i + H];
        out[2] = p[i + 2 * H];
    } else if (cfg->param_kind == 1) {
        int sh = cfg->num_splines + 1, i = sc->idx;
        for (int a = 0; a < 3; ++a) out[a] = sc->omq * p[i + a * sh] + sc->q * p[i + a * sh + 1];
    } else {
        int s = 10 * sc->idx;
        for (int a = 0; a < 3; ++a) {
            const float* pp = p + s + 4 * a;
            float phi = 0.5f * (((pp[2] - pp[1]) / 1.0f) + ((pp[1] - pp[0]) / 1.0f));
            float phin = 0.5f * (((pp[3] - pp[2]) / 1.0f) + ((pp[2] - pp[1]) / 1.0f));
            out[a] = sc->a * pp[1] + sc->b * phi + sc->c * pp[2] + sc->d * phin;
        }
    }
    (void)n_step;
}

/* decode + gravity compensation + mask + clip (NMPC:364-420, :270-314) */
static void forces(const oracle_cfg* cfg, const float* params, const step_coef* sc, const float c[4], float F[12]) {
    int PL = num_params_leg(cfg);
    float ns = c[0] + c[1] + c[2] + c[3];
    float fref = cfg->mg / ns;
    const float rx = 3.0f, ry = 3.0f;
    for (int leg = 0; leg < 4; ++leg) {
        float f[3];
        decode_leg(cfg, params + leg * PL, sc, 0, f);
        float fz = fref + f[2];
        float fx = f[0] * c[leg] / rx;
        float fy = f[1] * c[leg] / ry;
        fz = fz * c[leg];
        fz = (fz > cfg->grf_min) ? fz : cfg->grf_min;
        fz = (fz < cfg->grf_max) ? fz : cfg->grf_max;
        float lo = (-cfg->mu) * fz, hi = cfg->mu * fz;
        fx = (fx > lo) ? fx : lo;
        fx = (fx < hi) ? fx : hi;
        fy = (fy > lo) ? fy : lo;
        fy = (fy < hi) ? fy : hi;
        F[3 * leg] = fx;
        F[3 * leg + 1] = fy;
        F[3 * leg + 2] = fz;
    }
}

static const float QD[24] = {0, 0, 1500, 200, 200, 200, 500, 500, 0, 20, 20, 50, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};

/* One rollout (NMPC:316-496); params: P floats */
static float rollout_one(const oracle_cfg* cfg, const float Iinv[9], const step_coef* coefs, const float* state,
                         const float* ref, const float* contact, int stride, const float* params) {
    float x[24];
    memcpy(x, state, sizeof(x));
    float cost = 0.0f;
    for (int n = 0; n < cfg->H; ++n) {
        float c[4] = {contact[n], contact[stride + n], contact[2 * stride + n], contact[3 * stride + n]}, F[12];
        forces(cfg, params, &coefs[n], c, F);
        integrate(cfg, Iinv, x, F, c, cfg->dts[n]);
        float acc = 0.0f;
        for (int i = 0; i < 24; ++i) {
            float e = x[i] - ref[i];
            float t = (e * QD[i]) * e;
            acc = (i == 0) ? t : acc + t;
        }
        cost = cost + acc;
    }
    return cost;
}

int srbd_oracle_num_params(const oracle_cfg* cfg) { return 4 * num_params_leg(cfg); }

/* costs[k] for params = best + noise[k] (noise row-major N x P); unsaturated. */
int srbd_oracle_rollout_costs(const oracle_cfg* cfg, const float* state, const float* ref, const float* contact,
                              int stride, const float* best, const float* noise, int N, float* costs, int nthreads) {
    int P = srbd_oracle_num_params(cfg);
    if (cfg->H > OR_MAXH || P > OR_MAXP) return -1;
    float Iinv[9];
    inv3(cfg->inertia, Iinv);
    step_coef coefs[OR_MAXH];
    for (int n = 0; n < cfg->H; ++n) coefs[n] = make_coef(cfg, (float)n, cfg->H);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (int k = 0; k < N; ++k) {
        float p[OR_MAXP];
        for (int j = 0; j < P; ++j) p[j] = best[j] + noise[(size_t)k * P + j];
        costs[k] = rollout_one(cfg, Iinv, coefs, state, ref, contact, stride, p);
    }
    (void)nthreads;
    return 0;
}

/* Final GRF + predicted state at step 0 (NMPC:695-784) */
int srbd_oracle_final(const oracle_cfg* cfg, const float* state, const float* contact, int stride, const float* best,
                      float grf[12], float pred[24]) {
    float Iinv[9];
    inv3(cfg->inertia, Iinv);
    step_coef sc = make_coef(cfg, 0.0f, 1);
    float c[4] = {contact[0], contact[stride], contact[2 * stride], contact[3 * stride]};
    forces(cfg, best, &sc, c, grf);
    memcpy(pred, state, 24 * sizeof(float));
    integrate(cfg, Iinv, pred, grf, c, cfg->dts[0]);
    return 0;
}

/* ------------------------------------------------------------ Philox RNG */
static inline uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t* hi) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    *hi = (uint32_t)(p >> 32);
    return (uint32_t)p;
}

void srbd_oracle_philox(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3], k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        uint32_t hi0, hi1;
        uint32_t lo0 = mulhilo(0xD2511F53u, c0, &hi0);
        uint32_t lo1 = mulhilo(0xCD9E8D57u, c2, &hi1);
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
    }
    out[0] = c0;
    out[1] = c1;
    out[2] = c2;
    out[3] = c3;
}

static inline float u01(uint32_t x) { return ((float)(x >> 8) + 0.5f) * 5.9604644775390625e-08f; /* 2^-24 */ }

/* Standard normal / uniform draw (d, j) for key (seed) and stream counter (ctr). */
static void draw(uint64_t seed, uint64_t ctr, uint32_t d, uint32_t j, float* z, float* u) {
    uint32_t in[4] = {d, j >> 2, (uint32_t)ctr, (uint32_t)(ctr >> 32)}, key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)},
             o[4];
    srbd_oracle_philox(in, key, o);
    uint32_t q = j & 3u, base = q & 2u;
    float ua = u01(o[base]), ub = u01(o[base + 1]);
    float r = sqrtf(-2.0f * logf(ua));
    /* sin/cos(pi * 2ub): the device uses sincospif(2ub); evaluated here in double, rounded once */
    double th = 3.14159265358979323846 * (double)(2.0f * ub);
    *z = (q & 1u) ? r * (float)sin(th) : r * (float)cos(th);
    *u = u01(o[q]);
}

/* additional_random_parameters (N x P row-major) as the product RNG defines them. */
int srbd_oracle_gen_noise(const oracle_cfg* cfg, uint64_t seed, uint64_t ctr, const float* sigma, float* noise) {
    int N = cfg->N, P = srbd_oracle_num_params(cfg), t = N / 3;
    memset(noise, 0, sizeof(float) * (size_t)P);
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int r = 1; r < N; ++r) {
        for (int j = 0; j < P; ++j) {
            float z, u, v;
            if (cfg->method == 0) {
                if (r <= t) {
                    draw(seed, ctr, (uint32_t)(r - 1), (uint32_t)j, &z, &u);
                    v = cfg->sigma_rs[0] * z;
                } else if (r <= 2 * t) {
                    draw(seed, ctr, (uint32_t)(r - 1 - t), (uint32_t)j, &z, &u);
                    v = cfg->sigma_rs[1] * z;
                } else {
                    draw(seed, ctr, (uint32_t)(r - 1 - 2 * t), (uint32_t)j, &z, &u);
                    v = u * (2.0f * cfg->sigma_rs[2]) - cfg->sigma_rs[2];
                }
            } else {
                draw(seed, ctr, (uint32_t)(r - 1), (uint32_t)j, &z, &u);
                v = (cfg->method == 1) ? cfg->sigma_mppi * z : z * sigma[j];
            }
            noise[(size_t)r * P + j] = v;
        }
    }
    return 0;
}

/* Full MPPI/RS/CEM step on the CPU (used as the cpu_baseline workload).
 * noise: N x P scratch (generated here when gen != 0).  Outputs best (in/out), grf, pred, sigma (CEM). */
int srbd_oracle_step(const oracle_cfg* cfg, const float* state, const float* ref, const float* contact, int stride,
                     float* best, float* sigma, int gen, uint64_t seed, uint64_t ctr, float* noise, float* costs,
                     float grf[12], float pred[24], float* best_cost, int32_t* best_idx, int nthreads) {
    int N = cfg->N, P = srbd_oracle_num_params(cfg);
    if (gen) srbd_oracle_gen_noise(cfg, seed, ctr, sigma, noise);
    int rc = srbd_oracle_rollout_costs(cfg, state, ref, contact, stride, best, noise, N, costs, nthreads);
    if (rc) return rc;
    int bi = 0;
    for (int k = 0; k < N; ++k) {
        float c = costs[k];
        if (isnan(c) || isinf(c)) c = 1000000.0f;
        costs[k] = c;
        if (c < costs[bi]) bi = k;
    }
    float beta = costs[bi];
    if (cfg->method == 0) {
        for (int j = 0; j < P; ++j) best[j] = best[j] + noise[(size_t)bi * P + j];
    } else {
        double* acc = (double*)calloc((size_t)P, sizeof(double));
        float denom = 0.0f;
        for (int k = 0; k < N; ++k) denom += expf(-1.0f * (costs[k] - beta));
        for (int k = 0; k < N; ++k) {
            float w = expf(-1.0f * (costs[k] - beta)) / denom;
            if (w == 0.0f) continue;
            for (int j = 0; j < P; ++j) acc[j] += (double)(w * noise[(size_t)k * P + j]);
        }
        for (int j = 0; j < P; ++j) best[j] = best[j] + (float)acc[j];
        free(acc);
        if (cfg->method == 2 && sigma) {
            /* stable top-10 by (cost, index) */
            int idx[10], ne = N < 10 ? N : 10;
            for (int e = 0; e < ne; ++e) {
                int b = -1;
                for (int k = 0; k < N; ++k) {
                    int used = 0;
                    for (int q = 0; q < e; ++q) used |= (idx[q] == k);
                    if (used) continue;
                    if (b < 0 || costs[k] < costs[b]) b = k;
                }
                idx[e] = b;
            }
            for (int j = 0; j < P; ++j) {
                float m = 0.0f, v = 0.0f;
                for (int e = 0; e < ne; ++e) m += noise[(size_t)idx[e] * P + j];
                m = m / (float)ne;
                for (int e = 0; e < ne; ++e) {
                    float d = noise[(size_t)idx[e] * P + j] - m;
                    v += d * d;
                }
                v = v / (float)(ne - 1);
                float s = sqrtf(v + 1e-8f);
                s = (s > 5.0f) ? 5.0f : s;
                s = (s < 0.2f) ? 0.2f : s;
                sigma[j] = s;
            }
        }
    }
    *best_cost = beta;
    *best_idx = bi;
    return srbd_oracle_final(cfg, state, contact, stride, best, grf, pred);
}
