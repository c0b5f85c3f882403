// srbd_core.h -- float32 SRBD math shared by the CDNA4 kernels and the host-side
// merge (compiled by hipcc for both).  Every function follows the reference's
// float32 evaluation order (JAX, x64 off); the build uses -ffp-contract=off so
// no multiply-add is fused unless written as an explicit fmaf.
//
// Reference (paths relative to the reference repository root):
//   CMJ  = quadruped_pympc/controllers/sampling/centroidal_model_jax.py
//   NMPC = quadruped_pympc/controllers/sampling/centroidal_nmpc_jax.py
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/srbd_mpc.h"

#define SRBD_HD __host__ __device__ __forceinline__

namespace srbd {

constexpr int MAXH = SRBD_MAX_HORIZON;
constexpr int MAXP = SRBD_MAX_PARAMS;
constexpr int MAXK = SRBD_MAX_ELITE;
constexpr int REC_HDR = 4;
constexpr int MAX_TAIL = 48;  // 4 legs x 3 axes x 4 cubic control points

// Per-context constants, passed to every kernel by value (kernarg segment -> SGPRs).
struct ModelConst {
    int H, P, PL, kind, S, method, K;
    int N, n_local, row0, ldn;
    // reduction tree (tree_shape): global leaves, depth, the exchange level and its node count, the world size,
    // this rank's first global leaf and its leaf count
    int t_leaves, t_depth, t_xlevel, t_xnodes, t_xmax, t_world, leaf0, nleaf;
    float inv_m, mg, grf_min, grf_max, mu, neg_mu;
    float inertia[9], Iinv[9];
    float Q[12];
    float dts[MAXH];
    // rollout spline coefficients at step n (horizon_leg = H), NMPC:181-257
    int sidx[MAXH];
    float sq[MAXH], somq[MAXH], sa[MAXH], sb[MAXH], sc[MAXH], sd[MAXH];
    // final decode at step 0.0, horizon_leg 1 (NMPC:706-710)
    int fidx;
    float fq, fomq, fa, fb, fc, fd;
    float sigma_mppi, sigma_rs[3];
    // gait-adaptive sampling (srbd_set_gait): on/off, float32(mg) / n_stance for n_stance = 0..4
    // (GA:385; inf at 0), and the device array of injected per-row step frequencies (ldn entries)
    int ga;
    float fz_ns[5];
    const float* ga_freq;
    // columns the final decode reads (decode_leg at step 0.0, horizon_leg 1): in the column-split
    // merge the tail block computes and owns them (list + bit mask)
    int ntail;
    short tailc[MAX_TAIL];
    uint32_t tailmask[MAXP / 32];
    // opt-in cost terms (srbd_set_cost_terms); cost_on == 0: the reference's cost, terms skipped
    int cost_on;
    float cost_r[3], cost_smooth, cost_cone;
    // device noise stream (srbd_set_rng): RNG_PHILOX (Philox4x32-10, keyed by (seed, counter)) or the
    // reference's jax.random stream (RNG_JAX / RNG_JAX_LEGACY, keyed by the packed key `seed`; srbd_jaxrng.h)
    int rng;
};
SRBD_HD bool is_tail_col(const ModelConst& mc, int j) { return (mc.tailmask[j >> 5] >> (j & 31)) & 1u; }

constexpr int GA_MAXCB = 33;  // chunk boundaries of S <= 32 splines

// Per-step inputs: one pinned host copy -> one H2D per step.
struct StepInput {
    float state[24];
    float ref[24];
    float contact[4][MAXH];
    float fzref[MAXH];  // float32(mass*9.81) / n_stance(n)   (NMPC:377-380)
    float cost_feet;    // sum over feet of (e*0)*e: 0, or NaN when a foot error is not finite
    uint32_t seed_lo, seed_hi, ctr_lo, ctr_hi;
    int32_t noise_scaled;  // 0: noise holds unscaled CEM draws (device RNG), multiply by sigma on read
    // gait-adaptive sampling (srbd_set_gait): leg phases, PGG dt and duty factor, the per-call
    // frequency set, injected (1) or device-drawn (0) frequencies, and per chunk boundary i the
    // smallest integer step with step >= float32(linspace(0, H, S+1)[i]) (GA:196)
    int32_t ga_nfreq, ga_explicit;
    float ga_timing[4];
    float ga_dt, ga_duty;
    float ga_freqs[SRBD_MAX_FREQS];
    int32_t ga_cb[GA_MAXCB];
    int32_t pad[1];
    float best[MAXP];
    float sigma[MAXP];
};

static_assert(sizeof(StepInput) % 16 == 0 && offsetof(StepInput, best) % 16 == 0 &&
                  offsetof(StepInput, sigma) % 16 == 0,
              "StepInput is copied in 16-byte words (P is a multiple of 12, so P floats are too)");

// A column-split merge's in-launch hand-off (merge_body), in device memory right after the context's StepInput
// (d_in is allocated STEP_INPUT_ALLOC bytes): the slices' root sums of their columns and the weights' sum for the
// tail block, the tail block's top-K keys for the slices.  Every word is stored once per launch as one 8-byte
// atomic, tagged with the launch's epoch + 1 in its high half, so a reader polls the word itself (one memory
// round trip, no flag behind the data); the tail block advances the epoch once it holds every slice's sums (every
// slice read the epoch before storing them).
struct SplitXchg {
    uint32_t epoch;
    uint32_t drop;  // tests (srbd_debug_split_drop): != 0 makes slice 1 withhold a word; cleared by the reset
    uint32_t pad[2];
    uint64_t elite[2 * MAXK];  // the top-K keys' low and high halves
    uint64_t sums[MAXP + 1];   // column j: sum_r scale_r v_r[j]; [P]: sum_r scale_r s_r (float bits)
};
constexpr size_t STEP_INPUT_ALLOC = sizeof(StepInput) + sizeof(SplitXchg);

// A host step's input passed by value as a kernel argument (KS rollout launches, srbd_step): StepInput's
// prefix up to best[KSI_MAXP] -- no sigma, so MPPI / random sampling only.  The launch's block 0 writes it to
// the device StepInput, which the merge and any later reader use; no upload kernel runs.
constexpr int KSI_MAXP = 192;
struct StepInputK {
    unsigned char head[offsetof(StepInput, best)];
    float best[KSI_MAXP];
};
static_assert(offsetof(StepInputK, best) == offsetof(StepInput, best) && sizeof(StepInputK) % 16 == 0,
              "StepInputK is StepInput's prefix, copied in 16-byte words");
struct KsNone {  // the kernel argument of launches that read the device StepInput
    int unused;
};

struct StepOutput {
    float best[MAXP];
    float sigma[MAXP];
    float grf[12];
    float pred[24];
    float best_cost;
    int32_t best_index;
    int32_t status;
    float best_freq;  // gait-adaptive: step frequency of the best row
};

// Record strides are padded to whole 16-byte words, so a merge block can stage a run of records into
// LDS with dwordx4 loads (merge_body<true>); the padding floats are never read as values.
SRBD_HD int rec_pad4(int n) { return (n + 3) & ~3; }
SRBD_HD int rec_floats_wave(int P, int K) { return rec_pad4(REC_HDR + P + 2 * K); }
SRBD_HD int rec_floats_rank(int P, int K) { return rec_pad4(REC_HDR + P + 2 * K + K * P); }
SRBD_HD int num_elite(int method, int num_elite_cfg) { return method == SRBD_CEM_MPPI ? num_elite_cfg : 1; }

// ---- The reduction tree of one MPC step (MPPI / CEM weighted sums, random-sampling / CEM keys), fixed by global
// rows alone -- the same for every rollout form and every rank count W, so 1-GPU and W-GPU steps give the same
// bits.  A leaf is LEAF_ROWS consecutive global rows; its record holds m = its minimum cost, s = sum of
// e_i = exp(-(c_i - m)) and v[j] = sum of e_i noise_i[j], each sum in the DPP order of wave_sum_f32 over the 64
// rows (row i in lane i; rows past N contribute 0), and its K smallest (cost, row) keys.  Above the leaves every
// node folds up to TREE_FAN consecutive children in order: m = the children's minimum, scale_c = exp(-(m_c - m))
// (1 for random sampling), s = sum_c scale_c s_c and v[j] = sum_c scale_c v_c[j] summed child by child, keys =
// the K smallest of the children's.  The root's sums give the update v / s (centroidal_nmpc_jax.py:828-836).
// Level-d nodes cover LEAF_ROWS * TREE_FAN^d rows.  A W-rank problem is split at whole nodes of its exchange
// level X: rank r holds nodes [r xmax, (r + 1) xmax) (the last rank fewer), so the ranks' level-X node records
// gathered in rank order are the level's node list, and every rank folds that list to the root the same way.
constexpr int LEAF_ROWS = 64;
constexpr int TREE_FAN = 32;
SRBD_HD int tree_nodes(int leaves, int d) {  // ceil(leaves / TREE_FAN^d)
    int n = leaves;
    for (int i = 0; i < d; ++i) n = (n + TREE_FAN - 1) / TREE_FAN;
    return n;
}
SRBD_HD int tree_depth(int leaves) {  // the root level D: tree_nodes(leaves, D) == 1
    int d = 0;
    while (tree_nodes(leaves, d) > 1) ++d;
    return d;
}
SRBD_HD long long tree_node_rows(int d) {  // rows of a level-d node
    long long r = LEAF_ROWS;
    for (int i = 0; i < d; ++i) r *= TREE_FAN;
    return r;
}
struct TreeShape {
    int leaves, depth, xlevel, xnodes, xmax;  // xmax: level-X nodes per rank (the last rank may hold fewer)
    int node0, nnodes;                        // this rank's level-X nodes
    long long row0, nrows;                    // this rank's rows
    bool ok;                                  // every rank holds at least one node
};
// N rows over `world` ranks, rank `rank`'s share.  X: the highest level at which every rank gets at least one node
// and the largest rank share (ceil(nodes / W) nodes) is within 1/8 of the smallest largest share any level allows
// (world 1: the root level, one node holding everything).  Only the levels the ranks fold to and exchange move with
// X; the tree and so the bits do not.  Without the balance test, N just past a node boundary gave one rank nearly
// all the rows (N = 70 001, W = 2: 65 536 and 4 465 rows at level 2; 36 864 and 33 137 at level 1).
SRBD_HD long long tree_share(int leaves, long long N, int world, int x) {  // largest rank share at level x, 0: invalid
    const int n = tree_nodes(leaves, x), per = (n + world - 1) / world;
    if ((long long)(world - 1) * per >= n) return 0;
    const long long r = (long long)per * tree_node_rows(x);
    return r < N ? r : N;
}
SRBD_HD TreeShape tree_shape(long long N, int world, int rank) {
    TreeShape t;
    t.leaves = (int)((N + LEAF_ROWS - 1) / LEAF_ROWS);
    t.depth = tree_depth(t.leaves);
    long long best = 0;
    for (int l = 0; l <= t.depth; ++l) {
        const long long s = tree_share(t.leaves, N, world, l);
        if (s > 0 && (best == 0 || s < best)) best = s;
    }
    int x = t.depth;
    for (; x > 0; --x) {
        const long long s = tree_share(t.leaves, N, world, x);
        if (s > 0 && 8 * s <= 9 * best) break;
    }
    t.xlevel = x;
    t.xnodes = tree_nodes(t.leaves, x);
    t.xmax = (t.xnodes + world - 1) / world;
    t.ok = (long long)(world - 1) * t.xmax < t.xnodes;
    t.node0 = rank * t.xmax < t.xnodes ? rank * t.xmax : t.xnodes;
    const int e = (rank + 1) * t.xmax < t.xnodes ? (rank + 1) * t.xmax : t.xnodes;
    t.nnodes = e - t.node0;
    const long long nr = tree_node_rows(x);
    t.row0 = (long long)t.node0 * nr;
    const long long end = (long long)e * nr;
    t.nrows = (end < N ? end : N) - t.row0;
    if (t.nrows < 0) t.nrows = 0;
    return t;
}

SRBD_HD uint32_t f2u(float f) {
    union { float f; uint32_t u; } x;
    x.f = f;
    return x.u;
}
SRBD_HD float u2f(uint32_t u) {
    union { float f; uint32_t u; } x;
    x.u = u;
    return x.f;
}
// Sort key of a (saturated, non-negative) cost and its global row: ascending key order is
// ascending cost, ties by ascending row == jnp.nanargmin / stable jnp.argsort order.
SRBD_HD uint64_t cost_key(float c, uint32_t row) {
    return ((uint64_t)f2u(c + 0.0f) << 32) | (uint64_t)row;
}

// Correctly rounded x / d given r = RN(1/d) (Markstein): q0 = RN(x r), rem = x - q0 d (exact,
// fma), q = RN(q0 + rem r).  Equal to IEEE x / d for finite normal operands (tested in
// tests/test_gpu_parity.py::test_division and test_host_logic.py).
SRBD_HD float div_by(float x, float d, float r) {
    float q0 = x * r;
    float rem = fmaf(-q0, d, x);
    return fmaf(rem, r, q0);
}

constexpr float THIRD = 0.3333333432674407958984375f;  // RN(1/3)
SRBD_HD float div3(float x) { return div_by(x, 3.0f, THIRD); }

// ---- rollout arithmetic (round 3): the reference's float32 operations in its order, except that
// the three operations with a long correctly rounded sequence take their hardware forms, each within
// a few ulp of the IEEE result (the parity contract is the tolerance against the C oracle, SURVEY
// 8(c); every kernel -- thread, four-lane, gait-adaptive, merge tail -- calls these same helpers, so
// the layouts still agree bit for bit):
//   x / 3            -> x * RN(1/3)                       (<= 1 ulp)
//   1 / d            -> v_rcp_f32                         (<= 1 ulp)
//   sin(x), cos(x)   -> v_sin_f32 / v_cos_f32 of x / 2pi  (revolutions; no range reduction)
// Measured on the C2 four-lane rollout: 262 -> see DESIGN.md VALU instructions per lane-step.
SRBD_HD float third(float x) { return x * THIRD; }
SRBD_HD float rcp_(float d) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_rcpf(d);
#else
    return 1.0f / d;
#endif
}

// CMJ:67-91, entries divided by DET (IEEE reciprocal once, then Markstein per entry; falls back
// to plain division when DET is not a comfortably normal number).
SRBD_HD void inv3(const float A[9], float out[9]) {
    const float a11 = A[0], a12 = A[1], a13 = A[2], a21 = A[3], a22 = A[4], a23 = A[5], a31 = A[6], a32 = A[7],
                a33 = A[8];
    const float DET = a11 * (a33 * a22 - a32 * a23) - a21 * (a33 * a12 - a32 * a13) + a31 * (a23 * a12 - a22 * a13);
    const float M[9] = {(a33 * a22 - a32 * a23),  -(a33 * a12 - a32 * a13), (a23 * a12 - a22 * a13),
                        -(a33 * a21 - a31 * a23), (a33 * a11 - a31 * a13),  -(a23 * a11 - a21 * a13),
                        (a32 * a21 - a31 * a22),  -(a32 * a11 - a31 * a12), (a22 * a11 - a21 * a12)};
    const float ad = fabsf(DET);
    if (ad > 1e-30f && ad < 1e30f) {
        const float r = 1.0f / DET;
#pragma unroll
        for (int i = 0; i < 9; ++i) out[i] = div_by(M[i], DET, r);
    } else {
#pragma unroll
        for (int i = 0; i < 9; ++i) out[i] = M[i] / DET;
    }
}

SRBD_HD void mv3(const float M[9], const float v[3], float o[3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = M[3 * i] * v[0] + M[3 * i + 1] * v[1] + M[3 * i + 2] * v[2];
}

// jnp.dot(skew(v), f) (CMJ:100-101).  The reference's 0*f terms are dropped: f and v are finite
// here (forces are clipped; rows of non-finite states saturate to 1e6 either way), so only the
// sign of an exact zero can differ.
SRBD_HD void skew_dot(const float v[3], const float f[3], float o[3]) {
    o[0] = (-v[2]) * f[1] + v[1] * f[2];
    o[1] = v[2] * f[0] + (-v[0]) * f[2];
    o[2] = (-v[1]) * f[0] + v[0] * f[1];
}

constexpr float INV_2PI = 0.15915493667125701904296875f;  // RN(1/(2 pi))
SRBD_HD void sincos_(float x, float* s, float* c) {
#ifdef __HIP_DEVICE_COMPILE__
    const float t = x * INV_2PI;  // revolutions (v_sin/v_cos domain |t| <= 256: |x| <= 1608 rad)
    *s = __builtin_amdgcn_sinf(t);
    *c = __builtin_amdgcn_cosf(t);
#else
    *s = sinf(x);
    *c = cosf(x);
#endif
}

// Row c of calculate_inverse(conj) (CMJ:67-91 applied to CMJ:126-132) times omega.  conj has the
// constant entries a11 = 1, a12 = a21 = a31 = 0, so the reference's cofactor expression reduces to
//   DET = a33*a22 - a32*a23,  row0 = [1, a32*a13, -(a22*a13)]/DET,  row1 = [0, a33, -a23]/DET,
//   row2 = [0, -a32, a22]/DET
// with identical values (only the sign of an exact zero can differ, which cannot change a cost).
SRBD_HD void euler_rate_coefs(int c, float sr, float cr, float sp, float cp, float& k1, float& k2) {
    const float a13 = -sp, a22 = cr, a23 = cp * sr, a32 = -sr, a33 = cp * cr;
    const float DET = a33 * a22 - a32 * a23;
    const float n1 = c == 0 ? a32 * a13 : (c == 1 ? a33 : -a32);
    const float n2 = c == 0 ? -(a22 * a13) : (c == 1 ? -a23 : a22);
    const float r = rcp_(DET);  // |DET| >= |cos(pitch)| / 2 >= 8e-10: see euler_rates
    k1 = n1 * r;
    k2 = n2 * r;
}

SRBD_HD float euler_rate_row(int c, float k1, float k2, float w0, float w1, float w2) {
    return (c == 0 ? w0 + k1 * w1 : k1 * w1) + k2 * w2;
}

SRBD_HD void euler_rates(float sr, float cr, float sp, float cp, float w0, float w1, float w2, float er[3]) {
    const float a13 = -sp, a22 = cr, a23 = cp * sr, a32 = -sr, a33 = cp * cr;
    const float DET = a33 * a22 - a32 * a23;
    const float n[6] = {a32 * a13, -(a22 * a13), a33, -a23, -a32, a22};
    // n / DET as n * rcp(DET) (rcp_: <= 1 ulp; the product <= 2 ulp from the IEEE quotient).  1/DET
    // stays normal: DET = cp (cr^2 + sr^2), so |DET| >= |cos(pitch)| / 2, and over every finite
    // float32 pitch |cos| >= 1.6e-9 (exhaustive search, attained at 7.73e28); a non-finite angle
    // makes DET NaN, and NaN propagates to the cost either way.
    float k[6];
    const float r = rcp_(DET);
#pragma unroll
    for (int i = 0; i < 6; ++i) k[i] = n[i] * r;
    er[0] = euler_rate_row(0, k[0], k[1], w0, w1, w2);
    er[1] = euler_rate_row(1, k[2], k[3], w0, w1, w2);
    er[2] = euler_rate_row(2, k[4], k[5], w0, w1, w2);
}

// Model constants as the rollout reads them (the KC template parameter of integrate_k / clip_leg_k / shape_leg_k).
struct McConst {
    const ModelConst& m;
    SRBD_HD float inv_m() const { return m.inv_m; }
    SRBD_HD const float* inertia() const { return m.inertia; }
    SRBD_HD const float* Iinv() const { return m.Iinv; }
    SRBD_HD float grf_min() const { return m.grf_min; }
    SRBD_HD float grf_max() const { return m.grf_max; }
    SRBD_HD float mu() const { return m.mu; }
    SRBD_HD float neg_mu() const { return m.neg_mu; }
};

// Centroidal_Model_JAX.fd + integrate_jax (CMJ:93-174).  x: 12 evolving states, feet: 12
// (constant over the rollout), F: 12 clipped foot forces, c: 4 contact flags.
// The rigid-body part of the step, from the contact-weighted force sum temp = sum_i f_i c_i and torque sum
// temp2 = sum_i (p_i - p_com) x f_i c_i (integrate_k forms both).
template <class KC>
SRBD_HD void integrate_rb_k(const KC& kc, float x[12], const float temp[3], const float temp2[3], float dt) {
    float lin_acc[3];
    const float inv_m = kc.inv_m();
    lin_acc[0] = inv_m * temp[0] + 0.0f;
    lin_acc[1] = inv_m * temp[1] + 0.0f;
    lin_acc[2] = inv_m * temp[2] + (-9.81f);

    float sr, cr, sp, cp, sy, cy;
    sincos_(x[6], &sr, &cr);
    sincos_(x[7], &sp, &cp);
    sincos_(x[8], &sy, &cy);

    float er[3];
    euler_rates(sr, cr, sp, cp, x[9], x[10], x[11], er);

    const float R[9] = {cp * cy, cp * sy, -sp,
                        sr * sp * cy - cr * sy, sr * sp * sy + cr * cy, sr * cp,
                        cr * sp * cy + sr * sy, cr * sp * sy - sr * cy, cr * cp};
    float Iw[3], wxIw[3], a1[3], Rt[3], a2[3];
    mv3(kc.inertia(), x + 9, Iw);
    skew_dot(x + 9, Iw, wxIw);
    mv3(kc.Iinv(), wxIw, a1);
    mv3(R, temp2, Rt);
    mv3(kc.Iinv(), Rt, a2);

    const float d[12] = {x[3],  x[4],  x[5],  lin_acc[0],    lin_acc[1],    lin_acc[2],
                         er[0], er[1], er[2], -a1[0] + a2[0], -a1[1] + a2[1], -a1[2] + a2[2]};
#pragma unroll
    for (int k = 0; k < 12; ++k) x[k] = x[k] + d[k] * dt;
}
// (p_i - p_com) x f_i * c_i of one leg (CMJ:100-101).
SRBD_HD void leg_torque(const float foot[3], const float x[3], const float f[3], float c, float tc[3]) {
    const float v[3] = {foot[0] - x[0], foot[1] - x[1], foot[2] - x[2]};
    float t[3];
    skew_dot(v, f, t);
#pragma unroll
    for (int k = 0; k < 3; ++k) tc[k] = t[k] * c;
}
template <class KC>
SRBD_HD void integrate_k(const KC& kc, float x[12], const float feet[12], const float F[12], const float c[4],
                         float dt) {
    // leg sums pairwise, (leg0 + leg1) + (leg2 + leg3): the four-lane kernel forms them with one quad
    // butterfly over leg-parallel lanes (rollout_quad_kernel), and every layout uses this order
    float temp[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) temp[k] = (F[k] * c[0] + F[3 + k] * c[1]) + (F[6 + k] * c[2] + F[9 + k] * c[3]);
    float tc[4][3];  // (p_i - p_com) x f_i * c_i per leg
#pragma unroll
    for (int i = 0; i < 4; ++i) leg_torque(feet + 3 * i, x, F + 3 * i, c[i], tc[i]);
    float temp2[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) temp2[k] = (tc[0][k] + tc[1][k]) + (tc[2][k] + tc[3][k]);
    integrate_rb_k(kc, x, temp, temp2, dt);
}
SRBD_HD void integrate(const ModelConst& mc, float x[12], const float feet[12], const float F[12], const float c[4],
                       float dt) {
    integrate_k(McConst{mc}, x, feet, F, c, dt);
}

// NMPC:270-314: where(x > lo, x, lo) then where(x < hi, x, hi), so a NaN becomes the lower bound.
// On the device this is one v_med3_f32: with lo <= hi it is the clamp, and with a NaN operand
// gfx9's med3 returns min3(x, lo, hi) = lo, the reference's result.  Only the sign of an exact
// zero can differ from the two compare-selects (no cost or force value does).  lo <= hi holds
// because build_model requires 0 <= grf_min <= grf_max and mu >= 0.
SRBD_HD float clamp_cs(float x, float lo, float hi) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_fmed3f(x, lo, hi);
#else
    x = (x > lo) ? x : lo;
    return (x < hi) ? x : hi;
#endif
}

template <class KC>
SRBD_HD void clip_leg_k(const KC& kc, float& fx, float& fy, float& fz) {
    fz = clamp_cs(fz, kc.grf_min(), kc.grf_max());
    const float lo = kc.neg_mu() * fz, hi = kc.mu() * fz;
    fx = clamp_cs(fx, lo, hi);
    fy = clamp_cs(fy, lo, hi);
}
SRBD_HD void clip_leg(const ModelConst& mc, float& fx, float& fy, float& fz) { clip_leg_k(McConst{mc}, fx, fy, fz); }

// Gravity compensation + contact mask (NMPC:377-402), then clip.
template <class KC>
SRBD_HD void shape_leg_k(const KC& kc, float fref, float c, float& fx, float& fy, float& fz) {
    fz = fref + fz;
    fx = third(fx * c);
    fy = third(fy * c);
    fz = fz * c;
    clip_leg_k(kc, fx, fy, fz);
}
SRBD_HD void shape_leg(const ModelConst& mc, float fref, float c, float& fx, float& fy, float& fz) {
    shape_leg_k(McConst{mc}, fref, c, fx, fy, fz);
}

// Opt-in cost terms of one step n (srbd_set_cost_terms), thread-per-sample layout: per component q
// (x, y, z), leg by leg in order, (u r_q) u + (d w_smooth) d [n >= 1] + (v w_cone) v [q = x, y] with
// u = f_q (z: f_z - fref for a stance leg), d = f_q - f_q(step n-1), v = max(0, |f_q before the
// clip| - mu f_z); the component's sum joins cost3[q] after its tracking term.  F: clipped forces,
// RX / RY: each leg's decoded x / y.  The four-lane kernel forms the same terms in the same order.
SRBD_HD void extra_cost_step(const ModelConst& mc, int n, const float F[12], const float RX[4], const float RY[4],
                             const float c[4], float fref, float Fprev[12], float cost3[3]) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        float e = 0.0f;
#pragma unroll
        for (int leg = 0; leg < 4; ++leg) {
            const float f = F[3 * leg + q];
            const float u = q == 2 ? f - (c[leg] != 0.0f ? fref : 0.0f) : f;
            float term = (u * mc.cost_r[q]) * u;
            if (n > 0) {
                const float d = f - Fprev[3 * leg + q];
                term = term + (d * mc.cost_smooth) * d;
            }
            if (q < 2) {
                const float pre = third((q == 0 ? RX[leg] : RY[leg]) * c[leg]);
                float v = fabsf(pre) - mc.mu * F[3 * leg + 2];
                v = v > 0.0f ? v : 0.0f;
                term = term + (v * mc.cost_cone) * v;
            }
            e = e + term;
        }
        cost3[q] = cost3[q] + e;
    }
#pragma unroll
    for (int i = 0; i < 12; ++i) Fprev[i] = F[i];
}

// Spline decode of one leg (NMPC:181-268) with precomputed per-step coefficients.
// `p(j)` returns parameter j of this leg.
template <class Acc>
SRBD_HD void decode_leg(int kind, int H, int S, int idx, float q, float omq, float a, float b, float cc, float d,
                        int n_zero_order, const Acc& p, float& fx, float& fy, float& fz) {
    if (kind == SRBD_ZERO_ORDER) {
        fx = p(n_zero_order);
        fy = p(n_zero_order + H);
        fz = p(n_zero_order + 2 * H);
    } else if (kind == SRBD_LINEAR_SPLINE) {
        const int sh = S + 1;
        fx = omq * p(idx) + q * p(idx + 1);
        fy = omq * p(idx + sh) + q * p(idx + sh + 1);
        fz = omq * p(idx + 2 * sh) + q * p(idx + 2 * sh + 1);
    } else {
        const int s = 10 * idx;
        float o[3];
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) {
            const float p0 = p(s + 4 * ax), p1 = p(s + 4 * ax + 1), p2 = p(s + 4 * ax + 2), p3 = p(s + 4 * ax + 3);
            const float phi = 0.5f * ((p2 - p1) + (p1 - p0));
            const float phin = 0.5f * ((p3 - p2) + (p2 - p1));
            o[ax] = a * p1 + b * phi + cc * p2 + d * phin;
        }
        fx = o[0];
        fy = o[1];
        fz = o[2];
    }
}

// Final GRF decode at step 0 and the predicted state (NMPC:695-784).
SRBD_HD void final_grf_pred(const ModelConst& mc, const StepInput& in, const float* best, float grf[12],
                            float pred[24]) {
    const float c[4] = {in.contact[0][0], in.contact[1][0], in.contact[2][0], in.contact[3][0]};
#pragma unroll
    for (int leg = 0; leg < 4; ++leg) {
        const float* pl = best + leg * mc.PL;
        auto acc = [pl](int j) { return pl[j]; };
        float fx, fy, fz;
        decode_leg(mc.kind, mc.H, mc.S, mc.fidx, mc.fq, mc.fomq, mc.fa, mc.fb, mc.fc, mc.fd, 0, acc, fx, fy, fz);
        shape_leg(mc, in.fzref[0], c[leg], fx, fy, fz);
        grf[3 * leg] = fx;
        grf[3 * leg + 1] = fy;
        grf[3 * leg + 2] = fz;
    }
    float x[12];
    for (int i = 0; i < 12; ++i) x[i] = in.state[i];
    integrate(mc, x, in.state + 12, grf, c, mc.dts[0]);
    for (int i = 0; i < 12; ++i) pred[i] = x[i];
    for (int i = 12; i < 24; ++i) pred[i] = in.state[i];
}

}  // namespace srbd
