// srbd_kernels.hip -- CDNA4 (gfx950) kernels of the sampling SRBD MPC step and the TAMOLS
// foothold search.  Launchers are declared in srbd_launch.h.
//
// Kernels of one MPC step:
//   rng_kernel        Philox4x32-10 + Box-Muller -> additional_random_parameters, SoA [P][ldn]
//   transpose_kernel  parity mode: host noise (row-major N x P) -> SoA
//   rollout_kernel    one thread per sample: spline decode, gravity compensation, contact mask,
//                     friction-cone clip, H explicit-Euler SRBD steps, tracking cost, saturation;
//                     epilogue: per-block (min cost, sum exp, sum exp*noise[P], top-K keys) record
//   merge_kernel      merges block (or rank) records: global argmin, MPPI/CEM softmax-weighted
//                     update, CEM sigma, final GRF decode + predicted state
//   advance_kernel    device-resident warm start for back-to-back steps (benchmark chain)
#include "srbd_device.h"

#include <cstdlib>

namespace srbd {

__global__ void __launch_bounds__(256) rng_kernel(const ModelConst mc, const StepInput* __restrict__ in,
                                                  const RngJob job) {
    if (job.gate && (*job.gate & ARM_CANCEL)) return;  // armed chain that did not fire
    rng_items(mc, in, job, blockIdx.x * 256 + threadIdx.x, gridDim.x * 256);
}

// row-major (n x P) -> SoA [P][ldn]
__global__ void __launch_bounds__(256) transpose_kernel(const float* __restrict__ src, int n, int P, int ldn,
                                                        float* __restrict__ dst) {
    __shared__ float tile[32][33];
    const int bx = blockIdx.x * 32, by = blockIdx.y * 32;  // bx: rows (samples), by: params
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    for (int i = ty; i < 32; i += 8) {
        const int row = bx + i, col = by + tx;
        tile[i][tx] = (row < n && col < P) ? src[(size_t)row * P + col] : 0.0f;
    }
    __syncthreads();
    for (int i = ty; i < 32; i += 8) {
        const int col = by + i, row = bx + tx;
        if (col < P && row < n) dst[(size_t)col * ldn + row] = tile[tx][i];
    }
}

// ---- four lanes per sample: lane c in {0,1,2} owns component c (x, y, z) of every 3-vector of
// the model (forces per leg, torques, p, v, rpy, omega); lane 3 mirrors lane 2.  Cross-lane data
// moves are DPP quad permutations.  Every float operation is the one the thread-per-sample kernel
// performs, in the same order, so both kernels give bitwise identical costs; the 4x wave count
// and ~1.6x shorter per-lane instruction stream cut the latency when N is too small to fill
// the GPU one sample per lane.
constexpr int QP_B0 = 0x00, QP_B1 = 0x55, QP_B2 = 0xAA;  // quad_perm broadcast of lane 0/1/2
constexpr int QP_NEXT = 0x09;   // lanes (0,1,2,3) <- (1,2,0,0): component c+1 (mod 3)
constexpr int QP_NEXT2 = 0x52;  // lanes (0,1,2,3) <- (2,0,1,1): component c+2 (mod 3)
constexpr int QP_XOR1 = 0xB1;   // lanes (0,1,2,3) <- (1,0,3,2)
constexpr int QP_XOR2 = 0x4E;   // lanes (0,1,2,3) <- (2,3,0,1)

#ifndef SRBD_XS
#define SRBD_XS 0  // experiment knob: quad permutations through ds_swizzle (the LDS crossbar) instead of DPP
#endif
#ifndef SRBD_PRIO
#define SRBD_PRIO 0  // experiment knob: s_setprio of the rollout blocks' waves (the draw blocks stay at 0)
#endif
#ifndef SRBD_PRIO_MIN
#define SRBD_PRIO_MIN 0  // ... for launches of at least this many rollout blocks
#endif
template <int CTRL>
__device__ __forceinline__ float qp(float v) {
#if SRBD_XS
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x8000 | CTRL));
#else
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
#endif
}
__device__ __forceinline__ float sel3(int c, float a0, float a1, float a2) { return c == 0 ? a0 : (c == 1 ? a1 : a2); }

// Lane constants of the four-lane layout: lane c in {0,1,2} owns component c, lane 3 mirrors lane 2.
struct QuadLane {
    int c;
    float g, Ir0, Ir1, Ir2, Ii0, Ii1, Ii2;
};
__device__ __forceinline__ QuadLane quad_lane(const ModelConst& mc, int c) {
    QuadLane L;
    L.c = c;
    L.g = c == 2 ? -9.81f : 0.0f;
    L.Ir0 = sel3(c, mc.inertia[0], mc.inertia[3], mc.inertia[6]);
    L.Ir1 = sel3(c, mc.inertia[1], mc.inertia[4], mc.inertia[7]);
    L.Ir2 = sel3(c, mc.inertia[2], mc.inertia[5], mc.inertia[8]);
    L.Ii0 = sel3(c, mc.Iinv[0], mc.Iinv[3], mc.Iinv[6]);
    L.Ii1 = sel3(c, mc.Iinv[1], mc.Iinv[4], mc.Iinv[7]);
    L.Ii2 = sel3(c, mc.Iinv[2], mc.Iinv[5], mc.Iinv[8]);
    return L;
}

// One explicit-Euler step of the single rigid body (Centroidal_Model_JAX.fd + integrate_jax,
// CMJ:93-174) in the four-lane layout, from this lane's component of the contact-weighted force sum
// `temp` = sum_i f_i c_i and torque sum `temp2` = sum_i (p_i - p_com) x f_i c_i.  The float ops and
// their order are those of integrate() in srbd_core.h (rollout_kernel), so both layouts agree bit
// for bit.  All four lanes of each quad must be active (DPP quad permutations).
// Split in two so the merge tail can form the state-only part (rotation, Euler rates, gyroscopic
// term) while the weighted sums are still being reduced: quad_rb_prep needs only r and w,
// quad_rb_apply adds the forces.  quad_rigid_body = apply(prep); the float ops are unchanged.
struct QuadRB {
    float er, R0, R1, R2, a1;
};
__device__ __forceinline__ QuadRB quad_rb_prep(const QuadLane& L, float r, float w) {
    const int c = L.c;
    float sn, cs;
    sincos_(r, &sn, &cs);
    const float sr = qp<QP_B0>(sn), cr = qp<QP_B0>(cs);
    const float sp = qp<QP_B1>(sn), cp = qp<QP_B1>(cs);
    const float sy = qp<QP_B2>(sn), cy = qp<QP_B2>(cs);
    const float w0 = qp<QP_B0>(w), w1 = qp<QP_B1>(w), w2 = qp<QP_B2>(w);
    float k1, k2;
    euler_rate_coefs(c, sr, cr, sp, cp, k1, k2);
    // euler_rate_row, with both operands of every lane select computed first (straight-line code:
    // selects, not divergent branches)
    const float kw1 = k1 * w1;
    const float er0 = w0 + kw1;
    const float er = (c == 0 ? er0 : kw1) + k2 * w2;
    // row c of b_R_w (CMJ:136-150)
    const float A = c == 1 ? sr : cr;
    const float B0 = c == 1 ? -cr : sr, B1 = c == 1 ? cr : -sr;
    const float Asp = A * sp;
    const float r0a = cp * cy, r0b = Asp * cy + B0 * sy;
    const float r1a = cp * sy, r1b = Asp * sy + B1 * cy;
    const float r2b = A * cp;
    const float R0 = c == 0 ? r0a : r0b;
    const float R1 = c == 0 ? r1a : r1b;
    const float R2 = c == 0 ? -sp : r2b;
    const float Iw = L.Ir0 * w0 + L.Ir1 * w1 + L.Ir2 * w2;
    const float wx = (-qp<QP_NEXT2>(w)) * qp<QP_NEXT>(Iw) + qp<QP_NEXT>(w) * qp<QP_NEXT2>(Iw);
    const float a1 = L.Ii0 * qp<QP_B0>(wx) + L.Ii1 * qp<QP_B1>(wx) + L.Ii2 * qp<QP_B2>(wx);
    return QuadRB{er, R0, R1, R2, a1};
}
__device__ __forceinline__ void quad_rb_apply(const ModelConst& mc, const QuadLane& L, const QuadRB& q, float temp,
                                              float temp2, float dt, float& p, float& v, float& r, float& w) {
    const float lin = mc.inv_m * temp + L.g;
    const float Rt = q.R0 * qp<QP_B0>(temp2) + q.R1 * qp<QP_B1>(temp2) + q.R2 * qp<QP_B2>(temp2);
    const float a2 = L.Ii0 * qp<QP_B0>(Rt) + L.Ii1 * qp<QP_B1>(Rt) + L.Ii2 * qp<QP_B2>(Rt);
    const float aa = -q.a1 + a2;
    const float pn = p + v * dt, vn = v + lin * dt, rn = r + q.er * dt, wn = w + aa * dt;
    p = pn;
    v = vn;
    r = rn;
    w = wn;
}
// quad_rb_apply with the torque sum's three components already on every lane (the leg-parallel force phase):
// the same float operations, no broadcasts.
__device__ __forceinline__ void quad_rb_apply3(const ModelConst& mc, const QuadLane& L, const QuadRB& q, float temp,
                                               float t2x, float t2y, float t2z, float dt, float& p, float& v, float& r,
                                               float& w) {
    const float lin = mc.inv_m * temp + L.g;
    const float Rt = q.R0 * t2x + q.R1 * t2y + q.R2 * t2z;
    const float a2 = L.Ii0 * qp<QP_B0>(Rt) + L.Ii1 * qp<QP_B1>(Rt) + L.Ii2 * qp<QP_B2>(Rt);
    const float aa = -q.a1 + a2;
    const float pn = p + v * dt, vn = v + lin * dt, rn = r + q.er * dt, wn = w + aa * dt;
    p = pn;
    v = vn;
    r = rn;
    w = wn;
}
__device__ __forceinline__ void quad_rigid_body(const ModelConst& mc, const QuadLane& L, float temp, float temp2,
                                                float dt, float& p, float& v, float& r, float& w) {
    quad_rb_apply(mc, L, quad_rb_prep(L, r, w), temp, temp2, dt, p, v, r, w);
}

// This lane's component of (p_i - p_com) x f_i (jnp.dot(skew(v), f), CMJ:100-101, zero terms dropped).
__device__ __forceinline__ float quad_cross(float vl, float fl) {
    const float vn1 = qp<QP_NEXT>(vl), vn2 = qp<QP_NEXT2>(vl);
    const float fn1 = qp<QP_NEXT>(fl), fn2 = qp<QP_NEXT2>(fl);
    return (-vn2) * fn1 + vn1 * fn2;
}

// The in-launch final merge of the group records (GroupArgs::out), defined after merge_body.
template <int NT, bool XG>
__device__ void final_merge(const ModelConst& mc, const StepInput* in, const float* noise, int rec_stride,
                            const GroupArgs& grp, float* lds);
// The level-1 fold and the root merge of unsharded host steps with <= TREE_FAN level-1 nodes (GroupArgs::fast),
// defined after merge_body.
__device__ void fast_tail(const ModelConst& mc, const StepInput* in, const float* noise, const float* recs,
                          int rec_stride, const GroupArgs& grp, int nroll, float* st);

// FM: 1 the instantiation with the in-launch final merge (launched when GroupArgs::out is set), 2 with the sharded
// step's exchange too (GroupArgs::xa); the others carry none of its code (C2's launch, which never merges
// in-launch, measured 0.25 us slower with it; the exchange costs the plain final merge 23 VGPRs and a spill).
// KS: the host step's input arrives by value (StepInputK, GroupArgs::ksi); block 0 writes it to the device
// StepInput `in_dev` for the merge and later readers, so the step needs no upload kernel (one dependent launch
// and a PCIe read fewer).
// GEN (GroupArgs::gen, zero-order H 12 host steps, MPPI, device Philox draws): the launch makes the step's draws
// itself -- every fourth step each lane the three column quads (its leg's three components) of the next four
// steps: rng_item's Philox4x32-10 call and Box-Muller pairs, so the same bits.  No noise is read or written: the
// values stay raw in `pre` as the ZST loads leave them, and the LDS stage feeds the epilogue as before.
#ifndef SRBD_QUAD_WPE
#define SRBD_QUAD_WPE 4  // waves per SIMD the four-lane kernels are compiled for (a build-time knob for A/B builds)
#endif
template <int KIND, int HT, int ST, bool CEMT, bool EXT, int FM = 0, bool KS = false, bool GEN = false>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(SRBD_QUAD_WPE))) rollout_quad_kernel(
                                                           const std::conditional_t<KS, StepInputK, KsNone> ksi,
                                                           const ModelConst mc, const StepInput* __restrict__ in_dev,
                                                           const float* __restrict__ noise, float* __restrict__ costs,
                                                           float* __restrict__ recs, int rec_stride,
    const RngJob next_rng, int nroll, const GroupArgs grp) {
    const StepInput* __restrict__ in;
    if constexpr (KS) {
        // ksi is the first kernel argument: read it where it lies in the kernarg segment (taking &ksi makes
        // the compiler copy the struct to scratch once lanes index it)
        (void)ksi;
        const auto ka = (const __attribute__((address_space(4))) StepInput*)__builtin_amdgcn_kernarg_segment_ptr();
        in = (const StepInput*)ka;
        if (blockIdx.x == 0) {
            const auto src = (const __attribute__((address_space(4))) uint32_t*)ka;
            uint32_t* dst = reinterpret_cast<uint32_t*>(const_cast<StepInput*>(in_dev));
            for (int i = threadIdx.x; i < (int)(sizeof(StepInputK) / 4); i += blockDim.x) dst[i] = src[i];
        }
    } else {
        in = in_dev;
    }
    if (grp.gate && (*grp.gate & ARM_CANCEL)) {  // armed chain that did not fire: nothing to compute
        if (FM && blockIdx.x == 0 && threadIdx.x == 0)  // the in-launch final merge's cancel token
            __hip_atomic_store(grp.flag, grp.seq | ARM_CANCEL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    // blocks past the rollout grid generate the next step's noise on the CUs the rollout leaves idle
    SRBD_RSTAMP(0);
#if SRBD_PRIO
    // experiment knob: the rollout waves (horizon, epilogue, fold, tail) ahead of the draw waves in VALU arbitration
    if ((int)blockIdx.x < nroll && nroll >= SRBD_PRIO_MIN) __builtin_amdgcn_s_setprio(SRBD_PRIO);
#endif
    if ((int)blockIdx.x >= nroll) {
        rng_items(mc, in, next_rng, ((int)blockIdx.x - nroll) * (int)blockDim.x + (int)threadIdx.x,
                  ((int)gridDim.x - nroll) * (int)blockDim.x);
        SRBD_RSTAMP(5);
        return;
    }

    constexpr bool CT = HT > 0 && (KIND == SRBD_ZERO_ORDER || ST > 0);
    const int SPB = (int)blockDim.x >> 2;  // samples per block: 64 or 128
    const int H = CT ? HT : mc.H;
    const int S = CT ? ST : mc.S;
    const int PL = CT ? (KIND == SRBD_ZERO_ORDER ? 3 * HT : (KIND == SRBD_LINEAR_SPLINE ? 3 * (ST + 1) : 12 * ST))
                      : mc.PL;
    // ZST (zero-order, compile-time horizon): every noise value a lane reads stays in its registers raw (best is
    // added from an LDS copy at use), and after the horizon the block's 64 x P values go to LDS, sample-major,
    // where the epilogue's weighted sums read them (block_wsum_lds) instead of reading the noise from L2 / HBM
    // a second time (N = 65 536: the epilogue was 11 of the rollout's 28 us; scripts/vrun.sh noepi).  64 samples
    // per block (the launcher's quad block for zero-order).  The group reduction reuses the buffer.  H <= 12:
    // 38.5 KB of LDS per block keeps four blocks per CU (H = 16 would need 51 KB: three).
    constexpr bool ZST = CT && KIND == SRBD_ZERO_ORDER && !EXT && HT <= 12;
    static_assert(!GEN || (ZST && HT % 4 == 0 && !CEMT), "GEN: the zero-order LDS-staged form, H % 4 == 0");
    constexpr int PCT = ZST ? 12 * HT : 1;
    constexpr int ZSTR = PCT + 1;  // sample stride of the stage: odd, so the epilogue's row-per-lane reads hit 64 banks
    __shared__ __attribute__((aligned(16))) float zst[ZST ? (64 * ZSTR > GROUP_LDS_FLOATS ? 64 * ZSTR : GROUP_LDS_FLOATS) : 1];
    __shared__ float bls[ZST ? PCT : 1];
    __shared__ float sls[ZST && CEMT ? PCT : 1];
    const int tid = threadIdx.x;
    const int q4 = tid & 3;
    const int c = q4 < 3 ? q4 : 2;
    const int sib = tid >> 2;
    const int k = blockIdx.x * SPB + sib;
    const bool valid = k < mc.n_local;
    const size_t ldn = (size_t)mc.ldn;
    const float* __restrict__ nz = noise + k;
    const float* __restrict__ best = in->best;
    const bool zs = CEMT && zs_scaled(mc, in);  // CEMT: CEM kernels only carry the scaling code

    // lane constants
    const QuadLane L = quad_lane(mc, c);
    const float Qp = sel3(c, mc.Q[0], mc.Q[1], mc.Q[2]), Qv = sel3(c, mc.Q[3], mc.Q[4], mc.Q[5]);
    const float Qr = sel3(c, mc.Q[6], mc.Q[7], mc.Q[8]), Qw = sel3(c, mc.Q[9], mc.Q[10], mc.Q[11]);
    const float* st = in->state;
    const float* rf = in->ref;
    const float rp = sel3(c, rf[0], rf[1], rf[2]), rv = sel3(c, rf[3], rf[4], rf[5]);
    const float rr = sel3(c, rf[6], rf[7], rf[8]), rw = sel3(c, rf[9], rf[10], rf[11]);
    float feet[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) feet[l] = sel3(c, st[12 + 3 * l], st[13 + 3 * l], st[14 + 3 * l]);
    float p = sel3(c, st[0], st[1], st[2]), v = sel3(c, st[3], st[4], st[5]);
    float r = sel3(c, st[6], st[7], st[8]), w = sel3(c, st[9], st[10], st[11]);
    float cost = 0.0f;
    // EXT: opt-in cost terms (srbd_set_cost_terms), this lane's component of extra_cost_step
    const float rwc = sel3(c, mc.cost_r[0], mc.cost_r[1], mc.cost_r[2]);
    float fprev[4];
    // LEGP (every kernel but EXT): the force phase runs leg-parallel.  Lane q4 decodes, shapes and clips the
    // three components of leg q4 and forms its force and torque contributions f c, ((p_foot - p) x f) c;
    // one quad butterfly sums them over the legs in integrate()'s order (leg0 + leg1) + (leg2 + leg3),
    // leaving all six sums on every lane; the rigid-body step then runs component-parallel as before.
    // Lane 3 does real work in the force phase, the fz broadcast and the per-leg cross-product DPP moves
    // go away (C2 ZO step: see DESIGN.md).  EXT keeps the component-parallel form (its terms are per
    // component, in leg order).
    constexpr bool LEGP = !EXT;
    const int lq = q4;  // this lane's leg in the force phase
    uint32_t lmask[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) lmask[l] = lq == l ? ~0u : 0u;
    float footL[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) footL[q] = st[12 + 3 * lq + q];
    // ZST: this lane's leg's contact value of every step in registers, loaded once (lane-varying row: one vector
    // load per step, issued before the horizon), instead of four scalar loads and a 10-instruction lane select
    // per step
    constexpr int NCL = ZST ? HT : 1;
    float clreg[NCL];
    if constexpr (ZST) {
#pragma unroll
        for (int n = 0; n < HT; ++n) clreg[n] = in->contact[lq][n];
    }

    // Specialised shapes: every parameter this lane reads over the horizon (its component's block
    // of each leg) is loaded before the first step, so the horizon chain pays one memory round trip
    // instead of one per step (at N = 10 000 there is < 1 wave per SIMD to hide the latency).
    // ZO: H values per leg; linear: S + 1; cubic: 4 per chunk (start 10 * chunk, NMPC:225).
    constexpr int NPRE = !CT ? 1 : (KIND == SRBD_ZERO_ORDER ? HT : (KIND == SRBD_LINEAR_SPLINE ? ST + 1 : 4 * ST));
    // LEGP: pre[q][i] = component q's slot i of this lane's leg; else pre[l][i] = this lane's component's
    // slot i of leg l
    float pre[LEGP ? 3 : 4][NPRE];
    // noise through a buffer descriptor: per-lane part (leg or component block + sample) in voffset, the
    // uniform row in soffset -> no per-load address arithmetic (launch_rollout checks P*ldn*4 < 2^31)
    const int cblk = LEGP ? lq * PL
                          : (KIND == SRBD_ZERO_ORDER ? c * HT : (KIND == SRBD_LINEAR_SPLINE ? c * (ST + 1) : 4 * c));
    const auto nrs = __builtin_amdgcn_make_buffer_rsrc((void*)noise, (short)0, mc.P * mc.ldn * 4, 0x00020000);
    const int voff = (cblk * mc.ldn + k) * 4;
    const float* __restrict__ bl = best + cblk;
    const float* __restrict__ sl = in->sigma + cblk;
    if constexpr (ZST) {  // best (and sigma) -> LDS; their loads issue ahead of the noise loads (vmcnt is in order)
        for (int j = tid; j < PCT; j += 256) {
            bls[j] = best[j];
            if constexpr (CEMT) sls[j] = in->sigma[j];
        }
    }
    auto load_slot = [&](const int i) __attribute__((always_inline)) {
#pragma unroll
        for (int l = 0; l < (LEGP ? 3 : 4); ++l) {
            // row - cblk: LEGP component l of this leg (ZO l H + i, linear l (S + 1) + i, cubic 10 chunk + 4 l +
            // k); else leg l's block of this lane's component
            const int jr = LEGP ? (KIND == SRBD_ZERO_ORDER ? l * HT + i
                                   : (KIND == SRBD_LINEAR_SPLINE ? l * (ST + 1) + i : 10 * (i >> 2) + 4 * l + (i & 3)))
                                : l * PL + (KIND == SRBD_CUBIC_SPLINE ? 10 * (i >> 2) + (i & 3) : i);
#ifdef SRBD_DIAG_NOLOAD  // diagnostic build: no noise reads (timing only)
            const float nzv = (float)(voff + jr * mc.ldn) * 1e-9f;
#else
            const float nzv = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(nrs, voff, jr * mc.ldn * 4, 0));
#endif
            if constexpr (ZST) {
                pre[l][i] = nzv;  // raw: best is added at use, the value staged for the epilogue
            } else if constexpr (CEMT) {  // unscaled CEM device draws: Z * sigma_j (z * 1 == z; the load unconditional)
                const float sj = sl[jr];
                pre[l][i] = bl[jr] + nzv * (zs ? sj : 1.0f);
            } else {
                pre[l][i] = bl[jr] + nzv;
            }
        }
    };
    // Zero-order with the opt-in cost terms: a rolling window of PW slots (slot n + PW loads at step n)
    // instead of the whole horizon up front -- the terms' extra live values otherwise push the unrolled
    // horizon past 256 VGPRs into scratch.
    constexpr int PW = (EXT && KIND == SRBD_ZERO_ORDER) ? (NPRE < 4 ? NPRE : 4) : NPRE;
    // CEM cubic splines with S > 1: chunk q's four slots are loaded CLEAD steps before its first step
    // instead of up front.  C3 (H16 CEM): 80 -> 16 B of scratch per lane, rollout 41.8 -> 37.9 us, device
    // step 73.1 -> 65.5 us (r3d); leads 3 / 4 spill again (80 / 144 B), and the plain cubic kernels spill
    // more with the window (H16: 48 -> 144 B at lead 2), so they keep the up-front loads.
    constexpr int CLEAD = 2;
    constexpr bool CWIN = CT && CEMT && KIND == SRBD_CUBIC_SPLINE && ST > 1;
    if constexpr (GEN) {
        // nothing to load: the horizon makes the values (gen4)
    } else if constexpr (CWIN) {
#pragma unroll
        for (int i = 0; i < 4; ++i) load_slot(i);
    } else if constexpr (CT) {
        // slot-major issue order: step n's operands are the first to return (loads complete in order),
        // so the horizon starts while the later steps' parameters are still in flight
#pragma unroll
        for (int i = 0; i < PW; ++i) load_slot(i);
    }
    if constexpr (ZST) {  // the LDS copy of best is complete (the noise loads stay in flight)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }

    float dep = p;  // step_ptr dependency: set part-way through each step
    // GEN: steps 4 s .. 4 s + 3 of component q of this lane's leg are column quad lq PL / 4 + q HT / 4 + s of the row
    auto gen4 = [&](const int s, auto is) __attribute__((always_inline)) {
        const int r = mc.row0 + k;
        const bool live = r > 0 && valid;  // row 0 (the warm start) and the padding rows: zeros, as in the buffer
        const uint32_t d = (uint32_t)(r - 1);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            uint32_t cc[4] = {d, (uint32_t)(lq * (PL / 4) + q * (HT / 4) + s), is->ctr_lo, is->ctr_hi};
            philox4x32_10(cc, is->seed_lo, is->seed_hi);
            float v[4];
            box_muller(cc[0], cc[1], v[0], v[1]);
            box_muller(cc[2], cc[3], v[2], v[3]);
#pragma unroll
            for (int i = 0; i < 4; ++i) pre[q][(4 * s + i) % NPRE] = live ? mc.sigma_mppi * v[i] : 0.0f;
        }
    };
    auto step = [&](const int n, auto EX) __attribute__((always_inline)) {  // EX: as rollout_kernel
        // GEN: the key read through a pointer tied to the last step's cost, so the quads are made four steps at a
        // time, not hoisted to the start (as rollout_kernel's GEN)
        if constexpr (GEN)
            if (n % 4 == 0) gen4(n / 4, step_ptr(in, cost));
        if constexpr (CT && PW < NPRE)
            if (n + PW < NPRE) load_slot(n + PW);  // n is a compile-time constant here (unrolled horizon)
        if constexpr (CWIN) {
#pragma unroll
            for (int q = 1; q < (CWIN ? ST : 1); ++q) {
                const int at = q * HT / ST - CLEAD;
                if (n == (at > 0 ? at : 0))
#pragma unroll
                    for (int i = 4 * q; i < 4 * q + 4; ++i) load_slot(i);
            }
        }
        // this step's scalars through step_ptr: loaded per step, not hoisted across the unrolled horizon
        // (hoisted: SGPR spills to VGPR lanes, ~150 v_readlane per step in the cubic CEM kernel)
        const auto is = step_ptr(in, dep);
        float cl[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        if constexpr (!ZST)
#pragma unroll
            for (int l = 0; l < 4; ++l) cl[l] = is->contact[l][n];
        const float fref = is->fzref[n];
        const float dt = mc.dts[n];
        const float sq = mc.sq[n], somq = mc.somq[n], sa = mc.sa[n], sb = mc.sb[n], scc = mc.sc[n], sd = mc.sd[n];
        const int idx = CT && KIND != SRBD_ZERO_ORDER ? chunk_index(n, HT, ST) : mc.sidx[n];
        // force and torque sums over the legs, (leg0 + leg1) + (leg2 + leg3) as integrate() forms them.  No
        // per-leg branch on the contact flags: the straight-line horizon schedules better than it saves
        // (measured 15.9 -> 17.1 us at C2 with the branches)
        float temp, temp2, ex = 0.0f;
        if constexpr (LEGP) {
            // this lane's leg's contact value as bit masks (lmask[l] = ~0 on the lanes of leg l): a select chain
            // here became three nested divergent branches, each with its own scalar load and lgkmcnt(0) wait
            const float clq = ZST ? clreg[ZST ? n : 0]
                                  : __uint_as_float((__float_as_uint(cl[0]) & lmask[0]) | (__float_as_uint(cl[1]) & lmask[1]) |
                                                    (__float_as_uint(cl[2]) & lmask[2]) | (__float_as_uint(cl[3]) & lmask[3]));
            const int lbase = lq * PL;
            // component q of this leg's decoded force (slot i, parameter j of the leg when not prefetched)
            auto PQ = [&](int q, int i, int j) {
                if constexpr (ZST) {  // best + z as load_slot formed it (ZO: j = q H + n, i = n)
                    if constexpr (CEMT) return bls[lbase + j] + pre[q][i] * (zs ? sls[lbase + j] : 1.0f);
                    return bls[lbase + j] + pre[q][i];
                } else if constexpr (CT) {
                    return pre[q][i];
                } else {
                    const float z = nz[(size_t)(lbase + j) * ldn];
                    return best[lbase + j] + (zs ? z * in->sigma[lbase + j] : z);
                }
            };
            float rq[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                if (KIND == SRBD_ZERO_ORDER) {
                    rq[q] = PQ(q, n, n + q * H);
                } else if (KIND == SRBD_LINEAR_SPLINE) {
                    const int o = idx + q * (S + 1);
                    rq[q] = somq * PQ(q, idx, o) + sq * PQ(q, idx + 1, o + 1);
                } else {
                    const int o = 10 * idx + 4 * q;
                    const float p0 = PQ(q, 4 * idx, o), p1 = PQ(q, 4 * idx + 1, o + 1), p2 = PQ(q, 4 * idx + 2, o + 2),
                                p3 = PQ(q, 4 * idx + 3, o + 3);
                    const float phi = 0.5f * ((p2 - p1) + (p1 - p0));
                    const float phin = 0.5f * ((p3 - p2) + (p2 - p1));
                    rq[q] = sa * p1 + sb * phi + scc * p2 + sd * phin;
                }
            }
            // shape_leg / clip_leg (srbd_core.h), this lane's leg
            const float fz = clamp_cs((fref + rq[2]) * clq, mc.grf_min, mc.grf_max);
            const float lo = mc.neg_mu * fz, hi = mc.mu * fz;
            const float fx = clamp_cs(third(rq[0] * clq), lo, hi), fy = clamp_cs(third(rq[1] * clq), lo, hi);
            // integrate(): skew_dot(p_foot - p, f) * c (the position's components from their lanes)
            const float vx = footL[0] - qp<QP_B0>(p), vy = footL[1] - qp<QP_B1>(p), vz = footL[2] - qp<QP_B2>(p);
            float sm[6] = {fx * clq, fy * clq, fz * clq, ((-vz) * fy + vy * fz) * clq, (vz * fx + (-vx) * fz) * clq,
                           ((-vy) * fx + vx * fy) * clq};
#pragma unroll
            for (int i = 0; i < 6; ++i) {  // quad butterfly: (l0 + l1) + (l2 + l3) on every lane (adds commute)
                sm[i] = sm[i] + qp<QP_XOR1>(sm[i]);
                sm[i] = sm[i] + qp<QP_XOR2>(sm[i]);
            }
            temp = sel3(c, sm[0], sm[1], sm[2]);
            temp2 = sel3(c, sm[3], sm[4], sm[5]);
            dep = sm[5];  // the next step's scalar loads issue from here on (step_ptr)
            quad_rb_apply3(mc, L, quad_rb_prep(L, r, w), temp, sm[3], sm[4], sm[5], dt, p, v, r, w);
        } else {
        float tf[4], tt[4];
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const int base = l * PL;
            // parameter j of this leg (i: its slot in the prefetched block when the shape is specialised;
            // i is a compile-time constant there, so `pre` stays in registers)
            auto P = [&](int i, int j) {
                if constexpr (CT) {
                    return pre[l][i];
                } else {
                    const float z = nz[(size_t)(base + j) * ldn];
                    return best[base + j] + (zs ? z * in->sigma[base + j] : z);
                }
            };
            float raw;
            if (KIND == SRBD_ZERO_ORDER) {
                raw = P(n, n + c * H);
            } else if (KIND == SRBD_LINEAR_SPLINE) {
                const int o = idx + c * (S + 1);
                raw = somq * P(idx, o) + sq * P(idx + 1, o + 1);
            } else {
                const int o = 10 * idx + 4 * c;
                const float p0 = P(4 * idx, o), p1 = P(4 * idx + 1, o + 1), p2 = P(4 * idx + 2, o + 2),
                            p3 = P(4 * idx + 3, o + 3);
                const float phi = 0.5f * ((p2 - p1) + (p1 - p0));
                const float phin = 0.5f * ((p3 - p2) + (p2 - p1));
                raw = sa * p1 + sb * phi + scc * p2 + sd * phin;
            }
            // shape_leg / clip_leg, component-wise
            float zp = clamp_cs((fref + raw) * cl[l], mc.grf_min, mc.grf_max);
            const float xy = third(raw * cl[l]);
            const float fz = qp<QP_B2>(c == 2 ? zp : xy);
            const float f = c == 2 ? fz : clamp_cs(xy, mc.neg_mu * fz, mc.mu * fz);
            tf[l] = f * cl[l];
            tt[l] = quad_cross(feet[l] - p, f) * cl[l];
            if constexpr (decltype(EX)::value) {
                const float u = c == 2 ? f - (cl[l] != 0.0f ? fref : 0.0f) : f;
                float term = (u * rwc) * u;
                if (n > 0) {
                    const float d = f - fprev[l];
                    term = term + (d * mc.cost_smooth) * d;
                }
                {  // x / y lanes only, as a select (a divergent branch in the unrolled horizon spilled)
                    float vv = fabsf(xy) - mc.mu * fz;
                    vv = vv > 0.0f ? vv : 0.0f;
                    const float cone = (vv * mc.cost_cone) * vv;
                    term = c < 2 ? term + cone : term;
                }
                ex = ex + term;
                fprev[l] = f;
            }
        }
        temp = (tf[0] + tf[1]) + (tf[2] + tf[3]);
        temp2 = (tt[0] + tt[1]) + (tt[2] + tt[3]);
        dep = temp2;  // the next step's scalar loads issue from here on (step_ptr)
        quad_rigid_body(mc, L, temp, temp2, dt, p, v, r, w);
        }
        // tracking cost (NMPC:451), accumulated per component lane: cost_c += ((tp + tv) + tr) + tw,
        // the three lanes summed once after the horizon (see rollout_kernel for the same order)
        const float ep = p - rp, ev = v - rv, er_ = r - rr, ew = w - rw;
        const float tp = (ep * Qp) * ep, tv = (ev * Qv) * ev, tr = (er_ * Qr) * er_, tw = (ew * Qw) * ew;
        cost = cost + (((tp + tv) + tr) + tw);
        if constexpr (decltype(EX)::value) {
            cost = cost + ex;
            // The terms do not feed the dynamics, so the scheduler sank them to the end of the unrolled
            // horizon and kept every step's forces live (256 VGPRs + up to 800 B of scratch; 334
            // registers at H12 given 512).  An empty asm on the accumulator pins each step's terms to
            // that step: 122 VGPRs, no spill.  (The plain kernels' cost terms gain nothing from it.)
            asm volatile("" : "+v"(cost));
        }
    };
    auto horizon = [&](auto EX) __attribute__((always_inline)) {
        if constexpr (CT) {
            unroll_seq([&](auto nc) { step(decltype(nc)::value, EX); },
                       std::make_integer_sequence<int, (CT ? HT : 1)>{});
        } else {
            for (int n = 0; n < H; ++n) step(n, EX);
        }
    };
    horizon(std::bool_constant<EXT>{});
    SRBD_RSTAMP(2);
    cost = (qp<QP_B0>(cost) + qp<QP_B1>(cost)) + qp<QP_B2>(cost);
    cost = cost + in->cost_feet;  // 0, or NaN when a foot term is non-finite (Q_feet = 0)
    if (isnan(cost) || isinf(cost)) cost = 1000000.0f;
    if (valid && q4 == 0 && costs) costs[k] = cost;
    if constexpr (ZST) {  // the block's noise, sample-major (leg lq's block of columns lq PL .. lq PL + PL - 1)
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int i = 0; i < NPRE; ++i) zst[sib * ZSTR + lq * PL + q * HT + i] = pre[q][i];
    }
#ifdef SRBD_DIAG_NOEPI  // diagnostic build: no block epilogue (timing only)
    if (tid == 0) recs[blockIdx.x] = cost;
    return;
#endif
    const bool glast = block_epilogue<CEMT, ZST>(mc, in, SPB, q4 == 0 ? sib : -1, valid, cost, noise, recs, rec_stride,
                                                 0.0f, grp, nroll, ZST ? zst : nullptr, ZSTR);
    if constexpr (FM && ZST && !CEMT) {
        if (FM == 1 && grp.fast) {
            if (glast) fast_tail(mc, in, noise, recs, rec_stride, grp, nroll, zst);
        } else if (glast) {
            final_merge<256, FM == 2>(mc, in, noise, rec_stride, grp, zst);
        }
    }
    SRBD_RSTAMP(5);
}

// ---- gait-adaptive rollout in the four-lane layout (rollout_ga_kernel's float operations, in its
// order, component-wise as rollout_quad_kernel does): the sample's step frequency, contact masks,
// stance counters and per-leg spline coefficients are formed on each of its four lanes (the same
// values), the decode reads this lane's component.  Costs are rollout_ga_kernel's bit for bit.
// The opt-in cost terms run on rollout_ga_kernel (launch_rollout_ga).
template <int KIND, int HT>
__global__ void __launch_bounds__(512) rollout_ga_quad_kernel(const ModelConst mc, const StepInput* __restrict__ in,
                                                              const float* __restrict__ noise,
                                                              float* __restrict__ costs, float* __restrict__ recs,
                                                              int rec_stride, const RngJob next_rng, int nroll, const GroupArgs grp) {
    if (grp.gate && (*grp.gate & ARM_CANCEL)) return;  // armed chain that did not fire
    if ((int)blockIdx.x >= nroll) {
        rng_items(mc, in, next_rng, ((int)blockIdx.x - nroll) * (int)blockDim.x + (int)threadIdx.x,
                  ((int)gridDim.x - nroll) * (int)blockDim.x);
        return;
    }
    const int H = HT > 0 ? HT : mc.H, S = mc.S, PL = mc.PL;  // HT: horizon fixed at compile time
    const int tid = threadIdx.x;
    const int q4 = tid & 3;
    const int c = q4 < 3 ? q4 : 2;
    const int sib = tid >> 2;
    const int SPB = (int)blockDim.x >> 2;
    const int k = blockIdx.x * SPB + sib;
    const bool valid = k < mc.n_local;
    const size_t ldn = (size_t)mc.ldn;
    const float* __restrict__ nz = noise + k;
    const float* __restrict__ best = in->best;

    const float f = ga_sample_freq(mc, in, k);
    uint32_t mask[4];
    ga_contact_masks(in, H, f, mask);
    float seg[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) seg[l] = ((float)__popc(mask[l]) + 1.0f) / (float)S;
    int cnt[4] = {-1, -1, -1, -1};

    const QuadLane L = quad_lane(mc, c);
    const float Qp = sel3(c, mc.Q[0], mc.Q[1], mc.Q[2]), Qv = sel3(c, mc.Q[3], mc.Q[4], mc.Q[5]);
    const float Qr = sel3(c, mc.Q[6], mc.Q[7], mc.Q[8]), Qw = sel3(c, mc.Q[9], mc.Q[10], mc.Q[11]);
    const float* st_ = in->state;
    const float* rf = in->ref;
    const float rp = sel3(c, rf[0], rf[1], rf[2]), rv = sel3(c, rf[3], rf[4], rf[5]);
    const float rr = sel3(c, rf[6], rf[7], rf[8]), rw = sel3(c, rf[9], rf[10], rf[11]);
    float feet[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) feet[l] = sel3(c, st_[12 + 3 * l], st_[13 + 3 * l], st_[14 + 3 * l]);
    float p = sel3(c, st_[0], st_[1], st_[2]), v = sel3(c, st_[3], st_[4], st_[5]);
    float r = sel3(c, st_[6], st_[7], st_[8]), w = sel3(c, st_[9], st_[10], st_[11]);
    float cost = 0.0f;
    // unrolled when HT > 0: every step's parameter loads depend only on the contact masks, so they
    // issue ahead of the physics chain
    constexpr int UNR = HT > 0 ? HT : 1;
#pragma unroll UNR
    for (int n = 0; n < H; ++n) {
        float cl[4];
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const uint32_t b = (mask[l] >> n) & 1u;
            cl[l] = b ? 1.0f : 0.0f;
            cnt[l] += (int)b;
        }
        const float ns = ((cl[0] + cl[1]) + cl[2]) + cl[3];
        const float fref = mc.fz_ns[(int)ns];
        float tf[4], tt[4];  // per-leg force / torque contributions, summed pairwise (integrate()'s order)
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const int base = l * PL;
            auto acc = [&](int j) {
                j = j < 0 ? j + PL : j;
                return best[base + j] + nz[(size_t)(base + j) * ldn];
            };
            const int stc = cnt[l];
            float raw;
            if (KIND == SRBD_ZERO_ORDER) {
                raw = acc(stc + c * H);
            } else {
                int idx = 0;
                for (int i = 0; i <= S; ++i)
                    if (stc >= in->ga_cb[i]) idx = i;
                float tau = (float)stc / seg[l];
                tau = tau - (float)idx;
                const float q = tau / 1.0f;
                if (KIND == SRBD_LINEAR_SPLINE) {
                    const float omq = 1.0f - q;
                    const int o = idx + c * (S + 1);
                    raw = omq * acc(o) + q * acc(o + 1);
                } else {
                    const float a = 2.0f * q * q * q - 3.0f * q * q + 1.0f;
                    const float bb = (q * q * q - 2.0f * q * q + q) * 1.0f;
                    const float cc = -2.0f * q * q * q + 3.0f * q * q;
                    const float d = (q * q * q - q * q) * 1.0f;
                    const int o = 10 * idx + 4 * c;
                    const float p0 = acc(o), p1 = acc(o + 1), p2 = acc(o + 2), p3 = acc(o + 3);
                    const float phi = 0.5f * ((p2 - p1) + (p1 - p0));
                    const float phin = 0.5f * ((p3 - p2) + (p2 - p1));
                    raw = a * p1 + bb * phi + cc * p2 + d * phin;
                }
            }
            const float zp = clamp_cs((fref + raw) * cl[l], mc.grf_min, mc.grf_max);
            const float xy = third(raw * cl[l]);
            const float fz = qp<QP_B2>(c == 2 ? zp : xy);
            const float fo = c == 2 ? fz : clamp_cs(xy, mc.neg_mu * fz, mc.mu * fz);
            tf[l] = fo * cl[l];
            tt[l] = quad_cross(feet[l] - p, fo) * cl[l];
        }
        const float temp = (tf[0] + tf[1]) + (tf[2] + tf[3]), temp2 = (tt[0] + tt[1]) + (tt[2] + tt[3]);
        quad_rigid_body(mc, L, temp, temp2, mc.dts[n], p, v, r, w);
        const float ep = p - rp, ev = v - rv, er_ = r - rr, ew = w - rw;
        const float tp = (ep * Qp) * ep, tv = (ev * Qv) * ev, tr = (er_ * Qr) * er_, tw = (ew * Qw) * ew;
        cost = cost + (((tp + tv) + tr) + tw);
    }
    cost = (qp<QP_B0>(cost) + qp<QP_B1>(cost)) + qp<QP_B2>(cost);
    cost = cost + in->cost_feet;
    const float df = f - 1.3f;
    cost = cost + (df * 100.0f) * df;  // GA:500
    if (isnan(cost) || isinf(cost)) cost = 1000000.0f;
    if (valid && q4 == 0 && costs) costs[k] = cost;
    block_epilogue<false>(mc, in, SPB, q4 == 0 ? sib : -1, valid, cost, noise, recs, rec_stride, f, grp, nroll);
}

// ------------------------------------------------------------------ merge
__device__ __forceinline__ uint64_t rec_key(const float* R, int P, int q) {
    return ((uint64_t)f2u(R[REC_HDR + P + 2 * q + 1]) << 32) | (uint64_t)f2u(R[REC_HDR + P + 2 * q]);
}

constexpr int MERGE_THREADS = 1024;
constexpr int MERGE_RPT = 8;    // record headers per thread (nrec <= MERGE_RPT * MERGE_THREADS)
// The LDS-staged merge runs two waves per SIMD: its phases are short dependent chains that every
// wave repeats (index math, the beta reduction), so 16 waves pay ~2x the issue of 8, while fewer
// waves stage the records more slowly (C2 merge 9.0 / 8.4 / 9.8 us at 1024 / 512 / 256 threads).
constexpr int MERGE_STAGE_THREADS = 512;
// Block-wide K smallest record keys (ascending) into `elite`, by selection and ranks.  Every record's
// key list is the sorted K smallest keys of its samples, so its first key is its minimum, and the K
// smallest keys overall lie in the K records with the smallest minima (any other record's minimum already
// exceeds K keys of those records).  Keys are unique (cost bits, row); only the ~0 padding repeats.
//  1. the K smallest record minima, with their records: per chunk of NT records, every record's rank in
//     its wave's 64 minima (64 independent LDS-broadcast compares) sends the wave's K smallest to a
//     candidate list, then the candidates' ranks among themselves and the K carried from the chunks
//     before (<= NW K + K compares) keep the K smallest;
//  2. those records' K-key lists (K x K keys), ranked among themselves, give the K smallest keys.
// Compares are independent, so the phase is issue-bound (~4 us at C3's 1024 records) where K dependent
// rounds of DPP wave minima per level were latency-bound (10 us).  Caller syncs afterwards.
template <int NT>
struct TopkLds {
    static constexpr int NCT = (NT / 64) * MAXK + MAXK > MAXK * MAXK ? (NT / 64) * MAXK + MAXK : MAXK * MAXK;
    uint64_t keys[NT > MAXK * MAXK ? NT : MAXK * MAXK];  // a chunk's record minima, then step 2's K x K keys
    uint64_t cand[NCT];  // candidates (block_topk_nodes: a K x K table)
    int cand_r[NCT];
    int cnt[MAXK * MAXK];                   // block_topk_nodes' rank counts
    uint64_t top[MAXK], ntop[MAXK];         // carried K smallest minima (and the next chunk's)
    int top_r[MAXK], ntop_r[MAXK];
    int sel[MAXK];                          // block_topk_nodes: the selected level-0 nodes
};
template <int NT>
__device__ __forceinline__ void block_topk_rank(const float* __restrict__ recs, int nrec, int rec_stride, int P, int K,
                                                uint64_t* elite, TopkLds<NT>& t) {
    constexpr int NW = NT / 64;
    const int tid = threadIdx.x, T = NT, wv = tid >> 6;
    const int NC = NW * K + K;  // candidates per chunk: the waves' K smallest + the carried K
    if (tid < K) {
        t.top[tid] = KEY_NONE;
        t.top_r[tid] = 0;
    }
    for (int base = 0; base < nrec; base += T) {
        const int r = base + tid;
        const uint64_t x = r < nrec ? rec_key(recs + (size_t)r * rec_stride, P, 0) : KEY_NONE;
        t.keys[tid] = x;
        for (int i = tid; i < NW * K; i += T) t.cand[i] = KEY_NONE;
        __syncthreads();
        const uint64_t* wk = t.keys + (wv << 6);
        int cnt = 0;
#pragma unroll 16
        for (int j = 0; j < 64; ++j) cnt += wk[j] < x ? 1 : 0;
        if (cnt < K && x != KEY_NONE) {
            t.cand[wv * K + cnt] = x;
            t.cand_r[wv * K + cnt] = r;
        }
        if (tid < K) {
            t.cand[NW * K + tid] = t.top[tid];
            t.cand_r[NW * K + tid] = t.top_r[tid];
            t.ntop[tid] = KEY_NONE;
        }
        __syncthreads();
        if (tid < NC) {
            const uint64_t y = t.cand[tid];
            int c2 = 0;
            for (int j = 0; j < NC; ++j) c2 += t.cand[j] < y ? 1 : 0;
            if (c2 < K && y != KEY_NONE) {
                t.ntop[c2] = y;
                t.ntop_r[c2] = t.cand_r[tid];
            }
        }
        __syncthreads();
        if (tid < K) {
            t.top[tid] = t.ntop[tid];
            t.top_r[tid] = t.ntop_r[tid];
        }
        __syncthreads();
    }
    const int KK = K * K;
    for (int i = tid; i < KK; i += T) {
        const int e = i / K, q = i - e * K;
        t.keys[i] = t.top[e] != KEY_NONE ? rec_key(recs + (size_t)t.top_r[e] * rec_stride, P, q) : KEY_NONE;
    }
    if (tid < K) elite[tid] = KEY_NONE;
    __syncthreads();
    for (int i = tid; i < KK; i += T) {
        const uint64_t y = t.keys[i];
        int c3 = 0;
        for (int j = 0; j < KK; ++j) c3 += t.keys[j] < y ? 1 : 0;
        if (c3 < K && y != KEY_NONE) elite[c3] = y;
    }
}

// The same K smallest keys as block_topk_rank, from the keys the merge's header pass already holds: every
// record's key (its minimum) in t.keys[r] (KEY_NONE up to NT; nrec <= NT) and the tree's level-0 node keys
// nk[g] (the minimum of records [32 g, 32 g + 32)).  Far fewer compares (C3: ~2 k against ~95 k):
//  A. the K smallest node keys.  The K smallest record minima lie in those nodes: any other node has K nodes
//     below its minimum, so K records below each of its records;
//  B. in each selected node, every record's rank among the node's 32: its K smallest, in order, form row s of
//     a K x K candidate table;
//  C. a candidate's overall rank = the entries below it summed over the table's rows (one thread per
//     (candidate, row), counts added in LDS): the K smallest record minima and their records;
//  D. those records' key lists (each ascending) ranked the same way: the K smallest keys.
// Entry state, with a barrier since: t.sel[0, MAXK) = -1, t.top[0, MAXK) = KEY_NONE, t.cand[0, K K) = KEY_NONE,
// t.cnt[0, K K) = 0.  Caller syncs afterwards.
template <int NT>
__device__ __forceinline__ void block_topk_nodes(const float* __restrict__ recs, int nrec, int rec_stride, int P,
                                                 int K, const uint64_t* nk, uint64_t* elite, TopkLds<NT>& t,
                                                 uint64_t* dbg = nullptr) {
    const int tid = threadIdx.x, KK = K * K;
#define TOPK_MARK(i) \
    if (dbg && tid == 0 && blockIdx.x < 2) dbg[32 * blockIdx.x + 25 + (i)] = __builtin_amdgcn_s_memrealtime()
    const int n1 = (nrec + TREE_FAN - 1) / TREE_FAN;
    if (tid < n1) {  // A
        const uint64_t y = nk[tid];
        int c = 0;
#pragma unroll 8
        for (int g = 0; g < n1; ++g) c += nk[g] < y ? 1 : 0;
        if (c < K && y != KEY_NONE) t.sel[c] = tid;
    }
    __syncthreads();
    TOPK_MARK(0);
    for (int i = tid; i < K * TREE_FAN; i += NT) {  // B
        const int sl = i / TREE_FAN, g = t.sel[sl];
        if (g < 0) continue;
        const uint64_t* nodek = t.keys + g * TREE_FAN;
        const uint64_t y = nodek[i % TREE_FAN];  // KEY_NONE past nrec
        if (y == KEY_NONE) continue;
        int c = 0;
#pragma unroll
        for (int j = 0; j < TREE_FAN; ++j) c += nodek[j] < y ? 1 : 0;
        if (c < K) {
            t.cand[sl * K + c] = y;
            t.cand_r[sl * K + c] = g * TREE_FAN + i % TREE_FAN;
        }
    }
    __syncthreads();
    // cnt[i] = entries of the K x K table below entry i.  Every row is ascending (B: a node's K smallest record
    // minima by rank, KEY_NONE after them; D: a record's key list, ascending, KEY_NONE-padded) and the keys are
    // unique, so a row's count below y is its lower bound: found by binary lifting (five dependent LDS reads for
    // K <= 16) -- the same count as comparing every entry, a third of the LDS traffic (C3: 1.3 us per call so)
    static_assert(MAXK <= 31, "binary lifting from a step of 16");
    auto table_ranks = [&](const uint64_t* tab) {
        for (int i = tid; i < KK * K; i += NT) {
            const int c = i / K, b = i - c * K;
            const uint64_t y = tab[c];
            if (y == KEY_NONE) continue;
            const uint64_t* row = tab + b * K;
            int n = 0;
#pragma unroll
            for (int s = 16; s >= 1; s >>= 1)
                if (n + s <= K && row[n + s - 1] < y) n += s;
            if (n) atomicAdd(&t.cnt[c], n);
        }
    };
    TOPK_MARK(1);
    table_ranks(t.cand);  // C
    __syncthreads();
    TOPK_MARK(2);
    for (int c = tid; c < KK; c += NT) {
        const uint64_t y = t.cand[c];
        const int n = t.cnt[c];
        if (y != KEY_NONE && n < K) {
            t.top[n] = y;
            t.top_r[n] = t.cand_r[c];
        }
    }
    __syncthreads();
    for (int i = tid; i < KK; i += NT) {  // D
        const int e = i / K, q = i - e * K;
        t.keys[i] = t.top[e] != KEY_NONE ? rec_key(recs + (size_t)t.top_r[e] * rec_stride, P, q) : KEY_NONE;
        t.cnt[i] = 0;
    }
    if (tid < K) elite[tid] = KEY_NONE;
    __syncthreads();
    TOPK_MARK(3);
    table_ranks(t.keys);
    __syncthreads();
    TOPK_MARK(4);
#undef TOPK_MARK
    for (int i = tid; i < KK; i += NT) {
        const uint64_t y = t.keys[i];
        const int n = t.cnt[i];
        if (y != KEY_NONE && n < K) elite[n] = y;
    }
}

// One block merges `nrec` records (per-block records of one rank, or gathered rank records).
//  L. one memory round trip: record headers (min cost, best row) and the first MERGE_PREF weighted-
//     sum values of every (column j, record group g) thread;
//  1. global (min cost, first row) key beta;  2. per-record rescale exp(-(m_r - beta)) -> LDS;
//  3. sum_r scale_r * v_r[j] and sum_r scale_r * s_r in fixed order (groups, then columns);
//  4. top-K keys: per-thread sorted lists -> per-wave K-round DPP minima -> one wave over the 16
//     wave lists; 5. elite rows -> LDS;  6. outputs: rank record and/or final step outputs; with
//     `chain` the new parameters, sigma and RNG counter are written back into `in` (warm start).
// Column-split launch (split_cs > 0, final step outputs only): every block reads all record headers (beta
// and the normaliser are recomputed per block, in the same order, so they agree bit for bit); block b >= 1
// (a slice) folds the columns [(b-1)cs, b cs) and writes the non-tail ones and sigma; block 0 (the tail
// block) writes the mc.tailc columns final_grf_pred decodes, the GRFs, the predicted state and the step
// scalars.  They meet through SplitXchg (srbd_core.h) inside the launch: the slices publish their root sums
// and the tail block reads its columns' back (it folds none itself); for CEM the tail block computes the
// top-K once and the slices read it back.  Each block publishes flag[blockIdx.x] = seq.  This spreads the
// record reads over CUs and drops the single block's serial column loop (C2: 8.8 -> see DESIGN).
// STAGE: the block first copies its records into LDS with 16-byte loads (one memory round trip,
// a quarter of the load instructions of dword column reads; the whole per-block record array at C2 is
// 157 x 152 floats = 95 KB) and every later phase reads them from LDS.
// Host-published outputs (flag != NULL) are stored system-scope (write-through to the mapped host
// buffer); after every wave's vmcnt(0) and a barrier the flag store follows them, so the system-wide
// L2 write-back of __threadfence_system is not needed for them (fence_sys = 1 keeps it).
// The merge's fixed-size LDS, passed in so a caller can place it (the merge kernels declare it; the zero-order
// rollout's final merge carves it from its noise stage, rollout_quad_kernel).
// alignas(16): the dynamic LDS that follows it (staged records, read as float4) starts 16-byte aligned
// (an 8-byte aligned start cost the C2 merge 1 us)
template <int NT>
struct alignas(16) MergeShared {
    uint64_t red[NT / 64];
    uint64_t elite[MAXK];
    int elite_src[MAXK];
    TopkLds<NT> tk;  // block_topk_rank
    float Vs[MAXP + 1];
    float nb[MAXP];
    float tag_sh;  // header tag (gait-adaptive step frequency) of the record holding beta's row
    // tail lanes: StepInput fields (13), the force-independent step (5), the ModelConst values the tail
    // uses (16) -- read back in one batch (kernarg fields re-read lazily are serial scalar loads)
    float tail_sh[4][40];
    float osh[sizeof(StepOutput) / sizeof(float)];  // the step outputs assembled for the burst
};
// The merge's tail lanes (0..3, component qc of the four-lane layout): the step inputs they use (tail_pre: fzref[0],
// the legs' contact at step 0, p / v / rpy / omega and the feet, component qc), the force-independent part of the
// predicted state (NMPC:752-784 via CMJ:93-174) and the ModelConst values of the final GRFs, into the lane's row of
// tail_sh -- read back in one batch by the outputs phase.
template <class IN>
__device__ __forceinline__ void merge_tail_load(const IN* in, int qc, float* tail_pre) {
    tail_pre[0] = in->fzref[0];
#pragma unroll
    for (int l = 0; l < 4; ++l) tail_pre[1 + l] = in->contact[l][0];
#pragma unroll
    for (int q = 0; q < 4; ++q) tail_pre[5 + q] = in->state[3 * q + qc];  // p, v, rpy, omega
#pragma unroll
    for (int l = 0; l < 4; ++l) tail_pre[9 + l] = in->state[12 + 3 * l + qc];  // feet
}
__device__ __forceinline__ void merge_tail_lane(const ModelConst& mc, int qc, const float* tail_pre, float* row) {
    const QuadLane L = quad_lane(mc, qc);
    const QuadRB rb = quad_rb_prep(L, tail_pre[7], tail_pre[8]);
    row[36] = L.Ii0;
    row[37] = L.Ii1;
    row[38] = L.Ii2;
    row[39] = L.g;
#pragma unroll
    for (int i = 0; i < 13; ++i) row[i] = tail_pre[i];
    row[13] = rb.er;
    row[14] = rb.R0;
    row[15] = rb.R1;
    row[16] = rb.R2;
    row[17] = rb.a1;
    const int iv[5] = {mc.kind, mc.H, mc.PL, mc.S, mc.fidx};
#pragma unroll
    for (int i = 0; i < 5; ++i) row[18 + i] = __int_as_float(iv[i]);
    const float fv[13] = {mc.fq, mc.fomq, mc.fa, mc.fb, mc.fc, mc.fd, mc.grf_min,
                          mc.grf_max, mc.mu, mc.neg_mu, mc.inv_m, mc.dts[0], 0.0f};
#pragma unroll
    for (int i = 0; i < 13; ++i) row[23 + i] = fv[i];
}
// Final GRFs (NMPC:695-750) and the predicted state (NMPC:752-784) on tail lane c (four-lane layout, all four lanes
// of the quad active): lane c decodes component c of every leg from the new parameters `nb` (decode_leg at step 0.0,
// horizon_leg 1), shapes and clips it as shape_leg does (the rollout's component form), then one Euler step from
// the prepared rigid-body terms.  ts: the lane's merge_tail_lane row.  One straight-line read of the legs' parameters
// per kind, so the reads issue together.  merge_body and fast_tail share it, so both give the same bits.
__device__ __forceinline__ void merge_tail_grf(int c, const float* ts, const float* nb, float f[4], float& p, float& v,
                                               float& r, float& w) {
    const float* tail_pre = ts;
    const QuadRB rb{ts[13], ts[14], ts[15], ts[16], ts[17]};
    const int kind = __float_as_int(ts[18]), H = __float_as_int(ts[19]), PL = __float_as_int(ts[20]),
              S = __float_as_int(ts[21]), fidx = __float_as_int(ts[22]);
    const float fq = ts[23], fomq = ts[24], fa = ts[25], fb = ts[26], fc = ts[27], fd = ts[28];
    const float gmin = ts[29], gmax = ts[30], mu = ts[31], neg_mu = ts[32];
    float raw[4];
    if (kind == SRBD_ZERO_ORDER) {
#pragma unroll
        for (int l = 0; l < 4; ++l) raw[l] = nb[l * PL + c * H];
    } else if (kind == SRBD_LINEAR_SPLINE) {
        float x0[4], x1[4];
        const int o = fidx + c * (S + 1);
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            x0[l] = nb[l * PL + o];
            x1[l] = nb[l * PL + o + 1];
        }
#pragma unroll
        for (int l = 0; l < 4; ++l) raw[l] = fomq * x0[l] + fq * x1[l];
    } else {
        float x[4][4];
        const int o = 10 * fidx + 4 * c;
#pragma unroll
        for (int l = 0; l < 4; ++l)
#pragma unroll
            for (int k = 0; k < 4; ++k) x[l][k] = nb[l * PL + o + k];
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const float p0 = x[l][0], p1 = x[l][1], p2 = x[l][2], p3 = x[l][3];
            const float phi = 0.5f * ((p2 - p1) + (p1 - p0));
            const float phin = 0.5f * ((p3 - p2) + (p2 - p1));
            raw[l] = fa * p1 + fb * phi + fc * p2 + fd * phin;
        }
    }
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        const float cl = tail_pre[1 + l];
        const float zp = clamp_cs((tail_pre[0] + raw[l]) * cl, gmin, gmax);
        const float xy = third(raw[l] * cl);
        const float fz = qp<QP_B2>(c == 2 ? zp : xy);
        f[l] = c == 2 ? fz : clamp_cs(xy, neg_mu * fz, mu * fz);
    }
    p = tail_pre[5], v = tail_pre[6], r = tail_pre[7], w = tail_pre[8];
    const float c0 = tail_pre[1], c1 = tail_pre[2], c2 = tail_pre[3], c3 = tail_pre[4];
    const float temp = (f[0] * c0 + f[1] * c1) + (f[2] * c2 + f[3] * c3);  // integrate()'s order
    const float temp2 = (quad_cross(tail_pre[9] - p, f[0]) * c0 + quad_cross(tail_pre[10] - p, f[1]) * c1) +
                        (quad_cross(tail_pre[11] - p, f[2]) * c2 + quad_cross(tail_pre[12] - p, f[3]) * c3);
    {  // quad_rb_apply with the copies of inv_m / dt and this lane's constants
        const float lin = ts[33] * temp + ts[39];
        const float Rt = rb.R0 * qp<QP_B0>(temp2) + rb.R1 * qp<QP_B1>(temp2) + rb.R2 * qp<QP_B2>(temp2);
        const float a2 = ts[36] * qp<QP_B0>(Rt) + ts[37] * qp<QP_B1>(Rt) + ts[38] * qp<QP_B2>(Rt);
        const float aa = -rb.a1 + a2;
        const float dt = ts[34];
        const float pn = p + v * dt, vn = v + lin * dt, rn = r + rb.er * dt, wn = w + aa * dt;
        p = pn;
        v = vn;
        r = rn;
        w = wn;
    }
}

// smem: [STAGE: records] | scale[nrec_pad] | tree levels | node keys | erow[K*ncol] (merge_smem_bytes).  prestaged
// (STAGE): the records are already in smem.  The staged body's sums use G = MERGE_STAGE_THREADS / (ncol + 1)
// record groups whatever NT is, so a 256-thread block merges bit for bit as the 512-thread kernel does.
template <int NT, bool STAGE, bool SPLITX = false>
__device__ __forceinline__ void merge_body(const ModelConst& mc, StepInput* __restrict__ in,
                                           const float* __restrict__ recs, int nrec, int rec_stride, int rows_in_rec,
                                           const float* __restrict__ noise, float* __restrict__ rank_out,
                                           StepOutput* __restrict__ out, int chain, int ctr_inc,
                                           uint64_t* __restrict__ dbg, uint32_t* __restrict__ flag, uint32_t seq,
                                           int split_cs, int fence_sys, MergeShared<NT>& sh, float* smem,
                                           bool prestaged = false, int levels_up = 0, SplitXchg* xg = nullptr) {
    constexpr int NW = NT / 64;
    uint64_t* red = sh.red;
    uint64_t* elite = sh.elite;
    int* elite_src = sh.elite_src;
    TopkLds<NT>& tk = sh.tk;
    float* Vs = sh.Vs;
    float* nb = sh.nb;
    float& tag_sh = sh.tag_sh;
    auto& tail_sh = sh.tail_sh;
    const int sblk = split_cs > 0 ? (int)blockIdx.x : 0;  // stamps: a split launch's blocks 0 and 1, else this block
#define MERGE_STAMP(i) \
    if (dbg && threadIdx.x == 0 && sblk < 2) dbg[32 * sblk + (i)] = __builtin_amdgcn_s_memrealtime()
    // finer marks (diagnostic build of the phases call only: dbg[16 + i])
#define MERGE_MARK(i) MERGE_STAMP(16 + (i))
    MERGE_STAMP(0);
    if (dbg && threadIdx.x == 0 && sblk < 2) dbg[32 * sblk + 8] = __builtin_amdgcn_s_memtime();  // clock

    // T: the launch's block size, a template constant (blockDim.x is a dependent load)
    const int tid = threadIdx.x, T = NT, lane = tid & 63, wv = tid >> 6;
    const int P = mc.P, K = mc.K;
    const bool rs = mc.method == SRBD_RANDOM_SAMPLING, cem = mc.method == SRBD_CEM_MPPI;
    const bool split = split_cs > 0;
    const bool tailblk = split && blockIdx.x == 0;
    const bool sysout = flag != nullptr;  // outputs read by the host after the flag
    // Unsplit: the step outputs are assembled in LDS and written out in one burst at the end, so no
    // wave waits for a host store's completion mid-merge (a wave overwriting a register of a pending
    // store waits vmcnt(0), ~1 us for a PCIe write) and the publish waits for one round of them.
    // A column split's tail block assembles its outputs (its tail columns of best, the GRFs, the prediction and the
    // scalars) the same way and bursts only those (C3: its direct host stores cost ~1 us of register-reuse waits).
    float* osh = sh.osh;
    const bool shadow = !split || tailblk;
    auto ostore = [&](void* dst, float v) {
        if (shadow)
            osh[reinterpret_cast<float*>(dst) - reinterpret_cast<float*>(out)] = v;
        else if (sysout)
            __hip_atomic_store(reinterpret_cast<uint32_t*>(dst), __float_as_uint(v), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        else
            *reinterpret_cast<float*>(dst) = v;
    };
    // this block's columns: local index i -> parameter column jc(i)
    const int j0 = split && !tailblk ? ((int)blockIdx.x - 1) * split_cs : 0;
    const int ncol = !split ? P : (tailblk ? mc.ntail : min(split_cs, P - j0));
    auto jc = [&](int i) { return tailblk ? (int)mc.tailc[i] : j0 + i; };
    // parameters this block writes: all (unsplit), the tail columns (tail block), the others (slices)
    auto owns = [&](int jj) { return !split || tailblk || !is_tail_col(mc, jj); };
    const bool do_tail = out && (!split || tailblk);
    const int cols = ncol + 1;
    const int nrec_pad = (nrec + 3) & ~3;
    // the tree levels above the input records (merge_smem_bytes): even levels in lvA / nkA (n1 nodes at most), odd
    // levels in lvB / nkB (n1b), this block's cols columns each
    const int n1 = (nrec + TREE_FAN - 1) / TREE_FAN, n1b = (n1 + TREE_FAN - 1) / TREE_FAN;
    const int lvfA = (n1 * cols + 3) & ~3, lvfB = (n1b * cols + 3) & ~3;
    float* stage = smem;
    float* scale = STAGE ? smem + (size_t)nrec * rec_stride : smem;
    float* lvA = scale + nrec_pad;
    float* lvB = lvA + lvfA;
    uint64_t* nkA = reinterpret_cast<uint64_t*>(lvB + lvfB);  // 8-byte aligned: lvf* and nrec_pad are multiples of 4
    uint64_t* nkB = nkA + n1;
    float* erow = reinterpret_cast<float*>(nkB + n1b);

    // ---- L: loads.  The StepInput fields the output phases need are fetched first, so their latency
    // hides under the record loads instead of stalling the tail.
    const float best_pre = (out && tid < ncol && owns(jc(tid))) ? in->best[jc(tid)] : 0.0f;
    const int qc = tid < 3 ? tid : 2;  // tail lanes 0..3: component of the four-lane layout
    const bool tail_lane = do_tail && tid < 4;
    float tail_pre[13];  // kept in tail_sh across the merge (register pressure: 1024-thread block)
    if (tail_lane) merge_tail_load(in, qc, tail_pre);
    const float state_hi = (do_tail && tid >= 12 && tid < 24) ? in->state[tid] : 0.0f;
    // the predicted state's force-independent part (NMPC:752-784 via CMJ:93-174), formed while the
    // record loads are in flight
    auto tail_prep = [&]() {
        if (tail_lane) merge_tail_lane(mc, qc, tail_pre, tail_sh[tid]);
    };
    if constexpr (STAGE) {
        constexpr int U = 8;
        const int n4 = (nrec * rec_stride) >> 2;
        const float4* __restrict__ src = reinterpret_cast<const float4*>(recs);
        float4* dst = reinterpret_cast<float4*>(stage);
        auto chunk = [&](int base, bool first) __attribute__((always_inline)) {
            float4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = base + u * T + tid;
                v[u] = i < n4 ? src[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            }
            if (first) {
                tail_prep();
                MERGE_STAMP(7);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = base + u * T + tid;
                if (i < n4) dst[i] = v[u];
            }
        };
        if (prestaged) {
            tail_prep();
        } else {
            chunk(0, true);
            for (int base = U * T; base < n4; base += U * T) chunk(base, false);
        }
        __syncthreads();
        MERGE_STAMP(6);
        recs = stage;
    }
    // ---- 1. beta.  Staged: only the waves holding a record scan and reduce (nrec <= RPT * T, but a
    // step's few hundred records sit in the first waves), and the block minimum is over those waves.
    uint64_t mine = KEY_NONE, kk0 = KEY_NONE;
    float mtag = 0.0f;
    // the top-K's record minima are these headers' keys: kept for it when one chunk holds them all
    // Column split (SplitXchg after the StepInput): the slices fold every column's sums and publish them; the tail
    // block folds none and reads its columns' sums back.  CEM: the tail block computes the top-K once and publishes
    // it; the slices read it back (each slice recomputed both before: C3 merge 15.5 -> 12.8 us).
    const bool hand = SPLITX && split && !rs;  // SPLITX: merge_kernel, the only split launch, passes xg
    const uint32_t ep = hand ? __hip_atomic_load(&xg->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u : 0u;
    // a hand-off word (SplitXchg): polled until it carries this launch's tag, bounded (the tail block reports a
    // timed-out wait as status 1)
    int hand_late = 0;
    auto poll = [&](const uint64_t* w) -> uint32_t {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint64_t v;
        while ((uint32_t)((v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) != ep) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > XCHG_TIMEOUT_TICKS) {
                hand_late = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        return (uint32_t)v;
    };
    auto tagged = [&](uint32_t x) { return ((uint64_t)ep << 32) | x; };
    const bool topk_here = K > 1 && !rank_out && (!split || tailblk);
    const bool pre_topk = topk_here && nrec <= T;
    const int nhw = STAGE ? (nrec + 63) >> 6 : NW;  // waves that hold a record (staged: <= RPT * NW)
    // the tree's first level rides along (srbd_core.h: 32 consecutive records per node, so a node is a 32-lane half
    // of a wave here): its node keys (nkA) and each record's scale exp(-(m_r - m_node)), formed in this pass
    if (!STAGE || wv < nhw) {
#pragma unroll
        for (int i = 0; i < MERGE_RPT; ++i) {
            if (i * T >= nrec) break;
            const int r = tid + i * T;
            uint64_t kk = KEY_NONE;
            float m_r = 0.0f;
            if (r < nrec) {
                const float* R = recs + (size_t)r * rec_stride;
                m_r = R[0];
                kk = ((uint64_t)f2u(m_r) << 32) | (uint64_t)f2u(R[2]);
                const float tg = R[3];
                mtag = kk < mine ? tg : mtag;
                mine = umin64(mine, kk);
            }
            if (i == 0) kk0 = kk;
            if (!rs) {
                uint64_t nlo, nhi;
                half_wave_min_u64(kk, &nlo, &nhi);
                const uint64_t nk = lane < 32 ? nlo : nhi;
                if (r < nrec) {
                    if ((r & (TREE_FAN - 1)) == 0) nkA[r / TREE_FAN] = nk;
                    scale[r] = expf(-1.0f * (m_r - u2f((uint32_t)(nk >> 32))));
                }
            }
        }
        const uint64_t wmin = wave_min_u64(mine);
        if (lane == 0 && wv < NW) red[wv] = wmin;
    }
    if (pre_topk) {  // block_topk_nodes' entry state
        tk.keys[tid] = kk0;
        if (tid < MAXK) {
            tk.sel[tid] = -1;
            tk.top[tid] = KEY_NONE;
        }
        for (int i = tid; i < K * K; i += T) {
            tk.cand[i] = KEY_NONE;
            tk.cnt[i] = 0;
        }
    }
    MERGE_MARK(0);
    if constexpr (!STAGE)
        if (!(SPLITX && hand && tailblk)) tail_prep();  // a hand-off tail block: after its top-K (off its critical path)
    MERGE_MARK(1);
    __syncthreads();
    MERGE_MARK(2);
    uint64_t bkey = red[0];
    for (int i = 1; i < (STAGE ? (nhw < NW ? nhw : NW) : NW); ++i) bkey = umin64(bkey, red[i]);
    const float beta = u2f((uint32_t)(bkey >> 32));
    if (mine == bkey && mine != KEY_NONE) tag_sh = mtag;  // keys are unique: one writer
    MERGE_STAMP(1);

    // ---- 2./3. the reduction tree's sums (srbd_core.h): the input records folded level by level, TREE_FAN
    // consecutive children per node in order (the fold of fold_node_lds, srbd_device.h), to the root -- or, for a
    // rank record (rank_out), `levels_up` levels, up to this rank's nodes of the exchange level.  Every block of a
    // column split folds its own columns; all recompute the node keys the same way.
    auto off_of = [&](int jj) { return jj < ncol ? REC_HDR + jc(jj) : 1; };
    int nlev = nrec;            // nodes of the current level
    bool lev_recs = true;       // the current level is the input records
    const float* lvp = nullptr;  // values of the current level (lev_recs: the records)
    const uint64_t* nkp = nullptr;
    if (!rs && !(hand && tailblk)) {
        float* lv_out = lvA;
        uint64_t* nk_out = nkA;
        for (int L = 0; rank_out ? L < levels_up : nlev > 1; ++L) {
            const int n2 = (nlev + TREE_FAN - 1) / TREE_FAN;
            // level 0's keys and scales came with the beta pass; above it, one wave per node, lane = child
            for (int g2 = wv; L > 0 && g2 < n2; g2 += NW) {
                const int c = TREE_FAN * g2 + lane;
                const bool have = lane < TREE_FAN && c < nlev;
                const uint64_t kc = !have ? KEY_NONE
                                          : lev_recs ? ((uint64_t)f2u(recs[(size_t)c * rec_stride]) << 32) |
                                                           (uint64_t)f2u(recs[(size_t)c * rec_stride + 2])
                                                     : nkp[c];
                const uint64_t k = wave_min_u64(kc);
                if (lane == 0) nk_out[g2] = k;
                if (have) scale[c] = expf(-1.0f * (u2f((uint32_t)(kc >> 32)) - u2f((uint32_t)(k >> 32))));
            }
            if (L > 0) __syncthreads();
            if (L == 1) MERGE_MARK(6);
            for (int q = tid; q < n2 * cols; q += T) {  // (node, column) sums, child by child
                const int g2 = (int)((uint32_t)q / (uint32_t)cols), jq = (int)((uint32_t)q % (uint32_t)cols);
                const int c0 = TREE_FAN * g2, nc = min(TREE_FAN, nlev - c0);
                const float* src = lev_recs ? recs + (size_t)c0 * rec_stride + off_of(jq) : lvp + (size_t)c0 * cols + jq;
                const int sstride = lev_recs ? rec_stride : cols;
                float a = 0.0f;
                int cb = 0;
                for (; cb + 8 <= nc; cb += 8) {  // 8 children's loads in flight, then their adds in order
                    float x[8], sc[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        x[u] = src[(size_t)(cb + u) * sstride];
                        sc[u] = scale[c0 + cb + u];
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) a = a + sc[u] * x[u];
                }
                for (; cb < nc; ++cb) a = a + scale[c0 + cb] * src[(size_t)cb * sstride];
                lv_out[(size_t)g2 * cols + jq] = a;
            }
            __syncthreads();
            if (L == 0) MERGE_MARK(4);
            if (L == 1) MERGE_MARK(7);
            lvp = lv_out;
            nkp = nk_out;
            lev_recs = false;
            nlev = n2;
            lv_out = lv_out == lvA ? lvB : lvA;
            nk_out = nk_out == nkA ? nkB : nkA;
        }
        MERGE_MARK(5);
        if (!rank_out)  // the root
            for (int jj = tid; jj < cols; jj += T) Vs[jj] = lev_recs ? recs[off_of(jj)] : lvp[jj];
    }
    if (SPLITX && hand && !tailblk) {  // a slice publishes its columns' sums (block 1 also the weights' sum)
        __syncthreads();
        // srbd_debug_split_drop (tests): block 1 withholds the weights' sum, so the tail block's wait times out
        const bool drop = blockIdx.x == 1 && __hip_atomic_load(&xg->drop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int i = tid; i <= ncol; i += T)
            if (i < ncol || (blockIdx.x == 1 && !drop))
                __hip_atomic_store(&xg->sums[i < ncol ? jc(i) : P], tagged(f2u(Vs[i])), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    }
    MERGE_STAMP(2);

    if (rank_out) {  // ---- a rank record: this rank's nodes of the exchange level (unsplit: column i == i)
        const int rstride = rec_floats_rank(P, K);
        int span = 1;
        for (int L = 0; L < levels_up; ++L) span *= TREE_FAN;
        const bool zs = zs_scaled(mc, in);
        const int nout = (nrec + span - 1) / span;  // == nlev after the folds (random sampling folds no sums)
        for (int g = 0; g < nout; ++g) {
            const int r0 = g * span, r1 = min(r0 + span, nrec);
            float* R = rank_out + (size_t)g * rstride;
            // the node's key (its records' minimum) and the tag of the record holding it
            uint64_t km = KEY_NONE;
            for (int r = r0 + tid; r < r1; r += T)
                km = umin64(km, ((uint64_t)f2u(recs[(size_t)r * rec_stride]) << 32) | f2u(recs[(size_t)r * rec_stride + 2]));
            km = wave_min_u64(km);
            __syncthreads();
            if (lane == 0) red[wv] = km;
            __syncthreads();
            uint64_t nk = red[0];
            for (int i = 1; i < NW; ++i) nk = umin64(nk, red[i]);
            for (int r = r0 + tid; r < r1; r += T)
                if ((((uint64_t)f2u(recs[(size_t)r * rec_stride]) << 32) | f2u(recs[(size_t)r * rec_stride + 2])) == nk)
                    tag_sh = recs[(size_t)r * rec_stride + 3];
            if (K == 1) {
                if (tid == 0) elite[0] = nk;
            } else {
                block_topk_rank<NT>(recs + (size_t)r0 * rec_stride, r1 - r0, rec_stride, P, K, elite, tk);
            }
            __syncthreads();
            for (int jj = tid; jj < P; jj += T)
                R[REC_HDR + jj] = rs ? 0.0f : (lev_recs ? recs[(size_t)g * rec_stride + REC_HDR + jj] : lvp[(size_t)g * cols + jj]);
            for (int e = tid; e < K; e += T) {
                R[REC_HDR + P + 2 * e] = u2f((uint32_t)elite[e]);
                R[REC_HDR + P + 2 * e + 1] = u2f((uint32_t)(elite[e] >> 32));
            }
            const bool rows = rs || cem;  // the rows the root needs: random sampling's best, CEM's elite
            for (int t = tid; t < K * P; t += T) {
                const int e = t / P, jj = t % P;
                float v = 0.0f;
                if (rows && elite[e] != KEY_NONE) {
                    v = noise[(size_t)jj * mc.ldn + ((int)(uint32_t)elite[e] - mc.row0)];
                    if (zs) v = v * in->sigma[jj];
                }
                R[REC_HDR + P + 2 * K + t] = v;
            }
            if (tid == 0) {
                R[0] = u2f((uint32_t)(nk >> 32));
                R[1] = rs ? 1.0f : (lev_recs ? recs[(size_t)g * rec_stride + 1] : lvp[(size_t)g * cols + P]);
                R[2] = u2f((uint32_t)nk);
                R[3] = tag_sh;
            }
            __syncthreads();
        }
        return;
    }

    // ---- 4. top-K keys (ascending; keys are unique).  The tail block of a CEM split never reads
    // elite rows (sigma belongs to the slices), so it skips them.
    const bool want_elite = !tailblk || rs;
    if (K == 1) {
        if (tid == 0) elite[0] = bkey;
    } else if (SPLITX && !topk_here) {  // a CEM slice: the tail block's keys (halves: little-endian words)
        if (tid < 2 * K) reinterpret_cast<uint32_t*>(elite)[tid] = poll(&xg->elite[tid]);
    } else {
        if (pre_topk)
            block_topk_nodes<NT>(recs, nrec, rec_stride, P, K, nkA, elite, tk, dbg);
        else
            block_topk_rank<NT>(recs, nrec, rec_stride, P, K, elite, tk);
        if (SPLITX && split) {  // the tail block publishes them
            __syncthreads();
            if (tid < 2 * K)
                __hip_atomic_store(&xg->elite[tid], tagged(reinterpret_cast<const uint32_t*>(elite)[tid]),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (SPLITX && hand && tailblk) {  // the tail block's sums: the slices'
        if constexpr (!STAGE) tail_prep();
        for (int i = tid; i <= ncol; i += T) Vs[i] = u2f(poll(&xg->sums[i < ncol ? jc(i) : P]));
        // any thread's timed-out word fails the step (status bit 1; the host then resets SplitXchg)
        hand_late = __syncthreads_or(hand_late);
        // every slice has stored its sums, so every slice has read the epoch: advance it for the next launch.  Not
        // after a timeout: a slice may not have read it yet (it would tag its late sums with the next launch's epoch)
        if (tid == 0 && !hand_late) __hip_atomic_store(&xg->epoch, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (SPLITX && hand && !tailblk && !topk_here && K > 1) hand_late = __syncthreads_or(hand_late);  // elite keys
    __syncthreads();
    // record slot of every elite key (needed when rows travel inside the records)
    const bool need_rows = want_elite && (rs || cem);  // MPPI's update is the weighted sum alone
    if (rows_in_rec && need_rows) {
        for (int t = tid; t < nrec * K; t += T) {
            const int r = t / K, q = t % K;
            const uint64_t x = rec_key(recs + (size_t)r * rec_stride, P, q);
            for (int e = 0; e < K; ++e)
                if (x == elite[e] && x != KEY_NONE) elite_src[e] = t;
        }
        __syncthreads();
    }
    MERGE_STAMP(3);

    // ---- 5. elite rows (this block's columns) -> LDS
    int Kv = 0;
    for (int e = 0; e < K; ++e) Kv += elite[e] != KEY_NONE;
    const bool zs = zs_scaled(mc, in);
    for (int t = tid; need_rows && t < K * ncol; t += T) {
        const int e = t / ncol, i = t % ncol, jj = jc(i);
        float v = 0.0f;
        if (elite[e] != KEY_NONE) {
            if (rows_in_rec) {
                const int st = elite_src[e];
                v = recs[(size_t)(st / K) * rec_stride + REC_HDR + P + 2 * K + (size_t)(st % K) * P + jj];
            } else {
                v = noise[(size_t)jj * mc.ldn + ((int)(uint32_t)elite[e] - mc.row0)];
                if (zs) v = v * in->sigma[jj];
            }
        }
        erow[t] = v;
    }
    __syncthreads();

    // ---- 6. outputs
    if (out) {
        for (int i = tid; i < ncol; i += T) {
            const int jj = jc(i);
            if (owns(jj)) {
                const float b0 = i == tid ? best_pre : in->best[jj];
                const float v = rs ? b0 + erow[i] : b0 + Vs[i] / Vs[ncol];
                nb[jj] = v;
                ostore(&out->best[jj], v);
            }
            if (cem && !tailblk) {  // NMPC:1075-1081
                float s = 0.0f;
                for (int e = 0; e < Kv; ++e) s = s + erow[e * ncol + i];
                const float mean = s / (float)Kv;
                float var = 0.0f;
                for (int e = 0; e < Kv; ++e) {
                    const float d = erow[e * ncol + i] - mean;
                    var = var + d * d;
                }
                var = var / (float)(Kv - 1);
                float sg = sqrtf(var + 1e-8f);
                sg = sg > 5.0f ? 5.0f : sg;
                sg = sg < 0.2f ? 0.2f : sg;
                ostore(&out->sigma[jj], sg);
                if (chain) in->sigma[jj] = sg;
            }
        }
        __syncthreads();
        MERGE_STAMP(4);
        if (tail_lane) {
            float ts[40];  // one batch of LDS reads
#pragma unroll
            for (int i = 0; i < 40; ++i) ts[i] = tail_sh[tid][i];
            const int c = qc;
            float f[4], p, v, r, w;
            merge_tail_grf(c, ts, nb, f, p, v, r, w);
            if (tid < 3) {
#pragma unroll
                for (int l = 0; l < 4; ++l) ostore(&out->grf[3 * l + c], f[l]);
                ostore(&out->pred[c], p);
                ostore(&out->pred[3 + c], v);
                ostore(&out->pred[6 + c], r);
                ostore(&out->pred[9 + c], w);
            }
        }
        if (do_tail && tid >= 12 && tid < 24) ostore(&out->pred[tid], state_hi);
        if (do_tail && tid == 0) {
            ostore(&out->best_cost, beta);
            ostore(&out->best_index, __uint_as_float((uint32_t)bkey));
            ostore(&out->best_freq, tag_sh);
            // a column split: the host zeroes status before the launch, and a late block ORs its bit in (below)
            if (!split) ostore(&out->status, __int_as_float(0));
            // chain: the next draws come from the device RNG.  (Split: slices read noise_scaled too, but a
            // chain's steps all run with it 0 already -- reset_noise_scaled -- so this store never changes it.)
            if (chain) in->noise_scaled = 0;
            if (chain && ctr_inc) advance_key(mc, in, ctr_inc);
        }
        if (chain)
            for (int i = tid; i < ncol; i += T) {
                const int jj = jc(i);
                if (owns(jj)) in->best[jj] = nb[jj];
            }
    }
    if (out && shadow) {  // the burst: best[P] | sigma[P] (CEM) | grf, pred, scalars
        __syncthreads();
        constexpr int TAILF = (int)((sizeof(StepOutput) - offsetof(StepOutput, grf)) / sizeof(float));
        constexpr int TAIL0 = (int)(offsetof(StepOutput, grf) / sizeof(float));
        constexpr int SIG0 = (int)(offsetof(StepOutput, sigma) / sizeof(float));
        constexpr int STAT = (int)(offsetof(StepOutput, status) / sizeof(float));
        // unsplit: the whole StepOutput; a split's tail block: its columns of best, then grf .. the scalars except
        // status (the host zeroed it; a late block ORs its bit in)
        const int nb0 = split ? ncol : P;
        const int nsig = cem && !split ? P : 0;
        float* o = reinterpret_cast<float*>(out);
        for (int t = tid; t < nb0 + nsig + TAILF; t += T) {
            const int k = t < nb0 ? (split ? jc(t) : t) : (t < nb0 + nsig ? SIG0 + (t - nb0) : TAIL0 + (t - nb0 - nsig));
            if (split && k == STAT) continue;
            if (sysout)
                __hip_atomic_store(reinterpret_cast<uint32_t*>(o + k), __float_as_uint(osh[k]), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            else
                o[k] = osh[k];
        }
    }
    MERGE_STAMP(5);
    MERGE_MARK(8);
    if (dbg && threadIdx.x == 0 && sblk < 2) dbg[32 * sblk + 9] = __builtin_amdgcn_s_memtime();
#undef MERGE_STAMP
#undef MERGE_MARK
    // a hand-off word of the column split never arrived (bounded poll): tail block bit 1, a slice bit 2
    if (SPLITX && hand && hand_late && tid == 0 && out)
        __hip_atomic_fetch_or(reinterpret_cast<uint32_t*>(&out->status), tailblk ? 1u : 2u, __ATOMIC_RELAXED,
                              sysout ? __HIP_MEMORY_SCOPE_SYSTEM : __HIP_MEMORY_SCOPE_AGENT);
    if (flag) {  // every thread's output writes have completed before thread 0 publishes `seq`
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            if (fence_sys) {
                __threadfence_system();
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __hip_atomic_store(flag + (split ? blockIdx.x : 0), seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <int NT, bool STAGE>
__global__ void __launch_bounds__(NT) merge_kernel(const ModelConst mc, StepInput* __restrict__ in,
                                                              const float* __restrict__ recs, int nrec,
                                                              int rec_stride, int rows_in_rec,
                                                              const float* __restrict__ noise,
                                                              float* __restrict__ rank_out,
                                                              StepOutput* __restrict__ out, int chain,
                                                              int ctr_inc, uint64_t* __restrict__ dbg,
                                                              uint32_t* __restrict__ flag, uint32_t seq,
                                                              int split_cs, int fence_sys,
                                                              const uint32_t* __restrict__ gate, int levels_up) {
    if (gate && (*gate & ARM_CANCEL)) {  // armed chain that did not fire (Publish::gate)
        if (threadIdx.x == 0 && flag)
            __hip_atomic_store(flag + (split_cs > 0 ? blockIdx.x : 0), seq | ARM_CANCEL, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    __shared__ MergeShared<NT> sh;
    extern __shared__ __attribute__((aligned(16))) float dsm[];
    merge_body<NT, STAGE, true>(mc, in, recs, nrec, rec_stride, rows_in_rec, noise, rank_out, out, chain, ctr_inc, dbg, flag,
                          seq, split_cs, fence_sys, sh, dsm, false, levels_up, reinterpret_cast<SplitXchg*>(in + 1));
}

// Sharded step without a collective launch (xGMI exchange).
//  1. pass 1 merges this rank's block records into its rank record (a cached stage slot);
//  2. the record goes to slot `rank` of every peer's mailbox as system-scope (sc0 sc1, write-through)
//     stores; every storing wave waits for its stores (vmcnt 0), then after a block barrier one lane
//     per peer makes a system release and sets that peer's flag for this rank to the next epoch
//     (*x.epoch + 1; mailboxes are uncached device memory, IPC-mapped over xGMI);
//  3. the block waits for the W-1 flags of its own mailbox (bounded: on timeout it records an error,
//     publishes a failed status and skips the outputs), copies the peers' slots into the stage with
//     system-scope loads (one parallel round trip; nothing is read from a cache) and
//  4. pass 2 merges the W rank records in rank order, exactly as srbd_step_finish does.
// Costs (MI355X, one rank): all-thread agent + system fences and a system acquire here cost 7 us per
// step; this form measures within noise of no release at all (scripts/sharded_probe.py).
// NT / STAGE1: pass 1 as the single-rank merge runs it -- the LDS-staged 512-thread body when this
// rank's block records fit (C2: 157), else the 1024-thread direct body; pass 2 (W records) direct.
// xchg_exchange: steps 2-3 for one block, after pass 1 has written this rank's buffer `mine` (= x.stage slot rank):
// returns false after publishing the failure when a peer timed out, true with the gathered buffers in x.stage.
template <int NT>
__device__ __forceinline__ bool xchg_exchange(const XchgArgs& x, const float* mine, StepOutput* out, uint32_t* flag,
                                              uint32_t seq) {
    const int tid = threadIdx.x, T = NT;
    const int stride = x.stride;  // one rank's buffer: its exchange-level node records (t_xmax of them)
    const uint32_t epoch = *x.epoch + 1;
    // slot parity: epoch & 1.  A peer can run at most one exchange ahead of this rank (it cannot pass
    // its next wait before this rank has published that epoch, i.e. finished copying this one), so
    // its epoch+1 record lands in the other half and never overwrites a slot still being copied.
    const size_t half = (size_t)(epoch & 1u) * x.world * stride;
    for (int i = tid; i < (x.world - 1) * stride; i += T) {
        const int q = i / stride, k = i - q * stride;
        const int p = q < x.rank ? q : q + 1;
        __hip_atomic_store(reinterpret_cast<uint32_t*>(x.peer_mailbox[p]) + half + (size_t)x.rank * stride + k,
                           __float_as_uint(mine[k]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid < x.world && tid != x.rank) {
        __threadfence_system();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(x.peer_flags[tid] + x.rank, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __shared__ int timed_out;
    if (tid == 0) timed_out = 0;
    __syncthreads();
    if (tid < x.world && tid != x.rank) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        // >= (wrap-safe): a peer one exchange ahead has already moved its flag on to epoch + 1
        while ((int32_t)(__hip_atomic_load(x.flags + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > XCHG_TIMEOUT_TICKS) {
                timed_out = 1;
                break;
            }
        }
    }
    __syncthreads();
    if (tid == 0) *x.epoch = epoch;
    if (timed_out) {
        if (tid == 0) {
            *x.err = 1;
            if (out) out->status = -1;
            __threadfence_system();
            if (flag) __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return false;
    }
    for (int i = tid; i < (x.world - 1) * stride; i += T) {
        const int q = i / stride, k = i - q * stride;
        const size_t o = (size_t)(q < x.rank ? q : q + 1) * stride + k;
        x.stage[o] = __uint_as_float(__hip_atomic_load(reinterpret_cast<const uint32_t*>(x.mailbox) + half + o,
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    }
    __syncthreads();
    return true;
}
template <int NT, bool STAGE1>
__global__ void __launch_bounds__(NT) merge_xchg_kernel(const ModelConst mc, StepInput* __restrict__ in,
                                                        const float* __restrict__ recs, int nrec, int rec_stride,
                                                        const float* __restrict__ noise, XchgArgs x,
                                                        StepOutput* __restrict__ out, int chain, int ctr_inc,
                                                        uint32_t* __restrict__ flag, uint32_t seq, int levels_up) {
    __shared__ MergeShared<NT> sh;  // both passes (they run one after the other)
    extern __shared__ __attribute__((aligned(16))) float dsm[];
    float* mine = x.stage + (size_t)x.rank * x.stride;
    merge_body<NT, STAGE1>(mc, in, recs, nrec, rec_stride, 0, noise, mine, nullptr, 0, 0, nullptr, nullptr, 0, 0, 1, sh,
                           dsm, false, levels_up);
    __syncthreads();
    if (!xchg_exchange<NT>(x, mine, out, flag, seq)) return;
    // pass 2: the ranks' buffers side by side are the exchange level's node list (tree_shape)
    merge_body<NT, false>(mc, in, x.stage, mc.t_xnodes, rec_floats_rank(mc.P, mc.K), 1, noise, nullptr, out, chain,
                          ctr_inc, nullptr, flag, seq, 0, 1, sh, dsm);
}



// In-launch final merge (zero-order four-lane rollout, host steps; launch_rollout with GroupArgs::out): a
// group's last arriver, its group record stored write-through, counts itself in *gdone; the block that
// completes the count (every group record is then in memory) copies the ngroups records into LDS with sc1
// loads and runs the single-block merge on them -- merge_body<NT, STAGE> with the record groups of the
// 512-thread kernel, so the outputs are merge_kernel's bit for bit -- writing the step outputs and
// publishing `seq` (and resets the count for the next launch).  The merge's LDS is carved from the rollout's
// noise stage, dead by then (final_merge_lds).  Saves the merge launch and its record staging: N = 65 536
// (see DESIGN.md).
template <int NT, bool XG>
__device__ void final_merge(const ModelConst& mc, const StepInput* in, const float* noise, int rec_stride,
                            const GroupArgs& grp, float* lds) {
    __shared__ int fin;
#ifdef SRBD_ROLLOUT_STAMPS
    const uint64_t f1 = __builtin_amdgcn_s_memrealtime();
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's group record stores have completed
    __syncthreads();
#ifdef SRBD_ROLLOUT_STAMPS
    const uint64_t f2 = __builtin_amdgcn_s_memrealtime();
#endif
    if (threadIdx.x == 0) {
        const uint32_t old = __hip_atomic_fetch_add(grp.gdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fin = old == (uint32_t)(grp.ngroups - 1);
    }
    __syncthreads();
    if (!fin) return;
    uint64_t* dbg = nullptr;
#ifdef SRBD_ROLLOUT_STAMPS
    if (threadIdx.x == 0) {
        g_fstamp[0] = blockIdx.x + 1;
        g_fstamp[1] = f1;
        g_fstamp[2] = f2;
        g_fstamp[3] = __builtin_amdgcn_s_memrealtime();
    }
    dbg = g_fstamp + 32;
#endif
    if (threadIdx.x == 0) __hip_atomic_store(grp.gdone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    MergeShared<NT>& sh = *reinterpret_cast<MergeShared<NT>*>(lds);
    float* smem = lds + (sizeof(MergeShared<NT>) + 15) / 16 * 4;  // 16-byte aligned
    stage_recs16<5>(grp.grecs, smem, grp.ngroups * rec_stride);  // sc1 loads (other CUs wrote the records)
    __syncthreads();
#ifdef SRBD_ROLLOUT_STAMPS
    if (threadIdx.x == 0) g_fstamp[4] = __builtin_amdgcn_s_memrealtime();
#endif
    // sharded (grp.xa): pass 0 folds this rank's buffer, the exchange gathers the ranks' buffers (the exchange
    // level's node list), pass 1 merges them into the outputs.  One merge_body call site for both passes.
    int nrec = grp.ngroups, stride = rec_stride;
    for (int pass = 0;; ++pass) {
        const bool rank_pass = XG && pass == 0;
        float* mine = rank_pass ? grp.xa->stage + (size_t)grp.xa->rank * grp.xa->stride : nullptr;
        merge_body<NT, true>(mc, const_cast<StepInput*>(in), smem, nrec, stride, 0, noise, mine,
                             rank_pass ? nullptr : grp.out, 0, 0, rank_pass ? nullptr : dbg,
                             rank_pass ? nullptr : grp.flag, grp.seq, 0,
                             grp.fence_sys, sh, smem, true, rank_pass ? grp.levels_up : 0);
        if (!rank_pass) return;
        __syncthreads();
        if (!xchg_exchange<NT>(*grp.xa, mine, grp.out, grp.flag, grp.seq)) return;
        nrec = mc.t_xnodes;
        stride = rec_floats_rank(mc.P, mc.K);
        for (int i = threadIdx.x; i < nrec * stride; i += NT) smem[i] = grp.xa->stage[i];
        __syncthreads();
    }
}

size_t final_merge_lds(const ModelConst& mc, int ngroups, int rec_stride) {
    const size_t a = sizeof(float) * (size_t)ngroups * rec_stride + merge_smem_bytes(ngroups, mc.P, mc.K);
    // a sharded step's second pass: the gathered node records
    const size_t b =
        sizeof(float) * (size_t)mc.t_xnodes * rec_floats_rank(mc.P, mc.K) + merge_smem_bytes(mc.t_xnodes, mc.P, mc.K);
    return (sizeof(MergeShared<256>) + 15) / 16 * 16 + (a > b ? a : b);
}

// ---- fast_tail: unsharded host steps whose launch folds level 1 into 2..TREE_FAN node records (GroupArgs::fast,
// fast_tail_ok; MPPI / random sampling, zero-order four-lane, FM = 1).  The tree's arithmetic is that of the level-1
// fold (fold_node_lds) and of merge_body over <= TREE_FAN records (one level to the root), operation for operation,
// so the bits equal the two-stage form's; what changes is the hand-offs after the last leaf record:
//  - a node's last arriving block counts itself in *gdone as soon as it knows (the count's round trip overlaps the
//    staging of the node's leaf records), instead of after its fold and the drain of its node record;
//  - headers are formed on every wave alike (lane c = child c) and broadcast through a per-wave LDS row, so the
//    column sums (thread j: column j, thread P: the weights' sum) follow without a block barrier;
//  - a folder that is not the last to count hands its node record over as 8-byte words tagged with the launch's seq
//    (the header words as soon as the node key is known) and exits.  The last to count keeps its own node's sums in
//    registers, loads the other nodes' words straight into registers (each polled until it carries seq) and folds
//    the root column by column;
//  - outputs: the root sums go to LDS; after a barrier thread j forms best[j] = best_in[j] + V[j] / V[P] and writes
//    it to the host (as a tagged word, tagged_outputs, or into StepOutput followed by the flag); after a second
//    barrier the tail lanes (wave 3, which holds no column) form the GRFs and the predicted state (merge_tail_grf).
// LDS (carved from the rollout's noise stage `st`, ft_lds_floats): the node's leaf records, nb[P], V[P + 1], the tail
// lanes' rows (4 x 40), per-wave broadcast rows (child scales, root scales: 2 x 4 x 64).
// The tagged node records (gtag, FT_GTAG_WORDS): header words [64 nodes][4] (m, -, best row, tag), then column
// words [node][P + 1] (v[0..P), s).  A word that never arrives (bounded wait) makes the step publish status -1.
__device__ __forceinline__ uint64_t tag_word(uint32_t seq, float v) { return ((uint64_t)seq << 32) | f2u(v); }
__device__ __forceinline__ void st_tag(uint64_t* p, uint64_t w) {
    __hip_atomic_store(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sys(void* p, float v) {
    __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
constexpr int FT_TAIL0 = 192;  // the tail lanes: a quad of wave 3 (the P + 1 <= 192 columns sit in waves 0-2)
__host__ __device__ constexpr int ft_lds_floats(int P, int rec_stride) {
    return TREE_FAN * rec_stride + ((P + 3) & ~3) + ((P + 4) & ~3) + 4 * 40 + 2 * 4 * 64;
}
// ---- shared by fast_tail and direct_tail: the step input the outputs need (read while the sums are formed) and the
// outputs themselves.
// ft_prep: the tail lanes' merge_tail_lane rows into tsh (the predicted state's force-independent part), best_in[j]
// (thread j < P) and the state's pass-through half (threads 12..23), through a global pointer: generic (flat) loads
// count in lgkmcnt too, so every LDS read after them would wait for their memory round trip (the kernel argument
// segment is global memory as well).
__device__ __forceinline__ void ft_prep(const ModelConst& mc, const StepInput* in, float* tsh, float& b0,
                                        float& state_hi) {
    const int tid = threadIdx.x, P = mc.P;
    const auto gin = (const __attribute__((address_space(1))) StepInput*)in;
    if (tid >= FT_TAIL0 && tid < FT_TAIL0 + 4) {
        const int qc = tid - FT_TAIL0 < 3 ? tid - FT_TAIL0 : 2;
        float tail_pre[13];
        merge_tail_load(gin, qc, tail_pre);
        merge_tail_lane(mc, qc, tail_pre, tsh + 40 * (tid - FT_TAIL0));
    }
    if (tid < P) b0 = gin->best[tid];
    if (tid >= 12 && tid < 24) state_hi = gin->state[tid];
}
// ft_outputs (merge_body's values), every thread of the block: vsh[0..P] holds the root sums (V[P] the weights' sum)
// on entry (written before a barrier the caller passed); `late` != 0 on any thread publishes status -1.
// best[j] = best_in[j] + V[j] / V[P] (random sampling: + the best row's noise), then the tail lanes' GRFs / prediction
// (wave 3).  Host steps (GroupArgs::outt) write them as 8-byte words tagged with seq (tagged_outputs): the host takes
// the step when every word carries it, so no wave waits for its stores and no flag follows them; else StepOutput +
// the flag after every wave's stores have completed.
__device__ __forceinline__ void ft_outputs(const ModelConst& mc, const GroupArgs& grp, const float* noise, bool rs,
                                           int late, uint64_t bk, float beta, float btag, float b0, float state_hi,
                                           float* nbv, const float* vsh, const float* tsh) {
    const int tid = threadIdx.x, j = tid, P = mc.P;
    const uint32_t seq = grp.seq;
    late = __syncthreads_or(late);
    StepOutput* out = grp.out;
    uint64_t* ot = grp.outt;
    auto put = [&](int w, float* dst, float v) {
        if (ot)
            __hip_atomic_store(ot + w, tag_word(seq, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else
            st_sys(dst, v);
    };
    if (j < P) {
        const float v = rs ? b0 + noise[(size_t)j * mc.ldn + ((int)(uint32_t)bk - mc.row0)] : b0 + vsh[j] / vsh[P];
        nbv[j] = v;
        put(j, &out->best[j], v);
    }
    if (tid >= 12 && tid < 24) put(P + 12 + tid, &out->pred[tid], state_hi);
    if (tid == 0) {
        put(P + 36, &out->best_cost, beta);
        put(P + 37, reinterpret_cast<float*>(&out->best_index), __uint_as_float((uint32_t)bk));
        put(P + 38, &out->best_freq, btag);
        put(P + 39, reinterpret_cast<float*>(&out->status), __int_as_float(late ? -1 : 0));
    }
    __syncthreads();  // nb complete for the tail lanes
    if (tid >= FT_TAIL0 && tid < FT_TAIL0 + 4) {
        const int qc = tid - FT_TAIL0 < 3 ? tid - FT_TAIL0 : 2;
        float ts[40];
#pragma unroll
        for (int i = 0; i < 40; ++i) ts[i] = tsh[40 * (tid - FT_TAIL0) + i];
        float f[4], p, v, r, w;
        merge_tail_grf(qc, ts, nbv, f, p, v, r, w);
        if (tid - FT_TAIL0 < 3) {
#pragma unroll
            for (int l = 0; l < 4; ++l) put(P + 3 * l + qc, &out->grf[3 * l + qc], f[l]);
            put(P + 12 + qc, &out->pred[qc], p);
            put(P + 15 + qc, &out->pred[3 + qc], v);
            put(P + 18 + qc, &out->pred[6 + qc], r);
            put(P + 21 + qc, &out->pred[9 + qc], w);
        }
    }
    if (!ot) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's output stores have completed
        __syncthreads();
    }
    if (tid == 0) {
        __hip_atomic_store(grp.gdone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
        if (!ot) __hip_atomic_store(grp.flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__device__ void fast_tail(const ModelConst& mc, const StepInput* in, const float* noise, const float* recs,
                          int rec_stride, const GroupArgs& grp, int nroll, float* st) {
    __shared__ int last_sh, fin_sh;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int P = mc.P, TWV = P + 1;  // TWV: column words of a tagged node record
    const bool rs = mc.method == SRBD_RANDOM_SAMPLING;
    const int g = (int)blockIdx.x / TREE_FAN;  // one leaf per four-lane block
    const int nblk = min(TREE_FAN, nroll - g * TREE_FAN);
    const int nb = min(TREE_FAN, mc.nleaf - g * TREE_FAN);  // the node's leaves
    const int ng = grp.ngroups;
    const uint32_t seq = grp.seq;
#ifdef SRBD_ROLLOUT_STAMPS  // probe build: thread 0's time at mark i of the last folder
#define FT_MARK(i) if (tid == 0) g_fstamp[i] = __builtin_amdgcn_s_memrealtime()
#else
#define FT_MARK(i)
#endif
    SRBD_LSTAMP(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's leaf record stores have completed
    __syncthreads();
    SRBD_LSTAMP(1);
    if (tid == 0) {
        const uint32_t old = __hip_atomic_fetch_add(grp.cnt + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_sh = old == (uint32_t)(nblk - 1);
    }
    __syncthreads();
    if (!last_sh) return;
    SRBD_LSTAMP(2);
    uint32_t gd = 0;
    if (tid == 0) {
        __hip_atomic_store(grp.cnt + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
        gd = __hip_atomic_fetch_add(grp.gdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    stage_recs16<5>(recs + (size_t)g * TREE_FAN * rec_stride, st, nb * rec_stride);  // sc1 loads (other CUs' records)
    if (tid == 0) fin_sh = gd == (uint32_t)(ng - 1);
    __syncthreads();
    SRBD_LSTAMP(3);
    const bool fin = fin_sh;
    float* nbv = st + TREE_FAN * rec_stride;  // the new parameters (the tail lanes read them)
    float* vsh = nbv + ((P + 3) & ~3);        // the root sums V[0..P]
    float* tsh = vsh + ((P + 4) & ~3);        // the tail lanes' merge_tail_lane rows, 4 x 40
    float* wsc = tsh + 4 * 40 + 64 * wv;      // this wave's broadcast rows: child scales,
    float* wnsc = wsc + 4 * 64;               // root scales
    const int j = tid;
    const bool col = !rs && j <= P;                  // column j (P: the weights' sum s)
    const int jw = j < P ? REC_HDR + j : 1;          // its word in a record
    float b0 = 0.0f, state_hi = 0.0f;
    if (fin) ft_prep(mc, in, tsh, b0, state_hi);  // in flight during the fold
    // ---- the node (fold_node_lds's arithmetic): key and child scales on every wave (lane c = child c)
    const float* R = st + (size_t)(lane < TREE_FAN ? lane : 0) * rec_stride;
    const bool have = lane < nb;
    const float m = have ? R[0] : 0.0f;
    const uint64_t key = have ? ((uint64_t)__float_as_uint(m) << 32) | __float_as_uint(R[2]) : KEY_NONE;
    const float r3 = have ? R[3] : 0.0f;
    const uint64_t gk = wave_min_u64(key);
    const float gm = __uint_as_float((uint32_t)(gk >> 32));
    const float sc = have ? (rs ? 1.0f : expf(-1.0f * (m - gm))) : 0.0f;
    const float gtg = __int_as_float(
        __builtin_amdgcn_readlane(__float_as_int(r3), (int)__builtin_ctzll(__builtin_amdgcn_ballot_w64(key == gk))));
    wsc[lane] = sc;  // this wave's row: read back below by its own lanes (in order, no barrier)
    uint64_t* GH = grp.gtag + 4 * g;                // node g's header words
    uint64_t* GV = grp.gtag + 256 + (size_t)g * TWV;  // its column words
    if (!fin && tid == 0) {  // the header words first: the last folder's root key needs them before the sums
        st_tag(GH, tag_word(seq, gm));
        st_tag(GH + 2, tag_word(seq, __uint_as_float((uint32_t)gk)));
        st_tag(GH + 3, tag_word(seq, gtg));
        if (rs) st_tag(GV + P, tag_word(seq, 1.0f));
    }
    SRBD_LSTAMP(4);
    // column j: sum_c sc_c x_c in child order (fold_node_lds), 8 children's LDS loads in flight
    float a = 0.0f;
    if (col) {
        const float* src = st + jw;
        int cb = 0;
        for (; cb + 8 <= nb; cb += 8) {
            float x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = src[(size_t)(cb + u) * rec_stride];
            const float4 y0 = *reinterpret_cast<const float4*>(wsc + cb);
            const float4 y1 = *reinterpret_cast<const float4*>(wsc + cb + 4);
            const float y[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
#pragma unroll
            for (int u = 0; u < 8; ++u) a = a + y[u] * x[u];
        }
        for (; cb < nb; ++cb) a = a + wsc[cb] * src[(size_t)cb * rec_stride];
    }
    SRBD_LSTAMP(5);
    if (!fin) {  // hand the node record over: tagged words, no drain, no second count
        if (col) st_tag(GV + j, tag_word(seq, a));
        return;
    }
    FT_MARK(1);  // own fold done
#ifdef SRBD_ROLLOUT_STAMPS
    if (tid == 0) g_fstamp[0] = blockIdx.x + 1;
#endif
    // ---- the other nodes' words into registers, batches of 8 nodes issued while below ng (all 32 at once spilled;
    // two batches of 16 issued 11 needless loads per thread at C2's 5 nodes), through a buffer descriptor (h
    // uniform: an SGPR offset, one VGPR of address per thread), sc1 as an agent-scope atomic load
    // has it.  Every load unconditional and unmasked (a branch per load, or a select on its result right after it,
    // costs a wait per load); the words a thread does not need are skipped by the poll (`need`) and the sums.  The
    // gtag allocation covers every address formed here; the poll's re-reads are kept apart by an asm memory clobber.
    constexpr int HB = TREE_FAN / 4;  // four batches of 8 nodes, only those below ng issued (C2's 5 nodes: one)
    const auto grs = __builtin_amdgcn_make_buffer_rsrc((void*)grp.gtag, (short)0, FT_GTAG_WORDS(P) * 8, 0x00020000);
    auto ldv = [&](int h) -> uint64_t {  // column word j of node h
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(grs, 8 * (256 + j), 8 * h * TWV, 16);
        return ((uint64_t)v[1] << 32) | v[0];
    };
    auto ldh = [&](int i) -> uint64_t {  // header word i of node `lane`
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(grs, 8 * (4 * lane + i), 0, 16);
        return ((uint64_t)v[1] << 32) | v[0];
    };
    const bool hv = lane < ng && lane != g;
    uint64_t xq[4][HB], hw[3];
    auto issue = [&](uint64_t(&x)[HB], int h0) {
#pragma unroll
        for (int u = 0; u < HB; ++u) x[u] = ldv(h0 + u);
    };
    hw[0] = ldh(0);
    hw[1] = ldh(2);
    hw[2] = ldh(3);
#pragma unroll
    for (int b = 0; b < 4; ++b)
        if (ng > b * HB) issue(xq[b], b * HB);
    FT_MARK(2);  // words issued
    int late = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    auto poll = [&](uint64_t* x, int n, auto&& need, auto&& reload) {  // bounded: re-read needed words not tagged seq
        for (;;) {
            bool p = false;
            for (int u = 0; u < n; ++u) p |= need(u) && (uint32_t)(x[u] >> 32) != seq;
            if (!p) return;
            if (__builtin_amdgcn_s_memrealtime() - t0 > XCHG_TIMEOUT_TICKS) {
                late = 1;
                return;
            }
            __builtin_amdgcn_s_sleep(1);
            asm volatile("" ::: "memory");  // the words may have changed: re-read them
            for (int u = 0; u < n; ++u)
                if (need(u) && (uint32_t)(x[u] >> 32) != seq) x[u] = reload(u);
        }
    };
    // ---- the root (merge_body over ng records, one level): key and scales on every wave alike
    poll(hw, 3, [&](int) { return hv; }, [&](int i) { return ldh(i == 0 ? 0 : i + 1); });
    FT_MARK(3);  // headers in
    const bool hl = lane < ng;
    const float mh = lane == g ? gm : __uint_as_float((uint32_t)hw[0]);
    const uint32_t rowh = lane == g ? (uint32_t)gk : (uint32_t)hw[1];
    const float th = lane == g ? gtg : __uint_as_float((uint32_t)hw[2]);
    const uint64_t kh = hl ? ((uint64_t)__float_as_uint(mh) << 32) | rowh : KEY_NONE;
    const uint64_t bk = wave_min_u64(kh);
    const float beta = __uint_as_float((uint32_t)(bk >> 32));
    const float nsc = hl && !rs ? expf(-1.0f * (mh - beta)) : 0.0f;
    const float btag = __int_as_float(
        __builtin_amdgcn_readlane(__float_as_int(th), (int)__builtin_ctzll(__builtin_amdgcn_ballot_w64(kh == bk))));
    wnsc[lane] = nsc;
    FT_MARK(4);  // root key and scales
    if (col) {
        // column j's root sum V = sum_h nsc_h x_h in node order (merge_body's level): straight-line over all TREE_FAN
        // nodes, each term added only for h < ng (V never holds -0, so skipping and adding nothing agree)
        float V = 0.0f;
        auto need = [&](int h) { return h < ng && h != g; };
        auto accum = [&](const uint64_t(&x)[HB], int h0) {
            float w[HB];  // this batch's scales (registers: a whole row beside the batches spilled)
#pragma unroll
            for (int q = 0; q < HB / 4; ++q) {
                const float4 t = *reinterpret_cast<const float4*>(wnsc + h0 + 4 * q);
                w[4 * q] = t.x, w[4 * q + 1] = t.y, w[4 * q + 2] = t.z, w[4 * q + 3] = t.w;
            }
#pragma unroll
            for (int u = 0; u < HB; ++u) {
                const int h = h0 + u;
                const float t = w[u] * (h == g ? a : __uint_as_float((uint32_t)x[u]));
                V = h < ng ? V + t : V;
            }
        };
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            if (ng > b * HB) {
                poll(xq[b], HB, [&](int u) { return need(b * HB + u); }, [&](int u) { return ldv(b * HB + u); });
                if (b == 0) FT_MARK(6);  // batch A in
                if (b == 3) FT_MARK(8);  // the last batch in
                accum(xq[b], b * HB);
            }
        }
        vsh[j] = V;
    }
    FT_MARK(9);  // root sums
    FT_MARK(10);
    ft_outputs(mc, grp, noise, rs, late, bk, beta, btag, b0, state_hi, nbv, vsh, tsh);
    FT_MARK(13);  // published
#undef FT_MARK
}

// fast_tail's LDS fits the zero-order noise stage, the P + 1 columns sit in waves 0-2 (wave 3's quad is the tail's),
// and the root is one level.
bool fast_tail_ok(const ModelConst& mc, int mode, int ngroups, int rec_stride) {
    if (!final_merge_ok(mc, mode, ngroups, rec_stride) || ngroups < 2 || ngroups > TREE_FAN || mc.P + 1 > FT_TAIL0)
        return false;
    const int zst = 64 * (12 * mc.H + 1) > GROUP_LDS_FLOATS ? 64 * (12 * mc.H + 1) : GROUP_LDS_FLOATS;
    return ft_lds_floats(mc.P, rec_stride) <= zst;
}

// The step input as a kernel argument (StepInputK): zero-order H 10 / 12 rollouts (four-lane with the LDS noise
// stage, or the thread form), MPPI / random sampling (no sigma in the argument), P <= KSI_MAXP.
bool ks_ok(const ModelConst& mc, int mode) {
    if ((mode != ROLLOUT_QUAD && mode != ROLLOUT_THREAD) || mc.kind != SRBD_ZERO_ORDER) return false;
    return (mc.H == 10 || mc.H == 12) && mc.method != SRBD_CEM_MPPI && mc.P <= KSI_MAXP;
}

// The in-launch final merge: the zero-order four-lane kernel with the LDS noise stage (H 10 / 12), MPPI / random
// sampling, grouped records, and the merge's LDS inside the stage (64 x (12 H + 1) floats).
bool final_merge_ok(const ModelConst& mc, int mode, int ngroups, int rec_stride) {
    // (the gait-adaptive rollout and the cost terms, which can be switched on later, are checked per launch)
    if (mode != ROLLOUT_QUAD || mc.kind != SRBD_ZERO_ORDER) return false;
    if ((mc.H != 10 && mc.H != 12) || mc.method == SRBD_CEM_MPPI || ngroups < 1) return false;
    const size_t zst =
        sizeof(float) * (size_t)(64 * (12 * mc.H + 1) > GROUP_LDS_FLOATS ? 64 * (12 * mc.H + 1) : GROUP_LDS_FLOATS);
    return final_merge_lds(mc, ngroups, rec_stride) <= zst;
}

__global__ void advance_kernel(const ModelConst mc, StepInput* __restrict__ in, const StepOutput* __restrict__ out) {
    for (int j = threadIdx.x; j < mc.P; j += blockDim.x) {
        in->best[j] = out->best[j];
        if (mc.method == SRBD_CEM_MPPI) in->sigma[j] = out->sigma[j];
    }
    if (threadIdx.x == 0) advance_key(mc, in, 1);
}

__global__ void div_selftest_kernel(const float* a, const float* b, int n, float* o) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float d = b[i];
    if (d == 3.0f) {
        o[i] = div3(a[i]);
    } else {
        const float r = 1.0f / d;
        o[i] = div_by(a[i], d, r);
    }
}

// ------------------------------------------------------------------ launchers
template <int KIND, int HT, int ST, bool EXT = false>
static void launch_rollout_t(const ModelConst& mc, const StepInput* in, const float* noise, float* costs,
                             float* recs, int rec_stride, int mode, int threads, hipStream_t s, const RngJob* next,
                             const GroupArgs& grp) {
    const RngJob job = next ? *next : RngJob{nullptr, 0, 0, 0, 0};
    const int extra = next ? (rng_grid(mc) < 1024 ? rng_grid(mc) : 1024) : 0;
    const bool cem = mc.method == SRBD_CEM_MPPI;
    if (mode == ROLLOUT_QUAD) {  // `threads` = 4 lanes x samples per block (256 or 512)
        const int spb = threads / 4;
        const int blocks = (mc.n_local + spb - 1) / spb;
        const dim3 grid(blocks + extra * 256 / threads);
        if constexpr (KIND == SRBD_ZERO_ORDER && (HT == 10 || HT == 12) && !EXT) {
            if (!cem && grp.ksi) {  // ks_ok: the step input as a kernel argument
                if constexpr (HT == 12) {
                    if (grp.gen && grp.out && !grp.xa && !next) {  // gen_ok: the launch makes the step's draws
                        hipLaunchKernelGGL((rollout_quad_kernel<KIND, HT, ST, false, false, 1, true, true>), grid,
                                           dim3(threads), 0, s, *static_cast<const StepInputK*>(grp.ksi), mc, in,
                                           noise, costs, recs, rec_stride, job, blocks, grp);
                        return;
                    }
                }
                if (grp.out && grp.xa)
                    hipLaunchKernelGGL((rollout_quad_kernel<KIND, HT, ST, false, false, 2, true>), grid, dim3(threads),
                                       0, s, *static_cast<const StepInputK*>(grp.ksi), mc, in, noise, costs, recs, rec_stride, job, blocks, grp);
                else if (grp.out)
                    hipLaunchKernelGGL((rollout_quad_kernel<KIND, HT, ST, false, false, 1, true>), grid, dim3(threads),
                                       0, s, *static_cast<const StepInputK*>(grp.ksi), mc, in, noise, costs, recs, rec_stride, job, blocks, grp);
                else
                    hipLaunchKernelGGL((rollout_quad_kernel<KIND, HT, ST, false, false, 0, true>), grid,
                                       dim3(threads), 0, s, *static_cast<const StepInputK*>(grp.ksi), mc, in, noise, costs, recs, rec_stride, job, blocks,
                                       grp);
                return;
            }
            if (grp.out && !cem) {  // final_merge_ok: the in-launch final merge
                if (grp.xa)
                    hipLaunchKernelGGL((rollout_quad_kernel<KIND, HT, ST, false, false, 2>), grid, dim3(threads), 0, s,
                                       KsNone{}, mc, in, noise, costs, recs, rec_stride, job, blocks, grp);
                else
                    hipLaunchKernelGGL((rollout_quad_kernel<KIND, HT, ST, false, false, 1>), grid, dim3(threads), 0, s,
                                       KsNone{}, mc, in, noise, costs, recs, rec_stride, job, blocks, grp);
                return;
            }
        }
        if (cem)
            hipLaunchKernelGGL((rollout_quad_kernel<KIND, HT, ST, true, EXT>), grid, dim3(threads), 0, s, KsNone{}, mc, in, noise,
                               costs, recs, rec_stride, job, blocks, grp);
        else
            hipLaunchKernelGGL((rollout_quad_kernel<KIND, HT, ST, false, EXT>), grid, dim3(threads), 0, s, KsNone{}, mc, in, noise,
                               costs, recs, rec_stride, job, blocks, grp);
    } else {
        launch_rollout_thread(mc, in, noise, costs, recs, rec_stride, threads, s, next, grp);
    }
}

bool rollout_specialised(int kind, int H, int S) {
    if (kind == SRBD_ZERO_ORDER) return H == 10 || H == 12 || H == 16;
    return S == 2 && (H == 12 || H == 16);
}

// Same samples per block as the context's rollout mode (the merge reads one record per block).
static void launch_rollout_ga(const ModelConst& mc, const StepInput* in, const float* noise, float* costs,
                              float* recs, int rec_stride, int mode, int threads, hipStream_t s, const RngJob* next,
                              const GroupArgs& grp) {
    const RngJob job = next ? *next : RngJob{nullptr, 0, 0, 0, 0};
    const int extra = next ? (rng_grid(mc) < 1024 ? rng_grid(mc) : 1024) : 0;
    const int spb = rollout_spb(mode, threads);
    const int blocks = (mc.n_local + spb - 1) / spb;
    if (mode == ROLLOUT_QUAD && !mc.cost_on) {  // four lanes per sample, `threads` per block
        const dim3 grid(blocks + extra * 256 / threads), block(threads);
#define SRBD_GQ(K, HH)                                                                                            \
    {                                                                                                              \
        hipLaunchKernelGGL((rollout_ga_quad_kernel<K, HH>), grid, block, 0, s, mc, in, noise, costs, recs, rec_stride, \
                           job, blocks, grp);                                                                           \
        return;                                                                                                    \
    }
        const int H = mc.H;
        switch (mc.kind) {
            case SRBD_ZERO_ORDER:
                if (H == 10) SRBD_GQ(SRBD_ZERO_ORDER, 10);
                if (H == 12) SRBD_GQ(SRBD_ZERO_ORDER, 12);
                if (H == 16) SRBD_GQ(SRBD_ZERO_ORDER, 16);
                SRBD_GQ(SRBD_ZERO_ORDER, 0);
            case SRBD_LINEAR_SPLINE:
                if (H == 12) SRBD_GQ(SRBD_LINEAR_SPLINE, 12);
                if (H == 16) SRBD_GQ(SRBD_LINEAR_SPLINE, 16);
                SRBD_GQ(SRBD_LINEAR_SPLINE, 0);
            default:
                if (H == 12) SRBD_GQ(SRBD_CUBIC_SPLINE, 12);
                if (H == 16) SRBD_GQ(SRBD_CUBIC_SPLINE, 16);
                SRBD_GQ(SRBD_CUBIC_SPLINE, 0);
        }
#undef SRBD_GQ
    }
    launch_rollout_ga_thread(mc, in, noise, costs, recs, rec_stride, spb, s, next, grp);
}

void launch_rollout(const ModelConst& mc, const StepInput* in, const float* noise, float* costs, float* recs,
                    int rec_stride, int mode, int threads, hipStream_t s, const RngJob* next, const GroupArgs& grp_in) {
    GroupArgs grp = grp_in;
    // No KS kernel for this launch: copy the input up instead.  Not reached from the library (the context
    // decides KS once, at create, with this same shape test, and passes no input to the gait-adaptive or
    // cost-term kernels); a blocking copy, since `ksi` is the caller's stack object.
    if (grp.ksi && (mc.ga || mc.cost_on || !ks_ok(mc, mode))) {
        (void)hipStreamSynchronize(s);
        (void)hipMemcpy(const_cast<StepInput*>(in), grp.ksi, sizeof(StepInputK), hipMemcpyHostToDevice);
        grp.ksi = nullptr;
    }
    if (mc.ga) return launch_rollout_ga(mc, in, noise, costs, recs, rec_stride, mode, threads, s, next, grp);
    const int H = mc.H, S = mc.S;
    // the opt-in cost terms (mc.cost_on): the EXT instantiations, on the same compile-time shapes (with
    // each step's terms pinned to their step they no longer spill: C2 24.6 vs 23.3 us/step without the
    // terms, C3 cubic H16 N=10 000 48.8 vs 47.3; the runtime-shape form took 68.7)
#define SRBD_LR(K, HH, SS)                                                                                        \
    return mc.cost_on                                                                                             \
               ? launch_rollout_t<K, HH, SS, true>(mc, in, noise, costs, recs, rec_stride, mode, threads, s, next, \
                                                   grp)                                                           \
               : launch_rollout_t<K, HH, SS, false>(mc, in, noise, costs, recs, rec_stride, mode, threads, s, next, grp)
    switch (mc.kind) {
        case SRBD_ZERO_ORDER:
            if (H == 10) SRBD_LR(SRBD_ZERO_ORDER, 10, 0);
            if (H == 12) SRBD_LR(SRBD_ZERO_ORDER, 12, 0);
            if (H == 16) SRBD_LR(SRBD_ZERO_ORDER, 16, 0);
            SRBD_LR(SRBD_ZERO_ORDER, 0, 0);
        case SRBD_LINEAR_SPLINE:
            if (S == 2 && H == 12) SRBD_LR(SRBD_LINEAR_SPLINE, 12, 2);
            if (S == 2 && H == 16) SRBD_LR(SRBD_LINEAR_SPLINE, 16, 2);
            SRBD_LR(SRBD_LINEAR_SPLINE, 0, 0);
        default:
            if (S == 2 && H == 12) SRBD_LR(SRBD_CUBIC_SPLINE, 12, 2);
            if (S == 2 && H == 16) SRBD_LR(SRBD_CUBIC_SPLINE, 16, 2);
            SRBD_LR(SRBD_CUBIC_SPLINE, 0, 0);
    }
#undef SRBD_LR
}

int group_size(const ModelConst& mc) {
    // the level-1 fold runs in the launch when the merge would read more than GROUP_MIN_LEAVES leaf records, and
    // the rank's rows start at a level-1 node (world 1, or an exchange level >= 1).  Not for CEM: its folds (the
    // K-key merge of 32 children on top of the sums) lengthen the rollout's tail by more than they take off the
    // merge (C3 rollout 29.6 vs 38.3 us, merge 17 vs 13 us).
    const bool use = mc.nleaf > GROUP_MIN_LEAVES && (mc.t_world == 1 || mc.t_xlevel >= 1) &&
                     mc.method != SRBD_CEM_MPPI;
    return use ? TREE_FAN : 1;
}

int rng_grid(const ModelConst& mc) {
    // Philox: one item per (row, column quad); the JAX stream: one per element
    const long items = (long)mc.n_local * (mc.rng != RNG_PHILOX ? mc.P : (mc.P + 3) / 4);
    const long blocks = (items + 255) / 256;
    return (int)(blocks < 2048 ? blocks : 2048);
}

void launch_rng(const ModelConst& mc, const StepInput* in, uint64_t seed, uint64_t ctr, int dev_ctr, int ctr_offset,
                float* noise, hipStream_t s, const uint32_t* gate) {
    const RngJob job{noise, seed, ctr, dev_ctr, ctr_offset, gate};
    hipLaunchKernelGGL(rng_kernel, dim3(rng_grid(mc)), dim3(256), 0, s, mc, in, job);
}

void launch_transpose(const float* src, int n, int P, int ldn, float* dst, hipStream_t s) {
    dim3 grid((n + 31) / 32, (P + 31) / 32);
    hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, s, src, n, P, ldn, dst);
}

size_t merge_smem_bytes(int nrec, int P, int K, int cols) {
    // scale[nrec_pad] | tree-level values n1 x cols | n1b x cols | node keys n1 | n1b | erow[K P]  (merge_body)
    if (cols <= 0) cols = P + 1;
    const int nrec_pad = (nrec + 3) & ~3, n1 = (nrec + TREE_FAN - 1) / TREE_FAN, n1b = (n1 + TREE_FAN - 1) / TREE_FAN;
    const size_t lvfA = ((size_t)n1 * cols + 3) & ~(size_t)3, lvfB = ((size_t)n1b * cols + 3) & ~(size_t)3;
    return sizeof(float) * ((size_t)nrec_pad + lvfA + lvfB + 2 * (size_t)(n1 + n1b) + (size_t)K * P);
}

int merge_split_cols(const ModelConst& mc) {
    if (MERGE_SPLIT_COLS >= mc.P) return 0;  // 0: one block
    const int lo = (mc.P + MERGE_MAX_BLOCKS - 2) / (MERGE_MAX_BLOCKS - 1);  // at most MERGE_MAX_BLOCKS flags
    return MERGE_SPLIT_COLS > lo ? MERGE_SPLIT_COLS : lo;
}

int merge_blocks(const ModelConst& mc) {
    const int cs = merge_split_cols(mc);
    return cs ? 1 + (mc.P + cs - 1) / cs : 1;
}

// LDS staging of the records (merge_body<true>): when the block's records fit beside the merge's own
// dynamic LDS.  The publish flag follows the system-scope output stores without a system fence (the
// stores are write-through to the host; every wave waits vmcnt(0) first, merge_body).
constexpr size_t MERGE_LDS_DYN_MAX = 140 * 1024;  // + the staged merge's static LDS (block_topk_rank) <= 160 KB
// the exchange kernel's static LDS holds both passes' merge_body arrays: its dynamic limit is this much lower
constexpr size_t XCHG_LDS_STATIC = 24 * 1024;
static bool merge_stage_fits(int nrec_block, int rec_stride, int P, int K, size_t* smem) {
    const size_t base = merge_smem_bytes(nrec_block, P, K);
    const size_t st = sizeof(float) * (size_t)nrec_block * rec_stride;
    if ((rec_stride & 3) == 0 && base + st <= MERGE_LDS_DYN_MAX &&
        nrec_block <= MERGE_RPT * MERGE_STAGE_THREADS) {
        *smem = base + st;
        return true;
    }
    *smem = base;
    return false;
}
// Called once per context before any launch (not during a graph capture).
void merge_prepare() {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&merge_kernel<MERGE_STAGE_THREADS, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)MERGE_LDS_DYN_MAX);
    // its static LDS holds both passes' arrays (21 KB): XCHG_LDS_STATIC less dynamic LDS (launch_merge_xchg)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&merge_xchg_kernel<MERGE_STAGE_THREADS, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)(MERGE_LDS_DYN_MAX - XCHG_LDS_STATIC));
}
int merge_fence_sys() { return 0; }
static void launch_merge_kernel(bool stage, dim3 grid, size_t smem, hipStream_t s, const ModelConst& mc,
                                StepInput* in, const float* recs, int nrec, int rec_stride, int rows_in_rec,
                                const float* noise, float* rank_out, StepOutput* out, int chain, int ctr_inc,
                                uint64_t* dbg, uint32_t* flag, uint32_t seq, int split_cs,
                                const uint32_t* gate, int levels_up) {
    if (stage) {
        hipLaunchKernelGGL((merge_kernel<MERGE_STAGE_THREADS, true>), grid, dim3(MERGE_STAGE_THREADS), smem, s, mc, in,
                           recs, nrec, rec_stride,
                           rows_in_rec, noise, rank_out, out, chain, ctr_inc, dbg, flag, seq, split_cs,
                           merge_fence_sys(), gate, levels_up);
    } else {
        hipLaunchKernelGGL((merge_kernel<MERGE_THREADS, false>), grid, dim3(MERGE_THREADS), smem, s, mc, in, recs, nrec,
                           rec_stride,
                           rows_in_rec, noise, rank_out, out, chain, ctr_inc, dbg, flag, seq, split_cs,
                           merge_fence_sys(), gate, levels_up);
    }
}

int launch_merge(const ModelConst& mc, StepInput* in, const float* recs, int nrec, int rec_stride,
                 int rows_in_rec, const float* noise, float* rank_out, StepOutput* out, int chain, hipStream_t s,
                 uint64_t* dbg, int ctr_inc, Publish pub, int levels_up) {
    // step outputs only (no rank record): column-split over merge_blocks() blocks when the column work
    // is large (many records, or CEM's per-column elite statistics); a few hundred MPPI records merge
    // faster in one block (C2: 157 records, 24.9 vs 25.5 us/step)
    const bool split = out && !rank_out && (nrec > MERGE_SPLIT_MIN_RECS || mc.method == SRBD_CEM_MPPI);
    const int cs = split ? merge_split_cols(mc) : 0;
    const int nb = cs ? merge_blocks(mc) : 1;
    size_t smem = 0;
    const bool stage = !cs && merge_stage_fits(nrec, rec_stride, mc.P, mc.K, &smem);
    if (cs) smem = merge_smem_bytes(nrec, mc.P, mc.K, (cs > mc.ntail ? cs : mc.ntail) + 1);
    launch_merge_kernel(stage, dim3(nb), smem, s, mc, in, recs, nrec, rec_stride, rows_in_rec, noise, rank_out, out,
                        chain, chain ? ctr_inc : 0, dbg, pub.flag, pub.seq, cs, pub.gate, levels_up);
    return nb;
}

// Setup probe of the xGMI mailboxes: slot `rank` word 0 of every mailbox <- rank, flags <- epoch;
// then every slot of the local mailbox must hold its rank.  ok[0] = 1 on success.
__global__ void xchg_probe_kernel(XchgArgs x, int* ok) {
    const int tid = threadIdx.x;
    const uint32_t epoch = *x.epoch + 1;
    const size_t half = (size_t)(epoch & 1u) * x.world * x.stride;
    if (tid < x.world) x.peer_mailbox[tid][half + (size_t)x.rank * x.stride] = (float)x.rank;
    __threadfence_system();
    __syncthreads();
    if (tid < x.world)
        __hip_atomic_store(x.peer_flags[tid] + x.rank, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __shared__ int bad;
    if (tid == 0) bad = 0;
    __syncthreads();
    if (tid < x.world) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool seen = false;
        while (!(seen = (int32_t)(__hip_atomic_load(x.flags + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) -
                                  epoch) >= 0)) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > XCHG_TIMEOUT_TICKS) break;
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        if (!seen || x.mailbox[half + (size_t)tid * x.stride] != (float)tid) bad = 1;
    }
    __syncthreads();
    if (tid == 0) {
        *ok = bad ? 0 : 1;
        *x.epoch = epoch;
    }
}

void launch_xchg_probe(const XchgArgs& x, int* ok, hipStream_t s) {
    hipLaunchKernelGGL(xchg_probe_kernel, dim3(1), dim3(64), 0, s, x, ok);
}

void launch_merge_xchg(const ModelConst& mc, StepInput* in, const float* recs, int nrec, int rec_stride,
                       const float* noise, const XchgArgs& x, StepOutput* out, int chain, hipStream_t s, int ctr_inc,
                       Publish pub, int levels_up) {
    // the kernel holds both passes' static LDS (two merge_body instantiations), so the staged records
    // get XCHG_LDS_STATIC less dynamic LDS than merge_kernel's
    size_t smem = 0;
    bool stage = merge_stage_fits(nrec, rec_stride, mc.P, mc.K, &smem);
    if (stage && smem > MERGE_LDS_DYN_MAX - XCHG_LDS_STATIC) {
        stage = false;
        smem = merge_smem_bytes(nrec, mc.P, mc.K);
    }
    const size_t smem2 = merge_smem_bytes(mc.t_xnodes, mc.P, mc.K);
    smem = smem > smem2 ? smem : smem2;
    if (stage)
        hipLaunchKernelGGL((merge_xchg_kernel<MERGE_STAGE_THREADS, true>), dim3(1), dim3(MERGE_STAGE_THREADS), smem, s,
                           mc, in, recs, nrec, rec_stride, noise, x, out, chain, chain ? ctr_inc : 0, pub.flag, pub.seq,
                           levels_up);
    else
        hipLaunchKernelGGL((merge_xchg_kernel<MERGE_THREADS, false>), dim3(1), dim3(MERGE_THREADS), smem, s, mc, in,
                           recs, nrec, rec_stride, noise, x, out, chain, chain ? ctr_inc : 0, pub.flag, pub.seq,
                           levels_up);
}


// Two byte ranges [0, n0) and [off1, off1 + n1) (16-byte words) of src -> dst, one block.
__global__ void __launch_bounds__(256) copy16_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, int n0,
                                                     int off1, int n1) {
    for (int i = threadIdx.x; i < n0 + n1; i += blockDim.x) {
        const int k = i < n0 ? i : off1 + (i - n0);
        dst[k] = src[k];
    }
}
void launch_copy16(const void* src, void* dst, size_t bytes0, size_t off1, size_t bytes1, hipStream_t s) {
    hipLaunchKernelGGL(copy16_kernel, dim3(1), dim3(256), 0, s, (const uint4*)src, (uint4*)dst, (int)(bytes0 / 16),
                       (int)(off1 / 16), (int)(bytes1 / 16));
}

// Armed step (launch_arm_copy): the step's input copy, queued before the host has the input.
__global__ void __launch_bounds__(256) arm_copy_kernel(const uint32_t* __restrict__ go, uint32_t seq,
                                                       uint64_t deadline_ticks, const uint32_t* __restrict__ src,
                                                       uint32_t* __restrict__ dst, int n0, int off1, int n1,
                                                       uint32_t* __restrict__ fired) {
    __shared__ int fire;
    if (threadIdx.x == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t g = __hip_atomic_load(go, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        while (g != seq && g != (seq | ARM_CANCEL) && __builtin_amdgcn_s_memrealtime() - t0 < deadline_ticks) {
            __builtin_amdgcn_s_sleep(1);
            g = __hip_atomic_load(go, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        fire = g == seq;
        // the chain behind reads this word (Publish::gate / GroupArgs::gate / RngJob::gate) after the kernel
        // boundary: fired -> seq, cancelled or timed out -> seq | ARM_CANCEL (nothing computed, that token
        // published, the host re-runs the call unarmed)
        *fired = fire ? seq : (seq | ARM_CANCEL);
    }
    __syncthreads();
    if (!fire) return;
    // 32-bit words; system scope, so nothing is served from a cache line older than the host's stores
    for (int i = threadIdx.x; i < n0 + n1; i += blockDim.x) {
        const int k = i < n0 ? i : off1 + (i - n0);
        dst[k] = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
void launch_arm_copy(const uint32_t* go, uint32_t seq, uint64_t deadline_ticks, const void* src, void* dst,
                     size_t bytes0, size_t off1, size_t bytes1, uint32_t* fired, hipStream_t s) {
    hipLaunchKernelGGL(arm_copy_kernel, dim3(1), dim3(256), 0, s, go, seq, deadline_ticks, (const uint32_t*)src,
                       (uint32_t*)dst, (int)(bytes0 / 4), (int)(off1 / 4), (int)(bytes1 / 4), fired);
}

__global__ void empty_kernel() {}
void launch_empty(hipStream_t s) { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s); }

void launch_advance(const ModelConst& mc, StepInput* in, const StepOutput* out, hipStream_t s) {
    hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(256), 0, s, mc, in, out);
}

void launch_div_selftest(const float* a, const float* b, int n, float* o, hipStream_t s) {
    hipLaunchKernelGGL(div_selftest_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a, b, n, o);
}

__global__ void log1p_selftest_kernel(const float* t, int n, float* o) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = log1p_fast(t[i]);
}
void launch_log1p_selftest(const float* t, int n, float* o, hipStream_t s) {
    if (n > 0) hipLaunchKernelGGL(log1p_selftest_kernel, dim3((n + 255) / 256), dim3(256), 0, s, t, n, o);
}

}  // namespace srbd

#ifdef SRBD_ROLLOUT_STAMPS
// Probe build only: the last step launch's tail stamps -- host[0, 64) g_fstamp, then n4 words of g_lstamp (8 a block).
extern "C" int srbd_probe_fstamps(uint64_t* host, int n4) {
    if (n4 < 0 || n4 > srbd::RSTAMP_BLOCKS * 8) return -1;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(srbd::g_fstamp), sizeof(uint64_t) * 64) != hipSuccess) return -2;
    return hipMemcpyFromSymbol(host + 64, HIP_SYMBOL(srbd::g_lstamp), sizeof(uint64_t) * n4) == hipSuccess ? 0 : -2;
}
extern "C" int srbd_probe_fstamps_clear() {
    static uint64_t z[srbd::RSTAMP_BLOCKS * 8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(srbd::g_fstamp), z, sizeof(uint64_t) * 64) != hipSuccess) return -2;
    return hipMemcpyToSymbol(HIP_SYMBOL(srbd::g_lstamp), z, sizeof(z)) == hipSuccess ? 0 : -2;
}
// Probe build only: copy out the last rollout launch's block stamps (n <= RSTAMP_BLOCKS * RSTAMP_N).
extern "C" int srbd_probe_rstamps(uint64_t* host, int n) {
    if (n > srbd::RSTAMP_BLOCKS * srbd::RSTAMP_N) return -1;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(srbd::g_rstamp), sizeof(uint64_t) * n) == hipSuccess ? 0 : -2;
}
extern "C" int srbd_probe_rstamps_clear() {
    static uint64_t z[srbd::RSTAMP_BLOCKS * srbd::RSTAMP_N];
    return hipMemcpyToSymbol(HIP_SYMBOL(srbd::g_rstamp), z, sizeof(z)) == hipSuccess ? 0 : -2;
}
#endif
