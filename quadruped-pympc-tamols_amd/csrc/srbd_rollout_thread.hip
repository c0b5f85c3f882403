// srbd_rollout_thread.hip -- thread-per-sample rollout kernels (rollout_kernel, rollout_ga_kernel) and
// their launchers.  A translation unit of its own so it can be built with -fno-slp-vectorize: in the
// thread layout the SLP vectoriser pairs independent x / y / z chains into v_pk_* instructions whose
// operand pairs cost a v_mov each and whose SGPR-pair operands spilled (C5 rollout: 1 389 v_mov and
// 256 VGPRs + scratch with it, 97 VGPRs without; the four-lane kernels keep it: fewer instructions).
// Float results are unchanged by either choice (the v_pk ops round per lane, contraction stays off).
#undef SRBD_ROLLOUT_STAMPS  // the timeline probe stamps the four-lane kernel (srbd_kernels.hip) only
#include "srbd_device.h"

namespace srbd {

// One thread per sample.  Best throughput when samples fill the GPU (>= ~1 wave per SIMD).  The zero-order form
// is compiled for at least four waves per SIMD (a fifth measured slower: DESIGN.md section 4).
// KS: the host step's input by value (the first kernel argument, read in place from the kernarg segment; block
// 0 writes the device StepInput `in_dev`), as rollout_quad_kernel does.
// GEN (GroupArgs::gen, zero-order H 12, MPPI, device Philox draws): the launch makes the step's draws itself --
// every fourth step the twelve column quads of the next four steps (rng_item's Philox call and Box-Muller pairs,
// so the same bits); the epilogue regenerates the first gen - 1 quads (leaf_wsum_lanes, RG = 2) and reads the
// rest back, which the horizon stores as it makes them -- in place of the RNG launch's write of N P floats and
// the horizon's reads of them.
template <int KIND, int HT, int ST, bool CEMT, bool EXT, bool KS = false, bool GEN = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KIND == SRBD_ZERO_ORDER ? (GEN ? 3 : 4) : 1))) rollout_kernel(
                                                      const std::conditional_t<KS, StepInputK, KsNone> ksi,
                                                      const ModelConst mc, const StepInput* __restrict__ in_dev,
                                                      const float* __restrict__ noise, float* __restrict__ costs,
                                                      float* __restrict__ recs, int rec_stride,
    const RngJob next_rng, int nroll, const GroupArgs grp) {
    const StepInput* __restrict__ in;
    if constexpr (KS) {
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
    if (grp.gate && (*grp.gate & ARM_CANCEL)) return;  // armed chain that did not fire: nothing to compute
    // blocks past the rollout grid generate the next step's noise on the CUs the rollout leaves idle
    if ((int)blockIdx.x >= nroll) {
        rng_items(mc, in, next_rng, ((int)blockIdx.x - nroll) * (int)blockDim.x + (int)threadIdx.x,
                  ((int)gridDim.x - nroll) * (int)blockDim.x);
        return;
    }

    constexpr bool CT = HT > 0 && (KIND == SRBD_ZERO_ORDER || ST > 0);  // compile-time shape
    const int H = CT ? HT : mc.H;
    const int S = CT ? ST : mc.S;
    const int PL = CT ? (KIND == SRBD_ZERO_ORDER ? 3 * HT : (KIND == SRBD_LINEAR_SPLINE ? 3 * (ST + 1) : 12 * ST))
                      : mc.PL;
    constexpr int T = 256;  // launched with 256 threads (rollout_threads)
    const int tid = threadIdx.x;
    const int k = blockIdx.x * T + tid;  // local row (padded rows < ldn are readable zeros)
    const bool valid = k < mc.n_local;
    const size_t ldn = (size_t)mc.ldn;
    const bool zs = CEMT && zs_scaled(mc, in);  // CEMT: CEM kernels only carry the scaling code

    float x[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) x[i] = in->state[i];
    float cost3[3] = {0.0f, 0.0f, 0.0f};
    float Fprev[12];  // EXT: opt-in cost terms (srbd_set_cost_terms), a separate instantiation so the
                      // default horizon carries none of their code (a runtime test cost C3 17 %)
    // Zero-order with a compile-time horizon: step m's 12 noise values are issued at step m - ZD into a
    // ring of ZD + 1 slots (buffer loads: the row in soffset, the sample in voffset), and each step reads
    // its scalars (contact, fz_ref, dt, best) and the LDS constants through step_ptr, so nothing is hoisted
    // across the whole horizon.  (Hoisted, the 144 loads took 210 VGPRs plus SGPR spills to VGPR lanes:
    // 2 waves per SIMD and ~300 v_readlane per step at C5.)  P * ldn * 4 < 2^31: P <= 192 here and
    // n_local <= 8192 blocks x 256.
    static_assert(!GEN || (KIND == SRBD_ZERO_ORDER && HT % 4 == 0 && !CEMT && !EXT), "GEN: zero-order H % 4 == 0");
    constexpr bool ZR = CT && KIND == SRBD_ZERO_ORDER && !EXT && !GEN;
    constexpr int ZD = 2, ZRS = ZD + 1;
    float zr[ZR ? ZRS : 1][12];
    const auto nrs = __builtin_amdgcn_make_buffer_rsrc((void*)noise, (short)0, ZR ? mc.P * mc.ldn * 4 : 0, 0x00020000);
    const int voff = k * 4;
    auto zload = [&](const int m, const int ldn4) __attribute__((always_inline)) {
#pragma unroll
        for (int l = 0; l < 4; ++l)
#pragma unroll
            for (int q = 0; q < 3; ++q)
#ifdef SRBD_DIAG_NOLOAD  // diagnostic build: no noise reads (timing only)
                zr[m % ZRS][3 * l + q] = (float)(k + l * PL + q * HT + m + ldn4) * 1e-9f;
#else
                zr[m % ZRS][3 * l + q] =
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(nrs, voff, (l * PL + q * HT + m) * ldn4, 0));
#endif
    };
    if constexpr (ZR) {
        const int ldn4 = step_int(mc.ldn * 4, x[0]);
#pragma unroll
        for (int m = 0; m < ZD && m < HT; ++m) zload(m, ldn4);
    }
    float dep = x[0];  // step_ptr dependency: set part-way through each step
    // GEN: column quad l PL / 4 + q HT / 4 + s of this row holds steps 4 s .. 4 s + 3 of leg l's component q.  The
    // epilogue regenerates quads [0, nrg) and reads the others back, which the horizon stores (GroupArgs::gen - 1)
    float gz[GEN ? 12 : 1][4];
    const int nrg = GEN ? grp.gen - 1 : 0;
    // The twelve quads one after another: each quad's row word waits for the previous quad's last value (an empty
    // asm).  Chained per leg or not at all measured the same (C5 step launch 126.2 / 126.4 vs 126.6 us); the GEN
    // kernel runs at 3 waves per SIMD (147 VGPRs): capped at 4 it spills 104 B and the launch takes 137.4 us.
    auto gen4 = [&](const int s, auto is) __attribute__((always_inline)) {
        const int r = mc.row0 + k;
        const bool live = r > 0 && valid;  // row 0 (the warm start) and the padding rows: zeros, as in the buffer
        uint32_t d = (uint32_t)(r - 1);
#pragma unroll
        for (int l = 0; l < 4; ++l)
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                uint32_t c[4] = {d, (uint32_t)(l * (PL / 4) + q * (HT / 4) + s), is->ctr_lo, is->ctr_hi};
                philox4x32_10(c, is->seed_lo, is->seed_hi);
                float v[4];
                box_muller(c[0], c[1], v[0], v[1]);
                box_muller(c[2], c[3], v[2], v[3]);
                const int qq = l * (PL / 4) + q * (HT / 4) + s;
#pragma unroll
                for (int i = 0; i < 4; ++i) gz[3 * l + q][i] = live ? mc.sigma_mppi * v[i] : 0.0f;
                if (qq >= nrg) {  // a quad the epilogue reads back: stored (plain stores, kept in the XCD's L2)
                    float* o = const_cast<float*>(noise) + (size_t)(4 * qq) * ldn + k;
#pragma unroll
                    for (int i = 0; i < 4; ++i) o[(size_t)i * ldn] = gz[3 * l + q][i];
                }
                asm volatile("" : "+v"(d) : "v"(gz[3 * l + q][3]));
            }
    };
    auto step = [&](const int n, auto EX) __attribute__((always_inline)) {
        const auto is = step_ptr(in, dep);
        if constexpr (ZR)
            if (n + ZD < HT) zload(n + ZD, step_int(mc.ldn * 4, dep));  // n: a compile-time constant (unrolled)
        // the key read through a pointer tied to the last step's cost (its roll and angular-rate terms: the whole
        // rotation update; tied to the forces or to a position, all 36 quads were made before the first step)
        if constexpr (GEN)
            if (n % 4 == 0) gen4(n / 4, step_ptr(in, cost3[0]));
        const float c[4] = {is->contact[0][n], is->contact[1][n], is->contact[2][n], is->contact[3][n]};
        const float fref = is->fzref[n];
        const float dt = mc.dts[n];
        const int idx = CT && KIND != SRBD_ZERO_ORDER ? chunk_index(n, HT, ST) : mc.sidx[n];
        float F[12], RX[4], RY[4];
#pragma unroll
        for (int leg = 0; leg < 4; ++leg) {
            const int base = leg * PL;
            auto acc = [&](int j) {
                float z;
                if constexpr (GEN)
                    z = gz[3 * leg + (j - n) / HT][n % 4];
                else if constexpr (ZR)
                    z = zr[n % ZRS][3 * leg + (j - n) / HT];  // ZO reads j = n + q H (decode_leg)
                else
                    z = (step_gptr(noise, dep) + k)[(size_t)(base + j) * ldn];
                if constexpr (CEMT) {  // CEM device draws are unscaled: noise = Z * sigma_j (z * 1 == z)
                    const float sj = is->sigma[base + j];
                    return is->best[base + j] + z * (zs ? sj : 1.0f);
                }
                return is->best[base + j] + z;
            };
            float fx, fy, fz;
            decode_leg(KIND, H, S, idx, mc.sq[n], mc.somq[n], mc.sa[n], mc.sb[n], mc.sc[n], mc.sd[n], n, acc, fx,
                       fy, fz);
            RX[leg] = fx;
            RY[leg] = fy;
            shape_leg(mc, fref, c[leg], fx, fy, fz);
            F[3 * leg] = fx;
            F[3 * leg + 1] = fy;
            F[3 * leg + 2] = fz;
        }
        dep = F[11];  // the next step's loads issue from here on (step_ptr)
        integrate(mc, x, in->state + 12, F, c, dt);
        // tracking cost (NMPC:451) per component: cost_c += ((t_p + t_v) + t_rpy) + t_omega
        float t[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) {
            const float e = x[i] - in->ref[i];
            t[i] = (e * mc.Q[i]) * e;
        }
#pragma unroll
        for (int q = 0; q < 3; ++q) cost3[q] = cost3[q] + (((t[q] + t[3 + q]) + t[6 + q]) + t[9 + q]);
        if constexpr (decltype(EX)::value) extra_cost_step(mc, n, F, RX, RY, c, fref, Fprev, cost3);
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
    float cost = (cost3[0] + cost3[1]) + cost3[2];
    cost = cost + in->cost_feet;  // 0, or NaN when a foot term is non-finite (Q_feet = 0)
    // NMPC:686-687
    if (isnan(cost) || isinf(cost)) cost = 1000000.0f;
    if (valid && costs) costs[k] = cost;
#ifdef SRBD_DIAG_NOEPI  // diagnostic build: no block epilogue (timing only)
    if (tid == 0) recs[blockIdx.x] = cost;
    return;
#endif
    // RG: zero-order MPPI regenerates part of its draws in the epilogue (leaf_wsum_lanes, REGEN_QUADS)
    block_epilogue<CEMT, false, true, GEN ? 2 : (KIND == SRBD_ZERO_ORDER && !CEMT && !EXT ? 1 : 0)>(
        mc, in, T, tid, valid, cost, noise, recs, rec_stride, 0.0f, grp, nroll);
}

template <int KIND>
__global__ void __launch_bounds__(256) rollout_ga_kernel(const ModelConst mc, const StepInput* __restrict__ in,
                                                         const float* __restrict__ noise, float* __restrict__ costs,
                                                         float* __restrict__ recs, int rec_stride,
                                                         const RngJob next_rng, int nroll, const GroupArgs grp) {
    if (grp.gate && (*grp.gate & ARM_CANCEL)) return;  // armed chain that did not fire
    if ((int)blockIdx.x >= nroll) {
        rng_items(mc, in, next_rng, ((int)blockIdx.x - nroll) * (int)blockDim.x + (int)threadIdx.x,
                  ((int)gridDim.x - nroll) * (int)blockDim.x);
        return;
    }
    const int H = mc.H, S = mc.S, PL = mc.PL;
    const int tid = threadIdx.x, T = blockDim.x;
    const int k = blockIdx.x * T + tid;  // rows >= n_local are padding (readable zeros)
    const bool valid = k < mc.n_local;
    const size_t ldn = (size_t)mc.ldn;
    const float* __restrict__ nz = noise + k;
    const float* __restrict__ best = in->best;

    const float f = ga_sample_freq(mc, in, k);
    uint32_t mask[4];
    ga_contact_masks(in, H, f, mask);
    float seg[4];  // horizon_leg / S (GA:200 / :223), IEEE division
#pragma unroll
    for (int l = 0; l < 4; ++l) seg[l] = ((float)__popc(mask[l]) + 1.0f) / (float)S;
    int cnt[4] = {-1, -1, -1, -1};

    float x[12], feet[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        x[i] = in->state[i];
        feet[i] = in->state[12 + i];
    }
    float cost3[3] = {0.0f, 0.0f, 0.0f};
    const bool extra = mc.cost_on != 0;  // opt-in cost terms (srbd_set_cost_terms)
    float Fprev[12];
    for (int n = 0; n < H; ++n) {
        float c[4];
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const uint32_t b = (mask[l] >> n) & 1u;
            c[l] = b ? 1.0f : 0.0f;
            cnt[l] += (int)b;
        }
        const float ns = ((c[0] + c[1]) + c[2]) + c[3];
        const float fref = mc.fz_ns[(int)ns];
        float F[12], RX[4], RY[4];
#pragma unroll
        for (int leg = 0; leg < 4; ++leg) {
            const int base = leg * PL;
            auto acc = [&](int j) {
                j = j < 0 ? j + PL : j;
                return best[base + j] + nz[(size_t)(base + j) * ldn];
            };
            const int st = cnt[leg];
            int idx = 0;
            float q = 0.0f, omq = 0.0f, a = 0.0f, bb = 0.0f, cc = 0.0f, d = 0.0f;
            if (KIND != SRBD_ZERO_ORDER) {  // spline_coef of srbd_api.hip with (step, horizon_leg) per leg
                for (int i = 0; i <= S; ++i)
                    if (st >= in->ga_cb[i]) idx = i;
                float tau = (float)st / seg[leg];
                tau = tau - (float)idx;
                q = tau / 1.0f;
                omq = 1.0f - q;
                a = 2.0f * q * q * q - 3.0f * q * q + 1.0f;
                bb = (q * q * q - 2.0f * q * q + q) * 1.0f;
                cc = -2.0f * q * q * q + 3.0f * q * q;
                d = (q * q * q - q * q) * 1.0f;
            }
            float fx, fy, fz;
            decode_leg(KIND, H, S, idx, q, omq, a, bb, cc, d, st, acc, fx, fy, fz);
            RX[leg] = fx;
            RY[leg] = fy;
            shape_leg(mc, fref, c[leg], fx, fy, fz);
            F[3 * leg] = fx;
            F[3 * leg + 1] = fy;
            F[3 * leg + 2] = fz;
        }
        integrate(mc, x, feet, F, c, mc.dts[n]);
        float t[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) {
            const float e = x[i] - in->ref[i];
            t[i] = (e * mc.Q[i]) * e;
        }
#pragma unroll
        for (int q = 0; q < 3; ++q) cost3[q] = cost3[q] + (((t[q] + t[3 + q]) + t[6 + q]) + t[9 + q]);
        if (extra) extra_cost_step(mc, n, F, RX, RY, c, fref, Fprev, cost3);
    }
    float cost = (cost3[0] + cost3[1]) + cost3[2];
    cost = cost + in->cost_feet;
    const float df = f - 1.3f;
    cost = cost + (df * 100.0f) * df;  // GA:500
    if (isnan(cost) || isinf(cost)) cost = 1000000.0f;
    if (valid && costs) costs[k] = cost;
    block_epilogue<false, false, true>(mc, in, T, tid, valid, cost, noise, recs, rec_stride, f, grp, nroll);
}

// ------------------------------------------------------------------ launchers (srbd_launch.h)
template <int KIND, int HT, int ST, bool EXT>
static void launch_thread_t(const ModelConst& mc, const StepInput* in, const float* noise, float* costs, float* recs,
                            int rec_stride, int threads, hipStream_t s, const RngJob* next, const GroupArgs& grp) {
    const RngJob job = next ? *next : RngJob{nullptr, 0, 0, 0, 0};
    const int extra = next ? (rng_grid(mc) < 1024 ? rng_grid(mc) : 1024) : 0;
    threads = 256;  // the kernel is compiled for 256-thread blocks (rollout_threads)
    const int blocks = (mc.n_local + threads - 1) / threads;
    const dim3 grid(blocks + extra * (256 / threads));
    // thread form with the cost terms: runtime shapes only (the four-lane kernel is the default)
    constexpr int HTT = EXT ? 0 : HT, STT = EXT ? 0 : ST;
    if constexpr (KIND == SRBD_ZERO_ORDER && HT == 12 && !EXT) {
        // gen_ok: the launch makes the step's draws (host steps, the input by value; no next-step draws).  Only the
        // by-value form: with the input in global memory the same code spilled 368 B per lane.
        if (grp.gen && grp.ksi) {
            hipLaunchKernelGGL((rollout_kernel<KIND, HT, ST, false, false, true, true>), dim3(blocks), dim3(threads), 0,
                               s, *static_cast<const StepInputK*>(grp.ksi), mc, in, noise, costs, recs, rec_stride,
                               job, blocks, grp);
            return;
        }
    }
    if constexpr (KIND == SRBD_ZERO_ORDER && (HT == 10 || HT == 12) && !EXT) {
        if (grp.ksi && mc.method != SRBD_CEM_MPPI) {  // ks_ok: the step input as the first kernel argument
            hipLaunchKernelGGL((rollout_kernel<KIND, HT, ST, false, false, true>), grid, dim3(threads), 0, s,
                               *static_cast<const StepInputK*>(grp.ksi), mc, in, noise, costs, recs, rec_stride, job,
                               blocks, grp);
            return;
        }
    }
    if (mc.method == SRBD_CEM_MPPI)
        hipLaunchKernelGGL((rollout_kernel<KIND, HTT, STT, true, EXT>), grid, dim3(threads), 0, s, KsNone{}, mc, in, noise,
                           costs, recs, rec_stride, job, blocks, grp);
    else
        hipLaunchKernelGGL((rollout_kernel<KIND, HTT, STT, false, EXT>), grid, dim3(threads), 0, s, KsNone{}, mc, in,
                           noise, costs, recs, rec_stride, job, blocks, grp);
}

// The launch can make the step's draws itself (GroupArgs::gen); the caller also needs device draws (no injected
// noise) and no next-step draws in the launch.
bool gen_ok(const ModelConst& mc, int mode) {
    return (mode == ROLLOUT_THREAD || mode == ROLLOUT_QUAD) && mc.kind == SRBD_ZERO_ORDER && mc.H == 12 &&
           mc.method == SRBD_MPPI && mc.rng == RNG_PHILOX && !mc.ga && !mc.cost_on && mc.P % 4 == 0;
}

void launch_rollout_thread(const ModelConst& mc, const StepInput* in, const float* noise, float* costs, float* recs,
                           int rec_stride, int threads, hipStream_t s, const RngJob* next, const GroupArgs& grp) {
    const int H = mc.H, S = mc.S;
#define SRBD_LT(K, HH, SS)                                                                                        \
    return mc.cost_on                                                                                            \
               ? launch_thread_t<K, HH, SS, true>(mc, in, noise, costs, recs, rec_stride, threads, s, next, grp)    \
               : launch_thread_t<K, HH, SS, false>(mc, in, noise, costs, recs, rec_stride, threads, s, next, grp)
    switch (mc.kind) {
        case SRBD_ZERO_ORDER:
            if (H == 10) SRBD_LT(SRBD_ZERO_ORDER, 10, 0);
            if (H == 12) SRBD_LT(SRBD_ZERO_ORDER, 12, 0);
            if (H == 16) SRBD_LT(SRBD_ZERO_ORDER, 16, 0);
            SRBD_LT(SRBD_ZERO_ORDER, 0, 0);
        case SRBD_LINEAR_SPLINE:
            if (S == 2 && H == 12) SRBD_LT(SRBD_LINEAR_SPLINE, 12, 2);
            if (S == 2 && H == 16) SRBD_LT(SRBD_LINEAR_SPLINE, 16, 2);
            SRBD_LT(SRBD_LINEAR_SPLINE, 0, 0);
        default:
            if (S == 2 && H == 12) SRBD_LT(SRBD_CUBIC_SPLINE, 12, 2);
            if (S == 2 && H == 16) SRBD_LT(SRBD_CUBIC_SPLINE, 16, 2);
            SRBD_LT(SRBD_CUBIC_SPLINE, 0, 0);
    }
#undef SRBD_LT
}

void launch_rollout_ga_thread(const ModelConst& mc, const StepInput* in, const float* noise, float* costs,
                              float* recs, int rec_stride, int spb, hipStream_t s, const RngJob* next,
                              const GroupArgs& grp) {
    const RngJob job = next ? *next : RngJob{nullptr, 0, 0, 0, 0};
    const int extra = next ? (rng_grid(mc) < 1024 ? rng_grid(mc) : 1024) : 0;
    const int blocks = (mc.n_local + spb - 1) / spb;
    const dim3 grid(blocks + extra * 256 / spb), block(spb);
    if (mc.kind == SRBD_ZERO_ORDER)
        hipLaunchKernelGGL((rollout_ga_kernel<SRBD_ZERO_ORDER>), grid, block, 0, s, mc, in, noise, costs, recs,
                           rec_stride, job, blocks, grp);
    else if (mc.kind == SRBD_LINEAR_SPLINE)
        hipLaunchKernelGGL((rollout_ga_kernel<SRBD_LINEAR_SPLINE>), grid, block, 0, s, mc, in, noise, costs, recs,
                           rec_stride, job, blocks, grp);
    else
        hipLaunchKernelGGL((rollout_ga_kernel<SRBD_CUBIC_SPLINE>), grid, block, 0, s, mc, in, noise, costs, recs,
                           rec_stride, job, blocks, grp);
}

}  // namespace srbd
