// srbd_device.h -- device helpers shared by the rollout translation units (srbd_kernels.hip: RNG,
// four-lane rollouts, merge; srbd_rollout_thread.hip: thread-per-sample rollouts).
#pragma once

#include <utility>

#include "srbd_jaxrng.h"
#include "srbd_launch.h"

namespace srbd {

// Timeline probe (measurement build only, `make probe`): thread 0 of every rollout-launch block
// stores s_memrealtime (100 MHz) at fixed points after draining its outstanding memory operations.
#ifdef SRBD_ROLLOUT_STAMPS
constexpr int RSTAMP_N = 6, RSTAMP_BLOCKS = 8192;
__device__ uint64_t g_rstamp[RSTAMP_BLOCKS * RSTAMP_N];
#define SRBD_RSTAMP(i)                                                                  \
    do {                                                                                \
        if (threadIdx.x == 0 && blockIdx.x < RSTAMP_BLOCKS) {                           \
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                 \
            g_rstamp[blockIdx.x * RSTAMP_N + (i)] = __builtin_amdgcn_s_memrealtime(); \
        }                                                                               \
    } while (0)
// The step launch's tail: level1_fold marks per block (no drain), and the final merger's own marks
// (g_fstamp[0] = its block + 1, [1..4] final_merge, [32..63] its merge_body stamps).
__device__ uint64_t g_lstamp[RSTAMP_BLOCKS * 8];
__device__ uint64_t g_fstamp[64];
#define SRBD_LSTAMP(i)                                                                            \
    do {                                                                                          \
        if (threadIdx.x == 0 && blockIdx.x < RSTAMP_BLOCKS)                                       \
            g_lstamp[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime();                    \
    } while (0)
#else
#define SRBD_RSTAMP(i) \
    do {               \
    } while (0)
#define SRBD_LSTAMP(i) \
    do {               \
    } while (0)
#endif

// Per-step pointer of an unrolled horizon: the same address, passed through an empty asm that also
// reads `dep` (a value the previous step computes part-way through), so the loads through it issue
// during the previous step -- not hoisted to the top of the horizon, not merged with another step's
// loads.  (An asm "memory" clobber does not do this: the step input and the noise are readonly
// __restrict__ arguments, whose loads LLVM moves freely, and an asm without an input floats to the
// top.  Hoisted, the step scalars and noise took 210 VGPRs + SGPR spills in the C5 thread rollout and
// ~150 v_readlane per step in the cubic CEM kernel.)  Uniform loads stay scalar: nothing is clobbered.
// The returned pointer is in the constant address space, so uniform loads through it stay scalar
// (s_load); a generic pointer out of the asm would turn them into flat vector loads.  step_gptr: the
// same in the global address space (per-lane loads).
template <class T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* step_ptr(const T* p, float dep) {
    auto q = (const __attribute__((address_space(4))) T*)p;
    asm volatile("" : "+s"(q) : "v"(dep));
    return q;
}
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* step_gptr(const T* p, float dep) {
    auto q = (const __attribute__((address_space(1))) T*)p;
    asm volatile("" : "+s"(q) : "v"(dep));
    return q;
}
// The same for a uniform integer (a load offset formed from it).
__device__ __forceinline__ int step_int(int v, float dep) {
    asm volatile("" : "+s"(v) : "v"(dep));
    return v;
}

// ------------------------------------------------------------------ helpers
// 64-bit wave minimum with DPP (row_shr 1/2/4/8 within 16-lane rows, then row_bcast 15/31, gfx9
// family), result read from lane 63.  All 64 lanes must be active.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)(uint32_t)v, CTRL, ROWMASK, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)(uint32_t)(v >> 32), CTRL, ROWMASK, 0xF, false);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return b < a ? b : a; }
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
    v = umin64(v, dpp_u64<0x111, 0xF>(v));
    v = umin64(v, dpp_u64<0x112, 0xF>(v));
    v = umin64(v, dpp_u64<0x114, 0xF>(v));
    v = umin64(v, dpp_u64<0x118, 0xF>(v));
    v = umin64(v, dpp_u64<0x142, 0xA>(v));
    v = umin64(v, dpp_u64<0x143, 0xC>(v));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
    return ((uint64_t)hi << 32) | lo;
}

// Minimum of each 32-lane half (the reduction tree's level-0 nodes of 32 children): lanes 0..31 -> *lo, 32..63 -> *hi.
__device__ __forceinline__ void half_wave_min_u64(uint64_t v, uint64_t* lo, uint64_t* hi) {
    v = umin64(v, dpp_u64<0x111, 0xF>(v));
    v = umin64(v, dpp_u64<0x112, 0xF>(v));
    v = umin64(v, dpp_u64<0x114, 0xF>(v));
    v = umin64(v, dpp_u64<0x118, 0xF>(v));
    v = umin64(v, dpp_u64<0x142, 0xA>(v));
    *lo = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 31) << 32) |
          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 31);
    *hi = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63) << 32) |
          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
}

// Block-wide min; every thread gets the result.  `red` holds blockDim/64 words.
__device__ __forceinline__ uint64_t block_min_u64(uint64_t v, uint64_t* red) {
    v = wave_min_u64(v);
    const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    uint64_t r = red[0];
    for (int i = 1; i < nw; ++i) r = red[i] < r ? red[i] : r;
    return r;
}

__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        // one 32x32->64 multiply each (v_mad_u64_u32) instead of separate lo / hi multiplies
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = (uint32_t)p1;
        c[2] = n2;
        c[3] = (uint32_t)p0;
    }
}

__device__ __forceinline__ float u01(uint32_t x) { return ((float)(x >> 8) + 0.5f) * 5.9604644775390625e-08f; }

// Noise buffers hold unscaled CEM draws Z when they come from the device RNG (StepInput::noise_scaled
// == 0): readers form the noise value Z * sigma_j.  Injected noise is stored as given.
__device__ __forceinline__ bool zs_scaled(const ModelConst& mc, const StepInput* in) {
    return mc.method == SRBD_CEM_MPPI && in->noise_scaled == 0;
}

constexpr uint64_t KEY_NONE = ~0ull;

// Sorted (ascending) per-lane candidate list of at most KM keys; fully unrolled (registers only).
template <int KM>
__device__ __forceinline__ void lk_insert(uint64_t (&lk)[KM], uint64_t x) {
#pragma unroll
    for (int i = KM - 1; i >= 1; --i) lk[i] = (x < lk[i - 1]) ? lk[i - 1] : (x < lk[i] ? x : lk[i]);
    lk[0] = x < lk[0] ? x : lk[0];
}
// K rounds of a wave-wide minimum over the lanes' list heads; the (unique) winning lane pops.
template <int KM>
__device__ __forceinline__ void wave_topk(uint64_t (&lk)[KM], int K, uint64_t* out) {
    for (int e = 0; e < K; ++e) {
        const uint64_t m = wave_min_u64(lk[0]);
        const bool pop = lk[0] == m && m != KEY_NONE;
#pragma unroll
        for (int i = 0; i < KM - 1; ++i) lk[i] = pop ? lk[i + 1] : lk[i];
        lk[KM - 1] = pop ? KEY_NONE : lk[KM - 1];
        if ((threadIdx.x & 63) == 0) out[e] = m;
    }
}

// ------------------------------------------------------------------ RNG
// Noise row r (global), column j.  MPPI: sigma*Z(r-1, j); CEM: Z(r-1, j)*sigma_j; random sampling
// (NMPC:647-677): rows 1..t sigma0*Z(r-1), rows t+1..2t sigma1*Z(r-1-t) (same draws: the reference
// reuses one key, App. B #3), rows 2t+1..N-1 U(-s2, s2) from draw r-1-2t.  Row 0 is zero.
// One item = (local row k, column quad q): one Philox4x32-10 call, two Box-Muller pairs.
// Box-Muller on the hardware transcendentals: v_log_f32 (log2), v_sqrt_f32, and v_sin/v_cos_f32,
// which take revolutions, i.e. sin/cos(2 pi ub) directly with no range reduction (ub in (0, 1)).
// They differ from libm by a few ulp (the host oracle's draws agree to ~1e-6 relative).
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
    const float ua = u01(a), ub = u01(b);
    const float rr = __builtin_amdgcn_sqrtf(-1.38629436112f * __builtin_amdgcn_logf(ua));  // -2 ln ua
    z0 = rr * __builtin_amdgcn_cosf(ub);
    z1 = rr * __builtin_amdgcn_sinf(ub);
}

__device__ __forceinline__ void rng_item(const ModelConst& mc, const float* __restrict__ sigma, uint32_t key0,
                                         uint32_t key1, uint32_t c2, uint32_t c3, int k, int q,
                                         float* __restrict__ noise) {
    const int r = mc.row0 + k;
    uint32_t d = (uint32_t)(r - 1);
    float scale = mc.sigma_mppi;  // MPPI
    bool uniform = false;
    if (mc.method == SRBD_RANDOM_SAMPLING) {
        const int t = mc.N / 3;
        if (r <= t) {
            scale = mc.sigma_rs[0];
        } else if (r <= 2 * t) {
            scale = mc.sigma_rs[1];
            d = (uint32_t)(r - 1 - t);
        } else {
            uniform = true;
            d = (uint32_t)(r - 1 - 2 * t);
        }
    }
    uint32_t c[4] = {d, (uint32_t)q, c2, c3};
    philox4x32_10(c, key0, key1);
    float v[4];
    if (uniform) {
        const float s2 = mc.sigma_rs[2];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = u01(c[i]) * (2.0f * s2) - s2;
    } else {
        box_muller(c[0], c[1], v[0], v[1]);
        box_muller(c[2], c[3], v[2], v[3]);
        // CEM: the standard normals themselves (they do not depend on the step's sigma, so the next
        // step's draws can be made early); every reader multiplies by sigma_j (zs_scale), the same
        // float product Z * sigma the reference forms (NMPC:951-958)
        if (mc.method != SRBD_CEM_MPPI) {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = scale * v[i];
        }
    }
    const size_t ldn = (size_t)mc.ldn;
    float* __restrict__ o = noise + (size_t)(4 * q) * ldn + k;
#pragma unroll
    // Write-through (sc1) stores: the draws leave no dirty lines in the XCD L2s, so the end of the
    // launch that makes them has nothing to write back (the next step reads them from memory on other
    // XCDs anyway).  C2: 25.6 -> 24.1 us per step; the fused rollout launch 14.7 -> 14.2 us.
    for (int i = 0; i < 4; ++i)  // row 0: the warm start itself
        __hip_atomic_store(&o[i * ldn], r > 0 ? v[i] : 0.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The reference's jax.random stream (srbd_set_rng, srbd_jaxrng.h): element (row r, column j) of the
// sampler's draw, as NMPC:647-677 (random sampling: the two Gaussian blocks share key and shape, so block
// 2 reuses block 1's normals; the uniform block is a draw of its own shape from the same key), :806-812
// (MPPI: sigma * Z) and :951-958 (CEM: Z, scaled by sigma_j on read as for Philox).  One item per element,
// enumerated k-fastest like the Philox items (coalesced stores).
__device__ __forceinline__ float jax_noise_value(const ModelConst& mc, uint32_t k0, uint32_t k1, int r, int j,
                                                 bool part) {
    const uint64_t P = (uint64_t)mc.P;
    if (mc.method != SRBD_RANDOM_SAMPLING) {
        const float z = jax_normal(jax_bits(k0, k1, (uint64_t)(r - 1) * P + j, (uint64_t)(mc.N - 1) * P, part));
        return mc.method == SRBD_MPPI ? mc.sigma_mppi * z : z;
    }
    const int t = mc.N / 3;
    if (r <= 2 * t) {
        const int d = r <= t ? r - 1 : r - 1 - t;
        const float z = jax_normal(jax_bits(k0, k1, (uint64_t)d * P + j, (uint64_t)t * P, part));
        return (r <= t ? mc.sigma_rs[0] : mc.sigma_rs[1]) * z;
    }
    const float s2 = mc.sigma_rs[2], lo = -s2;
    return jax_uniform(jax_bits(k0, k1, (uint64_t)(r - 1 - 2 * t) * P + j, (uint64_t)(mc.N - 1 - 2 * t) * P, part),
                       lo, s2 - lo);
}

__device__ __forceinline__ void jax_rng_items(const ModelConst& mc, uint64_t key, const RngJob& job, int first,
                                              int stride) {
    const bool part = mc.rng == RNG_JAX;
    const uint32_t k0 = (uint32_t)(key >> 32), k1 = (uint32_t)key;
    const int n = mc.n_local, P = mc.P;
    const size_t ldn = (size_t)mc.ldn;
    int j = first / n, k = first - j * n;
    const int sj = stride / n, sk = stride - sj * n;
    while (j < P) {
        const int r = mc.row0 + k;
        const float v = r > 0 ? jax_noise_value(mc, k0, k1, r, j, part) : 0.0f;  // row 0: the warm start
        __hip_atomic_store(&job.noise[(size_t)j * ldn + k], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        k += sk;
        j += sj;
        if (k >= n) {
            k -= n;
            ++j;
        }
    }
}

// Device-resident chains: the next step's RNG key -- counter + inc, and for the JAX stream also the
// key itself, with_newkey inc times (NMPC:498-501).
__device__ __forceinline__ void advance_key(const ModelConst& mc, StepInput* in, int inc) {
    const uint64_t cc = (((uint64_t)in->ctr_hi << 32) | in->ctr_lo) + (uint64_t)inc;
    in->ctr_lo = (uint32_t)cc;
    in->ctr_hi = (uint32_t)(cc >> 32);
    if (mc.rng != RNG_PHILOX) {
        const uint64_t key = jax_next_key(((uint64_t)in->seed_hi << 32) | in->seed_lo, mc.rng == RNG_JAX, inc);
        in->seed_lo = (uint32_t)key;
        in->seed_hi = (uint32_t)(key >> 32);
    }
}

// Items (k, q) enumerated k-fastest so consecutive lanes store consecutive floats; the item index is
// advanced incrementally (no per-item division).  P is a multiple of 12, so quads are whole.
__device__ __forceinline__ void rng_items(const ModelConst& mc, const StepInput* __restrict__ in, const RngJob& job,
                                          int first, int stride) {
    uint64_t seed = job.seed, ctr = job.ctr;
    if (job.dev_ctr) {
        seed = ((uint64_t)in->seed_hi << 32) | in->seed_lo;
        ctr = (((uint64_t)in->ctr_hi << 32) | in->ctr_lo) + (uint64_t)job.ctr_offset;
        // the JAX key of a later step of the chain: with_newkey ctr_offset times
        if (mc.rng != RNG_PHILOX) seed = jax_next_key(seed, mc.rng == RNG_JAX, job.ctr_offset);
    }
    if (mc.rng != RNG_PHILOX) return jax_rng_items(mc, seed, job, first, stride);
    const int n = mc.n_local, nq = mc.P / 4;
    int q = first / n, k = first - q * n;
    const int sq = stride / n, sk = stride - sq * n;
    while (q < nq) {
        rng_item(mc, in->sigma, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ctr, (uint32_t)(ctr >> 32), k, q,
                 job.noise);
        k += sk;
        q += sq;
        if (k >= n) {
            k -= n;
            ++q;
        }
    }
}

// ------------------------------------------------------------------ rollout
// Compile-time chunk index of the linear/cubic spline (== max(where(n >= linspace(0,H,S+1))) for
// integer n, NMPC:187-189).
__host__ __device__ constexpr int chunk_index(int n, int H, int S) { return (n * S) / H; }

template <int N>
struct IntC {
    static constexpr int value = N;
};
template <class F, int... Ns>
__device__ __forceinline__ void unroll_seq(F&& f, std::integer_sequence<int, Ns...>) {
    (f(IntC<Ns>{}), ...);
}

// Record words are stored write-through (sc1: relaxed agent-scope atomic stores) and read back with sc1
// loads by a group's last arriver (group_reduce): the hand-off form of MI355X_MICROARCH.md's table row 1
// (every storing wave waits vmcnt(0), one lane per block adds to the group's counter after a barrier,
// the workgroup whose add returns last loads).  A record the merge kernel reads after the launch needs
// no more than the kernel boundary; the same stores serve both.
__device__ __forceinline__ void st_rec(float* p, float v) {
    __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_rec(const float* p) {
    return __uint_as_float(
        __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// Stage n floats (n even, src and dst 8-byte aligned) of records other blocks stored write-through: 8-byte sc1 loads,
// U per thread in flight (half the load instructions and round trips of ld_rec).
// stage_recs16: the same with 16-byte sc1 loads through a buffer descriptor (n a multiple of 4, src and dst 16-byte
// aligned: record strides are whole 16-byte words), U per thread in flight.  C2 host p50 -0.5 to -1.6 us against the
// 8-byte form in four same-box pairs (the node's 32 records staged by the fast tail's folder); 8-byte sc1 loads run
// at 0.54-0.70x the 16-byte rate (MI355X guide).
template <int U>
__device__ __forceinline__ void stage_recs16(const float* __restrict__ src, float* dst, int n) {
    const int tid = threadIdx.x, T = blockDim.x, n4 = n >> 2;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, n * 4, 0x00020000);
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int i0 = 0; i0 < n4; i0 += U * T) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // out-of-range offsets read zeros (the descriptor's range), never stored
            const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * (i0 + u * T + tid), 0, 16);
            v[u] = make_float4(__uint_as_float(x[0]), __uint_as_float(x[1]), __uint_as_float(x[2]),
                               __uint_as_float(x[3]));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * T + tid;
            if (i < n4) d4[i] = v[u];
        }
    }
}
template <int U>
__device__ __forceinline__ void stage_recs(const float* __restrict__ src, float* dst, int n) {
    const int tid = threadIdx.x, T = blockDim.x, n2 = n >> 1;
    const uint64_t* s2 = reinterpret_cast<const uint64_t*>(src);
    uint64_t* d2 = reinterpret_cast<uint64_t*>(dst);
    for (int i0 = 0; i0 < n2; i0 += U * T) {
        uint64_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * T + tid;
            v[u] = i < n2 ? __hip_atomic_load(s2 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * T + tid;
            if (i < n2) d2[i] = v[u];
        }
    }
}

// ---- The reduction tree in the rollout launch (srbd_core.h): leaf records and the level-1 fold ----
// Record words are stored write-through (st_rec) and read back with sc1 loads (ld_rec) by a level-1 node's last
// arriving block (the hand-off form of MI355X_MICROARCH.md's table row 1, GroupArgs).

// Fold nb (<= TREE_FAN) child records staged in LDS (`st`, rec_stride apart, in order) into one node record `G`
// (write-through stores): m = the children's minimum (cost, row) key, its record's tag; MPPI / CEM: s = sum_c
// scale_c s_c and v[j] = sum_c scale_c v_c[j] child by child with scale_c = exp(-(m_c - m)); random sampling:
// s = 1; the node's key (K == 1: the fold runs for MPPI / random sampling only, group_size).  The merge kernel's
// tree levels (merge_body) and the host restatement (srbd_api.hip host_fold) are the same arithmetic.  All threads
// of the block call it.
__device__ __forceinline__ void fold_node_lds(const ModelConst& mc, const float* st, int rec_stride, int nb, float* G) {
    __shared__ float sc_sh[TREE_FAN];
    __shared__ float gh_sh[2];  // node m, tag
    __shared__ uint64_t gk_sh[MAXK + 1];
    const int tid = threadIdx.x, T = blockDim.x;
    const int P = mc.P, K = mc.K;
    const bool rs = mc.method == SRBD_RANDOM_SAMPLING;
    if (tid < 64) {  // wave 0: headers, the node key, scales, top-K
        const float* R = st + (size_t)tid * rec_stride;
        const bool have = tid < nb;
        const float m = have ? R[0] : 0.0f;
        const uint32_t row = have ? __float_as_uint(R[2]) : 0u;
        const uint64_t key = have ? ((uint64_t)__float_as_uint(m) << 32) | row : KEY_NONE;
        const uint64_t gk = wave_min_u64(key);
        const float beta = __uint_as_float((uint32_t)(gk >> 32));
        if (key == gk) gh_sh[1] = R[3];  // keys are unique: one writer
        if (tid == 0) {
            gh_sh[0] = beta;
            gk_sh[MAXK] = gk;
        }
        if (have) sc_sh[tid] = rs ? 1.0f : expf(-1.0f * (m - beta));
        if (tid == 0) gk_sh[0] = gk;  // K == 1: the in-launch fold is not used for CEM (group_size)
    }
    __syncthreads();
    SRBD_LSTAMP(4);
    if (!rs) {  // column j < P: sum_c scale_c v_c[j]; column P: sum_c scale_c s_c (child order)
        for (int j = tid; j <= P; j += T) {
            const int off = j < P ? REC_HDR + j : 1;
            float a = 0.0f;
            int cb = 0;
            for (; cb + 8 <= nb; cb += 8) {  // 8 children's LDS loads in flight, then their adds in order
                float x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) x[u] = st[(size_t)(cb + u) * rec_stride + off];
#pragma unroll
                for (int u = 0; u < 8; ++u) a = a + sc_sh[cb + u] * x[u];
            }
            for (; cb < nb; ++cb) a = a + sc_sh[cb] * st[(size_t)cb * rec_stride + off];
            st_rec(&G[off], a);
        }
    }
    SRBD_LSTAMP(5);
    if (tid == 0) {
        st_rec(&G[0], gh_sh[0]);
        if (rs) st_rec(&G[1], 1.0f);
        st_rec(&G[2], __uint_as_float((uint32_t)gk_sh[MAXK]));
        st_rec(&G[3], gh_sh[1]);
    }
    if (tid < K) {
        const uint64_t kk = gk_sh[tid];
        st_rec(&G[REC_HDR + P + 2 * tid], __uint_as_float((uint32_t)kk));
        st_rec(&G[REC_HDR + P + 2 * tid + 1], __uint_as_float((uint32_t)(kk >> 32)));
    }
}

// Level-1 fold in the launch (GroupArgs::gsize > 1): the blocks of a level-1 node (TREE_FAN leaves, aligned to the
// global leaf index: the rank's first leaf is a multiple of TREE_FAN, tree_shape) count themselves in cnt[g]; the
// last one stages the node's leaf records (sc1 loads, all in flight together) into `st` (>= TREE_FAN * rec_stride
// floats of LDS) and folds them into grecs[g].  Returns true (every thread) in the block that wrote the node.
__device__ __forceinline__ bool level1_fold(const ModelConst& mc, const float* __restrict__ recs, int rec_stride,
                                            const GroupArgs& grp, int nroll, int lpb, float* st) {
    __shared__ int last_sh;
    const int tid = threadIdx.x;
    const int bpg = TREE_FAN / lpb;  // blocks per level-1 node
    const int g = (int)blockIdx.x / bpg;
    const int nblk = min(bpg, nroll - g * bpg);
    const int nb = min(TREE_FAN, mc.nleaf - g * TREE_FAN);  // the node's leaves
    SRBD_LSTAMP(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's record stores have completed
    __syncthreads();
    SRBD_LSTAMP(1);
    if (tid == 0) {
        const uint32_t old = __hip_atomic_fetch_add(grp.cnt + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_sh = old == (uint32_t)(nblk - 1);
    }
    __syncthreads();
    if (!last_sh) return false;
    SRBD_LSTAMP(2);
    if (tid == 0) __hip_atomic_store(grp.cnt + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    stage_recs16<5>(recs + (size_t)g * TREE_FAN * rec_stride, st, nb * rec_stride);  // the node's nb leaf records
    __syncthreads();
    SRBD_LSTAMP(3);
    fold_node_lds(mc, st, rec_stride, nb, grp.grecs + (size_t)g * rec_stride);
    return true;
}

// Wave sum in a fixed DPP tree (row_shr 1/2/4/8 within 16-lane rows, then row_bcast 15/31); the total
// lands in lane 63.  All 64 lanes must be active.  Lane 63's chain is the balanced pairwise tree over the lanes in
// order ((v0 + v1) + (v2 + v3)) + ... (no term ever adds the zero of an invalid source), the leaf sum of the
// reduction tree (srbd_core.h); block_epilogue's LDS path and the host (srbd_api.hip pairwise64) form the same tree.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWMASK, 0xF, false));
}
// The first LEVELS levels of that tree: 4 -> lane 16 r + 15 holds the pairwise sum of 16-lane row r, 5 -> lanes 31
// and 63 hold those of lanes 0..31 and 32..63, 6 -> lane 63 the wave's.
template <int LEVELS>
__device__ __forceinline__ float lane_tree_f32(float v) {
    v = v + dpp_f32<0x111, 0xF>(v);
    v = v + dpp_f32<0x112, 0xF>(v);
    v = v + dpp_f32<0x114, 0xF>(v);
    v = v + dpp_f32<0x118, 0xF>(v);
    if constexpr (LEVELS >= 5) v = v + dpp_f32<0x142, 0xA>(v);
    if constexpr (LEVELS >= 6) v = v + dpp_f32<0x143, 0xC>(v);
    return v;
}
__device__ __forceinline__ float wave_sum_f32(float v) { return lane_tree_f32<6>(v); }

// Leaf sums of the weighted noise, thread form with SPB = 64 SPL samples per block (SPL = 2 / 4): wave w takes
// columns w, w + NW, ...; lane l holds samples SPL l .. SPL l + SPL - 1 of a column (one coalesced load), pairs
// them in registers (the tree's first log2 SPL levels) and the DPP rows finish each leaf (64 / SPL lanes): leaf b's
// sum lands in lane (b + 1) 64 / SPL - 1, which writes it into the block's records in LDS (rbuf; block_epilogue
// stores them whole).  Column P: the e alone.  CB columns' loads are in flight together.
// Thread form, 4 leaves per block, MPPI on the device Philox stream: the first REGEN_QUADS column quads of the
// draws are regenerated here (the same Philox4x32-10 call and Box-Muller pairs rng_item made, so the same bits)
// instead of re-read; the rest are re-read.  That trades VALU issue for HBM reads where the launch has both to
// spare (C5 issue 71.6 of 104 us, 656 MB read).
// RG = 2 (the in-launch draws, GroupArgs::gen: the rollout made the step's draws itself and stored only quads
// [gen - 1, P / 4)): quads [0, gen - 1) are regenerated.
constexpr int REGEN_QUADS = 16;  // C5 step launch 106.8 / 98.3 / 96.5 / 97.1 / 98.7 us at 0 / 12 / 16 / 20 / 24 of 36
template <int SPL, int RG>
__device__ __forceinline__ void leaf_wsum_lanes(const ModelConst& mc, const StepInput* __restrict__ in,
                                                const float* __restrict__ base, bool zs, const float* e_sh,
                                                float* rbuf, int rec_stride, int k0, int gen = 0) {
    constexpr int CB = SPL == 4 ? 8 : 12;
    constexpr int LPL = 64 / SPL;  // lanes per leaf
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, NW = blockDim.x >> 6;
    const int P = mc.P;
    const size_t ldn = (size_t)mc.ldn;
    float e[SPL];
#pragma unroll
    for (int u = 0; u < SPL; ++u) e[u] = e_sh[SPL * lane + u];
    float* rec = rbuf + (lane / LPL) * rec_stride;
    const bool writer = (lane % LPL) == LPL - 1;
    int jreg = 0;  // columns [0, jreg) regenerated
    if constexpr (RG && SPL == 4) {
        if (RG == 2 || (mc.method == SRBD_MPPI && mc.rng == RNG_PHILOX && in->noise_scaled == 0 && 4 * REGEN_QUADS <= P)) {
            const uint32_t key0 = in->seed_lo, key1 = in->seed_hi, c2 = in->ctr_lo, c3 = in->ctr_hi;
            const int nq = RG == 2 ? gen - 1 : REGEN_QUADS;
            for (int q = w; q < nq; q += NW) {
                float zq[4][SPL];  // [column 4q + i][row u]
#pragma unroll
                for (int u = 0; u < SPL; ++u) {
                    const int k = k0 + SPL * lane + u, r = mc.row0 + k;
                    uint32_t c[4] = {(uint32_t)(r - 1), (uint32_t)q, c2, c3};
                    philox4x32_10(c, key0, key1);
                    float v[4];
                    box_muller(c[0], c[1], v[0], v[1]);
                    box_muller(c[2], c[3], v[2], v[3]);
                    // rng_item's value; row 0 (the warm start) and rows past n_local hold zeros in the buffer
                    const bool live = r > 0 && k < mc.n_local;
#pragma unroll
                    for (int i = 0; i < 4; ++i) zq[i][u] = live ? mc.sigma_mppi * v[i] : 0.0f;
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float p[SPL];
#pragma unroll
                    for (int u = 0; u < SPL; ++u) p[u] = e[u] * (zq[i][u] * 1.0f);  // the read path's x * 1
                    float a = (p[0] + p[1]) + (p[2] + p[3]);
                    a = lane_tree_f32<4>(a);
                    if (writer) rec[REC_HDR + 4 * q + i] = a;
                }
            }
            jreg = 4 * nq;
        }
    }
    for (int j0 = jreg + w; j0 <= P; j0 += CB * NW) {
        float z[CB][SPL];
#pragma unroll
        for (int b = 0; b < CB; ++b) {
            const int j = j0 + b * NW;
            const float* col = base + (size_t)(j < P ? j : 0) * ldn + SPL * lane;
            if constexpr (SPL == 4) {
                const float4 v = *reinterpret_cast<const float4*>(col);
                z[b][0] = v.x, z[b][1] = v.y, z[b][2] = v.z, z[b][3] = v.w;
            } else {
                const float2 v = *reinterpret_cast<const float2*>(col);
                z[b][0] = v.x, z[b][1] = v.y;
            }
        }
#pragma unroll
        for (int b = 0; b < CB; ++b) {
            const int j = j0 + b * NW;
            if (j > P) break;
            float p[SPL];
            if (j < P) {
                const float sj = zs ? in->sigma[j] : 1.0f;  // x * 1 == x
#pragma unroll
                for (int u = 0; u < SPL; ++u) p[u] = e[u] * (z[b][u] * sj);
            } else {
#pragma unroll
                for (int u = 0; u < SPL; ++u) p[u] = e[u];
            }
            float a;
            if constexpr (SPL == 4)
                a = (p[0] + p[1]) + (p[2] + p[3]);
            else
                a = p[0] + p[1];
            a = lane_tree_f32<SPL == 4 ? 4 : 5>(a);
            if (writer) rec[j < P ? REC_HDR + j : 1] = a;
        }
    }
}

// Leaf sums, one 64-sample leaf per block (four-lane form, thread form at 64 samples per block): thread j forms
// column j's 64 products from the LDS stage (ZS: row s at zst[s zstride]) or the SoA noise (16 float4 loads in
// flight) and adds them in the pairwise tree in registers; the last wave adds the e alone (column P) by DPP.
template <bool ZS>
__device__ __forceinline__ void leaf_wsum_cols(const ModelConst& mc, const StepInput* __restrict__ in,
                                               const float* __restrict__ base, const float* zst, int zstride, bool zs,
                                               const float* e_sh, float* __restrict__ rec) {
    const int tid = threadIdx.x, T = blockDim.x, P = mc.P;
    const size_t ldn = (size_t)mc.ldn;
    if ((tid >> 6) == (T >> 6) - 1) {
        const float t = wave_sum_f32(e_sh[tid & 63]);
        if ((tid & 63) == 63) st_rec(&rec[1], t);
    }
    for (int j = tid; j < P; j += T) {
        const float sj = zs ? in->sigma[j] : 1.0f;  // x * 1 == x
        float first = 0.0f, tot = 0.0f;
#pragma nounroll
        for (int h = 0; h < 2; ++h) {  // the tree's two 32-row halves one after the other (registers), then the root
            float lv[16];
            if constexpr (ZS) {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int r = 32 * h + 2 * i;
                    lv[i] = e_sh[r] * (zst[r * zstride + j] * sj) + e_sh[r + 1] * (zst[(r + 1) * zstride + j] * sj);
                }
            } else {
                const float4* row = reinterpret_cast<const float4*>(base + (size_t)j * ldn) + 8 * h;
                float4 v[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = row[i];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int r = 32 * h + 4 * i;
                    lv[2 * i] = e_sh[r] * (v[i].x * sj) + e_sh[r + 1] * (v[i].y * sj);
                    lv[2 * i + 1] = e_sh[r + 2] * (v[i].z * sj) + e_sh[r + 3] * (v[i].w * sj);
                }
            }
#pragma unroll
            for (int n = 8; n >= 1; n >>= 1)
#pragma unroll
                for (int i = 0; i < n; ++i) lv[i] = lv[2 * i] + lv[2 * i + 1];
            if (h == 0)
                first = lv[0];
            else
                tot = first + lv[0];
        }
        st_rec(&rec[REC_HDR + j], tot);
    }
}

// The block's leaf records (srbd_core.h): SPB samples = lpb = SPB / 64 leaves (four-lane: 1; thread form: 1, 2
// or 4), leaf b of block x at record x lpb + b.  The thread owning sample `sib` passes it (others -1) with its
// `tag` (the gait-adaptive step frequency, else 0), which the owner of the leaf's best row stores in the header.
//  keys -> LDS; leaf minima (one wave per leaf); CEM: each leaf's K smallest keys by ranks (every sample counts
//  the leaf's keys below its own; the `lps` lanes of a sample split the count, summed by DPP); e = exp(-(c - m));
//  the sums v[j] = sum_l e_l noise_l[j] and s = sum_l e_l of each leaf in the pairwise tree over its 64 rows
//  (leaf_wsum_cols at one leaf per block, from the LDS stage `zst` (ZS: four-lane zero-order) or the SoA noise;
//  leaf_wsum_lanes at 2 / 4 leaves per block).
// Then the level-1 fold (grp.gsize > 1).  All threads call it; returns level1_fold's verdict (false without one).
// TF: the thread form (2 / 4 leaves per block: records assembled in LDS); the four-lane kernels pass false and carry
// none of that LDS, nor (CEM: no in-launch fold) the fold's stage -- static LDS a fused launch's draw blocks share.
template <bool CEMT, bool ZS = false, bool TF = false, int RG = 0>
__device__ __forceinline__ bool block_epilogue(const ModelConst& mc, const StepInput* __restrict__ in, const int SPB,
                                               int sib, bool valid, float cost, const float* __restrict__ noise,
                                               float* __restrict__ recs, int rec_stride, float tag,
                                               const GroupArgs& grp, int nroll, float* zst = nullptr,
                                               int zstride = 0) {
    // ZS (four-lane, 64 samples per block): sized for one leaf, so the block's LDS (the noise stage) stays within a
    // quarter of the CU's 160 KB (four blocks per CU)
    __shared__ uint64_t ks[ZS ? 64 : 256];
    __shared__ float e_sh[ZS ? 64 : 256];
    __shared__ uint64_t lmin[4];
    __shared__ uint64_t lel[CEMT ? 4 : 1][CEMT ? MAXK : 1];
    // thread form with 2 / 4 leaves per block: the records are assembled in LDS and stored whole (consecutive
    // lanes, consecutive words) instead of word by word from the lanes that finish each sum
    __shared__ float rbuf[TF ? 4 * ((REC_HDR + MAXP + 2 * MAXK + 3) & ~3) : 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int lpb = SPB >> 6;
    const int P = mc.P, K = mc.K;
    const int k0 = blockIdx.x * SPB;
    const bool rs = mc.method == SRBD_RANDOM_SAMPLING;
    const uint64_t key = (sib >= 0 && valid) ? cost_key(cost, (uint32_t)(mc.row0 + k0 + sib)) : KEY_NONE;
    if (sib >= 0) ks[sib] = key;
    __syncthreads();
    // one leaf per block (the four-lane zero-order MPPI / random-sampling blocks): every wave forms the leaf minimum
    // itself (the same keys, the same value), so the exponentials need no second barrier
    constexpr bool ONE = ZS && !CEMT;
    uint64_t m1 = KEY_NONE;
    if constexpr (ONE) {
        m1 = wave_min_u64(ks[lane]);
    } else if (w < lpb) {
        const uint64_t m = wave_min_u64(ks[64 * w + lane]);
        if (lane == 0) lmin[w] = m;
    }
    if constexpr (CEMT) {
        if (K > 1) {
            for (int i = tid; i < lpb * MAXK; i += (int)blockDim.x) lel[i / MAXK][i % MAXK] = KEY_NONE;
            __syncthreads();
            const int lps = (int)blockDim.x / SPB, part = tid & (lps - 1), s = tid / lps, b = s >> 6;
            const uint64_t mine = ks[s];
            const int span = 64 / lps, i0 = 64 * b + part * span;
            int cnt = 0;
            for (int i = 0; i < span; ++i) cnt += ks[i0 + i] < mine ? 1 : 0;
            if (lps >= 2) cnt += __builtin_amdgcn_mov_dpp(cnt, 0xB1, 0xF, 0xF, true);  // quad lanes (1, 0, 3, 2)
            if (lps == 4) cnt += __builtin_amdgcn_mov_dpp(cnt, 0x4E, 0xF, 0xF, true);  // quad lanes (2, 3, 0, 1)
            if (part == 0 && cnt < K) lel[b][cnt] = mine;
        }
    }
    if constexpr (!ONE) __syncthreads();
    SRBD_RSTAMP(3);
    if (!rs) {
        const uint64_t lm = ONE ? m1 : (sib >= 0 ? lmin[sib >> 6] : KEY_NONE);
        if (sib >= 0) e_sh[sib] = valid ? expf(-1.0f * (cost - u2f((uint32_t)(lm >> 32)))) : 0.0f;
        __syncthreads();
        const bool zs = CEMT && zs_scaled(mc, in);
        if (SPB == 64)
            leaf_wsum_cols<ZS>(mc, in, noise + k0, zst, zstride, zs, e_sh, recs + (size_t)blockIdx.x * rec_stride);
        else if constexpr (TF) {
            if (SPB == 128)
                leaf_wsum_lanes<2, RG>(mc, in, noise + k0, zs, e_sh, rbuf, rec_stride, k0);
            else
                leaf_wsum_lanes<4, RG>(mc, in, noise + k0, zs, e_sh, rbuf, rec_stride, k0, grp.gen);
        }
    }
    SRBD_RSTAMP(4);
    const bool via_lds = TF && SPB > 64;
    float* const grec = recs + (size_t)blockIdx.x * lpb * rec_stride;  // the block's lpb records, consecutive
    auto put = [&](int b, int off, float v) {
        if (via_lds)
            rbuf[b * rec_stride + off] = v;
        else
            st_rec(&grec[(size_t)b * rec_stride + off], v);
    };
    // ONE: every thread holds the leaf minimum (m1); random sampling passed no barrier since lmin was written
    auto leafmin = [&](int b) { return ONE ? m1 : lmin[b]; };
    if (tid < lpb) {  // headers of leaf tid
        const uint64_t m = leafmin(tid);
        put(tid, 0, u2f((uint32_t)(m >> 32)));
        put(tid, 2, u2f((uint32_t)m));
        if (rs) put(tid, 1, 1.0f);
    }
    if (sib >= 0 && key == leafmin(sib >> 6)) put(sib >> 6, 3, tag);
    for (int i = tid; i < lpb * K; i += (int)blockDim.x) {  // keys
        const int b = i / K, q = i % K;
        uint64_t kk = leafmin(b);
        if constexpr (CEMT) kk = K > 1 ? lel[b][q] : kk;
        put(b, REC_HDR + P + 2 * q, u2f((uint32_t)kk));
        put(b, REC_HDR + P + 2 * q + 1, u2f((uint32_t)(kk >> 32)));
    }
    if (via_lds) {
        __syncthreads();
        for (int i = tid; i < lpb * rec_stride; i += (int)blockDim.x) st_rec(&grec[i], rbuf[i]);
    }
    if constexpr (!CEMT) {  // group_size: no in-launch fold for CEM
        if (grp.gsize > 1) {
            if (grp.fast) return true;  // the caller's fast_tail counts, folds and merges (srbd_kernels.hip)
            if constexpr (ZS) {
                return level1_fold(mc, recs, rec_stride, grp, nroll, lpb, zst);
            } else {
                __shared__ __attribute__((aligned(16))) float st[GROUP_LDS_FLOATS];  // stage_recs16: 16-byte stores
                return level1_fold(mc, recs, rec_stride, grp, nroll, lpb, st);
            }
        }
    }
    return false;
}

// ---- gait-adaptive rollout (centroidal_nmpc_jax_gait_adaptive.py:326-501).
// One thread per sample.  The sample's step frequency f is injected (ga_explicit) or drawn from the
// per-call set with one Philox call on the sample's own counter lane (jax.random.choice, GA:692/836;
// the threefry stream is not reproduced); its contact sequence is the JAX gait
// generator's (periodic_gait_generator_jax.py:68-151) run from the caller's leg phases, kept as one
// bit mask per leg; each leg's decode index counts its stance steps so far (n_, GA:339/353-356,
// -1 before the first touchdown: jnp's negative index wraps to the leg's last parameter) with
// horizon_leg = stance steps + 1 (GA:345-348); the cost gains (f - 1.3) * 100 * (f - 1.3) (GA:500).
constexpr uint32_t GA_FREQ_LANE = 0x10000u;  // Philox counter word 1 of the frequency draw (noise uses < P/4)

__device__ __forceinline__ float ga_sample_freq(const ModelConst& mc, const StepInput* __restrict__ in, int k) {
    if (in->ga_explicit) return mc.ga_freq[k];
    const uint64_t seed = ((uint64_t)in->seed_hi << 32) | in->seed_lo;
    if (mc.rng != RNG_PHILOX)  // jax.random.choice(key, freqs, (N,)) at the sample's global row
        return in->ga_freqs[jax_choice_index((uint32_t)(seed >> 32), (uint32_t)seed, (uint64_t)(mc.row0 + k),
                                             (uint64_t)mc.N, (uint32_t)in->ga_nfreq, mc.rng == RNG_JAX)];
    uint32_t c[4] = {(uint32_t)(mc.row0 + k), GA_FREQ_LANE, in->ctr_lo, in->ctr_hi};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t i = (uint32_t)(((uint64_t)c[0] * (uint32_t)in->ga_nfreq) >> 32);  // uniform in [0, n)
    return in->ga_freqs[i];
}

// Per-leg contact masks of one sample (bit n = stance at step n), PGGJ:136-151 with run :68-89:
// restart (t >= 1 -> 0), advance by pgg_dt * f (the product first), stance while t < duty.
__device__ __forceinline__ void ga_contact_masks(const StepInput* __restrict__ in, int H, float f, uint32_t mask[4]) {
    const float inc = in->ga_dt * f;
    float t[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        t[l] = in->ga_timing[l];
        mask[l] = 0u;
    }
    for (int n = 0; n < H; ++n)
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            t[l] = t[l] >= 1.0f ? 0.0f : t[l];
            t[l] = t[l] + inc;
            mask[l] |= (t[l] < in->ga_duty ? 1u : 0u) << n;
        }
}

}  // namespace srbd
