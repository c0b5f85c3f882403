// srbd_jaxrng.h -- the jax.random stream the reference draws its sampling noise from, for host and device
// (SRBD_RNG_JAX / SRBD_RNG_JAX_LEGACY, srbd_set_rng).
//
// Reference calls (paths relative to the reference repository root):
//   jax.random.PRNGKey(42)                          centroidal_nmpc_jax.py:167
//   master_key <- jax.random.split(master_key)[0]   centroidal_nmpc_jax.py:498-501 (with_newkey)
//   jax.random.normal(key, (n, P))                  centroidal_nmpc_jax.py:654, 663, 811, 957
//   jax.random.uniform(key, (n, P), -s, s)          centroidal_nmpc_jax.py:671-676
//   jax.random.choice(key, a, (N,))                 centroidal_nmpc_jax_gait_adaptive.py:692, 836-837
// JAX is not vendored in the reference and not installed here; this restates its published algorithm
// (jax._src.prng threefry2x32 / threefry_split / threefry_random_bits, jax._src.random _uniform /
// _normal_real / _randint, XLA's float32 ErfInv), the same as oracle/jax_random_oracle.py (the checker).
//   Threefry-2x32-20: ks = (k0, k1, k0 ^ k1 ^ 0x1BD11BDA), rotations 13 15 26 6 / 17 29 16 24, a key
//   injection after every four rounds (second word + injection count).
//   Counter layouts (jax_threefry_partitionable):
//     partitionable (JAX >= 0.5 default): element i of any draw = t0 ^ t1, (t0, t1) = tf(key, (hi32 i, lo32 i));
//       split(key)[j] = tf(key, (0, j));
//     legacy: a draw of M elements pairs counts (i, i + h), h = ceil(M / 2) (count M -> 0 when M is odd):
//       element i < h is word 0 of that pair's output, element h + i word 1; split(key) = bits of M = 4 as (2, 2).
//   bits -> [0, 1): bitcast((b >> 9) | 0x3F800000) - 1;  uniform = max(lo, fma(f, hi - lo, lo));
//   normal = sqrt(2) * erf_inv(uniform(nextafter(-1, 0), 1)), erf_inv: Giles' single-precision form with a
//   fused Horner chain; log1p correctly rounded (float64, one rounding).
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIP__) || defined(__HIPCC__)
#include <hip/hip_runtime.h>
#endif
#ifndef SRBD_HD
#if defined(__HIP__) || defined(__HIPCC__)
#define SRBD_HD __host__ __device__ __forceinline__
#else
#define SRBD_HD inline  // plain C++ (srbd_host.cpp)
#endif
#endif

namespace srbd {

enum { RNG_PHILOX = 0, RNG_JAX = 1, RNG_JAX_LEGACY = 2 };  // == SRBD_RNG_* (include/srbd_mpc.h)

SRBD_HD uint32_t tf_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

SRBD_HD void threefry2x32_20(uint32_t k0, uint32_t k1, uint32_t& x0, uint32_t& x1) {
    const uint32_t ks[3] = {k0, k1, k0 ^ k1 ^ 0x1BD11BDAu};
    constexpr int R[2][4] = {{13, 15, 26, 6}, {17, 29, 16, 24}};
    x0 += ks[0];
    x1 += ks[1];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            x0 += x1;
            x1 = tf_rotl(x1, R[i & 1][j]);
            x1 ^= x0;
        }
        x0 += ks[(i + 1) % 3];
        x1 += ks[(i + 2) % 3] + (uint32_t)(i + 1);
    }
}

// 32 random bits of element i (row-major flat index) of a draw of M elements.
SRBD_HD uint32_t jax_bits(uint32_t k0, uint32_t k1, uint64_t i, uint64_t M, bool partitionable) {
    uint32_t x0, x1;
    if (partitionable) {
        x0 = (uint32_t)(i >> 32);
        x1 = (uint32_t)i;
        threefry2x32_20(k0, k1, x0, x1);
        return x0 ^ x1;
    }
    const uint32_t h = (uint32_t)((M + 1) >> 1), ii = (uint32_t)i;
    if (ii < h) {
        x0 = ii;
        x1 = (uint64_t)ii + h < M ? ii + h : 0u;  // an odd M pads its counts with one 0
        threefry2x32_20(k0, k1, x0, x1);
        return x0;
    }
    x0 = ii - h;
    x1 = ii;
    threefry2x32_20(k0, k1, x0, x1);
    return x1;
}

// jax.random.split(key, 2) -> (a, b): a = [a0, a1], b = [b0, b1].
SRBD_HD void jax_split2(uint32_t k0, uint32_t k1, bool partitionable, uint32_t a[2], uint32_t b[2]) {
    if (partitionable) {
        uint32_t x0 = 0, x1 = 0;
        threefry2x32_20(k0, k1, x0, x1);
        a[0] = x0, a[1] = x1;
        x0 = 0, x1 = 1;
        threefry2x32_20(k0, k1, x0, x1);
        b[0] = x0, b[1] = x1;
        return;
    }
    // bits of iota(4): pairs (0, 2), (1, 3) -> [y0(0,2), y0(1,3), y1(0,2), y1(1,3)] reshaped (2, 2)
    uint32_t p0 = 0, p1 = 2, q0 = 1, q1 = 3;
    threefry2x32_20(k0, k1, p0, p1);
    threefry2x32_20(k0, k1, q0, q1);
    a[0] = p0, a[1] = q0;
    b[0] = p1, b[1] = q1;
}

// with_newkey: key <- split(key)[0], `times` times.  The 64-bit packing of a key is k0 << 32 | k1.
SRBD_HD uint64_t jax_next_key(uint64_t key, bool partitionable, int times = 1) {
    for (int t = 0; t < times; ++t) {
        uint32_t a[2], b[2];
        jax_split2((uint32_t)(key >> 32), (uint32_t)key, partitionable, a, b);
        key = ((uint64_t)a[0] << 32) | a[1];
    }
    return key;
}

SRBD_HD float jax_unit(uint32_t b) {
    union { uint32_t u; float f; } x;
    x.u = (b >> 9) | 0x3F800000u;
    return x.f - 1.0f;
}

// uniform(minval = lo, maxval) with range = f32(maxval - lo)
SRBD_HD float jax_uniform(uint32_t b, float lo, float range) {
    const float v = fmaf(jax_unit(b), range, lo);
    return v > lo ? v : lo;
}

SRBD_HD float log1p_cr(float x) { return (float)log1p((double)x); }

SRBD_HD float sqrt_rn(float x) {
#ifdef __HIP_DEVICE_COMPILE__
    return __fsqrt_rn(x);
#else
    return sqrtf(x);
#endif
}

// XLA ErfInv (float32)
SRBD_HD float jax_erf_inv(float x) {
    constexpr float A[9] = {2.81022636e-08f, 3.43273939e-07f, -3.5233877e-06f, -4.39150654e-06f, 0.00021858087f,
                            -0.00125372503f, -0.00417768164f, 0.246640727f,    1.50140941f};
    constexpr float B[9] = {-0.000200214257f, 0.000100950558f, 0.00134934322f, -0.00367342844f, 0.00573950773f,
                            -0.0076224613f,   0.00943887047f,  1.00167406f,    2.83297682f};
    float w = -log1p_cr(x * (-x));
    const bool lt = w < 5.0f;
    w = lt ? w - 2.5f : sqrt_rn(w) - 3.0f;
    float p = lt ? A[0] : B[0];
#pragma unroll
    for (int i = 1; i < 9; ++i) p = fmaf(p, w, lt ? A[i] : B[i]);
    return p * x;  // |x| == 1 (the +-inf edge) cannot occur: u lies in [nextafter(-1, 0), 1)
}

constexpr float JAX_NORMAL_LO = -0.99999994039535522461f;  // nextafter(-1, 0)
constexpr float JAX_SQRT2 = 1.41421353816986083984f;       // float32(sqrt(2))

SRBD_HD float jax_normal(uint32_t b) {
    // f32(1 - nextafter(-1, 0)) == 2.0f
    const float u = jax_uniform(b, JAX_NORMAL_LO, 2.0f);
    return JAX_SQRT2 * jax_erf_inv(u);
}

// jax.random.choice(key, a, (M,)) with replacement: index of element i in [0, n) (randint: split the key,
// 32 bits from each half, ((hi % n) * m + lo % n) % n with m = (2^16 % n)^2 % n, uint32 arithmetic).
SRBD_HD uint32_t jax_choice_index(uint32_t k0, uint32_t k1, uint64_t i, uint64_t M, uint32_t n, bool partitionable) {
    uint32_t a[2], b[2];
    jax_split2(k0, k1, partitionable, a, b);
    const uint32_t hi = jax_bits(a[0], a[1], i, M, partitionable);
    const uint32_t lo = jax_bits(b[0], b[1], i, M, partitionable);
    const uint32_t span = n < 1 ? 1u : n;
    uint32_t m = 65536u % span;
    m = (m * m) % span;
    const uint32_t off = (hi % span) * m + lo % span;
    return off % span;
}

}  // namespace srbd
