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
//   fused Horner chain; log1p: float64's, rounded once to float (log1p_fast: the same float from a short float64
//   evaluation, the float64 log1p only where that one is too close to a rounding boundary).
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

// ---- log1p_cr without float64's log1p on the common path (jax_erf_inv's argument t = -x^2 in (-1, 0]).
// LOG1P_TAB[k] = {c_k, -log(c_k)}: c_k = 1 / (1 + (k + 1/2) / 128) rounded to a multiple of 2^-8 (so m c_k - 1 is
// small, |.| <= 2^-7.4, for m in bin k of [1, 2)), -log(c_k) to double from a 60-digit evaluation
// (tests/test_jax_random.py checks the function against the float64 log1p).
struct Log1pEnt {
    double c, nlogc;
};
constexpr Log1pEnt LOG1P_TAB[128] = {
    {0.99609375, 0.003913899321136329}, {0.98828125, 0.01178795575204224}, {0.98046875, 0.01972450534777859}, {0.97265625, 0.027724548014854862},
    {0.96484375, 0.03578910785158528}, {0.95703125, 0.04391923393483549}, {0.953125, 0.048009219186360606}, {0.9453125, 0.05623971832287608},
    {0.9375, 0.06453852113757118}, {0.9296875, 0.07290677080808779}, {0.92578125, 0.07711730334443129}, {0.91796875, 0.08559193033540351},
    {0.91015625, 0.09413899091386191}, {0.90625, 0.09844007281325252}, {0.8984375, 0.1070981355563671}, {0.890625, 0.1158318155251217},
    {0.88671875, 0.1202274269981598}, {0.87890625, 0.12907704227514236}, {0.875, 0.13353139262452263}, {0.8671875, 0.14250006260728304},
    {0.86328125, 0.14701474296180966}, {0.85546875, 0.15610571466306167}, {0.8515625, 0.16068238169047347}, {0.84375, 0.16989903679539747},
    {0.83984375, 0.17453941635189968}, {0.83203125, 0.18388527877013736}, {0.828125, 0.18859116980755003}, {0.82421875, 0.19331931100349597},
    {0.81640625, 0.20284319251475147}, {0.8125, 0.2076393647782445}, {0.80859375, 0.2124586512141934}, {0.80078125, 0.2221674653411543},
    {0.796875, 0.22705745063534608}, {0.79296875, 0.23197146543777514}, {0.7890625, 0.2369097470783577}, {0.78125, 0.24686007793152578},
    {0.77734375, 0.2518726197550701}, {0.7734375, 0.2569104137850272}, {0.76953125, 0.26197371574157396}, {0.765625, 0.26706278524904525},
    {0.7578125, 0.27731928541623435}, {0.75390625, 0.2824872555746769}, {0.75, 0.2876820724517809}, {0.74609375, 0.2929040164329326},
    {0.7421875, 0.29815337231907635}, {0.73828125, 0.3034304294199201}, {0.734375, 0.3087354816496133}, {0.73046875, 0.31406882762497584},
    {0.7265625, 0.3194307707663612}, {0.72265625, 0.32482161940123766}, {0.71875, 0.33024168687057687}, {0.71484375, 0.33569129163814154},
    {0.7109375, 0.34117075740276714}, {0.70703125, 0.3466804132137367}, {0.703125, 0.3522205935893521}, {0.69921875, 0.3577916386388075},
    {0.6953125, 0.3633938941874773}, {0.69140625, 0.36902771190573336}, {0.6875, 0.3746934494414107}, {0.68359375, 0.38039147055604844},
    {0.6796875, 0.38612214526503347}, {0.67578125, 0.39188584998178355}, {0.671875, 0.39768296766610944}, {0.66796875, 0.40351388797690263},
    {0.6640625, 0.4093790074293007}, {0.66015625, 0.415278729556489}, {0.65625, 0.42121346507630353}, {0.65625, 0.42121346507630353},
    {0.65234375, 0.42718363206280735}, {0.6484375, 0.43318965612301924}, {0.64453125, 0.4392319705789819}, {0.640625, 0.44531101665536404},
    {0.63671875, 0.4514272436728001}, {0.63671875, 0.4514272436728001}, {0.6328125, 0.4575811092471784}, {0.62890625, 0.4637730794950995},
    {0.625, 0.4700036292457356}, {0.62109375, 0.47627324225933093}, {0.62109375, 0.47627324225933093}, {0.6171875, 0.48258241145259567},
    {0.61328125, 0.4889316391312544}, {0.609375, 0.4953214372300254}, {0.609375, 0.4953214372300254}, {0.60546875, 0.5017523275603158},
    {0.6015625, 0.5082248420659333}, {0.59765625, 0.514739523087127}, {0.59765625, 0.514739523087127}, {0.59375, 0.5212969236332861},
    {0.58984375, 0.5278976076646381}, {0.58984375, 0.5278976076646381}, {0.5859375, 0.5345421503833068}, {0.58203125, 0.5412311385341033},
    {0.58203125, 0.5412311385341033}, {0.578125, 0.5479651707154474}, {0.57421875, 0.5547448577008262}, {0.57421875, 0.5547448577008262},
    {0.5703125, 0.561570822771226}, {0.56640625, 0.5684437020589881}, {0.56640625, 0.5684437020589881}, {0.5625, 0.5753641449035618},
    {0.55859375, 0.5823328142196552}, {0.55859375, 0.5823328142196552}, {0.5546875, 0.5893503868783018}, {0.5546875, 0.5893503868783018},
    {0.55078125, 0.5964175541013942}, {0.546875, 0.6035350218702582}, {0.546875, 0.6035350218702582}, {0.54296875, 0.6107035113488707},
    {0.54296875, 0.6107035113488707}, {0.5390625, 0.6179237593223578}, {0.53515625, 0.6251965186514375}, {0.53515625, 0.6251965186514375},
    {0.53125, 0.6325225587435105}, {0.53125, 0.6325225587435105}, {0.52734375, 0.639902666041133}, {0.52734375, 0.639902666041133},
    {0.5234375, 0.6473376445286511}, {0.51953125, 0.6548283162578087}, {0.51953125, 0.6548283162578087}, {0.515625, 0.6623755218931916},
    {0.515625, 0.6623755218931916}, {0.51171875, 0.6699801212784109}, {0.51171875, 0.6699801212784109}, {0.5078125, 0.6776429940239801},
    {0.5078125, 0.6776429940239801}, {0.50390625, 0.6853650401178903}, {0.50390625, 0.6853650401178903}, {0.5, 0.6931471805599453},
};

// The float64 evaluation: |t| < 2^-7 the Taylor polynomial to t^6 / 6 (truncation < t^6 / 7 <= 2^-44.8 relative; t
// is exact in float64); else y = 1 + t (exact) = 2^e m, m in [1, 2), k = m's top 7 fraction bits, r = m c_k - 1 (one
// rounding: the product has <= 62 bits), log y = e ln2 + (-log c_k) + log1p(r) (polynomial to r^6 / 6: truncation
// < 2^-54.6 absolute).  Error < 2^-44 relative (|log y| >= 2^-7 on this branch, so the absolute 2^-51 of the sum
// stays small).
SRBD_HD double log1p_poly(double t) {
    constexpr double C6 = -1.0 / 6, C5 = 1.0 / 5, C4 = -1.0 / 4, C3 = 1.0 / 3, C2 = -1.0 / 2;
    double p = fma(t, C6, C5);
    p = fma(p, t, C4);
    p = fma(p, t, C3);
    p = fma(p, t, C2);
    p = fma(p, t, 1.0);
    return p * t;
}
SRBD_HD double log1p_tab(float t) {
    const bool small = t > -0.0078125f;  // |t| < 2^-7: the polynomial in t alone (no branch: selects below)
    const double y = 1.0 + (double)t;    // exact when !small: t's last bit is >= 2^-31 there
    union { double d; uint64_t u; } b;
    b.d = y;
    const int e = (int)((b.u >> 52) & 0x7FF) - 1023;
    const int k = (int)((b.u >> 45) & 127);
    b.u = (b.u & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull;  // m in [1, 2)
    const Log1pEnt E = LOG1P_TAB[k];
    // small: r = t, -log c = 0, e = 0, and the sum below is log1p_poly(t) itself (+0 + p == p for p != -0)
    const double r = small ? (double)t : fma(b.d, E.c, -1.0);
    const double nl = small ? 0.0 : E.nlogc;
    const double ed = small ? 0.0 : (double)e;
    constexpr double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;  // hi: 32 bits
    return (ed * LN2_HI + nl) + (log1p_poly(r) + ed * LN2_LO);
}
// log1p_cr(t) for t in (-1, 0] -- jax_erf_inv's argument -x^2 -- at a fraction of float64 log1p's cost, the same
// float: log1p_tab's value L is rounded to float when it lies farther than 2^13 of its own ulps (>= 2^-40 |L|, 16
// times its error bound) from the rounding midpoint (Ziv's test, on L's bits: float rounding drops the low 29 of the
// 52 fraction bits, and the midpoint is 2^28 there -- L is a normal float's neighbour, |L| in [2^-30, 17)), so the
// float64 log1p rounds the same way; else (about one draw in 2^15) the float64 log1p itself is evaluated.
// |t| < 2^-29: log1p(t) lies within 2^-30 relative of t, so it rounds to t.
// log1p_try: the float, or false where the float64 log1p must decide (srbd_selftest_log1p counts those).
SRBD_HD bool log1p_try(float t, float* out) {
    bool ok = t > -1.0f && t <= 0.0f;
    float f = t;
    if (ok && t <= -1.862645149230957e-09f) {  // 2^-29
        const double L = log1p_tab(t);
        f = (float)L;
        union { double d; uint64_t u; } b;
        b.d = L;
        const uint32_t r = (uint32_t)b.u & 0x1FFFFFFFu;
        const uint32_t dist = r > 0x10000000u ? r - 0x10000000u : 0x10000000u - r;
        ok = dist > 0x2000u;
    }
    *out = f;
    return ok;
}
SRBD_HD float log1p_fast(float t) {
    float f;
    if (!log1p_try(t, &f)) f = log1p_cr(t);
    return f;
}

// correctly rounded float sqrt (np.sqrt's float32 result).  On the device __builtin_sqrtf is the correctly rounded
// expansion (v_sqrt_f32 and a one-ulp fma correction); __fsqrt_rn lowers to the bare v_sqrt_f32 (within 1 ulp), which
// made 3 of C1's 15 360 draws differ by an ulp once erf_inv's w >= 5 branch stood alone.
SRBD_HD float sqrt_rn(float x) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_sqrtf(x);
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
    float w = -log1p_fast(x * (-x));
    float p;
    if (w < 5.0f) {  // |x| < 0.9966: all but a few lanes of a wave (a branch, not 9 coefficient selects)
        w = w - 2.5f;
        p = A[0];
#pragma unroll
        for (int i = 1; i < 9; ++i) p = fmaf(p, w, A[i]);
    } else {
        w = sqrt_rn(w) - 3.0f;
        p = B[0];
#pragma unroll
        for (int i = 1; i < 9; ++i) p = fmaf(p, w, B[i]);
    }
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
