"""Pins the restatement of the reference's jax.random noise stream (CPU; oracle/jax_random_oracle.py) and the
product's host key helpers (srbd_jax_prng_key / srbd_jax_split, include/srbd_host.h).

The reference draws its sampling noise with jax.random from PRNGKey(42), advanced by split each iteration
(centroidal_nmpc_jax.py:167, 498-501, 654-676, 811, 957).  JAX is not vendored in the reference and not
installed here (JAX itself: parity unpinned).  What pins the restatement:
  * the Threefry-2x32-20 core: Random123's known-answer vectors (kat_vectors, "threefry2x32 20" lines) and
    rocRAND's independent engine (oracle/_pin/threefry_rocrand, built from
    /opt/rocm/include/rocrand/rocrand_threefry2x32_20.h);
  * the layers above it (PRNGKey, split, the legacy counter layout, bits -> float, the uniform map, the
    float32 ErfInv, sqrt(2) scaling): outputs JAX's own documentation prints for
    jax_threefry_partitionable=False (the JAX Quickstart: normal(PRNGKey(0), (10,)); "Sharp bits", random
    numbers: normal(PRNGKey(0), (1,)), split(PRNGKey(0)) and normal(subkey, (1,))) -- 15 float32 values
    matched bit for bit;
  * the partitionable layout (JAX's default since 0.5.0) by construction: split(key)[0] is the Threefry
    output of counter (0, 0), and element i of any draw depends on i only (shape independence).
The GPU draws are checked against this restatement bit for bit in tests/test_gpu_jax_rng.py.
"""
import os
import subprocess
from fractions import Fraction

import numpy as np
import pytest

from oracle import jax_random_oracle as jr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PIN = os.path.join(ROOT, "oracle", "_pin", "threefry_rocrand")
f32 = np.float32

# Random123 kat_vectors, "threefry2x32 20": (ctr, key) -> out
R123 = [
    ((0x00000000, 0x00000000), (0x00000000, 0x00000000), (0x6B200159, 0x99BA4EFE)),
    ((0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF), (0x1CB996FC, 0xBB002BE7)),
    ((0x243F6A88, 0x85A308D3), (0x13198A2E, 0x03707344), (0xC4923A9C, 0x483DF7A0)),
]


@pytest.mark.parametrize("ctr,key,out", R123)
def test_threefry_random123_kat(ctr, key, out):
    y = jr.threefry2x32(key[0], key[1], ctr[0], ctr[1])
    assert (int(y[0]), int(y[1])) == out


def test_threefry_matches_rocrand():
    if not os.path.exists(PIN):
        r = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "_pin/threefry_rocrand"], capture_output=True)
        if r.returncode != 0:
            pytest.skip("rocRAND pin helper not buildable here")
    rng = np.random.default_rng(11)
    v = rng.integers(0, 2 ** 32, (500, 4), dtype=np.uint64).astype(np.uint32)
    lines = "\n".join(f"{a:x} {b:x} {c:x} {d:x}" for a, b, c, d in v) + "\n"
    out = subprocess.run([PIN], input=lines, capture_output=True, text=True, check=True).stdout.split()
    got = np.array([int(x, 16) for x in out], dtype=np.uint64).reshape(-1, 2)
    y0, y1 = jr.threefry2x32(v[:, 2], v[:, 3], v[:, 0], v[:, 1])
    np.testing.assert_array_equal(got[:, 0], y0)
    np.testing.assert_array_equal(got[:, 1], y1)


# Outputs printed in JAX's documentation (jax_threefry_partitionable=False, float32).
DOC_NORMAL10 = [-0.3721109, 0.26423115, -0.18252768, -0.7368197, -0.44030377, -0.1521442, -0.67135346, -0.5908641,
                0.73168886, 0.5673026]


def test_jax_documented_outputs_legacy_layout():
    key = jr.prng_key(0)
    np.testing.assert_array_equal(key, [0, 0])
    sp = jr.split(key, 2, partitionable=False)
    np.testing.assert_array_equal(sp, [[4146024105, 967050713], [2718843009, 1272950319]])
    assert jr.normal(key, (1,), partitionable=False)[0] == f32(-0.20584226)
    assert jr.normal(sp[1], (1,), partitionable=False)[0] == f32(-1.2515389)
    np.testing.assert_array_equal(jr.normal(key, (10,), partitionable=False), np.array(DOC_NORMAL10, f32))


def test_prng_key_of_the_reference():
    np.testing.assert_array_equal(jr.prng_key(42), [0, 42])  # centroidal_nmpc_jax.py:167
    np.testing.assert_array_equal(jr.prng_key(2 ** 33 + 5), [2, 5])


def test_partitionable_layout_properties():
    key = jr.prng_key(42)
    sp = jr.split(key, 3, partitionable=True)
    for i in range(3):
        y = jr.threefry2x32(key[0], key[1], 0, i)
        np.testing.assert_array_equal(sp[i], [int(y[0]), int(y[1])])
    # element i depends on i alone: a (5, 7) draw is the first 35 elements of a (100,) draw
    a = jr.random_bits(key, 35, partitionable=True)
    b = jr.random_bits(key, 100, partitionable=True)
    np.testing.assert_array_equal(a, b[:35])
    y = jr.threefry2x32(key[0], key[1], 0, 17)
    assert int(a[17]) == int(y[0]) ^ int(y[1])


def test_legacy_layout_odd_padding():
    key = jr.prng_key(7)
    M = 9  # odd: counts 0..8 padded with one 0, halves [0..4], [5..8, 0]
    bits = jr.random_bits(key, M, partitionable=False)
    for i in range(5):
        x1 = i + 5 if i + 5 < M else 0
        y0, y1 = jr.threefry2x32(key[0], key[1], i, x1)
        assert int(bits[i]) == int(y0)
        if i + 5 < M:
            assert int(bits[i + 5]) == int(y1)


def _fma_exact(a, b, c):
    v = Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c))
    return v


def test_fma32_is_correctly_rounded():
    rng = np.random.default_rng(3)
    a = rng.standard_normal(4000).astype(f32)
    b = rng.standard_normal(4000).astype(f32)
    c = (rng.standard_normal(4000) * 4).astype(f32)
    # adversarial: products landing at float32 midpoints after adding c
    a[:500] = f32(1.0) + np.arange(500, dtype=f32) * f32(2 ** -23)
    b[:500] = f32(1.0) + f32(2 ** -23)
    c[:500] = f32(-1.0)
    r = jr.fma32(a, b, c)
    for i in range(0, 4000, 7):
        exact = _fma_exact(a[i], b[i], c[i])
        got = Fraction(float(r[i]))
        lo = Fraction(float(np.nextafter(r[i], f32(-np.inf))))
        hi = Fraction(float(np.nextafter(r[i], f32(np.inf))))
        assert abs(got - exact) <= abs(lo - exact) and abs(got - exact) <= abs(hi - exact), i
    # against the hardware fma of numpy's float64 path where no double rounding can occur (|c| tiny)
    np.testing.assert_array_equal(jr.fma32(a[1000:], b[1000:], f32(0)), (a[1000:] * b[1000:]).astype(f32))


def test_normal_distribution_and_tails():
    key = jr.prng_key(42)
    for part in (True, False):
        z = jr.normal(key, (200000,), partitionable=part)
        assert abs(float(z.mean())) < 0.01 and abs(float(z.std()) - 1.0) < 0.01
        assert np.isfinite(z).all()
    # the extreme uniform values stay finite: u = nextafter(-1, 0) gives the w >= 5 branch
    b = np.array([0, 0xFFFFFFFF, 0x80000000, 0x7FFFFFFF], np.uint32)
    z = jr.normal_from_bits(b)
    assert np.isfinite(z).all() and z[0] < -5 and z[1] > 5


def test_sampling_noise_block_structure():
    """NMPC:647-677: the two Gaussian blocks share key and shape (block 2 = 15 x block 1); the uniform block is
    a draw of its own shape from the same key; row 0 is zero.  MPPI (:811) sigma * Z; CEM (:957) Z."""
    key = jr.with_newkey(jr.prng_key(42))
    N, P = 128, 120
    t = N // 3
    for part in (True, False):
        rs = jr.sampling_noise(key, 0, N, P, partitionable=part)
        assert not rs[0].any()
        z = jr.normal(key, (t, P), partitionable=part)
        np.testing.assert_array_equal(rs[1:1 + t], (f32(0.2) * z).astype(f32))
        np.testing.assert_array_equal(rs[1 + t:1 + 2 * t], (f32(3.0) * z).astype(f32))
        np.testing.assert_array_equal(rs[1 + 2 * t:], jr.uniform(key, (N - 1 - 2 * t, P), -10.0, 10.0, part))
        assert rs[1 + 2 * t:].min() >= -10 and rs[1 + 2 * t:].max() < 10
        mp = jr.sampling_noise(key, 1, N, P, sigma_mppi=3.0, partitionable=part)
        np.testing.assert_array_equal(mp[1:], (f32(3.0) * jr.normal(key, (N - 1, P), part)).astype(f32))
        cem = jr.sampling_noise(key, 2, N, P, partitionable=part)
        np.testing.assert_array_equal(cem[1:], jr.normal(key, (N - 1, P), part))


def test_choice_matches_randint_formula():
    key = jr.prng_key(5)
    a = np.array([1.3, 1.65, 2.0], f32)
    for part in (True, False):
        k1, k2 = jr.split(key, 2, part)
        hi = jr.random_bits(k1, 50, part).astype(np.uint64)
        lo = jr.random_bits(k2, 50, part).astype(np.uint64)
        m = (2 ** 16 % 3) ** 2 % 3
        idx = ((hi % 3) * m + lo % 3) % 3
        np.testing.assert_array_equal(jr.choice(key, a, 50, part), a[idx])


def test_product_host_key_helpers_match():
    """The product's C++ key helpers (what Sampling_MPC.with_newkey calls) equal the restatement."""
    from quadruped_pympc_amd import _lib

    np.testing.assert_array_equal(_lib.jax_prng_key(42), jr.prng_key(42))
    for part in (True, False):
        k = _lib.jax_prng_key(42)
        for _ in range(20):
            for num in (2, 3, 5):
                np.testing.assert_array_equal(_lib.jax_split(k, num, part), jr.split(k, num, part))
            k = _lib.jax_split(k, 2, part)[0]
    assert _lib.pack_key(np.array([1, 2], np.uint32)) == (1 << 32) | 2 == jr.pack_key([1, 2])


def test_controller_key_schedule_is_the_reference_s():
    """Sampling_MPC (rng 'jax'): master_key = PRNGKey(42); with_newkey = split(master_key)[0] (NMPC:167, 498-501)."""
    from quadruped_pympc_amd import config as mirror
    from quadruped_pympc_amd.controllers.sampling.centroidal_nmpc_hip import Sampling_MPC

    for part in (True, False):
        mirror.mpc_params["jax_threefry_partitionable"] = part
        try:
            mpc = Sampling_MPC(mirror)
        finally:
            mirror.mpc_params.pop("jax_threefry_partitionable")
        k = jr.prng_key(42)
        np.testing.assert_array_equal(mpc.master_key, k)
        for _ in range(4):
            mpc.with_newkey()
            k = jr.with_newkey(k, part)
            np.testing.assert_array_equal(mpc.master_key, k)
        assert mpc.master_key.dtype == np.uint32


def _log1p_sample():
    """Every 61st float32 in (-1, 0] (bit patterns 0x80000000 .. 0xBF7FFFFF), its neighbours of 1 and 0, and values
    whose float64 log1p lies near a float32 rounding boundary (the Ziv fallback's territory)."""
    u = np.arange(0x80000000, 0xBF800000, 61, dtype=np.uint64).astype(np.uint32)
    t = u.view(f32)
    edge = np.array([-0.0, 0.0, -np.finfo(f32).tiny, -1.862645149230957e-09, -1.8626452e-09, -0.0078125,
                     np.nextafter(f32(-0.0078125), f32(0)), np.nextafter(f32(-0.0078125), f32(-1)),
                     np.nextafter(f32(-1), f32(0)), -0.5, -0.25, -0.75], f32)
    # boundary cases: t whose log1p(t) (float64) is within 2^-34 relative of a float32 midpoint
    rng = np.random.default_rng(5)
    c = -rng.random(4_000_000).astype(f32)
    L = np.log1p(c.astype(np.float64))
    f = L.astype(f32).astype(np.float64)
    up = np.nextafter(L.astype(f32), f32(0)).astype(np.float64)
    dn = np.nextafter(L.astype(f32), f32(-np.inf)).astype(np.float64)
    near = np.minimum(np.abs(L - 0.5 * (f + up)), np.abs(L - 0.5 * (f + dn))) < np.abs(L) * 2.0 ** -34
    return np.concatenate([t, edge, c[near]])


def test_log1p_fast_equals_float64_log1p():
    """log1p_fast (the JAX normal's erf_inv argument, srbd_jaxrng.h): a short float64 evaluation rounded to float
    unless it lies within 2^13 of its ulps (>= 2^-40 relative) of the rounding midpoint, else the float64 log1p -- the same float32 as
    float32(log1p(float64 t)) for every t in (-1, 0] sampled, with fallbacks rare (about 2^-15 of uniform draws)."""
    from quadruped_pympc_amd import _lib

    t = _log1p_sample()
    out = np.empty_like(t)
    nfb = __import__("ctypes").c_int64(0)
    assert _lib.lib.srbd_selftest_log1p(_lib.fptr(t), t.size, _lib.fptr(out), None, __import__("ctypes").byref(nfb)) == 0
    want = np.log1p(t.astype(np.float64)).astype(f32)
    bad = np.flatnonzero(out.view(np.uint32) != want.view(np.uint32))
    assert bad.size == 0, (t[bad[:5]], out[bad[:5]], want[bad[:5]])
    # the uniform part of the sample: fallbacks well under 1e-3 of it
    assert nfb.value < 1e-3 * t.size, nfb.value
