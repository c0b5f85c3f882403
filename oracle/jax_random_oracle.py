"""CPU restatement (numpy) of the ``jax.random`` stream the reference samples its noise from.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker.  The product path
(``quadruped_pympc_amd``, ``libsrbd_hip.so``) has its own implementation (``csrc/srbd_jaxrng.h``).

What the reference calls (paths relative to the reference repository root):

* ``jax.random.PRNGKey(42)``                       centroidal_nmpc_jax.py:167
* ``newkey, subkey = jax.random.split(master_key)`` centroidal_nmpc_jax.py:498-501 (with_newkey);
  the interface passes ``master_key`` (= newkey) to the step, srbd_controller_interface.py:126,145,164
* ``jax.random.normal(key, (n, P))``               centroidal_nmpc_jax.py:654,663 (RS), :811 (MPPI), :957 (CEM)
* ``jax.random.uniform(key, (n, P), minval=-s, maxval=s)``  centroidal_nmpc_jax.py:671-676 (RS)
* ``jax.random.choice(key, a, (N,))``              centroidal_nmpc_jax_gait_adaptive.py:692, 836-837

JAX itself is a third-party dependency that is absent from ``/root/reference`` and not
installed here; it is unpinned (``pyproject.toml:52-55``).  This module restates the published
algorithm of ``jax._src.prng`` / ``jax._src.random`` / XLA's ``ErfInv``:

* Threefry-2x32 with 20 rounds (Salmon et al., SC'11; Random123's ``threefry2x32_20``), key
  schedule ``ks = [k0, k1, k0 ^ k1 ^ 0x1BD11BDA]``, rotations (13, 15, 26, 6), (17, 29, 16, 24),
  key injection after every four rounds with the injection count added to the second word.
* ``PRNGKey(seed)`` = ``[seed >> 32, seed & 0xFFFFFFFF]`` (``threefry_seed``; [0, seed] for the
  32-bit seeds the reference uses).
* ``jax_threefry_partitionable`` (the ``partitionable`` argument below) selects the counter layout:
  - True (JAX's default since 0.5.0): element i of a draw of any shape is
    ``t0 ^ t1`` with ``(t0, t1) = threefry(key, (hi32(i), lo32(i)))`` over the row-major flat index;
    ``split(key, n)[i] = threefry(key, (0, i))``;
  - False (earlier JAX): the M counts ``0..M-1`` (padded with one 0 when M is odd) are cut into
    halves x0 = counts[:h], x1 = counts[h:], h = ceil(M / 2); ``bits = concat(y0, y1)[:M]`` with
    ``(y0, y1) = threefry(key, (x0, x1))``; ``split(key, n)`` reshapes the 2n bits to (n, 2).
* bits -> float in [0, 1): ``bitcast((b >> 9) | 0x3F800000) - 1``; ``uniform(minval, maxval)`` =
  ``max(minval, f * (maxval - minval) + minval)``.
* ``normal`` = ``sqrt(2) * erf_inv(u)`` with u = uniform(nextafter(-1, 0), 1); ``erf_inv`` is XLA's
  single-precision form (M. Giles, "Approximating the erfinv function", GPU Computing Gems 2010):
  ``w = -log1p(-u * u)``; w < 5: w - 2.5 and the first coefficient set, else sqrt(w) - 3 and the
  second; a degree-8 Horner chain; times u.
* ``choice(key, a, (N,))`` with replacement = ``a[randint(key, (N,), 0, n)]``; randint splits the key
  into (k1, k2), draws 32 bits from each and forms ``((hi % n) * m + lo % n) % n`` with
  ``m = ((2**16 % n) ** 2) % n``.

Rounding choices (unpinned against JAX itself -- JAX is absent, so no JAX output can be compared):
* the two multiply-adds (``f * range + minval`` and every Horner step) are fused (one rounding),
  as XLA's LLVM backends emit them (fp-contract fast on NVPTX and x86-64 with FMA);
* ``log1p`` is the correctly rounded float32 log1p (computed in float64 and rounded once).  XLA
  calls the platform's log1pf (CUDA libdevice ``__nv_log1pf``, <= 1 ulp), so JAX's own draws can
  differ from these in the last bit or two where that library rounds differently.

Pins (``tests/test_jax_random.py``): the Threefry core against the Random123 known-answer vectors
and against rocRAND's independent ``threefry2x32_20`` engine (``oracle/threefry_rocrand.cpp``);
everything above the core against JAX's published example outputs where they exist.
"""
from __future__ import annotations

import numpy as np

u32 = np.uint32
f32 = np.float32

_ROT = ((13, 15, 26, 6), (17, 29, 16, 24))
_PARITY = 0x1BD11BDA


def _rotl(x, r):
    return (x << u32(r)) | (x >> u32(32 - r))


def threefry2x32(k0, k1, x0, x1):
    """Threefry-2x32-20 of counter pairs (x0, x1) under key (k0, k1); uint32 arrays (broadcast)."""
    k0 = np.asarray(k0, dtype=u32)
    k1 = np.asarray(k1, dtype=u32)
    ks = (k0, k1, k0 ^ k1 ^ u32(_PARITY))
    with np.errstate(over="ignore"):
        x0 = np.asarray(x0, dtype=u32) + ks[0]
        x1 = np.asarray(x1, dtype=u32) + ks[1]
        for i in range(5):
            for r in _ROT[i % 2]:
                x0 = x0 + x1
                x1 = _rotl(x1, r)
                x1 = x1 ^ x0
            x0 = x0 + ks[(i + 1) % 3]
            x1 = x1 + ks[(i + 2) % 3] + u32(i + 1)
    return x0.astype(u32), x1.astype(u32)


def prng_key(seed: int) -> np.ndarray:
    """jax.random.PRNGKey(seed) (threefry_seed): [seed >> 32, seed & 0xFFFFFFFF]."""
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return np.array([seed >> 32, seed & 0xFFFFFFFF], dtype=u32)


def _original_pairs(M):
    """Counter halves of threefry_2x32(key, iota(M)) (the padded odd case included)."""
    h = (M + 1) // 2
    x0 = np.arange(h, dtype=np.uint64)
    x1 = x0 + h
    x1[x1 >= M] = 0  # the padding count of an odd M
    return x0.astype(u32), x1.astype(u32), h


def random_bits(key, M: int, partitionable: bool = True) -> np.ndarray:
    """jax._src.prng.threefry_random_bits(key, 32, shape) for a shape of M elements, flattened."""
    key = np.asarray(key, dtype=u32)
    if M == 0:
        return np.zeros(0, dtype=u32)
    if partitionable:
        i = np.arange(M, dtype=np.uint64)
        t0, t1 = threefry2x32(key[0], key[1], (i >> np.uint64(32)).astype(u32), (i & np.uint64(0xFFFFFFFF)).astype(u32))
        return t0 ^ t1
    x0, x1, h = _original_pairs(M)
    y0, y1 = threefry2x32(key[0], key[1], x0, x1)
    return np.concatenate([y0, y1])[:M]


def split(key, num: int = 2, partitionable: bool = True) -> np.ndarray:
    """jax.random.split(key, num) -> (num, 2) uint32."""
    key = np.asarray(key, dtype=u32)
    if partitionable:
        i = np.arange(num, dtype=np.uint64)
        t0, t1 = threefry2x32(key[0], key[1], (i >> np.uint64(32)).astype(u32), (i & np.uint64(0xFFFFFFFF)).astype(u32))
        return np.stack([t0, t1], axis=1)
    return random_bits(key, 2 * num, partitionable=False).reshape(num, 2)


def with_newkey(key, partitionable: bool = True) -> np.ndarray:
    """Sampling_MPC.with_newkey (centroidal_nmpc_jax.py:498-501): master_key <- split(master_key)[0]."""
    return split(key, 2, partitionable)[0]


def fma32(a, b, c):
    """Correctly rounded float32 a * b + c (one rounding), vectorised.

    a * b is exact in float64; t = a*b + c in float64 with its exact error e (TwoSum).  Rounding t to
    float32 gives the right answer unless t is exactly halfway between two float32 values, where the
    sign of e decides (t and the exact value lie on the same side of every other float32 midpoint,
    since the midpoints are float64 numbers).
    """
    a = np.asarray(a, dtype=f32).astype(np.float64)
    b = np.asarray(b, dtype=f32).astype(np.float64)
    c = np.asarray(c, dtype=f32).astype(np.float64)
    s = a * b
    t = s + c
    bp = t - s
    e = (s - (t - bp)) + (c - bp)
    r = t.astype(f32)
    rd = r.astype(np.float64)
    lo = np.where(rd > t, np.nextafter(r, f32(-np.inf)), r)
    hi = np.where(rd < t, np.nextafter(r, f32(np.inf)), r)
    mid = (lo.astype(np.float64) + hi.astype(np.float64)) * 0.5
    tie = (lo != hi) & (t == mid) & (e != 0)
    return np.where(tie, np.where(e > 0, hi, lo), r).astype(f32)


def bits_to_unit(bits) -> np.ndarray:
    """float32 in [0, 1): bitcast((bits >> 9) | 0x3F800000) - 1 (jax._src.random._uniform)."""
    b = (np.asarray(bits, dtype=u32) >> u32(9)) | u32(0x3F800000)
    return (b.view(f32) - f32(1.0)).astype(f32)


def uniform_from_bits(bits, minval, maxval) -> np.ndarray:
    """_uniform's map of 32 random bits to [minval, maxval)."""
    lo, hi = f32(minval), f32(maxval)
    return np.maximum(lo, fma32(bits_to_unit(bits), f32(hi - lo), lo)).astype(f32)


_ERFINV_LT5 = (2.81022636e-08, 3.43273939e-07, -3.5233877e-06, -4.39150654e-06, 0.00021858087,
               -0.00125372503, -0.00417768164, 0.246640727, 1.50140941)
_ERFINV_GE5 = (-0.000200214257, 0.000100950558, 0.00134934322, -0.00367342844, 0.00573950773,
               -0.0076224613, 0.00943887047, 1.00167406, 2.83297682)


def log1p32(x) -> np.ndarray:
    """Correctly rounded float32 log1p (float64 log1p, one rounding)."""
    return np.log1p(np.asarray(x, dtype=f32).astype(np.float64)).astype(f32)


def erf_inv32(x) -> np.ndarray:
    """XLA's float32 ErfInv (Giles' single-precision approximation)."""
    x = np.asarray(x, dtype=f32)
    w = -log1p32(x * (-x))
    lt = w < f32(5.0)
    with np.errstate(invalid="ignore"):
        w = np.where(lt, w - f32(2.5), np.sqrt(w).astype(f32) - f32(3.0)).astype(f32)
    p = np.where(lt, f32(_ERFINV_LT5[0]), f32(_ERFINV_GE5[0])).astype(f32)
    for a, b in zip(_ERFINV_LT5[1:], _ERFINV_GE5[1:]):
        p = fma32(p, w, np.where(lt, f32(a), f32(b)))
    r = (p * x).astype(f32)
    return np.where(np.abs(x) == f32(1.0), x * f32(np.inf), r).astype(f32)


NORMAL_LO = np.nextafter(f32(-1.0), f32(0.0))  # -0.99999994


def normal_from_bits(bits) -> np.ndarray:
    """_normal_real: sqrt(2) * erf_inv(uniform(nextafter(-1, 0), 1))."""
    u = uniform_from_bits(bits, NORMAL_LO, f32(1.0))
    return (f32(np.sqrt(2)) * erf_inv32(u)).astype(f32)


def normal(key, shape, partitionable: bool = True) -> np.ndarray:
    """jax.random.normal(key, shape) (float32)."""
    M = int(np.prod(shape))
    return normal_from_bits(random_bits(key, M, partitionable)).reshape(shape)


def uniform(key, shape, minval=0.0, maxval=1.0, partitionable: bool = True) -> np.ndarray:
    """jax.random.uniform(key, shape, minval=, maxval=) (float32)."""
    M = int(np.prod(shape))
    return uniform_from_bits(random_bits(key, M, partitionable), minval, maxval).reshape(shape)


def randint(key, M: int, minval: int, maxval: int, partitionable: bool = True) -> np.ndarray:
    """jax.random.randint(key, (M,), minval, maxval) for int32 (jax._src.random._randint)."""
    k1, k2 = split(key, 2, partitionable)
    hi = random_bits(k1, M, partitionable).astype(np.uint64)
    lo = random_bits(k2, M, partitionable).astype(np.uint64)
    span = maxval - minval
    span = 1 if span <= 0 else span
    mult = (2 ** 16) % span
    mult = (mult * mult) % span
    off = ((hi % span) * mult + (lo % span)) & 0xFFFFFFFF  # uint32 arithmetic
    off = off % span
    return (minval + off).astype(np.int32)


def choice(key, a, M: int, partitionable: bool = True) -> np.ndarray:
    """jax.random.choice(key, a, shape=(M,)) with replacement and uniform p."""
    a = np.asarray(a)
    return a[randint(key, M, 0, a.shape[0], partitionable)]


def sampling_noise(key, method: int, N: int, P: int, sigma_mppi=3.0, sigma_rs=(0.2, 3.0, 10.0),
                   partitionable: bool = True) -> np.ndarray:
    """additional_random_parameters (N, P) exactly as the reference's samplers draw them.

    method 0 random sampling (centroidal_nmpc_jax.py:647-677), 1 MPPI (:806-812), 2 CEM (:951-958).
    CEM returns the unscaled standard normals Z (the reference forms Z * sigma; callers multiply).
    Row 0 is zero (the warm start).
    """
    out = np.zeros((N, P), dtype=f32)
    if method == 1:
        out[1:] = (f32(sigma_mppi) * normal(key, (N - 1, P), partitionable)).astype(f32)
    elif method == 2:
        out[1:] = normal(key, (N - 1, P), partitionable)
    else:
        t = int(N / 3)
        z = normal(key, (t, P), partitionable)  # the same key and shape for both Gaussian blocks
        out[1:1 + t] = (f32(sigma_rs[0]) * z).astype(f32)
        out[1 + t:1 + 2 * t] = (f32(sigma_rs[1]) * z).astype(f32)
        s = float(sigma_rs[2])
        out[1 + 2 * t:N] = uniform(key, (N - 1 - 2 * t, P), -s, s, partitionable)
    return out


def pack_key(key) -> int:
    """The 64-bit `seed` argument of srbd_step in the JAX stream mode: key[0] << 32 | key[1]."""
    key = np.asarray(key, dtype=u32)
    return (int(key[0]) << 32) | int(key[1])
