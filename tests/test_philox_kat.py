"""Pins the oracle's Philox4x32-10 + Box-Muller noise stream (CPU).

The reference draws with jax.random (threefry) -- a different generator, so sample-level
parity with it is impossible by construction; what is pinned instead:
  * Philox4x32-10 against the Random123 known-answer vectors (kat_vectors, philox4x32_10)
    and against rocRAND's host-callable engine (oracle/_pin/philox_rocrand),
  * the distribution and block structure the reference's samplers produce
    (centroidal_nmpc_jax.py:647-677 random sampling, :806-812 MPPI, :951-958 CEM).
The GPU generator is checked against this oracle bit for bit in tests/test_gpu_parity.py.
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import c_oracle as co
from quadruped_pympc_amd.config import ROBOTS

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PIN = os.path.join(ROOT, "oracle", "_pin", "philox_rocrand")

# Random123 kat_vectors, "philox4x32 10" lines: (ctr, key) -> out
R123 = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,out", R123)
def test_philox_random123_kat(ctr, key, out):
    assert tuple(co.philox(ctr, key)) == out


def test_philox_matches_rocrand():
    if not os.path.exists(PIN):
        r = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "_pin/philox_rocrand"], capture_output=True)
        if r.returncode != 0:
            pytest.skip("rocRAND pin helper not buildable here")
    rng = np.random.default_rng(5)
    for _ in range(20):
        c = [int(x) for x in rng.integers(0, 2 ** 32, 4)]
        k = [int(x) for x in rng.integers(0, 2 ** 32, 2)]
        out = subprocess.run([PIN] + [f"{x:x}" for x in c + k], capture_output=True, text=True, check=True).stdout
        assert [int(x, 16) for x in out.split()] == co.philox(c, k)


def cfg(method, N=3001, H=12):
    m, I = ROBOTS["go2"]
    return co.make_cfg(N=N, H=H, method=method, param_kind=0, mass=m, inertia=I)


def test_mppi_noise_distribution():
    c = cfg(1)
    z = co.gen_noise(c, 42, 7)
    assert np.all(z[0] == 0)
    body = z[1:].ravel() / np.float32(3.0)
    assert abs(body.mean()) < 0.01 and abs(body.std() - 1) < 0.01
    # tails of a standard normal
    assert 0.0440 < np.mean(np.abs(body) > 2) < 0.0470


def test_cem_noise_scales_per_parameter():
    c = cfg(2)
    sigma = np.linspace(0.2, 5, 144).astype(np.float32)
    z = co.gen_noise(c, 1, 0, sigma)
    z1 = co.gen_noise(c, 1, 0, np.ones(144, np.float32))
    np.testing.assert_array_equal(z, (z1 * sigma).astype(np.float32))


def test_random_sampling_blocks():
    N = 3001
    c = cfg(0, N)
    z = co.gen_noise(c, 3, 11)
    t = N // 3
    np.testing.assert_allclose(z[1 + t:1 + 2 * t], z[1:1 + t] * np.float32(3.0 / 0.2), rtol=1e-6)
    u = z[1 + 2 * t:]
    assert u.min() >= -10 and u.max() <= 10
    assert abs(u.mean()) < 0.1 and abs(u.std() - 20 / np.sqrt(12)) < 0.05


def test_counter_and_seed_select_independent_streams():
    c = cfg(1, 200)
    a = co.gen_noise(c, 42, 0)
    np.testing.assert_array_equal(a, co.gen_noise(c, 42, 0))
    b = co.gen_noise(c, 42, 1)
    d = co.gen_noise(c, 43, 0)
    assert np.mean(a[1:] == b[1:]) < 1e-3 and np.mean(a[1:] == d[1:]) < 1e-3
    assert abs(np.corrcoef(a[1:].ravel(), b[1:].ravel())[0, 1]) < 0.02
