"""GPU: the reference's jax.random noise stream on the device (srbd_set_rng SRBD_RNG_JAX / _LEGACY) against its
numpy restatement (oracle/jax_random_oracle.py, pinned in tests/test_jax_random.py).

  * draws: bit-exact at C1 (random sampling, N = 128, the shared-key Gaussian blocks and the uniform block),
    C2 (MPPI, N = 10 000) and C3 (CEM, N = 65 536; unscaled standard normals), both counter layouts, and for a
    shard (rows of rank 1 of 3 are the global rows: draws are indexed by global row);
  * a step on the device draws equals the same step with the restatement's draws injected, bit for bit
    (costs, parameters, GRFs, prediction);
  * key schedule: host steps keyed by master_key, split(master_key)[0], ... (with_newkey) hit the draws the
    previous launch made ahead (the next key computed on the device) and equal fresh injected-noise steps;
    device-resident chains advance the key on the device;
  * gait-adaptive: the step frequencies are jax.random.choice(key, set, (N,)) (GA:692, 836);
  * end to end at C2: Sampling_MPC (rng 'jax') driven through the interface's call sequence matches the
    numpy oracle fed the restatement's draws for the same keys (SURVEY 8(c) tolerances: costs rtol 2e-5 /
    atol 1e-3, GRFs rtol 1e-4 / atol 5e-3 N).
Reference: centroidal_nmpc_jax.py:167, 498-501, 647-677, 806-836, 951-958.
"""
import numpy as np
import pytest

from helpers import f32, make_case, product_cfg
from oracle import jax_random_oracle as jr

pytestmark = pytest.mark.gpu

METHOD = {"random_sampling": 0, "mppi": 1, "cem_mppi": 2}
LAYOUTS = [("jax", True), ("jax_legacy", False)]


@pytest.fixture(scope="module")
def lib():
    from quadruped_pympc_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X")
    return _lib


def first_key():
    return jr.with_newkey(jr.prng_key(42))  # the key of the interface's first call (SCI:126)


def expected_noise(case, key, part):
    w, o = case["w"], case["orc"]
    return jr.sampling_noise(key, METHOD[w.method], w.num_samples, o.P, sigma_mppi=3.0,
                             sigma_rs=(0.2, 3.0, 10.0), partitionable=part)


@pytest.mark.parametrize("kind,part", LAYOUTS)
@pytest.mark.parametrize("wkey,N,method,par,H", [
    ("c1", 128, "random_sampling", "zero_order", 10),
    ("c1", 301, "random_sampling", "linear_spline", 12),
    ("c2", 10000, "mppi", "zero_order", 12),
    ("c3", 65536, "cem_mppi", "cubic_spline", 16),
])
def test_device_draws_equal_restatement(lib, kind, part, wkey, N, method, par, H):
    case = make_case(wkey, N=N, method=method, par=par, H=H)
    ctx = lib.Context(product_cfg(case))
    try:
        ctx.set_rng(kind)
        key = first_key()
        got = ctx.draw_noise(jr.pack_key(key), 0)
    finally:
        ctx.close()
    np.testing.assert_array_equal(got, expected_noise(case, key, part))


@pytest.mark.parametrize("kind,part", LAYOUTS)
def test_shard_draws_are_global_rows(lib, kind, part):
    case = make_case("c2", N=3001, method="mppi")
    key = jr.prng_key(9)
    want = expected_noise(case, key, part)
    for rank in range(3):
        ctx = lib.Context(product_cfg(case, rank=rank, world_size=3))
        try:
            ctx.set_rng(kind)
            got = ctx.draw_noise(jr.pack_key(key), 5)
            np.testing.assert_array_equal(got, want[ctx.row0:ctx.row0 + ctx.n_local])
        finally:
            ctx.close()


def _step(lib, case, kind, key, noise=None, counter=1, best=None):
    ctx = lib.Context(product_cfg(case))
    try:
        ctx.set_rng(kind)
        b, s, res, costs = ctx.step(case["state"], case["ref"], case["contact"], case["best"] if best is None else best,
                                    sigma=case["sigma"], noise=noise, seed=jr.pack_key(key), counter=counter,
                                    want_costs=True)
        return b, s, res, costs
    finally:
        ctx.close()


def _same(a, b):
    np.testing.assert_array_equal(a[0], b[0])
    if a[1] is not None:
        np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(np.array(a[2].grf), np.array(b[2].grf))
    np.testing.assert_array_equal(np.array(a[2].predicted_state), np.array(b[2].predicted_state))
    assert a[2].best_index == b[2].best_index
    np.testing.assert_array_equal(a[3], b[3])


@pytest.mark.parametrize("kind,part", LAYOUTS)
@pytest.mark.parametrize("wkey,N,method,par,H", [
    ("c1", 128, "random_sampling", "zero_order", 10),
    ("c2", 10000, "mppi", "zero_order", 12),
    ("c2", 65536, "mppi", "zero_order", 12),
    ("c3", 20000, "cem_mppi", "cubic_spline", 16),
])
def test_step_on_device_draws_equals_injected(lib, kind, part, wkey, N, method, par, H):
    case = make_case(wkey, N=N, method=method, par=par, H=H, seed=3)
    key = first_key()
    noise = expected_noise(case, key, part)
    if method == "cem_mppi":  # the reference forms Z * sigma (NMPC:957); injected noise is stored as given
        noise = (noise * case["sigma"][None, :]).astype(f32)
    _same(_step(lib, case, kind, key), _step(lib, case, kind, key, noise=noise))


@pytest.mark.parametrize("kind,part", LAYOUTS)
@pytest.mark.parametrize("N", [10000, 65536, 131072])
def test_key_schedule_host_steps(lib, kind, part, N):
    """Host steps keyed by with_newkey's chain: the draws made ahead in each launch (next key computed on the
    device) serve the following call; every step equals a fresh injected-noise step."""
    case = make_case("c2", N=N, method="mppi", seed=4)
    key = first_key()
    ctx = lib.Context(product_cfg(case))
    try:
        ctx.set_rng(kind)
        best = case["best"]
        keys = []
        outs = []
        for i in range(4):
            keys.append(key)
            b, _, res, costs = ctx.step(case["state"], case["ref"], case["contact"], best, seed=jr.pack_key(key),
                                        counter=i + 1, want_costs=True)
            outs.append((b, None, res, costs))
            best = b
            key = jr.with_newkey(key, part)
    finally:
        ctx.close()
    best = case["best"]
    for i in range(4):
        ref = _step(lib, case, kind, keys[i], noise=expected_noise(case, keys[i], part), best=best)
        _same(outs[i], ref)
        best = ref[0]


@pytest.mark.parametrize("kind,part", LAYOUTS)
def test_device_chain_advances_the_key(lib, kind, part):
    case = make_case("c2", N=10000, method="mppi", seed=6)
    key = first_key()
    ctx = lib.Context(product_cfg(case))
    try:
        ctx.set_rng(kind)
        ctx.step(case["state"], case["ref"], case["contact"], case["best"], seed=jr.pack_key(key), counter=4)
        ctx.bench_device_steps(3)
        best, _, seed, ctr = ctx.get_state()
    finally:
        ctx.close()
    want_key = key
    b = case["best"]
    for i in range(3):  # chain step i replays the host step's input with key split^i
        b = _step(lib, case, kind, want_key, noise=expected_noise(case, want_key, part), best=b)[0]
        want_key = jr.with_newkey(want_key, part)
    assert seed == jr.pack_key(want_key) and ctr == 4 + 3
    np.testing.assert_allclose(best, b, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("kind,part", LAYOUTS)
@pytest.mark.parametrize("method", ["mppi", "random_sampling"])
def test_gait_adaptive_choice(lib, kind, part, method):
    from oracle.srbd_ga_oracle import GA_DUTY, freq_set

    case = make_case("c2", N=1500, method=method, seed=8)
    fs = np.asarray(freq_set(1 if method == "mppi" else 0, (1.4, 2.0, 2.4), 1.65, 1), f32)
    key = first_key()
    freqs = jr.choice(key, fs, 1500, part).astype(f32)
    noise = expected_noise(case, key, part)
    outs = []
    for inject in (False, True):
        ctx = lib.Context(product_cfg(case))
        try:
            ctx.set_rng(kind)
            ctx.set_gait((0.1, 0.6, 0.6, 0.1), 0.02, GA_DUTY, fs, freqs if inject else None)
            b, _, res, costs = ctx.step(case["state"], case["ref"], case["contact"], case["best"],
                                        noise=noise if inject else None, seed=jr.pack_key(key), counter=2,
                                        want_costs=True)
            outs.append((b, None, res, costs))
        finally:
            ctx.close()
    _same(outs[0], outs[1])
    assert outs[0][2].best_freq == freqs[outs[0][2].best_index]


@pytest.mark.parametrize("part", [True, False])
def test_end_to_end_c2_interface_on_jax_stream(lib, part):
    """Sampling_MPC (rng 'jax') through SRBDControllerInterface's call sequence for 3 MPC calls vs the numpy
    oracle fed jax.random draws of the same keys."""
    from quadruped_pympc_amd import config as mirror
    from quadruped_pympc_amd.controllers.sampling.centroidal_nmpc_hip import Sampling_MPC

    from test_gpu_parity import COST_ATOL, COST_RTOL

    case = make_case("c2", N=10000, method="mppi", seed=10)
    o = case["orc"]
    saved, robot = dict(mirror.mpc_params), mirror.robot
    mirror.set_robot(case["w"].robot)  # the case's robot (mass / inertia / grf_max), Go2
    mirror.mpc_params.update(num_parallel_computations=10000, sampling_method="mppi",
                             control_parametrization="zero_order", horizon=12, jax_threefry_partitionable=part)
    try:
        mpc = Sampling_MPC(mirror)
    finally:
        mirror.set_robot(robot)
        mirror.mpc_params.clear()
        mirror.mpc_params.update(saved)
    try:
        best_ref = np.zeros(o.P, f32)
        mpc.best_control_parameters = best_ref.copy()
        key = jr.prng_key(42)
        for it in range(3):
            mpc.with_newkey()
            key = jr.with_newkey(key, part)
            np.testing.assert_array_equal(mpc.master_key, key)
            r = mpc.jitted_compute_control(case["state"], case["ref"], case["contact"], mpc.best_control_parameters,
                                           mpc.master_key, None, 1.4, 0)
            mpc.best_control_parameters = r[3]
            ref = o.compute_control(case["state"], case["ref"], case["contact"], best_ref,
                                    jr.sampling_noise(key, 1, 10000, o.P, partitionable=part))
            np.testing.assert_allclose(np.asarray(r[6]), ref["costs"], rtol=COST_RTOL, atol=COST_ATOL)
            np.testing.assert_allclose(r[0], ref["grf"], rtol=1e-4, atol=5e-3)
            np.testing.assert_allclose(r[3], ref["best"], rtol=1e-4, atol=1e-3)
            best_ref = ref["best"]
    finally:
        mpc.close()


def test_log1p_fast_device_equals_host(lib):
    """The device log1p_fast (float64 polynomial + table, Ziv's test, OCML's float64 log1p as the fallback) gives the
    host's float32 for every sampled t in (-1, 0] (tests/test_jax_random.py pins the host against float64 log1p)."""
    import ctypes

    from test_jax_random import _log1p_sample

    t = _log1p_sample()
    host, dev = np.empty_like(t), np.empty_like(t)
    nfb = ctypes.c_int64(0)
    assert lib.lib.srbd_selftest_log1p(lib.fptr(t), t.size, lib.fptr(host), lib.fptr(dev), ctypes.byref(nfb)) == 0
    np.testing.assert_array_equal(dev.view(np.uint32), host.view(np.uint32))
