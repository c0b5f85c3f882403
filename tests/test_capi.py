"""CPU tests of the C-ABI boundary (include/srbd_mpc.h): exports, argument checks, host merge.

No compute kernel runs here (no GPU in this container).  The host-side record builder and
merger (srbd_make_record_host / srbd_finish_host) are product code shared with the sharded
path, so they are checked against the oracle's reduction (centroidal_nmpc_jax.py:686-692,
:820-842, :966-988, :1075-1081) on oracle costs.
"""
import ctypes as C
import glob
import os
import re
import subprocess

import numpy as np
import pytest

from quadruped_pympc_amd import _lib
from quadruped_pympc_amd.synthetic import CONFIGS, inputs

from oracle.srbd_oracle import SamplingMPCOracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = sorted(glob.glob(os.path.join(ROOT, "include", "*.h")))
f32 = np.float32


def header_functions():
    """Every function every include/*.h declares."""
    names = set()
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(srbd_\w+)\s*\(", text, flags=re.M))
    return sorted(names)


def test_header_symbols_exported():
    names = header_functions()
    assert len(names) >= 25, names
    dyn = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\sT\s(\w+)$", dyn.stdout, flags=re.M))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    for n in names:
        assert hasattr(_lib.lib, n)


def test_bindings_cover_header():
    assert set(header_functions()) == set(_lib.SIGNATURES)


def test_struct_layouts_match_header():
    # srbd_config: 10 int32 + 5 f32 + 9 + 32 + 24 + 1 + 3 floats
    assert C.sizeof(_lib.SrbdConfig) == 4 * (10 + 5 + 9 + _lib.MAX_HORIZON + 24 + 1 + 3)
    assert C.sizeof(_lib.SrbdResult) == 4 * (12 + 24 + 1 + 3)
    assert C.sizeof(_lib.TamolsParams) == 8 * 21


def test_abi_version_and_num_params():
    assert _lib.lib.srbd_abi_version() == 1
    for par, H, S, P in [("zero_order", 12, 2, 144), ("linear_spline", 12, 2, 36), ("cubic_spline", 16, 2, 96),
                         ("zero_order", 10, 2, 120), ("linear_spline", 12, 4, 60), ("cubic_spline", 16, 3, 144)]:
        cfg = _lib.make_config(num_samples=100, horizon=H, method="mppi", parametrization=par, num_splines=S,
                               mass=15.0, inertia=np.eye(3), dts=np.full(H, 0.02))
        assert _lib.num_params(cfg) == P


@pytest.mark.parametrize("field,value", [("horizon", 0), ("horizon", 33), ("num_samples", 0), ("method", 7),
                                         ("parametrization", 9), ("num_elite", 1)])
def test_invalid_configs_rejected(field, value):
    cfg = _lib.make_config(num_samples=100, horizon=12, method="cem_mppi", parametrization="zero_order", mass=15.0,
                           inertia=np.eye(3), dts=np.full(12, 0.02))
    setattr(cfg, field, value)
    h = C.c_void_p()
    rc = _lib.lib.srbd_create(C.byref(cfg), C.byref(h))
    assert rc == _lib.E_INVALID
    assert _lib.last_error(None)


def test_null_arguments_rejected():
    assert _lib.lib.srbd_create(None, None) == _lib.E_INVALID
    assert _lib.lib.srbd_step(None, None, None, None, 0, None, None, None, 0, 0, None, None) == _lib.E_INVALID
    assert _lib.lib.srbd_record_floats(None) == _lib.E_INVALID
    _lib.lib.srbd_destroy(None)


def test_no_device_fails_loudly():
    """No CPU fallback: without a HIP device, context creation fails with SRBD_E_NODEVICE."""
    if _lib.device_count() > 0:
        pytest.skip("a HIP device is visible")
    cfg = _lib.make_config(num_samples=100, horizon=12, method="mppi", parametrization="zero_order", mass=15.0,
                           inertia=np.eye(3), dts=np.full(12, 0.02))
    with pytest.raises(RuntimeError, match="srbd_create"):
        _lib.Context(cfg)
    h = C.c_void_p()
    assert _lib.lib.srbd_create(C.byref(cfg), C.byref(h)) == _lib.E_NODEVICE


def test_division_host_path_correctly_rounded():
    """The rollout's reciprocal-based division (Markstein) equals IEEE a/b, incl. the b == 3 path."""
    rng = np.random.default_rng(0)
    a = np.concatenate([rng.standard_normal(200000) * 10 ** rng.uniform(-6, 6, 200000),
                        np.arange(-5000, 5000) * 0.37]).astype(f32)
    b = np.concatenate([rng.uniform(0.5, 4.5, 100000), np.full(110000, 3.0)]).astype(f32)
    out = np.empty_like(a)
    rc = _lib.lib.srbd_selftest_div(_lib.fptr(a), _lib.fptr(b), a.size, _lib.fptr(out), None)
    assert rc == 0
    np.testing.assert_array_equal(out, a / b)


# ------------------------------------------------------------------------ host merge


def oracle_case(method, N, seed, key="c2", par="zero_order", H=12):
    w = CONFIGS[key]
    o = SamplingMPCOracle(mass=w.mass, inertia=w.inertia, horizon=H, num_samples=N, method=method,
                          parametrization=par)
    s, r, c = inputs(w, 2)
    rng = np.random.default_rng(seed)
    t = N // 3
    sigma = rng.uniform(0.3, 3, o.P).astype(f32)
    noise = o.assemble_noise(rng.standard_normal((N - 1, o.P)).astype(f32), sigma=sigma,
                             U=rng.uniform(-10, 10, (N - 1 - 2 * t, o.P)).astype(f32))
    best = (rng.standard_normal(o.P) * 2).astype(f32)
    s, r, c = s.astype(f32), r.astype(f32), c[:, :H].astype(f32)
    costs = o.saturate(o.rollout_costs(s, r, best[None] + noise, c))
    cfg = _lib.make_config(num_samples=N, horizon=H, method=method, parametrization=par, mass=w.mass,
                           inertia=w.inertia, dts=np.full(H, 0.02))
    return o, cfg, s, c, best, sigma, noise, costs


def _host_merge(cfg, world, costs, noise, s, c, best, sigma=None):
    recs = []
    for rank in range(world):
        a, n = _lib.shard_rows(cfg.num_samples, rank, world)
        recs.append(_lib.make_record_host(cfg, rank, world, costs[a:a + n], noise[a:a + n]))
    return _lib.finish_host(cfg, np.concatenate(recs), s, c, best, sigma)


@pytest.mark.parametrize("method", ["mppi", "cem_mppi", "random_sampling"])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_host_records_merge_matches_oracle(method, world):
    N = 997
    o, cfg, s, c, best, sigma, noise, costs = oracle_case(method, N, seed=world)
    ref = o.reduce(s, c, best, noise, costs)
    nb, ns, res = _host_merge(cfg, world, costs, noise, s, c, best, sigma if method == "cem_mppi" else None)
    assert res.best_index == ref["best_index"]
    assert f32(res.best_cost) == ref["best_cost"]
    np.testing.assert_allclose(nb, ref["best"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(np.array(res.grf), ref["grf"], rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(np.array(res.predicted_state), ref["pred"], rtol=1e-5, atol=1e-5)
    if method == "cem_mppi":
        np.testing.assert_allclose(ns, ref["sigma"], rtol=1e-5, atol=1e-6)


def test_host_merge_ties_pick_first_row():
    """nanargmin semantics across shards: equal costs -> lowest global row wins."""
    N, world = 300, 3
    o, cfg, s, c, best, sigma, noise, costs = oracle_case("mppi", N, seed=7)
    costs = np.full(N, 5.0, f32)
    costs[[13, 141, 299]] = 1.0  # one per shard
    _, _, res = _host_merge(cfg, world, costs, noise, s, c, best)
    assert res.best_index == 13


@pytest.mark.parametrize("method", ["mppi", "cem_mppi", "random_sampling"])
def test_host_merge_is_world_invariant(method):
    """The fixed reduction tree: every world size merges to the same bits (up to 8 ranks; N spans 3 levels)."""
    N = 70001
    o, cfg, s, c, best, sigma, noise, costs = oracle_case(method, N, seed=11)
    sg = sigma if method == "cem_mppi" else None
    b1, s1, r1 = _host_merge(cfg, 1, costs, noise, s, c, best, sg)
    for world in (2, 3, 5, 8):
        bw, sw, rw = _host_merge(cfg, world, costs, noise, s, c, best, sg)
        np.testing.assert_array_equal(bw, b1)
        if sg is not None:
            np.testing.assert_array_equal(sw, s1)
        np.testing.assert_array_equal(np.array(rw.grf), np.array(r1.grf))
        assert rw.best_index == r1.best_index and rw.best_cost == r1.best_cost


def test_host_merge_saturated_costs():
    N = 300
    o, cfg, s, c, best, sigma, noise, costs = oracle_case("mppi", N, seed=8)
    costs[:] = f32(1e6)
    costs[200] = f32(1e6)
    ref = o.reduce(s, c, best, noise, costs)
    rec = _lib.make_record_host(cfg, 0, 1, costs, noise)
    nb, _, res = _lib.finish_host(cfg, rec, s, c, best)
    assert res.best_index == ref["best_index"] == 0
    np.testing.assert_allclose(nb, ref["best"], rtol=1e-5, atol=1e-5)
