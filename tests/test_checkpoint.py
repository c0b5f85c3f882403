"""Checkpoint / restore: the controller's evolving state as plain arrays (CPU, no device),
and exact replays of device-resident chains through srbd_get_state / srbd_set_state (GPU)."""
import io

import numpy as np
import pytest

from quadruped_pympc_amd import config as mirror
from tests.helpers import make_case, product_cfg

f32 = np.float32


def _controller(method, rng=None):
    from quadruped_pympc_amd.controllers.sampling.centroidal_nmpc_hip import Sampling_MPC

    mirror.mpc_params["sampling_method"] = method
    if rng is not None:
        mirror.mpc_params["rng"] = rng
    try:
        return Sampling_MPC(mirror)
    finally:
        mirror.mpc_params["sampling_method"] = "mppi"
        mirror.mpc_params.pop("rng", None)


def test_set_state_rejects_other_stream_key():
    """A checkpoint's master_key must fit the controller's stream: uint64 (seed, counter) for Philox, a uint32 JAX
    key otherwise -- never silently cast (a Philox counter is not a JAX key)."""
    jx, ph = _controller("mppi", "jax"), _controller("mppi", "philox")
    with pytest.raises(ValueError):
        jx.set_state(ph.get_state())
    with pytest.raises(ValueError):
        ph.set_state(jx.get_state())
    jx.set_state(jx.get_state())
    ph.set_state(ph.get_state())


def test_set_state_warns_when_device_part_dropped():
    """A fresh controller cannot take a checkpoint's device-resident part: it says so (RuntimeWarning)."""
    mpc = _controller("mppi")
    st = mpc.get_state()
    st["device_best"] = np.zeros(mpc.num_control_parameters, f32)
    st["device_key"] = np.array([42, 3], np.uint64)
    with pytest.warns(RuntimeWarning, match="device-resident part"):
        mpc.set_state(st)
    assert mpc.master_key[1] == st["master_key"][1]


@pytest.mark.parametrize("stream", ["jax", "philox"])
@pytest.mark.parametrize("method", ["random_sampling", "mppi", "cem_mppi"])
def test_controller_state_round_trip_without_device(method, stream):
    """get_state -> np.savez -> np.load (no pickle) -> set_state restores every evolving attribute."""
    mpc = _controller(method, stream)
    rng = np.random.default_rng(3)
    mpc.best_control_parameters = rng.standard_normal(mpc.num_control_parameters).astype(f32)
    mpc.with_newkey().with_newkey()
    if method == "cem_mppi":
        mpc.sigma_cem_mppi = rng.uniform(0.2, 5.0, mpc.num_control_parameters).astype(f32)
    st = mpc.get_state()
    assert "device_best" not in st  # no context yet: nothing on a device
    buf = io.BytesIO()
    np.savez(buf, **st)
    buf.seek(0)
    loaded = dict(np.load(buf, allow_pickle=False))

    other = _controller(method, stream)
    other.set_state(loaded)
    np.testing.assert_array_equal(other.best_control_parameters, mpc.best_control_parameters)
    np.testing.assert_array_equal(other.master_key, mpc.master_key)
    assert other.master_key.dtype == mpc.master_key.dtype
    if stream == "philox":
        assert other.master_key[1] == 2
    else:  # two with_newkey calls from PRNGKey(42)
        from oracle import jax_random_oracle as jr

        np.testing.assert_array_equal(other.master_key, jr.with_newkey(jr.with_newkey(jr.prng_key(42))))
    if method == "cem_mppi":
        np.testing.assert_array_equal(other.sigma_cem_mppi, mpc.sigma_cem_mppi)


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["mppi", "cem_mppi", "random_sampling"])
def test_device_chain_replays_from_checkpoint(method):
    """A device-resident chain restarted from a checkpoint ends in the same state bit for bit."""
    from quadruped_pympc_amd import _lib

    case = make_case("c2", N=3000, method=method, seed=5)
    ctx = _lib.Context(product_cfg(case))
    try:
        ctx.step(case["state"], case["ref"], case["contact"], case["best"], sigma=case["sigma"], seed=11, counter=4)
        s0 = ctx.get_state()
        np.testing.assert_array_equal(s0[0], case["best"])  # a host step leaves its inputs as the state
        assert s0[2:] == (11, 4)
        ctx.bench_device_steps(7)
        s1 = ctx.get_state()
        assert s1[3] == 4 + 7  # one counter per device step
        assert not np.array_equal(s1[0], s0[0])
        ctx.bench_device_steps(3)  # move on, then restore
        ctx.set_state(*s0)
        np.testing.assert_array_equal(ctx.get_state()[0], s0[0])
        ctx.bench_device_steps(7)
        s1b = ctx.get_state()
        np.testing.assert_array_equal(s1b[0], s1[0])
        if method == "cem_mppi":
            np.testing.assert_array_equal(s1b[1], s1[1])
        assert s1b[2:] == s1[2:]
    finally:
        ctx.close()


@pytest.mark.gpu
def test_controller_replays_host_steps_from_checkpoint():
    """Sampling_MPC: the same compute calls after set_state(get_state()) give identical outputs."""
    mpc = _controller("mppi")
    case = make_case("c2", N=mpc.num_parallel_computations, method="mppi", seed=9)
    P = mpc.num_control_parameters
    state, ref, contact = case["state"], case["ref"], case["contact"][:, :mpc.horizon]
    try:
        mpc.best_control_parameters = np.zeros(P, f32)
        mpc.compute_control(state, ref, contact, mpc.best_control_parameters, mpc.master_key)
        st = mpc.get_state()

        def run(k):
            outs = []
            for _ in range(k):
                r = mpc.compute_control(state, ref, contact, mpc.best_control_parameters, mpc.master_key)
                mpc.best_control_parameters = r[3]
                mpc.with_newkey()
                outs.append((np.array(r[0]), np.array(r[2]), np.array(r[3])))
            return outs

        a = run(3)
        mpc.set_state(st)
        b = run(3)
        for x, y in zip(a, b):
            for u, v in zip(x, y):
                np.testing.assert_array_equal(u, v)
    finally:
        mpc.close()
