"""GPU: the thread-form epilogue's regenerated draws (srbd_device.h leaf_wsum_lanes, REGEN_QUADS).

Zero-order MPPI on the device Philox stream regenerates part of its draws in the epilogue instead of re-reading
them.  A step with device draws must equal, bit for bit, the same step fed those draws as injected noise (read
back with srbd_draw_noise), which takes the read path for every column.
"""
import numpy as np
import pytest

from helpers import f32, make_case, product_cfg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from quadruped_pympc_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X")
    return _lib


@pytest.mark.parametrize("wkey,N,H", [("c2", 262144, 12), ("c5", 524288, 12), ("c2", 100003, 10)])
def test_regenerated_draws_equal_read_draws(lib, wkey, N, H):
    case = make_case(wkey, N=N, method="mppi", par="zero_order", H=H, seed=N % 71)
    seed, counter = 1234, 5
    cx = lib.Context(product_cfg(case))
    try:
        drawn = cx.draw_noise(seed, counter)
        assert not np.any(drawn[0])  # row 0: the warm start
        b_dev, _, r_dev, c_dev = cx.step(case["state"], case["ref"], case["contact"], case["best"], seed=seed,
                                         counter=counter, want_costs=True)
    finally:
        cx.close()
    cx = lib.Context(product_cfg(case))
    try:
        b_inj, _, r_inj, c_inj = cx.step(case["state"], case["ref"], case["contact"], case["best"],
                                         noise=np.ascontiguousarray(drawn), want_costs=True)
    finally:
        cx.close()
    np.testing.assert_array_equal(c_dev, c_inj)
    assert r_dev.best_index == r_inj.best_index
    np.testing.assert_array_equal(b_dev, b_inj)
    np.testing.assert_array_equal(np.array(r_dev.grf, f32), np.array(r_inj.grf, f32))
    np.testing.assert_array_equal(np.array(r_dev.predicted_state, f32), np.array(r_inj.predicted_state, f32))


@pytest.mark.parametrize("wkey,N,rg", [("c5", 524288, None), ("c2", 300001, None), ("c5", 524288, "0"),
                                       ("c5", 524288, "36"),
                                       # the four-lane form (rollout_quad_kernel GEN): the north-star shape and a
                                       # ragged last block; its draws stay in registers and the LDS stage
                                       ("c2", 65536, None), ("c2", 40001, None)])
def test_in_launch_draws_equal_rng_launch(lib, monkeypatch, wkey, N, rg):
    """Host steps whose rollout launch makes the step's draws itself (gen_now: thread form, zero-order H 12, MPPI,
    device Philox; the horizon stores the quads the epilogue reads back) against the same steps with the RNG launch
    writing them first (SRBD_GEN=0; the rollout reads them, the epilogue regenerates REGEN_QUADS of them), and the
    opt-in four-lane form (SRBD_GEN_QUAD_MIN; each lane makes its leg's three quads every fourth step; no noise
    stored): bit for
    bit over three warm-started steps, costs included.  rg: SRBD_GEN_RG, the quads the epilogue regenerates
    (default GEN_REGEN_QUADS; 0: every quad stored and read back; 36: none stored).  N = 300 001: padding rows
    past n_local in the last block (zeros in the buffer, zeros generated)."""
    case = make_case(wkey, N=N, method="mppi", par="zero_order", H=12, seed=N % 83)
    if N <= 65536:  # the four-lane GEN form is opt-in
        monkeypatch.setenv("SRBD_GEN_QUAD_MIN", "1")
    monkeypatch.setenv("SRBD_GEN", "0")
    ref = lib.Context(product_cfg(case))
    monkeypatch.delenv("SRBD_GEN")
    if rg is not None:
        monkeypatch.setenv("SRBD_GEN_RG", rg)
    gen = lib.Context(product_cfg(case))
    monkeypatch.delenv("SRBD_GEN_RG", raising=False)
    monkeypatch.delenv("SRBD_GEN_QUAD_MIN", raising=False)
    try:
        bg, br = case["best"].copy(), case["best"].copy()
        for k in range(3):
            a = gen.step(case["state"], case["ref"], case["contact"], bg, seed=77, counter=k, want_costs=True)
            b = ref.step(case["state"], case["ref"], case["contact"], br, seed=77, counter=k, want_costs=True)
            np.testing.assert_array_equal(a[3], b[3])
            assert a[2].best_index == b[2].best_index
            np.testing.assert_array_equal(a[0], b[0])
            np.testing.assert_array_equal(np.array(a[2].grf, f32), np.array(b[2].grf, f32))
            np.testing.assert_array_equal(np.array(a[2].predicted_state, f32), np.array(b[2].predicted_state, f32))
            bg, br = a[0], b[0]
        assert gen.time_launch(3, 2)[1] & 32 and not ref.time_launch(3, 2)[1] & 32  # the forms the steps ran
    finally:
        gen.close()
        ref.close()
