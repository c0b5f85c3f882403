"""GPU: srbd_foothold_mpc_step chained on the device (srbd_foothold_chain: the TAMOLS launch also writes the MPC
step's device input -- the reference's feet = the footholds, the swing feet of the state = the footholds,
cost_feet -- and the rollout launch is queued right behind it, one host wait) against the same call run as the
sequence of calls (SRBD_FOOTHOLD_CHAIN=0: TAMOLS waited for, prepare_state and the step's staging on the host),
bit for bit, over C4's trot contacts (swing feet, lift-offs) and seeds out of reach (infeasible legs: the seed at
its terrain height), with the lattice and the full-scan TAMOLS queries and both noise streams.

The sequential form is itself pinned to the Python chain and the chained oracles (tests/test_gpu_c4_pipeline.py).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LEGS = ("FL", "FR", "RL", "RR")


def _compare(pf, pu, of, ou):
    for i in (0, 1):
        for n in LEGS:
            np.testing.assert_array_equal(of[i][n], ou[i][n])
            assert of[i][n].dtype == ou[i][n].dtype
    assert of[2:6] == ou[2:6]
    np.testing.assert_array_equal(of[6], ou[6])
    rf, ru = pf.last_ref_state, pu.last_ref_state
    assert rf.keys() == ru.keys()
    for key in ru:
        if key.startswith("ref_foot_constraints_"):
            assert (rf[key] is None) == (ru[key] is None)
            if ru[key] is not None:
                for a, b in zip(rf[key], ru[key]):
                    np.testing.assert_array_equal(a, b)
        else:
            np.testing.assert_array_equal(rf[key], ru[key])
    for n in LEGS:
        np.testing.assert_array_equal(pf.heightmaps[n].data, pu.heightmaps[n].data)
        np.testing.assert_array_equal(pf.vfa.footholds_adaptation[n], pu.vfa.footholds_adaptation[n])
    assert (pf.vfa.last_scores is None) == (pu.vfa.last_scores is None) == (not pu.vfa.keep_scores)
    if pu.vfa.keep_scores:
        np.testing.assert_array_equal(pf.vfa.last_scores, pu.vfa.last_scores)
    np.testing.assert_array_equal(pf.controller.best_control_parameters, pu.controller.best_control_parameters)
    np.testing.assert_array_equal(pf.controller.master_key, pu.controller.master_key)
    np.testing.assert_array_equal(pf.iface.previous_contact_mpc, pu.iface.previous_contact_mpc)
    a, b = pf.controller.last_result, pu.controller.last_result
    assert (a.best_index, a.best_cost, a.status) == (b.best_index, b.best_cost, b.status)
    np.testing.assert_array_equal(np.array(a.grf[:]), np.array(b.grf[:]))
    np.testing.assert_array_equal(np.array(a.predicted_state[:]), np.array(b.predicted_state[:]))


@pytest.mark.parametrize("lattice,method,rng,qfeet", [
    ("1", "mppi", "jax", 0.0),                # C4 as the bench runs it, the drop-in's default stream
    ("1", "mppi", "philox", 0.0),
    ("0", "mppi", "philox", 0.0),             # full-scan TAMOLS queries: 16 blocks per leg, the feed in the merging block
    ("1", "random_sampling", "philox", 0.0),
    ("1", "mppi", "philox", 2.5),             # feet weights: cost_feet summed on the device by the last leg
    ("0", "mppi", "jax", 2.5),
])
def test_chain_equals_sequential(monkeypatch, lattice, method, rng, qfeet):
    """Zero feet weights (the reference's Q) with a bounded scene: each leg writes its own feet into the step input
    and the host's cost_feet (+0) stands; nonzero feet weights: the last leg to finish sums cost_feet on the device
    as fill_input does (float, in order, no contraction)."""
    from quadruped_pympc_amd import _lib
    from quadruped_pympc_amd.helpers.foothold_pipeline import TamolsMpcStep
    from quadruped_pympc_amd.helpers.legs_attr import LegsAttr
    from quadruped_pympc_amd.helpers.terrain import GpuTerrain
    from quadruped_pympc_amd.synthetic import c4_config, c4_inputs

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X")
    monkeypatch.setenv("SRBD_TAMOLS_LATTICE", lattice)
    cfgs = [c4_config(), c4_config()]
    for c in cfgs:
        c.mpc_params.update(sampling_method=method, rng=rng)
    ter = GpuTerrain.stepping_stones()
    pf, pu = TamolsMpcStep(ter, cfgs[0]), TamolsMpcStep(ter, cfgs[1])
    assert pf._fusable() and pu._fusable()
    for p in (pf, pu):
        assert p.controller._ctx is None  # the context is made at the first step, from Q
        p.controller.Q[12:24] = qfeet
    invalid = lifts = 0
    try:
        for k in range(12):
            state, seeds, hips, ref_base, cs = c4_inputs(k)
            if k % 4 == 3:
                seeds = seeds + np.array([1.5, 0.0, 0.0])  # beyond the legs' reach
            prev = np.array(pu.iface.previous_contact_mpc, dtype=float)
            lifts += int(np.sum((prev == 1) & (cs[:, 0] == 0)))
            args = (state, LegsAttr(*seeds.copy()), LegsAttr(*hips), ref_base, cs.copy(), state["linear_velocity"],
                    state["orientation"], state["angular_velocity"], np.zeros(4), 1.4)
            for p in (pf, pu):  # the scores kept on some steps (opt-in), the patches pending on access in the chain
                p.vfa.keep_scores = k % 3 != 2
            of = pf.step(*args)
            monkeypatch.setenv("SRBD_FOOTHOLD_CHAIN", "0")
            ou = pu.step(state, LegsAttr(*seeds.copy()), *args[2:])
            monkeypatch.delenv("SRBD_FOOTHOLD_CHAIN")
            _compare(pf, pu, of, ou)
            invalid += int((pf._io_np["valid"] == 0).sum())
        assert pf.controller.context.foothold_chained() == 12  # each ran the form it was meant to
        assert pu.controller.context.foothold_chained() == 0
    finally:
        pf.close()
        pu.close()
        ter.close()
    assert invalid > 0 and lifts > 0
