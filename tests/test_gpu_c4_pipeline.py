"""C4 as one pipeline (BASELINE configs[3]: Go2 on stepping_stones_medium, TAMOLS foothold search + MPPI N = 10 000):
the heightmap raycast and TAMOLS (one launch), the adapted footholds into ref_state, prepare_state_and_reference
(swing feet replaced by their reference footholds, the warm start of lifted legs zeroed) and the MPPI step -- as
wb_interface.py:230-291 and srbd_controller_interface.py:113-180 chain them (helpers/foothold_pipeline.py) --
against the chained oracles: terrain_oracle -> tamols_oracle -> srbd_oracle.prepare_state_and_reference ->
SamplingMPCOracle on the same injected noise.

Tolerances: footholds atol 1e-12 and the same feasible legs (tests/test_gpu_tamols.py); state / reference arrays
bit for bit; the MPPI step as tests/test_gpu_parity.py's end-to-end bar (costs rtol 2e-5 atol 1e-3, GRFs rtol 1e-4
atol 5e-3 N, a near tie accepted only when the oracle's reduction of the GPU's own costs reproduces the GPU).
"""
import numpy as np
import pytest

from helpers import f32
from oracle import srbd_oracle as so
from oracle import terrain_oracle as T
from oracle.tamols_oracle import TamolsOracle
from test_gpu_parity import check_end_to_end

pytestmark = pytest.mark.gpu

LEGS = ("FL", "FR", "RL", "RR")


def oracle_footholds(cfg, state, seeds, hips, yaw, contact):
    """terrain_oracle's patches around the seeds, then tamols_oracle, then VFA's fallback for infeasible legs."""
    from quadruped_pympc_amd.helpers.terrain import stepping_stones_scene

    sc = stepping_stones_scene()
    hms = T.patches(sc["prims"], seeds, [yaw] * 4, 13, 7, 0.04, 0.04, 10.0, has_ground=sc["has_ground"],
                    ground_z=sc["ground_z"])
    orc = TamolsOracle(dict(cfg.simulation_params["tamols_params"]), cfg.robot)
    feet = np.stack([state["foot_" + n] for n in LEGS])
    fh, boxes, valid, _ = orc.compute(hms, seeds, hips, state["linear_velocity"], state["position"],
                                      np.asarray(contact, np.int32), feet)
    out = fh.copy()
    for i in range(4):
        if not valid[i]:  # VFA:223-228 through the patch's nearest-point lookup (+ 0.02)
            pts = hms[i].reshape(-1, 3)
            d = (pts[:, 0] - seeds[i, 0]) ** 2 + (pts[:, 1] - seeds[i, 1]) ** 2
            out[i] = seeds[i]
            out[i, 2] = pts[int(np.argmin(d)), 2] + 0.02
    return out, valid, hms


@pytest.fixture(scope="module")
def pipe():
    from quadruped_pympc_amd import _lib
    from quadruped_pympc_amd.helpers.foothold_pipeline import TamolsMpcStep
    from quadruped_pympc_amd.helpers.terrain import GpuTerrain

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible")
    from quadruped_pympc_amd.synthetic import CONFIGS, c4_config

    cfg, w = c4_config(), CONFIGS["c4"]
    ter = GpuTerrain.stepping_stones()
    p = TamolsMpcStep(ter, cfg)
    yield p, cfg, w
    p.close()
    ter.close()


def test_c4_pipeline_against_chained_oracles(pipe):
    from quadruped_pympc_amd.helpers.legs_attr import LegsAttr
    from quadruped_pympc_amd.synthetic import c4_inputs

    p, cfg, w = pipe
    state, seeds, hips, ref_base, cs = c4_inputs(0)
    yaw = state["orientation"][2]
    contact = cs[:, 0]
    prev = p.iface.previous_contact_mpc.copy()
    best_in = p.controller.best_control_parameters.copy()
    out = p.step(state, LegsAttr(*seeds), LegsAttr(*hips), ref_base, cs, state["linear_velocity"],
                 state["orientation"], state["angular_velocity"], np.zeros(4), 1.4)
    # 1. footholds: raycast + TAMOLS against terrain_oracle -> tamols_oracle
    fh_o, valid_o, hms_o = oracle_footholds(cfg, state, seeds, hips, yaw, contact)
    np.testing.assert_array_equal(np.stack([p.heightmaps[n].data[:, :, 0, :] for n in LEGS]), hms_o)
    got = np.stack([p.last_ref_state["ref_foot_" + n][0] for n in LEGS])
    np.testing.assert_allclose(got, fh_o, rtol=0, atol=1e-12)
    assert [p.last_constraints[n] is not None for n in LEGS] == list(valid_o)
    assert valid_o.any()
    np.testing.assert_array_equal(np.stack([out[1][n] for n in LEGS]), got)  # nmpc_footholds = the ref footholds
    assert np.isfinite(np.concatenate([out[0][n] for n in LEGS] + [out[6]])).all()
    # 2. prepare_state_and_reference against the oracle (bit for bit), from the same inputs
    PL = p.controller.num_control_parameters_single_leg
    s_o, r_o, b_o = so.prepare_state_and_reference(state, p.last_ref_state, contact, prev, best_in, PL)
    p.controller.best_control_parameters = best_in.copy()
    s_p, r_p = p.controller.prepare_state_and_reference(state, p.last_ref_state, contact, prev)
    np.testing.assert_array_equal(np.asarray(s_p, np.float64), s_o)
    np.testing.assert_array_equal(np.asarray(r_p, np.float64), r_o)
    np.testing.assert_array_equal(p.controller.best_control_parameters, b_o)
    # 3. the MPPI step on those arrays with injected noise against the oracle
    orc = so.SamplingMPCOracle(mass=w.mass, inertia=w.inertia, horizon=w.horizon, num_samples=w.num_samples,
                               method=w.method, parametrization=w.parametrization)
    rng = np.random.default_rng(44)
    noise = orc.assemble_noise(rng.standard_normal((w.num_samples - 1, orc.P)).astype(f32))
    grf, _, pred, best, _, _, costs = p.controller.compute_control_mppi(
        s_p, r_p, cs.astype(f32), p.controller.best_control_parameters, p.controller.master_key, noise=noise)
    g = dict(grf=np.asarray(grf, f32), pred=np.asarray(pred, f32), best=np.asarray(best, f32),
             costs=np.asarray(costs, f32), best_index=p.controller.last_result.best_index)
    case = dict(orc=orc, state=s_o.astype(f32), ref=r_o.astype(f32), contact=cs.astype(f32), best=b_o, noise=noise)
    check_end_to_end(case, g)


def test_c4_pipeline_steps(pipe):
    """Ten successive pipeline steps (device draws, the controller's key schedule): finite outputs, the adapted
    footholds are the controller's reference feet every step, and every step's footholds equal the oracle's."""
    from quadruped_pympc_amd.helpers.legs_attr import LegsAttr
    from quadruped_pympc_amd.synthetic import c4_inputs

    p, cfg, _ = pipe
    for k in range(10):
        state, seeds, hips, ref_base, cs = c4_inputs(k)
        out = p.step(state, LegsAttr(*seeds), LegsAttr(*hips), ref_base, cs, state["linear_velocity"],
                     state["orientation"], state["angular_velocity"], np.zeros(4), 1.4)
        got = np.stack([p.last_ref_state["ref_foot_" + n][0] for n in LEGS])
        fh_o, _, _ = oracle_footholds(cfg, state, seeds, hips, state["orientation"][2], cs[:, 0])
        np.testing.assert_allclose(got, fh_o, rtol=0, atol=1e-12)
        np.testing.assert_array_equal(np.stack([out[1][n] for n in LEGS]), got)
        assert np.isfinite(np.concatenate([out[0][n] for n in LEGS] + [out[6]])).all()


def test_c4_fused_step_equals_python_chain():
    """srbd_foothold_mpc_step (TamolsMpcStep's one-call path) against the same pipeline run through the Python
    chain (fused off), step by step from the same start: every returned array, the ref_state, the constraints, the
    heightmap patches, the scores, the warm start, the key and the step result bit for bit -- over trot contacts
    (swing feet, lift-offs) and seeds out of reach (infeasible legs: the seed at its terrain height)."""
    from quadruped_pympc_amd import _lib
    from quadruped_pympc_amd.helpers.foothold_pipeline import TamolsMpcStep
    from quadruped_pympc_amd.helpers.legs_attr import LegsAttr
    from quadruped_pympc_amd.helpers.terrain import GpuTerrain
    from quadruped_pympc_amd.synthetic import c4_config, c4_inputs

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible")
    ter = GpuTerrain.stepping_stones()
    pf, pu = TamolsMpcStep(ter, c4_config()), TamolsMpcStep(ter, c4_config())
    pu.fused = False
    assert pf._fusable() and not pu._fusable()
    invalid_seen = 0
    try:
        for k in range(12):
            state, seeds, hips, ref_base, cs = c4_inputs(k)
            if k % 4 == 3:
                seeds = seeds + np.array([1.5, 0.0, 0.0])  # beyond the legs' reach
            outs = []
            for p in (pf, pu):
                p.vfa.keep_scores = k % 3 != 2  # the scores are opt-in (VisualFootholdAdaptation.keep_scores)
                outs.append(p.step(state, LegsAttr(*seeds.copy()), LegsAttr(*hips), ref_base, cs.copy(),
                                   state["linear_velocity"], state["orientation"], state["angular_velocity"],
                                   np.zeros(4), 1.4))
            of, ou = outs
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
                    assert np.asarray(rf[key]).shape == np.asarray(ru[key]).shape
            for n in LEGS:
                np.testing.assert_array_equal(pf.heightmaps[n].data, pu.heightmaps[n].data)
                np.testing.assert_array_equal(pf.vfa.footholds_adaptation[n], pu.vfa.footholds_adaptation[n])
            assert (pf.vfa.last_scores is None) == (pu.vfa.last_scores is None) == (k % 3 == 2)
            if k % 3 != 2:
                np.testing.assert_array_equal(pf.vfa.last_scores, pu.vfa.last_scores)
            np.testing.assert_array_equal(pf.controller.best_control_parameters, pu.controller.best_control_parameters)
            np.testing.assert_array_equal(pf.controller.master_key, pu.controller.master_key)
            np.testing.assert_array_equal(pf.iface.previous_contact_mpc, pu.iface.previous_contact_mpc)
            a, b = pf.controller.last_result, pu.controller.last_result
            assert (a.best_index, a.best_cost, a.status) == (b.best_index, b.best_cost, b.status)
            invalid_seen += int((pf._io_np["valid"] == 0).sum())  # infeasible legs keep their old constraints
            assert pf.controller.context.step_id == pu.controller.context.step_id
    finally:
        pf.close()
        pu.close()
        ter.close()
    assert invalid_seen > 0


def test_c4_fused_step_error_leaves_the_chain_state():
    """A TAMOLS failure inside srbd_foothold_mpc_step (patches of 20 x 20 points: more than the 320 candidates a call
    takes) raises as the Python chain does and leaves the objects as the chain leaves them: the key not advanced, the
    warm start and previous contact untouched, the patches pending around the seeds, VFA not initialised."""
    from quadruped_pympc_amd import _lib
    from quadruped_pympc_amd.helpers.foothold_pipeline import TamolsMpcStep
    from quadruped_pympc_amd.helpers.legs_attr import LegsAttr
    from quadruped_pympc_amd.helpers.terrain import GpuTerrain
    from quadruped_pympc_amd.synthetic import c4_config, c4_inputs

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible")
    ter = GpuTerrain.stepping_stones()
    pf, pu = TamolsMpcStep(ter, c4_config(), 20, 20), TamolsMpcStep(ter, c4_config(), 20, 20)
    pu.fused = False
    try:
        state, seeds, hips, ref_base, cs = c4_inputs(0)
        for p in (pf, pu):
            key, best = np.array(p.controller.master_key), p.controller.best_control_parameters.copy()
            with pytest.raises(RuntimeError, match="patch must have"):
                p.step(state, LegsAttr(*seeds.copy()), LegsAttr(*hips), ref_base, cs, state["linear_velocity"],
                       state["orientation"], state["angular_velocity"], np.zeros(4), 1.4)
            np.testing.assert_array_equal(p.controller.master_key, key)
            np.testing.assert_array_equal(p.controller.best_control_parameters, best)
            np.testing.assert_array_equal(p.iface.previous_contact_mpc, [1, 1, 1, 1])
            assert not p.vfa.initialized
            for i, n in enumerate(LEGS):
                np.testing.assert_array_equal(p.heightmaps[n].pending[0], seeds[i])
                assert p.heightmaps[n].pending[1] == float(state["orientation"][2])
        assert pf.controller._calls == pu.controller._calls
    finally:
        pf.close()
        pu.close()
        ter.close()
