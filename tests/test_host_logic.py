"""CPU tests of the host-side mirror of the reference interface (no GPU compute).

Covers the Python contract of SURVEY 8(b): Sampling_MPC construction, attributes, key/sigma
plumbing, prepare_state_and_reference, shift_solution, the interface wrapper; the contact
producer (PeriodicGaitGenerator vs the scalar oracle restatement); LegsAttr; config; the TAMOLS
parameter packing and the TAMOLS oracle's known answers.  Compute calls must fail loudly here
(no HIP device, no CPU fallback).
"""
import copy
import ctypes as C
import types

import numpy as np
import pytest

from oracle.pgg_oracle import PGGOracle
from oracle.srbd_oracle import SamplingMPCOracle, prepare_state_and_reference
from oracle.tamols_oracle import FastHeightMap, TamolsOracle, synthetic_patch
from quadruped_pympc_amd import _lib
from quadruped_pympc_amd import config as base_config
from quadruped_pympc_amd.controllers.sampling.centroidal_nmpc_hip import Sampling_MPC
from quadruped_pympc_amd.helpers.legs_attr import LegsAttr
from quadruped_pympc_amd.helpers.periodic_gait_generator import PeriodicGaitGenerator
from quadruped_pympc_amd.helpers.terrain import TERRAINS
from quadruped_pympc_amd.helpers.visual_foothold_adaptation import tamols_params_struct

f32 = np.float32


def cfg_module(**mp):
    c = types.SimpleNamespace(**{k: copy.deepcopy(getattr(base_config, k)) for k in dir(base_config)
                                 if not k.startswith("__") and not callable(getattr(base_config, k))
                                 and not isinstance(getattr(base_config, k), types.ModuleType)})
    c.mpc_params.update(mp)
    return c


# ---------------------------------------------------------------- periodic gait generator (a16)
@pytest.mark.parametrize("gait", range(8))
@pytest.mark.parametrize("dts,lengths,H", [([0.02], [12], 12), ([0.01, 0.02], [2, 12], 12), ([0.02], [16], 16)])
def test_pgg_matches_scalar_oracle(gait, dts, lengths, H):
    duty, freq = 0.65, 1.4
    a = PeriodicGaitGenerator(duty, freq, gait, H)
    b = PGGOracle(duty, freq, gait, H)
    for k in range(300):
        np.testing.assert_array_equal(a.compute_contact_sequence(dts, lengths), b.compute_contact_sequence(dts, lengths))
        for _ in range(5):
            np.testing.assert_array_equal(a.run(0.002, freq), b.run(0.002, freq))
        np.testing.assert_allclose(a.phase_signal, b.phase, rtol=0, atol=0)


def test_pgg_init_hold():
    a = PeriodicGaitGenerator(0.6, 2.0, 0, 12)
    b = PGGOracle(0.6, 2.0, 0, 12)
    a.set_phase_signal(np.array([0.1, 0.2, 0.9, 0.4]), init=[True, False, True, True])
    b.phase, b.init = [0.1, 0.2, 0.9, 0.4], [True, False, True, True]
    for _ in range(100):
        np.testing.assert_array_equal(a.run(0.01, 2.0), b.run(0.01, 2.0))


def test_pgg_full_stance_sequence():
    a = PeriodicGaitGenerator(0.65, 1.4, 0, 12)
    a.set_full_stance()
    seq = a.compute_contact_sequence([0.02], [12])
    assert seq.shape == (4, 24) and np.all(seq == 1)
    a.restore_previous_gait()
    assert a.gait_type == 0


def test_pgg_c_abi_argument_checks():
    import ctypes as C
    g = _lib.SrbdPgg()
    assert _lib.lib.srbd_pgg_init(C.byref(g), 0, 0.65, 1.4, 0) == _lib.E_INVALID  # horizon < 1
    assert _lib.lib.srbd_pgg_init(C.byref(g), 0, 0.65, 1.4, 12) == _lib.OK
    out = np.zeros(4 * 12)
    dts, lens = np.array([0.02]), np.array([5], np.int32)  # the reference would run past its dts list
    assert _lib.lib.srbd_pgg_contact_sequence(C.byref(g), _lib.dptr(dts), _lib.iptr(lens), 1, _lib.dptr(out),
                                              out.size) == _lib.E_INVALID
    assert list(g.phase_signal) == [0.5, 1.0, 1.0, 0.5]  # state restored after the failure
    lens[0] = 12
    assert _lib.lib.srbd_pgg_contact_sequence(C.byref(g), _lib.dptr(dts), _lib.iptr(lens), 1, _lib.dptr(out),
                                              out.size - 1) == _lib.E_INVALID  # capacity
    assert _lib.lib.srbd_pgg_contact_sequence(C.byref(g), _lib.dptr(dts), _lib.iptr(lens), 1, _lib.dptr(out),
                                              out.size) == 12
    z = np.zeros(24)
    assert _lib.lib.srbd_prepare_state(None, _lib.dptr(z), None, None, 36, None, _lib.dptr(z),
                                       _lib.dptr(z)) == _lib.E_INVALID


# ---------------------------------------------------------------- LegsAttr / config
def test_legs_attr():
    la = LegsAttr(FL=1, FR=2, RL=3, RR=4)
    assert la["FR"] == 2 and la[2] == 3 and list(la) == [1, 2, 3, 4]
    la["RR"] = 9
    assert la.RR == 9 and la.to_list(("RR", "FL")) == [9, 1]


def test_config_set_robot():
    old = base_config.robot
    try:
        base_config.set_robot("aliengo")
        assert base_config.mass == base_config.ROBOTS["aliengo"][0]
        assert base_config.mpc_params["grf_max"] == base_config.mass * 9.81
        assert base_config.simulation_params["tamols_params"]["h_des"] == base_config.HIP_HEIGHTS["aliengo"]
        with pytest.raises(ValueError):
            base_config.set_robot("nope")
    finally:
        base_config.set_robot(old)


# ---------------------------------------------------------------- Sampling_MPC contract (8(b))
@pytest.mark.parametrize("method,par,P", [("mppi", "zero_order", 144), ("cem_mppi", "cubic_spline", 96),
                                          ("random_sampling", "linear_spline", 36)])
def test_sampling_mpc_attributes(method, par, P):
    m = Sampling_MPC(cfg_module(sampling_method=method, control_parametrization=par))
    assert m.num_control_parameters == P
    assert m.best_control_parameters.shape == (P,) and m.best_control_parameters.dtype == f32
    assert m.sampling_method == method and m.num_sampling_iterations == 1
    assert m.jitted_compute_control == m.compute_control
    if method == "cem_mppi":
        assert m.sigma_cem_mppi.shape == (P,) and np.all(m.sigma_cem_mppi == 3)
    assert m._ctx is None  # no device work at construction
    k0 = m.master_key.copy()
    np.testing.assert_array_equal(k0, [0, 42])  # jax.random.PRNGKey(42) (NMPC:167), the default 'jax' stream
    assert m.with_newkey() is m
    np.testing.assert_array_equal(m.master_key, _lib.jax_split(k0, 2)[0])  # NMPC:498-501
    assert m.with_newsigma(np.full(P, 2.0)) is m and np.all(m.get_sigma() == 2.0)
    cfg = m._srbd_config()
    assert _lib.num_params(cfg) == P
    assert cfg.mg == f32(m.mass * 9.81)


def test_sampling_mpc_rejects_cpu_device():
    with pytest.raises(RuntimeError, match="GPU only"):
        Sampling_MPC(cfg_module(device="cpu"))


def test_sampling_mpc_unknown_method_exits():
    with pytest.raises(SystemExit):
        Sampling_MPC(cfg_module(sampling_method="nope"))


def test_compute_without_device_fails_loudly():
    if _lib.device_count() > 0:
        pytest.skip("a HIP device is visible")
    m = Sampling_MPC(cfg_module(sampling_method="mppi", control_parametrization="zero_order"))
    z = np.zeros(24)
    with pytest.raises(RuntimeError, match="srbd_create"):
        m.jitted_compute_control(z, z, np.ones((4, 12)), m.best_control_parameters, m.master_key, None, 1.4, 0)


def dicts(rng):
    sc = {k: rng.standard_normal(3) for k in ("position", "linear_velocity", "orientation", "angular_velocity",
                                              "foot_FL", "foot_FR", "foot_RL", "foot_RR")}
    rs = {k: rng.standard_normal(3) for k in ("ref_position", "ref_linear_velocity", "ref_orientation",
                                              "ref_angular_velocity")}
    for n in ("FL", "FR", "RL", "RR"):
        rs["ref_foot_" + n] = rng.standard_normal((1, 3))
    return sc, rs


@pytest.mark.parametrize("cur,prev", [([1, 1, 1, 1], [1, 1, 1, 1]), ([0, 1, 1, 0], [1, 1, 1, 1]),
                                      ([0, 0, 0, 0], [1, 0, 1, 0]), ([1, 0, 0, 1], [0, 1, 1, 0])])
def test_prepare_state_and_reference_matches_oracle(cur, prev):
    rng = np.random.default_rng(sum(cur) * 7 + sum(prev))
    m = Sampling_MPC(cfg_module(sampling_method="mppi", control_parametrization="zero_order"))
    m.best_control_parameters = rng.standard_normal(m.num_control_parameters).astype(f32)
    sc, rs = dicts(rng)
    s_ref, r_ref, b_ref = prepare_state_and_reference(sc, rs, np.array(cur), np.array(prev),
                                                      m.best_control_parameters, m.num_control_parameters_single_leg)
    s, r = m.prepare_state_and_reference(sc, rs, np.array(cur), np.array(prev))
    np.testing.assert_array_equal(s, s_ref)
    np.testing.assert_array_equal(r, r_ref)
    np.testing.assert_array_equal(m.best_control_parameters, b_ref)


def test_prepare_state_staging_shapes_and_copies():
    """prepare_state_and_reference stages into persistent buffers: contacts as lists or (4, 1) columns, the warm start
    as (1, P) give the oracle's arrays; the returned arrays are copies (a second call does not change the first
    call's), and a size mismatch raises as np.reshape does.  float32 state arrays: the reference's array is float32
    (NMPC:575-596 concatenates without a dtype, so the swing feet it substitutes are rounded to float32); here it is
    float64 with the feet exact -- the same float32 values once srbd_step stages the state (checked below)."""
    rng = np.random.default_rng(5)
    m = Sampling_MPC(cfg_module(sampling_method="mppi", control_parametrization="zero_order"))
    PL = m.num_control_parameters_single_leg
    outs = []
    for k, (cur, prev) in enumerate([([0, 1, 1, 0], [1, 1, 1, 1]), ([1, 0, 0, 1], [0, 1, 1, 0])]):
        best = rng.standard_normal(m.num_control_parameters).astype(f32)
        sc, rs = dicts(rng)
        if k == 1:
            sc = {n: v.astype(f32) for n, v in sc.items()}
        s_ref, r_ref, b_ref = prepare_state_and_reference(sc, rs, np.array(cur), np.array(prev), best.copy(), PL)
        m.best_control_parameters = best.reshape(1, -1) if k == 0 else best
        c_in = list(cur) if k == 0 else np.array(cur, np.float64).reshape(4, 1)
        s, r = m.prepare_state_and_reference(sc, rs, c_in, prev)
        if k == 1:
            assert s_ref.dtype == f32 and s.dtype == np.float64
            np.testing.assert_array_equal(s.astype(f32), s_ref)
            s_ref = s_ref.astype(np.float64)
            s_ref[12:] = np.where(np.repeat(np.array(cur) == 0, 3), np.concatenate(
                [rs["ref_foot_" + n].reshape(3) for n in ("FL", "FR", "RL", "RR")]), s_ref[12:])
        np.testing.assert_array_equal(s, s_ref)
        np.testing.assert_array_equal(r, r_ref)
        np.testing.assert_array_equal(m.best_control_parameters, b_ref)
        outs.append((s, s.copy(), r, r.copy()))
    for s, s0, r, r0 in outs:
        np.testing.assert_array_equal(s, s0)
        np.testing.assert_array_equal(r, r0)
    with pytest.raises(ValueError):
        m.prepare_state_and_reference(sc, rs, [1, 1, 1], [1, 1, 1, 1])


@pytest.mark.parametrize("dtype", [np.float64, np.int64, np.float32, bool])
def test_grf_contact_masking_matches_per_leg_products(dtype):
    """compute_control's GRF masking as one (4, 3) x (4, 1) product: the dtype and values of the reference's four
    array x scalar products (SCI:175-178) for every contact dtype."""
    g = (np.arange(12, dtype=np.float32) - 5.5) * np.float32(1.37)
    cc = np.array([1, 0, 1, 1]).astype(dtype)
    per_leg = [g[0:3] * cc[0], g[3:6] * cc[1], g[6:9] * cc[2], g[9:12] * cc[3]]
    one = g.reshape(4, 3) * cc[:, None]
    for a, b in zip(per_leg, one):
        np.testing.assert_array_equal(a, b)
        assert a.dtype == b.dtype


@pytest.mark.parametrize("par,H", [("zero_order", 12), ("linear_spline", 12), ("cubic_spline", 16)])
def test_spline_host_matches_oracle(par, H):
    m = Sampling_MPC(cfg_module(sampling_method="mppi", control_parametrization=par, horizon=H))
    o = SamplingMPCOracle(mass=m.mass, inertia=m.inertia, horizon=H, num_samples=1, parametrization=par)
    rng = np.random.default_rng(1)
    p = rng.standard_normal(m.num_control_parameters_single_leg).astype(f32)
    for step in [0, 0.0, 0.01, 1, 3, 7.5, H - 1]:
        if par == "zero_order" and step != int(step):
            continue
        a = m.spline_host(p, step, H)
        b = o.spline(p[None], step, H)
        np.testing.assert_array_equal(np.array(a, f32), np.array([v[0] for v in b], f32))


def test_shift_solution_updates_first_entries_only():
    m = Sampling_MPC(cfg_module(sampling_method="mppi", control_parametrization="cubic_spline", horizon=16))
    rng = np.random.default_rng(2)
    best = rng.standard_normal(m.num_control_parameters).astype(f32)
    out = m.shift_solution(best, 0.01)
    PL = m.num_control_parameters_single_leg
    for leg in range(4):
        blk, ob = best[leg * PL:(leg + 1) * PL], out[leg * PL:(leg + 1) * PL]
        np.testing.assert_array_equal(np.delete(ob, [0, 2, 4]), np.delete(blk, [0, 2, 4]))
        np.testing.assert_array_equal(ob[[0, 2, 4]], np.array(m.spline_host(blk, 0.01, 16), f32))


def test_interface_rejects_out_of_scope_types():
    from quadruped_pympc_amd.interfaces.srbd_controller_interface import SRBDControllerInterface

    with pytest.raises(NotImplementedError):
        SRBDControllerInterface(cfg_module(type="nominal"))
    itf = SRBDControllerInterface(cfg_module(sampling_method="mppi", control_parametrization="zero_order"))
    assert isinstance(itf.controller, Sampling_MPC)


def test_interface_selects_gait_adaptive_controller():
    """optimize_step_freq selects the gait-adaptive Sampling_MPC (srbd_controller_interface.py:77-81);
    its CEM branch (broken in the reference) refuses before touching a device."""
    from quadruped_pympc_amd.controllers.sampling import centroidal_nmpc_hip_gait_adaptive as ga
    from quadruped_pympc_amd.interfaces.srbd_controller_interface import SRBDControllerInterface

    itf = SRBDControllerInterface(cfg_module(optimize_step_freq=True, sampling_method="mppi"))
    assert isinstance(itf.controller, ga.Sampling_MPC)
    np.testing.assert_array_equal(itf.controller._freq_set(1.65, 0), np.array([1.4, 2.0, 2.4], f32))
    rs = ga.Sampling_MPC(cfg_module(optimize_step_freq=True, sampling_method="random_sampling"))
    np.testing.assert_array_equal(rs._freq_set(1.65, 1), np.array([1.4, 2.0, 2.4], f32))
    np.testing.assert_array_equal(rs._freq_set(1.65, 0), np.full(3, f32(1.65)))
    cem = ga.Sampling_MPC(cfg_module(optimize_step_freq=True, sampling_method="cem_mppi"))
    with pytest.raises(NotImplementedError, match="App. B #2"):
        cem.jitted_compute_control(np.zeros(24), np.zeros(24), np.ones((4, 12)), cem.best_control_parameters,
                                   cem.master_key, 3.0)


def test_interface_masks_grfs_and_reassigns_params():
    """The interface's call sequence (srbd_controller_interface.py:118-180) over a fake controller."""
    from quadruped_pympc_amd.interfaces.srbd_controller_interface import SRBDControllerInterface

    itf = SRBDControllerInterface(cfg_module(sampling_method="mppi", control_parametrization="zero_order",
                                             num_sampling_iterations=3))
    calls = []

    def fake(state, ref, contact, best, key, *rest):
        calls.append((np.array(key), best.copy()))
        return np.arange(12, dtype=f32) + 1, np.zeros(12), np.zeros(24, f32), best + 1, f32(0), 1.4, None

    itf.controller.jitted_compute_control = fake
    rng = np.random.default_rng(3)
    sc, rs = dicts(rng)
    contact = np.ones((4, 12))
    contact[1, 0] = 0
    grfs, fh, _, _, _, freq, pred = itf.compute_control(sc, rs, contact, None, None, 1.4, 0)
    assert len(calls) == 3
    # with_newkey before each iteration: master_key <- split(master_key)[0] from PRNGKey(42) (NMPC:498-501)
    k = _lib.jax_prng_key(42)
    for key, _ in calls:
        k = _lib.jax_split(k, 2)[0]
        np.testing.assert_array_equal(key, k)
    np.testing.assert_array_equal(calls[2][1], calls[0][1] + 2)  # best reassigned between iterations
    np.testing.assert_array_equal(grfs.FR, np.zeros(3))
    np.testing.assert_array_equal(grfs.FL, [1, 2, 3])
    np.testing.assert_array_equal(fh.FL, rs["ref_foot_FL"][0])
    assert freq == 1.4


# ---------------------------------------------------------------- TAMOLS (a15) host side
def test_tamols_params_struct_packs_config():
    p = tamols_params_struct(base_config.simulation_params["tamols_params"], "aliengo")
    tp = base_config.simulation_params["tamols_params"]
    assert (p.w_edge, p.w_rough, p.w_dev, p.w_nominal, p.w_tracking, p.w_stability) == (
        tp["weight_edge_avoidance"], tp["weight_roughness"], tp["weight_deviation"], tp["weight_nominal_kinematic"],
        tp["weight_reference_tracking"], tp["weight_stability"])
    assert (p.l_min, p.l_max) == (0.1, 0.55)
    np.testing.assert_allclose(list(p.alphas), np.linspace(0.2, 0.8, 5))
    q = tamols_params_struct({}, "go2")  # VFA's own .get() fallbacks (visual_foothold_adaptation.py:298-305)
    assert (q.w_edge, q.w_dev, q.w_nominal, q.w_tracking, q.w_stability) == (15.0, 1.0, 20.0, 2.0, 10.0)


def test_tamols_oracle_flat_known_answer():
    """Flat patch: edge = roughness = 0; with deviation as the only soft cost the winner is the
    reachable candidate nearest the seed (SURVEY 8(c) KAT 7)."""
    params = dict(base_config.simulation_params["tamols_params"])
    params.update(weight_reference_tracking=0.0, weight_stability=0.0, weight_nominal_kinematic=0.0, h_des=0.25)
    orc = TamolsOracle(params, "go2")
    rng = np.random.default_rng(4)
    seeds = np.array([[0.30, 0.13, 0], [0.30, -0.13, 0], [-0.1, 0.13, 0], [-0.1, -0.13, 0]]) + \
        rng.uniform(-0.02, 0.02, (4, 3)) * [1, 1, 0]
    hips = seeds * [1, 1, 0] + [0, 0, 0.30]
    hms = np.stack([synthetic_patch(s[:2], 0.2, TERRAINS["flat"]) for s in seeds])
    fh, boxes, valid, scores = orc.compute(hms, seeds, hips, None)
    assert valid.all()
    orc.forward_vel = None
    for leg in range(4):
        hm = FastHeightMap(hms[leg])
        cands = np.column_stack([hm.points, hm.heights + 0.02 + 0.005])
        for c in cands[:10]:
            assert orc._edge(c, hm) == 0.0
            assert orc._rough(c, hm) < 1e-30
        feas = np.isfinite(scores[leg])
        d = np.sum((cands - seeds[leg]) ** 2, axis=1)
        d[~feas] = np.inf
        np.testing.assert_array_equal(fh[leg], cands[np.argmin(d)])
        np.testing.assert_allclose(boxes[leg, 1] - boxes[leg, 0], [0.1, 0.1, 0], atol=1e-15)


def test_tamols_oracle_unreachable_falls_back_to_seed_height():
    orc = TamolsOracle(dict(base_config.simulation_params["tamols_params"]), "go2")
    seeds = np.zeros((4, 3))
    hips = np.tile([0.0, 0.0, 5.0], (4, 1))  # every candidate far out of reach
    hms = np.stack([synthetic_patch(s[:2], 0.0, TERRAINS["flat"]) for s in seeds])
    fh, boxes, valid, scores = orc.compute(hms, seeds, hips, None)
    assert not valid.any() and np.isinf(scores).all()
    np.testing.assert_allclose(fh[:, 2], 0.02)


# ---------------------------------------------------------------- the per-step CPython glue (_srbd_fast)
def test_fast_glue_is_built_and_bound():
    assert _lib.fast is not None, "_srbd_fast is not built (make -C quadruped-pympc-tamols_amd)"


@pytest.mark.parametrize("gait", [0, 1, 7])
def test_pgg_fast_glue_equals_python_path(monkeypatch, gait):
    """compute_contact_sequence through _srbd_fast equals the ctypes path (same C call) for every dts / lens form
    the caller may pass (lists, int64 lengths), and keeps the same error."""
    a, b = PeriodicGaitGenerator(0.65, 1.4, gait, 12), PeriodicGaitGenerator(0.65, 1.4, gait, 12)
    for k in range(50):
        dts, lens = ([0.02], [12]) if k % 2 else (np.array([0.01, 0.02]), np.array([3, 12], np.int64))
        x = a.compute_contact_sequence(dts, lens)
        monkeypatch.setattr(_lib, "fast", None)
        y = b.compute_contact_sequence(dts, lens)
        monkeypatch.undo()
        assert x.dtype == y.dtype and x.shape == y.shape and x.flags["C_CONTIGUOUS"]
        np.testing.assert_array_equal(x, y)
        a.run(0.002 * (k % 5), 1.4)
        b.run(0.002 * (k % 5), 1.4)
    if gait != 7:
        with pytest.raises(ValueError, match="compute_contact_sequence failed"):
            a.compute_contact_sequence([0.02], [3])  # runs past the last dts entry (the reference: IndexError)


@pytest.mark.parametrize("fast", [True, False])
def test_pgg_short_lengths_follow_the_reference_loop(monkeypatch, fast):
    """Fewer contact_sequence_lenghts than dts: the library reads lengths[j] for j < len(dts) only, so both paths walk
    the reference's index (PGG:111-115) first -- IndexError exactly where the reference's loop would read past the
    lengths, the reference's sequence where it never does (the scalar oracle restates that loop)."""
    if not fast:
        monkeypatch.setattr(_lib, "fast", None)
    H = 12
    ok_cases = [([0.01, 0.02], [12]), ([0.01, 0.02], [H - 1]), ([0.01, 0.02, 0.03], [4, 12])]
    bad_cases = [([0.01, 0.02], [3]), ([0.01, 0.02, 0.03], [4, 8]), ([0.01, 0.02], [])]
    for dts, lens in ok_cases:
        a, b = PeriodicGaitGenerator(0.65, 1.4, 0, H), PGGOracle(0.65, 1.4, 0, H)
        np.testing.assert_array_equal(a.compute_contact_sequence(dts, lens), b.compute_contact_sequence(dts, lens))
    for dts, lens in bad_cases:
        a, b = PeriodicGaitGenerator(0.65, 1.4, 0, H), PGGOracle(0.65, 1.4, 0, H)
        with pytest.raises(IndexError):
            b.compute_contact_sequence(dts, lens)
        with pytest.raises(IndexError):
            a.compute_contact_sequence(dts, lens)
        # nothing ran here (the reference's loop has advanced its phases by the time it raises; the library's own
        # error path restores them, as test_pgg_c_abi_argument_checks pins)
        np.testing.assert_array_equal(a.phase_signal, [0.5, 1.0, 1.0, 0.5])


def test_interface_glue_declines_other_inputs():
    """interface_step returns None (the Python sequence then runs) for inputs it does not take, before it touches
    the context, the staging or the library -- so no device is needed to check it."""
    from quadruped_pympc_amd._lib import InterfaceIO

    io = InterfaceIO()
    io.horizon = 12
    rng = np.random.default_rng(0)
    sc, rs = dicts(rng)
    best = np.zeros(48, f32)
    cs = np.ones((4, 12))
    args = lambda s, r, c: (0, C.addressof(io), s, r, c, best, np.ones(4), np.array([42, 0], np.uint64), 0, 1, None,
                            np.zeros(48, f32), None, 0)
    assert _lib.fast.interface_step(*args({k: list(v) for k, v in sc.items()}, rs, cs)) is None
    assert _lib.fast.interface_step(*args({k: v.astype(f32) for k, v in sc.items()}, rs, cs)) is None
    assert _lib.fast.interface_step(*args(sc, rs, cs[:, :8])) is None       # shorter than the horizon
    assert _lib.fast.interface_step(*args(sc, rs, cs.astype(np.int64))) is None
    del sc["foot_RR"]
    assert _lib.fast.interface_step(*args(sc, rs, cs)) is None
    assert io.stage == 0 and not any(io.state_in)


def test_controller_copies_own_their_staging():
    """with_newkey / prepare_state cache raw addresses of per-controller staging; a deepcopy (or a pickle
    round trip) must make its own instead of writing into the original's (or freed) memory."""
    import pickle

    m = Sampling_MPC(cfg_module(sampling_method="mppi", control_parametrization="zero_order"))
    m.with_newkey()
    rng = np.random.default_rng(1)
    sc, rs = dicts(rng)
    m.prepare_state_and_reference(sc, rs, np.ones(4), np.ones(4))
    k_orig = m.master_key.copy()
    for c in (copy.deepcopy(m), pickle.loads(pickle.dumps(m))):
        assert c._ctx is None and "_split_buf" not in c.__dict__ and "_ps" not in c.__dict__
        c.with_newkey()
        c.prepare_state_and_reference(sc, rs, np.array([0, 1, 1, 0]), np.ones(4))
        np.testing.assert_array_equal(m.master_key, k_orig)
        np.testing.assert_array_equal(c.master_key, _lib.jax_split(k_orig, 2)[0])
    m.with_newkey()
    np.testing.assert_array_equal(m.master_key, _lib.jax_split(k_orig, 2)[0])
