"""GPU TAMOLS foothold search vs the float64 oracle (oracle/tamols_oracle.py).

Tolerances: identical feasibility (inf pattern) and winning candidate; finite scores atol 1e-9
(numpy's BLAS norms and SVD lstsq vs the kernel's closed forms differ by float64 rounding only);
footholds and boxes atol 1e-12.
"""
import numpy as np
import pytest

from oracle.tamols_oracle import TamolsOracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def search():
    from quadruped_pympc_amd import _lib
    from quadruped_pympc_amd.helpers.visual_foothold_adaptation import TamolsSearch

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible")
    s = TamolsSearch(0)
    yield s
    s.close()


def scene(terrain_name, yaw, rng, hip_h=0.30, shift=(0.0, 0.0)):
    from quadruped_pympc_amd.helpers.terrain import TERRAINS, PatchHeightMap

    if terrain_name == "rough":
        base = TERRAINS["flat"]
        amp = rng.uniform(0.0, 0.06, (64, 64))

        def terrain(x, y):
            i = np.clip(((np.asarray(x) + 2) * 16).astype(int), 0, 63)
            j = np.clip(((np.asarray(y) + 2) * 16).astype(int), 0, 63)
            return base(x, y) + amp[i, j]
    else:
        terrain = TERRAINS[terrain_name]
    feet = np.array([[0.62, 0.13, 0.0], [0.62, -0.13, 0.0], [0.24, 0.13, 0.0], [0.24, -0.13, 0.0]])
    feet[:, 0] += shift[0]
    feet[:, 1] += shift[1]
    seeds = feet + np.array([0.12, 0.0, 0.0]) + rng.uniform(-0.03, 0.03, (4, 3)) * [1, 1, 0]
    hips = feet + np.array([0.0, 0.0, hip_h])
    hms = []
    for i in range(4):
        hm = PatchHeightMap(terrain)
        hm.update_height_map(seeds[i], yaw)
        hms.append(hm.data)
    return np.stack(hms), seeds, hips, feet


def compare(search, hms, seeds, hips, vel, base, contact, feet, robot="go2"):
    from quadruped_pympc_amd import config
    from quadruped_pympc_amd.helpers.visual_foothold_adaptation import tamols_params_struct

    params = dict(config.simulation_params["tamols_params"])
    params["h_des"] = 0.25
    orc = TamolsOracle(params, robot)
    fh, boxes, valid, scores = orc.compute(hms, seeds, hips, vel, base, contact, feet)
    out = search.run(hms, seeds, hips, tamols_params_struct(params, robot), forward_vel=vel, base_position=base,
                     current_contact=contact, current_feet_pos=feet)
    np.testing.assert_array_equal(np.isinf(out["scores"]), np.isinf(scores))
    fin = np.isfinite(scores)
    np.testing.assert_allclose(out["scores"][fin], scores[fin], rtol=0, atol=1e-9)
    np.testing.assert_array_equal(out["valid"], valid)
    np.testing.assert_allclose(out["footholds"], fh, rtol=0, atol=1e-12)
    np.testing.assert_allclose(out["boxes"][valid], boxes[valid], rtol=0, atol=1e-12)
    return out, scores


@pytest.mark.parametrize("terrain", ["flat", "stepping_stones_medium", "rough"])
@pytest.mark.parametrize("yaw", [0.0, 0.3, -1.2])
def test_tamols_parity(search, terrain, yaw):
    rng = np.random.default_rng(int(abs(yaw) * 100) + len(terrain))
    hms, seeds, hips, feet = scene(terrain, yaw, rng)
    vel = np.array([0.4, 0.05, 0.0])
    base = feet.mean(0) + [0, 0, 0.3]
    contact = np.array([0, 1, 1, 0])
    out, scores = compare(search, hms, seeds, hips, vel, base, contact, feet)
    assert np.isfinite(scores).any()


def test_tamols_optional_inputs(search):
    rng = np.random.default_rng(3)
    hms, seeds, hips, feet = scene("stepping_stones_medium", 0.1, rng, shift=(0.5, 0.0))
    compare(search, hms, seeds, hips, None, None, None, None)
    compare(search, hms, seeds, hips, np.array([-0.3, 0.0, 0.0]), None, None, feet)
    compare(search, hms, seeds, hips, np.zeros(3), feet.mean(0), np.array([1, 1, 1, 1]), feet)


def test_tamols_all_infeasible_fallback(search):
    rng = np.random.default_rng(4)
    hms, seeds, hips, feet = scene("flat", 0.0, rng, hip_h=2.0)  # out of reach everywhere
    out, scores = compare(search, hms, seeds, hips, np.zeros(3), None, None, None)
    assert not out["valid"].any() and np.isinf(scores).all()
    np.testing.assert_allclose(out["footholds"][:, 2], 0.02, atol=1e-12)


def test_visual_foothold_adaptation_drop_in(search):
    """The product class with HeightMap-like objects and the reference's extra phase_signal kwarg."""
    from quadruped_pympc_amd.helpers.legs_attr import LegsAttr
    from quadruped_pympc_amd.helpers.terrain import TERRAINS, PatchHeightMap
    from quadruped_pympc_amd.helpers.visual_foothold_adaptation import VisualFootholdAdaptation
    from quadruped_pympc_amd import config

    legs = ["FL", "FR", "RL", "RR"]
    vfa = VisualFootholdAdaptation(legs, "tamols")
    rng = np.random.default_rng(9)
    _, seeds, hips, feet = scene("stepping_stones_medium", 0.0, rng, shift=(0.4, 0.0))
    hmaps = LegsAttr(*[PatchHeightMap(TERRAINS["stepping_stones_medium"]) for _ in legs])
    for i, n in enumerate(legs):
        hmaps[n].update_height_map(seeds[i], 0.0)
    ref = LegsAttr(*[s.copy() for s in seeds])
    ok = vfa.compute_adaptation(legs, ref, LegsAttr(*hips), hmaps, np.array([0.4, 0, 0]), np.zeros(3), np.zeros(3),
                                base_position=feet.mean(0) + [0, 0, 0.3], current_contact=np.array([0, 1, 1, 0]),
                                phase_signal=np.zeros(4), current_feet_pos=LegsAttr(*feet))
    assert ok and vfa.initialized
    adapted, boxes = vfa.get_footholds_adapted(ref)
    orc = TamolsOracle(dict(config.simulation_params["tamols_params"]), config.robot)
    fh, _, valid, _ = orc.compute(np.stack([h.data for h in hmaps]), seeds, hips, np.array([0.4, 0, 0]),
                                  feet.mean(0) + [0, 0, 0.3], np.array([0, 1, 1, 0]), feet)
    for i, n in enumerate(legs):
        np.testing.assert_allclose(adapted[n], fh[i], atol=1e-12)
