"""GPU heightmap patches (srbd_terrain_*, terrain_kernel.hip) vs oracle/terrain_oracle.py, and the
fused raycast + TAMOLS call vs TAMOLS on the same patches.  Bar: bit-exact (float64, same op order,
libm cos / sin on both host sides)."""
import math

import numpy as np
import pytest

from oracle import terrain_oracle as T

pytestmark = pytest.mark.gpu


def random_scene(rng, n_box=12, n_cyl=12, with_hf=True):
    prims = []
    for _ in range(n_box):
        prims.append(dict(type=T.BOX, cx=rng.uniform(-1, 1), cy=rng.uniform(-1, 1), cz=rng.uniform(-0.2, 0.1),
                          a=rng.uniform(0.02, 0.3), b=rng.uniform(0.02, 0.3), c=rng.uniform(0.01, 0.2),
                          yaw=rng.uniform(-math.pi, math.pi)))
    for _ in range(n_cyl):
        prims.append(dict(type=T.CYLINDER, cx=rng.uniform(-1, 1), cy=rng.uniform(-1, 1), cz=rng.uniform(-0.2, 0.1),
                          a=rng.uniform(0.02, 0.2), b=0.0, c=rng.uniform(0.01, 0.2), yaw=0.0))
    hf = None
    if with_hf:
        hf = dict(z=rng.uniform(-0.1, 0.15, (40, 33)), x0=-1.2, y0=-0.9, dx=0.06, dy=0.055)
    return prims, hf


@pytest.fixture(scope="module")
def lib():
    from quadruped_pympc_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible")
    return _lib


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("rows,cols", [(13, 7), (5, 3), (1, 1)])
def test_patches_bit_exact(lib, seed, rows, cols):
    from quadruped_pympc_amd.helpers.terrain import GpuTerrain

    rng = np.random.default_rng(seed)
    prims, hf = random_scene(rng, with_hf=seed != 2)
    has_ground = seed != 1
    ter = GpuTerrain(prims, has_ground=has_ground, ground_z=-0.05, hfield=hf, miss_z=-9.0)
    try:
        n = 37
        centers = np.column_stack([rng.uniform(-1.2, 1.2, n), rng.uniform(-1.2, 1.2, n), rng.uniform(0, 0.3, n)])
        yaws = rng.uniform(-math.pi, math.pi, n)
        got = ter.patches(centers, yaws, rows, cols, 0.04, 0.035, ray_z=0.12)
        want = T.patches(prims, centers, yaws, rows, cols, 0.04, 0.035, 0.12, has_ground=has_ground, ground_z=-0.05,
                         hfield=hf, miss_z=-9.0)
        np.testing.assert_array_equal(got, want)
        assert np.isfinite(got).all()
    finally:
        ter.close()


def test_stepping_stones_heightmap_matches_host_patch(lib):
    from quadruped_pympc_amd.helpers.terrain import GpuHeightMap, GpuTerrain, PatchHeightMap, stepping_stones

    ter = GpuTerrain.stepping_stones()
    try:
        g = GpuHeightMap(ter)
        h = PatchHeightMap(stepping_stones())
        for c in ([1.2, 0.13, 0.3], [2.03, -0.21, 0.3], [3.5, 0.0, 0.3]):  # clear of the platform edge
            g.update_height_map(np.array(c), yaw=0.0)
            h.update_height_map(np.array(c), yaw=0.0)
            np.testing.assert_array_equal(g.data, h.data)
            assert g.get_height(np.array(c)) == h.get_height(np.array(c))
    finally:
        ter.close()


@pytest.mark.parametrize("yaw", [0.0, 0.4])
def test_fused_raycast_tamols_equals_two_step(lib, yaw):
    from quadruped_pympc_amd import config
    from quadruped_pympc_amd.helpers.terrain import GpuTerrain
    from quadruped_pympc_amd.helpers.visual_foothold_adaptation import TamolsSearch, tamols_params_struct

    ter = GpuTerrain.stepping_stones()
    s = TamolsSearch(0)
    try:
        feet = np.array([[1.22, 0.13, 0.05], [1.22, -0.13, 0.05], [0.84, 0.13, 0.05], [0.84, -0.13, 0.05]])
        seeds = feet + np.array([0.12, 0.02, 0.0])
        hips = feet + np.array([0.0, 0.0, 0.3])
        params = dict(config.simulation_params["tamols_params"])
        params["h_des"] = 0.25
        ps = tamols_params_struct(params, "go2")
        vel, base = np.array([0.5, 0.0, 0.0]), np.array([1.03, 0.0, 0.35])
        contact = np.array([0, 1, 1, 0], np.int32)
        fused = s.run_terrain(ter, yaw, seeds, hips, ps, forward_vel=vel, base_position=base, current_contact=contact,
                              current_feet_pos=feet)
        hms = ter.patches(seeds, [yaw] * 4, 13, 7, 0.04, 0.04, ray_z=10.0)
        np.testing.assert_array_equal(fused["heightmaps"], hms)
        two = s.run(hms, seeds, hips, ps, forward_vel=vel, base_position=base, current_contact=contact,
                    current_feet_pos=feet)
        for k in ("footholds", "boxes", "valid", "scores", "seed_heights"):
            np.testing.assert_array_equal(fused[k], two[k])
        assert fused["valid"].any()
    finally:
        s.close()
        ter.close()


def test_argument_errors(lib):
    import ctypes as C

    h = C.c_void_p()
    bad = (lib.TerrainPrim * 1)()
    bad[0].type = 7
    assert lib.lib.srbd_terrain_create(0, bad, 1, 1, 0.0, None, 0, 0, 0, 0, 0, 0, 0.0, C.byref(h)) == lib.E_INVALID
    hf = np.zeros((1, 5))
    assert lib.lib.srbd_terrain_create(0, bad, 0, 1, 0.0, lib.dptr(hf), 1, 5, 0, 0, 0.1, 0.1, 0.0,
                                       C.byref(h)) == lib.E_INVALID


@pytest.mark.parametrize("n_box,n_cyl", [(500, 500), (560, 540)])
def test_large_scene_fused_tamols(lib, n_box, n_cyl):
    """Scenes at the LDS staging limit (1000 primitives: 80 KB of dynamic LDS beside the kernel's static
    ~23 KB, which needs the dynamic-LDS attribute srbd_tamols_create sets) and past it (1100: the fused
    kernel reads the primitives from global memory): raycast patches bit-exact vs the terrain oracle, and
    the fused raycast + TAMOLS call equal to TAMOLS on those patches."""
    from quadruped_pympc_amd import config
    from quadruped_pympc_amd.helpers.terrain import GpuTerrain
    from quadruped_pympc_amd.helpers.visual_foothold_adaptation import TamolsSearch, tamols_params_struct

    rng = np.random.default_rng(n_box)
    prims, hf = random_scene(rng, n_box=n_box, n_cyl=n_cyl)
    ter = GpuTerrain(prims, has_ground=True, ground_z=-0.05, hfield=hf, miss_z=-9.0)
    s = TamolsSearch(0)
    try:
        feet = np.array([[0.32, 0.13, 0.05], [0.32, -0.13, 0.05], [-0.06, 0.13, 0.05], [-0.06, -0.13, 0.05]])
        seeds = feet + np.array([0.12, 0.02, 0.0])
        hips = feet + np.array([0.0, 0.0, 0.3])
        want = T.patches(prims, seeds, [0.3] * 4, 13, 7, 0.04, 0.04, 10.0, has_ground=True, ground_z=-0.05,
                         hfield=hf, miss_z=-9.0)
        hms = ter.patches(seeds, [0.3] * 4, 13, 7, 0.04, 0.04, ray_z=10.0)
        np.testing.assert_array_equal(hms, want)
        params = dict(config.simulation_params["tamols_params"])
        params["h_des"] = 0.25
        ps = tamols_params_struct(params, "go2")
        kw = dict(forward_vel=np.array([0.5, 0.0, 0.0]), base_position=np.array([0.13, 0.0, 0.35]),
                  current_contact=np.array([0, 1, 1, 0], np.int32), current_feet_pos=feet)
        fused = s.run_terrain(ter, 0.3, seeds, hips, ps, **kw)
        np.testing.assert_array_equal(fused["heightmaps"], want)
        two = s.run(hms, seeds, hips, ps, **kw)
        for k in ("footholds", "boxes", "valid", "scores", "seed_heights"):
            np.testing.assert_array_equal(fused[k], two[k])
    finally:
        s.close()
        ter.close()


@pytest.mark.parametrize("yaw", [0.0, 0.4, math.pi / 2, -2.3])
def test_lattice_queries_equal_full_scan(lib, monkeypatch, yaw):
    """The raycast patch's nearest-neighbour queries on the lattice (four points per query, one block per leg)
    against every point scanned (SRBD_TAMOLS_LATTICE=0, 16 blocks per leg): every output bit-equal, with hips on
    half-lattice points (exact ties between two patch points: the first index wins both ways) and hips off the
    patch (queries clamped to its edge)."""
    from quadruped_pympc_amd import config
    from quadruped_pympc_amd.helpers.terrain import GpuTerrain
    from quadruped_pympc_amd.helpers.visual_foothold_adaptation import TamolsSearch, tamols_params_struct

    ter = GpuTerrain.stepping_stones()
    s = TamolsSearch(0)
    rng = np.random.default_rng(int(1000 * abs(yaw)) + 3)
    params = dict(config.simulation_params["tamols_params"])
    params["h_des"] = 0.25
    ps = tamols_params_struct(params, "go2")
    c, sn = math.cos(yaw), math.sin(yaw)
    try:
        for trial in range(6):
            feet = np.array([[1.22, 0.13, 0.05], [1.22, -0.13, 0.05], [0.84, 0.13, 0.05], [0.84, -0.13, 0.05]])
            feet[:, :2] += rng.uniform(-0.3, 0.3, 2)
            seeds = feet + np.array([0.12, 0.02, 0.0])
            # hips at (half-)lattice offsets from the seed in the patch frame, or far off the patch
            du, dv = rng.integers(-8, 9, 4) * 0.02, rng.integers(-8, 9, 4) * 0.02
            if trial % 3 == 2:
                du = du * 10.0
            hips = seeds.copy()
            hips[:, 0] += c * du - sn * dv
            hips[:, 1] += sn * du + c * dv
            hips[:, 2] += 0.3
            kw = dict(forward_vel=np.array([0.5, 0.1, 0.0]), base_position=feet.mean(0) + [0, 0, 0.3],
                      current_contact=np.array([0, 1, 1, 0], np.int32), current_feet_pos=feet)
            a = s.run_terrain(ter, yaw, seeds, hips, ps, **kw)
            monkeypatch.setenv("SRBD_TAMOLS_LATTICE", "0")
            b = s.run_terrain(ter, yaw, seeds, hips, ps, **kw)
            monkeypatch.delenv("SRBD_TAMOLS_LATTICE")
            for k in ("footholds", "boxes", "valid", "scores", "seed_heights", "heightmaps"):
                np.testing.assert_array_equal(a[k], b[k], err_msg=f"{k} trial {trial}")
    finally:
        s.close()
        ter.close()
