"""CPU tests of the terrain heightmap-patch oracle (oracle/terrain_oracle.py): patch layout, the
stepping-stones scene against the analytic terrain, height-field and box semantics."""
import math

import numpy as np
import pytest

from oracle import terrain_oracle as T
from quadruped_pympc_amd import _lib
from quadruped_pympc_amd.helpers.terrain import PatchHeightMap, stepping_stones, stepping_stones_scene


@pytest.mark.parametrize("yaw", [0.0, 0.3, -1.2, math.pi / 2])
def test_patch_layout_matches_host_heightmap(yaw):
    hm = PatchHeightMap(stepping_stones(), 13, 7, 0.04, 0.04)
    c = np.array([1.13, -0.21, 0.3])
    hm.update_height_map(c, yaw=yaw)
    xy = T.patch_points(c[None], [yaw], 13, 7, 0.04, 0.04)[0]
    np.testing.assert_allclose(xy, hm.data[:, :, 0, :2], rtol=0, atol=1e-15)
    if yaw == 0.0:
        np.testing.assert_array_equal(xy, hm.data[:, :, 0, :2])


def test_stepping_stones_scene_matches_analytic_terrain():
    rng = np.random.default_rng(3)
    x = rng.uniform(-1.0, 8.0, 20000)
    y = rng.uniform(-1.0, 1.0, 20000)
    # the two descriptions differ only next to the platform: the analytic function lets the platform
    # (z = 0) override the first row's stones for x < 0.4, the scene keeps the stones' tops
    keep = (x < 0.25) | (x > 0.4)
    x, y = x[keep], y[keep]
    sc = stepping_stones_scene()
    z = T.raycast(x, y, sc["prims"], 10.0, has_ground=True, ground_z=sc["ground_z"])
    np.testing.assert_array_equal(z, stepping_stones()(x, y))
    assert set(np.unique(z)) == {-0.5, 0.0, 0.05}


def test_height_field_is_piecewise_linear_and_exact_at_nodes():
    nx, ny = 9, 6
    gx, gy = np.meshgrid(np.arange(nx) * 0.1 - 0.3, np.arange(ny) * 0.05 + 0.2, indexing="ij")
    plane = 0.25 * gx - 0.5 * gy + 0.1
    hf = dict(z=plane, x0=-0.3, y0=0.2, dx=0.1, dy=0.05)
    rng = np.random.default_rng(1)
    x = rng.uniform(-0.3, 0.5, 5000)
    y = rng.uniform(0.2, 0.45, 5000)
    z = T.raycast(x, y, [], 10.0, has_ground=False, hfield=hf)
    np.testing.assert_allclose(z, 0.25 * x - 0.5 * y + 0.1, rtol=0, atol=1e-12)  # a plane is reproduced
    bumpy = rng.normal(size=(nx, ny))
    hf2 = dict(z=bumpy, x0=-0.3, y0=0.2, dx=0.1, dy=0.05)
    zn = T.raycast(-0.3 + np.arange(nx)[:, None] * 0.1 + 0 * gy, 0.2 + np.arange(ny)[None, :] * 0.05 + 0 * gx, [],
                   10.0, has_ground=False, hfield=hf2)
    np.testing.assert_allclose(zn, bumpy, rtol=0, atol=1e-12)
    # outside the field: miss
    assert np.isnan(T.raycast(np.array([0.6]), np.array([0.3]), [], 10.0, has_ground=False, hfield=hf2))[0]


def test_box_yaw_ray_start_and_miss():
    box = dict(type=T.BOX, cx=1.0, cy=0.0, cz=0.0, a=0.5, b=0.1, c=0.2, yaw=math.pi / 2)  # long axis along y
    z = T.raycast(np.array([1.0, 1.0, 1.3]), np.array([0.4, 0.6, 0.0]), [box], 10.0, has_ground=False, miss_z=-7.0)
    np.testing.assert_array_equal(z, [0.2, -7.0, -7.0])
    # a surface above the ray start is not hit; the ground below is
    z = T.raycast(np.array([1.0]), np.array([0.0]), [box], 0.1, has_ground=True, ground_z=-0.3)
    np.testing.assert_array_equal(z, [-0.3])
    cyl = dict(type=T.CYLINDER, cx=0.0, cy=0.0, cz=0.1, a=0.2, b=0.0, c=0.1, yaw=0.0)
    z = T.raycast(np.array([0.2, 0.2001]), np.array([0.0, 0.0]), [cyl, box], 10.0, has_ground=True)
    np.testing.assert_array_equal(z, [0.2, 0.0])  # boundary inclusive


def test_struct_layout():
    import ctypes as C
    assert C.sizeof(_lib.TerrainPrim) == 8 + 7 * 8
