"""NumPy restatement of the terrain heightmap-patch producer (TEST INFRASTRUCTURE ONLY).

SURVEY 8(f) row 3.  The reference samples each leg's 13 x 7 patch with gym_quadruped's
``HeightMap.update_height_map`` (one MuJoCo ``mj_ray`` per point; called at
quadruped_pympc/interfaces/wb_interface.py:233-234, built at simulation/simulation.py:490-511).
gym_quadruped and MuJoCo are absent here, so this oracle pins the semantics the C-ABI declares
(include/srbd_mpc.h, srbd_terrain_*): vertical rays from ray_z, the highest surface at or below
ray_z among the ground plane, box tops (yaw about z), upright-cylinder tops and a height field
split along the (i, j)-(i+1, j+1) diagonal; ``miss_z`` when nothing is hit.  Every float64
operation is written in the kernel's order (terrain_kernel.hip), and cos / sin come from libm
(``math``) as on the kernel's host side, so the comparison is exact.  Parity against the real
sensor is unpinned (no MuJoCo).  Only tests/ may import this module.
"""
from __future__ import annotations

import math

import numpy as np

BOX, CYLINDER = 0, 1


def patch_points(centers, yaws, rows, cols, dist_x, dist_y):
    """(npatch, rows, cols, 2) x, y of every ray, the kernel's arithmetic order."""
    centers = np.asarray(centers, dtype=np.float64).reshape(-1, 3)
    n = centers.shape[0]
    i = np.arange(rows, dtype=np.float64)[:, None]
    k = np.arange(cols, dtype=np.float64)[None, :]
    dx = (i - float(rows - 1) / 2.0) * dist_x
    dy = (k - float(cols - 1) / 2.0) * dist_y
    out = np.empty((n, rows, cols, 2))
    for p in range(n):
        c, s = math.cos(float(yaws[p])), math.sin(float(yaws[p]))
        out[p, :, :, 0] = centers[p, 0] + c * dx - s * dy
        out[p, :, :, 1] = centers[p, 1] + s * dx + c * dy
    return out


def raycast(x, y, prims, ray_z, has_ground=True, ground_z=0.0, hfield=None, miss_z=float("nan")):
    """Heights at points (x, y) (any matching shapes).  prims: list of dicts with keys type, cx, cy, cz,
    a, b, c, yaw (srbd_terrain_prim).  hfield: None or dict(z (nx, ny), x0, y0, dx, dy)."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    best = np.full(x.shape, -np.inf)
    hit = np.zeros(x.shape, dtype=bool)

    def consider(top, mask):
        take = mask & (top <= ray_z) & (top > best)
        best[take] = np.broadcast_to(top, x.shape)[take]
        hit[take] = True

    if has_ground:
        consider(np.float64(ground_z), np.ones(x.shape, dtype=bool))
    for pr in prims:
        ux, uy = x - pr["cx"], y - pr["cy"]
        if pr["type"] == BOX:
            cb, sb = math.cos(pr["yaw"]), math.sin(pr["yaw"])
            u, v = cb * ux + sb * uy, cb * uy - sb * ux
            inside = (np.abs(u) <= pr["a"]) & (np.abs(v) <= pr["b"])
        else:
            inside = ux * ux + uy * uy <= pr["a"] * pr["a"]
        consider(np.float64(pr["cz"] + pr["c"]), inside)
    if hfield is not None:
        z = np.asarray(hfield["z"], dtype=np.float64)
        nx, ny = z.shape
        fx = (x - hfield["x0"]) / hfield["dx"]
        fy = (y - hfield["y0"]) / hfield["dy"]
        inside = (fx >= 0.0) & (fy >= 0.0) & (fx <= float(nx - 1)) & (fy <= float(ny - 1))
        i0 = np.minimum(np.floor(np.where(inside, fx, 0.0)).astype(np.int64), nx - 2)
        j0 = np.minimum(np.floor(np.where(inside, fy, 0.0)).astype(np.int64), ny - 2)
        tx, ty = fx - i0, fy - j0
        z00, z10, z01, z11 = z[i0, j0], z[i0 + 1, j0], z[i0, j0 + 1], z[i0 + 1, j0 + 1]
        lower = z00 + tx * (z10 - z00) + ty * (z11 - z10)
        upper = z00 + ty * (z01 - z00) + tx * (z11 - z01)
        consider(np.where(tx >= ty, lower, upper), inside)
    return np.where(hit, best, miss_z)


def patches(prims, centers, yaws, rows, cols, dist_x, dist_y, ray_z, **scene):
    """(npatch, rows, cols, 3) as srbd_terrain_patches returns them."""
    xy = patch_points(centers, yaws, rows, cols, dist_x, dist_y)
    z = raycast(xy[..., 0], xy[..., 1], prims, ray_z, **scene)
    return np.concatenate([xy, z[..., None]], axis=-1)
