"""Synthetic terrains and a heightmap-patch producer (stand-in for gym_quadruped's HeightMap).

The reference samples a 13 x 7 patch at 0.04 m around each reference foothold with
MuJoCo ray casts (simulation.py:490-511, wb_interface.py:233-234).  Here the patch
is sampled from an analytic height field: ``flat`` or ``stepping_stones_medium``
(stones of radius 0.15 m, 0.40 m apart, 3 per row, alternate rows offset, top
+0.05 m, gaps at -0.5 m; geometry from docs/STEPPING_STONES_TERRAIN.md:9-50).
"""
from __future__ import annotations

import numpy as np


def flat(height: float = 0.0):
    return lambda x, y: np.full(np.broadcast(x, y).shape, height, dtype=np.float64)


def stepping_stones(radius=0.15, spacing=0.40, per_row=3, top=0.05, gap=-0.5, x0=0.4):
    """Rows along +x every ``spacing``; ``per_row`` stones across y; odd rows shifted by spacing/2.

    Flat ground (z = 0) for x < x0 (the start platform)."""
    ys = (np.arange(per_row) - (per_row - 1) / 2) * spacing

    def h(x, y):
        x = np.asarray(x, dtype=np.float64)
        y = np.asarray(y, dtype=np.float64)
        row = np.round((x - x0) / spacing)
        cx = x0 + row * spacing
        shift = np.where(np.mod(row, 2) == 1, spacing / 2, 0.0)
        best = np.full(np.broadcast(x, y).shape, np.inf)
        for yc in ys:
            d = np.hypot(x - cx, y - (yc + shift))
            best = np.minimum(best, d)
        z = np.where(best <= radius, top, gap)
        return np.where(x < x0, 0.0, z)

    return h


TERRAINS = {"flat": flat(), "stepping_stones_medium": stepping_stones()}


class PatchHeightMap:
    """``HeightMap``-like object: ``.data`` is (rows, cols, 1, 3) world points, ``get_height`` is
    nearest-point height + 0.02 (the lookup FastHeightMap accelerates, visual_foothold_adaptation.py:21-35)."""

    def __init__(self, terrain, num_rows=13, num_cols=7, dist_x=0.04, dist_y=0.04):
        self.terrain = terrain
        self.num_rows, self.num_cols, self.dist_x, self.dist_y = num_rows, num_cols, dist_x, dist_y
        self.data = None

    def update_height_map(self, center, yaw=0.0):
        r = (np.arange(self.num_rows) - (self.num_rows - 1) / 2) * self.dist_x
        c = (np.arange(self.num_cols) - (self.num_cols - 1) / 2) * self.dist_y
        dx, dy = np.meshgrid(r, c, indexing="ij")
        cy, sy = np.cos(yaw), np.sin(yaw)
        x = center[0] + cy * dx - sy * dy
        y = center[1] + sy * dx + cy * dy
        z = self.terrain(x, y)
        self.data = np.stack([x, y, z], -1)[:, :, None, :].astype(np.float64)
        return self.data

    def get_height(self, target):
        if self.data is None:
            return None
        pts = self.data[:, :, 0, :].reshape(-1, 3)
        d = (pts[:, 0] - target[0]) ** 2 + (pts[:, 1] - target[1]) ** 2
        return pts[int(np.argmin(d)), 2] + 0.02
