"""Terrains and heightmap-patch producers (stand-ins for gym_quadruped's HeightMap).

The reference samples a 13 x 7 patch at 0.04 m around each reference foothold with
MuJoCo ray casts (simulation.py:490-511, wb_interface.py:233-234).  Two producers here:

* ``GpuTerrain`` / ``GpuHeightMap``: the scene (ground plane, boxes, upright cylinders, a
  height field) lives on the GPU and every patch point is one lane's vertical ray cast
  (``srbd_terrain_patches``, terrain_kernel.hip).  ``TamolsSearch.run_terrain``
  feeds the raycast patches straight into the TAMOLS kernel without a host round trip.
* ``PatchHeightMap``: the same patch layout sampled from an analytic height function on the host
  (``flat`` or ``stepping_stones_medium``: stones of radius 0.15 m, 0.40 m apart, 3 per row,
  alternate rows offset, top +0.05 m, gaps at -0.5 m; geometry from
  docs/STEPPING_STONES_TERRAIN.md:9-50).  ``stepping_stones_scene`` builds the equivalent
  primitive scene for the GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .. import _lib


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


def stepping_stones_scene(radius=0.15, spacing=0.40, per_row=3, top=0.05, gap=-0.5, x0=0.4, n_rows=20,
                          platform_from=-10.0):
    """Primitive scene of ``stepping_stones`` for ``GpuTerrain``: ``n_rows`` rows of upright cylinders
    (top ``top``), the start platform as a box with top 0 over [platform_from, x0], the gaps as the
    ground plane at ``gap``.  Equal to the analytic terrain except within one stone radius before the
    platform edge, where the analytic function lets the platform (z = 0) cut the first row's stones and
    the scene keeps their tops (+0.05)."""
    ys = (np.arange(per_row) - (per_row - 1) / 2) * spacing
    prims = []
    for row in range(n_rows):
        shift = spacing / 2 if row % 2 == 1 else 0.0
        for yc in ys:
            prims.append(dict(type=_lib.PRIM_CYLINDER, cx=x0 + row * spacing, cy=float(yc + shift), cz=0.0,
                              a=radius, b=0.0, c=top, yaw=0.0))
    half = (x0 - platform_from) / 2
    prims.append(dict(type=_lib.PRIM_BOX, cx=platform_from + half, cy=0.0, cz=-0.25, a=half, b=50.0, c=0.25, yaw=0.0))
    return dict(prims=prims, has_ground=True, ground_z=gap)


class GpuTerrain:
    """A device-resident scene (``srbd_terrain``); ``patches`` casts one vertical ray per patch point."""

    def __init__(self, prims=(), has_ground=True, ground_z=0.0, hfield=None, miss_z=float("nan"), device_id=0):
        prims = list(prims)
        arr = (_lib.TerrainPrim * max(1, len(prims)))()
        for i, p in enumerate(prims):
            arr[i] = _lib.TerrainPrim(int(p["type"]), 0, float(p["cx"]), float(p["cy"]), float(p["cz"]),
                                      float(p["a"]), float(p.get("b", 0.0)), float(p["c"]), float(p.get("yaw", 0.0)))
        hf = None
        nx = ny = 0
        x0 = y0 = dx = dy = 0.0
        if hfield is not None:
            hf = np.ascontiguousarray(hfield["z"], dtype=np.float64)
            nx, ny = hf.shape
            x0, y0, dx, dy = (float(hfield[k]) for k in ("x0", "y0", "dx", "dy"))
        h = C.c_void_p()
        rc = _lib.lib.srbd_terrain_create(int(device_id), arr, len(prims), int(bool(has_ground)), float(ground_z),
                                          _lib.dptr(hf), nx, ny, x0, y0, dx, dy, float(miss_z), C.byref(h))
        if rc != _lib.OK:
            msg = _lib.lib.srbd_terrain_last_error(None)
            raise RuntimeError(f"srbd_terrain_create failed ({rc}): {msg.decode() if msg else ''}")
        self.h = h

    @classmethod
    def stepping_stones(cls, device_id=0, **kw):
        return cls(device_id=device_id, **stepping_stones_scene(**kw))

    def patches(self, centers, yaws, rows=13, cols=7, dist_x=0.04, dist_y=0.04, ray_z=10.0) -> np.ndarray:
        """(npatch, rows, cols, 3) points (x, y, z) around each centre (rows along the yawed x axis)."""
        c = np.ascontiguousarray(centers, dtype=np.float64).reshape(-1, 3)
        y = np.ascontiguousarray(np.broadcast_to(np.asarray(yaws, dtype=np.float64), (c.shape[0],)))
        out = np.empty((c.shape[0], rows, cols, 3))
        rc = _lib.lib.srbd_terrain_patches(self.h, _lib.dptr(c), _lib.dptr(y), c.shape[0], rows, cols, float(dist_x),
                                           float(dist_y), float(ray_z), _lib.dptr(out))
        if rc != _lib.OK:
            msg = _lib.lib.srbd_terrain_last_error(self.h)
            raise RuntimeError(f"srbd_terrain_patches failed ({rc}): {msg.decode() if msg else ''}")
        return out

    def close(self):
        if getattr(self, "h", None):
            _lib.lib.srbd_terrain_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GpuHeightMap:
    """``HeightMap``-like object over a ``GpuTerrain``: ``update_height_map`` records the patch (centre, yaw) and the
    raycast runs on the GPU when ``.data`` is first read; ``.data`` is (rows, cols, 1, 3); ``get_height`` is
    nearest-point height + 0.02, as ``PatchHeightMap``.  Lazy, so ``VisualFootholdAdaptation.compute_adaptation``
    can hand four pending patches over one terrain to the fused raycast + TAMOLS launch
    (``TamolsSearch.run_terrain``) instead of four raycast launches and their copies (wb_interface.py:230-240
    updates the four maps around the seeds and adapts at once)."""

    def __init__(self, terrain: GpuTerrain, num_rows=13, num_cols=7, dist_x=0.04, dist_y=0.04, ray_z=10.0):
        self.terrain = terrain
        self.num_rows, self.num_cols, self.dist_x, self.dist_y, self.ray_z = num_rows, num_cols, dist_x, dist_y, ray_z
        self._data = None
        self.pending = None  # (centre (3,), yaw) of a patch not raycast yet

    def update_height_map(self, center, yaw=0.0):
        c = np.asarray(center, dtype=np.float64).reshape(-1)[:3]
        if c.size < 3:
            c = np.concatenate([c, np.zeros(3 - c.size)])
        self.pending = (c.copy(), float(yaw))
        self._data = None

    @property
    def has_data(self) -> bool:
        return self.pending is not None or self._data is not None

    @property
    def data(self):
        if self.pending is not None:
            c, yaw = self.pending
            p = self.terrain.patches(c[None], [yaw], self.num_rows, self.num_cols, self.dist_x, self.dist_y,
                                     self.ray_z)
            self.set_data(p[0])
        return self._data

    def set_data(self, patch):
        """The raycast patch (rows, cols, 3) of the pending update (the fused launch's output)."""
        self._data = np.asarray(patch, dtype=np.float64)[:, :, None, :]
        self.pending = None

    get_height = PatchHeightMap.get_height
