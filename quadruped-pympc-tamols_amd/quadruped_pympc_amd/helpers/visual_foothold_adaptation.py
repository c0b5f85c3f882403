"""Visual foothold adaptation with the TAMOLS local search on the GPU.

Drop-in for ``quadruped_pympc/helpers/visual_foothold_adaptation.py``
(``VisualFootholdAdaptation``, :38-231) for the strategies ``'height'`` and
``'tamols'``.  The TAMOLS search (:153-229 and its cost helpers :261-714) runs as
one HIP kernel launch over the four legs (``srbd_tamols_run``); the candidate set
is every point of each leg's heightmap patch (:240-243), as in the reference.

Fixes relative to the reference (behaviour otherwise unchanged):

* ``compute_adaptation`` accepts and ignores extra keyword arguments such as the
  ``phase_signal=`` that ``wb_interface.py:235-240`` passes (a TypeError in the
  reference).

``'vfa'`` needs the closed-source VFA module and raises ImportError, as the
reference does when it is absent.
"""
from __future__ import annotations

import ctypes as C

import copy

import numpy as np

from .. import _lib
from ..runtime import active_config, resolve_device_id
from .legs_attr import LegsAttr

LEGS = ("FL", "FR", "RL", "RR")


def tamols_params_struct(tamols_params: dict, robot_name: str) -> "_lib.TamolsParams":
    """srbd_tamols_params from ``simulation_params['tamols_params']`` (config.py:209-243), with VFA's defaults."""
    g = tamols_params.get
    p = _lib.TamolsParams()
    p.gradient_delta = g("gradient_delta", 0.04)
    p.slope_threshold = g("slope_threshold", 0.7)
    p.w_edge = g("weight_edge_avoidance", 15.0)
    p.w_rough = g("weight_roughness", 10.0)
    p.w_dev = g("weight_deviation", 1.0)
    p.w_nominal = g("weight_nominal_kinematic", 20.0)
    p.w_tracking = g("weight_reference_tracking", 2.0)
    p.w_stability = g("weight_stability", 10.0)
    p.stability_margin = g("stability_margin", 0.06)
    p.swing_time = g("estimated_swing_time", 0.25)
    p.h_des = g("h_des", 0.25)
    p.l_min = g("l_min", {}).get(robot_name, 0.15)
    p.l_max = g("l_max", {}).get(robot_name, 0.45)
    p.box_dx = g("constraint_box_dx", 0.05)
    p.box_dy = g("constraint_box_dy", 0.05)
    p.stance_duration = 0.3
    for i, a in enumerate(np.linspace(0.2, 0.8, 5)):
        p.alphas[i] = float(a)
    return p


class TamolsSearch:
    """Owns one ``srbd_tamols_ctx``; ``run`` / ``run_terrain`` evaluate all four legs in one kernel launch.

    Inputs are copied into persistent staging arrays whose addresses are cached, and the outputs come
    back in persistent arrays (copied into the returned dict): a call costs a few slice copies plus the C
    call (``ndarray.ctypes`` conversions cost ~2.5 us each, more than the kernel itself)."""

    def __init__(self, device_id: int = 0):
        h = C.c_void_p()
        rc = _lib.lib.srbd_tamols_create(int(device_id), C.byref(h))
        if rc != _lib.OK:
            raise RuntimeError(f"srbd_tamols_create failed ({rc}): {_lib.last_error(None)}")
        self.h = h
        self._shape = None
        self._inp = np.zeros(42)  # seeds 0:12 | hips 12:24 | vel 24:27 | base 27:30 | feet 30:42
        self._contact = np.zeros(4, dtype=np.int32)
        self._res = np.zeros(40)  # footholds 0:12 | boxes 12:36 | seed heights 36:40
        self._valid = np.zeros(4, dtype=np.int32)
        a = self._inp.ctypes.data
        self._a_seeds, self._a_hips, self._a_vel, self._a_base, self._a_feet = a, a + 96, a + 192, a + 216, a + 240
        self._a_contact = self._contact.ctypes.data
        r = self._res.ctypes.data
        self._a_fh, self._a_box, self._a_seedh = r, r + 96, r + 288
        self._a_valid = self._valid.ctypes.data

    def _shape_bufs(self, rows, cols):
        if self._shape != (rows, cols):
            self._shape = (rows, cols)
            self._scores = np.zeros(4 * rows * cols)
            self._hm = np.zeros((4, rows, cols, 3))
            self._a_scores, self._a_hm = self._scores.ctypes.data, self._hm.ctypes.data

    def close(self):
        if getattr(self, "h", None):
            _lib.lib.srbd_tamols_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stage(self, seeds, hips, forward_vel, base_position, current_contact, current_feet_pos):
        inp = self._inp
        inp[0:12] = np.reshape(seeds, 12)
        inp[12:24] = np.reshape(hips, 12)
        a_vel = a_base = a_contact = a_feet = None
        if forward_vel is not None:
            inp[24:27] = np.asarray(forward_vel, dtype=np.float64).reshape(-1)[:3]
            a_vel = self._a_vel
        if base_position is not None:
            inp[27:30] = np.asarray(base_position, dtype=np.float64).reshape(-1)[:3]
            a_base = self._a_base
        if current_contact is not None:
            self._contact[:] = np.reshape(current_contact, 4)
            a_contact = self._a_contact
        if current_feet_pos is not None:
            inp[30:42] = np.reshape(current_feet_pos, 12)
            a_feet = self._a_feet
        return a_vel, a_base, a_contact, a_feet

    def _result(self, rows, cols, with_hm, with_scores=True):
        r = self._res
        out = dict(footholds=r[0:12].reshape(4, 3).copy(), boxes=r[12:36].reshape(4, 2, 3).copy(),
                   valid=self._valid.astype(bool), seed_heights=r[36:40].copy())
        if with_scores:
            out["scores"] = self._scores.reshape(4, rows * cols).copy()
        if with_hm:
            out["heightmaps"] = self._hm.copy()
        return out

    def _raise(self, name, rc):
        msg = _lib.lib.srbd_tamols_last_error(self.h)
        raise RuntimeError(f"{name} failed ({rc}): {msg.decode() if msg else ''}")

    def run(self, heightmaps, seeds, hips, params, forward_vel=None, base_position=None, current_contact=None,
            current_feet_pos=None, want_scores=True):
        """heightmaps (4, rows, cols, 3) or (4, rows, cols, 1, 3); seeds/hips (4, 3).

        Returns dict(footholds (4,3), boxes (4,2,3), valid (4,) bool, scores (4, rows*cols) (when
        want_scores), seed_heights (4,))."""
        hm = np.asarray(heightmaps, dtype=np.float64)
        rows, cols = hm.shape[1], hm.shape[2]
        self._shape_bufs(rows, cols)
        self._hm[...] = hm.reshape(4, rows, cols, 3)
        a_vel, a_base, a_contact, a_feet = self._stage(seeds, hips, forward_vel, base_position, current_contact,
                                                       current_feet_pos)
        rc = _lib.lib.srbd_tamols_run(self.h, self._a_hm, rows, cols, self._a_seeds, self._a_hips, a_vel, a_base,
                                      a_contact, a_feet, C.byref(params), self._a_fh, self._a_box, self._a_valid,
                                      self._a_scores if want_scores else None, self._a_seedh)
        if rc != _lib.OK:
            self._raise("srbd_tamols_run", rc)
        return self._result(rows, cols, False, want_scores)

    def run_terrain(self, terrain, yaw, seeds, hips, params, rows=13, cols=7, dist_x=0.04, dist_y=0.04, ray_z=10.0,
                    forward_vel=None, base_position=None, current_contact=None, current_feet_pos=None,
                    want_scores=True, want_heightmaps=True):
        """``run`` on patches raycast from a ``GpuTerrain`` around the seeds, in the same launch as the search
        (``srbd_tamols_run_terrain``).  The result also holds the patches (``heightmaps``, (4, rows, cols, 3))
        when want_heightmaps; without scores and patches nothing but the footholds crosses PCIe."""
        self._shape_bufs(rows, cols)
        a_vel, a_base, a_contact, a_feet = self._stage(seeds, hips, forward_vel, base_position, current_contact,
                                                       current_feet_pos)
        rc = _lib.lib.srbd_tamols_run_terrain(self.h, terrain.h, float(yaw), rows, cols, float(dist_x), float(dist_y),
                                              float(ray_z), self._a_seeds, self._a_hips, a_vel, a_base, a_contact,
                                              a_feet, C.byref(params), self._a_fh, self._a_box, self._a_valid,
                                              self._a_scores if want_scores else None, self._a_seedh,
                                              self._a_hm if want_heightmaps else None)
        if rc != _lib.OK:
            self._raise("srbd_tamols_run_terrain", rc)
        return self._result(rows, cols, want_heightmaps, want_scores)


def _rows(attr, names):
    """(len(names), 3) float64 copy of the per-leg 3-vectors (one slice store per leg instead of np.stack)."""
    out = np.empty((len(names), 3))
    for i, n in enumerate(names):
        out[i] = attr[n]
    return out


def _fused_patches(heightmaps, names, seeds):
    """(terrain, yaw, first map) when the four maps are GpuHeightMaps of one terrain with one patch geometry, each
    pending a patch around its seed at one yaw (what wb_interface.py:233-234 leaves before compute_adaptation);
    else None."""
    from .terrain import GpuHeightMap

    maps = [heightmaps[n] for n in names]
    if not all(isinstance(m, GpuHeightMap) and m.pending is not None for m in maps):
        return None
    g = maps[0]
    geo = (g.terrain, g.num_rows, g.num_cols, g.dist_x, g.dist_y, g.ray_z, g.pending[1])
    for m, sd in zip(maps, seeds):
        if (m.terrain, m.num_rows, m.num_cols, m.dist_x, m.dist_y, m.ray_z, m.pending[1]) != geo:
            return None
        # bitwise (a -0.0 / 0.0 mismatch only costs the unfused path); ~10x cheaper than np.array_equal
        if m.pending[0].tobytes() != np.asarray(sd, dtype=np.float64).reshape(-1)[:3].tobytes():
            return None
    return g.terrain, g.pending[1], g


class VisualFootholdAdaptation:
    def __init__(self, legs_order, adaptation_strategy="height", config_module=None, device_id=None):
        cfg = active_config(config_module)  # the reference's quadruped_pympc.config when installed
        self.footholds_adaptation = LegsAttr(FL=np.array([0, 0, 0]), FR=np.array([0, 0, 0]), RL=np.array([0, 0, 0]),
                                             RR=np.array([0, 0, 0]))
        self.footholds_constraints = LegsAttr(FL=None, FR=None, RL=None, RR=None)
        self.initialized = False
        self.adaptation_strategy = adaptation_strategy
        self.legs_order = tuple(legs_order)
        if adaptation_strategy == "vfa":
            raise ImportError("VFA strategy requested but VFA module could not be imported.")
        self._search = None
        self._device_id = cfg.mpc_params.get("device_id", "auto") if device_id is None else device_id
        if adaptation_strategy == "tamols":
            self.tamols_params = cfg.simulation_params.get("tamols_params", {})
            self.robot_name = cfg.robot
        # last_scores (an extension: the reference keeps no scores): the per-candidate TAMOLS scores of the last call,
        # (4, rows * cols), kept when keep_scores is set -- copying them to the host costs the C4 step ~2 us
        self.keep_scores = False
        self.last_scores = None
        self._params_src = self._params_struct = self._params_robot = None

    def _params(self):
        """tamols_params_struct of the current tamols_params, rebuilt only when they changed (a dict compare instead
        of 17 attribute stores and a linspace per call)."""
        if self._params_src is None or self._params_src != self.tamols_params or self._params_robot != self.robot_name:
            self._params_struct = tamols_params_struct(self.tamols_params, self.robot_name)
            self._params_src = copy.deepcopy(self.tamols_params)
            self._params_robot = self.robot_name
        return self._params_struct

    def update_footholds_adaptation(self, update_footholds_adaptation):
        self.footholds_adaptation = update_footholds_adaptation
        self.initialized = True

    def reset(self):
        self.initialized = False

    def get_footholds_adapted(self, reference_footholds):
        if not self.initialized:
            self.footholds_adaptation = reference_footholds
            return reference_footholds, self.footholds_constraints
        return self.footholds_adaptation, self.footholds_constraints

    @property
    def search(self) -> TamolsSearch:
        if self._search is None:
            self._device_id = resolve_device_id(self._device_id)
            self._search = TamolsSearch(self._device_id)
        return self._search

    def compute_adaptation(self, legs_order, reference_footholds, hip_positions, heightmaps, forward_vel,
                           base_orientation, base_orientation_rate, gait_phases=None, base_position=None,
                           current_contact=None, current_feet_pos=None, **_ignored):
        for leg_name in legs_order:
            hm = heightmaps[leg_name]
            if not (hm.has_data if hasattr(hm, "has_data") else hm.data is not None):
                return False

        if self.adaptation_strategy == "tamols" and tuple(legs_order) != LEGS:
            raise ValueError("TAMOLS expects legs_order FL, FR, RL, RR")

        if self.adaptation_strategy == "height":
            for leg_name in legs_order:
                h = heightmaps[leg_name].get_height(reference_footholds[leg_name])
                if h is not None:
                    reference_footholds[leg_name][2] = h

        elif self.adaptation_strategy == "tamols":
            names = list(legs_order)
            seeds = _rows(reference_footholds, names)
            hips = _rows(hip_positions, names)
            contact = None if current_contact is None else np.asarray(current_contact).astype(np.int32)
            feet = None
            if current_feet_pos is not None and base_position is not None:
                feet = _rows(current_feet_pos, LEGS)
            params = self._params()
            fused = _fused_patches(heightmaps, names, seeds)
            if fused is not None:  # GPU maps of one terrain, pending around the seeds: raycast + TAMOLS in one launch
                ter, yaw, g = fused
                out = self.search.run_terrain(ter, yaw, seeds, hips, params, rows=g.num_rows, cols=g.num_cols,
                                              dist_x=g.dist_x, dist_y=g.dist_y, ray_z=g.ray_z,
                                              forward_vel=forward_vel, base_position=base_position,
                                              current_contact=contact, current_feet_pos=feet,
                                              want_scores=self.keep_scores)
                for i, n in enumerate(names):
                    heightmaps[n].set_data(out["heightmaps"][i])
            else:
                data = np.stack([np.asarray(heightmaps[n].data, dtype=np.float64)[:, :, 0, :] for n in names])
                out = self.search.run(data, seeds, hips, params, forward_vel=forward_vel, base_position=base_position,
                                      current_contact=contact, current_feet_pos=feet, want_scores=self.keep_scores)
            self.last_scores = out.get("scores")
            for i, n in enumerate(names):
                if out["valid"][i]:
                    reference_footholds[n] = out["footholds"][i].copy()
                    self.footholds_constraints[n] = [out["boxes"][i, 0].copy(), out["boxes"][i, 1].copy()]
                else:
                    # VFA:223-228: the original heightmap's own lookup when it provides one
                    get = getattr(heightmaps[n], "get_height", None)
                    h = get(seeds[i]) if get is not None else out["seed_heights"][i]
                    if h is not None:
                        reference_footholds[n][2] = h
        self.update_footholds_adaptation(reference_footholds)
        return True
