"""CPU oracle (numpy float64) for the TAMOLS foothold local search.

TEST INFRASTRUCTURE ONLY (same import rule as ``srbd_oracle.py``).

Restates ``VisualFootholdAdaptation.compute_adaptation`` (strategy ``'tamols'``)
and its helpers from the reference file
``quadruped_pympc/helpers/visual_foothold_adaptation.py`` (VFA below), lines
cited per function, with parameters from ``quadruped_pympc/config.py:209-243``.
Nearest-neighbour height lookups use ``scipy.spatial.cKDTree`` exactly as the
reference's ``FastHeightMap`` does (VFA:21-35).

PARITY STATUS: parity unpinned against the reference itself (it imports
``gym_quadruped`` at module import, which is absent; the reference has no
tests or fixtures).  Pinned by analytic known-answer tests (flat patch: edge =
roughness = 0 and the winner is the reachable candidate nearest the seed).

The original ``HeightMap.get_height`` used by the all-infeasible fallback
(VFA:223-228) lives in the absent gym_quadruped; it is inferred to be the same
nearest-neighbour + 0.02 lookup that ``FastHeightMap`` accelerates (VFA:22).
"""
from __future__ import annotations

import numpy as np
from scipy.spatial import cKDTree

LEGS = ("FL", "FR", "RL", "RR")

# config.py:209-243 (tamols_params) values; the tests always pass this dict explicitly, so VFA's own
# .get() fallbacks (VFA:298-305, used by the product's tamols_params_struct) never apply here
DEFAULT_PARAMS = {
    "gradient_delta": 0.04,
    "weight_edge_avoidance": 10.0,
    "weight_roughness": 10,
    "weight_deviation": 2,
    "weight_kinematic": 2.0,
    "weight_nominal_kinematic": 0.0,
    "weight_reference_tracking": 10.0,
    "weight_stability": 20.0,
    "stability_margin": 0.06,
    "estimated_swing_time": 0.25,
    "h_des": 0.25,
    "slope_threshold": 0.7,
    "constraint_box_dx": 0.05,
    "constraint_box_dy": 0.05,
    "l_min": {"go1": 0.15, "go2": 0.15, "aliengo": 0.1, "b2": 0.25, "hyqreal1": 0.25, "hyqreal2": 0.25,
              "mini_cheetah": 0.12, "spot": 0.20},
    "l_max": {"go1": 0.45, "go2": 0.45, "aliengo": 0.55, "b2": 0.75, "hyqreal1": 0.75, "hyqreal2": 0.75,
              "mini_cheetah": 0.40, "spot": 0.60},
}


class FastHeightMap:
    """VFA:21-35.  data: (rows, cols, 1, 3) float64.

    ``nn="kdtree"`` is the reference's lookup (cKDTree.query).  ``nn="first"`` is the same nearest
    neighbour by brute force with the first index winning exact distance ties (the kernel's rule,
    tamols_kernel.hip).  The two differ only when a query is exactly equidistant from two patch points:
    cKDTree then returns the first tied point its traversal visits, which depends on the leaf order its
    median-split build leaves behind (an introselect permutation inside scipy), so that tie rule is not
    reproducible outside scipy (tests/test_tamols_ties.py measures how often it differs).
    """

    def __init__(self, data, nn="kdtree"):
        self.data = np.asarray(data, dtype=np.float64)
        self.points = self.data[:, :, 0, :2].reshape(-1, 2)
        self.heights = self.data[:, :, 0, 2].reshape(-1)
        self.nn = nn
        self.tree = cKDTree(self.points) if nn == "kdtree" else None

    def nearest(self, target):
        if self.tree is not None:
            return int(self.tree.query(target[:2])[1])
        d = (self.points[:, 0] - target[0]) ** 2 + (self.points[:, 1] - target[1]) ** 2
        return int(np.argmin(d))  # first index among exact ties

    def get_height(self, target):
        return self.heights[self.nearest(target)] + 0.02


class TamolsOracle:
    def __init__(self, params=None, robot_name="go2", nn="kdtree"):
        self.nn = nn  # FastHeightMap lookup: the reference's cKDTree, or "first" (first index on exact ties)
        self.p = dict(DEFAULT_PARAMS)
        if params:
            self.p.update(params)
        self.robot_name = robot_name

    # VFA:375-395
    def _kin(self, cand, hip):
        l_min = self.p["l_min"].get(self.robot_name, 0.15)
        l_max = self.p["l_max"].get(self.robot_name, 0.45)
        d = np.linalg.norm(cand - hip)
        if not (l_min <= d <= l_max):
            return False
        if self.forward_vel is not None:
            hip_lo = hip + self.forward_vel[:3] * 0.3
            d = np.linalg.norm(cand - hip_lo)
            if not (l_min <= d <= l_max):
                return False
        return True

    # VFA:397-420
    def _collision(self, cand, hip, hm):
        for alpha in np.linspace(0.2, 0.8, 5):
            p = (1 - alpha) * hip + alpha * cand
            h_ground = hm.get_height(p) - 0.02
            if p[2] < (h_ground + 0.02):
                return True
        return False

    # VFA:422-466
    def _edge(self, cand, hm):
        delta = self.p["gradient_delta"]
        thr = self.p["slope_threshold"]
        offs = [np.array([delta, 0, 0]), np.array([-delta, 0, 0]), np.array([0, delta, 0]), np.array([0, -delta, 0])]
        h = [hm.get_height(cand + o) for o in offs]
        gx = abs(h[0] - h[1]) / (2 * delta)
        gy = abs(h[2] - h[3]) / (2 * delta)
        g = np.sqrt(gx ** 2 + gy ** 2)
        return 0.0 if g <= thr else g - thr

    # VFA:468-521
    def _rough(self, cand, hm):
        delta = self.p["gradient_delta"]
        heights, pos = [], []
        for i in range(-1, 2):
            for j in range(-1, 2):
                q = cand.copy()
                q[0] += i * delta
                q[1] += j * delta
                heights.append(hm.get_height(q))
                pos.append([i * delta, j * delta])
        heights = np.array(heights)
        pos = np.array(pos)
        A = np.column_stack([pos[:, 0], pos[:, 1], np.ones(len(heights))])
        sol = np.linalg.lstsq(A, heights, rcond=None)[0]
        return np.var(heights - A @ sol)

    # VFA:523-553
    def _nominal(self, cand, hip):
        l_des = np.array([0.0, 0.0, -self.p["h_des"]])
        diff = hip - (cand - l_des)
        return np.dot(diff, diff)

    # VFA:555-609
    def _tracking(self, cand, seed):
        if self.forward_vel is None:
            dx = cand[0] - seed[0]
            return dx ** 2 if dx < 0 else 0.0
        v = self.forward_vel[:2]
        if np.linalg.norm(v) < 0.01:
            return 0.0
        dx = (cand[:2] - seed[:2])[0]
        if v[0] > 0 and dx < 0:
            return dx ** 2
        if v[0] < 0 and dx > 0:
            return dx ** 2
        return 0.0

    # VFA:611-714
    def _stability(self, cand, leg_id):
        if self.base_position is None or self.current_feet_pos is None:
            return 0.0
        margin = self.p["stability_margin"]
        diag = {0: 3, 1: 2, 2: 1, 3: 0}[leg_id]
        if self.current_contact is not None and self.current_contact[leg_id] == 1:
            return 0.0
        foot = np.asarray(self.current_feet_pos[diag], dtype=np.float64)
        c = self.base_position[:2] + self.forward_vel[:2] * self.p["estimated_swing_time"]
        p1, p2 = cand[:2], foot[:2]
        v = p2 - p1
        w = c - p1
        vv = np.dot(v, v)
        if vv < 1e-8:
            d = np.linalg.norm(c - p1)
        else:
            t = np.clip(np.dot(w, v) / vv, 0.0, 1.0)
            d = np.linalg.norm(c - (p1 + t * v))
        return (d - margin) ** 2 if d > margin else 0.0

    # VFA:261-373
    def score(self, cand, seed, hip, hm, leg_id):
        if not self._kin(cand, hip):
            return float("inf")
        if self._collision(cand, hip, hm):
            return float("inf")
        p = self.p
        edge = self._edge(cand, hm) * p["weight_edge_avoidance"]
        rough = self._rough(cand, hm) * p["weight_roughness"]
        dev = np.sum((cand - seed) ** 2) * p["weight_deviation"]
        nom = self._nominal(cand, hip) * p["weight_nominal_kinematic"]
        track = self._tracking(cand, seed) * p["weight_reference_tracking"]
        stab = self._stability(cand, leg_id) * p["weight_stability"]
        return 0.0 + edge + rough + dev + nom + track + stab

    # VFA:153-231
    def compute(self, heightmaps, seeds, hips, forward_vel, base_position=None, current_contact=None,
                current_feet_pos=None):
        """heightmaps: (4, rows, cols, 1, 3); seeds/hips: (4, 3).

        Returns footholds (4,3), boxes (4,2,3) (nan where no box), valid (4,) bool, scores (4, rows*cols)."""
        self.forward_vel = None if forward_vel is None else np.asarray(forward_vel, dtype=np.float64)
        self.base_position = None if base_position is None else np.asarray(base_position, dtype=np.float64)
        self.current_contact = np.array([0, 0, 0, 0]) if current_contact is None else np.asarray(current_contact)
        self.current_feet_pos = current_feet_pos
        heightmaps = np.asarray(heightmaps, dtype=np.float64)
        R, C = heightmaps.shape[1], heightmaps.shape[2]
        footholds = np.array(seeds, dtype=np.float64).copy()
        boxes = np.full((4, 2, 3), np.nan)
        valid = np.zeros(4, dtype=bool)
        scores = np.full((4, R * C), np.inf)
        for leg in range(4):
            seed = np.array(seeds[leg], dtype=np.float64).copy()
            hip = np.asarray(hips[leg], dtype=np.float64)
            hm = FastHeightMap(heightmaps[leg].reshape(R, C, 1, 3), self.nn)
            cands = hm.data[:, :, 0, :2].reshape(-1, 2).tolist()
            best, best_score = None, float("inf")
            for i, cxy in enumerate(cands):
                cand = np.array([cxy[0], cxy[1], 0.0])
                cand[2] = hm.get_height(cand) + 0.005
                s = self.score(cand, seed, hip, hm, leg)
                scores[leg, i] = s
                if s < best_score:
                    best_score, best = s, cand
            if best is not None:
                footholds[leg] = best
                dx, dy = self.p["constraint_box_dx"], self.p["constraint_box_dy"]
                v1, v2 = best.copy(), best.copy()
                v1[0] -= dx
                v1[1] -= dy
                v2[0] += dx
                v2[1] += dy
                boxes[leg] = [v1, v2]
                valid[leg] = True
            else:
                footholds[leg][2] = hm.get_height(seed)
        return footholds, boxes, valid, scores


def synthetic_patch(center_xy, yaw, terrain, rows=13, cols=7, res=0.04):
    """A (rows, cols, 1, 3) heightmap patch around ``center_xy`` rotated by ``yaw``.

    Layout follows simulation.py:490-511 (13 x 7 @ 0.04 m); ``terrain(x, y)`` gives ground height.
    """
    r = (np.arange(rows) - (rows - 1) / 2) * res
    c = (np.arange(cols) - (cols - 1) / 2) * res
    out = np.zeros((rows, cols, 1, 3))
    cy, sy = np.cos(yaw), np.sin(yaw)
    for i, dx in enumerate(r):
        for j, dy in enumerate(c):
            x = center_xy[0] + cy * dx - sy * dy
            y = center_xy[1] + sy * dx + cy * dy
            out[i, j, 0] = (x, y, terrain(x, y))
    return out
