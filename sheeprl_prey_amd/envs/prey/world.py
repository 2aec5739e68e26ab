"""Hexagonal predator-prey "cellworld", self-contained (no ``cellworld`` package, no downloads).

Reference behaviour: ``prey_env/prey_env/envs/gymnasium_env_bins.py``, ``Model.py``, ``Predator.py``,
``myPaths.py`` - they load a hex world ("hexagonal", "canonical", "%02i_%02i" occlusion set) from the
``cellworld`` resources server.  Here the same geometry is generated locally:

* arena: a regular hexagon centred at (0.5, 0.5), width 1, tiled by a radius-10 hex grid of
  cells (331 cells, centre spacing 1/21 - the canonical cellworld resolution);
* occlusions: the world name ``"%02i_%02i" % (layout, entropy)`` seeds a deterministic generator of
  clustered occlusion cells; higher entropy -> more, more scattered occlusions (layouts 0-10 are the
  "train" worlds, 11-19 "test", as in the reference);
* visibility: a segment is visible unless it passes within ``1.05 * cell_size/2`` of an occluded cell
  centre (the reference tests against 1.05-scaled hexagons; a circle of the hexagon's circumradius
  is used here) - evaluated vectorised over all occlusions;
* paths: shortest next-move table over free cells (BFS from every destination), replacing the
  downloaded A* path sets.
"""
from __future__ import annotations

import math
from functools import lru_cache
from typing import List, Optional, Tuple

import numpy as np

RADIUS = 10  # hex grid radius in cells -> 1 + 3R(R+1) = 331 cells
SPACING = 1.0 / (2 * RADIUS + 1)  # centre-to-centre distance
CELL_SIZE = SPACING  # cellworld's cell_transformation.size (goal / capture thresholds)
AXIAL_DIRS = [(1, 0), (1, -1), (0, -1), (-1, 0), (-1, 1), (0, 1)]


def normalize_angle(a: float) -> float:
    while a > math.pi:
        a -= 2 * math.pi
    while a < -math.pi:
        a += 2 * math.pi
    return a


def angle_difference(a: float, b: float) -> Tuple[float, float]:
    """(|difference|, direction) like cellworld's ``angle_difference`` (direction = +1 if b is
    clockwise of a)."""
    d = normalize_angle(b - a)
    return abs(d), (-1.0 if d > 0 else 1.0)


def atan_to(src: np.ndarray, dst: np.ndarray) -> float:
    """cellworld ``Location.atan``: angle measured from the +y axis, clockwise-positive."""
    return math.atan2(dst[0] - src[0], dst[1] - src[1])


def move(loc: np.ndarray, theta: float, dist: float) -> np.ndarray:
    return np.array([loc[0] + math.sin(theta) * dist, loc[1] + math.cos(theta) * dist])


class HexWorld:
    def __init__(self, name: str = "00_03"):
        self.name = name
        qs, rs = [], []
        for q in range(-RADIUS, RADIUS + 1):
            for r in range(max(-RADIUS, -q - RADIUS), min(RADIUS, -q + RADIUS) + 1):
                qs.append(q)
                rs.append(r)
        self.axial = np.stack([np.array(qs), np.array(rs)], -1)
        # pointy-top cells; the arena hexagon has its corners at (0, 0.5) and (1, 0.5)
        x = 0.5 + SPACING * (np.array(qs) + np.array(rs) * 0.5)
        y = 0.5 + SPACING * (np.array(rs) * math.sqrt(3) / 2)
        self.centers = np.stack([x, y], -1)
        self.n = len(qs)
        self.index = {(int(q), int(r)): i for i, (q, r) in enumerate(self.axial)}
        self.occluded = self._generate_occlusions(name)
        self.occ_centers = self.centers[self.occluded]
        self.occ_radius = CELL_SIZE / 2 * 1.05  # circumradius of the reference's 1.05-scaled occlusion hexagons
        self.neighbors = [[self.index.get((int(q) + dq, int(r) + dr), -1) for dq, dr in AXIAL_DIRS]
                          for q, r in self.axial]
        self.free = np.nonzero(~self.occluded)[0]
        self._next_hop: Optional[np.ndarray] = None

    # ------------------------------------------------------------------ occlusions
    def _generate_occlusions(self, name: str) -> np.ndarray:
        layout, entropy = (int(p) for p in name.split("_"))
        rng = np.random.default_rng(1000 * layout + entropy + 7)
        occ = np.zeros(self.n, dtype=bool)
        target = int(round(self.n * (0.04 + 0.025 * entropy)))  # ~4%..29% of the arena
        n_clusters = max(1, 2 + entropy + rng.integers(0, 3))
        protected = set()
        for loc in ((0.0, 0.5), (1.0, 0.5)):  # keep start/goal regions free
            d = np.linalg.norm(self.centers - np.array(loc), axis=1)
            protected.update(np.nonzero(d < 3.5 * SPACING)[0].tolist())
        tries = 0
        while occ.sum() < target and tries < 10000:
            tries += 1
            seed = int(rng.integers(0, self.n))
            if seed in protected:
                continue
            size = int(rng.integers(2, max(3, target // n_clusters + 2)))
            frontier = [seed]
            grown = 0
            while frontier and grown < size and occ.sum() < target:
                c = frontier.pop(int(rng.integers(0, len(frontier))))
                if occ[c] or c in protected:
                    continue
                occ[c] = True
                grown += 1
                frontier.extend(nb for nb in self.neighbors_of(c) if nb >= 0 and not occ[nb])
        return occ

    def neighbors_of(self, i: int) -> List[int]:
        q, r = self.axial[i]
        return [self.index.get((int(q) + dq, int(r) + dr), -1) for dq, dr in AXIAL_DIRS]

    # ------------------------------------------------------------------ geometry
    def cell_of(self, loc: np.ndarray) -> int:
        return int(np.argmin(((self.centers - loc) ** 2).sum(-1)))

    def in_arena(self, loc: np.ndarray) -> bool:
        # flat-topped hexagon of apothem 0.5*sqrt(3)/2*... : test the 3 slab constraints
        p = loc - 0.5
        apothem = (RADIUS + 0.5) * SPACING * math.sqrt(3) / 2
        for ang in (0.0, math.pi / 3, 2 * math.pi / 3):
            n = (math.sin(ang), math.cos(ang))
            if abs(p[0] * n[0] + p[1] * n[1]) > apothem:
                return False
        return True

    def is_valid_location(self, loc: np.ndarray) -> bool:
        if not self.in_arena(loc):
            return False
        if len(self.occ_centers) == 0:
            return True
        d2 = ((self.occ_centers - loc) ** 2).sum(-1)
        return bool(d2.min() > (self.occ_radius) ** 2)

    def is_visible(self, a: np.ndarray, b: np.ndarray) -> bool:
        if len(self.occ_centers) == 0:
            return True
        ab = b - a
        L2 = float(ab @ ab)
        if L2 < 1e-12:
            return True
        t = np.clip(((self.occ_centers - a) @ ab) / L2, 0.0, 1.0)
        closest = a + t[:, None] * ab
        d2 = ((self.occ_centers - closest) ** 2).sum(-1)
        return bool(d2.min() > self.occ_radius ** 2)

    def visible_mask(self, a: np.ndarray, points: np.ndarray) -> np.ndarray:
        """Visibility from ``a`` to every row of ``points`` (vectorised over points and occlusions)."""
        if len(self.occ_centers) == 0:
            return np.ones(len(points), dtype=bool)
        ab = points - a  # [P, 2]
        L2 = np.maximum((ab ** 2).sum(-1), 1e-12)
        rel = self.occ_centers - a  # [O, 2]
        t = np.clip((rel @ ab.T) / L2, 0.0, 1.0)  # [O, P]
        cx = a[0] + t * ab[:, 0]
        cy = a[1] + t * ab[:, 1]
        d2 = (self.occ_centers[:, :1] - cx) ** 2 + (self.occ_centers[:, 1:] - cy) ** 2
        return d2.min(0) > self.occ_radius ** 2

    # ------------------------------------------------------------------ paths
    @property
    def next_hop(self) -> np.ndarray:
        """``next_hop[src, dst]`` = neighbour of ``src`` on a shortest free path to ``dst`` (-1 if none)."""
        if self._next_hop is None:
            nh = np.full((self.n, self.n), -1, dtype=np.int32)
            free = ~self.occluded
            for dst in self.free:
                # BFS from dst: parent pointers give each cell's next hop towards dst
                nh[dst, dst] = dst
                frontier = [int(dst)]
                seen = np.zeros(self.n, dtype=bool)
                seen[dst] = True
                while frontier:
                    nxt = []
                    for c in frontier:
                        for nb in self.neighbors[c]:
                            if nb >= 0 and free[nb] and not seen[nb]:
                                seen[nb] = True
                                nh[nb, dst] = c
                                nxt.append(nb)
                    frontier = nxt
            self._next_hop = nh
        return self._next_hop

    def path(self, src: int, dst: int) -> List[int]:
        out = [src]
        cur = src
        for _ in range(self.n):
            if cur == dst:
                break
            nxt = int(self.next_hop[cur, dst])
            if nxt < 0 or nxt == cur:
                break
            out.append(nxt)
            cur = nxt
        return out

    def occlusion_features(self, loc: np.ndarray, theta: float, k: int = 3) -> List[Tuple[float, float]]:
        """(distance, signed angle) to the ``k`` nearest occluded cells (reference
        ``gymnasium_env_bins.py:70-80``); padded with (0, 0) when fewer exist."""
        if len(self.occ_centers) == 0:
            return [(0.0, 0.0)] * k
        d = np.sqrt(((self.occ_centers - loc) ** 2).sum(-1))
        order = np.argsort(d)[:k]
        out = []
        for i in order:
            diff, direction = angle_difference(atan_to(loc, self.occ_centers[i]), theta)
            out.append((float(d[i]), float(diff * direction)))
        while len(out) < k:
            out.append((0.0, 0.0))
        return out


@lru_cache(maxsize=64)
def get_world(name: str) -> HexWorld:
    """Worlds are immutable: cache them (the reference rebuilds one, plus matplotlib displays, on every reset)."""
    return HexWorld(name)
