"""Seeded synthetic workloads for BASELINE.json's configs.

config 1: two 360-beam scans, one alignment (ratio 5, and a ratio-1 variant)
config 2: 500-node odometry chain, 499 successive ICP edges, no loop closures
config 3: 2000 nodes, 1999 successive ICP edges + 200 loop closures (|i-j| >= 50, <= 2 m)
config 4: 5000 nodes, 4999 successive + 15001 loop-closure ICP edges (<= 5 m, nearest pairs
          first), 4999 odometry factors, 1 prior -> 25000 factors

World, trajectory and scans come from the C generator (dpg_synth.c).  Node estimated poses (the
values runIcp reads, dpg_slam.cc:364-368, and the GN initial values, dpg_slam.cc:111-118) are the
ground truth in node 0's frame plus Gaussian noise, as after an earlier optimisation; odometry
(odom_only_estimates_) is the ground-truth motion plus per-step noise.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass, field

import numpy as np

from . import _abi
from ._abi import FACTOR_DTYPE, lib, ptr
from . import api

ANGLE_MIN = -math.pi
ANGLE_MAX = math.pi
RANGE_MAX = 30.0
LASER = (0.2, 0.0, 0.0)   # parameters.h:319-339


@dataclass
class SynthConfig:
    name: str
    n_nodes: int
    n_beams: int = 5000
    seed: int = 4
    world_size: float = 40.0
    downsample: int = 5
    n_loop_closures: int = 0
    lc_max_dist: float = 5.0
    lc_min_sep: int = 2
    range_noise: float = 0.01
    est_noise: tuple = (0.05, 0.02)
    odom_noise: tuple = (0.05, 0.01)
    threads: int = 0


CONFIGS = {
    "config1": SynthConfig("config1", n_nodes=2, n_beams=360, seed=1, world_size=20.0),
    "config2": SynthConfig("config2", n_nodes=500, seed=2),
    "config3": SynthConfig("config3", n_nodes=2000, seed=3, n_loop_closures=200, lc_max_dist=2.0, lc_min_sep=50),
    "config4": SynthConfig("config4", n_nodes=5000, seed=4, n_loop_closures=15001, lc_max_dist=5.0, lc_min_sep=2),
}


@dataclass
class Workload:
    cfg: SynthConfig
    segs: np.ndarray            # world segments [S,4]
    gt: np.ndarray              # ground truth (world frame) [V,3] f64
    ranges: np.ndarray          # [V, n_beams] f32
    pts: np.ndarray             # concatenated full base_link clouds [P,2] f32
    offsets: np.ndarray         # [V+1] i64
    est: np.ndarray             # node estimated poses [V,3] f32 (node-0 frame)
    odom: np.ndarray            # odom_only_estimates_ [V,3] f32
    edges: np.ndarray           # ICP edges [E,2] = (node_1 target, node_2 source)
    n_successive: int
    base_factors: np.ndarray = field(default=None)   # prior + odometry factors
    icp_factor_first: int = 0

    @property
    def V(self) -> int:
        return len(self.gt)

    @property
    def E(self) -> int:
        return len(self.edges)

    def cloud(self, v: int) -> np.ndarray:
        return self.pts[self.offsets[v]:self.offsets[v + 1]]

    def node(self, v: int) -> api.Node:
        return api.Node(pose=self.est[v], cloud=self.cloud(v))

    def factors_with_icp(self, results: np.ndarray, params=None) -> np.ndarray:
        """Full factor list: base factors, then one BetweenFactor per ICP edge in edge order;
        successive edges always count, loop closures only when converged (zero information
        otherwise -- same H, g and error as leaving the factor out)."""
        p = params or _abi.default_icp_params()
        F = np.zeros(len(self.base_factors) + self.E, FACTOR_DTYPE)
        F[:len(self.base_factors)] = self.base_factors
        k = len(self.base_factors)
        F["kind"][k:] = _abi.DPG_FACTOR_BETWEEN
        F["i"][k:] = self.edges[:, 0]
        F["j"][k:] = self.edges[:, 1]
        F["z"][k:] = results["z"].astype(np.float64)
        keep = np.ones(self.E, bool)
        keep[self.n_successive:] = (results["converged"][self.n_successive:] != 0) & (
            results["status"][self.n_successive:] == _abi.DPG_ICP_OK)
        info = np.array([1.0 / float(np.float32(p.laser_x_variance)), 1.0 / float(np.float32(p.laser_y_variance)),
                         1.0 / float(np.float32(p.laser_theta_variance))])
        F["info"][k:] = np.where(keep[:, None], info[None, :], 0.0)
        return F

    def factors_placeholder(self) -> np.ndarray:
        """Factor list with the ICP slots present (measurements filled on device)."""
        F = np.zeros(len(self.base_factors) + self.E, FACTOR_DTYPE)
        F[:len(self.base_factors)] = self.base_factors
        k = len(self.base_factors)
        F["kind"][k:] = _abi.DPG_FACTOR_BETWEEN
        F["i"][k:] = self.edges[:, 0]
        F["j"][k:] = self.edges[:, 1]
        return F


def _relative(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """pose a in frame b (double)."""
    c, s = np.cos(b[..., 2]), np.sin(b[..., 2])
    dx, dy = a[..., 0] - b[..., 0], a[..., 1] - b[..., 1]
    th = np.arctan2(np.sin(a[..., 2] - b[..., 2]), np.cos(a[..., 2] - b[..., 2]))
    return np.stack([c * dx + s * dy, -s * dx + c * dy, th], -1)


def _compose(a: np.ndarray, d: np.ndarray) -> np.ndarray:
    c, s = math.cos(a[2]), math.sin(a[2])
    th = a[2] + d[2]
    return np.array([a[0] + c * d[0] - s * d[1], a[1] + s * d[0] + c * d[1], math.atan2(math.sin(th), math.cos(th))])


def loop_closure_pairs(est: np.ndarray, n: int, max_dist: float, min_sep: int) -> np.ndarray:
    """Reference distance rule (dpg_slam.cc:91-98): pairs (j, i), j < i - 1 (|i - j| >= min_sep),
    float32 ||p_j - p_i|| <= threshold; the n nearest pairs first (ties by (i, j))."""
    if n <= 0:
        return np.zeros((0, 2), np.int32)
    from scipy.spatial import cKDTree
    xy = est[:, :2].astype(np.float64)
    pairs = cKDTree(xy).query_pairs(max_dist * 1.0001, output_type="ndarray")
    if len(pairs) == 0:
        return np.zeros((0, 2), np.int32)
    j = np.minimum(pairs[:, 0], pairs[:, 1])
    i = np.maximum(pairs[:, 0], pairs[:, 1])
    sel = (i - j) >= max(min_sep, 2)
    i, j = i[sel], j[sel]
    d = est[j, :2].astype(np.float32) - est[i, :2].astype(np.float32)
    dist = np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]).astype(np.float32)
    ok = dist <= np.float32(max_dist)
    i, j, dist = i[ok], j[ok], dist[ok]
    order = np.lexsort((j, i, dist))[:n]
    return np.stack([j[order], i[order]], 1).astype(np.int32)


def generate(cfg: SynthConfig | str) -> Workload:
    if isinstance(cfg, str):
        cfg = CONFIGS[cfg]
    L = lib()
    segs = np.zeros((4096, 4), np.float32)
    ns = L.dpg_synth_world(cfg.seed, cfg.world_size, ptr(segs, C.c_float), len(segs))
    segs = np.ascontiguousarray(segs[:ns])
    V = cfg.n_nodes
    gt = np.zeros((V, 3), np.float64)
    _abi.check(L.dpg_synth_trajectory(cfg.seed, V, ptr(segs, C.c_float), ns, cfg.world_size, 1.0,
                                      ptr(gt, C.c_double)), "dpg_synth_trajectory")
    ranges = np.zeros((V, cfg.n_beams), np.float32)
    threads = cfg.threads or min(16, os.cpu_count() or 1)
    _abi.check(L.dpg_synth_scans(ptr(gt, C.c_double), V, ptr(segs, C.c_float), ns, cfg.n_beams, ANGLE_MIN,
                                 ANGLE_MAX, RANGE_MAX, LASER[0], LASER[1], LASER[2], cfg.range_noise,
                                 cfg.seed * 7919 + 1, threads, ptr(ranges, C.c_float)), "dpg_synth_scans")
    pts, offs = api.scans_to_clouds(ranges, ANGLE_MIN, ANGLE_MAX, RANGE_MAX, LASER)
    rng = np.random.default_rng(cfg.seed)
    rel = _relative(gt, gt[0])
    est = rel + np.concatenate([rng.normal(0, cfg.est_noise[0], (V, 2)), rng.normal(0, cfg.est_noise[1], (V, 1))], 1)
    est[0] = 0.0   # createNewPassFirstNode: (0, 0, 0)
    est = est.astype(np.float32)
    odom = np.zeros((V, 3), np.float64)
    for v in range(1, V):
        d = _relative(gt[v], gt[v - 1])
        d = d + np.array([rng.normal(0, cfg.odom_noise[0]), rng.normal(0, cfg.odom_noise[0]),
                          rng.normal(0, cfg.odom_noise[1])])
        odom[v] = _compose(odom[v - 1], d)
    odom = odom.astype(np.float32)
    succ = np.stack([np.arange(V - 1), np.arange(1, V)], 1).astype(np.int32)
    lc = loop_closure_pairs(est, cfg.n_loop_closures, cfg.lc_max_dist, cfg.lc_min_sep)
    edges = np.ascontiguousarray(np.concatenate([succ, lc], 0), np.int32)
    base = [api.prior_factor(0)]
    for v in range(1, V):
        f = api.odometry_factor(odom[v - 1], odom[v], v - 1, v)
        base.append(np.frombuffer(bytes(f), FACTOR_DTYPE).copy())
    base = np.concatenate(base).astype(FACTOR_DTYPE)
    return Workload(cfg=cfg, segs=segs, gt=gt, ranges=ranges, pts=pts, offsets=offs, est=est, odom=odom,
                    edges=edges, n_successive=len(succ), base_factors=base, icp_factor_first=len(base))


# ------------------------------------------------------------------ config 5 (dynamic passes)
@dataclass
class DynamicWorkload:
    """Multi-pass workload for DPG change detection (BASELINE config 5): one static world,
    a set of movable boxes of which each pass sees its own subset (boxes added or removed between
    passes), one trajectory per pass through the same area, exactly ray-cast scans per pass."""
    ranges: np.ndarray      # [V, n_beams] f32
    geom: np.ndarray        # [V, 3] f32: angle_min, angle_max, range_max
    est: np.ndarray         # [V, 3] f32 node poses (map frame = world frame)
    pass_of: np.ndarray     # [V] i32
    pass_start: np.ndarray  # [P + 1] first node of each pass
    boxes: np.ndarray       # [K, 4] x0, y0, x1, y1 of the movable boxes
    present: np.ndarray     # [P, K] bool

    @property
    def V(self) -> int:
        return len(self.est)


def _box_segs(b) -> list:
    x0, y0, x1, y1 = (float(v) for v in b)
    return [[x0, y0, x1, y0], [x1, y0, x1, y1], [x1, y1, x0, y1], [x0, y1, x0, y0]]


def make_dynamic(n_passes: int = 4, nodes_per_pass: int = 2500, n_beams: int = 5000, seed: int = 5,
                 world_size: float = 40.0, range_max: float = RANGE_MAX, n_boxes: int = 24,
                 range_noise: float = 0.01, threads: int = 0, fov_deg: float = 360.0,
                 p_add: float | None = None, p_remove: float | None = None) -> DynamicWorkload:
    """fov_deg: scan span centred on the laser's heading (360: ANGLE_MIN..ANGLE_MAX).  Box dynamics:
    by default each later pass flips about a third of the boxes in or out; with p_add / p_remove an
    absent box appears with probability p_add and a present one disappears with p_remove."""
    L = lib()
    segs = np.zeros((4096, 4), np.float32)
    ns = L.dpg_synth_world(seed, world_size, ptr(segs, C.c_float), len(segs))
    static = segs[:ns]
    rng = np.random.default_rng(seed)
    boxes = []
    for _ in range(n_boxes):
        w, h = rng.uniform(0.4, 1.2, 2)
        x, y = rng.uniform(2.0, world_size - 2.0 - 1.2, 2)
        boxes.append([x, y, x + w, y + h])
    boxes = np.asarray(boxes, np.float32)
    present = np.zeros((n_passes, n_boxes), bool)
    present[0] = rng.random(n_boxes) < 0.5
    for p in range(1, n_passes):   # each later pass moves about a third of the boxes in or out
        if p_add is None and p_remove is None:
            flip = rng.random(n_boxes) < 0.33
        else:
            u = rng.random(n_boxes)
            flip = np.where(present[p - 1], u < (p_remove or 0.0), u < (p_add or 0.0))
        present[p] = present[p - 1] ^ flip
    all_segs = np.ascontiguousarray(np.concatenate([static, np.asarray(sum((_box_segs(b) for b in boxes), []),
                                                                       np.float32)]), np.float32)
    threads = threads or min(16, os.cpu_count() or 1)
    if fov_deg >= 360.0:
        amin, amax = ANGLE_MIN, ANGLE_MAX
    else:
        amin, amax = -math.radians(fov_deg) / 2.0, math.radians(fov_deg) / 2.0
    gts, rs = [], []
    for p in range(n_passes):
        gt = np.zeros((nodes_per_pass, 3), np.float64)
        _abi.check(L.dpg_synth_trajectory(seed * 131 + p, nodes_per_pass, ptr(all_segs, C.c_float), len(all_segs),
                                          world_size, 1.0, ptr(gt, C.c_double)), "dpg_synth_trajectory")
        bs = [s for k in range(n_boxes) if present[p, k] for s in _box_segs(boxes[k])]
        world = np.ascontiguousarray(np.concatenate([static, np.asarray(bs, np.float32).reshape(-1, 4)]), np.float32)
        r = np.zeros((nodes_per_pass, n_beams), np.float32)
        _abi.check(L.dpg_synth_scans(ptr(gt, C.c_double), nodes_per_pass, ptr(world, C.c_float), len(world), n_beams,
                                     amin, amax, range_max, LASER[0], LASER[1], LASER[2], range_noise,
                                     seed * 7919 + 17 * p + 1, threads, ptr(r, C.c_float)), "dpg_synth_scans")
        gts.append(gt)
        rs.append(r)
    V = n_passes * nodes_per_pass
    geom = np.tile(np.array([amin, amax, range_max], np.float32), (V, 1))
    return DynamicWorkload(ranges=np.concatenate(rs), geom=geom, est=np.concatenate(gts).astype(np.float32),
                           pass_of=np.repeat(np.arange(n_passes, dtype=np.int32), nodes_per_pass),
                           pass_start=np.arange(n_passes + 1, dtype=np.int64) * nodes_per_pass,
                           boxes=boxes, present=present)


# ------------------------------------------------------------------ config 5 (patrol passes)
@dataclass
class PatrolWorkload:
    """BASELINE config 5 as a DpgSLAM run: a building of rooms x rooms rooms (2 m doors at the wall
    centres), furniture and movable boxes kept off the room centre lines, and n_passes passes that
    all start at the same pose and follow the same serpentine patrol route through every room
    (dpg_slam's passes start where pass 0 started: createNewPassFirstNode puts each pass's first
    node at the map origin).  Between passes movable boxes appear (p_add) or disappear (p_remove).
    Per pass: ground truth, odometry readings (noisy increments integrated from (0, 0, 0)) and one
    ray-cast scan per reading."""
    segs: np.ndarray        # static world segments
    boxes: np.ndarray       # [K, 4] movable boxes
    present: np.ndarray     # [P, K] bool
    gt: np.ndarray          # [P, N, 3] world frame (f64)
    odom: np.ndarray        # [P, N, 3] odometry readings (f32)
    ranges: np.ndarray      # [P * N, n_beams] f32
    geom: np.ndarray        # [P * N, 3] angle_min, angle_max, range_max

    @property
    def n_passes(self) -> int:
        return self.gt.shape[0]

    @property
    def steps(self) -> int:
        return self.gt.shape[1]

    def gt_map(self) -> np.ndarray:
        """Ground truth in the map frame (pass 0's start pose), [P, N, 3]."""
        return _relative(self.gt, self.gt[0, 0])


def _patrol_world(rooms: int, cell: float, rng, n_movable: int, lane: float):
    W = rooms * cell
    segs = [[0, 0, W, 0], [W, 0, W, W], [W, W, 0, W], [0, W, 0, 0]]
    for k in range(1, rooms):
        c = k * cell
        for m in range(rooms):
            a0, mid, a1 = m * cell, m * cell + cell / 2.0, (m + 1) * cell
            segs += [[c, a0, c, mid - 1.0], [c, mid + 1.0, c, a1], [a0, c, mid - 1.0, c], [mid + 1.0, c, a1, c]]

    def off_lane_box(r, c, hmax):
        cx, cy = (c + 0.5) * cell, (r + 0.5) * cell
        qx, qy = rng.choice([-1.0, 1.0], 2)
        h = rng.uniform(0.2, hmax, 2)
        lo, hi = lane + h + 0.2, cell / 2.0 - h - 0.4
        x = cx + qx * rng.uniform(lo[0], max(lo[0], hi[0]))
        y = cy + qy * rng.uniform(lo[1], max(lo[1], hi[1]))
        return [x - h[0], y - h[1], x + h[0], y + h[1]]

    for r in range(rooms):
        for c in range(rooms):
            for _ in range(2):
                segs += _box_segs(off_lane_box(r, c, 0.6))
    cells = rng.choice(rooms * rooms, size=min(n_movable, rooms * rooms), replace=False)
    boxes = np.asarray([off_lane_box(int(q) // rooms, int(q) % rooms, 0.5) for q in cells], np.float32).reshape(-1, 4)
    return np.asarray(segs, np.float32), boxes


def _serpentine(rooms: int, cell: float) -> np.ndarray:
    pts = []
    for r in range(rooms):
        cols = range(rooms) if r % 2 == 0 else range(rooms - 1, -1, -1)
        pts += [((c + 0.5) * cell, (r + 0.5) * cell) for c in cols]
    return np.asarray(pts, np.float64)


def make_patrol(n_passes: int = 4, steps: int = 2500, n_beams: int = 5000, rooms: int = 16, cell: float = 10.5,
                step: float = 1.05, fov_deg: float = 270.0, range_max: float = RANGE_MAX, range_noise: float = 0.002,
                n_movable: int = 64, p_add: float = 0.3, p_remove: float = 0.15, lateral: float = 0.35,
                odom_noise: tuple = (0.01, 0.003), seed: int = 5, threads: int = 0) -> PatrolWorkload:
    rng = np.random.default_rng(seed)
    static, boxes = _patrol_world(rooms, cell, rng, n_movable, lane=1.5)
    K = len(boxes)
    present = np.zeros((n_passes, K), bool)
    present[0] = rng.random(K) < 0.5
    for p in range(1, n_passes):
        u = rng.random(K)
        present[p] = present[p - 1] ^ np.where(present[p - 1], u < p_remove, u < p_add)
    # the route, sampled every `step` m of arc length
    way = _serpentine(rooms, cell)
    seg = np.diff(way, axis=0)
    seg_len = np.linalg.norm(seg, axis=1)
    cum = np.concatenate([[0.0], np.cumsum(seg_len)])
    if cum[-1] < step * steps:
        raise ValueError(f"route of {cum[-1]:.0f} m is shorter than {steps} steps of {step} m")
    amin, amax = (ANGLE_MIN, ANGLE_MAX) if fov_deg >= 360.0 else (-math.radians(fov_deg) / 2, math.radians(fov_deg) / 2)
    threads = threads or min(16, os.cpu_count() or 1)
    gts, odoms, rs = [], [], []
    for p in range(n_passes):
        s = np.arange(steps) * step
        k = np.minimum(np.searchsorted(cum, s, side="right") - 1, len(seg) - 1)
        d = seg[k] / seg_len[k, None]
        base = way[k] + d * (s - cum[k])[:, None]
        ph = rng.uniform(0, 2 * np.pi, 2)
        off = lateral * (0.6 * np.sin(2 * np.pi * s / 23.0 + ph[0]) + 0.4 * np.sin(2 * np.pi * s / 7.0 + ph[1]))
        off[0] = 0.0   # every pass starts at the same pose
        nrm = np.stack([-d[:, 1], d[:, 0]], 1)
        xy = base + nrm * off[:, None]
        th = np.arctan2(d[:, 1], d[:, 0]) + np.concatenate([[0.0], rng.normal(0, 0.02, steps - 1)])
        gt = np.concatenate([xy, th[:, None]], 1)
        od = np.zeros((steps, 3))
        for v in range(1, steps):
            inc = _relative(gt[v], gt[v - 1]) + np.array([rng.normal(0, odom_noise[0]), rng.normal(0, odom_noise[0]),
                                                          rng.normal(0, odom_noise[1])])
            od[v] = _compose(od[v - 1], inc)
        bs = [q for b in range(K) if present[p, b] for q in _box_segs(boxes[b])]
        world = np.ascontiguousarray(np.concatenate([static, np.asarray(bs, np.float32).reshape(-1, 4)]), np.float32)
        r = np.zeros((steps, n_beams), np.float32)
        gtc = np.ascontiguousarray(gt)
        _abi.check(lib().dpg_synth_scans(ptr(gtc, C.c_double), steps, ptr(world, C.c_float), len(world), n_beams, amin,
                                         amax, range_max, LASER[0], LASER[1], LASER[2], range_noise,
                                         seed * 7919 + 17 * p + 1, threads, ptr(r, C.c_float)), "dpg_synth_scans")
        gts.append(gt)
        odoms.append(od.astype(np.float32))
        rs.append(r)
    V = n_passes * steps
    geom = np.tile(np.array([amin, amax, range_max], np.float32), (V, 1))
    return PatrolWorkload(segs=static, boxes=boxes, present=present, gt=np.stack(gts), odom=np.stack(odoms),
                          ranges=np.concatenate(rs), geom=geom)
