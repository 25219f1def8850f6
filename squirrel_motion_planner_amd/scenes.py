"""Scene inputs for the BASELINE.json configurations, as occupied octomap keys.

A scene here is what the reference's node hands to setOctree() (squirrel_8dof_planner.cpp:862-917): a set
of occupied leaf voxels at resolution `res` in octomap key space (key = floor(coord / res) + 32768), plus
the floor square the node inserts around the robot (squirrel_8dof_planner.cpp:889-902).  The synthetic
generators are seeded and deterministic; data="synthetic" in bench.py.

  C1  empty 5 m x 5 m map (floor only)                                   -> empty_room()
  C2  10 x 10 x 2 m @ 5 cm, 20 axis-aligned boxes, seed 42              -> box_room()
  C4  narrow passage: wall at x = 0 with a 0.24 m slot at z 0.55-0.79   -> narrow_passage()
  C5  2 cm dense clutter from a 2e6-point synthetic cloud, seed 11       -> clutter_cloud()
"""
import math

import numpy as np

KEY_OFFSET = 32768

# Reference start/goal material: pose_folded_arm (parameters.yaml:38) and the last keyframe of the
# tuw-robotino2 folding trajectory (folding_poses_tuw-robotino2.yaml), an unfolded arm.
ARM_FOLDED = [-0.7, 1.9, 0.0, 1.7, 0.0]
ARM_UNFOLDED = [-0.707011701539749, 1.6149626484476989, 0.19002285249790796, 1.7589609723317974, 0.183945523562212]
ARM_REACH = [0.6, 0.9, 0.4, 0.8, 0.0]
# The first keyframe of folding_poses_tuw-robotino2.yaml, SURVEY C1's start ("folded arm"): the stowed hand rests its
# fingers inside the front shell's box primitive (robotino_plan.urdf:323-329), so the start is in self-collision --
# for the reference as well (its FCL box vs the hand meshes of squirrel-hand.dae, tools/gen_robot_model.py validate).
ARM_STOWED = [0.29201350928033476, 2.2600188129288705, 0.19001033369874476, -1.1680354608387098, 0.5320232345529955]


def coord_to_key(c, res):
    """octomap OcTreeBaseImpl::coordToKey: floor(resolution_factor * c) + 32768, resolution_factor = 1.0 / res."""
    return np.floor((1.0 / res) * np.asarray(c, np.float64)).astype(np.int64) + KEY_OFFSET


def _box_keys(lo, hi, res):
    """Keys of all voxels whose centre lies in [lo, hi) (metric, octree frame)."""
    klo = np.ceil(np.asarray(lo) / res - 0.5).astype(np.int64)
    khi = np.ceil(np.asarray(hi) / res - 0.5).astype(np.int64)
    if np.any(khi <= klo):
        return np.zeros((0, 3), np.int64)
    ax = [np.arange(klo[d], khi[d]) for d in range(3)]
    g = np.stack(np.meshgrid(*ax, indexing="ij"), -1).reshape(-1, 3)
    return g + KEY_OFFSET


def floor_keys(center_xy, res, distance=3.0):
    """squirrel_8dof_planner.cpp:889-902: a (2n+1)^2 key square at z-key(-res/2) around the robot."""
    k = coord_to_key([center_xy[0], center_xy[1], -res * 0.5], res)
    n = int(distance / res)
    xs = np.arange(k[0] - n, k[0] + n + 1)
    ys = np.arange(k[1] - n, k[1] + n + 1)
    g = np.stack(np.meshgrid(xs, ys, indexing="ij"), -1).reshape(-1, 2)
    return np.concatenate([g, np.full((len(g), 1), k[2])], 1)


def _walls(half_x, half_y, height, res, thick=0.1):
    return np.concatenate([
        _box_keys([-half_x - thick, -half_y - thick, 0.0], [-half_x, half_y + thick, height], res),
        _box_keys([half_x, -half_y - thick, 0.0], [half_x + thick, half_y + thick, height], res),
        _box_keys([-half_x, -half_y - thick, 0.0], [half_x, -half_y, height], res),
        _box_keys([-half_x, half_y, 0.0], [half_x, half_y + thick, height], res)])


def _unique(keys):
    keys = np.asarray(keys, np.int64).reshape(-1, 3)
    return np.unique(keys, axis=0)


class Scene:
    def __init__(self, name, keys, res, start, goal, env_x, env_y):
        self.name = name
        self.keys = _unique(keys)
        self.res = float(res)
        self.start = list(map(float, start))
        self.goal = list(map(float, goal))
        self.env_x = tuple(env_x)
        self.env_y = tuple(env_y)

    def bounds(self):
        """octree->getMetricMin/Max x,y (the env bounds of setPlanningSceneInfo, SP:1226-1232)."""
        if len(self.keys) == 0:
            return (0.0, 0.0), (0.0, 0.0)
        lo = (self.keys.min(0) - KEY_OFFSET) * self.res
        hi = (self.keys.max(0) - KEY_OFFSET + 1) * self.res
        return (float(lo[0]), float(hi[0])), (float(lo[1]), float(hi[1]))


def empty_room(res=0.05, stowed=False):
    """C1: empty 5 m x 5 m map, floor only (plumbing).  stowed=True: SURVEY's start (ARM_STOWED, in self-collision:
    init_planner fails, birrt_star.cpp:353-357); else pose_folded_arm (parameters.yaml:38)."""
    start = [0.0, 0.0, 0.0] + (ARM_STOWED if stowed else ARM_FOLDED)
    goal = [1.5, 1.0, 1.2] + ARM_UNFOLDED
    keys = floor_keys(start[:2], res, 2.5)
    s = Scene("C1-empty-5m", keys, res, start, goal, (0, 0), (0, 0))
    s.env_x, s.env_y = s.bounds()
    return s


def box_room(seed=42, res=0.05, n_boxes=20, start=None, goal=None):
    """C2: 10 x 10 x 2 m room (walls), 20 boxes xy U(0.2,1.0) m, height U(0.3,1.5) m, floor around start."""
    start = start or ([-3.0, -3.0, 0.0] + ARM_FOLDED)
    goal = goal or ([3.0, 3.0, 1.57] + ARM_UNFOLDED)
    rng = np.random.default_rng(seed)
    parts = [_walls(5.0, 5.0, 2.0, res), floor_keys(start[:2], res, 3.0)]
    placed = 0
    while placed < n_boxes:
        sx, sy = rng.uniform(0.2, 1.0, 2)
        h = rng.uniform(0.3, 1.5)
        cx, cy = rng.uniform(-5.0 + sx / 2, 5.0 - sx / 2), rng.uniform(-5.0 + sy / 2, 5.0 - sy / 2)
        near = False
        for p in (start, goal):
            dx = max(abs(cx - p[0]) - sx / 2, 0.0)
            dy = max(abs(cy - p[1]) - sy / 2, 0.0)
            if math.hypot(dx, dy) < 0.8:
                near = True
        if near:
            continue
        parts.append(_box_keys([cx - sx / 2, cy - sy / 2, 0.0], [cx + sx / 2, cy + sy / 2, h], res))
        placed += 1
    s = Scene("C2-boxes-10m-5cm", np.concatenate(parts), res, start, goal, (0, 0), (0, 0))
    s.env_x, s.env_y = s.bounds()
    return s


def narrow_passage(res=0.05, slot=0.24):
    """C4: wall at x = 0 with a slot `slot` m wide (2 x ~0.12 m arm-link width) at z 0.55-0.79.

    Start: folded arm 0.9 m in front of the wall.  Goal: the wrist inside the slot (hand_wrist_link at x 0.031,
    y -0.052, z 0.597), one of the 8 collision-free configurations of 1e6 random ones with the wrist in the slot
    (rejection sampling with the oracle, seed 4); the straight start->goal edge collides, so the query is planned,
    not connected directly (birrt_star.cpp:1072-1075)."""
    start = [-0.9, 0.0, 0.0] + ARM_FOLDED
    goal = [-0.391, -0.227, 1.184, -0.799, -0.055, 1.581, -0.13, 1.613]
    wall = _box_keys([0.0, -5.0, 0.0], [0.1, 5.0, 2.0], res)
    rel = (wall - KEY_OFFSET + 0.5) * res
    hole = (np.abs(rel[:, 1]) < slot / 2) & (rel[:, 2] > 0.55) & (rel[:, 2] < 0.79)
    keys = np.concatenate([_walls(5.0, 5.0, 2.0, res), wall[~hole], floor_keys(start[:2], res, 3.0)])
    s = Scene("C4-narrow-passage", keys, res, start, goal, (0, 0), (0, 0))
    s.env_x, s.env_y = s.bounds()
    return s


def clutter_cloud(seed=11, res=0.02, n_points=2_000_000):
    """C5: 10 x 10 x 2 m @ 2 cm from a synthetic cloud: clustered boxes + uniform noise, voxelised."""
    rng = np.random.default_rng(seed)
    start = [-3.0, -3.0, 0.0] + ARM_FOLDED
    goal = [3.0, 3.0, 1.57] + ARM_UNFOLDED
    n_cl = 60
    centers = np.column_stack([rng.uniform(-4.5, 4.5, n_cl), rng.uniform(-4.5, 4.5, n_cl), rng.uniform(0.1, 1.6, n_cl)])
    sizes = rng.uniform(0.05, 0.5, (n_cl, 3))
    keep = np.ones(n_cl, bool)
    for p in (start, goal):
        keep &= np.hypot(centers[:, 0] - p[0], centers[:, 1] - p[1]) > 1.0
    centers, sizes = centers[keep], sizes[keep]
    n_clust = int(n_points * 0.95)
    idx = rng.integers(0, len(centers), n_clust)
    pts = centers[idx] + (rng.uniform(-0.5, 0.5, (n_clust, 3)) * sizes[idx])
    noise = np.column_stack([rng.uniform(-5, 5, n_points - n_clust), rng.uniform(-5, 5, n_points - n_clust),
                             rng.uniform(0, 2, n_points - n_clust)])
    pts = np.concatenate([pts, noise])
    for p in (start, goal):  # keep the robot's own footprint clear of noise
        pts = pts[np.hypot(pts[:, 0] - p[0], pts[:, 1] - p[1]) > 0.9]
    keys = coord_to_key(pts, res)
    keys = np.concatenate([keys, _walls(5.0, 5.0, 2.0, res), floor_keys(start[:2], res, 3.0)])
    s = Scene("C5-clutter-2cm", keys, res, start, goal, (0, 0), (0, 0))
    s.env_x, s.env_y = s.bounds()
    return s


def random_queries(scene, n, seed=7, check=None, max_tries=100000):
    """C3: n (start, goal) pairs sampled with seed 7; `check(q) -> bool valid` filters invalid ones."""
    rng = np.random.default_rng(seed)
    (x0, x1), (y0, y1) = scene.env_x, scene.env_y
    out = []
    tries = 0
    while len(out) < n and tries < max_tries:
        tries += 1
        pair = []
        for arm in (ARM_FOLDED, ARM_UNFOLDED):
            q = [rng.uniform(x0 + 0.5, x1 - 0.5), rng.uniform(y0 + 0.5, y1 - 0.5), rng.uniform(-math.pi, math.pi)] + list(arm)
            pair.append(q)
        if check is None or (check(pair[0]) and check(pair[1])):
            out.append(pair)
    return out
