"""CPU tests of the node-side host entry points (§8f rows 1-2): octomap full format (.ot) and octomap_msgs payloads
-> scene, the floor insertion over free leaves, and Planner::normalizeTrajectory.  Parity: the .ot fixtures are
the reference's own maps (config/room{3,4,5}.ot, copied to tests/golden/); their occupied leaves must equal the
keys decoded from the reference's room{3,4,5}.bt (tests/golden/room*_keys.npz).  Synthetic trees come from the
oracle writer (oracle/octomap_bt.py); normalizeTrajectory is checked bit for bit against oracle/trajectory.py."""
import os

import numpy as np
import pytest

from oracle import octomap_bt, trajectory as OT
from squirrel_motion_planner_amd import _lib as L
from squirrel_motion_planner_amd import scenes
from squirrel_motion_planner_amd.planner import BiRRTstarPlanner, Scene, normalize_trajectory

GOLD = os.path.join(os.path.dirname(__file__), "golden")
KEY = 32768


def _same(a, b):
    (ba, da), (bb, db) = a.export(), b.export()
    assert a.info()["dims"] == b.info()["dims"] and a.info()["origin"] == b.info()["origin"]
    assert np.array_equal(ba, bb) and np.array_equal(da, db)


def _keyset(k):
    return set(map(tuple, np.asarray(k, np.int64).reshape(-1, 3).tolist()))


@pytest.mark.parametrize("room", ["room3", "room4", "room5"])
def test_ot_fixture_equals_bt_keys(room):
    data = open(os.path.join(GOLD, room + ".ot"), "rb").read()
    keys = np.load(os.path.join(GOLD, room + "_keys.npz"))["keys"].astype(np.int64)
    res, occ, free = octomap_bt.read_ot(data)
    assert res == 0.05 and not free
    assert _keyset(occ) == _keyset(keys)                       # oracle reader vs the .bt fixture
    _same(Scene.from_ot(data), Scene.from_keys(keys, 0.05))    # product reader
    # with the node's floor (squirrel_8dof_planner.cpp:886-904) at a robot pose
    fc = (0.5, -1.0)
    _same(Scene.from_ot(data, floor_center=fc), Scene.from_keys(np.concatenate([keys, scenes.floor_keys(fc, 0.05)]), 0.05))


def _covers(d, k, q):
    return all(k[a] - (KEY >> d) <= q[a] < k[a] - (KEY >> d) + ((2 * KEY) >> d) for a in range(3))


def _synthetic_tree():
    """Occupied / free leaves at depth 16 and pruned ones (depth 15: 2^3 voxels, depth 14: 4^3 voxels; centre keys
    as octomap's computeChildKey makes them), free ones across the floor plane z-key 32767."""
    big = [(15, (KEY + 21, KEY + 31, KEY + 11), np.float32(3.5)),       # keys +20..21, +30..31, +10..11
           (14, (KEY - 6, KEY + 10, KEY - 2), np.float32(-1.5))]        # keys -8..-5, +8..+11, -4..-1: holds z 32767
    rng = np.random.default_rng(3)
    leaves = list(big)
    seen = set()
    for _ in range(60):
        k = KEY + rng.integers(-40, 40, 3)
        k[2] = KEY + rng.integers(0, 20)
        k = tuple(int(v) for v in k)
        if k in seen or any(_covers(d, c, k) for d, c, _ in big):
            continue
        seen.add(k)
        leaves.append((16, k, np.float32(rng.uniform(0.0, 3.5))))
    # free depth-16 leaves on the floor plane: one stays free after a hit, one turns occupied; one off the floor
    leaves += [(16, (KEY + 3, KEY + 4, KEY - 1), np.float32(-2.0)), (16, (KEY + 5, KEY + 4, KEY - 1), np.float32(-0.5)),
               (16, (KEY + 7, KEY + 4, KEY + 22), np.float32(-2.0))]
    return leaves


def test_ot_synthetic_with_free_leaves_and_floor():
    leaves = _synthetic_tree()
    data = octomap_bt.write_ot(leaves, 0.05)
    res, occ, free = octomap_bt.read_ot(data)
    want = _keyset([k for d, k, v in leaves if d == 16 and v >= 0]) | {
        (KEY + 20 + dx, KEY + 30 + dy, KEY + 10 + dz) for dx in (0, 1) for dy in (0, 1) for dz in (0, 1)}
    assert _keyset(occ) == want and len(free) == 4
    _same(Scene.from_ot(data), Scene.from_keys(occ, 0.05))
    fc = (0.12, 0.31)
    floor = octomap_bt.floor_keys(fc, 0.05, 1.0, free)
    fs = _keyset(floor)
    assert (KEY + 3, KEY + 4, KEY - 1) not in fs and (KEY + 5, KEY + 4, KEY - 1) in fs
    assert (KEY - 8, KEY + 8, KEY - 1) not in fs and (KEY - 5, KEY + 11, KEY - 1) not in fs
    assert (KEY - 9, KEY + 8, KEY - 1) in fs and (KEY - 4, KEY + 8, KEY - 1) in fs
    _same(Scene.from_ot(data, floor_center=fc, floor_distance=1.0),
          Scene.from_keys(np.concatenate([occ, floor]), 0.05))
    # without free leaves the oracle floor is the plain square of scenes.floor_keys
    assert _keyset(octomap_bt.floor_keys(fc, 0.05, 1.0)) == _keyset(scenes.floor_keys(fc, 0.05, 1.0))


def test_octomap_msg_payloads():
    leaves = _synthetic_tree()
    full = octomap_bt.write_ot(leaves, 0.05, header=False)
    _same(Scene.from_octomap_msg("OcTree", 0.05, False, full), Scene.from_ot(octomap_bt.write_ot(leaves, 0.05)))
    keys = np.load(os.path.join(GOLD, "room4_keys.npz"))["keys"].astype(np.int64)
    bt = octomap_bt.write_bt(keys, 0.05)
    payload = bt[bt.index(b"\ndata\n") + 6:]
    fc = (1.0, 2.0)
    _same(Scene.from_octomap_msg("OcTree", 0.05, True, payload, floor_center=fc), Scene.from_bt(bt, floor_center=fc))
    empty = Scene.from_octomap_msg("OcTree", 0.1, True, b"")
    assert empty.info()["n_occupied"] == 0
    with pytest.raises(L.SmpError) as e:
        Scene.from_octomap_msg("ColorOcTree", 0.05, False, full)   # dynamic_cast<OcTree*> fails in the node
    assert e.value.status == L.SMP_ERR_PARSE
    with pytest.raises(L.SmpError):
        Scene.from_octomap_msg("OcTree", 0.05, False, full[:-3])   # truncated


def test_ot_parse_errors_and_shim_dispatch():
    with pytest.raises(L.SmpError):
        Scene.from_ot(b"# Octomap OcTree file\nid OcTree\nsize 1\nres 0.05\ndata\n\x00\x00")
    with pytest.raises(L.SmpError):
        Scene.from_ot(b"# Octomap OcTree file\nid OcTree\nsize 1\n")
    # BiRRTstarPlanner.setOctree picks the format from the first line (needs no GPU up to the upload)
    data = open(os.path.join(GOLD, "room5.ot"), "rb").read()
    assert data.startswith(b"# Octomap OcTree file")


def _wrap(a):
    return (a + np.pi) % (2 * np.pi) - np.pi


def _check_norm(raw, npose):
    a = normalize_trajectory(raw, npose)
    b = OT.normalize_trajectory([list(r) for r in raw], list(npose))
    if b is None:
        assert a is None
        return a
    assert a.shape == (len(b), len(npose))
    assert np.array_equal(a, np.array(b)), np.abs(a - np.array(b)).max()
    return a


def test_normalize_trajectory_matches_oracle():
    rng = np.random.default_rng(11)
    npose = [0.02, 0.02, 0.08, 0.08, 0.08, 0.08, 0.08, 0.08]   # parameters.yaml:41
    for _ in range(40):
        n = int(rng.integers(2, 12))
        raw = np.cumsum(rng.normal(0, 0.15, (n, 8)), 0)
        raw[:, 2] = _wrap(rng.uniform(-4, 4) + np.cumsum(rng.normal(0, 1.2, n)))  # theta across +-pi
        if rng.random() < 0.3:
            raw[1:, 2] += rng.choice([-2 * np.pi, 2 * np.pi])   # unwrapped input (the wrap at 1564-1572)
        out = _check_norm(raw, npose)
        assert np.all(np.abs(out[:, 2]) <= np.pi + 1e-12)
        np.testing.assert_array_equal(out[0], np.where(np.abs(raw[0]) > 10, raw[0], out[0]))
    # 5-DoF folding keyframes (squirrel_8dof_planner.cpp:60-67): no angular special case
    for _ in range(10):
        raw = rng.uniform(-2, 2, (int(rng.integers(2, 6)), 5))
        _check_norm(raw, [0.08] * 5)


def test_normalize_trajectory_edge_cases():
    npose = [0.5] * 8
    assert _check_norm(np.zeros((1, 8)), npose) is None          # <= 1 pose: output untouched
    assert normalize_trajectory(np.zeros((3, 8)), [0.5] * 5) is None   # dimension mismatch
    # all poses within one normalized distance: first and last only
    raw = np.zeros((4, 8)); raw[:, 0] = [0, 0.1, 0.2, 0.3]
    assert _check_norm(raw, npose).shape == (2, 8)
    # an exact multiple of the distance: (UInt)frac + 1 samples at step 1 / ceil(frac) (one past the pose)
    raw = np.zeros((2, 8)); raw[1, 0] = 1.0
    out = _check_norm(raw, npose)
    assert out.shape == (4, 8) and out[-1, 0] == 1.5
    # theta crossing +-pi takes the short way round
    raw = np.zeros((2, 8)); raw[0, 2] = 3.0; raw[1, 2] = -3.0
    out = _check_norm(raw, npose)
    assert np.all(np.abs(out[:, 2]) >= 3.0 - 1e-12)
    with pytest.raises(L.SmpError):
        normalize_trajectory(np.ones((2, 8)) * [[0], [1]], [0.0] * 8)   # 0/0: refused, not UB
