"""The C++ drop-in shim (include/smp_birrt_star.hpp) compiled with g++ and driven through the node's call
sequence (tests/cpp/shim_plan.cpp).  CPU: it builds, links libsmp_gpu.so and fails loudly without a GPU.
GPU: the trajectory it returns equals the oracle's for the same scene, seed and budget."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from oracle import octomap_bt, oracle as O
from squirrel_motion_planner_amd import scenes

LIBDIR = os.path.join(ROOT, "squirrel_motion_planner_amd", "lib")
MODEL = os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json")
URDF = os.path.join(ROOT, "tests", "golden", "robotino_plan.urdf")  # the node's robot description (+ .srdf beside it)


def build_shim(tmpdir):
    exe = os.path.join(str(tmpdir), "shim_plan")
    cmd = ["g++", "-std=c++11", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cpp", "shim_plan.cpp"), "-L", LIBDIR, "-lsmp_gpu",
           "-Wl,-rpath," + LIBDIR, "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def room3_case(tmpdir):
    f = np.load(os.path.join(ROOT, "tests", "golden", "room3_keys.npz"))
    keys = np.concatenate([f["keys"].astype(np.int64), scenes.floor_keys([0.0, 0.0], 0.05, 3.0)])
    bt = os.path.join(str(tmpdir), "room3_floor.bt")
    open(bt, "wb").write(octomap_bt.write_bt(keys, 0.05))
    sc = scenes.Scene("room3", keys, 0.05, [0.3, -0.4, 0.0] + scenes.ARM_FOLDED,
                      [1.4, 1.1, 1.2] + scenes.ARM_UNFOLDED, (0, 0), (0, 0))
    sc.env_x, sc.env_y = sc.bounds()
    return sc, bt


def run_shim(exe, model, bt, sc, iters, seed):
    args = [exe, model, bt, str(iters), str(seed)] + ["%.17g" % v for v in list(sc.start) + list(sc.goal)]
    args += ["%.17g" % v for v in list(sc.env_x) + list(sc.env_y)]
    return subprocess.run(args, capture_output=True, text=True, timeout=300)


def test_shim_builds_and_fails_loudly_without_gpu(tmp_path):
    exe = build_shim(tmp_path)
    sc, bt = room3_case(tmp_path)
    p = run_shim(exe, URDF, bt, sc, 10, 1)
    if p.returncode == 3:  # no GPU here: the shim throws, no CPU fallback
        assert "no usable GPU" in p.stdout or "NO_DEVICE" in p.stdout.upper(), p.stdout
    else:
        assert p.returncode == 0, p.stderr


@pytest.mark.gpu
def test_shim_node_sequence_matches_oracle(tmp_path):
    exe = build_shim(tmp_path)
    sc, bt = room3_case(tmp_path)
    iters, seed = 200, 5
    p = run_shim(exe, URDF, bt, sc, iters, seed)  # initialize() builds the robot from the URDF + SRDF text
    assert p.returncode == 0, p.stdout + p.stderr
    lines = p.stdout.splitlines()
    assert lines[0] in ("status 0", "status 1")
    n = int(lines[1].split()[1])
    checked = int(lines[1].split()[3])
    path = np.array([[float(v) for v in ln.split()] for ln in lines[2:2 + n]]).reshape(-1, 8)
    assert lines[2 + n] == "dim_mismatch_rejected 1"
    assert lines[3 + n] == "start_valid 1"
    res, keys = octomap_bt.read_bt(open(bt, "rb").read())
    orc = O.Oracle(O.OracleRobot(MODEL), O.OracleScene(keys, res))
    # findGoalPose / getFullPoseFromEEPose through the shim
    ee = [sc.start[0] + 0.6, sc.start[1] + 0.2, 0.5, 1.57, 0.0, 0.3]
    gs = lines[4 + n].split()
    ores, opose, _, _, _ = orc.find_goal_pose(ee, sc.start, 20.0, True, True)
    assert gs[0] == "goal_search" and int(gs[1]) == ores
    if ores == 0:
        assert np.array_equal(np.array([float(v) for v in gs[2:]]), opose)
    ik = lines[5 + n].split()
    init = [ee[0] - 0.47, ee[1], 0.99, -1.2, 1.1, 0.0, 0.7, -1.5]
    oi = orc.ik_solve(O.ik_tasks(ee, [init]))
    assert ik[0] == "ee_ik" and int(ik[1]) == oi["reached"][0]
    if oi["reached"][0]:
        assert np.array_equal(np.array([float(v) for v in ik[2:]]), oi["q"][0])
    # getCollisions (SP:839) of three probes: the start, its arm at the upper joint limits, the map's corner
    probes = [list(sc.start) for _ in range(3)]
    probes[1][3:8] = [1.5, 2.6, 1.8, 2.4, 2.9]
    probes[2][0], probes[2][1] = sc.env_x[1], sc.env_y[1]
    for k, q in enumerate(probes):
        f = lines[6 + n + k].split()
        assert f[0] == "collisions"
        ns, nm = int(f[1]), int(f[2])
        got_self = [(f[3 + 2 * i], f[4 + 2 * i]) for i in range(ns)]
        got_map = f[3 + 2 * ns:3 + 2 * ns + nm]
        want_self, want_map = orc.collisions(q)
        assert got_self == want_self and got_map == want_map, (k, got_self, got_map, want_self, want_map)
    o = orc.plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, max_iter=iters, seed=seed)
    assert lines[0] == "status %d" % o["status"]
    assert checked == o["checked"]
    assert path.shape == o["path"].reshape(-1, 8).shape
    assert np.array_equal(path, o["path"].reshape(-1, 8))


def test_shim_normalize_trajectory_matches_oracle(tmp_path):
    """smp_node::normalizeTrajectory (the node's Planner::normalizeTrajectory, SP:1557-1637) through the C++ shim,
    bit for bit against oracle/trajectory.py; host only, no GPU."""
    from oracle import trajectory as OT
    exe = os.path.join(str(tmp_path), "shim_normalize")
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "shim_normalize.cpp"), "-L", LIBDIR, "-lsmp_gpu",
                    "-Wl,-rpath," + LIBDIR, "-o", exe], check=True, capture_output=True, text=True)
    rng = np.random.default_rng(2)
    cases = []
    for k in range(12):
        dim = 8 if k % 3 else 5
        n = int(rng.integers(1, 7))
        raw = np.cumsum(rng.normal(0, 0.2, (n, dim)), 0)
        if dim == 8:
            raw[:, 2] = rng.uniform(-3.5, 3.5, n)
        npose = [0.02, 0.02, 0.08, 0.08, 0.08, 0.08, 0.08, 0.08][:dim] if dim == 8 else [0.08] * 5
        cases.append((raw, npose))
    txt = ""
    for raw, npose in cases:
        txt += "%d %d\n" % (raw.shape[1], len(raw))
        txt += "\n".join(" ".join("%.17g" % v for v in r) for r in raw) + "\n"
        txt += " ".join("%.17g" % v for v in npose) + "\n"
    p = subprocess.run([exe], input=txt, capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    lines = p.stdout.splitlines()
    i = 0
    for raw, npose in cases:
        want = OT.normalize_trajectory(raw.tolist(), npose)
        if want is None:
            assert lines[i] == "untouched"
            i += 1
            continue
        assert lines[i] == "rows %d" % len(want)
        got = np.array([[float(v) for v in ln.split()] for ln in lines[i + 1:i + 1 + len(want)]])
        assert np.array_equal(got, np.array(want))
        i += 1 + len(want)


def build_multi(tmpdir):
    exe = os.path.join(str(tmpdir), "shim_multi")
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "shim_multi.cpp"), "-L", LIBDIR, "-lsmp_gpu",
                    "-Wl,-rpath," + LIBDIR, "-o", exe], check=True, capture_output=True, text=True)
    return exe


def run_multi(exe, bt, sc, devices, iters, nq):
    args = [exe, URDF, bt, devices, str(iters), str(nq)] + ["%.17g" % v for v in list(sc.start) + list(sc.goal)]
    args += ["%.17g" % v for v in list(sc.env_x) + list(sc.env_y)]
    return subprocess.run(args, capture_output=True, text=True, timeout=300)


def parse_multi(out):
    lines, res, i = out.splitlines(), [], 0
    while i < len(lines):
        f = lines[i].split()
        assert f[0] == "query"
        n = int(f[4])
        res.append((int(f[2]), int(f[3]), np.array([[float(v) for v in ln.split()] for ln in lines[i + 1:i + 1 + n]])))
        i += 1 + n
    return res


def test_shim_multi_builds_and_fails_loudly_without_gpu(tmp_path):
    exe = build_multi(tmp_path)
    sc, bt = room3_case(tmp_path)
    p = run_multi(exe, bt, sc, "0", 10, 2)
    if p.returncode == 3:
        assert "no usable GPU" in p.stdout or "NO_DEVICE" in p.stdout.upper(), p.stdout
    else:
        assert p.returncode == 0, p.stderr


@pytest.mark.gpu
def test_shim_multi_gpu_planner_matches_single_planner(tmp_path):
    """smp_node::MultiGpuPlanner: the scene shared device to device to a second planner (listed on the same GPU here)
    and 5 queries dealt over both give exactly what one planner gives, and query 0 equals the oracle's run."""
    exe = build_multi(tmp_path)
    sc, bt = room3_case(tmp_path)
    two = run_multi(exe, bt, sc, "0,0", 150, 5)
    one = run_multi(exe, bt, sc, "0", 150, 5)
    assert two.returncode == 0 and one.returncode == 0, two.stdout + two.stderr + one.stderr
    a, b = parse_multi(two.stdout), parse_multi(one.stdout)
    assert len(a) == len(b) == 5
    for x, y in zip(a, b):
        assert x[0] == y[0] and x[1] == y[1] and np.array_equal(x[2], y[2])
    res, keys = octomap_bt.read_bt(open(bt, "rb").read())
    orc = O.Oracle(O.OracleRobot(MODEL), O.OracleScene(keys, res))
    o = orc.plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, max_iter=150, seed=100, query=0)
    assert a[0][1] == o["checked"]
    if o["status"] == 0:
        assert a[0][0] == 0 and np.array_equal(a[0][2], o["path"].reshape(-1, 8))
