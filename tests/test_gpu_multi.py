"""Multi-GPU entry points on the one-GPU box: several planners of one process (smp_plan_multi,
smp_planners_share_scene), the device-resident scene form (smp_planner_scene_device / smp_planner_set_scene_device)
and the rank-to-rank device broadcast (distributed.broadcast_planner_scene, here over gloo with two ranks on cuda:0;
bench.py --gpus N uses it over RCCL).  Every planner that received a scene device to device must answer exactly as
the planner that built it from the host scene: same validity flags, same planning results bit for bit."""
import math
import os
import socket

import numpy as np
import pytest

from squirrel_motion_planner_amd import _lib as L
from squirrel_motion_planner_amd import scenes
from squirrel_motion_planner_amd.planner import GpuPlanner, Robot, Scene

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c2():
    sc = scenes.box_room()
    return sc, Scene.from_keys(sc.keys, sc.res)


def _configs(sc, n, seed):
    rng = np.random.default_rng(seed)
    (x0, x1), (y0, y1) = sc.env_x, sc.env_y
    return np.column_stack([rng.uniform(x0, x1, n), rng.uniform(y0, y1, n)] +
                           [rng.uniform(-2.5, 2.5, n) for _ in range(6)])


def _same_result(a, b):
    for k in ("status", "iterations", "configs_checked", "configs_valid", "nodes_start", "nodes_goal",
              "first_solution_iter"):
        assert a[k] == b[k], (k, a[k], b[k])
    assert np.array_equal(np.asarray(a["cost_best"]), np.asarray(b["cost_best"]))
    assert np.array_equal(np.asarray(a["path"]), np.asarray(b["path"]))


def _queries(sc, n, iters=300):
    pairs = [(sc.start, sc.goal)] * n
    return [GpuPlanner.make_query(s, g, sc.env_x, sc.env_y, iterations=iters, seed=11 + k, query_id=k)
            for k, (s, g) in enumerate(pairs)]


def test_share_scene_and_plan_multi(c2):
    sc, scene = c2
    robot = Robot()
    a = GpuPlanner(robot, device=0, path_optimality_threshold=-math.inf)
    b = GpuPlanner(robot, device=0, path_optimality_threshold=-math.inf)
    a.set_scene(scene)
    GpuPlanner.share_scene([a, b], src=0)
    q = _configs(sc, 20000, 3)
    assert np.array_equal(a.check_configs(q), b.check_configs(q))
    qs = _queries(sc, 5)
    ref = [a.plan(x) for x in qs]
    got = GpuPlanner.plan_multi([a, b], qs)
    assert len(got) == len(qs)
    for r, g in zip(ref, got):
        _same_result(r, g)
    # a planner listed twice would be driven from two threads: refused
    with pytest.raises(L.SmpError):
        GpuPlanner.plan_multi([a, a], qs[:2])


def _roundtrip(rank, out_dir):
    """Body of test_scene_device_roundtrip_through_torch, in a fresh process: torch's HIP runtime initialises before
    the library's there (torch ships its own libamdhip64 beside /opt/rocm's; in a process where the library already
    ran many planners, torch's later initialisation was seen to find no GPU)."""
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from squirrel_motion_planner_amd import _lib as LL, scenes as S
    from squirrel_motion_planner_amd.planner import GpuPlanner as G, Robot as R, Scene as Sc
    dev = torch.device("cuda", 0)
    torch.empty(1, device=dev)
    sc = S.box_room()
    scene = Sc.from_keys(sc.keys, sc.res)
    robot = R()
    a = G(robot, device=0)
    a.set_scene(scene)
    v = a.scene_device()
    checks = [tuple(v.dims) == scene.info()["dims"], v.n_cells == int(np.prod(v.dims)), v.n_prim == 6, v.has_d2b == 1]
    bricks = torch.empty(v.n_bricks, dtype=torch.int64, device=dev)
    d2 = torch.empty(v.n_cells, dtype=torch.int16, device=dev)
    d2b = torch.empty(v.n_cells, dtype=torch.uint8, device=dev)
    slab = torch.empty(v.n_prim * v.dims[0] * v.dims[1], dtype=torch.int16, device=dev)
    a.scene_device(bricks=bricks.data_ptr(), d2=d2.data_ptr(), d2b=d2b.data_ptr(), slab=slab.data_ptr())
    torch.cuda.synchronize()
    # the device arrays are the host builder's: the box-gap field equals the host scene's export
    _, d2_host = scene.export()
    checks.append(bool(np.array_equal(d2.cpu().numpy().view(np.uint16), d2_host)))
    checks.append(bool(np.array_equal(d2b.cpu().numpy(), np.minimum(d2_host, 255).astype(np.uint8))))
    c = G(robot, device=0)
    c.set_scene_device(v, bricks.data_ptr(), d2.data_ptr(), d2b.data_ptr(), slab.data_ptr())
    del bricks, d2, d2b, slab  # copied by the library
    q = _configs(sc, 20000, 5)
    checks.append(bool(np.array_equal(a.check_configs(q), c.check_configs(q))))
    qs = _queries(sc, 1, iters=200)
    ra, rc = a.plan(qs[0]), c.plan(qs[0])
    checks.append(all(ra[k] == rc[k] for k in ("status", "iterations", "configs_checked", "nodes_start", "nodes_goal")))
    checks.append(bool(np.array_equal(ra["path"], rc["path"])) and ra["cost_best"] == rc["cost_best"])
    # a layout that does not fit this robot / grid is refused; no scene yet: nothing to export
    bad = a.scene_device()
    bad.n_prim = 5
    for f in (lambda: c.set_scene_device(bad, 1, 1, 1, 1), lambda: G(robot, device=0).scene_device()):
        try:
            f()
            checks.append(False)
        except LL.SmpError:
            checks.append(True)
    np.save(os.path.join(out_dir, "roundtrip.npy"), np.array(checks))


def test_scene_device_roundtrip_through_torch(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_roundtrip, args=(str(tmp_path),), nprocs=1, join=True)
    checks = np.load(os.path.join(str(tmp_path), "roundtrip.npy"))
    assert checks.all(), checks.tolist()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank(rank, world, port, out_dir):
    import sys
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from squirrel_motion_planner_amd import distributed as D, scenes as S
    from squirrel_motion_planner_amd.planner import GpuPlanner as G, Scene as Sc
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = S.box_room()
    gp = G(device=0, path_optimality_threshold=-math.inf)
    if rank == 0:
        gp.set_scene(Sc.from_keys(sc.keys, sc.res))
    nbytes = D.broadcast_planner_scene(gp, src=0)
    q = G.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=200, seed=21, query_id=0)
    r = gp.plan(q)
    flags = gp.check_configs(_configs(sc, 5000, 9))
    np.savez(os.path.join(out_dir, "r%d.npz" % rank), nbytes=nbytes, flags=flags, path=np.asarray(r["path"]),
             counters=np.array([r["status"], r["iterations"], r["configs_checked"], r["nodes_start"], r["nodes_goal"]]),
             cost=np.asarray(r["cost_best"]))
    dist.destroy_process_group()


def test_broadcast_planner_scene_two_ranks(tmp_path):
    import torch.multiprocessing as mp
    port = _free_port()
    mp.spawn(_rank, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    a = np.load(os.path.join(str(tmp_path), "r0.npz"))
    b = np.load(os.path.join(str(tmp_path), "r1.npz"))
    assert int(a["nbytes"]) == int(b["nbytes"]) > 4_000_000  # C2: bricks + d2 + d2b + 6 slab planes, one broadcast
    assert np.array_equal(a["flags"], b["flags"])
    assert np.array_equal(a["counters"], b["counters"]) and np.array_equal(a["cost"], b["cost"])
    assert np.array_equal(a["path"], b["path"])
