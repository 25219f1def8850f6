"""World-size-2 gloo tests of the multi-rank path (bench.py with --gpus N > 1 uses the same functions over
RCCL): the scene broadcast reproduces rank 0's grid exactly, queries shard without overlap, and the
counter reduction gives sums and maxima over ranks."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from squirrel_motion_planner_amd import distributed as D, scenes
    from squirrel_motion_planner_amd.planner import Scene
    sc = scenes.box_room()
    scene = Scene.from_keys(sc.keys, sc.res) if rank == 0 else None
    got = D.broadcast_scene(scene)
    bits, d2 = got.export()
    info = got.info()
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), bits=bits, d2=d2, dims=np.array(info["dims"]),
             origin=np.array(info["origin"]), res=info["res"], n_occ=info["n_occupied"],
             shard=np.array(D.shard_queries(64, world, rank)))
    s, m = D.reduce_counters([float(rank + 1), 10.0 * (rank + 1)])
    np.save(os.path.join(out_dir, "red%d.npy" % rank), np.array(s + m))
    dist.destroy_process_group()


def _plan_worker(rank, world, port, out_dir):
    """bench.py's multi-GPU dealing with the oracle in place of the GPU: each rank plans the queries
    D.shard_queries deals it (C3 pairs, short budgets) and the counters are reduced as bench.py reduces them."""
    import math
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    from squirrel_motion_planner_amd import distributed as D, scenes
    sc = scenes.box_room()
    orc = O.Oracle(O.OracleRobot(os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json")),
                   O.OracleScene(sc.keys, sc.res))
    pairs = scenes.random_queries(sc, 8, seed=7, check=lambda q: bool(orc.check_configs(np.array([q]))[0]))
    mine = D.shard_queries(len(pairs), world, rank)
    vals = [0.0, 0.0, 0.0]
    for qid in mine:
        r = orc.plan(pairs[qid][0], pairs[qid][1], env_x=sc.env_x, env_y=sc.env_y, seed=1, query=qid,
                     opt_thresh=-math.inf, max_iter=40)
        vals = [vals[0] + r["checked"], vals[1] + r["iterations"], vals[2] + r["valid"]]
    s, m = D.reduce_counters(vals)
    np.save(os.path.join(out_dir, "plan%d.npy" % rank), np.array(s + [float(q) for q in mine]))
    dist.destroy_process_group()


def test_bench_dealing_reduces_to_single_rank_totals(tmp_path, orobot):
    """With WORLD_SIZE > 1 bench.py plans the C3 share: the dealt queries partition the job's pairs, and the reduced
    per-rank counters equal one rank planning every query."""
    import math
    from oracle import oracle as O
    from squirrel_motion_planner_amd import scenes
    world, port = 2, _free_port()
    mp.spawn(_plan_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    got = [np.load(os.path.join(str(tmp_path), "plan%d.npy" % r)) for r in range(world)]
    assert got[0][:3].tolist() == got[1][:3].tolist()
    ids = sorted(int(v) for g in got for v in g[3:])
    assert ids == list(range(8))
    sc = scenes.box_room()
    orc = O.Oracle(orobot, O.OracleScene(sc.keys, sc.res))
    pairs = scenes.random_queries(sc, 8, seed=7, check=lambda q: bool(orc.check_configs(np.array([q]))[0]))
    tot = [0.0, 0.0, 0.0]
    for qid in range(8):
        r = orc.plan(pairs[qid][0], pairs[qid][1], env_x=sc.env_x, env_y=sc.env_y, seed=1, query=qid,
                     opt_thresh=-math.inf, max_iter=40)
        tot = [tot[0] + r["checked"], tot[1] + r["iterations"], tot[2] + r["valid"]]
    assert got[0][:3].tolist() == tot and tot[0] > 0


def _scaling_worker(rank, world, port, out_dir):
    """bench.py's multi-rank line with the oracle in place of the GPU: the timed region over every rank's C3 share, the
    reduced rate, then rank 0's share again alone (D.single_rank_reference) and the scaling fields (D.scaling_fields)."""
    import json
    import math
    import sys
    import time
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    from squirrel_motion_planner_amd import distributed as D, scenes
    sc = scenes.box_room()
    orc = O.Oracle(O.OracleRobot(os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json")),
                   O.OracleScene(sc.keys, sc.res))
    pairs = scenes.random_queries(sc, 4, seed=7, check=lambda q: bool(orc.check_configs(np.array([q]))[0]))
    mine = D.shard_queries(len(pairs), world, rank)

    def timed(sync):
        if sync:
            dist.barrier()
        t0, checked = time.perf_counter(), 0
        for qid in mine:
            r = orc.plan(pairs[qid][0], pairs[qid][1], env_x=sc.env_x, env_y=sc.env_y, seed=1, query=qid,
                         opt_thresh=-math.inf, max_iter=30)
            checked += r["checked"]
        if sync:
            dist.barrier()
        return time.perf_counter() - t0, checked

    el, ch = timed(True)
    s, m = D.reduce_counters([el, float(ch)])
    alone = D.single_rank_reference(lambda: timed(False), rank)
    if rank == 0:
        out = D.scaling_fields(s[1] / m[0], world, (alone[1], alone[0]))
        out["value"] = s[1] / m[0]
        out["rank0_checked"] = ch
        json.dump(out, open(os.path.join(out_dir, "scaling.json"), "w"))
    else:
        assert alone is None
    dist.destroy_process_group()


def test_bench_scaling_fields_world2(tmp_path):
    """With WORLD_SIZE > 1 the line carries single_gpu_same_workload (rank 0's share planned again alone, the same
    configurations) and scaling_efficiency = value / (world x that rate)."""
    import json
    world, port = 2, _free_port()
    mp.spawn(_scaling_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    out = json.load(open(os.path.join(str(tmp_path), "scaling.json")))
    single = out["single_gpu_same_workload"]
    assert single["configs_checked"] == out["rank0_checked"] > 0
    assert single["unit"] == "configs/s" and single["value"] == single["configs_checked"] / single["seconds"]
    assert abs(out["scaling_efficiency"] - out["value"] / (world * single["value"])) < 1e-12


def test_scene_broadcast_and_sharding_world2(tmp_path):
    world, port = 2, _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    a = np.load(os.path.join(str(tmp_path), "rank0.npz"))
    b = np.load(os.path.join(str(tmp_path), "rank1.npz"))
    assert np.array_equal(a["bits"], b["bits"]) and np.array_equal(a["d2"], b["d2"])
    assert np.array_equal(a["dims"], b["dims"]) and np.array_equal(a["origin"], b["origin"])
    assert float(a["res"]) == float(b["res"]) and int(a["n_occ"]) == int(b["n_occ"]) > 0
    s0, s1 = set(a["shard"].tolist()), set(b["shard"].tolist())
    assert not (s0 & s1) and s0 | s1 == set(range(64)) and len(s0) == len(s1) == 32
    for r in range(world):
        red = np.load(os.path.join(str(tmp_path), "red%d.npy" % r))
        assert red.tolist() == [3.0, 30.0, 2.0, 20.0]


def test_rehearsal_scaling_fields_carry_no_efficiency():
    """Ranks sharing one GPU (ranks_per_gpu > 1): the line is labelled a rehearsal and derives no efficiency."""
    from squirrel_motion_planner_amd import distributed as D
    f = D.scaling_fields(10.0, 2, (400, 100.0), ranks_per_gpu=2)
    assert f["scaling_efficiency"] is None and f["ranks_per_gpu"] == 2 and "rehearsal" in f
    assert f["single_gpu_same_workload"]["value"] == 4.0
    g = D.scaling_fields(10.0, 2, (400, 100.0))
    assert g["scaling_efficiency"] == 10.0 / (2 * 4.0) and "rehearsal" not in g
