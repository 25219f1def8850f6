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
