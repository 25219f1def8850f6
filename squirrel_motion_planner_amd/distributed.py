"""Multi-GPU plumbing of the planner: one process per GPU, queries sharded over ranks,
the scene built once on rank 0 and broadcast (RCCL over xGMI on GPUs, gloo on CPU in the tests).  There is no
collective on the planning data path: each rank plans its own queries against its copy of the grid.

The reference has no multi-process path (a single ROS node, squirrel_8dof_planner_node.cpp:6-15); the
sharding unit is an independent start/goal query.
"""
import numpy as np
import torch
import torch.distributed as dist

from .planner import Scene


def shard_queries(n_queries, world, rank):
    """Query indices of `rank` when n_queries independent queries are dealt round-robin over `world` ranks."""
    return list(range(rank, n_queries, world))


def broadcast_scene(scene, device="cpu", src=0):
    """Rank `src` passes its Scene (others None); every rank returns an equivalent Scene.

    One broadcast of the header (dims, origin, resolution) and one each of the occupancy bitset and the
    box-gap field; ranks other than `src` rebuild their brick masks from the bitset (smp_scene_from_grid).
    """
    rank = dist.get_rank()
    meta = torch.zeros(7, dtype=torch.float64, device=device)
    if rank == src:
        info = scene.info()
        meta[:] = torch.tensor(list(info["dims"]) + list(info["origin"]) + [info["res"]], dtype=torch.float64)
    dist.broadcast(meta, src)
    dims = [int(v) for v in meta[:3].tolist()]
    origin = meta[3:6].tolist()
    res = float(meta[6])
    nw = ((dims[0] + 63) // 64) * dims[1] * dims[2]
    nc = dims[0] * dims[1] * dims[2]
    nd = (nc + 3) // 4  # the uint16 field travels packed in int64 words (gloo has no 16-bit type)
    tb = torch.zeros(nw, dtype=torch.int64, device=device)
    td = torch.zeros(nd, dtype=torch.int64, device=device)
    if rank == src:
        bits, d2 = scene.export()
        packed = np.zeros(nd * 4, np.uint16)
        packed[:nc] = d2
        tb.copy_(torch.from_numpy(bits.view(np.int64)))
        td.copy_(torch.from_numpy(packed.view(np.int64)))
    dist.broadcast(tb, src)
    dist.broadcast(td, src)
    if rank == src:
        return scene
    d2 = td.cpu().numpy().view(np.uint16)[:nc].copy()
    return Scene.from_grid(tb.cpu().numpy().view(np.uint64), d2, dims, origin, res)


def reduce_counters(values, device="cpu"):
    """(sum over ranks, max over ranks) of a list of float counters."""
    t = torch.tensor(values, dtype=torch.float64, device=device)
    tmax = t.clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist(), tmax.tolist()
