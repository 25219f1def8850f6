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
    """Rank `src` passes its Scene (others None); every rank returns an equivalent Scene (host form, for ranks that
    need the host grid; planners take broadcast_planner_scene's device-to-device path instead).

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


def _scene_offsets(n_bricks, n_cells, n_prim, plane, has_d2b):
    """Byte offsets of the arrays of a device scene in one flat broadcast buffer (8-byte aligned) and its size."""
    al = lambda n: (n + 7) // 8 * 8
    o_bricks = 0
    o_d2 = o_bricks + al(8 * n_bricks)
    o_d2b = o_d2 + al(2 * n_cells)
    o_slab = o_d2b + (al(n_cells) if has_d2b else 0)
    return o_bricks, o_d2, o_d2b, o_slab, o_slab + al(2 * plane * n_prim)


def broadcast_planner_scene(gp, src=0, device=None):
    """The scene of rank `src`'s planner to every rank's planner, device to device: one broadcast of a small header
    and ONE broadcast of the device-resident arrays (bricks, box-gap field, its byte copy, the primitives' slab fields)
    -- RCCL over xGMI with the nccl backend -- straight from the sender's planner buffers into the receivers'
    (smp_planner_scene_device / smp_planner_set_scene_device); nothing is rebuilt or staged on a host.

    Rank `src` must have set its planner's scene (GpuPlanner.set_scene); the ranks' robots must be the same model.
    Returns the number of payload bytes broadcast."""
    from . import _lib as L
    rank = dist.get_rank()
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    meta = torch.zeros(11, dtype=torch.float64, device=dev)
    if rank == src:
        v = gp.scene_device()
        meta[:] = torch.tensor(list(v.dims) + list(v.origin) + [v.resolution, v.n_bricks, v.n_cells, v.n_prim,
                                                                 v.has_d2b], dtype=torch.float64)
    dist.broadcast(meta, src)
    m = meta.tolist()
    dims = [int(x) for x in m[0:3]]
    n_bricks, n_cells, n_prim, has_d2b = int(m[7]), int(m[8]), int(m[9]), int(m[10])
    plane = dims[0] * dims[1]
    o_b, o_d, o_db, o_s, total = _scene_offsets(n_bricks, n_cells, n_prim, plane, has_d2b)
    buf = torch.empty(total, dtype=torch.uint8, device=dev)
    base = buf.data_ptr()
    ptrs = dict(bricks=base + o_b, d2=base + o_d, d2b=base + o_db if has_d2b else 0, slab=base + o_s if n_prim else 0)
    if rank == src:
        gp.scene_device(**ptrs)  # the planner's arrays into the broadcast buffer (device copies)
    dist.broadcast(buf, src)
    if rank != src:
        v = L.SceneDevice()
        for k in range(3):
            v.dims[k] = dims[k]
            v.origin[k] = m[3 + k]
        v.resolution = m[6]
        v.n_bricks, v.n_cells, v.n_prim, v.has_d2b = n_bricks, n_cells, n_prim, has_d2b
        torch.cuda.synchronize(dev)  # the broadcast has landed before the library's stream reads the buffer
        gp.set_scene_device(v, **ptrs)
    return total


def reduce_counters(values, device="cpu"):
    """(sum over ranks, max over ranks) of a list of float counters."""
    t = torch.tensor(values, dtype=torch.float64, device=device)
    tmax = t.clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist(), tmax.tolist()


def single_rank_reference(run, rank, src=0):
    """The same-workload single-GPU reference of a multi-rank measurement (bench.py with WORLD_SIZE > 1): after the
    multi-rank timed region, rank `src` runs `run()` -- its own per-GPU share of the job again, timed -- while every
    other rank waits at a barrier, so the GPU runs alone.  Returns run()'s result on `src`, None elsewhere."""
    dist.barrier()
    out = run() if rank == src else None
    dist.barrier()
    return out


def scaling_fields(value_all, world, alone, ranks_per_gpu=1):
    """The line's scaling fields: `alone` = (configurations checked, seconds) of one GPU planning the same per-GPU
    share alone; scaling_efficiency = whole-job rate / (world x that single-GPU rate) (weak scaling: the per-GPU work
    is the same).  With ranks_per_gpu > 1 (a rehearsal: more ranks than GPUs, each planner provisioned with its share of
    one device, SMP_SLOT_SHARE) rank 0's "alone" run still held only its share of the GPU, so the quotient is not a
    multi-GPU efficiency: the line carries the rehearsal's fields and scaling_efficiency None."""
    checked, seconds = alone
    single = checked / seconds if seconds > 0 else None
    out = {"single_gpu_same_workload": {"value": single, "unit": "configs/s", "configs_checked": checked,
                                        "seconds": seconds},
           "scaling_efficiency": value_all / (world * single) if single and ranks_per_gpu == 1 else None}
    if ranks_per_gpu > 1:
        out["ranks_per_gpu"] = ranks_per_gpu
        out["rehearsal"] = ("ranks share %d per GPU; single_gpu_same_workload ran at 1/%d of the device's slots, so no "
                            "scaling efficiency is derived" % (ranks_per_gpu, ranks_per_gpu))
    return out

