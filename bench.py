#!/usr/bin/env python3
"""Benchmark of the BiRRT* hot path on MI355X (BASELINE.json metric).

A step = one planning query of the C2 configuration (single query, 10 m x 10 m x 2 m octomap @ 5 cm with 20
box obstacles, iteration budget --iterations; path_optimality_threshold = -inf so the whole budget runs,
SURVEY.md 8d) through the C ABI.  value = collision-checked configurations per second over all ranks
(reference semantics: every isInCollision call up to the first collision of an edge).  With N GPUs each rank
plans its own queries against the scene rank 0 broadcast over RCCL (weak scaling, no per-iteration
collectives).  rank 0 prints one JSON line.
"""
import argparse
import json
import math
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

S_SPHERES = 64          # spheres per configuration in the collision model
BYTES_PER_CONFIG = 64 + 8 * S_SPHERES   # config in + one 8-byte occupancy word per sphere
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8 TB/s


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--iterations", type=int, default=int(os.environ.get("SMP_BENCH_ITERS", 1_000_000)))
    ap.add_argument("--warmup-iterations", type=int, default=2000)
    ap.add_argument("--queries-per-gpu", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args()


def cpu_baseline(sc, seconds, seed):
    """The oracle (sequential C++ restatement, 1 thread) on the same query for a bounded time."""
    from oracle import oracle as O
    rob = O.OracleRobot(os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json"))
    orc = O.Oracle(rob, O.OracleScene(sc.keys, sc.res))
    r = orc.plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, max_time=seconds, seed=seed,
                 opt_thresh=-math.inf)
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": r["checked"] / r["t_total"], "unit": "configs/s", "cores": 1, "kind": "port",
            "sample": "C2 query (seed %d), oracle/smp_oracle.cpp single thread, time budget %.0f s: %d iterations, "
                      "%d configs checked in %.2f s on %s" % (seed, seconds, r["iterations"], r["checked"],
                                                           r["t_total"], cpu),
            "iterations": r["iterations"], "time_first_solution_s": r["t_first"],
            "iters_per_s": r["iterations"] / r["t_total"]}


def main():
    a = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from squirrel_motion_planner_amd import scenes
    from squirrel_motion_planner_amd.planner import GpuPlanner, Scene

    sc = scenes.box_room()
    # scene: rank 0 builds the grid (octomap keys -> bitset + squared EDT) and broadcasts it once (RCCL/xGMI)
    if rank == 0:
        s0 = Scene.from_keys(sc.keys, sc.res)
        info = s0.info()
        bits, d2 = s0.export()
    if world > 1:
        meta = torch.zeros(7, dtype=torch.float64, device="cuda")
        if rank == 0:
            meta[:] = torch.tensor(list(info["dims"]) + list(info["origin"]) + [info["res"]], dtype=torch.float64)
        dist.broadcast(meta, 0)
        dims = [int(v) for v in meta[:3].tolist()]
        origin = meta[3:6].tolist()
        res = float(meta[6])
        nw = ((dims[0] + 63) // 64) * dims[1] * dims[2]
        nc = dims[0] * dims[1] * dims[2]
        tb = torch.zeros(nw, dtype=torch.int64, device="cuda")
        td = torch.zeros(nc, dtype=torch.int16, device="cuda")
        if rank == 0:
            tb.copy_(torch.from_numpy(bits.view(np.int64)))
            td.copy_(torch.from_numpy(d2.view(np.int16)))
        dist.broadcast(tb, 0)
        dist.broadcast(td, 0)
        scene = Scene.from_grid(tb.cpu().numpy().view(np.uint64), td.cpu().numpy().view(np.uint16), dims, origin, res)
    else:
        scene = s0

    gp = GpuPlanner(device=local, path_optimality_threshold=-math.inf)
    gp.set_scene(scene)

    def queries(step, iters):
        out = []
        for k in range(a.queries_per_gpu):
            qid = rank * a.queries_per_gpu + k
            out.append(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=iters,
                                             seed=a.seed + 1000 * step, query_id=qid))
        return out

    for w in range(a.warmup):
        gp.plan_batch(queries(-1 - w, a.warmup_iterations))

    totals = dict(checked=0, valid=0, iters=0, nn=0, near=0, plan_ms=0.0, launches=0)
    first_t = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for step in range(a.steps):
        rs = gp.plan_batch(queries(step, a.iterations))
        for r in rs:
            if r["status"] not in (0, -4):
                raise RuntimeError("plan failed with status %d" % r["status"])
            totals["checked"] += r["configs_checked"]
            totals["valid"] += r["configs_valid"]
            totals["iters"] += r["iterations"]
            totals["nn"] += r["nn_nodes_scanned"]
            totals["near"] += r["near_nodes_scanned"]
            if r["time_first_solution"] >= 0:
                first_t.append(r["time_first_solution"])
        _, pms, nl = gp.last_kernel_ms()
        totals["plan_ms"] += pms
        totals["launches"] += nl
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    local_vec = [elapsed, totals["checked"], totals["valid"], totals["iters"], totals["nn"], totals["near"],
                 totals["plan_ms"], totals["launches"]]
    if world > 1:
        tt = torch.tensor(local_vec, dtype=torch.float64, device="cuda")
        tmax = tt.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        elapsed = float(tmax[0])
        checked, valid, iters, nn, near, plan_ms, launches = [float(v) for v in tt[1:].tolist()]
        plan_ms_rank0 = totals["plan_ms"]
    else:
        checked, valid, iters, nn, near, plan_ms, launches = local_vec[1:]
        plan_ms_rank0 = plan_ms

    if rank == 0:
        alg_bytes_rank0 = 64.0 * totals["nn"] + 72.0 * totals["near"] + BYTES_PER_CONFIG * totals["checked"]
        achieved = alg_bytes_rank0 / (plan_ms_rank0 * 1e-3) / 1e9 if plan_ms_rank0 > 0 else 0.0
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_plan_kernel.json")
        if os.path.exists(pmc):
            try:
                traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
        out = {
            "metric": "collision-checked samples/sec + time-to-first-feasible-path, 8-DoF, 5 cm octomap",
            "value": checked / elapsed,
            "unit": "configs/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded box scene + seeded Philox samples)",
            "config": {"workload": "C2: single start->goal query, 10x10x2 m octomap @5 cm, 20 boxes, %d-iteration "
                                   "budget, path_optimality_threshold=-inf" % a.iterations,
                       "queries_per_gpu": a.queries_per_gpu, "iterations_per_query": a.iterations,
                       "robot": "robotino 8-DoF, 64-sphere model", "parallelism": "one workgroup per query, "
                       "queries sharded over ranks, scene broadcast once"},
            "valid_configs_per_s": valid / elapsed,
            "iterations_per_s": iters / elapsed,
            "time_to_first_feasible_path_s": (sum(first_t) / len(first_t)) if first_t else None,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "smp::plan_kernel", "kernel_ms_rank0": plan_ms_rank0,
                         "launches_rank0": totals["launches"],
                         "algorithmic_bytes_rank0": alg_bytes_rank0},
        }
        if not a.no_cpu and world == 1:
            out["cpu_baseline"] = cpu_baseline(sc, a.cpu_seconds, a.seed)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
