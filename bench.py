#!/usr/bin/env python3
"""Benchmark of the BiRRT* hot path on MI355X (BASELINE.json metric).

A step = one planning query of the C2 configuration (BASELINE.json configs[1]: single query, 10 m x 10 m x 2 m
octomap @ 5 cm with 20 box obstacles, budget of 1e6 collision-checked samples; path_optimality_threshold = -inf
so the whole budget runs) through the C ABI.  value = collision-checked configurations per second over all ranks
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

S_SPHERES = 50 + 6      # collision model 2: 50 spheres + 6 exact box / cylinder primitives (one map test each)
BYTES_PER_CONFIG = 64 + 8 * S_SPHERES   # config in + one 8-byte occupancy word per sphere
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8 TB/s


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--samples", type=int, default=int(os.environ.get("SMP_BENCH_SAMPLES", 1_000_000)),
                    help="budget of collision-checked configurations per query")
    ap.add_argument("--warmup-samples", type=int, default=None,
                    help="budget of each warmup query (default: --samples, so warmup launches match timed ones)")
    ap.add_argument("--queries-per-gpu", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--helpers", type=int, default=0,
                    help="helper workgroups per query (0 automatic, -1 none: e.g. for counter passes, which "
                         "serialise dispatches)")
    ap.add_argument("--scout", type=int, default=1,
                    help="scout workgroups per query (1 automatic, 0 none, 2..8 that many)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--workload", choices=("c2", "c3", "c5"), default=None,
                    help="c2 (default on one GPU, BASELINE configs[1]): the single C2 query; c3 (default with "
                         "WORLD_SIZE > 1, configs[2]: 64 queries sharded 8 per GPU at 8 GPUs): random (start, goal) "
                         "pairs on the C2 scene, 8 per GPU; c5: 2 cm dense clutter, 8 random queries per GPU "
                         "(configs[4])")
    ap.add_argument("--iterations", type=int, default=None,
                    help="iteration budget per query instead of --samples (C3: 1e5 in SURVEY.md 8d)")
    ap.add_argument("--cpu-iterations", type=int, default=20000,
                    help="with --iterations above this, the CPU baseline is a bounded window at the end of the run: "
                         "the oracle continues the GPU's own state at iteration N - --cpu-window (same trees) to N, "
                         "timed against the GPU's time for the same iterations (its cost rows)")
    ap.add_argument("--cpu-window", type=int, default=1000,
                    help="iterations of the CPU window of --iterations runs above --cpu-iterations")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args()


def workload_name(a, sc):
    if a.workload == "c2":
        return ("C2: single start->goal query, 10x10x2 m octomap @5 cm, 20 boxes, budget %s, "
                "path_optimality_threshold=-inf" % (("%d iterations" % a.iterations) if a.iterations else
                                                   ("%d collision-checked samples" % a.samples)))
    if a.workload == "c3":
        return ("C3: random collision-free start/goal pairs (seed 7) on the C2 scene, %d queries per GPU, "
                "path_optimality_threshold=-inf" % a.queries_per_gpu)
    return ("C5: 10x10x2 m @2 cm dense clutter voxelised from a 2e6-point synthetic cloud (seed 11), %d random "
            "queries per GPU, path_optimality_threshold=-inf" % a.queries_per_gpu)


def host_cpu():
    """CPU model and the core count this process may use (the GPU box gives each GPU a share of its cores:
    OMP_NUM_THREADS; nproc / os.cpu_count() report the whole machine there)."""
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    share = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    return cpu, max(1, min(share, len(os.sched_getaffinity(0))))


def cpu_baseline(sc, pair, a, step0_seed, step_seeds=()):
    """The oracle (C++ restatement of the reference loop) on query 0 of GPU step 0: one thread (the north_star's
    single-thread reference) and all of this process's cores (OpenMP on the two scans, as the reference's
    BS:4092 / BS:4283).

    Same scene, (start, goal), seed, query id and budget, so the CPU runs plan the identical trees; the bench
    records whether the counters match the GPU's (a parity check of the measured run itself)."""
    from oracle import oracle as O
    rob = O.OracleRobot(os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json"))
    orc = O.Oracle(rob, O.OracleScene(sc.keys, sc.res))
    bounded = bool(a.iterations and a.iterations > a.cpu_iterations)
    budget = (dict(max_iter=min(a.iterations, a.cpu_iterations)) if a.iterations else
              dict(max_checked=a.samples, max_iter=0))
    cpu, cores = host_cpu()
    r = orc.plan(pair[0], pair[1], env_x=sc.env_x, env_y=sc.env_y, seed=step0_seed, query=0,
                 opt_thresh=-math.inf, threads=1, **budget)
    rm = orc.plan(pair[0], pair[1], env_x=sc.env_x, env_y=sc.env_y, seed=step0_seed, query=0,
                  opt_thresh=-math.inf, threads=cores, **budget) if cores > 1 else r
    ttff = [first_solution(orc, sc, pair, sd) for sd in step_seeds]
    full = None
    if bounded and a.workload == "c2":
        # the committed 1e5-iteration fixture (oracle run of C2 seed 7, timed when it was made in the build
        # container, not on this host): the full-run CPU time beside the bounded sample
        try:
            import numpy as np
            z = np.load(os.path.join(ROOT, "tests", "golden", "plan_c2_1e5.npz"))
            if int(z["iterations"]) == a.iterations and int(z["seed"]) == step0_seed:
                full = {"iterations": int(z["iterations"]), "checked": int(z["checked"]),
                        "t_total_s": float(z["t_total"]), "configs_per_s": float(z["checked"]) / float(z["t_total"]),
                        "source": "tests/golden/plan_c2_1e5.npz (oracle single thread, build container CPU)"}
        except (OSError, KeyError, ValueError):
            full = None
    return {"value": r["checked"] / r["t_total"], "unit": "configs/s", "cores": 1, "kind": "port",
            "sample": "%s query 0 (seed %d), oracle/smp_oracle.cpp single thread, %s: %d iterations, "
                      "%d configs checked in %.2f s on %s" % (
                          a.workload.upper(), step0_seed,
                          "first %d iterations of the same query (bounded sample; its trees are smaller, so the CPU "
                          "rate is an upper bound for the full run)" % a.cpu_iterations if bounded else "same budget",
                          r["iterations"], r["checked"], r["t_total"], cpu),
            "bounded_sample": bounded, "full_run_oracle": full,
            "cpu_model": cpu,
            "valid_configs_per_s": r["valid"] / r["t_total"],
            "iterations": r["iterations"], "checked": r["checked"], "time_first_solution_s": r["t_first"],
            "iters_per_s": r["iterations"] / r["t_total"], "cost_best": r["cost"][0],
            "all_cores": {"value": rm["checked"] / rm["t_total"], "unit": "configs/s", "cores": cores,
                          "valid_configs_per_s": rm["valid"] / rm["t_total"], "t_total_s": rm["t_total"],
                          "same_trees_as_1_thread": bool(rm["checked"] == r["checked"] and
                                                         rm["iterations"] == r["iterations"]),
                          "how": "oracle with the nearest / near scans as OpenMP loops on %d threads "
                                 "(BS:4092, BS:4283)" % cores},
            # the oracle's time to the first feasible path for every timed step's seed (short runs, same query,
            # timed from run() entry), beside the GPU's per-step lists
            "time_first_solution_steps_s": ttff or None,
            "time_first_solution_stats_s": stats3(ttff)}


def cpu_window(a, gp, sc, pair, seed, step0):
    """CPU baseline of a long run (--iterations above --cpu-iterations), at the run's own tree sizes: the GPU plans
    the same query to N - K iterations (untimed, after the timed region) and hands its state to the oracle
    (GpuPlanner.export_state -> Oracle.resume: both trees, child order, in-edges, loop scalars), which continues it to
    N on one thread and with its scans on all of this process's cores.  The window's GPU time is the timed step 0's
    device clock between the cost rows of iterations N - K and N; both sides check the same configurations in it
    (the oracle's end state is compared with the GPU's step 0)."""
    import numpy as np
    from oracle import oracle as O
    from squirrel_motion_planner_amd.planner import GpuPlanner
    n, k = a.iterations, min(a.cpu_window, a.iterations - 1)
    gp.plan(GpuPlanner.make_query(pair[0], pair[1], sc.env_x, sc.env_y, iterations=n - k, seed=seed, query_id=0))
    st = gp.export_state()
    rob = O.OracleRobot(os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json"))
    orc = O.Oracle(rob, O.OracleScene(sc.keys, sc.res))
    cpu, cores = host_cpu()
    kw = dict(env_x=sc.env_x, env_y=sc.env_y, seed=seed, query=0, opt_thresh=-math.inf, max_iter=n)
    r1 = orc.resume(pair[0], pair[1], st, threads=1, **kw)
    rm = orc.resume(pair[0], pair[1], st, threads=cores, **kw) if cores > 1 else r1
    rows = step0["cost_rows"]
    gpu_s = float(rows[n - 1][1] - rows[n - k - 1][1]) if len(rows) >= n else None
    checked = r1["checked"] - int(st["iv"][1])
    same = bool(r1["checked"] == step0["configs_checked"] and r1["n_start"] == step0["nodes_start"] and
                r1["n_goal"] == step0["nodes_goal"] and r1["cost"][0] == step0["cost_best"][0])
    nodes = (len(st["start"]["parent"]), len(st["goal"]["parent"]))
    return {"value": checked / r1["t_total"], "unit": "configs/s", "cores": 1, "kind": "port",
            "sample": "C2 query 0 (seed %d), oracle/smp_oracle.cpp single thread, continuing the GPU's state at "
                      "iteration %d (trees of %d / %d nodes) to %d: %d configs checked in %.2f s on %s" % (
                          seed, n - k, nodes[0], nodes[1], n, checked, r1["t_total"], cpu),
            "bounded_sample": True, "window": {"from_iteration": n - k, "to_iteration": n, "tree_nodes": nodes,
                                                "configs_checked": checked, "gpu_seconds": gpu_s,
                                                "gpu_configs_per_s": checked / gpu_s if gpu_s else None,
                                                "cpu_seconds_1_thread": r1["t_total"],
                                                "cpu_seconds_all_cores": rm["t_total"]},
            "cpu_model": cpu, "valid_configs_per_s": (r1["valid"] - int(st["iv"][2])) / r1["t_total"],
            "iterations": k, "checked": checked, "iters_per_s": k / r1["t_total"], "cost_best": r1["cost"][0],
            "all_cores": {"value": checked / rm["t_total"], "unit": "configs/s", "cores": cores,
                          "t_total_s": rm["t_total"],
                          "same_trees_as_1_thread": bool(rm["checked"] == r1["checked"] and
                                                         rm["n_start"] == r1["n_start"]),
                          "how": "oracle with the nearest / near scans as OpenMP loops on %d threads "
                                 "(BS:4092, BS:4283), the same window" % cores},
            "same_result_as_gpu_step0": same}


def _oracle_worker(args):
    """One independent oracle process of the many-query CPU baseline: plans its share of the queries."""
    workload, jobs, budget = args
    from oracle import oracle as O
    from squirrel_motion_planner_amd import scenes
    sc = scenes.clutter_cloud() if workload == "c5" else scenes.box_room()
    rob = O.OracleRobot(os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json"))
    orc = O.Oracle(rob, O.OracleScene(sc.keys, sc.res))
    out = []
    for qid, s, g, seed in jobs:
        t = time.perf_counter()
        r = orc.plan(s, g, env_x=sc.env_x, env_y=sc.env_y, seed=seed, query=qid, opt_thresh=-math.inf, threads=1,
                     **budget)
        out.append((qid, r["checked"], r["iterations"], r["valid"], time.perf_counter() - t))
    return out


def cpu_many_queries(a, pairs, seed, procs, gpu_results):
    """The many-query CPU baseline (C3 / C5): `procs` independent single-thread oracle processes, each planning its
    share of this rank's queries (same pairs, seeds, query ids and budget as the GPU step 0), the whole set timed
    on the wall clock from the first process start to the last result (scene set-up excluded: each process builds
    its scene before its clock starts)."""
    import multiprocessing as mp
    budget = dict(max_iter=a.iterations) if a.iterations else dict(max_checked=a.samples, max_iter=0)
    jobs = [(k, list(pairs[k][0]), list(pairs[k][1]), seed) for k in range(len(gpu_results))]
    shares = [jobs[i::procs] for i in range(procs)]
    ctx = mp.get_context("spawn")  # fresh interpreters: nothing of this (GPU) process is inherited
    with ctx.Pool(procs) as pool:
        res = pool.map(_oracle_worker, [(a.workload, sh, budget) for sh in shares if sh])
    flat = sorted(x for part in res for x in part)
    busy = [sum(x[4] for x in part) for part in res]
    span = max(busy)
    checked = sum(x[1] for x in flat)
    used = len(res)  # processes that planned something: min(procs, queries)
    same = all(x[1] == r["configs_checked"] and x[2] == r["iterations"] for x, r in zip(flat, gpu_results))
    return {"value": checked / span, "unit": "configs/s", "cores": used, "processes": used,
            "queries": len(flat), "checked": checked, "span_s": span,
            "how": "%d independent oracle processes (one thread each) of the %d cores available, the %d queries dealt "
                   "round-robin; value = all configurations checked / the busiest process's planning time" % (
                       used, procs, len(flat)),
            "same_results_as_gpu_step0": bool(same)}


def stats3(v):
    v = sorted(x for x in v if x is not None)
    if not v:
        return None
    return {"min": v[0], "median": v[len(v) // 2] if len(v) % 2 else 0.5 * (v[len(v) // 2 - 1] + v[len(v) // 2]),
            "max": v[-1], "n": len(v)}


def first_solution(orc, sc, pair, seed, max_iter=600):
    """Oracle time to the first feasible path of query 0 with this seed (None if not within max_iter)."""
    r = orc.plan(pair[0], pair[1], env_x=sc.env_x, env_y=sc.env_y, seed=seed, query=0, opt_thresh=-math.inf,
                 max_iter=max_iter)
    return r["t_first"] if r["t_first"] >= 0 else None


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = "nccl"
    if world > 1:
        ndev = max(1, torch.cuda.device_count())
        if ndev < world:
            # more ranks than GPUs (a rehearsal on a one-GPU box): ranks share a GPU, each planner provisions its share
            # of the device's co-resident workgroups (read when the planner is created); RCCL refuses two ranks on one
            # device, so the rehearsal's few collectives (scene broadcast, barriers, counter reductions) go over gloo
            os.environ["SMP_SLOT_SHARE"] = str((world + ndev - 1) // ndev)
            backend = "gloo"
        local = local % ndev
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    from squirrel_motion_planner_amd import distributed as D, scenes
    from squirrel_motion_planner_amd.planner import GpuPlanner, Scene

    # one GPU: the headline C2 query (configs[1]); several: BASELINE configs[2], the C3 share of 8 random queries per
    # GPU (64 at 8 GPUs), so that the driver's scaling runs measure the multi-GPU configuration
    if a.workload is None:
        a.workload = "c3" if world > 1 else "c2"
    if a.workload != "c2" and a.queries_per_gpu == 1:
        a.queries_per_gpu = 8
    # every rank builds the same scene description (seeded); only rank 0 turns it into the grid
    sc = scenes.clutter_cloud() if a.workload == "c5" else scenes.box_room()
    # scene: rank 0 builds the grid (octomap keys -> bitset + box-gap field + slab fields) and sets it on its GPU;
    # the other ranks receive its device arrays in one RCCL broadcast over xGMI, device to device (no host rebuild)
    gp = GpuPlanner(device=local, path_optimality_threshold=-math.inf, helpers=a.helpers, scout=a.scout)
    if rank == 0:
        gp.set_scene(Scene.from_keys(sc.keys, sc.res))
    if world > 1:
        D.broadcast_planner_scene(gp, src=0)

    # (start, goal) of every query of the job: C2 repeats its own pair; C3/C5 draw world * queries_per_gpu
    # collision-free pairs (scenes.random_queries, seed 7: the first k pairs are the same for any job size) and each
    # rank plans the ones D.shard_queries deals it (no collective)
    n_job = world * a.queries_per_gpu
    mine = D.shard_queries(n_job, world, rank)
    if a.workload == "c2":
        pairs = [(sc.start, sc.goal)] * n_job
    else:
        pairs = scenes.random_queries(sc, n_job, seed=7, check=lambda q: bool(gp.check_configs([q])[0]))
        if len(pairs) < n_job:
            raise RuntimeError("only %d collision-free query pairs" % len(pairs))

    def queries(step, samples):
        out = []
        for qid in mine:
            s, g = pairs[qid]
            budget = dict(iterations=a.iterations) if a.iterations else dict(samples=samples)
            out.append(GpuPlanner.make_query(s, g, sc.env_x, sc.env_y, seed=a.seed + 1000 * step, query_id=qid,
                                             **budget))
        return out

    for w in range(a.warmup):
        gp.plan_batch(queries(-1 - w, a.warmup_samples or a.samples))

    def timed_steps(sync_ranks=True):
        """The timed region: exactly a.steps planning steps of this rank's queries, bracketed by a barrier (several
        ranks; not for rank 0's run alone) and a device synchronisation on both sides."""
        totals = dict(checked=0, valid=0, iters=0, nn=0, near=0, plan_ms=0.0, launches=0)
        first_t, first_host, steps0 = [], [], []
        if world > 1 and sync_ranks:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for step in range(a.steps):
            rs = gp.plan_batch(queries(step, a.samples))
            if not steps0:
                steps0.append(rs)
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
                    first_host.append(r["time_first_solution_host"])
            _, pms, nl = gp.last_kernel_ms()
            totals["plan_ms"] += pms
            totals["launches"] += nl
        torch.cuda.synchronize()
        if world > 1 and sync_ranks:
            dist.barrier()
        return time.perf_counter() - t0, totals, steps0[0], first_t, first_host

    elapsed, totals, step0_all, first_t, first_host = timed_steps()
    step0 = step0_all[0]

    local_vec = [elapsed, totals["checked"], totals["valid"], totals["iters"], totals["nn"], totals["near"],
                 totals["plan_ms"], totals["launches"]]
    alone = None
    if world > 1:
        tsum, tmax = D.reduce_counters(local_vec, device="cuda" if backend == "nccl" else "cpu")
        elapsed = tmax[0]
        checked, valid, iters, nn, near, plan_ms, launches = tsum[1:]
        plan_ms_rank0 = totals["plan_ms"]
        # the same per-GPU share on rank 0's GPU alone (the other ranks at a barrier): the single-GPU rate of THIS
        # workload, so that the line carries its own scaling efficiency (the N = 1 line of a scaling run is C2)
        alone = D.single_rank_reference(lambda: timed_steps(sync_ranks=False), rank)
    else:
        checked, valid, iters, nn, near, plan_ms, launches = local_vec[1:]
        plan_ms_rank0 = plan_ms

    if rank == 0:
        alg_bytes_rank0 = 64.0 * totals["nn"] + 72.0 * totals["near"] + BYTES_PER_CONFIG * totals["checked"]
        # per launch: algorithmic bytes of one launch / its average duration (HIP events on the planner stream)
        achieved = alg_bytes_rank0 / (plan_ms_rank0 * 1e-3) / 1e9 if plan_ms_rank0 > 0 else 0.0
        traffic, traffic_src = None, None
        # HBM bytes per launch: not measurable inside this run (counter passes need rocprofv3); taken from the newest
        # committed FETCH_SIZE + WRITE_SIZE passes of THIS workload (profiles/r*_pmc_<tag>.json, tools/profile_round.sh),
        # else null.  From round 5 on one plan_kernel dispatch holds the leader, its scouts and helpers, so those passes
        # run the benched configuration (round 4's ran --helpers -1: counter collection serialised the helper kernel).
        import glob
        tag = a.workload + ("_iter%d" % a.iterations if a.iterations else "")
        pmcs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_%s.json" % tag)))
        if pmcs:
            try:
                traffic = json.load(open(pmcs[-1])).get("hbm_bytes_per_launch")
                name = os.path.basename(pmcs[-1])
                traffic_src = ("profiles/" + name + " (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this workload, " +
                               ("with --helpers -1)" if name < "r05" else "the benched configuration: one dispatch)"))
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
            "config": {"workload": workload_name(a, sc),
                       "queries_per_gpu": a.queries_per_gpu,
                       "budget_per_query": ("%d iterations" % a.iterations) if a.iterations else
                                           ("%d collision-checked samples" % a.samples),
                       "robot": "robotino 8-DoF, 50 spheres + 6 exact box / cylinder primitives (collision model 2)",
                       # helper workgroups per query as the library resolved them (0 = auto: the CUs left over by
                       # the queries; with a scout, split between the leader's and the scout's tiles + the sampler)
                       "helpers_per_query": int(step0["helpers"]), "scout": int(step0["scout"]),
                       "parallelism": "one leader workgroup per query + helper workgroups sharing its collision "
                       "tiles; queries sharded over ranks, scene broadcast once",
                       "backend": backend if world > 1 else None},
            "valid_configs_per_s": valid / elapsed,
            "iterations_per_s": iters / elapsed,
            # time to the first feasible path on the host's clock from smp_plan entry (start / goal checks, uploads,
            # launch and the kernel's iterations; SURVEY 8d counts from run_planner entry) and, beside it, the
            # kernel's own device-clock value (from its planning start)
            "time_to_first_feasible_path_s": (sum(first_host) / len(first_host)) if first_host else None,
            "time_to_first_feasible_path_host_steps_s": first_host if a.queries_per_gpu == 1 else None,
            "time_to_first_feasible_path_host_stats_s": stats3(first_host),
            "time_to_first_feasible_path_device_steps_s": first_t if a.queries_per_gpu == 1 else None,
            "time_to_first_feasible_path_device_stats_s": stats3(first_t),
            # priced against HBM (no dense contraction); the measured limiter is the dependent latency of
            # one query's iteration chain, not bandwidth: trees and grid stay in L2 / Infinity Cache
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "limiter": "latency (sequential iteration chain of one query)",
                         # the latency bound beside the bandwidth one: one query's iterations are a dependent chain
                         # (each reads the trees the last one wrote); per query, the time of one iteration and the
                         # collision-checked configurations it yields
                         "latency": {"us_per_iteration_per_query": (elapsed * 1e6 * a.queries_per_gpu * world / iters)
                                     if iters else None,
                                     "configs_per_iteration": checked / iters if iters else None},
                         "kernel": "smp::plan_kernel", "kernel_ms_rank0": plan_ms_rank0,
                         "avg_launch_ms": plan_ms_rank0 / max(totals["launches"], 1),
                         "launches_rank0": totals["launches"],
                         "algorithmic_bytes_rank0": alg_bytes_rank0},
        }
        if alone is not None:
            rpg = int(os.environ.get("SMP_SLOT_SHARE", "1")) if backend == "gloo" else 1
            out.update(D.scaling_fields(checked / elapsed, world, (alone[1]["checked"], alone[0]), ranks_per_gpu=rpg))
            out["single_gpu_same_workload"]["how"] = (
                "rank 0 planned its own per-GPU share (the same %d queries, seeds and budgets) again alone, the other "
                "ranks waiting at a barrier" % len(mine))
        if not a.no_cpu and world == 1 and a.workload == "c2" and a.iterations and a.iterations > a.cpu_iterations:
            out["cpu_baseline"] = cpu_window(a, gp, sc, pairs[0], a.seed, step0)
        elif not a.no_cpu and world == 1:
            cb = cpu_baseline(sc, pairs[0], a, step0_seed=a.seed, step_seeds=[a.seed + 1000 * step for step in
                                                                             range(a.steps)]
                              if a.queries_per_gpu == 1 else ())
            if cb["full_run_oracle"]:
                cb["full_run_oracle"]["same_result_as_gpu_step0"] = bool(
                    cb["full_run_oracle"]["checked"] == step0["configs_checked"])
            cb["same_result_as_gpu_step0"] = bool(not cb["bounded_sample"] and cb["checked"] == step0["configs_checked"] and
                                                  cb["iterations"] == step0["iterations"] and
                                                  cb["cost_best"] == step0["cost_best"][0])
            if a.queries_per_gpu > 1:
                # many queries: the host's answer is one oracle per core, not OpenMP scans inside one query
                cb["all_cores"] = cpu_many_queries(a, pairs, a.seed, host_cpu()[1], step0_all)
            out["cpu_baseline"] = cb
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
