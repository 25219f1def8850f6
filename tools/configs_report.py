#!/usr/bin/env python3
"""Reports of the BASELINE configs that are not bench.py's headline line (run on the GPU box).

  python tools/configs_report.py c4 OUT.json [--seconds S]
      C4 narrow passage (2 x arm-width slot): rewire-cost convergence c_best(t) of the GPU planner (time budget S,
      path_optimality_threshold = -inf), and the CPU oracle (1 thread) on the same query for the same number of
      iterations -- both runs plan identical trees, so the rows differ only in their time column.  Rows are
      birrt_star.cpp:1325-1331's [iteration, time, c_best, c_best_rev, c_best_prism], kept where c_best changes.
  python tools/configs_report.py c5-sweep OUT.json [--libs a.so,b.so,...] [--iterations N]
      C5 2 cm dense clutter, 8 random queries on one GPU, once per library build (tile-size variants: configurations
      per job tile staged in LDS, SMP_HELPER_CT): configs/s, iterations/s and the tile's LDS bytes.
"""
import argparse
import json
import math
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def changes(rows):
    out, last = [], None
    for r in rows:
        if last is None or r[2] != last:
            out.append([float(x) for x in r])
            last = r[2]
    return out


def c4(a):
    import numpy as np
    from oracle import oracle as O
    from squirrel_motion_planner_amd import scenes
    from squirrel_motion_planner_amd.planner import GpuPlanner, Scene
    sc = scenes.narrow_passage()
    gp = GpuPlanner(path_optimality_threshold=-math.inf)
    gp.set_scene(Scene.from_keys(sc.keys, sc.res))
    gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=200, seed=a.seed))  # warm
    t0 = time.perf_counter()
    r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, seconds=a.seconds, seed=a.seed))
    wall = time.perf_counter() - t0
    rob = O.OracleRobot(os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json"))
    o = O.Oracle(rob, O.OracleScene(sc.keys, sc.res)).plan(
        sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, seed=a.seed, opt_thresh=-math.inf,
        max_iter=int(r["iterations"]))
    same = bool(o["iterations"] == r["iterations"] and o["checked"] == r["configs_checked"] and
                o["cost"] == r["cost_best"])
    orows = [[row[0], t, row[2], row[3], row[4]] for row, t in zip(o["cost_rows"], o["cost_row_times"])]
    rg, ro = changes(r["cost_rows"]), changes(orows)
    out = {"config": "C4 narrow passage, slot 0.24 m at z 0.55-0.79, seed %d, path_optimality_threshold=-inf"
                     % a.seed,
           "gpu": {"seconds_budget": a.seconds, "wall_s": wall, "iterations": int(r["iterations"]),
                   "configs_checked": int(r["configs_checked"]), "configs_per_s": r["configs_checked"] / wall,
                   "time_first_solution_s": r["time_first_solution"], "cost_best": r["cost_best"],
                   "rows_at_changes": rg},
           "cpu_oracle_1_thread": {"iterations": int(o["iterations"]), "t_total_s": o["t_total"],
                                   "configs_per_s": o["checked"] / o["t_total"], "time_first_solution_s": o["t_first"],
                                   "cost_best": o["cost"], "rows_at_changes": ro},
           "same_trees": same}
    # c_best reached by both at matching wall-clock marks
    marks = []
    for t in (0.01, 0.03, 0.1, 0.3, 1.0, 3.0):
        def at(rows):
            c = None
            for row in rows:
                if row[1] <= t:
                    c = row[2]
            return c
        marks.append({"t_s": t, "gpu_c_best": at(rg), "cpu_c_best": at(ro)})
    out["c_best_at_wall_clock"] = marks
    return out


def c5_sweep(a):
    res = []
    for lib in a.libs.split(","):
        env = dict(os.environ, SMP_LIB=os.path.join(ROOT, lib) if not os.path.isabs(lib) else lib)
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c5", "--no-cpu", "--steps", "1",
               "--warmup", "1", "--iterations", str(a.iterations)]
        t0 = time.perf_counter()
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
        if p.returncode != 0:
            res.append({"lib": lib, "error": p.stderr[-2000:]})
            break
        line = json.loads(p.stdout.strip().splitlines()[-1])
        res.append({"lib": lib, "wall_s": time.perf_counter() - t0, "configs_per_s": line["value"],
                    "iterations_per_s": line["iterations_per_s"], "valid_configs_per_s": line["valid_configs_per_s"],
                    "ms_per_step": line["ms_per_step"], "config": line["config"]})
        print(json.dumps(res[-1]), flush=True)
    return {"config": "C5 LDS tile sweep: configurations per job tile (SMP_HELPER_CT)", "runs": res}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=("c4", "c5-sweep"))
    ap.add_argument("out")
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--iterations", type=int, default=3000)
    ap.add_argument("--libs", default="squirrel_motion_planner_amd/lib/libsmp_gpu.so")
    a = ap.parse_args()
    out = c4(a) if a.what == "c4" else c5_sweep(a)
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k not in ("gpu", "cpu_oracle_1_thread", "runs")}))


if __name__ == "__main__":
    main()
