#!/usr/bin/env python3
"""IK goal search report on one GPU: findGoalPose latency and batched controller throughput,
GPU (smp_find_goal_pose / smp_ik_solve) beside the CPU oracle on the same inputs (one host core), results compared.

    python tools/ik_report.py [out.json]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Robot, Scene  # noqa: E402

MODEL = os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json")


def cpu_name():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def goals(sc, n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        d = rng.uniform(0.4, 1.0)
        a = rng.uniform(-np.pi, np.pi)
        out.append([sc.start[0] + d * np.cos(a), sc.start[1] + d * np.sin(a), rng.uniform(0.1, 0.8),
                    rng.uniform(-np.pi, np.pi), rng.uniform(-1.5, 1.5), rng.uniform(-np.pi, np.pi)])
    return out


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "ik_report.json")
    sc = scenes.box_room()
    gp = GpuPlanner(Robot())
    gp.set_scene(Scene.from_keys(sc.keys, sc.res))
    orc = O.Oracle(O.OracleRobot(MODEL), O.OracleScene(sc.keys, sc.res))
    cur = np.array(sc.start, float)
    rep = {"scene": "C2 box scene (10x10x2 m @5 cm, 20 boxes), robot at its start pose", "cpu": cpu_name(),
           "cpu_threads": 1, "goal_search": [], "batch": []}
    gp.find_goal_pose(goals(sc, 1, 0)[0], cur, 20.0)  # warm-up (module load, first launch)
    for disc in (20.0, 10.0, 5.0):  # 10 deg: the node's setting (parameters.yaml:33)
        rows = []
        for ee in goals(sc, 16, 1):
            t0 = time.perf_counter()
            res, pose, info = gp.find_goal_pose(ee, cur, disc)
            t_gpu = time.perf_counter() - t0
            t0 = time.perf_counter()
            ores, opose, tried, chosen, iters = orc.find_goal_pose(ee, cur, disc)
            t_cpu = time.perf_counter() - t0
            same = res == ores and info["chosen"] == chosen and (res != 0 or np.array_equal(pose, opose))
            rows.append(dict(result=res, same=bool(same), candidates=info["n_candidates"], chosen=chosen,
                             cpu_tried=int(tried), cpu_ik_iterations=int(iters), gpu_ms=t_gpu * 1e3,
                             gpu_kernel_ms=info["kernel_ms"], cpu_ms=t_cpu * 1e3))
        g = np.array([r["gpu_ms"] for r in rows])
        c = np.array([r["cpu_ms"] for r in rows])
        rep["goal_search"].append(dict(discretization_deg=disc, goals=len(rows), all_same=all(r["same"] for r in rows),
                                       gpu_ms_median=float(np.median(g)), cpu_ms_median=float(np.median(c)),
                                       gpu_ms_mean=float(g.mean()), cpu_ms_mean=float(c.mean()),
                                       speedup_median=float(np.median(c / g)), rows=rows))
        print("disc %.0f: gpu median %.2f ms, cpu median %.2f ms, same %s" % (
            disc, np.median(g), np.median(c), all(r["same"] for r in rows)), flush=True)
    # batched controller runs: candidates of many goals at once (e.g. grasp-pose screening)
    for n_goals in (16, 256):
        tasks_ee, tasks_q = [], []
        for ee in goals(sc, n_goals, 2):
            t, _ = O.goal_candidates(ee, cur, 20.0)
            tasks_ee += [ee] * len(t)
            tasks_q += list(t[:, 19:27])
        tasks_ee, tasks_q = np.array(tasks_ee), np.array(tasks_q)
        gp.ik_solve(tasks_ee[:64], tasks_q[:64])
        t0 = time.perf_counter()
        r = gp.ik_solve(tasks_ee, tasks_q)
        t_gpu = time.perf_counter() - t0
        k_ms = gp.last_kernel_ms()[0]
        m = min(len(tasks_q), 272)
        t0 = time.perf_counter()
        o = orc.ik_solve(O.ik_tasks(tasks_ee[:m], tasks_q[:m]))
        t_cpu = time.perf_counter() - t0
        same = bool(np.array_equal(r["q"][:m], o["q"], equal_nan=True) and np.array_equal(r["iterations"][:m], o["iters"]))
        it_gpu = int(r["iterations"].sum())
        it_cpu = int(o["iters"].sum())
        rep["batch"].append(dict(runs=len(tasks_q), gpu_ms=t_gpu * 1e3, gpu_kernel_ms=k_ms, iterations=it_gpu,
                                 gpu_iterations_per_s=it_gpu / (k_ms * 1e-3),
                                 max_iterations_one_run=int(r["iterations"].max()),
                                 gpu_us_per_iteration_longest_run=k_ms * 1e3 / max(1, int(r["iterations"].max())),
                                 cpu_sample_runs=m, cpu_ms=t_cpu * 1e3, cpu_iterations_per_s=it_cpu / t_cpu,
                                 same_as_cpu_on_sample=same))
        print("batch %d runs: kernel %.2f ms (%.3g it/s), cpu %.3g it/s, same %s" % (
            len(tasks_q), k_ms, it_gpu / (k_ms * 1e-3), it_cpu / t_cpu, same), flush=True)
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    json.dump(rep, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
