"""Host-side mirror of the reference planner interface, over the C ABI.

`BiRRTstarPlanner` keeps the member names, argument meaning and bool/error behaviour of
birrt_star_motion_planning::BiRRTstarPlanner (birrt_star.h:27-110) as the squirrel_8dof_planner node uses it
(squirrel_8dof_planner.cpp:1221-1248): initialize, setOctree, setDisabledLinkMapCollisions,
reset_planner_and_config, setPlanningSceneInfo, init_planner, run_planner, getJointTrajectoryRef,
isConfigValid.  Every call lands in libsmp_gpu.so (HIP kernels on the GPU); nothing here computes planning
or collision results on the CPU.
"""
import ctypes

import numpy as np

from . import _lib as L
from ._lib import check, lib

_pd = ctypes.POINTER(ctypes.c_double)


def default_params(**kw):
    p = L.Params()
    lib().smp_params_default(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class Robot:
    """Robot model (KDL chain + collision model): from the committed model JSON, or (from_urdf) from the robot
    description the node holds -- URDF and SRDF text plus the sphere covers of the mesh links."""

    def __init__(self, model_json=L.MODEL_JSON, _handle=None):
        if _handle is not None:
            self.h = _handle
            return
        with open(model_json, "rb") as f:
            text = f.read()
        h = ctypes.c_void_p()
        check(lib().smp_robot_create_json(text, ctypes.byref(h)), "smp_robot_create_json")
        self.h = h

    @classmethod
    def from_urdf(cls, urdf, srdf, spheres=None):
        """smp_robot_create_urdf: KDLRobotModel + CollisionChecker construction from the description text
        (birrt_star.cpp:36-73, collision_checker.hpp:176-393)."""
        if spheres is None:
            spheres = open(L.SPHERES_JSON).read()
        enc = lambda t: t.encode() if isinstance(t, str) else bytes(t)
        h = ctypes.c_void_p()
        check(lib().smp_robot_create_urdf(enc(urdf), enc(srdf), enc(spheres), ctypes.byref(h)), "smp_robot_create_urdf")
        return cls(_handle=h)

    def device_bytes(self):
        """The device model (RobotDev) as bytes -- for comparing construction paths."""
        n = lib().smp_probe_robot_dev(self.h, None, 0)
        b = ctypes.create_string_buffer(n)
        lib().smp_probe_robot_dev(self.h, b, n)
        return b.raw

    @property
    def link_names(self):
        n = lib().smp_robot_num_links(self.h)
        return [lib().smp_robot_link_name(self.h, i).decode() for i in range(n)]

    def __del__(self):
        if getattr(self, "h", None):
            lib().smp_robot_destroy(self.h)
            self.h = None


class Scene:
    """Occupancy scene: octomap leaf keys (or a .bt stream) -> padded bitset + squared-EDT prefilter."""

    def __init__(self, h):
        self.h = h

    @classmethod
    def from_keys(cls, keys, res, z_offset=-0.02, floor_center=None, floor_distance=3.0):
        keys = np.ascontiguousarray(np.asarray(keys).reshape(-1, 3), np.uint16)
        o = L.SceneOpts()
        lib().smp_scene_opts_default(ctypes.byref(o))
        o.resolution = res
        o.z_offset = z_offset
        if floor_center is not None:
            o.insert_floor = 1
            o.floor_center[0], o.floor_center[1] = floor_center
            o.floor_distance = floor_distance
        h = ctypes.c_void_p()
        check(lib().smp_scene_from_keys(keys.ctypes.data_as(ctypes.c_void_p), len(keys), ctypes.byref(o),
                                        ctypes.byref(h)), "smp_scene_from_keys")
        return cls(h)

    @staticmethod
    def _opts(z_offset, floor_center, floor_distance):
        o = L.SceneOpts()
        lib().smp_scene_opts_default(ctypes.byref(o))
        o.z_offset = z_offset
        if floor_center is not None:
            o.insert_floor = 1
            o.floor_center[0], o.floor_center[1] = floor_center
            o.floor_distance = floor_distance
        return o

    @classmethod
    def from_bt(cls, data, z_offset=-0.02, floor_center=None, floor_distance=3.0):
        """Octomap binary file (.bt) bytes."""
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        o = cls._opts(z_offset, floor_center, floor_distance)
        h = ctypes.c_void_p()
        check(lib().smp_scene_from_bt(buf, len(data), ctypes.byref(o), ctypes.byref(h)), "smp_scene_from_bt")
        return cls(h)

    @classmethod
    def from_ot(cls, data, z_offset=-0.02, floor_center=None, floor_distance=3.0):
        """Octomap full-format file (.ot) bytes (the octomap_server's map, launch/simulation.launch:51)."""
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        o = cls._opts(z_offset, floor_center, floor_distance)
        h = ctypes.c_void_p()
        check(lib().smp_scene_from_ot(buf, len(data), ctypes.byref(o), ctypes.byref(h)), "smp_scene_from_ot")
        return cls(h)

    @classmethod
    def from_octomap_msg(cls, id, resolution, binary, data, z_offset=-0.02, floor_center=None, floor_distance=3.0):
        """octomap_msgs/Octomap fields (squirrel_8dof_planner.cpp:875-883): binaryMsgToMap / fullMsgToMap."""
        data = bytes(data)
        buf = ctypes.create_string_buffer(data, max(len(data), 1))
        o = cls._opts(z_offset, floor_center, floor_distance)
        h = ctypes.c_void_p()
        check(lib().smp_scene_from_octomap_msg(id.encode() if isinstance(id, str) else id, float(resolution),
                                               int(bool(binary)), buf, len(data), ctypes.byref(o), ctypes.byref(h)),
              "smp_scene_from_octomap_msg")
        return cls(h)

    @classmethod
    def from_grid(cls, bits, d2, dims, origin, res):
        bits = np.ascontiguousarray(bits, np.uint64)
        d2 = np.ascontiguousarray(d2, np.uint16)
        dd = (ctypes.c_int * 3)(*dims)
        oo = (ctypes.c_double * 3)(*origin)
        h = ctypes.c_void_p()
        check(lib().smp_scene_from_grid(bits.ctypes.data_as(ctypes.c_void_p), d2.ctypes.data_as(ctypes.c_void_p), dd,
                                        oo, res, ctypes.byref(h)), "smp_scene_from_grid")
        return cls(h)

    def info(self):
        dims = (ctypes.c_int * 3)()
        org = (ctypes.c_double * 3)()
        res = ctypes.c_double()
        nocc = ctypes.c_int64()
        bmin = (ctypes.c_double * 3)()
        bmax = (ctypes.c_double * 3)()
        check(lib().smp_scene_info(self.h, dims, org, ctypes.byref(res), ctypes.byref(nocc), bmin, bmax))
        return dict(dims=tuple(dims), origin=tuple(org), res=res.value, n_occupied=nocc.value,
                    bbox_min=tuple(bmin), bbox_max=tuple(bmax))

    def export(self):
        i = self.info()
        nx, ny, nz = i["dims"]
        wx = (nx + 63) // 64
        bits = np.zeros(wx * ny * nz, np.uint64)
        d2 = np.zeros(nx * ny * nz, np.uint16)
        check(lib().smp_scene_export(self.h, bits.ctypes.data_as(ctypes.c_void_p), d2.ctypes.data_as(ctypes.c_void_p)))
        return bits, d2

    def __del__(self):
        if getattr(self, "h", None):
            lib().smp_scene_destroy(self.h)
            self.h = None


class GpuPlanner:
    """Thin owner of an smp_planner (one GPU, one robot, one scene at a time)."""

    def __init__(self, robot=None, device=0, **params):
        self.robot = robot or Robot()
        self.params = default_params(**params)
        h = ctypes.c_void_p()
        check(lib().smp_planner_create(device, self.robot.h, ctypes.byref(self.params), ctypes.byref(h)),
              "smp_planner_create")
        self.h = h
        self.scene = None

    def set_scene(self, scene):
        check(lib().smp_planner_set_scene(self.h, scene.h), "smp_planner_set_scene")
        self.scene = scene

    def scene_device(self, bricks=0, d2=0, d2b=0, slab=0):
        """smp_planner_scene_device: geometry and sizes of the planner's device-resident scene; each non-zero device
        address (e.g. a torch tensor's data_ptr() on any GPU) receives a device-to-device copy of that array."""
        v = L.SceneDevice()
        v.bricks, v.d2, v.d2b, v.slab = bricks or None, d2 or None, d2b or None, slab or None
        check(lib().smp_planner_scene_device(self.h, ctypes.byref(v)), "smp_planner_scene_device")
        return v

    def set_scene_device(self, layout, bricks, d2, d2b=0, slab=0):
        """smp_planner_set_scene_device: the scene from device arrays laid out as `layout` (scene_device() of the
        sending planner), given by device address; copied, so the caller may release them afterwards."""
        v = L.SceneDevice()
        ctypes.pointer(v)[0] = layout
        v.bricks, v.d2, v.d2b, v.slab = bricks or None, d2 or None, d2b or None, slab or None
        check(lib().smp_planner_set_scene_device(self.h, ctypes.byref(v)), "smp_planner_set_scene_device")
        self.scene = None

    def set_disabled_map_links(self, names):
        arr = (ctypes.c_char_p * max(len(names), 1))(*[n.encode() for n in names])
        check(lib().smp_set_disabled_map_links(self.h, arr, len(names)))

    def check_configs(self, q, check_self=True, check_map=True):
        q = np.asarray(q, np.float64).reshape(-1, 8)
        soa = np.ascontiguousarray(q.T)
        out = np.zeros(len(q), np.uint8)
        check(lib().smp_check_configs(self.h, soa.ctypes.data_as(_pd), len(q), int(check_self), int(check_map),
                                      out.ctypes.data_as(ctypes.c_void_p)), "smp_check_configs")
        return out

    def check_sequence(self, poses, check_self=True, check_map=True):
        """Index of the first pose in collision (-1: all valid), one batched check (fold / unfold keyframes)."""
        q = np.ascontiguousarray(np.asarray(poses, np.float64).reshape(-1, 8))
        first = ctypes.c_int64()
        check(lib().smp_check_sequence(self.h, q.ctypes.data_as(_pd), len(q), int(check_self), int(check_map),
                                       ctypes.byref(first)), "smp_check_sequence")
        return first.value

    def get_collisions(self, q):
        """getCollisions (birrt_star.cpp:6910-6914): (self pairs [(link a, link b)] in pair order, map-colliding links
        in name order) of one configuration, as link names; disabled links are listed too, as in the reference."""
        qa = np.ascontiguousarray(np.asarray(q, np.float64).reshape(8))
        names = self.robot.link_names
        cap_s, cap_m = 256, len(names)
        sp = (ctypes.c_int32 * (2 * cap_s))()
        ml = (ctypes.c_int32 * max(cap_m, 1))()
        ns, nm = ctypes.c_int(), ctypes.c_int()
        check(lib().smp_get_collisions(self.h, qa.ctypes.data_as(_pd), sp, cap_s, ctypes.byref(ns), ml, cap_m,
                                       ctypes.byref(nm)), "smp_get_collisions")
        if ns.value > cap_s or nm.value > cap_m:
            raise L.SmpError(L.SMP_ERR_ARG, "smp_get_collisions: more results than capacity")
        return ([(names[sp[2 * k]], names[sp[2 * k + 1]]) for k in range(ns.value)],
                [names[ml[k]] for k in range(nm.value)])

    def ik_solve(self, ee_poses, q_inits, deviation=None, max_iter=1000):
        """getFullPoseFromEEPose's controller (run_VDLS_Control_Connector) for n (end-effector pose, start
        configuration) pairs, one wavefront each.  ee_poses: (n, 6) or one (6,) pose for every start; deviation: (6, 2)
        error bands (default: findGoalPose's).  Returns dict of arrays q (n, 8), reached, iterations, error, manip."""
        q_inits = np.asarray(q_inits, np.float64).reshape(-1, 8)
        ee = np.asarray(ee_poses, np.float64).reshape(-1, 6)
        if len(ee) == 1:
            ee = np.repeat(ee, len(q_inits), 0)
        if len(ee) != len(q_inits):
            raise ValueError("ik_solve: %d end-effector poses for %d start configurations" % (len(ee), len(q_inits)))
        dev = np.asarray(IK_DEVIATION if deviation is None else deviation, np.float64).reshape(6, 2)
        n = len(q_inits)
        reqs = (L.IkRequest * max(n, 1))()
        for i in range(n):
            r = reqs[i]
            for k in range(6):
                r.ee_pose[k] = float(ee[i, k])
                r.deviation[k][0], r.deviation[k][1] = float(dev[k, 0]), float(dev[k, 1])
            for j in range(8):
                r.q_init[j] = float(q_inits[i, j])
            r.max_iter = int(max_iter)
        res = (L.IkResult * max(n, 1))()
        check(lib().smp_ik_solve(self.h, reqs, n, res), "smp_ik_solve")
        return dict(q=np.array([list(r.q) for r in res[:n]]).reshape(n, 8),
                    reached=np.array([r.reached for r in res[:n]], np.int32),
                    iterations=np.array([r.iterations for r in res[:n]], np.int32),
                    fallback=np.array([r.fallback_iterations for r in res[:n]], np.int32),
                    error=np.array([list(r.error) for r in res[:n]]).reshape(n, 6),
                    manip=np.array([r.manipulability for r in res[:n]]))

    def find_goal_pose(self, ee_pose, pose_current, discretization_deg=20.0, check_self=True, check_map=True):
        """Planner::findGoalPose -> (result 0 found / 1 collision / 2 no IK solution, pose_goal or None, info dict)."""
        ee = np.ascontiguousarray(ee_pose, np.float64).reshape(6)
        cur = np.ascontiguousarray(pose_current, np.float64).reshape(8)
        goal = np.zeros(8)
        res = ctypes.c_int()
        info = L.GoalSearch()
        check(lib().smp_find_goal_pose(self.h, ee.ctypes.data_as(_pd), cur.ctypes.data_as(_pd),
                                       float(discretization_deg), int(check_self), int(check_map),
                                       goal.ctypes.data_as(_pd), ctypes.byref(res), ctypes.byref(info)),
              "smp_find_goal_pose")
        d = {f: getattr(info, f) for f, _ in L.GoalSearch._fields_}
        return res.value, (goal if res.value == 0 else None), d

    def last_kernel_ms(self):
        a, b = ctypes.c_double(), ctypes.c_double()
        n = ctypes.c_int64()
        check(lib().smp_last_kernel_ms(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(n)))
        return a.value, b.value, n.value

    @staticmethod
    def make_query(start, goal, env_x=(0, 0), env_y=(0, 0), check_self=True, check_map=True, iterations=None,
                   seconds=None, samples=None, seed=1, query_id=0):
        """One query; the budget is `seconds`, else `samples` (collision-checked configurations), else
        `iterations` (default 1000)."""
        q = L.Query()
        for j in range(8):
            q.start[j] = float(start[j])
            q.goal[j] = float(goal[j])
        q.env_x[0], q.env_x[1] = env_x
        q.env_y[0], q.env_y[1] = env_y
        q.check_self, q.check_map = int(check_self), int(check_map)
        if seconds is not None:
            q.budget_kind, q.budget = L.BUDGET_SECONDS, float(seconds)
        elif samples is not None:
            q.budget_kind, q.budget = L.BUDGET_SAMPLES, float(samples)
        else:
            q.budget_kind, q.budget = L.BUDGET_ITERATIONS, float(1000 if iterations is None else iterations)
        q.seed = seed
        q.query_id = query_id
        return q

    def plan_batch(self, queries):
        n = len(queries)
        qa = (L.Query * n)(*queries)
        ra = (L.Result * n)()
        rc = lib().smp_plan_batch(self.h, qa, n, ra)
        out = []
        for r in ra:
            d = _result_dict(r)
            lib().smp_result_free(ctypes.byref(r))
            out.append(d)
        # per-query outcomes (a path, no path, invalid start / goal / budget, a full tree) come back in the results;
        # a failure of the call itself (HIP error, no device, the no-progress guard) raises
        failed = [d["status"] for d in out if d["status"] in _CALL_FAILURES]
        if rc in _CALL_FAILURES or failed:
            raise L.SmpError(rc if rc in _CALL_FAILURES else failed[0], "smp_plan_batch")
        return out

    def plan(self, query):
        return self.plan_batch([query])[0]

    @staticmethod
    def share_scene(planners, src=0):
        """smp_planners_share_scene: planners[src]'s scene to the others (xGMI peer copies across GPUs)."""
        arr = (ctypes.c_void_p * len(planners))(*[p.h.value for p in planners])
        check(lib().smp_planners_share_scene(arr, len(planners), int(src)), "smp_planners_share_scene")
        for k, p in enumerate(planners):
            if k != src:
                p.scene = planners[src].scene

    @staticmethod
    def plan_multi(planners, queries):
        """smp_plan_multi: query i on planners[i % len(planners)], all planners concurrently; results in query
        order (per-query outcomes in the dicts, call failures raise as plan_batch)."""
        n = len(queries)
        arr = (ctypes.c_void_p * len(planners))(*[p.h.value for p in planners])
        qa = (L.Query * n)(*queries)
        ra = (L.Result * n)()
        rc = lib().smp_plan_multi(arr, len(planners), qa, n, ra)
        if rc == L.SMP_ERR_ARG and all(r.status == L.SMP_ERR_ARG for r in ra):
            raise L.SmpError(rc, "smp_plan_multi")
        out = []
        for r in ra:
            d = _result_dict(r)
            lib().smp_result_free(ctypes.byref(r))
            out.append(d)
        failed = [d["status"] for d in out if d["status"] in _CALL_FAILURES]
        if rc in _CALL_FAILURES or failed:
            raise L.SmpError(rc if rc in _CALL_FAILURES else failed[0], "smp_plan_multi")
        return out

    def tree(self, which):
        n = lib().smp_get_tree(self.h, which, None, None, None)
        if n < 0:
            raise L.SmpError(L.SMP_ERR_ARG, "smp_get_tree")
        par = np.zeros(n, np.int32)
        conf = np.zeros((n, 8))
        cost = np.zeros((n, 3))
        lib().smp_get_tree(self.h, which, par.ctypes.data_as(ctypes.c_void_p), conf.ctypes.data_as(ctypes.c_void_p),
                           cost.ctypes.data_as(ctypes.c_void_p))
        return par, conf, cost

    def export_state(self):
        """The last query's state in the form oracle.Oracle.resume() takes (test infrastructure: the oracle continues
        the GPU's run from it -- large-tree parity and the CPU timed at the GPU's tree sizes)."""
        iv = np.zeros(16, np.int64)
        dv = np.zeros(25)
        check(lib().smp_probe_export_state(self.h, iv.ctypes.data_as(ctypes.c_void_p), dv.ctypes.data_as(_pd)),
              "smp_probe_export_state")
        st = {"iv": iv[:12].copy(), "dv": dv}
        for which, name in ((0, "start"), (1, "goal")):
            par, conf, cost = self.tree(which)
            n = len(par)
            fc, ns = np.zeros(n, np.int32), np.zeros(n, np.int32)
            es, et = np.zeros((n, 8)), np.zeros((n, 8))
            check(lib().smp_probe_export_tree(self.h, which, fc.ctypes.data_as(ctypes.c_void_p),
                                              ns.ctypes.data_as(ctypes.c_void_p), es.ctypes.data_as(_pd),
                                              et.ctypes.data_as(_pd)), "smp_probe_export_tree")
            # the reference's out-edge order: the GPU's child lists (head insertion) reversed
            off = np.zeros(n + 1, np.int32)
            ids = []
            for i in range(n):
                off[i] = len(ids)
                ch = []
                c = int(fc[i])
                while c >= 0:
                    ch.append(c)
                    c = int(ns[c])
                ids.extend(reversed(ch))
            off[n] = len(ids)
            st[name] = {"parent": par, "conf": conf, "cost": cost, "e_start": es, "e_target": et, "child_off": off,
                        "child_ids": np.array(ids, np.int32), "edges": int(iv[12 + which]),
                        "rewires": int(iv[14 + which])}
        return st

    def __del__(self):
        if getattr(self, "h", None):
            lib().smp_planner_destroy(self.h)
            self.h = None


# findGoalPose's endEffectorDeviations (squirrel_8dof_planner.cpp:1131-1137)
IK_DEVIATION = [(-0.005, 0.005)] * 3 + [(-0.025, 0.025)] * 3

_CALL_FAILURES = (L.SMP_ERR_HIP, L.SMP_ERR_NO_DEVICE, L.SMP_ERR_PARSE)


def _result_dict(r):
    s = r.stats
    d = {f: getattr(s, f) for f, _ in L.Stats._fields_}
    d["cost_best"] = list(s.cost_best)
    d["cost_theoretical"] = list(s.cost_theoretical)
    names = ["sample", "nearest", "expand", "near", "choose_parent", "rewire", "connect", "collide_tiles",
             "n_tiles", "edge_costs", "via_chains", "n_via_steps", "tile_local_frames|job_publish", "tile_chain|job_own_tiles",
             "tile_centres_w0|job_wait", "tile_tests|n_jobs", "tiles_in_expand", "tiles_in_choose", "tiles_in_rewire",
             "tiles_in_connect", "checked_expand", "checked_choose", "checked_rewire", "checked_connect",
             "slots_expand", "slots_choose", "slots_rewire", "slots_connect"]
    d["phases"] = {n: s.phase_seconds[i] for i, n in enumerate(names)}
    d["phase_raw"] = list(s.phase_seconds)
    d["scout_phases"] = list(s.scout_phase_seconds)
    d["status"] = r.status
    n = r.n_waypoints
    d["path"] = np.ctypeslib.as_array(r.waypoints, shape=(n, 8)).copy() if n else np.zeros((0, 8))
    m = r.n_cost_rows
    d["cost_rows"] = np.ctypeslib.as_array(r.cost_rows, shape=(m, 5)).copy() if m else np.zeros((0, 5))
    return d


class BiRRTstarPlanner:
    """Drop-in mirror of birrt_star_motion_planning::BiRRTstarPlanner for the C-space (search_space = 1) path.

    Call sequence of the node (squirrel_8dof_planner.cpp:1221-1248):
        initialize(); setOctree(...); setDisabledLinkMapCollisions([...]);
        reset_planner_and_config(); setPlanningSceneInfo(x, y, name);
        init_planner(start, goal, 1, self, map) -> bool; run_planner(1, 1, T, False, 0.0, n) -> bool;
        getJointTrajectoryRef()
    Extra (not in the reference): seed / query_id for reproducible runs, `stats` of the last run.
    """

    def __init__(self, device=0, seed=1):
        self.device = device
        self.seed = seed
        self.query_id = 0
        self._gpu = None
        self._env = [(0.0, 0.0), (0.0, 0.0)]
        self._start = self._goal = None
        self._flags = (True, True)
        self._traj = []
        self.stats = None

    def initialize(self, planning_group="robotino_robot", **params):
        if planning_group != "robotino_robot":
            raise ValueError("only the robotino_robot group (robotino_plan.srdf:4-6) is modelled")
        self._gpu = GpuPlanner(device=self.device, **params)

    def setOctree(self, octree, resolution=None, floor_center=None, floor_distance=3.0):
        """octree: .bt or .ot file bytes, or an (n, 3) array of occupied octomap keys (then `resolution` is
        required).  The first line tells the formats apart (AbstractOcTree::read / OcTree::readBinary)."""
        if isinstance(octree, (bytes, bytearray)):
            full = bytes(octree).startswith(b"# Octomap OcTree file")
            sc = (Scene.from_ot if full else Scene.from_bt)(octree, floor_center=floor_center,
                                                            floor_distance=floor_distance)
        else:
            sc = Scene.from_keys(octree, resolution, floor_center=floor_center, floor_distance=floor_distance)
        self._gpu.set_scene(sc)

    def setDisabledLinkMapCollisions(self, links):
        self._gpu.set_disabled_map_links(list(links))

    def setPlanningSceneInfo(self, size_x, size_y, scene_name="scenario"):
        self._env = [(float(size_x[0]), float(size_x[1])), (float(size_y[0]), float(size_y[1]))]

    def reset_planner_and_config(self):
        self._env = [(0.0, 0.0), (0.0, 0.0)]
        self._start = self._goal = None
        self._traj = []

    def isConfigValid(self, config, check_self_collision=True, check_map_collision=True):
        return bool(self._gpu.check_configs([config], check_self_collision, check_map_collision)[0])

    def getCollisions(self, joint_positions, self_collisions, map_collisions):
        """birrt_star.cpp:6910-6914: appends to the two lists, as the reference does."""
        s, m = self._gpu.get_collisions(joint_positions)
        self_collisions.extend(s)
        map_collisions.extend(m)

    def init_planner(self, start_conf, goal_conf, search_space=1, check_self_collision=True, check_map_collision=True):
        if len(start_conf) != 8 or len(goal_conf) != 8 or search_space != 1:
            return False  # birrt_star.cpp:338-342 (control-space search is out of scope)
        v = self._gpu.check_configs([start_conf, goal_conf], check_self_collision, check_map_collision)
        if not v[0] or not v[1]:
            return False  # birrt_star.cpp:350-362
        self._start, self._goal = list(start_conf), list(goal_conf)
        self._flags = (check_self_collision, check_map_collision)
        return True

    def run_planner(self, search_space=1, flag_iter_or_time=1, max_iter_time=30.0, show_tree_vis=False,
                    iter_sleep=0.0, planner_run_number=0):
        if self._start is None or search_space != 1:
            return False
        kw = dict(seconds=max_iter_time) if flag_iter_or_time else dict(iterations=int(max_iter_time))
        q = GpuPlanner.make_query(self._start, self._goal, self._env[0], self._env[1], self._flags[0],
                                  self._flags[1], seed=self.seed, query_id=self.query_id, **kw)
        r = self._gpu.plan(q)
        self.stats = r
        if r["status"] not in (L.SMP_OK, L.SMP_ERR_NO_SOLUTION):
            raise L.SmpError(r["status"], "run_planner")
        self._traj = [list(map(float, w)) for w in r["path"]]
        return r["status"] == L.SMP_OK

    def getJointTrajectoryRef(self):
        return self._traj

    def getFullPoseFromEEPose(self, endEffectorPose, endEffectorDeviations, poseInit, poseSolution):
        """birrt_star.cpp:1627-1686: the VDLS controller from poseInit towards endEffectorPose (x, y, z, roll, pitch,
        yaw); on REACHED fills the list poseSolution with the final configuration and returns True."""
        r = self._gpu.ik_solve([endEffectorPose], [poseInit], deviation=endEffectorDeviations)
        if not r["reached"][0]:
            return False
        poseSolution[:] = [float(v) for v in r["q"][0]]
        return True


def normalize_trajectory(raw, normalized_pose):
    """Planner::normalizeTrajectory (squirrel_8dof_planner.cpp:1557-1637) through the C ABI: the resampled poses as
    an (m, dim) array, or None where the reference returns without touching its output (dim < 1, <= 1 pose)."""
    np_ = np.ascontiguousarray(np.asarray(normalized_pose, np.float64).reshape(-1))
    raw = np.ascontiguousarray(np.asarray(raw, np.float64))
    dim = len(np_)
    if raw.ndim != 2 or len(raw) <= 1 or dim < 1 or raw.shape[1] != dim:
        return None
    n_out = ctypes.c_int64()
    check(lib().smp_normalize_trajectory(raw.ctypes.data_as(_pd), len(raw), dim, np_.ctypes.data_as(_pd), None, 0,
                                         ctypes.byref(n_out)), "smp_normalize_trajectory")
    out = np.zeros((n_out.value, dim))
    check(lib().smp_normalize_trajectory(raw.ctypes.data_as(_pd), len(raw), dim, np_.ctypes.data_as(_pd),
                                         out.ctypes.data_as(_pd), n_out.value, ctypes.byref(n_out)),
          "smp_normalize_trajectory")
    return out
