"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes front end of oracle/_build/liboracle.so (the sequential CPU restatement of the reference BiRRT*
C-space planner, see smp_oracle.cpp) plus an independent numpy/scipy construction of the scene grid
(occupancy bitset + squared-EDT prefilter field).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module.  Parity is "unpinned" against the original binaries:
the reference ships no tests or golden vectors and cannot be built here.
"""
import ctypes
import json
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

_i = ctypes.c_int
_d = ctypes.c_double
_pi = ctypes.POINTER(ctypes.c_int)
_pd = ctypes.POINTER(ctypes.c_double)


class RobotDesc(ctypes.Structure):
    _fields_ = [("n_links", _i), ("parent", _pi), ("joint", _pi), ("type", _pi),
                ("axis", _pd), ("origin", _pd), ("R", _pd), ("p", _pd),
                ("n_seg", _i), ("seg_joint", _pi), ("seg_type", _pi),
                ("seg_axis", _pd), ("seg_origin", _pd), ("seg_R", _pd), ("seg_p", _pd),
                ("n_sph", _i), ("sph_link", _pi), ("sph_c", _pd), ("sph_r", _pd),
                ("lb_has", _pi), ("lb_c", _pd), ("lb_r", _pd),
                ("n_pairs", _i), ("pair_a", _pi), ("pair_b", _pi),
                ("q_min", _pd), ("q_max", _pd), ("rev", _pi), ("root_z", _d),
                ("n_chain", _i), ("ch_type", _pi), ("ch_joint", _pi), ("ch_body", _pi),
                ("ch_axis", _pd), ("ch_origin", _pd), ("ch_R", _pd), ("ch_p", _pd),
                ("n_body", _i), ("sph_body", _pi), ("lb_body", _pi), ("sph_cb", _pd), ("lb_cb", _pd),
                ("n_prim", _i), ("prim_type", _pi), ("prim_body", _pi), ("prim_link", _pi),
                ("prim_cb", _pd), ("prim_ab", _pd), ("prim_h", _pd), ("prim_rxy", _pd)]


class SceneDesc(ctypes.Structure):
    _fields_ = [("nx", _i), ("ny", _i), ("nz", _i), ("ox", _d), ("oy", _d), ("oz", _d), ("res", _d),
                ("bits", ctypes.POINTER(ctypes.c_uint64)), ("d2", ctypes.POINTER(ctypes.c_uint16)),
                ("n_slab", _i), ("slab", ctypes.POINTER(ctypes.c_uint16))]


class Params(ctypes.Structure):
    _fields_ = [("near_r", _d), ("step", _d), ("n_pts", _i), ("max_near", _i), ("opt_thresh", _d),
                ("tree_opt", _i), ("informed", _i), ("env_x", _d * 2), ("env_y", _d * 2),
                ("self_", _i), ("map", _i), ("seed", ctypes.c_uint64), ("query", ctypes.c_uint32),
                ("max_iter", _i), ("max_time", _d), ("max_checked", ctypes.c_longlong), ("threads", _i)]


class Result(ctypes.Structure):
    _fields_ = [("status", _i), ("iterations", ctypes.c_longlong), ("first_iter", ctypes.c_longlong),
                ("last_iter", ctypes.c_longlong), ("checked", ctypes.c_longlong), ("valid", ctypes.c_longlong),
                ("ck_calls", ctypes.c_longlong), ("t_first", _d), ("t_total", _d), ("cost", _d * 3), ("h0", _d * 3),
                ("n_start", _i), ("n_goal", _i), ("edges_start", _i), ("edges_goal", _i),
                ("rewires_start", _i), ("rewires_goal", _i), ("conn_start", _i), ("conn_b", _i), ("conn_a", _i),
                ("n_wp", _i)]


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_create.restype = ctypes.c_void_p
        L.orc_create.argtypes = [ctypes.POINTER(RobotDesc), ctypes.POINTER(SceneDesc), ctypes.c_void_p]
        L.orc_destroy.argtypes = [ctypes.c_void_p]
        L.orc_check_configs.argtypes = [ctypes.c_void_p, _pd, _i, _i, _i, ctypes.c_void_p]
        L.orc_collisions.argtypes = [ctypes.c_void_p, _pd, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_fk.argtypes = [ctypes.c_void_p, _pd, _i, _pd, _pd]
        L.orc_sincos.argtypes = [_pd, _i, _pd, _pd]
        L.orc_body_fk.argtypes = [ctypes.c_void_p, _pd, _i, _pd]
        L.orc_philox.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_u01.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, _i, _pd]
        L.orc_plan.argtypes = [ctypes.c_void_p, _pd, _pd, ctypes.POINTER(Params), ctypes.POINTER(Result)]
        L.orc_get_path.argtypes = [ctypes.c_void_p, _pd]
        L.orc_get_tree.argtypes = [ctypes.c_void_p, _i, _pi, _pd, _pd]
        L.orc_get_tree.restype = _i
        L.orc_get_cost_rows.argtypes = [ctypes.c_void_p, _pd]
        L.orc_get_cost_rows.restype = _i
        L.orc_get_cost_row_times.argtypes = [ctypes.c_void_p, _pd]
        L.orc_get_cost_row_times.restype = _i
        L.orc_ik_solve.argtypes = [ctypes.c_void_p, _pd, _i, _i, _pd, _pi]
        L.orc_ik_goal.argtypes = [_pd, _pd]
        L.orc_ik_fk_jac.argtypes = [ctypes.c_void_p, _pd, _i, _pd, _pd]
        L.orc_goal_candidates.argtypes = [_pd, _pd, _d, _pd, _pi]
        L.orc_goal_candidates.restype = _i
        L.orc_find_goal_pose.argtypes = [ctypes.c_void_p, _pd, _pd, _d, _i, _i, _pd,
                                         ctypes.POINTER(ctypes.c_longlong)]
        L.orc_find_goal_pose.restype = _i
        L.orc_resume_begin.argtypes = [ctypes.c_void_p, _pd, _pd, ctypes.POINTER(Params)]
        L.orc_resume_begin.restype = _i
        L.orc_resume_tree.argtypes = [ctypes.c_void_p, _i, _i, _pi, _pd, _pd, _pd, _pd, _pi, _pi, _i, _i]
        L.orc_resume_run.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong), _pd, ctypes.POINTER(Result)]
        L.orc_resume_run.restype = _i
        L.orc_export_tree.argtypes = [ctypes.c_void_p, _i, _pd, _pd, _pi, _pi]
        L.orc_export_tree.restype = _i
        L.orc_export_state.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong), _pd]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


# ------------------------------------------------------------------------------------------ robot
class OracleRobot:
    """Flat arrays of the robot model JSON (squirrel_motion_planner_amd/data/robotino_model.json)."""

    TYPES = {"None": 0, "RotAxis": 1, "TransAxis": 2}

    def __init__(self, model):
        if isinstance(model, str):
            with open(model) as f:
                model = json.load(f)
        self.model = model
        L = model["links"]
        n = len(L)
        self.n_links = n
        self.parent = np.array([e["parent"] for e in L], np.int32)
        self.joint = np.array([e["joint"] for e in L], np.int32)
        self.type = np.array([self.TYPES[e["type"]] for e in L], np.int32)
        self.axis = np.array([e["axis"] for e in L], np.float64).ravel()
        self.origin = np.array([e["origin"] for e in L], np.float64).ravel()
        self.R = np.array([e["R"] for e in L], np.float64).ravel()
        self.p = np.array([e["p"] for e in L], np.float64).ravel()
        C = model["chain"]
        self.n_seg = len(C)
        self.seg_joint = np.array([e["joint"] for e in C], np.int32)
        self.seg_type = np.array([self.TYPES[e["type"]] for e in C], np.int32)
        self.seg_axis = np.array([e["axis"] for e in C], np.float64).ravel()
        self.seg_origin = np.array([e["origin"] for e in C], np.float64).ravel()
        self.seg_R = np.array([e["ftip_R"] for e in C], np.float64).ravel()
        self.seg_p = np.array([e["ftip_p"] for e in C], np.float64).ravel()
        S = model["spheres"]
        self.n_sph = len(S)
        self.sph_link = np.array([s["link"] for s in S], np.int32)
        self.sph_c = np.array([s["c"] for s in S], np.float64).ravel()
        self.sph_r = np.array([s["r"] for s in S], np.float64)
        self.lb_has = np.zeros(n, np.int32)
        self.lb_c = np.zeros(3 * n, np.float64)
        self.lb_r = np.zeros(n, np.float64)
        for b in model["link_bounds"]:
            self.lb_has[b["link"]] = 1
            self.lb_c[3 * b["link"]:3 * b["link"] + 3] = b["c"]
            self.lb_r[b["link"]] = b["r"]
        P = model["self_pairs"]
        self.n_pairs = len(P)
        self.pair_a = np.array([a for a, b in P], np.int32)
        self.pair_b = np.array([b for a, b in P], np.int32)
        self.q_min = np.array(model["q_min"], np.float64)
        self.q_max = np.array(model["q_max"], np.float64)
        self.rev = np.array(model["joint_is_revolute"], np.int32)
        self.root_z = float(model["root_z"])
        self.link_names = [e["name"] for e in L]
        BC = model["body_chain"]
        self.n_chain = len(BC)
        self.ch_type = np.array([self.TYPES[e["type"]] for e in BC], np.int32)
        self.ch_joint = np.array([e["joint"] for e in BC], np.int32)
        self.ch_body = np.array([e["body"] for e in BC], np.int32)
        self.ch_axis = np.array([e["axis"] for e in BC], np.float64).ravel()
        self.ch_origin = np.array([e["origin"] for e in BC], np.float64).ravel()
        self.ch_R = np.array([e["R"] for e in BC], np.float64).ravel()
        self.ch_p = np.array([e["p"] for e in BC], np.float64).ravel()
        self.n_body = len(model["bodies"])
        self.sph_body = np.array([s["body"] for s in S], np.int32)
        self.sph_cb = np.array([s["cb"] for s in S], np.float64).ravel()
        self.lb_body = np.zeros(n, np.int32)
        self.lb_cb = np.zeros(3 * n, np.float64)
        for b in model["link_bounds"]:
            self.lb_body[b["link"]] = b["body"]
            self.lb_cb[3 * b["link"]:3 * b["link"] + 3] = b["cb"]
        PR = model.get("prims", [])
        self.n_prim = len(PR)
        self.prim_type = np.array([1 if p["type"] == "box" else 2 for p in PR] or [0], np.int32)
        self.prim_body = np.array([p["body"] for p in PR] or [0], np.int32)
        self.prim_link = np.array([p["link"] for p in PR] or [0], np.int32)
        self.prim_cb = np.array([p["cb"] for p in PR] or [[0.0] * 3], np.float64).ravel()
        self.prim_ab = np.array([p["ab"] for p in PR] or [[0.0] * 3], np.float64).ravel()
        self.prim_h = np.array([p["half"] for p in PR] or [[0.0] * 3], np.float64).ravel()
        self.prim_rxy = np.array([p["rxy"] for p in PR] or [0.0], np.float64)

    def desc(self):
        d = RobotDesc()
        d.n_links = self.n_links
        d.parent, d.joint, d.type = _p(self.parent, _i), _p(self.joint, _i), _p(self.type, _i)
        d.axis, d.origin, d.R, d.p = _p(self.axis, _d), _p(self.origin, _d), _p(self.R, _d), _p(self.p, _d)
        d.n_seg = self.n_seg
        d.seg_joint, d.seg_type = _p(self.seg_joint, _i), _p(self.seg_type, _i)
        d.seg_axis, d.seg_origin = _p(self.seg_axis, _d), _p(self.seg_origin, _d)
        d.seg_R, d.seg_p = _p(self.seg_R, _d), _p(self.seg_p, _d)
        d.n_sph = self.n_sph
        d.sph_link, d.sph_c, d.sph_r = _p(self.sph_link, _i), _p(self.sph_c, _d), _p(self.sph_r, _d)
        d.lb_has, d.lb_c, d.lb_r = _p(self.lb_has, _i), _p(self.lb_c, _d), _p(self.lb_r, _d)
        d.n_pairs = self.n_pairs
        d.pair_a, d.pair_b = _p(self.pair_a, _i), _p(self.pair_b, _i)
        d.q_min, d.q_max, d.rev = _p(self.q_min, _d), _p(self.q_max, _d), _p(self.rev, _i)
        d.root_z = self.root_z
        d.n_chain = self.n_chain
        d.ch_type, d.ch_joint, d.ch_body = _p(self.ch_type, _i), _p(self.ch_joint, _i), _p(self.ch_body, _i)
        d.ch_axis, d.ch_origin = _p(self.ch_axis, _d), _p(self.ch_origin, _d)
        d.ch_R, d.ch_p = _p(self.ch_R, _d), _p(self.ch_p, _d)
        d.n_body = self.n_body
        d.sph_body, d.lb_body = _p(self.sph_body, _i), _p(self.lb_body, _i)
        d.sph_cb, d.lb_cb = _p(self.sph_cb, _d), _p(self.lb_cb, _d)
        d.n_prim = self.n_prim
        d.prim_type, d.prim_body, d.prim_link = _p(self.prim_type, _i), _p(self.prim_body, _i), _p(self.prim_link, _i)
        d.prim_cb, d.prim_ab = _p(self.prim_cb, _d), _p(self.prim_ab, _d)
        d.prim_h, d.prim_rxy = _p(self.prim_h, _d), _p(self.prim_rxy, _d)
        return d


# ------------------------------------------------------------------------------------------ scene
KEY_OFFSET = 32768  # octomap tree_max_val


def grid_pad_cells(res):
    """Padding around the occupied key bbox: sphere / primitive reaches are <= 0.45 m."""
    return int(math.ceil(0.45 / res)) + 2


class OracleScene:
    """Dense padded grid built from occupied octree keys (independent of the product's C++ builder)."""

    def __init__(self, keys, res, z_offset=-0.02):
        keys = np.asarray(keys, dtype=np.int64).reshape(-1, 3)
        self.res = float(res)
        if len(keys) == 0:
            self.nx = self.ny = self.nz = 1
            self.ox = self.oy = 0.0
            self.oz = 0.0 + z_offset
            occ = np.zeros((1, 1, 1), bool)
        else:
            pad = grid_pad_cells(res)
            kmin = keys.min(0) - pad
            kmax = keys.max(0) + pad
            self.nx, self.ny, self.nz = [int(v) for v in (kmax - kmin + 1)]
            self.ox = float((kmin[0] - KEY_OFFSET)) * self.res
            self.oy = float((kmin[1] - KEY_OFFSET)) * self.res
            self.oz = float((kmin[2] - KEY_OFFSET)) * self.res + z_offset
            occ = np.zeros((self.nz, self.ny, self.nx), bool)
            rel = keys - kmin
            occ[rel[:, 2], rel[:, 1], rel[:, 0]] = True
        self.occ = occ
        wx = (self.nx + 63) // 64
        padded = np.zeros((self.nz, self.ny, wx * 64), bool)
        padded[:, :, :self.nx] = occ
        self.bits = np.packbits(padded.reshape(-1, 64), axis=1, bitorder="little").view("<u8").astype(np.uint64).ravel()
        if occ.any():
            # squared box-to-box gap to the nearest occupied cell = squared EDT of the 3x3x3-dilated occupancy
            from scipy.ndimage import binary_dilation, distance_transform_edt
            d = distance_transform_edt(~binary_dilation(occ, structure=np.ones((3, 3, 3), bool)))
            d2 = np.rint(d * d)
            self.d2 = np.minimum(d2, 65535).astype(np.uint16).ravel()
        else:
            self.d2 = np.full(self.nx * self.ny * self.nz, 65535, np.uint16)

    def slabs(self, zranges):
        """Per primitive, the 2-D box-gap field of the occupancy projected over the layers whose cells meet its z range
        (zlo, zhi): squared EDT (cells) of the 3x3-dilated projection, clamped to 65535 (scipy, independent of the
        product's C++ builder)."""
        from scipy.ndimage import binary_dilation, distance_transform_edt
        out = []
        for zlo, zhi in zranges:
            k0 = max(0, int(math.floor((zlo - self.oz) / self.res)) - 1)
            k1 = min(self.nz - 1, int(math.floor((zhi - self.oz) / self.res)) + 1)
            while k0 <= k1 and self.oz + (k0 + 1) * self.res < zlo:
                k0 += 1
            while k1 >= k0 and self.oz + k1 * self.res > zhi:
                k1 -= 1
            proj = self.occ[k0:k1 + 1].any(0) if k0 <= k1 else np.zeros((self.ny, self.nx), bool)
            if proj.any():
                d = distance_transform_edt(~binary_dilation(proj, structure=np.ones((3, 3), bool)))
                out.append(np.minimum(np.rint(d * d), 65535).astype(np.uint16).ravel())
            else:
                out.append(np.full(self.nx * self.ny, 65535, np.uint16))
        return out

    def desc(self, slabs=()):
        d = SceneDesc()
        d.nx, d.ny, d.nz = self.nx, self.ny, self.nz
        d.ox, d.oy, d.oz, d.res = self.ox, self.oy, self.oz, self.res
        d.bits = _p(self.bits, ctypes.c_uint64)
        d.d2 = _p(self.d2, ctypes.c_uint16)
        self._slab = np.ascontiguousarray(np.concatenate(slabs) if len(slabs) else np.zeros(1, np.uint16))
        d.n_slab = len(slabs)
        d.slab = _p(self._slab, ctypes.c_uint16)
        return d


# ------------------------------------------------------------------------------------------ planner
DEFAULT_PARAMS = dict(near_r=4.0, step=0.5, n_pts=20, max_near=20, opt_thresh=1.0, tree_opt=1, informed=1,
                      env_x=(0.0, 0.0), env_y=(0.0, 0.0), self_=1, map=1, seed=1, query=0, max_iter=1000,
                      max_time=0.0, max_checked=0, threads=1)


class Oracle:
    def __init__(self, robot, scene=None, map_enabled=None):
        self.robot = robot if isinstance(robot, OracleRobot) else OracleRobot(robot)
        self.scene = scene
        self._rd = self.robot.desc()
        self._sd = None
        if scene is not None:
            rb = self.robot
            slabs = []
            if rb.n_prim:
                # the primitives' bodies are planar: their centre z is the one of q = 0 (margin 1e-6 m)
                h0 = lib().orc_create(ctypes.byref(self._rd), None, None)
                fr = np.zeros((1, rb.n_body, 12))
                lib().orc_body_fk(h0, _p(np.zeros(8), _d), 1, _p(fr, _d))
                lib().orc_destroy(h0)
                zr = []
                for k in range(rb.n_prim):
                    B = fr[0, rb.prim_body[k]]
                    cb = rb.prim_cb[3 * k:3 * k + 3]
                    zc = (B[6] * cb[0] + B[7] * cb[1] + B[8] * cb[2]) + B[11]
                    hz = rb.prim_h[3 * k + 2] if rb.prim_type[k] == 1 else rb.prim_h[3 * k + 1]
                    zr.append((zc - hz - 1e-6, zc + hz + 1e-6))
                slabs = scene.slabs(zr)
            self._sd = scene.desc(slabs)
        me = None
        if map_enabled is not None:
            self._me = np.ascontiguousarray(map_enabled, np.uint8)
            me = self._me.ctypes.data_as(ctypes.c_void_p)
        self.h = lib().orc_create(ctypes.byref(self._rd), ctypes.byref(self._sd) if self._sd else None, me)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_destroy(self.h)
            self.h = None

    def check_configs(self, q, self_=True, map_=True):
        q = np.ascontiguousarray(q, np.float64).reshape(-1, 8)
        out = np.zeros(len(q), np.uint8)
        lib().orc_check_configs(self.h, _p(q, _d), len(q), int(self_), int(map_), out.ctypes.data_as(ctypes.c_void_p))
        return out

    def collisions(self, q):
        """getCollisions restated (smp_oracle.cpp orc_collisions): ([(link a, link b)] of the overlapping model pairs in
        pair order, [links touching the map] in name order), as link names."""
        q = np.ascontiguousarray(q, np.float64).reshape(8)
        rb = self.robot
        lm = np.zeros(rb.n_links, np.uint8)
        ps = np.zeros(max(rb.n_pairs, 1), np.uint8)
        lib().orc_collisions(self.h, _p(q, _d), lm.ctypes.data_as(ctypes.c_void_p), ps.ctypes.data_as(ctypes.c_void_p))
        names = [e["name"] for e in rb.model["links"]]
        pairs = [(names[rb.pair_a[k]], names[rb.pair_b[k]]) for k in range(rb.n_pairs) if ps[k]]
        return pairs, sorted(names[l] for l in range(rb.n_links) if lm[l])

    def fk(self, q):
        q = np.ascontiguousarray(q, np.float64).reshape(-1, 8)
        fr = np.zeros((len(q), self.robot.n_links, 12))
        z = np.zeros(len(q))
        lib().orc_fk(self.h, _p(q, _d), len(q), _p(fr, _d), _p(z, _d))
        return fr, z

    def body_fk(self, q):
        q = np.ascontiguousarray(q, np.float64).reshape(-1, 8)
        fr = np.zeros((len(q), self.robot.n_body, 12))
        lib().orc_body_fk(self.h, _p(q, _d), len(q), _p(fr, _d))
        return fr

    def ik_solve(self, tasks, max_iter=1000):
        """run_VDLS_Control_Connector for rows of ik_tasks() -> dict of q (n x 8), err (n x 6), manip, reached,
        iters, fallback."""
        tasks = np.ascontiguousarray(tasks, np.float64).reshape(-1, 27)
        n = len(tasks)
        out = np.zeros((n, 15))
        st = np.zeros((n, 3), np.int32)
        lib().orc_ik_solve(self.h, _p(tasks, _d), n, int(max_iter), _p(out, _d), _p(st, _i))
        return dict(q=out[:, :8], err=out[:, 8:14], manip=out[:, 14], reached=st[:, 0], iters=st[:, 1],
                    fallback=st[:, 2])

    def ik_fk_jac(self, q):
        """compute_FK poses (n, 7: x y z qx qy qz qw) and float-cast KDL Jacobians (n, 6, 8)."""
        q = np.ascontiguousarray(q, np.float64).reshape(-1, 8)
        ee = np.zeros((len(q), 7))
        J = np.zeros((len(q), 6, 8))
        lib().orc_ik_fk_jac(self.h, _p(q, _d), len(q), _p(ee, _d), _p(J, _d))
        return ee, J

    def find_goal_pose(self, ee, cur, disc_deg=20.0, self_=True, map_=True):
        """Planner::findGoalPose -> (result 0/1/2, pose_goal or None, tried, chosen, summed IK iterations)."""
        ee = np.ascontiguousarray(ee, np.float64)
        cur = np.ascontiguousarray(cur, np.float64)
        pose = np.zeros(8)
        info = (ctypes.c_longlong * 3)()
        r = lib().orc_find_goal_pose(self.h, _p(ee, _d), _p(cur, _d), float(disc_deg), int(self_), int(map_),
                                     _p(pose, _d), info)
        return r, (pose if r == 0 else None), info[0], info[1], info[2]

    def export_state(self, res):
        """The last run's state in the form resume() takes (res: that run's plan() / resume() output)."""
        st = {"iv": np.zeros(12, np.int64), "dv": np.zeros(25)}
        lib().orc_export_state(self.h, st["iv"].ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), _p(st["dv"], _d))
        for which, name in ((0, "start"), (1, "goal")):
            n = len(res[name + "_parent"])
            es, et = np.zeros((n, 8)), np.zeros((n, 8))
            off = np.zeros(n + 1, np.int32)
            k = lib().orc_export_tree(self.h, which, None, None, None, None)
            ids = np.zeros(max(k, 1), np.int32)
            lib().orc_export_tree(self.h, which, _p(es, _d), _p(et, _d), _p(off, _i), _p(ids, _i))
            st[name] = {"parent": res[name + "_parent"], "conf": res[name + "_conf"], "cost": res[name + "_cost"],
                        "e_start": es, "e_target": et, "child_off": off, "child_ids": ids[:k],
                        "edges": res["edges_" + name], "rewires": res["rewires_" + name]}
        return st

    def resume(self, start, goal, state, **kw):
        """Continues a run from `state` (export_state, or the GPU planner's GpuPlanner.export_state) to the budget of
        **kw (max_iter counts from the run's start); the output is plan()'s, timed from the resume."""
        p = dict(DEFAULT_PARAMS)
        p.update(kw)
        P = Params()
        for k, v in p.items():
            if k in ("env_x", "env_y"):
                getattr(P, k)[0], getattr(P, k)[1] = v
            else:
                setattr(P, k, v)
        s = np.ascontiguousarray(start, np.float64)
        g = np.ascontiguousarray(goal, np.float64)
        st = lib().orc_resume_begin(self.h, _p(s, _d), _p(g, _d), ctypes.byref(P))
        if st:
            raise ValueError("resume: init_planner failed (%d)" % st)
        for which, name in ((0, "start"), (1, "goal")):
            t = state[name]
            par = np.ascontiguousarray(t["parent"], np.int32)
            conf = np.ascontiguousarray(t["conf"], np.float64)
            cost = np.ascontiguousarray(t["cost"], np.float64)
            es = np.ascontiguousarray(t["e_start"], np.float64)
            et = np.ascontiguousarray(t["e_target"], np.float64)
            off = np.ascontiguousarray(t["child_off"], np.int32)
            ids = np.ascontiguousarray(t["child_ids"], np.int32)
            if len(ids) == 0:
                ids = np.zeros(1, np.int32)
            lib().orc_resume_tree(self.h, which, len(par), _p(par, _i), _p(conf, _d), _p(cost, _d), _p(es, _d),
                                  _p(et, _d), _p(off, _i), _p(ids, _i), int(t["edges"]), int(t["rewires"]))
        iv = np.ascontiguousarray(state["iv"], np.int64)
        dv = np.ascontiguousarray(state["dv"], np.float64)
        R = Result()
        lib().orc_resume_run(self.h, iv.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), _p(dv, _d), ctypes.byref(R))
        return self._collect(R)

    def plan(self, start, goal, **kw):
        p = dict(DEFAULT_PARAMS)
        p.update(kw)
        P = Params()
        for k, v in p.items():
            if k in ("env_x", "env_y"):
                getattr(P, k)[0], getattr(P, k)[1] = v
            else:
                setattr(P, k, v)
        s = np.ascontiguousarray(start, np.float64)
        g = np.ascontiguousarray(goal, np.float64)
        R = Result()
        lib().orc_plan(self.h, _p(s, _d), _p(g, _d), ctypes.byref(P), ctypes.byref(R))
        return self._collect(R)

    def _collect(self, R):
        out = {f: getattr(R, f) for f, _ in Result._fields_}
        out["cost"] = list(R.cost)
        out["h0"] = list(R.h0)
        if R.status in (0, 1):
            wp = np.zeros((R.n_wp, 8))
            if R.n_wp:
                lib().orc_get_path(self.h, _p(wp, _d))
            out["path"] = wp
            for which, name in ((0, "start"), (1, "goal")):
                n = R.n_start if which == 0 else R.n_goal
                par = np.zeros(n, np.int32)
                conf = np.zeros((n, 8))
                cost = np.zeros((n, 3))
                lib().orc_get_tree(self.h, which, _p(par, _i), _p(conf, _d), _p(cost, _d))
                out[name + "_parent"], out[name + "_conf"], out[name + "_cost"] = par, conf, cost
            nr = lib().orc_get_cost_rows(self.h, None)
            rows = np.zeros((nr, 5))
            if nr:
                lib().orc_get_cost_rows(self.h, _p(rows, _d))
            out["cost_rows"] = rows
            # wall-clock seconds of each row from the planning start (reports only; the rows keep time 0)
            tr = np.zeros(nr)
            if nr:
                lib().orc_get_cost_row_times(self.h, _p(tr, _d))
            out["cost_row_times"] = tr
        return out


def ik_goal(ee):
    """[x, y, z, qx, qy, qz, qw] of an end-effector pose [x, y, z, roll, pitch, yaw] (BS:1630-1645)."""
    ee = np.ascontiguousarray(ee, np.float64)
    g = np.zeros(7)
    lib().orc_ik_goal(_p(ee, _d), _p(g, _d))
    return g


IK_DEV = np.array([[-0.005, 0.005]] * 3 + [[-0.025, 0.025]] * 3)  # findGoalPose's endEffectorDeviations (SP:1131-1137)


def ik_tasks(ee, q_init, dev=IK_DEV):
    """Rows of 27 doubles (goal quaternion pose, deviation lo[6], hi[6], q_init[8]) for Oracle.ik_solve."""
    q_init = np.asarray(q_init, np.float64).reshape(-1, 8)
    ee = np.asarray(ee, np.float64).reshape(-1, 6)
    if len(ee) == 1:
        ee = np.repeat(ee, len(q_init), 0)
    dev = np.asarray(dev, np.float64).reshape(6, 2)
    t = np.zeros((len(q_init), 27))
    for i in range(len(q_init)):
        t[i, :7] = ik_goal(ee[i])
        t[i, 7:13] = dev[:, 0]
        t[i, 13:19] = dev[:, 1]
        t[i, 19:27] = q_init[i]
    return t


def goal_candidates(ee, cur, disc_deg=20.0):
    """findGoalPose's candidate tasks (rows as ik_tasks) and the downward flag."""
    ee = np.ascontiguousarray(ee, np.float64)
    cur = np.ascontiguousarray(cur, np.float64)
    n = lib().orc_goal_candidates(_p(ee, _d), _p(cur, _d), float(disc_deg), None, None)
    t = np.zeros((n, 27))
    down = ctypes.c_int(0)
    lib().orc_goal_candidates(_p(ee, _d), _p(cur, _d), float(disc_deg), _p(t, _d), ctypes.byref(down))
    return t, bool(down.value)


def sincos(x):
    x = np.ascontiguousarray(x, np.float64)
    s, c = np.zeros_like(x), np.zeros_like(x)
    lib().orc_sincos(_p(x, _d), len(x), _p(s, _d), _p(c, _d))
    return s, c


def u01(seed, query, ctr):
    ctr = np.ascontiguousarray(ctr, np.uint32).reshape(-1, 4)
    out = np.zeros(len(ctr))
    lib().orc_u01(seed, query, ctr.ctypes.data_as(ctypes.c_void_p), len(ctr), _p(out, _d))
    return out


def philox(ctr, key):
    c = np.ascontiguousarray(ctr, np.uint32)
    k = np.ascontiguousarray(key, np.uint32)
    out = np.zeros(4, np.uint32)
    lib().orc_philox(c.ctypes.data_as(ctypes.c_void_p), k.ctypes.data_as(ctypes.c_void_p),
                     out.ctypes.data_as(ctypes.c_void_p))
    return out
