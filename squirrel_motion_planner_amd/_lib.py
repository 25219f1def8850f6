"""ctypes binding of the C ABI (include/smp_gpu.h) of libsmp_gpu.so.

This is the reference-side binding a maintainer would add: every call goes through the C ABI into the HIP
kernels.  There is no CPU fallback -- if the library is missing the import fails loudly, and without a GPU
smp_planner_create returns SMP_ERR_NO_DEVICE.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SMP_LIB") or os.path.join(HERE, "lib", "libsmp_gpu.so")  # SMP_LIB: experiment builds
MODEL_JSON = os.path.join(HERE, "data", "robotino_model.json")
SPHERES_JSON = os.path.join(HERE, "data", "robotino_spheres.json")

SMP_OK = 0
SMP_ERR_ARG = -1
SMP_ERR_START_INVALID = -2
SMP_ERR_GOAL_INVALID = -3
SMP_ERR_NO_SOLUTION = -4
SMP_ERR_HIP = -5
SMP_ERR_PARSE = -6
SMP_ERR_CAPACITY = -7
SMP_ERR_NO_DEVICE = -8

BUDGET_ITERATIONS = 0
BUDGET_SECONDS = 1
BUDGET_SAMPLES = 2

_d = ctypes.c_double
_i = ctypes.c_int
_i64 = ctypes.c_int64
_p = ctypes.c_void_p
_pd = ctypes.POINTER(ctypes.c_double)


class SceneOpts(ctypes.Structure):
    _fields_ = [("resolution", _d), ("z_offset", _d), ("insert_floor", _i), ("floor_center", _d * 2),
                ("floor_distance", _d)]


class Params(ctypes.Structure):
    _fields_ = [("near_threshold", _d), ("step_factor", _d), ("num_traj_segments", _i), ("max_near_nodes", _i),
                ("path_optimality_threshold", _d), ("tree_optimization", _i), ("informed_sampling", _i),
                ("node_capacity", _i64), ("helpers", _i), ("scout", _i)]


class Query(ctypes.Structure):
    _fields_ = [("start", _d * 8), ("goal", _d * 8), ("env_x", _d * 2), ("env_y", _d * 2), ("check_self", _i),
                ("check_map", _i), ("budget_kind", _i), ("budget", _d), ("seed", ctypes.c_uint64),
                ("query_id", ctypes.c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [("iterations", _i64), ("first_solution_iter", _i64), ("last_solution_iter", _i64),
                ("configs_checked", _i64), ("configs_valid", _i64), ("time_first_solution", _d), ("time_total", _d),
                ("cost_best", _d * 3), ("cost_theoretical", _d * 3), ("nodes_start", _i64), ("nodes_goal", _i64),
                ("edges_start", _i64), ("edges_goal", _i64), ("rewires_start", _i64), ("rewires_goal", _i64),
                ("connected_tree_is_start", ctypes.c_int32), ("conn_node_b", ctypes.c_int32),
                ("conn_node_a", ctypes.c_int32), ("nn_nodes_scanned", _i64), ("near_nodes_scanned", _i64),
                ("samples_precomputed", _i64), ("phase_seconds", _d * 32), ("scout_nn_hits", _i64),
                ("scout_near_hits", _i64), ("scout_edge_hits", _i64), ("scout_edge_misses", _i64),
                ("scout_wait_seconds", _d), ("scout_phase_seconds", _d * 32), ("helpers", ctypes.c_int32),
                ("scout", ctypes.c_int32), ("time_first_solution_host", _d)]


class Result(ctypes.Structure):
    _fields_ = [("status", _i), ("n_waypoints", _i64), ("waypoints", _pd), ("stats", Stats), ("n_cost_rows", _i64),
                ("cost_rows", _pd)]


class IkRequest(ctypes.Structure):
    _fields_ = [("ee_pose", _d * 6), ("deviation", (_d * 2) * 6), ("q_init", _d * 8), ("max_iter", _i)]


class IkResult(ctypes.Structure):
    _fields_ = [("reached", _i), ("iterations", _i), ("fallback_iterations", _i), ("q", _d * 8), ("error", _d * 6),
                ("manipulability", _d)]


class GoalSearch(ctypes.Structure):
    _fields_ = [("n_candidates", _i), ("n_reached", _i), ("chosen", _i), ("downward", _i), ("kernel_ms", _d)]


class SceneDevice(ctypes.Structure):
    """smp_scene_device: a planner's device-resident scene (geometry, sizes, device pointers)."""
    _fields_ = [("dims", _i * 3), ("origin", _d * 3), ("resolution", _d), ("n_bricks", _i64), ("n_cells", _i64),
                ("n_prim", _i), ("has_d2b", _i), ("bricks", _p), ("d2", _p), ("d2b", _p), ("slab", _p)]


# (name, restype, argtypes) of every symbol declared in include/smp_gpu.h
EXPORTS = [
    ("smp_params_default", None, [ctypes.POINTER(Params)]),
    ("smp_scene_opts_default", None, [ctypes.POINTER(SceneOpts)]),
    ("smp_robot_create_json", _i, [ctypes.c_char_p, ctypes.POINTER(_p)]),
    ("smp_robot_create_urdf", _i, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(_p)]),
    ("smp_robot_destroy", None, [_p]),
    ("smp_robot_num_links", _i, [_p]),
    ("smp_robot_link_name", ctypes.c_char_p, [_p, _i]),
    ("smp_scene_from_keys", _i, [_p, _i64, ctypes.POINTER(SceneOpts), ctypes.POINTER(_p)]),
    ("smp_scene_from_bt", _i, [_p, ctypes.c_size_t, ctypes.POINTER(SceneOpts), ctypes.POINTER(_p)]),
    ("smp_scene_from_ot", _i, [_p, ctypes.c_size_t, ctypes.POINTER(SceneOpts), ctypes.POINTER(_p)]),
    ("smp_scene_from_octomap_msg", _i, [ctypes.c_char_p, _d, _i, _p, ctypes.c_size_t, ctypes.POINTER(SceneOpts),
                                        ctypes.POINTER(_p)]),
    ("smp_scene_from_grid", _i, [_p, _p, ctypes.POINTER(_i), _pd, _d, ctypes.POINTER(_p)]),
    ("smp_scene_destroy", None, [_p]),
    ("smp_scene_info", _i, [_p, ctypes.POINTER(_i), _pd, _pd, ctypes.POINTER(_i64), _pd, _pd]),
    ("smp_scene_export", _i, [_p, _p, _p]),
    ("smp_planner_create", _i, [_i, _p, ctypes.POINTER(Params), ctypes.POINTER(_p)]),
    ("smp_planner_destroy", None, [_p]),
    ("smp_planner_set_scene", _i, [_p, _p]),
    ("smp_planner_set_params", _i, [_p, ctypes.POINTER(Params)]),
    ("smp_planner_get_params", _i, [_p, ctypes.POINTER(Params)]),
    ("smp_set_disabled_map_links", _i, [_p, ctypes.POINTER(ctypes.c_char_p), _i]),
    ("smp_plan", _i, [_p, ctypes.POINTER(Query), ctypes.POINTER(Result)]),
    ("smp_plan_batch", _i, [_p, ctypes.POINTER(Query), _i, ctypes.POINTER(Result)]),
    ("smp_plan_multi", _i, [ctypes.POINTER(_p), _i, ctypes.POINTER(Query), _i, ctypes.POINTER(Result)]),
    ("smp_planner_scene_device", _i, [_p, ctypes.POINTER(SceneDevice)]),
    ("smp_planner_set_scene_device", _i, [_p, ctypes.POINTER(SceneDevice)]),
    ("smp_planners_share_scene", _i, [ctypes.POINTER(_p), _i, _i]),
    ("smp_result_free", None, [ctypes.POINTER(Result)]),
    ("smp_get_tree", _i64, [_p, _i, _p, _p, _p]),
    ("smp_check_configs", _i, [_p, _pd, _i64, _i, _i, _p]),
    ("smp_is_config_valid", _i, [_p, _pd, _i, _i, ctypes.POINTER(_i)]),
    ("smp_check_sequence", _i, [_p, _pd, _i64, _i, _i, ctypes.POINTER(_i64)]),
    ("smp_get_collisions", _i, [_p, _pd, ctypes.POINTER(ctypes.c_int32), _i, ctypes.POINTER(_i),
                                ctypes.POINTER(ctypes.c_int32), _i, ctypes.POINTER(_i)]),
    ("smp_normalize_trajectory", _i, [_pd, _i64, _i, _pd, _pd, _i64, ctypes.POINTER(_i64)]),
    ("smp_ik_solve", _i, [_p, ctypes.POINTER(IkRequest), _i, ctypes.POINTER(IkResult)]),
    ("smp_find_goal_pose", _i, [_p, _pd, _pd, _d, _i, _i, _pd, ctypes.POINTER(_i), ctypes.POINTER(GoalSearch)]),
    ("smp_last_kernel_ms", _i, [_p, _pd, _pd, ctypes.POINTER(_i64)]),
    ("smp_strerror", ctypes.c_char_p, [_i]),
]

PROBES = [
    ("smp_probe_sincos", _i, [_i, _pd, _i, _pd, _pd]),
    ("smp_probe_u01", _i, [_i, ctypes.c_uint64, ctypes.c_uint32, _p, _i, _pd]),
    ("smp_probe_fk", _i, [_p, _pd, _i, _pd, _pd]),
    ("smp_probe_sqrt_div", _i, [_i, _pd, _pd, _i, _pd, _pd]),
    ("smp_probe_near", _i, [_i, _pd, _pd, _i, _pd, _p, _i, ctypes.c_double, _i, _p, _p, _p, _p,
                            ctypes.POINTER(ctypes.c_uint64), _pd]),
    ("smp_probe_check_latency", _i, [_p, _pd, _i64, _i, _i, _i, _i, _pd, ctypes.POINTER(ctypes.c_uint64), _pd]),
    ("smp_probe_check_shape", _i, [_p, _pd, _i64, _i, _i, _i, _i, _p]),
    ("smp_probe_export_tree", _i, [_p, _i, _p, _p, _pd, _pd]),
    ("smp_probe_export_state", _i, [_p, _p, _pd]),
    ("smp_probe_robot_dev", _i64, [_p, _p, _i64]),
    ("smp_probe_scene_slabs", _i64, [_p, _p, _p, _i64]),
]

_lib = None


def lib():
    """Load libsmp_gpu.so (build it with `make -C squirrel_motion_planner_amd` / __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libsmp_gpu.so not built at %s -- run __graft_entry__.build(); there is no CPU fallback"
                              % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in EXPORTS + PROBES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class SmpError(RuntimeError):
    def __init__(self, status, what=""):
        self.status = status
        msg = lib().smp_strerror(status).decode()
        super().__init__("%s%s (status %d)" % (what + ": " if what else "", msg, status))


def check(status, what=""):
    if status != SMP_OK:
        raise SmpError(status, what)
    return status
