/* smp_gpu.h -- C ABI of the MI355X BiRRT* sampling / collision hot path.
 *
 * Drop-in boundary for the planner core that squirrel_8dof_planner drives
 * (tpatten/squirrel_motion_planner).  Each entry point replaces one interface of the reference:
 *
 *   smp_robot_create_json      KDLRobotModel + CollisionChecker construction
 *                              (birrt_star.cpp:61-73, kdl_kuka_model.cpp:12-236, collision_checker.hpp:65-74)
 *   smp_robot_create_urdf      the same from robot_description / SRDF text (collision_checker.hpp:176-393)
 *   smp_scene_from_keys        BiRRTstarPlanner::setOctree -> CollisionChecker::setOcTree
 *                              (birrt_star.cpp:1621-1624, collision_checker.hpp:76-88) for occupied leaf keys
 *   smp_scene_from_bt          the same from an octomap binary (.bt / binary octomap_msgs payload), with the
 *                              node's floor insertion (squirrel_8dof_planner.cpp:862-917)
 *   smp_scene_from_ot          the same from an octomap full-format file (.ot, the octomap_server's input,
 *                              launch/simulation.launch:51)
 *   smp_scene_from_octomap_msg the same from an octomap_msgs/Octomap payload (id, resolution, binary flag, data):
 *                              binaryMsgToMap / fullMsgToMap (squirrel_8dof_planner.cpp:875-883)
 *   smp_scene_from_grid        the same from a broadcast grid (multi-GPU: one RCCL broadcast per scene)
 *   smp_planner_create         BiRRTstarPlanner::initialize (birrt_star.cpp:11-326) on one GPU
 *   smp_planner_set_scene      BiRRTstarPlanner::setOctree (copies; caller keeps ownership)
 *   smp_set_disabled_map_links BiRRTstarPlanner::setDisabledLinkMapCollisions (birrt_star.cpp:6916-6919)
 *   smp_plan                   reset_planner_and_config + setPlanningSceneInfo + init_planner + run_planner
 *                              + getJointTrajectoryRef (squirrel_8dof_planner.cpp:1221-1248,
 *                              birrt_star.cpp:335-536, 983-1407, 1688-1691)
 *   smp_plan_batch             independent queries against one scene (one workgroup each)
 *   smp_plan_multi             the same over several planners / GPUs of one process (the node is one process:
 *                              squirrel_8dof_planner_node.cpp:6-15), queries dealt round-robin
 *   smp_planner_scene_device   setOctree's copy of the map for further GPUs: the planner's device-resident scene
 *   smp_planner_set_scene_device  (RCCL broadcast between ranks, xGMI peer copies between planners) instead of a
 *   smp_planners_share_scene   host rebuild per GPU
 *   smp_check_configs          batched isConfigValid (birrt_star.cpp:6897-6908) -> valid flags
 *   smp_is_config_valid        BiRRTstarPlanner::isConfigValid for one configuration
 *   smp_get_collisions         BiRRTstarPlanner::getCollisions (birrt_star.cpp:6910-6914 -> collision_checker.hpp:
 *                              123-132, 594-630): colliding self pairs and map-colliding links of one configuration
 *   smp_check_sequence         the node's keyframe loops over isConfigValid (fold / unfold arm,
 *                              squirrel_8dof_planner.cpp:759-784, 814-823): first invalid pose, one kernel launch
 *   smp_normalize_trajectory   Planner::normalizeTrajectory (squirrel_8dof_planner.cpp:1557-1637), host only
 *   smp_ik_solve               BiRRTstarPlanner::getFullPoseFromEEPose (birrt_star.cpp:1627-1686) ->
 *                              RobotController::run_VDLS_Control_Connector (control_laws.cpp:3283-3712):
 *                              n independent controller runs, one wavefront each
 *   smp_find_goal_pose         Planner::findGoalPose (squirrel_8dof_planner.cpp:1129-1201): every candidate base
 *                              angle's controller run at once, each REACHED pose checked in the same kernel, the
 *                              first valid one in the reference's order (later candidates stop once it is known)
 *   smp_result_free            releases library-owned result buffers
 *   smp_strerror               text of a status code
 *
 * Conventions: the caller owns every input buffer; results are library-allocated and released with
 * smp_result_free.  Every function returns SMP_OK (0) or a negative status.  One smp_planner per host
 * thread (the reference planner is not thread-safe either, squirrel_8dof_planner_node.cpp:12).
 * Configurations are 8 fp64 values in chain order [x, y, theta, arm1..arm5].
 */
#ifndef SMP_GPU_H
#define SMP_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  SMP_OK = 0,
  SMP_ERR_ARG = -1,           /* bad argument / dimension mismatch (birrt_star.cpp:338-342) */
  SMP_ERR_START_INVALID = -2, /* start configuration in collision (birrt_star.cpp:353-357) */
  SMP_ERR_GOAL_INVALID = -3,  /* goal configuration in collision (birrt_star.cpp:358-362) */
  SMP_ERR_NO_SOLUTION = -4,   /* budget exhausted without a path (birrt_star.cpp:1405) */
  SMP_ERR_HIP = -5,           /* HIP runtime error, or a launch the call gave up waiting for (a seconds budget's
                                 4x + 60 s): the planner then sets its abort word, which every leader polls each 64
                                 iterations, and answers SMP_ERR_HIP to every call until that launch has drained */
  SMP_ERR_PARSE = -6,         /* model / octomap parse error */
  SMP_ERR_CAPACITY = -7,      /* tree capacity exceeded (raise smp_params.node_capacity) */
  SMP_ERR_NO_DEVICE = -8      /* no usable GPU: the library never falls back to the CPU */
};

enum { SMP_BUDGET_ITERATIONS = 0, SMP_BUDGET_SECONDS = 1, SMP_BUDGET_SAMPLES = 2 };

typedef struct smp_robot smp_robot;
typedef struct smp_scene smp_scene;
typedef struct smp_planner smp_planner;

typedef struct smp_scene_opts {
  double resolution;      /* metres per voxel (used by smp_scene_from_keys) */
  double z_offset;        /* octree transform z (collision_checker.hpp:87: -0.02) */
  int insert_floor;       /* 1: insert the node's floor square (squirrel_8dof_planner.cpp:889-902) */
  double floor_center[2]; /* robot x, y at planning time */
  double floor_distance;  /* floor_collision_distance (parameters.yaml:24: 3.0) */
} smp_scene_opts;

typedef struct smp_params {
  double near_threshold;   /* near_threshold_interpolation (birrt_star.cpp:183, default 4.0) */
  double step_factor;      /* unconstraint_extend_step_factor (birrt_star.cpp:189, default 0.5) */
  int num_traj_segments;   /* num_traj_segments_interp (birrt_star.cpp:186, default 20) */
  int max_near_nodes;      /* max_near_nodes (birrt_star.cpp:195, default 20) */
  double path_optimality_threshold; /* birrt_star.cpp:201 (default 1.0) */
  int tree_optimization;   /* m_tree_optimization_active (default 1) */
  int informed_sampling;   /* m_informed_sampling_active (default 1) */
  int64_t node_capacity;   /* per-tree node capacity on the device (0: derived from the budget) */
  int helpers;             /* helper workgroups per query that share its collision tiles across CUs
                              (0: automatic, up to 200 with scouts / 63 without; -1: none, the query runs on
                              its own workgroup) */
  int scout;               /* 1 (default): scout workgroups compute the coming iterations' scans and collision jobs
                              ahead of the leader -- 4 when a query has 64 CUs or more, 2 from 18 CUs, 1 from 6
                              (before the first solution they take the iterations in turn; after it scouts 0 and 1
                              alternate, two ahead, and the others retire); 2..8: that many (with >= 4 helpers);
                              0: off.  Results are identical either way */
} smp_params;

typedef struct smp_query {
  double start[8];
  double goal[8];
  double env_x[2];         /* setPlanningSceneInfo size_x (0,0 = unconfined) */
  double env_y[2];
  int check_self;
  int check_map;
  int budget_kind;         /* SMP_BUDGET_*: iterations (flag_iter_or_time = 0), seconds (= 1), or
                              collision-checked configurations (checked before each iteration) */
  double budget;
  uint64_t seed;
  uint32_t query_id;       /* RNG stream of this query */
} smp_query;

typedef struct smp_stats {
  int64_t iterations;
  int64_t first_solution_iter;   /* -1 if none */
  int64_t last_solution_iter;
  int64_t configs_checked;       /* isInCollision calls of the reference semantics */
  int64_t configs_valid;         /* ... of which collision free */
  double time_first_solution;    /* seconds from the kernel's planning start (device clock; see also
                                    time_first_solution_host) */
  double time_total;             /* seconds of the planning loop (device clock) */
  double cost_best[3];           /* total, revolute, prismatic */
  double cost_theoretical[3];
  int64_t nodes_start, nodes_goal, edges_start, edges_goal, rewires_start, rewires_goal;
  int32_t connected_tree_is_start;
  int32_t conn_node_b, conn_node_a;
  int64_t nn_nodes_scanned;      /* nodes streamed by nearest-neighbour scans (64 B each) */
  int64_t near_nodes_scanned;    /* nodes streamed by near-vertex scans (72 B each) */
  int64_t samples_precomputed;   /* iterations whose sample came from the run-ahead sampler workgroup */
  double phase_seconds[32];      /* device time per planner phase (sample, nn, expand, near, choose-parent,
                                    rewire, connect, collision tiles, #tiles, edge costs, via chains, #via,
                                    tile stages, tile time per calling phase, then counts of checked
                                    configurations and of tile slots per calling phase) */
  int64_t scout_nn_hits;         /* nearest-neighbour scans answered from the scout's record */
  int64_t scout_near_hits;       /* near-vertex scans answered from the scout's record */
  int64_t scout_edge_hits;       /* needed edges whose collision check the scout had done */
  int64_t scout_edge_misses;     /* needed edges checked by the leader's own jobs while the scout was asked */
  double scout_wait_seconds;     /* time the leader waited for the scout */
  double scout_phase_seconds[32]; /* the scout's time per stage (0 sample, 1 nearest, 2 expand, 3 near, 4 choose,
                                    5 via chain, 6 rewire, 28 idle, 29 publishing, 31 busy; 30 = iterations) */
  int32_t helpers;               /* helper workgroups per query used */
  int32_t scout;                 /* scout workgroups per query used (0: none) */
  double time_first_solution_host; /* seconds from smp_plan entry until the host saw the first feasible path (host
                                    clock: start / goal checks, allocation, uploads and launch included; SURVEY 8d
                                    counts from run_planner entry, birrt_star.cpp:1075-1081); -1 if none */
} smp_stats;

typedef struct smp_result {
  int status;               /* SMP_OK or a negative code */
  int64_t n_waypoints;
  double* waypoints;        /* n_waypoints x 8, row-major (library-owned) */
  smp_stats stats;
  int64_t n_cost_rows;
  double* cost_rows;        /* n_cost_rows x 5: [iteration, time, c_best, c_rev, c_prism] (birrt_star.cpp:1325-1331) */
} smp_result;

void smp_params_default(smp_params* p);
void smp_scene_opts_default(smp_scene_opts* o);

int smp_robot_create_json(const char* model_json, smp_robot** out);
int smp_robot_create_urdf(const char* urdf_xml, const char* srdf_xml, const char* spheres_json, smp_robot** out);
void smp_robot_destroy(smp_robot* r);
int smp_robot_num_links(const smp_robot* r);
const char* smp_robot_link_name(const smp_robot* r, int i);

int smp_scene_from_keys(const uint16_t* keys_xyz, int64_t n, const smp_scene_opts* opts, smp_scene** out);
int smp_scene_from_bt(const uint8_t* data, size_t size, const smp_scene_opts* opts, smp_scene** out);
/* Octomap full format (.ot): per node a float log-odds and a child-existence byte; leaves with log-odds >= 0 are
 * occupied.  Floor insertion (opts->insert_floor) leaves cells of free leaves free when one hit does not make them
 * occupied, as updateNode(key, true) does. */
int smp_scene_from_ot(const uint8_t* data, size_t size, const smp_scene_opts* opts, smp_scene** out);
/* octomap_msgs/Octomap fields: id must be "OcTree" (other tree types: SMP_ERR_PARSE, the node's "empty octomap"),
 * binary != 0: writeBinaryData payload, else writeData payload; neither carries a text header. */
int smp_scene_from_octomap_msg(const char* id, double resolution, int binary, const uint8_t* data, size_t size,
                               const smp_scene_opts* opts, smp_scene** out);
/* A scene from an exported grid (bitset + d2), e.g. after the RCCL broadcast of rank 0's scene. */
int smp_scene_from_grid(const uint64_t* bits, const uint16_t* d2, const int dims[3], const double origin[3],
                        double resolution, smp_scene** out);
void smp_scene_destroy(smp_scene* s);
/* Grid geometry of a scene: dims[3], origin[3], resolution; bitset/d2 copies for inspection (may be NULL). */
int smp_scene_info(const smp_scene* s, int dims[3], double origin[3], double* resolution,
                   int64_t* n_occupied, double bbox_min[3], double bbox_max[3]);
int smp_scene_export(const smp_scene* s, uint64_t* bits, uint16_t* d2);

int smp_planner_create(int device, const smp_robot* robot, const smp_params* params, smp_planner** out);
void smp_planner_destroy(smp_planner* p);
int smp_planner_set_scene(smp_planner* p, const smp_scene* s);
/* Planner parameters for subsequent smp_plan calls (activate/deactivateTreeOptimization,
 * activate/deactivateInformedSampling, birrt_star.h:57-63; setEdgeCostWeights keeps weights 1). */
int smp_planner_set_params(smp_planner* p, const smp_params* params);
int smp_planner_get_params(const smp_planner* p, smp_params* params);
int smp_set_disabled_map_links(smp_planner* p, const char* const* link_names, int n);

/* Multi-GPU (queries shard, the scene is sent once per scene, no per-iteration collective).
 * The device-resident form of a planner's scene: the arrays smp_planner_set_scene derived for the planner's robot
 * (4x4x4 occupancy bricks, the box-gap field, its byte copy when every sphere threshold is below 255, one 2-D slab field
 * per exact primitive).  They move device to device: between ranks by an RCCL broadcast into caller buffers
 * (squirrel_motion_planner_amd/distributed.py), between the planners of one process by peer copies over xGMI
 * (smp_planners_share_scene).  The sender's and the receiver's robot must be the same model. */
typedef struct smp_scene_device {
  int dims[3];             /* cells x, y, z */
  double origin[3];
  double resolution;
  int64_t n_bricks;        /* uint64 words: ceil(x/4) * ceil(y/4) * ceil(z/4) */
  int64_t n_cells;         /* x * y * z: uint16 box-gap values (and bytes of the byte copy) */
  int n_prim;              /* slab planes of x * y uint16 values */
  int has_d2b;             /* the byte copy is part of the scene */
  uint64_t* bricks;        /* device pointers (any GPU of this process, or caller-owned buffers on the planner's GPU) */
  uint16_t* d2;
  uint8_t* d2b;
  uint16_t* slab;
} smp_scene_device;
/* Geometry and sizes of the planner's device scene; each non-NULL pointer of *io receives a device-to-device copy of
 * that array (caller-allocated, on any GPU).  SMP_ERR_ARG if the planner has no scene. */
int smp_planner_scene_device(const smp_planner* p, smp_scene_device* io);
/* Sets the planner's scene from device arrays laid out as above (copied: the caller keeps ownership); the robot-derived
 * parts must match this planner's robot (SMP_ERR_ARG otherwise).  Replaces smp_planner_set_scene on receiving ranks. */
int smp_planner_set_scene_device(smp_planner* p, const smp_scene_device* in);
/* ps[src]'s scene to every other planner of the array (peer copies over xGMI for planners on other GPUs). */
int smp_planners_share_scene(smp_planner* const* ps, int n, int src);

int smp_plan(smp_planner* p, const smp_query* q, smp_result* out);
int smp_plan_batch(smp_planner* p, const smp_query* q, int n, smp_result* out);
/* Independent queries over several planners (typically one per GPU, sharing a scene): query i runs on planner
 * i % n_planners, all planners concurrently (one host thread each); out[i] is query i's result, identical to what
 * smp_plan on that planner returns.  Each planner may appear once; planners on one GPU split that GPU's co-resident
 * workgroups among them for the call (each query's workgroups must all be resident).  Scenes set from grids
 * (smp_planner_set_scene / _device) must keep every occupied cell 0.45 m plus one cell from the grid's faces
 * (SMP_ERR_ARG otherwise): a sphere or primitive centred outside the grid is taken as free of the map. */
int smp_plan_multi(smp_planner* const* planners, int n_planners, const smp_query* q, int n, smp_result* out);
void smp_result_free(smp_result* r);

/* Tree dump of the last smp_plan (which: 0 start tree, 1 goal tree) for parity checks; arrays may be NULL. */
int64_t smp_get_tree(smp_planner* p, int which, int32_t* parent, double* conf, double* cost);

int smp_check_configs(smp_planner* p, const double* q_soa, int64_t n, int check_self, int check_map, uint8_t* valid);
int smp_is_config_valid(smp_planner* p, const double q[8], int check_self, int check_map, int* valid);
/* Every self pair that collides (2 link indices each, smp_robot_link_name, in the model's pair order -- the SRDF-enabled
 * link pairs i < j in link order, CC:378-388) and every collision link that touches the map (link indices in name
 * order, as the reference's std::map; disabled links included, CC:610-630).  Writes at most max_self pairs /
 * max_map links; *n_self / *n_map receive the full counts (the caller compares them with its capacity).
 * Rigid pairs are left out, here as in every validity check: the 65 SRDF-enabled pairs of links on one rigid body
 * (the reference's getSelfCollisions, CC:594-608, tests all 230) have the same relative pose in every configuration,
 * so their outcome does not depend on it; an overlapping one would make every configuration invalid in the
 * reference, and 7 of them overlap only under the conservative sphere covers (hand couplers / cranks against the
 * hand base and finger links, door against shell) -- tests/test_host_cpu.py pins both facts. */
int smp_get_collisions(smp_planner* p, const double q[8], int32_t* self_pairs, int max_self, int* n_self,
                       int32_t* map_links, int max_map, int* n_map);
/* n poses, row-major n x 8: *first_invalid = index of the first pose in collision, -1 if all are valid. */
int smp_check_sequence(smp_planner* p, const double* q_rows, int64_t n, int check_self, int check_map,
                       int64_t* first_invalid);
/* n poses of `dim` values, row-major.  *n_out = rows of the normalized trajectory; with out == NULL only counts,
 * else writes them (SMP_ERR_CAPACITY if out_cap < *n_out).  For dim < 1 or n <= 1 the reference leaves its output
 * untouched: *n_out = 0.  Host only (no GPU needed). */
int smp_normalize_trajectory(const double* raw, int64_t n, int dim, const double* normalized_pose, double* out,
                             int64_t out_cap, int64_t* n_out);

/* End-effector goal -> 8-DoF pose (IK of the node's goal search). */
typedef struct smp_ik_request {
  double ee_pose[6];        /* x, y, z, roll, pitch, yaw: getFullPoseFromEEPose's endEffectorPose (birrt_star.cpp:1627) */
  double deviation[6][2];   /* (lower, upper) permitted error per task coordinate: endEffectorDeviations
                               (setVariableConstraints, control_laws.cpp:1740-1761) */
  double q_init[8];         /* poseInit (setStartConf, control_laws.cpp:1464-1495) */
  int max_iter;             /* controller iterations, >= 1 (the reference passes 1000, birrt_star.cpp:1670) */
} smp_ik_request;

typedef struct smp_ik_result {
  int reached;              /* 1: REACHED -- getFullPoseFromEEPose returns true; 0: ADVANCED (control_laws.cpp:3691-3710) */
  int iterations;           /* controller iterations run */
  int fallback_iterations;  /* iterations whose manipulability needed the Jacobi eigenvalue path (near-singular J) */
  double q[8];              /* poseSolution = joint_trajectory.back() (birrt_star.cpp:1675) */
  double error[6];          /* last task-space error (zero inside the deviation band) */
  double manipulability;    /* last manipulability measure (control_laws.cpp:6050-6089) */
} smp_ik_result;

/* Parity: bit for bit against the oracle (oracle/smp_oracle.cpp), which is unpinned against the reference here:
 * the reference's manipulability (float Eigen::JacobiSVD, CL:6061-6084) and damped pseudo-inverse (fp64 SVD,
 * CL:5574-5596) are restated as det / Gauss-Jordan with a Jacobi eigen-decomposition fallback (DESIGN.md "IK goal
 * search"), equal in exact arithmetic; near singular Jacobians the iteration counts and REACHED / ADVANCED can
 * differ from the reference binaries.  fallback_iterations counts the fallback branch; tests/test_gpu_ik.py checks
 * that kernel and oracle take the same branch on singular starts. */
int smp_ik_solve(smp_planner* p, const smp_ik_request* reqs, int n, smp_ik_result* out);

typedef struct smp_goal_search {
  int n_candidates;         /* base angles of the search (17 at the default 20 degrees) */
  int n_reached;            /* candidates whose controller run REACHED the pose; candidates after the chosen one may
                               have stopped early (they can no longer be chosen), so this counts the ones that ran */
  int chosen;               /* candidate index of pose_goal, -1 if none */
  int downward;             /* 1 if the hand points downward (squirrel_8dof_planner.cpp:1140) */
  double kernel_ms;         /* IK + validity kernels, HIP events */
} smp_goal_search;

/* findGoalPose for end-effector pose ee_pose (x, y, z, roll, pitch, yaw in the planning frame) from the robot's
 * current pose, candidate spacing in degrees (goal_pose_search_discretization, default 20; values < 1 count as 1).
 * *result: 0 = pose found (pose_goal written), 1 = every pose the controller reached collides (COLLISION_GOAL_POSE),
 * 2 = the controller reached no pose (INVALID_END_EFFECTOR_POSE) -- the reference's return codes.  info may be NULL. */
/* (Unpinned against the reference near singular Jacobians as smp_ik_solve.) */
int smp_find_goal_pose(smp_planner* p, const double ee_pose[6], const double pose_current[8], double discretization_deg,
                       int check_self, int check_map, double pose_goal[8], int* result, smp_goal_search* info);

/* Kernel timing of the last smp_check_configs / smp_plan call: milliseconds on the launch stream. */
int smp_last_kernel_ms(const smp_planner* p, double* check_ms, double* plan_ms, int64_t* plan_launches);

const char* smp_strerror(int status);

#ifdef __cplusplus
}
#endif
#endif /* SMP_GPU_H */
