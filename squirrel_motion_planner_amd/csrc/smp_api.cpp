// C ABI implementation (include/smp_gpu.h): device memory, launches, result assembly.
// No CPU fallback: without a usable GPU every compute entry point returns SMP_ERR_NO_DEVICE.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <set>
#include <stdexcept>
#include <string>
#include <array>
#include <thread>
#include <vector>

#include "../../include/smp_gpu.h"
#include "smp_host.h"
#include "smp_ik.h"
#include "smp_math.h"
#include "smp_plan.h"
#include "smp_types.h"

namespace smp {
void launch_check(int ct, int grid, hipStream_t st, const RobotDev* rb, SceneDev sc, const MapCfg* mc, const double* q,
                  long long n, int self, int map, uint8_t* valid, unsigned long long* prof);
__global__ void plan_kernel(const RobotDev* rb, SceneDev sc, const MapCfg* mc, QueryDev* qs, int nq, int scout_base,
                            int helper_base, int iters);
__global__ void path_kernel(QueryDev* qs, int* counts);
__global__ void path_edges_kernel(const QueryDev* qs, int q, int ns, int ng, double* out);
__global__ void boards_reset_kernel(const QueryDev* qs, int ns);
size_t check_kernels_private_bytes();
size_t ik_kernels_private_bytes();
void launch_collisions(hipStream_t st, const RobotDev* rb, SceneDev sc, const MapCfg* mc, const double* q, int map,
                       uint8_t* link_map, uint8_t* pair_self);
void launch_ik(bool search, int n, hipStream_t st, const RobotDev* rb, const IkTaskDev* tasks, IkOutDev* out,
               SceneDev sc, const MapCfg* mc, int self, int map, int* best);
__global__ void sincos_kernel(const double* x, int n, double* s, double* c);
__global__ void u01_kernel(unsigned long long seed, unsigned query, const uint32_t* ctr, int n, double* out);
__global__ void fk_kernel(const RobotDev* rb, const double* q, int n, double* frames, double* eez);
__global__ void sqrt_div_kernel(const double* a, const double* b, int n, double* sq, double* dv);
__global__ void near_probe_kernel(const double* tq, const double* tcost, int cap, int n, const double* queries,
                                  const int* excl, int m, double r, int reps, int* nn, int* nk, int* lo, int* hi,
                                  unsigned long long* ticks, const float* tqf);
__global__ void near_probe_inl_kernel(const double* tq, const double* tcost, int cap, int n, const double* queries,
                                      const int* excl, int m, double r, int reps, int* nn, int* nk, int* lo, int* hi,
                                      unsigned long long* ticks, const float* tqf);
}  // namespace smp

using namespace smp;

struct smp_robot {
  RobotHost h;
};

struct smp_scene {
  SceneHost h;
};

namespace {

#define HIPCHK(x)                                                                         \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "smp_gpu: HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return SMP_ERR_HIP;                                                                 \
    }                                                                                     \
  } while (0)

template <typename T>
struct DBuf {  // device buffer that only grows
  T* p = nullptr;
  size_t n = 0;
  hipError_t reserve(size_t want) {
    if (want <= n) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipMalloc(&p, std::max<size_t>(want, 1) * sizeof(T));
    if (e == hipSuccess) n = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

struct QueryBuffers {
  DBuf<QState> st;
  DBuf<double> q, cost, e_start, e_target, rows;
  DBuf<float> qf;
  DBuf<int> parent, first_child, next_sib, prev_sib, stack, path_nodes;
  DBuf<ViaNode> via;
  DBuf<JobBoard> jb;               // the leader's collision-job board
  DBuf<JobBoard> sjb[MAX_SCOUTS];  // the scouts' collision-job boards, record boards and via scratch
  DBuf<ScoutBoard> scb[MAX_SCOUTS];
  DBuf<ViaNode> svia[MAX_SCOUTS];
  size_t cap = 0;
  void release() {
    st.release(); q.release(); qf.release(); cost.release(); e_start.release(); e_target.release(); rows.release();
    parent.release(); first_child.release(); next_sib.release(); prev_sib.release(); stack.release();
    path_nodes.release(); via.release(); jb.release();
    for (int s = 0; s < MAX_SCOUTS; ++s) { sjb[s].release(); scb[s].release(); svia[s].release(); }
    cap = 0;
  }
};

}  // namespace

struct smp_planner {
  int device = 0;
  hipStream_t stream = nullptr;
  RobotHost robot;
  smp_params params;
  RobotDev* d_rb = nullptr;
  MapCfg mc_host;
  MapCfg* d_mc = nullptr;
  DBuf<uint64_t> d_bricks;
  DBuf<uint16_t> d_d2;
  DBuf<uint8_t> d_d2b;
  DBuf<uint16_t> d_slab;           // per-primitive 2-D slab fields (SceneDev::slab), n_prim x nx x ny
  SceneDev sc{};
  bool have_scene = false;
  double scene_res = 0.05;
  std::set<std::string> disabled;
  std::vector<QueryBuffers> qb;
  DBuf<QueryDev> d_qdev;
  DBuf<int> d_counts;
  DBuf<unsigned> d_lfin;  // finished queries of the current launch
  DBuf<double> d_cq;
  DBuf<uint8_t> d_valid;
  DBuf<IkTaskDev> d_ik_tasks;
  DBuf<IkOutDev> d_ik_out;
  DBuf<int> d_ik_best;
  DBuf<double> d_path_edges;       // path_edges_kernel output (the path's edges, one copy to the host)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  double last_check_ms = 0, last_plan_ms = 0;
  int64_t last_plan_launches = 0;
  double wall_rate_hz = 1e8;
  int num_cus = 256;
  int num_xcd = 8;                 // XCDs (hipDeviceAttributeNumberOfXccs): the per-XCD helper budget of provision()
  unsigned* h_ttff = nullptr;      // host-mapped first-solution flags, one per query (QueryDev::ttff)
  unsigned* h_abort = nullptr;     // host-mapped abort word of the planner's launches (QueryDev::abort)
  QState* h_st = nullptr;          // pinned host copies of the queries' loop states (asynchronous uploads)
  int n_st = 0;
  int n_ttff = 0;
  // last plan (query 0) bookkeeping for smp_get_tree
  int last_n[2] = {0, 0};
  int slots_cache = 0;  // resident_slots (occupancy queries) once per planner
  int slot_share = 1;   // planners planning on this planner's GPU at once (smp_plan_multi): its share of the slots
  // processes planning on this GPU at once (SMP_SLOT_SHARE, e.g. several ranks of one job on a one-GPU box): every
  // workgroup of a query must be co-resident, so each process provisions its share of the device
  int proc_share = 1;
  // a planning call gave up (SMP_ERR_HIP) while its kernels may still run on these buffers: every later call that
  // would touch them fails with SMP_ERR_HIP until both streams are idle again (busy_check), and destroy leaks them
  // rather than freeing memory a live kernel uses
  bool busy = false;
};

// SMP_OK once no kernel of an abandoned planning call runs any more (smp_planner::busy), else SMP_ERR_HIP.
static int busy_check(smp_planner* p) {
  if (!p->busy) return SMP_OK;
  (void)hipSetDevice(p->device);
  if (hipStreamQuery(p->stream) == hipErrorNotReady) return SMP_ERR_HIP;
  (void)hipGetLastError();
  p->busy = false;
  return SMP_OK;
}

// Workgroups of BLOCK threads that can be resident at once on the device for plan_kernel (leaders, scouts and helpers
// of a launch are its blocks): occupancy per CU (registers, LDS) x CUs.
static int resident_slots(smp_planner* p) {
  if (p->slots_cache > 0) return std::max(1, p->slots_cache / std::max(1, p->slot_share));
  int occ_plan = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_plan, reinterpret_cast<const void*>(&plan_kernel), BLOCK, 0) !=
      hipSuccess) {
    (void)hipGetLastError();
    return p->num_cus;
  }
  p->slots_cache = p->num_cus * std::max(1, occ_plan);
  return std::max(1, p->slots_cache / std::max(1, p->slot_share));
}

static int update_mapcfg(smp_planner* p) {
  const RobotDev& d = p->robot.dev;
  std::memset(&p->mc_host, 0, sizeof(MapCfg));
  p->mc_host.has_map = p->have_scene ? 1 : 0;
  for (int s = 0; s < d.n_sph; ++s) {
    p->mc_host.T[s] = p->have_scene ? sphere_threshold(d.sph_r[s], p->scene_res) : 0;
    int link = d.cl_link[d.sph_clink[s]];
    p->mc_host.map_on[s] = p->disabled.count(p->robot.link_names[link]) ? 0 : 1;
  }
  for (int k = 0; k < d.n_prim; ++k) {
    p->mc_host.pT[k] = p->have_scene ? sphere_threshold(d.prim_rxy[k], p->scene_res) : 0;
    p->mc_host.p_map_on[k] = p->disabled.count(p->robot.link_names[d.cl_link[d.prim_clink[k]]]) ? 0 : 1;
  }
  HIPCHK(hipMemcpyAsync(p->d_mc, &p->mc_host, sizeof(MapCfg), hipMemcpyHostToDevice, p->stream));
  HIPCHK(hipStreamSynchronize(p->stream));
  return SMP_OK;
}

extern "C" int smp_debug_bounds(int* out);
#ifdef SMP_RING_CHECK
extern "C" void smp_ringchk_dump();
#endif

extern "C" {

void smp_params_default(smp_params* p) {
  p->near_threshold = 4.0;
  p->step_factor = 0.5;
  p->num_traj_segments = 20;
  p->max_near_nodes = 20;
  p->path_optimality_threshold = 1.0;
  p->tree_optimization = 1;
  p->informed_sampling = 1;
  p->node_capacity = 0;
  p->helpers = 0;
  p->scout = 1;
}

void smp_scene_opts_default(smp_scene_opts* o) {
  o->resolution = 0.05;
  o->z_offset = -0.02;
  o->insert_floor = 0;
  o->floor_center[0] = o->floor_center[1] = 0.0;
  o->floor_distance = 3.0;
}

const char* smp_strerror(int s) {
  switch (s) {
    case SMP_OK: return "ok";
    case SMP_ERR_ARG: return "invalid argument";
    case SMP_ERR_START_INVALID: return "start configuration is invalid";
    case SMP_ERR_GOAL_INVALID: return "goal configuration is invalid";
    case SMP_ERR_NO_SOLUTION: return "no solution found within the budget";
    case SMP_ERR_HIP: return "HIP runtime error";
    case SMP_ERR_PARSE: return "parse error";
    case SMP_ERR_CAPACITY: return "tree capacity exceeded";
    case SMP_ERR_NO_DEVICE: return "no usable GPU (the library has no CPU fallback)";
    default: return "unknown status";
  }
}

int smp_robot_create_json(const char* model_json, smp_robot** out) {
  if (!model_json || !out) return SMP_ERR_ARG;
  smp_robot* r = new smp_robot();
  try {
    robot_from_json(model_json, &r->h);
  } catch (const std::exception& e) {
    fprintf(stderr, "smp_gpu: %s\n", e.what());
    delete r;
    return SMP_ERR_PARSE;
  }
  *out = r;
  return SMP_OK;
}

int smp_robot_create_urdf(const char* urdf_xml, const char* srdf_xml, const char* spheres_json, smp_robot** out) {
  if (!urdf_xml || !srdf_xml || !spheres_json || !out) return SMP_ERR_ARG;
  smp_robot* r = new smp_robot();
  try {
    robot_from_urdf(urdf_xml, srdf_xml, spheres_json, &r->h);
  } catch (const std::exception& e) {
    fprintf(stderr, "smp_gpu: %s\n", e.what());
    delete r;
    return SMP_ERR_PARSE;
  }
  *out = r;
  return SMP_OK;
}

void smp_robot_destroy(smp_robot* r) { delete r; }
int smp_robot_num_links(const smp_robot* r) { return r ? (int)r->h.link_names.size() : 0; }
const char* smp_robot_link_name(const smp_robot* r, int i) {
  if (!r || i < 0 || i >= (int)r->h.link_names.size()) return nullptr;
  return r->h.link_names[i].c_str();
}

int smp_scene_from_keys(const uint16_t* keys, int64_t n, const smp_scene_opts* o, smp_scene** out) {
  if (!o || !out || (n > 0 && !keys) || !(o->resolution > 0)) return SMP_ERR_ARG;
  std::vector<uint16_t> k(keys, keys + 3 * std::max<int64_t>(n, 0));
  if (o->insert_floor) floor_keys(o->floor_center[0], o->floor_center[1], o->resolution, o->floor_distance, &k);
  smp_scene* s = new smp_scene();
  scene_from_keys(k.data(), (int64_t)k.size() / 3, o->resolution, o->z_offset, &s->h);
  *out = s;
  return SMP_OK;
}

// Occupied keys + free leaves of an octomap stream -> scene (with the node's floor insertion when asked).
static int scene_from_octomap(bool full, bool header, const uint8_t* data, size_t size, double res,
                              const smp_scene_opts* o, smp_scene** out) {
  std::vector<uint16_t> k;
  std::vector<FreeLeaf> fl;
  try {
    if (full) octomap_ot_keys(data, size, &res, &k, &fl, header);
    else octomap_bt_keys(data, size, &res, &k, &fl, header);
  } catch (const std::exception& e) {
    fprintf(stderr, "smp_gpu: %s\n", e.what());
    return SMP_ERR_PARSE;
  }
  if (!(res > 0)) return SMP_ERR_ARG;
  if (o->insert_floor) floor_keys(o->floor_center[0], o->floor_center[1], res, o->floor_distance, &k, &fl);
  smp_scene* s = new smp_scene();
  scene_from_keys(k.data(), (int64_t)k.size() / 3, res, o->z_offset, &s->h);
  *out = s;
  return SMP_OK;
}

int smp_scene_from_bt(const uint8_t* data, size_t size, const smp_scene_opts* o, smp_scene** out) {
  if (!data || !o || !out) return SMP_ERR_ARG;
  return scene_from_octomap(false, true, data, size, 0.0, o, out);
}

int smp_scene_from_ot(const uint8_t* data, size_t size, const smp_scene_opts* o, smp_scene** out) {
  if (!data || !o || !out) return SMP_ERR_ARG;
  return scene_from_octomap(true, true, data, size, 0.0, o, out);
}

int smp_scene_from_octomap_msg(const char* id, double resolution, int binary, const uint8_t* data, size_t size,
                               const smp_scene_opts* o, smp_scene** out) {
  if (!id || !o || !out || (size > 0 && !data) || !(resolution > 0)) return SMP_ERR_ARG;
  // binaryMsgToMap / fullMsgToMap + dynamic_cast<octomap::OcTree*> (squirrel_8dof_planner.cpp:875-883): any
  // other tree type is an empty octomap for the node
  if (std::strcmp(id, "OcTree") != 0) return SMP_ERR_PARSE;
  return scene_from_octomap(binary == 0, false, data, size, resolution, o, out);
}

int smp_scene_from_grid(const uint64_t* bits, const uint16_t* d2, const int dims[3], const double origin[3],
                        double res, smp_scene** out) {
  if (!bits || !d2 || !dims || !origin || !out || !(res > 0) || dims[0] <= 0 || dims[1] <= 0 || dims[2] <= 0)
    return SMP_ERR_ARG;
  smp_scene* s = new smp_scene();
  SceneHost& h = s->h;
  h.nx = dims[0]; h.ny = dims[1]; h.nz = dims[2]; h.wx = (h.nx + 63) / 64;
  h.ox = origin[0]; h.oy = origin[1]; h.oz = origin[2]; h.res = res;
  size_t nw = (size_t)h.wx * h.ny * h.nz, nc = (size_t)h.nx * h.ny * h.nz;
  h.bits.assign(bits, bits + nw);
  h.d2.assign(d2, d2 + nc);
  h.n_occupied = 0;
  for (uint64_t w : h.bits) h.n_occupied += __builtin_popcountll(w);
  build_bricks(&h);
  *out = s;
  return SMP_OK;
}

void smp_scene_destroy(smp_scene* s) { delete s; }

int smp_scene_info(const smp_scene* s, int dims[3], double origin[3], double* resolution, int64_t* n_occupied,
                   double bbox_min[3], double bbox_max[3]) {
  if (!s) return SMP_ERR_ARG;
  if (dims) { dims[0] = s->h.nx; dims[1] = s->h.ny; dims[2] = s->h.nz; }
  if (origin) { origin[0] = s->h.ox; origin[1] = s->h.oy; origin[2] = s->h.oz; }
  if (resolution) *resolution = s->h.res;
  if (n_occupied) *n_occupied = s->h.n_occupied;
  for (int d = 0; d < 3; ++d) {
    if (bbox_min) bbox_min[d] = s->h.bbox_min[d];
    if (bbox_max) bbox_max[d] = s->h.bbox_max[d];
  }
  return SMP_OK;
}

int smp_scene_export(const smp_scene* s, uint64_t* bits, uint16_t* d2) {
  if (!s) return SMP_ERR_ARG;
  if (bits) std::memcpy(bits, s->h.bits.data(), s->h.bits.size() * sizeof(uint64_t));
  if (d2) std::memcpy(d2, s->h.d2.data(), s->h.d2.size() * sizeof(uint16_t));
  return SMP_OK;
}

static bool params_ok(const smp_params& q) {
  return q.max_near_nodes >= 1 && q.max_near_nodes <= 20 && q.num_traj_segments >= 1 && q.num_traj_segments <= MAX_PTS &&
         q.near_threshold > 0 && q.step_factor > 0 && q.node_capacity >= 0 && q.scout >= 0 && q.scout <= MAX_SCOUTS;
}

int smp_planner_set_params(smp_planner* p, const smp_params* params) {
  if (!p || !params || !params_ok(*params)) return SMP_ERR_ARG;
  p->params = *params;
  return SMP_OK;
}

int smp_planner_get_params(const smp_planner* p, smp_params* params) {
  if (!p || !params) return SMP_ERR_ARG;
  *params = p->params;
  return SMP_OK;
}

int smp_planner_create(int device, const smp_robot* robot, const smp_params* params, smp_planner** out) {
  if (!robot || !out) return SMP_ERR_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) return SMP_ERR_NO_DEVICE;
  HIPCHK(hipSetDevice(device));
  smp_planner* p = new smp_planner();
  p->device = device;
  p->robot = robot->h;
  if (params) p->params = *params; else smp_params_default(&p->params);
  if (!params_ok(p->params)) {
    delete p;
    return SMP_ERR_ARG;
  }
  // The runtime sizes a dispatch's scratch from the device stack limit (hipLimitStackSize, 1 KB per work-item by
  // default), not from the kernel's private segment: a kernel whose fixed private segment exceeds the limit reads
  // and writes scratch beyond its allocation (HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION).  Raise the limit to the
  // largest private segment of the planner's kernels.
  {
    size_t need = 0;
    hipFuncAttributes fa;
    const void* ks[] = {reinterpret_cast<const void*>(&plan_kernel), reinterpret_cast<const void*>(&path_kernel)};
    for (const void* k : ks)
      if (hipFuncGetAttributes(&fa, k) == hipSuccess) need = std::max(need, (size_t)fa.localSizeBytes);
    need = std::max(need, check_kernels_private_bytes());
    need = std::max(need, ik_kernels_private_bytes());
    size_t cur = 0;
    if (hipDeviceGetLimit(&cur, hipLimitStackSize) == hipSuccess && cur < need) {
      need = (need + 255) / 256 * 256;
      if (hipDeviceSetLimit(hipLimitStackSize, need) != hipSuccess) {
        delete p;
        return SMP_ERR_HIP;
      }
    }
  }
  // every failure from here on releases what was created so far (smp_planner_destroy skips null handles)
  if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&p->d_rb, sizeof(RobotDev)) != hipSuccess || hipMalloc(&p->d_mc, sizeof(MapCfg)) != hipSuccess ||
      hipMemcpy(p->d_rb, &p->robot.dev, sizeof(RobotDev), hipMemcpyHostToDevice) != hipSuccess ||
      hipEventCreate(&p->ev0) != hipSuccess || hipEventCreate(&p->ev1) != hipSuccess) {
    smp_planner_destroy(p);
    return SMP_ERR_HIP;
  }
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0)
    p->wall_rate_hz = khz * 1000.0;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
    p->num_cus = cus;
  if (const char* e = std::getenv("SMP_SLOT_SHARE")) p->proc_share = std::max(1, std::atoi(e));
  p->slot_share = p->proc_share;
  int xcc = 0;
  if (hipDeviceGetAttribute(&xcc, hipDeviceAttributeNumberOfXccs, device) == hipSuccess && xcc > 0) p->num_xcd = xcc;
  else (void)hipGetLastError();
  std::memset(&p->sc, 0, sizeof(p->sc));
  int st = update_mapcfg(p);
  if (st) { smp_planner_destroy(p); return st; }
  *out = p;
  return SMP_OK;
}

void smp_planner_destroy(smp_planner* p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  if (busy_check(p) != SMP_OK) {  // a kernel still runs on the buffers: leak them rather than free them under it
    fprintf(stderr, "smp_gpu: planner destroyed while a planning launch still runs; its device memory is leaked\n");
    return;
  }
  if (p->stream) (void)hipStreamSynchronize(p->stream);
  for (auto& q : p->qb) q.release();
  p->d_qdev.release(); p->d_counts.release(); p->d_lfin.release(); p->d_cq.release(); p->d_valid.release();
  p->d_ik_tasks.release(); p->d_ik_out.release(); p->d_ik_best.release(); p->d_path_edges.release();
  p->d_bricks.release(); p->d_d2.release(); p->d_d2b.release(); p->d_slab.release();
  if (p->d_rb) (void)hipFree(p->d_rb);
  if (p->d_mc) (void)hipFree(p->d_mc);
  if (p->ev0) (void)hipEventDestroy(p->ev0);
  if (p->ev1) (void)hipEventDestroy(p->ev1);
  if (p->stream) (void)hipStreamDestroy(p->stream);
  if (p->h_ttff) (void)hipHostFree(p->h_ttff);
  if (p->h_abort) (void)hipHostFree(p->h_abort);
  if (p->h_st) (void)hipHostFree(p->h_st);
  delete p;
}

// The collision tests treat a sphere or primitive whose centre lies outside the grid as free of the map (centre_cell,
// prim_candidate): exact only while every occupied cell keeps GRID_REACH (+ one cell of rounding margin) from every
// face of the grid, which scene_from_keys' padding guarantees.  Grids from elsewhere (smp_scene_from_grid, a device
// scene) are checked here: false if an occupied cell of the 4x4x4 bricks lies closer to a face.
static bool occupancy_clear_of_faces(const uint64_t* bricks, int nx, int ny, int nz, double res) {
  const int m = (int)std::ceil(GRID_REACH / res) + 1;
  const int bnx = (nx + 3) / 4, bny = (ny + 3) / 4, bnz = (nz + 3) / 4;
  const int lo[3] = {m, m, m}, hi[3] = {nx - 1 - m, ny - 1 - m, nz - 1 - m};
  for (int bk = 0; bk < bnz; ++bk)
    for (int bj = 0; bj < bny; ++bj)
      for (int bi = 0; bi < bnx; ++bi) {
        uint64_t w = bricks[((size_t)bk * bny + bj) * bnx + bi];
        if (!w) continue;
        if (4 * bi >= lo[0] && 4 * bi + 3 <= hi[0] && 4 * bj >= lo[1] && 4 * bj + 3 <= hi[1] && 4 * bk >= lo[2] &&
            4 * bk + 3 <= hi[2])
          continue;
        for (; w; w &= w - 1) {
          const int bit = __builtin_ctzll(w);
          const int c[3] = {4 * bi + (bit & 3), 4 * bj + ((bit >> 2) & 3), 4 * bk + (bit >> 4)};
          for (int d = 0; d < 3; ++d)
            if (c[d] < lo[d] || c[d] > hi[d]) return false;
        }
      }
  return true;
}

int smp_planner_set_scene(smp_planner* p, const smp_scene* s) {
  if (!p || !s) return SMP_ERR_ARG;
  if (int b_ = busy_check(const_cast<smp_planner*>(p))) return b_;
  if (!occupancy_clear_of_faces(s->h.bricks.data(), s->h.nx, s->h.ny, s->h.nz, s->h.res)) {
    fprintf(stderr, "smp_gpu: an occupied cell lies within %.2f m of the grid's faces (pad the grid)\n", GRID_REACH);
    return SMP_ERR_ARG;
  }
  HIPCHK(hipSetDevice(p->device));
  HIPCHK(p->d_bricks.reserve(s->h.bricks.size()));
  HIPCHK(p->d_d2.reserve(s->h.d2.size()));
  HIPCHK(hipMemcpyAsync(p->d_bricks.p, s->h.bricks.data(), s->h.bricks.size() * sizeof(uint64_t), hipMemcpyHostToDevice, p->stream));
  HIPCHK(hipMemcpyAsync(p->d_d2.p, s->h.d2.data(), s->h.d2.size() * sizeof(uint16_t), hipMemcpyHostToDevice, p->stream));
  p->sc.nx = s->h.nx; p->sc.ny = s->h.ny; p->sc.nz = s->h.nz;
  p->sc.bnx = s->h.bnx; p->sc.bny = s->h.bny;
  p->sc.ox = s->h.ox; p->sc.oy = s->h.oy; p->sc.oz = s->h.oz; p->sc.res = s->h.res; p->sc.inv_res = 1.0 / s->h.res;
  p->sc.bricks = p->d_bricks.p;
  p->sc.d2 = p->d_d2.p;
  {
    const RobotDev& d = p->robot.dev;
    for (int k = 0; k < d.n_prim; ++k)
      if (d.prim_rxy[k] > GRID_REACH) {  // the padding would not keep a primitive outside the grid free
        fprintf(stderr, "smp_gpu: primitive reach %.3f m exceeds the grid padding\n", d.prim_rxy[k]);
        return SMP_ERR_ARG;
      }
    for (int k = 0; k < MAX_PRIM; ++k) p->sc.slab[k] = nullptr;
    if (d.n_prim > 0) {
      std::vector<std::vector<uint16_t>> slabs;
      prim_slabs(d, s->h, &slabs);
      const size_t plane = (size_t)s->h.nx * s->h.ny;
      std::vector<uint16_t> all(plane * d.n_prim);
      for (int k = 0; k < d.n_prim; ++k) std::memcpy(all.data() + k * plane, slabs[k].data(), plane * sizeof(uint16_t));
      HIPCHK(p->d_slab.reserve(all.size()));
      HIPCHK(hipMemcpyAsync(p->d_slab.p, all.data(), all.size() * sizeof(uint16_t), hipMemcpyHostToDevice, p->stream));
      HIPCHK(hipStreamSynchronize(p->stream));  // `all` is released on return
      for (int k = 0; k < d.n_prim; ++k) p->sc.slab[k] = p->d_slab.p + k * plane;
    }
  }
  // byte copy of the field when every sphere's threshold is below 255 (SceneDev.d2b)
  uint32_t tmax = 0;
  for (int k = 0; k < p->robot.dev.n_sph; ++k) tmax = std::max(tmax, sphere_threshold(p->robot.dev.sph_r[k], s->h.res));
  p->sc.d2b = nullptr;
  if (tmax < 255) {
    std::vector<uint8_t> b(s->h.d2.size());
    for (size_t i = 0; i < b.size(); ++i) b[i] = (uint8_t)std::min<uint16_t>(s->h.d2[i], 255);
    HIPCHK(p->d_d2b.reserve(b.size()));
    HIPCHK(hipMemcpyAsync(p->d_d2b.p, b.data(), b.size(), hipMemcpyHostToDevice, p->stream));
    HIPCHK(hipStreamSynchronize(p->stream));  // b is released on return
    p->sc.d2b = p->d_d2b.p;
  }
  p->have_scene = true;
  p->scene_res = s->h.res;
  return update_mapcfg(p);
}

// Device-resident scene of a planner (multi-GPU): the arrays smp_planner_set_scene derived for
// this robot (bricks, box-gap field, its byte copy, the primitives' slab fields) travel device to device -- an RCCL
// broadcast between ranks, or peer copies over xGMI between the planners of one process -- instead of being rebuilt
// from a host scene on every GPU.
static void scene_layout(const smp_planner* p, smp_scene_device* o) {
  o->dims[0] = p->sc.nx; o->dims[1] = p->sc.ny; o->dims[2] = p->sc.nz;
  o->origin[0] = p->sc.ox; o->origin[1] = p->sc.oy; o->origin[2] = p->sc.oz;
  o->resolution = p->sc.res;
  o->n_bricks = (int64_t)p->sc.bnx * p->sc.bny * (((int64_t)p->sc.nz + 3) / 4);
  o->n_cells = (int64_t)p->sc.nx * p->sc.ny * p->sc.nz;
  o->n_prim = p->robot.dev.n_prim;
  o->has_d2b = p->sc.d2b != nullptr;
}

int smp_planner_scene_device(const smp_planner* p, smp_scene_device* io) {
  if (!p || !io) return SMP_ERR_ARG;
  if (int b_ = busy_check(const_cast<smp_planner*>(p))) return b_;
  if (!p->have_scene) return SMP_ERR_ARG;
  HIPCHK(hipSetDevice(p->device));
  uint64_t* bricks = io->bricks;
  uint16_t* d2 = io->d2;
  uint8_t* d2b = io->d2b;
  uint16_t* slab = io->slab;
  scene_layout(p, io);
  io->bricks = bricks; io->d2 = d2; io->d2b = d2b; io->slab = slab;
  const size_t plane = (size_t)p->sc.nx * p->sc.ny;
  if (bricks) HIPCHK(hipMemcpyAsync(bricks, p->sc.bricks, io->n_bricks * sizeof(uint64_t), hipMemcpyDefault, p->stream));
  if (d2) HIPCHK(hipMemcpyAsync(d2, p->sc.d2, io->n_cells * sizeof(uint16_t), hipMemcpyDefault, p->stream));
  if (d2b && io->has_d2b) HIPCHK(hipMemcpyAsync(d2b, p->sc.d2b, io->n_cells, hipMemcpyDefault, p->stream));
  if (slab && io->n_prim > 0)
    HIPCHK(hipMemcpyAsync(slab, p->d_slab.p, plane * io->n_prim * sizeof(uint16_t), hipMemcpyDefault, p->stream));
  HIPCHK(hipStreamSynchronize(p->stream));
  return SMP_OK;
}

int smp_planner_set_scene_device(smp_planner* p, const smp_scene_device* in) {
  if (!p || !in || !in->bricks || !in->d2) return SMP_ERR_ARG;
  if (int b_ = busy_check(const_cast<smp_planner*>(p))) return b_;
  const int nx = in->dims[0], ny = in->dims[1], nz = in->dims[2];
  if (nx <= 0 || ny <= 0 || nz <= 0 || !(in->resolution > 0)) return SMP_ERR_ARG;
  const RobotDev& d = p->robot.dev;
  const int bnx = (nx + 3) / 4, bny = (ny + 3) / 4, bnz = (nz + 3) / 4;
  const size_t nb = (size_t)bnx * bny * bnz, nc = (size_t)nx * ny * nz, plane = (size_t)nx * ny;
  // the derived arrays depend on the robot (slab z ranges, the byte field's threshold condition): the sender's
  // robot must be this one's
  uint32_t tmax = 0;
  for (int k = 0; k < d.n_sph; ++k) tmax = std::max(tmax, sphere_threshold(d.sph_r[k], in->resolution));
  if (in->n_bricks != (int64_t)nb || in->n_cells != (int64_t)nc || in->n_prim != d.n_prim ||
      (in->has_d2b != 0) != (tmax < 255) || (in->has_d2b && !in->d2b) || (d.n_prim > 0 && !in->slab))
    return SMP_ERR_ARG;
  for (int k = 0; k < d.n_prim; ++k)
    if (d.prim_rxy[k] > GRID_REACH) return SMP_ERR_ARG;
  HIPCHK(hipSetDevice(p->device));
  {  // the occupancy must keep the collision tests' reach from the grid's faces (occupancy_clear_of_faces)
    std::vector<uint64_t> hb(nb);
    HIPCHK(hipMemcpy(hb.data(), in->bricks, nb * sizeof(uint64_t), hipMemcpyDefault));
    if (!occupancy_clear_of_faces(hb.data(), nx, ny, nz, in->resolution)) return SMP_ERR_ARG;
  }
  HIPCHK(p->d_bricks.reserve(nb));
  HIPCHK(p->d_d2.reserve(nc));
  // hipMemcpyDefault: a source on another GPU is a peer copy (xGMI), one on this GPU a device copy
  HIPCHK(hipMemcpyAsync(p->d_bricks.p, in->bricks, nb * sizeof(uint64_t), hipMemcpyDefault, p->stream));
  HIPCHK(hipMemcpyAsync(p->d_d2.p, in->d2, nc * sizeof(uint16_t), hipMemcpyDefault, p->stream));
  p->sc.d2b = nullptr;
  if (in->has_d2b) {
    HIPCHK(p->d_d2b.reserve(nc));
    HIPCHK(hipMemcpyAsync(p->d_d2b.p, in->d2b, nc, hipMemcpyDefault, p->stream));
    p->sc.d2b = p->d_d2b.p;
  }
  for (int k = 0; k < MAX_PRIM; ++k) p->sc.slab[k] = nullptr;
  if (d.n_prim > 0) {
    HIPCHK(p->d_slab.reserve(plane * d.n_prim));
    HIPCHK(hipMemcpyAsync(p->d_slab.p, in->slab, plane * d.n_prim * sizeof(uint16_t), hipMemcpyDefault, p->stream));
    for (int k = 0; k < d.n_prim; ++k) p->sc.slab[k] = p->d_slab.p + k * plane;
  }
  HIPCHK(hipStreamSynchronize(p->stream));  // the caller may release its buffers on return
  p->sc.nx = nx; p->sc.ny = ny; p->sc.nz = nz;
  p->sc.bnx = bnx; p->sc.bny = bny;
  p->sc.ox = in->origin[0]; p->sc.oy = in->origin[1]; p->sc.oz = in->origin[2];
  p->sc.res = in->resolution; p->sc.inv_res = 1.0 / in->resolution;
  p->sc.bricks = p->d_bricks.p;
  p->sc.d2 = p->d_d2.p;
  p->have_scene = true;
  p->scene_res = in->resolution;
  return update_mapcfg(p);
}

int smp_planners_share_scene(smp_planner* const* ps, int n, int src) {
  if (!ps || n <= 0 || src < 0 || src >= n || !ps[src]) return SMP_ERR_ARG;
  smp_scene_device v{};
  int rc = smp_planner_scene_device(ps[src], &v);
  if (rc != SMP_OK) return rc;
  v.bricks = ps[src]->d_bricks.p;
  v.d2 = ps[src]->d_d2.p;
  v.d2b = ps[src]->sc.d2b ? ps[src]->d_d2b.p : nullptr;
  v.slab = v.n_prim > 0 ? ps[src]->d_slab.p : nullptr;
  for (int i = 0; i < n; ++i) {
    if (i == src) continue;
    if (!ps[i]) return SMP_ERR_ARG;
    if (ps[i]->device != ps[src]->device) {
      // direct peer reads over xGMI where the pair allows it (else the runtime stages the copy)
      int can = 0;
      HIPCHK(hipDeviceCanAccessPeer(&can, ps[i]->device, ps[src]->device));
      if (can) {
        HIPCHK(hipSetDevice(ps[i]->device));
        const hipError_t e = hipDeviceEnablePeerAccess(ps[src]->device, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHK(e);
        (void)hipGetLastError();
      }
    }
    rc = smp_planner_set_scene_device(ps[i], &v);
    if (rc != SMP_OK) return rc;
  }
  return SMP_OK;
}

int smp_set_disabled_map_links(smp_planner* p, const char* const* names, int n) {
  if (!p || (n > 0 && !names)) return SMP_ERR_ARG;
  if (int b_ = busy_check(const_cast<smp_planner*>(p))) return b_;
  HIPCHK(hipSetDevice(p->device));
  p->disabled.clear();
  for (int i = 0; i < n; ++i) if (names[i]) p->disabled.insert(names[i]);
  return update_mapcfg(p);
}

int smp_check_configs(smp_planner* p, const double* q_soa, int64_t n, int check_self, int check_map, uint8_t* valid) {
  if (!p || n < 0 || (n > 0 && (!q_soa || !valid))) return SMP_ERR_ARG;
  if (int b_ = busy_check(const_cast<smp_planner*>(p))) return b_;
  if (n == 0) return SMP_OK;
  HIPCHK(hipSetDevice(p->device));
  HIPCHK(p->d_cq.reserve((size_t)n * NJ));
  HIPCHK(p->d_valid.reserve((size_t)n));
  HIPCHK(hipMemcpyAsync(p->d_cq.p, q_soa, (size_t)n * NJ * sizeof(double), hipMemcpyHostToDevice, p->stream));
  long long tiles = (n + 31) / 32;
  int grid = (int)std::min<long long>(tiles, 256 * 8);
  HIPCHK(hipEventRecord(p->ev0, p->stream));
  launch_check(32, grid, p->stream, p->d_rb, p->sc, p->d_mc, p->d_cq.p, (long long)n, check_self,
               check_map && p->have_scene, p->d_valid.p, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(p->ev1, p->stream));
  HIPCHK(hipMemcpyAsync(valid, p->d_valid.p, (size_t)n, hipMemcpyDeviceToHost, p->stream));
  HIPCHK(hipStreamSynchronize(p->stream));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, p->ev0, p->ev1));
  p->last_check_ms = ms;
  return SMP_OK;
}

// getCollisions (birrt_star.cpp:6910-6914 -> collision_checker.hpp:123-132, 594-630): one configuration's
// colliding self pairs (pair order, CC:378-388) and map-colliding links (std::map name order, CC:189, 615).
int smp_get_collisions(smp_planner* p, const double q[8], int32_t* self_pairs, int max_self, int* n_self,
                       int32_t* map_links, int max_map, int* n_map) {
  if (!p || !q || !n_self || !n_map || max_self < 0 || max_map < 0 || (max_self > 0 && !self_pairs) ||
      (max_map > 0 && !map_links))
    return SMP_ERR_ARG;
  if (int b_ = busy_check(const_cast<smp_planner*>(p))) return b_;
  const RobotDev& d = p->robot.dev;
  HIPCHK(hipSetDevice(p->device));
  HIPCHK(p->d_cq.reserve(NJ));
  HIPCHK(p->d_valid.reserve(MAX_CLINK + MAX_PAIRS));
  HIPCHK(hipMemcpyAsync(p->d_cq.p, q, NJ * sizeof(double), hipMemcpyHostToDevice, p->stream));
  launch_collisions(p->stream, p->d_rb, p->sc, p->d_mc, p->d_cq.p, p->have_scene ? 1 : 0, p->d_valid.p,
                    p->d_valid.p + MAX_CLINK);
  HIPCHK(hipGetLastError());
  uint8_t flags[MAX_CLINK + MAX_PAIRS];
  HIPCHK(hipMemcpyAsync(flags, p->d_valid.p, sizeof(flags), hipMemcpyDeviceToHost, p->stream));
  HIPCHK(hipStreamSynchronize(p->stream));
  int ns = 0;
  for (int k = 0; k < d.n_pairs; ++k) {
    if (!flags[MAX_CLINK + k]) continue;
    if (ns < max_self) {
      self_pairs[2 * ns] = d.cl_link[d.pair_a[k]];
      self_pairs[2 * ns + 1] = d.cl_link[d.pair_b[k]];
    }
    ++ns;
  }
  std::vector<int> links;
  for (int c = 0; c < d.n_clink; ++c)
    if (flags[c]) links.push_back(d.cl_link[c]);
  const std::vector<std::string>& names = p->robot.link_names;
  std::sort(links.begin(), links.end(), [&](int a, int b) { return names[a] < names[b]; });
  for (int k = 0; k < (int)links.size() && k < max_map; ++k) map_links[k] = links[k];
  *n_self = ns;
  *n_map = (int)links.size();
  return SMP_OK;
}

int smp_check_sequence(smp_planner* p, const double* q_rows, int64_t n, int check_self, int check_map,
                       int64_t* first_invalid) {
  if (!p || !first_invalid || n < 0 || (n > 0 && !q_rows)) return SMP_ERR_ARG;
  if (int b_ = busy_check(const_cast<smp_planner*>(p))) return b_;
  *first_invalid = -1;
  if (n == 0) return SMP_OK;
  std::vector<double> soa((size_t)n * NJ);
  for (int64_t i = 0; i < n; ++i)
    for (int j = 0; j < NJ; ++j) soa[(size_t)j * n + i] = q_rows[i * NJ + j];
  std::vector<uint8_t> v((size_t)n);
  const int st = smp_check_configs(p, soa.data(), n, check_self, check_map, v.data());
  if (st != SMP_OK) return st;
  for (int64_t i = 0; i < n; ++i)
    if (!v[i]) { *first_invalid = i; break; }
  return SMP_OK;
}

int smp_is_config_valid(smp_planner* p, const double q[8], int check_self, int check_map, int* valid) {
  if (!p || !q || !valid) return SMP_ERR_ARG;
  if (int b_ = busy_check(const_cast<smp_planner*>(p))) return b_;
  double soa[8];
  for (int j = 0; j < 8; ++j) soa[j] = q[j];
  uint8_t v = 0;
  int st = smp_check_configs(p, soa, 1, check_self, check_map, &v);
  *valid = v;
  return st;
}

// IK controller runs (getFullPoseFromEEPose, birrt_star.cpp:1627-1686): one wavefront per task, on p->stream.
// search != 0: the candidates of one findGoalPose -- a run that REACHED checks its pose (isConfigValid,
// birrt_star.cpp:6897-6908) in the same kernel and runs that can no longer be chosen stop early.
static int ik_run(smp_planner* p, const std::vector<IkTaskDev>& tasks, std::vector<IkOutDev>& outs, int search,
                  int check_self, int check_map, double* ms) {
  const int n = (int)tasks.size();
  outs.assign(n, IkOutDev{});
  if (n == 0) return SMP_OK;
  HIPCHK(hipSetDevice(p->device));
  HIPCHK(p->d_ik_tasks.reserve(n));
  HIPCHK(p->d_ik_out.reserve(n));
  HIPCHK(p->d_ik_best.reserve(1));
  HIPCHK(hipMemcpyAsync(p->d_ik_tasks.p, tasks.data(), n * sizeof(IkTaskDev), hipMemcpyHostToDevice, p->stream));
  HIPCHK(hipMemsetAsync(p->d_ik_best.p, 0x7f, sizeof(int), p->stream));
  HIPCHK(hipEventRecord(p->ev0, p->stream));
  launch_ik(search != 0, n, p->stream, p->d_rb, p->d_ik_tasks.p, p->d_ik_out.p, p->sc, p->d_mc, check_self,
            check_map && p->have_scene, p->d_ik_best.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(p->ev1, p->stream));
  HIPCHK(hipMemcpyAsync(outs.data(), p->d_ik_out.p, n * sizeof(IkOutDev), hipMemcpyDeviceToHost, p->stream));
  HIPCHK(hipStreamSynchronize(p->stream));
  float f = 0;
  HIPCHK(hipEventElapsedTime(&f, p->ev0, p->ev1));
  if (ms) *ms = f;
  return SMP_OK;
}

int smp_ik_solve(smp_planner* p, const smp_ik_request* reqs, int n, smp_ik_result* out) {
  if (!p || n < 0 || (n > 0 && (!reqs || !out))) return SMP_ERR_ARG;
  if (int b_ = busy_check(const_cast<smp_planner*>(p))) return b_;
  if (n == 0) return SMP_OK;
  std::vector<IkTaskDev> tasks(n);
  for (int i = 0; i < n; ++i) {
    const smp_ik_request& r = reqs[i];
    if (r.max_iter < 1) return SMP_ERR_ARG;
    IkTaskDev& t = tasks[i];
    std::memset(&t, 0, sizeof(t));
    ik_goal_quat(r.ee_pose, t.goal);
    for (int k = 0; k < 6; ++k) { t.lo[k] = r.deviation[k][0]; t.hi[k] = r.deviation[k][1]; }
    for (int j = 0; j < NJ; ++j) t.q[j] = r.q_init[j];
    t.max_iter = r.max_iter;
  }
  std::vector<IkOutDev> outs;
  double ms = 0;
  const int st = ik_run(p, tasks, outs, 0, 0, 0, &ms);
  if (st != SMP_OK) return st;
  p->last_check_ms = ms;
  for (int i = 0; i < n; ++i) {
    smp_ik_result& o = out[i];
    o.reached = outs[i].reached;
    o.iterations = outs[i].iters;
    o.fallback_iterations = outs[i].fallback;
    for (int j = 0; j < NJ; ++j) o.q[j] = outs[i].q[j];
    for (int k = 0; k < 6; ++k) o.error[k] = outs[i].err[k];
    o.manipulability = outs[i].manip;
  }
  return SMP_OK;
}

int smp_find_goal_pose(smp_planner* p, const double ee_pose[6], const double pose_current[8], double discretization_deg,
                       int check_self, int check_map, double pose_goal[8], int* result, smp_goal_search* info) {
  if (!p || !ee_pose || !pose_current || !pose_goal || !result || !(discretization_deg == discretization_deg))
    return SMP_ERR_ARG;
  if (int b_ = busy_check(const_cast<smp_planner*>(p))) return b_;
  int n = 0;
  ik_goal_candidates(ee_pose, pose_current, discretization_deg, nullptr, 0, &n);
  std::vector<IkTaskDev> tasks(n);
  const int down = ik_goal_candidates(ee_pose, pose_current, discretization_deg, tasks.data(), n, &n);
  std::vector<IkOutDev> outs;
  double ms = 0;
  const int st = ik_run(p, tasks, outs, 1, check_self, check_map, &ms);
  if (st != SMP_OK) return st;
  p->last_check_ms = ms;
  // candidates below the chosen one always run to the end; those above it may have stopped early (IK_ABANDONED)
  int chosen = -1, reached = 0;
  for (int i = 0; i < n; ++i) {
    if (!outs[i].reached) continue;
    ++reached;
    if (chosen < 0 && (outs[i].flags & IK_VALID)) chosen = i;
  }
  *result = chosen >= 0 ? 0 : (reached ? 1 : 2);
  if (chosen >= 0)
    for (int j = 0; j < NJ; ++j) pose_goal[j] = outs[chosen].q[j];
  if (info) {
    info->n_candidates = n;
    info->n_reached = reached;
    info->chosen = chosen;
    info->downward = down;
    info->kernel_ms = ms;
  }
  return SMP_OK;
}

int smp_last_kernel_ms(const smp_planner* p, double* check_ms, double* plan_ms, int64_t* plan_launches) {
  if (!p) return SMP_ERR_ARG;
  if (check_ms) *check_ms = p->last_check_ms;
  if (plan_ms) *plan_ms = p->last_plan_ms;
  if (plan_launches) *plan_launches = p->last_plan_launches;
  return SMP_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------ planning
// C = H * diag(1, .., 1, det H), H = I - 2 v v^T / v^T v, v = e1 - a (DESIGN.md "Informed sampling");
// a non-finite direction (start == goal in a block) falls back to a = e1 (the reference divides by zero).
static void householder_C(const double* a_in, int n, double* C) {
  double a[6], v[6], vv = 0.0;
  bool fin = true;
  for (int i = 0; i < n; ++i) { a[i] = a_in[i]; if (!std::isfinite(a[i])) fin = false; }
  if (!fin) for (int i = 0; i < n; ++i) a[i] = (i == 0) ? 1.0 : 0.0;
  for (int i = 0; i < n; ++i) { v[i] = (i == 0 ? 1.0 : 0.0) - a[i]; vv += v[i] * v[i]; }
  double det = vv == 0.0 ? 1.0 : -1.0;
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < n; ++k) {
      double h = (i == k ? 1.0 : 0.0) - (vv == 0.0 ? 0.0 : 2.0 * v[i] * v[k] / vv);
      C[i * n + k] = (k == n - 1) ? h * det : h;
    }
}

static void init_qstate(const smp_planner* p, const smp_query& q, int64_t cap, int via_cap, QState* S) {
  std::memset(S, 0, sizeof(QState));
  const RobotDev& rb = p->robot.dev;
  S->status = 0;
  S->phase = 0;
  S->A = 0;
  S->n[0] = S->n[1] = 1;
  S->cap = (int)cap;
  S->via_cap = via_cap;
  S->max_iter = q.budget_kind == SMP_BUDGET_ITERATIONS ? (long long)q.budget : (long long)1 << 62;
  S->max_checked = q.budget_kind == SMP_BUDGET_SAMPLES ? std::max<long long>((long long)q.budget, 1) : 0;
  S->first_iter = -1;
  S->last_iter = -1;
  S->cbest[0] = S->cbest[1] = S->cbest[2] = 10000.0;
  double a = 0, r = 0, pp = 0;  // distance_heuristics.cpp:160-217
  for (int j = 0; j < NJ; ++j) {
    double d = q.goal[j] - q.start[j];
    a += d * d;
    if (rb.rev[j]) r += d * d; else pp += d * d;
  }
  S->h0[0] = std::sqrt(a); S->h0[1] = std::sqrt(r); S->h0[2] = std::sqrt(pp);
  for (int j = 0; j < NJ; ++j) { S->qs[j] = q.start[j]; S->qg[j] = q.goal[j]; }
  double arev[6], apr[2];
  int ir = 0, ip = 0;
  for (int j = 0; j < NJ; ++j) {  // jointConfigEllipseInitialization (birrt_star.cpp:3472-3604)
    if (rb.rev[j]) { S->ctr_rev[ir] = (q.start[j] + q.goal[j]) / 2.0; arev[ir++] = (q.goal[j] - q.start[j]) / S->h0[1]; }
    else { S->ctr_pr[ip] = (q.start[j] + q.goal[j]) / 2.0; apr[ip++] = (q.goal[j] - q.start[j]) / S->h0[2]; }
  }
  householder_C(arev, 6, S->Crev);
  householder_C(apr, 2, S->Cpr);
  S->env_x[0] = q.env_x[0]; S->env_x[1] = q.env_x[1];
  S->env_y[0] = q.env_y[0]; S->env_y[1] = q.env_y[1];
  S->near_r = p->params.near_threshold;
  S->step = p->params.step_factor;
  S->opt_thresh = p->params.path_optimality_threshold;
  S->n_pts = p->params.num_traj_segments;
  S->max_near = p->params.max_near_nodes;
  S->tree_opt = p->params.tree_optimization;
  S->informed = p->params.informed_sampling;
  S->self = q.check_self;
  S->map = q.check_map && p->have_scene;
  S->seed = q.seed;
  S->query = q.query_id;
}

static hipError_t alloc_query(QueryBuffers& b, size_t cap, int via_cap, long long rows) {
  hipError_t e;
  if ((e = b.st.reserve(1))) return e;
  if ((e = b.q.reserve(cap * NJ * 2))) return e;
  if ((e = b.qf.reserve(cap * NJ * 2))) return e;
  if ((e = b.cost.reserve(cap * 3 * 2))) return e;
  if ((e = b.e_start.reserve(cap * NJ * 2))) return e;
  if ((e = b.e_target.reserve(cap * NJ * 2))) return e;
  if ((e = b.parent.reserve(cap * 2))) return e;
  if ((e = b.first_child.reserve(cap * 2))) return e;
  if ((e = b.next_sib.reserve(cap * 2))) return e;
  if ((e = b.prev_sib.reserve(cap * 2))) return e;
  if ((e = b.stack.reserve(cap))) return e;
  if ((e = b.path_nodes.reserve(cap * 2))) return e;
  if ((e = b.via.reserve(via_cap))) return e;
  if ((e = b.rows.reserve(std::max<long long>(rows, 1) * 5))) return e;
  if ((e = b.jb.reserve(1))) return e;
  for (int s = 0; s < MAX_SCOUTS; ++s) {
    if ((e = b.sjb[s].reserve(1))) return e;
    if ((e = b.scb[s].reserve(1))) return e;
    if ((e = b.svia[s].reserve(via_cap))) return e;
  }
  b.cap = cap;
  return hipSuccess;
}

static QueryDev make_qdev(QueryBuffers& b, size_t cap, long long rows) {
  QueryDev d;
  std::memset(&d, 0, sizeof(d));
  d.st = b.st.p;
  for (int t = 0; t < 2; ++t) {
    TreeDev& T = d.tr[t];
    T.q = b.q.p + (size_t)t * cap * NJ;
    T.qf = b.qf.p + (size_t)t * cap * NJ;
    T.cost = b.cost.p + (size_t)t * cap * 3;
    T.e_start = b.e_start.p + (size_t)t * cap * NJ;
    T.e_target = b.e_target.p + (size_t)t * cap * NJ;
    T.parent = b.parent.p + (size_t)t * cap;
    T.first_child = b.first_child.p + (size_t)t * cap;
    T.next_sib = b.next_sib.p + (size_t)t * cap;
    T.prev_sib = b.prev_sib.p + (size_t)t * cap;
  }
  d.via = b.via.p;
  d.stack = b.stack.p;
  d.rows = b.rows.p;
  d.rows_cap = rows;
  d.path_nodes = b.path_nodes.p;
  d.jb = nullptr;
  d.sampler_jb = nullptr;
  d.nscouts = 0;
  d.pre_delay = 0;
  d.pre_commit = 0;
  d.pre_refresh = 0;
  for (int s = 0; s < MAX_SCOUTS; ++s) {
    d.scbs[s] = nullptr; d.sjbs[s] = nullptr; d.svias[s] = nullptr; d.sworkers_s[s] = 1;
  }
  d.scb = nullptr;
  d.sjb = nullptr;
  d.svia = nullptr;
  d.sworkers = 1;
  d.nworkers = 1;
  // configurations per job tile: by job size (smp_plan.h job_tile_ct); SMP_TILE_CT = 1 / 2 / 4 / 8 fixes it (experiments)
  d.tile_ct = 0;
  if (const char* e = std::getenv("SMP_TILE_CT")) {
    const int v = std::atoi(e);
    if (v == 1 || v == 2 || v == 4 || v == 8) d.tile_ct = v;
  }
  d.sampler = 0;
  d.trace = nullptr;
  d.ttff = nullptr;
  d.abort = nullptr;
  d.lfin = nullptr;
  d.lquota = 0;
  // scans of trees of at least this many nodes are split over the helpers (DESIGN.md "Scans of large trees");
  // SMP_SCAN_MIN overrides it (experiments and tests; 0: never)
  d.scan_min = 12288;
  if (const char* e = std::getenv("SMP_SCAN_MIN")) d.scan_min = std::max(0, std::atoi(e));
  // participants of one split scan: a nearest result is 3 granules, a near result 122 -- fewer, longer slices for
  // near: one per 2^scan_nshift nodes (4096), 8 to 32 (SMP_SCAN_PNN / SMP_SCAN_PNEAR cap them, SMP_SCAN_NSHIFT sets
  // the shift)
  d.scan_pnn = 64;
  d.scan_pnear = SCAN_PNEAR;
  if (const char* e = std::getenv("SMP_SCAN_PNN")) d.scan_pnn = std::atoi(e);
  if (const char* e = std::getenv("SMP_SCAN_PNEAR")) d.scan_pnear = std::atoi(e);
  d.scan_nshift = 12;
  if (const char* e = std::getenv("SMP_SCAN_NSHIFT")) d.scan_nshift = std::min(20, std::max(6, std::atoi(e)));
  d.scan_ps0 = 0;
  if (const char* e = std::getenv("SMP_SCAN_PS0")) d.scan_ps0 = std::min(4, std::max(0, std::atoi(e)));
  d.scan_pnn = std::min(SCAN_P, std::max(2, d.scan_pnn));
  d.scan_pnear = std::min(SCAN_PNEAR, std::max(2, d.scan_pnear));
  return d;
}

// smp_plan_batch's body.  done[i] is set once out[i] holds query i's complete result; a call that fails on the way
// (a HIP error, the no-progress guard) returns early, and smp_plan_batch then reports that status in every
// result not yet complete.
static int plan_batch_impl(smp_planner* p, const smp_query* qs, int nq, smp_result* out, std::vector<char>& done) {
  const auto t_entry = std::chrono::steady_clock::now();
  HIPCHK(hipSetDevice(p->device));
  // arguments; init_planner's validity of start and goal (birrt_star.cpp:350-362) is the kernel's first step (its
  // first launch checks both with the query's own self / map flags: no separate check launch and wait here)
  std::vector<int> status(nq, SMP_OK);
  for (int i = 0; i < nq; ++i) {
    const int bk = qs[i].budget_kind;
    if (!(qs[i].budget >= 0) || (bk != SMP_BUDGET_ITERATIONS && bk != SMP_BUDGET_SECONDS && bk != SMP_BUDGET_SAMPLES))
      status[i] = SMP_ERR_ARG;
  }
  // SMP_HOST_PROF: microseconds from smp_plan entry to each host stage of the first launch (experiments)
  const bool hprof = std::getenv("SMP_HOST_PROF") != nullptr;
  auto hstamp = [&](const char* what) {
    if (hprof)
      std::fprintf(stderr, "[smp host] %-22s %8.1f us\n", what,
                   std::chrono::duration<double>(std::chrono::steady_clock::now() - t_entry).count() * 1e6);
  };
  hstamp("arguments checked");
  if ((int)p->qb.size() < nq) p->qb.resize(nq);
  std::vector<QueryDev> qdev(nq);
  // the loop states in pinned host memory: their uploads and read-backs are true asynchronous copies (a pageable
  // source is staged synchronously: tens of microseconds before the first launch, inside the time to a first path)
  if (p->n_st < nq) {
    if (p->h_st) (void)hipHostFree(p->h_st);
    p->h_st = nullptr;
    p->n_st = 0;
    HIPCHK(hipHostMalloc(&p->h_st, (size_t)nq * sizeof(QState), hipHostMallocDefault));
    p->n_st = nq;
  }
  QState* S = p->h_st;
  hstamp("host states");
  std::vector<long long> rows_cap(nq, 0);
  for (int i = 0; i < nq; ++i) {
    const smp_query& q = qs[i];
    int64_t cap = p->params.node_capacity;
    const bool by_iter = q.budget_kind == SMP_BUDGET_ITERATIONS;
    long long iters = by_iter ? (long long)q.budget : 0;
    if (cap <= 0) {
      if (by_iter) cap = std::min<int64_t>(1024 + 16 * iters, (int64_t)1 << 27);
      else if (q.budget_kind == SMP_BUDGET_SAMPLES) cap = std::min<int64_t>(1024 + (int64_t)q.budget / 2, (int64_t)1 << 27);
      else cap = (int64_t)4 << 20;
    }
    rows_cap[i] = by_iter ? std::max<long long>(iters, 1) : 1 << 20;
    // via nodes one connect / choose-parent chain may add (a chain of step_factor steps across the workspace: a few
    // dozen on a 10 m map); an eighth of the tree capacity, so that a seconds budget's stop margin (two chains) leaves
    // three quarters of an explicit node_capacity usable.  A longer chain ends the run with SMP_ERR_CAPACITY.
    const int via_cap = (int)std::max<int64_t>(64, std::min<int64_t>(4096, cap / 8));
    HIPCHK(alloc_query(p->qb[i], (size_t)cap, via_cap, rows_cap[i]));
    if (i == 0) hstamp("query 0 buffers");
    qdev[i] = make_qdev(p->qb[i], (size_t)cap, rows_cap[i]);
    init_qstate(p, q, cap, via_cap, &S[i]);
    if (i == 0) hstamp("query 0 state");
    if (q.budget_kind == SMP_BUDGET_SECONDS) {
      // the budget counts from smp_plan entry (start / goal checks and first-call allocation included); the kernel
      // turns the rest into a deadline when it records the planning start
      const double left = q.budget - std::chrono::duration<double>(std::chrono::steady_clock::now() - t_entry).count();
      S[i].has_deadline = 1;
      S[i].budget_ticks = (unsigned long long)(std::max(left, 0.0) * p->wall_rate_hz);
      S[i].stop_margin = 2 * via_cap + 4;  // nodes one iteration can add at most (two via chains + x_new + connection)
    }
    if (status[i] != SMP_OK) { S[i].status = status[i]; S[i].phase = 2; }
    if (by_iter && iters <= 0 && S[i].phase == 0) S[i].max_iter = 0;
    // (the two roots are written by the kernel's first launch from QState::qs / qg: no per-word uploads)
    HIPCHK(hipMemcpyAsync(qdev[i].st, &S[i], sizeof(QState), hipMemcpyHostToDevice, p->stream));
  }
  // Workgroups per query (one per CU): the leader, its scouts and the helpers (DESIGN.md "Helpers", "Scouts").
  // Scouts: smp_params.scout of them (1: automatic -- 4 from 64 CUs per query (scouts 2 and 3 take every other
  // iteration before the first solution and retire after it: time to first path 2.1 -> 1.7 ms on C2), 2 from 18,
  // 1 from 6).  Helpers: the leader's tile helpers, each scout's, and the run-ahead sampler (the last one); up to 200
  // with scouts (C2: 127 -> 200 helpers 3.65 -> 3.75 M configs/s with four scouts; 250 no longer all fit and stall).
  // Every workgroup of a query (leader, scouts, helpers) polls the others, so all of them must be resident at once:
  // the budget is the device's co-resident capacity for these kernels (occupancy x CUs), not a fixed count.  With
  // automatic helpers the provisioning is redone for the queries still running whenever a launch ends with some of
  // them finished (DESIGN.md "Many queries").
  const int nh_req = p->params.helpers;
  const bool want_scout = p->params.scout != 0;
  const int slots = resident_slots(p);
  int cap_s = 200;  // SMP_HELPER_CAP: experiments with other helper caps
  if (const char* e = std::getenv("SMP_HELPER_CAP")) cap_s = std::max(1, std::atoi(e));
  int lead_div = 3;  // SMP_LEAD_DIV: the leader's share of the helpers (C2: 1/3 3.82, 1/5 3.75, 1/8 3.73 M configs/s)
  if (const char* e = std::getenv("SMP_LEAD_DIV")) lead_div = std::max(1, std::atoi(e));
  // SMP_PRE_HELPERS: helpers of each pre-solution-only scout (its jobs: expand + connect edge, 42 configurations).  12
  // (round 6; ct 4 tiles instead of 8): time to first path median 1.68 -> 1.61 ms over the 20 seeds on one box, C2 equal
  // (57.5 / 57.7 us per iteration); 16 1.61 ms but C2 69.0 against 68.4 us at 30000 iterations
  int pre_h = 12;
  if (const char* e = std::getenv("SMP_PRE_HELPERS")) pre_h = std::max(0, std::atoi(e));
  // before the first solution a scout starts record k when the leader reaches k - pre_delay (DESIGN.md "Pre-solution
  // commits"); SMP_PRE_DELAY overrides it for experiments (0: at the request)
  int pre_delay = 3;
  if (const char* e = std::getenv("SMP_PRE_DELAY")) pre_delay = std::atoi(e);
  int early_ask = 0;  // SMP_EARLY_ASK=1: after the first solution, iteration k + 2 is asked for before k's rewires (DESIGN.md "Early asks")
  if (const char* e = std::getenv("SMP_EARLY_ASK")) early_ask = std::atoi(e);
  // SMP_PRE_REFRESH: a pre-solution scout rechecks its nearest on the leader's newer sizes after its expand job (bit 0)
  // and / or before it publishes (bit 1), starting the pass over (at most twice) when a newer node is nearer
  // (DESIGN.md "Pre-solution refresh"; bit 0 alone measured best)
  int pre_refresh = 1;
  if (const char* e = std::getenv("SMP_PRE_REFRESH")) pre_refresh = std::atoi(e);
  int conn_check = 0;  // SMP_CONN_CHECK=1: connect's edges checked by the scouts with their SC_CONN scans (experiments)
  if (const char* e = std::getenv("SMP_CONN_CHECK")) conn_check = std::atoi(e);
  int pre_commit = 1;  // SMP_PRE_COMMIT=0: every iteration runs the full path (experiments)
  if (const char* e = std::getenv("SMP_PRE_COMMIT")) pre_commit = std::atoi(e);
  int rebalance = nh_req == 0 ? 1 : 0;  // SMP_REBALANCE=0: keep the first launch's provisioning (experiments)
  if (const char* e = std::getenv("SMP_REBALANCE")) rebalance = rebalance && std::atoi(e) != 0;
  // SMP_REBALANCE_DIV: a launch ends once 1/rb_div of its queries finished (C3, 64 queries: 2 / 4 / 8 all 10.1-10.3
  // M configs/s; C5, 8 queries: 0.49 / 0.61 / 0.62 M)
  // several queries run in time slices (SMP_SLICE_MS, default 50; 0: chunks of 256 .. 4096 iterations): a launch
  // ends at its slice or when a quarter of its queries finished, never waiting for the slowest query's chunk --
  // C5's queries differ 5x in iteration time (tools/batch_probe.py)
  double slice_ms = 50.0;
  if (const char* e = std::getenv("SMP_SLICE_MS")) slice_ms = std::max(0.0, std::atof(e));
  int rb_div = 4;
  if (const char* e = std::getenv("SMP_REBALANCE_DIV")) rb_div = std::max(1, std::atoi(e));
  int xcd_margin = 1;
  if (const char* e = std::getenv("SMP_XCD_MARGIN")) xcd_margin = std::max(0, std::atoi(e));
  int nh = 0, ns = 0, ns_base = 0;
  int pre_scouts = 1;
  int pre_lead_div = 5;  // SMP_PRE_LEAD_DIV: the leader's share of a pre-solution query's helpers (1 / n)
  if (const char* e = std::getenv("SMP_PRE_LEAD_DIV")) pre_lead_div = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("SMP_PRE_SCOUTS")) pre_scouts = std::atoi(e);
  auto provision = [&](const std::vector<int>& act) {
    const int na = std::max(1, (int)act.size());
    const int cpq = std::max(1, slots / na);
    nh = nh_req;
    ns = 0;
    if (nh == 0) {
      if (want_scout) ns = cpq >= 64 ? 4 : cpq >= 18 ? 2 : cpq >= 6 ? 1 : 0;
      if (want_scout && p->params.scout > 1) ns = std::min(p->params.scout, MAX_SCOUTS);
      nh = want_scout ? std::min(cap_s, std::max(0, cpq - 1 - ns)) : std::min(63, std::max(0, cpq - 1));
    } else if (nh > 0 && want_scout) {
      ns = nh >= 16 ? 2 : nh >= 4 ? 1 : 0;
    }
    if (want_scout && p->params.scout > 1) ns = std::min(p->params.scout, MAX_SCOUTS);  // explicit count
    if (nh < 0) nh = 0;
    if (nh < 4) ns = 0;
    // per query: where the automatic count is two, a query still without a path takes four (scouts 2 and 3 take every
    // other pre-solution iteration and retire at the first path; C5 query 1 alone, 59 helpers: 25.5 -> 14.0 us per
    // iteration); ns is then the launch's largest count (grid, boards, XCD budget).  SMP_PRE_SCOUTS=0: uniform
    ns_base = ns;
    if (pre_scouts && nh_req == 0 && p->params.scout == 1 && ns == 2)
      for (int i : act)
        if (!S[i].have_sol) { ns = 4; break; }
    // per XCD: the workgroups of a launch are dealt round-robin over the 8 XCDs (blocks b and b + 8 share one), and a
    // workgroup dealt to a full XCD waits there -- a persistent helper that never starts leaves its tiles to the
    // leader's timeout on every job.  plan_kernel puts query q's leader and scouts on XCD slot q % 8, so the fullest
    // XCD holds (1 + ns) ceil(na / 8) of them; the helpers, dealt evenly, get what that XCD leaves, less
    // SMP_XCD_MARGIN CUs (default 1: the two launches race for the CUs).  C5, 8 queries rebalanced to 6 and 4:
    // 39 / 59 helpers each (some never resident) 0.65 M configs/s, 26 each 1.12 M.
    // (a device of one XCD has no such round-robin: no cap)
    const int nx = p->num_xcd;
    if (nx > 1 && p->num_cus >= nx) {
      const int per_xcd = p->num_cus / nx / std::max(1, p->slot_share);
      const int plan_max = (1 + ns) * ((na + nx - 1) / nx);
      const int free_xcd = std::max(0, per_xcd - plan_max - xcd_margin);
      const int hcap = nx * free_xcd / na;
      // (an explicit request beyond it gets no more than the automatic count either)
      if (nh > hcap) nh = std::max(0, nh_req > 0 ? std::min(hcap, cap_s) : hcap);
      // scouts need helpers of their own (and the boards' reset needs nh > 0): below four, none (as above)
      if (nh < 4) { ns = 0; ns_base = 0; }
    }
    // an explicit request larger than what can be resident is clamped to the automatic count: a helper that never
    // starts would leave its tiles to the leader's 8 us timeout on every job (helper sweeps: 250 helpers beside four
    // scouts no longer all start on 256 CUs and stall)
    if (1 + ns + nh > cpq) {
      nh = std::max(0, want_scout ? std::min(cap_s, cpq - 1 - ns) : std::min(63, cpq - 1));
      if (nh < 4) { ns = 0; ns_base = 0; nh = std::max(0, std::min(nh, cpq - 1)); }
    }
    // after the first solution scouts 0 and 1 check choose-parent / rewire candidate batches (many tiles); scouts 2
    // and 3 only work before it, one edge per job (3 tiles); the leader's own jobs (edges no record had) are rare
    auto split = [&](int nsq, int& h_lead, int* h_s) {
      h_lead = 0;
      for (int s = 0; s < MAX_SCOUTS; ++s) h_s[s] = 0;
      if (nh < 1) return;  // (nh < 4 has no scouts: nothing to split)
      if (nsq > ns_base) {  // a query's pre-solution scouts: their records carry its iterations, one in four each
        const int avail = nh - 1;
        h_lead = avail / pre_lead_div;
        const int per = (avail - h_lead) / nsq;
        for (int s = 0; s < nsq; ++s) h_s[s] = per;
        h_s[0] += avail - h_lead - per * nsq;
      } else if (nsq > 0) {
        const int avail = nh - 1;  // minus the sampler
        h_lead = nsq >= 2 ? avail / lead_div : avail / 2;
        int rest = avail - h_lead;
        for (int s = 2; s < nsq; ++s) { h_s[s] = std::min(pre_h, rest); rest -= h_s[s]; }
        if (nsq >= 2) { h_s[0] = rest - rest / 2; h_s[1] = rest / 2; } else { h_s[0] = rest; }
      }
    };
    for (int i : act) {
      const int nsq = ns > ns_base && S[i].have_sol ? ns_base : ns;
      int h_lead = 0, h_s[MAX_SCOUTS];
      split(nsq, h_lead, h_s);
      qdev[i].jb = nh > 0 ? p->qb[i].jb.p : nullptr;
      qdev[i].sampler = nh >= 2;              // with two or more helpers, the last one runs ahead sampling
      qdev[i].nworkers = nsq > 0 ? 1 + h_lead : (nh >= 2 ? nh : 1 + nh);
      qdev[i].nscouts = nsq;
      qdev[i].pre_delay = pre_delay;
      qdev[i].pre_commit = pre_commit;
      qdev[i].early_ask = early_ask;
      qdev[i].pre_refresh = pre_refresh;
      qdev[i].conn_check = conn_check;
      qdev[i].sampler_jb = p->qb[i].jb.p;
      for (int s = 0; s < ns; ++s) {
        qdev[i].sjbs[s] = p->qb[i].sjb[s].p;
        qdev[i].scbs[s] = p->qb[i].scb[s].p;
        qdev[i].svias[s] = p->qb[i].svia[s].p;
        qdev[i].sworkers_s[s] = 1 + h_s[s];
      }
    }
  };
  // the queries to launch: those not decided on the host (an invalid start / goal or argument)
  std::vector<int> act;
  for (int i = 0; i < nq; ++i)
    if (S[i].phase != 2 && S[i].status == 0) act.push_back(i);
  std::vector<int> all(nq);
  for (int i = 0; i < nq; ++i) all[i] = i;
  std::vector<int> sol_seen(nq, 0);
  provision(act.empty() ? all : act);
  const int nh_first = nh, ns_first = ns;
  static int* trace_host = nullptr;
  const bool debug = std::getenv("SMP_DEBUG") != nullptr;
  if (debug && !trace_host) HIPCHK(hipHostMalloc(&trace_host, 256 * sizeof(int), hipHostMallocMapped));
  if (debug) {
    int* trace_dev = nullptr;
    std::memset(trace_host, 0, 256 * sizeof(int));
    HIPCHK(hipHostGetDevicePointer((void**)&trace_dev, trace_host, 0));
    qdev[0].trace = trace_dev;
  }
  // first feasible path on the host's clock (from run_planner entry): the kernel sets a host-mapped flag
  // when it commits the first solution and the launch loop below polls it
  if (p->n_ttff < nq) {
    if (p->h_ttff) (void)hipHostFree(p->h_ttff);
    p->h_ttff = nullptr;
    p->n_ttff = 0;
    HIPCHK(hipHostMalloc(&p->h_ttff, nq * sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent));
    p->n_ttff = nq;
  }
  for (int i = 0; i < nq; ++i) __atomic_store_n(&p->h_ttff[i], 0u, __ATOMIC_RELAXED);
  {
    unsigned* dflag = nullptr;
    HIPCHK(hipHostGetDevicePointer((void**)&dflag, p->h_ttff, 0));
    for (int i = 0; i < nq; ++i) qdev[i].ttff = dflag + i;
  }
  // the abort word (QueryDev::abort): cleared for this call (busy_check has seen every earlier launch drain)
  if (!p->h_abort) HIPCHK(hipHostMalloc(&p->h_abort, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent));
  __atomic_store_n(p->h_abort, 0u, __ATOMIC_RELEASE);
  {
    unsigned* dabort = nullptr;
    HIPCHK(hipHostGetDevicePointer((void**)&dabort, p->h_abort, 0));
    for (int i = 0; i < nq; ++i) qdev[i].abort = dabort;
  }
  std::vector<double> host_ttff(nq, -1.0);
  auto poll_ttff = [&]() {
    for (int i = 0; i < nq; ++i)
      if (host_ttff[i] < 0 && __atomic_load_n(&p->h_ttff[i], __ATOMIC_ACQUIRE))
        host_ttff[i] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_entry).count();
  };
  HIPCHK(p->d_qdev.reserve(nq));
  HIPCHK(p->d_counts.reserve(2 * nq));
  HIPCHK(p->d_lfin.reserve(1));
  // the launch's query records, compacted to the queries still running
  std::vector<QueryDev> qlaunch;
  auto upload_active = [&]() -> int {
    qlaunch.clear();
    const int quota = rebalance && act.size() >= 2 ? std::max(1, (int)act.size() / rb_div) : 0;
    for (int i : act) {
      qdev[i].lfin = p->d_lfin.p;
      qdev[i].lquota = quota;
      qdev[i].lticks = act.size() >= 2 && slice_ms > 0 ? (long long)(slice_ms * 1e-3 * p->wall_rate_hz) : 0;
      qlaunch.push_back(qdev[i]);
    }
    // (qlaunch outlives the copy: it changes only after the next launch has completed)
    if (!qlaunch.empty())
      HIPCHK(hipMemcpyAsync(p->d_qdev.p, qlaunch.data(), qlaunch.size() * sizeof(QueryDev), hipMemcpyHostToDevice,
                            p->stream));
    return SMP_OK;
  };
  hstamp("queries uploaded");
  if (int st = upload_active()) return st;
  hstamp("provisioned");

  // launch loop: each launch advances every running query by up to `chunk` iterations; time budgets use a device
  // deadline
  double tmax = 0;
  for (int i = 0; i < nq; ++i) if (qs[i].budget_kind == SMP_BUDGET_SECONDS) tmax = std::max(tmax, qs[i].budget);
  auto t_begin = std::chrono::steady_clock::now();
  // a seconds budget bounds the host's wait for a launch at 4x the budget + this slack (SMP_WAIT_SLACK_S: tests)
  double wait_slack = 60.0;
  if (const char* e = std::getenv("SMP_WAIT_SLACK_S")) wait_slack = std::atof(e);
  // a single query runs its whole budget in one launch (the loop state is resumable, but a relaunch costs the host
  // round trip, the board reset and the scouts' restart: C2, 5 launches of 256 .. 4096 iterations, ~1 ms each);
  // several queries start at 256 iterations and double, so that finished ones free their CUs early (rebalance)
  int chunk = nq == 1 || slice_ms > 0 ? (1 << 30) : 256;
  if (const char* e = std::getenv("SMP_CHUNK0")) chunk = std::max(1, std::atoi(e));  // experiments
  std::vector<std::array<unsigned long long, 32>> scout_prof(nq);
  for (auto& a : scout_prof) a.fill(0);
  float total_ms = 0;
  int64_t launches = 0;
  long long max_iters = 0;
  for (int i = 0; i < nq; ++i)
    if (qs[i].budget_kind != SMP_BUDGET_SECONDS) max_iters = std::max(max_iters, (long long)qs[i].budget);
  while (!act.empty()) {
    // no progress: never spin forever (a launch ended early by finished queries counts too)
    if (tmax == 0 && launches > max_iters / 256 + 64 + 2 * nq +
                                    (slice_ms > 0 ? (long long)(total_ms / slice_ms) * 2 : 0))
      return SMP_ERR_HIP;
    if (tmax > 0 && std::chrono::duration<double>(std::chrono::steady_clock::now() - t_begin).count() > tmax * 4 + wait_slack)
      return SMP_ERR_HIP;
    const int na = (int)act.size();
    HIPCHK(hipMemsetAsync(p->d_lfin.p, 0, sizeof(unsigned), p->stream));
    if (nh > 0) {
      // fresh boards before the launch (its helpers poll them from their start and leave on the leader's stop)
      hipLaunchKernelGGL(boards_reset_kernel, dim3(na * (1 + 2 * ns)), dim3(BLOCK), 0, p->stream, p->d_qdev.p, ns);
      HIPCHK(hipGetLastError());
    }
    if (launches == 0) hstamp("boards reset issued");
    HIPCHK(hipEventRecord(p->ev0, p->stream));
    // one dispatch for every workgroup of the launch (plan_kernel): leaders at blocks [0, na), scout s of query q at
    // scout_base + s * round8(na) + q, helper h of query q at helper_base + h * na + q; scout_base and helper_base are
    // multiples of 8, so blocks b and b + 8 are dealt to the same XCD (a query's leader and scouts share one).  The
    // leaders and scouts come first in dispatch order, so their workgroups find CUs first.
    const int r8 = (na + 7) / 8 * 8;
    const int scout_base = ns > 0 ? r8 : 0;
    const int helper_base = nh > 0 ? (ns > 0 ? scout_base + ns * r8 : r8) : (1 << 30);
    const int grid = nh > 0 ? helper_base + na * nh : (ns > 0 ? scout_base + (ns - 1) * r8 + na : na);
    hipLaunchKernelGGL(plan_kernel, dim3(grid), dim3(BLOCK), 0, p->stream, p->d_rb, p->sc,
                       p->d_mc, p->d_qdev.p, na, scout_base, helper_base, chunk);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(p->ev1, p->stream));
    if (launches == 0) hstamp("kernels launched");
    launches++;
    // time the first feasible path on the host: poll the flags while the launch runs -- spinning (with a yield) until
    // every query has its first path, then sleeping between polls; a seconds budget bounds the wait (SMP_DEBUG builds
    // skip this loop for the bounded diagnostic wait below)
    if (!debug) {
      hipError_t qe;
      while ((qe = hipEventQuery(p->ev1)) == hipErrorNotReady) {
        poll_ttff();
        bool all = true;
        for (int i : act) all = all && host_ttff[i] >= 0;
        if (all) std::this_thread::sleep_for(std::chrono::microseconds(50));
        else std::this_thread::yield();
        if (tmax > 0 && std::chrono::duration<double>(std::chrono::steady_clock::now() - t_begin).count() > tmax * 4 + wait_slack) {
          // the launch still runs on this planner's buffers: ask it to end (its leaders poll the abort word every
          // ABORT_EVERY iterations) and refuse calls until it has drained (busy_check)
          __atomic_store_n(p->h_abort, 1u, __ATOMIC_RELEASE);
          p->busy = true;
          return SMP_ERR_HIP;
        }
      }
      if (qe != hipSuccess) HIPCHK(qe);
      poll_ttff();
    }
    if (debug) {  // bounded wait: print the leader's progress markers if the launch does not finish
      auto tw = std::chrono::steady_clock::now();
      hipError_t qe;
      while ((qe = hipStreamQuery(p->stream)) == hipErrorNotReady || qe != hipSuccess) {
        if (qe != hipErrorNotReady || std::chrono::duration<double>(std::chrono::steady_clock::now() - tw).count() > 10.0) {
          if (qe != hipErrorNotReady) std::fprintf(stderr, "[smp] launch %lld failed: %s\n", (long long)launches, hipGetErrorString(qe));
          std::fprintf(stderr, "[smp] launch %lld did not finish in 10 s; leader trace:", (long long)launches);
          for (int i = 0; i < 8; ++i) std::fprintf(stderr, " %d", trace_host[i]);
          std::fprintf(stderr, "\n");
          std::_Exit(3);
        }
      }
    }
    for (int i : act)
      HIPCHK(hipMemcpyAsync(&S[i], qdev[i].st, sizeof(QState), hipMemcpyDeviceToHost, p->stream));
    if (ns > 0) {  // every scout's phase clocks, summed (per-pass averages divide by the summed pass count)
      HIPCHK(hipStreamSynchronize(p->stream));
      for (int i : act)
        for (int sc = 0; sc < ns; ++sc) {
          unsigned long long sp[32];
          HIPCHK(hipMemcpy(sp, qdev[i].scbs[sc]->prof, sizeof(sp), hipMemcpyDeviceToHost));
          for (int k = 0; k < 32; ++k) scout_prof[i][k] += sp[k];
          if (i == 0 && std::getenv("SMP_DEBUG_SCOUTS")) {  // per-scout passes and XCD (experiments)
            int xcc = 0;
            HIPCHK(hipMemcpy(&xcc, &qdev[i].scbs[sc]->xcc, sizeof(int), hipMemcpyDeviceToHost));
            std::fprintf(stderr, "[smp] launch %lld scout %d: passes %llu busy %.1f us idle %.1f us xcc %d\n",
                         (long long)launches, sc, sp[30], sp[31] / (p->wall_rate_hz * 1e-6), sp[28] / (p->wall_rate_hz * 1e-6),
                         xcc - 1);
          }
        }
    }
    HIPCHK(hipStreamSynchronize(p->stream));
    if (std::getenv("SMP_BOUNDS")) {
      int dbg[8];
      if (smp_debug_bounds(dbg) == 0 && dbg[0])
        std::fprintf(stderr, "[smp] bounds: line %d id %d block %d tree %d limit %d (launch %lld)\n", dbg[0], dbg[1],
                     dbg[2], dbg[3], dbg[4], (long long)launches);
    }
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, p->ev0, p->ev1));
    total_ms += ms;
    if (std::getenv("SMP_DEBUG")) {
      JobBoard jbh;
      const int i0 = act[0];
      if (nh > 0) HIPCHK(hipMemcpy(&jbh, qdev[i0].jb, sizeof(JobBoard), hipMemcpyDeviceToHost));
      std::fprintf(stderr, "[smp] launch %lld queries %d grid %d chunk %d: %.3f ms phase %d status %d iter %lld checked %lld"
                   " board stop %d job %u tile0 %llx\n", (long long)launches, na, na * (1 + nh), chunk, ms, S[i0].phase,
                   S[i0].status, S[i0].iter, S[i0].checked, nh ? jbh.stop : -1, nh ? (unsigned)(jbh.pay[0] >> 32) : 0u,
                   nh ? jbh.res[0] : 0ull);
    }
    std::vector<int> still;
    int solved_before = 0, solved_now = 0;
    for (int i : act) solved_before += sol_seen[i];
    for (int i : act)
      if (!(S[i].phase == 2 || S[i].status != 0)) still.push_back(i);
    for (int i : act) { sol_seen[i] = S[i].have_sol ? 1 : 0; solved_now += sol_seen[i]; }
    const bool shrank = still.size() < act.size();
    act.swap(still);
    if (act.empty()) break;
    // (a query that found its first path gives its pre-solution scouts back: re-provisioned too)
    if (shrank || (ns > ns_base && solved_now != solved_before)) {
      if (rebalance) provision(act);
      if (int st = upload_active()) return st;
    }
    if (chunk < 4096) chunk *= 2;
  }
  hstamp("launch loop done");
#ifdef SMP_RING_CHECK
  smp_ringchk_dump();
#endif
  // path extraction reads every query's record: the full array again
  HIPCHK(hipMemcpyAsync(p->d_qdev.p, qdev.data(), nq * sizeof(QueryDev), hipMemcpyHostToDevice, p->stream));
  nh = nh_first;
  ns = ns_first;
  p->last_plan_ms = total_ms;
  p->last_plan_launches = launches;

  // path extraction
  hipLaunchKernelGGL(path_kernel, dim3(nq), dim3(64), 0, p->stream, p->d_qdev.p, p->d_counts.p);
  HIPCHK(hipGetLastError());
  std::vector<int> counts(2 * nq);
  HIPCHK(hipMemcpyAsync(counts.data(), p->d_counts.p, 2 * nq * sizeof(int), hipMemcpyDeviceToHost, p->stream));
  HIPCHK(hipStreamSynchronize(p->stream));
  int rc = SMP_OK;
  for (int i = 0; i < nq; ++i) {
    QState& s = S[i];
    smp_result& r = out[i];
    size_t cap = p->qb[i].cap;
    r.status = s.status != 0 ? s.status : (s.have_sol ? SMP_OK : SMP_ERR_NO_SOLUTION);
    smp_stats& st = r.stats;
    st.iterations = s.iter;
    st.first_solution_iter = s.first_iter;
    st.last_solution_iter = s.last_iter;
    st.configs_checked = s.checked;
    st.configs_valid = s.valid;
    st.time_first_solution = s.have_sol && s.t_first >= s.t0 ? (double)(s.t_first - s.t0) / p->wall_rate_hz : -1.0;
    st.time_total = s.t_end >= s.t0 ? (double)(s.t_end - s.t0) / p->wall_rate_hz : 0.0;
    st.time_first_solution_host = s.have_sol ? host_ttff[i] : -1.0;
    for (int k = 0; k < 3; ++k) { st.cost_best[k] = s.cbest[k]; st.cost_theoretical[k] = s.h0[k]; }
    st.nodes_start = s.n[0]; st.nodes_goal = s.n[1];
    st.edges_start = s.edges[0]; st.edges_goal = s.edges[1];
    st.rewires_start = s.rewires[0]; st.rewires_goal = s.rewires[1];
    st.connected_tree_is_start = s.conn_start;
    st.conn_node_b = s.nB.id; st.conn_node_a = s.nA.id;
    st.nn_nodes_scanned = s.nn_nodes;
    st.near_nodes_scanned = s.near_nodes;
    st.samples_precomputed = s.smp_hits;
    st.scout_nn_hits = s.sc_nn;
    st.scout_near_hits = s.sc_near;
    st.scout_edge_hits = s.sc_edge_hit;
    st.scout_edge_misses = s.sc_edge_miss;
    st.scout_wait_seconds = (double)s.sc_wait / p->wall_rate_hz;
    for (int k = 0; k < 32; ++k) {
      const bool count = k == 8 || k == 11 || (k >= 20 && k < 28) || k == 30;
      st.scout_phase_seconds[k] = count ? (double)scout_prof[i][k] : (double)scout_prof[i][k] / p->wall_rate_hz;
    }
    st.helpers = nh;
    st.scout = ns;
    for (int k = 0; k < 32; ++k)
      st.phase_seconds[k] = (k == 8 || k == 11 || k >= 20) ? (double)s.prof[k] : (double)s.prof[k] / p->wall_rate_hz;
    if (i == 0) { p->last_n[0] = s.n[0]; p->last_n[1] = s.n[1]; }
    // cost rows
    r.n_cost_rows = s.n_rows;
    if (s.n_rows > 0) {
      r.cost_rows = (double*)malloc(sizeof(double) * 5 * s.n_rows);
      HIPCHK(hipMemcpy(r.cost_rows, p->qb[i].rows.p, sizeof(double) * 5 * s.n_rows, hipMemcpyDeviceToHost));
      for (int64_t k = 0; k < s.n_rows; ++k) r.cost_rows[k * 5 + 1] /= p->wall_rate_hz;
    }
    if (r.status != SMP_OK) { done[i] = 1; continue; }
    int ns = counts[2 * i], ng = counts[2 * i + 1];
    const int np = p->params.num_traj_segments;
    // the path's edges (e_start, e_target of every path node, start-tree nodes root first, then the goal-tree nodes
    // from the connection) gathered on the device: one copy instead of one per value
    std::vector<double> pe((size_t)(ns + ng) * 2 * NJ);
    if (ns + ng > 0) {
      HIPCHK(p->d_path_edges.reserve(pe.size()));
      const int nthr = (int)pe.size();
      hipLaunchKernelGGL(path_edges_kernel, dim3((nthr + 255) / 256), dim3(256), 0, p->stream, p->d_qdev.p, i, ns, ng,
                         p->d_path_edges.p);
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpyAsync(pe.data(), p->d_path_edges.p, pe.size() * sizeof(double), hipMemcpyDeviceToHost, p->stream));
      HIPCHK(hipStreamSynchronize(p->stream));
    }
    (void)cap;
    std::vector<double> wp;
    for (int k = 0; k < ns + ng; ++k) {
      // start-tree edges contribute points 0 .. np-1; goal-tree edges reversed: points np .. 1, then point 0 of the
      // last one (computeFinalSolutionPathTrajectories, birrt_star.cpp:6173-6274)
      const double* a = &pe[(size_t)k * 2 * NJ];
      const double* b = a + NJ;
      double stp[NJ];
      for (int j = 0; j < NJ; ++j) stp[j] = (b[j] - a[j]) / double(np);
      if (k < ns) {
        for (int inc = 0; inc < np; ++inc)
          for (int j = 0; j < NJ; ++j) wp.push_back(a[j] + inc * stp[j]);
      } else {
        for (int inc = np; inc > 0; --inc)
          for (int j = 0; j < NJ; ++j) wp.push_back(a[j] + inc * stp[j]);
        if (k == ns + ng - 1)
          for (int j = 0; j < NJ; ++j) wp.push_back(a[j] + 0 * stp[j]);
      }
    }
    r.n_waypoints = (int64_t)(wp.size() / NJ);
    if (!wp.empty()) {
      r.waypoints = (double*)malloc(sizeof(double) * wp.size());
      std::memcpy(r.waypoints, wp.data(), sizeof(double) * wp.size());
    }
    done[i] = 1;
  }
  for (int i = 0; i < nq; ++i) if (out[i].status != SMP_OK && rc == SMP_OK) rc = out[i].status;
  hstamp("results assembled");
  return rc;
}

extern "C" int smp_plan_batch(smp_planner* p, const smp_query* qs, int nq, smp_result* out) {
  if (!p || !qs || nq <= 0 || !out) return SMP_ERR_ARG;
  for (int i = 0; i < nq; ++i) std::memset(&out[i], 0, sizeof(smp_result));
  if (int b_ = busy_check(p)) {
    for (int i = 0; i < nq; ++i) out[i].status = b_;
    return b_;
  }
  std::vector<char> done(nq, 0);
  const int rc = plan_batch_impl(p, qs, nq, out, done);
  // the runtime's last-error slot still holds a failed call's error (e.g. an allocation): clear it, so the next
  // call's launch checks do not report it again
  if (rc == SMP_ERR_HIP) (void)hipGetLastError();
  // a call that stopped early leaves no result looking like a success
  for (int i = 0; i < nq; ++i) {
    if (done[i]) continue;
    smp_result_free(&out[i]);
    out[i].status = rc != SMP_OK ? rc : SMP_ERR_HIP;
  }
  return rc;
}

extern "C" int smp_plan(smp_planner* p, const smp_query* q, smp_result* out) { return smp_plan_batch(p, q, 1, out); }

// Queries dealt round-robin over the planners (query i -> planner i % np), one host thread per planner, so the
// planners' GPUs plan concurrently; out[i] is query i's result.  The return code is the first non-OK status in query
// order, as smp_plan_batch's.
extern "C" int smp_plan_multi(smp_planner* const* ps, int np, const smp_query* qs, int nq, smp_result* out) {
  if (!ps || np <= 0 || !qs || nq <= 0 || !out) return SMP_ERR_ARG;
  for (int i = 0; i < nq; ++i) std::memset(&out[i], 0, sizeof(smp_result));
  for (int k = 0; k < np; ++k)
    for (int j = 0; j <= k; ++j)
      if (!ps[k] || (j < k && ps[k] == ps[j])) {  // a planner is not thread-safe: each at most once
        for (int i = 0; i < nq; ++i) out[i].status = SMP_ERR_ARG;
        return SMP_ERR_ARG;
      }
  const int used = std::min(np, nq);
  std::vector<std::vector<smp_query>> part(used);
  std::vector<std::vector<smp_result>> res(used);
  for (int i = 0; i < nq; ++i) part[i % used].push_back(qs[i]);
  std::vector<int> rcs(used, SMP_OK);
  // planners on the same GPU run at once: each provisions its share of that GPU's co-resident workgroups (every
  // workgroup of a query polls the others, so all of them must be resident)
  for (int k = 0; k < used; ++k) {
    int same = 0;
    for (int j = 0; j < used; ++j) same += ps[j]->device == ps[k]->device;
    ps[k]->slot_share = same * ps[k]->proc_share;
  }
  std::vector<std::thread> th;
  th.reserve(used);
  for (int k = 0; k < used; ++k) {
    res[k].resize(part[k].size());
    th.emplace_back([&, k] { rcs[k] = smp_plan_batch(ps[k], part[k].data(), (int)part[k].size(), res[k].data()); });
  }
  for (auto& t : th) t.join();
  for (int k = 0; k < used; ++k) ps[k]->slot_share = ps[k]->proc_share;
  int rc = SMP_OK;
  for (int i = 0; i < nq; ++i) {
    out[i] = res[i % used][i / used];
    if (rc == SMP_OK && out[i].status != SMP_OK) rc = out[i].status;
  }
  for (int k = 0; k < used; ++k)
    if (rc == SMP_OK && rcs[k] != SMP_OK) rc = rcs[k];
  return rc;
}

extern "C" void smp_result_free(smp_result* r) {
  if (!r) return;
  free(r->waypoints);
  free(r->cost_rows);
  r->waypoints = nullptr;
  r->cost_rows = nullptr;
  r->n_waypoints = r->n_cost_rows = 0;
}

// The last query's state in the oracle's terms (test infrastructure, DESIGN.md "Large trees": the oracle continues
// the same run from it, orc_resume_*): per tree the child lists (first child, next sibling: the GPU inserts children
// at the head, so the reference's out-edge order is the list reversed) and every node's in-edge (interpolation start
// and target, n x 8 row-major); then the loop scalars (iv: iteration, checked, valid, first_iter, last_iter,
// have_sol, conn_start, tree_A of the next iteration, nB id / parent, nA id / parent, edges / rewires of both trees;
// dv: c_best[3], nB q[8] / cost[3], nA q[8] / cost[3]).
extern "C" int smp_probe_export_tree(smp_planner* p, int which, int32_t* first_child, int32_t* next_sib,
                                     double* e_start, double* e_target) {
  if (!p || p->qb.empty() || which < 0 || which > 1) return SMP_ERR_ARG;
  if (int b_ = busy_check(const_cast<smp_planner*>(p))) return b_;
  HIPCHK(hipSetDevice(p->device));
  QueryBuffers& b = p->qb[0];
  const size_t cap = b.cap;
  const int n = p->last_n[which];
  if (first_child) HIPCHK(hipMemcpy(first_child, b.first_child.p + which * cap, n * sizeof(int), hipMemcpyDeviceToHost));
  if (next_sib) HIPCHK(hipMemcpy(next_sib, b.next_sib.p + which * cap, n * sizeof(int), hipMemcpyDeviceToHost));
  std::vector<double> tmp((size_t)n);
  double* const outs[2] = {e_start, e_target};
  double* const srcs[2] = {b.e_start.p, b.e_target.p};
  for (int o = 0; o < 2; ++o) {
    if (!outs[o]) continue;
    for (int j = 0; j < NJ; ++j) {
      HIPCHK(hipMemcpy(tmp.data(), srcs[o] + which * cap * NJ + (size_t)j * cap, n * sizeof(double), hipMemcpyDeviceToHost));
      for (int i = 0; i < n; ++i) outs[o][(size_t)i * NJ + j] = tmp[i];
    }
  }
  return SMP_OK;
}

extern "C" int smp_probe_export_state(smp_planner* p, int64_t* iv, double* dv) {
  if (!p || p->qb.empty() || !iv || !dv) return SMP_ERR_ARG;
  if (int b_ = busy_check(const_cast<smp_planner*>(p))) return b_;
  HIPCHK(hipSetDevice(p->device));
  QState S;
  HIPCHK(hipMemcpy(&S, p->qb[0].st.p, sizeof(QState), hipMemcpyDeviceToHost));
  iv[0] = S.iter; iv[1] = S.checked; iv[2] = S.valid; iv[3] = S.first_iter; iv[4] = S.last_iter;
  iv[5] = S.have_sol; iv[6] = S.conn_start; iv[7] = S.A;
  iv[8] = S.nB.id; iv[9] = S.nB.parent; iv[10] = S.nA.id; iv[11] = S.nA.parent;
  iv[12] = S.edges[0]; iv[13] = S.edges[1]; iv[14] = S.rewires[0]; iv[15] = S.rewires[1];
  dv[0] = S.cbest[0]; dv[1] = S.cbest[1]; dv[2] = S.cbest[2];
  const NodeRef* nb[2] = {&S.nB, &S.nA};
  for (int k = 0; k < 2; ++k) {
    for (int j = 0; j < NJ; ++j) dv[3 + 11 * k + j] = nb[k]->q[j];
    for (int c = 0; c < 3; ++c) dv[11 + 11 * k + c] = nb[k]->c[c];
  }
  return SMP_OK;
}

extern "C" int64_t smp_get_tree(smp_planner* p, int which, int32_t* parent, double* conf, double* cost) {
  if (!p || p->qb.empty() || which < 0 || which > 1) return -1;
  if (hipSetDevice(p->device) != hipSuccess) return -1;
  QueryBuffers& b = p->qb[0];
  size_t cap = b.cap;
  int n = p->last_n[which];
  if (parent && hipMemcpy(parent, b.parent.p + (size_t)which * cap, n * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  std::vector<double> tmp((size_t)n);
  if (conf)
    for (int j = 0; j < NJ; ++j) {
      if (hipMemcpy(tmp.data(), b.q.p + (size_t)which * cap * NJ + (size_t)j * cap, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) return -1;
      for (int i = 0; i < n; ++i) conf[(size_t)i * NJ + j] = tmp[i];
    }
  if (cost)
    for (int k = 0; k < 3; ++k) {
      if (hipMemcpy(tmp.data(), b.cost.p + (size_t)which * cap * 3 + (size_t)k * cap, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) return -1;
      for (int i = 0; i < n; ++i) cost[(size_t)i * 3 + k] = tmp[i];
    }
  return n;
}

// ------------------------------------------------------------------------------------------ parity probes
// The per-primitive slab fields a planner would build for this robot and scene (n_prim x ny x nx), host only.
extern "C" int64_t smp_probe_scene_slabs(const smp_robot* r, const smp_scene* s, uint16_t* out, int64_t cap) {
  if (!r || !s) return SMP_ERR_ARG;
  std::vector<std::vector<uint16_t>> slabs;
  prim_slabs(r->h.dev, s->h, &slabs);
  int64_t n = 0;
  for (auto& v : slabs) {
    if (out && n + (int64_t)v.size() <= cap) std::memcpy(out + n, v.data(), v.size() * sizeof(uint16_t));
    n += (int64_t)v.size();
  }
  return n;
}

// The device model of a robot (tests: the URDF + SRDF path and the JSON path give the same bytes).  Host only.
extern "C" int64_t smp_probe_robot_dev(const smp_robot* r, void* out, int64_t cap) {
  if (!r) return SMP_ERR_ARG;
  if (out && cap >= (int64_t)sizeof(RobotDev)) std::memcpy(out, &r->h.dev, sizeof(RobotDev));
  return (int64_t)sizeof(RobotDev);
}

// Device evaluations of the shared arithmetic (tests only): portable sin/cos, the Philox draw, body FK,
// end-effector z and the fp64 sqrt / division used throughout.
extern "C" int smp_probe_sincos(int device, const double* x, int n, double* s, double* c) {
  if (hipSetDevice(device) != hipSuccess) return SMP_ERR_NO_DEVICE;
  double *dx, *ds, *dc;
  HIPCHK(hipMalloc(&dx, n * sizeof(double))); HIPCHK(hipMalloc(&ds, n * sizeof(double))); HIPCHK(hipMalloc(&dc, n * sizeof(double)));
  HIPCHK(hipMemcpy(dx, x, n * sizeof(double), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(sincos_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, dx, n, ds, dc);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(s, ds, n * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c, dc, n * sizeof(double), hipMemcpyDeviceToHost));
  (void)hipFree(dx); (void)hipFree(ds); (void)hipFree(dc);
  return SMP_OK;
}

extern "C" int smp_probe_u01(int device, uint64_t seed, uint32_t query, const uint32_t* ctr, int n, double* out) {
  if (hipSetDevice(device) != hipSuccess) return SMP_ERR_NO_DEVICE;
  uint32_t* dc;
  double* d;
  HIPCHK(hipMalloc(&dc, 4 * n * sizeof(uint32_t))); HIPCHK(hipMalloc(&d, n * sizeof(double)));
  HIPCHK(hipMemcpy(dc, ctr, 4 * n * sizeof(uint32_t), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(u01_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, (unsigned long long)seed, query, dc, n, d);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, d, n * sizeof(double), hipMemcpyDeviceToHost));
  (void)hipFree(dc); (void)hipFree(d);
  return SMP_OK;
}

extern "C" int smp_probe_fk(smp_planner* p, const double* q, int n, double* frames, double* eez) {
  if (!p) return SMP_ERR_ARG;
  if (int b_ = busy_check(const_cast<smp_planner*>(p))) return b_;
  HIPCHK(hipSetDevice(p->device));
  int nb = p->robot.dev.n_body;
  double *dq, *df, *dz;
  HIPCHK(hipMalloc(&dq, (size_t)n * NJ * sizeof(double)));
  HIPCHK(hipMalloc(&df, (size_t)n * nb * 12 * sizeof(double)));
  HIPCHK(hipMalloc(&dz, (size_t)n * sizeof(double)));
  HIPCHK(hipMemcpy(dq, q, (size_t)n * NJ * sizeof(double), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(fk_kernel, dim3((n + 127) / 128), dim3(128), 0, 0, p->d_rb, dq, n, df, dz);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(frames, df, (size_t)n * nb * 12 * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(eez, dz, (size_t)n * sizeof(double), hipMemcpyDeviceToHost));
  (void)hipFree(dq); (void)hipFree(df); (void)hipFree(dz);
  return SMP_OK;
}

// Latency probe of the collision tile: check_kernel with `grid` workgroups (grid 1: one workgroup streams
// every tile back to back); ticks[0..3] = block 0's device-clock ticks in tile stages A, B, C-centres, C;
// ticks[4] / ticks[5] = block 0's shader cycles / device-clock ticks over the kernel (effective shader clock);
// ticks[6..8] = wave 0's detail clocks (collide_tile: centres + map sweeps, self test; collide_wide (tile < 0):
// primitive sweeps, sphere sweeps, self test).  `ticks` holds 12 entries.
extern "C" int smp_probe_check_latency(smp_planner* p, const double* q_soa, int64_t n, int check_self, int check_map,
                                       int grid, int tile, double* ms, unsigned long long* ticks, double* clock_hz) {
  if (!p || n <= 0 || !q_soa || grid <= 0) return SMP_ERR_ARG;
  if (int b_ = busy_check(const_cast<smp_planner*>(p))) return b_;
  HIPCHK(hipSetDevice(p->device));
  HIPCHK(p->d_cq.reserve((size_t)n * NJ));
  HIPCHK(p->d_valid.reserve((size_t)n));
  unsigned long long* dprof = nullptr;
  HIPCHK(hipMalloc(&dprof, 16 * sizeof(unsigned long long)));
  HIPCHK(hipMemset(dprof, 0, 16 * sizeof(unsigned long long)));
  HIPCHK(hipMemcpy(p->d_cq.p, q_soa, (size_t)n * NJ * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipEventRecord(p->ev0, p->stream));
  launch_check(tile, grid, p->stream, p->d_rb, p->sc, p->d_mc, p->d_cq.p, (long long)n, check_self,
               check_map && p->have_scene, p->d_valid.p, dprof);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(p->ev1, p->stream));
  HIPCHK(hipStreamSynchronize(p->stream));
  float f = 0;
  HIPCHK(hipEventElapsedTime(&f, p->ev0, p->ev1));
  *ms = f;
  HIPCHK(hipMemcpy(ticks, dprof, 12 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  (void)hipFree(dprof);
  *clock_hz = p->wall_rate_hz;
  return SMP_OK;
}

// Validity flags of n configurations checked in tiles of the given shape (launch_check: 8 / 16 / 32 = the batch
// checker's collide_tile, -1 / -2 / -4 / -8 = the job tiles' collide_wide with that many configurations): the parity
// test of the job-tile shapes against the batch checker (tests/test_gpu_parity.py).
extern "C" int smp_probe_check_shape(smp_planner* p, const double* q_soa, int64_t n, int check_self, int check_map,
                                     int tile, int grid, uint8_t* valid) {
  if (!p || n <= 0 || !q_soa || !valid || grid <= 0) return SMP_ERR_ARG;
  if (int b_ = busy_check(const_cast<smp_planner*>(p))) return b_;
  if (!(tile == 8 || tile == 16 || tile == 32 || tile == -1 || tile == -2 || tile == -4 || tile == -8)) return SMP_ERR_ARG;
  HIPCHK(hipSetDevice(p->device));
  HIPCHK(p->d_cq.reserve((size_t)n * NJ));
  HIPCHK(p->d_valid.reserve((size_t)n));
  HIPCHK(hipMemcpyAsync(p->d_cq.p, q_soa, (size_t)n * NJ * sizeof(double), hipMemcpyHostToDevice, p->stream));
  launch_check(tile, grid, p->stream, p->d_rb, p->sc, p->d_mc, p->d_cq.p, (long long)n, check_self,
               check_map && p->have_scene, p->d_valid.p, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(valid, p->d_valid.p, (size_t)n, hipMemcpyDeviceToHost, p->stream));
  HIPCHK(hipStreamSynchronize(p->stream));
  return SMP_OK;
}

extern "C" int smp_probe_sqrt_div(int device, const double* a, const double* b, int n, double* sq, double* dv) {
  if (hipSetDevice(device) != hipSuccess) return SMP_ERR_NO_DEVICE;
  double *da, *db, *ds, *dd;
  HIPCHK(hipMalloc(&da, n * sizeof(double))); HIPCHK(hipMalloc(&db, n * sizeof(double)));
  HIPCHK(hipMalloc(&ds, n * sizeof(double))); HIPCHK(hipMalloc(&dd, n * sizeof(double)));
  HIPCHK(hipMemcpy(da, a, n * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(db, b, n * sizeof(double), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(sqrt_div_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, da, db, n, ds, dd);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(sq, ds, n * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(dv, dd, n * sizeof(double), hipMemcpyDeviceToHost));
  (void)hipFree(da); (void)hipFree(db); (void)hipFree(ds); (void)hipFree(dd);
  return SMP_OK;
}

// Tree-scan probe (near_probe_kernel): nearest and near_set<20> of m queries against one tree of n nodes
// (q_soa [NJ][n], cost [n]); lo / hi: m x 20 ids (-1 padded); ticks[2]: device-clock ticks of all nearest /
// near_set calls (clock_hz ticks per second); ticks[2..13]: the workgroup's profiling slots 20..31 (SMP_NEAR_PROF
// builds: near_set step clocks and path counts).
extern "C" int smp_probe_near(int device, const double* q_soa, const double* cost, int n, const double* queries,
                              const int* excl, int m, double r, int reps, int* nn, int* nk, int* lo, int* hi,
                              unsigned long long* ticks, double* clock_hz) {
  // reps < 0: the distributed scans' slice functions over the whole tree (tools/slice_probe.py)
  if (n <= 0 || m <= 0 || reps == 0 || !q_soa || !cost || !queries || !excl) return SMP_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return SMP_ERR_NO_DEVICE;
  double *dq, *dc, *dqq;
  int *dx, *dnn, *dnk, *dlo, *dhi;
  unsigned long long* dt;
  HIPCHK(hipMalloc(&dq, (size_t)n * NJ * sizeof(double)));
  HIPCHK(hipMalloc(&dc, (size_t)n * sizeof(double)));
  HIPCHK(hipMalloc(&dqq, (size_t)m * NJ * sizeof(double)));
  HIPCHK(hipMalloc(&dx, (size_t)m * sizeof(int)));
  HIPCHK(hipMalloc(&dnn, (size_t)m * sizeof(int)));
  HIPCHK(hipMalloc(&dnk, (size_t)m * sizeof(int)));
  HIPCHK(hipMalloc(&dlo, (size_t)m * 20 * sizeof(int)));
  HIPCHK(hipMalloc(&dhi, (size_t)m * 20 * sizeof(int)));
  HIPCHK(hipMalloc(&dt, 14 * sizeof(unsigned long long)));
  HIPCHK(hipMemcpy(dq, q_soa, (size_t)n * NJ * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dc, cost, (size_t)n * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dqq, queries, (size_t)m * NJ * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dx, excl, (size_t)m * sizeof(int), hipMemcpyHostToDevice));
  // the tree's fp32 copy (TreeDev::qf: the planner writes it with every node)
  std::vector<float> qf((size_t)n * NJ);
  for (size_t k = 0; k < qf.size(); ++k) qf[k] = (float)q_soa[k];
  float* dqf;
  HIPCHK(hipMalloc(&dqf, qf.size() * sizeof(float)));
  HIPCHK(hipMemcpy(dqf, qf.data(), qf.size() * sizeof(float), hipMemcpyHostToDevice));
  // modes 4 / 5 (the helpers' inlined slice forms) run in a kernel of their own, so that neither kernel's register
  // allocation carries the other's code
  const bool inl = reps < 0 && 1 + ((-reps) >> 20) >= 4;
  hipLaunchKernelGGL(inl ? near_probe_inl_kernel : near_probe_kernel, dim3(1), dim3(BLOCK), 0, 0, dq, dc, n, n, dqq, dx,
                     m, r, reps, dnn, dnk, dlo, dhi, dt, (const float*)dqf);
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(nn, dnn, (size_t)m * sizeof(int), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(nk, dnk, (size_t)m * sizeof(int), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(lo, dlo, (size_t)m * 20 * sizeof(int), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(hi, dhi, (size_t)m * 20 * sizeof(int), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(ticks, dt, 14 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  (void)hipFree(dq); (void)hipFree(dc); (void)hipFree(dqq); (void)hipFree(dx); (void)hipFree(dnn);
  (void)hipFree(dnk); (void)hipFree(dlo); (void)hipFree(dhi); (void)hipFree(dt); (void)hipFree(dqf);
  int dev_clock_khz = 0;
  HIPCHK(hipDeviceGetAttribute(&dev_clock_khz, hipDeviceAttributeWallClockRate, device));
  *clock_hz = dev_clock_khz * 1000.0;
  return SMP_OK;
}
