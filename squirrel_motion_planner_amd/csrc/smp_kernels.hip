// HIP kernels for gfx950: batched configuration validity and the device-resident BiRRT* planner.
//
// Design: one 256-thread workgroup owns one planning query for its whole run_planner loop
// (birrt_star.cpp:983-1407).  The sequential decisions of the reference are taken by one lane and broadcast
// through LDS; the data-parallel parts run on the whole workgroup:
//   * nearest-neighbour argmin and radius-near selection over SoA node arrays (birrt_star.cpp:4076-4133,
//     4272-4324) -- coalesced fp64 streams, wave shuffles + LDS reduction, lowest-index tie break;
//   * edge validity (isEdgeValid, birrt_star.cpp:6864-6895) as 32-configuration collision tiles in LDS;
//   * candidate edges of choose-parent / rewire / connect evaluated speculatively in one batch and then
//     committed in the reference's sequential order, so trees are identical to the sequential planner.
// Several queries (C3/C5) run as several workgroups of one launch; each launch advances every query by a
// bounded number of iterations and persists the state (QState) in HBM.
#include <hip/hip_runtime.h>

#include <vector>

#include "smp_collide.h"
#include "smp_math.h"
#include "smp_plan.h"
#include "smp_types.h"

// Wave reductions of the device library (ockl, DPP-based); hip's header declares the 64-bit ones only under
// HIP_ENABLE_EXTRA_WARP_SYNC_TYPES.
extern "C" __device__ __attribute__((const)) unsigned long long __ockl_wfred_min_u64(unsigned long long);
extern "C" __device__ __attribute__((const)) unsigned long long __ockl_wfred_max_u64(unsigned long long);

namespace smp {

// ============================================================================================ batch check
// valid[i] = !isInCollision(q_i) for n configurations given as SoA q[j*n + i].
constexpr int CHECK_CT = 32;

// Robot model and map configuration staged in LDS by every kernel that runs collision tiles.
__shared__ RobotDev g_rb;
__shared__ MapCfg g_mc;

// Copies the robot model and the map configuration into LDS (read by every collision stage).
__device__ __forceinline__ void stage_model(const RobotDev* rb, const MapCfg* mc, RobotDev* rbl, MapCfg* mcl) {
  static_assert(sizeof(RobotDev) % 8 == 0 && sizeof(MapCfg) % 4 == 0, "staging granularity");
  for (int i = threadIdx.x; i < (int)(sizeof(RobotDev) / 8); i += BLOCK)
    reinterpret_cast<uint64_t*>(rbl)[i] = reinterpret_cast<const uint64_t*>(rb)[i];
  for (int i = threadIdx.x; i < (int)(sizeof(MapCfg) / 4); i += BLOCK)
    reinterpret_cast<uint32_t*>(mcl)[i] = reinterpret_cast<const uint32_t*>(mc)[i];
  __syncthreads();
}

template <int CT>
__global__ void __launch_bounds__(BLOCK) check_kernel_t(const RobotDev* __restrict__ rb, SceneDev sc,
                                                        const MapCfg* __restrict__ mc, const double* __restrict__ q,
                                                        long long n, int self, int map, uint8_t* __restrict__ valid,
                                                        unsigned long long* prof) {
  __shared__ TileLds<CT> L;
  __shared__ double ql[CT][NJ];
  unsigned long long* pr = blockIdx.x == 0 ? prof : nullptr;  // stage clocks of block 0 (latency probe)
  unsigned long long c0 = 0, w0 = 0;
  if (pr && threadIdx.x == 0) { c0 = __builtin_amdgcn_s_memtime(); w0 = wall_clock64(); }
  stage_model(rb, mc, &g_rb, &g_mc);
  const long long ntiles = (n + CT - 1) / CT;
  for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    long long base = t * CT;
    int nc = (int)min((long long)CT, n - base);
    for (int it = threadIdx.x; it < nc * NJ; it += BLOCK) {
      int c = it / NJ, j = it - c * NJ;
      ql[c][j] = q[(long long)j * n + base + c];
    }
    __syncthreads();
    collide_tile<CT>(&g_rb, sc, &g_mc, nc, ql, self, map, L, nullptr, pr, pr ? pr + 6 : nullptr);
    if (threadIdx.x < nc) valid[base + threadIdx.x] = L.coll[threadIdx.x] ? 0 : 1;
    __syncthreads();
  }
  if (pr && threadIdx.x == 0) { pr[4] = __builtin_amdgcn_s_memtime() - c0; pr[5] = wall_clock64() - w0; }
}

// The job tiles' shape (collide_wide, ct configurations spread over the workgroup) as a batch check: grid-stride over
// tiles of ct configurations.  Latency / rate probe of the helpers' tiles (smp_probe_check_latency, tile = -ct).
__global__ void __launch_bounds__(BLOCK) check_wide_kernel(const RobotDev* __restrict__ rb, SceneDev sc,
                                                           const MapCfg* __restrict__ mc, const double* __restrict__ q,
                                                           long long n, int ct, int self, int map,
                                                           uint8_t* __restrict__ valid, unsigned long long* prof) {
  __shared__ WideLds L;
  __shared__ double ql[TILE_CT_MAX][NJ];
  unsigned long long* pr = blockIdx.x == 0 ? prof : nullptr;
  unsigned long long c0 = 0, w0 = 0;
  if (pr && threadIdx.x == 0) { c0 = __builtin_amdgcn_s_memtime(); w0 = wall_clock64(); }
  stage_model(rb, mc, &g_rb, &g_mc);
  const long long ntiles = (n + ct - 1) / ct;
  for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const long long base = t * ct;
    const int nc = (int)min((long long)ct, n - base);
    if (threadIdx.x < nc * NJ) {
      const int c = threadIdx.x / NJ, j = threadIdx.x - c * NJ;
      ql[c][j] = q[(long long)j * n + base + c];
    }
    if (threadIdx.x < TILE_CT_MAX) L.coll[threadIdx.x] = 0;
    __syncthreads();
    collide_wide(&g_rb, sc, &g_mc, ct, nc, ql, self, map, L, nullptr, pr, pr ? pr + 6 : nullptr);
    if (threadIdx.x < nc) valid[base + threadIdx.x] = L.coll[threadIdx.x] ? 0 : 1;
    __syncthreads();
  }
  if (pr && threadIdx.x == 0) { pr[4] = __builtin_amdgcn_s_memtime() - c0; pr[5] = wall_clock64() - w0; }
}

// Batched isConfigValid (birrt_star.cpp:6897-6908): grid-stride over tiles of CT configurations.
// Largest per-work-item private segment (scratch) of the batch check kernels (smp_planner_create raises the
// device stack limit to cover every kernel of the library).
size_t check_kernels_private_bytes() {
  size_t need = 0;
  hipFuncAttributes fa;
  const void* ks[] = {reinterpret_cast<const void*>(&check_kernel_t<8>), reinterpret_cast<const void*>(&check_kernel_t<16>),
                      reinterpret_cast<const void*>(&check_kernel_t<CHECK_CT>),
                      reinterpret_cast<const void*>(&check_wide_kernel)};
  for (const void* k : ks)
    if (hipFuncGetAttributes(&fa, k) == hipSuccess && (size_t)fa.localSizeBytes > need) need = fa.localSizeBytes;
  return need;
}

void launch_check(int ct, int grid, hipStream_t st, const RobotDev* rb, SceneDev sc, const MapCfg* mc, const double* q,
                  long long n, int self, int map, uint8_t* valid, unsigned long long* prof) {
  if (ct == -1 || ct == -2 || ct == -4 || ct == -8) {  // job-tile shape (collide_wide)
    hipLaunchKernelGGL(check_wide_kernel, dim3(grid), dim3(BLOCK), 0, st, rb, sc, mc, q, n, -ct, self, map, valid, prof);
    return;
  }
  switch (ct) {
    case 8: hipLaunchKernelGGL(check_kernel_t<8>, dim3(grid), dim3(BLOCK), 0, st, rb, sc, mc, q, n, self, map, valid, prof); break;
    case 16: hipLaunchKernelGGL(check_kernel_t<16>, dim3(grid), dim3(BLOCK), 0, st, rb, sc, mc, q, n, self, map, valid, prof); break;
    default: hipLaunchKernelGGL(check_kernel_t<CHECK_CT>, dim3(grid), dim3(BLOCK), 0, st, rb, sc, mc, q, n, self, map, valid, prof); break;
  }
}

// ============================================================================================ collision listing
// getCollisions (birrt_star.cpp:6910-6914 -> collision_checker.hpp:123-132): for one configuration, which collision
// links touch the map (getMapCollisions, CC:610-630: every link with geometry, the disabled ones included) and which
// self pairs overlap (getSelfCollisions, CC:594-608: every pair, no early exit).  One wavefront; the map test of a
// sphere is the planner's (box-gap prefilter, then the exact sweep), the self test the planner's sphere-pair test.
__global__ void __launch_bounds__(64) collisions_kernel(const RobotDev* __restrict__ rb, SceneDev sc,
                                                        const MapCfg* __restrict__ mc, const double* __restrict__ q,
                                                        int map, uint8_t* __restrict__ link_map,
                                                        uint8_t* __restrict__ pair_self) {
  __shared__ Frame B[MAX_BODY];
  __shared__ double wc[MAX_SPH][3];
  __shared__ uint32_t cand[(MAX_SPH + 31) / 32];
  __shared__ int lm[MAX_CLINK];
  __shared__ double pwl[MAX_PRIM][5];
  const int lane = threadIdx.x;
  if (lane == 0) {
    double qq[NJ];
    for (int j = 0; j < NJ; ++j) qq[j] = q[j];
    Frame F[MAX_BODY];
    body_frames(rb, qq, F);
    for (int b = 0; b < rb->n_body; ++b) B[b] = F[b];
  }
  if (lane < (MAX_SPH + 31) / 32) cand[lane] = 0u;
  if (lane < MAX_CLINK) lm[lane] = 0;
  __syncthreads();
  const int nsph = rb->n_sph;
  for (int s = lane; s < nsph; s += 64) {
    double w[3];
    xform(B[rb->sph_body[s]], &rb->sph_cb[s * 3], w);
    wc[s][0] = w[0]; wc[s][1] = w[1]; wc[s][2] = w[2];
    if (map) {
      const long long cell = centre_cell(sc, w);
      const uint32_t dv = cell < 0 ? 0xffffffffu : (sc.d2b ? (uint32_t)sc.d2b[cell] : (uint32_t)sc.d2[cell]);
      if (dv <= mc->T[s]) atomicOr(&cand[s >> 5], 1u << (s & 31));
    }
  }
  for (int p = lane; p < rb->n_prim; p += 64) prim_world(rb, p, &B[rb->prim_body[p]].R[0], pwl[p]);
  __syncthreads();
  // primitives: exact sweep of every one whose slab prefilter does not clear it (disabled links included)
  if (map)
    for (int p = 0; p < rb->n_prim; ++p) {
      const double pw[5] = {pwl[p][0], pwl[p][1], pwl[p][2], pwl[p][3], pwl[p][4]};
      if (!prim_candidate(sc, sc.slab[p], mc->pT[p], pw)) continue;
      const bool hit = wave_prim_map(sc, rb->prim_type[p], &rb->prim_h[p * 3], pw, lane);
      if (hit && lane == 0) lm[rb->prim_clink[p]] = 1;
    }
  __syncthreads();
  for (int wd = 0; wd < (nsph + 31) / 32; ++wd) {
    uint32_t m = cand[wd];
    while (m) {
      const int s = wd * 32 + __builtin_ctz(m);
      m &= m - 1;
      const int c = rb->sph_clink[s];
      if (lm[c]) continue;  // the link is listed already
      const bool hit = wave_sphere_map(sc, wc[s], rb->sph_r[s], lane);
      __syncthreads();
      if (hit && lane == 0) lm[c] = 1;
      __syncthreads();
    }
  }
  for (int c = lane; c < rb->n_clink; c += 64) link_map[c] = (uint8_t)lm[c];
  for (int p = lane; p < rb->n_pairs; p += 64) {
    const int a = rb->pair_a[p], b = rb->pair_b[p];
    bool hit = false;
    if (rb->cl_prim[a] >= 0 || rb->cl_prim[b] >= 0) {
      const int pr = rb->cl_prim[a] >= 0 ? rb->cl_prim[a] : rb->cl_prim[b], sl = rb->cl_prim[a] >= 0 ? b : a;
      for (int s = rb->cl_sph0[sl]; s < rb->cl_sph0[sl] + rb->cl_nsph[sl] && !hit; ++s)
        hit = sphere_prim(rb->prim_type[pr], &rb->prim_h[pr * 3], pwl[pr], wc[s], rb->sph_r[s]);
      pair_self[p] = hit ? 1 : 0;
      continue;
    }
    for (int sa = rb->cl_sph0[a]; sa < rb->cl_sph0[a] + rb->cl_nsph[a] && !hit; ++sa)
      for (int sb = rb->cl_sph0[b]; sb < rb->cl_sph0[b] + rb->cl_nsph[b]; ++sb) {
        const double rs = rb->sph_r[sa] + rb->sph_r[sb];
        const double ex = wc[sa][0] - wc[sb][0], ey = wc[sa][1] - wc[sb][1], ez = wc[sa][2] - wc[sb][2];
        if (ex * ex + ey * ey + ez * ez <= rs * rs) { hit = true; break; }
      }
    pair_self[p] = hit ? 1 : 0;
  }
}

void launch_collisions(hipStream_t st, const RobotDev* rb, SceneDev sc, const MapCfg* mc, const double* q, int map,
                       uint8_t* link_map, uint8_t* pair_self) {
  hipLaunchKernelGGL(collisions_kernel, dim3(1), dim3(64), 0, st, rb, sc, mc, q, map, link_map, pair_self);
}

// ============================================================================================ parity kernels
__global__ void sincos_kernel(const double* x, int n, double* s, double* c) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) psincos(x[i], s + i, c + i);
}

__global__ void u01_kernel(unsigned long long seed, unsigned query, const uint32_t* ctr, int n, double* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = u01(seed, query, ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]);
}

// body frames (n x n_body x 12) and end-effector z of n configurations (row-major q).
__global__ void __launch_bounds__(128) fk_kernel(const RobotDev* __restrict__ rb, const double* q, int n, double* frames, double* eez) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double qq[NJ];
  for (int j = 0; j < NJ; ++j) qq[j] = q[i * NJ + j];
  Frame B[MAX_BODY];
  body_frames(rb, qq, B);
  for (int b = 0; b < rb->n_body; ++b) {
    for (int k = 0; k < 9; ++k) frames[((size_t)i * rb->n_body + b) * 12 + k] = B[b].R[k];
    for (int k = 0; k < 3; ++k) frames[((size_t)i * rb->n_body + b) * 12 + 9 + k] = B[b].p[k];
  }
  eez[i] = ee_z(rb, qq);
}

__global__ void sqrt_div_kernel(const double* a, const double* b, int n, double* sq, double* dv) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { sq[i] = sqrt(a[i]); dv[i] = a[i] / b[i]; }
}

// ============================================================================================ planner
// Distributed scans of large trees (DESIGN.md "Scans of large trees").  ScanLds: one workgroup's slice (the per-wave
// lists of the near scan, the slice's merged lists, the nearest reduction); MergeLds: every participant's partial
// result as the leader collects and merges them.
constexpr int SCAN_K = 20;  // near-list ends a scan keeps (near_set<20>; max_near_nodes <= 20)
constexpr int NEAR_BINS = 256;   // near_set register path: cost histogram bins
constexpr int NEAR_BUF = 128;    // near_set register path: candidate buffer entries per end
#ifndef SMP_NEAR_NBK
#define SMP_NEAR_NBK 16
#endif
constexpr int NEAR_NBK = SMP_NEAR_NBK;  // near_set register path: 64-node batches per wave held in registers
struct ScanLds {
  union {
    struct {  // slice_near_body (per-wave sorted lists)
      unsigned long long wlk[BLOCK / 64][SCAN_K], whk[BLOCK / 64][SCAN_K];
      int wli[BLOCK / 64][SCAN_K], whi[BLOCK / 64][SCAN_K];
    };
    struct {  // slice_near_hist (near_set's register path): cost histogram and the two candidate buffers
      alignas(16) unsigned hist[NEAR_BINS];
      unsigned long long ck[2][NEAR_BUF];
      int ci[2][NEAR_BUF];
    };
  };
  unsigned long long hmin[BLOCK / 64], hmax[BLOCK / 64];
  int hcnt[2], hblo, hbhi, fast;
  int wtot[BLOCK / 64];
  unsigned long long blo, bhi;                       // near_batch's block bounds
  unsigned long long lk[SCAN_K], hk[SCAN_K];        // the slice's lowest (ascending) / highest (descending) entries
  int li[SCAN_K], hi[SCAN_K];
  int cnt, take;
  unsigned long long wk[BLOCK / 64];
  int wi[BLOCK / 64];
};
constexpr int MERGE_LS = SCAN_K | 1;  // words per participant list in MergeLds (odd: conflict-free lane-per-list reads)
struct MergeLds {
  // [0] lows ascending, [1] highs descending, per participant: key halves and ids.  A list takes MERGE_LS (odd) words:
  // the tournament's lane w reads list w, and an odd stride puts the 32 lists' heads in 32 different LDS banks (a
  // stride of 40 words -- the key halves interleaved -- put every 8th list in one bank: 16-way conflicts per read)
  unsigned kl[2][SCAN_PNEAR][MERGE_LS], kh[2][SCAN_PNEAR][MERGE_LS];
  int id[2][SCAN_PNEAR][MERGE_LS];
  int len[SCAN_P], cnt[SCAN_P], done[SCAN_P], bad[SCAN_P];
  unsigned hv[SCAN_P][3];             // collection: near header (count, take) / nearest (key halves, id)
  unsigned hn[SCAN_PNEAR][3];         // collection: a fused scan's nearest (key halves, id)
  unsigned long long nk[SCAN_P];      // nearest: per participant (distance key, id)
  int ni[SCAN_P];
  int ndone, go[2], steal;
};
__device__ __forceinline__ unsigned long long merge_key(const MergeLds& M, int s, int w, int e) {
  return (unsigned long long)M.kh[s][w][e] << 32 | M.kl[s][w][e];
}
// LDS of job mode (leader and helper kernel): the published job + one job tile.
struct JobLds {
#ifdef SMP_NO_SCAN_UNION
  ScanLds scan;
  WideLds T;
#else
  union {
    ScanLds scan;                          // helper: its slice of a scan job
    WideLds T;                             // one job tile (collide_wide)
  };
#endif
  double tq[TILE_CT_MAX][NJ];
  double start[MAXE][NJ], step[MAXE][NJ];  // the job's edges (needed edges of the batch, compacted)
  unsigned words[JOB_WORDS];               // helper: the payload words as received
  uint8_t rmask[JOB_TILES];                // leader: collision mask per tile
  uint8_t rdone[JOB_TILES];                // leader: tile result known
  int emap[MAXE];                          // leader: job edge -> batch edge
  int first[MAXE];                         // leader: first colliding point per job edge
  int E, np1, nslots, ntiles, ct, self, map, seq, steal, hidx, left;  // ct: configurations per tile
  int skip, sfv, tskip;                    // job in skip mode / stop-first-valid; tile wholly skipped
  int tgrp[TILE_CT_MAX], tord[TILE_CT_MAX];  // skip mode: the tile's TileOrder (edge, point or "skip")
  unsigned long long tprof[4];             // SMP_JOB_PROF builds: this helper's tile stage clocks
  int go[2];  // poll-loop decisions, double-buffered by iteration parity (a slow wave may still read the last one)
};
// Sampling scratch (sample_ellipse: first valid inner getRandomConf draw of each outer attempt).
struct SmpLds {
  double q[64][NJ];
  int ok[64];
  int win;
};
// LDS of the run-ahead sampler workgroup.
struct SamplerLds {
  QState S;        // the query's constants, with have_sol / cbest of the version being served
  SmpLds W;
  double out[NJ];
  long long next;  // next iteration to sample
  int ver, go[2];
};
#ifndef SMP_PLAN_CT
#define SMP_PLAN_CT 8  // (the local path of a query without helpers, and init_planner's start / goal check)
#endif
constexpr int PLAN_CT = SMP_PLAN_CT;  // configurations per collision tile of the planner
constexpr int PATCH_K = 32;           // leader: recently appended nodes kept in LDS per tree (power of two)
struct PlanLds {
  QState S;
  union {
    struct {
      TileLds<PLAN_CT> T;
      double tq[PLAN_CT][NJ];
    } tile;
    JobLds job;  // job mode: the leader's LDS copy of its published job + one job tile
    double seg[MAXE][MAX_PTS][3];
    SmpLds smp;
    SamplerLds smpl;  // a helper block of plan_kernel that runs the run-ahead sampler
  } u;
  // scan scratch (outside the union u: a scan may run while a collision job holds u.job, overlap_work): a local near set's
  // lists, or a distributed scan's own slice and merge area -- a scan is one or the other
  union {
    struct {
      struct {  // near_set: per-wave sorted low / high ends of the near list
        unsigned long long wlk[BLOCK / 64][MAX_NEAR], whk[BLOCK / 64][MAX_NEAR];
        int wli[BLOCK / 64][MAX_NEAR], whi[BLOCK / 64][MAX_NEAR];
        int wtot[BLOCK / 64];
      } nr;
      struct {  // near_set, register path: cost histogram and the two candidate buffers
        alignas(16) unsigned hist[NEAR_BINS];
        unsigned long long ck[2][NEAR_BUF];
        int ci[2][NEAR_BUF];
        unsigned long long wmin[BLOCK / 64], wmax[BLOCK / 64];
        int wtot[BLOCK / 64];
        int cnt[2], blo, bhi, fast;
      } nh;
    };
    struct {  // a distributed scan (scan_run)
      ScanLds s;
      MergeLds m;
    } sc;
  };
  // edge batch
  double eg_start[MAXE][NJ], eg_target[MAXE][NJ], eg_step[MAXE][NJ], eg_end[MAXE][NJ];
  double eg_base[MAXE][3], eg_cost[MAXE][3];
  double eg_acc[MAXE][3];             // edge_costs: the segment-norm sums (eg_cost = eg_base + eg_acc)
  int eg_first[MAXE], eg_need[MAXE], eg_near[MAXE], eg_ptr[MAXE];
  int rw_par[MAXE], rw_next;          // rewire: candidates' parents (refreshed after every commit), resume point
  double rw_cost[MAXE][3];            // rewire: candidates' costs
  int tile_e[PLAN_CT], tile_i[PLAN_CT], tile_n;
  int count_slot;  // profiling: phase the checked configurations are attributed to
  int job_seq;     // last job published by this leader (this launch)
  int in_job;      // a collision job is in flight (its helpers are busy): scans stay local
  int go_end;      // the launch's finished-query quota is reached
  int smp_ver, smp_have_sol, smp_hit;  // run-ahead sampler: published parameter version / snapshot, slot hit
  int smp_pub;                         // the version changed this iteration: publish the parameters
  int spec, spec_nn;                   // overlap_work: what was computed during the last collision job, its result
  long long spec_cnt;                  // ... and the nodes it scanned (counted only if the result is used)
  double smp_cbest[3];
  // near lists (ascending (cost,id) for the first max_near; last max_near in ascending order)
  int nk;
  unsigned long long near_blo, near_bhi;  // near_set: block-wide bounds on the K-th smallest / largest key
  int lo_i[MAX_NEAR], hi_i[MAX_NEAR];
  double lo_c[MAX_NEAR], hi_c[MAX_NEAR];
  int n_lo, n_hi;
  // working nodes
  NodeRef nn, xn, xc, cur, g;
  double xr[NJ], ext[NJ], ox[NJ];
  double en_start[NJ], en_target[NJ];
  int ext_nn, ext_bp, flag, found, nn_id, cnt;
  int reached;
  // via list (connectGraphs / choose_parent): count, tree-local next id
  int n_via, nn_t, tree_expand;
  NodeRef sel;
  double sel_start[NJ], sel_target[NJ];
  double csp[3], best_nv;
  double sol[3];
  // wave reductions
  double wd[BLOCK / 64];
  unsigned long long wk[BLOCK / 64];
  int wi[BLOCK / 64];
  long long wcount[BLOCK / 64];
  // scout (DESIGN.md "Scout").  Leader: the scout's record of this iteration as far as received (sp_stage), sp_on =
  // still worth asking; eg_hit[e] = first colliding point of batch edge e taken from the record, -2 = none.
  // Scout: the record it builds.
  ScoutRec sr;
  PreRec prer;                  // pre-solution record: the leader's copy (pre_read) / the scout's, being written
  int prer_ok;                  // leader: prer holds this iteration's complete record
#ifdef SMP_TRACE
  int trole;                    // SMP_TRACE builds: 0 leader, 1 / 2 scout (trace records of this workgroup)
  unsigned tn;                  // records of this role so far
  long long tit;                // iteration the records belong to
#endif
  int sp_on, sp_stage, sp_go[2];
  double fnn_d;                 // near_set<K, true>: the nearest node of the same configuration (distance, id)
  int fnn_id;
#ifdef SMP_SCAN_PROF
  unsigned long long spc_t;     // SMP_SCAN_PROF: end of the last scan's collection
#endif
  int sc_same[MAX_SCOUTS];      // leader: scout s runs on this XCD (1), another (0), not yet known (-1)
  unsigned sc_seen, sc_dead;    // leader: scouts that delivered a pre-solution record / that never did and timed out
  int asked[SCOUT_SLOTS];       // leader: scout s + 1 asked for iteration k in slot k % SCOUT_SLOTS, 0 = none
  int asked_conn[SCOUT_SLOTS];  // leader: that record will carry connect's scans (stage SC_CONN)
  int asked_pre[SCOUT_SLOTS];   // leader: asked before the first solution (a pre-solution record)
  int conn_rec;                 // leader: connect of this iteration takes its scans from the record (g_L.sr.cc)
  int two_scouts;               // scout: two scouts share the iterations (post-solution records get SC_CONN)
  unsigned sc_mod;              // scout: rewire commits of its pass's tree when the pass read it (stage granules carry it)
  unsigned rw_at0;              // leader: rewire commits of tree_A at the start of the iteration (records must match)
  int n_at0;                    // leader: nodes of tree_A at the start of the iteration (early asks' snapshot)
  int sc_t, sc_rerun;           // scout: the pass's tree; 1 = the tree was rewired under the pass (rebuild it)
  int rb_go[2];                 // scout: decision words of the rebuild wait (double-buffered like sp_go)
  long long sc_k;               // scout: the pass's iteration
  int eg_hit[MAXE];
  int eg_rec[MAXE];             // leader: record edge (index into sr.e) equal to batch edge e, -1 = none
  int rec_grp;                  // leader: the record stage eg_rec was matched against (-1 = not matched)
  int rec_all, ev_job;          // rec_match: every edge matched; edge_validity: a job is needed
  // leader: configurations of the last PATCH_K nodes appended to each tree, by node index mod PATCH_K (kept by
  // insert_node / insert_via, loaded at launch start); before the first solution no node changes after its insert,
  // so pre_commit's patch scans over the nodes appended since a record's snapshot read these
  double pc_q[2][PATCH_K][NJ];
};

// The planner's LDS objects live at namespace scope so that every device function addresses them as LDS
// (ds_read/ds_write) rather than through generic pointers.
__shared__ PlanLds g_L;

struct Ctx {
  SceneDev sc;
  QueryDev Q;
};

// SMP_TRACE builds (tools/trace_probe.py): thread 0 of the leader and of the scouts appends (role, source line,
// device clock) records for the iterations [SMP_TRACE_IT0, SMP_TRACE_IT1) of query 0; smp_debug_tlog reads them.
#ifdef SMP_TRACE
#ifndef SMP_TRACE_IT0
#define SMP_TRACE_IT0 3000
#endif
#ifndef SMP_TRACE_IT1
#define SMP_TRACE_IT1 3040
#endif
constexpr unsigned TLOG_CAP = 1u << 18, TLOG_ROLE = TLOG_CAP / 4;  // records per role (0 leader, 1-2 scouts)
__device__ unsigned long long g_tlog[TLOG_CAP];
__device__ unsigned g_tlog_n[4];
// No atomics: each workgroup keeps its role's record count in LDS (loaded at launch start by tlog_begin) and
// stores it back after every record (plain stores, nothing waited on), so tracing adds ~0.1 us per record.
#define TR()                                                                                                  \
  if (threadIdx.x == 0 && g_L.tit >= SMP_TRACE_IT0 && g_L.tit < SMP_TRACE_IT1 && g_L.tn < TLOG_ROLE) {        \
    g_tlog[g_L.trole * TLOG_ROLE + g_L.tn] =                                                                   \
        ((unsigned long long)g_L.trole << 62) | ((unsigned long long)((g_L.tit - SMP_TRACE_IT0) & 0xff) << 54) | \
        ((unsigned long long)(__LINE__ & 0x3fff) << 40) | (wall_clock64() & 0xffffffffffull);                  \
    g_tlog_n[g_L.trole] = ++g_L.tn;                                                                            \
  }
#else
#define TR()
#endif

// Phase clocks (thread 0, s_memrealtime ticks): where an iteration spends its time.
enum { P_SAMPLE, P_NN, P_EXPAND, P_NEAR, P_CHOOSE, P_REWIRE, P_CONNECT, P_TILES, P_NTILES, P_COSTS, P_VIA, P_NVIA,
       P_TFK, P_TCHAIN, P_TCENTRE, P_TTEST, P_XEXPAND, P_XCHOOSE, P_XREWIRE, P_XCONNECT };
// Phase clocks read the device wall clock (s_memrealtime, a scalar memory round trip each); SMP_NOCLK builds
// compile them out of the phase / stage accounting (the timeouts and the planning clock keep theirs).
#ifdef SMP_NOCLK
__device__ __forceinline__ unsigned long long pclk() { return 0; }
#else
__device__ __forceinline__ unsigned long long pclk() { return wall_clock64(); }
#endif
#define PROF_BEGIN() unsigned long long _pt = threadIdx.x == 0 ? pclk() : 0
#ifdef SMP_DETAIL_PROF  // thread-0 clocks of serial sections into prof[28..31] (perf_probe.py SMP_DETAIL_PROF=1)
#define DETAIL_BEGIN(v) const unsigned long long v = threadIdx.x == 0 ? wall_clock64() : 0
#define DETAIL_END(v, k) if (threadIdx.x == 0) g_L.S.prof[k] += wall_clock64() - v
#else
#define DETAIL_BEGIN(v)
#define DETAIL_END(v, k)
#endif
#define PROF_END(k) if (threadIdx.x == 0) { g_L.S.prof[k] += pclk() - _pt; }

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
// Block-uniform control value read from LDS, made provably wave-uniform (a scalar register): every loop
// or branch that contains a __syncthreads() must be steered by such a value, or the compiler may lower it
// as a divergent region and desynchronise the waves' barrier counts.
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }
// A block-uniform pointer made scalar (SGPR pair) and typed as global memory, so that streaming loads issue as
// global_load with a scalar base instead of re-reading the pointer through the (scratch-resident) Ctx and
// going through flat addressing.
typedef const double __attribute__((address_space(1)))* gcdptr;
__device__ __forceinline__ gcdptr uni_gptr(const double* p) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((int)(unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
  return (gcdptr)(((unsigned long long)hi << 32) | lo);
}

// A global pointer made wave-uniform (SGPR pair): a pointer argument of a non-inlined function arrives in VGPRs.
__device__ __forceinline__ gcdptr uni_g(gcdptr p) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((int)(unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
  return (gcdptr)(((unsigned long long)hi << 32) | lo);
}
// The column bases of a tree's configurations ([NJ][cap]) as scalar pointers: a scan's loads then issue as global_load
// with a scalar base and a 32-bit lane offset, unconditionally (the scans clamp the index of lanes past the range to its
// last node and ignore their values) -- no address arithmetic in 64-bit vector registers, no branch per load.
__device__ __forceinline__ void tree_cols(gcdptr tq, int cap, gcdptr* c) {
#pragma unroll
  for (int j = 0; j < NJ; ++j) c[j] = uni_g(tq + (size_t)j * (unsigned)cap);
}
// Wave-uniform test of a scan's load group: true if the wavefront's 64 nodes starting at node `first` (a wave-uniform
// index) reach into the range [.., end).  A group wholly beyond the range skips its loads (a scalar branch): the clamped
// loads of such a group all read the range's last node, but each still costs its wave-instruction's address and data
// cycles in the CU's load pipeline -- 7 of a round's 8 groups on a 512-node tree.
__device__ __forceinline__ bool wave_group_live(int first, int end) {
  return __builtin_amdgcn_readfirstlane((int)(first < end)) != 0;
}
// Element i of a column with a scalar base: the byte offset is formed in 32 bits (cap <= 2^27 nodes), so the load issues as
// global_load with the base in SGPRs and one offset VGPR shared by every column of the node (no 64-bit vector address
// arithmetic per column).  The scans issue a group's loads unconditionally (indices clamped to the range) and decide
// validity afterwards: a load inside a per-batch branch whose other arm supplies a default value makes the compiler
// wait for the load (s_waitcnt vmcnt(0)) at the branch's join, so each batch would cost its own memory round trip.
__device__ __forceinline__ double ld_col(gcdptr col, unsigned i) {
  return *(gcdptr)((const char __attribute__((address_space(1)))*)col + i * 8u);
}
typedef const float __attribute__((address_space(1)))* gcfptr;
__device__ __forceinline__ float ld_col(gcfptr col, unsigned i) {  // as ld_col(gcdptr, ..)
  return *(gcfptr)((const char __attribute__((address_space(1)))*)col + i * 4u);
}
// One round of a scan's loads: NPT nodes per thread, b0 + u * BLOCK (u < NPT), of which the first K (a wave-uniform count)
// are loaded -- all at once, indices clamped to the range -- and the rest take `fill` (their results are masked out).
template <int K, int NPT, typename P, typename T>
__device__ __forceinline__ void load_round_k(T (*a)[NJ], const P* cols, int b0, int i1, const T* fill) {
#pragma unroll
  for (int u = 0; u < NPT; ++u) {
    if (u < K) {
      const unsigned ii = (unsigned)min(b0 + u * BLOCK, i1 - 1);
#pragma unroll
      for (int j = 0; j < NJ; ++j) a[u][j] = ld_col(cols[j], ii);
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j) a[u][j] = fill[j];
    }
  }
}
// The live nodes of a round are a prefix of the u (b0 - lane + u * BLOCK < i1): the round loads 1, 2, 4 or NPT of them by a
// wave-uniform switch, so one memory round trip covers it and a small tree's round does not load NPT nodes per thread.
template <int NPT, typename P, typename T>
__device__ __forceinline__ void load_round(T (*a)[NJ], const P* cols, int b0, int i1, const T* fill) {
  static_assert(NPT == 8, "rounds of 8 nodes per thread");
  const int first = b0 - lane_id();
  const int nl = uni(min(NPT, (i1 - first + BLOCK - 1) / BLOCK));
  if (nl > 4) load_round_k<8, NPT>(a, cols, b0, i1, fill);
  else if (nl > 2) load_round_k<4, NPT>(a, cols, b0, i1, fill);
  else if (nl > 1) load_round_k<2, NPT>(a, cols, b0, i1, fill);
  else load_round_k<1, NPT>(a, cols, b0, i1, fill);
}

// Stores into the tree arrays that the scout reads (q, cost, parent).  Plain stores: the lines stay in this XCD's
// L2, where a scout on the same XCD (the usual placement, plan_kernel) and the leader's own scans find them;
// scout_request publishes them (drain, plus an agent release when the scout runs on another XCD).
__device__ __forceinline__ void st_tree(double* p, double v) { *p = v; }
__device__ __forceinline__ void st_tree(int* p, int v) { *p = v; }
__device__ __forceinline__ void st_tree(float* p, float v) { *p = v; }
// Node coordinate j of node i of tree T: the fp64 value and its fp32 copy (the distributed scans' prefilter, TreeDev::qf).
__device__ __forceinline__ void st_coord(const TreeDev& T, int cap, int j, int i, double v) {
  st_tree(&T.q[(size_t)j * cap + i], v);
  st_tree(&T.qf[(size_t)j * cap + i], (float)v);
}
// XCD of this workgroup (HW_REG_XCC_ID): placement knowledge for speed only.
__device__ __forceinline__ int xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20); }
// Bitwise equality of two configurations (cache keys of the scout's records).
__device__ __forceinline__ bool same8(const double* a, const double* b) {
  bool s = true;
#pragma unroll
  for (int j = 0; j < NJ; ++j) s &= __double_as_longlong(a[j]) == __double_as_longlong(b[j]);
  return s;
}

// --------------------------------------------------------------------------------------- node access
// SMP_BOUNDS builds (debugging): out-of-range node ids are recorded in g_dbg (first one: source line, id, block,
// tree) and replaced by 0 instead of being dereferenced; smp_debug_bounds() reads the record.
#ifdef SMP_BOUNDS
__device__ int g_dbg[8];
#define BCHK(id, lim, line, t)                                                                          \
  if ((unsigned)(id) >= (unsigned)(lim)) {                                                             \
    if (atomicCAS(&g_dbg[0], 0, (line)) == 0) { g_dbg[1] = (id); g_dbg[2] = blockIdx.x; g_dbg[3] = (t); g_dbg[4] = (lim); } \
    id = 0;                                                                                            \
  }
#else
#define BCHK(id, lim, line, t)
#endif
#define load_node(C, t, id, o) load_node_at(C, t, id, o, __LINE__)
__device__ __forceinline__ void load_node_at(const Ctx& C, int t, int id, NodeRef* o, int line) {
  const TreeDev& T = C.Q.tr[t];
  const int cap = g_L.S.cap;  // (the leader and scouts stage their QState in LDS: no dependent global load for it)
  BCHK(id, cap, line, t);
  (void)line;
  for (int j = 0; j < NJ; ++j) o->q[j] = T.q[(size_t)j * cap + id];
  for (int k = 0; k < 3; ++k) o->c[k] = T.cost[(size_t)k * cap + id];
  o->id = id;
  o->parent = T.parent[id];
}

// insertNode (birrt_star.cpp:3298-3322), single lane.  Appends at index n[t] (== node id).
__device__ void insert_node(const Ctx& C, int t, const double* e_start, const double* e_target, const NodeRef& x) {
  QState& S = g_L.S;
  int i = S.n[t];
  if (i >= S.cap || x.id != i) { S.status = -7; S.phase = 2; return; }
  const TreeDev& T = C.Q.tr[t];
  int cap = S.cap;
  for (int j = 0; j < NJ; ++j) {
    st_coord(T, cap, j, i, x.q[j]);
    T.e_start[(size_t)j * cap + i] = e_start[j];
    T.e_target[(size_t)j * cap + i] = e_target[j];
    g_L.pc_q[t][i & (PATCH_K - 1)][j] = x.q[j];
  }
  for (int k = 0; k < 3; ++k) st_tree(&T.cost[(size_t)k * cap + i], x.c[k]);
  st_tree(&T.parent[i], x.parent);
  T.first_child[i] = -1;
  int p = x.parent;
  int f = T.first_child[p];
  T.next_sib[i] = f;
  T.prev_sib[i] = -1;
  if (f >= 0) T.prev_sib[f] = i;
  T.first_child[p] = i;
  S.n[t] = i + 1;
  S.edges[t]++;
}

// --------------------------------------------------------------------------------------- scans
// find_nearest_neighbour_interpolation: first strict minimum of the Euclidean joint distance (DH:128-156).
// sqrt is monotone, so a node can only beat the running minimum if its squared distance is below the minimum's
// squared distance; the (correctly rounded) sqrt is taken only then and compared exactly as the reference does.
__device__ bool spec_stage(const Ctx& C, int s, unsigned long long wait = 0);
// Distributed scans (defined with the job protocol below): true if a scan of `nodes` nodes is split over the helpers.
// Participants of a distributed scan: this workgroup and up to SCAN_P - 1 helpers (SCAN_PNEAR for a near scan).  While a
// collision job runs (overlap_work), its tiles hold workers 1 .. ntiles and participant p >= 1 is worker W - p: the scan
// takes the helpers the job leaves free, at least 8 participants (a busy helper takes its slice after its tile).
// A near scan takes one participant per 2^scan_nshift nodes (4096 by default, at least 8): its result collection grows
// with the participants (122 granules each), a nearest result is 3 granules.
__device__ __forceinline__ int scan_parts(const Ctx& C, int near, int nodes) {
  int P = min(min(C.Q.nworkers, SCAN_P), near ? min(min(C.Q.scan_pnear, SCAN_PNEAR), max(8, nodes >> C.Q.scan_nshift)) : C.Q.scan_pnn);
  if (g_L.in_job) P = min(P, max(C.Q.nworkers - g_L.u.job.ntiles, 8));
  return uni(P);
}
__device__ __forceinline__ bool scan_split(const Ctx& C, int nodes) {
  return uni(C.Q.jb != nullptr && C.Q.scan_min > 0 && nodes >= C.Q.scan_min && C.Q.nworkers >= 8);
}
__device__ int nearest_dist(const Ctx& C, int t, const double* q, int i0, int n, double* d_out);
__device__ void near_set_dist(const Ctx& C, int t, const double* q, int excl, bool nn);
// A local scan of at least this many nodes reads the tree's fp32 copy (the distributed slices' prefilter, exact).
constexpr int LOCAL_F32_MIN = 2048;
struct ScanLds;
__device__ __forceinline__ void slice_nn_body32(gcdptr tq, const float* tqf, int cap, int i0, int i1, const double* q,
                                                ScanLds& X);
// Block argmin of the nodes [i_begin, n) of tree t: the first strict minimum (d, id) of the distances, d = 10000
// if none is below it.  All threads; result in (g_L.wd[0], g_L.wi[0]) via nearest_scan's return.
__device__ __forceinline__ int nearest_scan(const Ctx& C, int t, const double* q, int i_begin, double* d_out) {
  TR();
  if (scan_split(C, uni(g_L.S.n[t]) - i_begin)) {
    int id;
    [[clang::always_inline]] id = nearest_dist(C, t, q, i_begin, uni(g_L.S.n[t]), d_out);
    return id;
  }
  const gcdptr tq = uni_gptr(C.Q.tr[t].q);
  const int n = uni(g_L.S.n[t]), cap = uni(g_L.S.cap);
  if (n - i_begin >= LOCAL_F32_MIN) {
    slice_nn_body32(tq, C.Q.tr[t].qf, cap, i_begin, n, q, g_L.sc.s);
    *d_out = __longlong_as_double((long long)g_L.sc.s.wk[0]);
    const int id = g_L.sc.s.wi[0];
    __syncthreads();
    return id;
  }
  gcdptr tqc[NJ];
  tree_cols(tq, cap, tqc);
  double qq[NJ];
  for (int j = 0; j < NJ; ++j) qq[j] = q[j];
  double best = 10000.0, best_s = 1e300;
  int bid = 0x7fffffff;
  // NPT nodes per thread per round, all loads of a round issued together: a round costs about one memory latency
  // plus one 8-term dependent sum, so few rounds matter more than few loads (a 4k-node tree is 1 round)
  constexpr int NPT = 8;
  for (int i0 = i_begin + threadIdx.x; i0 < n; i0 += NPT * BLOCK) {
    double a[NPT][NJ];
    load_round<NPT>(a, tqc, i0, n, qq);
    double s[NPT];
#pragma unroll
    for (int u = 0; u < NPT; ++u) s[u] = 0.0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int u = 0; u < NPT; ++u) {
        const double d = qq[j] - a[u][j];
        s[u] += d * d;
      }
    }
    // this thread's nodes in increasing index order (first strict minimum)
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int i = i0 + u * BLOCK;
      if (i < n && s[u] < best_s) {
        const double dist = sqrt(s[u]);
        if (dist < best) { best = dist; bid = i; best_s = s[u]; }
      }
    }
  }
  TR();
  // (distance, id) lexicographic minimum: distances are non-negative doubles, whose bit patterns order like the
  // values, so the wave minimum is two DPP integer reductions (distance bits, then the lowest id among the lanes
  // holding that distance) instead of fp64 compares through shuffles
  const unsigned long long key = (unsigned long long)__double_as_longlong(best);
  const unsigned long long wk = __ockl_wfred_min_u64(key);
  const int wi = __ockl_wfred_min_i32(key == wk ? bid : 0x7fffffff);
  if (lane_id() == 0) { g_L.wk[wave_id()] = wk; g_L.wi[wave_id()] = wi; }
  __syncthreads();
  unsigned long long bk = g_L.wk[0];
  int bi = g_L.wi[0];
#pragma unroll
  for (int w = 1; w < BLOCK / 64; ++w) {
    const unsigned long long k = g_L.wk[w];
    const int i = g_L.wi[w];
    if (k < bk || (k == bk && i < bi)) { bk = k; bi = i; }
  }
  __syncthreads();
  *d_out = __longlong_as_double((long long)bk);
  TR();
  return bi;
}

// nearest_scan over the nodes [i0, n) of tree t, n - i0 <= PATCH_K, from the leader's LDS copy of the recently
// appended nodes (valid before the first solution): wave 0, one node per lane, the same distance and the same
// (distance, id) minimum.  All threads; returns the id, *d_out = its distance (10000 if none is below it).
__device__ int patch_scan(int t, const double* q, int i0, int n, double* d_out) {
  if (threadIdx.x < 64) {
    const int i = i0 + (int)threadIdx.x;
    double best = 10000.0;
    int bid = 0x7fffffff;
    if (i < n) {
      const double* x = g_L.pc_q[t][i & (PATCH_K - 1)];
      double s = 0.0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const double d = q[j] - x[j];
        s += d * d;
      }
      const double dist = sqrt(s);
      if (dist < best) { best = dist; bid = i; }
    }
    const unsigned long long key = (unsigned long long)__double_as_longlong(best);
    const unsigned long long wk = __ockl_wfred_min_u64(key);
    const int wi = __ockl_wfred_min_i32(key == wk ? bid : 0x7fffffff);
    if (threadIdx.x == 0) { g_L.wk[0] = wk; g_L.wi[0] = wi; }
  }
  __syncthreads();
  *d_out = __longlong_as_double((long long)g_L.wk[0]);
  const int id = g_L.wi[0];
  __syncthreads();
  return id;
}

// find_nearest_neighbour_interpolation (birrt_star.cpp:4076-4133).  With `spec`, the scout's scan of the same
// sample over the tree's first X nodes is taken if it matches, and only the nodes appended since are scanned: one
// of them replaces the scout's node only with a strictly smaller distance (it has a larger index).
__device__ int nearest(const Ctx& C, int t, const double* q, bool spec = false) {
  const int n = uni(g_L.S.n[t]);
  if (threadIdx.x == 0) g_L.S.nn_nodes += n;
  if (spec && spec_stage(C, SC_NN)) {
    const ScoutNN& R = g_L.sr.nn;
    if (uni(R.ok && R.t == t && R.X <= n && same8(q, R.q))) {
      if (threadIdx.x == 0) g_L.S.sc_nn++;
      if (uni(R.X < n)) {  // nodes appended since the snapshot (none: the scout's answer stands)
        double dp;
        const int ip = nearest_scan(C, t, q, R.X, &dp);
        if (dp < R.d) return ip;
      }
      return R.d < 10000.0 ? R.id : 0;
    }
  }
  double bd;
  const int bi = nearest_scan(C, t, q, 0, &bd);
  return bd < 10000.0 ? bi : 0;
}

// The leader's nearest with a record (iteration): the record's path inline -- at most 64 appended nodes scanned by one
// wave from global memory (tail_scan) -- and a full scan only as a call, so that the scan's registers are saved only
// when it runs (a call that saves ~50 VGPRs at 512 threads costs ~1.5 us).  Same answer as nearest(C, t, q, true).
__device__ __noinline__ int nearest_scan_call(const Ctx& C, int t, const double* q, int i_begin, double* d_out) {
  return nearest_scan(C, t, q, i_begin, d_out);
}
// nearest_scan over at most 64 nodes [i0, n) of tree t: wave 0, one node per lane, the (distance, id) minimum as
// nearest_scan's (patch_scan's from global memory: after the first solution rewires may leave the LDS copy stale).
// All threads; returns the id, *d_out = its distance (10000 if none is below it).
__device__ int tail_scan(const Ctx& C, int t, const double* q, int i0, int n, double* d_out) {
  if (threadIdx.x < 64) {
    const int i = i0 + (int)threadIdx.x;
    double best = 10000.0;
    int bid = 0x7fffffff;
    if (i < n) {
      const double* x = C.Q.tr[t].q;
      const int cap = g_L.S.cap;
      double s = 0.0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const double d = q[j] - x[(size_t)j * cap + i];
        s += d * d;
      }
      const double dist = sqrt(s);
      if (dist < best) { best = dist; bid = i; }
    }
    const unsigned long long key = (unsigned long long)__double_as_longlong(best);
    const unsigned long long wk = __ockl_wfred_min_u64(key);
    const int wi = __ockl_wfred_min_i32(key == wk ? bid : 0x7fffffff);
    if (threadIdx.x == 0) { g_L.wk[0] = wk; g_L.wi[0] = wi; }
  }
  __syncthreads();
  *d_out = __longlong_as_double((long long)g_L.wk[0]);
  const int id = g_L.wi[0];
  __syncthreads();
  return id;
}
__device__ __forceinline__ int nearest_leader(const Ctx& C, int t, const double* q) {
  const int n = uni(g_L.S.n[t]);
  if (threadIdx.x == 0) g_L.S.nn_nodes += n;
  if (spec_stage(C, SC_NN)) {
    const ScoutNN& R = g_L.sr.nn;
    if (uni(R.ok && R.t == t && R.X <= n && same8(q, R.q))) {
      if (threadIdx.x == 0) g_L.S.sc_nn++;
      if (uni(R.X < n)) {
        double dp;
        const int ip = uni(n - R.X <= 64) ? tail_scan(C, t, q, R.X, n, &dp) : nearest_scan_call(C, t, q, R.X, &dp);
        if (dp < R.d) return ip;
      }
      return R.d < 10000.0 ? R.id : 0;
    }
  }
  double bd;
  const int bi = nearest_scan_call(C, t, q, 0, &bd);
  return bd < 10000.0 ? bi : 0;
}

// (cost,id) lexicographic order of the near list (std::sort order made total).  Costs are
// non-negative doubles, whose bit patterns order like the values, so keys compare as integers (64-bit integer
// compares stay in the scalar / VALU integer pipe and need no fp64 compare-to-mask step).
__device__ __forceinline__ bool ki_less(unsigned long long ka, int ia, unsigned long long kb, int ib) {
  return ka < kb || (ka == kb && ia < ib);
}
// Lane i | 1 (the odd lane of lane i's pair: DPP quad_perm [1, 1, 3, 3], no LDS round trip; the whole quad active).
__device__ __forceinline__ int odd_lane_of_pair(int v) { return __builtin_amdgcn_mov_dpp(v, 0xF5, 0xF, 0xF, false); }
// Lane i ^ 1 / i ^ 2 of a quad (DPP quad_perm, no LDS round trip; the whole quad active).
__device__ __forceinline__ int quad_xor1(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ int quad_xor2(int v) { return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false); }
// Wave-uniform lane read (v_readlane: scalar result, no LDS round trip).
__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int l) {
  const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)v, l);
  const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
  return ((unsigned long long)hi << 32) | lo;
}
// Lane i receives lane i-1's value (DPP wave_shr:1, a GFX9 whole-wave shift); lane 0 keeps its own.
__device__ __forceinline__ int wave_shr1(int v) { return __builtin_amdgcn_update_dpp(v, v, 0x138, 0xF, 0xF, false); }
__device__ __forceinline__ unsigned long long wave_shr1_u64(unsigned long long v) {
  const unsigned lo = wave_shr1((int)(unsigned)v), hi = wave_shr1((int)(unsigned)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

// One 64-node batch into a wave's two lane-distributed sorted lists (lane k holds entry k).  Only candidates
// beating the wave's K-th entry and the block-wide bound are inserted; an insertion is a readlane, a compare +
// ballot + popcount and a DPP shift of the list (~30 dependent instructions, so the bound matters).  Once the
// wave holds K entries its K-th key tightens the block bound (LDS atomic): any wave's K entries are K near nodes,
// so a node whose key lies beyond another wave's K-th key cannot be among the block's K smallest (largest).
template <int K>
__device__ __forceinline__ void near_batch(bool near, unsigned long long key, int base, int lane,
                                           unsigned long long& lk, int& li, unsigned long long& hk, int& hi,
                                           unsigned long long& blo_r, unsigned long long& bhi_r) {
  const int i = base + lane;
  const unsigned long long blo = blo_r, bhi = bhi_r;
  {
    const unsigned long long tk = readlane_u64(lk, K - 1);
    const int ti = __builtin_amdgcn_readlane(li, K - 1);
    unsigned long long m = __ballot(near && key <= blo && ki_less(key, i, tk, ti));
    if (m) {
      do {
        const int src = __builtin_ctzll(m);
        m &= m - 1;
        const unsigned long long kk = readlane_u64(key, src);
        const int ii = src + base;
        const unsigned long long uk = wave_shr1_u64(lk);
        const int ui = wave_shr1(li);
        const int pos = __popcll(__ballot(ki_less(lk, li, kk, ii)));
        if (lane >= pos) {
          if (lane == pos) { lk = kk; li = ii; } else { lk = uk; li = ui; }
        }
      } while (m);
      const unsigned long long nk = readlane_u64(lk, K - 1);
      if (lane == 0 && nk < blo && __builtin_amdgcn_readlane(li, K - 1) != 0x7fffffff) atomicMin(&blo_r, nk);
    }
  }
  {
    const unsigned long long tk = readlane_u64(hk, K - 1);
    const int ti = __builtin_amdgcn_readlane(hi, K - 1);
    unsigned long long m = __ballot(near && key >= bhi && ki_less(tk, ti, key, i));
    if (m) {
      do {
        const int src = __builtin_ctzll(m);
        m &= m - 1;
        const unsigned long long kk = readlane_u64(key, src);
        const int ii = src + base;
        const unsigned long long uk = wave_shr1_u64(hk);
        const int ui = wave_shr1(hi);
        const int pos = __popcll(__ballot(ki_less(kk, ii, hk, hi)));
        if (lane >= pos) {
          if (lane == pos) { hk = kk; hi = ii; } else { hk = uk; hi = ui; }
        }
      } while (m);
      const unsigned long long nk = readlane_u64(hk, K - 1);
      if (lane == 0 && nk > bhi && __builtin_amdgcn_readlane(hi, K - 1) != -1) atomicMax(&bhi_r, nk);
    }
  }
}

// One node's part of a nearest scan inside a near scan (NN): the first strict minimum of the Euclidean distance (DH:128-156)
// from its squared distance, the sqrt taken only when it can win.
__device__ __forceinline__ void nn_take(bool valid, double s, int i, double& best, double& best_s, int& bid) {
  if (valid && s < best_s) {
    const double dist = sqrt(s);
    if (dist < best) { best = dist; bid = i; best_s = s; }
  }
}
// Histogram bin of a near cost (monotone in the cost: bins order like costs; near_set's register path).
__device__ __forceinline__ int near_bin(unsigned long long key, double cmin, double scale) {
  return (int)((__longlong_as_double((long long)key) - cmin) * scale);
}

// Radius test sqrt(s) < r of the reference, decided on s against r^2 (1 -+ 1e-12); the (correctly rounded)
// sqrt is only taken inside that band, where the two could disagree.
__device__ __forceinline__ bool near_radius(bool valid, double s, double r, double r2lo, double r2hi, bool& amb) {
  amb = valid && s >= r2lo && s <= r2hi;
  return valid && s < r2lo;
}

// near_set, streaming path (trees above NEAR_NBK * BLOCK nodes, or cost distributions the histogram cannot
// split, e.g. many equal costs):
//   1. scan: four 64-node batches in flight per wave (q and cost loaded together); each wave keeps the K
//      smallest and K largest (key, id) of its nodes (near_batch);
//   2. rank merge: every wave entry finds its rank among all NW*K entries by binary searches in the other
//      waves' sorted lists (advanced in lock-step) and is written to its place if the rank is below K.
// The nearest-node part of a fused near_set<K, true>: the threads' candidates -> g_L.fnn_d / fnn_id.  All threads.
__device__ __forceinline__ void fnn_reduce(double best, int bid) {
  const unsigned long long key = (unsigned long long)__double_as_longlong(best);
  const unsigned long long wk = __ockl_wfred_min_u64(key);
  const int wi = __ockl_wfred_min_i32(key == wk ? bid : 0x7fffffff);
  if (lane_id() == 0) { g_L.wk[wave_id()] = wk; g_L.wi[wave_id()] = wi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long bk = g_L.wk[0];
    int bi = g_L.wi[0];
    for (int w = 1; w < BLOCK / 64; ++w)
      if (g_L.wk[w] < bk || (g_L.wk[w] == bk && g_L.wi[w] < bi)) { bk = g_L.wk[w]; bi = g_L.wi[w]; }
    g_L.fnn_d = __longlong_as_double((long long)bk);
    g_L.fnn_id = bi;
  }
  __syncthreads();
}

template <int K, bool NN>
__device__ __noinline__ void near_set_stream(const Ctx& C, int t, const double* q, int excl) {
  static_assert(K <= 64, "lane-distributed lists");
  double nb = 10000.0, nb_s = 1e300;  // NN: this thread's nearest candidate
  int nbi = 0x7fffffff;
  constexpr int NW = BLOCK / 64, NB = 4;
  const gcdptr tq = uni_gptr(C.Q.tr[t].q), tc = uni_gptr(C.Q.tr[t].cost);
  const int n = uni(g_L.S.n[t]), cap = uni(g_L.S.cap);
  gcdptr tqc[NJ];
  tree_cols(tq, cap, tqc);
  const double r = g_L.S.near_r;
  const double r2 = r * r, r2lo = r2 * (1.0 - 1e-12), r2hi = r2 * (1.0 + 1e-12);
  const int lane = lane_id(), wave = wave_id();
  if (threadIdx.x == 0) g_L.S.near_nodes += n;
  double qq[NJ];
  for (int j = 0; j < NJ; ++j) qq[j] = q[j];
  const unsigned long long KMAX = ~0ull;
  unsigned long long lk = KMAX, hk = 0;
  int li = 0x7fffffff, hi = -1;
  int wc = 0;
  for (int base = wave * 64; base < n; base += NB * BLOCK) {
    double x[NB][NJ];
    unsigned long long key[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int i = base + b * BLOCK + lane;
      if (wave_group_live(base + b * BLOCK, n)) {
        const unsigned ii = (unsigned)min(i, n - 1);
#pragma unroll
        for (int j = 0; j < NJ; ++j) x[b][j] = tqc[j][ii];
        key[b] = i < n ? (unsigned long long)__double_as_longlong(tc[ii]) : 0ull;
      } else {
#pragma unroll
        for (int j = 0; j < NJ; ++j) x[b][j] = qq[j];
        key[b] = 0ull;
      }
    }
    bool nr[NB], amb[NB];
    bool any_amb = false;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int i = base + b * BLOCK + lane;
      double sb = 0.0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        double d = qq[j] - x[b][j];
        sb += d * d;
      }
      nr[b] = near_radius(i < n && i != excl, sb, r, r2lo, r2hi, amb[b]);
      if (NN) nn_take(i < n, sb, i, nb, nb_s, nbi);
      x[b][0] = sb;
      any_amb |= amb[b];
    }
    if (__ballot(any_amb)) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
        if (amb[b]) nr[b] = sqrt(x[b][0]) < r;
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int bb = base + b * BLOCK;
      if (bb < n) {
        wc += __popcll(__ballot(nr[b]));
        near_batch<K>(nr[b], key[b], bb, lane, lk, li, hk, hi, g_L.near_blo, g_L.near_bhi);
      }
    }
  }
  if (lane < K) {
    g_L.nr.wlk[wave][lane] = lk; g_L.nr.wli[wave][lane] = li;
    g_L.nr.whk[wave][lane] = hk; g_L.nr.whi[wave][lane] = hi;
  }
  if (lane == 0) g_L.nr.wtot[wave] = wc;
  __syncthreads();
  int tot = 0;
  for (int w = 0; w < NW; ++w) tot += g_L.nr.wtot[w];
  const int take = min(K, tot);
  // threads [0, NW*K): low entries; [256, 256 + NW*K): high entries
  static_assert(NW * K <= 256, "rank merge thread map");
  const int hsel = threadIdx.x >= 256;
  const int e = threadIdx.x - hsel * 256;
  if (e < NW * K) {
    const int w = e / K, k = e - w * K;
    const unsigned long long ck = hsel ? g_L.nr.whk[w][k] : g_L.nr.wlk[w][k];
    const int ci = hsel ? g_L.nr.whi[w][k] : g_L.nr.wli[w][k];
    if (ci != (hsel ? -1 : 0x7fffffff)) {
      // per list o: number of entries ahead of (ck, ci) in that list's order (ascending low, descending high)
      int lo[NW];
#pragma unroll
      for (int o = 0; o < NW; ++o) lo[o] = 0;
      constexpr int P = K >= 32 ? 32 : K >= 16 ? 16 : K >= 8 ? 8 : K >= 4 ? 4 : K >= 2 ? 2 : 1;
#pragma unroll
      for (int step = P; step > 0; step >>= 1) {
        // lock-step binary search over the NW lists: entries [0, lo[o]) of list o are ahead
#pragma unroll
        for (int o = 0; o < NW; ++o) {
          const int m = lo[o] + step - 1;
          if (m < K) {
            const unsigned long long ok = hsel ? g_L.nr.whk[o][m] : g_L.nr.wlk[o][m];
            const int oi = hsel ? g_L.nr.whi[o][m] : g_L.nr.wli[o][m];
            const bool ahead = hsel ? ki_less(ck, ci, ok, oi) : ki_less(ok, oi, ck, ci);
            if (ahead) lo[o] += step;
          }
        }
      }
      int rank = k;
#pragma unroll
      for (int o = 0; o < NW; ++o)
        if (o != w) rank += lo[o];
      if (rank < take) {
        if (!hsel) { g_L.lo_c[rank] = __longlong_as_double((long long)ck); g_L.lo_i[rank] = ci; }
        else { g_L.hi_c[take - 1 - rank] = __longlong_as_double((long long)ck); g_L.hi_i[take - 1 - rank] = ci; }
      }
    }
  }
  if (threadIdx.x == 0) { g_L.nk = tot; g_L.n_lo = take; g_L.n_hi = take; g_L.near_blo = KMAX; g_L.near_bhi = 0; }
  __syncthreads();
  if (NN) fnn_reduce(nb, nbi);
}

// ------------------------------------------------------------------------------- slices of distributed scans
// Nearest over the nodes [i0, i1): the first strict minimum as nearest_scan, reduced to (distance key, id) in X.wk[0],
// X.wi[0] (key of 10000.0 and id INT_MAX if no node is below 10000).  All threads.
// Block reduction of the threads' nearest candidates (distance, id; each thread's first strict minimum over its nodes in
// increasing index order) to the (distance key, id) minimum in X.wk[0], X.wi[0].  All threads.
__device__ __forceinline__ void slice_nn_reduce(double best, int bid, ScanLds& X) {
  const unsigned long long key = (unsigned long long)__double_as_longlong(best);
  const unsigned long long wk = __ockl_wfred_min_u64(key);
  const int wi = __ockl_wfred_min_i32(key == wk ? bid : 0x7fffffff);
  if (lane_id() == 0) { X.wk[wave_id()] = wk; X.wi[wave_id()] = wi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long bk = X.wk[0];
    int bi = X.wi[0];
    for (int w = 1; w < BLOCK / 64; ++w)
      if (X.wk[w] < bk || (X.wk[w] == bk && X.wi[w] < bi)) { bk = X.wk[w]; bi = X.wi[w]; }
    X.wk[0] = bk;
    X.wi[0] = bi;
  }
  __syncthreads();
}

__device__ __forceinline__ void slice_nn_body(gcdptr tq, int cap, int i0, int i1, const double* q, ScanLds& X) {
  gcdptr tqc[NJ];
  tree_cols(tq, cap, tqc);
  double qq[NJ];
  for (int j = 0; j < NJ; ++j) qq[j] = q[j];
  double best = 10000.0, best_s = 1e300;
  int bid = 0x7fffffff;
  constexpr int NPT = 8;
  for (int b0 = i0 + (int)threadIdx.x; b0 < i1; b0 += NPT * BLOCK) {
    double a[NPT][NJ];
    load_round<NPT>(a, tqc, b0, i1, qq);
    double s[NPT];
#pragma unroll
    for (int u = 0; u < NPT; ++u) s[u] = 0.0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int u = 0; u < NPT; ++u) {
        const double d = qq[j] - a[u][j];
        s[u] += d * d;
      }
    }
#pragma unroll
    for (int u = 0; u < NPT; ++u) nn_take(b0 + u * BLOCK < i1, s[u], b0 + u * BLOCK, best, best_s, bid);
  }
  slice_nn_reduce(best, bid, X);
}
// ---- fp32 prefilter of the distributed scans (DESIGN.md "Scans of large trees").  A slice reads the tree's fp32 copy
// (TreeDev::qf, 32 B per node instead of 64) and decides in fp64 only where fp32 cannot.  With u = 2^-24 and c = 6u *
// max(|q_j|, |x_j|) (4u M bounds the error of one fp32 difference, M the largest magnitude; x1.5 margin), the fp32
// squared distance s32 of a node differs from the fp64 one s by at most E(s) = 4 (2 sqrt(8) c sqrt(s) + 8 c^2 + 9 u s)
// (the cross terms by Cauchy-Schwarz, the squares' and the eight-term sum's roundings; x4 margin).  Near test: a node
// with s32 + E < r2lo is near, one with s32 - E > r2hi is not (E taken at s = 2 r2hi, which covers every node that can
// fall between), the rest are decided from their fp64 coordinates exactly as before.  Nearest: a node can tie or beat
// the minimum only if its s32 is within 2 E(2 m) of the smallest s32 m; each thread keeps its smallest and second
// smallest s32, so the candidates are the threads' smallest nodes, and a thread whose second smallest is also within
// the margin rescans its nodes in fp64 -- the first strict minimum in fp64, as the reference, decides.
__device__ __forceinline__ gcfptr uni_gf(const float* p) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((int)(unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
  return (gcfptr)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ void tree_cols_f(const float* tqf, int cap, gcfptr* c) {
  const gcfptr b = uni_gf(tqf);
#pragma unroll
  for (int j = 0; j < NJ; ++j) c[j] = b + (size_t)j * (unsigned)cap;
}
constexpr double F32_U = 0x1p-24;
// The float nearest x from below / above (conservative thresholds).
__device__ __forceinline__ float f32_down(double x) {
  const float f = (float)x;
  return (double)f > x ? nextafterf(f, -__builtin_inff()) : f;
}
__device__ __forceinline__ float f32_up(double x) {
  const float f = (float)x;
  return (double)f < x ? nextafterf(f, __builtin_inff()) : f;
}
__device__ __forceinline__ double s32_err(double s, double c) {
  return 4.0 * (5.6568543 * c * sqrt(s) + 8.0 * c * c + 9.0 * F32_U * s);
}
// One node's fp32 squared distance and its coordinates' largest magnitude.
__device__ __forceinline__ float s32_of(const float* qf, const float* xf, float& xm) {
  float s = 0.0f;
  xm = 0.0f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const float d = qf[j] - xf[j];
    s += d * d;
    xm = fmaxf(xm, fabsf(xf[j]));
  }
  return s;
}
// The thread's two smallest s32 (b1 with its node, b2) and the largest magnitude seen.
__device__ __forceinline__ void nn32_track(bool valid, float s, int i, float xm, float& b1, float& b2, int& bi1,
                                           float& cm) {
  if (valid) {
    if (s < b1) { b2 = b1; b1 = s; bi1 = i; }
    else if (s < b2) b2 = s;
    cm = fmaxf(cm, xm);
  }
}
// Exact finish of a prefiltered nearest scan over the nodes i0 + threadIdx.x + k * BLOCK of [i0, i1) (every thread's node
// set in both slice forms): the candidates in fp64, the (distance key, id) minimum in X.wk[0], X.wi[0] (slice_nn_reduce).
__device__ __forceinline__ void nn32_finish(const gcdptr* tqc, int i0, int i1, const double* qq, float qm, float b1,
                                            float b2, int bi1, float cm, ScanLds& X) {
  const unsigned mb = __ockl_wfred_min_u32(__float_as_uint(b1));  // non-negative floats order like their bits
  const unsigned cb = __ockl_wfred_max_u32(__float_as_uint(cm));
  if (lane_id() == 0) { X.wi[wave_id()] = (int)mb; X.wk[wave_id()] = cb; }
  __syncthreads();
  unsigned m = (unsigned)X.wi[0], c = (unsigned)X.wk[0];
#pragma unroll
  for (int w = 1; w < BLOCK / 64; ++w) { m = min(m, (unsigned)X.wi[w]); c = max(c, (unsigned)X.wk[w]); }
  __syncthreads();  // (slice_nn_reduce writes X.wk / X.wi next)
  const double md = (double)__uint_as_float(m);
  const double th = md + 2.0 * s32_err(2.0 * md + 1e-300, 6.0 * F32_U * (double)fmaxf(__uint_as_float(c), qm));
  double best = 10000.0, best_s = 1e300;
  int bid = 0x7fffffff;
  if ((double)b2 <= th) {
    for (int i = i0 + (int)threadIdx.x; i < i1; i += BLOCK) {
      double sd = 0.0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const double d = qq[j] - tqc[j][(unsigned)i];
        sd += d * d;
      }
      nn_take(true, sd, i, best, best_s, bid);
    }
  } else if ((double)b1 <= th) {
    double sd = 0.0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const double d = qq[j] - tqc[j][(unsigned)bi1];
      sd += d * d;
    }
    nn_take(true, sd, bi1, best, best_s, bid);
  }
  slice_nn_reduce(best, bid, X);
}
// slice_nn over the fp32 copy (tqf), exact through nn32_finish.
__device__ __forceinline__ void slice_nn_body32(gcdptr tq, const float* tqf, int cap, int i0, int i1, const double* q,
                                                ScanLds& X) {
  gcdptr tqc[NJ];
  tree_cols(tq, cap, tqc);
  gcfptr tfc[NJ];
  tree_cols_f(tqf, cap, tfc);
  double qq[NJ];
  float qf[NJ], qm = 0.0f;
  for (int j = 0; j < NJ; ++j) { qq[j] = q[j]; qf[j] = (float)q[j]; qm = fmaxf(qm, fabsf(qf[j])); }
  float b1 = __builtin_inff(), b2 = __builtin_inff(), cm = 0.0f;
  int bi1 = 0x7fffffff;
  constexpr int NPT = 8;
  for (int b0 = i0 + (int)threadIdx.x; b0 < i1; b0 += NPT * BLOCK) {
    float a[NPT][NJ];
    load_round<NPT>(a, tfc, b0, i1, qf);
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      float xm;
      const float sv = s32_of(qf, a[u], xm);
      nn32_track(b0 + u * BLOCK < i1, sv, b0 + u * BLOCK, xm, b1, b2, bi1, cm);
    }
  }
  nn32_finish(tqc, i0, i1, qq, qm, b1, b2, bi1, cm, X);
}
__device__ void slice_nn(gcdptr tq, int cap, int i0, int i1, const double* q, ScanLds& X) {
  slice_nn_body(tq, cap, i0, i1, q, X);
}

// Near set over the nodes [i0, i1) (find_near_vertices_interpolation's radius test, excluding `excl`): count X.cnt,
// its SCAN_K lowest (cost, id) entries ascending in X.lk / X.li and SCAN_K highest descending in X.hk / X.hi (X.take
// each).  near_set_stream's per-wave lists and rank merge over a range.  All threads.
// NN: also the nearest node of q over the range (no exclusion), in X.wk[0] / X.wi[0] as slice_nn (fused scans: connect's
// nearest node and near set of the same configuration in one pass over the tree).
template <bool NN>
__device__ __forceinline__ void slice_near_body(gcdptr tq, gcdptr tc, int cap, int i0, int i1, const double* q,
                                                int excl, double r, ScanLds& X) {
  constexpr int K = SCAN_K, NW = BLOCK / 64, NB = 4;
  double nb = 10000.0, nb_s = 1e300;
  int nbi = 0x7fffffff;
  const double r2 = r * r, r2lo = r2 * (1.0 - 1e-12), r2hi = r2 * (1.0 + 1e-12);
  const int lane = lane_id(), wave = wave_id();
  gcdptr tqc[NJ];
  tree_cols(tq, cap, tqc);
  tc = uni_g(tc);
  double qq[NJ];
  for (int j = 0; j < NJ; ++j) qq[j] = q[j];
  const unsigned long long KMAX = ~0ull;
  if (threadIdx.x == 0) { X.blo = KMAX; X.bhi = 0; }
  __syncthreads();
  unsigned long long lk = KMAX, hk = 0;
  int li = 0x7fffffff, hi = -1;
  int wc = 0;
  for (int base = i0 + wave * 64; base < i1; base += NB * BLOCK) {
    double x[NB][NJ];
    unsigned long long key[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int i = base + b * BLOCK + lane;
      if (wave_group_live(base + b * BLOCK, i1)) {
        const unsigned ii = (unsigned)min(i, i1 - 1);
#pragma unroll
        for (int j = 0; j < NJ; ++j) x[b][j] = tqc[j][ii];
        key[b] = i < i1 ? (unsigned long long)__double_as_longlong(tc[ii]) : 0ull;
      } else {
#pragma unroll
        for (int j = 0; j < NJ; ++j) x[b][j] = qq[j];
        key[b] = 0ull;
      }
    }
    bool nr[NB], amb[NB];
    bool any_amb = false;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int i = base + b * BLOCK + lane;
      double sb = 0.0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        double d = qq[j] - x[b][j];
        sb += d * d;
      }
      nr[b] = near_radius(i < i1 && i != excl, sb, r, r2lo, r2hi, amb[b]);
      if (NN) nn_take(i < i1, sb, i, nb, nb_s, nbi);
      x[b][0] = sb;
      any_amb |= amb[b];
    }
    if (__ballot(any_amb)) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
        if (amb[b]) nr[b] = sqrt(x[b][0]) < r;
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int bb = base + b * BLOCK;
      if (bb < i1) {
        wc += __popcll(__ballot(nr[b]));
        near_batch<K>(nr[b], key[b], bb, lane, lk, li, hk, hi, X.blo, X.bhi);
      }
    }
  }
  if (lane < K) {
    X.wlk[wave][lane] = lk; X.wli[wave][lane] = li;
    X.whk[wave][lane] = hk; X.whi[wave][lane] = hi;
  }
  if (lane == 0) X.wtot[wave] = wc;
  __syncthreads();
  int tot = 0;
  for (int w = 0; w < NW; ++w) tot += X.wtot[w];
  const int take = min(K, tot);
  static_assert(NW * K <= 256, "rank merge thread map");
  const int hsel = threadIdx.x >= 256;
  const int e = threadIdx.x - hsel * 256;
  if (e < NW * K) {
    const int w = e / K, k = e - w * K;
    const unsigned long long ck = hsel ? X.whk[w][k] : X.wlk[w][k];
    const int ci = hsel ? X.whi[w][k] : X.wli[w][k];
    if (ci != (hsel ? -1 : 0x7fffffff)) {
      int lo[NW];
#pragma unroll
      for (int o = 0; o < NW; ++o) lo[o] = 0;
#pragma unroll
      for (int step = 16; step > 0; step >>= 1) {
#pragma unroll
        for (int o = 0; o < NW; ++o) {
          const int m = lo[o] + step - 1;
          if (m < K) {
            const unsigned long long ok = hsel ? X.whk[o][m] : X.wlk[o][m];
            const int oi = hsel ? X.whi[o][m] : X.wli[o][m];
            const bool ahead = hsel ? ki_less(ck, ci, ok, oi) : ki_less(ok, oi, ck, ci);
            if (ahead) lo[o] += step;
          }
        }
      }
      int rank = k;
#pragma unroll
      for (int o = 0; o < NW; ++o)
        if (o != w) rank += lo[o];
      if (rank < take) {
        if (!hsel) { X.lk[rank] = ck; X.li[rank] = ci; }
        else { X.hk[rank] = ck; X.hi[rank] = ci; }
      }
    }
  }
  if (threadIdx.x == 0) { X.cnt = tot; X.take = take; }
  __syncthreads();
  if (NN) slice_nn_reduce(nb, nbi, X);
}
// The same outputs by near_set's register path (histogram of the chunk's near costs, candidates at or beyond the bins of
// the K-th lowest / highest, ranked by counting), chunk by chunk with the running lists X.lk / X.hk: a slice of a few
// thousand nodes is one chunk, one pass of barrier-separated steps, instead of a per-wave insertion per candidate.
// Returns false (outputs undefined) if a chunk's histogram cannot split its costs (many equal costs): the caller then
// runs slice_near_body.  All threads.
// F32: the radius test and the nearest node from the tree's fp32 copy tqf (the prefilter above), fp64 where it cannot
// decide.
// pf (probe kernels only; null in the planner): thread 0's shader-clock ticks per step, accumulated into pf[0..6] (scan and
// radius test, chunk min / max, histogram or direct gather, bin prefix, gather, rank, nearest finish), pf[7] / pf[8] the
// chunks taking the direct / histogram path.
#define SNH_CLOCK(k)                                                                                              \
  if (pf && threadIdx.x == 0) {                                                                                   \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                                                   \
    pf[k] += _t - _tp;                                                                                            \
    _tp = _t;                                                                                                     \
  }
template <bool NN, bool F32 = false>
__device__ __forceinline__ bool slice_near_hist(gcdptr tq, gcdptr tc, int cap, int i0, int i1, const double* q, int excl,
                                                double r, ScanLds& X, const float* tqf = nullptr,
                                                unsigned long long* pf = nullptr) {
  constexpr int K = SCAN_K, NW = BLOCK / 64, CH = NEAR_NBK * BLOCK;
  unsigned long long _tp = pf && threadIdx.x == 0 ? __builtin_amdgcn_s_memtime() : 0;
  double nb = 10000.0, nb_s = 1e300;  // NN: this thread's nearest candidate
  int nbi = 0x7fffffff;
  float b1 = __builtin_inff(), b2 = __builtin_inff(), cm = 0.0f;  // NN with F32: nn32_track's state
  int bi1 = 0x7fffffff;
  static_assert(K <= 64 && NEAR_BUF == 128 && NEAR_BINS == 4 * 64, "register path layout");
  const double r2 = r * r, r2lo = r2 * (1.0 - 1e-12), r2hi = r2 * (1.0 + 1e-12);
  const int lane = lane_id(), wave = wave_id();
  gcdptr tqc[NJ];
  tree_cols(tq, cap, tqc);
  gcfptr tfc[NJ];
  if (F32) tree_cols_f(tqf, cap, tfc);
  tc = uni_g(tc);
  double qq[NJ];
  float qf[NJ], qm = 0.0f;
  for (int j = 0; j < NJ; ++j) { qq[j] = q[j]; qf[j] = (float)q[j]; qm = fmaxf(qm, fabsf(qf[j])); }
  // F32: E(2 r2hi) = c K1 + 32 c^2 + K2 for a node's c (s32_err at s = 2 r2hi)
  const double K1 = 4.0 * 5.6568543 * sqrt(2.0 * r2hi), K2 = 4.0 * 9.0 * F32_U * 2.0 * r2hi;
  // ... evaluated per node in fp32: E(m) <= m (kM + kM2 m) + K2 with m = max(|x_j|, |q_j|) and the constants rounded up; the
  // thresholds r2lo - K2 and r2hi + K2 carry a slack of 4 fp32 ulps of r^2, which covers the roundings of the fp32 threshold
  // expressions, so s32 < kA - m (kM + kM2 m) implies s32 + E < r2lo and s32 > kB + m (kM + kM2 m) implies s32 - E > r2hi
  const double slack = r2hi * 0x1p-21;
  const float kA = f32_down(r2lo - K2 - slack), kB = f32_up(r2hi + K2 + slack);
  const float kM = f32_up(6.0 * F32_U * K1), kM2 = f32_up(32.0 * 36.0 * F32_U * F32_U);
  int tot_all = 0;  // near nodes of the chunks before this one (block-uniform)
  int prev = 0;     // both running lists hold this many entries (block-uniform; X.take once the scan is done)
  // Three barriers per chunk: the chunk's min / max, its histogram, its gathered candidates.  Every wave derives the
  // bins of the K-th entries from the histogram itself (no barrier after a one-wave prefix), the running lists enter the
  // candidate buffers before the histogram's barrier, and the ranked lists need no barrier of their own: the next
  // chunk reads them only after its first barrier, the caller after the last one.
  for (int c0 = i0; c0 < i1; c0 += CH) {
    unsigned long long key[NEAR_NBK];
    unsigned nmask = 0;
    unsigned long long kmin = ~0ull, kmax = 0;
    int wc = 0;
#pragma unroll
    for (int g = 0; g < NEAR_NBK; g += 4) {
      key[g] = key[g + 1] = key[g + 2] = key[g + 3] = 0;
      if (F32 && c0 + g * BLOCK + wave * 64 < i1) {
        float xf[4][NJ];
#pragma unroll
        for (int b = 0; b < 4; ++b) {  // every load of the group at once (clamped indices; see ld_col)
          const int i = c0 + (g + b) * BLOCK + wave * 64 + lane;
          const unsigned ii = (unsigned)min(i, i1 - 1);
#pragma unroll
          for (int j = 0; j < NJ; ++j) xf[b][j] = ld_col(tfc[j], ii);
          const unsigned long long kb = (unsigned long long)__double_as_longlong(ld_col(tc, ii));
          key[g + b] = i < i1 ? kb : 0ull;
        }
        bool nr[4], und[4];
        bool any_und = false;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int i = c0 + (g + b) * BLOCK + wave * 64 + lane;
          const bool valid = i < i1 && i != excl;
          float xm;
          const float sv = s32_of(qf, xf[b], xm);
          const float m = fmaxf(xm, qm), em = m * (kM + kM2 * m);
          nr[b] = valid && sv < kA - em;
          und[b] = valid && !nr[b] && !(sv > kB + em);
          if (NN) nn32_track(i < i1, sv, i, xm, b1, b2, bi1, cm);
          any_und |= und[b];
        }
        if (__ballot(any_und)) {
          // nodes the fp32 test cannot decide: their fp64 coordinates, near_set's test
#pragma unroll
          for (int b = 0; b < 4; ++b)
            if (und[b]) {
              const unsigned ii = (unsigned)(c0 + (g + b) * BLOCK + wave * 64 + lane);
              double sb = 0.0;
#pragma unroll
              for (int j = 0; j < NJ; ++j) {
                const double d = qq[j] - tqc[j][ii];
                sb += d * d;
              }
              bool amb;
              nr[b] = near_radius(true, sb, r, r2lo, r2hi, amb);
              if (amb) nr[b] = sqrt(sb) < r;
            }
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          if (nr[b]) {
            nmask |= 1u << (g + b);
            kmin = min(kmin, key[g + b]);
            kmax = max(kmax, key[g + b]);
          }
          wc += __popcll(__ballot(nr[b]));
        }
      } else if (!F32 && c0 + g * BLOCK + wave * 64 < i1) {
        double x[4][NJ];
#pragma unroll
        for (int b = 0; b < 4; ++b) {  // every load of the group at once (clamped indices; see ld_col)
          const int i = c0 + (g + b) * BLOCK + wave * 64 + lane;
          const unsigned ii = (unsigned)min(i, i1 - 1);
#pragma unroll
          for (int j = 0; j < NJ; ++j) x[b][j] = ld_col(tqc[j], ii);
          const unsigned long long kb = (unsigned long long)__double_as_longlong(ld_col(tc, ii));
          key[g + b] = i < i1 ? kb : 0ull;
        }
        bool nr[4], amb[4];
        bool any_amb = false;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int i = c0 + (g + b) * BLOCK + wave * 64 + lane;
          double sb = 0.0;
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            double d = qq[j] - x[b][j];
            sb += d * d;
          }
          nr[b] = near_radius(i < i1 && i != excl, sb, r, r2lo, r2hi, amb[b]);
          if (NN) nn_take(i < i1, sb, i, nb, nb_s, nbi);
          x[b][0] = sb;
          any_amb |= amb[b];
        }
        if (__ballot(any_amb)) {
#pragma unroll
          for (int b = 0; b < 4; ++b)
            if (amb[b]) nr[b] = sqrt(x[b][0]) < r;
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          if (nr[b]) {
            nmask |= 1u << (g + b);
            kmin = min(kmin, key[g + b]);
            kmax = max(kmax, key[g + b]);
          }
          wc += __popcll(__ballot(nr[b]));
        }
      }
    }
    SNH_CLOCK(0);
    kmin = __ockl_wfred_min_u64(kmin);
    kmax = __ockl_wfred_max_u64(kmax);
    if (lane == 0) { X.hmin[wave] = kmin; X.hmax[wave] = kmax; X.wtot[wave] = wc; }
    if (threadIdx.x < NEAR_BINS) X.hist[threadIdx.x] = 0;
    __syncthreads();
    SNH_CLOCK(1);
    int tot = 0;
    kmin = ~0ull; kmax = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      tot += X.wtot[w];
      kmin = min(kmin, X.hmin[w]);
      kmax = max(kmax, X.hmax[w]);
    }
    tot = uni(tot);
    if (tot == 0) {  // nothing near in this chunk: lists unchanged (the barrier: every wave has read X.wtot / hmin / hmax)
      __syncthreads();
      continue;
    }
    const int take_c = min(K, tot);
    if (uni(tot <= NEAR_BUF && prev == 0)) {
      // few near nodes and no running lists: every near node of the chunk into one buffer (wave w's at the wave prefix
      // of the counts), each ranked by counting -- rank r below K is the r-th lowest entry, m - 1 - r below K the
      // (m - 1 - r)-th highest: no histogram
      int base = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) base += w < wave ? X.wtot[w] : 0;
      const unsigned long long below = (1ull << lane) - 1;
#pragma unroll
      for (int g = 0; g < NEAR_NBK; ++g) {
        if (c0 + g * BLOCK + wave * 64 < i1) {
          const bool nr = nmask >> g & 1;
          const unsigned long long ml = __ballot(nr);
          if (nr) {
            const int slot = base + __popcll(ml & below);
            X.ck[0][slot] = key[g];
            X.ci[0][slot] = c0 + g * BLOCK + wave * 64 + lane;
          }
          base += __popcll(ml);
        }
      }
      __syncthreads();
      {
        const int c = threadIdx.x >> 2, sl = threadIdx.x & 3;  // 4 lanes per entry (m <= 128)
        int rank = 0;
        unsigned long long ck = 0;
        int ci = 0;
        if (c < tot) {
          ck = X.ck[0][c];
          ci = X.ci[0][c];
          for (int j = sl; j < tot; j += 4) rank += ki_less(X.ck[0][j], X.ci[0][j], ck, ci);
        }
        rank += quad_xor1(rank);
        rank += quad_xor2(rank);
        if (c < tot && sl == 0) {
          if (rank < take_c) { X.lk[rank] = ck; X.li[rank] = ci; }
          const int h = tot - 1 - rank;
          if (h < take_c) { X.hk[h] = ck; X.hi[h] = ci; }
        }
      }
      tot_all += tot;
      prev = take_c;
      SNH_CLOCK(2);
      if (pf && threadIdx.x == 0) pf[7]++;
      continue;
    }
    const double cmin = __longlong_as_double((long long)kmin), cmax = __longlong_as_double((long long)kmax);
    const double scale = cmax > cmin ? (NEAR_BINS * (1.0 - 1e-9)) / (cmax - cmin) : 0.0;
    unsigned bins[NEAR_NBK / 4] = {};  // 8-bit bin of every near key
#pragma unroll
    for (int b = 0; b < NEAR_NBK; ++b)
      if (nmask >> b & 1) {
        const int bin = near_bin(key[b], cmin, scale);
        bins[b >> 2] |= (unsigned)bin << (8 * (b & 3));
        atomicAdd(&X.hist[bin], 1u);
      }
    // the running lists take the first buffer slots (no wave reads the buffers until after the gather's barrier)
    if (threadIdx.x < prev) {
      X.ck[0][threadIdx.x] = X.lk[threadIdx.x];
      X.ci[0][threadIdx.x] = X.li[threadIdx.x];
    }
    if (threadIdx.x >= 64 && threadIdx.x < 64 + prev) {
      X.ck[1][threadIdx.x - 64] = X.hk[threadIdx.x - 64];
      X.ci[1][threadIdx.x - 64] = X.hi[threadIdx.x - 64];
    }
    if (threadIdx.x == 0) { X.hcnt[0] = prev; X.hcnt[1] = prev; }
    __syncthreads();
    SNH_CLOCK(2);
    if (pf && threadIdx.x == 0) pf[8]++;
    int blo, bhi;
    bool fast;
    {
      // lane l owns bins 4l .. 4l+3: inclusive cumulative counts (near_set)
      const uint4 hv = reinterpret_cast<const uint4*>(X.hist)[lane];  // (one 16-byte read: a stride of 4 words per lane
      const unsigned h0 = hv.x, h1 = hv.y, h2 = hv.z, h3 = hv.w;        // read word by word met 4-way bank conflicts)
      const int inc = wave_incl_scan(h0 + h1 + h2 + h3);
      const int c3 = inc, c2 = c3 - (int)h3, c1 = c2 - (int)h2, c0b = c1 - (int)h1;
      const int e0 = c0b - (int)h0;
      const int flo = c0b >= take_c ? 0 : c1 >= take_c ? 1 : c2 >= take_c ? 2 : c3 >= take_c ? 3 : 4;
      const int Llo = __builtin_ctzll(__ballot(flo < 4));
      const int blo_w = 4 * Llo + __builtin_amdgcn_readlane(flo, Llo);
      const int cnt_lo = __builtin_amdgcn_readlane(flo == 0 ? c0b : flo == 1 ? c1 : flo == 2 ? c2 : c3, Llo);
      const int lim = tot - take_c;
      const int fhi = c2 <= lim ? 3 : c1 <= lim ? 2 : c0b <= lim ? 1 : e0 <= lim ? 0 : -1;
      const int Lhi = 63 - __builtin_clzll(__ballot(fhi >= 0));
      const int fh = __builtin_amdgcn_readlane(fhi, Lhi);
      const int cnt_hi = tot - __builtin_amdgcn_readlane(fhi == 3 ? c2 : fhi == 2 ? c1 : fhi == 1 ? c0b : e0, Lhi);
      blo = blo_w;
      bhi = 4 * Lhi + fh;
      fast = cnt_lo + prev <= NEAR_BUF && cnt_hi + prev <= NEAR_BUF;
    }
    SNH_CLOCK(3);
    if (!fast) {  // (wave-uniform, the same in every wave)
      __syncthreads();
      return false;
    }
    // gather in one pass: a candidate takes its buffer slot with an LDS atomic (the buffers' order does not matter: the
    // rank below counts (key, id) pairs, which are distinct)
#pragma unroll
    for (int g = 0; g < NEAR_NBK; ++g) {
      if (c0 + g * BLOCK + wave * 64 < i1) {
        const bool nr = nmask >> g & 1;
        const int bin = bins[g >> 2] >> (8 * (g & 3)) & 255;
        const int i = c0 + g * BLOCK + wave * 64 + lane;
        if (nr && bin <= blo) {
          const int slot = atomicAdd(&X.hcnt[0], 1);
          X.ck[0][slot] = key[g];
          X.ci[0][slot] = i;
        }
        if (nr && bin >= bhi) {
          const int slot = atomicAdd(&X.hcnt[1], 1);
          X.ck[1][slot] = key[g];
          X.ci[1][slot] = i;
        }
      }
    }
    __syncthreads();
    SNH_CLOCK(4);
    const int take = min(K, tot_all + tot);
    {
      // rank: threads [0, 256) the low buffer, [256, 512) the high buffer; L lanes per entry; the low list ascending,
      // the high list descending (its rank counts the entries above it)
      const int e = threadIdx.x >= 256;
      const int idx = threadIdx.x & 255;
      const int m = X.hcnt[e];
      const int L = m <= 64 ? 4 : 2;
      const int c = L == 4 ? idx >> 2 : idx >> 1, sl = idx & (L - 1);
      int rank = 0;
      unsigned long long ck = 0;
      int ci = 0;
      if (c < m) {
        ck = X.ck[e][c];
        ci = X.ci[e][c];
        for (int j = sl; j < m; j += L) {
          const unsigned long long ok = X.ck[e][j];
          const int oi = X.ci[e][j];
          rank += e == 0 ? ki_less(ok, oi, ck, ci) : ki_less(ck, ci, ok, oi);
        }
      }
      rank += quad_xor1(rank);
      if (L == 4) rank += quad_xor2(rank);
      if (c < m && sl == 0 && rank < take) {
        if (e == 0) { X.lk[rank] = ck; X.li[rank] = ci; }
        else { X.hk[rank] = ck; X.hi[rank] = ci; }
      }
    }
    tot_all += tot;
    prev = take;
    SNH_CLOCK(5);
  }
  if (threadIdx.x == 0) { X.cnt = tot_all; X.take = prev; }
  __syncthreads();
  if (NN && F32) nn32_finish(tqc, i0, i1, qq, qm, b1, b2, bi1, cm, X);
  else if (NN) slice_nn_reduce(nb, nbi, X);
  SNH_CLOCK(6);
  return true;
}
#undef SNH_CLOCK

template <bool NN>
__device__ __noinline__ void slice_near(gcdptr tq, gcdptr tc, int cap, int i0, int i1, const double* q, int excl,
                                        double r, ScanLds& X) {
  if (uni(slice_near_hist<NN>(tq, tc, cap, i0, i1, q, excl, r, X))) return;
  slice_near_body<NN>(tq, tc, cap, i0, i1, q, excl, r, X);
}
template <bool NN>
__device__ __noinline__ void slice_near_slow(gcdptr tq, gcdptr tc, int cap, int i0, int i1, const double* q, int excl,
                                             double r, ScanLds& X) {
  slice_near_body<NN>(tq, tc, cap, i0, i1, q, excl, r, X);
}
// The helpers' form of slice_near: the register path inlined into the helper loop, so that a scan job costs no call --
// a non-inlined callee at 512 threads saves and restores every callee-saved VGPR it uses, ~100 of them here (≈200 KB
// of scratch stores and loads per call through the CU's load pipeline, and most of a large tree's write traffic).
template <bool NN, bool F32 = false>
__device__ __forceinline__ void slice_near_inl(gcdptr tq, gcdptr tc, int cap, int i0, int i1, const double* q, int excl,
                                               double r, ScanLds& X, const float* tqf = nullptr,
                                               unsigned long long* pf = nullptr) {
  if (uni(slice_near_hist<NN, F32>(tq, tc, cap, i0, i1, q, excl, r, X, tqf, pf))) return;
  slice_near_slow<NN>(tq, tc, cap, i0, i1, q, excl, r, X);
}

// find_near_vertices_interpolation (birrt_star.cpp:4272-4324): count k, the first K and the last K entries of
// the (cost,id)-sorted near list.  The tree is taken in chunks of NEAR_NBK * BLOCK nodes; the radius test leaves
// every thread with up to NEAR_NBK (key, near) pairs of the chunk in registers; then
//   1. block min / max of the chunk's near keys, and a NEAR_BINS-bin LDS histogram of cost over [min, max] (the
//      bin map (c - cmin) * scale is monotone in c, so bins order like costs);
//   2. wave 0 scans the histogram: b_lo = first bin where the cumulative count reaches K, b_hi = last bin whose
//      suffix count reaches K;
//   3. the chunk's near nodes in bins <= b_lo (>= b_hi) and the running low (high) list of the previous chunks
//      are gathered in an LDS buffer (one atomic per wave and list) and every entry is ranked by counting the
//      entries ahead of it (2-4 lanes per entry): the entries of rank < K are the new running list.
// A buffer that would exceed NEAR_BUF entries (ties, clustered costs) sends the call to near_set_stream.
#ifdef SMP_NEAR_PROF  // clocks of the barrier-separated steps into prof[20..24]; path counts in prof[26], prof[27]
#define NEAR_CLOCK(k)                                                                    \
  if (threadIdx.x == 0) {                                                                \
    const unsigned long long _t = wall_clock64();                                        \
    if (k > 0) g_L.S.prof[19 + k] += _t - _tn;                                           \
    _tn = _t;                                                                            \
  }
#define NEAR_COUNT(k) if (threadIdx.x == 0) g_L.S.prof[k]++
#elif defined(SMP_TRACE)
#define NEAR_CLOCK(k) TR()
#define NEAR_COUNT(k)
#else
#define NEAR_CLOCK(k)
#define NEAR_COUNT(k)
#endif

// NN: also the nearest node of q over the whole tree (no exclusion; nearest()'s answer) in g_L.fnn_d / fnn_id -- connect's
// two scans of x_new in tree_B in one pass (no scout record then: spec must be false).
// near_set's record path: the scout's near set of the same configuration, merged with the near nodes appended since its
// snapshot (at most 64), if the record applies (returns false otherwise).  No tree scan: light enough to inline.
template <int K>
__device__ __forceinline__ bool near_set_rec(const Ctx& C, int t, const double* q, int excl) {
  if (!spec_stage(C, SC_NEAR)) return false;
  const int n = uni(g_L.S.n[t]);
  const gcdptr tq = uni_gptr(C.Q.tr[t].q), tc = uni_gptr(C.Q.tr[t].cost);
  const int cap = uni(g_L.S.cap);
  const double r = g_L.S.near_r;
  const double r2 = r * r, r2lo = r2 * (1.0 - 1e-12), r2hi = r2 * (1.0 + 1e-12);
  const int lane = lane_id();
  // the scout's near set of the same configuration over the tree's first X nodes, with the near nodes appended since
  // (at most 64: else the full scan below) merged in exactly: the costs of the first X nodes are those the record
  // saw (no rewire of this tree in between), so the K lowest / highest (cost, id) entries of the whole set are among
  // the record's low / high lists and the appended near nodes
  const ScoutNear& R = g_L.sr.nr;
  if (uni(R.ok && R.t == t && R.X <= n && n - R.X <= 64 && same8(q, R.q))) {
    const int X = uni(R.X);
    if (threadIdx.x < 64) {
      const int i = X + lane;
      bool nr = false;
      unsigned long long key = 0;
      if (i < n) {
        double sb = 0.0;
        for (int j = 0; j < NJ; ++j) {
          const double d = q[j] - (tq + (size_t)j * cap)[(unsigned)i];
          sb += d * d;
        }
        bool amb;
        nr = near_radius(i != excl, sb, r, r2lo, r2hi, amb);
        if (amb) nr = sqrt(sb) < r;
        if (nr) key = (unsigned long long)__double_as_longlong(tc[(unsigned)i]);
      }
      const unsigned long long mk = __ballot(nr);
      if (nr) {
        const int s = __popcll(mk & ((1ull << lane) - 1));
        g_L.nh.ck[0][s] = key;
        g_L.nh.ci[0][s] = i;
      }
      if (lane == 0) g_L.nh.cnt[0] = __popcll(mk);
    }
    __syncthreads();
    const int m = uni(g_L.nh.cnt[0]);
    const int take = min(K, R.nk + m);
    if (m == 0) {
      if (threadIdx.x < K) {
        g_L.lo_i[threadIdx.x] = R.lo_i[threadIdx.x]; g_L.lo_c[threadIdx.x] = R.lo_c[threadIdx.x];
        g_L.hi_i[threadIdx.x] = R.hi_i[threadIdx.x]; g_L.hi_c[threadIdx.x] = R.hi_c[threadIdx.x];
      }
    } else if (threadIdx.x < 128) {
      // wave 0 ranks the low side (the record's low list + the appended), wave 1 the high side; entries c = lane,
      // lane + 64 of N <= K + 64, each ranked against all N as near_set's merge does
      const int e = threadIdx.x >> 6;
      const int nl = e == 0 ? R.n_lo : R.n_hi, N = nl + m;
      for (int c = lane; c < N; c += 64) {
        unsigned long long ck;
        int ci;
        if (c < nl) {
          ck = (unsigned long long)__double_as_longlong(e == 0 ? R.lo_c[c] : R.hi_c[c]);
          ci = e == 0 ? R.lo_i[c] : R.hi_i[c];
        } else {
          ck = g_L.nh.ck[0][c - nl];
          ci = g_L.nh.ci[0][c - nl];
        }
        int rank = 0;
        for (int o = 0; o < N; ++o) {
          const unsigned long long ok = o < nl ? (unsigned long long)__double_as_longlong(e == 0 ? R.lo_c[o] : R.hi_c[o])
                                               : g_L.nh.ck[0][o - nl];
          const int oi = o < nl ? (e == 0 ? R.lo_i[o] : R.hi_i[o]) : g_L.nh.ci[0][o - nl];
          rank += e == 0 ? ki_less(ok, oi, ck, ci) : ki_less(ck, ci, ok, oi);
        }
        if (rank < take) {
          if (e == 0) { g_L.lo_c[rank] = __longlong_as_double((long long)ck); g_L.lo_i[rank] = ci; }
          else { g_L.hi_c[take - 1 - rank] = __longlong_as_double((long long)ck); g_L.hi_i[take - 1 - rank] = ci; }
        }
      }
    }
    if (threadIdx.x == 0) {
      g_L.nk = R.nk + m; g_L.n_lo = m == 0 ? R.n_lo : take; g_L.n_hi = m == 0 ? R.n_hi : take;
      g_L.S.near_nodes += n;
      g_L.S.sc_near++;
    }
    __syncthreads();
    TR();
    return true;
  }
  return false;
}

template <int K, bool NN = false>
__device__ void near_set(const Ctx& C, int t, const double* q, int excl, bool spec = false) {
#ifdef SMP_NEAR_PROF
  unsigned long long _tn = 0;
#endif
  static_assert(K <= 64 && NEAR_BUF == 128 && NEAR_BINS == 4 * 64, "register path layout");
  static_assert(K <= MAX_NEAR, "scout record lists");
  constexpr int NW = BLOCK / 64, CH = NEAR_NBK * BLOCK;
  const int n = uni(g_L.S.n[t]);
  const gcdptr tq = uni_gptr(C.Q.tr[t].q), tc = uni_gptr(C.Q.tr[t].cost);
  const int cap = uni(g_L.S.cap);
  gcdptr tqc[NJ];
  tree_cols(tq, cap, tqc);
  const double r = g_L.S.near_r;
  const double r2 = r * r, r2lo = r2 * (1.0 - 1e-12), r2hi = r2 * (1.0 + 1e-12);
  const int lane = lane_id(), wave = wave_id();
  TR();
  if (!NN && spec && near_set_rec<K>(C, t, q, excl)) return;
  if (K == SCAN_K && scan_split(C, n)) {
    [[clang::always_inline]] near_set_dist(C, t, q, excl, NN);
    TR();
    return;
  }
  if (K == SCAN_K && n >= LOCAL_F32_MIN) {
    // the slice form over the whole tree with the fp32 prefilter (exact): its lists into near_set's outputs
    ScanLds& X = g_L.sc.s;
    slice_near_inl<NN, true>(tq, tc, cap, 0, n, q, excl, r, X, C.Q.tr[t].qf);
    const int take = X.take;
    if (threadIdx.x < take) {
      const int e = threadIdx.x;
      g_L.lo_c[e] = __longlong_as_double((long long)X.lk[e]); g_L.lo_i[e] = X.li[e];
      g_L.hi_c[take - 1 - e] = __longlong_as_double((long long)X.hk[e]); g_L.hi_i[take - 1 - e] = X.hi[e];
    }
    if (threadIdx.x == 0) {
      g_L.nk = X.cnt; g_L.n_lo = take; g_L.n_hi = take; g_L.S.near_nodes += n;
      if (NN) { g_L.fnn_d = __longlong_as_double((long long)X.wk[0]); g_L.fnn_id = X.wi[0]; }
    }
    __syncthreads();
    TR();
    return;
  }
  double nb = 10000.0, nb_s = 1e300;  // NN: this thread's nearest candidate
  int nbi = 0x7fffffff;
  double qq[NJ];
  for (int j = 0; j < NJ; ++j) qq[j] = q[j];
  int tot_all = 0;  // near nodes of the chunks before this one (block-uniform)
  if (threadIdx.x == 0) { g_L.n_lo = 0; g_L.n_hi = 0; }
  for (int c0 = 0; c0 < n; c0 += CH) {
    NEAR_CLOCK(0);
    unsigned long long key[NEAR_NBK];
    unsigned nmask = 0;
    unsigned long long kmin = ~0ull, kmax = 0;
    int wc = 0;
#pragma unroll
    for (int g = 0; g < NEAR_NBK; g += 4) {
      key[g] = key[g + 1] = key[g + 2] = key[g + 3] = 0;
      if (c0 + g * BLOCK + wave * 64 < n) {
        double x[4][NJ];
#pragma unroll
        for (int b = 0; b < 4; ++b) {  // every load of the group at once (clamped indices; see ld_col)
          const int i = c0 + (g + b) * BLOCK + wave * 64 + lane;
          const unsigned ii = (unsigned)min(i, n - 1);
#pragma unroll
          for (int j = 0; j < NJ; ++j) x[b][j] = ld_col(tqc[j], ii);
          const unsigned long long kb = (unsigned long long)__double_as_longlong(ld_col(tc, ii));
          key[g + b] = i < n ? kb : 0ull;
        }
        bool nr[4], amb[4];
        bool any_amb = false;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int i = c0 + (g + b) * BLOCK + wave * 64 + lane;
          double sb = 0.0;
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            double d = qq[j] - x[b][j];
            sb += d * d;
          }
          nr[b] = near_radius(i < n && i != excl, sb, r, r2lo, r2hi, amb[b]);
          if (NN) nn_take(i < n, sb, i, nb, nb_s, nbi);
          x[b][0] = sb;
          any_amb |= amb[b];
        }
        if (__ballot(any_amb)) {
#pragma unroll
          for (int b = 0; b < 4; ++b)
            if (amb[b]) nr[b] = sqrt(x[b][0]) < r;
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          if (nr[b]) {
            nmask |= 1u << (g + b);
            kmin = min(kmin, key[g + b]);
            kmax = max(kmax, key[g + b]);
          }
          wc += __popcll(__ballot(nr[b]));
        }
      }
    }
    kmin = __ockl_wfred_min_u64(kmin);
    kmax = __ockl_wfred_max_u64(kmax);
    if (lane == 0) { g_L.nh.wmin[wave] = kmin; g_L.nh.wmax[wave] = kmax; g_L.nh.wtot[wave] = wc; }
    if (threadIdx.x < NEAR_BINS) g_L.nh.hist[threadIdx.x] = 0;
    __syncthreads();
    NEAR_CLOCK(1);
    int tot = 0;
    kmin = ~0ull; kmax = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      tot += g_L.nh.wtot[w];
      kmin = min(kmin, g_L.nh.wmin[w]);
      kmax = max(kmax, g_L.nh.wmax[w]);
    }
    tot = uni(tot);
    if (tot == 0) {  // nothing near in this chunk: lists unchanged (the barrier: every wave has read wtot / wmin / wmax)
      __syncthreads();
      continue;
    }
    const int take_c = min(K, tot);
    const int prev_lo = g_L.n_lo, prev_hi = g_L.n_hi;
    if (uni(tot <= NEAR_BUF && prev_lo == 0 && prev_hi == 0)) {
      // few near nodes and no running lists: one buffer, ranked by counting (slice_near_hist's direct path)
      int base = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) base += w < wave ? g_L.nh.wtot[w] : 0;
      const unsigned long long below = (1ull << lane) - 1;
#pragma unroll
      for (int g = 0; g < NEAR_NBK; ++g) {
        if (c0 + g * BLOCK + wave * 64 < n) {
          const bool nr = nmask >> g & 1;
          const unsigned long long ml = __ballot(nr);
          if (nr) {
            const int slot = base + __popcll(ml & below);
            g_L.nh.ck[0][slot] = key[g];
            g_L.nh.ci[0][slot] = c0 + g * BLOCK + wave * 64 + lane;
          }
          base += __popcll(ml);
        }
      }
      __syncthreads();
      {
        const int c = threadIdx.x >> 2, sl = threadIdx.x & 3;  // 4 lanes per entry (m <= 128)
        int rank = 0;
        unsigned long long ck = 0;
        int ci = 0;
        if (c < tot) {
          ck = g_L.nh.ck[0][c];
          ci = g_L.nh.ci[0][c];
          for (int j = sl; j < tot; j += 4) rank += ki_less(g_L.nh.ck[0][j], g_L.nh.ci[0][j], ck, ci);
        }
        rank += quad_xor1(rank);
        rank += quad_xor2(rank);
        if (c < tot && sl == 0) {
          if (rank < take_c) { g_L.lo_c[rank] = __longlong_as_double((long long)ck); g_L.lo_i[rank] = ci; }
          const int h = tot - 1 - rank;
          if (h < take_c) { g_L.hi_c[take_c - 1 - h] = __longlong_as_double((long long)ck); g_L.hi_i[take_c - 1 - h] = ci; }
        }
      }
      tot_all += tot;
      __syncthreads();
      if (threadIdx.x == 0) { g_L.n_lo = take_c; g_L.n_hi = take_c; }
      __syncthreads();
      NEAR_COUNT(27);
      continue;
    }
    const double cmin = __longlong_as_double((long long)kmin), cmax = __longlong_as_double((long long)kmax);
    const double scale = cmax > cmin ? (NEAR_BINS * (1.0 - 1e-9)) / (cmax - cmin) : 0.0;
    unsigned bins[NEAR_NBK / 4] = {};  // 8-bit bin of every near key
#pragma unroll
    for (int b = 0; b < NEAR_NBK; ++b)
      if (nmask >> b & 1) {
        const int bin = near_bin(key[b], cmin, scale);
        bins[b >> 2] |= (unsigned)bin << (8 * (b & 3));
        atomicAdd(&g_L.nh.hist[bin], 1u);
      }
    __syncthreads();
    NEAR_CLOCK(2);
    if (wave == 0) {
      // lane l owns bins 4l .. 4l+3: inclusive cumulative counts
      const uint4 hv = reinterpret_cast<const uint4*>(g_L.nh.hist)[lane];  // (one 16-byte read per lane)
      const unsigned h0 = hv.x, h1 = hv.y, h2 = hv.z, h3 = hv.w;
      const int inc = wave_incl_scan(h0 + h1 + h2 + h3);
      const int c3 = inc, c2 = c3 - (int)h3, c1 = c2 - (int)h2, c0b = c1 - (int)h1;  // inclusive
      const int e0 = c0b - (int)h0;                                                   // exclusive of bin 4l
      // b_lo: first bin with inclusive count >= take_c
      const int flo = c0b >= take_c ? 0 : c1 >= take_c ? 1 : c2 >= take_c ? 2 : c3 >= take_c ? 3 : 4;
      const int Llo = __builtin_ctzll(__ballot(flo < 4));
      const int blo = 4 * Llo + __builtin_amdgcn_readlane(flo, Llo);
      const int cnt_lo = __builtin_amdgcn_readlane(flo == 0 ? c0b : flo == 1 ? c1 : flo == 2 ? c2 : c3, Llo);
      // b_hi: last bin whose exclusive count is <= tot - take_c (suffix count >= take_c)
      const int lim = tot - take_c;
      const int fhi = c2 <= lim ? 3 : c1 <= lim ? 2 : c0b <= lim ? 1 : e0 <= lim ? 0 : -1;
      const int Lhi = 63 - __builtin_clzll(__ballot(fhi >= 0));
      const int fh = __builtin_amdgcn_readlane(fhi, Lhi);
      const int bhi = 4 * Lhi + fh;
      const int cnt_hi = tot - __builtin_amdgcn_readlane(fhi == 3 ? c2 : fhi == 2 ? c1 : fhi == 1 ? c0b : e0, Lhi);
      if (lane == 0) {
        g_L.nh.blo = blo;
        g_L.nh.bhi = bhi;
        g_L.nh.fast = cnt_lo + prev_lo <= NEAR_BUF && cnt_hi + prev_hi <= NEAR_BUF;
        g_L.nh.cnt[0] = prev_lo;  // the running lists take the first buffer slots
        g_L.nh.cnt[1] = prev_hi;
      }
    }
    if (threadIdx.x < prev_lo) {
      g_L.nh.ck[0][threadIdx.x] = (unsigned long long)__double_as_longlong(g_L.lo_c[threadIdx.x]);
      g_L.nh.ci[0][threadIdx.x] = g_L.lo_i[threadIdx.x];
    }
    if (threadIdx.x >= 64 && threadIdx.x < 64 + prev_hi) {
      g_L.nh.ck[1][threadIdx.x - 64] = (unsigned long long)__double_as_longlong(g_L.hi_c[threadIdx.x - 64]);
      g_L.nh.ci[1][threadIdx.x - 64] = g_L.hi_i[threadIdx.x - 64];
    }
    __syncthreads();
    NEAR_CLOCK(3);
    if (!uni(g_L.nh.fast)) {
      NEAR_COUNT(26);
      __syncthreads();
      near_set_stream<K, NN>(C, t, q, excl);
      return;
    }
    const int blo = g_L.nh.blo, bhi = g_L.nh.bhi;
    // gather in one pass: a candidate takes its buffer slot with an LDS atomic (order-free: the rank counts (key, id))
#pragma unroll
    for (int g = 0; g < NEAR_NBK; ++g) {
      if (c0 + g * BLOCK + wave * 64 < n) {
        const bool nr = nmask >> g & 1;
        const int bin = bins[g >> 2] >> (8 * (g & 3)) & 255;
        const int i = c0 + g * BLOCK + wave * 64 + lane;
        if (nr && bin <= blo) {
          const int slot = atomicAdd(&g_L.nh.cnt[0], 1);
          g_L.nh.ck[0][slot] = key[g];
          g_L.nh.ci[0][slot] = i;
        }
        if (nr && bin >= bhi) {
          const int slot = atomicAdd(&g_L.nh.cnt[1], 1);
          g_L.nh.ck[1][slot] = key[g];
          g_L.nh.ci[1][slot] = i;
        }
      }
    }
    __syncthreads();
    NEAR_CLOCK(4);
    const int take = min(K, tot_all + tot);
    {
      // rank: threads [0, 256) the low buffer, [256, 512) the high buffer; L lanes per entry
      const int e = threadIdx.x >= 256;
      const int idx = threadIdx.x & 255;
      const int m = g_L.nh.cnt[e];
      const int L = m <= 64 ? 4 : 2;
      const int c = L == 4 ? idx >> 2 : idx >> 1, sl = idx & (L - 1);
      int rank = 0;
      unsigned long long ck = 0;
      int ci = 0;
      if (c < m) {
        ck = g_L.nh.ck[e][c];
        ci = g_L.nh.ci[e][c];
        for (int j = sl; j < m; j += L) {
          const unsigned long long ok = g_L.nh.ck[e][j];
          const int oi = g_L.nh.ci[e][j];
          rank += e == 0 ? ki_less(ok, oi, ck, ci) : ki_less(ck, ci, ok, oi);
        }
      }
      rank += quad_xor1(rank);
      if (L == 4) rank += quad_xor2(rank);
      if (c < m && sl == 0 && rank < take) {
        if (e == 0) { g_L.lo_c[rank] = __longlong_as_double((long long)ck); g_L.lo_i[rank] = ci; }
        else { g_L.hi_c[take - 1 - rank] = __longlong_as_double((long long)ck); g_L.hi_i[take - 1 - rank] = ci; }
      }
    }
    tot_all += tot;
    if (threadIdx.x == 0) { g_L.n_lo = take; g_L.n_hi = take; }
    __syncthreads();
    NEAR_CLOCK(5);
    NEAR_COUNT(27);
  }
  if (threadIdx.x == 0) { g_L.nk = tot_all; g_L.S.near_nodes += n; }
  __syncthreads();
  if (NN) fnn_reduce(nb, nbi);
  TR();
}

// near_set without a record, as a call (the leader: the record's path, near_set_rec, runs inline before it).
template <int K, bool NN>
__device__ __noinline__ void near_set_scan(const Ctx& C, int t, const double* q, int excl) {
  [[clang::always_inline]] near_set<K, NN>(C, t, q, excl, false);
}

// --------------------------------------------------------------------------------------- edges
// Bit j set: joint j is revolute (RobotDev::rev as one register).
__device__ __forceinline__ unsigned rev_mask(const RobotDev* rb) {
  unsigned m = 0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) m |= (rb->rev[j] != 0 ? 1u : 0u) << j;
  return m;
}

// A double from lane l (two v_readlane: a wave-uniform value in scalar registers).
__device__ __forceinline__ double readlane_d(double v, int l) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Segment s of the interpolated edge st -> st + np * stp: the squared lengths behind its total / revolute / prismatic norms
// (compute_edge_cost_interpolation's per-segment terms, birrt_star.cpp:4162-4242; the joint sums in joint order).
__device__ __forceinline__ void seg_terms(unsigned rm, const double* st, const double* stp, int s, double& t, double& r,
                                          double& p) {
  t = 0.0; r = 0.0; p = 0.0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const double a = st[j] + s * stp[j];
    const double b = st[j] + (s + 1) * stp[j];
    const double d = (b - a) * (b - a);
    t += d * 1.0;
    const bool rv = (rm >> j) & 1u;
    r += rv ? d : 0.0;
    p += rv ? 0.0 : d;
  }
}
// ... and their square roots (the norms)
__device__ __forceinline__ void seg_norms(unsigned rm, const double* st, const double* stp, int s, double& t, double& r,
                                          double& p) {
  seg_terms(rm, st, stp, s, t, r, p);
  t = sqrt(t); r = sqrt(r); p = sqrt(p);
}

// connectNodesInterpolation + compute_edge_cost_interpolation (birrt_star.cpp:4380-4440, 4443-4526,
// 4162-4242) for E <= MAXE edges eg_start -> eg_target, base costs eg_base.  Segment norms in parallel,
// ordered sums per edge.  Fills eg_step, eg_end (the child configuration) and eg_cost.
__device__ void edge_costs(const Ctx& C, int E) {
  TR();
  PROF_BEGIN();
  const int np = g_L.S.n_pts;
  const RobotDev* rb = (&g_rb);
  if (threadIdx.x < E * NJ) {
    int e = threadIdx.x / NJ, j = threadIdx.x - e * NJ;
    double st = (g_L.eg_target[e][j] - g_L.eg_start[e][j]) / double(np);
    g_L.eg_step[e][j] = st;
    g_L.eg_end[e][j] = g_L.eg_start[e][j] + np * st;
  }
  __syncthreads();
  const unsigned rm = rev_mask(rb);
  for (int it = threadIdx.x; it < E * np; it += BLOCK) {
    const int e = it / np, s = it - e * np;
    double st[NJ], stp[NJ], t, r, p;
#pragma unroll
    for (int j = 0; j < NJ; ++j) { st[j] = g_L.eg_start[e][j]; stp[j] = g_L.eg_step[e][j]; }
    seg_norms(rm, st, stp, s, t, r, p);
    g_L.u.seg[e][s][0] = t;
    g_L.u.seg[e][s][1] = r;
    g_L.u.seg[e][s][2] = p;
  }
  __syncthreads();
  if (threadIdx.x < E * 3) {
    int e = threadIdx.x / 3, k = threadIdx.x - e * 3;
    // the segment norms in order (the reference's sum), all MAX_PTS loads issued before the first add, unconditionally
    // (a runtime-bound loop, or loads under `s < np`, waited one LDS round trip per segment; the words past np are
    // read and not added)
    double sg[MAX_PTS];
#pragma unroll
    for (int s = 0; s < MAX_PTS; ++s) sg[s] = g_L.u.seg[e][s][k];
    double acc = 0.0;
#pragma unroll
    for (int s = 0; s < MAX_PTS; ++s)
      if (s < np) acc += sg[s];
    g_L.eg_acc[e][k] = acc;
    g_L.eg_cost[e][k] = g_L.eg_base[e][k] + acc;
  }
  __syncthreads();
  PROF_END(P_COSTS);
  TR();
}

// edge_costs for E edges whose segment-norm sums the scout computed (acc[e], the same function of the same two
// configurations): only the interpolation step / end point are formed here.
__device__ void edge_costs_acc(int E, const double (*acc)[3]) {
  const int np = g_L.S.n_pts;
  if (threadIdx.x < E * NJ) {
    const int e = threadIdx.x / NJ, j = threadIdx.x - e * NJ;
    const double st = (g_L.eg_target[e][j] - g_L.eg_start[e][j]) / double(np);
    g_L.eg_step[e][j] = st;
    g_L.eg_end[e][j] = g_L.eg_start[e][j] + np * st;
  } else if (threadIdx.x >= 256 && threadIdx.x < 256 + E * 3) {
    const int i = threadIdx.x - 256, e = i / 3, k = i - e * 3;
    const double a = acc[e][k];
    g_L.eg_acc[e][k] = a;
    g_L.eg_cost[e][k] = g_L.eg_base[e][k] + a;
  }
  __syncthreads();
}

// isEdgeValid for the edges with eg_need[e] set: eg_first[e] = index of the first colliding configuration,
// or n_pts + 1 if the edge is free.  Each 32-configuration tile takes the next unchecked points of the
// unresolved needed edges in edge order, so an edge leaves the schedule at its first collision and every
// point before eg_first[e] has been checked.  With stop_first_valid the scan ends as soon as the first needed
// edge not in collision is fully checked (choose-parent and the connect near loop consume the edges in
// order and stop there); eg_first of the edges after it is then undefined.
// --------------------------------------------------------------------------------------- jobs (helpers)
#define TRACE(C, slot, v) \
  if ((C).Q.trace) __hip_atomic_store(&(C).Q.trace[slot], (int)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
__device__ __forceinline__ void st_agent(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_agent(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_agent(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Waits until this wave's vector-memory operations (stores, atomics) are performed.
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Granule = (job << 32) | 32-bit word (smp_plan.h JobBoard).
__device__ __forceinline__ unsigned long long granule(int seq, unsigned w) {
  return ((unsigned long long)(unsigned)seq << 32) | w;
}

// Skip mode (a job of more tiles than workers, JobLds::skip): before tile t of its second or later round, a worker
// reads the results of tiles [0, t) that have arrived (JobBoard::res, the leader's own included) -> each job edge's
// lowest known colliding point (J.first) and, for a stop-first-valid job (choose-parent, the connect near loop), the
// first edge known to be free (every tile of it arrived without a collision).  A configuration beyond its edge's
// known collision, or on an edge after a known free one, cannot change what the job's consumer reads (the first
// collision of each edge up to the first free one: eg_first of later edges is undefined, as in the local path), so
// it is not checked.  Returns true if no configuration of the tile is left; else J.tgrp / J.tord / J.first are the
// tile's TileOrder.  All threads.
__device__ __forceinline__ bool job_tile_skip(const Ctx& C, JobLds& J, int t, int seq) {
  const JobBoard* jb = C.Q.jb;
  const int np1 = uni(J.np1), ne = uni(J.E), ct = uni(J.ct);
  for (int u = threadIdx.x; u < t; u += BLOCK) {
    if (!J.rdone[u]) {
      const unsigned long long v = ld_agent(&jb->res[u]);
      if ((int)(v >> 32) == seq) { J.rmask[u] = (unsigned)v; J.rdone[u] = 1; }
    }
  }
  if (threadIdx.x < ne) J.first[threadIdx.x] = np1;
  __syncthreads();
  for (int u = threadIdx.x; u < t; u += BLOCK) {
    if (!J.rdone[u]) continue;
    unsigned m = J.rmask[u];
    while (m) {
      const int sl = u * ct + __builtin_ctz(m), k = sl / np1;
      m &= m - 1;
      atomicMin(&J.first[k], sl - k * np1);
    }
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    bool fr = false;
    if (J.sfv && lane < ne && (lane + 1) * np1 <= t * ct && J.first[lane] >= np1) {
      fr = true;
      for (int u = (lane * np1) / ct; u <= ((lane + 1) * np1 - 1) / ct; ++u)
        if (!J.rdone[u]) { fr = false; break; }
    }
    const unsigned long long fb = __ballot(fr);
    const int ff = fb ? __builtin_ctzll(fb) : (1 << 30);
    const int base = t * ct, nc = min(ct, J.nslots - base);
    bool live = false;
    if (lane < nc) {
      const int sl = base + lane, k = sl / np1, i = sl - k * np1;
      live = k <= ff && i <= J.first[k];
      J.tgrp[lane] = k;
      J.tord[lane] = live ? i : (1 << 30);
    }
    const unsigned long long lb = __ballot(live);
    if (lane == 0) J.tskip = lb == 0;
  }
  __syncthreads();
  return uni(J.tskip) != 0;
}

// Configurations of job tile t -> J.tq: slot s = job edge s / np1, point s % np1, configuration start + i * step
// (the leader's arithmetic).  Then the collision tile; returns the tile's collision mask in every thread.
// `seq` >= 0 in skip mode: configurations skipped by job_tile_skip report no collision.
__device__ __forceinline__ unsigned job_tile_mask(const Ctx& C, JobLds& J, int t, unsigned long long* prof = nullptr,
                                                  int seq = -1) {
  const int ct = uni(J.ct), base = t * ct, nc = min(ct, uni(J.nslots) - base);
  const bool sk = seq >= 0 && uni(J.skip) && t >= uni(C.Q.nworkers);
  if (sk && job_tile_skip(C, J, t, seq)) return 0u;
  if (threadIdx.x < nc * NJ) {
    const int c = threadIdx.x / NJ, j = threadIdx.x - c * NJ;
    const int sl = base + c, k = sl / J.np1, i = sl - k * J.np1;
    J.tq[c][j] = J.start[k][j] + i * J.step[k][j];
  }
  if (threadIdx.x < TILE_CT_MAX) J.T.coll[threadIdx.x] = 0;
  __syncthreads();
  const TileOrder order{J.tgrp, J.tord, J.first, false};
  collide_wide((&g_rb), C.sc, (&g_mc), ct, nc, J.tq, J.self, J.map, J.T, sk ? &order : nullptr, prof);
  unsigned m = 0;
  for (int c = 0; c < nc; ++c) m |= (J.T.coll[c] ? 1u : 0u) << c;
  __syncthreads();
  return m;
}

// job_tile_mask as a call, for the publisher's own and stolen tiles (rare while it has helpers): the collision tile's
// registers and code stay out of edge_validity and of the workgroups that inline it (the scouts).
__device__ __noinline__ unsigned job_tile_mask_out(const Ctx& C, JobLds& J, int t, int seq) {
  return job_tile_mask(C, J, t, nullptr, seq);
}

// Work the leader does while a collision job's tiles are checked by the helpers (see edge_validity).
enum { OV_NONE = 0, OV_NEAR_EXPAND = 1, OV_NN = 2, OV_NEAR_XN = 3 };
__device__ void overlap_work(const Ctx& C, int ov, int t);
// Takes the result of overlap_work `ov` if that is what the last job computed: counts its scanned nodes.
__device__ __forceinline__ bool take_spec(int ov) {
  const bool hit = uni(g_L.spec) == ov;
  __syncthreads();
  if (hit && threadIdx.x == 0) {
    (ov == OV_NN ? g_L.S.nn_nodes : g_L.S.near_nodes) += g_L.spec_cnt;
    g_L.spec = OV_NONE;
  }
  __syncthreads();
  return hit;
}

// Leader: publishes the needed edges of the batch as one job (every point of every needed edge); tile t belongs
// to worker (t + 1) % W, so the helpers take the first W - 1 tiles and the leader only tiles W - 1, 2W - 1, ...
// While they are checked, the leader does `ov` (overlap_work), then its own tiles, then collects the helpers'
// tile results and reduces them to the first collision of each edge (eg_first).  A helper's tile that does not
// arrive within 8 us of the last progress is checked by the leader itself (a duplicate result is identical, so
// no claim is needed).
__device__ __forceinline__ void edge_validity_job(const Ctx& C, int E, int pslot, int ov, int ovt, bool sfv) {
  JobBoard* jb = C.Q.jb;
  auto& J = g_L.u.job;
  const int np1 = g_L.S.n_pts + 1;
  const int W = max(1, C.Q.nworkers);  // (a workgroup without helpers takes every tile itself)
  if (threadIdx.x < 64) {
    const int e = threadIdx.x;
    const bool need = e < E && g_L.eg_need[e] && g_L.eg_hit[e] < 0;  // edges the scout checked are not published
    const unsigned long long m = __ballot(need);
    const int k = __popcll(m & ((1ull << e) - 1));
    if (need) J.emap[k] = e;
    if (e == 0) {
      const int ne = __popcll(m);
      J.E = ne;
      J.np1 = np1;
      J.nslots = ne * np1;
      J.ct = job_tile_ct(ne * np1, W, C.Q.tile_ct);
      J.ntiles = (ne * np1 + J.ct - 1) / J.ct;
      J.self = g_L.S.self; J.map = g_L.S.map;
      J.seq = ++g_L.job_seq;
#ifdef SMP_NO_SKIP
      J.skip = 0;
#else
      J.skip = J.ntiles > W;  // more tiles than workers: later rounds skip what earlier ones decided
#endif
      J.sfv = J.skip && sfv;
    }
  }
  if (threadIdx.x < E) g_L.eg_first[threadIdx.x] = np1;
  __syncthreads();
  const int ne = uni(J.E), nt = uni(J.ntiles), seq = uni(J.seq), ct = uni(J.ct);
  if (ne == 0) {
    // nothing to check (the scout's record had every edge): no job whose latency the scan would hide, and its
    // result may not be needed (OV_NEAR_EXPAND when the expand edge collides) -- the caller scans if it must
    overlap_work(C, OV_NONE, ovt);
    return;
  }
  const unsigned long long tj0 = threadIdx.x == 0 ? wall_clock64() : 0;
  for (int it = threadIdx.x; it < ne * NJ; it += BLOCK) {
    const int k = it / NJ, j = it - k * NJ, e = J.emap[k];
    J.start[k][j] = g_L.eg_start[e][j];
    J.step[k][j] = g_L.eg_step[e][j];
  }
  for (int t = threadIdx.x; t < nt; t += BLOCK) J.rdone[t] = 0;
  if (threadIdx.x < ne) J.first[threadIdx.x] = np1;
  __syncthreads();
  // payload granules (no flag and no drain: each granule carries the job number)
  for (int i = threadIdx.x; i < 1 + 32 * ne; i += BLOCK) {
    unsigned w;
    if (i == 0) {
      w = (unsigned)ne | (unsigned)np1 << 8 | (unsigned)(J.self != 0) << 16 | (unsigned)(J.map != 0) << 17 |
          (unsigned)J.skip << 19 | (unsigned)J.sfv << 20 | (unsigned)__builtin_ctz((unsigned)J.ct) << 21;
    } else {
      const int m = i - 1, k = m >> 5, r = m & 31, j = (r & 15) >> 1;
      const unsigned long long bits = (unsigned long long)__double_as_longlong(r < 16 ? J.start[k][j] : J.step[k][j]);
      w = (r & 1) ? (unsigned)(bits >> 32) : (unsigned)bits;
    }
    st_agent(&jb->pay[i], granule(seq, w));
  }
#ifdef SMP_JOB_PROF
  if (threadIdx.x == 0) st_agent(&jb->dbg[0], wall_clock64());
#endif
  PROF_BEGIN();
  if (threadIdx.x == 0) { g_L.S.prof[P_TFK] += _pt - tj0; g_L.S.prof[P_TTEST]++; }  // job publication
  TR();
  if (threadIdx.x == 0) g_L.in_job = 1;  // the helpers are on this job's tiles: overlap scans stay local
  __syncthreads();
  overlap_work(C, ov, ovt);
  if (threadIdx.x == 0) g_L.in_job = 0;
  TR();
  // the leader's own tiles (in skip mode published too: the helpers' skip decisions read every earlier tile)
  const bool skip = uni(J.skip) != 0;
  for (int t = W - 1; t < nt; t += W) {
    const unsigned m = job_tile_mask_out(C, J, t, skip ? seq : -1);
    if (threadIdx.x == 0) {
      J.rmask[t] = m;
      J.rdone[t] = 1;
      if (skip) st_agent(&jb->res[t], granule(seq, m));
    }
  }
  __syncthreads();
  const unsigned long long tj1 = threadIdx.x == 0 ? wall_clock64() : 0;
  if (threadIdx.x == 0) g_L.S.prof[P_TCHAIN] += tj1 - _pt;  // the leader's own tiles
  // collect the helpers' results (wave 0 polls the result granules; block-level decision double-buffered)
  unsigned long long t_prog = tj1, t_wait = tj1;
  int last_left = 1 << 30;
  for (int k = 0;; k ^= 1) {
    if (threadIdx.x < 64) {
      int left = 0;
      for (int t = threadIdx.x; t < nt; t += 64) {
        if (J.rdone[t]) continue;
        const unsigned long long v = ld_agent(&jb->res[t]);
        if ((int)(v >> 32) == seq) { J.rmask[t] = (unsigned)v; J.rdone[t] = 1; }
        else ++left;
      }
      left = __ockl_wfred_add_i32(left);  // (DPP reduction: a shuffle tree costs six LDS-latency bpermutes)
      if (threadIdx.x == 0) {
        const unsigned long long now = wall_clock64();
        if (left != last_left) { last_left = left; t_prog = now; }
        int st = left == 0 ? 1 : (now - t_prog > 800ull ? 2 : 0);
        if (st != 1 && now - t_wait > 200000000ull) {  // 2 s: a job never takes that long -- fail, never hang
          g_L.S.status = -5;
          g_L.S.phase = 2;
          g_L.S.prof[28] = (unsigned long long)left;
          g_L.S.prof[29] = (unsigned long long)nt;
          g_L.S.prof[31] = (unsigned long long)seq;
          st = 1;
        }
        J.go[k] = st;
      }
    }
    __syncthreads();
    const int go = uni(J.go[k]);
    if (go == 1) break;
    if (go == 2) {
      // check the first missing tile here
      if (threadIdx.x < 64) {
        int cand = 1 << 30;
        for (int t = threadIdx.x; t < nt; t += 64)
          if (!J.rdone[t]) { cand = t; break; }
        cand = __ockl_wfred_min_i32(cand);
        if (threadIdx.x == 0) J.steal = cand < nt ? cand : -1;
      }
      __syncthreads();
      const int t = uni(J.steal);
      if (t >= 0) {
        const unsigned m = job_tile_mask_out(C, J, t, -1);
        if (threadIdx.x == 0) { J.rmask[t] = m; J.rdone[t] = 1; }
      }
      if (threadIdx.x == 0) t_prog = wall_clock64();
      __syncthreads();
      continue;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  TR();
  if (threadIdx.x == 0) g_L.S.prof[P_TCENTRE] += pclk() - tj1;  // waiting for helpers' tiles
  // first collision per job edge from the tile masks
  for (int t = threadIdx.x; t < nt; t += BLOCK) {
    unsigned m = J.rmask[t];
    while (m) {
      const int c = __builtin_ctz(m);
      m &= m - 1;
      const int sl = t * ct + c, kk = sl / np1;
      atomicMin(&J.first[kk], sl - kk * np1);
    }
  }
  __syncthreads();
  if (threadIdx.x < ne) g_L.eg_first[J.emap[threadIdx.x]] = J.first[threadIdx.x];
  PROF_END(P_TILES);
  if (threadIdx.x == 0) {
    g_L.S.prof[pslot] += pclk() - _pt;
    g_L.S.prof[P_NTILES] += nt;
    g_L.S.prof[pslot + 8] += J.nslots;
  }
  __syncthreads();
}

// --------------------------------------------------------------------------------------- distributed scans
// A nearest or near scan of a large tree (scan_split: at least QueryDev::scan_min nodes, eight or more workers, no
// collision job in flight) is split into P = min(workers, SCAN_P) slices of equal size: the workgroup publishes a scan
// job (header + the query configuration, range, excluded id and radius: 33 payload words, within the helpers' first
// poll), scans slice 0 itself, and collects the helpers' partial results (data-tagged granules of JobBoard::sres).
// A slice whose result does not arrive within 20 us of the last progress is scanned here (a duplicate is identical).
// The merge is exact: nearest takes the (distance, id) minimum of the slices -- the slices partition the range, and
// each slice's answer is its first strict minimum; the near lists take every entry whose rank over all slices' lists
// is below SCAN_K (an entry beyond a slice's K-th cannot rank below K: K entries are ahead of it).
constexpr unsigned SCAN_HDR = 1u | 1u << 18;  // edge-count field 1 (33 payload words), scan job bit
// SMP_SCAN_PROF builds (tools/scan_probe.py): clocks of the distributed scans, summed over every scan of the leader and
// the scouts, read by smp_debug_scanprof: [0] scans, [1] write-back + publication, [2] own slice, [3] collection,
// [4] merge, [5] stolen slices, [6] collection rounds, [7] helper slices, [8] helper pickup (publication -> acquire),
// [9] helper acquire, [10] helper slice, [11] publication -> helper result stored, [12] near scans, [13] their
// collection, [14] participants, [15] nodes, [16] near scans' own slice, [17] near merge, [18] near helper slices,
// [19] their slice clocks
#ifdef SMP_SCAN_PROF
__device__ unsigned long long g_scanprof[24];
#define SCANPROF_ADD(k, v) atomicAdd(&g_scanprof[k], (unsigned long long)(v))
#else
#define SCANPROF_ADD(k, v)
#endif
constexpr unsigned long long SCAN_WAIT = 2000;  // device-clock ticks (20 us) without progress before stealing a slice

// Slice w of [i0, n) over P participants, in index order, 64-node multiples.  The publisher's slice 0 is a fraction
// 1 / 2^ps0 of a helper's (QueryDev::scan_ps0): it publishes first and collects and merges after its slice, so equal
// slices would make it the last to finish.
__device__ __forceinline__ void scan_range(int i0, int n, int P, int w, int ps0, int* lo, int* hi) {
  const int m = n - i0;
  // helpers' chunk c with c / 2^ps0 + (P - 1) c >= m
  int chunk = (int)(((long long)m << ps0) / (((long long)(P - 1) << ps0) + 1)) + 1;
  chunk = (chunk + 63) & ~63;
  const int c0 = ((chunk >> ps0) + 63) & ~63;
  *lo = w == 0 ? i0 : min(n, i0 + c0 + (w - 1) * chunk);
  *hi = w == 0 ? min(n, i0 + c0) : min(n, *lo + chunk);
}

// Publishes scan job `seq` (all threads).
__device__ void scan_publish(const Ctx& C, int seq, int near, int t, const double* q, int i0, int n, int excl, double r,
                             int P) {
  JobBoard* jb = C.Q.jb;
  const int i = threadIdx.x;
  if (i < SCAN_WORDS) {
    unsigned w = 0;
    if (i == 0) {
      w = SCAN_HDR | (unsigned)(near != 0) << 19 | (unsigned)t << 20 | (unsigned)(near == 2) << 21;
    } else if (i <= 16) {
      const unsigned long long b = (unsigned long long)__double_as_longlong(q[(i - 1) >> 1]);
      w = ((i - 1) & 1) ? (unsigned)(b >> 32) : (unsigned)b;
    } else if (i == 17) {
      w = (unsigned)i0;
    } else if (i == 18) {
      w = (unsigned)n;
    } else if (i == 19) {
      w = (unsigned)excl;
    } else if (i == 20 || i == 21) {
      const unsigned long long b = (unsigned long long)__double_as_longlong(r);
      w = i == 21 ? (unsigned)(b >> 32) : (unsigned)b;
    } else if (i == 22) {
      w = (unsigned)P;
    }
    st_agent(&jb->spay[i], granule(seq, w));
  }
}

// Participant w's slice of a scan, its result as granules of sres[w] (helper) or into the merge area (workgroup).
// INL: the helpers' form (slices inlined, scan_helper).
template <bool INL = false>
__device__ void scan_slice(const Ctx& C, int near, int t, const double* q, int i0, int n, int excl, double r, int P, int w,
                           ScanLds& X) {
  const gcdptr tq = uni_gptr(C.Q.tr[t].q), tc = uni_gptr(C.Q.tr[t].cost);
  const int cap = uni(__hip_atomic_load(&C.Q.st->cap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  int lo, hi;
  scan_range(i0, n, P, w, C.Q.scan_ps0, &lo, &hi);
  if (INL) {
    // the fp32 prefilter (the tree's qf copy): half the bytes per node
    const float* tqf = C.Q.tr[t].qf;
    if (near == 2) slice_near_inl<true, true>(tq, tc, cap, lo, hi, q, excl, r, X, tqf);
    else if (near) slice_near_inl<false, true>(tq, tc, cap, lo, hi, q, excl, r, X, tqf);
    else slice_nn_body32(tq, tqf, cap, lo, hi, q, X);
    return;
  }
  if (near == 2) slice_near<true>(tq, tc, cap, lo, hi, q, excl, r, X);
  else if (near) slice_near<false>(tq, tc, cap, lo, hi, q, excl, r, X);
  else slice_nn(tq, cap, lo, hi, q, X);
}

// Helper side of a scan job already in J.words (seq): worker w is participant W - w (smp_plan.h SCAN_P); its slice, then
// the result granules.
__device__ __forceinline__ void scan_helper(const Ctx& C, JobLds& J, int worker, int seq) {
  const unsigned hdr = J.words[0];
  const int near = ((hdr >> 21) & 1) ? 2 : (int)((hdr >> 19) & 1), t = (hdr >> 20) & 1;
  double q[NJ];
  for (int j = 0; j < NJ; ++j) q[j] = __hiloint2double((int)J.words[2 + 2 * j], (int)J.words[1 + 2 * j]);
  const int i0 = (int)J.words[17], n = (int)J.words[18], excl = (int)J.words[19], P = (int)J.words[22];
  const double r = __hiloint2double((int)J.words[21], (int)J.words[20]);
  const int w = C.Q.nworkers - worker;
  if (w < 1 || w >= P) return;
#ifdef SMP_SCAN_PROF
  const unsigned long long hp0 = wall_clock64();
#endif
  // tree words stored by the leader since this CU last cached them: drop stale copies (consumer form: one acquire,
  // its wait, a barrier, then plain loads)
  if (threadIdx.x < 64) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    drain();
  }
  __syncthreads();
#ifdef SMP_SCAN_PROF
  const unsigned long long hp1 = wall_clock64();
#endif
  ScanLds& X = J.scan;
  scan_slice<true>(C, near, t, q, i0, n, excl, r, P, w, X);
#ifdef SMP_SCAN_PROF
  if (threadIdx.x == 0) {
    const unsigned long long hp2 = wall_clock64(), pub = ld_agent(&C.Q.jb->dbg[8]);
    SCANPROF_ADD(7, 1); SCANPROF_ADD(8, hp0 - pub); SCANPROF_ADD(9, hp1 - hp0); SCANPROF_ADD(10, hp2 - hp1);
    SCANPROF_ADD(11, hp2 - pub);
    if (near) { SCANPROF_ADD(18, 1); SCANPROF_ADD(19, hp2 - hp1); }
  }
#endif
  unsigned long long* out = C.Q.jb->sres[w];
  if (!near) {
    if (threadIdx.x == 0) {
      st_agent(&out[0], granule(seq, (unsigned)X.wk[0]));
      st_agent(&out[1], granule(seq, (unsigned)(X.wk[0] >> 32)));
      st_agent(&out[2], granule(seq, (unsigned)X.wi[0]));
    }
  } else {
    // fixed places: entry e of side s in granules 2 + 3 * (s * SCAN_K + e) .. + 2, so that the collector can
    // load a whole result at once
    const int take = X.take;
    const int i = threadIdx.x;
    if (i == 0) st_agent(&out[0], granule(seq, (unsigned)X.cnt));
    if (i == 1) st_agent(&out[1], granule(seq, (unsigned)take));
    if (i < 6 * take) {
      const int side = i >= 3 * take, j = i - side * 3 * take, e = j / 3, f = j - 3 * e;
      const unsigned long long k = side ? X.hk[e] : X.lk[e];
      const int id = side ? X.hi[e] : X.li[e];
      const unsigned v = f == 0 ? (unsigned)k : f == 1 ? (unsigned)(k >> 32) : (unsigned)id;
      st_agent(&out[2 + 3 * side * SCAN_K + j], granule(seq, v));
    }
    // a fused scan's nearest node after the near lists: key halves, id
    if (near == 2 && i >= 256 && i < 259) {
      const int f = i - 256;
      const unsigned v = f == 0 ? (unsigned)X.wk[0] : f == 1 ? (unsigned)(X.wk[0] >> 32) : (unsigned)X.wi[0];
      st_agent(&out[2 + 6 * SCAN_K + f], granule(seq, v));
    }
  }
  __syncthreads();
}

// Slot w of the merge area from a slice result in X (all threads).
__device__ __forceinline__ void merge_put(MergeLds& M, const ScanLds& X, int near, int w) {
  if (near != 1) {  // nearest, or a fused scan's nearest part
    if (threadIdx.x == 0) { M.nk[w] = X.wk[0]; M.ni[w] = X.wi[0]; }
  }
  if (near) {
    const int take = X.take;
    if (threadIdx.x < SCAN_K) {
      const int e = threadIdx.x;
      if (e < take) {
        M.kl[0][w][e] = (unsigned)X.lk[e]; M.kh[0][w][e] = (unsigned)(X.lk[e] >> 32); M.id[0][w][e] = X.li[e];
        M.kl[1][w][e] = (unsigned)X.hk[e]; M.kh[1][w][e] = (unsigned)(X.hk[e] >> 32); M.id[1][w][e] = X.hi[e];
      }
    }
    if (threadIdx.x == 0) { M.len[w] = take; M.cnt[w] = X.cnt; }
  }
  if (threadIdx.x == 0) M.done[w] = 1;
}

// Publishes a scan of [i0, n) over P participants, scans slice 0, collects (or steals) the other slices into
// g_L.sc.m.  All threads.
__device__ void scan_run(const Ctx& C, int near, int t, const double* q, int i0, int n, int excl, double r, int P) {
  MergeLds& M = g_L.sc.m;
  ScanLds& X = g_L.sc.s;
  __syncthreads();
  const int seq = uni(g_L.job_seq) + 1;
  if (threadIdx.x < SCAN_P) { M.done[threadIdx.x] = 0; M.bad[threadIdx.x] = 0; }
  __syncthreads();
  if (threadIdx.x == 0) { g_L.job_seq = seq; M.ndone = 0; }
#ifdef SMP_SCAN_PROF
  const unsigned long long sp0 = wall_clock64();
#endif
  // the helpers read the tree through their own CUs and XCDs: the tree stores (this workgroup's, or the leader's on
  // this XCD for a scout) are written back before the job is published (MI355X_MICROARCH.md producer form)
  drain();
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain();
  }
  __syncthreads();
#ifdef SMP_SCAN_PROF
  const unsigned long long sp1 = wall_clock64();
  if (threadIdx.x == 0) st_agent(&C.Q.jb->dbg[8], sp1);
#endif
  TR();
  scan_publish(C, seq, near, t, q, i0, n, excl, r, P);
  scan_slice<true>(C, near, t, q, i0, n, excl, r, P, 0, X);
  TR();
  merge_put(M, X, near, 0);
  __syncthreads();
#ifdef SMP_SCAN_PROF
  const unsigned long long sp2 = wall_clock64();
  int sp_rounds = 0, sp_steals = 0;
#endif
  const JobBoard* jb = C.Q.jb;
  unsigned long long t_prog = wall_clock64();
  int last_done = 0;
  // One collection round loads every granule of every outstanding result at once (up to 4 per thread per pass:
  // independent loads, one round trip), then keeps the results whose needed granules all carry this job's number.
  // (a fused scan's result: the near lists, then its nearest node's 3 granules)
  constexpr int NG = 2 + 6 * SCAN_K;
  const int per = near ? NG + (near == 2 ? 3 : 0) : 3;
  const int total = (P - 1) * per;
  for (int k = 0;; k ^= 1) {
    for (int base = 0; base < total; base += 4 * BLOCK) {
      unsigned val[4];
      unsigned okm = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int g = base + u * BLOCK + (int)threadIdx.x;
        val[u] = 0;
        if (g < total) {
          const int w = 1 + g / per;
          if (!M.done[w]) {
            const unsigned long long v = ld_agent(&jb->sres[w][g - (w - 1) * per]);
            val[u] = (unsigned)v;
            if ((int)(v >> 32) == seq) okm |= 1u << u;
          }
        }
      }
      // nearest values and near headers (every granule needed)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int g = base + u * BLOCK + (int)threadIdx.x;
        if (g < total) {
          const int w = 1 + g / per, i = g - (w - 1) * per;
          if (!M.done[w] && i < (near ? 2 : 3)) {
            M.hv[w][i] = val[u];
            if (!((okm >> u) & 1u)) M.bad[w] = 1;
          }
          if (near == 2 && !M.done[w] && i >= NG) {
            M.hn[w][i - NG] = val[u];
            if (!((okm >> u) & 1u)) M.bad[w] = 1;
          }
        }
      }
      if (near) {
        __syncthreads();
        // near entries: needed below the result's take
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int g = base + u * BLOCK + (int)threadIdx.x;
          if (g < total) {
            const int w = 1 + g / per, i = g - (w - 1) * per;
            if (!M.done[w] && i >= 2 && i < NG) {
              const int j = i - 2, side = j >= 3 * SCAN_K ? 1 : 0, jj = j - side * 3 * SCAN_K, e = jj / 3, f = jj - 3 * e;
              if (e < min((int)M.hv[w][1], SCAN_K)) {
                if (!((okm >> u) & 1u)) M.bad[w] = 1;
                else if (f == 0) M.kl[side][w][e] = val[u];
                else if (f == 1) M.kh[side][w][e] = val[u];
                else M.id[side][w][e] = (int)val[u];
              }
            }
          }
        }
      }
    }
    __syncthreads();
    {
      const int w = threadIdx.x;
      if (w >= 1 && w < P && !M.done[w]) {
        if (!M.bad[w]) {
          if (near) {
            M.len[w] = min((int)M.hv[w][1], SCAN_K);
            M.cnt[w] = (int)M.hv[w][0];
          } else {
            M.nk[w] = (unsigned long long)M.hv[w][1] << 32 | M.hv[w][0];
            M.ni[w] = (int)M.hv[w][2];
          }
          if (near == 2) {
            M.nk[w] = (unsigned long long)M.hn[w][1] << 32 | M.hn[w][0];
            M.ni[w] = (int)M.hn[w][2];
          }
          M.done[w] = 1;
          atomicAdd(&M.ndone, 1);
        }
        M.bad[w] = 0;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long now = wall_clock64();
      const int nd = M.ndone;
      if (nd != last_done) { last_done = nd; t_prog = now; }
      // a slice missing SCAN_WAIT after the last progress is scanned here (stealing guarantees progress: no timeout
      // status is needed, and a slow scan is not an error)
      int st = nd >= P - 1 ? 1 : (now - t_prog > SCAN_WAIT ? 2 : 0);
      if (st == 2) {
        int w = 1;
        while (w < P && M.done[w]) ++w;
        M.steal = w < P ? w : -1;
        if (M.steal < 0) st = 1;
      }
      M.go[k] = st;
    }
    __syncthreads();
    const int go = uni(M.go[k]);
#ifdef SMP_SCAN_PROF
    ++sp_rounds;
#endif
    if (go == 1) break;
    TR();
    if (go == 2) {
      const int w = uni(M.steal);
      scan_slice<true>(C, near, t, q, i0, n, excl, r, P, w, X);
      merge_put(M, X, near, w);
      if (threadIdx.x == 0) { M.ndone++; t_prog = wall_clock64(); }
#ifdef SMP_SCAN_PROF
      ++sp_steals;
#endif
      __syncthreads();
      continue;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  __syncthreads();
#ifdef SMP_SCAN_PROF
  if (threadIdx.x == 0) {
    const unsigned long long sp3 = wall_clock64();
    SCANPROF_ADD(0, 1); SCANPROF_ADD(1, sp1 - sp0); SCANPROF_ADD(2, sp2 - sp1); SCANPROF_ADD(3, sp3 - sp2);
    SCANPROF_ADD(5, sp_steals); SCANPROF_ADD(6, sp_rounds); SCANPROF_ADD(14, P); SCANPROF_ADD(15, n - i0);
    if (near) { SCANPROF_ADD(12, 1); SCANPROF_ADD(13, sp3 - sp2); SCANPROF_ADD(16, sp2 - sp1); }
    g_L.spc_t = sp3;
  }
#endif
}

// The (distance key, id) minimum of the P slices' nearest results (each wave computes it: lane w reads slice w; a serial
// loop would wait on one LDS read per slice).
__device__ __forceinline__ void merge_nearest(const MergeLds& M, int P, unsigned long long& bk, int& bi) {
  const int w = lane_id();
  const unsigned long long k = w < P ? M.nk[w] : ~0ull;
  const int i = w < P ? M.ni[w] : 0x7fffffff;
  bk = __ockl_wfred_min_u64(k);
  bi = __ockl_wfred_min_i32(k == bk ? i : 0x7fffffff);
}
__device__ int nearest_dist(const Ctx& C, int t, const double* q, int i0, int n, double* d_out) {
  const int P = scan_parts(C, 0, n - i0);
  scan_run(C, 0, t, q, i0, n, -1, 0.0, P);
  const MergeLds& M = g_L.sc.m;
  unsigned long long bk;
  int bi;
  merge_nearest(M, P, bk, bi);
  __syncthreads();
#ifdef SMP_SCAN_PROF
  if (threadIdx.x == 0) SCANPROF_ADD(4, wall_clock64() - g_L.spc_t);
#endif
  *d_out = __longlong_as_double((long long)bk);
  return bi;
}

// near_set's outputs (g_L.nk, n_lo, n_hi, lo_*, hi_*) from the merged slices: the lowest SCAN_K (cost, id) entries of
// the P ascending low lists and the highest SCAN_K of the P descending high lists, by a tournament -- wave 0 the low
// side, wave 1 the high side, lane w the head of participant w's list; each round one wave minimum (maximum) of the
// heads, whose lane advances.  The slices partition the range, so ids are distinct and every round has one winner.
__device__ void near_set_dist(const Ctx& C, int t, const double* q, int excl, bool nn) {
  const int n = uni(g_L.S.n[t]);
  const int P = scan_parts(C, 1, n);
  scan_run(C, nn ? 2 : 1, t, q, 0, n, excl, g_L.S.near_r, P);
  TR();
  const MergeLds& M = g_L.sc.m;
  static_assert(SCAN_PNEAR <= 64, "one lane per list");
  int tot = 0, take = 0;
  if (threadIdx.x < 128) {
    const int side = (int)threadIdx.x >> 6, w = lane_id();
    tot = __ockl_wfred_add_i32(w < P ? M.cnt[w] : 0);  // (lane-parallel: a serial sum waits on one LDS read per list)
    take = min(SCAN_K, tot);
    const int len = w < P ? M.len[w] : 0;
    const unsigned long long KN = side ? 0ull : ~0ull;
    const int IN = side ? -1 : 0x7fffffff;
    // per round: the extreme head by two 32-bit wave reductions (high word, then the low word among the lanes holding
    // that high word: DPP min / max steps on 32 bits, cheaper than one 64-bit reduction), the id reduction only when
    // two heads hold equal keys; each lane has its list's next entry loaded ahead, so a winning lane's new head is in
    // registers when the next round starts (a threshold merge -- candidates up to the extreme of the full lists' last
    // entries, ranked by counting -- measured slower: 7.5 -> 10.8 us per merge at 1e5 iterations)
    int p = 0;
    unsigned long long k = len > 0 ? merge_key(M, side, w, 0) : KN;
    int id = len > 0 ? M.id[side][w][0] : IN;
    unsigned long long kn = len > 1 ? merge_key(M, side, w, 1) : KN;
    int idn = len > 1 ? M.id[side][w][1] : IN;
    for (int r = 0; r < take; ++r) {
      const unsigned kh = (unsigned)(k >> 32), kl = (unsigned)k;
      unsigned mh, ml;
      if (side) { mh = __ockl_wfred_max_u32(kh); ml = __ockl_wfred_max_u32(kh == mh ? kl : 0u); }
      else { mh = __ockl_wfred_min_u32(kh); ml = __ockl_wfred_min_u32(kh == mh ? kl : ~0u); }
      const unsigned long long mk = (unsigned long long)mh << 32 | ml;
      const unsigned long long tie = __ballot(k == mk);
      int mi = id;
      if (__popcll(tie) > 1)
        mi = side ? __ockl_wfred_max_i32(k == mk ? id : -1) : __ockl_wfred_min_i32(k == mk ? id : 0x7fffffff);
      if (k == mk && id == mi) {
        if (!side) { g_L.lo_c[r] = __longlong_as_double((long long)mk); g_L.lo_i[r] = mi; }
        else { g_L.hi_c[take - 1 - r] = __longlong_as_double((long long)mk); g_L.hi_i[take - 1 - r] = mi; }
        ++p;
        k = kn; id = idn;
        if (p + 1 < len) { kn = merge_key(M, side, w, p + 1); idn = M.id[side][w][p + 1]; }
        else { kn = KN; idn = IN; }
      }
    }
  }
  TR();
  if (threadIdx.x == 0) {
    g_L.nk = tot; g_L.n_lo = take; g_L.n_hi = take; g_L.S.near_nodes += n;
  }
  if (nn && threadIdx.x < 64) {  // the fused scan's nearest node: the (distance key, id) minimum of the slices
    unsigned long long bk;
    int bi;
    merge_nearest(M, P, bk, bi);
    if (threadIdx.x == 0) { g_L.fnn_d = __longlong_as_double((long long)bk); g_L.fnn_id = bi; }
  }
  __syncthreads();
#ifdef SMP_SCAN_PROF
  if (threadIdx.x == 0) { SCANPROF_ADD(4, wall_clock64() - g_L.spc_t); SCANPROF_ADD(17, wall_clock64() - g_L.spc_t); }
#endif
}

#ifndef SMP_HELPER_SLEEP
#define SMP_HELPER_SLEEP 2  // s_sleep units (64 clocks) between an idle helper's polls of its job board
#endif
#ifndef SMP_POLL_N
#define SMP_POLL_N 128  // payload granules read by an idle helper's poll (64 per wave-0 load instruction)
#endif
// Helper workgroup w (1 .. W-1): wave 0 polls the first SMP_POLL_N payload granules of its board's collision job (two
// per lane: a header and three edges, so the pre-solution scouts' expand + connect jobs arrive within the poll) and the
// scan job's granules (one per lane); a job is taken once every granule it needs carries its header's job number (a
// longer collision payload takes one more read).  A new scan job goes first -- its publisher collects the slices before
// its collision job's tiles (overlap_work) -- and this helper scans its slice if it is a participant (scan_helper).  Then
// tiles w - 1, w - 1 + W, ... of a collision job, each result stored as one granule.  Leaves on the stop flag, or after
// two idle seconds should the leader never start.
__device__ __noinline__ void helper_main(const Ctx& C, int hidx, JobLds& J) {
  JobBoard* jb = C.Q.jb;
  const int w = 1 + hidx, W = C.Q.nworkers;
  int last = 0, last_scan = 0;
  unsigned long long t_last = wall_clock64();
  constexpr int PU = SMP_POLL_N / 64;
  static_assert(PU >= 1 && PU * 64 <= JOB_WORDS, "poll width");
  static_assert(SCAN_WORDS <= 64, "a scan payload is one granule per lane");
  for (int k = 0;; k ^= 1) {
    // 0 = nothing new, > 0 = collision job number complete in J.words, -1 = leave, -2 = collision payload longer than
    // the poll, -3 = scan job complete in J.words
    if (threadIdx.x < 64) {
      unsigned long long v[PU];
#pragma unroll
      for (int u = 0; u < PU; ++u) v[u] = ld_agent(&jb->pay[u * 64 + threadIdx.x]);
      const unsigned long long sv = ld_agent(&jb->spay[threadIdx.x]);
      const unsigned stag = __builtin_amdgcn_readfirstlane((unsigned)(sv >> 32));
      const unsigned tag0 = __builtin_amdgcn_readfirstlane((unsigned)(v[0] >> 32));
      const unsigned hdr = __builtin_amdgcn_readfirstlane((unsigned)v[0]);
      int go = 0;
      if (stag != 0 && (int)stag != last_scan) {
        const bool stale = (int)threadIdx.x < SCAN_WORDS && (unsigned)(sv >> 32) != stag;
        if (!__ballot(stale)) {
          if ((int)threadIdx.x < SCAN_WORDS) J.words[threadIdx.x] = (unsigned)sv;
          go = -3;
        }
      }
      if (go == 0 && tag0 != 0 && (int)tag0 != last) {
        const int nw = 1 + 32 * (int)(hdr & 255);
        bool stale = false;
#pragma unroll
        for (int u = 0; u < PU; ++u) stale |= u * 64 + (int)threadIdx.x < nw && (unsigned)(v[u] >> 32) != tag0;
        if (!__ballot(stale)) {
#pragma unroll
          for (int u = 0; u < PU; ++u)
            if (u * 64 + (int)threadIdx.x < nw) J.words[u * 64 + threadIdx.x] = (unsigned)v[u];
          go = nw <= PU * 64 ? (int)tag0 : -2;
        }
      }
      if (threadIdx.x == 0) {
        if (go == 0 && (ld_agent(&jb->stop) || wall_clock64() - t_last > 200000000ull)) go = -1;  // 2 s idle
        J.go[k] = go;
        J.seq = go == -3 ? (int)stag : (int)tag0;
      }
    }
    __syncthreads();
    const int go = uni(J.go[k]);
    if (go == -1) break;
    if (go == 0) {
      __builtin_amdgcn_s_sleep(SMP_HELPER_SLEEP);
      continue;
    }
    const int seq = uni(J.seq);
    if (go == -3) {  // scan job: this helper's slice, if it is a participant
      scan_helper(C, J, w, seq);
      last_scan = seq;
      t_last = wall_clock64();
      continue;
    }
    const unsigned hdr = J.words[0];
    const int ne = min((int)(hdr & 255), MAXE), nw = 1 + 32 * ne;
    if (go == -2) {
      // the rest of a long payload (one read; granules not yet current abandon the job to the next poll, which
      // sees it again since `last` is unchanged)
      int bad = 0;
      for (int i = PU * 64 + threadIdx.x; i < nw; i += BLOCK) {
        const unsigned long long v = ld_agent(&jb->pay[i]);
        if ((int)(v >> 32) != seq) bad = 1;
        J.words[i] = (unsigned)v;
      }
      if (threadIdx.x == 0) J.left = 0;
      __syncthreads();
      if (bad) J.left = 1;
      __syncthreads();
      if (uni(J.left)) continue;
    }
    for (int it = threadIdx.x; it < ne * 2 * NJ; it += BLOCK) {
      const int kk = it / (2 * NJ), r = it - kk * 2 * NJ;  // r < NJ: start[j], else step[j - NJ]
      const int wi = 1 + 32 * kk + 2 * r;
      const double d = __hiloint2double((int)J.words[wi + 1], (int)J.words[wi]);
      if (r < NJ) J.start[kk][r] = d; else J.step[kk][r - NJ] = d;
    }
    if (threadIdx.x == 0) {
      J.E = ne;
      J.np1 = (int)((hdr >> 8) & 255);
      J.self = (hdr >> 16) & 1;
      J.map = (hdr >> 17) & 1;
      J.skip = (hdr >> 19) & 1;
      J.sfv = (hdr >> 20) & 1;
      J.nslots = ne * J.np1;
      J.ct = 1 << ((hdr >> 21) & 3);
      J.ntiles = (J.nslots + J.ct - 1) / J.ct;
    }
    if (hdr & (1u << 19))
      for (int t = threadIdx.x; t < JOB_TILES; t += BLOCK) J.rdone[t] = 0;
    __syncthreads();
    last = seq;
    const int nt = uni(J.ntiles);
#ifdef SMP_JOB_PROF
    if (threadIdx.x == 0 && w - 1 < nt) {
      const unsigned long long tp = ld_agent(&jb->dbg[0]);
      atomicAdd(&jb->dbg[1], wall_clock64() - tp);
      atomicAdd(&jb->dbg[2], 1ull);
    }
#endif
#ifdef SMP_JOB_PROF
    if (threadIdx.x == 0) for (int i = 0; i < 4; ++i) J.tprof[i] = 0;
    unsigned long long* tp = J.tprof;
#else
    unsigned long long* tp = nullptr;
#endif
    for (int t = w - 1; t < nt; t += W) {
      const unsigned m = job_tile_mask(C, J, t, tp, seq);
      if (threadIdx.x == 0) st_agent(&jb->res[t], granule(seq, m));
#ifdef SMP_JOB_PROF
      if (threadIdx.x == 0) atomicAdd(&jb->dbg[3], wall_clock64() - ld_agent(&jb->dbg[0]));
#endif
    }
#ifdef SMP_JOB_PROF
    if (threadIdx.x == 0 && w - 1 < nt) for (int i = 0; i < 4; ++i) atomicAdd(&jb->dbg[4 + i], J.tprof[i]);
#endif
    t_last = wall_clock64();
  }
}

// --------------------------------------------------------------------------------------- scout hand-off
// Copies nbytes of LDS record section p (inside g_L.sr) to / from record `par` of the scout board, 8-byte words
// with agent-scope (sc1) stores / loads.  All threads.
__device__ __forceinline__ void sc_copy_out(ScoutBoard* sb, int par, const void* p, int nbytes) {
  const size_t off = (const char*)p - (const char*)&g_L.sr;
  const unsigned long long* src = (const unsigned long long*)p;
  unsigned long long* dst = (unsigned long long*)((char*)&sb->rec[par] + off);
  for (int w = threadIdx.x; w < nbytes / 8; w += BLOCK) st_agent(&dst[w], src[w]);
}
__device__ __forceinline__ void sc_copy_in(const ScoutBoard* sb, int par, void* p, int nbytes) {
  const size_t off = (const char*)p - (const char*)&g_L.sr;
  unsigned long long* dst = (unsigned long long*)p;
  const unsigned long long* src = (const unsigned long long*)((const char*)&sb->rec[par] + off);
  for (int w = threadIdx.x; w < nbytes / 8; w += BLOCK) dst[w] = ld_agent(&src[w]);
}
static_assert(sizeof(ScoutNN) % 8 == 0 && sizeof(ScoutNear) % 8 == 0 && sizeof(ScoutEdge) % 8 == 0 &&
              sizeof(ScoutExpand) % 8 == 0 && offsetof(ScoutRec, ex) % 8 == 0 && offsetof(ScoutRec, nr) % 8 == 0 &&
              sizeof(ScoutConnect) % 8 == 0 && offsetof(ScoutRec, cn) % 8 == 0 && sizeof(ScoutConn) % 8 == 0 &&
              sizeof(ScoutPre) % 8 == 0 && offsetof(ScoutRec, pre) % 8 == 0 && sizeof(ViaNode) % 8 == 0 &&
              offsetof(ScoutRec, cc) % 8 == 0 && offsetof(ScoutRec, n_choose) % 8 == 0 && offsetof(ScoutRec, e) % 8 == 0,
              "scout record sections are 8-byte words");

constexpr unsigned long long SCOUT_WAIT = 6000;  // device-clock ticks (60 us) the leader waits for one scout stage

// Leader: waits until the scout's record of this iteration reached stage s (or the scout is not working on this
// iteration, or SCOUT_WAIT passes: then the scout is not asked again this iteration) and copies the sections of
// the stages received since the last call into g_L.sr.  All threads; returns whether stage s is there.
__device__ void spec_copy(const ScoutBoard* sb, int par, int have, int st);
__device__ bool spec_stage(const Ctx& C, int s, unsigned long long wait) {
  if (!uni(g_L.sp_on)) return false;
  if (wait == 0) wait = SCOUT_WAIT;
  const int have = uni(g_L.sp_stage);
  if (have >= s) return true;
  const ScoutBoard* sb = C.Q.scbs[uni(g_L.asked[g_L.S.iter & (SCOUT_SLOTS - 1)]) - 1];
  const int par = (int)(g_L.S.iter & (SCOUT_SLOTS - 1));
  const unsigned tag = (unsigned)(g_L.S.iter + 1);
  const unsigned long long t0 = threadIdx.x == 0 ? wall_clock64() : 0;
  TR();
  int got;
  for (int k = 0;; k ^= 1) {
    if (threadIdx.x == 0) {
      const unsigned long long v = ld_agent(&sb->stage[par]);
      const unsigned lo = (unsigned)v;
      // a stage counts only if the scout built it on the tree as this iteration found it (its rewire commits)
      const bool cur = ((lo >> 8) & 0xfffu) == (g_L.rw_at0 & 0xfffu);
      int go = 0;
      if ((unsigned)(v >> 32) != tag) go = -1;           // the scout is not on this iteration
      else if (cur && (int)(lo & 0xffu) >= s) go = 1 + (int)(lo & 0xffu);
      else if (wall_clock64() - t0 > wait) go = -1;
      g_L.sp_go[k] = go;
    }
    __syncthreads();
    got = uni(g_L.sp_go[k]);
    if (got != 0) break;
    __builtin_amdgcn_s_sleep(1);
  }
  if (threadIdx.x == 0) g_L.S.sc_wait += wall_clock64() - t0;
#ifdef SMP_WAIT_PROF  // the leader's waits by stage into prof[28..31]: nn / expand, near / choose, rewire, connect
  if (threadIdx.x == 0) g_L.S.prof[s <= SC_EXPAND ? 28 : s <= SC_CHOOSE ? 29 : s == SC_DONE ? 30 : 31] += wall_clock64() - t0;
#endif
  TR();
  if (got < 0) {
    if (threadIdx.x == 0) g_L.sp_on = 0;
    __syncthreads();
    return false;
  }
  spec_copy(sb, par, have, got - 1);  // stages (have, st] arrived
  return true;
}

// Copies the sections of record stages (have, st] of record slot par into g_L.sr; all threads.  The sections are
// concatenated into one list of 8-byte words, each thread taking words tid, tid + BLOCK, ... with every load of a
// thread issued before its LDS stores: one memory round trip for the whole copy (a loop per section would queue
// one round trip per section behind the other).
__device__ void spec_copy(const ScoutBoard* sb, int par, int have, int st) {
  ScoutRec& R = g_L.sr;
  // choose-parent / rewire candidates only in iterations that have those steps (tree optimisation, a solution)
  const bool opt_now = uni(g_L.S.tree_opt && g_L.S.have_sol) != 0;
  int off[8], nw[8], ns = 0;
  auto add = [&](const void* p, int nbytes) {
    off[ns] = (int)((const char*)p - (const char*)&R) / 8;
    nw[ns] = nbytes / 8;
    ++ns;
  };
  if (have < SC_NN && st >= SC_NN) add(&R.nn, sizeof(ScoutNN));
  if (have < SC_EXPAND && st >= SC_EXPAND) { add(&R.e[0], sizeof(ScoutEdge)); add(&R.ex, sizeof(ScoutExpand)); }
  if (have < SC_NEAR && st >= SC_NEAR) add(&R.nr, sizeof(ScoutNear));
  if ((have < SC_CHOOSE && st >= SC_CHOOSE) || (have < SC_DONE && st >= SC_DONE)) add(&R.n_choose, 4 * sizeof(int));
  if (opt_now && have < SC_CHOOSE && st >= SC_CHOOSE) add(&R.e[SCOUT_CHOOSE0], MAX_NEAR * sizeof(ScoutEdge));
  if (opt_now && have < SC_DONE && st >= SC_DONE) add(&R.e[SCOUT_REWIRE0], MAX_NEAR * sizeof(ScoutEdge));
  if (!opt_now && have < SC_DONE && st >= SC_DONE) { add(&R.cn, sizeof(ScoutConnect)); add(&R.pre, sizeof(ScoutPre)); }
  if (have < SC_CONN && st >= SC_CONN) add(&R.cc, sizeof(ScoutConn));
  int total = 0;
  for (int i = 0; i < ns; ++i) total += nw[i];
  const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&sb->rec[par]);
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(&R);
  constexpr int U = 4;  // words per thread per round (a round holds 4 * BLOCK words: every section set fits)
  static_assert(sizeof(ScoutRec) / 8 <= U * BLOCK, "one round per record copy");
  int idx[U];
  unsigned long long v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int w = (int)threadIdx.x + u * BLOCK;
    idx[u] = -1;
    if (w < total) {
      int rem = w, i = 0;
      while (rem >= nw[i]) { rem -= nw[i]; ++i; }
      idx[u] = off[i] + rem;
      v[u] = ld_agent(&src[idx[u]]);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (idx[u] >= 0) dst[idx[u]] = v[u];
  __syncthreads();
  if (threadIdx.x == 0) g_L.sp_stage = st;
  __syncthreads();
}

// Leader, at the start of iteration j (after its sample): asks a scout for iteration j + 1, which expands tree `t`
// (= tree_B of iteration j), unless it was asked already.  Before the first solution (no choose-parent / rewire,
// so the trees only grow) and with a second scout, it also asks for iteration j + 2, which expands tree_A of
// iteration j: the scouts alternate by iteration parity, each with two leader iterations for its pass, since a
// pre-solution pass (nearest + expand job) is longer than the leader's own iteration.  The first n[t] nodes of a
// requested tree stay as they are until the record is used (only appends before then), and their stores are
// drained here, so the scout reads them as the leader will.  Iteration j looks a record up only if it was asked
// for (asked[j % 4]); every scout also gets the leader's current iteration (its staleness test).
// Thread 0: asks a scout for iteration k (expanding `tree`, whose first n[tree] nodes are final for it): before the
// first solution scout k mod nscouts, after it scout k mod 2 (scouts 0 and 1).
__device__ void scout_ask(const Ctx& C, long long k, int tree, bool pre, bool& fenced, int x_snap = -1) {
  const QState& S = g_L.S;
  const int ns = C.Q.nscouts;
  // (32-bit remainder: a 64-bit one is a long software division on the leader's path; which scout takes a record only
  // has to be the one asked, so the wrap at 2^32 iterations is harmless)
  int which = 1 + (int)(pre ? (unsigned)k % (unsigned)ns : (ns >= 2 ? (unsigned)(k & 1) : 0u));
  if ((g_L.sc_dead >> (which - 1)) & 1u) {  // a scout that never delivered: the next live one before the first
    if (!pre) return;                         // solution, none after it (the iteration takes the full path)
    int w = -1;
    for (int d = 1; d < ns && w < 0; ++d) {
      const int c = (int)((unsigned)(k + d) % (unsigned)ns);
      if (!((g_L.sc_dead >> c) & 1u)) w = c;
    }
    if (w < 0) return;
    // a scout holds one request slot (req[0..2], newest tag wins): if it still has an outstanding request of its own,
    // a second one could replace it before it is taken and its record would never come (the leader would wait out
    // SCOUT_WAIT for it), so iteration k takes the full path instead
    for (int x = 0; x < SCOUT_SLOTS; ++x)
      if (g_L.asked[x] == 1 + w) return;
    which = 1 + w;
  }
  ScoutBoard* sb = C.Q.scbs[which - 1];
  int& same = g_L.sc_same[which - 1];
  if (same < 0) {
    const int x = ld_agent(&sb->xcc);
    if (x > 0) same = (x - 1) == xcc_id() ? 1 : 0;
  }
  // a scout on another XCD reads through its own L2: write this XCD's dirty lines back first
  if (same != 1 && !fenced) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain();
    fenced = true;
  }
  const unsigned tag = (unsigned)(k + 1);
  const unsigned w0 = (unsigned)(x_snap >= 0 ? x_snap : S.n[tree]) | (unsigned)tree << 28 | (unsigned)(!pre) << 29;
  st_agent(&sb->req[2], granule(tag, (unsigned)S.n[1 - tree]));
  // the sampler version (low 20 bits; the ring tags use 8) and the rewire commits of the tree the record expands
  st_agent(&sb->req[1], granule(tag, ((unsigned)g_L.smp_ver & 0xfffffu) | ((unsigned)S.rewires[tree] & 0xfffu) << 20));
  st_agent(&sb->req[0], granule(tag, w0));
  g_L.asked[k & (SCOUT_SLOTS - 1)] = which;
  g_L.asked_conn[k & (SCOUT_SLOTS - 1)] = !pre && ns >= 2;
  g_L.asked_pre[k & (SCOUT_SLOTS - 1)] = pre;
}

// Leader, start of iteration j, before any store of the iteration: the requests for the coming iterations not yet
// asked for.  Their snapshots include the nodes the last iteration appended, whose stores are drained first -- only
// when something is asked (after the first solution the next iteration was usually asked for by
// scout_request_ahead2), and before this iteration's own stores, so the drain finds the last iteration's long done.
// Iteration j - 1's record slot is free again, j's record is looked up only if it was asked for, and every scout
// gets the leader's iteration (its staleness test).
// scout_slots (thread 0, LDS only, before the iteration's first memory round): iteration j - 1's slot is free
// again, and j's record is looked up only if it was asked for.  scout_asks (thread 0, after that round, whose drain
// covers the last iteration's stores): the leader's iteration for every scout, before the first solution the tree
// sizes for the scouts' late snapshots, and the requests for the coming iterations not yet asked for (their snapshots
// include the nodes the last iteration appended).
// Early ask (after the first solution, two scouts on this XCD): iteration j + 2 is asked for as soon as its scout
// (the one of iteration j) has finished record j's main pass -- before iteration j's inserts and rewire commits, not
// after them.  The record reads tree_A(j) as it is then: nodes appended later are patched in by the leader as usual, and
// a rewire commit on that tree makes the scout rebuild the pass (ScoutBoard::rwb / rwe; stage granules carry the count
// of rewire commits the record was built on, and the leader takes only a record of the tree as it found it).  Thread 0.
__device__ void scout_ask_early(const Ctx& C, int stage_j) {
  const QState& S = g_L.S;
  if (!C.Q.early_ask || C.Q.nscouts < 2 || !(S.tree_opt && S.have_sol) || stage_j < SC_DONE) return;
  const long long k = S.iter + 2;
  if (g_L.asked[k & (SCOUT_SLOTS - 1)]) return;
  const int w = (int)(k & 1);
  if (g_L.sc_same[w] != 1 || ((g_L.sc_dead >> w) & 1u)) return;
  bool fenced = true;  // same XCD: no write-back needed
  // the snapshot is tree_A as the iteration found it (those nodes' stores were drained by sample_read's round); the
  // nodes this iteration inserts count as appended, as j + 1's connect nodes do
  scout_ask(C, k, S.A, false, fenced, g_L.n_at0);
}

__device__ void scout_slots() {
  const QState& S = g_L.S;
  const long long j = S.iter;
  g_L.rw_at0 = (unsigned)S.rewires[S.A];
  g_L.n_at0 = S.n[S.A];
  g_L.asked[(j - 1) & (SCOUT_SLOTS - 1)] = 0;
  g_L.asked_conn[(j - 1) & (SCOUT_SLOTS - 1)] = 0;
  // a record asked for before the first solution (found in iteration f) is exact only while the tree it expands has
  // not been rewired since its snapshot: f + 1 rewires tree_B(f), which f + 3 expands, and f + 2 rewires tree_A(f)
  // after its own expand, so records of f + 1 and f + 2 hold and later ones are not looked up
  g_L.sp_on = g_L.asked[j & (SCOUT_SLOTS - 1)] != 0 &&
              !(g_L.asked_pre[j & (SCOUT_SLOTS - 1)] && S.have_sol && j >= S.first_iter + 3);
  g_L.sp_stage = -1;
}
// Wave 0, before scout_asks: the leader's iteration for every scout (and, before the first solution, the tree sizes
// for the late snapshots of the scouts on this XCD) -- lane s stores scout s's, so the boards' stores issue together
// instead of one dependent chain per scout in thread 0.
__device__ __forceinline__ void scout_cur_lanes(const Ctx& C) {
  const QState& S = g_L.S;
  const long long j = S.iter;
  const int s = (int)lane_id();
  if (s >= C.Q.nscouts) return;
  const bool pre = !(S.tree_opt && S.have_sol);
  const int nsc = pre ? C.Q.nscouts : min(C.Q.nscouts, 2);  // scouts 2 and up retire after the first solution
  ScoutBoard* sb = C.Q.scbs[s];
  // from first_iter + 3 on no record asked before the first solution is looked up (scout_slots): scouts 2 and up
  // stop (with their helpers) instead of polling beside the leader for the rest of the launch
  if (!pre && j == S.first_iter + 3 && s >= 2) st_agent(&sb->stop, 1);
  if (s >= nsc) return;
  st_agent(&sb->cur, (unsigned long long)j);
  // only to a scout on this XCD: the sizes hand over nodes stored without an agent release (a scout on another XCD
  // takes its request's sizes, whose nodes scout_ask released)
  if (pre && S.n[0] < (1 << 20) && S.n[1] < (1 << 20) && g_L.sc_same[s] == 1)
    st_agent(&sb->cur_sz, ((unsigned long long)(j & 0xffffff) << 40) | ((unsigned long long)S.n[0] << 20) |
                              (unsigned long long)S.n[1]);
}
// Thread 0: the requests for the coming iterations not yet asked for.
__device__ void scout_asks(const Ctx& C, int t) {
  const QState& S = g_L.S;
  const long long j = S.iter;
  const bool pre = !(S.tree_opt && S.have_sol);
  bool fenced = false;
  // before the first solution every scout has a request out (the trees only grow: records stay exact up to the
  // appended nodes); iteration j + a expands tree t for odd a, the other one for even a
  for (int ahead = 1; ahead <= (pre ? C.Q.nscouts : 1); ++ahead) {
    const long long k = j + ahead;
    if (g_L.asked[k & (SCOUT_SLOTS - 1)]) continue;
    scout_ask(C, k, (ahead & 1) ? t : 1 - t, pre, fenced);
  }
}

// After the first solution, with two scouts: iteration j asks for iteration j + 2 once its own rewire commits are
// done (or where they would be).  j + 2 expands tree_A of iteration j, which no later step of iteration j changes
// and iteration j + 1 only appends to (its connect step), so the record stays exact up to the appended nodes, which
// the leader patches in as before; each scout gets two leader iterations for its pass.
__device__ void scout_request_ahead2(const Ctx& C, int tA) {
  if (C.Q.nscouts < 2) return;
  drain();
  __syncthreads();
  if (threadIdx.x == 0) {
    const long long j = g_L.S.iter, k = j + 2;
    bool fenced = false;
    if (!g_L.asked[k & (SCOUT_SLOTS - 1)]) scout_ask(C, k, tA, false, fenced);
    // tree_A of this iteration is tree_B of iteration j + 1 and final for its connect step (which comes before any
    // other write to it): the scout of record j + 1 may run connect's scans now
    const long long k1 = j + 1;
    const int w1 = g_L.asked[k1 & (SCOUT_SLOTS - 1)];
    if (w1 && g_L.asked_conn[k1 & (SCOUT_SLOTS - 1)]) {
      ScoutBoard* sb = C.Q.scbs[w1 - 1];
      if (!fenced && g_L.sc_same[w1 - 1] != 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        drain();
      }
      st_agent(&sb->cgo, granule((int)(k1 + 1), (unsigned)g_L.S.n[tA]));
    }
  }
  __syncthreads();
}

// Leader: matches the batch's first E edges against the candidate edges of scout record stage sgrp (SC_CHOOSE:
// choose-parent candidates, SC_DONE: rewire candidates; equal start and target bit for bit) -> eg_rec[e], and
// returns whether every one of them has a record edge.  Wave 0, lane e: the record edge at the same position first
// (the scout builds its candidate lists with the leader's code, so they usually line up), then the others.
__device__ bool rec_match(const Ctx& C, int E, int sgrp) {
  const bool rec = spec_stage(C, sgrp);
  if (threadIdx.x < 64) {
    const int e = threadIdx.x;
    const int g0 = sgrp == SC_EXPAND ? 0 : sgrp == SC_CHOOSE ? SCOUT_CHOOSE0 : SCOUT_REWIRE0;
    const int gn = !rec ? 0 : sgrp == SC_EXPAND ? 1 : sgrp == SC_CHOOSE ? g_L.sr.n_choose : g_L.sr.n_rewire;
    int m = -1;
    if (e < E) {
      const int d = e < gn ? e : -1;
      for (int u = 0; u < gn; ++u) {
        const int k = g0 + (d < 0 ? u : (u == 0 ? d : (u <= d ? u - 1 : u)));
        const ScoutEdge& R = g_L.sr.e[k];
        if (same8(g_L.eg_start[e], R.s) && same8(g_L.eg_target[e], R.g)) { m = k; break; }
      }
    }
    if (e < MAXE) g_L.eg_rec[e] = m;
    const unsigned long long miss = __ballot(e < E && m < 0);
    if (e == 0) { g_L.rec_grp = sgrp; g_L.rec_all = miss == 0; }
  }
  __syncthreads();
  return uni(g_L.rec_all) != 0;
}

// edge_costs of E batch edges that all have record edges (rec_match): the record's segment-norm sums.
__device__ void edge_costs_rec(int E) {
  const int np = g_L.S.n_pts;
  if (threadIdx.x < E * NJ) {
    const int e = threadIdx.x / NJ, j = threadIdx.x - e * NJ;
    const double st = (g_L.eg_target[e][j] - g_L.eg_start[e][j]) / double(np);
    g_L.eg_step[e][j] = st;
    g_L.eg_end[e][j] = g_L.eg_start[e][j] + np * st;
  } else if (threadIdx.x >= 256 && threadIdx.x < 256 + E * 3) {
    const int i = threadIdx.x - 256, e = i / 3, k = i - e * 3;
    const double a = g_L.sr.e[g_L.eg_rec[e]].acc[k];
    g_L.eg_acc[e][k] = a;
    g_L.eg_cost[e][k] = g_L.eg_base[e][k] + a;
  }
  __syncthreads();
}

// One local collision tile of edge_validity's path without helpers (a call: the tile's registers stay out of the
// callers that inline edge_validity).
__device__ __noinline__ void local_tile(const Ctx& C, int nc) {
  const TileOrder order{g_L.tile_e, g_L.tile_i, g_L.eg_first, false};
  collide_tile<PLAN_CT>((&g_rb), C.sc, (&g_mc), nc, g_L.u.tile.tq, g_L.S.self, g_L.S.map, g_L.u.tile.T, &order,
                        &g_L.S.prof[P_TFK]);
}

// Validity of the batch's needed edges -> eg_first.  `ov` (OV_*, tree `ovt`): scan work whose inputs are final
// before the check, done while a collision job runs (after the check without helpers); overlap_work records it
// in g_L.spec for the caller.
// `sgrp` (leader, job mode): the scout record stage whose candidate edges may hold these edges' results
// (SC_EXPAND: the expand edge, SC_CHOOSE: choose-parent candidates, SC_DONE: rewire candidates).  A needed edge
// whose start and target equal a checked record edge bit for bit takes that edge's first collision (a pure
// function of the two configurations) and is left out of the job.
__device__ __forceinline__ void edge_validity(const Ctx& C, int E, bool stop_first_valid, int pslot, int ov = 0, int ovt = 0,
                              int sgrp = -1) {
  const int np1 = g_L.S.n_pts + 1;
  if (threadIdx.x == 0) g_L.count_slot = pslot + 4;
  TR();
  if (C.Q.jb) {
    // the record's results for the needed edges (matched by rec_match for this batch, else here)
    const bool matched = uni(g_L.rec_grp) == sgrp && sgrp >= 0;
    const bool rec = sgrp >= 0 && (matched || spec_stage(C, sgrp));
    TR();
    if (threadIdx.x < 64) {
      const int e = threadIdx.x;
      const bool need = e < E && g_L.eg_need[e];
      int hit = -2;
      if (rec && need) {
        if (matched) {
          const int k = g_L.eg_rec[e];
          if (k >= 0 && g_L.sr.e[k].first >= 0) hit = g_L.sr.e[k].first;
        } else {
          const int g0 = sgrp == SC_EXPAND ? 0 : sgrp == SC_CHOOSE ? SCOUT_CHOOSE0 : SCOUT_REWIRE0;
          const int gn = sgrp == SC_EXPAND ? 1 : sgrp == SC_CHOOSE ? g_L.sr.n_choose : g_L.sr.n_rewire;
          const int d = e < gn ? e : -1;
          for (int u = 0; u < gn; ++u) {
            const int k = g0 + (d < 0 ? u : (u == 0 ? d : (u <= d ? u - 1 : u)));
            const ScoutEdge& R = g_L.sr.e[k];
            if (R.first >= 0 && same8(g_L.eg_start[e], R.s) && same8(g_L.eg_target[e], R.g)) { hit = R.first; break; }
          }
        }
      }
      if (e < MAXE) g_L.eg_hit[e] = hit;
      const unsigned long long mh = __ballot(need && hit >= 0), mm = __ballot(need && hit < 0);
      if (rec && e == 0) { g_L.S.sc_edge_hit += __popcll(mh); g_L.S.sc_edge_miss += __popcll(mm); }
      // every needed edge answered by the record: no job
      if (mm == 0 && e < E) g_L.eg_first[e] = need ? hit : np1;
      if (e == 0) {
        g_L.ev_job = mm != 0;
        g_L.rec_grp = -1;
        if (mm == 0) g_L.spec = OV_NONE;
      }
    }
    __syncthreads();
    if (!uni(g_L.ev_job)) { TR(); return; }
    edge_validity_job(C, E, pslot, ov, ovt, stop_first_valid);
    if (threadIdx.x < E && g_L.eg_hit[threadIdx.x] >= 0) g_L.eg_first[threadIdx.x] = g_L.eg_hit[threadIdx.x];
    __syncthreads();
    TR();
    return;
  }
  if (threadIdx.x < E) { g_L.eg_first[threadIdx.x] = np1; g_L.eg_ptr[threadIdx.x] = 0; }
  __syncthreads();
  for (;;) {
    // wave 0 (lane e = edge e): stop check, then the next tile's slots by a prefix sum of remaining points
    if (threadIdx.x < 64) {
      const int e = threadIdx.x;
      const bool live = e < E && g_L.eg_need[e] && g_L.eg_first[e] >= np1;  // needed, no collision found
      const int ptr = e < E ? g_L.eg_ptr[e] : np1;
      bool stop = false;
      if (stop_first_valid) {
        const unsigned long long m = __ballot(live);
        if (m) stop = __shfl(ptr, __builtin_ctzll(m)) >= np1;  // first live candidate fully checked: free
      }
      const int rem = (live && ptr < np1) ? np1 - ptr : 0;
      int inc = rem;
      for (int off = 1; off < 32; off <<= 1) {
        int v = __shfl_up(inc, off);
        if (e >= off) inc += v;
      }
      const int start = inc - rem;
      const int take = stop ? 0 : max(0, min(rem, PLAN_CT - start));
      for (int i = 0; i < take; ++i) { g_L.tile_e[start + i] = e; g_L.tile_i[start + i] = ptr + i; }
      if (e < E) g_L.eg_ptr[e] = ptr + take;
      const int total = __shfl(inc, 31);
      if (e == 0) g_L.tile_n = stop ? 0 : min(PLAN_CT, total);
    }
    __syncthreads();
    const int nc = uni(g_L.tile_n);
    if (nc == 0) break;
    if (threadIdx.x < nc * NJ) {
      int c = threadIdx.x / NJ, j = threadIdx.x - c * NJ;
      int e = g_L.tile_e[c];
      g_L.u.tile.tq[c][j] = g_L.eg_start[e][j] + g_L.tile_i[c] * g_L.eg_step[e][j];
    }
    __syncthreads();
    PROF_BEGIN();
    local_tile(C, nc);
    PROF_END(P_TILES);
    if (threadIdx.x == 0) {
      g_L.S.prof[pslot] += pclk() - _pt;
      g_L.S.prof[P_NTILES]++;
      g_L.S.prof[pslot + 8] += nc;
    }
  }
  __syncthreads();
  overlap_work(C, ov, ovt);
}

// Scans whose inputs are final before a collision job, run while its tiles are checked (edge_validity):
//   OV_NEAR_EXPAND  near set of the expand edge's end in tree t (x_new if the edge is valid);
//   OV_NN           nearest node of tree t to x_new (connect's tree_B lookup, during the rewire job);
//   OV_NEAR_XN      near set of x_new in tree t (connect's near loop, during its direct-edge job).
// The nodes a scan streams are held back (spec_cnt) and counted by the caller only if it uses the result.
__device__ void overlap_work(const Ctx& C, int ov, int t) {
  ov = uni(ov);
  t = uni(t);
  if (ov == OV_NONE) {
    if (threadIdx.x == 0) g_L.spec = OV_NONE;
    __syncthreads();
    return;
  }
  const long long c0 = ov == OV_NN ? g_L.S.nn_nodes : g_L.S.near_nodes;
  __syncthreads();
  if (ov == OV_NEAR_EXPAND) near_set<20>(C, t, g_L.eg_end[0], g_L.S.n[t], true);
  else if (ov == OV_NEAR_XN) near_set<20>(C, t, g_L.xn.q, g_L.xn.id);
  else {
    const int id = nearest(C, t, g_L.xn.q);
    if (threadIdx.x == 0) g_L.spec_nn = id;
  }
  if (threadIdx.x == 0) {
    long long& cnt = ov == OV_NN ? g_L.S.nn_nodes : g_L.S.near_nodes;
    g_L.spec_cnt = cnt - c0;
    cnt = c0;
    g_L.spec = ov;
  }
  __syncthreads();
}

// Reference-semantics accounting of one isEdgeValid call (stops at the first collision).
__device__ __forceinline__ void count_edge(int first) {
  int np1 = g_L.S.n_pts + 1;
  g_L.S.prof[g_L.count_slot] += first >= np1 ? np1 : first + 1;
  if (first >= np1) { g_L.S.checked += np1; g_L.S.valid += np1; }
  else { g_L.S.checked += first + 1; g_L.S.valid += first; }
}

// count_edge over the needed edges of a batch, wave-parallel: every needed edge e < E (stop_first: up to and
// including the first needed one that is free, which is returned; -1 if none).  All threads.
__device__ int count_edges(int E, bool stop_first) {
  if (threadIdx.x < 64) {
    const int e = threadIdx.x, np1 = g_L.S.n_pts + 1;
    const bool need = e < E && g_L.eg_need[e];
    const int f = need ? g_L.eg_first[e] : 0;
    const unsigned long long mfree = __ballot(need && f >= np1);
    const int ev = (stop_first && mfree) ? __builtin_ctzll(mfree) : 64;
    int chk = 0, val = 0;
    if (need && e <= ev) { chk = f >= np1 ? np1 : f + 1; val = f >= np1 ? np1 : f; }
    chk = __ockl_wfred_add_i32(chk); val = __ockl_wfred_add_i32(val);
    if (e == 0) {
      g_L.S.prof[g_L.count_slot] += chk;
      g_L.S.checked += chk;
      g_L.S.valid += val;
      g_L.found = ev < 64 ? ev : -1;
    }
  }
  __syncthreads();
  return uni(g_L.found);
}

// stepTowardsRandSample (birrt_star.cpp:5712-5868), one lane (or every lane of a wave on the same values).  The
// revolute / prismatic split is a select on the mask bit, not a branch: a sum takes +0.0 for the joints of the other
// kind, which leaves it unchanged bit for bit (the sums are of squares, never -0.0), and a joint of a finished kind
// keeps 0.0 as the reference's extension does.
__device__ __forceinline__ bool step_towards_m(unsigned rm, const double* nn, double* x, double f) {
  double ed[NJ], srev = 0.0, spr = 0.0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const bool rv = (rm >> j) & 1u;
    ed[j] = x[j] - nn[j];
    const double d = ed[j] * ed[j];
    srev += rv ? d : 0.0;
    spr += rv ? 0.0 : d;
  }
  const double lrev = sqrt(srev), lpr = sqrt(spr);
  const bool rev_done = lrev < 0.001, pr_done = lpr < 0.001;
  double ext[NJ];
  srev = 0.0; spr = 0.0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const bool rv = (rm >> j) & 1u;
    const bool done = rv ? rev_done : pr_done;
    const double c = f * (ed[j] / (rv ? lrev : lpr));
    ext[j] = done ? 0.0 : nn[j] + c;
    const double cc = done ? 0.0 : c * c;
    srev += rv ? cc : 0.0;
    spr += rv ? 0.0 : cc;
  }
  const double elp = spr == 0.0 ? 1000.0 : sqrt(spr);
  const double elr = srev == 0.0 ? 1000.0 : sqrt(srev);
  const bool tr = elr < lrev, tp = elp < lpr;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const bool rv = (rm >> j) & 1u;
    if (rv ? tr : tp) x[j] = ext[j];
  }
  return !(tr || tp);
}
__device__ bool step_towards(const RobotDev* rb, const double* nn, double* x, double f) {
  return step_towards_m(rev_mask(rb), nn, x, f);
}

// step_towards_m for a whole wave (every lane active, the same nn / x / f in every lane, the same result).  An fp64
// division or square root costs a wave ~70 / ~90 cycles of issue however few lanes it serves, so the per-joint
// divisions run once, lane l dividing joint l % 8's difference, and the revolute / prismatic square roots once, even
// and odd lanes; every lane takes the results back by v_readlane.  nn_l / x_l are lane l's copies of nn[l % 8] and
// x[l % 8] (kept beside the arrays: picking an array element by lane compiles to a private-memory round trip); x_l
// is updated with x.  The operations and their order per value are step_towards_m's.
__device__ __forceinline__ bool step_towards_w(unsigned rm, const double* nn, double* x, double f, int lane, double nn_l,
                                               double& x_l) {
  double ed[NJ], srev = 0.0, spr = 0.0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const bool rv = (rm >> j) & 1u;
    ed[j] = x[j] - nn[j];
    const double d = ed[j] * ed[j];
    srev += rv ? d : 0.0;
    spr += rv ? 0.0 : d;
  }
  const double l2 = sqrt((lane & 1) ? spr : srev);
  const double lrev = readlane_d(l2, 0), lpr = readlane_d(l2, 1);
  const bool rev_done = lrev < 0.001, pr_done = lpr < 0.001;
  const bool rvl = (rm >> (lane & 7)) & 1u;
  const double ql = (x_l - nn_l) / (rvl ? lrev : lpr);
  double ext[NJ];
  srev = 0.0; spr = 0.0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const bool rv = (rm >> j) & 1u;
    const bool done = rv ? rev_done : pr_done;
    const double c = f * readlane_d(ql, j);
    ext[j] = done ? 0.0 : nn[j] + c;
    const double cc = done ? 0.0 : c * c;
    srev += rv ? cc : 0.0;
    spr += rv ? 0.0 : cc;
  }
  const double e2 = sqrt((lane & 1) ? spr : srev);
  const double elr = srev == 0.0 ? 1000.0 : readlane_d(e2, 0);
  const double elp = spr == 0.0 ? 1000.0 : readlane_d(e2, 1);
  const bool tr = elr < lrev, tp = elp < lpr;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const bool rv = (rm >> j) & 1u;
    if (rv ? tr : tp) x[j] = ext[j];
  }
  if (rvl ? tr : tp) x_l = (rvl ? rev_done : pr_done) ? 0.0 : nn_l + f * ql;
  return !(tr || tp);
}

// Stepping loop shared by choose_parent / connectGraphs: from `cur` towards `target` with
// unconstraint_extend_step_factor, collecting via nodes (ids nn_t, nn_t+1, ...) until the target is
// reached; the last edge becomes `sel` (id nn_t at that point).  No collision checks (reference behaviour).
// Wave 0 alone, the chain's state in registers (every lane holds the same values; lane s of the first half forms
// segment s of a step's edge cost as edge_costs does): no barrier per step.  On return g_L.cur, ox, reached, nn_t,
// n_via and edge slot 0 hold what the last step left, as a step-by-step block loop would.
__device__ __noinline__ void via_chain_w(const Ctx& C, const double* target) {
  const int lane = lane_id(), s = lane & 31;
  const int np = g_L.S.n_pts, via_cap = g_L.S.via_cap;
  const double f = g_L.S.step;
  double cur[NJ], cc[3], tg[NJ], ox[NJ], stp[NJ], end[NJ], acc[3], cost[3];
  int cid = g_L.cur.id, cpar = g_L.cur.parent;
#pragma unroll
  for (int j = 0; j < NJ; ++j) { cur[j] = g_L.cur.q[j]; tg[j] = target[j]; }
#pragma unroll
  for (int k = 0; k < 3; ++k) cc[k] = g_L.cur.c[k];
  int nn_t = g_L.nn_t, n_via = g_L.n_via, nsteps = 0;
  const unsigned rm = rev_mask(&g_rb);
  double cur_l = g_L.cur.q[lane & 7], ox_l;  // lane l's copies of cur[l % 8] / ox[l % 8] (step_towards_w)
  const double tg_l = target[lane & 7];
  static_assert(NJ == 8, "lane copies of the joints");
#ifdef SMP_VIA_PROF  // lane-0 clocks into prof[28..31]: entry, stepping, edge costs, calls
  unsigned long long _v0 = wall_clock64(), _v1;
#define VIA_CLK(k) { _v1 = wall_clock64(); if (lane == 0) g_L.S.prof[k] += _v1 - _v0; _v0 = _v1; }
#else
#define VIA_CLK(k)
#endif
  VIA_CLK(31);
  bool reached, overflow = false;
  double lst[NJ], lcc[3];  // the last step's edge start and base cost (edge slot 0)
  for (;;) {
    ++nsteps;
#pragma unroll
    for (int j = 0; j < NJ; ++j) ox[j] = tg[j];
    ox_l = tg_l;
    reached = step_towards_w(rm, cur, ox, f, lane, cur_l, ox_l);
    // the step of the edge: lane l divides joint l % 8's difference (one division for the wave)
    const double ql = (ox_l - cur_l) / double(np);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      stp[j] = readlane_d(ql, j);
      end[j] = cur[j] + np * stp[j];
    }
    VIA_CLK(28);
    // the segment norms: with np <= 21, lane 21 k + s takes norm k (total, revolute, prismatic) of segment s, one
    // square root for the wave; else lane s all three of segment s
    if (np <= 21) {
      const int k = lane / 21, sg = lane - 21 * k;
      double t, r, p;
      seg_terms(rm, cur, stp, sg, t, r, p);
      const double v = sqrt(k == 0 ? t : k == 1 ? r : p);
      if (sg < np && k < 3) g_L.u.seg[0][sg][k] = v;
    } else {
      double t, r, p;
      seg_norms(rm, cur, stp, s, t, r, p);
      if (lane < np) { g_L.u.seg[0][lane][0] = t; g_L.u.seg[0][lane][1] = r; g_L.u.seg[0][lane][2] = p; }
    }
    VIA_CLK(29);
    // the ordered sums (edge_costs' third stage): lanes 0..2 sum the segments through LDS (in order; one wave, so
    // its LDS writes are seen by its later reads), and every lane takes the three sums by v_readlane
    double al = 0.0;
    if (lane < 3) {
      double sg[MAX_PTS];
#pragma unroll
      for (int i = 0; i < MAX_PTS; ++i) sg[i] = g_L.u.seg[0][i][lane];  // (unconditional: see edge_costs)
#pragma unroll
      for (int i = 0; i < MAX_PTS; ++i)
        if (i < np) al += sg[i];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) acc[k] = readlane_d(al, k);
    VIA_CLK(30);
#pragma unroll
    for (int k = 0; k < 3; ++k) cost[k] = cc[k] + acc[k];
#pragma unroll
    for (int j = 0; j < NJ; ++j) lst[j] = cur[j];
#pragma unroll
    for (int k = 0; k < 3; ++k) lcc[k] = cc[k];
    if (reached) break;
    const int id = nn_t++;
    if (n_via >= via_cap) { overflow = true; reached = true; break; }
    if (lane == 0) {
      ViaNode& v = C.Q.via[n_via];
#pragma unroll
      for (int j = 0; j < NJ; ++j) { v.q[j] = end[j]; v.e_start[j] = cur[j]; v.e_target[j] = ox[j]; }
#pragma unroll
      for (int k = 0; k < 3; ++k) v.c[k] = cost[k];
      v.id = id;
      v.parent = cid;
    }
    ++n_via;
    cpar = cid;
    cid = id;
    cur_l = cur_l + np * ql;  // end[l % 8]
#pragma unroll
    for (int j = 0; j < NJ; ++j) cur[j] = end[j];
#pragma unroll
    for (int k = 0; k < 3; ++k) cc[k] = cost[k];
  }
#undef VIA_CLK
  if (lane == 0) {
    QState& S = g_L.S;
    S.prof[P_NVIA] += nsteps;
    if (overflow) { S.status = -7; S.phase = 2; }
    else {
      NodeRef& g = g_L.sel;
#pragma unroll
      for (int j = 0; j < NJ; ++j) { g.q[j] = end[j]; g_L.sel_start[j] = cur[j]; g_L.sel_target[j] = ox[j]; }
#pragma unroll
      for (int k = 0; k < 3; ++k) g.c[k] = cost[k];
      g.id = nn_t;
      g.parent = cid;
    }
    g_L.reached = 1;
    g_L.nn_t = nn_t;
    g_L.n_via = n_via;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      g_L.cur.q[j] = cur[j];
      g_L.ox[j] = ox[j];
      g_L.eg_start[0][j] = lst[j];
      g_L.eg_target[0][j] = ox[j];
      g_L.eg_step[0][j] = stp[j];
      g_L.eg_end[0][j] = end[j];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      g_L.cur.c[k] = cc[k];
      g_L.eg_base[0][k] = lcc[k];
      g_L.eg_acc[0][k] = acc[k];
      g_L.eg_cost[0][k] = cost[k];
    }
    g_L.cur.id = cid;
    g_L.cur.parent = cpar;
  }
}
__device__ void via_chain(const Ctx& C, const double* target) {
  TR();
  PROF_BEGIN();
  if (threadIdx.x < 64) via_chain_w(C, target);
  __syncthreads();
  PROF_END(P_VIA);
  TR();
}

// Inserts the pending via nodes (insertNode, birrt_star.cpp:3298-3322, once per node in order).  They form a
// chain -- via k's parent is via k-1, the first one's an existing node p0 -- so the result of the sequential
// inserts is known up front: node n0+k gets first child n0+k+1 (none for the last), and only p0's child list
// changes among the existing nodes.  One thread per node; thread 0 also links the first node under p0.
// rec (pre-solution commits): the nodes come from a scout record's via chain instead of C.Q.via, read
// with agent-scope loads; their ids (and parents) at or above rec_x are the scout's, relative to its snapshot size
// rec_x, and are rebased onto this tree's size.
__device__ void insert_via(const Ctx& C, int t, const ViaNode* rec = nullptr, int rec_x = 0) {
  TR();
  DETAIL_BEGIN(_di);
  const int nv = uni(g_L.n_via);
  if (nv > 0) {
    QState& S = g_L.S;
    const TreeDev& T = C.Q.tr[t];
    const int n0 = uni(S.n[t]), cap = uni(S.cap);
    if (n0 + nv > cap) {
      if (threadIdx.x == 0) { S.status = -7; S.phase = 2; }
    } else {
      for (int k = threadIdx.x; k < nv; k += BLOCK) {
        const ViaNode& w = rec ? rec[k] : C.Q.via[k];
        // record words are read with agent-scope loads (the scout may run on another XCD)
        auto ldd = [&](const double* p) {
          return rec ? __longlong_as_double((long long)ld_agent(reinterpret_cast<const unsigned long long*>(p))) : *p;
        };
        int wid = rec ? ld_agent(&w.id) : w.id, wpar = rec ? ld_agent(&w.parent) : w.parent;
        if (rec) {
          const int off = n0 - rec_x;
          if (wid >= rec_x) wid += off;
          if (wpar >= rec_x) wpar += off;
        }
        const int i = n0 + k;
        if (wid != i || (k > 0 && wpar != i - 1)) S.status = -7;  // not the chain insert_node expects
        for (int j = 0; j < NJ; ++j) {
          const double qj = ldd(&w.q[j]);
          st_coord(T, cap, j, i, qj);
          g_L.pc_q[t][i & (PATCH_K - 1)][j] = qj;
          T.e_start[(size_t)j * cap + i] = ldd(&w.e_start[j]);
          T.e_target[(size_t)j * cap + i] = ldd(&w.e_target[j]);
        }
        for (int c = 0; c < 3; ++c) st_tree(&T.cost[(size_t)c * cap + i], ldd(&w.c[c]));
        st_tree(&T.parent[i], wpar);
        T.first_child[i] = k + 1 < nv ? i + 1 : -1;
        T.prev_sib[i] = -1;
        if (k > 0) {
          T.next_sib[i] = -1;
        } else {
          const int p = wpar, f = T.first_child[p];
          T.next_sib[i] = f;
          if (f >= 0) T.prev_sib[f] = i;
          T.first_child[p] = i;
        }
      }
      if (threadIdx.x == 0) {
        S.n[t] = n0 + nv;
        S.edges[t] += nv;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (g_L.S.status == -7) g_L.S.phase = 2;
    g_L.n_via = 0;
  }
  DETAIL_END(_di, 31);
  __syncthreads();
  TR();
}

#ifdef SMP_RING_CHECK
__device__ unsigned long long g_ringchk[64];
__device__ unsigned long long g_ringdbg[SMP_RING][16];  // sampler: parameters of the slot's sample
extern "C" void smp_ringchk_dump() {
  unsigned long long v[64];
  if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_ringchk), sizeof(v)) == hipSuccess) {
    double d[64];
    __builtin_memcpy(d, v, sizeof(d));
    std::fprintf(stderr, "[smp] ring check: uniform(it) %llu, it-1 %llu, it+1 %llu, other %llu; first mismatch it %llu\n",
                 v[0], v[1], v[2], v[3], v[4]);
    std::fprintf(stderr, "[smp]   ring  :");
    for (int j = 0; j < 8; ++j) std::fprintf(stderr, " %.17g", d[24 + j]);
    std::fprintf(stderr, "\n[smp]   leader:");
    for (int j = 0; j < 8; ++j) std::fprintf(stderr, " %.17g", d[32 + j]);
    std::fprintf(stderr, "\n[smp]   sampler h0 %.17g Crev0 %.17g Crev7 %.17g ctr0 %.17g qmin2 %.17g qmax2 %.17g rev %llx\n",
                 d[40], d[41], d[42], d[43], d[44], d[45], v[46]);
    std::fprintf(stderr, "[smp]   leader  h0 %.17g Crev0 %.17g Crev7 %.17g ctr0 %.17g qmin2 %.17g qmax2 %.17g rev %llx\n",
                 d[48], d[49], d[50], d[51], d[52], d[53], v[54]);
  }
}
#endif
// --------------------------------------------------------------------------------------- sampling
// getRandomConf (control_laws.cpp:1120-1188) draw `inner` of outer attempt `outer` in iteration `it`; the
// caller keeps the first draw with EE z >= 0.
__device__ __forceinline__ void rand_conf_lane(const QState& S, uint32_t it, uint32_t outer, uint32_t inner, double* q) {
  const RobotDev* rb = (&g_rb);
  bool env0 = S.env_x[0] == 0.0 && S.env_x[1] == 0.0 && S.env_y[0] == 0.0 && S.env_y[1] == 0.0;
  double u[NJ];
#pragma unroll
  for (int p = 0; p < NJ / 2; ++p) u01_pair(S.seed, S.query, it, outer, inner, p, &u[2 * p], &u[2 * p + 1]);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    double lo = rb->q_min[j], hi = rb->q_max[j];
    if (!env0 && j == 0) { lo = S.env_x[0]; hi = S.env_x[1]; }
    if (!env0 && j == 1) { lo = S.env_y[0]; hi = S.env_y[1]; }
    q[j] = u[j] * (hi - lo) + lo;
  }
}

// sampleJointConfig_JntArray (birrt_star.cpp:3832-3878) of iteration `it` -> out[NJ] (LDS); wave 0 tries 64
// attempts at once.  All threads; returns 0, or -1 if no valid sample was found.
__device__ __forceinline__ int sample_uniform(const QState& S, uint32_t it, SmpLds& W, double* out) {
  if (wave_id() == 0) {
    int st = -1;
    for (uint32_t base = 0; base < (1u << 24); base += 64) {  // no valid sample in 16M attempts: give up loudly
      double q[NJ];
      rand_conf_lane(S, it, 0, base + lane_id(), q);
      bool ok = 0.0 <= ee_z((&g_rb), q);
      unsigned long long m = __ballot(ok);
      if (m) {
        int w = __ffsll((long long)m) - 1;
        if (lane_id() == w) for (int j = 0; j < NJ; ++j) out[j] = q[j];
        st = 0;
        break;
      }
    }
    if (lane_id() == 0) W.win = st;
  }
  __syncthreads();
  return uni(W.win);
}

// sampleJointConfigfromEllipse_JntArray (birrt_star.cpp:3607-3829) of iteration `it` -> out[NJ] (LDS): outer
// attempt b draws getRandomConf inner attempts 0, 1, ... until one has EE z >= 0, maps it into the informed
// ellipse, and the lowest outer attempt whose mapped sample is above ground and inside the environment wins.
// SE_OUT outer attempts per round:
//   1. waves 0-3 (one per SIMD: the FK chain is fp64-latency bound, more waves would only queue behind each
//      other): lane (b, i) evaluates inner attempt i < 8 of outer attempt b; the first valid i of each b goes to
//      LDS;
//   2. wave 0, lane b < SE_OUT: an outer attempt without a valid inner attempt in 0..7 continues serially from 8
//      (p ~ 2^-8 each); ellipse map + EE z + environment test; the lowest valid b wins.
// All threads; returns 0, or -1 if no valid sample was found.
__device__ __forceinline__ int sample_ellipse(const QState& S, uint32_t it, SmpLds& W, double* out) {
  const RobotDev* rb = (&g_rb);
  const bool env0 = S.env_x[0] == 0.0 && S.env_x[1] == 0.0 && S.env_y[0] == 0.0 && S.env_y[1] == 0.0;
  const int lane = lane_id();
  constexpr int SE_OUT = 32;
  for (uint32_t base = 0;; base += SE_OUT) {
    if (base >= (1u << 20)) return -1;
    if (threadIdx.x < SE_OUT * 8) {
      const uint32_t b = base + (threadIdx.x >> 3), inner = threadIdx.x & 7;
      double q[NJ];
      rand_conf_lane(S, it, 1 + b, inner, q);
      const bool ok = 0.0 <= ee_z(rb, q);
      const unsigned long long m = __ballot(ok);
      const unsigned grp = (unsigned)(m >> (lane & ~7)) & 0xffu;  // the 8 lanes of outer attempt b
      const int first = grp ? __builtin_ctz(grp) : 8;
      if ((int)inner == first)
        for (int j = 0; j < NJ; ++j) W.q[threadIdx.x >> 3][j] = q[j];
      if (inner == 0) W.ok[threadIdx.x >> 3] = grp != 0;
    }
    __syncthreads();
    if (wave_id() == 0) {
      const uint32_t b = base + lane;
      double q[NJ];
      if (lane >= SE_OUT) {
        for (int j = 0; j < NJ; ++j) q[j] = 1.0;  // idle lanes: excluded from the ballot below
      } else if (W.ok[lane]) {
        for (int j = 0; j < NJ; ++j) q[j] = W.q[lane][j];
      } else {
        for (uint32_t inner = 8; inner < (1u << 16); ++inner) {
          rand_conf_lane(S, it, 1 + b, inner, q);
          if (0.0 <= ee_z(rb, q)) break;
        }
      }
      // the revolute / prismatic parts in joint order, through static indices only (packing them through running
      // counters into private arrays came out shifted by one slot in the run-ahead sampler's build: samples of the
      // wrong joints; tests/test_gpu_parity.py::test_c5_informed_samples_from_the_ring)
      double br[6] = {}, bp[2] = {}, sr = 0.0, sp = 0.0;
      {
        int cr = 0, cp = 0;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const bool rv = rb->rev[j] != 0;
#pragma unroll
          for (int i = 0; i < 6; ++i) br[i] = rv && cr == i ? q[j] : br[i];
#pragma unroll
          for (int i = 0; i < 2; ++i) bp[i] = !rv && cp == i ? q[j] : bp[i];
          cr += rv ? 1 : 0;
          cp += rv ? 0 : 1;
        }
      }
      for (int i = 0; i < 6; ++i) sr += br[i] * br[i];
      for (int i = 0; i < 2; ++i) sp += bp[i] * bp[i];
      double nr = sqrt(sr), npn = sqrt(sp);
      double ps = u01(S.seed, S.query, it, 1 + b, 0, 8);
      for (int i = 0; i < 6; ++i) br[i] = ps * (br[i] / nr);
      for (int i = 0; i < 2; ++i) bp[i] = ps * (bp[i] / npn);
      double srev = sqrt(S.cbest[1] * S.cbest[1] - S.h0[1] * S.h0[1]) / 2.0;
      double spr = sqrt(S.cbest[2] * S.cbest[2] - S.h0[2] * S.h0[2]) / 2.0;
      double lr[6], lp[2];
      for (int i = 0; i < 6; ++i) lr[i] = i == 0 ? S.cbest[1] / 2.0 : srev;
      for (int i = 0; i < 2; ++i) lp[i] = i == 0 ? S.cbest[2] / 2.0 : spr;
      double r[NJ];
      double rr[6], rp[2];
      for (int i = 0; i < 6; ++i) {
        double s = 0.0;
        for (int k = 0; k < 6; ++k) s += (S.Crev[i * 6 + k] * lr[k]) * br[k];
        rr[i] = s + S.ctr_rev[i];
      }
      for (int i = 0; i < 2; ++i) {
        double s = 0.0;
        for (int k = 0; k < 2; ++k) s += (S.Cpr[i * 2 + k] * lp[k]) * bp[k];
        rp[i] = s + S.ctr_pr[i];
      }
      {
        int cr = 0, cp = 0;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const bool rv = rb->rev[j] != 0;
          double v = 0.0;
#pragma unroll
          for (int i = 0; i < 6; ++i) v = rv && cr == i ? rr[i] : v;
#pragma unroll
          for (int i = 0; i < 2; ++i) v = !rv && cp == i ? rp[i] : v;
          r[j] = v;
          cr += rv ? 1 : 0;
          cp += rv ? 0 : 1;
        }
      }
      bool above = 0.0 <= ee_z(rb, r);
      bool inside = (r[0] < S.env_x[1] && r[0] > S.env_x[0] && r[1] < S.env_y[1] && r[1] > S.env_y[0]) || env0;
      unsigned long long m = __ballot(above && inside && lane < SE_OUT);
      const int w = m ? __ffsll((long long)m) - 1 : -1;
      if (lane == w) for (int j = 0; j < NJ; ++j) out[j] = r[j];
      if (lane == 0) W.win = w;
    }
    __syncthreads();
    if (uni(W.win) >= 0) return 0;
  }
}

// The sample of iteration `it` for the planner state S (uniform, or informed once a solution exists).
__device__ __forceinline__ int sample_conf(const QState& S, uint32_t it, SmpLds& W, double* out) {
  if (uni(S.informed && S.have_sol)) return sample_ellipse(S, it, W, out);
  return sample_uniform(S, it, W, out);
}

// Leader, start of an iteration, thread 0, LDS only: a new informed-sampling parameter version when have_sol or
// c_best changed (the ring is then read at the new version); sample_publish (thread 0, after the iteration's first
// memory round) stores its iteration and, on a change, the parameters for the run-ahead sampler.
__device__ void sample_version(const Ctx& C) {
  QState& S = g_L.S;
  g_L.smp_pub = 0;
  if (!C.Q.sampler) return;
  const bool changed = g_L.smp_ver == 0 || g_L.smp_have_sol != S.have_sol || g_L.smp_cbest[0] != S.cbest[0] ||
                       g_L.smp_cbest[1] != S.cbest[1] || g_L.smp_cbest[2] != S.cbest[2];
  if (changed) {
    g_L.smp_have_sol = S.have_sol;
    for (int k = 0; k < 3; ++k) g_L.smp_cbest[k] = S.cbest[k];
    ++g_L.smp_ver;
    g_L.smp_pub = 1;
  }
}
// before_read: published ahead of this iteration's own sample read (the first launch, before the pre-loop connection):
// the iteration is announced as the one before, so the run-ahead sampler starts with this iteration's sample.
__device__ void sample_publish(const Ctx& C, bool before_read = false) {
  if (!C.Q.sampler) return;
  const QState& S = g_L.S;
  JobBoard* jb = C.Q.jb;
  if (g_L.smp_pub) {
    st_agent(&jb->s_have_sol, g_L.smp_have_sol);
    for (int k = 0; k < 3; ++k) st_agent(&jb->s_cbest[k], (unsigned long long)__double_as_longlong(g_L.smp_cbest[k]));
    drain();  // payload before the version
    st_agent(&jb->s_ver, g_L.smp_ver);
  }
  st_agent(reinterpret_cast<unsigned long long*>(&jb->s_iter), (unsigned long long)(S.iter - (before_read ? 1 : 0)));
}

// Second part: the sample from the ring (one round of tagged granules, wave 0) -- and, in the same round (wave 1),
// a look at the stage of this iteration's scout record, whose sections are then copied ahead of the steps that
// use them -- else drawn here.
// Leader, one round of the pre-solution record's granules (threads 64 .. 64 + PRE_GRANULES - 1, waves 1-3): each
// thread's 32-bit half goes to g_L.prer; returns, in every thread, whether its own granule carried this iteration's
// tag (the caller combines them at its barrier).  No ordering is needed: each granule says itself whether it is
// current.
__device__ __forceinline__ bool pre_read_round(const ScoutBoard* sb, int par, unsigned tag) {
  const int g = (int)threadIdx.x - 64;
  if (g < 0 || g >= PRE_GRANULES) return true;
  const unsigned long long v = ld_agent(&sb->pre_g[par][g]);
  reinterpret_cast<unsigned*>(&g_L.prer)[g] = (unsigned)v;
  return (unsigned)(v >> 32) == tag;
}

__device__ __forceinline__ void sample_read(const Ctx& C) {
  TR();
  QState& S = g_L.S;
  const uint32_t it = (uint32_t)S.iter;
  const bool pre = uni(g_L.sp_on && g_L.sp_stage < 0) != 0;
  const int sw = uni(g_L.asked[S.iter & (SCOUT_SLOTS - 1)]);
  const ScoutBoard* sb = sw > 0 ? C.Q.scbs[sw - 1] : nullptr;
  const int par = (int)(S.iter & (SCOUT_SLOTS - 1));
  // before the first solution the record is the data-tagged PreRec (read whole in this round); after it, a look at
  // the stage of the staged record, whose sections are then copied ahead of the steps that use them
  const bool prerec = pre && !uni(S.have_sol);
  bool pre_ok = true;
  if (prerec) pre_ok = pre_read_round(sb, par, (unsigned)(S.iter + 1));
  if (threadIdx.x == 64) {
    int st = -1;
    if (pre && !prerec) {
      const unsigned long long v = ld_agent(&sb->stage[par]);
      const unsigned lo = (unsigned)v;
      if ((unsigned)(v >> 32) == (unsigned)(S.iter + 1) && ((lo >> 8) & 0xfffu) == (g_L.rw_at0 & 0xfffu))
        st = (int)(lo & 0xffu);
    }
    g_L.sp_go[0] = st;
  }
  if (C.Q.sampler && threadIdx.x < 64) {
    JobBoard* jb = C.Q.jb;
    // the slot's 16 granules in one round; current iff every tag is this iteration's with the current version
    const unsigned want = ring_tag(it, (unsigned)__builtin_amdgcn_readfirstlane(g_L.smp_ver));
    unsigned long long v = 0;
    if (threadIdx.x < RING_G) v = ld_agent(&jb->ring[it % SMP_RING].g[threadIdx.x]);
    // current: every granule this iteration's at this version, and the parameters it was drawn with the leader's
    const int pk = (int)threadIdx.x - 2 * NJ;
    const bool ok = threadIdx.x >= RING_G ||
                    ((unsigned)(v >> 32) == want && (pk < 0 || (unsigned)v == ring_param(pk, S.have_sol, S.cbest)));
    const unsigned hi = (unsigned)odd_lane_of_pair((int)(unsigned)v);
    if (threadIdx.x < 2 * NJ && !(threadIdx.x & 1))
      g_L.xr[threadIdx.x >> 1] = __longlong_as_double((long long)(((unsigned long long)hi << 32) | (unsigned)v));
    const bool all = __ballot(!ok) == 0;
    if (threadIdx.x == 0) { g_L.smp_hit = all; if (all) S.smp_hits++; }
  } else if (threadIdx.x == 0) {
    g_L.smp_hit = 0;
  }
  // this round's loads and the last iteration's stores (tree inserts the requests below hand to the scouts) complete
  // together; then thread 0's stores of the iteration
  drain();
  const bool stale_granule = __syncthreads_or(!pre_ok) != 0;  // also the round's barrier
  TR();
  const bool prer_ok = prerec && !stale_granule;
  // the iteration's stores, over two waves: wave 0 the sampler's and the scout boards' iteration (a lane per scout),
  // thread 64 the new requests (only LDS fields of its own; the last iteration's tree stores a request hands over
  // were drained by every wave above)
  if (threadIdx.x < 64) {
    if (threadIdx.x == 0) {
      g_L.prer_ok = prer_ok;
      if (prer_ok) g_L.sc_seen |= 1u << (sw - 1);
      sample_publish(C);
    }
    TR();
    if (C.Q.nscouts > 0) scout_cur_lanes(C);
    TR();
  } else if (threadIdx.x == 64 && C.Q.nscouts > 0) {
    scout_asks(C, 1 - g_L.S.A);
    scout_ask_early(C, g_L.sp_go[0]);  // record j's stage as this round found it
  }
  TR();
  const int st = uni(g_L.sp_go[0]);
  __syncthreads();
  if (pre && !prerec && st >= 0) spec_copy(sb, par, -1, st);
  if (prer_ok && !uni(g_L.smp_hit) && uni(g_L.prer.t >= 0)) {
    // a valid record holds this iteration's sample (the ring's, at the pre-solution parameter version; an empty
    // record, t = -1, carries none)
    if (threadIdx.x < NJ) g_L.xr[threadIdx.x] = g_L.prer.xr[threadIdx.x];
    if (threadIdx.x == 0) g_L.smp_hit = 1;
    __syncthreads();
  }
  if (!uni(g_L.smp_hit)) {
    if (sample_conf(S, it, g_L.u.smp, g_L.xr) < 0 && threadIdx.x == 0) { S.status = -1; S.phase = 2; }
    __syncthreads();
  }
#ifdef SMP_RING_CHECK  // debugging: a sample taken from the ring or a record, recomputed here and compared (prof[28..30])
  else {
    __shared__ double chk_xr[NJ];
    __shared__ int chk_bad;
    sample_conf(S, it, g_L.u.smp, chk_xr);
    if (threadIdx.x == 0) {
      int bad = 0;
      for (int j = 0; j < NJ; ++j) bad |= __double_as_longlong(chk_xr[j]) != __double_as_longlong(g_L.xr[j]);
      chk_bad = bad;
      S.prof[30]++;
      if (bad) { S.prof[28]++; if (!S.prof[29]) S.prof[29] = (unsigned long long)it + 1; }
      if (bad && g_ringchk[21] == 0) {
        const RobotDev* rb = (&g_rb);
        g_ringchk[21] = 1;
        g_ringchk[4] = (unsigned long long)it;
        for (int j = 0; j < NJ; ++j) {
          g_ringchk[24 + j] = (unsigned long long)__double_as_longlong(g_L.xr[j]);
          g_ringchk[32 + j] = (unsigned long long)__double_as_longlong(chk_xr[j]);
        }
        for (int k = 0; k < 7; ++k) g_ringchk[40 + k] = ld_agent(&g_ringdbg[it % SMP_RING][8 + k]);
        const double lv[6] = {S.h0[1], S.Crev[0], S.Crev[7], S.ctr_rev[0], rb->q_min[2], rb->q_max[2]};
        for (int k = 0; k < 6; ++k) g_ringchk[48 + k] = (unsigned long long)__double_as_longlong(lv[k]);
        unsigned long long rv = 0;
        for (int j = 0; j < NJ; ++j) rv |= (unsigned long long)(rb->rev[j] != 0) << j;
        g_ringchk[54] = rv;
      }
    }
    __syncthreads();
    if (uni(chk_bad)) {  // which sample the ring held: prof[20] the uniform one of this iteration, [21] iteration
      // it - 1's, [22] it + 1's (current parameters), [23] none of them
      int cls = 23;
      for (int v = 0; v < 3 && cls == 23; ++v) {
        if (v == 0) sample_uniform(S, it, g_L.u.smp, chk_xr);
        else sample_conf(S, v == 1 ? it - 1 : it + 1, g_L.u.smp, chk_xr);
        if (threadIdx.x == 0) {
          int same = 1;
          for (int j = 0; j < NJ; ++j) same &= __double_as_longlong(chk_xr[j]) == __double_as_longlong(g_L.xr[j]);
          chk_bad = same;
        }
        __syncthreads();
        if (uni(chk_bad)) cls = 20 + v;
        __syncthreads();
      }
      if (threadIdx.x == 0) {
        g_ringchk[cls - 20]++;
      }
      __syncthreads();
    }
  }
#endif
}

// --------------------------------------------------------------------------------------- tree updates
// recursiveNodeCostUpdate (birrt_star.cpp:5495-5606): subtree walk over child lists, single lane.
__device__ void cost_update(const Ctx& C, int t, int v, const double* red) {
  QState& S = g_L.S;
  const TreeDev& T = C.Q.tr[t];
  const int cap = S.cap;
  int* stack = C.Q.stack;
  int sp = 0;
  stack[sp++] = v;
  const bool connected = (t == 0) == (S.conn_start != 0);
  int visits = 0;
  while (sp > 0) {
    if (++visits > S.n[t]) { S.status = -7; S.phase = 2; return; }  // a loop in the tree: fail loudly
    int id = stack[--sp];
    BCHK(id, cap, __LINE__, t);
    double nc[3];
    for (int k = 0; k < 3; ++k) { nc[k] = T.cost[(size_t)k * cap + id] + red[k]; st_tree(&T.cost[(size_t)k * cap + id], nc[k]); }
    if (S.have_sol) {
      if (id == S.nB.id && connected) {
        for (int k = 0; k < 3; ++k) { S.cbest[k] = S.cbest[k] + red[k]; S.nB.c[k] = nc[k]; }
        S.last_iter = S.iter;
      }
      if (id == S.nA.id && !connected) {
        for (int k = 0; k < 3; ++k) { S.cbest[k] = S.cbest[k] + red[k]; S.nA.c[k] = nc[k]; }
        S.last_iter = S.iter;
      }
    }
    for (int c = T.first_child[id]; c >= 0; c = T.next_sib[c]) {
      if (sp >= cap) { S.status = -7; S.phase = 2; return; }
      stack[sp++] = c;
    }
  }
}

// choose_node_parent_interpolation, unconstrained (birrt_star.cpp:4594-4738, 4916-4935).
// Uses g_L.lo_* (near list prefix) and g_L.xn / g_L.nn; may update g_L.xn, g_L.en_*; returns via g_L.ext_bp.
// choose_parent's candidate prefix (birrt_star.cpp:4594-4620): the near nodes in (cost, id) order up to the first whose
// cost is not below x_new's, at most max_near -- wave 0, one lane per list entry, the prefix length by a ballot (a loop
// on one thread waited one LDS round trip per entry).  Returns the count in every lane of wave 0 (0 without near nodes).
__device__ __forceinline__ int choose_prefix() {
  const int lane = lane_id();
  const int m = g_L.nk > 0 ? min(g_L.n_lo, g_L.S.max_near) : 0;
  const bool below = lane < m && g_L.lo_c[lane] < g_L.xn.c[0];
  return min(m, (int)__builtin_ctzll(~__ballot(below)));  // (m <= 20: lane 63 is never `below`)
}
__device__ void choose_parent(const Ctx& C, int t) {
  if (threadIdx.x < 64) {
    const int E = choose_prefix();  // candidate prefix: stop at the first near node whose cost is not below x_new's
    if (threadIdx.x == 0) {
      g_L.ext_bp = 0;
      g_L.found = -1;
      g_L.cnt = E;
      if (g_L.nk > 0) g_L.xn.parent = g_L.nn.id;
    }
  }
  __syncthreads();
  const int E = uni(g_L.cnt);
  if (E > 0) {
    if (threadIdx.x < E) {
      int e = threadIdx.x;
      NodeRef nd;
      load_node(C, t, g_L.lo_i[e], &nd);
      for (int j = 0; j < NJ; ++j) { g_L.eg_start[e][j] = nd.q[j]; g_L.eg_target[e][j] = g_L.xn.q[j]; }
      for (int k = 0; k < 3; ++k) g_L.eg_base[e][k] = nd.c[k];
      g_L.eg_near[e] = nd.id;
    }
    __syncthreads();
    if (C.Q.jb && rec_match(C, E, SC_CHOOSE)) edge_costs_rec(E);
    else edge_costs(C, E);
    if (threadIdx.x < E) g_L.eg_need[threadIdx.x] = g_L.eg_cost[threadIdx.x][0] <= g_L.xn.c[0];
    for (int e = E + threadIdx.x; e < MAXE; e += BLOCK) g_L.eg_need[e] = 0;
    __syncthreads();
    edge_validity(C, E, true, P_XCHOOSE, 0, 0, SC_CHOOSE);
    count_edges(E, true);  // -> g_L.found
    if (threadIdx.x == 0) {
      if (g_L.found >= 0) {
        g_L.ext_bp = 1;
        g_L.n_via = 0;
        g_L.nn_t = g_L.S.n[t];
        load_node(C, t, g_L.eg_near[g_L.found], &g_L.cur);
      }
    }
    __syncthreads();
    if (uni(g_L.found) >= 0) {
      via_chain(C, g_L.xn.q);
      if (threadIdx.x == 0) {
        // x_new <- last stepped edge (birrt_star.cpp:4692-4711)
        g_L.xn.id = g_L.sel.id;
        g_L.xn.parent = g_L.sel.parent;
        for (int j = 0; j < NJ; ++j) g_L.xn.q[j] = g_L.sel.q[j];
        for (int k = 0; k < 3; ++k) g_L.xn.c[k] = g_L.sel.c[k];
        for (int j = 0; j < NJ; ++j) { g_L.en_start[j] = g_L.sel_start[j]; g_L.en_target[j] = g_L.sel_target[j]; }
      }
      __syncthreads();
      insert_via(C, t);
    }
  }
  __syncthreads();
}

// rewireTreeInterpolation's candidates (birrt_star.cpp:5088-5096): the last min(k, max_near) near nodes, from the
// end, whose cost exceeds x_new's -> g_L.cnt.  The hi list is in ascending (cost, id) order, so they are a suffix
// of it; wave 0 tests them with one load each (lane l: position n_hi - 1 - l) and counts by ballot.
__device__ void rewire_count(const TreeDev& T) {
  if (threadIdx.x < 64) {
    const int n = g_L.nk, lane = threadIdx.x;
    const int m = n >= g_L.S.max_near ? g_L.S.max_near : n;
    bool ok = false;
    if (lane < m) {
      int hv = g_L.n_hi - 1 - lane;
      BCHK(hv, MAX_NEAR, __LINE__, 9);
      int v = g_L.hi_i[hv];
      BCHK(v, g_L.S.cap, __LINE__, 9);
      ok = g_L.xn.c[0] < T.cost[v];
    }
    const int cnt = __popcll(__ballot(ok));
    if (lane == 0) g_L.cnt = cnt;
  }
  __syncthreads();
}

// rewireTreeInterpolation, unconstrained (birrt_star.cpp:5056-5230).  Validity of every candidate edge
// x_new -> near is independent of the tree state, so all are checked at once; commits stay sequential.
__device__ void rewire(const Ctx& C, int t) {
  const int cap = g_L.S.cap;
  const TreeDev& T = C.Q.tr[t];
  rewire_count(T);
  const int cnt = uni(g_L.cnt);
  if (cnt == 0) return;
  // candidates k = n-1 .. n-cnt  ->  edge slot e = n-1-k
  if (threadIdx.x < cnt) {
    int e = threadIdx.x;
    int pos = g_L.n_hi - 1 - e;
    int v = g_L.hi_i[pos];
    NodeRef nd;
    load_node(C, t, v, &nd);
    for (int j = 0; j < NJ; ++j) { g_L.eg_start[e][j] = g_L.xn.q[j]; g_L.eg_target[e][j] = nd.q[j]; }
    for (int k = 0; k < 3; ++k) g_L.eg_base[e][k] = g_L.xn.c[k];
    g_L.eg_near[e] = v;
  }
  __syncthreads();
  if (C.Q.jb && rec_match(C, cnt, SC_DONE)) edge_costs_rec(cnt);
  else edge_costs(C, cnt);
  if (threadIdx.x == 0 && g_L.sp_on) scout_ask_early(C, g_L.sp_stage);  // before this iteration's commits
  if (threadIdx.x < cnt) {
    int e = threadIdx.x, v = g_L.eg_near[e];
    // costs only decrease during the loop, so a candidate failing against the current cost never passes
    int vv = v;
    BCHK(vv, g_L.S.cap, __LINE__, t);
    g_L.eg_need[e] = (vv != g_L.xn.parent) && (T.parent[vv] != 0) && (g_L.eg_cost[e][0] < T.cost[vv]);
  }
  for (int e = cnt + threadIdx.x; e < MAXE; e += BLOCK) g_L.eg_need[e] = 0;
  __syncthreads();
  edge_validity(C, cnt, false, P_XREWIRE, OV_NN, 1 - t, SC_DONE);
  TR();
  DETAIL_BEGIN(_dr);
  // Sequential commits (birrt_star.cpp:5096-5228).  The candidates' parents and costs are gathered into LDS by
  // one thread each; thread 0 walks the candidates from the resume point and stops after a commit, which may
  // change later candidates' costs (subtree update) -- the block then re-gathers and resumes.
  for (int e0 = 0;;) {
    if (threadIdx.x >= e0 && threadIdx.x < cnt) {
      const int e = threadIdx.x, v = g_L.eg_near[e];
      int vv = v;
      BCHK(vv, g_L.S.cap, __LINE__, t);
      g_L.rw_par[e] = T.parent[vv];
      for (int k = 0; k < 3; ++k) g_L.rw_cost[e][k] = T.cost[(size_t)k * cap + vv];
    }
    __syncthreads();
    // wave 0: the candidates from e0 on that act (birrt_star.cpp:5094-5110: not x_new's parent, not a child of the
    // root, cheaper through x_new), the first acting one that is free commits; every acting candidate up to it is
    // counted as the sequential loop counts it
    if (threadIdx.x < 64) {
      const int e = threadIdx.x, np1 = g_L.S.n_pts + 1;
      const bool act = e >= e0 && e < cnt && g_L.S.status == 0 && g_L.eg_near[e] != g_L.xn.parent &&
                       g_L.rw_par[e] != 0 && g_L.eg_cost[e][0] < g_L.rw_cost[e][0];
      const int f = act ? g_L.eg_first[e] : 0;
      const unsigned long long mc = __ballot(act && f >= np1);
      const int ec = mc ? __builtin_ctzll(mc) : 64;
      int chk = 0, val = 0;
      if (act && e <= ec) { chk = f >= np1 ? np1 : f + 1; val = f >= np1 ? np1 : f; }
      chk = __ockl_wfred_add_i32(chk); val = __ockl_wfred_add_i32(val);
      if (e == 0) {
        g_L.S.prof[g_L.count_slot] += chk;
        g_L.S.checked += chk;
        g_L.S.valid += val;
        g_L.rw_next = ec;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      QState& S = g_L.S;
      int next = cnt;
      for (int e = g_L.rw_next; e < cnt; ++e) {  // at most one pass: e is the committing candidate
        const int v = g_L.eg_near[e];
        double red[3];
        for (int k = 0; k < 3; ++k) red[k] = g_L.eg_cost[e][k] - g_L.rw_cost[e][k];
        // early asks: every scout learns that tree t changes before any of this commit's stores can be seen (without
        // early asks no record is asked for before its tree's rewires are done: nothing to publish)
        const bool pub = C.Q.early_ask && C.Q.nscouts >= 2;
        if (pub) {
          // (the iteration's earlier stores, its `cur` for the scouts among them, are performed first: a scout that
          // sees the commit also sees that the leader is at this iteration, whose own commits need no rebuild)
          drain();
          for (int s2 = 0; s2 < 2; ++s2) st_agent(reinterpret_cast<int*>(&C.Q.scbs[s2]->rwb[t]), S.rewires[t] + 1);
          drain();
        }
        // unlink from the old parent (the reference erases the outgoing edge, birrt_star.cpp:5124-5169)
        const int p = g_L.rw_par[e];
        const int pv = T.prev_sib[v], nx = T.next_sib[v];
        if (pv >= 0) T.next_sib[pv] = nx; else T.first_child[p] = nx;
        if (nx >= 0) T.prev_sib[nx] = pv;
        S.edges[t]--;
        st_tree(&T.parent[v], g_L.xn.id);
        if (S.have_sol) {
          bool connected = (t == 0) == (S.conn_start != 0);
          if (v == S.nB.id && connected) S.nB.parent = g_L.xn.id;
          else if (v == S.nA.id && !connected) S.nA.parent = g_L.xn.id;
        }
        for (int j = 0; j < NJ; ++j) {
          st_coord(T, cap, j, v, g_L.eg_end[e][j]);
          T.e_start[(size_t)j * cap + v] = g_L.eg_start[e][j];
          T.e_target[(size_t)j * cap + v] = g_L.eg_target[e][j];
        }
        int f = T.first_child[g_L.xn.id];
        T.next_sib[v] = f;
        T.prev_sib[v] = -1;
        if (f >= 0) T.prev_sib[f] = v;
        T.first_child[g_L.xn.id] = v;
        DETAIL_BEGIN(_dc);
        cost_update(C, t, v, red);
        DETAIL_END(_dc, 29);
        S.edges[t]++;
        S.rewires[t]++;
        if (pub) {
          drain();  // the commit's tree stores are performed (a same-XCD scout reads them through the shared L2)
          for (int s2 = 0; s2 < 2; ++s2) st_agent(reinterpret_cast<int*>(&C.Q.scbs[s2]->rwe[t]), S.rewires[t]);
        }
        next = e + 1;
        break;
      }
      if (S.status != 0) next = cnt;
      g_L.rw_next = next;
    }
    __syncthreads();
    e0 = uni(g_L.rw_next);
    if (e0 >= cnt) break;
  }
  DETAIL_END(_dr, 28);
  __syncthreads();
  TR();
}

// connectGraphsInterpolation, unconstrained branch + commit (birrt_star.cpp:2608-3046, 3219-3288).
// t = tree_B; g_L.xc = its nearest node to x_new; g_L.xn = x_new (node of the other tree).
__device__ void connect_tail(const Ctx& C, int t);
__device__ void connect_graphs(const Ctx& C, int t) {
  if (threadIdx.x == 0) {
    g_L.tree_expand = 0;
    g_L.best_nv = 10000.0;
    g_L.n_via = 0;
    for (int k = 0; k < 3; ++k) g_L.csp[k] = g_L.S.cbest[k];
    for (int j = 0; j < NJ; ++j) { g_L.eg_start[0][j] = g_L.xc.q[j]; g_L.eg_target[0][j] = g_L.xn.q[j]; }
    for (int k = 0; k < 3; ++k) g_L.eg_base[0][k] = g_L.xc.c[k];
    g_L.sel.id = -1;
  }
  __syncthreads();
  const bool crec = uni(g_L.conn_rec) != 0;
  if (crec) edge_costs_acc(1, (const double (*)[3])g_L.sr.cc.acc0);
  else edge_costs(C, 1);
  if (threadIdx.x == 0) {
    for (int k = 0; k < 3; ++k) g_L.sol[k] = g_L.eg_cost[0][k] + g_L.xn.c[k];
    g_L.eg_need[0] = g_L.sol[0] < g_L.csp[0];
  }
  __syncthreads();
  if (threadIdx.x == 0) g_L.spec = OV_NONE;
  __syncthreads();
  if (uni(g_L.eg_need[0])) {
    if (uni(!g_L.S.have_sol && g_L.sp_on && g_L.sp_stage >= SC_DONE && g_L.sr.cn.ok && g_L.sr.cn.t == t &&
            same8(g_L.sr.cn.e.s, g_L.eg_start[0]) && same8(g_L.sr.cn.e.g, g_L.eg_target[0]))) {
      // the scout checked this edge (before the first solution: no near set to overlap)
      if (threadIdx.x == 0) { g_L.eg_first[0] = g_L.sr.cn.e.first; g_L.S.sc_edge_hit++; }
      __syncthreads();
    } else if (crec && uni(g_L.sr.cc.nfirst >= 0)) {
      // after the first solution: the record's connect edges were checked with its scans (scout_connect); the direct
      // edge is the record's nearest node -> x_new, the same configurations
      if (threadIdx.x == 0) { g_L.eg_first[0] = g_L.sr.cc.first0; g_L.S.sc_edge_hit++; }
      __syncthreads();
    } else {
      edge_validity(C, 1, false, P_XCONNECT, (g_L.S.have_sol && !crec) ? OV_NEAR_XN : OV_NONE, t);
    }
    if (threadIdx.x == 0) {
      int f = g_L.eg_first[0];
      count_edge(f);
      g_L.flag = 0;
      if (f > g_L.S.n_pts) {  // valid: connect, stepping without collision checks
        for (int k = 0; k < 3; ++k) g_L.csp[k] = g_L.sol[k];
        g_L.flag = 1;
      } else {
        int lv = f == 0 ? 0 : f - 1;
        if (lv != 0) {  // extend towards the last valid configuration
          for (int j = 0; j < NJ; ++j) g_L.ext[j] = g_L.eg_start[0][j] + lv * g_L.eg_step[0][j];
          g_L.flag = 2;
        }
      }
      g_L.nn_t = g_L.S.n[t];
      g_L.cur = g_L.xc;
    }
    __syncthreads();
    const int flag = uni(g_L.flag);
    if (flag == 1) {
      via_chain(C, g_L.xn.q);
      if (threadIdx.x == 0) g_L.tree_expand = 0;
    } else if (flag == 2) {
      via_chain(C, g_L.ext);
      if (threadIdx.x == 0) { g_L.tree_expand = 1; g_L.best_nv = g_L.sol[0]; }
    }
    __syncthreads();
  }
  if (uni(g_L.S.have_sol)) {
    if (!take_spec(OV_NEAR_XN)) {
      if (crec) {  // the record's near set of x_new over the same final tree
        const ScoutConn& R = g_L.sr.cc;
        if (threadIdx.x < MAX_NEAR) {
          g_L.lo_i[threadIdx.x] = R.lo_i[threadIdx.x]; g_L.lo_c[threadIdx.x] = R.lo_c[threadIdx.x];
          g_L.hi_i[threadIdx.x] = R.hi_i[threadIdx.x]; g_L.hi_c[threadIdx.x] = R.hi_c[threadIdx.x];
        }
        if (threadIdx.x == 0) {
          g_L.nk = R.nk; g_L.n_lo = R.n_lo; g_L.n_hi = R.n_hi;
          g_L.S.near_nodes += g_L.S.n[t];
          g_L.S.sc_near++;
        }
        __syncthreads();
      } else {
        near_set<20>(C, t, g_L.xn.q, g_L.xn.id);
      }
    }
    if (threadIdx.x == 0) {
      int m = min(g_L.n_lo, g_L.S.max_near);
      g_L.cnt = m;
    }
    __syncthreads();
    const int E = uni(g_L.cnt);
    if (E > 0) {
      if (threadIdx.x < E) {
        int e = threadIdx.x;
        NodeRef nd;
        load_node(C, t, g_L.lo_i[e], &nd);
        for (int j = 0; j < NJ; ++j) { g_L.eg_start[e][j] = nd.q[j]; g_L.eg_target[e][j] = g_L.xn.q[j]; }
        for (int k = 0; k < 3; ++k) g_L.eg_base[e][k] = nd.c[k];
        g_L.eg_near[e] = nd.id;
      }
      __syncthreads();
      if (crec) edge_costs_acc(E, g_L.sr.cc.acc);
      else edge_costs(C, E);
      if (threadIdx.x < E) {
        int e = threadIdx.x;
        double s0 = g_L.eg_cost[e][0] + g_L.xn.c[0];
        g_L.eg_need[e] = (g_L.lo_c[e] < g_L.xn.c[0]) && (s0 < g_L.csp[0]);
      }
      for (int e = E + threadIdx.x; e < MAXE; e += BLOCK) g_L.eg_need[e] = 0;
      __syncthreads();
      if (crec && uni(g_L.sr.cc.nfirst >= E)) {  // the record's candidates, checked to the end (scout_connect)
        if (threadIdx.x < 64) {  // (E <= max_near <= 20: wave 0)
          if ((int)threadIdx.x < E) g_L.eg_first[threadIdx.x] = g_L.sr.cc.first[threadIdx.x];
          const int hits = __popcll(__ballot((int)threadIdx.x < E && g_L.eg_need[threadIdx.x]));
          if (threadIdx.x == 0) g_L.S.sc_edge_hit += hits;
        }
        __syncthreads();
      } else {
        edge_validity(C, E, true, P_XCONNECT);
      }
      DETAIL_BEGIN(_dn);
      // replay of the near loop (birrt_star.cpp:2820-3030).  An edge acts (connects: 1, extends: 2) only on
      // conditions of state that changes when an edge acts, so wave 0 evaluates every remaining edge against
      // the current state and the first acting one is processed; the configurations of the needed edges up to
      // it are counted as the sequential loop counts them.
      for (int e0 = 0;;) {
        if (threadIdx.x < 64) {
          const int e = threadIdx.x;
          const int np1 = g_L.S.n_pts + 1;
          const bool act = e >= e0 && e < E && g_L.eg_need[e];
          int fl = 0, f = 0;
          if (act) {
            f = g_L.eg_first[e];
            const double sol0 = g_L.eg_cost[e][0] + g_L.xn.c[0];
            if (f > g_L.S.n_pts) fl = 1;
            else if (g_L.csp[0] == g_L.S.cbest[0] && sol0 < g_L.best_nv && f >= 2) fl = 2;  // lv = f - 1 != 0
          }
          const unsigned long long m = __ballot(fl != 0);
          const int ev = m ? __builtin_ctzll(m) : 64;
          int chk = 0, val = 0;
          if (act && e <= ev) { chk = f >= np1 ? np1 : f + 1; val = f >= np1 ? np1 : f; }
          chk = __ockl_wfred_add_i32(chk); val = __ockl_wfred_add_i32(val);
          if (e == 0) {
            g_L.S.prof[g_L.count_slot] += chk;
            g_L.S.checked += chk;
            g_L.S.valid += val;
            g_L.flag = 0;
            g_L.rw_next = ev;
            if (ev < 64) {
              const int fe = g_L.eg_first[ev];
              const double sol0 = g_L.eg_cost[ev][0] + g_L.xn.c[0];
              if (fe > g_L.S.n_pts) {
                g_L.csp[0] = sol0;
                g_L.csp[1] = g_L.eg_cost[ev][1] + g_L.xn.c[1];
                g_L.csp[2] = g_L.eg_cost[ev][2] + g_L.xn.c[2];
                g_L.flag = 1;
              } else {
                const int lv = fe - 1;
                for (int j = 0; j < NJ; ++j) g_L.ext[j] = g_L.eg_start[ev][j] + lv * g_L.eg_step[ev][j];
                g_L.flag = 2;
                g_L.sol[0] = sol0;
              }
              g_L.n_via = 0;
              g_L.nn_t = g_L.S.n[t];
              load_node(C, t, g_L.eg_near[ev], &g_L.cur);
            }
          }
        }
        __syncthreads();
        const int flag_e = uni(g_L.flag);
        if (flag_e == 0) break;
        if (flag_e == 1) {
          via_chain(C, g_L.xn.q);
          if (threadIdx.x == 0) g_L.tree_expand = 0;
          __syncthreads();
          break;
        }
        e0 = uni(g_L.rw_next) + 1;
        via_chain(C, g_L.ext);
        if (threadIdx.x == 0) { g_L.tree_expand = 1; g_L.best_nv = g_L.sol[0]; }
        __syncthreads();
      }
      DETAIL_END(_dn, 30);
    }
  }
  insert_via(C, t);
  connect_tail(C, t);
}

// connectGraphs' commit (birrt_star.cpp:3219-3288), after the via nodes are inserted: the connection node on a
// cheaper solution (the first one sets the first-solution iteration and time), else the extension's last node.
__device__ void connect_tail(const Ctx& C, int t) {
  if (threadIdx.x == 0) {
    QState& S = g_L.S;
    if (g_L.csp[0] < S.cbest[0]) {
      if (!S.have_sol) {
        S.first_iter = S.iter;
        S.t_first = wall_clock64();
        // host-visible flag: smp_plan times the first feasible path on its own clock (system-scope vector store)
        if (C.Q.ttff) __hip_atomic_store(C.Q.ttff, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      S.have_sol = 1;
      insert_node(C, t, g_L.sel_start, g_L.sel_target, g_L.sel);
      S.conn_start = (t == 0);
      S.nB = g_L.sel;
      S.nA = g_L.xn;
      for (int k = 0; k < 3; ++k) S.cbest[k] = g_L.csp[k];
      S.last_iter = S.iter;
    } else if (g_L.tree_expand) {
      insert_node(C, t, g_L.sel_start, g_L.sel_target, g_L.sel);
    }
  }
  __syncthreads();
}

// Leader, connect step of an iteration after the first solution: takes connect's scans from the scout's record
// (stage SC_CONN) if it is there within 10 us and was made for this x_new over the final tree_B (same size, same
// configuration, same excluded id) -> g_L.conn_rec.  All threads.
__device__ bool conn_stage(const Ctx& C, int B) {
  if (threadIdx.x == 0) g_L.conn_rec = 0;
  __syncthreads();
  if (!uni(g_L.asked_conn[g_L.S.iter & (SCOUT_SLOTS - 1)])) return false;
  if (!spec_stage(C, SC_CONN, 1000)) return false;
  const ScoutConn& R = g_L.sr.cc;
  const bool ok = uni(R.ok && R.t == B && R.X == g_L.S.n[B] && R.excl == g_L.xn.id && same8(R.q, g_L.xn.q));
  if (ok && threadIdx.x == 0) g_L.conn_rec = 1;
  __syncthreads();
  return ok;
}

// Leader, an iteration before the first solution committed from its complete scout record (DESIGN.md "Pre-solution
// commits").  Before the first solution nothing rewires, so a tree only grows and a record computed on the first X
// nodes of a tree is exact up to the nodes appended since, which the leader scans here: one of them replaces the
// record's nearest node only with a strictly smaller distance (it has a larger index, birrt_star.cpp:4122).  If none
// does, the iteration is the record's -- expand edge (birrt_star.cpp:2224-2256), x_new, connect's nearest node,
// direct edge and via chain (connectGraphs without a solution has no near loop, birrt_star.cpp:2608-2812) -- and the
// leader only counts and inserts.  Returns false, having changed nothing, if the record does not hold (the caller
// runs the iteration itself); a record whose connect part does not hold is completed by connect_graphs.
// Outcome counters of pre_commit in prof[28..31] (committed / no usable record / a newer nearest node / connect
// completed by connect_graphs); those slots belong to the profiling builds' own clocks otherwise.
#if defined(SMP_DETAIL_PROF) || defined(SMP_JOB_PROF) || defined(SMP_NEAR_PROF) || defined(SMP_SAMPLE_PROF) || \
    defined(SMP_VIA_PROF) || defined(SMP_WAIT_PROF)
#define PRE_COUNT(k)
#else
#define PRE_COUNT(k) if (threadIdx.x == 0) g_L.S.prof[28 + (k)]++
#endif
// Leader: the pre-solution record of this iteration, complete in g_L.prer -- from sample_read's round, else polled
// (every granule tagged) until it is or SCOUT_WAIT passes or the scout has left.  All threads.
__device__ bool pre_wait(const Ctx& C) {
  TR();
  if (uni(g_L.prer_ok)) return true;
  TR();
  const int par = (int)(g_L.S.iter & (SCOUT_SLOTS - 1));
  const ScoutBoard* sb = C.Q.scbs[uni(g_L.asked[par]) - 1];
  const unsigned tag = (unsigned)(g_L.S.iter + 1);
  const unsigned long long t0 = threadIdx.x == 0 ? wall_clock64() : 0;
  for (int k = 0;; k ^= 1) {
    __builtin_amdgcn_s_sleep(1);
    const bool ok = pre_read_round(sb, par, tag);
    if (threadIdx.x == 0) g_L.sp_go[k] = wall_clock64() - t0 > SCOUT_WAIT || ld_agent(&sb->stop);
    const bool bad = __syncthreads_or(!ok) != 0;
    if (!bad) break;
    if (uni(g_L.sp_go[k])) {
      if (threadIdx.x == 0) {
        g_L.S.sc_wait += wall_clock64() - t0;
        // a scout that timed out without ever having delivered a record is taken as not running (its workgroup
        // may start late): it is asked no more in this launch, and its outstanding iterations are asked again of
        // the others instead of each waiting out SCOUT_WAIT
        const int w = g_L.asked[par];
        if (!((g_L.sc_seen >> (w - 1)) & 1u) && !ld_agent(&sb->stop)) {
          g_L.sc_dead |= 1u << (w - 1);
          for (int x = 0; x < SCOUT_SLOTS; ++x)
            if (x != par && g_L.asked[x] == w) g_L.asked[x] = 0;
        }
      }
      __syncthreads();  // every wave has read sp_go[k] before the next poll loop writes it again
      return false;
    }
  }
  if (threadIdx.x == 0) {
    g_L.S.sc_wait += wall_clock64() - t0;
    g_L.prer_ok = 1;
    g_L.sc_seen |= 1u << (g_L.asked[par] - 1);
  }
  TR();
  __syncthreads();
  return true;
}

#ifdef SMP_PRE_VERIFY
// Debugging build: every record-committed decision is recomputed the full way and compared; g_pv[0] counts checks,
// g_pv[1] holds the first mismatch: iteration | kind << 40 (1 nearest, 2 expand edge, 3 connect nearest, 4 connect
// edge, 5 x_new / edge costs) | block << 48; read by smp_debug_preverify.
__device__ unsigned long long g_pv[4];
__device__ void pv_fail(int kind) {
  if (threadIdx.x == 0)
    atomicCAS(&g_pv[1], 0ull, (unsigned long long)g_L.S.iter | ((unsigned long long)kind << 40) |
                                  ((unsigned long long)blockIdx.x << 48));
}
__device__ void pre_verify_expand(const Ctx& C, int A) {
  const PreRec& P = g_L.prer;
  double d;
  int full = nearest_scan(C, A, g_L.xr, 0, &d);
  full = d < 10000.0 ? full : 0;
  if (threadIdx.x == 0) atomicAdd(&g_pv[0], 1ull);
  if (uni(full != (P.nn_d < 10000.0 ? P.nn_id : 0))) pv_fail(1);
  if (threadIdx.x == 0) {
    NodeRef nn;
    load_node(C, A, full, &nn);
    for (int j = 0; j < NJ; ++j) { g_L.ext[j] = g_L.xr[j]; }
    step_towards((&g_rb), nn.q, g_L.ext, g_L.S.step);
    for (int j = 0; j < NJ; ++j) { g_L.eg_start[0][j] = nn.q[j]; g_L.eg_target[0][j] = g_L.ext[j]; }
    for (int k = 0; k < 3; ++k) g_L.eg_base[0][k] = nn.c[k];
    g_L.eg_need[0] = 1;
    g_L.rec_grp = -1;
  }
  for (int e = 1 + threadIdx.x; e < MAXE; e += BLOCK) g_L.eg_need[e] = 0;
  __syncthreads();
  edge_costs(C, 1);
  edge_validity(C, 1, false, P_XEXPAND);
  bool bad_costs = false;
  for (int j = 0; j < NJ; ++j) bad_costs |= g_L.eg_end[0][j] != P.end[j] || g_L.eg_start[0][j] != P.nn_q[j];
  for (int k = 0; k < 3; ++k) bad_costs |= g_L.eg_cost[0][k] != P.nn_c[k] + P.acc[k];
  if (uni(g_L.eg_first[0] != P.first)) pv_fail(2);
  if (uni(bad_costs)) pv_fail(5);
  __syncthreads();
}
__device__ void pre_verify_connect(const Ctx& C, int B, int cid) {
  const PreRec& P = g_L.prer;
  double d;
  int full = nearest_scan(C, B, g_L.xn.q, 0, &d);
  full = d < 10000.0 ? full : 0;
  if (uni(full != cid)) pv_fail(3);
  if (threadIdx.x == 0) {
    NodeRef xc;
    load_node(C, B, full, &xc);
    for (int j = 0; j < NJ; ++j) { g_L.eg_start[0][j] = xc.q[j]; g_L.eg_target[0][j] = g_L.xn.q[j]; }
    for (int k = 0; k < 3; ++k) g_L.eg_base[0][k] = xc.c[k];
    g_L.eg_need[0] = 1;
    g_L.rec_grp = -1;
  }
  for (int e = 1 + threadIdx.x; e < MAXE; e += BLOCK) g_L.eg_need[e] = 0;
  __syncthreads();
  edge_costs(C, 1);
  edge_validity(C, 1, false, P_XCONNECT);
  if (uni(P.pre_ok && P.need && g_L.eg_first[0] != P.cn_first)) pv_fail(4);
  __syncthreads();
  if (!uni(P.pre_ok)) return;
  // the connect outcome the full path would take (connect_graphs without a solution): flag, via chain, last node
  if (threadIdx.x == 0) {
    QState& S = g_L.S;
    double sol[3];
    for (int k = 0; k < 3; ++k) sol[k] = g_L.eg_cost[0][k] + g_L.xn.c[k];
    const int need = sol[0] < S.cbest[0];
    int flag = 0;
    if (need) {
      const int f = g_L.eg_first[0];
      if (f > S.n_pts) flag = 1;
      else {
        const int lv = f == 0 ? 0 : f - 1;
        if (lv != 0) { for (int j = 0; j < NJ; ++j) g_L.ext[j] = g_L.eg_start[0][j] + lv * g_L.eg_step[0][j]; flag = 2; }
      }
    }
    bool bad = need != P.need || flag != P.flag;
    for (int k = 0; k < 3; ++k) bad |= sol[k] != P.sol[k];
    if (bad) pv_fail(8);
    g_L.flag = flag;
    g_L.n_via = 0;
    g_L.nn_t = S.n[B];
    load_node(C, B, cid, &g_L.cur);
  }
  __syncthreads();
  const int flag = uni(g_L.flag);
  if (!flag) return;
  via_chain(C, flag == 1 ? g_L.xn.q : g_L.ext);
  if (threadIdx.x == 0) {
    const int par = (int)(g_L.S.iter & (SCOUT_SLOTS - 1));
    const ScoutBoard* sb = C.Q.scbs[g_L.asked[par] - 1];
    const int off = g_L.S.n[B] - P.XB;
    bool bad = g_L.n_via != P.nv;
    for (int k = 0; k < g_L.n_via && k < P.nv && !bad; ++k) {
      const ViaNode& a = C.Q.via[k];
      const ViaNode& b = sb->pre_via[par][k];
      for (int j = 0; j < NJ; ++j)
        bad |= a.q[j] != __longlong_as_double((long long)ld_agent((const unsigned long long*)&b.q[j])) ||
               a.e_start[j] != __longlong_as_double((long long)ld_agent((const unsigned long long*)&b.e_start[j])) ||
               a.e_target[j] != __longlong_as_double((long long)ld_agent((const unsigned long long*)&b.e_target[j]));
      for (int c = 0; c < 3; ++c) bad |= a.c[c] != __longlong_as_double((long long)ld_agent((const unsigned long long*)&b.c[c]));
      const int bid = ld_agent(&b.id), bpar = ld_agent(&b.parent);
      bad |= a.id != (bid >= P.XB ? bid + off : bid) || a.parent != (bpar >= P.XB ? bpar + off : bpar);
    }
    if (bad) pv_fail(6);
    bool bs = false;
    for (int j = 0; j < NJ; ++j) bs |= g_L.sel.q[j] != P.sel_q[j] || g_L.sel_start[j] != P.sel_start[j] || g_L.sel_target[j] != P.sel_target[j];
    for (int k = 0; k < 3; ++k) bs |= g_L.sel.c[k] != P.sel_c[k];
    bs |= g_L.sel.id != (P.sel_id >= P.XB ? P.sel_id + off : P.sel_id);
    bs |= g_L.sel.parent != (P.sel_parent >= P.XB ? P.sel_parent + off : P.sel_parent);
    if (bs) pv_fail(7);
    g_L.n_via = 0;
  }
  __syncthreads();
}
#endif

__device__ __forceinline__ bool pre_commit(const Ctx& C, int A, int B) {
  if (!uni(g_L.sp_on) || !pre_wait(C)) { PRE_COUNT(1); return false; }
  const PreRec& P = g_L.prer;
  const int nA = uni(g_L.S.n[A]);
  if (!uni(P.t == A && P.X <= nA && same8(P.xr, g_L.xr))) { PRE_COUNT(1); return false; }
  if (uni(P.X < nA)) {
    double dp;
    if (uni(nA - P.X <= PATCH_K)) patch_scan(A, g_L.xr, P.X, nA, &dp);
    else nearest_scan(C, A, g_L.xr, P.X, &dp);
    if (uni(dp < P.nn_d)) { PRE_COUNT(2); return false; }
  }
  PRE_COUNT(0);
  TR();
#ifdef SMP_PRE_VERIFY
  pre_verify_expand(C, A);
#endif
  if (threadIdx.x == 0) {
    QState& S = g_L.S;
    S.nn_nodes += nA;
    S.sc_nn++;
    S.sc_edge_hit++;
    const int nid = P.nn_d < 10000.0 ? P.nn_id : 0;
    g_L.count_slot = P_XEXPAND + 4;
    count_edge(P.first);
    g_L.ext_nn = P.first > S.n_pts;
    g_L.ext_bp = 0;
    if (g_L.ext_nn) {
      for (int j = 0; j < NJ; ++j) { g_L.xn.q[j] = P.end[j]; g_L.en_start[j] = P.nn_q[j]; g_L.en_target[j] = P.ext[j]; }
      for (int k = 0; k < 3; ++k) g_L.xn.c[k] = P.nn_c[k] + P.acc[k];
      g_L.xn.id = S.n[A];
      g_L.xn.parent = nid;
      insert_node(C, A, g_L.en_start, g_L.en_target, g_L.xn);
    }
  }
  __syncthreads();
  if (!uni(g_L.ext_nn)) return true;
  // connect (birrt_star.cpp:1256-1275): tree_B's nearest node of x_new (the record's x_new is P.end)
  const int nB = uni(g_L.S.n[B]);
  bool rec = uni(P.cn_ok && P.XB <= nB) != 0;
  int cid;
  if (rec) {
    cid = P.cn_d < 10000.0 ? P.cn_id : 0;
    if (uni(P.XB < nB)) {
      double dp;
      const int ip = uni(nB - P.XB <= PATCH_K) ? patch_scan(B, g_L.xn.q, P.XB, nB, &dp)
                                                : nearest_scan(C, B, g_L.xn.q, P.XB, &dp);
      if (uni(dp < P.cn_d)) { cid = ip; rec = false; }
    }
    if (threadIdx.x == 0) { g_L.S.nn_nodes += nB; g_L.S.sc_nn++; }
  } else {
    cid = nearest(C, B, g_L.xn.q);
  }
  TR();
#ifdef SMP_PRE_VERIFY
  if (rec) pre_verify_connect(C, B, cid);
#endif
  if (!rec || !uni(P.pre_ok) || C.Q.pre_commit == 2) {
    PRE_COUNT(3);
    if (threadIdx.x == 0) load_node(C, B, cid, &g_L.xc);
    __syncthreads();
    connect_graphs(C, B);
    return true;
  }
  // the record's connect outcome: count the direct edge, insert its via chain and the last node
  if (threadIdx.x == 0) {
    QState& S = g_L.S;
    const int off = S.n[B] - P.XB;
    g_L.tree_expand = 0;
    g_L.best_nv = 10000.0;
    for (int k = 0; k < 3; ++k) g_L.csp[k] = S.cbest[k];
    if (P.need) {
      g_L.count_slot = P_XCONNECT + 4;
      count_edge(P.cn_first);
      S.sc_edge_hit++;
      if (P.flag == 1) {
        for (int k = 0; k < 3; ++k) g_L.csp[k] = P.sol[k];
      } else if (P.flag == 2) {
        g_L.tree_expand = 1;
        g_L.best_nv = P.sol[0];
      }
    }
    g_L.n_via = P.nv;
    for (int j = 0; j < NJ; ++j) {
      g_L.sel.q[j] = P.sel_q[j];
      g_L.sel_start[j] = P.sel_start[j];
      g_L.sel_target[j] = P.sel_target[j];
    }
    for (int k = 0; k < 3; ++k) g_L.sel.c[k] = P.sel_c[k];
    g_L.sel.id = P.sel_id >= P.XB ? P.sel_id + off : P.sel_id;
    g_L.sel.parent = P.sel_parent >= P.XB ? P.sel_parent + off : P.sel_parent;
  }
  __syncthreads();
  const int par = (int)(g_L.S.iter & (SCOUT_SLOTS - 1));
  const ScoutBoard* sb = C.Q.scbs[uni(g_L.asked[par]) - 1];
  insert_via(C, B, sb->pre_via[par], P.XB);
  connect_tail(C, B);
  TR();
  return true;
}

// One C-space iteration of run_planner (birrt_star.cpp:1163-1338).  Always inlined into plan_kernel: builds in
// which the inliner outlined it (a larger scout) fault the GPU with a memory-aperture violation in the first
// iterations (tools/experiments/README.md), builds that inline it run clean.
__device__ __forceinline__ void iteration(const Ctx& C) {
  const int A = uni(g_L.S.A), B = 1 - A;
  unsigned long long _t0 = threadIdx.x == 0 ? pclk() : 0, _t1;
#ifdef SMP_TRACE
  if (threadIdx.x == 0) g_L.tit = g_L.S.iter;
#endif
  if (threadIdx.x == 0) g_L.conn_rec = 0;
  TR();
#define PHASE(k) if (threadIdx.x == 0) { _t1 = pclk(); g_L.S.prof[k] += _t1 - _t0; _t0 = _t1; }
  // two waves in parallel (disjoint LDS fields; each a serial chain of LDS reads)
  if (threadIdx.x == 0) sample_version(C);
  else if (threadIdx.x == 64 && C.Q.nscouts > 0) scout_slots();
  __syncthreads();
  TR();
  sample_read(C);
  TR();
  PHASE(P_SAMPLE);
  const bool opt = uni(g_L.S.tree_opt && g_L.S.have_sol);
  if (C.Q.pre_commit && C.Q.nscouts > 0 && !uni(g_L.S.have_sol) && pre_commit(C, A, B)) {
    PHASE(P_CONNECT);
  } else {
  int nid = nearest_leader(C, A, g_L.xr);
  TR();
  PHASE(P_NN);
  if (threadIdx.x == 0) {
    // expandTree single step (birrt_star.cpp:2224-2256).  If the scout's record of this iteration already holds
    // its expand stage for the same sample, tree and nearest node, the step target and the interpolation data are
    // its (the same function of the same inputs); else computed here.
    const ScoutRec& R = g_L.sr;
    const bool rid = g_L.sp_on && g_L.sp_stage >= SC_EXPAND && R.ex.ok && R.nn.ok && R.nn.t == A && R.nn.id == nid &&
                     same8(R.nn.q, g_L.xr);
    if (rid) {
      // the record's nearest node is this one: its configuration is the record's edge start (configurations never
      // change) and its costs the record's (a staged record is taken only on the tree's rewire count as this
      // iteration found it, and only rewires change the costs of existing nodes) -- no dependent global load
      for (int j = 0; j < NJ; ++j) g_L.nn.q[j] = R.e[0].s[j];
      for (int k = 0; k < 3; ++k) g_L.nn.c[k] = R.nn.c[k];
      g_L.nn.id = nid;
      g_L.nn.parent = -1;  // (not used by the iteration)
    } else {
      load_node(C, A, nid, &g_L.nn);
    }
    bool rec = rid && same8(R.e[0].g, R.ex.ext);
    g_L.flag = rec;
    if (rec) {
      for (int j = 0; j < NJ; ++j) {
        g_L.eg_start[0][j] = g_L.nn.q[j];
        g_L.eg_target[0][j] = R.ex.ext[j];
        g_L.eg_step[0][j] = R.ex.step[j];
        g_L.eg_end[0][j] = R.ex.end[j];
      }
      for (int k = 0; k < 3; ++k) {
        g_L.eg_base[0][k] = g_L.nn.c[k];
        g_L.eg_acc[0][k] = R.ex.acc[k];
        g_L.eg_cost[0][k] = g_L.nn.c[k] + R.ex.acc[k];
      }
    } else {
      for (int j = 0; j < NJ; ++j) g_L.ext[j] = g_L.xr[j];
      step_towards((&g_rb), g_L.nn.q, g_L.ext, g_L.S.step);
      for (int j = 0; j < NJ; ++j) { g_L.eg_start[0][j] = g_L.nn.q[j]; g_L.eg_target[0][j] = g_L.ext[j]; }
      for (int k = 0; k < 3; ++k) g_L.eg_base[0][k] = g_L.nn.c[k];
    }
    g_L.eg_need[0] = 1;
  }
  __syncthreads();
  TR();
  if (!uni(g_L.flag)) edge_costs(C, 1);
  edge_validity(C, 1, false, P_XEXPAND, opt ? OV_NEAR_EXPAND : OV_NONE, A, SC_EXPAND);
  TR();
  if (threadIdx.x == 0) {
    int f = g_L.eg_first[0];
    count_edge(f);
    g_L.ext_nn = f > g_L.S.n_pts;
    if (g_L.ext_nn) {
      for (int j = 0; j < NJ; ++j) { g_L.xn.q[j] = g_L.eg_end[0][j]; g_L.en_start[j] = g_L.eg_start[0][j]; g_L.en_target[j] = g_L.eg_target[0][j]; }
      for (int k = 0; k < 3; ++k) g_L.xn.c[k] = g_L.eg_cost[0][k];
      g_L.xn.id = g_L.S.n[A];
      g_L.xn.parent = g_L.nn.id;
    } else {  // x_new = x_rand with cost 10000 (birrt_star.cpp:1213-1217, 2252-2255)
      for (int j = 0; j < NJ; ++j) g_L.xn.q[j] = g_L.xr[j];
      g_L.xn.c[0] = 10000.0; g_L.xn.c[1] = 0.0; g_L.xn.c[2] = 0.0;
      g_L.xn.id = g_L.S.n[A];
      g_L.xn.parent = g_L.nn.id;
    }
    g_L.ext_bp = 0;
  }
  __syncthreads();
  PHASE(P_EXPAND);
  if (opt) {
    // x_new is the expand edge's end exactly when the edge is valid: then its near set was computed during the job
    TR();
    if (!(uni(g_L.ext_nn) && take_spec(OV_NEAR_EXPAND)) && !near_set_rec<20>(C, A, g_L.xn.q, g_L.xn.id))
      near_set_scan<20, false>(C, A, g_L.xn.q, g_L.xn.id);
    TR();
    PHASE(P_NEAR);
    choose_parent(C, A);
    TR();
    PHASE(P_CHOOSE);
  }
  if (uni(g_L.ext_nn || g_L.ext_bp)) {
    if (threadIdx.x == 0) insert_node(C, A, g_L.en_start, g_L.en_target, g_L.xn);
    __syncthreads();
    if (threadIdx.x == 0) g_L.spec = OV_NONE;
    __syncthreads();
    TR();
    if (opt) {
      rewire(C, A);
      scout_request_ahead2(C, A);
    }
    TR();
    PHASE(P_REWIRE);
    int cid;
    const bool crec = opt && conn_stage(C, B);
    if (take_spec(OV_NN)) {
      cid = uni(g_L.spec_nn);
    } else if (crec) {
      cid = uni(g_L.sr.cc.d < 10000.0 ? g_L.sr.cc.id : 0);
      if (threadIdx.x == 0) { g_L.S.nn_nodes += g_L.S.n[B]; g_L.S.sc_nn++; }
    } else if (uni(!opt && g_L.sp_on) && spec_stage(C, SC_DONE, 2500) &&
               uni(g_L.sr.cn.ok && g_L.sr.cn.t == B &&
                   g_L.sr.cn.X <= g_L.S.n[B] && same8(g_L.sr.cn.q, g_L.xn.q))) {
      // the scout's nearest node over the first X nodes; only the nodes appended since are scanned (one of them
      // replaces it only with a strictly smaller distance: it has a larger index)
      const int n = uni(g_L.S.n[B]);
      double dp = 10000.0;
      int ip = 0;
      if (uni(g_L.sr.cn.X < n)) ip = nearest_scan(C, B, g_L.xn.q, g_L.sr.cn.X, &dp);
      if (threadIdx.x == 0) { g_L.S.nn_nodes += n; g_L.S.sc_nn++; }
      cid = uni(dp < g_L.sr.cn.d ? ip : (g_L.sr.cn.d < 10000.0 ? g_L.sr.cn.id : 0));
    } else {
      cid = nearest(C, B, g_L.xn.q);
    }
    if (threadIdx.x == 0) load_node(C, B, cid, &g_L.xc);
    __syncthreads();
    TR();
    PHASE(P_NN);
    connect_graphs(C, B);
    TR();
    PHASE(P_CONNECT);
  }
  else if (opt) {
    scout_request_ahead2(C, A);
  }
  }
#undef PHASE
  if (threadIdx.x == 0) {
    QState& S = g_L.S;
    S.A = B;
    S.iter++;
    if (C.Q.rows && S.n_rows < C.Q.rows_cap) {
      double* row = C.Q.rows + S.n_rows * 5;
      row[0] = (double)S.iter;
      row[1] = (double)(wall_clock64() - S.t0);
      row[2] = S.cbest[0]; row[3] = S.cbest[1]; row[4] = S.cbest[2];
      S.n_rows++;
    }
    if ((S.cbest[0] - S.h0[0]) < S.opt_thresh) S.phase = 2;  // birrt_star.cpp:1333-1338
    if (S.iter >= S.max_iter) S.phase = 2;
    if (S.max_checked && S.checked >= S.max_checked) S.phase = 2;
    if (S.has_deadline && wall_clock64() >= S.deadline) S.phase = 2;
    // a time budget sizes no tree: stop with the best path so far before a tree could overflow (a run without a
    // path reports the capacity instead)
    if (S.stop_margin && (S.n[0] + S.stop_margin > S.cap || S.n[1] + S.stop_margin > S.cap)) {
      S.phase = 2;
      if (!S.have_sol) S.status = -7;
    }
  }
  __syncthreads();
}

// ----------------------------------------------------------------------------------------------- scout
// Scout: publishes `nbytes` of section p of its record, then (stage >= 0) the stage granule once every wave's
// stores are drained.
__device__ void sc_publish(const Ctx& C, int par, unsigned tag, int stage) {
  const unsigned long long t0 = threadIdx.x == 0 ? pclk() : 0;
  drain();
  __syncthreads();
  if (threadIdx.x == 0) {
    st_agent(&C.Q.scb->stage[par], granule(tag, (unsigned)stage | (g_L.sc_mod & 0xfffu) << 8));
    g_L.S.prof[29] += pclk() - t0;
  }
  __syncthreads();
}
#define SC_PHASE(k) if (threadIdx.x == 0) { const unsigned long long _t = pclk(); g_L.S.prof[k] += _t - _ts; _ts = _t; }
// True (block-uniform) once the leader has moved past the iteration with record tag `tag` (iteration tag - 1):
// the rest of the record would not be used.
__device__ bool sc_stale(const Ctx& C, unsigned tag) {
  if (threadIdx.x == 0) g_L.sp_go[0] = (long long)ld_agent(&C.Q.scb->cur) > (long long)tag - 1 || ld_agent(&C.Q.scb->stop);
  __syncthreads();
  const int s = uni(g_L.sp_go[0]);
  __syncthreads();
  return s != 0;
}

// True (block-uniform) if the leader began a rewire commit on the pass's tree since the pass read it (early asks): the
// pass stops and scout_main rebuilds it on the tree as it is now.
__device__ bool sc_moved(const Ctx& C) {
  // (once the leader is at the pass's iteration, the commits are its own, after it took the record's stages; without
  // early asks the leader publishes no rewire commits: rwb / rwe keep their launch-start values)
  if (!C.Q.early_ask) return false;
  if (threadIdx.x == 0)
    g_L.sc_rerun = (ld_agent(&C.Q.scb->rwb[g_L.sc_t]) & 0xfffu) != g_L.sc_mod &&
                   (long long)ld_agent(&C.Q.scb->cur) < g_L.sc_k;
  __syncthreads();
  const int r = uni(g_L.sc_rerun);
  __syncthreads();
  return r != 0;
}

// Scout, after its record's rewire stage (two scouts, after the first solution): waits until the leader reports
// tree_B of iteration `it` final (its size in the cgo granule) and computes connect's scans for x_new (g_L.xn):
// nearest node, near set, and the segment-norm sums of the direct edge and of the near candidates (stage SC_CONN).
// Publishes SC_CONN with cc.ok = 0 if the leader moved on first.
__device__ void scout_connect(const Ctx& C, long long it, int t, int par, unsigned tag) {
  ScoutRec& R = g_L.sr;
  ScoutBoard* sb = C.Q.scb;
  const int tb = 1 - t;
  for (int k = 0;; k ^= 1) {
    if (threadIdx.x == 0) {
      const unsigned long long v = ld_agent(&sb->cgo);
      int go = 0;
      if ((unsigned)(v >> 32) == tag) { go = 1; g_L.cnt = (int)(unsigned)v; }
      else if ((long long)ld_agent(&sb->cur) > it || ld_agent(&sb->stop)) go = -1;
      g_L.sp_go[k] = go;
    }
    __syncthreads();
    const int go = uni(g_L.sp_go[k]);
    if (go < 0) {  // stale: nobody waits for this record any more
      __syncthreads();  // every wave has read sp_go[k] before scout_main's poll writes it again
      return;
    }
    if (go > 0) break;
    __builtin_amdgcn_s_sleep(2);
  }
  // the tree's stores are the leader's (drained before cgo): drop stale cached copies
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (threadIdx.x == 0) g_L.S.n[tb] = g_L.cnt;
  __syncthreads();
  // the near set of x_new and its nearest node (no exclusion) in one pass over tree_B
  [[clang::always_inline]] near_set<20, true>(C, tb, g_L.xn.q, g_L.xn.id);
  if (threadIdx.x == 0) {
    double d = g_L.fnn_d;
    int cid = g_L.fnn_id;
    if (!(d < 10000.0)) { cid = 0; d = 10000.0; }
    R.cc.d = d; R.cc.id = cid;
    load_node(C, tb, cid, &g_L.xc);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int E = min(g_L.n_lo, g_L.S.max_near);
    g_L.cnt = E;
    for (int j = 0; j < NJ; ++j) { g_L.eg_start[0][j] = g_L.xc.q[j]; g_L.eg_target[0][j] = g_L.xn.q[j]; }
    for (int k = 0; k < 3; ++k) g_L.eg_base[0][k] = 0.0;
  }
  __syncthreads();
  const int E = uni(g_L.cnt);
  if (threadIdx.x < E) {
    const int e = threadIdx.x;
    NodeRef nd;
    load_node(C, tb, g_L.lo_i[e], &nd);
    for (int j = 0; j < NJ; ++j) { g_L.eg_start[1 + e][j] = nd.q[j]; g_L.eg_target[1 + e][j] = g_L.xn.q[j]; }
    for (int k = 0; k < 3; ++k) g_L.eg_base[1 + e][k] = 0.0;
  }
  __syncthreads();
  edge_costs(C, 1 + E);
  // QueryDev::conn_check: the validity of every connect edge (the direct one and each near candidate's, checked to the
  // end) in one more job, so that the leader's connect takes them instead of its own two jobs (direct edge, near loop).
  // Off by default: it lengthens the scout's turn (C2: scout busy 106 -> 121 us per pass, 67.8 -> 71.9 us per leader
  // iteration -- the two post-solution scouts, not the leader's connect, bound the iteration)
  if (uni(C.Q.conn_check)) {
    if (threadIdx.x < MAXE) g_L.eg_need[threadIdx.x] = threadIdx.x < 1 + E;
    if (threadIdx.x == 0) g_L.rec_grp = -1;
    __syncthreads();
    [[clang::always_inline]] edge_validity(C, 1 + E, false, P_XCONNECT);
    if (threadIdx.x < E) R.cc.first[threadIdx.x] = g_L.eg_first[1 + threadIdx.x];
    if (threadIdx.x == 0) { R.cc.first0 = g_L.eg_first[0]; R.cc.nfirst = E; }
  }
  if (threadIdx.x < MAX_NEAR) {
    R.cc.lo_i[threadIdx.x] = g_L.lo_i[threadIdx.x]; R.cc.lo_c[threadIdx.x] = g_L.lo_c[threadIdx.x];
    R.cc.hi_i[threadIdx.x] = g_L.hi_i[threadIdx.x]; R.cc.hi_c[threadIdx.x] = g_L.hi_c[threadIdx.x];
  }
  if (threadIdx.x < E * 3) {
    const int e = threadIdx.x / 3, k = threadIdx.x - e * 3;
    R.cc.acc[e][k] = g_L.eg_acc[1 + e][k];
  }
  if (threadIdx.x == 0) {
    for (int j = 0; j < NJ; ++j) R.cc.q[j] = g_L.xn.q[j];
    for (int k = 0; k < 3; ++k) R.cc.acc0[k] = g_L.eg_acc[0][k];
    R.cc.X = g_L.S.n[tb]; R.cc.t = tb; R.cc.excl = g_L.xn.id;
    R.cc.nk = g_L.nk; R.cc.n_lo = g_L.n_lo; R.cc.n_hi = g_L.n_hi;
    R.cc.ok = 1;
  }
  __syncthreads();
  sc_copy_out(sb, par, &R.cc, sizeof(ScoutConn));
  sc_publish(C, par, tag, SC_CONN);
}

// Scout: ends a record without connect's scans; a post-solution record of two scouts still reaches stage SC_CONN
// (with cc.ok = 0), so the leader never waits for it.
__device__ void sc_end(const Ctx& C, int par, unsigned tag, int opt) {
  if (opt && uni(g_L.two_scouts)) {
    if (threadIdx.x == 0) g_L.sr.cc.ok = 0;
    __syncthreads();
    sc_copy_out(C.Q.scb, par, &g_L.sr.cc, sizeof(ScoutConn));
    sc_publish(C, par, tag, SC_CONN);
  } else {
    sc_publish(C, par, tag, SC_DONE);
  }
}

// Scout, before the first solution, once connect's direct edge is checked (g_L.xc = x_new's nearest node in tree tb,
// g_L.xn = x_new, batch edge 0 = xc -> x_new with its costs and first collision): connectGraphs' outcome without a
// solution (birrt_star.cpp:2608-2812; no near loop then) -> R.pre: the stepping flag and the via chain towards x_new
// (connect) or the last valid point (extend), whose nodes go to the board's pre_via[par].  A chain longer than
// PRE_VIA is not recorded (pre.ok = 0; the leader steps it itself).
__device__ void scout_pre_connect(const Ctx& C, int par, int tb) {
  ScoutRec& R = g_L.sr;
  QState& S = g_L.S;
  if (threadIdx.x == 0) {
    ScoutPre& P = R.pre;
    for (int k = 0; k < 3; ++k) P.sol[k] = g_L.eg_cost[0][k] + g_L.xn.c[k];
    P.need = P.sol[0] < S.cbest[0];
    int flag = 0;
    if (P.need) {
      const int f = g_L.eg_first[0];
      if (f > S.n_pts) {
        flag = 1;
      } else {
        const int lv = f == 0 ? 0 : f - 1;
        if (lv != 0) {
          for (int j = 0; j < NJ; ++j) g_L.ext[j] = g_L.eg_start[0][j] + lv * g_L.eg_step[0][j];
          flag = 2;
        }
      }
    }
    P.flag = flag;
    P.nv = 0;
    P.ok = 1;
    P.sel.id = -1;
    P.sel.parent = -1;
    g_L.flag = flag;
    g_L.n_via = 0;
    g_L.nn_t = S.n[tb];
    g_L.cur = g_L.xc;
  }
  __syncthreads();
  const int flag = uni(g_L.flag);
  if (!flag) return;
  const int vcap = S.via_cap, st0 = S.status, ph0 = S.phase;
  __syncthreads();
  if (threadIdx.x == 0) S.via_cap = PRE_VIA;  // a longer chain stops with status -7 (restored below)
  __syncthreads();
  via_chain(C, flag == 1 ? g_L.xn.q : g_L.ext);
  if (threadIdx.x == 0) {
    ScoutPre& P = R.pre;
    P.ok = S.status == st0;
    S.status = st0;
    S.phase = ph0;
    S.via_cap = vcap;
    P.nv = g_L.n_via;
    P.sel = g_L.sel;
    for (int j = 0; j < NJ; ++j) { P.sel_start[j] = g_L.sel_start[j]; P.sel_target[j] = g_L.sel_target[j]; }
    g_L.n_via = 0;
  }
  // the chain's nodes (plain stores of thread 0 into the scout's via scratch) -> the record slot, agent scope
  drain();
  __syncthreads();
  const int nw = uni(R.pre.ok ? R.pre.nv : 0) * (int)(sizeof(ViaNode) / 8);
  const unsigned long long* src = reinterpret_cast<const unsigned long long*>(C.Q.via);
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(&C.Q.scb->pre_via[par][0]);
  for (int w = threadIdx.x; w < nw; w += BLOCK) st_agent(&dst[w], ld_agent(&src[w]));
}

// Scout, end of a pre-solution pass: the record as PreRec granules (DESIGN.md "Pre-solution commits"); `valid` = 0
// publishes an empty one (t = -1: the leader stops waiting for it).  A via chain's node copies (scout_pre_connect)
// are drained first, so a leader that has the whole record finds them.
__device__ void scout_pre_publish(const Ctx& C, int par, unsigned tag, bool valid) {
  const ScoutRec& R = g_L.sr;
  PreRec& P = g_L.prer;
  if (threadIdx.x == 0) {
    P.t = valid ? R.nn.t : -1;  // (an empty record's other fields are stale and never read)
    P.X = R.nn.X;
    P.nn_id = R.nn.id;
    P.nn_d = R.nn.d;
    P.first = R.e[0].first;
    for (int j = 0; j < NJ; ++j) {
      P.xr[j] = R.nn.q[j]; P.nn_q[j] = R.e[0].s[j]; P.ext[j] = R.ex.ext[j]; P.end[j] = R.ex.end[j];
      P.sel_q[j] = R.pre.sel.q[j]; P.sel_start[j] = R.pre.sel_start[j]; P.sel_target[j] = R.pre.sel_target[j];
    }
    for (int k = 0; k < 3; ++k) {
      P.nn_c[k] = R.nn.c[k]; P.acc[k] = R.ex.acc[k]; P.cn_c[k] = R.cn.c[k]; P.sol[k] = R.pre.sol[k];
      P.sel_c[k] = R.pre.sel.c[k];
    }
    P.cn_ok = R.cn.ok;
    P.cn_d = R.cn.d;
    P.cn_id = R.cn.id;
    P.XB = R.cn.X;
    P.cn_first = R.cn.e.first;
    P.pre_ok = R.cn.ok && R.pre.ok;
    P.flag = R.pre.flag;
    P.nv = R.pre.nv;
    P.need = R.pre.need;
    P.sel_id = R.pre.sel.id;
    P.sel_parent = R.pre.sel.parent;
    P.pad[0] = P.pad[1] = 0;
  }
  __syncthreads();
  if (uni(P.pre_ok && P.nv > 0)) {
    drain();
    __syncthreads();
  }
  for (int g = threadIdx.x; g < PRE_GRANULES; g += BLOCK)
    st_agent(&C.Q.scb->pre_g[par][g], granule((int)tag, reinterpret_cast<const unsigned*>(&P)[g]));
  __syncthreads();
}

// Before the first solution the leader appends nodes while a scout pass runs; one of them nearer to the sample than
// the record's nearest node would make the leader redo the iteration.  True (all threads) when the leader's latest
// drained size of tree t (g_L.cnt, with tree B's in g_L.found) holds such a node: the pass then starts over on those
// sizes, with the record's fields and the snapshot sizes reset (DESIGN.md "Pre-solution refresh").
__device__ __forceinline__ bool pre_newer(const Ctx& C, int t, int X, int XB) {
  QState& S = g_L.S;
  ScoutRec& R = g_L.sr;
  if (threadIdx.x == 0) {
    const unsigned long long sz = ld_agent(&C.Q.scb->cur_sz);
    const int n0 = (int)((sz >> 20) & 0xfffff), n1 = (int)(sz & 0xfffff);
    g_L.cnt = max(X, t == 0 ? n0 : n1);
    g_L.found = max(XB, t == 0 ? n1 : n0);
  }
  __syncthreads();
  const int Xn = uni(g_L.cnt), XBn = uni(g_L.found);
  __syncthreads();
  if (Xn <= X) return false;
  // the nodes [X, Xn) were stored by the leader after this CU may have cached their lines (a line holds 16 nodes of a
  // column): drop stale copies before any load of them, as before a pass (scout_main)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  drain();
  __syncthreads();
  bool again = Xn - X > 64;
  if (!again) {
    double dp;
    tail_scan(C, t, g_L.xr, X, Xn, &dp);
    again = dp < R.nn.d;  // (both uniform: LDS values read after tail_scan's barriers)
  }
  if (!again) return false;
  if (threadIdx.x == 0) {
    S.n[t] = Xn;
    S.n[1 - t] = XBn;
    S.prof[26]++;
    R.cn.ok = 0;
    R.pre.ok = 0;
    R.nn.ok = 0; R.ex.ok = 0; R.nr.ok = 0; R.n_choose = 0; R.n_rewire = 0; R.cc.ok = 0; R.cc.nfirst = -1;
  }
  __syncthreads();
  return true;
}

// The scout's pass for iteration `it` of the leader, which expands tree t from a snapshot of its first X nodes:
// the leader's steps up to its rewire collision job (iteration / choose_parent / rewire, same functions on the
// scout's own LDS, job board, helpers and via-node scratch), recording the results the leader keys on; nothing is
// written to the trees.  The sample is the run-ahead sampler's for (it, ver).
__device__ void scout_iteration(const Ctx& C, long long it, int t, int X, int opt, unsigned ver, int XB) {
  QState& S = g_L.S;
  ScoutRec& R = g_L.sr;
  ScoutBoard* sb = C.Q.scb;
  JobBoard* jb = C.Q.jb;  // this Ctx's board is the scout's; the sampler ring lives on the leader's (sampler_jb)
  const int par = (int)(it & (SCOUT_SLOTS - 1));
  const unsigned tag = (unsigned)(it + 1);
  (void)jb;
  unsigned long long _ts = threadIdx.x == 0 ? pclk() : 0;
#ifdef SMP_TRACE
  if (threadIdx.x == 0) g_L.tit = it;
#endif
  TR();
  if (threadIdx.x == 0) {
    S.prof[30]++;
    S.n[t] = X;
    S.n[1 - t] = XB;
    R.cn.ok = 0;
    R.pre.ok = 0;
    R.nn.ok = 0; R.ex.ok = 0; R.nr.ok = 0; R.n_choose = 0; R.n_rewire = 0; R.cc.ok = 0; R.cc.nfirst = -1;
  }
  if (opt) sc_publish(C, par, tag, SC_STARTED);  // (a pre-solution pass publishes its record once, at its end)
  // the sample: the sampler's ring slot for (it, ver), if it is there within ~20 us
  if (threadIdx.x < 64) {  // wave 0 polls the slot's 16 granules (one round each time)
    const JobBoard* lb = C.Q.sampler_jb;
    const unsigned want = ring_tag(it, ver);
    const unsigned long long t0 = wall_clock64();
    int ok = 0;
    for (;;) {
      unsigned long long v = 0;
      if (threadIdx.x < 2 * NJ) v = ld_agent(&lb->ring[it % SMP_RING].g[threadIdx.x]);
      const bool cur = threadIdx.x >= 2 * NJ || (unsigned)(v >> 32) == want;
      if (__ballot(!cur) == 0) {
        const unsigned hi = (unsigned)odd_lane_of_pair((int)(unsigned)v);
        if (threadIdx.x < 2 * NJ && !(threadIdx.x & 1))
          g_L.xr[threadIdx.x >> 1] = __longlong_as_double((long long)(((unsigned long long)hi << 32) | (unsigned)v));
        ok = 1;
        break;
      }
      if (__builtin_amdgcn_readfirstlane((int)(wall_clock64() - t0 > 2000))) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (threadIdx.x == 0) g_L.flag = ok;
  }
  __syncthreads();
  SC_PHASE(0);
  TR();
  if (!uni(g_L.flag) && !opt) {
    scout_pre_publish(C, par, tag, false);
    return;
  }
  if (!uni(g_L.flag)) {
    sc_copy_out(sb, par, &R.nn, sizeof(ScoutNN));
    sc_copy_out(sb, par, &R.nr, sizeof(ScoutNear));
    sc_copy_out(sb, par, &R.cn, sizeof(ScoutConnect));
    sc_copy_out(sb, par, &R.pre, sizeof(ScoutPre));
    sc_copy_out(sb, par, &R.n_choose, 4 * sizeof(int));
    sc_end(C, par, tag, opt);
    return;
  }
  int rp = 0;  // passes redone on newer tree sizes (pre_refresh)
redo:
  // nearest + expand edge (iteration())
  if (opt && sc_moved(C)) return;
  int nid;
  [[clang::always_inline]] nid = nearest(C, t, g_L.xr);
  if (threadIdx.x < 64) {
    // wave 0: the nearest node's row (lane 0's loads), its distance, and the step towards the sample (step_towards_w:
    // one division and two square-root pairs for the wave instead of a single lane's eight and four)
    const int lane = threadIdx.x;
    if (lane == 0) load_node(C, t, nid, &g_L.nn);
    wave_sync();
    double nq[NJ], xe[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) { nq[j] = g_L.nn.q[j]; xe[j] = g_L.xr[j]; }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) { const double d = xe[j] - nq[j]; s += d * d; }
    const double d = sqrt(s);
    const double nn_l = g_L.nn.q[lane & 7];
    double x_l = g_L.xr[lane & 7];
    step_towards_w(rev_mask(&g_rb), nq, xe, S.step, lane, nn_l, x_l);
    if (lane < NJ) {
      R.nn.q[lane] = g_L.xr[lane];
      g_L.ext[lane] = x_l;
      g_L.eg_start[0][lane] = nn_l;
      g_L.eg_target[0][lane] = x_l;
    } else if (lane < NJ + 3) {
      const int k = lane - NJ;
      R.nn.c[k] = g_L.nn.c[k];
      g_L.eg_base[0][k] = g_L.nn.c[k];
    } else if (lane == NJ + 3) {
      R.nn.d = d < 10000.0 ? d : 10000.0;
      R.nn.id = nid; R.nn.X = X; R.nn.t = t; R.nn.ok = 1;
      g_L.eg_need[0] = 1;
    }
  }
  __syncthreads();
  if (opt) {
    sc_copy_out(sb, par, &R.nn, sizeof(ScoutNN));
    sc_publish(C, par, tag, SC_NN);
  }
  SC_PHASE(1);
  TR();
  if (opt && sc_moved(C)) return;
  edge_costs(C, 1);
  if (threadIdx.x == 0) {  // the expand edge's interpolation data, for the leader (published with SC_EXPAND)
    for (int j = 0; j < NJ; ++j) { R.ex.ext[j] = g_L.eg_target[0][j]; R.ex.step[j] = g_L.eg_step[0][j]; R.ex.end[j] = g_L.eg_end[0][j]; }
    for (int k = 0; k < 3; ++k) R.ex.acc[k] = g_L.eg_acc[0][k];
    R.ex.ok = 1;
  }
  // the near set of the edge's end (x_new if the edge is valid) is scanned while the helpers check the edge.
  // Before the first solution connect's direct edge goes into the same job: x_new is the expand edge's end if that
  // edge is valid, so its nearest node in the other tree (over that tree's first XB nodes; it only grows until then)
  // and the edge from it are known now; the connect half is dropped when the expand edge collides.
  if (threadIdx.x == 0) g_L.spec = OV_NONE;
  const bool spec_conn = !opt && !sc_stale(C, tag);
  int cid_s = 0;
  if (spec_conn) {
    const int tb = 1 - t;
    [[clang::always_inline]] cid_s = nearest(C, tb, g_L.eg_end[0]);
    if (threadIdx.x == 0) {
      load_node(C, tb, cid_s, &g_L.xc);
      for (int j = 0; j < NJ; ++j) { g_L.eg_start[1][j] = g_L.xc.q[j]; g_L.eg_target[1][j] = g_L.eg_end[0][j]; }
      for (int k = 0; k < 3; ++k) g_L.eg_base[1][k] = g_L.xc.c[k];
      g_L.eg_need[1] = 1;
    }
    for (int e = 2 + threadIdx.x; e < MAXE; e += BLOCK) g_L.eg_need[e] = 0;
    __syncthreads();
    edge_costs(C, 2);
    [[clang::always_inline]] edge_validity(C, 2, false, P_XEXPAND, OV_NONE, t);
  } else {
    [[clang::always_inline]] edge_validity(C, 1, false, P_XEXPAND, opt ? OV_NEAR_EXPAND : OV_NONE, t);
  }
  if (threadIdx.x == 0) {
    for (int j = 0; j < NJ; ++j) { R.e[0].s[j] = g_L.eg_start[0][j]; R.e[0].g[j] = g_L.eg_target[0][j]; }
    for (int k = 0; k < 3; ++k) R.e[0].acc[k] = g_L.eg_acc[0][k];
    R.e[0].first = g_L.eg_first[0];
    const int f = g_L.eg_first[0];
    g_L.ext_nn = f > S.n_pts;
    if (g_L.ext_nn) {
      for (int j = 0; j < NJ; ++j) g_L.xn.q[j] = g_L.eg_end[0][j];
      for (int k = 0; k < 3; ++k) g_L.xn.c[k] = g_L.eg_cost[0][k];
    } else {
      for (int j = 0; j < NJ; ++j) g_L.xn.q[j] = g_L.xr[j];
      g_L.xn.c[0] = 10000.0; g_L.xn.c[1] = 0.0; g_L.xn.c[2] = 0.0;
    }
    g_L.xn.id = X;
    g_L.xn.parent = g_L.nn.id;
    g_L.ext_bp = 0;
  }
  __syncthreads();
  if (!opt && (C.Q.pre_refresh & 1) && rp < 2 && pre_newer(C, t, X, XB)) {
    X = uni(g_L.cnt);
    XB = uni(g_L.found);
    rp++;
    goto redo;
  }
  if (opt) {
    sc_copy_out(sb, par, &R.e[0], sizeof(ScoutEdge));
    sc_copy_out(sb, par, &R.ex, sizeof(ScoutExpand));
  }
  if (spec_conn && uni(g_L.ext_nn)) {
    // before the first solution the iteration goes on with connect (connectGraphs): x_new is the expand edge's
    // end, and its direct edge from the nearest node of the other tree (whose check always runs while there is
    // no solution, c_best = inf) was checked in the expand job; its data move to edge slot 0
    const int tb = 1 - t;
    const int cid = cid_s;
    if (threadIdx.x < NJ) {
      const int j = threadIdx.x;
      g_L.eg_start[0][j] = g_L.eg_start[1][j]; g_L.eg_target[0][j] = g_L.eg_target[1][j];
      g_L.eg_step[0][j] = g_L.eg_step[1][j]; g_L.eg_end[0][j] = g_L.eg_end[1][j];
    }
    if (threadIdx.x < 3) {
      const int k = threadIdx.x;
      g_L.eg_base[0][k] = g_L.eg_base[1][k]; g_L.eg_acc[0][k] = g_L.eg_acc[1][k]; g_L.eg_cost[0][k] = g_L.eg_cost[1][k];
    }
    if (threadIdx.x == 0) {
      g_L.eg_first[0] = g_L.eg_first[1];
      double s = 0.0;
      for (int j = 0; j < NJ; ++j) { double d = g_L.xn.q[j] - g_L.xc.q[j]; s += d * d; }
      const double d = sqrt(s);
      for (int j = 0; j < NJ; ++j) R.cn.q[j] = g_L.xn.q[j];
      R.cn.d = d < 10000.0 ? d : 10000.0;
      R.cn.id = cid; R.cn.X = XB; R.cn.t = tb;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int j = 0; j < NJ; ++j) { R.cn.e.s[j] = g_L.eg_start[0][j]; R.cn.e.g[j] = g_L.eg_target[0][j]; }
      for (int k = 0; k < 3; ++k) { R.cn.e.acc[k] = g_L.eg_acc[0][k]; R.cn.c[k] = g_L.xc.c[k]; }
      R.cn.e.first = g_L.eg_first[0];
      R.cn.ok = 1;
    }
    __syncthreads();
    scout_pre_connect(C, par, tb);
  }
  if (!opt && (C.Q.pre_refresh & 2) && rp < 2 && pre_newer(C, t, X, XB)) {
    X = uni(g_L.cnt);
    XB = uni(g_L.found);
    rp++;
    goto redo;
  }
  if (!opt) {
    scout_pre_publish(C, par, tag, true);
    return;
  }
  if (sc_stale(C, tag)) {
    sc_copy_out(sb, par, &R.nr, sizeof(ScoutNear));
    sc_copy_out(sb, par, &R.n_choose, 4 * sizeof(int));
    sc_publish(C, par, tag, SC_DONE);
    return;
  }
  sc_publish(C, par, tag, SC_EXPAND);
  SC_PHASE(2);
  TR();
  if (sc_moved(C)) return;
  // near set of x_new (the leader's, before choose_parent)
  if (!(uni(g_L.ext_nn) && take_spec(OV_NEAR_EXPAND))) {
    [[clang::always_inline]] near_set<20>(C, t, g_L.xn.q, X);
  }
  if (threadIdx.x < 20) {
    R.nr.lo_i[threadIdx.x] = g_L.lo_i[threadIdx.x]; R.nr.lo_c[threadIdx.x] = g_L.lo_c[threadIdx.x];
    R.nr.hi_i[threadIdx.x] = g_L.hi_i[threadIdx.x]; R.nr.hi_c[threadIdx.x] = g_L.hi_c[threadIdx.x];
  }
  if (threadIdx.x == 0) {
    for (int j = 0; j < NJ; ++j) R.nr.q[j] = g_L.xn.q[j];
    R.nr.nk = g_L.nk; R.nr.n_lo = g_L.n_lo; R.nr.n_hi = g_L.n_hi;
    R.nr.X = X; R.nr.t = t; R.nr.ok = 1;
  }
  __syncthreads();
  sc_copy_out(sb, par, &R.nr, sizeof(ScoutNear));
  sc_publish(C, par, tag, SC_NEAR);
  SC_PHASE(3);
  TR();
  if (sc_moved(C)) return;
  // choose_parent's candidate edges (all needed ones checked: the job computes every tile)
  if (threadIdx.x < 64) {
    const int E = choose_prefix();
    if (threadIdx.x == 0) {
      g_L.cnt = E;
      g_L.found = -1;
    }
  }
  __syncthreads();
  const int E = uni(g_L.cnt);
  if (E > 0) {
    if (threadIdx.x < E) {
      const int e = threadIdx.x;
      NodeRef nd;
      load_node(C, t, g_L.lo_i[e], &nd);
      for (int j = 0; j < NJ; ++j) { g_L.eg_start[e][j] = nd.q[j]; g_L.eg_target[e][j] = g_L.xn.q[j]; }
      for (int k = 0; k < 3; ++k) g_L.eg_base[e][k] = nd.c[k];
      g_L.eg_near[e] = nd.id;
    }
    __syncthreads();
    edge_costs(C, E);
    if (threadIdx.x < E) g_L.eg_need[threadIdx.x] = g_L.eg_cost[threadIdx.x][0] <= g_L.xn.c[0];
    for (int e = E + threadIdx.x; e < MAXE; e += BLOCK) g_L.eg_need[e] = 0;
    __syncthreads();
    [[clang::always_inline]] edge_validity(C, E, false, P_XCHOOSE);
    if (threadIdx.x < E) {
      const int e = threadIdx.x;
      ScoutEdge& w = R.e[SCOUT_CHOOSE0 + e];
      for (int j = 0; j < NJ; ++j) { w.s[j] = g_L.eg_start[e][j]; w.g[j] = g_L.eg_target[e][j]; }
      for (int k = 0; k < 3; ++k) w.acc[k] = g_L.eg_acc[e][k];
      w.first = g_L.eg_need[e] ? g_L.eg_first[e] : -1;
    }
    if (threadIdx.x < 64) {  // the first needed candidate that is free (ballot: E <= 20)
      const bool fr = (int)threadIdx.x < E && g_L.eg_need[threadIdx.x] && g_L.eg_first[threadIdx.x] > S.n_pts;
      const unsigned long long fm = __ballot(fr);
      if (threadIdx.x == 0) {
        R.n_choose = E;
        if (fm) g_L.found = (int)__builtin_ctzll(fm);
      }
    }
    __syncthreads();
  }
  sc_copy_out(sb, par, &R.n_choose, 4 * sizeof(int));
  sc_copy_out(sb, par, &R.e[SCOUT_CHOOSE0], E * (int)sizeof(ScoutEdge));
  if (sc_stale(C, tag)) { sc_publish(C, par, tag, SC_DONE); return; }
  sc_publish(C, par, tag, SC_CHOOSE);
  SC_PHASE(4);
  TR();
  if (uni(g_L.found) >= 0) {
    // x_new <- the last edge of the via chain from the chosen parent (choose_parent)
    if (threadIdx.x == 0) {
      g_L.n_via = 0;
      g_L.nn_t = X;
      load_node(C, t, g_L.eg_near[g_L.found], &g_L.cur);
    }
    __syncthreads();
    via_chain(C, g_L.xn.q);
    if (threadIdx.x == 0) {
      g_L.xn.id = g_L.sel.id;
      g_L.xn.parent = g_L.sel.parent;
      for (int j = 0; j < NJ; ++j) g_L.xn.q[j] = g_L.sel.q[j];
      for (int k = 0; k < 3; ++k) g_L.xn.c[k] = g_L.sel.c[k];
      g_L.ext_bp = 1;
      g_L.n_via = 0;
    }
    __syncthreads();
  }
  SC_PHASE(5);
  TR();
  if (!uni(g_L.ext_nn || g_L.ext_bp)) { sc_end(C, par, tag, opt); return; }
  if (sc_moved(C)) return;
  // rewire's candidate edges (rewire())
  const TreeDev& T = C.Q.tr[t];
  rewire_count(T);
  const int cnt = uni(g_L.cnt);
  if (cnt > 0) {
    if (threadIdx.x < cnt) {
      const int e = threadIdx.x, v = g_L.hi_i[g_L.n_hi - 1 - e];
      NodeRef nd;
      load_node(C, t, v, &nd);
      for (int j = 0; j < NJ; ++j) { g_L.eg_start[e][j] = g_L.xn.q[j]; g_L.eg_target[e][j] = nd.q[j]; }
      for (int k = 0; k < 3; ++k) g_L.eg_base[e][k] = g_L.xn.c[k];
      g_L.eg_near[e] = v;
    }
    __syncthreads();
    edge_costs(C, cnt);
    if (threadIdx.x < cnt) {
      const int e = threadIdx.x, v = g_L.eg_near[e];
      g_L.eg_need[e] = (v != g_L.xn.parent) && (T.parent[v] != 0) && (g_L.eg_cost[e][0] < T.cost[v]);
    }
    for (int e = cnt + threadIdx.x; e < MAXE; e += BLOCK) g_L.eg_need[e] = 0;
    __syncthreads();
    [[clang::always_inline]] edge_validity(C, cnt, false, P_XREWIRE);
    if (threadIdx.x < cnt) {
      const int e = threadIdx.x;
      ScoutEdge& w = R.e[SCOUT_REWIRE0 + e];
      for (int j = 0; j < NJ; ++j) { w.s[j] = g_L.eg_start[e][j]; w.g[j] = g_L.eg_target[e][j]; }
      for (int k = 0; k < 3; ++k) w.acc[k] = g_L.eg_acc[e][k];
      w.first = g_L.eg_need[e] ? g_L.eg_first[e] : -1;
    }
    if (threadIdx.x == 0) R.n_rewire = cnt;
    __syncthreads();
  }
  sc_copy_out(sb, par, &R.n_choose, 4 * sizeof(int));
  sc_copy_out(sb, par, &R.e[SCOUT_REWIRE0], cnt * (int)sizeof(ScoutEdge));
  sc_publish(C, par, tag, SC_DONE);
  SC_PHASE(6);
  TR();
  if (sc_moved(C)) return;
  if (uni(g_L.two_scouts)) {
    [[clang::always_inline]] scout_connect(C, it, t, par, tag);
  }
  TR();
}
#undef SC_PHASE

// Scout workgroup `which` of a query (plan_kernel): takes the leader's newest request, runs scout_iteration on it,
// repeats; leaves on the stop flag (then stops its helpers) or after two idle seconds.
// A scout's context: its own record board, job board, helpers and via scratch; collision jobs go to its own board and
// helpers, the run-ahead sampler's ring stays the leader's.
__device__ __forceinline__ void scout_ctx(Ctx& C, int which) {
  C.Q.scb = C.Q.scbs[which];
  C.Q.sjb = C.Q.sjbs[which];
  C.Q.svia = C.Q.svias[which];
  C.Q.sworkers = C.Q.sworkers_s[which];
  C.Q.sampler_jb = C.Q.jb;
  C.Q.jb = C.Q.sjb;
  C.Q.nworkers = C.Q.sworkers;
  C.Q.via = C.Q.svia;
  C.Q.rows = nullptr;
  C.Q.trace = nullptr;
  C.Q.ttff = nullptr;
}

__device__ __noinline__ void scout_main(Ctx& C, int which) {
  {
    const int* src = reinterpret_cast<const int*>(C.Q.st);
    int* dst = reinterpret_cast<int*>(&g_L.S);
    for (int i = threadIdx.x; i < (int)(sizeof(QState) / sizeof(int)); i += BLOCK) dst[i] = src[i];
  }
  __syncthreads();
  if (threadIdx.x < 32) g_L.S.prof[threadIdx.x] = 0;
  if (threadIdx.x == 0) {
    g_L.count_slot = 0;
    g_L.job_seq = 0;
    g_L.in_job = 0;
    g_L.n_via = 0;
    g_L.near_blo = ~0ull;
    g_L.near_bhi = 0;
    g_L.spec = OV_NONE;
    g_L.sp_on = 0;
    st_agent(&C.Q.scb->xcc, xcc_id() + 1);
    g_L.two_scouts = C.Q.nscouts >= 2;
    g_L.rec_grp = -1;
#ifdef SMP_TRACE
    g_L.trole = which + 1 < 3 ? which + 1 : 3;
    g_L.tit = -1;
    g_L.tn = g_tlog_n[g_L.trole];
#endif
  }
  __syncthreads();
  unsigned last = 0;
  unsigned long long t_last = wall_clock64();
  // scouts 2 and up only serve iterations before the first solution (scout_ask): in a launch that starts after it
  // they retire at once, with their helpers, instead of polling beside the leader for the whole launch
#ifdef SMP_NO_RETIRE
  const bool retired = false;
#else
  const bool retired = which >= 2 && uni(g_L.S.tree_opt && g_L.S.have_sol);
#endif
  // the last pass's request: a post-solution pass is rebuilt when the leader rewires its tree after asking for it
  // (early asks, ScoutBoard::rwb / rwe) and the leader has not yet moved past the iteration
  unsigned l_w0 = 0, l_ver = 0;
  int l_X = 0, l_XB = 0;
  if (threadIdx.x == 0) { g_L.sc_mod = 0; g_L.sc_t = 0; g_L.sc_rerun = 0; }
  for (int k = 0; !retired; k ^= 1) {
    if (threadIdx.x == 0) {
      int go = 0;
      if (ld_agent(&C.Q.scb->stop)) {
        go = -1;
      } else {
        const unsigned long long r0 = ld_agent(&C.Q.scb->req[0]), r1 = ld_agent(&C.Q.scb->req[1]);
        const unsigned long long r2 = ld_agent(&C.Q.scb->req[2]);
        const unsigned tag = (unsigned)(r0 >> 32);
        if (tag > last && (unsigned)(r1 >> 32) == tag && (unsigned)(r2 >> 32) == tag) {
          go = 1;
          g_L.cnt = (int)(unsigned)r0;        // X | t << 28 | opt << 29
          g_L.nn_t = (int)(unsigned)r1;       // sampler parameter version | rewire commits of tree t << 20
          g_L.found = (int)(unsigned)r2;      // XB
          g_L.tree_expand = (int)tag;
        } else if (last && C.Q.early_ask && ((l_w0 >> 29) & 1u) &&
                   (ld_agent(&C.Q.scb->rwb[(l_w0 >> 28) & 1u]) & 0xfffu) != g_L.sc_mod &&
                   (long long)ld_agent(&C.Q.scb->cur) < (long long)last - 1) {
          go = 2;  // the last record's tree was rewired after it was built: rebuild it
        } else if (wall_clock64() - t_last > 200000000ull) {
          go = -1;  // 2 s idle
        }
      }
      g_L.sp_go[k] = go;
    }
    __syncthreads();
    const int go = uni(g_L.sp_go[k]);
    if (go < 0) break;
    if (go == 0) {
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    unsigned w0, ver, tag;
    int X, XB;
    if (go == 1) {
      const unsigned r1w = (unsigned)uni(g_L.nn_t);
      w0 = (unsigned)uni(g_L.cnt);
      ver = r1w & 0xfffffu;
      tag = (unsigned)uni(g_L.tree_expand);
      XB = uni(g_L.found);
      X = (int)(w0 & ((1u << 28) - 1));
      __syncthreads();
      if (threadIdx.x == 0) g_L.sc_mod = (r1w >> 20) & 0xfffu;
    } else {
      w0 = l_w0; ver = l_ver; tag = last; X = l_X; XB = l_XB;
    }
    const int t = (int)(w0 >> 28) & 1, opt = (int)(w0 >> 29) & 1;
    __syncthreads();
    if (go == 1 && !opt && C.Q.pre_delay > 0) {
      // before the first solution: start once the leader is pre_delay iterations from this one, on the tree sizes
      // it published after its latest drain (trees only grow until the first solution, so they are at least the
      // request's): fewer nodes appended between the snapshot and the record's use, fewer records a newer node beats
      const long long k = (long long)tag - 1;
      for (int r = 0;; r ^= 1) {
        if (threadIdx.x == 0) {
          const long long cur = (long long)ld_agent(&C.Q.scb->cur);
          const int go = cur >= k - C.Q.pre_delay || ld_agent(&C.Q.scb->stop);
          if (go) {
            const unsigned long long sz = ld_agent(&C.Q.scb->cur_sz);
            const int n0 = (int)((sz >> 20) & 0xfffff), n1 = (int)(sz & 0xfffff);
            g_L.cnt = max(X, t == 0 ? n0 : n1);
            g_L.found = max(XB, t == 0 ? n1 : n0);
          }
          g_L.sp_go[r] = go;
        }
        __syncthreads();
        if (uni(g_L.sp_go[r])) break;
        __builtin_amdgcn_s_sleep(2);
      }
      X = uni(g_L.cnt);
      XB = uni(g_L.found);
      __syncthreads();
    }
    l_w0 = w0; l_ver = ver; l_X = X; l_XB = XB;
    const unsigned long long tb = wall_clock64();
    if (threadIdx.x == 0) g_L.S.prof[28] += tb - t_last;  // idle: waiting for a request
    for (;;) {  // the pass, rebuilt while the leader rewires its tree under it
      if (opt && C.Q.early_ask) {
        // the tree as the leader left it: a begun rewire commit is waited for until its words are stored
        int st = 0;
        for (int r = 0;; r ^= 1) {
          if (threadIdx.x == 0) {
            const unsigned b = ld_agent(&C.Q.scb->rwb[t]);
            int v;
            if ((b & 0xfffu) == g_L.sc_mod) v = 1;
            else if (ld_agent(&C.Q.scb->stop) || (long long)ld_agent(&C.Q.scb->cur) > (long long)tag - 1) v = -1;
            else if (ld_agent(&C.Q.scb->rwe[t]) == b) { v = 1; g_L.sc_mod = b & 0xfffu; }
            else v = 0;
            g_L.rb_go[r] = v;
          }
          __syncthreads();
          st = uni(g_L.rb_go[r]);
          if (st != 0) break;
          __builtin_amdgcn_s_sleep(1);
        }
        __syncthreads();  // every wave has read rb_go before it is written again
        if (st < 0) break;
      }
      if (threadIdx.x == 0) { g_L.sc_t = t; g_L.sc_rerun = 0; g_L.sc_k = (long long)tag - 1; }
      // tree words stored by the leader since this CU / XCD last cached them: drop stale copies (the invalidate
      // completes asynchronously: every wave waits for it before its first plain load, MI355X_MICROARCH.md consumer
      // form)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      drain();
      __syncthreads();
      [[clang::always_inline]] scout_iteration(C, (long long)tag - 1, t, X, opt, ver, XB);
      if (!opt || !uni(g_L.sc_rerun)) break;
      __syncthreads();
    }
    last = tag;
    t_last = wall_clock64();
    if (threadIdx.x == 0) g_L.S.prof[31] += t_last - tb;
  }
  if (threadIdx.x == 0) {
    st_agent(&C.Q.jb->stop, 1);
    for (int k = 0; k < 32; ++k) st_agent(&C.Q.scb->prof[k], g_L.S.prof[k]);
  }
}

// Run-ahead sampler (DESIGN.md "Sampler"): keeps the samples of the leader's next SMP_RING - 1 iterations in
// the ring, computed with the latest published parameters and tagged (iteration, version); a parameter change
// restarts the window.  Never writes the slot of an iteration the leader may be reading: it fills iterations
// up to (published iteration) + SMP_RING - 1 only.  Leaves on the stop flag or after two idle seconds.
// (not inlined into helper_main, like scan_helper: the tile helpers' loop is compiled without the sampler's and the
// scan slices' registers live around it -- C2 73.1 -> 71.8 us per iteration, perf_probe.py with SMP_JOB_PROF, round 3)
__device__ __forceinline__ void sampler_body(const Ctx& C, SamplerLds& L) {
  JobBoard* jb = C.Q.jb;
  {
    const int* src = reinterpret_cast<const int*>(C.Q.st);
    int* dst = reinterpret_cast<int*>(&L.S);
    for (int i = threadIdx.x; i < (int)(sizeof(QState) / sizeof(int)); i += BLOCK) dst[i] = src[i];
  }
  if (threadIdx.x == 0) { L.ver = 0; L.next = 0; }
  __syncthreads();
  unsigned long long t_last = wall_clock64();
  for (int k = 0;; k ^= 1) {
    if (threadIdx.x == 0) {
      int go = 0;
      if (ld_agent(&jb->stop)) {
        go = -1;
      } else {
        const int ver = ld_agent(&jb->s_ver);
        const long long cur = (long long)ld_agent(reinterpret_cast<const unsigned long long*>(&jb->s_iter));
        if (ver != L.ver) {
          L.S.have_sol = ld_agent(&jb->s_have_sol);
          for (int c = 0; c < 3; ++c) L.S.cbest[c] = __longlong_as_double((long long)ld_agent(&jb->s_cbest[c]));
          if (ld_agent(&jb->s_ver) == ver) { L.ver = ver; L.next = cur + 1; }  // else re-read next poll
        }
        if (L.next < cur + 1) L.next = cur + 1;
        if (L.ver > 0 && ver == L.ver && L.next <= cur + SMP_RING - 1) go = 1;
        else if (wall_clock64() - t_last > 200000000ull) go = -1;  // 2 s idle
      }
      L.go[k] = go;
    }
    __syncthreads();
    const int go = uni(L.go[k]);
    if (go < 0) break;
    if (go == 0) {
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    const long long it = L.next;
    const int st = sample_conf(L.S, (uint32_t)it, L.W, L.out);
#ifdef SMP_RING_CHECK
    if (threadIdx.x == 0) {
      unsigned long long* d = g_ringdbg[it % SMP_RING];
      st_agent(&d[0], (unsigned long long)it); st_agent(&d[1], (unsigned long long)L.ver);
      st_agent(&d[2], (unsigned long long)L.S.have_sol);
      for (int k = 0; k < 3; ++k) st_agent(&d[3 + k], (unsigned long long)__double_as_longlong(L.S.cbest[k]));
      st_agent(&d[6], (unsigned long long)L.S.informed);
      const RobotDev* rb = (&g_rb);
      const double lv[6] = {L.S.h0[1], L.S.Crev[0], L.S.Crev[7], L.S.ctr_rev[0], rb->q_min[2], rb->q_max[2]};
      for (int k = 0; k < 6; ++k) st_agent(&d[8 + k], (unsigned long long)__double_as_longlong(lv[k]));
      unsigned long long rv = 0;
      for (int j = 0; j < NJ; ++j) rv |= (unsigned long long)(rb->rev[j] != 0) << j;
      st_agent(&d[14], rv);
    }
#endif
    if (st == 0 && threadIdx.x < RING_G) {
      unsigned w;
      if (threadIdx.x < 2 * NJ) {
        const unsigned long long bits = (unsigned long long)__double_as_longlong(L.out[threadIdx.x >> 1]);
        w = (threadIdx.x & 1) ? (unsigned)(bits >> 32) : (unsigned)bits;
      } else {
        w = ring_param((int)threadIdx.x - 2 * NJ, L.S.have_sol, L.S.cbest);
      }
      st_agent(&jb->ring[it % SMP_RING].g[threadIdx.x], granule((int)ring_tag(it, L.ver), w));
    }
    if (threadIdx.x == 0) L.next = it + 1;
    t_last = wall_clock64();
    __syncthreads();
  }
}

__device__ __noinline__ void sampler_main(const Ctx& C, SamplerLds& L) { sampler_body(C, L); }


// Advances every query (one workgroup each) by at most `iters` planner iterations.  One launch holds every workgroup of
// its queries (DESIGN.md "Execution model"): blocks [0, nq) are the leaders (the planner loop); scout s of query q is
// block scout_base + s * r8 + q (scout_base and r8 = nq rounded up to 8 are multiples of 8, and blocks are dealt to the 8
// XCDs round-robin: a query's leader and scouts share an XCD); from helper_base (a multiple of 8) block helper_base + h *
// nq + q is helper h of query q -- the leader's tile helpers first, then each scout's, the run-ahead sampler last.  Every
// role of a query runs in this one dispatch: the helpers are co-resident with the workgroups that publish their jobs,
// and a kernel trace or a counter pass sees the whole query as one kernel.
__global__ void __launch_bounds__(BLOCK) plan_kernel(const RobotDev* __restrict__ rb, SceneDev sc,
                                                     const MapCfg* __restrict__ mc, QueryDev* qs, int nq, int scout_base,
                                                     int helper_base, int iters) {
  const int b = (int)blockIdx.x;
  const int r8 = (nq + 7) / 8 * 8;
  const int so = b - scout_base, srole = scout_base > 0 && b >= scout_base && b < helper_base ? so / r8 : -1;
  const int sq = srole >= 0 ? so - srole * r8 : b;
  // the block's context in LDS: every function takes it by reference, and a private copy would live in scratch (each
  // field read a scratch load, invalidated with the L1 by every acquire)
  __shared__ Ctx g_ctx;
  __shared__ int g_role;
  if (b >= helper_base) {
    // helper block: -1 nothing to do, -2 run-ahead sampler, else tile helper h of the leader or of a scout
    if (threadIdx.x == 0) {
      Ctx c;
      c.sc = sc;
      c.Q = qs[(b - helper_base) % nq];
      const int hidx = (b - helper_base) / nq, nh = ((int)gridDim.x - helper_base) / nq;
      int role = hidx;
      if (!c.Q.jb) {
        role = -1;
      } else if (c.Q.sampler && hidx == nh - 1) {
        role = -2;
      } else if (role >= c.Q.nworkers - 1) {  // the leader's tile helpers first, then each scout's
        role -= c.Q.nworkers - 1;
        int s = 0;
        for (; s < c.Q.nscouts && role >= c.Q.sworkers_s[s] - 1; ++s) role -= c.Q.sworkers_s[s] - 1;
        if (s >= c.Q.nscouts) {
          role = -1;
        } else {
          c.Q.jb = c.Q.sjbs[s];
          c.Q.nworkers = c.Q.sworkers_s[s];
        }
      }
      g_ctx = c;
      g_role = role;
    }
    stage_model(rb, mc, &g_rb, &g_mc);  // (ends with a barrier)
    const int role = uni(g_role);
    if (role == -2) sampler_main(g_ctx, g_L.u.smpl);
    else if (role >= 0) helper_main(g_ctx, role, g_L.u.job);
    return;
  }
  if (b >= nq && (srole < 0 || sq >= nq)) return;
  if (threadIdx.x == 0) {
    Ctx c;
    c.sc = sc;
    c.Q = qs[sq];
    if (srole >= 0 && srole < c.Q.nscouts) scout_ctx(c, srole);
    g_ctx = c;
  }
  stage_model(rb, mc, &g_rb, &g_mc);  // (ends with a barrier)
  Ctx& C = g_ctx;
  if (srole >= 0) {
    if (srole < C.Q.nscouts) scout_main(C, srole);  // one call site: inlined
    return;
  }
  if (threadIdx.x == 0) {
    g_L.sp_on = 0;
    for (int k = 0; k < MAX_SCOUTS; ++k) g_L.sc_same[k] = -1;
    g_L.sc_seen = 0;
    g_L.sc_dead = 0;
    for (int k = 0; k < SCOUT_SLOTS; ++k) { g_L.asked[k] = 0; g_L.asked_conn[k] = 0; g_L.asked_pre[k] = 0; }
    g_L.conn_rec = 0;
    g_L.rec_grp = -1;
    g_L.count_slot = 0;
    g_L.job_seq = 0;
    g_L.in_job = 0;
    g_L.S = *C.Q.st;
    if (g_L.S.phase == 0 && g_L.S.t0 == 0) {
      g_L.S.t0 = wall_clock64();
      // run_planner reads the wall clock every iteration (birrt_star.cpp:1313-1320): the budget counts from here
      if (g_L.S.has_deadline) g_L.S.deadline = g_L.S.t0 + g_L.S.budget_ticks;
    }
    g_L.n_via = 0;
    g_L.near_blo = ~0ull;
    g_L.near_bhi = 0;
    g_L.smp_ver = 0;
    // the scouts' rewire-commit counters start at the trees' counts (the boards were zeroed for this launch)
    for (int s = 0; s < C.Q.nscouts && s < 2; ++s)
      for (int t = 0; t < 2; ++t) {
        st_agent(reinterpret_cast<int*>(&C.Q.scbs[s]->rwb[t]), g_L.S.rewires[t]);
        st_agent(reinterpret_cast<int*>(&C.Q.scbs[s]->rwe[t]), g_L.S.rewires[t]);
      }
    drain();  // before any request reaches a scout
#ifdef SMP_TRACE
    g_L.trole = 0;
    g_L.tit = 0;  // the pre-loop's records go with iteration 0's
    g_L.tn = g_tlog_n[0];
#endif
  }
  __syncthreads();
  TR();
  if (uni(g_L.S.status == 0 && g_L.S.phase == 0)) {
    // first launch: init_planner's validity of start and goal (birrt_star.cpp:350-362), one collision tile
    if (threadIdx.x < 2 * NJ) {
      const int c = threadIdx.x / NJ, j = threadIdx.x - c * NJ;
      g_L.u.tile.tq[c][j] = c == 0 ? g_L.S.qs[j] : g_L.S.qg[j];
    }
    __syncthreads();
    collide_tile<PLAN_CT>((&g_rb), C.sc, (&g_mc), 2, g_L.u.tile.tq, g_L.S.self, g_L.S.map, g_L.u.tile.T);
    if (threadIdx.x == 0 && (g_L.u.tile.T.coll[0] || g_L.u.tile.T.coll[1])) {
      g_L.S.status = g_L.u.tile.T.coll[0] ? -2 : -3;  // SMP_ERR_START_INVALID / SMP_ERR_GOAL_INVALID
      g_L.S.phase = 2;
    }
    __syncthreads();
    TR();
  }
  if (uni(g_L.S.status == 0 && g_L.S.phase == 0) && threadIdx.x < 2) {
    // first launch: the two roots (init_planner, birrt_star.cpp:386-443) from the query's start / goal
    const int t = threadIdx.x, cap = g_L.S.cap;
    const TreeDev& T = C.Q.tr[t];
    for (int j = 0; j < NJ; ++j) st_coord(T, cap, j, 0, t == 0 ? g_L.S.qs[j] : g_L.S.qg[j]);
    for (int k = 0; k < 3; ++k) T.cost[(size_t)k * cap] = 0.0;
    T.parent[0] = 0;
    T.first_child[0] = -1;
    T.next_sib[0] = -1;
    T.prev_sib[0] = -1;
  }
  __syncthreads();
  // the last PATCH_K nodes of each tree -> the LDS copy kept by insert_node / insert_via
  for (int it = threadIdx.x; it < 2 * PATCH_K * NJ; it += BLOCK) {
    const int t = it / (PATCH_K * NJ), r = it - t * (PATCH_K * NJ), k = r / NJ, j = r - k * NJ;
    const int i = g_L.S.n[t] - PATCH_K + k;
    if (i >= 0) g_L.pc_q[t][i & (PATCH_K - 1)][j] = C.Q.tr[t].q[(size_t)j * g_L.S.cap + i];
  }
  __syncthreads();
  if (uni(g_L.S.status == 0 && g_L.S.phase == 0 && C.Q.nscouts > 0 && C.Q.pre_commit && C.Q.sampler)) {
    // first launch, before the pre-loop connection: the sampling parameters (version 1: the run-ahead sampler starts
    // filling its ring now) and the first iterations' pre-solution records.  Until the first solution the trees only
    // grow, so a record of the roots' snapshot stays exact up to the nodes appended since -- the connection's via nodes
    // included -- which the leader patches in as for any record: the scouts work while the leader checks the direct
    // connection, instead of starting with iteration 0.
    drain();  // the roots' stores
    __syncthreads();
    if (threadIdx.x == 0) {
      sample_version(C);
      sample_publish(C, true);
      bool fenced = false;
      const long long j = g_L.S.iter;
      for (int ahead = 0; ahead < C.Q.nscouts; ++ahead)
        scout_ask(C, j + ahead, (ahead & 1) ? 1 - g_L.S.A : g_L.S.A, true, fenced);
    }
    __syncthreads();
  }
  if (uni(g_L.S.status == 0 && g_L.S.phase == 0)) {
    // pre-loop direct connection of the two roots (birrt_star.cpp:1072-1075)
    if (threadIdx.x == 0) {
      load_node(C, 1, 0, &g_L.xn);
      load_node(C, 0, 0, &g_L.xc);
    }
    __syncthreads();
    connect_graphs(C, 0);
    if (threadIdx.x == 0)
      g_L.S.phase = (g_L.S.have_sol || (g_L.S.max_checked && g_L.S.checked >= g_L.S.max_checked)) ? 2 : 1;
    __syncthreads();
  }
  const unsigned long long t_launch = wall_clock64();
  for (int k = 0; k < iters; ++k) {
    if (uni(g_L.S.status != 0 || g_L.S.phase != 1)) break;
    if (((C.Q.lquota > 0 || C.Q.lticks > 0) && (k & 7) == 7) || (C.Q.abort && (k & (ABORT_EVERY - 1)) == ABORT_EVERY - 1)) {
      // enough of the launch's queries finished, its time slice is over, or the host abandoned the call: end it
      // (resumable; the stop words below send the scouts and helpers home)
      if (threadIdx.x == 0)
        g_L.go_end = (C.Q.lquota > 0 && ld_agent(C.Q.lfin) >= (unsigned)C.Q.lquota) ||
                     (C.Q.lticks > 0 && (long long)(wall_clock64() - t_launch) > C.Q.lticks) ||
                     (C.Q.abort && __hip_atomic_load(C.Q.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u);
      __syncthreads();
      if (uni(g_L.go_end)) break;
    }
    iteration(C);
  }
  if (threadIdx.x == 0) {
    if (C.Q.lquota > 0 && (g_L.S.phase == 2 || g_L.S.status != 0))
      __hip_atomic_fetch_add(C.Q.lfin, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (g_L.S.phase == 2 && g_L.S.t_end == 0) g_L.S.t_end = wall_clock64();
#ifdef SMP_JOB_PROF
    if (C.Q.jb) {
      g_L.S.prof[28] += ld_agent(&C.Q.jb->dbg[1]);
      g_L.S.prof[29] += ld_agent(&C.Q.jb->dbg[2]);
      g_L.S.prof[30] += ld_agent(&C.Q.jb->dbg[3]);
      for (int i = 0; i < 4; ++i) g_L.S.prof[P_TFK + i] += ld_agent(&C.Q.jb->dbg[4 + i]);  // helper tile stages
    }
#endif
    *C.Q.st = g_L.S;
    if (C.Q.jb) st_agent(&C.Q.jb->stop, 1);
    for (int s = 0; s < C.Q.nscouts; ++s) st_agent(&C.Q.scbs[s]->stop, 1);
  }
}

// Fresh job / scout boards for a launch (all zero: no granule carries a job number, no stop flag): block b clears
// board b % (1 + 2 ns) of query b / (1 + 2 ns) -- the leader's job board, then each scout's job and record board.
// One launch instead of a memset per board (each costs the host a few microseconds before the planner starts).
__global__ void __launch_bounds__(BLOCK) boards_reset_kernel(const QueryDev* qs, int ns) {
  const int per = 1 + 2 * ns, q = (int)blockIdx.x / per, w = (int)blockIdx.x - q * per;
  const QueryDev& Q = qs[q];
  char* base = w == 0 ? (char*)Q.jb : w <= ns ? (char*)Q.sjbs[w - 1] : (char*)Q.scbs[w - 1 - ns];
  const size_t bytes = w == 0 || w <= ns ? sizeof(JobBoard) : sizeof(ScoutBoard);
  uint4* p4 = reinterpret_cast<uint4*>(base);
  const size_t n4 = bytes / sizeof(uint4);
  for (size_t i = threadIdx.x; i < n4; i += BLOCK) p4[i] = make_uint4(0u, 0u, 0u, 0u);
  for (size_t i = n4 * sizeof(uint4) + threadIdx.x; i < bytes; i += BLOCK) base[i] = 0;
}

__global__ void path_kernel(QueryDev* qs, int* counts) {
  QueryDev Q = qs[blockIdx.x];
  if (threadIdx.x != 0) return;
  const QState& S = *Q.st;
  int cap = S.cap;
  int* ps = Q.path_nodes;
  int* pg = Q.path_nodes + cap;
  int ns = 0, ng = 0;
  if (S.have_sol) {
    int s_id = S.conn_start ? S.nB.id : S.nA.id, s_par = S.conn_start ? S.nB.parent : S.nA.parent;
    int g_id = S.conn_start ? S.nA.id : S.nB.id, g_par = S.conn_start ? S.nA.parent : S.nB.parent;
    while (s_id != 0 && ns < cap) { ps[ns++] = s_id; s_id = s_par; s_par = Q.tr[0].parent[s_id]; }
    while (g_id != 0 && ng < cap) { pg[ng++] = g_id; g_id = g_par; g_par = Q.tr[1].parent[g_id]; }
    for (int i = 0; i < ns / 2; ++i) { int t = ps[i]; ps[i] = ps[ns - 1 - i]; ps[ns - 1 - i] = t; }
  }
  counts[blockIdx.x * 2] = ns;
  counts[blockIdx.x * 2 + 1] = ng;
}


// The edges of query q's path (path_kernel's node lists: ns start-tree nodes, then ng goal-tree nodes) gathered for
// one device-to-host copy: per path node its edge's e_start[0..7] then e_target[0..7].
__global__ void path_edges_kernel(const QueryDev* qs, int q, int ns, int ng, double* out) {
  const QueryDev& Q = qs[q];
  const int cap = Q.st->cap;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < (ns + ng) * 2 * NJ; k += gridDim.x * blockDim.x) {
    const int e = k / (2 * NJ), w = k - e * (2 * NJ), j = w % NJ;
    const int t = e < ns ? 0 : 1;
    const int id = e < ns ? Q.path_nodes[e] : Q.path_nodes[cap + (e - ns)];
    const double* src = w < NJ ? Q.tr[t].e_start : Q.tr[t].e_target;
    out[k] = src[(size_t)j * cap + id];
  }
}

// Probe of the tree scans alone (tests and tools/near_probe.py): one workgroup runs nearest() and
// near_set<20>() for m query configurations against one tree (SoA q [NJ][cap], total cost [cap]), `reps` times
// each; out: nearest id, near count, the first / last 20 near ids; ticks[0] / ticks[1] = device-clock ticks of
// all nearest / near_set calls.
template <bool INL>
__device__ __forceinline__ void near_probe_body(const double* tqv, const double* tcost, int cap, int n,
                                                const double* queries, const int* excl, int m, double r, int reps, int* nn,
                                                int* nk, int* lo, int* hi, unsigned long long* ticks, const float* tqf) {
  Ctx C;
  C.Q.jb = nullptr;  // single workgroup: no helpers, scans stay local
  C.Q.scan_min = 0;
  C.Q.tr[0].q = const_cast<double*>(tqv);
  C.Q.tr[0].qf = const_cast<float*>(tqf);
  C.Q.tr[0].cost = const_cast<double*>(tcost);
  if (threadIdx.x == 0) {
    g_L.in_job = 0;
    g_L.S.n[0] = n;
    g_L.S.cap = cap;
    g_L.S.near_r = r;
    g_L.near_blo = ~0ull;
    g_L.near_bhi = 0;
    for (int k = 0; k < 32; ++k) g_L.S.prof[k] = 0;
  }
  const unsigned long long m0 = __builtin_amdgcn_s_memtime(), w0 = wall_clock64();
  unsigned long long t_nn = 0, t_near = 0;
  // reps < 0: -(reps + ((mode - 1) << 20)), mode 1 the slice functions of distributed scans (slice_nn / slice_near over
  // [0, n)) instead of nearest / near_set, 2 the fused near_set<20, true>, 3 the fused slice_near<true> (nearest and near
  // set in one pass: the near timing holds both, the nearest timing nothing), 4 / 5 the helpers' inlined forms of modes 1
  // / 3 (slice_near_inl: no call)
  int mode = 0;
  if (reps < 0) { reps = -reps; mode = 1 + (reps >> 20); reps &= (1 << 20) - 1; }
  const bool slice = mode == 1 || mode == 3 || mode == 4 || mode == 5;
  const gcdptr tq = uni_gptr(tqv), tc = uni_gptr(tcost);
  for (int k = 0; k < m; ++k) {
    if (threadIdx.x < NJ) g_L.xr[threadIdx.x] = queries[(size_t)k * NJ + threadIdx.x];
    __syncthreads();
    int id = 0;
    unsigned long long t0 = wall_clock64();
    for (int rep = 0; rep < reps && (mode < 2 || mode == 4); ++rep) {
      if constexpr (INL) {
        slice_nn_body32(tq, tqf, cap, 0, n, g_L.xr, g_L.sc.s);
        id = __longlong_as_double((long long)g_L.sc.s.wk[0]) < 10000.0 ? g_L.sc.s.wi[0] : 0;
      } else {
        if (slice) {
          slice_nn(tq, cap, 0, n, g_L.xr, g_L.sc.s);
          id = __longlong_as_double((long long)g_L.sc.s.wk[0]) < 10000.0 ? g_L.sc.s.wi[0] : 0;
        } else {
          id = nearest(C, 0, g_L.xr);
        }
      }
    }
    unsigned long long t1 = wall_clock64();
    for (int rep = 0; rep < reps; ++rep) {
      if constexpr (INL) {
        if (mode == 4) slice_near_inl<false, true>(tq, tc, cap, 0, n, g_L.xr, excl[k], r, g_L.sc.s, tqf, &g_L.S.prof[20]);
        else slice_near_inl<true, true>(tq, tc, cap, 0, n, g_L.xr, excl[k], r, g_L.sc.s, tqf, &g_L.S.prof[20]);
      } else {
        if (mode == 1) slice_near<false>(tq, tc, cap, 0, n, g_L.xr, excl[k], r, g_L.sc.s);
        else if (mode == 3) slice_near<true>(tq, tc, cap, 0, n, g_L.xr, excl[k], r, g_L.sc.s);
        else if (mode == 2) near_set<20, true>(C, 0, g_L.xr, excl[k]);
        else near_set<20>(C, 0, g_L.xr, excl[k]);
      }
    }
    if (mode == 2) id = g_L.fnn_d < 10000.0 ? g_L.fnn_id : 0;
    if (mode == 3 || mode == 5) id = __longlong_as_double((long long)g_L.sc.s.wk[0]) < 10000.0 ? g_L.sc.s.wi[0] : 0;
    unsigned long long t2 = wall_clock64();
    t_nn += t1 - t0;
    t_near += t2 - t1;
    if (slice) {
      const ScanLds& X = g_L.sc.s;
      if (threadIdx.x == 0) { nn[k] = id; nk[k] = X.cnt; }
      if (threadIdx.x < 20) {
        lo[k * 20 + threadIdx.x] = (int)threadIdx.x < X.take ? X.li[threadIdx.x] : -1;
        hi[k * 20 + threadIdx.x] = (int)threadIdx.x < X.take ? X.hi[X.take - 1 - threadIdx.x] : -1;
      }
    } else {
      if (threadIdx.x == 0) { nn[k] = id; nk[k] = g_L.nk; }
      if (threadIdx.x < 20) {
        lo[k * 20 + threadIdx.x] = threadIdx.x < g_L.n_lo ? g_L.lo_i[threadIdx.x] : -1;
        hi[k * 20 + threadIdx.x] = threadIdx.x < g_L.n_hi ? g_L.hi_i[threadIdx.x] : -1;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    ticks[0] = t_nn;
    ticks[1] = t_near;
    for (int k = 0; k < 10; ++k) ticks[2 + k] = g_L.S.prof[20 + k];
    // shader clock over the whole probe: s_memtime (shader cycles) and wall-clock ticks
    ticks[12] = __builtin_amdgcn_s_memtime() - m0;
    ticks[13] = wall_clock64() - w0;
  }
}
__global__ void __launch_bounds__(BLOCK) near_probe_kernel(const double* tqv, const double* tcost, int cap, int n,
                                                           const double* queries, const int* excl, int m, double r,
                                                           int reps, int* nn, int* nk, int* lo, int* hi,
                                                           unsigned long long* ticks, const float* tqf) {
  near_probe_body<false>(tqv, tcost, cap, n, queries, excl, m, r, reps, nn, nk, lo, hi, ticks, tqf);
}
// Modes 4 / 5 only (the helpers' inlined slice forms, over the fp32 copy tqf as in the planner), in a kernel of their own.
__global__ void __launch_bounds__(BLOCK) near_probe_inl_kernel(const double* tqv, const double* tcost, int cap, int n,
                                                               const double* queries, const int* excl, int m, double r,
                                                               int reps, int* nn, int* nk, int* lo, int* hi,
                                                               unsigned long long* ticks, const float* tqf) {
  near_probe_body<true>(tqv, tcost, cap, n, queries, excl, m, r, reps, nn, nk, lo, hi, ticks, tqf);
}

}  // namespace smp

#ifdef SMP_TRACE
// Copies the records of every role (out: cap >= TLOG_CAP words, roles in blocks of TLOG_ROLE, unused words 0).
extern "C" int smp_debug_tlog(unsigned long long* out, int cap, int reset) {
  if (cap < (int)smp::TLOG_CAP) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(smp::g_tlog), smp::TLOG_CAP * sizeof(unsigned long long)) != hipSuccess) return -1;
  unsigned n[4];
  if (hipMemcpyFromSymbol(n, HIP_SYMBOL(smp::g_tlog_n), sizeof(n)) != hipSuccess) return -1;
  if (reset) {
    std::vector<unsigned long long> z(smp::TLOG_CAP, 0);
    unsigned zn[4] = {0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(smp::g_tlog), z.data(), z.size() * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(smp::g_tlog_n), zn, sizeof(zn)) != hipSuccess) return -1;
  }
  return (int)(n[0] + n[1] + n[2]);
}
#else
extern "C" int smp_debug_tlog(unsigned long long*, int, int) { return -1; }
#endif

#ifdef SMP_SCAN_PROF
extern "C" int smp_debug_scanprof(unsigned long long* out, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(smp::g_scanprof), 24 * sizeof(unsigned long long)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[24] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(smp::g_scanprof), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#else
extern "C" int smp_debug_scanprof(unsigned long long*, int) { return -1; }
#endif

#ifdef SMP_PRE_VERIFY
extern "C" int smp_debug_preverify(unsigned long long* out, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(smp::g_pv), 4 * sizeof(unsigned long long)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[4] = {0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(smp::g_pv), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#else
extern "C" int smp_debug_preverify(unsigned long long*, int) { return -1; }
#endif

#ifdef SMP_BOUNDS
extern "C" int smp_debug_bounds(int* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(smp::g_dbg), 8 * sizeof(int)) == hipSuccess ? 0 : -1;
}
#else
extern "C" int smp_debug_bounds(int* out) { for (int i = 0; i < 8; ++i) out[i] = 0; return 1; }
#endif
