// Device-side kinematics and collision tests (gfx950).  Included by smp_kernels.hip only.
//
// Collision model (DESIGN.md "Collision model"): the robot is 64 spheres on 6 rigid bodies; a
// configuration collides if (map) a sphere of a map-enabled link touches an occupied voxel box, or (self)
// two spheres of an enabled link pair (SRDF-enabled, non-rigid) overlap.  The reference evaluates the same
// predicate with FCL on meshes (collision_checker.hpp:541-592); the numbers are unpinned, the structure is
// the same: map first, then self (collision_checker.hpp:104-121).
#pragma once
#include <hip/hip_runtime.h>

#include "smp_math.h"
#include "smp_types.h"

namespace smp {

// Body frames of one configuration from sin/cos of its joints (sc[j] = {sin q_j, cos q_j}): tree recursion
// along base_link_origin -> arm_link5 (CC:519-539).
__device__ __forceinline__ void body_frames_sc(const RobotDev* __restrict__ rb, const double* q, const double (*sc)[2],
                                               Frame* B) {
  Frame T;
  frame_identity(&T);
  T.p[2] = rb->root_z;
  for (int k = 0; k < rb->n_chain; ++k) {
    Frame L;
    int ty = rb->ch_type[k];
    if (ty == 1) {
      int j = rb->ch_joint[k];
      rot2_sc(&rb->ch_axis[k * 3], sc[j][0], sc[j][1], L.R);
      L.p[0] = rb->ch_origin[k * 3]; L.p[1] = rb->ch_origin[k * 3 + 1]; L.p[2] = rb->ch_origin[k * 3 + 2];
    } else if (ty == 2) {
      frame_identity(&L);
      double qq = q[rb->ch_joint[k]];
      for (int d = 0; d < 3; ++d) L.p[d] = rb->ch_origin[k * 3 + d] + rb->ch_axis[k * 3 + d] * qq;
    } else {
      for (int i = 0; i < 9; ++i) L.R[i] = rb->ch_R[k * 9 + i];
      for (int d = 0; d < 3; ++d) L.p[d] = rb->ch_p[k * 3 + d];
    }
    fmul(T, L, &T);
    int b = rb->ch_body[k];
    if (b >= 0) B[b] = T;
  }
}

// Body frames of one configuration: tree recursion along base_link_origin -> arm_link5 (CC:519-539).
__device__ __forceinline__ void body_frames(const RobotDev* __restrict__ rb, const double* q, Frame* B) {
  Frame T;
  frame_identity(&T);
  T.p[2] = rb->root_z;
  for (int k = 0; k < rb->n_chain; ++k) {
    Frame L;
    int ty = rb->ch_type[k];
    if (ty == 1) {
      rot2(&rb->ch_axis[k * 3], q[rb->ch_joint[k]], L.R);
      L.p[0] = rb->ch_origin[k * 3]; L.p[1] = rb->ch_origin[k * 3 + 1]; L.p[2] = rb->ch_origin[k * 3 + 2];
    } else if (ty == 2) {
      frame_identity(&L);
      double qq = q[rb->ch_joint[k]];
      for (int d = 0; d < 3; ++d) L.p[d] = rb->ch_origin[k * 3 + d] + rb->ch_axis[k * 3 + d] * qq;
    } else {
      for (int i = 0; i < 9; ++i) L.R[i] = rb->ch_R[k * 9 + i];
      for (int d = 0; d < 3; ++d) L.p[d] = rb->ch_p[k * 3 + d];
    }
    fmul(T, L, &T);
    int b = rb->ch_body[k];
    if (b >= 0) B[b] = T;
  }
}

// End-effector z of the 12-segment KDL chain (kdl_kuka_model.cpp:278-305): p_out = I; p_out *= J(q)*f_tip.
__device__ __forceinline__ double ee_z(const RobotDev* __restrict__ rb, const double* q) {
  Frame P;
  frame_identity(&P);
  for (int s = 0; s < rb->n_seg; ++s) {
    Frame J;
    frame_identity(&J);
    int ty = rb->seg_type[s];
    if (ty == 1) {
      rot2(&rb->seg_axis[s * 3], q[rb->seg_joint[s]], J.R);
      J.p[0] = rb->seg_origin[s * 3]; J.p[1] = rb->seg_origin[s * 3 + 1]; J.p[2] = rb->seg_origin[s * 3 + 2];
    } else if (ty == 2) {
      double qq = q[rb->seg_joint[s]];
      for (int d = 0; d < 3; ++d) J.p[d] = rb->seg_origin[s * 3 + d] + rb->seg_axis[s * 3 + d] * qq;
    }
    Frame F;
    for (int i = 0; i < 9; ++i) F.R[i] = rb->seg_R[s * 9 + i];
    for (int d = 0; d < 3; ++d) F.p[d] = rb->seg_p[s * 3 + d];
    Frame L;
    fmul(J, F, &L);
    fmul(P, L, &P);
  }
  return P.p[2];
}

// Grid cell of a sphere centre, or -1 outside the grid (such a sphere is free: the grid is padded by more
// than the largest radius around every occupied cell).
__device__ __forceinline__ long long centre_cell(const SceneDev& s, const double* c) {
  double fx = floor((c[0] - s.ox) / s.res), fy = floor((c[1] - s.oy) / s.res), fz = floor((c[2] - s.oz) / s.res);
  if (!(fx >= 0 && fx < s.nx && fy >= 0 && fy < s.ny && fz >= 0 && fz < s.nz)) return -1;
  return ((long long)(int)fz * s.ny + (int)fy) * s.nx + (int)fx;
}

// Cells that can hold a box within r of c (one cell of margin against rounding), clipped to the grid.
__device__ __forceinline__ void sphere_reach(const SceneDev& s, const double* c, double r, int* lo, int* hi) {
  lo[0] = max((int)floor((c[0] - r - s.ox) / s.res) - 1, 0);
  lo[1] = max((int)floor((c[1] - r - s.oy) / s.res) - 1, 0);
  lo[2] = max((int)floor((c[2] - r - s.oz) / s.res) - 1, 0);
  hi[0] = min((int)floor((c[0] + r - s.ox) / s.res) + 1, s.nx - 1);
  hi[1] = min((int)floor((c[1] + r - s.oy) / s.res) + 1, s.ny - 1);
  hi[2] = min((int)floor((c[2] + r - s.oz) / s.res) + 1, s.nz - 1);
}

// Exact sphere vs the box of cell (i,j,k), if that cell is occupied.
__device__ __forceinline__ bool cell_hit(const SceneDev& s, const double* c, double r2, int i, int j, int k) {
  uint64_t w = s.bricks[((size_t)(k >> 2) * s.bny + (j >> 2)) * s.bnx + (i >> 2)];
  if (!((w >> (((k & 3) << 4) | ((j & 3) << 2) | (i & 3))) & 1ull)) return false;
  double xlo = s.ox + (double)i * s.res, xhi = s.ox + (double)(i + 1) * s.res;
  double ylo = s.oy + (double)j * s.res, yhi = s.oy + (double)(j + 1) * s.res;
  double zlo = s.oz + (double)k * s.res, zhi = s.oz + (double)(k + 1) * s.res;
  double dx = c[0] < xlo ? xlo - c[0] : (c[0] > xhi ? c[0] - xhi : 0.0);
  double dy = c[1] < ylo ? ylo - c[1] : (c[1] > yhi ? c[1] - yhi : 0.0);
  double dz = c[2] < zlo ? zlo - c[2] : (c[2] > zhi ? c[2] - zhi : 0.0);
  return dx * dx + dy * dy + dz * dz <= r2;
}

// Self-collision sphere test of one (a, b) sphere pair (collision_checker.hpp:541-552 on the sphere model).
__device__ __forceinline__ bool spheres_touch(const double* wa, const double* wb, double ra, double rb) {
  double ex = wa[0] - wb[0], ey = wa[1] - wb[1], ez = wa[2] - wb[2];
  double r2 = ra + rb;
  return ex * ex + ey * ey + ez * ez <= r2 * r2;
}

// Makes this wave's earlier LDS writes visible to all of its lanes (LDS ops of one wave complete in order;
// the fence keeps the compiler from caching or reordering across it).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Local frame of body-chain step k (the same construction as body_frames_sc).
__device__ __forceinline__ void chain_local(const RobotDev* __restrict__ rb, int k, const double* q, const double (*sc)[2],
                                            Frame* L) {
  int ty = rb->ch_type[k];
  if (ty == 1) {
    int j = rb->ch_joint[k];
    rot2_sc(&rb->ch_axis[k * 3], sc[j][0], sc[j][1], L->R);
    L->p[0] = rb->ch_origin[k * 3]; L->p[1] = rb->ch_origin[k * 3 + 1]; L->p[2] = rb->ch_origin[k * 3 + 2];
  } else if (ty == 2) {
    frame_identity(L);
    double qq = q[rb->ch_joint[k]];
    for (int d = 0; d < 3; ++d) L->p[d] = rb->ch_origin[k * 3 + d] + rb->ch_axis[k * 3 + d] * qq;
  } else {
    for (int i = 0; i < 9; ++i) L->R[i] = rb->ch_R[k * 9 + i];
    for (int d = 0; d < 3; ++d) L->p[d] = rb->ch_p[k * 3 + d];
  }
}

__device__ __forceinline__ double sel3(int i, double a, double b, double c) { return i == 0 ? a : (i == 1 ? b : c); }

// Element e (R[0..8], p[9..11]) of the KDL product a * b, with fmul's evaluation order.  a is in LDS; b's
// column is picked with selects (no dynamically indexed private array).
__device__ __forceinline__ double fmul_elem(const double* a, const Frame& b, int e) {
  const bool rot = e < 9;
  const int r = rot ? e / 3 : e - 9, c = rot ? e - r * 3 : 0;
  double b0 = rot ? sel3(c, b.R[0], b.R[1], b.R[2]) : b.p[0];
  double b1 = rot ? sel3(c, b.R[3], b.R[4], b.R[5]) : b.p[1];
  double b2 = rot ? sel3(c, b.R[6], b.R[7], b.R[8]) : b.p[2];
  double m = a[r * 3 + 0] * b0 + a[r * 3 + 1] * b1 + a[r * 3 + 2] * b2;
  return rot ? m : m + a[9 + r];
}

constexpr int NWAVE = BLOCK / 64;
constexpr int FK_LANES = 12;                 // one lane per frame element
constexpr int FK_GROUPS = 64 / FK_LANES;     // configurations per wave in the FK stage

// LDS work area of one collision tile of CT configurations.
template <int CT>
struct TileLds {
  double fr[CT][MAX_BODY][12];    // body frames (R row-major, p)
  double tf[CT][2][12];           // FK chain product, ping-pong
  double scs[CT][NJ][2];          // sin / cos of every joint
  double wc[NWAVE][MAX_SPH][3];   // sphere world centres of the configuration a wave is testing
  double lbw[NWAVE][MAX_CLINK][3];// link-bound world centres of that configuration
  int coll[CT];                   // 1 = in collision
};

// Optional ordering of a tile's configurations: configuration c is point ord[c] of group grp[c] (an edge);
// grp_first[g] is the lowest colliding point index of group g found so far.  A configuration whose index
// exceeds it is skipped (it cannot change the group's first collision); a colliding one lowers it.
struct TileOrder {
  const int* grp;
  const int* ord;
  int* grp_first;
};

// Cooperative exact map test of sphere centre cc, radius r by one wavefront: lanes over the cells in reach.
__device__ __forceinline__ bool wave_sphere_map(const SceneDev& sc, const double* cc, double r, int lane) {
  int lo[3], hi[3];
  sphere_reach(sc, cc, r, lo, hi);
  const int ni = hi[0] - lo[0] + 1, nj = hi[1] - lo[1] + 1, nk = hi[2] - lo[2] + 1;
  const int nv = ni * nj * nk;
  const double r2 = r * r;
  for (int v0 = 0; v0 < nv; v0 += 64) {
    int v = v0 + lane;
    bool hit = false;
    if (v < nv) {
      int i = v % ni, t = v / ni;
      int j = t % nj, k = t / nj;
      hit = cell_hit(sc, cc, r2, lo[0] + i, lo[1] + j, lo[2] + k);
    }
    if (__ballot(hit)) return true;
  }
  return false;
}

// Collision test of nc <= CT configurations already placed in q_lds[c][8] (LDS), all block threads.
// On return coll[c] is 1 for colliding configurations (0 for free or skipped ones).
//   A. sin/cos of every joint (one lane each);
//   B. body frames: 12 lanes per configuration, one frame element each, chain steps in order;
//   C. one wavefront per configuration: lanes over spheres (world centre + box-gap prefilter), the rare
//      spheres near an occupied box swept cooperatively (lanes over cells in reach, ballot early exit);
//      then lanes over link pairs (bound test) and, per overlapping pair, lanes over its sphere pairs.
// Stage C has no block barrier: each wave moves on to its next configuration as soon as it is decided.
template <int CT>
__device__ __forceinline__ void collide_tile(const RobotDev* __restrict__ rb, const SceneDev& sc,
                                             const MapCfg* __restrict__ mc, int nc, const double (*q_lds)[NJ],
                                             int self, int map, TileLds<CT>& L, const TileOrder* ord = nullptr,
                                             unsigned long long* prof = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  unsigned long long t0 = (prof && tid == 0) ? wall_clock64() : 0;
  for (int it = tid; it < nc * NJ; it += BLOCK) {
    int c = it / NJ, j = it - c * NJ;
    psincos(q_lds[c][j], &L.scs[c][j][0], &L.scs[c][j][1]);
  }
  if (tid < nc) L.coll[tid] = 0;
  __syncthreads();
  {
    const int e = lane % FK_LANES, g = lane / FK_LANES;
    for (int c0 = 0; c0 < nc; c0 += NWAVE * FK_GROUPS) {
      const int c = c0 + wave * FK_GROUPS + g;
      const bool act = g < FK_GROUPS && c < nc;
      if (act) L.tf[c][0][e] = (e == 0 || e == 4 || e == 8) ? 1.0 : (e == 11 ? rb->root_z : 0.0);
      wave_sync();
      int cur = 0;
      for (int k = 0; k < rb->n_chain; ++k) {
        if (act) {
          Frame Lk;
          chain_local(rb, k, q_lds[c], L.scs[c], &Lk);
          double v = fmul_elem(L.tf[c][cur], Lk, e);
          L.tf[c][cur ^ 1][e] = v;
          int b = rb->ch_body[k];
          if (b >= 0) L.fr[c][b][e] = v;
        }
        wave_sync();
        cur ^= 1;
      }
    }
  }
  __syncthreads();
  unsigned long long t1 = (prof && tid == 0) ? wall_clock64() : 0;
  const int nsph = rb->n_sph, ncl = rb->n_clink, npair = rb->n_pairs;
  const bool do_map = map && mc->has_map;
  double (*wc)[3] = L.wc[wave];
  double (*lbw)[3] = L.lbw[wave];
  for (int c = wave; c < nc; c += NWAVE) {
    if (ord && ord->ord[c] > __atomic_load_n(&ord->grp_first[ord->grp[c]], __ATOMIC_RELAXED)) continue;
    const double* F = &L.fr[c][0][0];
    bool hit = false;
    for (int s0 = 0; s0 < nsph && !hit; s0 += 64) {
      const int s = s0 + lane;
      bool need = false;
      if (s < nsph) {
        const double* B = F + rb->sph_body[s] * 12;
        const double* p = &rb->sph_cb[s * 3];
        double w[3];
        for (int r = 0; r < 3; ++r) {
          double m = B[r * 3 + 0] * p[0] + B[r * 3 + 1] * p[1] + B[r * 3 + 2] * p[2];
          w[r] = m + B[9 + r];
        }
        wc[s][0] = w[0]; wc[s][1] = w[1]; wc[s][2] = w[2];
        if (do_map && mc->map_on[s]) {
          long long cell = centre_cell(sc, w);
          need = cell >= 0 && (uint32_t)sc.d2[cell] <= mc->T[s];
        }
      }
      wave_sync();
      uint64_t m = __ballot(need);
      while (m) {
        const int sl = s0 + __builtin_ctzll(m);
        m &= m - 1;
        const double cc[3] = {wc[sl][0], wc[sl][1], wc[sl][2]};
        if (wave_sphere_map(sc, cc, rb->sph_r[sl], lane)) { hit = true; break; }
      }
    }
    if (!hit && self) {
      for (int l = lane; l < ncl; l += 64) {
        const double* B = F + rb->cl_body[l] * 12;
        const double* p = &rb->cl_cb[l * 3];
        for (int r = 0; r < 3; ++r) {
          double m = B[r * 3 + 0] * p[0] + B[r * 3 + 1] * p[1] + B[r * 3 + 2] * p[2];
          lbw[l][r] = m + B[9 + r];
        }
      }
      wave_sync();
      for (int p0 = 0; p0 < npair && !hit; p0 += 64) {
        const int pp = p0 + lane;
        bool over = false;
        if (pp < npair) {
          int a = rb->pair_a[pp], b = rb->pair_b[pp];
          double dx = lbw[a][0] - lbw[b][0], dy = lbw[a][1] - lbw[b][1], dz = lbw[a][2] - lbw[b][2];
          double rr = rb->cl_r[a] + rb->cl_r[b];
          over = !(dx * dx + dy * dy + dz * dz > rr * rr);
        }
        uint64_t m = __ballot(over);
        while (m) {
          const int pq = p0 + __builtin_ctzll(m);
          m &= m - 1;
          const int a = rb->pair_a[pq], b = rb->pair_b[pq];
          const int sa0 = rb->cl_sph0[a], sb0 = rb->cl_sph0[b], nb = rb->cl_nsph[b];
          const int K = rb->cl_nsph[a] * nb;
          bool h = false;
          for (int l0 = 0; l0 < K && !h; l0 += 64) {
            const int l = l0 + lane;
            bool t = false;
            if (l < K) {
              const int sa = sa0 + l / nb, sb = sb0 + l % nb;
              t = spheres_touch(wc[sa], wc[sb], rb->sph_r[sa], rb->sph_r[sb]);
            }
            h = __ballot(t) != 0;
          }
          if (h) { hit = true; break; }
        }
      }
    }
    if (hit && lane == 0) {
      L.coll[c] = 1;
      if (ord) atomicMin(&ord->grp_first[ord->grp[c]], ord->ord[c]);
    }
    wave_sync();
  }
  __syncthreads();
  if (prof && tid == 0) {
    unsigned long long t2 = wall_clock64();
    prof[0] += t1 - t0; prof[1] += t2 - t1;
  }
}

}  // namespace smp
