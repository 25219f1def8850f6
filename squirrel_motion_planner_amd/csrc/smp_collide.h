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
// Only z is wanted, so only row 2 of p_out's rotation and p_out.z are carried: each of those entries of
// P * L is the same three-term sum as in the full frame product (smp_math.h fmul), so the value is the one the
// full product gives.  Fixed and prismatic segments skip the product with their identity joint rotation:
// 1*a + 0*b + 0*c == a exactly up to the sign of a zero, which no later operation turns into a different
// non-zero value and which `z >= 0` does not see.
__device__ __forceinline__ double ee_z(const RobotDev* __restrict__ rb, const double* q) {
  double r0 = 0.0, r1 = 0.0, r2 = 1.0, pz = 0.0;  // row 2 of P.R, P.p[2]
  for (int s = 0; s < rb->n_seg; ++s) {
    const int ty = rb->seg_type[s];
    const double* FR = &rb->seg_R[s * 9];
    const double* Fp = &rb->seg_p[s * 3];
    double LR[9], Lp[3];
    if (ty == 1) {
      double JR[9];
      rot2(&rb->seg_axis[s * 3], q[rb->seg_joint[s]], JR);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c)
          LR[r * 3 + c] = JR[r * 3 + 0] * FR[0 * 3 + c] + JR[r * 3 + 1] * FR[1 * 3 + c] + JR[r * 3 + 2] * FR[2 * 3 + c];
        Lp[r] = (JR[r * 3 + 0] * Fp[0] + JR[r * 3 + 1] * Fp[1] + JR[r * 3 + 2] * Fp[2]) + rb->seg_origin[s * 3 + r];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 9; ++i) LR[i] = FR[i];
      if (ty == 2) {
        const double qq = q[rb->seg_joint[s]];
#pragma unroll
        for (int d = 0; d < 3; ++d) Lp[d] = Fp[d] + (rb->seg_origin[s * 3 + d] + rb->seg_axis[s * 3 + d] * qq);
      } else {
#pragma unroll
        for (int d = 0; d < 3; ++d) Lp[d] = Fp[d];
      }
    }
    const double n0 = r0 * LR[0] + r1 * LR[3] + r2 * LR[6];
    const double n1 = r0 * LR[1] + r1 * LR[4] + r2 * LR[7];
    const double n2 = r0 * LR[2] + r1 * LR[5] + r2 * LR[8];
    pz = (r0 * Lp[0] + r1 * Lp[1] + r2 * Lp[2]) + pz;
    r0 = n0; r1 = n1; r2 = n2;
  }
  return pz;
}

// Grid cell of a sphere centre, or -1 outside the grid (such a sphere is free: the grid is padded by more
// than the largest radius around every occupied cell).
// Multiplying by 1/res instead of dividing may put a centre within an ulp of a cell face into the neighbour
// cell; that cell's closed box still contains the centre up to that ulp, far inside the 1e-6 m margin of T.
__device__ __forceinline__ long long centre_cell(const SceneDev& s, const double* c) {
  double fx = floor((c[0] - s.ox) * s.inv_res), fy = floor((c[1] - s.oy) * s.inv_res), fz = floor((c[2] - s.oz) * s.inv_res);
  if (!(fx >= 0 && fx < s.nx && fy >= 0 && fy < s.ny && fz >= 0 && fz < s.nz)) return -1;
  return ((long long)(int)fz * s.ny + (int)fy) * s.nx + (int)fx;
}

// Cells that can hold a box within r of c (one cell of margin against rounding), clipped to the grid.
__device__ __forceinline__ void sphere_reach(const SceneDev& s, const double* c, double r, int* lo, int* hi) {
  lo[0] = max((int)floor((c[0] - r - s.ox) * s.inv_res) - 1, 0);
  lo[1] = max((int)floor((c[1] - r - s.oy) * s.inv_res) - 1, 0);
  lo[2] = max((int)floor((c[2] - r - s.oz) * s.inv_res) - 1, 0);
  hi[0] = min((int)floor((c[0] + r - s.ox) * s.inv_res) + 1, s.nx - 1);
  hi[1] = min((int)floor((c[1] + r - s.oy) * s.inv_res) + 1, s.ny - 1);
  hi[2] = min((int)floor((c[2] + r - s.oz) * s.inv_res) + 1, s.nz - 1);
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

// Makes this wave's earlier LDS writes visible to all of its lanes (LDS ops of one wave complete in order;
// the fence keeps the compiler from caching or reordering across it).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Local frame of body-chain step k (the same construction as body_frames / body_frames_sc).
__device__ __forceinline__ void chain_local(const RobotDev* __restrict__ rb, int k, const double* q, double st, double ct,
                                            Frame* L) {
  int ty = rb->ch_type[k];
  if (ty == 1) {
    rot2_sc(&rb->ch_axis[k * 3], st, ct, L->R);
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

__device__ __forceinline__ uint32_t shfl_u32(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src); }

// Inclusive prefix sum over the 64 lanes of a wavefront (all lanes active): ockl's DPP scan (row shifts and row
// broadcasts, six VALU steps) instead of a shuffle tree, whose six ds_bpermute steps each wait an LDS round trip.
extern "C" __device__ int __ockl_wfscan_add_i32(int, bool);
__device__ __forceinline__ int wave_incl_scan(int v) { return __ockl_wfscan_add_i32(v, true); }

// The scene's scalars in scalar registers.  A caller's SceneDev may live in private (scratch) memory -- the planner
// keeps its context there -- and every use of a field would then be a scratch load, several of them dependent per
// sphere centre (centre_cell) and per exact sweep (sphere_reach); read once here, they are wave-uniform SGPRs.
__device__ __forceinline__ double rfl_f64(double v) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)b);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
template <class T>
__device__ __forceinline__ T* rfl_ptr(T* p) {
  const unsigned long long b = (unsigned long long)(uintptr_t)p;
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)b);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(b >> 32));
  return (T*)(uintptr_t)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ SceneDev uniform_scene(const SceneDev& s) {
  SceneDev o;
  o.nx = __builtin_amdgcn_readfirstlane(s.nx); o.ny = __builtin_amdgcn_readfirstlane(s.ny);
  o.nz = __builtin_amdgcn_readfirstlane(s.nz); o.bnx = __builtin_amdgcn_readfirstlane(s.bnx);
  o.bny = __builtin_amdgcn_readfirstlane(s.bny);
  o.ox = rfl_f64(s.ox); o.oy = rfl_f64(s.oy); o.oz = rfl_f64(s.oz); o.res = rfl_f64(s.res); o.inv_res = rfl_f64(s.inv_res);
  o.bricks = rfl_ptr(s.bricks); o.d2 = rfl_ptr(s.d2); o.d2b = rfl_ptr(s.d2b);
  return o;
}

// Value of lane I of this lane's quad (DPP quad_perm broadcast, both 32-bit halves).  The whole quad must be active.
template <int I>
__device__ __forceinline__ double quad_bcast(double v) {
  constexpr int ctrl = I | (I << 2) | (I << 4) | (I << 6);
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, ctrl, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), ctrl, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// Cooperative exact map test of sphere centre cc, radius r by one wavefront.  The brick words covering the
// reach (<= 64) are loaded once, one per lane, and handed to the lanes testing their cells by shuffles; then
// lanes sweep the cells in reach (exact box test, ballot early exit).  Larger reaches load per cell.
__device__ __forceinline__ bool wave_sphere_map(const SceneDev& sc, const double* cc, double r, int lane) {
  int lo[3], hi[3];
  sphere_reach(sc, cc, r, lo, hi);
  const int ni = hi[0] - lo[0] + 1, nj = hi[1] - lo[1] + 1, nk = hi[2] - lo[2] + 1;
  const int nv = ni * nj * nk;
  const double r2 = r * r;
  const int bi0 = lo[0] >> 2, bj0 = lo[1] >> 2, bk0 = lo[2] >> 2;
  const int nbi = (hi[0] >> 2) - bi0 + 1, nbj = (hi[1] >> 2) - bj0 + 1, nbk = (hi[2] >> 2) - bk0 + 1;
  const int nb = nbi * nbj * nbk;
  if (nb <= 64) {
    uint64_t w = 0;
    if (lane < nb) {
      int bi = lane % nbi, t = lane / nbi;
      int bj = t % nbj, bk = t / nbj;
      w = sc.bricks[((size_t)(bk0 + bk) * sc.bny + (bj0 + bj)) * sc.bnx + (bi0 + bi)];
    }
    const uint32_t wlo = (uint32_t)w, whi = (uint32_t)(w >> 32);
    for (int v0 = 0; v0 < nv; v0 += 64) {
      const int v = v0 + lane;
      int i = 0, j = 0, k = 0, src = 0;
      if (v < nv) {
        int t = v / ni;
        i = lo[0] + (v - t * ni);
        j = lo[1] + t % nj;
        k = lo[2] + t / nj;
        src = ((k >> 2) - bk0) * nbj * nbi + ((j >> 2) - bj0) * nbi + ((i >> 2) - bi0);
      }
      const uint32_t a = shfl_u32(wlo, src), b = shfl_u32(whi, src);
      bool hit = false;
      if (v < nv) {
        const int bit = ((k & 3) << 4) | ((j & 3) << 2) | (i & 3);
        const uint32_t word = bit < 32 ? a : b;
        if ((word >> (bit & 31)) & 1u) {
          double xlo = sc.ox + (double)i * sc.res, xhi = sc.ox + (double)(i + 1) * sc.res;
          double ylo = sc.oy + (double)j * sc.res, yhi = sc.oy + (double)(j + 1) * sc.res;
          double zlo = sc.oz + (double)k * sc.res, zhi = sc.oz + (double)(k + 1) * sc.res;
          double dx = cc[0] < xlo ? xlo - cc[0] : (cc[0] > xhi ? cc[0] - xhi : 0.0);
          double dy = cc[1] < ylo ? ylo - cc[1] : (cc[1] > yhi ? cc[1] - yhi : 0.0);
          double dz = cc[2] < zlo ? zlo - cc[2] : (cc[2] > zhi ? cc[2] - zhi : 0.0);
          hit = dx * dx + dy * dy + dz * dz <= r2;
        }
      }
      if (__ballot(hit)) return true;
    }
    return false;
  }
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

// The brick box of a sphere's reach (sphere_reach, then the 4x4x4 bricks covering it): first brick and counts.
__device__ __forceinline__ int sphere_bricks(const SceneDev& sc, const double* cc, double r, int* lo, int* hi, int* b0,
                                             int* nbx) {
  sphere_reach(sc, cc, r, lo, hi);
  b0[0] = lo[0] >> 2; b0[1] = lo[1] >> 2; b0[2] = lo[2] >> 2;
  nbx[0] = (hi[0] >> 2) - b0[0] + 1; nbx[1] = (hi[1] >> 2) - b0[1] + 1; nbx[2] = (hi[2] >> 2) - b0[2] + 1;
  return nbx[0] * nbx[1] * nbx[2];
}

constexpr int MAP_STAGE_W = 96;  // brick words staged per configuration (its dead body-frame rows, TileLds::fr)

constexpr int MAP_LIST = 256;  // occupied cells of one sphere's reach listed at once (sweep_occupied)
// reaches of at most this many cells are swept cell by cell (a 5 cm scene's spheres reach <= 216 cells: four passes
// cost less than listing; a 2 cm scene's reach up to 1728)
constexpr int MAP_LIST_MIN = 4 * 64;

// Exact map test of a sphere (centre cc, radius r, reach lo..hi, its brick box b0 / nbx of nbs <= 64 bricks, lane b
// holding brick b's occupancy word) over the occupied cells of its reach only: each word masked to the reach, bricks
// farther than r + 1e-9 from the centre dropped (every cell of them fails the exact test), the remaining occupied cells
// listed in LDS (`list`, MAP_LIST entries) and tested 64 at a time.  A reach of a 2 cm scene holds up to 12^3 cells,
// mostly free: cell-by-cell passes take up to 27 rounds where the list takes one or two.  Returns 1 hit, 0 free,
// 2 = more than MAP_LIST occupied cells (the caller sweeps cell by cell).
__device__ __forceinline__ int sweep_occupied(const SceneDev& sc, const double* cc, double r, const int* lo, const int* hi,
                                              const int* b0, const int* nbx, int nbs, uint64_t w, uint16_t* list,
                                              int lane) {
  const double r2 = r * r;
  if (lane < nbs && w) {
    const int bi = lane % nbx[0], t = lane / nbx[0];
    const int bj = t % nbx[1], bk = t / nbx[1];
    const int gi = b0[0] + bi, gj = b0[1] + bj, gk = b0[2] + bk;
    const int il = max(lo[0] - 4 * gi, 0), ih = min(hi[0] - 4 * gi, 3);
    const int jl = max(lo[1] - 4 * gj, 0), jh = min(hi[1] - 4 * gj, 3);
    const int kl = max(lo[2] - 4 * gk, 0), kh = min(hi[2] - 4 * gk, 3);
    const uint32_t xm = ((2u << ih) - 1u) & ~((1u << il) - 1u);
    uint32_t row = 0;
    for (int jj = jl; jj <= jh; ++jj) row |= xm << (4 * jj);
    uint64_t m = 0;
    for (int kk = kl; kk <= kh; ++kk) m |= (uint64_t)row << (16 * kk);
    w &= m;
    if (w) {
      const double x0 = sc.ox + (double)(4 * gi + il) * sc.res, x1 = sc.ox + (double)(4 * gi + ih + 1) * sc.res;
      const double y0 = sc.oy + (double)(4 * gj + jl) * sc.res, y1 = sc.oy + (double)(4 * gj + jh + 1) * sc.res;
      const double z0 = sc.oz + (double)(4 * gk + kl) * sc.res, z1 = sc.oz + (double)(4 * gk + kh + 1) * sc.res;
      const double dx = cc[0] < x0 ? x0 - cc[0] : (cc[0] > x1 ? cc[0] - x1 : 0.0);
      const double dy = cc[1] < y0 ? y0 - cc[1] : (cc[1] > y1 ? cc[1] - y1 : 0.0);
      const double dz = cc[2] < z0 ? z0 - cc[2] : (cc[2] > z1 ? cc[2] - z1 : 0.0);
      const double re = r + 1e-9;
      if (dx * dx + dy * dy + dz * dz > re * re) w = 0;
    }
  } else {
    w = 0;
  }
  const int cnt = __popcll(w);
  const int inc = wave_incl_scan(cnt);
  const int T = __builtin_amdgcn_readlane(inc, 63);
  if (T > MAP_LIST) return 2;
  for (int pos = inc - cnt; w; ++pos) {
    const int bit = __builtin_ctzll(w);
    w &= w - 1;
    list[pos] = (uint16_t)(lane << 6 | bit);
  }
  wave_sync();
  int res = 0;
  for (int t0 = 0; t0 < T; t0 += 64) {
    const int t = t0 + lane;
    bool hit = false;
    if (t < T) {
      const int code = list[t], bb = code >> 6, bit = code & 63;
      const int bi = bb % nbx[0], tt = bb / nbx[0];
      const int bj = tt % nbx[1], bk = tt / nbx[1];
      const int i = 4 * (b0[0] + bi) + (bit & 3), j = 4 * (b0[1] + bj) + ((bit >> 2) & 3);
      const int k = 4 * (b0[2] + bk) + (bit >> 4);
      const double xlo = sc.ox + (double)i * sc.res, xhi = sc.ox + (double)(i + 1) * sc.res;
      const double ylo = sc.oy + (double)j * sc.res, yhi = sc.oy + (double)(j + 1) * sc.res;
      const double zlo = sc.oz + (double)k * sc.res, zhi = sc.oz + (double)(k + 1) * sc.res;
      const double dx = cc[0] < xlo ? xlo - cc[0] : (cc[0] > xhi ? cc[0] - xhi : 0.0);
      const double dy = cc[1] < ylo ? ylo - cc[1] : (cc[1] > yhi ? cc[1] - yhi : 0.0);
      const double dz = cc[2] < zlo ? zlo - cc[2] : (cc[2] > zhi ? cc[2] - zhi : 0.0);
      hit = dx * dx + dy * dy + dz * dz <= r2;
    }
    if (__ballot(hit)) { res = 1; break; }
  }
  wave_sync();  // the list is rewritten by the next sphere
  return res;
}

// Exact map tests of all candidate spheres of one configuration by one wavefront, their brick words fetched in ONE
// memory round trip: lanes over spheres give each candidate (<= 64 bricks) its slot range of the staging buffer `buf`
// (MAP_STAGE_W words, in sphere order; owner[w] = the sphere of word w, off[s] = its first slot), lanes over slots
// load the words, then the candidates are swept in sphere order from LDS (the cells and the exact box test of
// wave_sphere_map).  A candidate that does not fit (more than 64 bricks, or the buffer full) is swept by
// wave_sphere_map itself.  The outcome (any candidate touching an occupied cell) is the same as sweeping them one
// after the other; wave_sphere_map pays one load round trip per candidate.
template <int CAP = MAP_STAGE_W, typename OffT = uint8_t>
__device__ __forceinline__ bool wave_map_staged(const RobotDev* __restrict__ rb, const SceneDev& sc, const double (*wc)[3],
                                                const uint32_t* cand, int nsph, uint64_t* buf, uint8_t* owner,
                                                OffT* off, int lane, uint16_t* list = nullptr) {
  constexpr OffT NONE = (OffT)~(OffT)0;
  static_assert(CAP < (int)NONE, "slot offsets");
  // slots: sphere s = g * 64 + lane of group g.  Staged are the candidates (of at most 64 bricks) whose inclusive
  // prefix of brick counts still ends within the buffer: a prefix of them in sphere order, so the words [0, base)
  // all have an owner; off[s] = first slot of a staged candidate, else 255
  int base = 0;
  uint64_t spill[2] = {0, 0};  // candidates of group 0 / 1 (bit per lane) swept by wave_sphere_map
  for (int g = 0; g < 2 && g * 64 < nsph; ++g) {
    const int s = g * 64 + lane;
    const bool is_c = s < nsph && ((cand[s >> 5] >> (s & 31)) & 1u);
    int nb = 0;
    if (is_c) {
      int lo[3], hi[3], b0[3], nbx[3];
      nb = sphere_bricks(sc, wc[s], rb->sph_r[s], lo, hi, b0, nbx);
      if (nb > 64) nb = 0;  // swept by wave_sphere_map (its per-cell loads)
    }
    const int inc = wave_incl_scan(nb);
    const bool staged = nb > 0 && base + inc <= CAP;
    const int start = base + inc - nb;
    if (s < nsph) off[s] = staged ? (OffT)start : NONE;
    if (staged)
      for (int b = 0; b < nb; ++b) owner[start + b] = (uint8_t)s;
    spill[g] = __ballot(is_c && !staged);
    const uint64_t sm = __ballot(staged);
    if (sm) base += __builtin_amdgcn_readlane(inc, 63 - __builtin_clzll(sm));
  }
  wave_sync();
  // one round: every staged word loaded (two slots per lane), then stored
  constexpr int SU = (CAP + 63) / 64;
  uint64_t v[SU];
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    v[u] = 0;
    const int w = u * 64 + lane;
    if (w < base) {
      const int s = owner[w];
      int lo[3], hi[3], b0[3], nbx[3];
      sphere_bricks(sc, wc[s], rb->sph_r[s], lo, hi, b0, nbx);
      const int b = w - off[s], bi = b % nbx[0], t = b / nbx[0];
      const int bj = t % nbx[1], bk = t / nbx[1];
      v[u] = sc.bricks[((size_t)(b0[2] + bk) * sc.bny + (b0[1] + bj)) * sc.bnx + (b0[0] + bi)];
    }
  }
#pragma unroll
  for (int u = 0; u < SU; ++u)
    if (u * 64 + lane < base) buf[u * 64 + lane] = v[u];
  wave_sync();
  // sweeps of the staged candidates in sphere order (scalar loop over the candidate mask)
  for (int wd = 0; wd * 32 < nsph; ++wd) {
    uint32_t m = cand[wd];
    while (m) {
      const int s = wd * 32 + __builtin_ctz(m);
      m &= m - 1;
      const int o = off[s];
      if (o == (int)NONE) continue;
      const double cc[3] = {wc[s][0], wc[s][1], wc[s][2]};
      const double r = rb->sph_r[s], r2 = r * r;
      int lo[3], hi[3], b0[3], nbx[3];
      const int nbs = sphere_bricks(sc, cc, r, lo, hi, b0, nbx);
      const int ni = hi[0] - lo[0] + 1, nj = hi[1] - lo[1] + 1, nk = hi[2] - lo[2] + 1;
      const int nv = ni * nj * nk;
      if (list && nv > MAP_LIST_MIN) {
        const int h = sweep_occupied(sc, cc, r, lo, hi, b0, nbx, nbs, lane < nbs ? buf[o + lane] : 0ull, list, lane);
        if (h == 1) return true;
        if (h == 0) continue;
      }
      for (int v0 = 0; v0 < nv; v0 += 64) {
        const int vv = v0 + lane;
        bool hit = false;
        if (vv < nv) {
          const int t = vv / ni;
          const int i = lo[0] + (vv - t * ni), j = lo[1] + t % nj, k = lo[2] + t / nj;
          const int src = ((k >> 2) - b0[2]) * nbx[1] * nbx[0] + ((j >> 2) - b0[1]) * nbx[0] + ((i >> 2) - b0[0]);
          const uint64_t word = buf[o + src];
          const int bit = ((k & 3) << 4) | ((j & 3) << 2) | (i & 3);
          if ((word >> bit) & 1ull) {
            const double xlo = sc.ox + (double)i * sc.res, xhi = sc.ox + (double)(i + 1) * sc.res;
            const double ylo = sc.oy + (double)j * sc.res, yhi = sc.oy + (double)(j + 1) * sc.res;
            const double zlo = sc.oz + (double)k * sc.res, zhi = sc.oz + (double)(k + 1) * sc.res;
            const double dx = cc[0] < xlo ? xlo - cc[0] : (cc[0] > xhi ? cc[0] - xhi : 0.0);
            const double dy = cc[1] < ylo ? ylo - cc[1] : (cc[1] > yhi ? cc[1] - yhi : 0.0);
            const double dz = cc[2] < zlo ? zlo - cc[2] : (cc[2] > zhi ? cc[2] - zhi : 0.0);
            hit = dx * dx + dy * dy + dz * dz <= r2;
          }
        }
        if (__ballot(hit)) return true;
      }
    }
  }
  // candidates that did not fit the staging buffer
  for (int g = 0; g < 2; ++g) {
    uint64_t m = spill[g];
    while (m) {
      const int s = g * 64 + __builtin_ctzll(m);
      m &= m - 1;
      const double cc[3] = {wc[s][0], wc[s][1], wc[s][2]};
      if (list) {  // its brick words one per lane (one round trip), then the occupied cells only
        int lo[3], hi[3], b0[3], nbx[3];
        const int nbs = sphere_bricks(sc, cc, rb->sph_r[s], lo, hi, b0, nbx);
        if (nbs <= 64 && (hi[0] - lo[0] + 1) * (hi[1] - lo[1] + 1) * (hi[2] - lo[2] + 1) > MAP_LIST_MIN) {
          uint64_t w = 0;
          if (lane < nbs) {
            const int bi = lane % nbx[0], t = lane / nbx[0];
            const int bj = t % nbx[1], bk = t / nbx[1];
            w = sc.bricks[((size_t)(b0[2] + bk) * sc.bny + (b0[1] + bj)) * sc.bnx + (b0[0] + bi)];
          }
          const int h = sweep_occupied(sc, cc, rb->sph_r[s], lo, hi, b0, nbx, nbs, w, list, lane);
          if (h == 1) return true;
          if (h == 0) continue;
        }
      }
      if (wave_sphere_map(sc, cc, rb->sph_r[s], lane)) return true;
    }
  }
  return false;
}

// ---------------------------------------------------------------------------------------------- exact primitives
// World centre and horizontal x axis (c, s) of primitive p from its body's frame B (R row-major, then p): the same
// three-term sums as a sphere centre (KDL Frame * Vector); the axis is R times ab without the translation.
__device__ __forceinline__ void prim_world(const RobotDev* __restrict__ rb, int p, const double* B, double* o) {
  const double* cb = &rb->prim_cb[p * 3];
  const double* ab = &rb->prim_ab[p * 3];
  for (int r = 0; r < 3; ++r) {
    const double m = B[r * 3 + 0] * cb[0] + B[r * 3 + 1] * cb[1] + B[r * 3 + 2] * cb[2];
    o[r] = m + B[9 + r];
  }
  o[3] = B[0] * ab[0] + B[1] * ab[1] + B[2] * ab[2];
  o[4] = B[3] * ab[0] + B[4] * ab[1] + B[5] * ab[2];
}

// Exact test of an upright primitive (ty 1 box with half extents h[0..2], 2 cylinder of radius h[0] and half length
// h[1]; centre pw[0..2], x axis (pw[3], pw[4])) against the closed box of cell (i, j, k): z intervals overlap, and in
// the plane the separating-axis test of the rotated rectangle against the cell's square (axes x, y, the box's own
// two), or the circle against the square.  Shared term by term with the oracle (smp_oracle.cpp prim_cell).
__device__ __forceinline__ bool prim_cell(int ty, const double* __restrict__ h, const double* pw, const SceneDev& sc, int i,
                                          int j, int k) {
  const double zlo = sc.oz + (double)k * sc.res, zhi = sc.oz + (double)(k + 1) * sc.res;
  const double hz = ty == 1 ? h[2] : h[1];
  if (zhi < pw[2] - hz || zlo > pw[2] + hz) return false;
  const double xlo = sc.ox + (double)i * sc.res, xhi = sc.ox + (double)(i + 1) * sc.res;
  const double ylo = sc.oy + (double)j * sc.res, yhi = sc.oy + (double)(j + 1) * sc.res;
  if (ty == 2) {
    const double qx = pw[0] < xlo ? xlo - pw[0] : (pw[0] > xhi ? pw[0] - xhi : 0.0);
    const double qy = pw[1] < ylo ? ylo - pw[1] : (pw[1] > yhi ? pw[1] - yhi : 0.0);
    return qx * qx + qy * qy <= h[0] * h[0];
  }
  const double c = pw[3], s = pw[4], ac = fabs(c), as = fabs(s), hw = 0.5 * sc.res;
  const double dx = 0.5 * (xlo + xhi) - pw[0], dy = 0.5 * (ylo + yhi) - pw[1];
  if (fabs(dx) > hw + (ac * h[0] + as * h[1])) return false;
  if (fabs(dy) > hw + (as * h[0] + ac * h[1])) return false;
  if (fabs(c * dx + s * dy) > h[0] + hw * (ac + as)) return false;
  if (fabs(c * dy - s * dx) > h[1] + hw * (ac + as)) return false;
  return true;
}

// Cells whose boxes can meet the primitive's axis-aligned bounds, trimmed with the cell test's own comparisons (a
// trimmed cell fails that test), clipped to the grid.  Returns false if the range is empty.
__device__ __forceinline__ bool prim_reach(int ty, const double* __restrict__ h, const double* pw, const SceneDev& sc,
                                           int* lo, int* hi) {
  const double ac = fabs(pw[3]), as = fabs(pw[4]);
  const double ex = ty == 1 ? ac * h[0] + as * h[1] : h[0];
  const double ey = ty == 1 ? as * h[0] + ac * h[1] : h[0];
  const double ez = ty == 1 ? h[2] : h[1];
  const double a[3] = {pw[0] - ex, pw[1] - ey, pw[2] - ez}, b[3] = {pw[0] + ex, pw[1] + ey, pw[2] + ez};
  const double o[3] = {sc.ox, sc.oy, sc.oz};
  const int n[3] = {sc.nx, sc.ny, sc.nz};
  for (int d = 0; d < 3; ++d) {
    int l = (int)floor((a[d] - o[d]) * sc.inv_res) - 1, u = (int)floor((b[d] - o[d]) * sc.inv_res) + 1;
    l = max(l, 0);
    u = min(u, n[d] - 1);
    while (l <= u && o[d] + (double)(l + 1) * sc.res < a[d]) ++l;
    while (u >= l && o[d] + (double)u * sc.res > b[d]) --u;
    if (l > u) return false;
    lo[d] = l;
    hi[d] = u;
  }
  return true;
}

// Relation of an upright primitive to the axis-aligned box [x0, x1] x [y0, y1] x [z0, z1] (a brick's cells in reach),
// decided with a margin eps far above the rounding of prim_cell: 0 = separated by more than eps (every cell of the box
// fails prim_cell: a separating axis of the box separates each of its cells by at least as much), 2 = inside by more
// than eps (every cell of the box passes prim_cell), 1 = undecided (the cells are tested one by one).
__device__ __forceinline__ int prim_box_relation(int ty, const double* __restrict__ h, const double* pw, double x0,
                                                 double x1, double y0, double y1, double z0, double z1) {
  constexpr double eps = 1e-9;
  const double hz = ty == 1 ? h[2] : h[1];
  if (z1 < pw[2] - hz - eps || z0 > pw[2] + hz + eps) return 0;
  const bool zin = z0 > pw[2] - hz + eps && z1 < pw[2] + hz - eps;
  const double wx = 0.5 * (x1 - x0), wy = 0.5 * (y1 - y0);
  const double dx = 0.5 * (x0 + x1) - pw[0], dy = 0.5 * (y0 + y1) - pw[1];
  if (ty == 2) {
    const double qx = fmax(fabs(dx) - wx, 0.0), qy = fmax(fabs(dy) - wy, 0.0);
    const double re = h[0] + eps;
    if (qx * qx + qy * qy > re * re) return 0;
    const double fx = fabs(dx) + wx, fy = fabs(dy) + wy, ri = h[0] - eps;  // the farthest corner
    return zin && ri > 0.0 && fx * fx + fy * fy < ri * ri ? 2 : 1;
  }
  const double c = pw[3], s = pw[4], ac = fabs(c), as = fabs(s);
  if (fabs(dx) > wx + (ac * h[0] + as * h[1]) + eps) return 0;
  if (fabs(dy) > wy + (as * h[0] + ac * h[1]) + eps) return 0;
  if (fabs(c * dx + s * dy) > h[0] + (wx * ac + wy * as) + eps) return 0;
  if (fabs(c * dy - s * dx) > h[1] + (wx * as + wy * ac) + eps) return 0;
  // inside: the box's extent along the primitive's two axes lies within its half extents
  const bool xin = fabs(c * dx + s * dy) + (wx * ac + wy * as) < h[0] - eps;
  const bool yin = fabs(c * dy - s * dx) + (wx * as + wy * ac) < h[1] - eps;
  return zin && xin && yin ? 2 : 1;
}

// Cooperative exact map test of one primitive by a wavefront: one brick word per lane over the reach, masked to the
// reach's cells, and each brick's cells in reach classified at once (prim_box_relation): a brick with an occupied cell
// inside the primitive is a hit, a separated brick is skipped, and the undecided bricks are swept one after the other
// with a lane per cell (prim_cell, ballot early exit).  The outcome is the exhaustive per-cell test's; a lane no longer
// walks its brick's occupied cells serially (up to 64 dependent prim_cell tests next to a solid obstacle).
__device__ __forceinline__ bool wave_prim_map(const SceneDev& sc, int ty, const double* __restrict__ h, const double* pw,
                                              int lane) {
  int lo[3], hi[3];
  if (!prim_reach(ty, h, pw, sc, lo, hi)) return false;
  const int bi0 = lo[0] >> 2, bj0 = lo[1] >> 2, bk0 = lo[2] >> 2;
  const int nbi = (hi[0] >> 2) - bi0 + 1, nbj = (hi[1] >> 2) - bj0 + 1, nbk = (hi[2] >> 2) - bk0 + 1;
  const int nb = nbi * nbj * nbk;
  for (int b0 = 0; b0 < nb; b0 += 64) {
    const int b = b0 + lane;
    uint64_t w = 0;
    int bi = 0, bj = 0, bk = 0, rel = 0;
    if (b < nb) {
      bi = bi0 + b % nbi;
      const int t = b / nbi;
      bj = bj0 + t % nbj;
      bk = bk0 + t / nbj;
      w = sc.bricks[((size_t)bk * sc.bny + bj) * sc.bnx + bi];
      if (w) {
        const int il = max(lo[0] - 4 * bi, 0), ih = min(hi[0] - 4 * bi, 3);
        const int jl = max(lo[1] - 4 * bj, 0), jh = min(hi[1] - 4 * bj, 3);
        const int kl = max(lo[2] - 4 * bk, 0), kh = min(hi[2] - 4 * bk, 3);
        const uint32_t xm = ((2u << ih) - 1u) & ~((1u << il) - 1u);
        uint32_t row = 0;
        for (int jj = jl; jj <= jh; ++jj) row |= xm << (4 * jj);
        uint64_t m = 0;
        for (int kk = kl; kk <= kh; ++kk) m |= (uint64_t)row << (16 * kk);
        w &= m;
        if (w)
          rel = prim_box_relation(ty, h, pw, sc.ox + (double)(4 * bi + il) * sc.res, sc.ox + (double)(4 * bi + ih + 1) * sc.res,
                                  sc.oy + (double)(4 * bj + jl) * sc.res, sc.oy + (double)(4 * bj + jh + 1) * sc.res,
                                  sc.oz + (double)(4 * bk + kl) * sc.res, sc.oz + (double)(4 * bk + kh + 1) * sc.res);
      }
    }
    if (__ballot(rel == 2)) return true;
    // the undecided bricks, a lane per cell
    for (uint64_t um = __ballot(rel == 1); um;) {
      const int src = __builtin_ctzll(um);  // (wave-uniform: the brick's words and indices by v_readlane)
      um &= um - 1;
      const uint32_t wlo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)w, src);
      const uint32_t whi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(w >> 32), src);
      const int sbi = __builtin_amdgcn_readlane(bi, src), sbj = __builtin_amdgcn_readlane(bj, src);
      const int sbk = __builtin_amdgcn_readlane(bk, src);
      const bool set = ((lane < 32 ? wlo >> lane : whi >> (lane - 32)) & 1u) != 0;
      const bool hit = set && prim_cell(ty, h, pw, sc, 4 * sbi + (lane & 3), 4 * sbj + ((lane >> 2) & 3), 4 * sbk + (lane >> 4));
      if (__ballot(hit)) return true;
    }
  }
  return false;
}

// Slab prefilter of primitive p (SceneDev::slab): true if p may touch the map (its centre's column holds a squared
// gap of at most pT); a centre outside the grid is free (the grid is padded by more than any rxy).
__device__ __forceinline__ bool prim_candidate(const SceneDev& sc, const uint16_t* __restrict__ slab, uint32_t pT,
                                               const double* pw) {
  const double fx = floor((pw[0] - sc.ox) * sc.inv_res), fy = floor((pw[1] - sc.oy) * sc.inv_res);
  if (!(fx >= 0 && fx < sc.nx && fy >= 0 && fy < sc.ny)) return false;
  return (uint32_t)slab[(size_t)(int)fy * sc.nx + (int)fx] <= pT;
}

// Exact sphere (world centre w, radius rs) vs upright primitive test: the squared distance from the centre to the
// solid box (in the box's frame) or cylinder against rs^2.  Shared term by term with the oracle (sphere_prim).
__device__ __forceinline__ bool sphere_prim(int ty, const double* __restrict__ h, const double* pw, const double* w,
                                            double rs) {
  const double dx = w[0] - pw[0], dy = w[1] - pw[1], dz = w[2] - pw[2];
  const double az = fabs(dz);
  if (ty == 1) {
    const double lx = fabs(pw[3] * dx + pw[4] * dy), ly = fabs(pw[3] * dy - pw[4] * dx);
    const double qx = lx > h[0] ? lx - h[0] : 0.0, qy = ly > h[1] ? ly - h[1] : 0.0, qz = az > h[2] ? az - h[2] : 0.0;
    return qx * qx + qy * qy + qz * qz <= rs * rs;
  }
  const double rho = sqrt(dx * dx + dy * dy);
  const double qr = rho > h[0] ? rho - h[0] : 0.0, qz = az > h[1] ? az - h[1] : 0.0;
  return qr * qr + qz * qz <= rs * rs;
}

constexpr int NWAVE = BLOCK / 64;

// LDS work area of one collision tile of CT configurations (CT a multiple of the wave count).
template <int CT>
struct TileLds {
  static constexpr int CPW = CT / NWAVE;  // configurations per wavefront in stage C
  static constexpr int SW = (MAX_SPH + 31) / 32;
  double fr[CT][MAX_BODY][12];              // body frames (R row-major, p)
  double tf[CT][2][12];                     // stage B: chain product, ping-pong
  union {
    double lf[CT][MAX_CHAIN][12];           // stages A/B: local frame of every chain step
    struct {
      double wc[CT][MAX_SPH][3];            // stage C: sphere world centres
      double pw[CT][MAX_PRIM][5];           // stage C: primitive centres and x axes
    } c;
  } u;
  uint32_t cand[CT][SW];                    // spheres needing the exact map sweep
  uint32_t pcand[CT];                       // primitives needing the exact map sweep
  int coll[CT];                             // 1 = in collision
};

// Optional ordering of a tile's configurations: configuration c is point ord[c] of group grp[c] (an edge);
// grp_first[g] is the lowest colliding point index of group g found so far.  A configuration whose index
// exceeds it is skipped (it cannot change the group's first collision); a colliding one lowers it.
// grp_first may live in LDS (one workgroup) or in HBM shared by several workgroups (agent = true: reads are
// agent-scope loads, so a stale L1 line of an earlier job can never cause a skip).
struct TileOrder {
  const int* grp;
  const int* ord;
  int* grp_first;
  bool agent;
  __device__ __forceinline__ int first(int g) const {
    return agent ? __hip_atomic_load(&grp_first[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                 : __atomic_load_n(&grp_first[g], __ATOMIC_RELAXED);
  }
};

// Collision test of nc <= CT configurations already placed in q_lds[c][8] (LDS), all block threads.
// On return coll[c] is 1 for colliding configurations (0 for free or skipped ones).
//   A. local frame of every (configuration, chain step), sin/cos included, one lane each;
//   B. body frames: one lane per configuration multiplies its chain in order (KDL Frame*Frame);
//   C. wavefront w owns configurations w, w + 8, ...: lanes over (configuration, sphere) items with the d2
//      loads of all of them issued together; the rare spheres near an occupied box are swept by the whole
//      wave; then lanes over the flat list of sphere pairs of the enabled link pairs, the wave's
//      configurations interleaved per pair.  No block barrier inside stage C.
// Every stage is laid out as many short independent chains per lane rather than one long chain (a dependent fp64
// mul / add is ~5 cycles on gfx950, an LDS round trip 50-100: tools/micro/fp64_latency.hip).
template <int CT>
__device__ __forceinline__ void collide_tile(const RobotDev* __restrict__ rb, const SceneDev& sc_in,
                                             const MapCfg* __restrict__ mc, int nc, const double (*q_lds)[NJ],
                                             int self, int map, TileLds<CT>& L, const TileOrder* ord = nullptr,
                                             unsigned long long* prof = nullptr, unsigned long long* prof2 = nullptr) {
  static_assert(CT % NWAVE == 0, "tile size");
  const SceneDev sc = uniform_scene(sc_in);
  constexpr int CPW = TileLds<CT>::CPW, SW = TileLds<CT>::SW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  unsigned long long t0 = (prof && tid == 0) ? wall_clock64() : 0;
  const int nch = rb->n_chain;
  static_assert(CT <= 4 * NWAVE, "stages A/B: four configurations per wavefront");
  // A: wavefront w builds the local frames of its configurations 4w .. 4w+3 (sin/cos included), one
  // (configuration, chain step) per lane, so that B (same wavefront) needs no block barrier.
  {
    const int cb = wave * 4;
    for (int it = lane; it < 4 * nch; it += 64) {
      const int c = cb + it / nch, k = it - (it / nch) * nch;
      if (c >= nc) break;
      double st = 0.0, ct = 1.0;
      if (rb->ch_type[k] == 1) psincos(q_lds[c][rb->ch_joint[k]], &st, &ct);
      Frame F;
      chain_local(rb, k, q_lds[c], st, ct, &F);
      double* o = L.u.lf[c][k];
      for (int i = 0; i < 9; ++i) o[i] = F.R[i];
      o[9] = F.p[0]; o[10] = F.p[1]; o[11] = F.p[2];
    }
    for (int it = tid; it < CT * SW; it += BLOCK) (&L.cand[0][0])[it] = 0u;
    if (tid < CT) L.pcand[tid] = 0u;
    if (tid < nc) L.coll[tid] = 0;
    wave_sync();
  }
  unsigned long long ta = (prof && tid == 0) ? wall_clock64() : 0;
  // B: one lane per element of the chain product, 16 lanes per configuration (rows r = 0..2 of four lanes:
  // columns 0..2 of R, then p; the fourth row of lanes idles).  Element (r, col) of T * L is row r of T times
  // column col of L -- fmul's three-term sum in its order, p adding T.p[r] last -- and row r of T is read from
  // the lane's own quad by DPP broadcasts, so a chain step costs one dependent mul/add/add plus the broadcast
  // and each lane issues five fp64 operations per step instead of twenty (stage B is issue-bound in one wave).
  {
    const int c = wave * 4 + (lane >> 4), r = (lane >> 2) & 3, col = lane & 3;
    if (c < nc && r < 3) {
      const int lo = col < 3 ? col : 9, ls = col < 3 ? 3 : 1;  // column col of L: lf[lo + i * ls], i = 0..2
      double v = col < 3 ? (r == col ? 1.0 : 0.0) : (r == 2 ? rb->root_z : 0.0);
      const double* lf = L.u.lf[c][0];
      double l0 = lf[lo], l1 = lf[lo + ls], l2 = lf[lo + 2 * ls];
      int bd = rb->ch_body[0];
      const int oidx = col < 3 ? r * 3 + col : 9 + r;
      for (int k = 0; k < nch; ++k) {
        const int kn = k + 1 < nch ? k + 1 : k;
        const double* ln = L.u.lf[c][kn];
        const double n0 = ln[lo], n1 = ln[lo + ls], n2 = ln[lo + 2 * ls];
        const int bdn = rb->ch_body[kn];
        const double t0 = quad_bcast<0>(v), t1 = quad_bcast<1>(v), t2 = quad_bcast<2>(v);
        const double s = t0 * l0 + t1 * l1 + t2 * l2;
        const double sp = s + v;
        v = col < 3 ? s : sp;
        if (bd >= 0) L.fr[c][bd][oidx] = v;
        l0 = n0; l1 = n1; l2 = n2;
        bd = bdn;
      }
    }
  }
  __syncthreads();
  unsigned long long t1 = (prof && tid == 0) ? wall_clock64() : 0;
  // C
  const int nsph = rb->n_sph;
  const bool do_map = map && mc->has_map;
  // live configurations of this wave (skipped ones stay coll = 0)
  uint32_t live = 0;
  for (int k = 0; k < CPW; ++k) {
    const int c = k * NWAVE + wave;
    if (c < nc && !(ord && ord->ord[c] > ord->first(ord->grp[c])))
      live |= 1u << k;
  }
  if (live) {
    constexpr int MAXU = (CPW * MAX_SPH + 63) / 64;
    long long cell[MAXU];
#pragma unroll
    for (int u = 0; u < MAXU; ++u) {
      const int it = u * 64 + lane;
      cell[u] = -1;
      const int k = it / nsph, s = it - k * nsph;
      if (k < CPW && ((live >> k) & 1u)) {
        const int c = k * NWAVE + wave;
        const double* B = L.fr[c][rb->sph_body[s]];
        const double* p = &rb->sph_cb[s * 3];
        double w[3];
        for (int r = 0; r < 3; ++r) {
          double m = B[r * 3 + 0] * p[0] + B[r * 3 + 1] * p[1] + B[r * 3 + 2] * p[2];
          w[r] = m + B[9 + r];
        }
        L.u.c.wc[c][s][0] = w[0]; L.u.c.wc[c][s][1] = w[1]; L.u.c.wc[c][s][2] = w[2];
        if (do_map && mc->map_on[s]) cell[u] = centre_cell(sc, w);
      }
    }
    uint32_t dv[MAXU];
    if (sc.d2b) {
#pragma unroll
      for (int u = 0; u < MAXU; ++u) dv[u] = cell[u] >= 0 ? (uint32_t)sc.d2b[cell[u]] : 0xffffffffu;
    } else {
#pragma unroll
      for (int u = 0; u < MAXU; ++u) dv[u] = cell[u] >= 0 ? (uint32_t)sc.d2[cell[u]] : 0xffffffffu;
    }
#pragma unroll
    for (int u = 0; u < MAXU; ++u) {
      const int it = u * 64 + lane;
      const int k = it / nsph, s = it - k * nsph;
      if (cell[u] >= 0 && dv[u] <= mc->T[s]) atomicOr(&L.cand[k * NWAVE + wave][s >> 5], 1u << (s & 31));
    }
    // primitives: world frames (for the self test too) and the slab prefilter, lanes over (configuration, primitive)
    const int npr = rb->n_prim;
    for (int it = lane; it < CPW * npr; it += 64) {
      const int k = it / npr, p = it - k * npr;
      if (!((live >> k) & 1u)) continue;
      const int c = k * NWAVE + wave;
      double* pw = L.u.c.pw[c][p];
      prim_world(rb, p, L.fr[c][rb->prim_body[p]], pw);
      if (do_map && mc->p_map_on[p] && prim_candidate(sc, sc_in.slab[p], mc->pT[p], pw))
        atomicOr(&L.pcand[c], 1u << p);
    }
    wave_sync();
    if (prof && tid == 0) prof[2] += wall_clock64() - t1;
    // map sweeps
    uint32_t hitm = 0;
    for (int k = 0; k < CPW; ++k) {
      if (!((live >> k) & 1u)) continue;
      const int c = k * NWAVE + wave;
      bool hit = false;
      for (uint32_t pm = L.pcand[c]; pm && !hit;) {
        const int p = __builtin_ctz(pm);
        pm &= pm - 1;
        const double pw[5] = {L.u.c.pw[c][p][0], L.u.c.pw[c][p][1], L.u.c.pw[c][p][2], L.u.c.pw[c][p][3],
                              L.u.c.pw[c][p][4]};
        hit = wave_prim_map(sc, rb->prim_type[p], &rb->prim_h[p * 3], pw, lane);
      }
      // the candidate spheres' brick words in one round trip, staged in this configuration's body-frame rows (dead
      // once its centres and primitive frames are formed) -- one round trip per candidate before
      uint32_t any = 0;
      for (int wd = 0; wd < SW; ++wd) any |= L.cand[c][wd];
      if (!hit && any) {
        static_assert(sizeof(L.fr[0]) >= MAP_STAGE_W * sizeof(uint64_t), "staging buffer in the body-frame rows");
        static_assert(sizeof(L.tf[0]) >= MAP_STAGE_W + MAX_SPH, "slot owners and offsets in the stage-B rows");
        uint8_t* tb = reinterpret_cast<uint8_t*>(&L.tf[c][0][0]);
        hit = wave_map_staged(rb, sc, L.u.c.wc[c], L.cand[c], nsph, reinterpret_cast<uint64_t*>(&L.fr[c][0][0]), tb,
                              tb + MAP_STAGE_W, lane);
      }
      if (hit) hitm |= 1u << k;
    }
    const unsigned long long tm = (prof2 && tid == 0) ? wall_clock64() : 0;
    if (self) {
      // every sphere pair of the enabled link pairs, the CPW configurations of this wave interleaved
      const uint32_t todo = live & ~hitm;
      if (todo) {
        const int nsp = rb->n_spairs;
        uint32_t sh = 0;
#pragma unroll 4
        for (int p = lane; p < nsp; p += 64) {
          const uint32_t ab = rb->sp_ab[p];
          const int a = ab & 0xff, b = ab >> 8;
          const double rr2 = rb->sp_rr2[p];
#pragma unroll
          for (int k = 0; k < CPW; ++k) {
            const double* wa = L.u.c.wc[k * NWAVE + wave][a];
            const double* wb = L.u.c.wc[k * NWAVE + wave][b];
            const double ex = wa[0] - wb[0], ey = wa[1] - wb[1], ez = wa[2] - wb[2];
            if (ex * ex + ey * ey + ez * ez <= rr2) sh |= 1u << k;
          }
        }
        // (primitive, sphere) pairs
        const int npp = rb->n_ppairs;
        for (int p = lane; p < npp; p += 64) {
          const uint32_t ps = rb->pp_ps[p];
          const int pr = ps & 0xff, sp = ps >> 8;
          const int ty = rb->prim_type[pr];
          const double rs = rb->sph_r[sp];
#pragma unroll
          for (int k = 0; k < CPW; ++k)
            if (sphere_prim(ty, &rb->prim_h[pr * 3], L.u.c.pw[k * NWAVE + wave][pr], L.u.c.wc[k * NWAVE + wave][sp], rs))
              sh |= 1u << k;
        }
        for (int k = 0; k < CPW; ++k)
          if (((todo >> k) & 1u) && __ballot((sh >> k) & 1u)) hitm |= 1u << k;
      }
    }
    if (prof2 && tid == 0) {
      const unsigned long long ts = wall_clock64();
      prof2[0] += tm - t1;  // wave 0: centres + map sweeps
      prof2[1] += ts - tm;  // wave 0: self test
    }
    if (lane == 0) {
      for (int k = 0; k < CPW; ++k) {
        if (!((hitm >> k) & 1u)) continue;
        const int c = k * NWAVE + wave;
        L.coll[c] = 1;
        if (ord) atomicMin(&ord->grp_first[ord->grp[c]], ord->ord[c]);
      }
    }
  }
  __syncthreads();
  if (prof && tid == 0) {
    unsigned long long t2 = wall_clock64();
    prof[0] += ta - t0; prof[1] += t1 - ta; prof[3] += t2 - t1;
  }
}

// ------------------------------------------------------------------------------------------ job tiles (collide_wide)
// brick words a wavefront of collide_wide stages for its candidate spheres in one round trip (a 2 cm sphere needs up to
// 64: collide_tile's 96 held one of them)
#ifndef SMP_WIDE_STAGE_W
#define SMP_WIDE_STAGE_W 320
#endif
constexpr int WIDE_STAGE_W = SMP_WIDE_STAGE_W;
// LDS of one wavefront of collide_wide: the configuration's kinematics, centres and staging, private to the wavefront.
struct WideWave {
  union {
    double lf[MAX_CHAIN][12];               // stages A/B: local frame of every chain step
    struct {
      double wc[MAX_SPH][3];                // C: sphere world centres
      double pw[MAX_PRIM][5];               // C: primitive centres and x axes
    } c;
  } u;
  struct {
    double fr[MAX_BODY][12];                // B -> centres: body frames (R row-major, p)
  } v;
  uint32_t cand[(MAX_SPH + 31) / 32];       // this wavefront's candidate spheres (map sweep)
  uint32_t pcand;                           // this wavefront's candidate primitives
  uint64_t stage[WIDE_STAGE_W];             // map sweeps: the candidates' brick words (wave_map_staged)
  uint16_t off[MAX_SPH];                    // wave_map_staged: first slot per sphere
  uint8_t owner[WIDE_STAGE_W];              // wave_map_staged: slot owners
  uint16_t list[MAP_LIST];                  // sweep_occupied: the occupied cells of one candidate's reach
};
struct WideLds {
  WideWave w[NWAVE];
  int coll[NWAVE];                          // configuration c: 1 = in collision
};

// Collision test of nc <= ct configurations q_lds[c], ct in {1, 2, 4, 8}, all block threads.  Configuration c belongs
// to the G = 8 / ct wavefronts c*G .. c*G + G - 1 (its group): a job tile of one configuration is spread over the whole
// workgroup instead of one wavefront.  Every wavefront of a group computes the configuration's kinematics, all sphere
// centres and all primitive frames by itself (the same values; the stages A/B/centres need no block barrier), then
// takes its share of the tests -- the map tests of spheres and primitives s with s % G == g (g = its rank in the group:
// box-gap / slab prefilter, exact sweeps of the candidates in one load round trip, as collide_tile) and the self pairs
// of the 64-pair chunks k with k % G == g.  A configuration collides iff any test hits (the reference's
// isInCollision is map || self, collision_checker.hpp:104-121), so the split changes no result; a wavefront stops
// after its first hit or once another wavefront of the group reported one.  The caller zeroes L.coll[0 .. ct) before
// the barrier that publishes q_lds; on return (after a block barrier) L.coll[c] is 1 for the colliding configurations.
// prof (thread 0): stage clocks A, B, centres + prefilter loads, whole tile, as collide_tile's.
__device__ __forceinline__ void collide_wide(const RobotDev* __restrict__ rb, const SceneDev& sc_in,
                                             const MapCfg* __restrict__ mc, int ct, int nc, const double (*q_lds)[NJ],
                                             int self, int map, WideLds& L, const TileOrder* ord = nullptr,
                                             unsigned long long* prof = nullptr, unsigned long long* prof2 = nullptr) {
  const SceneDev sc = uniform_scene(sc_in);
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int G = __builtin_amdgcn_readfirstlane(NWAVE / ct);
  const int c = wave / G, g = wave - c * G;
  WideWave& W = L.w[wave];
  const unsigned long long t0 = (prof && threadIdx.x == 0) ? wall_clock64() : 0;
  unsigned long long ta = t0, tb = t0, tc = t0;
  int live = c < nc;
  if (live && ord) live = !(ord->ord[c] > ord->first(ord->grp[c]));
  if (__builtin_amdgcn_readfirstlane(live)) {
    const double* q = q_lds[c];
    const int nch = rb->n_chain;
    // A: local frame of every chain step (sin/cos included), one lane each
    if (lane < nch) {
      double st = 0.0, cs = 1.0;
      if (rb->ch_type[lane] == 1) psincos(q[rb->ch_joint[lane]], &st, &cs);
      Frame F;
      chain_local(rb, lane, q, st, cs, &F);
      double* o = W.u.lf[lane];
      for (int i = 0; i < 9; ++i) o[i] = F.R[i];
      o[9] = F.p[0]; o[10] = F.p[1]; o[11] = F.p[2];
    }
    if (lane < (MAX_SPH + 31) / 32) W.cand[lane] = 0u;
    if (lane == 0) W.pcand = 0u;
    wave_sync();
    if (prof && threadIdx.x == 0) ta = wall_clock64();
    // B: the chain product, one lane per element (rows r = 0..2 of four lanes: columns 0..2 of R, then p), as
    // collide_tile's stage B (fmul's three-term sums in KDL order; row r of T from the lane's quad by DPP broadcasts)
    if (lane < 12) {
      const int r = lane >> 2, col = lane & 3;
      const int lo = col < 3 ? col : 9, ls = col < 3 ? 3 : 1;
      double v = col < 3 ? (r == col ? 1.0 : 0.0) : (r == 2 ? rb->root_z : 0.0);
      double l0 = W.u.lf[0][lo], l1 = W.u.lf[0][lo + ls], l2 = W.u.lf[0][lo + 2 * ls];
      int bd = rb->ch_body[0];
      const int oidx = col < 3 ? r * 3 + col : 9 + r;
      for (int k = 0; k < nch; ++k) {
        const int kn = k + 1 < nch ? k + 1 : k;
        const double* ln = W.u.lf[kn];
        const double n0 = ln[lo], n1 = ln[lo + ls], n2 = ln[lo + 2 * ls];
        const int bdn = rb->ch_body[kn];
        const double t0v = quad_bcast<0>(v), t1v = quad_bcast<1>(v), t2v = quad_bcast<2>(v);
        const double s = t0v * l0 + t1v * l1 + t2v * l2;
        const double sp = s + v;
        v = col < 3 ? s : sp;
        if (bd >= 0) W.v.fr[bd][oidx] = v;
        l0 = n0; l1 = n1; l2 = n2;
        bd = bdn;
      }
    }
    wave_sync();
    if (prof && threadIdx.x == 0) tb = wall_clock64();
    // centres of every sphere and frames of every primitive (the self pairs need them all); the prefilter loads of
    // this wavefront's share, all issued together
    const int nsph = rb->n_sph, npr = rb->n_prim;
    const bool do_map = map && mc->has_map;
    // (the cells first, then every load -- box-gap bytes of the spheres, slab words of the primitives -- issued before
    // any is used: in a 2 cm scene the 25 MB field lives in the Infinity Cache, and dependent rounds cost ~1 us each)
    long long cell[2], pcell[2];
    const uint16_t* pslab[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int it = u * 64 + lane;
      cell[u] = -1;
      pcell[u] = -1;
      pslab[u] = nullptr;
      if (it < nsph) {
        const double* B = W.v.fr[rb->sph_body[it]];
        const double* p = &rb->sph_cb[it * 3];
        double w[3];
        for (int r = 0; r < 3; ++r) {
          const double m = B[r * 3 + 0] * p[0] + B[r * 3 + 1] * p[1] + B[r * 3 + 2] * p[2];
          w[r] = m + B[9 + r];
        }
        W.u.c.wc[it][0] = w[0]; W.u.c.wc[it][1] = w[1]; W.u.c.wc[it][2] = w[2];
        if (do_map && mc->map_on[it] && it % G == g) cell[u] = centre_cell(sc, w);
      } else if (it < nsph + npr) {
        const int p = it - nsph;
        double pw[5];
        prim_world(rb, p, W.v.fr[rb->prim_body[p]], pw);
        for (int i = 0; i < 5; ++i) W.u.c.pw[p][i] = pw[i];
        if (do_map && mc->p_map_on[p] && p % G == g) {  // prim_candidate: its centre's column, else free
          const double fx = floor((pw[0] - sc.ox) * sc.inv_res), fy = floor((pw[1] - sc.oy) * sc.inv_res);
          if (fx >= 0 && fx < sc.nx && fy >= 0 && fy < sc.ny) {
            pcell[u] = (long long)(int)fy * sc.nx + (int)fx;
            pslab[u] = sc_in.slab[p];
          }
        }
      }
    }
    uint32_t dv[2], sv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      dv[u] = cell[u] < 0 ? 0xffffffffu : (sc.d2b ? (uint32_t)sc.d2b[cell[u]] : (uint32_t)sc.d2[cell[u]]);
      sv[u] = pcell[u] < 0 ? 0xffffffffu : (uint32_t)pslab[u][pcell[u]];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int it = u * 64 + lane;
      if (cell[u] >= 0 && dv[u] <= mc->T[it]) atomicOr(&W.cand[it >> 5], 1u << (it & 31));
      if (pcell[u] >= 0 && sv[u] <= mc->pT[it - nsph]) atomicOr(&W.pcand, 1u << (it - nsph));
    }
    wave_sync();
    if (prof && threadIdx.x == 0) tc = wall_clock64();
    // map: this wavefront's candidate primitives, then its candidate spheres (their brick words in one round trip)
    bool hit = false;
    unsigned long long tp0 = (prof2 && threadIdx.x == 0) ? wall_clock64() : 0, tp1 = tp0, tp2 = tp0;
    for (uint32_t pm = (uint32_t)__builtin_amdgcn_readfirstlane((int)W.pcand); pm && !hit;) {
      const int p = __builtin_ctz(pm);
      pm &= pm - 1;
      if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&L.coll[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
        break;
      const double pw[5] = {W.u.c.pw[p][0], W.u.c.pw[p][1], W.u.c.pw[p][2], W.u.c.pw[p][3], W.u.c.pw[p][4]};
      hit = wave_prim_map(sc, rb->prim_type[p], &rb->prim_h[p * 3], pw, lane);
    }
    if (prof2 && threadIdx.x == 0) tp1 = wall_clock64();
    uint32_t any = 0;
    for (int wd = 0; wd < (MAX_SPH + 31) / 32; ++wd) any |= W.cand[wd];
    if (!hit && __builtin_amdgcn_readfirstlane((int)(any != 0)) &&
        !__builtin_amdgcn_readfirstlane(__hip_atomic_load(&L.coll[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
      hit = wave_map_staged<WIDE_STAGE_W, uint16_t>(rb, sc, W.u.c.wc, W.cand, nsph, W.stage, W.owner, W.off, lane,
                                                    W.list);
    if (prof2 && threadIdx.x == 0) tp2 = wall_clock64();
    // self: this wavefront's 64-pair chunks of the sphere pairs, then of the (primitive, sphere) pairs
    if (self && !hit &&
        !__builtin_amdgcn_readfirstlane(__hip_atomic_load(&L.coll[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) {
      const int nsp = rb->n_spairs, npp = rb->n_ppairs, ks = (nsp + 63) >> 6;
      bool sh = false;
#pragma unroll 4
      for (int k = g; k < ks; k += G) {
        const int p = k * 64 + lane;
        if (p < nsp) {
          const uint32_t ab = rb->sp_ab[p];
          const double* wa = W.u.c.wc[ab & 0xff];
          const double* wb = W.u.c.wc[ab >> 8];
          const double ex = wa[0] - wb[0], ey = wa[1] - wb[1], ez = wa[2] - wb[2];
          sh |= ex * ex + ey * ey + ez * ez <= rb->sp_rr2[p];
        }
      }
      // chunk numbers continue after the sphere pairs', so that G > ks wavefronts share the primitive pairs
      for (int k = (g - ks % G + G) % G; k * 64 < npp; k += G) {
        const int p = k * 64 + lane;
        if (p < npp) {
          const uint32_t ps = rb->pp_ps[p];
          const int pr = ps & 0xff, sp = ps >> 8;
          sh |= sphere_prim(rb->prim_type[pr], &rb->prim_h[pr * 3], W.u.c.pw[pr], W.u.c.wc[sp], rb->sph_r[sp]);
        }
      }
      hit = __ballot(sh) != 0;
    }
    if (prof2 && threadIdx.x == 0) {  // wave 0: primitive sweeps, sphere sweeps, self test
      const unsigned long long tp3 = wall_clock64();
      prof2[0] += tp1 - tp0; prof2[1] += tp2 - tp1; prof2[2] += tp3 - tp2;
    }
    if (hit && lane == 0) {
      atomicOr(&L.coll[c], 1);
      if (ord) atomicMin(&ord->grp_first[ord->grp[c]], ord->ord[c]);
    }
  }
  __syncthreads();
  if (prof && threadIdx.x == 0) {
    prof[0] += ta - t0; prof[1] += tb - ta; prof[2] += tc - tb; prof[3] += wall_clock64() - tb;
  }
}

}  // namespace smp
