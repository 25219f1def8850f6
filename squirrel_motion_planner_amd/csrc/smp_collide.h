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

constexpr int BLOCK = 256;

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

__device__ __forceinline__ bool occ_bit(const SceneDev& s, int i, int j, int k) {
  return (s.bits[((size_t)k * s.ny + j) * s.wx + (i >> 6)] >> (i & 63)) & 1ull;
}

// One sphere vs the occupied voxel boxes: d2 prefilter, then the exact box test over the reach.
__device__ __forceinline__ bool sphere_hits_map(const SceneDev& s, const double* c, double r, uint32_t T) {
  double fx = floor((c[0] - s.ox) / s.res), fy = floor((c[1] - s.oy) / s.res), fz = floor((c[2] - s.oz) / s.res);
  if (!(fx >= 0 && fx < s.nx && fy >= 0 && fy < s.ny && fz >= 0 && fz < s.nz)) return false;
  int ci = (int)fx, cj = (int)fy, ck = (int)fz;
  if ((uint32_t)s.d2[((size_t)ck * s.ny + cj) * s.nx + ci] > T) return false;
  int i0 = (int)floor((c[0] - r - s.ox) / s.res) - 1, i1 = (int)floor((c[0] + r - s.ox) / s.res) + 1;
  int j0 = (int)floor((c[1] - r - s.oy) / s.res) - 1, j1 = (int)floor((c[1] + r - s.oy) / s.res) + 1;
  int k0 = (int)floor((c[2] - r - s.oz) / s.res) - 1, k1 = (int)floor((c[2] + r - s.oz) / s.res) + 1;
  i0 = max(i0, 0); j0 = max(j0, 0); k0 = max(k0, 0);
  i1 = min(i1, s.nx - 1); j1 = min(j1, s.ny - 1); k1 = min(k1, s.nz - 1);
  double r2 = r * r;
  for (int k = k0; k <= k1; ++k) {
    double zlo = s.oz + (double)k * s.res, zhi = s.oz + (double)(k + 1) * s.res;
    double dz = c[2] < zlo ? zlo - c[2] : (c[2] > zhi ? c[2] - zhi : 0.0);
    double dz2 = dz * dz;
    if (dz2 > r2) continue;  // exact early-out: dx*dx + dy*dy + dz2 >= dz2 in IEEE (no negative terms)
    for (int j = j0; j <= j1; ++j) {
      double ylo = s.oy + (double)j * s.res, yhi = s.oy + (double)(j + 1) * s.res;
      double dy = c[1] < ylo ? ylo - c[1] : (c[1] > yhi ? c[1] - yhi : 0.0);
      const uint64_t* row = s.bits + ((size_t)k * s.ny + j) * s.wx;
      for (int i = i0; i <= i1; ++i) {
        if (!((row[i >> 6] >> (i & 63)) & 1ull)) continue;
        double xlo = s.ox + (double)i * s.res, xhi = s.ox + (double)(i + 1) * s.res;
        double dx = c[0] < xlo ? xlo - c[0] : (c[0] > xhi ? c[0] - xhi : 0.0);
        if (dx * dx + dy * dy + dz * dz <= r2) return true;
      }
    }
  }
  return false;
}

// LDS work area of one collision tile of CT configurations.
template <int CT>
struct TileLds {
  Frame frames[CT][MAX_BODY];     // 32 x 6 x 96 B used
  double wc[CT][MAX_SPH][3];      // sphere world centres
  double lbw[CT][MAX_CLINK][3];   // link-bound world centres
  int coll[CT];                   // 1 = in collision
};

// Collision test of nc <= CT configurations already placed in q_lds[c][8] (LDS), all block threads.
// On return coll[c] is 1 for colliding configurations.  Uses three barriers.
template <int CT>
__device__ __forceinline__ void collide_tile(const RobotDev* __restrict__ rb, const SceneDev& sc,
                                             const MapCfg* __restrict__ mc, int nc, const double (*q_lds)[NJ],
                                             int self, int map, TileLds<CT>& L, unsigned long long* prof = nullptr) {
  const int tid = threadIdx.x;
  unsigned long long t0 = (prof && tid == 0) ? wall_clock64() : 0;
  if (tid < nc) {
    double q[NJ];
    for (int j = 0; j < NJ; ++j) q[j] = q_lds[tid][j];
    body_frames(rb, q, L.frames[tid]);
    L.coll[tid] = 0;
  }
  __syncthreads();
  unsigned long long t1 = (prof && tid == 0) ? wall_clock64() : 0;
  const int nsph = rb->n_sph, ncl = rb->n_clink;
  for (int it = tid; it < nc * nsph; it += BLOCK) {
    int c = it / nsph, s = it - c * nsph;
    double w[3];
    xform(L.frames[c][rb->sph_body[s]], &rb->sph_cb[s * 3], w);
    L.wc[c][s][0] = w[0]; L.wc[c][s][1] = w[1]; L.wc[c][s][2] = w[2];
    if (map && mc->has_map && mc->map_on[s] && sphere_hits_map(sc, w, rb->sph_r[s], mc->T[s])) L.coll[c] = 1;
  }
  if (self) {
    for (int it = tid; it < nc * ncl; it += BLOCK) {
      int c = it / ncl, l = it - c * ncl;
      double w[3];
      xform(L.frames[c][rb->cl_body[l]], &rb->cl_cb[l * 3], w);
      L.lbw[c][l][0] = w[0]; L.lbw[c][l][1] = w[1]; L.lbw[c][l][2] = w[2];
    }
  }
  __syncthreads();
  unsigned long long t2 = (prof && tid == 0) ? wall_clock64() : 0;
  if (self) {
    const int np = rb->n_pairs;
    for (int it = tid; it < nc * np; it += BLOCK) {
      int c = it / np, p = it - c * np;
      if (L.coll[c]) continue;
      int a = rb->pair_a[p], b = rb->pair_b[p];
      double dx = L.lbw[c][a][0] - L.lbw[c][b][0], dy = L.lbw[c][a][1] - L.lbw[c][b][1], dz = L.lbw[c][a][2] - L.lbw[c][b][2];
      double rr = rb->cl_r[a] + rb->cl_r[b];
      if (dx * dx + dy * dy + dz * dz > rr * rr) continue;
      int sa0 = rb->cl_sph0[a], sa1 = sa0 + rb->cl_nsph[a];
      int sb0 = rb->cl_sph0[b], sb1 = sb0 + rb->cl_nsph[b];
      bool hit = false;
      for (int sa = sa0; sa < sa1 && !hit; ++sa)
        for (int sb = sb0; sb < sb1; ++sb) {
          double ex = L.wc[c][sa][0] - L.wc[c][sb][0], ey = L.wc[c][sa][1] - L.wc[c][sb][1], ez = L.wc[c][sa][2] - L.wc[c][sb][2];
          double r2 = rb->sph_r[sa] + rb->sph_r[sb];
          if (ex * ex + ey * ey + ez * ez <= r2 * r2) { hit = true; break; }
        }
      if (hit) L.coll[c] = 1;
    }
  }
  __syncthreads();
  if (prof && tid == 0) {
    unsigned long long t3 = wall_clock64();
    prof[0] += t1 - t0; prof[1] += t2 - t1; prof[2] += t3 - t2;
  }
}

}  // namespace smp
