// Plain-old-data layouts shared by the host builder and the HIP kernels.
#pragma once
#include <stdint.h>

namespace smp {

constexpr int MAX_CHAIN = 16;   // body chain steps (11 for robotino)
constexpr int MAX_SEG = 16;     // end-effector chain segments (12)
constexpr int MAX_SPH = 72;     // collision spheres (64)
constexpr int MAX_CLINK = 32;   // collision links (27)
constexpr int MAX_PAIRS = 256;  // self-collision link pairs (165 non-rigid of the 230 SRDF-enabled)
constexpr int MAX_BODY = 8;     // moving bodies (6)
constexpr int MAX_SPAIRS = 768; // sphere pairs of the enabled link pairs (499)
constexpr int MAX_PRIM = 8;     // exact box / cylinder primitives (6: the URDF's box and cylinder links)
constexpr int MAX_PPAIRS = 320; // (primitive, sphere) pairs of the enabled link pairs (187)
constexpr int NJ = 8;           // planning joints
constexpr int BLOCK = 512;      // threads per workgroup (8 wavefronts, 2 per SIMD)

// Robot model (kinematics + collision model).  Collision links are re-indexed into compact "clink" slots; spheres are
// sorted by clink so each link owns a contiguous range.  A link is either a set of spheres (mesh covers) or one exact
// primitive: an upright box or cylinder on a planar body (world frame Trans(x, y, z0) Rz(a)), collided exactly as the
// reference's fcl::Box / fcl::Cylinder (collision_checker.hpp:282-288).
struct RobotDev {
  int n_chain, n_seg, n_sph, n_clink, n_pairs, n_body;
  double root_z;
  int ch_type[MAX_CHAIN], ch_joint[MAX_CHAIN], ch_body[MAX_CHAIN];  // type: 0 fixed 1 revolute 2 prismatic
  double ch_axis[MAX_CHAIN * 3], ch_origin[MAX_CHAIN * 3], ch_R[MAX_CHAIN * 9], ch_p[MAX_CHAIN * 3];
  int seg_type[MAX_SEG], seg_joint[MAX_SEG];
  double seg_axis[MAX_SEG * 3], seg_origin[MAX_SEG * 3], seg_R[MAX_SEG * 9], seg_p[MAX_SEG * 3];
  int sph_body[MAX_SPH], sph_clink[MAX_SPH];
  double sph_cb[MAX_SPH * 3], sph_r[MAX_SPH];
  int cl_sph0[MAX_CLINK], cl_nsph[MAX_CLINK], cl_body[MAX_CLINK], cl_link[MAX_CLINK];
  double cl_cb[MAX_CLINK * 3], cl_r[MAX_CLINK];
  int pair_a[MAX_PAIRS], pair_b[MAX_PAIRS];
  // primitives: type 1 box (half extents hx, hy, hz), 2 cylinder (radius, half length, 0); centre cb and x axis ab in
  // the body frame (the z axis is the body's, vertical); rxy bounds the horizontal reach from the centre
  int n_prim;
  int prim_type[MAX_PRIM], prim_body[MAX_PRIM], prim_clink[MAX_PRIM];
  double prim_cb[MAX_PRIM * 3], prim_ab[MAX_PRIM * 3], prim_h[MAX_PRIM * 3], prim_rxy[MAX_PRIM];
  int cl_prim[MAX_CLINK];  // primitive of a collision link, -1 for a sphere link
  // flat (primitive, sphere) list of the enabled link pairs: prim | sphere << 8
  int n_ppairs;
  uint16_t pp_ps[MAX_PPAIRS];
  // flat self-collision list: every sphere pair of every enabled link pair, (a | b << 8) and (ra + rb)^2
  int n_spairs;
  uint16_t sp_ab[MAX_SPAIRS];
  double sp_rr2[MAX_SPAIRS];
  double q_min[NJ], q_max[NJ];
  int rev[NJ];
};


// Occupancy grid of one scene (device pointers).  Cell (i,j,k) is the box [o + i*res, o + (i+1)*res] per
// axis.  bricks: one 64-bit occupancy mask per 4x4x4 cells, bit (k&3)*16 + (j&3)*4 + (i&3) of brick
// ((k>>2)*bny + (j>>2))*bnx + (i>>2).  d2: per cell the squared box-to-box gap (voxel units, clamped to
// 65535) to the nearest occupied cell -- a lower bound of (distance to any occupied box / res)^2.
// d2b: the same field clamped to 255, one byte per cell (half the bytes, so a 5 cm 10x10x2 m grid stays
// resident in one XCD's 4 MB L2); set only when every sphere threshold T is below 255, where
// min(d2, 255) > T  <=>  d2 > T, so the prefilter decides identically.
// slab[p]: per primitive p, the 2-D box-gap field (nx x ny, x fastest; squared gap in cells, <= 65535) of the
// occupancy projected over the grid layers that p's constant z range [zc - hz, zc + hz] touches: p's footprint lies
// within rxy of its centre, so p is free of the map when slab[p] at its centre's column exceeds pT[p].
struct SceneDev {
  int nx, ny, nz, bnx, bny;
  double ox, oy, oz, res, inv_res;
  const uint64_t* bricks;
  const uint16_t* d2;
  const uint8_t* d2b;
  const uint16_t* slab[MAX_PRIM];
};

// Per (scene, disabled-link set) sphere constants.
struct MapCfg {
  uint32_t T[MAX_SPH];      // d2 prefilter threshold: free if d2 > T = floor(((r + 1e-6) / res)^2)
  int32_t map_on[MAX_SPH];  // 0 if the sphere's link is excluded from the map check
  int32_t has_map;          // scene present
  uint32_t pT[MAX_PRIM];    // slab prefilter threshold of a primitive: floor(((rxy + 1e-6) / res)^2)
  int32_t p_map_on[MAX_PRIM];
};

}  // namespace smp
