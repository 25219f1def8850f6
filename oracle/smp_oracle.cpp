// ORACLE -- TEST INFRASTRUCTURE ONLY.
//
// Sequential CPU restatement of the BiRRT* C-space planner that squirrel_8dof_planner drives
// (tpatten/squirrel_motion_planner, birrt_star_algorithm).  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load this library, and only as the checker / the CPU baseline.  The
// product (squirrel_motion_planner_amd/) never links or calls it.
//
// Parity status: the reference cannot be built here (ROS, KDL, FCL, octomap, Eigen, boost all absent;
// SURVEY.md 8c) and ships no tests or golden vectors, so this restatement is "parity unpinned" against the
// original binaries.  Every decision the reference leaves unpinned is fixed here and in DESIGN.md:
//   RNG (Philox4x32-10 counters instead of the unseeded boost mt19937), portable sin/cos, the sphere
//   collision model, the informed-sampling rotation C, and the (cost,id) order of the near list.
//
// Abbreviations used in citations: BS = birrt_star_algorithm/src/birrt_star.cpp,
// CC = birrt_star_algorithm/include/birrt_star_algorithm/collision_checker.hpp,
// CL = kuka_motion_control/src/control_laws.cpp, DH = planning_heuristics/src/distance_heuristics.cpp,
// KM = kuka_motion_control/src/kdl_kuka_model.cpp.
//
// Build: oracle/Makefile (g++ -O3 -fno-fast-math -ffp-contract=off).

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace orc {

// ------------------------------------------------------------------------------------------ math
// Portable sin/cos (fdlibm kernels + Cody-Waite reduction).  Same definition as the product kernels so
// FK agrees bit for bit; glibc and ocml sin/cos may differ by an ulp (hard parts).
static inline void psincos(double x, double* s, double* c) {
  const double inv_pio2 = 6.36619772367581382433e-01;
  const double pio2_1 = 1.57079632673412561417e+00;
  const double pio2_2 = 6.07710050630396597660e-11;
  const double pio2_3 = 2.02226624871116645580e-21;
  double fn = std::floor(x * inv_pio2 + 0.5);
  double r = ((x - fn * pio2_1) - fn * pio2_2) - fn * pio2_3;
  long long n = (long long)fn;
  double z = r * r;
  double sr = r + (r * z) * (-1.66666666666666324348e-01 +
                 z * (8.33333333332248946124e-03 + z * (-1.98412698298579493134e-04 +
                 z * (2.75573137070700676789e-06 + z * (-2.50507602534068634195e-08 +
                 z * 1.58969099521155010221e-10)))));
  double cr = 1.0 - (0.5 * z - z * (z * (4.16666666666666019037e-02 +
                 z * (-1.38888888888741095749e-03 + z * (2.48015872894767294178e-05 +
                 z * (-2.75573143513906633035e-07 + z * (2.08757232129817482790e-09 +
                 z * -1.13596475577881948265e-11)))))));
  switch ((int)(n & 3)) {
    case 0: *s = sr; *c = cr; break;
    case 1: *s = cr; *c = -sr; break;
    case 2: *s = -sr; *c = -cr; break;
    default: *s = -cr; *c = sr; break;
  }
}

struct Frame {
  double R[9];
  double p[3];
};

static inline Frame fmul(const Frame& a, const Frame& b) {  // KDL Frame operator*
  Frame o;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      o.R[r * 3 + c] = a.R[r * 3 + 0] * b.R[0 * 3 + c] + a.R[r * 3 + 1] * b.R[1 * 3 + c] + a.R[r * 3 + 2] * b.R[2 * 3 + c];
  for (int r = 0; r < 3; ++r) {
    double m = a.R[r * 3 + 0] * b.p[0] + a.R[r * 3 + 1] * b.p[1] + a.R[r * 3 + 2] * b.p[2];
    o.p[r] = m + a.p[r];
  }
  return o;
}

static inline void rot2(const double* ax, double q, double* R) {  // KDL Rotation::Rot2
  double st, ct;
  psincos(q, &st, &ct);
  double vt = 1 - ct;
  double m_vt_0 = vt * ax[0], m_vt_1 = vt * ax[1], m_vt_2 = vt * ax[2];
  double m_st_0 = ax[0] * st, m_st_1 = ax[1] * st, m_st_2 = ax[2] * st;
  double m_vt_0_1 = m_vt_0 * ax[1], m_vt_0_2 = m_vt_0 * ax[2], m_vt_1_2 = m_vt_1 * ax[2];
  R[0] = ct + m_vt_0 * ax[0]; R[1] = -m_st_2 + m_vt_0_1; R[2] = m_st_1 + m_vt_0_2;
  R[3] = m_st_2 + m_vt_0_1;  R[4] = ct + m_vt_1 * ax[1]; R[5] = -m_st_0 + m_vt_1_2;
  R[6] = -m_st_1 + m_vt_0_2; R[7] = m_st_0 + m_vt_1_2;  R[8] = ct + m_vt_2 * ax[2];
}

// Philox4x32-10 (Salmon et al. 2011) -- counter-based so that every draw is addressable by
// (seed, query, iteration, attempt, joint); the reference RNG is unseeded (control_laws.h:368).
static inline void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
  }
}

static inline double u01(uint64_t seed, uint32_t query, uint32_t it, uint32_t outer, uint32_t inner, uint32_t idx) {
  uint32_t c[4] = {it, outer, inner, idx >> 1};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32) ^ query);
  uint32_t a = c[(idx & 1) * 2], b = c[(idx & 1) * 2 + 1];
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// ------------------------------------------------------------------------------------------ model
struct Robot {
  int n_links;
  std::vector<int> parent, joint, type;   // type: 0 fixed, 1 revolute, 2 prismatic
  std::vector<double> axis, origin, R, p; // per link
  int n_seg;
  std::vector<int> seg_joint, seg_type;
  std::vector<double> seg_axis, seg_origin, seg_R, seg_p;  // f_tip per segment
  int n_sph;
  std::vector<int> sph_link;
  std::vector<double> sph_c, sph_r;
  std::vector<int> lb_has;                 // per link: has bound
  std::vector<double> lb_c, lb_r;
  int n_pairs;
  std::vector<int> pair_a, pair_b;
  double q_min[8], q_max[8];
  int rev[8];
  double root_z;
  std::vector<std::vector<int>> link_sph;  // spheres of each link
  // rigid-body collapse (DESIGN.md "Kinematics"): body chain steps, sphere / bound centres in body frames
  int n_chain;
  std::vector<int> ch_type, ch_joint, ch_body;
  std::vector<double> ch_axis, ch_origin, ch_R, ch_p;
  int n_body;
  std::vector<int> sph_body, lb_body;
  std::vector<double> sph_cb, lb_cb;
  // exact upright primitives (URDF box / cylinder links on the planar base): type 1 box (half extents), 2 cylinder
  // (radius, half length); centre and x axis in the body frame
  struct Prim { int type, body, link; double cb[3], ab[3], h[3], rxy; };
  std::vector<Prim> prims;
  std::vector<int> link_prim;  // per link: its primitive, -1 for sphere links
};

struct Scene {
  int nx, ny, nz, wx;  // wx = 64-bit words per x-row
  double ox, oy, oz, res;
  std::vector<uint64_t> bits;
  std::vector<uint16_t> d2;
  std::vector<std::vector<uint16_t>> slab;  // per primitive: 2-D box-gap field of its z slab (oracle.py Oracle)
};

static inline bool occ(const Scene& s, int i, int j, int k) {
  return (s.bits[((size_t)k * s.ny + j) * s.wx + (i >> 6)] >> (i & 63)) & 1ull;
}

// Map test of one sphere against the occupied voxel boxes (DESIGN.md "Collision model").  d2 holds, per
// cell, the squared box-to-box gap (voxel units) to the nearest occupied cell -- a lower bound of the
// distance from any point of the cell to any occupied box -- so a sphere whose centre cell has
// d2 > floor(((r + 1e-6) / res)^2) is free; otherwise every voxel box in reach is tested exactly.
static inline bool sphere_hits_map(const Scene& s, const double* c, double r, uint32_t T) {
  double fx = std::floor((c[0] - s.ox) / s.res), fy = std::floor((c[1] - s.oy) / s.res), fz = std::floor((c[2] - s.oz) / s.res);
  if (!(fx >= 0 && fx < s.nx && fy >= 0 && fy < s.ny && fz >= 0 && fz < s.nz)) return false;
  int ci = (int)fx, cj = (int)fy, ck = (int)fz;
  if ((uint32_t)s.d2[((size_t)ck * s.ny + cj) * s.nx + ci] > T) return false;
  int i0 = (int)std::floor((c[0] - r - s.ox) / s.res) - 1, i1 = (int)std::floor((c[0] + r - s.ox) / s.res) + 1;
  int j0 = (int)std::floor((c[1] - r - s.oy) / s.res) - 1, j1 = (int)std::floor((c[1] + r - s.oy) / s.res) + 1;
  int k0 = (int)std::floor((c[2] - r - s.oz) / s.res) - 1, k1 = (int)std::floor((c[2] + r - s.oz) / s.res) + 1;
  i0 = std::max(i0, 0); j0 = std::max(j0, 0); k0 = std::max(k0, 0);
  i1 = std::min(i1, s.nx - 1); j1 = std::min(j1, s.ny - 1); k1 = std::min(k1, s.nz - 1);
  double r2 = r * r;
  for (int k = k0; k <= k1; ++k) {
    double zlo = s.oz + (double)k * s.res, zhi = s.oz + (double)(k + 1) * s.res;
    double dz = c[2] < zlo ? zlo - c[2] : (c[2] > zhi ? c[2] - zhi : 0.0);
    for (int j = j0; j <= j1; ++j) {
      double ylo = s.oy + (double)j * s.res, yhi = s.oy + (double)(j + 1) * s.res;
      double dy = c[1] < ylo ? ylo - c[1] : (c[1] > yhi ? c[1] - yhi : 0.0);
      for (int i = i0; i <= i1; ++i) {
        if (!occ(s, i, j, k)) continue;
        double xlo = s.ox + (double)i * s.res, xhi = s.ox + (double)(i + 1) * s.res;
        double dx = c[0] < xlo ? xlo - c[0] : (c[0] > xhi ? c[0] - xhi : 0.0);
        if (dx * dx + dy * dy + dz * dz <= r2) return true;
      }
    }
  }
  return false;
}

// ---- exact primitives (DESIGN.md "Collision model"): restated term by term from the product's spec (the same
// expressions, so both decide every case alike); the reference collides fcl::Box / fcl::Cylinder (CC:282-288).
// prim: centre pw[0..2], horizontal x axis (pw[3], pw[4]).
static inline bool prim_cell(int ty, const double* h, const double* pw, const Scene& s, int i, int j, int k) {
  const double zlo = s.oz + (double)k * s.res, zhi = s.oz + (double)(k + 1) * s.res;
  const double hz = ty == 1 ? h[2] : h[1];
  if (zhi < pw[2] - hz || zlo > pw[2] + hz) return false;
  const double xlo = s.ox + (double)i * s.res, xhi = s.ox + (double)(i + 1) * s.res;
  const double ylo = s.oy + (double)j * s.res, yhi = s.oy + (double)(j + 1) * s.res;
  if (ty == 2) {
    const double qx = pw[0] < xlo ? xlo - pw[0] : (pw[0] > xhi ? pw[0] - xhi : 0.0);
    const double qy = pw[1] < ylo ? ylo - pw[1] : (pw[1] > yhi ? pw[1] - yhi : 0.0);
    return qx * qx + qy * qy <= h[0] * h[0];
  }
  const double c = pw[3], sn = pw[4], ac = std::fabs(c), as = std::fabs(sn), hw = 0.5 * s.res;
  const double dx = 0.5 * (xlo + xhi) - pw[0], dy = 0.5 * (ylo + yhi) - pw[1];
  if (std::fabs(dx) > hw + (ac * h[0] + as * h[1])) return false;
  if (std::fabs(dy) > hw + (as * h[0] + ac * h[1])) return false;
  if (std::fabs(c * dx + sn * dy) > h[0] + hw * (ac + as)) return false;
  if (std::fabs(c * dy - sn * dx) > h[1] + hw * (ac + as)) return false;
  return true;
}

// Slab prefilter, then every occupied cell of the primitive's axis-aligned reach.
static inline bool prim_hits_map(const Scene& s, int p, int ty, const double* h, double rxy_T, const double* pw) {
  const double fx = std::floor((pw[0] - s.ox) / s.res), fy = std::floor((pw[1] - s.oy) / s.res);
  if (!(fx >= 0 && fx < s.nx && fy >= 0 && fy < s.ny)) return false;
  if ((uint32_t)s.slab[p][(size_t)(int)fy * s.nx + (int)fx] > (uint32_t)rxy_T) return false;
  const double ac = std::fabs(pw[3]), as = std::fabs(pw[4]);
  const double ex = ty == 1 ? ac * h[0] + as * h[1] : h[0];
  const double ey = ty == 1 ? as * h[0] + ac * h[1] : h[0];
  const double ez = ty == 1 ? h[2] : h[1];
  const double lo[3] = {pw[0] - ex, pw[1] - ey, pw[2] - ez}, hi[3] = {pw[0] + ex, pw[1] + ey, pw[2] + ez};
  const double o[3] = {s.ox, s.oy, s.oz};
  const int n[3] = {s.nx, s.ny, s.nz};
  int a[3], b[3];
  for (int d = 0; d < 3; ++d) {
    a[d] = std::max((int)std::floor((lo[d] - o[d]) / s.res) - 2, 0);
    b[d] = std::min((int)std::floor((hi[d] - o[d]) / s.res) + 2, n[d] - 1);
  }
  for (int k = a[2]; k <= b[2]; ++k)
    for (int j = a[1]; j <= b[1]; ++j)
      for (int i = a[0]; i <= b[0]; ++i)
        if (occ(s, i, j, k) && prim_cell(ty, h, pw, s, i, j, k)) return true;
  return false;
}

// Sphere (centre w, radius rs) vs primitive: squared distance to the solid box / cylinder against rs^2.
static inline bool sphere_prim(int ty, const double* h, const double* pw, const double* w, double rs) {
  const double dx = w[0] - pw[0], dy = w[1] - pw[1], dz = w[2] - pw[2];
  const double az = std::fabs(dz);
  if (ty == 1) {
    const double lx = std::fabs(pw[3] * dx + pw[4] * dy), ly = std::fabs(pw[3] * dy - pw[4] * dx);
    const double qx = lx > h[0] ? lx - h[0] : 0.0, qy = ly > h[1] ? ly - h[1] : 0.0, qz = az > h[2] ? az - h[2] : 0.0;
    return qx * qx + qy * qy + qz * qz <= rs * rs;
  }
  const double rho = std::sqrt(dx * dx + dy * dy);
  const double qr = rho > h[0] ? rho - h[0] : 0.0, qz = az > h[1] ? az - h[1] : 0.0;
  return qr * qr + qz * qz <= rs * rs;
}

static inline uint32_t sphere_threshold(double r, double res) {
  double a = (r + 1e-6) / res;
  return (uint32_t)std::floor(a * a);
}

// Tree FK of every link (CC:519-539): movable links use joint->pose(q) only, the rest their stored
// frame-to-tip (with the collision-origin adjust folded in); root at z = +0.02 (CC:201).
static void link_frames(const Robot& rb, const double* q, Frame* T) {
  for (int i = 0; i < rb.n_links; ++i) {
    if (rb.parent[i] < 0) {
      std::memset(&T[i], 0, sizeof(Frame));
      T[i].R[0] = T[i].R[4] = T[i].R[8] = 1.0;
      T[i].p[2] = rb.root_z;
      continue;
    }
    Frame L;
    if (rb.type[i] == 1) {
      rot2(&rb.axis[i * 3], q[rb.joint[i]], L.R);
      for (int d = 0; d < 3; ++d) L.p[d] = rb.origin[i * 3 + d];
    } else if (rb.type[i] == 2) {
      static const double I9[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
      std::memcpy(L.R, I9, sizeof(I9));
      double qq = q[rb.joint[i]];
      for (int d = 0; d < 3; ++d) L.p[d] = rb.origin[i * 3 + d] + rb.axis[i * 3 + d] * qq;
    } else {
      std::memcpy(L.R, &rb.R[i * 9], 9 * sizeof(double));
      std::memcpy(L.p, &rb.p[i * 3], 3 * sizeof(double));
    }
    T[i] = fmul(T[rb.parent[i]], L);
  }
}

// Body frames: the tree recursion restricted to the path base_link_origin -> arm_link5 (CC:519-539).
static void body_frames(const Robot& rb, const double* q, Frame* B) {
  Frame T;
  std::memset(&T, 0, sizeof(T));
  T.R[0] = T.R[4] = T.R[8] = 1.0;
  T.p[2] = rb.root_z;
  for (int k = 0; k < rb.n_chain; ++k) {
    Frame L;
    if (rb.ch_type[k] == 1) {
      rot2(&rb.ch_axis[k * 3], q[rb.ch_joint[k]], L.R);
      for (int d = 0; d < 3; ++d) L.p[d] = rb.ch_origin[k * 3 + d];
    } else if (rb.ch_type[k] == 2) {
      static const double I9[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
      std::memcpy(L.R, I9, sizeof(I9));
      double qq = q[rb.ch_joint[k]];
      for (int d = 0; d < 3; ++d) L.p[d] = rb.ch_origin[k * 3 + d] + rb.ch_axis[k * 3 + d] * qq;
    } else {
      std::memcpy(L.R, &rb.ch_R[k * 9], 9 * sizeof(double));
      std::memcpy(L.p, &rb.ch_p[k * 3], 3 * sizeof(double));
    }
    T = fmul(T, L);
    if (rb.ch_body[k] >= 0) B[rb.ch_body[k]] = T;
  }
}

static inline void xform(const Frame& F, const double* c, double* o) {  // KDL Frame * Vector
  for (int r = 0; r < 3; ++r) {
    double m = F.R[r * 3 + 0] * c[0] + F.R[r * 3 + 1] * c[1] + F.R[r * 3 + 2] * c[2];
    o[r] = m + F.p[r];
  }
}

// Chain FK (KM:278-305, KDL ChainFkSolverPos_recursive): p_out = I; p_out = p_out * (joint.pose(q) * f_tip).
static double ee_z(const Robot& rb, const double* q) {
  Frame P;
  std::memset(&P, 0, sizeof(P));
  P.R[0] = P.R[4] = P.R[8] = 1.0;
  for (int s = 0; s < rb.n_seg; ++s) {
    Frame J;
    std::memset(&J, 0, sizeof(J));
    if (rb.seg_type[s] == 1) {
      rot2(&rb.seg_axis[s * 3], q[rb.seg_joint[s]], J.R);
      for (int d = 0; d < 3; ++d) J.p[d] = rb.seg_origin[s * 3 + d];
    } else if (rb.seg_type[s] == 2) {
      J.R[0] = J.R[4] = J.R[8] = 1.0;
      double qq = q[rb.seg_joint[s]];
      for (int d = 0; d < 3; ++d) J.p[d] = rb.seg_origin[s * 3 + d] + rb.seg_axis[s * 3 + d] * qq;
    } else {
      J.R[0] = J.R[4] = J.R[8] = 1.0;
    }
    Frame F;
    std::memcpy(F.R, &rb.seg_R[s * 9], 9 * sizeof(double));
    std::memcpy(F.p, &rb.seg_p[s * 3], 3 * sizeof(double));
    P = fmul(P, fmul(J, F));
  }
  return P.p[2];
}

struct Checker {
  const Robot* rb;
  const Scene* sc;
  std::vector<uint32_t> T;          // per-sphere map threshold
  std::vector<uint8_t> map_enabled; // per link (setDisabledLinkMapCollisions, CC:90-102)
  std::vector<Frame> frames;
  std::vector<double> wc;           // world sphere centres
  std::vector<uint32_t> pT;         // per-primitive slab threshold
  std::vector<double> pw;           // world primitive centres + x axes (5 per primitive)
  long long calls = 0;

  void init(const Robot* r, const Scene* s) {
    rb = r; sc = s;
    T.resize(r->n_sph);
    for (int i = 0; i < r->n_sph; ++i) T[i] = s ? sphere_threshold(r->sph_r[i], s->res) : 0;
    pT.resize(r->prims.size());
    for (size_t i = 0; i < r->prims.size(); ++i) pT[i] = s ? sphere_threshold(r->prims[i].rxy, s->res) : 0;
    pw.resize(5 * r->prims.size());
    map_enabled.assign(r->n_links, 1);
    frames.resize(r->n_body > r->n_links ? r->n_body : r->n_links);
    wc.resize(r->n_sph * 3);
  }

  // CollisionChecker::isInCollision (CC:104-121): map first, then self.
  bool in_collision(const double* q, bool self, bool map) {
    ++calls;
    if (!self && !map) return false;
    body_frames(*rb, q, frames.data());
    for (int i = 0; i < rb->n_sph; ++i) xform(frames[rb->sph_body[i]], &rb->sph_cb[i * 3], &wc[i * 3]);
    prim_frames();
    if (map && sc) {
      for (int i = 0; i < rb->n_sph; ++i)
        if (map_enabled[rb->sph_link[i]] && sphere_hits_map(*sc, &wc[i * 3], rb->sph_r[i], T[i])) return true;
      for (size_t p = 0; p < rb->prims.size(); ++p)
        if (map_enabled[rb->prims[p].link] && prim_map(p)) return true;
    }
    if (self) {
      for (int pi = 0; pi < rb->n_pairs; ++pi) {
        int a = rb->pair_a[pi], b = rb->pair_b[pi];
        if (rb->link_prim[a] >= 0 || rb->link_prim[b] >= 0) {
          if (pair_prim(a, b)) return true;
          continue;
        }
        double ca[3], cb[3];  // link bounding-sphere prefilter
        xform(frames[rb->lb_body[a]], &rb->lb_cb[a * 3], ca);
        xform(frames[rb->lb_body[b]], &rb->lb_cb[b * 3], cb);
        double dx = ca[0] - cb[0], dy = ca[1] - cb[1], dz = ca[2] - cb[2];
        double rr = rb->lb_r[a] + rb->lb_r[b];
        if (dx * dx + dy * dy + dz * dz > rr * rr) continue;
        for (int sa : rb->link_sph[a])
          for (int sb : rb->link_sph[b]) {
            double ex = wc[sa * 3] - wc[sb * 3], ey = wc[sa * 3 + 1] - wc[sb * 3 + 1], ez = wc[sa * 3 + 2] - wc[sb * 3 + 2];
            double r2 = rb->sph_r[sa] + rb->sph_r[sb];
            if (ex * ex + ey * ey + ez * ez <= r2 * r2) return true;
          }
      }
    }
    return false;
  }

  // world centre and x axis of every primitive (the sphere centres' KDL Frame * Vector; the axis without translation)
  void prim_frames() {
    for (size_t p = 0; p < rb->prims.size(); ++p) {
      const Robot::Prim& P = rb->prims[p];
      const Frame& B = frames[P.body];
      xform(B, P.cb, &pw[p * 5]);
      pw[p * 5 + 3] = B.R[0] * P.ab[0] + B.R[1] * P.ab[1] + B.R[2] * P.ab[2];
      pw[p * 5 + 4] = B.R[3] * P.ab[0] + B.R[4] * P.ab[1] + B.R[5] * P.ab[2];
    }
  }
  bool prim_map(size_t p) const {
    const Robot::Prim& P = rb->prims[p];
    return prim_hits_map(*sc, (int)p, P.type, P.h, pT[p], &pw[p * 5]);
  }
  // a primitive link against a sphere link: any sphere of it touching the primitive
  bool pair_prim(int a, int b) const {
    const int p = rb->link_prim[a] >= 0 ? rb->link_prim[a] : rb->link_prim[b], sl = rb->link_prim[a] >= 0 ? b : a;
    const Robot::Prim& P = rb->prims[p];
    for (int s : rb->link_sph[sl])
      if (sphere_prim(P.type, P.h, &pw[p * 5], &wc[s * 3], rb->sph_r[s])) return true;
    return false;
  }
};

// ------------------------------------------------------------------------------------------ planner
using Conf = std::array<double, 8>;

struct Costs { double total = 0, rev = 0, prism = 0; };

struct Edge {                 // DS:11-19 (ee trajectory dropped: output-only in C-space)
  int root_node_id = 0, child_node_id = 0;
  std::vector<Conf> traj;     // 21 interpolated configs (BS:4443-4526)
  Conf s{}, g{};              // interpolation start / target (export for orc_resume_*; the GPU's in-edge)
};

struct Node {                 // DS:29-45
  int node_id = 0, parent_id = 0;
  Conf q{};
  Costs cost;
  std::vector<Edge> out;      // outgoing edges
};

struct Tree {
  bool is_start;
  std::vector<Node> nodes;
  int num_nodes = 0, num_edges = 0, num_rewire = 0;
};

struct Params {
  double near_r = 4.0;         // BS:183 compiled default (squirrel_effective)
  double step = 0.5;           // BS:189
  int n_pts = 20;              // BS:186
  int max_near = 20;           // BS:195
  double opt_thresh = 1.0;     // BS:201
  int tree_opt = 1, informed = 1;
  double env_x[2] = {0, 0}, env_y[2] = {0, 0};
  int self = 1, map = 1;
  uint64_t seed = 1;
  uint32_t query = 0;
  int max_iter = 1000;
  double max_time = 0;         // >0: time budget instead of iterations (flag_iter_or_time = 1)
  long long max_checked = 0;   // >0: budget of collision-checked configurations instead of iterations
  int threads = 1;             // >1: the two scans run as OpenMP loops on this many threads (BS:4092, BS:4283)
};

struct Stats {
  long long iterations = 0, first_iter = -1, last_iter = -1;
  long long checked = 0, valid = 0;  // configs collision-checked (reference semantics) / found free
  double t_first = -1, t_total = 0;
};

struct Planner {
  const Robot* rb;
  Checker* ck;
  Params P;
  Tree ta, tb;  // start / goal
  Conf qs, qg;
  Costs h0;     // cost_h of the roots (BS:382, 396-398)
  double cbest = 10000.0, cbest_rev = 10000.0, cbest_prism = 10000.0;
  bool have_sol = false;
  bool conn_start = false;  // m_connected_tree_name == "START"
  Node nB, nA;              // m_node_tree_B / m_node_tree_A (copies, BS:3254-3255)
  double Crev[36], Cpr[4], ctr_rev[6], ctr_pr[2];
  long long iter = 0;
  Stats st;
  std::vector<std::array<double, 5>> cost_rows;  // BS:1325-1331 (time column = 0 for determinism)
  std::vector<double> cost_row_time;              // the rows' wall-clock seconds from the planning start (reports)
  std::chrono::steady_clock::time_point t0;

  double dist(const Conf& a, const Conf& b) const {  // DH:128-156
    double s = 0.0;
    for (int i = 0; i < 8; ++i) { double d = b[i] - a[i]; s += d * d; }
    return std::sqrt(s);
  }

  // isEdgeValid (BS:6878-6895): stops at the first colliding config; counts checked / free configs.
  bool edge_valid(const Edge& e, int* last_valid) {
    int lv = 0;
    for (size_t i = 0; i < e.traj.size(); ++i) {
      ++st.checked;
      if (ck->in_collision(e.traj[i].data(), P.self, P.map)) { if (last_valid) *last_valid = lv; return false; }
      ++st.valid;
      lv = (int)i;
    }
    if (last_valid) *last_valid = lv;
    return true;
  }

  // connectNodesInterpolation + interpolateConfigurations + compute_edge_cost_interpolation
  // (BS:4380-4440, 4443-4526, 4162-4242)
  void connect_nodes(Tree& t, const Node& near, const Node& end, Node& xn, Edge& e) {
    double step[8];
    for (int j = 0; j < 8; ++j) step[j] = (end.q[j] - near.q[j]) / double(P.n_pts);
    e.traj.resize(P.n_pts + 1);
    for (int inc = 0; inc <= P.n_pts; ++inc)
      for (int j = 0; j < 8; ++j) e.traj[inc][j] = near.q[j] + inc * step[j];
    e.s = near.q;
    e.g = end.q;
    double ct = 0, cr = 0, cp = 0;
    for (int wp = 0; wp < P.n_pts; ++wp) {
      double st_ = 0, sr = 0, sp = 0;
      for (int j = 0; j < 8; ++j) {
        double d = (e.traj[wp + 1][j] - e.traj[wp][j]) * (e.traj[wp + 1][j] - e.traj[wp][j]);
        st_ += d * 1.0;
        if (rb->rev[j]) sr += d; else sp += d;
      }
      ct += std::sqrt(st_); cr += std::sqrt(sr); cp += std::sqrt(sp);
    }
    xn.node_id = end.node_id;
    xn.parent_id = near.node_id;
    e.root_node_id = near.node_id;
    e.child_node_id = xn.node_id;
    xn.cost.total = near.cost.total + ct;
    xn.cost.rev = near.cost.rev + cr;
    xn.cost.prism = near.cost.prism + cp;
    xn.q = e.traj[P.n_pts];
    xn.out.clear();
    (void)t;
  }

  // stepTowardsRandSample (BS:5712-5868)
  bool step_towards(const Node& nn, Node& x, double f) {
    double ed[8], srev = 0, spr = 0;
    for (int j = 0; j < 8; ++j) {
      ed[j] = x.q[j] - nn.q[j];
      double d = ed[j] * ed[j];
      if (rb->rev[j]) srev += d; else spr += d;
    }
    double lrev = std::sqrt(srev), lpr = std::sqrt(spr);
    bool rev_done = lrev < 0.001, pr_done = lpr < 0.001;
    double ext[8] = {0};
    srev = 0; spr = 0;
    for (int j = 0; j < 8; ++j) {
      if (!rb->rev[j]) {
        if (!pr_done) { ed[j] = ed[j] / lpr; double c = f * ed[j]; ext[j] = nn.q[j] + c; spr += c * c; }
      } else {
        if (!rev_done) { ed[j] = ed[j] / lrev; double c = f * ed[j]; ext[j] = nn.q[j] + c; srev += c * c; }
      }
    }
    double elp = spr == 0.0 ? 1000.0 : std::sqrt(spr);
    double elr = srev == 0.0 ? 1000.0 : std::sqrt(srev);
    bool reached = true;
    if (elr < lrev) { for (int j = 0; j < 8; ++j) if (rb->rev[j]) x.q[j] = ext[j]; reached = false; }
    if (elp < lpr) { for (int j = 0; j < 8; ++j) if (!rb->rev[j]) x.q[j] = ext[j]; reached = false; }
    return reached;
  }

  // insertNode (BS:3298-3322)
  void insert(Tree& t, const Edge& e, const Node& x) {
    t.nodes[x.parent_id].out.push_back(e);
    t.nodes.push_back(x);
    t.nodes.back().out.clear();
    t.num_nodes++;
    t.num_edges++;
  }

  // find_nearest_neighbour_interpolation (BS:4076-4133): first strict minimum, min initialised to 10000.
  int nearest(const Tree& t, const Conf& q) const {
    int id = 0;
    double mn = 10000.0;
#ifdef _OPENMP
    if (P.threads > 1) {
      // the reference's parallel scan (BS:4092-4130: omp parallel for, critical(closervertex)), with the tie the
      // sequential loop takes: the lowest index among equal minima
      const long long nn = (long long)t.nodes.size();
#pragma omp parallel num_threads(P.threads)
      {
        int lid = 0;
        double lmn = 10000.0;
#pragma omp for schedule(static) nowait
        for (long long n = 0; n < nn; ++n) {
          double d = dist(t.nodes[n].q, q);
          if (d < lmn) { lid = t.nodes[n].node_id; lmn = d; }
        }
#pragma omp critical(closervertex)
        if (lmn < mn || (lmn == mn && lmn < 10000.0 && lid < id)) { mn = lmn; id = lid; }
      }
      return id;
    }
#endif
    for (size_t n = 0; n < t.nodes.size(); ++n) {
      double d = dist(t.nodes[n].q, q);
      if (d < mn) { id = t.nodes[n].node_id; mn = d; }
    }
    return id;
  }

  // find_near_vertices_interpolation (BS:4272-4324); order = ascending (cost, id).
  std::vector<int> near_set(const Tree& t, const Node& x) const {
    std::vector<std::pair<double, int>> v;
#ifdef _OPENMP
    if (P.threads > 1) {
      // BS:4283-4302: omp parallel for, critical(nodeinsertion); the (cost, id) sort makes the order schedule-free
      const long long nn = (long long)t.nodes.size();
#pragma omp parallel num_threads(P.threads)
      {
        std::vector<std::pair<double, int>> lv;
#pragma omp for schedule(static) nowait
        for (long long n = 0; n < nn; ++n) {
          double d = dist(t.nodes[n].q, x.q);
          if (d < P.near_r && x.node_id != t.nodes[n].node_id) lv.push_back({t.nodes[n].cost.total, t.nodes[n].node_id});
        }
#pragma omp critical(nodeinsertion)
        v.insert(v.end(), lv.begin(), lv.end());
      }
    } else
#endif
    for (size_t n = 0; n < t.nodes.size(); ++n) {
      double d = dist(t.nodes[n].q, x.q);
      if (d < P.near_r && x.node_id != t.nodes[n].node_id) v.push_back({t.nodes[n].cost.total, t.nodes[n].node_id});
    }
    std::sort(v.begin(), v.end());
    std::vector<int> ids(v.size());
    for (size_t i = 0; i < v.size(); ++i) ids[i] = v[i].second;
    return ids;
  }

  // --- sampling (CL:1120-1188, BS:3832-3878, BS:3607-3829)
  void rand_conf(uint32_t outer, uint32_t& inner, Conf& q) {
    bool env0 = P.env_x[0] == 0.0 && P.env_x[1] == 0.0 && P.env_y[0] == 0.0 && P.env_y[1] == 0.0;
    for (;; ++inner) {
      for (int j = 0; j < 8; ++j) {
        double lo = rb->q_min[j], hi = rb->q_max[j];
        if (!env0 && j == 0) { lo = P.env_x[0]; hi = P.env_x[1]; }
        if (!env0 && j == 1) { lo = P.env_y[0]; hi = P.env_y[1]; }
        double u = u01(P.seed, P.query, (uint32_t)iter, outer, inner, j);
        q[j] = u * (hi - lo) + lo;
      }
      if (0.0 <= ee_z(*rb, q.data())) return;
    }
  }

  void sample_uniform(Conf& q) {
    uint32_t inner = 0;
    rand_conf(0, inner, q);
  }

  void ellipse_init() {  // jointConfigEllipseInitialization (BS:3472-3604) with the C of DESIGN.md
    double arev[6], apr[2];
    int ir = 0, ip = 0;
    for (int j = 0; j < 8; ++j) {
      if (rb->rev[j]) { ctr_rev[ir] = (qs[j] + qg[j]) / 2.0; arev[ir++] = (qg[j] - qs[j]) / h0.rev; }
      else { ctr_pr[ip] = (qs[j] + qg[j]) / 2.0; apr[ip++] = (qg[j] - qs[j]) / h0.prism; }
    }
    householder_C(arev, 6, Crev);
    householder_C(apr, 2, Cpr);
  }

  // C = H * diag(1,..,1,det H), H = I - 2 v v^T / (v^T v), v = e1 - a (a non-finite -> a = e1).
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

  void sample_ellipse(Conf& out) {
    bool env0 = P.env_x[0] == 0.0 && P.env_x[1] == 0.0 && P.env_y[0] == 0.0 && P.env_y[1] == 0.0;
    for (uint32_t b = 0;; ++b) {
      Conf q;
      uint32_t inner = 0;
      rand_conf(1 + b, inner, q);
      double br[6], bp[2], sr = 0, sp = 0;
      int ir = 0, ip = 0;
      for (int j = 0; j < 8; ++j) { if (rb->rev[j]) br[ir++] = q[j]; else bp[ip++] = q[j]; }
      for (int i = 0; i < 6; ++i) sr += br[i] * br[i];
      for (int i = 0; i < 2; ++i) sp += bp[i] * bp[i];
      double nr = std::sqrt(sr), np = std::sqrt(sp);
      double ps = u01(P.seed, P.query, (uint32_t)iter, 1 + b, 0, 8);
      double lr[6], lp[2];
      for (int i = 0; i < 6; ++i) br[i] = ps * (br[i] / nr);
      for (int i = 0; i < 2; ++i) bp[i] = ps * (bp[i] / np);
      double srev = std::sqrt(cbest_rev * cbest_rev - h0.rev * h0.rev) / 2.0;
      double spr = std::sqrt(cbest_prism * cbest_prism - h0.prism * h0.prism) / 2.0;
      for (int i = 0; i < 6; ++i) lr[i] = i == 0 ? cbest_rev / 2.0 : srev;
      for (int i = 0; i < 2; ++i) lp[i] = i == 0 ? cbest_prism / 2.0 : spr;
      double rr[6], rp[2];
      for (int i = 0; i < 6; ++i) {
        double s = 0.0;
        for (int k = 0; k < 6; ++k) s += (Crev[i * 6 + k] * lr[k]) * br[k];
        rr[i] = s + ctr_rev[i];
      }
      for (int i = 0; i < 2; ++i) {
        double s = 0.0;
        for (int k = 0; k < 2; ++k) s += (Cpr[i * 2 + k] * lp[k]) * bp[k];
        rp[i] = s + ctr_pr[i];
      }
      Conf r;
      ir = 0; ip = 0;
      for (int j = 0; j < 8; ++j) r[j] = rb->rev[j] ? rr[ir++] : rp[ip++];
      bool above = 0.0 <= ee_z(*rb, r.data());
      bool inside = (r[0] < P.env_x[1] && r[0] > P.env_x[0] && r[1] < P.env_y[1] && r[1] > P.env_y[0]) || env0;
      if (above && inside) { out = r; return; }
      if (b > 100000000u) { out = r; return; }  // unreachable guard
    }
  }

  // ----------------------------------------------------------------------------------------------
  // expandTree, unconstrained single-step branch (BS:2221-2256)
  bool expand(Tree& t, const Node& nn, const Node& xr, Node& xn, Edge& en) {
    Node ext;
    ext.q = xr.q;
    step_towards(nn, ext, P.step);
    connect_nodes(t, nn, ext, xn, en);
    bool ok = edge_valid(en, nullptr);
    if (ok) {
      xn.node_id = t.num_nodes;
      en.child_node_id = xn.node_id;
    } else {
      xn = xr;
    }
    return ok;
  }

  // choose_node_parent_interpolation, unconstrained (BS:4594-4738, 4916-4935)
  bool choose_parent(Tree& t, const std::vector<int>& nv, const Node& nn, Edge& en, Node& xn) {
    if (nv.empty()) return false;
    bool found = false;
    std::vector<Node> vn;
    std::vector<Edge> ve;
    xn.parent_id = nn.node_id;
    for (size_t i = 0; i < nv.size(); ++i) {
      if ((int)i == P.max_near) break;
      if (t.nodes[nv[i]].cost.total < xn.cost.total) {
        Node g;
        Edge ge;
        connect_nodes(t, t.nodes[nv[i]], xn, g, ge);
        if (g.cost.total <= xn.cost.total) {
          if (edge_valid(ge, nullptr)) {
            found = true;
            int nn_t = t.num_nodes;
            Node cur = t.nodes[nv[i]];
            bool reached = false;
            while (!reached) {
              Node ox = xn;
              reached = step_towards(cur, ox, P.step);
              connect_nodes(t, cur, ox, g, ge);
              if (!reached) {
                g.node_id = nn_t++;
                g.parent_id = cur.node_id;
                ge.child_node_id = g.node_id;
                vn.push_back(g);
                ve.push_back(ge);
                cur = g;
              } else {
                xn.node_id = nn_t;
                xn.parent_id = cur.node_id;
                xn.q = g.q;
                xn.cost = g.cost;
                en = ge;
                en.child_node_id = xn.node_id;
              }
            }
            break;
          }
        }
      } else {
        break;
      }
    }
    if (found)
      for (size_t i = 0; i < vn.size(); ++i) insert(t, ve[i], vn[i]);
    return found;
  }

  // recursiveNodeCostUpdate (BS:5495-5606)
  void cost_update(Tree& t, int id, const Costs& red) {
    Node& nd = t.nodes[id];
    Costs old = nd.cost;
    nd.cost.total = old.total + red.total;
    nd.cost.rev = old.rev + red.rev;
    nd.cost.prism = old.prism + red.prism;
    if (have_sol) {
      bool connected = (t.is_start == conn_start);
      if (id == nB.node_id && connected) {
        cbest = cbest + red.total; cbest_rev = cbest_rev + red.rev; cbest_prism = cbest_prism + red.prism;
        nB.cost = nd.cost;
        st.last_iter = iter;
      }
      if (id == nA.node_id && !connected) {
        cbest = cbest + red.total; cbest_rev = cbest_rev + red.rev; cbest_prism = cbest_prism + red.prism;
        nA.cost = nd.cost;
        st.last_iter = iter;
      }
    }
    std::vector<int> kids;
    for (const Edge& e : t.nodes[id].out) kids.push_back(e.child_node_id);
    for (int c : kids) cost_update(t, c, red);
  }

  // rewireTreeInterpolation, unconstrained (BS:5056-5230)
  void rewire(Tree& t, const std::vector<int>& nv, const Node& xn) {
    int n = (int)nv.size();
    if (n == 0) return;
    int lower = n >= P.max_near ? n - P.max_near : 0;
    int cnt = 0;
    for (int k = n - 1; k >= lower; --k)
      if (xn.cost.total < t.nodes[nv[k]].cost.total) cnt++;
    for (int k = n - 1; k >= n - cnt; --k) {
      int v = nv[k];
      if (v != xn.parent_id && t.nodes[v].parent_id != 0) {
        Node g;
        Edge ge;
        connect_nodes(t, xn, t.nodes[v], g, ge);
        if (g.cost.total < t.nodes[v].cost.total) {
          if (edge_valid(ge, nullptr)) {
            Costs red;
            red.total = g.cost.total - t.nodes[v].cost.total;
            red.rev = g.cost.rev - t.nodes[v].cost.rev;
            red.prism = g.cost.prism - t.nodes[v].cost.prism;
            Node& par = t.nodes[t.nodes[v].parent_id];
            int ei = -1;
            for (size_t e = 0; e < par.out.size(); ++e)
              if (par.out[e].child_node_id == t.nodes[v].node_id) { ei = (int)e; t.num_edges--; break; }
            if (ei >= 0) par.out.erase(par.out.begin() + ei);
            t.nodes[v].parent_id = xn.node_id;
            if (have_sol) {
              bool connected = (t.is_start == conn_start);
              if (t.nodes[v].node_id == nB.node_id && connected) nB.parent_id = xn.node_id;
              else if (t.nodes[v].node_id == nA.node_id && !connected) nA.parent_id = xn.node_id;
            }
            t.nodes[v].q = g.q;
            t.nodes[xn.node_id].out.push_back(ge);
            cost_update(t, v, red);
            t.num_edges++;
            t.num_rewire++;
          }
        }
      }
    }
  }

  // connectGraphsInterpolation, unconstrained branch + commit (BS:2608-3046, 3219-3288).
  // `t` is tree_B (x_connect's tree); x_new belongs to the other tree.
  void connect_graphs(Tree& t, Node xc, const Node& xnew) {
    bool tree_expand = false;
    double best_nv_sol = 10000.0;
    Node sel;
    Edge sel_e;
    std::vector<Node> vn;
    std::vector<Edge> ve;
    double csp[3] = {cbest, cbest_rev, cbest_prism};
    Node g;
    Edge ge;
    connect_nodes(t, xc, xnew, g, ge);
    double sol[3] = {g.cost.total + xnew.cost.total, g.cost.rev + xnew.cost.rev, g.cost.prism + xnew.cost.prism};
    if (sol[0] < csp[0]) {
      int lv = 0;
      if (edge_valid(ge, &lv)) {
        csp[0] = sol[0]; csp[1] = sol[1]; csp[2] = sol[2];
        int nn_t = t.num_nodes;
        bool reached = false;
        while (!reached) {
          Node ox = xnew;
          reached = step_towards(xc, ox, P.step);
          connect_nodes(t, xc, ox, g, ge);
          if (!reached) {
            g.node_id = nn_t++;
            g.parent_id = xc.node_id;
            ge.child_node_id = g.node_id;
            vn.push_back(g); ve.push_back(ge);
            xc = g;
          } else {
            sel = g; sel.node_id = nn_t; sel.parent_id = xc.node_id;
            sel_e = ge; sel_e.child_node_id = sel.node_id;
            tree_expand = false;
          }
        }
      } else if (lv != 0) {
        Node ext;
        ext.q = ge.traj[lv];
        int nn_t = t.num_nodes;
        bool reached = false;
        Node en;
        Edge ee;
        while (!reached) {
          Node oe = ext;
          reached = step_towards(xc, oe, P.step);
          connect_nodes(t, xc, oe, en, ee);
          if (!reached) {
            en.node_id = nn_t++;
            en.parent_id = xc.node_id;
            ee.child_node_id = en.node_id;
            vn.push_back(en); ve.push_back(ee);
            xc = en;
          } else {
            sel = en; sel.node_id = nn_t; sel.parent_id = xc.node_id;
            sel_e = ee; sel_e.child_node_id = sel.node_id;
            tree_expand = true;
            best_nv_sol = sol[0];
          }
        }
      }
    }
    if (have_sol) {
      std::vector<int> nv = near_set(t, xnew);
      for (size_t i = 0; i < nv.size(); ++i) {
        if ((int)i == P.max_near) break;
        if (t.nodes[nv[i]].cost.total < xnew.cost.total) {
          Node en;
          Edge ee;
          connect_nodes(t, t.nodes[nv[i]], xnew, en, ee);
          sol[0] = en.cost.total + xnew.cost.total;
          sol[1] = en.cost.rev + xnew.cost.rev;
          sol[2] = en.cost.prism + xnew.cost.prism;
          if (sol[0] < csp[0]) {
            int lv = 0;
            if (edge_valid(ee, &lv)) {
              csp[0] = sol[0]; csp[1] = sol[1]; csp[2] = sol[2];
              vn.clear(); ve.clear();
              int nn_t = t.num_nodes;
              Node cur = t.nodes[nv[i]];
              bool reached = false;
              while (!reached) {
                Node ox = xnew;
                reached = step_towards(cur, ox, P.step);
                connect_nodes(t, cur, ox, en, ee);
                if (!reached) {
                  en.node_id = nn_t++;
                  en.parent_id = cur.node_id;
                  ee.child_node_id = en.node_id;
                  vn.push_back(en); ve.push_back(ee);
                  cur = en;
                } else {
                  sel = en; sel.node_id = nn_t; sel.parent_id = cur.node_id;
                  sel_e = ee; sel_e.child_node_id = sel.node_id;
                  tree_expand = false;
                }
              }
              break;
            } else {
              if (csp[0] == cbest && sol[0] < best_nv_sol) {
                if (lv != 0) {
                  Node ext;
                  ext.q = ee.traj[lv];
                  vn.clear(); ve.clear();
                  int nn_t = t.num_nodes;
                  Node cur = t.nodes[nv[i]];
                  bool reached = false;
                  while (!reached) {
                    Node oe = ext;
                    reached = step_towards(cur, oe, P.step);
                    connect_nodes(t, cur, oe, en, ee);
                    if (!reached) {
                      en.node_id = nn_t++;
                      en.parent_id = cur.node_id;
                      ee.child_node_id = en.node_id;
                      vn.push_back(en); ve.push_back(ee);
                      cur = en;
                    } else {
                      sel = en; sel.node_id = nn_t; sel.parent_id = cur.node_id;
                      sel_e = ee; sel_e.child_node_id = sel.node_id;
                      tree_expand = true;
                      best_nv_sol = sol[0];
                    }
                  }
                }
              }
            }
          }
        }
      }
    }
    for (size_t i = 0; i < vn.size(); ++i) insert(t, ve[i], vn[i]);
    if (csp[0] < cbest) {
      if (!have_sol) {
        st.first_iter = iter;
        st.t_first = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      }
      have_sol = true;
      insert(t, sel_e, sel);
      conn_start = t.is_start;
      nB = sel;
      nA = xnew;
      cbest = csp[0]; cbest_rev = csp[1]; cbest_prism = csp[2];
      st.last_iter = iter;
    } else if (tree_expand) {
      insert(t, sel_e, sel);
    }
  }

  // init_planner (BS:335-536) -- returns 0, or -2 / -3 for an invalid start / goal.
  int init(const Conf& s, const Conf& g) {
    qs = s; qg = g;
    if (ck->in_collision(s.data(), P.self, P.map)) return -2;
    if (ck->in_collision(g.data(), P.self, P.map)) return -3;
    double a = 0, r = 0, p = 0;  // DH:160-217
    for (int j = 0; j < 8; ++j) {
      double d = g[j] - s[j];
      a += d * d;
      if (rb->rev[j]) r += d * d; else p += d * d;
    }
    h0.total = std::sqrt(a); h0.rev = std::sqrt(r); h0.prism = std::sqrt(p);
    ta = Tree(); tb = Tree();
    ta.is_start = true; tb.is_start = false;
    Node gn; gn.q = g; tb.nodes.push_back(gn); tb.num_nodes = 1;
    Node sn; sn.q = s; ta.nodes.push_back(sn); ta.num_nodes = 1;
    ellipse_init();
    return 0;
  }

  // run_planner C-space branch (BS:983-1407), iteration budget (flag_iter_or_time = 0) or time budget.
  bool run() {
    t0 = std::chrono::steady_clock::now();
    Tree* A = &ta;
    Tree* B = &tb;
    iter = 0;
    connect_graphs(*A, A->nodes[0], B->nodes[0]);
    if (have_sol) {
      st.iterations = iter;
      st.t_total = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      return have_sol;
    }
    return loop(A, B);
  }

  // The same loop continued from a state set from outside (orc_resume_*: another run's trees and loop scalars after
  // `iter` iterations, tree_A of the next iteration `a_is_goal`); timed from here.
  bool resume(bool a_is_goal) {
    t0 = std::chrono::steady_clock::now();
    return a_is_goal ? loop(&tb, &ta) : loop(&ta, &tb);
  }

  bool loop(Tree* A, Tree* B) {
    for (;;) {
      double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (P.max_checked > 0) {
        if (!(st.checked < P.max_checked)) break;
      } else if (P.max_time > 0 ? !(el < P.max_time) : !(iter < P.max_iter)) {
        break;
      }
      Node xr;
      if (P.informed && have_sol) sample_ellipse(xr.q); else sample_uniform(xr.q);
      xr.node_id = (int)A->nodes.size();
      xr.cost.total = 0; xr.cost.rev = 0; xr.cost.prism = 0;
      Node nn = A->nodes[nearest(*A, xr.q)];
      Node xn;
      Edge en;
      bool ext_nn = expand(*A, nn, xr, xn, en);
      if (!ext_nn) xn.cost.total = 10000.0;
      std::vector<int> nv;
      bool ext_bp = false;
      if (P.tree_opt && have_sol) {
        nv = near_set(*A, xn);
        ext_bp = choose_parent(*A, nv, nn, en, xn);
      }
      if (ext_nn || ext_bp) {
        insert(*A, en, xn);
        if (P.tree_opt && have_sol) rewire(*A, nv, xn);
        Node xc = B->nodes[nearest(*B, xn.q)];
        connect_graphs(*B, xc, xn);
      }
      std::swap(A, B);
      iter++;
      cost_rows.push_back({(double)iter, 0.0, cbest, cbest_rev, cbest_prism});
      cost_row_time.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
      if ((cbest - h0.total) < P.opt_thresh) break;  // BS:1333-1338 (start root cost_h.total = h0.total)
    }
    st.iterations = iter;
    st.t_total = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return have_sol;
  }

  // computeFinalSolutionPathTrajectories (BS:6173-6274)
  std::vector<Conf> final_path() {
    std::vector<Conf> out;
    if (!have_sol) return out;
    Node sn = conn_start ? nB : nA;
    Node gn = conn_start ? nA : nB;
    std::vector<const Edge*> es, eg;
    while (sn.node_id != 0) {
      const Node& par = ta.nodes[sn.parent_id];
      for (const Edge& e : par.out) if (e.child_node_id == sn.node_id) { es.insert(es.begin(), &e); break; }
      sn = ta.nodes[sn.parent_id];
    }
    while (gn.node_id != 0) {
      const Node& par = tb.nodes[gn.parent_id];
      for (const Edge& e : par.out) if (e.child_node_id == gn.node_id) { eg.push_back(&e); break; }
      gn = tb.nodes[gn.parent_id];
    }
    for (const Edge* e : es)
      for (size_t k = 0; k + 1 < e->traj.size(); ++k) out.push_back(e->traj[k]);
    for (size_t s = 0; s < eg.size(); ++s) {
      for (size_t k = eg[s]->traj.size() - 1; k > 0; --k) out.push_back(eg[s]->traj[k]);
      if (s == eg.size() - 1) out.push_back(eg[s]->traj[0]);
    }
    return out;
  }
};

// ------------------------------------------------------------------------------------------ IK goal search
// Planner::findGoalPose (SP = squirrel_8dof_planner/src/squirrel_8dof_planner.cpp:1129-1201) ->
// BiRRTstarPlanner::getFullPoseFromEEPose (BS:1627-1686) -> RobotController::run_VDLS_Control_Connector
// (CL:3283-3712).  Unpinned choices (DESIGN.md "IK goal search"): portable sin/cos; KDL's Jacobian and
// GetQuaternion as published (orocos_kdl chainjnttojacsolver.cpp, frames.cpp); the damped pseudo-inverse
// sum_i s_i/(s_i^2+d^2) v_i u_i^T (CL:5591-5596) evaluated as J^T (J J^T + d^2 I)^-1 by Cholesky; the
// manipulability product of the singular values > 1e-5 (CL:6061-6084) as prod(diag chol(J J^T)) when
// chol(J J^T - 1e-10 I) has positive pivots (every singular value > 1e-5), else by cyclic Jacobi eigenvalues.

static const int MAX_IK_SEG = 16;

struct IkTask {
  double goal[7];      // x, y, z, qx, qy, qz, qw (BS:1639-1645)
  double lo[6], hi[6]; // endEffectorDeviations (setVariableConstraints, CL:1740-1761)
  double q[8];         // poseInit (setStartConf, CL:1464-1495)
  int max_iter;        // 1000 (BS:1670)
};

struct IkOut {
  double q[8];
  double err[6];
  double manip;
  int reached;  // REACHED (1) / ADVANCED (0), CL:3691-3710
  int iters;
  int fallback; // iterations that needed the Jacobi eigenvalue path
};

static const double IK_DT = 0.1;                      // delta_t_ (CL:3325)
static const double IK_GAIN = 1.0;                    // error_gain_ (CL:306)
static const double IK_MANIP_THR = (double)0.03f;     // min_manip_treshold_ (CL:3299), a float parameter (CL:5505)
static const double IK_DAMP_MAX = (double)0.07f;      // max_damping_factor_ (CL:320), float parameter
static const double IK_SV_EPS = 0.00001;              // CL:6073
static const double IK_BOUND = 0.0001;                // is_error_within_bounds (CL:6925)

// Goal quaternion of getFullPoseFromEEPose (BS:1630-1645).
static void ik_goal_quat(const double* ee, double* g) {
  double sx, cx, sy, cy, sz, cz;
  psincos(ee[3] / 2, &sx, &cx);
  psincos(ee[4] / 2, &sy, &cy);
  psincos(ee[5] / 2, &sz, &cz);
  g[0] = ee[0]; g[1] = ee[1]; g[2] = ee[2];
  g[3] = sx * cy * cz - cx * sy * sz;
  g[4] = cx * sy * cz + sx * cy * sz;
  g[5] = cx * cy * sz - sx * sy * cz;
  g[6] = cx * cy * cz + sx * sy * sz;
}

// KDL Rotation::GetQuaternion (frames.cpp), used by compute_FK (KM:302).
static void get_quaternion(const double* R, double* x, double* y, double* z, double* w) {
  double trace = R[0] + R[4] + R[8];
  if (trace > 1e-12) {
    double s = 0.5 / std::sqrt(trace + 1.0);
    *w = 0.25 / s;
    *x = (R[7] - R[5]) * s;
    *y = (R[2] - R[6]) * s;
    *z = (R[3] - R[1]) * s;
  } else if (R[0] > R[4] && R[0] > R[8]) {
    double s = 2.0 * std::sqrt(1.0 + R[0] - R[4] - R[8]);
    *w = (R[7] - R[5]) / s;
    *x = 0.25 * s;
    *y = (R[1] + R[3]) / s;
    *z = (R[2] + R[6]) / s;
  } else if (R[4] > R[8]) {
    double s = 2.0 * std::sqrt(1.0 + R[4] - R[0] - R[8]);
    *w = (R[2] - R[6]) / s;
    *x = (R[1] + R[3]) / s;
    *y = 0.25 * s;
    *z = (R[5] + R[7]) / s;
  } else {
    double s = 2.0 * std::sqrt(1.0 + R[8] - R[0] - R[4]);
    *w = (R[3] - R[1]) / s;
    *x = (R[2] + R[6]) / s;
    *y = (R[5] + R[7]) / s;
    *z = 0.25 * s;
  }
}

// A segment whose joint does not rotate (prismatic or fixed) and whose f_tip rotation is the identity has the
// identity as local rotation.
static bool ik_rot_identity(const Robot& rb, int s) {
  if (rb.seg_type[s] == 1) return false;
  for (int i = 0; i < 9; ++i)
    if (rb.seg_R[s * 9 + i] != ((i % 4 == 0) ? 1.0 : 0.0)) return false;
  return true;
}

// Segment frames of the 12-segment chain (KDL ChainFkSolverPos_recursive, KM:278-305; the same products as
// ChainJntToJacSolver's T_tmp * segment.pose(q)): T[0] = I, T[s+1] = T[s] * (joint(q) * f_tip).
static void chain_frames(const Robot& rb, const double* q, Frame* T) {
  std::memset(&T[0], 0, sizeof(Frame));
  T[0].R[0] = T[0].R[4] = T[0].R[8] = 1.0;
  for (int s = 0; s < rb.n_seg; ++s) {
    Frame J;
    std::memset(&J, 0, sizeof(J));
    if (rb.seg_type[s] == 1) {
      rot2(&rb.seg_axis[s * 3], q[rb.seg_joint[s]], J.R);
      for (int d = 0; d < 3; ++d) J.p[d] = rb.seg_origin[s * 3 + d];
    } else if (rb.seg_type[s] == 2) {
      J.R[0] = J.R[4] = J.R[8] = 1.0;
      double qq = q[rb.seg_joint[s]];
      for (int d = 0; d < 3; ++d) J.p[d] = rb.seg_origin[s * 3 + d] + rb.seg_axis[s * 3 + d] * qq;
    } else {
      J.R[0] = J.R[4] = J.R[8] = 1.0;
    }
    Frame F;
    std::memcpy(F.R, &rb.seg_R[s * 9], 9 * sizeof(double));
    std::memcpy(F.p, &rb.seg_p[s * 3], 3 * sizeof(double));
    const Frame L = fmul(J, F);
    if (ik_rot_identity(rb, s)) {
      // the local rotation is exactly I: T.R * I == T.R up to the sign of a zero, so only the translation is applied
      T[s + 1] = T[s];
      for (int r = 0; r < 3; ++r) {
        const double m = T[s].R[r * 3 + 0] * L.p[0] + T[s].R[r * 3 + 1] * L.p[1] + T[s].R[r * 3 + 2] * L.p[2];
        T[s + 1].p[r] = m + T[s].p[r];
      }
    } else {
      T[s + 1] = fmul(T[s], L);
    }
  }
}

// compute_FK (KM:278-305): [x, y, z, qx, qy, qz, qw] of the chain tip.
static void ee_pose(const Robot& rb, const Frame* T, double* ee) {
  const Frame& E = T[rb.n_seg];
  ee[0] = E.p[0]; ee[1] = E.p[1]; ee[2] = E.p[2];
  get_quaternion(E.R, &ee[3], &ee[4], &ee[5], &ee[6]);
}

// Cartesian error (set_EE_goal_pose CL:1690-1720 without, update_error_vec CL:2203-2239 with the deviation
// clamp): position des - cur, orientation eta_c eps_d - eta_d eps_c - S(eps_d) eps_c.
static void ik_error(const double* cur, const IkTask& t, bool clamp, double* e) {
  const double* d = t.goal;
  const double S[3][3] = {{0.0, -d[5], d[4]}, {d[5], 0.0, -d[3]}, {-d[4], d[3], 0.0}};
  for (int i = 0; i < 6; ++i) {
    if (i < 3) e[i] = d[i] - cur[i];
    else e[i] = cur[6] * d[i] - d[6] * cur[i] - (S[i - 3][0] * cur[3] + S[i - 3][1] * cur[4] + S[i - 3][2] * cur[5]);
  }
  if (clamp)
    for (int i = 0; i < 6; ++i) e[i] = (e[i] < t.lo[i] || e[i] > t.hi[i]) ? e[i] : 0.0;
}

// KDL ChainJntToJacSolver::JntToJac for the frames T of q: column k of the k-th movable segment s is
// T[s].M * (joint twist referred to the segment tip), then referred to the chain tip (KDL: Twist::RefPoint to every
// later tip in turn; the sum of those offsets telescopes to one).  Rows 0-2 linear, 3-5 angular; cast to float
// (getJacobian, CL:5273-5301).
static void jacobian(const Robot& rb, const double* q, const Frame* T, double J[6][8]) {
  int k = 0;
  for (int s = 0; s < rb.n_seg; ++s) {
    if (rb.seg_type[s] == 0) continue;
    const double* ax = &rb.seg_axis[s * 3];
    double M[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (rb.seg_type[s] == 1) rot2(ax, q[rb.seg_joint[s]], M);
    const double* fp = &rb.seg_p[s * 3];
    double v[3], rl[3], vl[3];
    for (int r = 0; r < 3; ++r) v[r] = M[r * 3 + 0] * fp[0] + M[r * 3 + 1] * fp[1] + M[r * 3 + 2] * fp[2];
    for (int d = 0; d < 3; ++d) {
      rl[d] = rb.seg_type[s] == 1 ? ax[d] * 1.0 : 0.0;
      vl[d] = rb.seg_type[s] == 2 ? ax[d] * 1.0 : 0.0;
    }
    double c0 = rl[1] * v[2] - rl[2] * v[1], c1 = rl[2] * v[0] - rl[0] * v[2], c2 = rl[0] * v[1] - rl[1] * v[0];
    vl[0] = vl[0] + c0; vl[1] = vl[1] + c1; vl[2] = vl[2] + c2;
    const double* B = T[s].R;
    double vel[3], rot[3];
    for (int r = 0; r < 3; ++r) {
      vel[r] = B[r * 3 + 0] * vl[0] + B[r * 3 + 1] * vl[1] + B[r * 3 + 2] * vl[2];
      rot[r] = B[r * 3 + 0] * rl[0] + B[r * 3 + 1] * rl[1] + B[r * 3 + 2] * rl[2];
    }
    // KDL moves the column to every later tip in turn (Twist::RefPoint(T[i+1].p - T[i].p), i > s); the offsets
    // telescope, so the column is moved once, to the chain tip
    {
      double dl[3];
      for (int d = 0; d < 3; ++d) dl[d] = T[rb.n_seg].p[d] - T[s + 1].p[d];
      double x0 = rot[1] * dl[2] - rot[2] * dl[1], x1 = rot[2] * dl[0] - rot[0] * dl[2], x2 = rot[0] * dl[1] - rot[1] * dl[0];
      vel[0] = vel[0] + x0; vel[1] = vel[1] + x1; vel[2] = vel[2] + x2;
    }
    for (int d = 0; d < 3; ++d) {
      J[d][k] = (double)(float)vel[d];
      J[3 + d][k] = (double)(float)rot[d];
    }
    ++k;
  }
}

// Gauss-Jordan elimination of the augmented [B | rhs] (6 x 7, no pivoting: B is symmetric positive definite on
// this path): step k divides every other row's column-k entry by the pivot and subtracts that multiple of row k
// from the row's columns > k.  The pivots are those of B's LDL^T; the solution is z_i = M[i][6] / M[i][i].
static void gauss_jordan6(double M[6][7], double* z) {
  for (int k = 0; k < 6; ++k)
    for (int i = 0; i < 6; ++i) {
      if (i == k) continue;
      const double f = M[i][k] / M[k][k];
      for (int j = k + 1; j < 7; ++j) M[i][j] = M[i][j] - f * M[k][j];
    }
  for (int i = 0; i < 6; ++i) z[i] = M[i][6] / M[i][i];
}

// Positive definiteness of A - tau I by symmetric elimination of the upper triangle (the LDL^T pivots): every
// singular value of J exceeds sqrt(tau) iff every pivot is > 0.
static bool shifted_pd6(const double A[6][6], double tau) {
  double P[6][6];
  for (int i = 0; i < 6; ++i)
    for (int j = i; j < 6; ++j) P[i][j] = i == j ? A[i][i] + (-tau) : A[i][j];
  bool pd = true;
  for (int k = 0; k < 6; ++k) {
    if (!(P[k][k] > 0.0)) pd = false;
    for (int i = k + 1; i < 6; ++i) {
      const double f = P[k][i] / P[k][k];
      for (int j = i; j < 6; ++j) P[i][j] = P[i][j] - f * P[k][j];
    }
  }
  return pd;
}

// Cyclic Jacobi eigen-decomposition of a symmetric 6x6: eigenvalues on the diagonal of a, eigenvectors in the
// columns of V (rows p < q in order, at most 30 sweeps).
static void jacobi_eigen6(const double A[6][6], double a[6][6], double V[6][6]) {
  std::memcpy(a, A, sizeof(double) * 36);
  for (int i = 0; i < 6; ++i)
    for (int k = 0; k < 6; ++k) V[i][k] = i == k ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 30; ++sweep) {
    double off = 0.0;
    for (int p = 0; p < 5; ++p)
      for (int q = p + 1; q < 6; ++q) off = off + a[p][q] * a[p][q];
    if (off == 0.0) break;
    for (int p = 0; p < 5; ++p)
      for (int q = p + 1; q < 6; ++q) {
        double apq = a[p][q];
        if (apq == 0.0) continue;
        double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
        double t = (theta >= 0.0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 6; ++k) {
          double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
          if (k == p || k == q) continue;
          double akp = a[k][p], akq = a[k][q];
          double np = c * akp - s * akq, nq = s * akp + c * akq;
          a[k][p] = np; a[p][k] = np; a[k][q] = nq; a[q][k] = nq;
        }
        double app = a[p][p] - t * apq, aqq = a[q][q] + t * apq;
        a[p][p] = app; a[q][q] = aqq; a[p][q] = 0.0; a[q][p] = 0.0;
      }
  }
}

// run_VDLS_Control_Connector (CL:3283-3712) for one start configuration and one goal pose.
static void ik_solve(const Robot& rb, const IkTask& t, IkOut* o) {
  double q[8];
  for (int j = 0; j < 8; ++j) q[j] = t.q[j];
  Frame T[MAX_IK_SEG + 1];
  double ee[7], err[6];
  chain_frames(rb, q, T);
  ee_pose(rb, T, ee);
  ik_error(ee, t, false, err);  // set_EE_goal_pose (CL:1689-1720)
  bool within = false;          // CL:3328
  int iter = 0, fallback = 0;
  double manip = 0.0;
  const double tau = IK_SV_EPS * IK_SV_EPS;
  while (!within) {
    double J[6][8], A[6][6], M[6][7], E[6][6], V[6][6], z[6], ep[6];
    jacobian(rb, q, T, J);
    for (int i = 0; i < 6; ++i)
      for (int k = 0; k < 6; ++k) {  // pairwise sums (a short dependent chain on the GPU)
        double p[8];
        for (int c = 0; c < 8; ++c) p[c] = J[i][c] * J[k][c];
        A[i][k] = ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
      }
    for (int i = 0; i < 6; ++i) ep[i] = 0.0 + IK_GAIN * err[i];  // current_goal_ee_vel_ + error_gain_ * error_
    for (int i = 0; i < 6; ++i) {
      for (int k = 0; k < 6; ++k) M[i][k] = A[i][k];
      M[i][6] = ep[i];
    }
    // computeManipulabilityMeasure (CL:6050-6089): product of the singular values > 1e-5.  Every singular value
    // exceeds 1e-5 (every eigenvalue of A exceeds tau) if det A > tau * tr(A)^5 (lambda_min >= det / lambda_max^5),
    // else exactly when A - tau I is positive definite.
    gauss_jordan6(M, z);
    double pr = 1.0;
    for (int k = 0; k < 6; ++k) pr = pr * M[k][k];
    const double tr = ((((A[0][0] + A[1][1]) + A[2][2]) + A[3][3]) + A[4][4]) + A[5][5];
    const double tr5 = (((tr * tr) * tr) * tr) * tr;
    const bool normal = pr > tau * tr5 || shifted_pd6(A, tau);
    if (normal) {
      manip = std::sqrt(pr);
    } else {
      jacobi_eigen6(A, E, V);
      manip = 1.0;
      for (int j = 0; j < 6; ++j) {
        double sv = std::sqrt(E[j][j] > 0.0 ? E[j][j] : 0.0);
        if (std::fabs(sv) > IK_SV_EPS) manip = manip * std::fabs(sv);
      }
      ++fallback;
    }
    if (manip == 1.0 || manip < 0.00001) manip = 0.0001;
    // compute_J_vdls (CL:5505-5614) applied to the error (CL:3455-3497): q_dot = J_vdls e = J^T (J J^T + d^2 I)^-1 e,
    // the inverse applied by Gauss-Jordan, or (a singular value <= 1e-5) through the eigenvectors u_i of J J^T:
    // sum_i u_i (u_i^T e) / (max(lambda_i, 0) + d^2)
    double damp = 0.0;
    if (manip < IK_MANIP_THR)
      damp = IK_DAMP_MAX * ((1 - (manip / IK_MANIP_THR)) * (1 - (manip / IK_MANIP_THR)));
    if (normal && damp != 0.0) {
      for (int i = 0; i < 6; ++i) {
        for (int k = 0; k < 6; ++k) M[i][k] = i == k ? A[i][i] + damp * damp : A[i][k];
        M[i][6] = ep[i];
      }
      gauss_jordan6(M, z);
    }
    if (!normal) {
      double g[6];
      for (int i = 0; i < 6; ++i) {
        double t = V[0][i] * ep[0];
        for (int j = 1; j < 6; ++j) t = t + V[j][i] * ep[j];
        g[i] = (1.0 / ((E[i][i] > 0.0 ? E[i][i] : 0.0) + damp * damp)) * t;
      }
      for (int k = 0; k < 6; ++k) {
        double y = g[0] * V[k][0];
        for (int i = 1; i < 6; ++i) y = y + g[i] * V[k][i];
        z[k] = y;
      }
    }
    double qd[8];
    for (int c = 0; c < 8; ++c) {
      double p[6];
      for (int i = 0; i < 6; ++i) p[i] = J[i][c] * z[i];
      qd[c] = ((p[0] + p[1]) + (p[2] + p[3])) + (p[4] + p[5]);
    }
    // joint update with the joint-limit check (CL:3504-3550, KM:680-703)
    int c = 0;
    for (int s = 0; s < rb.n_seg; ++s) {
      if (rb.seg_type[s] == 0) continue;
      int j = rb.seg_joint[s];
      double nv = q[j] + qd[c] * IK_DT;
      if (!(nv < rb.q_min[j] || nv > rb.q_max[j])) q[j] = nv;
      ++c;
    }
    chain_frames(rb, q, T);
    ee_pose(rb, T, ee);
    ik_error(ee, t, true, err);
    within = true;
    for (int i = 0; i < 6; ++i)
      if (std::fabs(err[i]) > IK_BOUND) within = false;
    ++iter;
    if (iter == t.max_iter) break;
  }
  for (int j = 0; j < 8; ++j) o->q[j] = q[j];
  for (int i = 0; i < 6; ++i) o->err[i] = err[i];
  o->manip = manip;
  o->reached = iter == t.max_iter ? 0 : 1;
  o->iters = iter;
  o->fallback = fallback;
}

// Base-angle candidates and start configurations of Planner::findGoalPose (SP:1129-1194), in the order the
// reference tries them.  getEndEffectorDirection (SP:1639-1661): the y axis of tf setRPY(roll, pitch, yaw).
static bool ee_downward(const double* ee) {
  double sr, cr, sp, cp, sy, cy;
  psincos(ee[3] * 0.5, &sr, &cr);
  psincos(ee[4] * 0.5, &sp, &cp);
  psincos(ee[5] * 0.5, &sy, &cy);
  double x = sr * cp * cy - cr * sp * sy, y = cr * sp * cy + sr * cp * sy;
  double z = cr * cp * sy - sr * sp * cy, w = cr * cp * cy + sr * sp * sy;
  double d = x * x + y * y + z * z + w * w, s = 2.0 / d;
  double xs = x * s, ys = y * s, zs = z * s;
  double wx = w * xs, yy = y * ys, yz = y * zs, xx = x * xs;
  double az = (x * zs - w * ys) * 0.0 + (yz + wx) * 1.0 + (1.0 - (xx + yy)) * 0.0;
  return !(std::fabs(az) < 0.9);
}

static int goal_candidates(const double* ee, const double* cur, double disc_deg, std::vector<IkTask>& tasks) {
  if (disc_deg < 1) disc_deg = 1.0;  // SP:80-83
  const double disc = disc_deg * (M_PI / 180.0);
  const bool down = ee_downward(ee);
  const double dist = down ? 0.44 : 0.47;
  const double arm_down[5] = {-0.8, 0.8, 0.0, -1.5, 0.0}, arm_side[5] = {-1.2, 1.1, 0.0, 0.7, -1.5};
  const double gx = ee[0] - cur[0], gy = ee[1] - cur[1];
  const double start = gy > 0 ? std::acos(gx / std::sqrt(std::pow(gx, 2) + std::pow(gy, 2)))
                              : -std::acos(gx / std::sqrt(std::pow(gx, 2) + std::pow(gy, 2)));
  IkTask t;
  double g[7];
  ik_goal_quat(ee, g);
  for (int i = 0; i < 7; ++i) t.goal[i] = g[i];
  for (int i = 0; i < 3; ++i) { t.lo[i] = -0.005; t.hi[i] = 0.005; t.lo[i + 3] = -0.025; t.hi[i + 3] = 0.025; }
  t.max_iter = 1000;
  double diff = 0.0;
  while (std::fabs(diff) < M_PI) {
    const double a = start + diff;
    double sa, ca;
    psincos(a, &sa, &ca);
    t.q[0] = ee[0] - dist * ca;
    t.q[1] = ee[1] - dist * sa;
    t.q[2] = a + 0.99;
    for (int j = 0; j < 5; ++j) t.q[3 + j] = down ? arm_down[j] : arm_side[j];
    tasks.push_back(t);
    diff *= -1;
    diff += 0.0;
    if (diff >= 0.0) diff += disc;
  }
  return down ? 1 : 0;
}

}  // namespace orc

// ============================================================================================ C ABI
// Flat arrays only; the Python side (oracle/oracle.py) builds them from the model JSON and the scene.
extern "C" {

struct orc_robot_desc {
  int n_links;
  const int *parent, *joint, *type;
  const double *axis, *origin, *R, *p;
  int n_seg;
  const int *seg_joint, *seg_type;
  const double *seg_axis, *seg_origin, *seg_R, *seg_p;
  int n_sph;
  const int* sph_link;
  const double *sph_c, *sph_r;
  const int* lb_has;
  const double *lb_c, *lb_r;
  int n_pairs;
  const int *pair_a, *pair_b;
  const double *q_min, *q_max;
  const int* rev;
  double root_z;
  int n_chain;
  const int *ch_type, *ch_joint, *ch_body;
  const double *ch_axis, *ch_origin, *ch_R, *ch_p;
  int n_body;
  const int *sph_body, *lb_body;
  const double *sph_cb, *lb_cb;
  int n_prim;
  const int *prim_type, *prim_body, *prim_link;
  const double *prim_cb, *prim_ab, *prim_h, *prim_rxy;
};

struct orc_scene_desc {
  int nx, ny, nz;
  double ox, oy, oz, res;
  const uint64_t* bits;
  const uint16_t* d2;
  int n_slab;
  const uint16_t* slab;  // n_slab x ny x nx
};

struct orc_params {
  double near_r, step;
  int n_pts, max_near;
  double opt_thresh;
  int tree_opt, informed;
  double env_x[2], env_y[2];
  int self, map;
  uint64_t seed;
  uint32_t query;
  int max_iter;
  double max_time;
  long long max_checked;
  int threads;           // OpenMP threads of the two scans (<= 1: sequential)
};

struct orc_result {
  int status;            // 0 ok (solution), 1 no solution, -2 start invalid, -3 goal invalid
  long long iterations, first_iter, last_iter, checked, valid, ck_calls;
  double t_first, t_total;
  double cost[3], h0[3];
  int n_start, n_goal, edges_start, edges_goal, rewires_start, rewires_goal;
  int conn_start;        // 1 if the connection node lives in the start tree
  int conn_b, conn_a;    // node ids of m_node_tree_B / m_node_tree_A
  int n_wp;
};

static orc::Robot* mk_robot(const orc_robot_desc* d) {
  orc::Robot* r = new orc::Robot();
  r->n_links = d->n_links;
  r->parent.assign(d->parent, d->parent + d->n_links);
  r->joint.assign(d->joint, d->joint + d->n_links);
  r->type.assign(d->type, d->type + d->n_links);
  r->axis.assign(d->axis, d->axis + 3 * d->n_links);
  r->origin.assign(d->origin, d->origin + 3 * d->n_links);
  r->R.assign(d->R, d->R + 9 * d->n_links);
  r->p.assign(d->p, d->p + 3 * d->n_links);
  r->n_seg = d->n_seg;
  r->seg_joint.assign(d->seg_joint, d->seg_joint + d->n_seg);
  r->seg_type.assign(d->seg_type, d->seg_type + d->n_seg);
  r->seg_axis.assign(d->seg_axis, d->seg_axis + 3 * d->n_seg);
  r->seg_origin.assign(d->seg_origin, d->seg_origin + 3 * d->n_seg);
  r->seg_R.assign(d->seg_R, d->seg_R + 9 * d->n_seg);
  r->seg_p.assign(d->seg_p, d->seg_p + 3 * d->n_seg);
  r->n_sph = d->n_sph;
  r->sph_link.assign(d->sph_link, d->sph_link + d->n_sph);
  r->sph_c.assign(d->sph_c, d->sph_c + 3 * d->n_sph);
  r->sph_r.assign(d->sph_r, d->sph_r + d->n_sph);
  r->lb_has.assign(d->lb_has, d->lb_has + d->n_links);
  r->lb_c.assign(d->lb_c, d->lb_c + 3 * d->n_links);
  r->lb_r.assign(d->lb_r, d->lb_r + d->n_links);
  r->n_pairs = d->n_pairs;
  r->pair_a.assign(d->pair_a, d->pair_a + d->n_pairs);
  r->pair_b.assign(d->pair_b, d->pair_b + d->n_pairs);
  for (int j = 0; j < 8; ++j) { r->q_min[j] = d->q_min[j]; r->q_max[j] = d->q_max[j]; r->rev[j] = d->rev[j]; }
  r->root_z = d->root_z;
  r->n_chain = d->n_chain;
  r->ch_type.assign(d->ch_type, d->ch_type + d->n_chain);
  r->ch_joint.assign(d->ch_joint, d->ch_joint + d->n_chain);
  r->ch_body.assign(d->ch_body, d->ch_body + d->n_chain);
  r->ch_axis.assign(d->ch_axis, d->ch_axis + 3 * d->n_chain);
  r->ch_origin.assign(d->ch_origin, d->ch_origin + 3 * d->n_chain);
  r->ch_R.assign(d->ch_R, d->ch_R + 9 * d->n_chain);
  r->ch_p.assign(d->ch_p, d->ch_p + 3 * d->n_chain);
  r->n_body = d->n_body;
  r->sph_body.assign(d->sph_body, d->sph_body + d->n_sph);
  r->sph_cb.assign(d->sph_cb, d->sph_cb + 3 * d->n_sph);
  r->lb_body.assign(d->lb_body, d->lb_body + d->n_links);
  r->lb_cb.assign(d->lb_cb, d->lb_cb + 3 * d->n_links);
  r->link_sph.assign(d->n_links, {});
  for (int i = 0; i < d->n_sph; ++i) r->link_sph[d->sph_link[i]].push_back(i);
  r->link_prim.assign(d->n_links, -1);
  for (int k = 0; k < d->n_prim; ++k) {
    orc::Robot::Prim P;
    P.type = d->prim_type[k]; P.body = d->prim_body[k]; P.link = d->prim_link[k]; P.rxy = d->prim_rxy[k];
    for (int i = 0; i < 3; ++i) { P.cb[i] = d->prim_cb[k * 3 + i]; P.ab[i] = d->prim_ab[k * 3 + i]; P.h[i] = d->prim_h[k * 3 + i]; }
    r->prims.push_back(P);
    r->link_prim[P.link] = k;
  }
  return r;
}

static orc::Scene* mk_scene(const orc_scene_desc* d) {
  if (!d) return nullptr;
  orc::Scene* s = new orc::Scene();
  s->nx = d->nx; s->ny = d->ny; s->nz = d->nz; s->wx = (d->nx + 63) / 64;
  s->ox = d->ox; s->oy = d->oy; s->oz = d->oz; s->res = d->res;
  size_t nw = (size_t)s->wx * d->ny * d->nz, nc = (size_t)d->nx * d->ny * d->nz;
  s->bits.assign(d->bits, d->bits + nw);
  s->d2.assign(d->d2, d->d2 + nc);
  const size_t plane = (size_t)d->nx * d->ny;
  for (int k = 0; k < d->n_slab; ++k) s->slab.emplace_back(d->slab + k * plane, d->slab + (k + 1) * plane);
  return s;
}

struct orc_handle {
  orc::Robot* rb;
  orc::Scene* sc;
  orc::Checker ck;
  orc::Planner* pl = nullptr;
  std::vector<orc::Conf> path;
};

void* orc_create(const orc_robot_desc* rd, const orc_scene_desc* sd, const uint8_t* map_enabled) {
  orc_handle* h = new orc_handle();
  h->rb = mk_robot(rd);
  h->sc = mk_scene(sd);
  if (h->sc && h->sc->slab.size() < h->rb->prims.size()) {  // every primitive needs its slab field
    fprintf(stderr, "oracle: scene without the primitives' slab fields\n");
    std::abort();
  }
  h->ck.init(h->rb, h->sc);
  if (map_enabled) for (int i = 0; i < rd->n_links; ++i) h->ck.map_enabled[i] = map_enabled[i];
  return h;
}

void orc_destroy(void* hp) {
  orc_handle* h = (orc_handle*)hp;
  delete h->pl;
  delete h->rb;
  delete h->sc;
  delete h;
}

// Batch validity: valid[i] = !isInCollision(q_i).  q is row-major n x 8.
void orc_check_configs(void* hp, const double* q, int n, int self, int map, uint8_t* valid) {
  orc_handle* h = (orc_handle*)hp;
  for (int i = 0; i < n; ++i) valid[i] = h->ck.in_collision(q + 8 * i, self, map) ? 0 : 1;
}

// getCollisions (birrt_star.cpp:6910-6914 -> collision_checker.hpp:123-132): link_map[link] = 1 if a sphere of the
// link touches the map (getMapCollisions, CC:610-630: disabled links included), pair_self[p] = 1 if model pair p
// overlaps (getSelfCollisions, CC:594-608: every pair, no early exit).
void orc_collisions(void* hp, const double* q, uint8_t* link_map, uint8_t* pair_self) {
  orc_handle* h = (orc_handle*)hp;
  orc::Checker& ck = h->ck;
  const orc::Robot& rb = *ck.rb;
  orc::body_frames(rb, q, ck.frames.data());
  for (int i = 0; i < rb.n_sph; ++i) orc::xform(ck.frames[rb.sph_body[i]], &rb.sph_cb[i * 3], &ck.wc[i * 3]);
  ck.prim_frames();
  for (int l = 0; l < rb.n_links; ++l) link_map[l] = 0;
  if (ck.sc) {
    for (int i = 0; i < rb.n_sph; ++i)
      if (orc::sphere_hits_map(*ck.sc, &ck.wc[i * 3], rb.sph_r[i], ck.T[i])) link_map[rb.sph_link[i]] = 1;
    for (size_t p = 0; p < rb.prims.size(); ++p)
      if (ck.prim_map(p)) link_map[rb.prims[p].link] = 1;
  }
  for (int pi = 0; pi < rb.n_pairs; ++pi) {
    if (rb.link_prim[rb.pair_a[pi]] >= 0 || rb.link_prim[rb.pair_b[pi]] >= 0) {
      pair_self[pi] = ck.pair_prim(rb.pair_a[pi], rb.pair_b[pi]) ? 1 : 0;
      continue;
    }
    bool hit = false;
    for (int sa : rb.link_sph[rb.pair_a[pi]])
      for (int sb : rb.link_sph[rb.pair_b[pi]]) {
        const double* a = &ck.wc[sa * 3];
        const double* b = &ck.wc[sb * 3];
        double ex = a[0] - b[0], ey = a[1] - b[1], ez = a[2] - b[2];
        double r2 = rb.sph_r[sa] + rb.sph_r[sb];
        if (ex * ex + ey * ey + ez * ez <= r2 * r2) hit = true;
      }
    pair_self[pi] = hit ? 1 : 0;
  }
}

// Link world frames (n_links x 12: R row-major then p) and the chain end-effector z.
void orc_fk(void* hp, const double* q, int n, double* frames, double* eez) {
  orc_handle* h = (orc_handle*)hp;
  std::vector<orc::Frame> T(h->rb->n_links);
  for (int i = 0; i < n; ++i) {
    orc::link_frames(*h->rb, q + 8 * i, T.data());
    if (frames)
      for (int l = 0; l < h->rb->n_links; ++l) {
        std::memcpy(frames + ((size_t)i * h->rb->n_links + l) * 12, T[l].R, 9 * sizeof(double));
        std::memcpy(frames + ((size_t)i * h->rb->n_links + l) * 12 + 9, T[l].p, 3 * sizeof(double));
      }
    if (eez) eez[i] = orc::ee_z(*h->rb, q + 8 * i);
  }
}

// Body frames (n x n_body x 12) of the collision model.
void orc_body_fk(void* hp, const double* q, int n, double* frames) {
  orc_handle* h = (orc_handle*)hp;
  std::vector<orc::Frame> B(h->rb->n_body);
  for (int i = 0; i < n; ++i) {
    orc::body_frames(*h->rb, q + 8 * i, B.data());
    for (int b = 0; b < h->rb->n_body; ++b) {
      std::memcpy(frames + ((size_t)i * h->rb->n_body + b) * 12, B[b].R, 9 * sizeof(double));
      std::memcpy(frames + ((size_t)i * h->rb->n_body + b) * 12 + 9, B[b].p, 3 * sizeof(double));
    }
  }
}

// Raw Philox4x32-10 block (known-answer tests).
void orc_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
  uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
  orc::philox(c, key[0], key[1]);
  for (int i = 0; i < 4; ++i) out[i] = c[i];
}

void orc_sincos(const double* x, int n, double* s, double* c) {
  for (int i = 0; i < n; ++i) orc::psincos(x[i], s + i, c + i);
}

void orc_u01(uint64_t seed, uint32_t query, const uint32_t* ctr, int n, double* out) {
  for (int i = 0; i < n; ++i) out[i] = orc::u01(seed, query, ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]);
}

static int fill_result(orc_handle* h, bool ok, orc_result* res);

static void set_params(orc::Planner& pl, const orc_params* p) {
  pl.P.near_r = p->near_r; pl.P.step = p->step; pl.P.n_pts = p->n_pts; pl.P.max_near = p->max_near;
  pl.P.opt_thresh = p->opt_thresh; pl.P.tree_opt = p->tree_opt; pl.P.informed = p->informed;
  pl.P.env_x[0] = p->env_x[0]; pl.P.env_x[1] = p->env_x[1]; pl.P.env_y[0] = p->env_y[0]; pl.P.env_y[1] = p->env_y[1];
  pl.P.self = p->self; pl.P.map = p->map; pl.P.seed = p->seed; pl.P.query = p->query;
  pl.P.max_iter = p->max_iter; pl.P.max_time = p->max_time; pl.P.max_checked = p->max_checked;
  pl.P.threads = p->threads;
}

// Continuing another run (test infrastructure: the GPU planner's state after some iterations, DESIGN.md "Large
// trees"): begin = init_planner of the same query, then both trees and the loop scalars replace the fresh state, then
// the loop runs on to the budget of `p` (max_iter counts from the run's start, as the GPU's budget).
int orc_resume_begin(void* hp, const double* start, const double* goal, const orc_params* p) {
  orc_handle* h = (orc_handle*)hp;
  delete h->pl;
  h->pl = new orc::Planner();
  orc::Planner& pl = *h->pl;
  pl.rb = h->rb;
  pl.ck = &h->ck;
  set_params(pl, p);
  orc::Conf s, g;
  for (int j = 0; j < 8; ++j) { s[j] = start[j]; g[j] = goal[j]; }
  h->ck.calls = 0;
  return pl.init(s, g);
}

// One tree: n nodes (parent id, configuration, costs, in-edge interpolation start / target) and every node's children
// in the reference's out-edge order (child_ids[child_off[i] .. child_off[i + 1]]).
void orc_resume_tree(void* hp, int which, int n, const int* parent, const double* q, const double* cost,
                     const double* e_start, const double* e_target, const int* child_off, const int* child_ids,
                     int num_edges, int num_rewire) {
  orc_handle* h = (orc_handle*)hp;
  orc::Planner& pl = *h->pl;
  orc::Tree& t = which ? pl.tb : pl.ta;
  t.nodes.assign(n, orc::Node());
  for (int i = 0; i < n; ++i) {
    orc::Node& nd = t.nodes[i];
    nd.node_id = i;
    nd.parent_id = parent[i];
    for (int j = 0; j < 8; ++j) nd.q[j] = q[8 * (size_t)i + j];
    nd.cost.total = cost[3 * (size_t)i]; nd.cost.rev = cost[3 * (size_t)i + 1]; nd.cost.prism = cost[3 * (size_t)i + 2];
  }
  for (int i = 0; i < n; ++i)
    for (int k = child_off[i]; k < child_off[i + 1]; ++k) {
      const int c = child_ids[k];
      orc::Edge e;
      e.root_node_id = i;
      e.child_node_id = c;
      // connectNodesInterpolation's trajectory from the child's in-edge (the arithmetic of connect_nodes)
      double step[8];
      for (int j = 0; j < 8; ++j) step[j] = (e_target[8 * (size_t)c + j] - e_start[8 * (size_t)c + j]) / double(pl.P.n_pts);
      e.traj.resize(pl.P.n_pts + 1);
      for (int inc = 0; inc <= pl.P.n_pts; ++inc)
        for (int j = 0; j < 8; ++j) e.traj[inc][j] = e_start[8 * (size_t)c + j] + inc * step[j];
      for (int j = 0; j < 8; ++j) { e.s[j] = e_start[8 * (size_t)c + j]; e.g[j] = e_target[8 * (size_t)c + j]; }
      t.nodes[i].out.push_back(e);
    }
  t.num_nodes = n;
  t.num_edges = num_edges;
  t.num_rewire = num_rewire;
}

// The loop scalars (iv: iteration, checked, valid, first_iter, last_iter, have_sol, conn_start, tree_A of the next
// iteration (1 = goal), nB id / parent, nA id / parent; dv: c_best[3], nB q[8] / cost[3], nA q[8] / cost[3]), then the
// loop to the budget.
int orc_resume_run(void* hp, const long long* iv, const double* dv, orc_result* res) {
  orc_handle* h = (orc_handle*)hp;
  orc::Planner& pl = *h->pl;
  std::memset(res, 0, sizeof(*res));
  pl.iter = iv[0];
  pl.st.checked = iv[1]; pl.st.valid = iv[2]; pl.st.first_iter = iv[3]; pl.st.last_iter = iv[4];
  pl.have_sol = iv[5] != 0;
  pl.conn_start = iv[6] != 0;
  pl.cbest = dv[0]; pl.cbest_rev = dv[1]; pl.cbest_prism = dv[2];
  orc::Node* nb[2] = {&pl.nB, &pl.nA};
  for (int k = 0; k < 2; ++k) {
    nb[k]->node_id = (int)iv[8 + 2 * k];
    nb[k]->parent_id = (int)iv[9 + 2 * k];
    for (int j = 0; j < 8; ++j) nb[k]->q[j] = dv[3 + 11 * k + j];
    nb[k]->cost.total = dv[11 + 11 * k]; nb[k]->cost.rev = dv[12 + 11 * k]; nb[k]->cost.prism = dv[13 + 11 * k];
    nb[k]->out.clear();
  }
  return fill_result(h, pl.resume(iv[7] != 0), res);
}

// The state orc_resume_* takes, of this handle's last run: per tree the in-edge (interpolation start / target) of every
// node and the children in out-edge order (child_off: n + 1 offsets; returns the total), then the loop scalars.
int orc_export_tree(void* hp, int which, double* e_start, double* e_target, int* child_off, int* child_ids) {
  orc_handle* h = (orc_handle*)hp;
  const orc::Tree& t = which ? h->pl->tb : h->pl->ta;
  int k = 0;
  for (size_t i = 0; i < t.nodes.size(); ++i) {
    if (child_off) child_off[i] = k;
    for (const orc::Edge& e : t.nodes[i].out) {
      if (child_ids) child_ids[k] = e.child_node_id;
      if (e_start) std::memcpy(e_start + 8 * (size_t)e.child_node_id, e.s.data(), 8 * sizeof(double));
      if (e_target) std::memcpy(e_target + 8 * (size_t)e.child_node_id, e.g.data(), 8 * sizeof(double));
      ++k;
    }
  }
  if (child_off) child_off[t.nodes.size()] = k;
  return k;
}

void orc_export_state(void* hp, long long* iv, double* dv) {
  const orc::Planner& pl = *((orc_handle*)hp)->pl;
  iv[0] = pl.iter; iv[1] = pl.st.checked; iv[2] = pl.st.valid; iv[3] = pl.st.first_iter; iv[4] = pl.st.last_iter;
  iv[5] = pl.have_sol; iv[6] = pl.conn_start; iv[7] = pl.iter & 1;  // tree_A alternates, starting with the start tree
  const orc::Node* nb[2] = {&pl.nB, &pl.nA};
  dv[0] = pl.cbest; dv[1] = pl.cbest_rev; dv[2] = pl.cbest_prism;
  for (int k = 0; k < 2; ++k) {
    iv[8 + 2 * k] = nb[k]->node_id;
    iv[9 + 2 * k] = nb[k]->parent_id;
    for (int j = 0; j < 8; ++j) dv[3 + 11 * k + j] = nb[k]->q[j];
    dv[11 + 11 * k] = nb[k]->cost.total; dv[12 + 11 * k] = nb[k]->cost.rev; dv[13 + 11 * k] = nb[k]->cost.prism;
  }
}

int orc_plan(void* hp, const double* start, const double* goal, const orc_params* p, orc_result* res) {
  orc_handle* h = (orc_handle*)hp;
  delete h->pl;
  h->pl = new orc::Planner();
  orc::Planner& pl = *h->pl;
  pl.rb = h->rb;
  pl.ck = &h->ck;
  set_params(pl, p);
  orc::Conf s, g;
  for (int j = 0; j < 8; ++j) { s[j] = start[j]; g[j] = goal[j]; }
  std::memset(res, 0, sizeof(*res));
  h->ck.calls = 0;
  int st = pl.init(s, g);
  if (st) { res->status = st; return st; }
  return fill_result(h, pl.run(), res);
}

static int fill_result(orc_handle* h, bool ok, orc_result* res) {
  orc::Planner& pl = *h->pl;
  h->path = pl.final_path();
  res->status = ok ? 0 : 1;
  res->iterations = pl.st.iterations; res->first_iter = pl.st.first_iter; res->last_iter = pl.st.last_iter;
  res->checked = pl.st.checked; res->valid = pl.st.valid; res->ck_calls = h->ck.calls;
  res->t_first = pl.st.t_first; res->t_total = pl.st.t_total;
  res->cost[0] = pl.cbest; res->cost[1] = pl.cbest_rev; res->cost[2] = pl.cbest_prism;
  res->h0[0] = pl.h0.total; res->h0[1] = pl.h0.rev; res->h0[2] = pl.h0.prism;
  res->n_start = (int)pl.ta.nodes.size(); res->n_goal = (int)pl.tb.nodes.size();
  res->edges_start = pl.ta.num_edges; res->edges_goal = pl.tb.num_edges;
  res->rewires_start = pl.ta.num_rewire; res->rewires_goal = pl.tb.num_rewire;
  res->conn_start = pl.conn_start ? 1 : 0;
  res->conn_b = pl.nB.node_id; res->conn_a = pl.nA.node_id;
  res->n_wp = (int)h->path.size();
  return res->status;
}

void orc_get_path(void* hp, double* wp) {
  orc_handle* h = (orc_handle*)hp;
  for (size_t i = 0; i < h->path.size(); ++i) std::memcpy(wp + 8 * i, h->path[i].data(), 8 * sizeof(double));
}

// Tree dump for parity: parent ids, configs (n x 8) and costs (n x 3) of the start (which=0) or goal tree.
int orc_get_tree(void* hp, int which, int* parent, double* conf, double* cost) {
  orc_handle* h = (orc_handle*)hp;
  const orc::Tree& t = which ? h->pl->tb : h->pl->ta;
  for (size_t i = 0; i < t.nodes.size(); ++i) {
    if (parent) parent[i] = t.nodes[i].parent_id;
    if (conf) std::memcpy(conf + 8 * i, t.nodes[i].q.data(), 8 * sizeof(double));
    if (cost) { cost[3 * i] = t.nodes[i].cost.total; cost[3 * i + 1] = t.nodes[i].cost.rev; cost[3 * i + 2] = t.nodes[i].cost.prism; }
  }
  return (int)t.nodes.size();
}

// IK (getFullPoseFromEEPose -> run_VDLS_Control_Connector) for n tasks: tasks[i] = goal[7], lo[6], hi[6], q[8]
// (27 doubles), max_iter shared; out[i] = q[8], err[6], manip (15 doubles); st[i] = reached, iters, fallback.
void orc_ik_solve(void* hp, const double* tasks, int n, int max_iter, double* out, int* st) {
  orc_handle* h = (orc_handle*)hp;
  for (int i = 0; i < n; ++i) {
    orc::IkTask t;
    const double* a = tasks + (size_t)27 * i;
    std::memcpy(t.goal, a, 7 * sizeof(double));
    std::memcpy(t.lo, a + 7, 6 * sizeof(double));
    std::memcpy(t.hi, a + 13, 6 * sizeof(double));
    std::memcpy(t.q, a + 19, 8 * sizeof(double));
    t.max_iter = max_iter;
    orc::IkOut o;
    orc::ik_solve(*h->rb, t, &o);
    std::memcpy(out + (size_t)15 * i, o.q, 8 * sizeof(double));
    std::memcpy(out + (size_t)15 * i + 8, o.err, 6 * sizeof(double));
    out[(size_t)15 * i + 14] = o.manip;
    st[3 * i] = o.reached; st[3 * i + 1] = o.iters; st[3 * i + 2] = o.fallback;
  }
}

// compute_FK pose (7) and the float-cast KDL Jacobian (6 x 8, row-major) of n configurations (checker input).
void orc_ik_fk_jac(void* hp, const double* q, int n, double* ee, double* J) {
  orc_handle* h = (orc_handle*)hp;
  orc::Frame T[orc::MAX_IK_SEG + 1];
  for (int i = 0; i < n; ++i) {
    orc::chain_frames(*h->rb, q + 8 * i, T);
    if (ee) orc::ee_pose(*h->rb, T, ee + 7 * i);
    if (J) {
      double Jm[6][8];
      orc::jacobian(*h->rb, q + 8 * i, T, Jm);
      std::memcpy(J + 48 * i, Jm, sizeof(Jm));
    }
  }
}

// Goal quaternion of an end-effector pose [x, y, z, roll, pitch, yaw] (BS:1630-1645).
void orc_ik_goal(const double* ee, double* g) { orc::ik_goal_quat(ee, g); }

// Candidate tasks of findGoalPose (27 doubles each as orc_ik_solve); returns their number (tasks may be NULL).
int orc_goal_candidates(const double* ee, const double* cur, double disc_deg, double* tasks, int* downward) {
  std::vector<orc::IkTask> ts;
  int d = orc::goal_candidates(ee, cur, disc_deg, ts);
  if (downward) *downward = d;
  if (tasks)
    for (size_t i = 0; i < ts.size(); ++i) {
      double* a = tasks + 27 * i;
      std::memcpy(a, ts[i].goal, 7 * sizeof(double));
      std::memcpy(a + 7, ts[i].lo, 6 * sizeof(double));
      std::memcpy(a + 13, ts[i].hi, 6 * sizeof(double));
      std::memcpy(a + 19, ts[i].q, 8 * sizeof(double));
    }
  return (int)ts.size();
}

// Planner::findGoalPose (SP:1129-1201): candidates in order, IK then isConfigValid, first valid wins.
// Returns 0 (pose_goal set), 1 (an IK solution exists but collides) or 2 (no IK solution); info = {candidates
// tried, candidate chosen or -1, IK iterations summed over the tried candidates}.
int orc_find_goal_pose(void* hp, const double* ee, const double* cur, double disc_deg, int self, int map,
                       double* pose_goal, long long* info) {
  orc_handle* h = (orc_handle*)hp;
  std::vector<orc::IkTask> ts;
  orc::goal_candidates(ee, cur, disc_deg, ts);
  bool found = false;
  long long iters = 0;
  for (size_t i = 0; i < ts.size(); ++i) {
    orc::IkOut o;
    orc::ik_solve(*h->rb, ts[i], &o);
    iters += o.iters;
    if (o.reached) {
      found = true;
      if (!h->ck.in_collision(o.q, self, map)) {
        std::memcpy(pose_goal, o.q, 8 * sizeof(double));
        if (info) { info[0] = (long long)i + 1; info[1] = (long long)i; info[2] = iters; }
        return 0;
      }
    }
  }
  if (info) { info[0] = (long long)ts.size(); info[1] = -1; info[2] = iters; }
  return found ? 1 : 2;
}

int orc_get_cost_row_times(void* hp, double* t) {
  orc_handle* h = (orc_handle*)hp;
  if (t) for (size_t i = 0; i < h->pl->cost_row_time.size(); ++i) t[i] = h->pl->cost_row_time[i];
  return (int)h->pl->cost_row_time.size();
}

int orc_get_cost_rows(void* hp, double* rows) {
  orc_handle* h = (orc_handle*)hp;
  if (rows) for (size_t i = 0; i < h->pl->cost_rows.size(); ++i) std::memcpy(rows + 5 * i, h->pl->cost_rows[i].data(), 5 * sizeof(double));
  return (int)h->pl->cost_rows.size();
}

}  // extern "C"
