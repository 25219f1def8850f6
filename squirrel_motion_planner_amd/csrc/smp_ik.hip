// VDLS inverse-kinematics controller (gfx950): one wavefront per controller run.
//
// RobotController::run_VDLS_Control_Connector (control_laws.cpp:3283-3712) as getFullPoseFromEEPose drives it
// (birrt_star.cpp:1627-1686): per iteration the KDL Jacobian of the 12-segment chain at q (cast to float,
// control_laws.cpp:5273-5301), the manipulability measure (control_laws.cpp:6050-6089), the variable damping
// (control_laws.cpp:5557-5569), the damped pseudo-inverse applied to the error (control_laws.cpp:3455-3497), the
// joint update with the joint-limit check (control_laws.cpp:3504-3550), forward kinematics and the clamped error
// (control_laws.cpp:2167-2245).  An iteration is a dependent chain of small steps (a dependent fp64 mul / add costs ~5
// cycles on gfx950, a division ~70, an LDS round trip ~50-100: tools/micro/fp64_latency.hip), so a run stays on one
// wavefront and each step is laid out to be short and wide:
//   J    lanes 0-7: Jacobian column c (the joint rotations come from the previous FK) and, in the same
//        instruction stream, the quaternion and error component min(c, 5) of the previous FK (the goal terms in
//        registers for the whole run);
//   A    lanes 0-35: J J^T; lanes 36-41: the error column of the augmented system;
//   GJ   6 Gauss-Jordan steps on [J J^T | e] (lanes 0-41, one entry each); when det < 1e-10 tr^5 also the
//        symmetric elimination of J J^T - 1e-10 I, whose pivot signs decide the manipulability path;
//   FK   lanes 0-11: joint update of the segment's column (q_dot_c = (J^T z)_c, limit check) and the local frame
//        of every segment; lanes 0-2: one frame row each through the chain.
// Robot constants live in registers (each lane always owns the same segment / column), the iteration touches
// only LDS, and phases are separated by wavefront syncs (one wave per workgroup: no s_barrier).  Every value is
// computed with the same operations in the same order as oracle/smp_oracle.cpp (ik_solve): -ffp-contract=off,
// IEEE sqrt and division, so the two agree bit for bit.
//
// Goal search (findGoalPose, squirrel_8dof_planner.cpp:1129-1201): the candidates of one search run as one grid;
// a run that REACHED checks its pose for collision itself (collide_tile, the batch checker's tile) and, if free,
// lowers the search's `best` candidate index; a run whose index is above `best` can no longer be chosen and stops.
// Runs below `best` always finish, so the first valid candidate in the reference's order is found exactly.
#include <hip/hip_runtime.h>

#include "smp_collide.h"
#include "smp_ik.h"
#include "smp_math.h"
#include "smp_types.h"

namespace smp {

namespace {

constexpr double IK_DT = 0.1;                       // delta_t_ (control_laws.cpp:3325)
constexpr double IK_GAIN = 1.0;                     // error_gain_ (control_laws.cpp:306)
constexpr double IK_MANIP_THR = (double)0.03f;      // min_manip_treshold_ (control_laws.cpp:3299), float parameter
constexpr double IK_DAMP_MAX = (double)0.07f;       // max_damping_factor_ (control_laws.cpp:320), float parameter
constexpr double IK_SV_EPS = 0.00001;               // control_laws.cpp:6073
constexpr double IK_BOUND = 0.0001;                 // is_error_within_bounds (control_laws.cpp:6925)

struct IkLds {
  double q[NJ];
  double L[MAX_SEG][12];      // local frame joint(q) * f_tip of every segment (R row-major, p)
  double JR[MAX_SEG][9];      // joint rotation of every revolute segment (the Jacobian's joint.pose(q).M)
  double T[MAX_SEG + 1][12];  // T[0] = I, T[s+1] = T[s] * L[s]
  double J[6][NJ];
  double A[6][6];             // J J^T
  double M[6][7];             // [J J^T (+ d^2 I) | e], Gauss-Jordan in place
  double P[6][6];             // upper triangle of J J^T - 1e-10 I, eliminated in place
  double E[6][6], V[6][6];    // Jacobi fallback: eigenvalues on the diagonal, eigenvectors in the columns
  double z[6];                // (J J^T + d^2 I)^-1 e of the fallback path
  double err[6];
  double manip, damp;
  double ql[8][NJ];           // goal search: the pose to check (collide_tile input)
};

// KDL Rotation::GetQuaternion (frames.cpp), as compute_FK uses it (kdl_kuka_model.cpp:302): q = x, y, z, w.  Written
// without branches: the trace selects one of KDL's four cases, and the case's own operations are applied (the
// square root's argument, s, and per component either x * s or x / s), so that it runs in one instruction stream
// beside the Jacobian column.
__device__ __forceinline__ void get_quaternion_sel(const double* R, double* q) {
  const double trace = R[0] + R[4] + R[8];
  const bool c0 = trace > 1e-12;
  const bool c1 = !c0 && R[0] > R[4] && R[0] > R[8];
  const bool c2 = !c0 && !c1 && R[4] > R[8];
  const double a1 = 1.0 + R[0] - R[4] - R[8], a2 = 1.0 + R[4] - R[0] - R[8], a3 = 1.0 + R[8] - R[0] - R[4];
  const double r = sqrt(c0 ? trace + 1.0 : (c1 ? a1 : (c2 ? a2 : a3)));
  const double s = c0 ? 0.5 / r : 2.0 * r;
  const double d75 = R[7] - R[5], d26 = R[2] - R[6], d31 = R[3] - R[1];
  const double s13 = R[1] + R[3], s26 = R[2] + R[6], s57 = R[5] + R[7];
  const double x3 = c0 ? 0.25 : (c1 ? d75 : (c2 ? d26 : d31));
  const double x0 = c0 ? d75 : (c1 ? 0.25 : (c2 ? s13 : s26));
  const double x1 = c0 ? d26 : (c1 ? s13 : (c2 ? 0.25 : s57));
  const double x2 = c0 ? d31 : (c1 ? s26 : (c2 ? s57 : 0.25));
  const double v0 = x0 / s, v1 = x1 / s, v2 = x2 / s, m0 = x0 * s, m1 = x1 * s, m2 = x2 * s;
  q[3] = x3 / s;
  q[0] = (c0 || c1) ? m0 : v0;
  q[1] = (c0 || c2) ? m1 : v1;
  q[2] = c0 ? m2 : (c1 || c2 ? v2 : m2);
}

// Constants of the segment a lane owns in the FK (lane s < n_seg) and of the Jacobian column it owns (lane c < 8).
struct LaneConst {
  int f_ty, f_jn, f_col;  // f_col: the segment's Jacobian column (movable segments)
  double f_ax[3], f_org[3], f_R[9], f_p[3], f_lo, f_hi;
  int j_s, j_ty;
  double j_ax[3], j_fp[3];
};

__device__ __forceinline__ void load_const(const RobotDev* __restrict__ rb, int lane, LaneConst& k) {
  const int ns = rb->n_seg;
  k.f_ty = 0; k.f_jn = 0; k.f_col = 0; k.f_lo = 0.0; k.f_hi = 0.0;
  for (int d = 0; d < 3; ++d) { k.f_ax[d] = 0.0; k.f_org[d] = 0.0; k.f_p[d] = 0.0; k.j_ax[d] = 0.0; k.j_fp[d] = 0.0; }
  for (int i = 0; i < 9; ++i) k.f_R[i] = 0.0;
  if (lane < ns) {
    k.f_ty = rb->seg_type[lane];
    k.f_jn = rb->seg_joint[lane] < 0 ? 0 : rb->seg_joint[lane];
    for (int d = 0; d < 3; ++d) {
      k.f_ax[d] = rb->seg_axis[lane * 3 + d];
      k.f_org[d] = rb->seg_origin[lane * 3 + d];
      k.f_p[d] = rb->seg_p[lane * 3 + d];
    }
    for (int i = 0; i < 9; ++i) k.f_R[i] = rb->seg_R[lane * 9 + i];
    for (int s = 0; s < lane; ++s) k.f_col += rb->seg_type[s] != 0 ? 1 : 0;
    k.f_lo = rb->q_min[k.f_jn];
    k.f_hi = rb->q_max[k.f_jn];
  }
  // the lane-th movable segment
  k.j_s = 0; k.j_ty = 0;
  int c = 0;
  for (int s = 0; s < ns; ++s) {
    if (rb->seg_type[s] == 0) continue;
    if (c == lane) k.j_s = s;
    ++c;
  }
  if (lane < NJ) {
    const int s = k.j_s;
    k.j_ty = rb->seg_type[s];
    for (int d = 0; d < 3; ++d) { k.j_ax[d] = rb->seg_axis[s * 3 + d]; k.j_fp[d] = rb->seg_p[s * 3 + d]; }
  }
}

// Segment frames of S.q (ChainFkSolverPos_recursive, kdl_kuka_model.cpp:278-305 -- the same products as the T_tmp
// chain of ChainJntToJacSolver): T[0] = I, T[s+1] = T[s] * (joint(q) * f_tip).
// upd (after an iteration's solve): the lane of a movable segment first applies the joint update of its column,
// q_dot_c = (J^T z)_c and the limit check (control_laws.cpp:3455-3550), z = [J J^T (+ d^2 I) | e] solved (upd 1)
// or the fallback's z (upd 2) -- the update and the frame it moves in one step, no LDS round trip between them.
__device__ __forceinline__ void chain_fk(int ns, unsigned rid, IkLds& S, int lane, const LaneConst& k, int upd) {
  if (lane < ns) {
    double qq = S.q[k.f_jn];
    if (upd != 0 && k.f_ty != 0) {
      // (one uniform branch around all six: a select per term compiled to six branches, each one LDS round trip
      // and one division after the other)
      double z[6];
      if (upd == 1) {
        double nu[6], de[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          nu[i] = S.M[i][6];
          de[i] = S.M[i][i];
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) z[i] = nu[i] / de[i];
      } else {
#pragma unroll
        for (int i = 0; i < 6; ++i) z[i] = S.z[i];
      }
      double pz[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) pz[i] = S.J[i][k.f_col] * z[i];
      const double v = ((pz[0] + pz[1]) + (pz[2] + pz[3])) + (pz[4] + pz[5]);
      const double nv = qq + v * IK_DT;
      if (!(nv < k.f_lo || nv > k.f_hi)) {
        qq = nv;
        S.q[k.f_jn] = nv;
      }
    }
    Frame Jf;
    frame_identity(&Jf);
    if (k.f_ty == 1) {
      rot2(k.f_ax, qq, Jf.R);
      for (int d = 0; d < 3; ++d) Jf.p[d] = k.f_org[d];
      for (int i = 0; i < 9; ++i) S.JR[lane][i] = Jf.R[i];
    } else if (k.f_ty == 2) {
      for (int d = 0; d < 3; ++d) Jf.p[d] = k.f_org[d] + k.f_ax[d] * qq;
    }
    Frame F, Lf;
    for (int i = 0; i < 9; ++i) F.R[i] = k.f_R[i];
    for (int d = 0; d < 3; ++d) F.p[d] = k.f_p[d];
    fmul(Jf, F, &Lf);
    for (int i = 0; i < 9; ++i) S.L[lane][i] = Lf.R[i];
    for (int d = 0; d < 3; ++d) S.L[lane][9 + d] = Lf.p[d];
  }
  wave_sync();
  if (lane < 3) {  // row r of every T[s]: the three-term sums of KDL Frame*Frame (smp_math.h fmul)
    const int r = lane;
    double t0 = r == 0 ? 1.0 : 0.0, t1 = r == 1 ? 1.0 : 0.0, t2 = r == 2 ? 1.0 : 0.0, tp = 0.0;
    S.T[0][r * 3 + 0] = t0; S.T[0][r * 3 + 1] = t1; S.T[0][r * 3 + 2] = t2; S.T[0][9 + r] = tp;
    double l[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) l[i] = S.L[0][i];
    for (int s = 0; s < ns; ++s) {
      double ln[12];  // next local frame loaded ahead of this step's products
      const int sn = s + 1 < ns ? s + 1 : s;
#pragma unroll
      for (int i = 0; i < 12; ++i) ln[i] = S.L[sn][i];
      const double m = t0 * l[9] + t1 * l[10] + t2 * l[11];
      tp = m + tp;
      if (!((rid >> s) & 1u)) {  // else the local rotation is exactly I: the row stays (oracle chain_frames)
        const double n0 = t0 * l[0] + t1 * l[3] + t2 * l[6];
        const double n1 = t0 * l[1] + t1 * l[4] + t2 * l[7];
        const double n2 = t0 * l[2] + t1 * l[5] + t2 * l[8];
        t0 = n0; t1 = n1; t2 = n2;
      }
      S.T[s + 1][r * 3 + 0] = t0; S.T[s + 1][r * 3 + 1] = t1; S.T[s + 1][r * 3 + 2] = t2; S.T[s + 1][9 + r] = tp;
#pragma unroll
      for (int i = 0; i < 12; ++i) l[i] = ln[i];
    }
  }
  wave_sync();
}

// Lanes 0-7: KDL ChainJntToJacSolver::JntToJac column of movable segment s = T[s].M * (joint twist referred to
// the tip of s), referred to the chain tip (KDL's Twist::RefPoint(T[i+1].p - T[i].p) for every later segment i,
// telescoped); cast to float (getJacobian).
// Lanes 0-5 also: error component lane of the end-effector pose T[ns] (set_EE_goal_pose unclamped, update_error_vec
// clamped).  Returns the ballot of components outside the 1e-4 bound (is_error_within_bounds).
// The goal terms of a lane's error component (lanes 0-7: component min(lane, 5)), read once per run: in the
// iteration they were global loads on the error's dependent chain.
struct ErrConst {
  double di, g6, s0, s1, s2, lo, hi;
};

__device__ __forceinline__ void load_err_const(const IkTaskDev& t, int lane, ErrConst& ec) {
  const int i = lane < 6 ? lane : 5;
  const int rr = i < 3 ? 0 : i - 3;
  const double* g = t.goal;
  ec.di = g[i];
  ec.g6 = g[6];
  ec.s0 = rr == 0 ? 0.0 : (rr == 1 ? g[5] : -g[4]);
  ec.s1 = rr == 0 ? -g[5] : (rr == 1 ? 0.0 : g[3]);
  ec.s2 = rr == 0 ? g[4] : (rr == 1 ? -g[3] : 0.0);
  ec.lo = t.lo[i];
  ec.hi = t.hi[i];
}

__device__ __forceinline__ unsigned long long jacobian_and_error(int ns, const ErrConst& ec, IkLds& S, int lane,
                                                                 const LaneConst& k, bool clamp) {
  bool out = false;
  if (lane < NJ) {
    // error component i (lanes 6 and 7 repeat component 5 and keep it to themselves) in the same instruction stream
    // as the Jacobian column: the two dependent chains overlap instead of running as two divergent lane groups
    const int i = lane < 6 ? lane : 5;
    const double* E = S.T[ns];
    double c[7] = {E[9], E[10], E[11], 0.0, 0.0, 0.0, 0.0};
    get_quaternion_sel(E, &c[3]);
    const int rr = i < 3 ? 0 : i - 3;
    const double ci = i < 3 ? (i == 0 ? c[0] : (i == 1 ? c[1] : c[2])) : (rr == 0 ? c[3] : (rr == 1 ? c[4] : c[5]));
    const double di = ec.di;
    const double e_lin = di - ci;
    const double e_rot = c[6] * di - ec.g6 * ci - (ec.s0 * c[3] + ec.s1 * c[4] + ec.s2 * c[5]);
    double e = i < 3 ? e_lin : e_rot;
    if (clamp) e = (e < ec.lo || e > ec.hi) ? e : 0.0;

    const int s = k.j_s;
    double M[9];
#pragma unroll
    for (int x = 0; x < 9; ++x) {
      const double jr = S.JR[s][x];  // (unwritten for a prismatic segment: not selected)
      M[x] = k.j_ty == 1 ? jr : (x % 4 == 0 ? 1.0 : 0.0);
    }
    double v[3], rl[3], vl[3];
    for (int r = 0; r < 3; ++r) v[r] = M[r * 3 + 0] * k.j_fp[0] + M[r * 3 + 1] * k.j_fp[1] + M[r * 3 + 2] * k.j_fp[2];
    for (int d = 0; d < 3; ++d) {
      rl[d] = k.j_ty == 1 ? k.j_ax[d] * 1.0 : 0.0;
      vl[d] = k.j_ty == 2 ? k.j_ax[d] * 1.0 : 0.0;
    }
    const double c0 = rl[1] * v[2] - rl[2] * v[1], c1 = rl[2] * v[0] - rl[0] * v[2], c2 = rl[0] * v[1] - rl[1] * v[0];
    vl[0] = vl[0] + c0; vl[1] = vl[1] + c1; vl[2] = vl[2] + c2;
    const double* B = S.T[s];
    double vel[3], rot[3];
    for (int r = 0; r < 3; ++r) {
      vel[r] = B[r * 3 + 0] * vl[0] + B[r * 3 + 1] * vl[1] + B[r * 3 + 2] * vl[2];
      rot[r] = B[r * 3 + 0] * rl[0] + B[r * 3 + 1] * rl[1] + B[r * 3 + 2] * rl[2];
    }
    // referred to the chain tip: KDL's RefPoint offsets to every later tip telescope to T[ns].p - T[s+1].p
    {
      const double d0 = S.T[ns][9] - S.T[s + 1][9], d1 = S.T[ns][10] - S.T[s + 1][10], d2 = S.T[ns][11] - S.T[s + 1][11];
      const double x0 = rot[1] * d2 - rot[2] * d1, x1 = rot[2] * d0 - rot[0] * d2, x2 = rot[0] * d1 - rot[1] * d0;
      vel[0] = vel[0] + x0; vel[1] = vel[1] + x1; vel[2] = vel[2] + x2;
    }
    for (int d = 0; d < 3; ++d) {
      S.J[d][lane] = (double)(float)vel[d];
      S.J[3 + d][lane] = (double)(float)rot[d];
    }
    if (lane < 6) {
      S.err[i] = e;
      out = fabs(e) > IK_BOUND;
    }
  }
  const unsigned long long b = __ballot(out);
  wave_sync();
  return b;
}

// Cyclic Jacobi eigen-decomposition of the symmetric 6x6 A (rows p < q in order, at most 30 sweeps): eigenvalues
// on the diagonal of a, eigenvectors in the columns of V; one lane.
__device__ void jacobi_eigen6(const double (*A)[6], double (*a)[6], double (*V)[6]) {
  for (int i = 0; i < 6; ++i)
    for (int k = 0; k < 6; ++k) {
      a[i][k] = A[i][k];
      V[i][k] = i == k ? 1.0 : 0.0;
    }
  for (int sweep = 0; sweep < 30; ++sweep) {
    double off = 0.0;
    for (int p = 0; p < 5; ++p)
      for (int q = p + 1; q < 6; ++q) off = off + a[p][q] * a[p][q];
    if (off == 0.0) break;
    for (int p = 0; p < 5; ++p)
      for (int q = p + 1; q < 6; ++q) {
        const double apq = a[p][q];
        if (apq == 0.0) continue;
        const double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
        const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 6; ++k) {
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
          if (k == p || k == q) continue;
          const double akp = a[k][p], akq = a[k][q];
          const double np = c * akp - s * akq, nq = s * akp + c * akq;
          a[k][p] = np; a[p][k] = np; a[k][q] = nq; a[q][k] = nq;
        }
        const double app = a[p][p] - t * apq, aqq = a[q][q] + t * apq;
        a[p][p] = app; a[q][q] = aqq; a[p][q] = 0.0; a[q][p] = 0.0;
      }
  }
}

// Upper-triangle entry (i, j), i <= j, of shifted-elimination lane u (u < 21).
__device__ __forceinline__ void upper_pair(int u, int* i, int* j) {
  int r = 0, base = 0;
  while (u >= base + (6 - r)) { base += 6 - r; ++r; }
  *i = r;
  *j = r + (u - base);
}

}  // namespace

#ifdef SMP_IK_PROF
// Phase clocks (s_memtime) of block 0's iterations: tools/ik_phase_probe.py (profiling build only).
__device__ unsigned long long g_ik_prof[8];
#define IKP(k)                                                                \
  if (lane == 0 && b == 0) {                                                  \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();               \
    _pf[k] += _t - _tp;                                                       \
    _tp = _t;                                                                 \
  }
#else
#define IKP(k)
#endif

// One controller run per wavefront (block = 64 threads).  SEARCH: goal-search mode (collision check of a REACHED
// pose, `best` candidate index shared by the grid, runs that can no longer be chosen stop).
template <bool SEARCH>
__global__ void __launch_bounds__(IK_THREADS) ik_kernel_t(const RobotDev* __restrict__ rb,
                                                          const IkTaskDev* __restrict__ tasks, int n,
                                                          IkOutDev* __restrict__ out, SceneDev sc,
                                                          const MapCfg* __restrict__ mc, int self, int map, int* best) {
  __shared__ IkLds S;
  __shared__ TileLds<8> TL;
  const int lane = threadIdx.x;
  const int b = blockIdx.x;
  if (b >= n) return;
  const IkTaskDev& t = tasks[b];
  const int ns = rb->n_seg;
  LaneConst k;
  load_const(rb, lane, k);
  ErrConst ec;
  load_err_const(t, lane, ec);
  const int max_iter = t.max_iter;
  const double tau = IK_SV_EPS * IK_SV_EPS;
  // main Gauss-Jordan lane (gi, gj) of the 6 x 7 system, or shifted-elimination lane (si, sj) of the upper triangle
  const int gi = lane / 7, gj = lane - 7 * (lane / 7);
  int si = 0, sj = 0;
  const bool sh = lane < 21;
  if (sh) upper_pair(lane, &si, &sj);
  // segments whose local rotation is exactly I (no revolute joint, identity f_tip rotation)
  unsigned rid = 0;
  for (int s = 0; s < ns; ++s) {
    bool id = rb->seg_type[s] != 1;
    for (int i = 0; i < 9; ++i) id = id && rb->seg_R[s * 9 + i] == ((i % 4 == 0) ? 1.0 : 0.0);
    rid |= id ? 1u << s : 0u;
  }
  if (lane < NJ) S.q[lane] = t.q[lane];
  wave_sync();
  chain_fk(ns, rid, S, lane, k, 0);
  int iter = 0, fallback = 0, abandoned = 0;
#ifdef SMP_IK_PROF
  unsigned long long _pf[8] = {0, 0, 0, 0, 0, 0, 0, 0}, _tp = __builtin_amdgcn_s_memtime();
#endif
  while (true) {
    const unsigned long long outb = jacobian_and_error(ns, ec, S, lane, k, iter > 0);
    IKP(0);
    if (iter > 0) {
      if (iter == max_iter) break;
      if (outb == 0ull) break;
    }
    // goal search: read the best candidate now, act on it after this iteration (the load overlaps the iteration)
    int bst = 0x7fffffff;
    if (SEARCH) bst = __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // J J^T, the augmented error column, the shifted upper triangle
    if (lane < 36) {
      const int i = lane / 6, c = lane - 6 * (lane / 6);
      double pp[NJ];
#pragma unroll
      for (int x = 0; x < NJ; ++x) pp[x] = S.J[i][x] * S.J[c][x];
      const double s = ((pp[0] + pp[1]) + (pp[2] + pp[3])) + ((pp[4] + pp[5]) + (pp[6] + pp[7]));
      S.A[i][c] = s;
      S.M[i][c] = s;
      if (i <= c) S.P[i][c] = i == c ? s + (-tau) : s;
    } else if (lane < 42) {
      S.M[lane - 36][6] = 0.0 + IK_GAIN * S.err[lane - 36];
    }
    wave_sync();
    IKP(1);
    // Gauss-Jordan on [A | e]; every lane multiplies the pivots
    double pr = 1.0;
    for (int s = 0; s < 6; ++s) {
      pr = pr * S.M[s][s];
      if (lane < 42 && gi != s && gj > s) {
        const double f = S.M[gi][s] / S.M[s][s];
        S.M[gi][gj] = S.M[gi][gj] - f * S.M[s][gj];
      }
      wave_sync();
    }
    IKP(2);
    // computeManipulabilityMeasure (control_laws.cpp:6050-6089) and the damping (control_laws.cpp:5557-5569): every
    // singular value exceeds 1e-5 if det A > tau tr(A)^5, else exactly when A - tau I is positive definite (the
    // symmetric elimination of its upper triangle, lanes 0-20; rare)
    const double tr = ((((S.A[0][0] + S.A[1][1]) + S.A[2][2]) + S.A[3][3]) + S.A[4][4]) + S.A[5][5];
    const double tr5 = (((tr * tr) * tr) * tr) * tr;
    bool normal = pr > tau * tr5;
    if (!normal) {
      for (int s = 0; s < 6; ++s) {
        if (sh && si > s) {
          const double f = S.P[s][si] / S.P[s][s];
          S.P[si][sj] = S.P[si][sj] - f * S.P[s][sj];
        }
        wave_sync();
      }
      normal = true;
#pragma unroll
      for (int s = 0; s < 6; ++s) normal = normal && S.P[s][s] > 0.0;
    }
    double m_all = sqrt(pr), d_all = 0.0;  // the normal path's manipulability and damping, in every lane
    if (m_all == 1.0 || m_all < 0.00001) m_all = 0.0001;
    if (m_all < IK_MANIP_THR) d_all = IK_DAMP_MAX * ((1 - (m_all / IK_MANIP_THR)) * (1 - (m_all / IK_MANIP_THR)));
    if (!normal && lane == 0) {
      double m;
      {
        jacobi_eigen6(S.A, S.E, S.V);
        m = 1.0;
        for (int j = 0; j < 6; ++j) {
          const double lam = S.E[j][j];
          const double sv = sqrt(lam > 0.0 ? lam : 0.0);
          if (fabs(sv) > IK_SV_EPS) m = m * fabs(sv);
        }
      }
      if (m == 1.0 || m < 0.00001) m = 0.0001;
      double d = 0.0;
      if (m < IK_MANIP_THR) d = IK_DAMP_MAX * ((1 - (m / IK_MANIP_THR)) * (1 - (m / IK_MANIP_THR)));
      if (!normal) {
        double ep[6], g[6];
        for (int i = 0; i < 6; ++i) ep[i] = 0.0 + IK_GAIN * S.err[i];
        for (int i = 0; i < 6; ++i) {
          double tt = S.V[0][i] * ep[0];
          for (int j = 1; j < 6; ++j) tt = tt + S.V[j][i] * ep[j];
          g[i] = (1.0 / ((S.E[i][i] > 0.0 ? S.E[i][i] : 0.0) + d * d)) * tt;
        }
        for (int r = 0; r < 6; ++r) {
          double y = g[0] * S.V[r][0];
          for (int i = 1; i < 6; ++i) y = y + g[i] * S.V[r][i];
          S.z[r] = y;
        }
      }
      S.manip = m;
      S.damp = d;
    }
    fallback += normal ? 0 : 1;
    if (!normal) wave_sync();
    const double damp = normal ? d_all : S.damp;
    if (normal && lane == 0) S.manip = m_all;
    IKP(3);
    if (normal && damp != 0.0) {  // damped system (A + d^2 I) z = e
      if (lane < 36) {
        const int i = lane / 6, c = lane - 6 * (lane / 6);
        S.M[i][c] = i == c ? S.A[i][i] + damp * damp : S.A[i][c];
      } else if (lane < 42) {
        S.M[lane - 36][6] = 0.0 + IK_GAIN * S.err[lane - 36];
      }
      wave_sync();
      for (int s = 0; s < 6; ++s) {
        if (lane < 42 && gi != s && gj > s) {
          const double f = S.M[gi][s] / S.M[s][s];
          S.M[gi][gj] = S.M[gi][gj] - f * S.M[s][gj];
        }
        wave_sync();
      }
    }
    IKP(4);
    // q_dot = J_vdls e = J^T z (control_laws.cpp:3455-3497), joint update with the limit check (:3504-3550), FK
    chain_fk(ns, rid, S, lane, k, normal ? 1 : 2);
    IKP(5);
    ++iter;
    if (SEARCH && bst < b) {  // a lower candidate is REACHED and valid: this run can no longer be chosen
      abandoned = 1;
      break;
    }
  }
  const int reached = (abandoned || iter == max_iter) ? 0 : 1;
  int flags = abandoned ? IK_ABANDONED : 0;
  if (SEARCH && reached) {
    if (lane < NJ) S.ql[0][lane] = S.q[lane];
    __syncthreads();
    collide_tile<8>(rb, sc, mc, 1, S.ql, self, map, TL);
    flags |= IK_CHECKED | (TL.coll[0] ? 0 : IK_VALID);
    if (lane == 0 && !TL.coll[0]) __hip_atomic_fetch_min(best, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#ifdef SMP_IK_PROF
  if (lane == 0 && b == 0) {
    for (int i = 0; i < 6; ++i) g_ik_prof[i] += _pf[i];
    g_ik_prof[6] += iter;
  }
#endif
  IkOutDev& o = out[b];
  if (lane < NJ) o.q[lane] = S.q[lane];
  if (lane < 6) o.err[lane] = S.err[lane];
  if (lane == 0) {
    o.manip = S.manip;
    o.reached = reached;
    o.iters = iter;
    o.fallback = fallback;
    o.flags = flags;
  }
}

void launch_ik(bool search, int n, hipStream_t st, const RobotDev* rb, const IkTaskDev* tasks, IkOutDev* out,
               SceneDev sc, const MapCfg* mc, int self, int map, int* best) {
  if (search)
    hipLaunchKernelGGL(ik_kernel_t<true>, dim3(n), dim3(IK_THREADS), 0, st, rb, tasks, n, out, sc, mc, self, map, best);
  else
    hipLaunchKernelGGL(ik_kernel_t<false>, dim3(n), dim3(IK_THREADS), 0, st, rb, tasks, n, out, sc, mc, self, map,
                       best);
}

#ifdef SMP_IK_PROF
extern "C" int smp_probe_ik_prof(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ik_prof), sizeof(g_ik_prof)) != hipSuccess) return -5;
  static const unsigned long long zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_ik_prof), zero, sizeof(zero)) == hipSuccess ? 0 : -5;
}
#endif

size_t ik_kernels_private_bytes() {
  size_t need = 0;
  hipFuncAttributes fa;
  const void* ks[] = {reinterpret_cast<const void*>(&ik_kernel_t<false>), reinterpret_cast<const void*>(&ik_kernel_t<true>)};
  for (const void* kk : ks)
    if (hipFuncGetAttributes(&fa, kk) == hipSuccess && (size_t)fa.localSizeBytes > need) need = fa.localSizeBytes;
  return need;
}

}  // namespace smp
