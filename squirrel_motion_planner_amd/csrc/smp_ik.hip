// VDLS inverse-kinematics controller (gfx950): one wavefront per controller run.
//
// RobotController::run_VDLS_Control_Connector (control_laws.cpp:3283-3712) as getFullPoseFromEEPose drives it
// (birrt_star.cpp:1627-1686): per iteration the KDL Jacobian of the 12-segment chain at q (cast to float,
// control_laws.cpp:5273-5301), the manipulability measure (control_laws.cpp:6050-6089), the variable damping
// (control_laws.cpp:5557-5569), the damped pseudo-inverse applied to the error (control_laws.cpp:3455-3497), the
// joint update with the joint-limit check (control_laws.cpp:3504-3550), forward kinematics and the clamped error
// (control_laws.cpp:2167-2245).  The work of an iteration is a dependent chain of small steps (a 12-frame product,
// 6x6 Cholesky columns, triangular solves), so a run stays on one wavefront and spreads each step over its lanes:
// local frames per segment, frame rows per lane, Jacobian columns per lane, J J^T entries per lane, Cholesky rows
// per lane (the plain and the shifted factorization side by side), solve columns per lane.  Every value is
// computed with the same operations in the same order as oracle/smp_oracle.cpp (ik_solve), so the two agree bit
// for bit (-ffp-contract=off, IEEE sqrt and division).
#include <hip/hip_runtime.h>

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
  double T[MAX_SEG + 1][12];  // T[0] = I, T[s+1] = T[s] * L[s]
  double dl[MAX_SEG][3];      // T[s+1].p - T[s].p (Twist::RefPoint offsets)
  double J[6][NJ];
  double A[6][6];             // J J^T
  double C[2][6][6];          // Cholesky factors: [0] of A (+ d^2 I), [1] of A - 1e-10 I
  double piv_ok[2][6];
  double ee[7];
  double err[6];
  double manip, damp;
  int mov[NJ];                // segment of Jacobian column c
};

// KDL Rotation::GetQuaternion (frames.cpp), as compute_FK uses it (kdl_kuka_model.cpp:302).
__device__ __forceinline__ void get_quaternion(const double* R, double* q) {
  double trace = R[0] + R[4] + R[8];
  if (trace > 1e-12) {
    double s = 0.5 / sqrt(trace + 1.0);
    q[3] = 0.25 / s;
    q[0] = (R[7] - R[5]) * s;
    q[1] = (R[2] - R[6]) * s;
    q[2] = (R[3] - R[1]) * s;
  } else if (R[0] > R[4] && R[0] > R[8]) {
    double s = 2.0 * sqrt(1.0 + R[0] - R[4] - R[8]);
    q[3] = (R[7] - R[5]) / s;
    q[0] = 0.25 * s;
    q[1] = (R[1] + R[3]) / s;
    q[2] = (R[2] + R[6]) / s;
  } else if (R[4] > R[8]) {
    double s = 2.0 * sqrt(1.0 + R[4] - R[0] - R[8]);
    q[3] = (R[2] - R[6]) / s;
    q[0] = (R[1] + R[3]) / s;
    q[1] = 0.25 * s;
    q[2] = (R[5] + R[7]) / s;
  } else {
    double s = 2.0 * sqrt(1.0 + R[8] - R[0] - R[4]);
    q[3] = (R[3] - R[1]) / s;
    q[0] = (R[2] + R[6]) / s;
    q[1] = (R[5] + R[7]) / s;
    q[2] = 0.25 * s;
  }
}

// Segment frames of q (ChainFkSolverPos_recursive, kdl_kuka_model.cpp:278-305, and the T_tmp chain of
// ChainJntToJacSolver) and the end-effector pose [x, y, z, qx, qy, qz, qw].
__device__ __forceinline__ void chain_fk(const RobotDev* __restrict__ rb, IkLds& S, int lane) {
  const int ns = rb->n_seg;
  if (lane < ns) {
    const int s = lane;
    Frame J;
    for (int i = 0; i < 9; ++i) J.R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    J.p[0] = J.p[1] = J.p[2] = 0.0;
    const int ty = rb->seg_type[s];
    if (ty == 1) {
      rot2(&rb->seg_axis[s * 3], S.q[rb->seg_joint[s]], J.R);
      for (int d = 0; d < 3; ++d) J.p[d] = rb->seg_origin[s * 3 + d];
    } else if (ty == 2) {
      const double qq = S.q[rb->seg_joint[s]];
      for (int d = 0; d < 3; ++d) J.p[d] = rb->seg_origin[s * 3 + d] + rb->seg_axis[s * 3 + d] * qq;
    }
    Frame F, Lf;
    for (int i = 0; i < 9; ++i) F.R[i] = rb->seg_R[s * 9 + i];
    for (int d = 0; d < 3; ++d) F.p[d] = rb->seg_p[s * 3 + d];
    fmul(J, F, &Lf);
    for (int i = 0; i < 9; ++i) S.L[s][i] = Lf.R[i];
    for (int d = 0; d < 3; ++d) S.L[s][9 + d] = Lf.p[d];
  }
  __syncthreads();
  if (lane < 3) {  // row r of every T[s]: the three-term sums of KDL Frame*Frame (smp_math.h fmul)
    const int r = lane;
    double t0 = r == 0 ? 1.0 : 0.0, t1 = r == 1 ? 1.0 : 0.0, t2 = r == 2 ? 1.0 : 0.0, tp = 0.0;
    S.T[0][r * 3 + 0] = t0; S.T[0][r * 3 + 1] = t1; S.T[0][r * 3 + 2] = t2; S.T[0][9 + r] = tp;
    for (int s = 0; s < ns; ++s) {
      const double* Lr = S.L[s];
      double n0 = t0 * Lr[0] + t1 * Lr[3] + t2 * Lr[6];
      double n1 = t0 * Lr[1] + t1 * Lr[4] + t2 * Lr[7];
      double n2 = t0 * Lr[2] + t1 * Lr[5] + t2 * Lr[8];
      double m = t0 * Lr[9] + t1 * Lr[10] + t2 * Lr[11];
      tp = m + tp;
      t0 = n0; t1 = n1; t2 = n2;
      S.T[s + 1][r * 3 + 0] = t0; S.T[s + 1][r * 3 + 1] = t1; S.T[s + 1][r * 3 + 2] = t2; S.T[s + 1][9 + r] = tp;
    }
  }
  __syncthreads();
  if (lane == 0) {
    const double* E = S.T[ns];
    S.ee[0] = E[9]; S.ee[1] = E[10]; S.ee[2] = E[11];
    get_quaternion(E, &S.ee[3]);
  }
  __syncthreads();
}

// Cartesian error (set_EE_goal_pose control_laws.cpp:1689-1720 unclamped; update_error_vec
// control_laws.cpp:2203-2239 clamped to zero inside the deviation band).  Returns 1 if every component is within
// 1e-4 (is_error_within_bounds).  Uniform across the wavefront.
__device__ __forceinline__ int ik_error(const IkTaskDev& t, IkLds& S, int lane, bool clamp) {
  double e = 0.0;
  if (lane < 6) {
    const double* d = t.goal;
    const double* c = S.ee;
    if (lane < 3) {
      e = d[lane] - c[lane];
    } else {
      const int i = lane - 3;
      const double s0 = i == 0 ? 0.0 : (i == 1 ? d[5] : -d[4]);
      const double s1 = i == 0 ? -d[5] : (i == 1 ? 0.0 : d[3]);
      const double s2 = i == 0 ? d[4] : (i == 1 ? -d[3] : 0.0);
      e = c[6] * d[lane] - d[6] * c[lane] - (s0 * c[3] + s1 * c[4] + s2 * c[5]);
    }
    if (clamp) e = (e < t.lo[lane] || e > t.hi[lane]) ? e : 0.0;
    S.err[lane] = e;
  }
  const unsigned long long out = __ballot(lane < 6 && fabs(e) > IK_BOUND);
  __syncthreads();
  return out == 0ull;
}

// KDL ChainJntToJacSolver::JntToJac: column c (lane c) = T[s].M * (joint twist referred to the tip of segment s),
// then Twist::RefPoint(T[i+1].p - T[i].p) for every later segment i; cast to float (getJacobian).
__device__ __forceinline__ void jacobian(const RobotDev* __restrict__ rb, IkLds& S, int lane) {
  const int ns = rb->n_seg;
  if (lane < 3 * ns) {
    const int s = lane / 3, d = lane - 3 * s;
    S.dl[s][d] = S.T[s + 1][9 + d] - S.T[s][9 + d];
  }
  __syncthreads();
  if (lane < NJ) {
    const int s = S.mov[lane];
    const int ty = rb->seg_type[s];
    const double* ax = &rb->seg_axis[s * 3];
    double M[9] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0};
    if (ty == 1) rot2(ax, S.q[rb->seg_joint[s]], M);
    const double* fp = &rb->seg_p[s * 3];
    double v[3], rl[3], vl[3];
    for (int r = 0; r < 3; ++r) v[r] = M[r * 3 + 0] * fp[0] + M[r * 3 + 1] * fp[1] + M[r * 3 + 2] * fp[2];
    for (int d = 0; d < 3; ++d) {
      rl[d] = ty == 1 ? ax[d] * 1.0 : 0.0;
      vl[d] = ty == 2 ? ax[d] * 1.0 : 0.0;
    }
    const double c0 = rl[1] * v[2] - rl[2] * v[1], c1 = rl[2] * v[0] - rl[0] * v[2], c2 = rl[0] * v[1] - rl[1] * v[0];
    vl[0] = vl[0] + c0; vl[1] = vl[1] + c1; vl[2] = vl[2] + c2;
    const double* B = S.T[s];
    double vel[3], rot[3];
    for (int r = 0; r < 3; ++r) {
      vel[r] = B[r * 3 + 0] * vl[0] + B[r * 3 + 1] * vl[1] + B[r * 3 + 2] * vl[2];
      rot[r] = B[r * 3 + 0] * rl[0] + B[r * 3 + 1] * rl[1] + B[r * 3 + 2] * rl[2];
    }
    for (int i = s + 1; i < ns; ++i) {
      const double d0 = S.dl[i][0], d1 = S.dl[i][1], d2 = S.dl[i][2];
      const double x0 = rot[1] * d2 - rot[2] * d1, x1 = rot[2] * d0 - rot[0] * d2, x2 = rot[0] * d1 - rot[1] * d0;
      vel[0] = vel[0] + x0; vel[1] = vel[1] + x1; vel[2] = vel[2] + x2;
    }
    for (int d = 0; d < 3; ++d) {
      S.J[d][lane] = (double)(float)vel[d];
      S.J[3 + d][lane] = (double)(float)rot[d];
    }
  }
  __syncthreads();
}

// Cholesky of A + shift I, column by column: lanes g*8 + i (i < 6) own row i of factor g (g < ng).
// Pivot flags piv_ok[g][j] = (pivot > 0).
__device__ __forceinline__ void cholesky(IkLds& S, int lane, int ng, double shift0, double shift1) {
  const int g = lane >> 3, i = lane & 7;
  const bool act = g < ng && i < 6;
  const double shift = g == 0 ? shift0 : shift1;
  double(*L)[6] = S.C[g < 2 ? g : 0];
  for (int j = 0; j < 6; ++j) {
    double s = 0.0;
    if (act && i >= j) {
      s = i == j ? S.A[i][j] + shift : S.A[i][j];
      for (int k = 0; k < j; ++k) s = s - L[i][k] * L[j][k];
      if (i == j) {
        S.piv_ok[g][j] = (s > 0.0) ? 1.0 : 0.0;
        L[j][j] = sqrt(s);
      }
    }
    __syncthreads();
    if (act && i > j) L[i][j] = s / L[j][j];
    __syncthreads();
  }
}

// Cyclic Jacobi eigen-decomposition of the symmetric 6x6 A (rows p < q in order, at most 30 sweeps): eigenvalues
// on the diagonal of the LDS scratch a, eigenvectors in the columns of V; one lane.
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

}  // namespace

__global__ void __launch_bounds__(IK_THREADS) ik_kernel(const RobotDev* __restrict__ rb,
                                                        const IkTaskDev* __restrict__ tasks, int n,
                                                        IkOutDev* __restrict__ out) {
  __shared__ IkLds S;
  __shared__ double Eg[6][6], Ev[6][6], coef[6];  // Jacobi fallback: eigenvalues (diagonal), eigenvectors, 1/(s^2+d^2)
  const int lane = threadIdx.x;
  const int b = blockIdx.x;
  if (b >= n) return;
  const IkTaskDev& t = tasks[b];
  const int ns = rb->n_seg;
  if (lane < NJ) S.q[lane] = t.q[lane];
  if (lane == 0) {
    int c = 0;
    for (int s = 0; s < ns && c < NJ; ++s)
      if (rb->seg_type[s] != 0) S.mov[c++] = s;
  }
  __syncthreads();
  chain_fk(rb, S, lane);
  int within = 0;
  ik_error(t, S, lane, false);  // set_EE_goal_pose: error_within_bounds stays false (control_laws.cpp:3328)
  int iter = 0, fallback = 0;
  const double tau = IK_SV_EPS * IK_SV_EPS;
  while (!within) {
    jacobian(rb, S, lane);
    if (lane < 36) {
      const int i = lane / 6, k = lane - 6 * (lane / 6);
      double s = S.J[i][0] * S.J[k][0];
      for (int c = 1; c < NJ; ++c) s = s + S.J[i][c] * S.J[k][c];
      S.A[i][k] = s;
    }
    __syncthreads();
    cholesky(S, lane, 2, 0.0, -tau);
    // computeManipulabilityMeasure (control_laws.cpp:6050-6089)
    bool normal = true;
    for (int j = 0; j < 6; ++j) normal = normal && S.piv_ok[1][j] != 0.0;
    if (lane == 0) {
      double m = 1.0;
      if (normal) {
        for (int j = 0; j < 6; ++j) m = m * S.C[0][j][j];
      } else {
        jacobi_eigen6(S.A, Eg, Ev);
        for (int j = 0; j < 6; ++j) {
          const double lam = Eg[j][j];
          const double sv = sqrt(lam > 0.0 ? lam : 0.0);
          if (fabs(sv) > IK_SV_EPS) m = m * fabs(sv);
        }
      }
      if (m == 1.0 || m < 0.00001) m = 0.0001;
      double d = 0.0;
      if (m < IK_MANIP_THR) d = IK_DAMP_MAX * ((1 - (m / IK_MANIP_THR)) * (1 - (m / IK_MANIP_THR)));
      S.manip = m;
      S.damp = d;
      if (!normal)
        for (int i = 0; i < 6; ++i) coef[i] = 1.0 / ((Eg[i][i] > 0.0 ? Eg[i][i] : 0.0) + d * d);
    }
    fallback += normal ? 0 : 1;
    __syncthreads();
    const double damp = S.damp;
    if (normal && damp != 0.0) cholesky(S, lane, 1, damp * damp, 0.0);
    // damped pseudo-inverse times the error (control_laws.cpp:3455-3497), then the joint update with the limit
    // check (control_laws.cpp:3504-3550): lane c owns column c of (A + d^2 I)^-1 J, i.e. row c of J_vdls -- by the
    // Cholesky factor, or (a singular value <= 1e-5) sum_i (J^T u_i)_c u_i / (max(lambda_i, 0) + d^2)
    if (lane < NJ) {
      double x[6];
      if (normal) {
        const double(*L)[6] = S.C[0];
        double y[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          double s = S.J[i][lane];
#pragma unroll
          for (int k = 0; k < i; ++k) s = s - L[i][k] * y[k];
          y[i] = s / L[i][i];
        }
#pragma unroll
        for (int i = 5; i >= 0; --i) {
          double s = y[i];
#pragma unroll
          for (int k = i + 1; k < 6; ++k) s = s - L[k][i] * x[k];
          x[i] = s / L[i][i];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 6; ++j) x[j] = 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          double w = S.J[0][lane] * Ev[0][i];
#pragma unroll
          for (int k = 1; k < 6; ++k) w = w + S.J[k][lane] * Ev[k][i];
          const double cw = coef[i] * w;
#pragma unroll
          for (int j = 0; j < 6; ++j) x[j] = x[j] + cw * Ev[j][i];
        }
      }
      double v = 0.0;
#pragma unroll
      for (int j = 0; j < 6; ++j) v = v + x[j] * (0.0 + IK_GAIN * S.err[j]);
      const int s = S.mov[lane];
      const int jn = rb->seg_joint[s];
      const double nv = S.q[jn] + v * IK_DT;
      if (!(nv < rb->q_min[jn] || nv > rb->q_max[jn])) S.q[jn] = nv;
    }
    __syncthreads();
    chain_fk(rb, S, lane);
    within = ik_error(t, S, lane, true);
    ++iter;
    if (iter == t.max_iter) break;
  }
  IkOutDev& o = out[b];
  if (lane < NJ) o.q[lane] = S.q[lane];
  if (lane < 6) o.err[lane] = S.err[lane];
  if (lane == 0) {
    o.manip = S.manip;
    o.reached = iter == t.max_iter ? 0 : 1;
    o.iters = iter;
    o.fallback = fallback;
    o.pad = 0;
  }
}

// Gathers the final configurations of n runs into the structure-of-arrays layout of the batch check kernel.
__global__ void ik_gather_kernel(const IkOutDev* __restrict__ out, int n, double* __restrict__ q_soa) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n * NJ) {
    const int c = i / NJ, j = i - c * NJ;
    q_soa[(size_t)j * n + c] = out[c].q[j];
  }
}

size_t ik_kernels_private_bytes() {
  size_t need = 0;
  hipFuncAttributes fa;
  const void* ks[] = {reinterpret_cast<const void*>(&ik_kernel), reinterpret_cast<const void*>(&ik_gather_kernel)};
  for (const void* k : ks)
    if (hipFuncGetAttributes(&fa, k) == hipSuccess && (size_t)fa.localSizeBytes > need) need = fa.localSizeBytes;
  return need;
}

}  // namespace smp
