// Shared fp64 arithmetic of the planner hot path (device kernels + host-side output assembly).
//
// Every function fixes an evaluation order so that the HIP path and the CPU oracle agree bit for bit.
// Build with -ffp-contract=off (no FMA contraction) and without fast-math.  KDL formulas follow
// orocos_kdl frames.inl / frames.cpp (Frame*Frame, Rotation::Rot2), which the reference uses through
// ChainFkSolverPos_recursive (kdl_kuka_model.cpp:278-305) and collision_checker.hpp:519-539.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SMP_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#define SMP_HD static inline
#endif

namespace smp {

struct Frame {
  double R[9];
  double p[3];
};

// Portable sin/cos: Cody-Waite reduction by pi/2 (3-part constant) + fdlibm minimax kernels.
// glibc and ocml differ by an ulp for some inputs, so neither is used on the FK path.
SMP_HD void psincos(double x, double* s, double* c) {
  const double inv_pio2 = 6.36619772367581382433e-01;
  const double pio2_1 = 1.57079632673412561417e+00;
  const double pio2_2 = 6.07710050630396597660e-11;
  const double pio2_3 = 2.02226624871116645580e-21;
  double fn = floor(x * inv_pio2 + 0.5);
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
  int q = (int)(n & 3);
  double ss = q == 0 ? sr : (q == 1 ? cr : (q == 2 ? -sr : -cr));
  double cc = q == 0 ? cr : (q == 1 ? -sr : (q == 2 ? -cr : sr));
  *s = ss;
  *c = cc;
}

SMP_HD void frame_identity(Frame* f) {
  for (int i = 0; i < 9; ++i) f->R[i] = (i % 4 == 0) ? 1.0 : 0.0;
  f->p[0] = f->p[1] = f->p[2] = 0.0;
}

// KDL Frame operator*: (M1*M2, M1*p2 + p1)
SMP_HD void fmul(const Frame& a, const Frame& b, Frame* o) {
  Frame t;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      t.R[r * 3 + c] = a.R[r * 3 + 0] * b.R[0 * 3 + c] + a.R[r * 3 + 1] * b.R[1 * 3 + c] + a.R[r * 3 + 2] * b.R[2 * 3 + c];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    double m = a.R[r * 3 + 0] * b.p[0] + a.R[r * 3 + 1] * b.p[1] + a.R[r * 3 + 2] * b.p[2];
    t.p[r] = m + a.p[r];
  }
  *o = t;
}

// KDL Frame * Vector
SMP_HD void xform(const Frame& F, const double* c, double* o) {
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    double m = F.R[r * 3 + 0] * c[0] + F.R[r * 3 + 1] * c[1] + F.R[r * 3 + 2] * c[2];
    o[r] = m + F.p[r];
  }
}

// KDL Rotation::Rot2(axis, angle) from sin/cos of the angle
SMP_HD void rot2_sc(const double* ax, double st, double ct, double* R) {
  double vt = 1 - ct;
  double m_vt_0 = vt * ax[0], m_vt_1 = vt * ax[1], m_vt_2 = vt * ax[2];
  double m_st_0 = ax[0] * st, m_st_1 = ax[1] * st, m_st_2 = ax[2] * st;
  double m_vt_0_1 = m_vt_0 * ax[1], m_vt_0_2 = m_vt_0 * ax[2], m_vt_1_2 = m_vt_1 * ax[2];
  R[0] = ct + m_vt_0 * ax[0]; R[1] = -m_st_2 + m_vt_0_1; R[2] = m_st_1 + m_vt_0_2;
  R[3] = m_st_2 + m_vt_0_1;  R[4] = ct + m_vt_1 * ax[1]; R[5] = -m_st_0 + m_vt_1_2;
  R[6] = -m_st_1 + m_vt_0_2; R[7] = m_st_0 + m_vt_1_2;  R[8] = ct + m_vt_2 * ax[2];
}

// KDL Rotation::Rot2(axis, angle)
SMP_HD void rot2(const double* ax, double q, double* R) {
  double st, ct;
  psincos(q, &st, &ct);
  rot2_sc(ax, st, ct, R);
}

// Philox4x32-10 counter RNG.  Draw (seed, query, iteration, outer attempt, inner attempt, joint idx).
SMP_HD void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
  }
}

SMP_HD double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

SMP_HD double u01(uint64_t seed, uint32_t query, uint32_t it, uint32_t outer, uint32_t inner, uint32_t idx) {
  uint32_t c[4] = {it, outer, inner, idx >> 1};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32) ^ query);
  return (idx & 1) ? u53(c[2], c[3]) : u53(c[0], c[1]);
}

// The two draws idx = 2 * pair and 2 * pair + 1 of u01, which share one Philox block.
SMP_HD void u01_pair(uint64_t seed, uint32_t query, uint32_t it, uint32_t outer, uint32_t inner, uint32_t pair,
                     double* even, double* odd) {
  uint32_t c[4] = {it, outer, inner, pair};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32) ^ query);
  *even = u53(c[0], c[1]);
  *odd = u53(c[2], c[3]);
}

}  // namespace smp
