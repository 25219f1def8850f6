// Trajectory post-processing of the node (host side, no GPU work): Planner::normalizeTrajectory
// (squirrel_8dof_planner.cpp:1557-1637) with its angle helpers (squirrel_8dof_planner.cpp:2026-2056), behind the
// C ABI so that the shim (include/smp_birrt_star.hpp) and the Python mirror share one implementation.
// Built with the library's strict IEEE flags (-ffp-contract=off): the arithmetic follows the reference term by term.
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/smp_gpu.h"

namespace {

constexpr double kPi = 3.14159265358979323846;  // M_PI

// findAngularDistance (squirrel_8dof_planner.cpp:2026-2033)
inline double angular_distance(double a1, double a2) {
  const double dist = std::fabs(a2 - a1);
  if (dist <= kPi) return dist;
  return 2 * kPi - dist;
}

// findAngularDistanceSigned (squirrel_8dof_planner.cpp:2035-2047)
inline double angular_distance_signed(double a1, double a2) {
  const double d = a2 - a1;
  if (std::fabs(d) <= kPi) return d;
  if (d > 0.0) return -2.0 * kPi + d;
  return 2.0 * kPi + d;
}

// normalizeAngle (squirrel_8dof_planner.cpp:2049-2055)
inline void normalize_angle(double& a) {
  if (a < -kPi) a += 2.0 * kPi;
  else if (a > kPi) a -= 2.0 * kPi;
}

constexpr int64_t kMaxRows = 100000000;  // refuse resamplings that would not fit memory (tiny distances)

}  // namespace

extern "C" int smp_normalize_trajectory(const double* raw, int64_t n, int dim, const double* normalized_pose,
                                        double* out, int64_t out_cap, int64_t* n_out) {
  if (!n_out || n < 0 || (n > 0 && !raw) || (dim > 0 && !normalized_pose)) return SMP_ERR_ARG;
  *n_out = 0;
  // the reference returns without touching its output for these (squirrel_8dof_planner.cpp:1561-1562)
  if (dim < 1 || n <= 1) return SMP_OK;
  const bool full = dim == 8;  // base theta (index 2) is an angle only for full 8-DoF poses
  std::vector<double> traj(raw, raw + n * dim);
  if (dim > 2) {
    // wrap theta into [-pi, pi] once (squirrel_8dof_planner.cpp:1564-1572; the reference does this for any
    // dimension, index 2 being arm joint 3 for the 5-DoF folding keyframes)
    for (int64_t i = 0; i < n; ++i) {
      double& a = traj[i * dim + 2];
      if (a > kPi) a -= 2.0 * kPi;
      else if (a < -kPi) a += 2.0 * kPi;
    }
  }
  std::vector<double> res(traj.begin(), traj.begin() + dim);  // front pose
  std::vector<double> last(dim), diff(dim);
  int64_t next = 1;
  for (;;) {
    const double* pn = &traj[next * dim];
    const double* pl = &res[res.size() - dim];
    double frac = std::fabs(pn[0] - pl[0]) / normalized_pose[0];
    for (int i = 1; i < dim; ++i) {
      double f;
      if (full && i == 2) f = angular_distance(pn[i], pl[i]) / normalized_pose[i];
      else f = std::fabs(pn[i] - pl[i]) / normalized_pose[i];
      if (f > frac) frac = f;
    }
    if (frac < 1.0) {
      ++next;
      if (next == n) {
        res.insert(res.end(), traj.end() - dim, traj.end());  // the last raw pose
        break;
      }
      continue;
    }
    if (!(frac < (double)kMaxRows)) return SMP_ERR_ARG;  // also NaN
    const int64_t counter_max = (int64_t)(unsigned)frac + 1;  // (UInt)frac + 1, before the ceil
    frac = std::ceil(frac);
    const double recip = 1.0 / frac;
    std::memcpy(last.data(), &res[res.size() - dim], dim * sizeof(double));
    for (int i = 0; i < dim; ++i) diff[i] = (full && i == 2) ? angular_distance_signed(last[i], pn[i]) : pn[i] - last[i];
    if ((int64_t)(res.size() / dim) + counter_max > kMaxRows) return SMP_ERR_ARG;
    for (int64_t c = 1; c <= counter_max; ++c) {
      const size_t b = res.size();
      res.insert(res.end(), last.begin(), last.end());
      for (int j = 0; j < dim; ++j) {
        res[b + j] += (double)c * diff[j] * recip;
        if (full && j == 2) normalize_angle(res[b + j]);
      }
    }
    ++next;
    if (next == n) break;
  }
  const int64_t rows = (int64_t)(res.size() / dim);
  *n_out = rows;
  if (!out) return SMP_OK;
  if (out_cap < rows) return SMP_ERR_CAPACITY;
  std::memcpy(out, res.data(), res.size() * sizeof(double));
  return SMP_OK;
}
