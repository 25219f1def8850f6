// Host side of the IK goal search: the goal quaternion of an end-effector pose and the candidate controller runs
// of Planner::findGoalPose (squirrel_8dof_planner.cpp:1129-1194), in the order the reference tries them.
#include <cmath>

#include "smp_ik.h"
#include "smp_math.h"

namespace smp {

// getFullPoseFromEEPose (birrt_star.cpp:1630-1645): XYZ Euler angles -> quaternion [x, y, z, w].
void ik_goal_quat(const double* ee, double* g) {
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

namespace {

// getEndEffectorDirection (squirrel_8dof_planner.cpp:1639-1661): the hand's y axis rotated by tf's
// setRPY(roll, pitch, yaw) quaternion (Matrix3x3::setRotation); "downward" when |z| >= 0.9 (:1140).
bool ee_downward(const double* ee) {
  double sr, cr, sp, cp, sy, cy;
  psincos(ee[3] * 0.5, &sr, &cr);
  psincos(ee[4] * 0.5, &sp, &cp);
  psincos(ee[5] * 0.5, &sy, &cy);
  const double x = sr * cp * cy - cr * sp * sy, y = cr * sp * cy + sr * cp * sy;
  const double z = cr * cp * sy - sr * sp * cy, w = cr * cp * cy + sr * sp * sy;
  const double d = x * x + y * y + z * z + w * w, s = 2.0 / d;
  const double xs = x * s, ys = y * s, zs = z * s;
  const double wx = w * xs, yy = y * ys, yz = y * zs, xx = x * xs;
  const double az = (x * zs - w * ys) * 0.0 + (yz + wx) * 1.0 + (1.0 - (xx + yy)) * 0.0;
  return !(std::fabs(az) < 0.9);
}

}  // namespace

// Candidates of findGoalPose: base angle start + 0, +d, -d, +2d, -2d, ... while |diff| < pi (:1172-1194), the base
// placed `dist` behind the end effector, theta = angle + 0.99, the arm in the downward / sideways preset
// (:1139-1163); deviations (:1131-1137); 1000 controller iterations (birrt_star.cpp:1670).  Writes at most cap
// tasks, *n = the number of candidates; returns 1 if the hand points downward.
int ik_goal_candidates(const double* ee, const double* cur, double disc_deg, IkTaskDev* tasks, int cap, int* n) {
  if (disc_deg < 1) disc_deg = 1.0;  // squirrel_8dof_planner.cpp:80-83
  const double disc = disc_deg * (M_PI / 180.0);
  const bool down = ee_downward(ee);
  const double dist = down ? 0.44 : 0.47;
  const double arm_down[5] = {-0.8, 0.8, 0.0, -1.5, 0.0}, arm_side[5] = {-1.2, 1.1, 0.0, 0.7, -1.5};
  const double gx = ee[0] - cur[0], gy = ee[1] - cur[1];
  const double start = gy > 0 ? std::acos(gx / std::sqrt(std::pow(gx, 2) + std::pow(gy, 2)))
                              : -std::acos(gx / std::sqrt(std::pow(gx, 2) + std::pow(gy, 2)));
  IkTaskDev t{};
  ik_goal_quat(ee, t.goal);
  for (int i = 0; i < 3; ++i) { t.lo[i] = -0.005; t.hi[i] = 0.005; t.lo[i + 3] = -0.025; t.hi[i + 3] = 0.025; }
  t.max_iter = 1000;
  int k = 0;
  double diff = 0.0;
  while (std::fabs(diff) < M_PI) {
    const double a = start + diff;
    double sa, ca;
    psincos(a, &sa, &ca);
    t.q[0] = ee[0] - dist * ca;
    t.q[1] = ee[1] - dist * sa;
    t.q[2] = a + 0.99;
    for (int j = 0; j < 5; ++j) t.q[3 + j] = down ? arm_down[j] : arm_side[j];
    if (k < cap) tasks[k] = t;
    ++k;
    diff *= -1;
    diff += 0.0;
    if (diff >= 0.0) diff += disc;
  }
  *n = k;
  return down ? 1 : 0;
}

}  // namespace smp
