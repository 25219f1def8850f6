// IK goal search: shared layouts of the VDLS controller kernel (smp_ik.hip) and its host side (smp_ik_host.cpp).
//
// Reference: Planner::findGoalPose (squirrel_8dof_planner.cpp:1129-1201) -> BiRRTstarPlanner::
// getFullPoseFromEEPose (birrt_star.cpp:1627-1686) -> RobotController::run_VDLS_Control_Connector
// (control_laws.cpp:3283-3712).  The candidate base angles of one goal search are independent controller runs,
// so each runs on its own wavefront; DESIGN.md "IK goal search" states the arithmetic both this kernel and the
// oracle (oracle/smp_oracle.cpp ik_solve) follow.
#pragma once
#include <stdint.h>

#include "smp_types.h"

namespace smp {

constexpr int IK_THREADS = 64;  // one wavefront per controller run

struct IkTaskDev {
  double goal[7];       // x, y, z, qx, qy, qz, qw (birrt_star.cpp:1638-1645)
  double lo[6], hi[6];  // permitted error band per task coordinate (setVariableConstraints, control_laws.cpp:1740)
  double q[8];          // start configuration (setStartConf, control_laws.cpp:1464-1495)
  int32_t max_iter;     // controller iterations (1000 in getFullPoseFromEEPose, birrt_star.cpp:1670)
  int32_t pad;
};

struct IkOutDev {
  double q[8];          // joint_trajectory.back()
  double err[6];        // last (clamped) error vector
  double manip;         // last manipulability measure
  int32_t reached;      // REACHED 1 / ADVANCED 0 (control_laws.cpp:3691-3710)
  int32_t iters;
  int32_t fallback;     // iterations whose manipulability needed the Jacobi eigenvalue path
  int32_t flags;        // goal search: IK_CHECKED | IK_VALID | IK_ABANDONED (0 for plain controller runs)
};

enum { IK_CHECKED = 1, IK_VALID = 2, IK_ABANDONED = 4 };

// Host side (smp_ik_host.cpp): goal quaternion of [x, y, z, roll, pitch, yaw] (birrt_star.cpp:1630-1645) and the
// candidate controller runs of findGoalPose in the reference's order; returns 1 if the hand points downward.
void ik_goal_quat(const double* ee, double* g);
int ik_goal_candidates(const double* ee, const double* cur, double disc_deg, IkTaskDev* tasks, int cap, int* n);

}  // namespace smp
