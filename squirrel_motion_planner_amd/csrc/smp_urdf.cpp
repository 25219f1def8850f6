// URDF + SRDF -> robot model (the path the ROS node takes: kdl_parser::treeFromParam + parseSRDF,
// collision_checker.hpp:176-393).  Filled in by the URDF reader; see smp_host.h.
#include <stdexcept>
#include <string>

#include "smp_host.h"

namespace smp {

void robot_from_urdf(const std::string& urdf, const std::string& srdf, const std::string& spheres_json, RobotHost* out) {
  (void)urdf; (void)srdf; (void)spheres_json; (void)out;
  throw std::runtime_error("smp_robot_create_urdf: URDF reader not built in this version; use smp_robot_create_json");
}

}  // namespace smp
