// Replays squirrel_8dof_planner.cpp's planner call sequence (SP:16, 482, 872-915, 1221-1248) through the C++
// drop-in shim include/smp_birrt_star.hpp, the way the ROS node would after swapping the include.
//
//   shim_plan <robot.urdf> <scene.bt> <iterations> <seed> <start x8> <goal x8> <env_x0 env_x1 env_y0 env_y1>
//
// The robot description is the URDF given and the SRDF beside it (same name, .srdf), handed to the planner as the node
// holds them (robot_description / robot_description_semantic); a .json argument names a prebuilt model instead.
//
// Prints "status <0|1>" and the trajectory rows; exit 0 on success, 2 on usage error, 3 when no GPU is usable
// (the shim throws: there is no CPU fallback).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "smp_birrt_star.hpp"

namespace {
// Minimal stand-in for octomap::OcTree: the shim only needs getResolution() and writeBinaryConst().
struct BtFileTree {
  std::string bytes;
  double res;
  double getResolution() const { return res; }
  std::ostream& writeBinaryConst(std::ostream& s) const { return s.write(bytes.data(), (std::streamsize)bytes.size()); }
};
}  // namespace

int main(int argc, char** argv) {
  if (argc != 1 + 4 + 16 + 4) {
    std::fprintf(stderr, "usage: shim_plan model.json scene.bt iterations seed start[8] goal[8] env[4]\n");
    return 2;
  }
  const std::string robot = argv[1];
  setenv("SMP_SEED", argv[4], 1);
  birrt_star_motion_planning::BiRRTstarPlanner planner;
  if (robot.size() > 5 && robot.compare(robot.size() - 5, 5, ".urdf") == 0) {
    auto slurp = [](const std::string& p) {
      std::ifstream in(p, std::ios::binary);
      return std::string(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
    };
    planner.setRobotDescription(slurp(robot), slurp(robot.substr(0, robot.size() - 5) + ".srdf"));
  } else {
    setenv("SMP_ROBOT_MODEL", argv[1], 1);
  }
  std::ifstream f(argv[2], std::ios::binary);
  BtFileTree tree{std::string(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>()), 0.05};
  std::vector<double> start(8), goal(8);
  for (int j = 0; j < 8; ++j) { start[j] = std::atof(argv[5 + j]); goal[j] = std::atof(argv[13 + j]); }
  std::vector<double> ex = {std::atof(argv[21]), std::atof(argv[22])}, ey = {std::atof(argv[23]), std::atof(argv[24])};
  try {
    planner.initialize("robotino_robot");                        // SP:16
  } catch (const std::exception& e) {
    std::printf("error %s\n", e.what());
    return 3;
  }
  planner.setOctree(&tree);                                       // SP:872-873 (floor already in the tree)
  planner.setDisabledLinkMapCollisions(std::vector<std::string>());  // SP:482
  planner.reset_planner_and_config();                             // SP:1224
  planner.setPlanningSceneInfo(ex, ey, "scenario");               // SP:1232
  if (!planner.init_planner(start, goal, 1, true, true)) {        // SP:1234
    std::printf("status init_failed\n");
    return 0;
  }
  bool ok = planner.run_planner(1, false, std::atof(argv[3]), false, 0.0, 0);  // SP:1238 (iteration budget)
  std::printf("status %d\n", ok ? 0 : 1);
  const std::vector<std::vector<double> >& traj = planner.getJointTrajectoryRef();  // SP:1241
  std::printf("waypoints %zu checked %lld\n", traj.size(), (long long)planner.lastStats().configs_checked);
  for (const auto& w : traj) {
    for (int j = 0; j < 8; ++j) std::printf("%s%.17g", j ? " " : "", w[j]);
    std::printf("\n");
  }
  // dimension mismatch: init_planner returns false (birrt_star.cpp:338-342)
  std::vector<double> short_conf(start.begin(), start.begin() + 7);
  std::printf("dim_mismatch_rejected %d\n", planner.init_planner(short_conf, goal, 1, true, true) ? 0 : 1);
  std::printf("start_valid %d\n", planner.isConfigValid(start, true, true) ? 1 : 0);
  // goal search of find_plan_end_effector (SP:578, 1129-1201) and one getFullPoseFromEEPose call (SP:1179)
  std::vector<double> ee = {start[0] + 0.6, start[1] + 0.2, 0.5, 1.57, 0.0, 0.3}, pose_goal;
  int res = planner.findGoalPose(ee, start, 20.0, true, true, pose_goal);
  std::printf("goal_search %d", res);
  for (double v : pose_goal) std::printf(" %.17g", v);
  std::printf("\n");
  std::vector<std::pair<double, double> > dev(3, std::make_pair(-0.005, 0.005));
  dev.resize(6, std::make_pair(-0.025, 0.025));
  std::vector<double> init = {ee[0] - 0.47, ee[1], 0.99, -1.2, 1.1, 0.0, 0.7, -1.5}, sol;
  bool ik = planner.getFullPoseFromEEPose(ee, dev, init, sol);
  std::printf("ee_ik %d", ik ? 1 : 0);
  for (double v : sol) std::printf(" %.17g", v);
  std::printf("\n");
  // the print-and-show-collisions service (SP:833-860): getCollisions of the start, of the start's arm at its
  // joint limits and of the start's arm at the corner of the map
  std::vector<std::vector<double> > probes(3, start);
  const double hi[5] = {1.5, 2.6, 1.8, 2.4, 2.9};
  for (int j = 0; j < 5; ++j) probes[1][3 + j] = hi[j];
  probes[2][0] = ex[1];
  probes[2][1] = ey[1];
  for (const std::vector<double>& q : probes) {
    std::vector<std::pair<std::string, std::string> > self;
    std::vector<std::string> map;
    planner.getCollisions(q, self, map);
    std::printf("collisions %zu %zu", self.size(), map.size());
    for (const auto& pr : self) std::printf(" %s %s", pr.first.c_str(), pr.second.c_str());
    for (const auto& m : map) std::printf(" %s", m.c_str());
    std::printf("\n");
  }
  return 0;
}
