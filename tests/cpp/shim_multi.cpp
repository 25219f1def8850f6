// smp_node::MultiGpuPlanner (include/smp_birrt_star.hpp) on a list of devices: the octree set once and shared device to
// device, a batch of queries dealt over the planners and planned concurrently.
//
//   shim_multi <robot.urdf> <scene.bt> <devices, e.g. 0,0> <iterations> <n_queries> <start x8> <goal x8> <env x4>
//
// Query k plans start -> goal with seed 100 + k.  Prints per query "query k status checked waypoints" and the
// trajectory rows; exit 0 on success, 2 on usage error, 3 when no GPU is usable (no CPU fallback).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <sstream>
#include <string>
#include <vector>

#include "smp_birrt_star.hpp"

int main(int argc, char** argv) {
  if (argc != 1 + 5 + 16 + 4) {
    std::fprintf(stderr, "usage: shim_multi robot.urdf scene.bt devices iterations n_queries start[8] goal[8] env[4]\n");
    return 2;
  }
  auto slurp = [](const std::string& p) {
    std::ifstream in(p, std::ios::binary);
    return std::string(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
  };
  const std::string urdf = argv[1];
  std::vector<int> devices;
  {
    std::stringstream ss(argv[3]);
    std::string tok;
    while (std::getline(ss, tok, ',')) devices.push_back(std::atoi(tok.c_str()));
  }
  smp_node::MultiGpuPlanner mp(devices);
  mp.setRobotDescription(slurp(urdf), slurp(urdf.substr(0, urdf.size() - 5) + ".srdf"));
  try {
    mp.initialize();
  } catch (const std::exception& e) {
    std::printf("error %s\n", e.what());
    return 3;
  }
  const std::string bt = slurp(argv[2]);
  mp.setOctreeBinary(reinterpret_cast<const uint8_t*>(bt.data()), bt.size(), 0.05);
  std::vector<smp_node::MultiGpuPlanner::Query> qs(std::atoi(argv[5]));
  for (size_t k = 0; k < qs.size(); ++k) {
    auto& q = qs[k];
    q.start.resize(8);
    q.goal.resize(8);
    for (int j = 0; j < 8; ++j) { q.start[j] = std::atof(argv[6 + j]); q.goal[j] = std::atof(argv[14 + j]); }
    q.env_x[0] = std::atof(argv[22]); q.env_x[1] = std::atof(argv[23]);
    q.env_y[0] = std::atof(argv[24]); q.env_y[1] = std::atof(argv[25]);
    q.budget = std::atof(argv[4]);
    q.seed = 100 + k;
  }
  const auto out = mp.plan(qs);
  for (size_t k = 0; k < out.size(); ++k) {
    std::printf("query %zu %d %lld %zu\n", k, out[k].status, (long long)out[k].stats.configs_checked,
                out[k].trajectory.size());
    for (const auto& w : out[k].trajectory) {
      for (int j = 0; j < 8; ++j) std::printf("%s%.17g", j ? " " : "", w[j]);
      std::printf("\n");
    }
  }
  return 0;
}
