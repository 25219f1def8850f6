// Sanitizer harness of the host-side parsers (ASAN / UBSAN on host code).  Built by
// tests/test_host_sanitize_cpu.py with g++ -fsanitize=address,undefined from the product sources smp_host.cpp,
// smp_urdf.cpp and smp_traj.cpp (no HIP: these files are plain C++).  The inputs arrive from the wire in the node
// (octomap service payloads, squirrel_8dof_planner.cpp:862-917; the robot description parameter, SP:1744-1767):
// every parser gets the intact input, every truncation on a stride, byte flips and random garbage.  A parser may
// throw std::runtime_error (reported to callers as SMP_ERR_PARSE); it may not read or write out of bounds, overflow
// or run away in memory.
//
//   fuzz_host <file> <kind: bt|ot|urdf|json> [<srdf> <spheres.json>] -> prints "ok <cases> <accepted> <rejected>"
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <iterator>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/smp_gpu.h"
#include "../../squirrel_motion_planner_amd/csrc/smp_host.h"

using namespace smp;

namespace {
std::string slurp(const char* p) {
  std::ifstream f(p, std::ios::binary);
  if (!f) throw std::runtime_error(std::string("cannot open ") + p);
  return std::string(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
}

long long n_ok = 0, n_rej = 0, n_cases = 0;

template <class F>
void attempt(F f) {
  ++n_cases;
  try {
    f();
    ++n_ok;
  } catch (const std::exception&) {
    ++n_rej;
  }
}

void octomap_case(const std::string& d, bool full) {
  // with the text header (a .bt / .ot file) and, after it, as a headerless message payload
  attempt([&] {
    double res = 0;
    std::vector<uint16_t> keys;
    std::vector<FreeLeaf> fl;
    if (full) octomap_ot_keys((const uint8_t*)d.data(), d.size(), &res, &keys, &fl, true);
    else octomap_bt_keys((const uint8_t*)d.data(), d.size(), &res, &keys, &fl, true);
    if (!keys.empty() && keys.size() / 3 < 100000) {
      SceneHost s;
      scene_from_keys(keys.data(), (int64_t)keys.size() / 3, res > 0 ? res : 0.05, -0.02, &s);
    }
  });
  const size_t h = d.find("\ndata\n");
  if (h != std::string::npos) {
    const std::string body = d.substr(h + 6);
    attempt([&] {
      double res = 0.05;
      std::vector<uint16_t> keys;
      if (full) octomap_ot_keys((const uint8_t*)body.data(), body.size(), &res, &keys, nullptr, false);
      else octomap_bt_keys((const uint8_t*)body.data(), body.size(), &res, &keys, nullptr, false);
    });
  }
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: fuzz_host <file> <bt|ot|urdf|json> [srdf spheres]\n");
    return 2;
  }
  const std::string data = slurp(argv[1]);
  const std::string kind = argv[2];
  set_max_octomap_voxels((size_t)1 << 20);  // a flipped bit can make a coarse occupied leaf: keep the runs short
  std::mt19937_64 rng(12345);
  std::vector<std::string> inputs = {data};
  const size_t stride = std::max<size_t>(1, data.size() / 400);
  for (size_t n = 0; n < data.size(); n += stride) inputs.push_back(data.substr(0, n));  // truncations
  for (int k = 0; k < 300; ++k) {                                                         // byte flips
    std::string m = data;
    const int flips = 1 + (int)(rng() % 8);
    for (int f = 0; f < flips && !m.empty(); ++f) m[rng() % m.size()] ^= (char)(1u << (rng() % 8));
    inputs.push_back(m);
  }
  for (int k = 0; k < 50; ++k) {                                                          // garbage after the header
    std::string m = data.substr(0, std::min<size_t>(data.size(), 64));
    const size_t n = rng() % 4096;
    for (size_t i = 0; i < n; ++i) m.push_back((char)(rng() & 0xff));
    inputs.push_back(m);
  }
  std::string srdf, spheres;
  if (kind == "urdf") {
    if (argc < 5) return 2;
    srdf = slurp(argv[3]);
    spheres = slurp(argv[4]);
    // structural mutations byte flips rarely reach: collision geometry moved onto each link in turn (the root and the
    // links fixed to it have no planning joint above them), each joint axis zeroed, every collision element removed
    const std::string col = "<collision><geometry><box size=\"0.1 0.1 0.1\"/></geometry></collision>";
    for (size_t p = data.find("<link name="); p != std::string::npos; p = data.find("<link name=", p + 1)) {
      const size_t e = data.find('>', p);
      if (e == std::string::npos) break;
      std::string m = data;
      if (m[e - 1] == '/') m.replace(e - 1, 2, ">" + col + "</link>");
      else m.insert(e + 1, col);
      inputs.push_back(m);
    }
    for (size_t p = data.find("<axis xyz=\""); p != std::string::npos; p = data.find("<axis xyz=\"", p + 1)) {
      const size_t q = data.find('"', p + 11);
      if (q == std::string::npos) break;
      std::string m = data;
      m.replace(p + 11, q - (p + 11), "0 0 0");
      inputs.push_back(m);
    }
    std::string nc = data;
    for (size_t p; (p = nc.find("<collision")) != std::string::npos;) {
      const size_t q = nc.find("</collision>", p);
      if (q == std::string::npos) break;
      nc.erase(p, q + 12 - p);
    }
    inputs.push_back(nc);
  }
  for (const std::string& in : inputs) {
    if (kind == "bt" || kind == "ot") {
      octomap_case(in, kind == "ot");
    } else if (kind == "urdf") {
      attempt([&] { RobotHost r; robot_from_urdf(in, srdf, spheres, &r); });
      attempt([&] { RobotHost r; robot_from_urdf(srdf, in, spheres, &r); });
    } else if (kind == "json") {
      attempt([&] { RobotHost r; robot_from_json(in, &r); });
    }
  }
  // trajectory normalisation (smp_traj.cpp) on random shapes, including degenerate ones
  for (int k = 0; k < 200; ++k) {
    const int dim = (int)(rng() % 10) - 1, n = (int)(rng() % 6);
    std::vector<double> raw((size_t)std::max(0, n * std::max(dim, 0)) + 1), np((size_t)std::max(dim, 0) + 1);
    std::uniform_real_distribution<double> u(-4.0, 4.0), s(0.0, 0.2);
    for (double& v : raw) v = u(rng);
    for (double& v : np) v = (k % 7 == 0) ? 0.0 : s(rng);
    int64_t n_out = 0;
    ++n_cases;
    if (smp_normalize_trajectory(raw.data(), n, dim, np.data(), nullptr, 0, &n_out) == SMP_OK && n_out > 0 &&
        n_out < 1000000) {
      std::vector<double> out((size_t)n_out * (size_t)std::max(dim, 1));
      smp_normalize_trajectory(raw.data(), n, dim, np.data(), out.data(), n_out, &n_out);
    }
  }
  std::printf("ok %lld %lld %lld\n", n_cases, n_ok, n_rej);
  return 0;
}
