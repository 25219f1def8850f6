// Host-side builders: robot model (JSON / URDF+SRDF), occupancy scene (keys / octomap .bt), squared EDT.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "smp_types.h"

namespace smp {

struct RobotHost {
  RobotDev dev;
  std::vector<std::string> link_names;  // all tree links
  std::vector<int> clink_of_link;       // -1 if the link has no collision geometry
};

struct SceneHost {
  int nx = 1, ny = 1, nz = 1, wx = 1;
  double ox = 0, oy = 0, oz = 0, res = 0.05;
  std::vector<uint64_t> bits;     // x-major rows of 64-bit words
  std::vector<uint16_t> d2;       // squared box-to-box gap (voxels) to the nearest occupied cell, <= 65535
  int bnx = 1, bny = 1, bnz = 1;  // 4x4x4 bricks
  std::vector<uint64_t> bricks;   // bit (z&3)*16 + (y&3)*4 + (x&3) of brick (z>>2, y>>2, x>>2)
  int64_t n_occupied = 0;
  double bbox_min[3] = {0, 0, 0}, bbox_max[3] = {0, 0, 0};  // metric bbox of the occupied keys (octree frame)
};

namespace json { struct Value; }
// Throws std::runtime_error on malformed input.
void robot_from_model_value(const json::Value& m, RobotHost* out);
void robot_from_json(const std::string& text, RobotHost* out);
void robot_from_urdf(const std::string& urdf, const std::string& srdf, const std::string& spheres_json, RobotHost* out);

constexpr int KEY_OFFSET = 32768;  // octomap tree_max_val

constexpr double GRID_REACH = 0.45;  // m: largest horizontal reach of a sphere or primitive from its centre
int grid_pad_cells(double res);
void scene_from_keys(const uint16_t* keys, int64_t n, double res, double z_offset, SceneHost* out);
// A free octree leaf (depth, centre key, float log-odds): kept for the floor insertion, which leaves a floor cell
// free when it falls in a free leaf whose log-odds plus one hit stay below 0.
struct FreeLeaf {
  int depth;
  int k[3];
  float v;
};
constexpr float kHitLogOdds = 0.847297860387203f;        // octomap prob_hit 0.7: logodds(0.7)
constexpr float kClampMinLogOdds = -2.000027830777221f;   // clamping_thres_min 0.1192: logodds(0.1192)
// Octomap binary stream (.bt file, or with header = false an octomap_msgs binary payload) -> occupied leaf keys
// (expanded to depth 16) and, if `free` is given, the free leaves.  *res is read from the header.
void octomap_bt_keys(const uint8_t* data, size_t size, double* res, std::vector<uint16_t>* keys,
                     std::vector<FreeLeaf>* free = nullptr, bool header = true);
// Expansion limit of pruned occupied leaves per stream (default 2^26 voxels; the parser throws beyond it).
void set_max_octomap_voxels(size_t n);
// Octomap full stream (.ot file, or with header = false an octomap_msgs full payload), same outputs.
void octomap_ot_keys(const uint8_t* data, size_t size, double* res, std::vector<uint16_t>* keys,
                     std::vector<FreeLeaf>* free = nullptr, bool header = true);
// squirrel_8dof_planner.cpp:889-902 floor square around (cx, cy) at the key of z = -res/2 (updateNode(key, true)
// on each cell; cells inside a free leaf that one hit does not make occupied are skipped).
void floor_keys(double cx, double cy, double res, double distance, std::vector<uint16_t>* keys,
                const std::vector<FreeLeaf>* free = nullptr);
// Exact squared Euclidean distance transform (voxel units) of a dense occupancy mask (x fastest).
void edt_squared(const std::vector<uint8_t>& occ, int nx, int ny, int nz, std::vector<uint16_t>* d2);
// Squared box-to-box gap field (voxel units): EDT of the 3x3x3-dilated occupancy.
void box_gap_squared(const std::vector<uint8_t>& occ, int nx, int ny, int nz, std::vector<uint16_t>* d2);
// 4x4x4 occupancy bricks from the bitset.
void build_bricks(SceneHost* h);
uint32_t sphere_threshold(double r, double res);
// Per-primitive 2-D box-gap fields of a scene (SceneDev::slab): occupancy projected over the layers the primitive's
// constant z range touches, dilated 3x3, squared EDT (cells).
void prim_slabs(const RobotDev& d, const SceneHost& s, std::vector<std::vector<uint16_t>>* out);
// Flat self-collision pair lists (sphere pairs, primitive-sphere pairs) from pair_a / pair_b.
void finish_pairs(RobotDev* d);

}  // namespace smp
