// Device-resident BiRRT* planner state (one workgroup per query).  Shared by smp_kernels.hip and the host.
#pragma once
#include <stdint.h>

#include "smp_types.h"

namespace smp {

constexpr int MAX_PTS = 32;    // num_traj_segments_interp upper bound (reference default 20)
constexpr int MAX_NEAR = 32;   // max_near_nodes upper bound (reference default 20)
constexpr int MAXE = 24;       // edges per validity / cost batch

struct NodeRef {               // what the reference passes by value (Node, data_structs.h:29-45)
  double q[NJ];
  double c[3];                 // cost_reach total, revolute, prismatic
  int id;
  int parent;
};

struct TreeDev {               // SoA node arrays of one tree; capacity `cap`
  double* q;                   // [NJ][cap]
  double* cost;                // [3][cap]
  int* parent;
  int* first_child;
  int* next_sib;
  int* prev_sib;
  double* e_start;             // [NJ][cap] in-edge: interpolation start (parent config at creation)
  double* e_target;            // [NJ][cap] in-edge: interpolation target
};

struct QState {                // per query, persisted in global memory across launches
  int status;                  // 0 ok / running, negative SMP_ERR_*
  int phase;                   // 0: pre-loop connect pending, 1: planning loop, 2: finished
  int A;                       // tree acting as tree_A next iteration (0 start, 1 goal)
  int have_sol, conn_start;
  int n[2], edges[2], rewires[2];
  int cap, via_cap;
  long long iter, max_iter;
  long long max_checked;       // > 0: stop once this many configurations were collision-checked
  long long checked, valid, first_iter, last_iter;
  long long nn_nodes, near_nodes;  // nodes streamed by nearest / near scans (algorithmic bytes)
  long long smp_hits;              // samples taken from the run-ahead sampler
  unsigned long long prof[32];     // device-clock ticks per planner phase (SMP_PROF_* in smp_kernels.hip)
  unsigned long long t0, t_first, t_end, deadline;  // device wall clock (0 deadline = none)
  double cbest[3], h0[3];
  NodeRef nB, nA;              // m_node_tree_B / m_node_tree_A
  double qs[NJ], qg[NJ];
  double Crev[36], Cpr[4], ctr_rev[6], ctr_pr[2];
  double env_x[2], env_y[2];
  double near_r, step, opt_thresh;
  int n_pts, max_near, tree_opt, informed, self, map;
  unsigned long long seed;
  unsigned query;
  long long n_rows;
};

struct ViaNode {               // via node pending insertion (selected_via_nodes / edges)
  double q[NJ];
  double c[3];
  double e_start[NJ];
  double e_target[NJ];
  int id, parent;
};

// Collision-check job of one query, shared by its leader workgroup and its helper workgroups through HBM
// (DESIGN.md "Helpers").  Both directions use data-tagged 8-byte granules (MI355X_MICROARCH.md hand-off table:
// "data-tagged granules"; an aligned 8-byte store is single-copy atomic): the high 32 bits of every granule are
// the job number, the low 32 bits data, so a reader knows a granule is current without any flag, fence or
// drain.  Granules are stored and read with agent-scope (sc1) relaxed atomics.
#ifndef SMP_HELPER_CT
#define SMP_HELPER_CT 8
#endif
constexpr int HELPER_CT = SMP_HELPER_CT;          // configurations per job tile
static_assert(HELPER_CT <= 32, "a tile's collision mask is one 32-bit word");
constexpr int JOB_SLOTS = MAXE * (MAX_PTS + 1); // (edge, point) slots of one job
constexpr int JOB_TILES = (JOB_SLOTS + HELPER_CT - 1) / HELPER_CT;
constexpr int JOB_WORDS = 1 + 4 * NJ * MAXE;     // payload words: header + (start, step) halves per edge
constexpr int SMP_RING = 16;                     // run-ahead sampler: samples kept ahead of the leader
struct JobBoard {
  int stop;                    // 1 once the leader left the launch: helpers exit
  int pad0[7];
  unsigned long long dbg[12];  // SMP_JOB_PROF builds: publish time, helper pickup / finish delay sums and counts,
                               // helper tile stage clocks (collide_tile A, B, C-centres, C)
  // leader -> helpers: word 0 = header (edges | np1 << 8 | self << 16 | map << 17); word 1 + 32k + 2j (+1) =
  // low (high) half of edge k's start[j], word 1 + 32k + 16 + 2j (+1) = of its step[j]
  unsigned long long pay[JOB_WORDS];
  int pad1[32 - (2 * JOB_WORDS) % 32];
  // helpers -> leader: tile t's collision mask (bit c = configuration c of the tile collides)
  unsigned long long res[JOB_TILES];
  int pad2[32 - (2 * JOB_TILES) % 32];
  // run-ahead sampler (DESIGN.md "Sampler").  Leader -> sampler: its current iteration and the informed-
  // sampling parameters, versioned (payload stores drained before the version store).
  int s_ver, s_have_sol;
  long long s_iter;
  unsigned long long s_cbest[3];  // fp64 bit patterns
  int pad6[22];
  // sampler -> leader: the sample of iteration i in slot i % SMP_RING, tag = (i << 32) | version, stored after
  // the drained configuration.
  struct {
    unsigned long long tag;
    unsigned long long q[NJ];     // fp64 bit patterns
    int pad[14];
  } ring[SMP_RING];
};

struct QueryDev {
  QState* st;
  JobBoard* jb;                // null: no helpers
  int* trace;                  // debug only (SMP_DEBUG): host-mapped progress markers of the leader
  int nworkers;                // leader + tile helper workgroups (tile w, w + nworkers, ... is worker w's)
  int sampler;                 // 1: the last helper workgroup is the run-ahead sampler
  TreeDev tr[2];
  ViaNode* via;                // [via_cap]
  int* stack;                  // [cap] DFS stack of recursiveNodeCostUpdate
  double* rows;                // [max_iter][5] cost evolution rows (may be null)
  long long rows_cap;
  int* path_nodes;             // [2][cap] path extraction scratch
};

}  // namespace smp
