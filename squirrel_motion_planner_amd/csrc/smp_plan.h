// Device-resident BiRRT* planner state (one workgroup per query).  Shared by smp_kernels.hip and the host.
#pragma once
#include <stdint.h>

#include "smp_types.h"

namespace smp {

constexpr int MAX_PTS = 32;    // num_traj_segments_interp upper bound (reference default 20)
constexpr int MAX_NEAR = 32;   // max_near_nodes upper bound (reference default 20)
#ifndef SMP_MAXE
#define SMP_MAXE 24
#endif
constexpr int MAXE = SMP_MAXE;  // edges per validity / cost batch 

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
  float* qf;                   // [NJ][cap] q rounded to fp32: the distributed scans' prefilter (DESIGN.md "Scans of
                               // large trees"), written with q
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
  long long sc_nn, sc_near, sc_edge_hit, sc_edge_miss;  // scout results used: nearest, near sets, edges (+ misses)
  unsigned long long sc_wait;      // device-clock ticks the leader waited for the scout
  unsigned long long prof[32];     // device-clock ticks per planner phase (SMP_PROF_* in smp_kernels.hip)
  unsigned long long t0, t_first, t_end, deadline;  // device wall clock (0 deadline = none)
  unsigned long long budget_ticks;  // seconds budget in device-clock ticks (has_deadline): deadline = t0 + this
  int has_deadline;
  int stop_margin;             // > 0 (seconds budgets): end the run once a tree is within this many nodes of cap
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
// Job tiles (DESIGN.md "Helpers"): a job of S configurations (its slots) checked by W workers (the leader + W - 1
// helpers) is cut into tiles of ct configurations, ct the smallest of 1, 2, 4 whose tiles the helpers take in one
// round, else 8 (the tiles of one round then exceed the helpers: skip mode).  A tile of ct configurations is spread
// over the whole workgroup (collide_wide: 8 / ct wavefronts per configuration), so the fewer configurations per tile,
// the shorter the tile and the job's round trip.
constexpr int TILE_CT_MAX = BLOCK / 64;         // configurations per tile at most (one per wavefront)
constexpr int JOB_SLOTS = MAXE * (MAX_PTS + 1); // (edge, point) slots of one job
constexpr int JOB_TILES = 256;                  // tiles of one job at most (W - 1 <= 255 for ct < 8)
static_assert(JOB_TILES * TILE_CT_MAX >= JOB_SLOTS, "a job of 8-configuration tiles fits the result granules");
// ct of a job of `slots` configurations and W workers; `fixed` > 0 forces 1, 2, 4 or 8 (QueryDev::tile_ct, experiments).
__host__ __device__ inline int job_tile_ct(int slots, int W, int fixed) {
  if (fixed > 0) return (slots + fixed - 1) / fixed <= JOB_TILES ? fixed : TILE_CT_MAX;
  const int helpers = W - 1 < JOB_TILES ? W - 1 : JOB_TILES;
  for (int ct = 1; ct < TILE_CT_MAX; ct <<= 1)
    if ((slots + ct - 1) / ct <= helpers) return ct;
  return TILE_CT_MAX;
}
constexpr int JOB_WORDS = 1 + 4 * NJ * MAXE;     // payload words: header + (start, step) halves per edge
constexpr int SMP_RING = 16;                     // run-ahead sampler: samples kept ahead of the leader
// Distributed tree scans (DESIGN.md "Scans of large trees"): a workgroup splits a nearest / near scan of a large tree
// over itself and up to SCAN_P - 1 of its helpers; participant w's partial result is SCAN_W granules of sres[w]:
// nearest: key low / high half, id; near set: count, list lengths (lo | hi << 16), then per entry of the low and the
// high list (key low half, key high half, id).
// Participant p >= 1 of a scan is worker W - p (W = the workgroup's workers: the helpers from the top down), so that a scan
// published while a collision job runs (the job's tiles go to workers 1, 2, ... from the bottom up) takes the helpers the
// job leaves free.  A near scan has at most SCAN_PNEAR participants (its merge ranks every list entry).
constexpr int SCAN_P = 64;
constexpr int SCAN_PNEAR = 32;
constexpr int SCAN_W = 2 + 2 * 3 * MAX_NEAR;
constexpr int SCAN_WORDS = 33;  // payload granules of a scan job (JobBoard::spay)
// Tag of the run-ahead sampler's ring granules: iteration (low 24 bits) and parameter version (low 8 bits).  A slot
// holds only iteration i (mod SMP_RING) and the version changes at most once per iteration, so the short fields
// cannot alias within a run of fewer than 2^24 iterations.
__host__ __device__ inline unsigned ring_tag(long long it, unsigned ver) {
  return ((unsigned)it & 0xffffffu) << 8 | (ver & 0xffu);
}
constexpr int RING_PARAMS = 5;               // ring slot: have_sol, cbest[1] (lo, hi), cbest[2] (lo, hi)
constexpr int RING_G = 2 * NJ + RING_PARAMS;  // granules per ring slot
// The parameter word k of a ring slot (sampler and leader).
__device__ inline unsigned ring_param(int k, int have_sol, const double* cbest) {
  if (k == 0) return (unsigned)have_sol;
  const unsigned long long b = (unsigned long long)__double_as_longlong(cbest[1 + ((k - 1) >> 1)]);
  return ((k - 1) & 1) ? (unsigned)(b >> 32) : (unsigned)b;
}
struct JobBoard {
  int stop;                    // 1 once the leader left the launch: helpers exit
  int pad0[7];
  unsigned long long dbg[12];  // SMP_JOB_PROF builds: publish time, helper pickup / finish delay sums and counts,
                               // helper tile stage clocks (collide_tile A, B, C-centres, C)
  // leader -> helpers: word 0 = header (edges | np1 << 8 | self << 16 | map << 17 | scan job << 18 | skip << 19 |
  // stop-first-valid << 20 | log2(tile ct) << 21); word 1 + 32k + 2j (+1) = low (high) half of edge k's start[j],
  // word 1 + 32k + 16 + 2j (+1) = of its step[j]
  unsigned long long pay[JOB_WORDS];
  int pad1[32 - (2 * JOB_WORDS) % 32];
  // helpers -> leader: tile t's collision mask (bit c = configuration c of the tile collides)
  unsigned long long res[JOB_TILES];
  int pad2[32 - (2 * JOB_TILES) % 32];
  // leader -> helpers: a scan job (DESIGN.md "Scans of large trees"), in its own granules beside `pay`, so that a scan may
  // run while a collision job holds `pay`: word 0 = header (scan bit << 18 | near << 19 | tree << 20 | near == 2 << 21,
  // bit 21 marking a fused nearest + near set of one configuration, slice_near<true>), words 1-16 the query
  // configuration's halves, 17 range start, 18 range end, 19 excluded id, 20-21 radius halves, 22 participants.  A scan
  // job thus fills words 0-22; SCAN_WORDS = 33 is the count an idle helper's first poll covers (the scan header's
  // edge-count field 1 = one edge's 32 granules + the header, as a collision job of one edge), words 23-32 unused.
  unsigned long long spay[64];
  // run-ahead sampler (DESIGN.md "Sampler").  Leader -> sampler: its current iteration and the informed-
  // sampling parameters, versioned (payload stores drained before the version store).
  int s_ver, s_have_sol;
  long long s_iter;
  unsigned long long s_cbest[3];  // fp64 bit patterns
  int pad6[22];
  // sampler -> leader: the sample of iteration i in slot i % SMP_RING.
  // Each configuration value travels as two data-tagged granules (low, high 32 bits) whose tag is
  // ring_tag(iteration, version), so one round of loads both reads a slot and tells whether it is current; then
  // RING_PARAMS granules of the sampling parameters the sample was drawn with (have_sol, the halves of cbest[1] and
  // cbest[2]: everything else it reads is a query constant), which the leader compares with its own -- a sample is
  // taken only if drawn with exactly the leader's parameters, whatever the version bookkeeping did.
  struct {
    unsigned long long g[RING_G];
  } ring[SMP_RING];
  unsigned long long sres[SCAN_P][SCAN_W];  // scan jobs: participant w's partial result (w >= 1)
};

// Scout (DESIGN.md "Scout"): a second workgroup per query computes the expand / near / choose-parent / rewire
// scans and collision jobs of the leader's NEXT iteration on a snapshot of the tree that iteration expands (its
// first X nodes, which no step of the current iteration modifies; the current iteration only appends to it).  The
// leader takes a result only if its key matches exactly (same tree, same query configuration, same edge end
// points) and patches the scans with the nodes appended since the snapshot, so its trees are the ones it would
// have built alone.  Records are double-buffered by iteration parity; every word is written with sc1 stores and
// drained before the record's stage granule, (tag << 32) | stage with tag = iteration + 1.
constexpr int SCOUT_EDGES = 1 + 2 * MAX_NEAR;  // expand edge, choose-parent candidates, rewire candidates
constexpr int SCOUT_CHOOSE0 = 1, SCOUT_REWIRE0 = 1 + MAX_NEAR;
enum { SC_STARTED = 0, SC_NN = 1, SC_EXPAND = 2, SC_NEAR = 3, SC_CHOOSE = 4, SC_DONE = 5, SC_CONN = 6 };
struct ScoutNN {               // stage SC_NN: nearest node of the sample in the snapshot
  double q[NJ];                // the sample scanned
  double d;                    // its distance (the running minimum of the reference scan, 10000 if none)
  double c[3];                 // that node's cost (a node's cost never changes before the first solution)
  int id, X, t, ok;            // node id, snapshot size, tree, 1 = valid
};
struct ScoutNear {             // stage SC_NEAR: near set of x_new in the snapshot
  double q[NJ];
  int nk, n_lo, n_hi, ok, X, t;  // count, list lengths, 1 = valid, snapshot size, tree
  int lo_i[MAX_NEAR], hi_i[MAX_NEAR];
  double lo_c[MAX_NEAR], hi_c[MAX_NEAR];
};
struct ScoutEdge {             // one candidate edge: interpolation start / target, first colliding point
  double s[NJ], g[NJ];
  double acc[3];               // segment-norm sums (edge_costs' eg_acc; cost = start node's cost + acc)
  int first, pad;              // first: as eg_first (n_pts + 1 = free), -1 = not checked
};
struct ScoutExpand {           // stage SC_EXPAND: the expand edge's interpolation data (edge_costs of edge 0)
  double ext[NJ];              // step target (stepTowardsRandSample from the nearest node towards the sample)
  double step[NJ], end[NJ];    // interpolation step and end point
  double acc[3];               // segment-norm sums (cost = nearest node's cost + acc)
  int ok, pad;
};
struct ScoutConnect {          // stage SC_DONE, before the first solution: connect's nearest node and direct edge
  double q[NJ];                // x_new (the expand edge's end)
  double d;                    // its nearest node's distance over the other tree's first X nodes (10000 if none)
  double c[3];                 // that node's cost
  int id, X, t, ok;            // that node, the snapshot size, the tree, 1 = valid
  ScoutEdge e;                 // the direct edge nearest -> x_new (segment-norm sums, first colliding point)
};
// Stage SC_DONE, before the first solution, with cn.ok: connect's outcome on the snapshot (connectGraphs before a
// solution has no near loop, so it is a function of x_new, its nearest node and the direct edge): the stepping flag
// and the via chain (nodes in ScoutBoard::pre_via of the record's slot, ids from the snapshot size XB upward, which
// the leader rebases onto its tree size).  The leader commits it when its own nearest node is the record's.
constexpr int PRE_VIA = 16;
struct ScoutPre {
  int ok;                      // 1: recorded (0: chain longer than PRE_VIA, the leader steps it itself)
  int flag;                    // 0 nothing, 1 connect (stepped to x_new), 2 extend (stepped to the last valid point)
  int nv, need;                // via nodes; the direct edge was checked (its cost is below c_best)
  double sol[3];               // direct edge cost + x_new's cost
  NodeRef sel;                 // the last stepped edge's node (id / parent relative to XB as above)
  double sel_start[NJ], sel_target[NJ];
};
// Stage SC_CONN (two scouts, after the first solution): connect's scans of the iteration, computed once the leader
// reports that the tree connect searches (tree_B of the iteration = tree_A of the one before) is final (its rewire
// commits are done; nothing appends to it before connect): the nearest node of x_new, its near set (excluding the
// id x_new has in its own tree, as find_near_vertices does) and the segment-norm sums of connect's edges.
struct ScoutConn {
  double q[NJ];                // x_new
  double d;                    // distance of the nearest node (10000 if none)
  int id, X, t, excl;          // nearest node, tree size scanned, tree, excluded id
  int nk, n_lo, n_hi, ok;      // near count, list lengths, 1 = valid
  int lo_i[MAX_NEAR], hi_i[MAX_NEAR];
  double lo_c[MAX_NEAR], hi_c[MAX_NEAR];
  double acc0[3];              // direct edge nearest -> x_new
  double pad0;
  double acc[MAX_NEAR][3];     // near candidate lo_i[e] -> x_new (e < min(n_lo, max_near))
  // first colliding point of the direct edge and of every near candidate's edge (as eg_first: n_pts + 1 = free), all
  // checked to the end (a pure function of the two configurations): connect takes them instead of its two jobs
  int first0, nfirst;          // nfirst: candidates checked (-1: none, the record carries no validity)
  int first[MAX_NEAR];
};
// Pre-solution record (DESIGN.md "Pre-solution commits"): everything pre_commit needs, written by the scout at the
// end of its pass as data-tagged granules (tag = iteration + 1 in the high 32 bits, one 32-bit half of the struct
// in the low 32), so the leader reads it whole in one round and knows it complete when every tag matches.
struct PreRec {
  double xr[NJ];               // the sample
  double nn_q[NJ];             // its nearest node's configuration over the snapshot (the expand edge's start)
  double nn_c[3];              // that node's cost
  double nn_d;                 // its distance (10000 if none)
  double ext[NJ], end[NJ];     // the expand edge's step target and end point (x_new)
  double acc[3];               // the expand edge's segment-norm sums
  double cn_d, cn_c[3];        // connect: x_new's nearest node in the other tree (distance, cost)
  double sol[3];               // connect: direct edge cost + x_new's cost
  double sel_q[NJ], sel_c[3];  // connect: the last stepped edge's node
  double sel_start[NJ], sel_target[NJ];
  int nn_id, X, t, first;      // nearest node, snapshot size, tree, expand edge's first collision
  int cn_id, XB, cn_ok, cn_first;  // connect's nearest node, other tree's snapshot size, 1 = computed, first collision
  int pre_ok, flag, nv, need;  // as ScoutPre
  int sel_id, sel_parent, pad[2];
};
constexpr int PRE_GRANULES = (int)(sizeof(PreRec) / 4);
static_assert(sizeof(PreRec) % 8 == 0 && PRE_GRANULES <= 4 * 64, "pre-solution record: one granule per lane of 4 waves");

struct ScoutRec {
  ScoutNN nn;
  ScoutExpand ex;
  ScoutConnect cn;
  ScoutPre pre;
  ScoutNear nr;
  ScoutConn cc;
  int n_choose, n_rewire, pad[2];
  ScoutEdge e[SCOUT_EDGES];    // [0] expand, [SCOUT_CHOOSE0 ..) choose-parent, [SCOUT_REWIRE0 ..) rewire
};
// Record slots of a scout board, by iteration mod SCOUT_SLOTS: a scout may be asked for iteration k + MAX_SCOUTS
// while the leader still reads its record of k (before the first solution the scouts take the iterations in turn,
// up to MAX_SCOUTS ahead).
constexpr int MAX_SCOUTS = 8;
constexpr int SCOUT_SLOTS = 16;
static_assert(SCOUT_SLOTS > MAX_SCOUTS && (SCOUT_SLOTS & (SCOUT_SLOTS - 1)) == 0, "record slots");
struct ScoutBoard {
  // leader -> scout: the request for iteration k carries tag k + 1; req[0] low word = X | t << 28 | opt << 29,
  // req[1] low word = the sampler parameter version, req[2] low word = XB (nodes of the other tree)
  unsigned long long req[3];
  int stop;                    // the leader left the launch
  int xcc;                     // the scout's XCD (XCC_ID) + 1, 0 = not yet known
  // leader -> scout, after the first solution: rewire commits on tree t begun (rwb) and finished (rwe), counted in
  // QState::rewires.  A record asked for before its tree's last rewires (early asks) is rebuilt by the scout when rwb
  // moves; both counters equal again = the tree's words are stored (DESIGN.md "Early asks")
  unsigned rwb[2], rwe[2];
  int pad0[4];
  unsigned long long cur;      // leader -> scout: the leader's current iteration (a record of an earlier one is stale)
  // leader -> scout, before the first solution: (iteration & 0xffffff) << 40 | n[0] << 20 | n[1], stored after the
  // iteration's drain, so both trees' first n nodes are visible (a scout binds its snapshot to it late)
  unsigned long long cur_sz;
  int pad2[28];
  unsigned long long stage[SCOUT_SLOTS];  // scout -> leader, by iteration mod SCOUT_SLOTS
  unsigned long long cgo;      // leader -> scout: granule (iteration k + 1, n of tree_B(k)) once tree_B(k) is final
  int pad1[14];
  unsigned long long prof[32]; // the scout's phase clocks of the launch (written when it leaves)
  ScoutRec rec[SCOUT_SLOTS];
  ViaNode pre_via[SCOUT_SLOTS][PRE_VIA];  // ScoutPre's via chains, by record slot
  unsigned long long pre_g[SCOUT_SLOTS][PRE_GRANULES];  // PreRec granules, by record slot
};

constexpr int ABORT_EVERY = 64;  // iterations between a leader's polls of the host's abort word (QueryDev::abort)
struct QueryDev {
  QState* st;
  JobBoard* jb;                // null: no helpers
  JobBoard* sampler_jb;        // scout: the leader's board (run-ahead sampler ring)
  // scouts (DESIGN.md "Scouts"): nscouts workgroups compute records of the leader's coming iterations -- before the
  // first solution iteration k goes to scout k mod nscouts (up to nscouts ahead), after it to scout k mod 2 (two
  // ahead); each has its record board, collision-job board, helpers and via-node scratch
  int nscouts;
  int pre_delay;               // before the first solution a scout starts record k once the leader is at k - pre_delay
  int pre_commit;              // 1: pre-solution iterations are committed from complete scout records
  int early_ask;               // 1: after the first solution, iteration k + 2 is asked for as soon as its scout is free
  int conn_check;              // 1: the scout's SC_CONN record carries the validity of connect's edges (scout_connect)
  int pre_refresh;             // bits 0/1: a pre-solution scout restarts its pass when a newer node is nearer
  ScoutBoard* scbs[MAX_SCOUTS];
  JobBoard* sjbs[MAX_SCOUTS];
  ViaNode* svias[MAX_SCOUTS];
  int sworkers_s[MAX_SCOUTS];  // scout + its tile helper workgroups
  // a scout workgroup's own board, job board, via scratch and workers (set by scout_main)
  ScoutBoard* scb;
  JobBoard* sjb;
  ViaNode* svia;
  int sworkers;
  int* trace;                  // debug only (SMP_DEBUG): host-mapped progress markers of the leader
  // queries of this launch that finished in it (shared by all of the launch's queries); once it reaches lquota > 0
  // every leader ends the launch after its current iteration, so that the host re-provisions the CUs of the
  // finished queries to the others (DESIGN.md "Many queries")
  unsigned* lfin;
  int lquota;
  long long lticks;            // > 0: the launch ends this many device-clock ticks after it started (resumable), so
                               // that the host re-provisions (DESIGN.md "Many queries")
  unsigned* ttff;              // host-mapped word set to 1 when the first feasible path is committed (null: none)
  // host-mapped word the host sets when it abandons a planning call (its wait timed out): every leader polls it every
  // ABORT_EVERY iterations and ends the launch (its stop words send its scouts and helpers home), so an abandoned
  // launch drains instead of holding the CUs to the end of its budget (null: none)
  const unsigned* abort;
  int scan_min;                // nodes in a scan's range from which it is split over the helpers (0: never)
  int scan_pnn, scan_pnear;    // participants (this workgroup + helpers) of a split nearest / near scan, <= SCAN_P
  int scan_nshift;             // a split near scan takes one participant per 2^scan_nshift nodes (at least 8)
  int scan_ps0;                // the publisher's slice is 1 / 2^scan_ps0 of a helper's
  int nworkers;                // leader + tile helper workgroups (tile w, w + nworkers, ... is worker w's)
  int tile_ct;                 // configurations per job tile: 0 = by job size (job_tile_ct), else 1 / 2 / 4 / 8
  int sampler;                 // 1: the last helper workgroup is the run-ahead sampler
  TreeDev tr[2];
  ViaNode* via;                // [via_cap]
  int* stack;                  // [cap] DFS stack of recursiveNodeCostUpdate
  double* rows;                // [max_iter][5] cost evolution rows (may be null)
  long long rows_cap;
  int* path_nodes;             // [2][cap] path extraction scratch
};

}  // namespace smp
