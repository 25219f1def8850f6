// Host-side builders of the device model and scene.  See smp_host.h.
#include "smp_host.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <map>
#include <stdexcept>

#include "smp_json.h"

namespace smp {

static int type_code(const std::string& t) {
  if (t == "RotAxis") return 1;
  if (t == "TransAxis") return 2;
  return 0;
}

static void copy3(const json::Value& v, double* o, int n = 3) {
  if (v.size() != (size_t)n) throw std::runtime_error("model: bad vector length");
  for (int i = 0; i < n; ++i) o[i] = v[i].d();
}

// Robot model JSON (tools/gen_robot_model.py).  Mirrors KDLRobotModel + CollisionChecker construction.
void robot_from_json(const std::string& text, RobotHost* out) {
  const json::Value m = json::parse(text.c_str());
  robot_from_model_value(m, out);
}

// The model's key / value form -> RobotDev (shared by the JSON path and the URDF + SRDF path, smp_urdf.cpp).
void robot_from_model_value(const json::Value& m, RobotHost* out) {
  RobotDev& d = out->dev;
  std::memset(&d, 0, sizeof(d));
  d.root_z = m["root_z"].d();
  const json::Value& links = m["links"];
  out->link_names.clear();
  for (size_t i = 0; i < links.size(); ++i) out->link_names.push_back(links[i]["name"].s());
  const json::Value& bc = m["body_chain"];
  d.n_chain = (int)bc.size();
  if (d.n_chain > MAX_CHAIN) throw std::runtime_error("model: body chain too long");
  for (int k = 0; k < d.n_chain; ++k) {
    const json::Value& e = bc[k];
    d.ch_type[k] = type_code(e["type"].s());
    d.ch_joint[k] = e["joint"].i();
    d.ch_body[k] = e["body"].i();
    copy3(e["axis"], &d.ch_axis[k * 3]);
    copy3(e["origin"], &d.ch_origin[k * 3]);
    copy3(e["R"], &d.ch_R[k * 9], 9);
    copy3(e["p"], &d.ch_p[k * 3]);
  }
  d.n_body = (int)m["bodies"].size();
  if (d.n_body > MAX_BODY) throw std::runtime_error("model: too many bodies");
  const json::Value& ch = m["chain"];
  d.n_seg = (int)ch.size();
  if (d.n_seg > MAX_SEG) throw std::runtime_error("model: chain too long");
  for (int s = 0; s < d.n_seg; ++s) {
    const json::Value& e = ch[s];
    d.seg_type[s] = type_code(e["type"].s());
    d.seg_joint[s] = e["joint"].i();
    copy3(e["axis"], &d.seg_axis[s * 3]);
    copy3(e["origin"], &d.seg_origin[s * 3]);
    copy3(e["ftip_R"], &d.seg_R[s * 9], 9);
    copy3(e["ftip_p"], &d.seg_p[s * 3]);
  }

  // collision links -> compact slots (order of link_bounds)
  const json::Value& lb = m["link_bounds"];
  d.n_clink = (int)lb.size();
  if (d.n_clink > MAX_CLINK) throw std::runtime_error("model: too many collision links");
  out->clink_of_link.assign(links.size(), -1);
  for (int c = 0; c < d.n_clink; ++c) {
    int li = lb[c]["link"].i();
    out->clink_of_link[li] = c;
    d.cl_link[c] = li;
    d.cl_body[c] = lb[c]["body"].i();
    copy3(lb[c]["cb"], &d.cl_cb[c * 3]);
    d.cl_r[c] = lb[c]["r"].d();
  }
  // spheres sorted by clink slot (stable)
  const json::Value& S = m["spheres"];
  d.n_sph = (int)S.size();
  if (d.n_sph > MAX_SPH) throw std::runtime_error("model: too many spheres");
  std::vector<int> order(d.n_sph);
  for (int i = 0; i < d.n_sph; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    return out->clink_of_link[S[a]["link"].i()] < out->clink_of_link[S[b]["link"].i()];
  });
  for (int c = 0; c < d.n_clink; ++c) { d.cl_sph0[c] = 0; d.cl_nsph[c] = 0; }
  for (int k = 0; k < d.n_sph; ++k) {
    const json::Value& s = S[order[k]];
    int c = out->clink_of_link[s["link"].i()];
    if (c < 0) throw std::runtime_error("model: sphere on a link without bounds");
    d.sph_clink[k] = c;
    d.sph_body[k] = s["body"].i();
    copy3(s["cb"], &d.sph_cb[k * 3]);
    d.sph_r[k] = s["r"].d();
    if (d.cl_nsph[c] == 0) d.cl_sph0[c] = k;
    d.cl_nsph[c]++;
  }
  for (int j = 0; j < NJ; ++j) {
    d.q_min[j] = m["q_min"][j].d();
    d.q_max[j] = m["q_max"][j].d();
    d.rev[j] = m["joint_is_revolute"][j].i();
  }
  // exact primitives (format 2; a format-1 model has none)
  for (int c = 0; c < d.n_clink; ++c) d.cl_prim[c] = -1;
  d.n_prim = 0;
  if (m.has("prims")) {
    const json::Value& PR = m["prims"];
    d.n_prim = (int)PR.size();
    if (d.n_prim > MAX_PRIM) throw std::runtime_error("model: too many primitives");
    for (int k = 0; k < d.n_prim; ++k) {
      const json::Value& e = PR[k];
      const int c = out->clink_of_link[e["link"].i()];
      if (c < 0 || d.cl_nsph[c] > 0 || d.cl_prim[c] >= 0) throw std::runtime_error("model: bad primitive link");
      const std::string ty = e["type"].s();
      d.prim_type[k] = ty == "box" ? 1 : ty == "cylinder" ? 2 : 0;
      if (!d.prim_type[k]) throw std::runtime_error("model: unknown primitive type " + ty);
      d.prim_body[k] = e["body"].i();
      d.prim_clink[k] = c;
      d.cl_prim[c] = k;
      copy3(e["cb"], &d.prim_cb[k * 3]);
      copy3(e["ab"], &d.prim_ab[k * 3]);
      copy3(e["half"], &d.prim_h[k * 3]);
      d.prim_rxy[k] = e["rxy"].d();
    }
  }
  for (int c = 0; c < d.n_clink; ++c)
    if (d.cl_nsph[c] == 0 && d.cl_prim[c] < 0) throw std::runtime_error("model: collision link without geometry");
  const json::Value& P = m["self_pairs"];
  d.n_pairs = (int)P.size();
  if (d.n_pairs > MAX_PAIRS) throw std::runtime_error("model: too many pairs");
  for (int p = 0; p < d.n_pairs; ++p) {
    d.pair_a[p] = out->clink_of_link[P[p][0].i()];
    d.pair_b[p] = out->clink_of_link[P[p][1].i()];
    if (d.pair_a[p] < 0 || d.pair_b[p] < 0) throw std::runtime_error("model: pair on a link without geometry");
  }
  finish_pairs(&d);
}

// Flat self-collision lists of the enabled link pairs: every sphere pair of two sphere links in (link pair, sphere
// of a, sphere of b) order with (ra + rb)^2 rounded as the device would, and every (primitive, sphere) pair of a
// primitive link and a sphere link.  Two primitive links in one pair would have to be rigidly attached (both sit on
// the planar base), and rigid pairs are not in the model.
void finish_pairs(RobotDev* dp) {
  RobotDev& d = *dp;
  d.n_spairs = 0;
  d.n_ppairs = 0;
  for (int p = 0; p < d.n_pairs; ++p) {
    int a = d.pair_a[p], b = d.pair_b[p];
    if (d.cl_prim[a] >= 0 && d.cl_prim[b] >= 0) throw std::runtime_error("model: primitive-primitive pair");
    if (d.cl_prim[a] >= 0 || d.cl_prim[b] >= 0) {
      const int pr = d.cl_prim[a] >= 0 ? d.cl_prim[a] : d.cl_prim[b], sl = d.cl_prim[a] >= 0 ? b : a;
      for (int s = d.cl_sph0[sl]; s < d.cl_sph0[sl] + d.cl_nsph[sl]; ++s) {
        if (d.n_ppairs >= MAX_PPAIRS) throw std::runtime_error("model: too many primitive-sphere pairs");
        d.pp_ps[d.n_ppairs++] = (uint16_t)(pr | (s << 8));
      }
      continue;
    }
    for (int sa = d.cl_sph0[a]; sa < d.cl_sph0[a] + d.cl_nsph[a]; ++sa)
      for (int sb = d.cl_sph0[b]; sb < d.cl_sph0[b] + d.cl_nsph[b]; ++sb) {
        if (d.n_spairs >= MAX_SPAIRS) throw std::runtime_error("model: too many sphere pairs");
        if (sa > 255 || sb > 255) throw std::runtime_error("model: sphere index out of range");
        volatile double rs = d.sph_r[sa] + d.sph_r[sb];
        d.sp_ab[d.n_spairs] = (uint16_t)(sa | (sb << 8));
        d.sp_rr2[d.n_spairs] = rs * rs;
        d.n_spairs++;
      }
  }
}

// ------------------------------------------------------------------------------------------ scene
// Padding around the occupied keys: more than the largest horizontal reach of any sphere (<= 0.30 m) or primitive
// (rxy <= 0.45 m; robotino's front shell box 0.389 m) plus a cell, so a centre outside the grid is free of the map.
int grid_pad_cells(double res) { return (int)std::ceil(GRID_REACH / res) + 2; }

// World z of every primitive's centre: its body is planar (tools/gen_robot_model.py), so the body frame at q = 0
// gives the z every configuration has (up to rounding; the slab adds a margin).
static void prim_z(const RobotDev& d, double* zc) {
  double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, P[3] = {0, 0, d.root_z};
  double BR[MAX_BODY][9], BP[MAX_BODY][3];
  for (int k = 0; k < d.n_chain; ++k) {
    double LR[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, LP[3];
    for (int i = 0; i < 3; ++i) LP[i] = d.ch_origin[k * 3 + i];
    if (d.ch_type[k] == 0) {
      for (int i = 0; i < 9; ++i) LR[i] = d.ch_R[k * 9 + i];
      for (int i = 0; i < 3; ++i) LP[i] = d.ch_p[k * 3 + i];
    }
    double NR[9], NP[3];
    for (int r = 0; r < 3; ++r) {
      for (int c = 0; c < 3; ++c) NR[r * 3 + c] = R[r * 3] * LR[c] + R[r * 3 + 1] * LR[3 + c] + R[r * 3 + 2] * LR[6 + c];
      NP[r] = (R[r * 3] * LP[0] + R[r * 3 + 1] * LP[1] + R[r * 3 + 2] * LP[2]) + P[r];
    }
    std::memcpy(R, NR, sizeof(R));
    std::memcpy(P, NP, sizeof(P));
    if (d.ch_body[k] >= 0) { std::memcpy(BR[d.ch_body[k]], R, sizeof(R)); std::memcpy(BP[d.ch_body[k]], P, sizeof(P)); }
  }
  for (int p = 0; p < d.n_prim; ++p) {
    const double* B = BR[d.prim_body[p]];
    const double* c = &d.prim_cb[p * 3];
    zc[p] = (B[6] * c[0] + B[7] * c[1] + B[8] * c[2]) + BP[d.prim_body[p]][2];
  }
}

void prim_slabs(const RobotDev& d, const SceneHost& s, std::vector<std::vector<uint16_t>>* out) {
  out->assign(d.n_prim, {});
  double zc[MAX_PRIM];
  prim_z(d, zc);
  for (int p = 0; p < d.n_prim; ++p) {
    const double hz = d.prim_type[p] == 1 ? d.prim_h[p * 3 + 2] : d.prim_h[p * 3 + 1];
    const double zlo = zc[p] - hz - 1e-6, zhi = zc[p] + hz + 1e-6;
    // layers whose cell boxes meet [zlo, zhi]
    int k0 = std::max(0, (int)std::floor((zlo - s.oz) / s.res) - 1), k1 = std::min(s.nz - 1, (int)std::floor((zhi - s.oz) / s.res) + 1);
    while (k0 <= k1 && s.oz + (double)(k0 + 1) * s.res < zlo) ++k0;
    while (k1 >= k0 && s.oz + (double)k1 * s.res > zhi) --k1;
    std::vector<uint8_t> proj((size_t)s.nx * s.ny, 0);
    for (int k = k0; k <= k1; ++k)
      for (int j = 0; j < s.ny; ++j) {
        const uint64_t* row = s.bits.data() + ((size_t)k * s.ny + j) * s.wx;
        for (int w = 0; w < s.wx; ++w)
          for (uint64_t m = row[w]; m; m &= m - 1) proj[(size_t)j * s.nx + w * 64 + __builtin_ctzll(m)] = 1;
      }
    box_gap_squared(proj, s.nx, s.ny, 1, &(*out)[p]);
  }
}

// d2 is a lower bound of (distance from any point of the cell to any occupied box / res)^2, so a sphere of
// radius r whose centre cell has d2 > T cannot touch an occupied box; the 1e-6 m margin absorbs rounding.
uint32_t sphere_threshold(double r, double res) {
  double a = (r + 1e-6) / res;
  return (uint32_t)std::floor(a * a);
}

// 1-D squared distance transform of f (Felzenszwalb & Huttenlocher 2012), in place.
static void dt1d(double* f, int n, int stride, std::vector<double>& tmp, std::vector<int>& v, std::vector<double>& z) {
  const double INF = std::numeric_limits<double>::infinity();
  tmp.resize(n);
  v.resize(n);
  z.resize(n + 1);
  for (int i = 0; i < n; ++i) tmp[i] = f[(size_t)i * stride];
  int k = -1;
  for (int q = 0; q < n; ++q) {
    if (tmp[q] == INF) continue;
    double s = 0.0;
    while (k >= 0) {  // z[0] = -inf, so the first parabola is never popped
      int vk = v[k];
      s = ((tmp[q] + (double)q * q) - (tmp[vk] + (double)vk * vk)) / (2.0 * q - 2.0 * vk);
      if (s <= z[k]) --k; else break;
    }
    if (k < 0) { k = 0; v[0] = q; z[0] = -INF; z[1] = INF; continue; }
    ++k;
    v[k] = q;
    z[k] = s;
    z[k + 1] = INF;
  }
  if (k < 0) return;  // all infinite: unchanged
  int j = 0;
  for (int q = 0; q < n; ++q) {
    while (z[j + 1] < q) ++j;
    double dq = (double)(q - v[j]);
    f[(size_t)q * stride] = dq * dq + tmp[v[j]];
  }
}

void edt_squared(const std::vector<uint8_t>& occ, int nx, int ny, int nz, std::vector<uint16_t>* d2) {
  const double INF = std::numeric_limits<double>::infinity();
  size_t n = (size_t)nx * ny * nz;
  std::vector<double> f(n);
  bool any = false;
  for (size_t i = 0; i < n; ++i) { f[i] = occ[i] ? 0.0 : INF; any |= occ[i] != 0; }
  d2->assign(n, 65535);
  if (!any) return;
  std::vector<double> tmp, z;
  std::vector<int> v;
  for (int k = 0; k < nz; ++k)
    for (int j = 0; j < ny; ++j) dt1d(&f[((size_t)k * ny + j) * nx], nx, 1, tmp, v, z);
  for (int k = 0; k < nz; ++k)
    for (int i = 0; i < nx; ++i) dt1d(&f[(size_t)k * ny * nx + i], ny, nx, tmp, v, z);
  for (int j = 0; j < ny; ++j)
    for (int i = 0; i < nx; ++i) dt1d(&f[(size_t)j * nx + i], nz, nx * ny, tmp, v, z);
  for (size_t i = 0; i < n; ++i) (*d2)[i] = f[i] >= 65535.0 ? 65535 : (uint16_t)f[i];
}

void box_gap_squared(const std::vector<uint8_t>& occ, int nx, int ny, int nz, std::vector<uint16_t>* d2) {
  // 3x3x3 dilation (separable max over +-1 per axis), then the EDT: the squared distance from cell u to the
  // dilated set is min over occupied o of sum_axis max(|u - o| - 1, 0)^2, the box-to-box gap.
  std::vector<uint8_t> a(occ), b(occ.size());
  const size_t sx = 1, sy = (size_t)nx, sz = (size_t)nx * ny;
  const int n[3] = {nx, ny, nz};
  const size_t st[3] = {sx, sy, sz};
  for (int ax = 0; ax < 3; ++ax) {
    for (int k = 0; k < nz; ++k)
      for (int j = 0; j < ny; ++j)
        for (int i = 0; i < nx; ++i) {
          size_t c = (size_t)k * sz + (size_t)j * sy + i;
          int pos = ax == 0 ? i : (ax == 1 ? j : k);
          uint8_t v = a[c];
          if (pos > 0) v |= a[c - st[ax]];
          if (pos + 1 < n[ax]) v |= a[c + st[ax]];
          b[c] = v;
        }
    a.swap(b);
  }
  edt_squared(a, nx, ny, nz, d2);
}

void build_bricks(SceneHost* h) {
  h->bnx = (h->nx + 3) / 4;
  h->bny = (h->ny + 3) / 4;
  h->bnz = (h->nz + 3) / 4;
  h->bricks.assign((size_t)h->bnx * h->bny * h->bnz, 0);
  for (int k = 0; k < h->nz; ++k)
    for (int j = 0; j < h->ny; ++j) {
      const uint64_t* row = h->bits.data() + ((size_t)k * h->ny + j) * h->wx;
      for (int w = 0; w < h->wx; ++w) {
        uint64_t m = row[w];
        while (m) {
          int i = w * 64 + __builtin_ctzll(m);
          m &= m - 1;
          size_t b = ((size_t)(k >> 2) * h->bny + (j >> 2)) * h->bnx + (i >> 2);
          h->bricks[b] |= 1ull << (((k & 3) << 4) | ((j & 3) << 2) | (i & 3));
        }
      }
    }
}

void scene_from_keys(const uint16_t* keys, int64_t n, double res, double z_offset, SceneHost* out) {
  out->res = res;
  out->n_occupied = 0;
  if (n <= 0) {
    out->nx = out->ny = out->nz = 1;
    out->wx = 1;
    out->ox = out->oy = 0.0;
    out->oz = 0.0 + z_offset;
    out->bits.assign(1, 0);
    out->d2.assign(1, 65535);
    for (int d = 0; d < 3; ++d) out->bbox_min[d] = out->bbox_max[d] = 0.0;
    build_bricks(out);
    return;
  }
  int kmin[3] = {1 << 30, 1 << 30, 1 << 30}, kmax[3] = {-1, -1, -1};
  for (int64_t i = 0; i < n; ++i)
    for (int d = 0; d < 3; ++d) {
      int k = keys[i * 3 + d];
      kmin[d] = std::min(kmin[d], k);
      kmax[d] = std::max(kmax[d], k);
    }
  int pad = grid_pad_cells(res);
  for (int d = 0; d < 3; ++d) {
    out->bbox_min[d] = (double)(kmin[d] - KEY_OFFSET) * res;
    out->bbox_max[d] = (double)(kmax[d] - KEY_OFFSET + 1) * res;
    kmin[d] -= pad;
    kmax[d] += pad;
  }
  out->nx = kmax[0] - kmin[0] + 1;
  out->ny = kmax[1] - kmin[1] + 1;
  out->nz = kmax[2] - kmin[2] + 1;
  out->wx = (out->nx + 63) / 64;
  out->ox = (double)(kmin[0] - KEY_OFFSET) * res;
  out->oy = (double)(kmin[1] - KEY_OFFSET) * res;
  out->oz = (double)(kmin[2] - KEY_OFFSET) * res + z_offset;
  size_t ncell = (size_t)out->nx * out->ny * out->nz;
  std::vector<uint8_t> occ(ncell, 0);
  out->bits.assign((size_t)out->wx * out->ny * out->nz, 0);
  for (int64_t i = 0; i < n; ++i) {
    int x = keys[i * 3] - kmin[0], y = keys[i * 3 + 1] - kmin[1], z = keys[i * 3 + 2] - kmin[2];
    size_t c = ((size_t)z * out->ny + y) * out->nx + x;
    if (!occ[c]) {
      occ[c] = 1;
      out->n_occupied++;
      out->bits[((size_t)z * out->ny + y) * out->wx + (x >> 6)] |= 1ull << (x & 63);
    }
  }
  box_gap_squared(occ, out->nx, out->ny, out->nz, &out->d2);
  build_bricks(out);
}

void floor_keys(double cx, double cy, double res, double distance, std::vector<uint16_t>* keys,
                const std::vector<FreeLeaf>* free) {
  // octree->coordToKey(x, y, -res/2): key = floor(coord * (1 / res)) + 32768 (octomap OcTreeBaseImpl::coordToKey,
  // resolution_factor = 1.0 / resolution)
  const double f = 1.0 / res;
  int kx = (int)std::floor(f * cx) + KEY_OFFSET;
  int ky = (int)std::floor(f * cy) + KEY_OFFSET;
  int kz = (int)std::floor(f * (-res * 0.5)) + KEY_OFFSET;
  int nd = (int)(distance / res);
  // updateNode(key, true) adds prob_hit_log (logodds(0.7), float) to an existing leaf: a free leaf stays free
  // when its log-odds plus the hit stay below the occupancy threshold (logodds(0.5) = 0).  Only the free leaves
  // whose key range holds the floor plane matter.
  // a leaf at depth d with centre key k covers keys [k - h, k - h + s), h = 32768 >> d, s = 65536 >> d
  auto inside = [](const FreeLeaf& l, int a, int v) {
    const int lo = l.k[a] - (KEY_OFFSET >> l.depth);
    return v >= lo && v < lo + ((2 * KEY_OFFSET) >> l.depth);
  };
  std::vector<FreeLeaf> fl;
  if (free)
    for (const FreeLeaf& l : *free)
      if (inside(l, 2, kz) && !(l.v + kHitLogOdds >= 0.0f)) fl.push_back(l);
  for (int x = kx - nd; x <= kx + nd; ++x)
    for (int y = ky - nd; y <= ky + nd; ++y) {
      bool stays_free = false;
      for (const FreeLeaf& l : fl)
        if (inside(l, 0, x) && inside(l, 1, y)) { stays_free = true; break; }
      if (stays_free) continue;
      keys->push_back((uint16_t)x);
      keys->push_back((uint16_t)y);
      keys->push_back((uint16_t)kz);
    }
}

// Occupied leaf (depth, centre key) -> its depth-16 keys; a pruned leaf at depth d covers [k - h, k + h - 1],
// h = 32768 >> d, on every axis.
namespace {
// Occupied voxels one stream may expand to (a pruned leaf at depth d stands for (2^(16-d))^3 of them): a corrupted or
// hostile payload must not exhaust memory.  2^26 voxels is a 2 cm grid of 27 x 27 x 2 m fully occupied.
size_t kMaxVoxels = (size_t)1 << 26;

void emit_leaf(std::vector<uint16_t>* keys, int depth, int kx, int ky, int kz) {
  if (depth < 6) throw std::runtime_error("octomap: occupied leaf too coarse to expand");
  const size_t side = depth >= 16 ? 1 : (size_t)2 * (KEY_OFFSET >> depth);
  if (keys->size() / 3 + side * side * side > kMaxVoxels) throw std::runtime_error("octomap: too many occupied voxels");
  if (depth >= 16) {
    keys->push_back((uint16_t)kx); keys->push_back((uint16_t)ky); keys->push_back((uint16_t)kz);
    return;
  }
  int h = KEY_OFFSET >> depth;
  for (int z = kz - h; z < kz + h; ++z)
    for (int y = ky - h; y < ky + h; ++y)
      for (int x = kx - h; x < kx + h; ++x) {
        keys->push_back((uint16_t)x); keys->push_back((uint16_t)y); keys->push_back((uint16_t)z);
      }
}

// Child i of a node at depth d with centre key k (octomap computeChildKey): bit 0/1/2 of i selects +x/+y/+z.
inline void child_key(int depth, int i, const int* k, int* c) {
  const int half = KEY_OFFSET >> (depth + 1);
  for (int a = 0; a < 3; ++a) c[a] = k[a] + (((i >> a) & 1) ? half : -half - (half ? 0 : 1));
}

// Octomap binary format (OccupancyOcTreeBase::readBinaryNode): per inner node two bytes, 2 bits per child --
// 00 unknown, bit 2i only: free leaf (log-odds clamping_thres_min), bit 2i+1 only: occupied leaf
// (clamping_thres_max), both: inner node -- then the inner children recursively in child order.
struct BtReader {
  const uint8_t* p;
  const uint8_t* end;
  std::vector<uint16_t>* keys;
  std::vector<FreeLeaf>* free;
  void node(int depth, const int* k) {
    if (end - p < 2) throw std::runtime_error("octomap: truncated binary stream");
    const uint8_t c14 = *p++, c58 = *p++;
    int inner[8];
    for (int i = 0; i < 8; ++i) {
      const uint8_t byte = i < 4 ? c14 : c58;
      const int b = (i & 3) * 2;
      const int b0 = (byte >> b) & 1, b1 = (byte >> (b + 1)) & 1;
      inner[i] = b0 && b1;
      int c[3];
      child_key(depth, i, k, c);
      if (!b0 && b1) emit_leaf(keys, depth + 1, c[0], c[1], c[2]);
      else if (b0 && !b1 && free) free->push_back({depth + 1, {c[0], c[1], c[2]}, kClampMinLogOdds});
    }
    for (int i = 0; i < 8; ++i) {
      if (!inner[i]) continue;
      if (depth + 1 >= 16) throw std::runtime_error("octomap: inner node below max depth");
      int c[3];
      child_key(depth, i, k, c);
      node(depth + 1, c);
    }
  }
};

// Octomap full format (OcTreeDataNode::readData / OcTreeBaseImpl::readNodesRecurs): per node its value (float
// log-odds) and one byte whose bit i says child i exists, then the existing children recursively in child order.
// A node without children is a leaf, occupied iff log-odds >= occ_prob_thres_log = logodds(0.5) = 0
// (OccupancyOcTreeBase::isNodeOccupied).
struct OtReader {
  const uint8_t* p;
  const uint8_t* end;
  std::vector<uint16_t>* keys;
  std::vector<FreeLeaf>* free;
  void node(int depth, const int* k) {
    if (end - p < 5) throw std::runtime_error("octomap: truncated full stream");
    float v;
    std::memcpy(&v, p, 4);
    const uint8_t m = p[4];
    p += 5;
    if (m == 0) {
      if (v >= 0.0f) emit_leaf(keys, depth, k[0], k[1], k[2]);
      else if (free) free->push_back({depth, {k[0], k[1], k[2]}, v});
      return;
    }
    if (depth >= 16) throw std::runtime_error("octomap: children below max depth");
    for (int i = 0; i < 8; ++i) {
      if (!((m >> i) & 1)) continue;
      int c[3];
      child_key(depth, i, k, c);
      node(depth + 1, c);
    }
  }
};

// Text header of .bt / .ot files (AbstractOcTree::readHeader): comment lines, "id", "size", "res", then "data".
// Returns the first byte after the "data" line; *nodes = -1 when no size line was given.
const uint8_t* octomap_header(const uint8_t* data, size_t size, double* res, long long* nodes) {
  const uint8_t* p = data;
  const uint8_t* end = data + size;
  bool have_res = false;
  std::string id;
  *nodes = -1;
  for (;;) {
    const uint8_t* nl = (const uint8_t*)memchr(p, '\n', end - p);
    if (!nl) throw std::runtime_error("octomap: header not terminated");
    std::string line((const char*)p, nl - p);
    p = nl + 1;
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.empty() || line[0] == '#') continue;
    if (line.rfind("id ", 0) == 0) id = line.substr(3);
    else if (line.rfind("size ", 0) == 0) *nodes = atoll(line.c_str() + 5);
    else if (line.rfind("res ", 0) == 0) { *res = strtod(line.c_str() + 4, nullptr); have_res = true; }
    else if (line == "data") break;
  }
  if (!have_res || !(*res > 0) || (id != "OcTree" && !id.empty())) throw std::runtime_error("octomap: unsupported header");
  return p;
}
}  // namespace

void set_max_octomap_voxels(size_t n) { kMaxVoxels = n; }

void octomap_bt_keys(const uint8_t* data, size_t size, double* res, std::vector<uint16_t>* keys,
                     std::vector<FreeLeaf>* free, bool header) {
  const uint8_t* p = data;
  if (header) {
    long long nodes;
    p = octomap_header(data, size, res, &nodes);
    if (nodes == 0) return;
  }
  if (p == data + size) return;  // empty tree
  BtReader r{p, data + size, keys, free};
  const int root[3] = {KEY_OFFSET, KEY_OFFSET, KEY_OFFSET};
  r.node(0, root);
}

void octomap_ot_keys(const uint8_t* data, size_t size, double* res, std::vector<uint16_t>* keys,
                     std::vector<FreeLeaf>* free, bool header) {
  const uint8_t* p = data;
  if (header) {
    long long nodes;
    p = octomap_header(data, size, res, &nodes);
    if (nodes == 0) return;
  }
  if (p == data + size) return;  // empty tree
  OtReader r{p, data + size, keys, free};
  const int root[3] = {KEY_OFFSET, KEY_OFFSET, KEY_OFFSET};
  r.node(0, root);
}

}  // namespace smp
