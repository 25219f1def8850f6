// URDF + SRDF (+ the sphere covers of the mesh links) -> robot model: the path the ROS node takes at start-up,
// BiRRTstarPlanner::initialize -> KDLRobotModel (kdl_kuka_model.cpp:12-236: chain, float-cast limits) and
// CollisionChecker (collision_checker.hpp:176-193 KDL tree, 263-351 collision geometry, 353-393 SRDF self pairs).
//
// The model is assembled as the same key/value structure tools/gen_robot_model.py writes (robotino_model.json), with
// the same arithmetic in the same order, and handed to the JSON path's assembly: both routes give the identical
// RobotDev (tests/test_host_cpu.py compares them byte for byte).  Geometry rules (DESIGN.md "Collision model"):
//   * box / cylinder collision links are exact primitives when upright on a planar body (the robotino base), unless
//     the sphere spec lists spheres for them;
//   * mesh links are the spheres of the spec (meshes are not read here);
//   * a pair of links whose relative pose depends on no planning joint is rigid and is left out (its state is the
//     same for every configuration).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "smp_host.h"
#include "smp_json.h"

namespace smp {
namespace {

// ------------------------------------------------------------------------------------------ minimal XML reader
struct XNode {
  std::string tag;
  std::map<std::string, std::string> attr;
  std::vector<XNode> kids;
  const XNode* child(const std::string& t) const {
    for (const XNode& k : kids)
      if (k.tag == t) return &k;
    return nullptr;
  }
  const std::string* get(const std::string& a) const {
    auto it = attr.find(a);
    return it == attr.end() ? nullptr : &it->second;
  }
};

class XmlReader {
 public:
  explicit XmlReader(const std::string& t) : s_(t), p_(0) {}
  XNode root() {
    for (;;) {
      skip_misc();
      if (p_ >= s_.size()) throw std::runtime_error("xml: no root element");
      if (s_[p_] == '<') return element();
      ++p_;  // stray text before the root
    }
  }

 private:
  const std::string& s_;
  size_t p_;
  bool starts(const char* t) const { return s_.compare(p_, std::strlen(t), t) == 0; }
  void skip_to(const char* t) {
    size_t q = s_.find(t, p_);
    if (q == std::string::npos) throw std::runtime_error(std::string("xml: unterminated ") + t);
    p_ = q + std::strlen(t);
  }
  // comments, processing instructions, doctype and whitespace
  void skip_misc() {
    for (;;) {
      while (p_ < s_.size() && std::isspace((unsigned char)s_[p_])) ++p_;
      if (starts("<!--")) skip_to("-->");
      else if (starts("<?")) skip_to("?>");
      else if (starts("<!")) skip_to(">");
      else return;
    }
  }
  std::string name() {
    size_t b = p_;
    while (p_ < s_.size() && !std::isspace((unsigned char)s_[p_]) && s_[p_] != '>' && s_[p_] != '/' && s_[p_] != '=')
      ++p_;
    if (b == p_) throw std::runtime_error("xml: expected a name");
    return s_.substr(b, p_ - b);
  }
  static std::string unescape(const std::string& v) {
    std::string o;
    for (size_t i = 0; i < v.size(); ++i) {
      if (v[i] != '&') { o += v[i]; continue; }
      size_t e = v.find(';', i);
      if (e == std::string::npos) { o += v[i]; continue; }
      const std::string ent = v.substr(i + 1, e - i - 1);
      if (ent == "lt") o += '<';
      else if (ent == "gt") o += '>';
      else if (ent == "amp") o += '&';
      else if (ent == "quot") o += '"';
      else if (ent == "apos") o += '\'';
      else o += v.substr(i, e - i + 1);
      i = e;
    }
    return o;
  }
  XNode element(int depth = 0) {
    if (depth > 256) throw std::runtime_error("xml: elements nested too deeply");
    XNode n;
    ++p_;  // '<'
    n.tag = name();
    for (;;) {
      while (p_ < s_.size() && std::isspace((unsigned char)s_[p_])) ++p_;
      if (p_ >= s_.size()) throw std::runtime_error("xml: unterminated tag " + n.tag);
      if (s_[p_] == '/') {
        if (p_ + 1 >= s_.size() || s_[p_ + 1] != '>') throw std::runtime_error("xml: bad empty tag " + n.tag);
        p_ += 2;
        return n;
      }
      if (s_[p_] == '>') { ++p_; break; }
      const std::string a = name();
      while (p_ < s_.size() && std::isspace((unsigned char)s_[p_])) ++p_;
      if (p_ >= s_.size() || s_[p_] != '=') throw std::runtime_error("xml: attribute without value in " + n.tag);
      ++p_;
      while (p_ < s_.size() && std::isspace((unsigned char)s_[p_])) ++p_;
      if (p_ >= s_.size() || (s_[p_] != '"' && s_[p_] != '\'')) throw std::runtime_error("xml: unquoted attribute");
      const char q = s_[p_++];
      const size_t e = s_.find(q, p_);
      if (e == std::string::npos) throw std::runtime_error("xml: unterminated attribute");
      n.attr[a] = unescape(s_.substr(p_, e - p_));
      p_ = e + 1;
    }
    // content: children, text (ignored), comments, CDATA
    for (;;) {
      if (p_ >= s_.size()) throw std::runtime_error("xml: unterminated element " + n.tag);
      if (starts("<!--")) { skip_to("-->"); continue; }
      if (starts("<![CDATA[")) { skip_to("]]>"); continue; }
      if (starts("<?")) { skip_to("?>"); continue; }
      if (starts("</")) {
        p_ += 2;
        const std::string t = name();
        if (t != n.tag) throw std::runtime_error("xml: </" + t + "> closes <" + n.tag + ">");
        while (p_ < s_.size() && s_[p_] != '>') ++p_;
        if (p_ >= s_.size()) throw std::runtime_error("xml: unterminated closing tag");
        ++p_;
        return n;
      }
      if (s_[p_] == '<') { n.kids.push_back(element(depth + 1)); continue; }
      ++p_;
    }
  }
};

// ------------------------------------------------------------------------------------------ KDL-style algebra
// Term by term as tools/gen_robot_model.py (fp64, no contraction): the two builders must give the same doubles.
struct F {
  double R[9];
  double p[3];
};
const F IDENT = {{1, 0, 0, 0, 1, 0, 0, 0, 1}, {0, 0, 0}};

void rot_mul(const double* a, const double* b, double* o) {
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) o[r * 3 + c] = a[r * 3 + 0] * b[0 * 3 + c] + a[r * 3 + 1] * b[1 * 3 + c] + a[r * 3 + 2] * b[2 * 3 + c];
}
void rot_vec(const double* a, const double* v, double* o) {
  for (int r = 0; r < 3; ++r) o[r] = a[r * 3 + 0] * v[0] + a[r * 3 + 1] * v[1] + a[r * 3 + 2] * v[2];
}
F frame_mul(const F& f1, const F& f2) {
  F o;
  rot_mul(f1.R, f2.R, o.R);
  double mp[3];
  rot_vec(f1.R, f2.p, mp);
  for (int i = 0; i < 3; ++i) o.p[i] = mp[i] + f1.p[i];
  return o;
}
// urdfdom Rotation::setFromRPY + normalize
void quat_from_rpy(double roll, double pitch, double yaw, double* q) {
  const double phi = roll / 2.0, the = pitch / 2.0, psi = yaw / 2.0;
  const double x = std::sin(phi) * std::cos(the) * std::cos(psi) - std::cos(phi) * std::sin(the) * std::sin(psi);
  const double y = std::cos(phi) * std::sin(the) * std::cos(psi) + std::sin(phi) * std::cos(the) * std::sin(psi);
  const double z = std::cos(phi) * std::cos(the) * std::sin(psi) - std::sin(phi) * std::sin(the) * std::cos(psi);
  const double w = std::cos(phi) * std::cos(the) * std::cos(psi) + std::sin(phi) * std::sin(the) * std::sin(psi);
  const double s = std::sqrt(x * x + y * y + z * z + w * w);
  if (s == 0.0) { q[0] = q[1] = q[2] = 0.0; q[3] = 1.0; return; }
  q[0] = x / s; q[1] = y / s; q[2] = z / s; q[3] = w / s;
}
// KDL::Rotation::Quaternion
void rot_from_quat(const double* q, double* R) {
  const double x = q[0], y = q[1], z = q[2], w = q[3];
  const double x2 = x * x, y2 = y * y, z2 = z * z, w2 = w * w;
  R[0] = w2 + x2 - y2 - z2; R[1] = 2 * x * y - 2 * w * z; R[2] = 2 * x * z + 2 * w * y;
  R[3] = 2 * x * y + 2 * w * z; R[4] = w2 - x2 + y2 - z2; R[5] = 2 * y * z - 2 * w * x;
  R[6] = 2 * x * z - 2 * w * y; R[7] = 2 * y * z + 2 * w * x; R[8] = w2 - x2 - y2 + z2;
}
// KDL::Rotation::Rot2 (builder side, libm sin / cos; only ever evaluated at q = 0 here)
void rot2(const double* ax, double angle, double* R) {
  const double ct = std::cos(angle), st = std::sin(angle);
  const double vt = 1 - ct;
  const double m_vt_0 = vt * ax[0], m_vt_1 = vt * ax[1], m_vt_2 = vt * ax[2];
  const double m_st_0 = ax[0] * st, m_st_1 = ax[1] * st, m_st_2 = ax[2] * st;
  const double m_vt_0_1 = m_vt_0 * ax[1], m_vt_0_2 = m_vt_0 * ax[2], m_vt_1_2 = m_vt_1 * ax[2];
  R[0] = ct + m_vt_0 * ax[0]; R[1] = -m_st_2 + m_vt_0_1; R[2] = m_st_1 + m_vt_0_2;
  R[3] = m_st_2 + m_vt_0_1; R[4] = ct + m_vt_1 * ax[1]; R[5] = -m_st_0 + m_vt_1_2;
  R[6] = -m_st_1 + m_vt_0_2; R[7] = m_st_0 + m_vt_1_2; R[8] = ct + m_vt_2 * ax[2];
}
// KDL::Vector::Norm
double kdl_norm(const double* v) {
  auto sq = [](double x) { return x * x; };
  const double a0 = std::fabs(v[0]), a1 = std::fabs(v[1]), a2 = std::fabs(v[2]);
  if (a0 >= a1) {
    if (a0 >= a2) {
      if (a0 == 0) return 0.0;
      return a0 * std::sqrt(1 + sq(v[1] / v[0]) + sq(v[2] / v[0]));
    }
    return a2 * std::sqrt(1 + sq(v[0] / v[2]) + sq(v[1] / v[2]));
  }
  if (a1 >= a2) return a1 * std::sqrt(1 + sq(v[0] / v[1]) + sq(v[2] / v[1]));
  return a2 * std::sqrt(1 + sq(v[0] / v[2]) + sq(v[1] / v[2]));
}
F frame_inverse(const F& f) {
  F o;
  const double* R = f.R;
  const double Rt[9] = {R[0], R[3], R[6], R[1], R[4], R[7], R[2], R[5], R[8]};
  std::memcpy(o.R, Rt, sizeof(Rt));
  double mp[3];
  rot_vec(Rt, f.p, mp);
  for (int i = 0; i < 3; ++i) o.p[i] = -mp[i];
  return o;
}

std::vector<double> floats(const std::string* s, size_t n) {
  std::vector<double> v;
  if (!s) return std::vector<double>(n, 0.0);
  const char* c = s->c_str();
  for (;;) {
    while (*c && std::isspace((unsigned char)*c)) ++c;
    if (!*c) break;
    char* e = nullptr;
    const double x = std::strtod(c, &e);
    if (e == c) throw std::runtime_error("urdf: bad number list '" + *s + "'");
    v.push_back(x);
    c = e;
  }
  return v;
}
std::vector<double> vec3(const std::string* s) {
  std::vector<double> v = floats(s, 3);
  if (v.size() != 3) throw std::runtime_error("urdf: expected three numbers, got '" + (s ? *s : std::string()) + "'");
  return v;
}

// kdl_parser joint: origin frame, KDL joint type, axis rotated into the parent frame and normalised
struct Joint {
  std::string name, type, parent, child;
  F Fo;
  double axis[3] = {0, 0, 0};
  double lower = 0.0, upper = 0.0;
  int kdl = 0;  // 0 None, 1 RotAxis, 2 TransAxis
  explicit Joint(const XNode& el) {
    const std::string* n = el.get("name");
    const std::string* t = el.get("type");
    const XNode* pa = el.child("parent");
    const XNode* ch = el.child("child");
    if (!n || !t || !pa || !ch || !pa->get("link") || !ch->get("link")) throw std::runtime_error("urdf: incomplete joint");
    name = *n; type = *t; parent = *pa->get("link"); child = *ch->get("link");
    const XNode* o = el.child("origin");
    const std::vector<double> xyz = vec3(o ? o->get("xyz") : nullptr), rpy = vec3(o ? o->get("rpy") : nullptr);
    double q[4];
    quat_from_rpy(rpy[0], rpy[1], rpy[2], q);
    rot_from_quat(q, Fo.R);
    for (int i = 0; i < 3; ++i) Fo.p[i] = xyz[i];
    const XNode* ax = el.child("axis");
    std::vector<double> au = {1.0, 0.0, 0.0};
    if (ax) au = vec3(ax->get("xyz"));
    const XNode* lim = el.child("limit");
    if (lim && lim->get("lower") && !lim->get("lower")->empty()) lower = std::strtod(lim->get("lower")->c_str(), nullptr);
    if (lim && lim->get("upper") && !lim->get("upper")->empty()) upper = std::strtod(lim->get("upper")->c_str(), nullptr);
    if (type == "revolute" || type == "continuous" || type == "prismatic") {
      double a[3];
      rot_vec(Fo.R, au.data(), a);
      const double nn = kdl_norm(a);
      if (!(nn > 0.0)) throw std::runtime_error("urdf: joint axis of zero length");
      for (int i = 0; i < 3; ++i) axis[i] = a[i] / nn;
      kdl = type == "prismatic" ? 2 : 1;
    }
  }
  F pose(double q) const {  // KDL::Joint::pose
    F o = IDENT;
    if (kdl == 1) {
      rot2(axis, q, o.R);
      for (int i = 0; i < 3; ++i) o.p[i] = Fo.p[i];
    } else if (kdl == 2) {
      for (int i = 0; i < 3; ++i) o.p[i] = Fo.p[i] + axis[i] * q;
    }
    return o;
  }
  F f_tip() const { return frame_mul(frame_inverse(pose(0.0)), Fo); }   // Segment ctor
  F frame_to_tip() const { return frame_mul(pose(0.0), f_tip()); }    // Segment::getFrameToTip
  const char* kdl_name() const { return kdl == 1 ? "RotAxis" : kdl == 2 ? "TransAxis" : "None"; }
};

// ------------------------------------------------------------------------------------------ json builders
json::Value num(double x) { json::Value v; v.kind = json::Value::Num; v.num = x; return v; }
json::Value str(const std::string& s) { json::Value v; v.kind = json::Value::Str; v.str = s; return v; }
json::Value arr() { json::Value v; v.kind = json::Value::Arr; return v; }
json::Value obj() { json::Value v; v.kind = json::Value::Obj; return v; }
json::Value nums(const double* x, int n) {
  json::Value v = arr();
  for (int i = 0; i < n; ++i) v.arr.push_back(num(x[i]));
  return v;
}

struct TreeLink {
  std::string name;
  int parent = -1, joint = -1;
  std::string type = "None";
  double axis[3] = {0, 0, 0}, origin[3] = {0, 0, 0};
  F f = IDENT;
  bool collision = false;
};

}  // namespace

void robot_from_model_value(const json::Value& m, RobotHost* out);

void robot_from_urdf(const std::string& urdf_text, const std::string& srdf_text, const std::string& spheres_json,
                     RobotHost* out) {
  const XNode urdf = XmlReader(urdf_text).root();
  const XNode srdf = XmlReader(srdf_text).root();
  if (urdf.tag != "robot" || srdf.tag != "robot") throw std::runtime_error("urdf / srdf: root element is not <robot>");
  const json::Value spec_doc = json::parse(spheres_json.c_str());
  const json::Value& spec = spec_doc["links"];

  // links in document order (kdl_parser / urdf::Model), joints (direct children of <robot> only)
  std::vector<std::string> link_order;
  std::map<std::string, const XNode*> links;
  std::vector<Joint> joints;
  for (const XNode& k : urdf.kids) {
    if (k.tag == "link") {
      const std::string* n = k.get("name");
      if (!n) throw std::runtime_error("urdf: link without a name");
      if (!links.count(*n)) link_order.push_back(*n);
      links[*n] = &k;
    } else if (k.tag == "joint") {
      joints.emplace_back(k);
    }
  }
  std::map<std::string, const Joint*> by_child;
  for (const Joint& j : joints) by_child[j.child] = &j;
  // urdf initTree iterates its joint map, sorted by name: children of a link in joint-name order
  std::vector<const Joint*> sorted_j;
  for (const Joint& j : joints) sorted_j.push_back(&j);
  std::stable_sort(sorted_j.begin(), sorted_j.end(), [](const Joint* a, const Joint* b) { return a->name < b->name; });
  std::map<std::string, std::vector<std::string>> children;
  for (const Joint* j : sorted_j) children[j->parent].push_back(j->child);
  std::vector<std::string> roots;
  for (const std::string& n : link_order)
    if (!by_child.count(n)) roots.push_back(n);
  if (roots.size() != 1) throw std::runtime_error("urdf: the tree needs exactly one root link");

  // ---- planning chain: the SRDF group's chain (robotino_plan.srdf:4-6), KDL segments with float-cast limits
  const XNode* grp = srdf.child("group");
  const XNode* chel = grp ? grp->child("chain") : nullptr;
  if (!chel || !chel->get("base_link") || !chel->get("tip_link")) throw std::runtime_error("srdf: no group chain");
  const std::string base = *chel->get("base_link"), tip = *chel->get("tip_link");
  std::vector<const Joint*> seq;
  for (std::string n = tip; n != base;) {
    auto it = by_child.find(n);
    if (it == by_child.end() || seq.size() > joints.size())
      throw std::runtime_error("urdf: chain tip does not lead to the base " + base);
    seq.push_back(it->second);
    n = it->second->parent;
  }
  std::reverse(seq.begin(), seq.end());
  json::Value chain = arr(), qmin = arr(), qmax = arr(), jrev = arr(), jnames = arr();
  std::vector<std::string> plan_links;  // child links of the chain's movable joints (collision_checker.hpp:216-255)
  for (const Joint* j : seq) {
    const F ft = j->f_tip();
    json::Value e = obj();
    e.obj["name"] = str(j->child);
    e.obj["joint_name"] = str(j->name);
    e.obj["type"] = str(j->kdl_name());
    e.obj["axis"] = nums(j->axis, 3);
    e.obj["origin"] = nums(j->Fo.p, 3);
    e.obj["ftip_R"] = nums(ft.R, 9);
    e.obj["ftip_p"] = nums(ft.p, 3);
    if (j->kdl) {
      e.obj["joint"] = num((double)jnames.arr.size());
      jnames.arr.push_back(str(j->name));
      jrev.arr.push_back(num(j->kdl == 1 ? 1 : 0));
      double lo, hi;
      if (j->type == "continuous") {  // kdl_kuka_model.cpp:176-184, stored through float
        lo = (double)(float)(-M_PI);
        hi = (double)(float)M_PI;
      } else {
        lo = (double)(float)j->lower;
        hi = (double)(float)j->upper;
      }
      qmin.arr.push_back(num(lo));
      qmax.arr.push_back(num(hi));
      plan_links.push_back(j->child);
    } else {
      e.obj["joint"] = num(-1);
    }
    chain.arr.push_back(e);
  }
  if ((int)jnames.arr.size() != NJ) throw std::runtime_error("urdf: the planning chain must have 8 joints");

  // ---- collision tree in KDL DFS order (collision_checker.hpp:195-261)
  std::vector<TreeLink> tree;
  std::map<std::string, int> index;
  TreeLink root;
  root.name = roots[0];
  tree.push_back(root);
  index[roots[0]] = 0;
  struct Frame_ { std::string name; int idx; size_t next; };
  std::vector<Frame_> stack = {{roots[0], 0, 0}};
  while (!stack.empty()) {  // recursion of expand() as an explicit stack: children in joint-name order, depth first
    Frame_& top = stack.back();
    const std::vector<std::string>& ch = children[top.name];
    if (top.next >= ch.size()) { stack.pop_back(); continue; }
    const std::string c = ch[top.next++];
    if (index.count(c)) throw std::runtime_error("urdf: link " + c + " reached twice (the joints do not form a tree)");
    const Joint* j = by_child[c];
    TreeLink t;
    t.name = c;
    t.parent = top.idx;
    auto pl = std::find(plan_links.begin(), plan_links.end(), c);
    if (pl != plan_links.end()) {
      t.joint = (int)(pl - plan_links.begin());
      t.type = j->kdl_name();
      for (int i = 0; i < 3; ++i) { t.axis[i] = j->axis[i]; t.origin[i] = j->Fo.p[i]; }
    } else {
      t.f = j->frame_to_tip();
    }
    tree.push_back(t);
    index[c] = (int)tree.size() - 1;
    stack.push_back({c, (int)tree.size() - 1, 0});
  }

  // ---- collision geometry (first <collision> of a link) + the transformToParent *= frameAdjust quirk
  // (collision_checker.hpp:329-336, 530: applied to fixed links, ignored for movable ones)
  struct Geom { std::string kind; std::vector<double> dims; };
  std::map<std::string, Geom> geom;
  for (const std::string& name : link_order) {
    const XNode* c = links[name]->child("collision");
    if (!c) continue;
    const XNode* g = c->child("geometry");
    if (!g || g->kids.empty()) throw std::runtime_error("urdf: collision without geometry in " + name);
    const XNode& sh = g->kids[0];
    const XNode* o = c->child("origin");
    const std::vector<double> xyz = vec3(o ? o->get("xyz") : nullptr), rpy = vec3(o ? o->get("rpy") : nullptr);
    Geom gm;
    gm.kind = sh.tag;
    if (sh.tag == "box") {
      gm.dims = vec3(sh.get("size"));
      if (!(gm.dims[0] > 0 && gm.dims[1] > 0 && gm.dims[2] > 0)) continue;  // a degenerate box is no geometry
    } else if (sh.tag == "cylinder") {
      if (!sh.get("radius") || !sh.get("length")) throw std::runtime_error("urdf: cylinder without radius / length");
      gm.dims = {std::strtod(sh.get("radius")->c_str(), nullptr), std::strtod(sh.get("length")->c_str(), nullptr)};
    } else if (sh.tag == "sphere") {
      gm.dims = {sh.get("radius") ? std::strtod(sh.get("radius")->c_str(), nullptr) : 0.0};
    } else {
      gm.kind = "mesh";
    }
    geom[name] = gm;
    F adj;
    double q[4];
    quat_from_rpy(rpy[0], rpy[1], rpy[2], q);
    rot_from_quat(q, adj.R);
    for (int i = 0; i < 3; ++i) adj.p[i] = xyz[i];
    auto it = index.find(name);
    if (it == index.end()) throw std::runtime_error("urdf: collision link outside the tree: " + name);
    TreeLink& e = tree[it->second];
    if (e.joint < 0) e.f = frame_mul(e.f, adj);
    e.collision = true;
  }

  // ---- spheres of the mesh links (tree order, spec order)
  struct Sph { int link; double c[3], r; int body = 0; double cb[3]; };
  std::vector<Sph> S;
  for (const auto& kv : spec.obj) {
    auto it = index.find(kv.first);
    if (it == index.end() || !tree[it->second].collision)
      throw std::runtime_error("sphere spec names a link without collision geometry: " + kv.first);
  }
  for (size_t i = 0; i < tree.size(); ++i) {
    if (!spec.has(tree[i].name)) continue;
    const json::Value& ss = spec[tree[i].name];
    for (size_t k = 0; k < ss.size(); ++k) {
      if (ss[k].size() != 4) throw std::runtime_error("sphere spec: entries are [x, y, z, r]");
      Sph s;
      s.link = (int)i;
      for (int d = 0; d < 3; ++d) s.c[d] = ss[k][d].d();
      s.r = ss[k][3].d();
      S.push_back(s);
    }
  }
  std::vector<int> coll_links, prim_links;
  for (size_t i = 0; i < tree.size(); ++i)
    if (tree[i].collision) coll_links.push_back((int)i);
  for (int i : coll_links) {
    const Geom& g = geom[tree[i].name];
    const bool prim = (g.kind == "box" || g.kind == "cylinder") && !spec.has(tree[i].name);
    if (prim) prim_links.push_back(i);
    else if (!spec.has(tree[i].name)) throw std::runtime_error("no collision geometry for " + tree[i].name + " (give spheres)");
  }

  // ---- self pairs: SRDF-enabled, non-rigid (collision_checker.hpp:353-393)
  std::set<std::pair<std::string, std::string>> dis;
  for (const XNode& k : srdf.kids)
    if (k.tag == "disable_collisions" && k.get("link1") && k.get("link2")) {
      dis.insert({*k.get("link1"), *k.get("link2")});
      dis.insert({*k.get("link2"), *k.get("link1")});
    }
  auto joint_set = [&](int i) {
    std::set<int> js;
    for (; i >= 0; i = tree[i].parent)
      if (tree[i].joint >= 0) js.insert(tree[i].joint);
    return js;
  };
  json::Value pairs = arr();
  int n_enabled = 0;
  for (size_t a = 0; a < coll_links.size(); ++a)
    for (size_t b = a + 1; b < coll_links.size(); ++b) {
      const int la = coll_links[a], lb = coll_links[b];
      if (dis.count({tree[la].name, tree[lb].name})) continue;
      ++n_enabled;
      if (joint_set(la) == joint_set(lb)) continue;  // rigid: no planning joint moves one against the other
      json::Value pr = arr();
      pr.arr.push_back(num(la));
      pr.arr.push_back(num(lb));
      pairs.arr.push_back(pr);
    }
  (void)n_enabled;

  // ---- rigid-body collapse (collision_checker.hpp:519-539 recursion, pre-composed into body frames)
  auto body_of = [&](int i) {
    const int i0 = i;
    while (i >= 0 && tree[i].joint < 0) i = tree[i].parent;
    // a collision link on the root, or fixed to it, has no planning joint above it: the model cannot place it
    if (i < 0) throw std::runtime_error("urdf: no planning joint above collision link " + tree[i0].name);
    return i;
  };
  auto offset = [&](int body, int i, bool* ident) {
    std::vector<int> path;
    for (; i != body; i = tree[i].parent) path.push_back(i);
    F f = IDENT;
    bool first = true;
    for (auto it = path.rbegin(); it != path.rend(); ++it) {
      f = first ? tree[*it].f : frame_mul(f, tree[*it].f);
      first = false;
    }
    *ident = first;
    return f;
  };
  auto to_body = [&](int b, int i, const double* c, double* o) {
    bool ident;
    const F f = offset(b, i, &ident);
    if (ident) { for (int d = 0; d < 3; ++d) o[d] = c[d]; return; }
    double m[3];
    rot_vec(f.R, c, m);
    for (int d = 0; d < 3; ++d) o[d] = m[d] + f.p[d];
  };
  std::set<int> bset;
  for (const Sph& s : S) bset.insert(body_of(s.link));
  for (int i : prim_links) bset.insert(body_of(i));
  const std::vector<int> bodies(bset.begin(), bset.end());
  if (bodies.empty()) throw std::runtime_error("urdf: no collision link below a planning joint");
  auto bidx = [&](int b) { return (int)(std::find(bodies.begin(), bodies.end(), b) - bodies.begin()); };
  json::Value body_chain = arr();
  for (int k = 1; k <= bodies.back(); ++k) {
    const TreeLink& e = tree[k];
    if (e.parent != k - 1) throw std::runtime_error("urdf: the moving bodies must lie on one path from the root");
    json::Value v = obj();
    v.obj["link"] = num(k);
    v.obj["type"] = str(e.type);
    v.obj["joint"] = num(e.joint);
    v.obj["axis"] = nums(e.axis, 3);
    v.obj["origin"] = nums(e.origin, 3);
    v.obj["R"] = nums(e.f.R, 9);
    v.obj["p"] = nums(e.f.p, 3);
    v.obj["body"] = num(bset.count(k) ? bidx(k) : -1);
    body_chain.arr.push_back(v);
  }
  auto planar = [&](int b) {
    for (int k = 1; k <= b; ++k) {
      const TreeLink& e = tree[k];
      if (e.joint >= 0) {
        if (e.type == "TransAxis" && e.axis[2] != 0.0) return false;
        if (e.type == "RotAxis" && !(e.axis[0] == 0.0 && e.axis[1] == 0.0 && std::fabs(e.axis[2]) == 1.0)) return false;
      } else {
        const double* R = e.f.R;
        if (!(R[2] == 0.0 && R[5] == 0.0 && R[6] == 0.0 && R[7] == 0.0 && R[8] == 1.0)) return false;
      }
    }
    return true;
  };
  json::Value spheres = arr();
  for (Sph& s : S) {
    const int b = body_of(s.link);
    s.body = bidx(b);
    to_body(b, s.link, s.c, s.cb);
    json::Value v = obj();
    v.obj["link"] = num(s.link);
    v.obj["c"] = nums(s.c, 3);
    v.obj["r"] = num(s.r);
    v.obj["body"] = num(s.body);
    v.obj["cb"] = nums(s.cb, 3);
    spheres.arr.push_back(v);
  }
  json::Value prims = arr();
  std::map<int, std::pair<std::vector<double>, double>> prim_bound;  // link -> (cb, r)
  for (int i : prim_links) {
    const int b = body_of(i);
    const Geom& g = geom[tree[i].name];
    bool ident;
    const F f = offset(b, i, &ident);
    if (!planar(b)) throw std::runtime_error("primitive on a non-planar body (give it spheres): " + tree[i].name);
    const double* R = f.R;
    if (std::fabs(R[2]) > 1e-9 || std::fabs(R[5]) > 1e-9 || std::fabs(R[8] - 1.0) > 1e-9 || std::fabs(R[6]) > 1e-9)
      throw std::runtime_error("primitive not upright in its planar body: " + tree[i].name);
    double half[3], rxy, rall;
    if (g.kind == "box") {
      for (int d = 0; d < 3; ++d) half[d] = 0.5 * g.dims[d];
      rxy = std::sqrt(half[0] * half[0] + half[1] * half[1]);
      rall = std::sqrt(half[0] * half[0] + half[1] * half[1] + half[2] * half[2]);
    } else {
      half[0] = g.dims[0]; half[1] = 0.5 * g.dims[1]; half[2] = 0.0;
      rxy = g.dims[0];
      rall = std::sqrt(half[0] * half[0] + half[1] * half[1]);
    }
    const double cb[3] = {ident ? 0.0 : f.p[0], ident ? 0.0 : f.p[1], ident ? 0.0 : f.p[2]};
    const double ab[3] = {ident ? 1.0 : R[0], ident ? 0.0 : R[3], 0.0};
    json::Value v = obj();
    v.obj["link"] = num(i);
    v.obj["body"] = num(bidx(b));
    v.obj["type"] = str(g.kind);
    v.obj["half"] = nums(half, 3);
    v.obj["cb"] = nums(cb, 3);
    v.obj["ab"] = nums(ab, 3);
    v.obj["rxy"] = num(rxy + 1e-6);
    v.obj["r"] = num(rall + 1e-6);
    prims.arr.push_back(v);
    prim_bound[i] = {std::vector<double>(cb, cb + 3), rall + 1e-6};
  }
  // per-link bounding spheres (sums in list order, margin 1e-6)
  json::Value lbs = arr();
  for (int i : coll_links) {
    const int b = body_of(i);
    double c[3] = {0, 0, 0}, cb[3], r = 0.0;
    if (prim_bound.count(i)) {
      for (int d = 0; d < 3; ++d) cb[d] = prim_bound[i].first[d];
      r = prim_bound[i].second;
    } else {
      int n = 0;
      for (const Sph& s : S)
        if (s.link == i) { for (int d = 0; d < 3; ++d) c[d] = c[d] + s.c[d]; ++n; }
      for (int d = 0; d < 3; ++d) c[d] = c[d] / n;
      for (const Sph& s : S)
        if (s.link == i) {
          const double dx = s.c[0] - c[0], dy = s.c[1] - c[1], dz = s.c[2] - c[2];
          r = std::max(r, std::sqrt(dx * dx + dy * dy + dz * dz) + s.r);
        }
      r = r + 1e-6;
      to_body(b, i, c, cb);
    }
    json::Value v = obj();
    v.obj["link"] = num(i);
    v.obj["c"] = nums(c, 3);
    v.obj["r"] = num(r);
    v.obj["body"] = num(bidx(b));
    v.obj["cb"] = nums(cb, 3);
    lbs.arr.push_back(v);
  }
  json::Value tree_v = arr();
  for (const TreeLink& t : tree) {
    json::Value v = obj();
    v.obj["name"] = str(t.name);
    tree_v.arr.push_back(v);
  }
  json::Value bodies_v = arr();
  for (int b : bodies) bodies_v.arr.push_back(num(b));

  json::Value m = obj();
  m.obj["root_z"] = num(0.02);  // collision_checker.hpp:201 (the octree's -0.02 is the scene's z_offset, CC:87)
  m.obj["links"] = tree_v;
  m.obj["body_chain"] = body_chain;
  m.obj["bodies"] = bodies_v;
  m.obj["chain"] = chain;
  m.obj["link_bounds"] = lbs;
  m.obj["spheres"] = spheres;
  m.obj["prims"] = prims;
  m.obj["self_pairs"] = pairs;
  m.obj["q_min"] = qmin;
  m.obj["q_max"] = qmax;
  m.obj["joint_is_revolute"] = jrev;
  robot_from_model_value(m, out);
}

}  // namespace smp
