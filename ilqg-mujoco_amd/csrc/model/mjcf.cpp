// MJCF subset compiler: XML -> HostModel (MuJoCo 2.0 compiler semantics for
// the features in SURVEY.md Appendix B.1).  Host-only model compilation; not
// on the hot path.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>

#include "ilqg_model_blob.h"
#include "model.h"

namespace ilqg {
namespace {

constexpr double kPi = 3.14159265358979323846;
constexpr double kMinVal = 1e-15;

// ---------------------------------------------------------------- XML ----
struct Elem {
  std::string name;
  std::vector<std::pair<std::string, std::string>> attrs;
  std::vector<std::unique_ptr<Elem>> kids;
  const std::string* attr(const std::string& k) const {
    for (auto& a : attrs)
      if (a.first == k) return &a.second;
    return nullptr;
  }
};

struct XmlParser {
  const std::string& s;
  size_t i = 0;
  std::string err;
  explicit XmlParser(const std::string& src) : s(src) {}

  void skip_ws() {
    while (i < s.size() && isspace((unsigned char)s[i])) i++;
  }
  bool starts(const char* t) const { return s.compare(i, strlen(t), t) == 0; }
  // skip comments, processing instructions and text
  void skip_misc() {
    for (;;) {
      while (i < s.size() && s[i] != '<') i++;
      if (starts("<!--")) {
        size_t e = s.find("-->", i + 4);
        i = (e == std::string::npos) ? s.size() : e + 3;
      } else if (starts("<?") || starts("<!")) {
        size_t e = s.find('>', i);
        i = (e == std::string::npos) ? s.size() : e + 1;
      } else {
        return;
      }
    }
  }
  std::unique_ptr<Elem> parse_elem() {
    skip_misc();
    if (i >= s.size() || s[i] != '<') { err = "expected element"; return nullptr; }
    i++;
    auto e = std::make_unique<Elem>();
    while (i < s.size() && !isspace((unsigned char)s[i]) && s[i] != '>' && s[i] != '/') e->name += s[i++];
    for (;;) {
      skip_ws();
      if (i >= s.size()) { err = "unterminated tag " + e->name; return nullptr; }
      if (s[i] == '/') {
        if (i + 1 < s.size() && s[i + 1] == '>') { i += 2; return e; }
        err = "bad '/' in tag " + e->name;
        return nullptr;
      }
      if (s[i] == '>') { i++; break; }
      std::string k, v;
      while (i < s.size() && s[i] != '=' && !isspace((unsigned char)s[i])) k += s[i++];
      skip_ws();
      if (i >= s.size() || s[i] != '=') { err = "attribute without value in " + e->name; return nullptr; }
      i++;
      skip_ws();
      char q = s[i];
      if (q != '"' && q != '\'') { err = "unquoted attribute in " + e->name; return nullptr; }
      i++;
      size_t end = s.find(q, i);
      if (end == std::string::npos) { err = "unterminated attribute"; return nullptr; }
      v = s.substr(i, end - i);
      i = end + 1;
      e->attrs.emplace_back(k, v);
    }
    // children until closing tag
    for (;;) {
      skip_misc();
      if (i >= s.size()) { err = "missing </" + e->name + ">"; return nullptr; }
      if (starts("</")) {
        size_t end = s.find('>', i);
        std::string nm = s.substr(i + 2, end - i - 2);
        while (!nm.empty() && isspace((unsigned char)nm.back())) nm.pop_back();
        if (nm != e->name) { err = "mismatched </" + nm + "> for <" + e->name + ">"; return nullptr; }
        i = end + 1;
        return e;
      }
      auto c = parse_elem();
      if (!c) return nullptr;
      e->kids.push_back(std::move(c));
    }
  }
};

// Lenient number list: whitespace-separated tokens, each read with strtod.
// A token such as "0.13/2" (hopper.xml:23) yields its numeric prefix (0.13);
// the malformed value only sets a body frame origin, which is dynamics-neutral
// under coordinate="global".
std::vector<double> numbers(const std::string& v) {
  std::vector<double> out;
  std::istringstream ss(v);
  std::string tok;
  while (ss >> tok) {
    char* end = nullptr;
    double x = strtod(tok.c_str(), &end);
    if (end != tok.c_str()) out.push_back(x);
  }
  return out;
}

// ------------------------------------------------------------ math -------
void quat_mul(double* r, const double* a, const double* b) {
  double t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                 a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                 a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                 a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  for (int k = 0; k < 4; k++) r[k] = t[k];
}
void quat2mat(double* r, const double* q) {
  double q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  double q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  double q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  r[0] = q00 + q11 - q22 - q33; r[4] = q00 - q11 + q22 - q33; r[8] = q00 - q11 - q22 + q33;
  r[1] = 2 * (q12 - q03); r[2] = 2 * (q13 + q02); r[3] = 2 * (q12 + q03);
  r[5] = 2 * (q23 - q01); r[6] = 2 * (q13 - q02); r[7] = 2 * (q23 + q01);
}
void rot(double* r, const double* v, const double* q) {
  double m[9];
  quat2mat(m, q);
  double t[3] = {m[0] * v[0] + m[1] * v[1] + m[2] * v[2], m[3] * v[0] + m[4] * v[1] + m[5] * v[2],
                 m[6] * v[0] + m[7] * v[1] + m[8] * v[2]};
  r[0] = t[0]; r[1] = t[1]; r[2] = t[2];
}
void conj(double* r, const double* q) { r[0] = q[0]; r[1] = -q[1]; r[2] = -q[2]; r[3] = -q[3]; }
void normalize4(double* q) {
  double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < kMinVal) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  for (int k = 0; k < 4; k++) q[k] /= n;
}
double normalize3(double* v) {
  double n = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (n < kMinVal) { v[0] = 1; v[1] = v[2] = 0; return n; }
  for (int k = 0; k < 3; k++) v[k] /= n;
  return n;
}
// rotation taking +z to vec (MuJoCo mju_quatZ2Vec)
void quat_z2vec(double* q, const double* vec) {
  double vn[3] = {vec[0], vec[1], vec[2]}, z[3] = {0, 0, 1}, axis[3];
  q[0] = 1; q[1] = q[2] = q[3] = 0;
  if (normalize3(vn) < kMinVal) return;
  axis[0] = z[1] * vn[2] - z[2] * vn[1];
  axis[1] = z[2] * vn[0] - z[0] * vn[2];
  axis[2] = z[0] * vn[1] - z[1] * vn[0];
  double a = normalize3(axis);
  if (std::fabs(a) < kMinVal) {
    if (vn[2] < 0) { q[0] = 0; q[1] = 1; }
    return;
  }
  double ang = std::atan2(a, vn[2]);
  double s = std::sin(ang / 2);
  q[0] = std::cos(ang / 2); q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}
// symmetric 3x3 eigen-decomposition (cyclic Jacobi); columns of V are eigenvectors
void eig3(const double* A, double* evals, double* V) {
  double a[9];
  for (int k = 0; k < 9; k++) a[k] = A[k];
  for (int k = 0; k < 9; k++) V[k] = (k % 4 == 0) ? 1 : 0;
  for (int sweep = 0; sweep < 64; sweep++) {
    double off = a[1] * a[1] + a[2] * a[2] + a[5] * a[5];
    if (off < 1e-40) break;
    for (int p = 0; p < 2; p++)
      for (int q = p + 1; q < 3; q++) {
        double apq = a[3 * p + q];
        if (std::fabs(apq) < 1e-300) continue;
        double app = a[3 * p + p], aqq = a[3 * q + q];
        double theta = (aqq - app) / (2 * apq);
        double t = (theta >= 0 ? 1 : -1) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
        double c = 1 / std::sqrt(t * t + 1), s = t * c;
        for (int k = 0; k < 3; k++) {  // A <- J' A J
          double akp = a[3 * k + p], akq = a[3 * k + q];
          a[3 * k + p] = c * akp - s * akq;
          a[3 * k + q] = s * akp + c * akq;
        }
        for (int k = 0; k < 3; k++) {
          double apk = a[3 * p + k], aqk = a[3 * q + k];
          a[3 * p + k] = c * apk - s * aqk;
          a[3 * q + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < 3; k++) {
          double vkp = V[3 * k + p], vkq = V[3 * k + q];
          V[3 * k + p] = c * vkp - s * vkq;
          V[3 * k + q] = s * vkp + c * vkq;
        }
      }
  }
  for (int k = 0; k < 3; k++) evals[k] = a[4 * k];
  // right-handed
  double det = V[0] * (V[4] * V[8] - V[5] * V[7]) - V[1] * (V[3] * V[8] - V[5] * V[6]) +
               V[2] * (V[3] * V[7] - V[4] * V[6]);
  if (det < 0)
    for (int k = 0; k < 3; k++) V[3 * k + 2] = -V[3 * k + 2];
}
void mat2quat(double* q, const double* m) {
  double tr = m[0] + m[4] + m[8];
  if (tr > 0) {
    double s = std::sqrt(tr + 1.0) * 2;
    q[0] = 0.25 * s; q[1] = (m[7] - m[5]) / s; q[2] = (m[2] - m[6]) / s; q[3] = (m[3] - m[1]) / s;
  } else if (m[0] > m[4] && m[0] > m[8]) {
    double s = std::sqrt(1.0 + m[0] - m[4] - m[8]) * 2;
    q[0] = (m[7] - m[5]) / s; q[1] = 0.25 * s; q[2] = (m[1] + m[3]) / s; q[3] = (m[2] + m[6]) / s;
  } else if (m[4] > m[8]) {
    double s = std::sqrt(1.0 + m[4] - m[0] - m[8]) * 2;
    q[0] = (m[2] - m[6]) / s; q[1] = (m[1] + m[3]) / s; q[2] = 0.25 * s; q[3] = (m[5] + m[7]) / s;
  } else {
    double s = std::sqrt(1.0 + m[8] - m[0] - m[4]) * 2;
    q[0] = (m[3] - m[1]) / s; q[1] = (m[2] + m[6]) / s; q[2] = (m[5] + m[7]) / s; q[3] = 0.25 * s;
  }
  normalize4(q);
}

// --------------------------------------------------------- compiler ------
enum { JNT_FREE = 0, JNT_BALL, JNT_SLIDE, JNT_HINGE };
enum { GEOM_PLANE = 0, GEOM_HFIELD, GEOM_SPHERE, GEOM_CAPSULE };

struct AttrSource {
  const Elem* e;
  const std::map<std::string, std::string>* def;
  const std::string* get(const std::string& k) const {
    if (const std::string* v = e->attr(k)) return v;
    if (def) {
      auto it = def->find(k);
      if (it != def->end()) return &it->second;
    }
    return nullptr;
  }
  std::vector<double> vec(const std::string& k, std::vector<double> dflt) const {
    const std::string* v = get(k);
    if (!v) return dflt;
    std::vector<double> x = numbers(*v);
    // partially specified vectors keep the trailing defaults (solimp has 5)
    for (size_t i = x.size(); i < dflt.size(); i++) x.push_back(dflt[i]);
    return x;
  }
  double num(const std::string& k, double dflt) const {
    const std::string* v = get(k);
    if (!v) return dflt;
    std::vector<double> x = numbers(*v);
    return x.empty() ? dflt : x[0];
  }
  int boolean(const std::string& k, int dflt) const {
    const std::string* v = get(k);
    if (!v) return dflt;
    return *v == "true" ? 1 : 0;
  }
  std::string str(const std::string& k, const std::string& dflt) const {
    const std::string* v = get(k);
    return v ? *v : dflt;
  }
};

struct BodyTmp {
  int parent;
  double gpos[3], gquat[4];  // global frame at qpos0
  double lpos[3], lquat[4];  // frame relative to parent
};

struct Compiler {
  HostModel& m;
  std::string& err;
  bool degree = true, global = false;
  std::map<std::string, std::string> djoint, dgeom, dmotor;
  std::vector<BodyTmp> bodies;
  std::map<std::string, int> jnt_by_name;
  // per-geom (body frame) for inertia
  std::vector<double> gmass, ginert;  // ngeom, 3*ngeom (principal, geom frame)

  Compiler(HostModel& mm, std::string& e) : m(mm), err(e) {}

  double ang(double x) const { return degree ? x * kPi / 180.0 : x; }

  // global <-> body-local helpers
  void to_local_pos(int b, const double* g, double* l) const {
    double d[3] = {g[0] - bodies[b].gpos[0], g[1] - bodies[b].gpos[1], g[2] - bodies[b].gpos[2]}, qc[4];
    conj(qc, bodies[b].gquat);
    rot(l, d, qc);
  }
  void to_local_vec(int b, const double* g, double* l) const {
    double qc[4];
    conj(qc, bodies[b].gquat);
    rot(l, g, qc);
  }
  void to_local_quat(int b, const double* g, double* l) const {
    double qc[4];
    conj(qc, bodies[b].gquat);
    quat_mul(l, qc, g);
    normalize4(l);
  }

  bool add_body(const Elem* e, int parent) {
    int id = (int)bodies.size();
    AttrSource a{e, nullptr};
    BodyTmp bt{};
    bt.parent = parent;
    std::vector<double> pos = a.vec("pos", {0, 0, 0});
    std::vector<double> quat = a.vec("quat", {1, 0, 0, 0});
    normalize4(quat.data());
    if (global) {
      for (int k = 0; k < 3; k++) bt.gpos[k] = pos[k];
      for (int k = 0; k < 4; k++) bt.gquat[k] = quat[k];
      const BodyTmp& p = bodies[parent];
      double d[3] = {pos[0] - p.gpos[0], pos[1] - p.gpos[1], pos[2] - p.gpos[2]}, qc[4];
      conj(qc, p.gquat);
      rot(bt.lpos, d, qc);
      quat_mul(bt.lquat, qc, quat.data());
      normalize4(bt.lquat);
    } else {
      for (int k = 0; k < 3; k++) bt.lpos[k] = pos[k];
      for (int k = 0; k < 4; k++) bt.lquat[k] = quat[k];
      const BodyTmp& p = bodies[parent];
      double t[3];
      rot(t, pos.data(), p.gquat);
      for (int k = 0; k < 3; k++) bt.gpos[k] = p.gpos[k] + t[k];
      quat_mul(bt.gquat, p.gquat, quat.data());
      normalize4(bt.gquat);
    }
    bodies.push_back(bt);
    m.body_names.push_back(a.str("name", ""));
    m.body_parentid.push_back(parent);
    m.body_rootid.push_back(parent == 0 ? id : m.body_rootid[parent]);
    m.body_jntadr.push_back(-1);
    m.body_jntnum.push_back(0);
    m.body_dofadr.push_back(-1);
    m.body_dofnum.push_back(0);
    m.body_geomadr.push_back(-1);
    m.body_geomnum.push_back(0);
    for (int k = 0; k < 3; k++) m.body_pos.push_back(bt.lpos[k]);
    for (int k = 0; k < 4; k++) m.body_quat.push_back(bt.lquat[k]);
    // joints first (XML order), then geoms, then child bodies (DFS preorder)
    for (auto& c : e->kids)
      if (c->name == "joint" || c->name == "freejoint")
        if (!add_joint(c.get(), id, c->name == "freejoint")) return false;
    for (auto& c : e->kids)
      if (c->name == "geom")
        if (!add_geom(c.get(), id)) return false;
    for (auto& c : e->kids)
      if (c->name == "body")
        if (!add_body(c.get(), id)) return false;
    for (auto& c : e->kids)
      if (c->name == "inertial") { err = "<inertial> not supported (inertiafromgeom only)"; return false; }
    return true;
  }

  bool add_joint(const Elem* e, int b, bool isfree) {
    AttrSource a{e, isfree ? nullptr : &djoint};
    int id = (int)m.jnt_type.size();
    int type;
    std::string t = isfree ? "free" : a.str("type", "hinge");
    if (t == "free") type = JNT_FREE;
    else if (t == "ball") type = JNT_BALL;
    else if (t == "slide") type = JNT_SLIDE;
    else if (t == "hinge") type = JNT_HINGE;
    else { err = "unknown joint type " + t; return false; }
    if (m.body_jntnum[b] == 0) m.body_jntadr[b] = id;
    m.body_jntnum[b]++;
    m.jnt_names.push_back(a.str("name", ""));
    jnt_by_name[a.str("name", "")] = id;
    m.jnt_type.push_back(type);
    m.jnt_bodyid.push_back(b);
    m.jnt_qposadr.push_back((int)m.qpos0.size());
    m.jnt_dofadr.push_back((int)m.dof_bodyid.size());
    std::vector<double> pos = a.vec("pos", {0, 0, 0}), axis = a.vec("axis", {0, 0, 1});
    double lp[3], la[3];
    if (global && !isfree) {
      to_local_pos(b, pos.data(), lp);
      to_local_vec(b, axis.data(), la);
    } else {
      for (int k = 0; k < 3; k++) { lp[k] = pos[k]; la[k] = axis[k]; }
    }
    normalize3(la);
    for (int k = 0; k < 3; k++) { m.jnt_pos.push_back(isfree ? 0 : lp[k]); m.jnt_axis.push_back(isfree ? (k == 2) : la[k]); }
    int limited = isfree ? 0 : a.boolean("limited", 0);
    std::vector<double> range = a.vec("range", {0, 0});
    if (type == JNT_HINGE || type == JNT_BALL) { range[0] = ang(range[0]); range[1] = ang(range[1]); }
    m.jnt_limited.push_back(limited);
    m.jnt_range.push_back(range[0]);
    m.jnt_range.push_back(range[1]);
    std::vector<double> sr = a.vec("solreflimit", {0.02, 1}), si = a.vec("solimplimit", {0.9, 0.95, 0.001, 0.5, 2});
    m.jnt_solref.push_back(sr[0]); m.jnt_solref.push_back(sr[1]);
    for (int k = 0; k < 5; k++) m.jnt_solimp.push_back(si[k]);
    m.jnt_stiffness.push_back(isfree ? 0 : a.num("stiffness", 0));
    m.jnt_margin.push_back(isfree ? 0 : a.num("margin", 0));
    double armature = isfree ? 0 : a.num("armature", 0), damping = isfree ? 0 : a.num("damping", 0);
    int ndof = type == JNT_FREE ? 6 : (type == JNT_BALL ? 3 : 1);
    if (m.body_dofnum[b] == 0) m.body_dofadr[b] = (int)m.dof_bodyid.size();
    m.body_dofnum[b] += ndof;
    for (int k = 0; k < ndof; k++) {
      m.dof_bodyid.push_back(b);
      m.dof_jntid.push_back(id);
      m.dof_armature.push_back(armature);
      m.dof_damping.push_back(damping);
    }
    // qpos0 / springref
    if (type == JNT_FREE) {
      for (int k = 0; k < 3; k++) m.qpos0.push_back(bodies[b].gpos[k]);
      for (int k = 0; k < 4; k++) m.qpos0.push_back(bodies[b].gquat[k]);
      for (int k = 0; k < 7; k++) m.qpos_spring.push_back(m.qpos0[m.qpos0.size() - 7 + k]);
    } else if (type == JNT_BALL) {
      double q[4] = {1, 0, 0, 0};
      for (int k = 0; k < 4; k++) { m.qpos0.push_back(q[k]); m.qpos_spring.push_back(q[k]); }
    } else {
      double ref = a.num("ref", 0), sref = a.num("springref", 0);
      if (type == JNT_HINGE) { ref = ang(ref); sref = ang(sref); }
      m.qpos0.push_back(ref);
      m.qpos_spring.push_back(sref);
    }
    return true;
  }

  bool add_geom(const Elem* e, int b) {
    AttrSource a{e, &dgeom};
    int id = (int)m.geom_type.size();
    std::string t = a.str("type", "sphere");
    int type;
    if (t == "plane") type = GEOM_PLANE;
    else if (t == "sphere") type = GEOM_SPHERE;
    else if (t == "capsule") type = GEOM_CAPSULE;
    else { err = "geom type '" + t + "' not supported"; return false; }
    if (m.body_geomnum[b] == 0) m.body_geomadr[b] = id;
    m.body_geomnum[b]++;
    m.geom_names.push_back(a.str("name", ""));
    m.geom_type.push_back(type);
    m.geom_bodyid.push_back(b);
    m.geom_contype.push_back((int)a.num("contype", 1));
    m.geom_conaffinity.push_back((int)a.num("conaffinity", 1));
    m.geom_condim.push_back((int)a.num("condim", 3));
    int cd = m.geom_condim.back();
    if (cd != 1 && cd != 3) { err = "condim must be 1 or 3"; return false; }
    std::vector<double> fr = a.vec("friction", {1, 0.005, 0.0001});
    for (int k = 0; k < 3; k++) m.geom_friction.push_back(fr[k]);
    m.geom_margin.push_back(a.num("margin", 0));
    m.geom_gap.push_back(a.num("gap", 0));
    std::vector<double> sr = a.vec("solref", {0.02, 1}), si = a.vec("solimp", {0.9, 0.95, 0.001, 0.5, 2});
    m.geom_solref.push_back(sr[0]); m.geom_solref.push_back(sr[1]);
    for (int k = 0; k < 5; k++) m.geom_solimp.push_back(si[k]);
    m.geom_solmix.push_back(a.num("solmix", 1));
    std::vector<double> size = a.vec("size", {0, 0, 0});
    double pos[3], quat[4];
    if (const std::string* ft = a.get("fromto")) {
      std::vector<double> f = numbers(*ft);
      if (f.size() < 6) { err = "bad fromto"; return false; }
      double vec[3] = {f[3] - f[0], f[4] - f[1], f[5] - f[2]};
      for (int k = 0; k < 3; k++) pos[k] = 0.5 * (f[k] + f[3 + k]);
      quat_z2vec(quat, vec);
      size[1] = 0.5 * std::sqrt(vec[0] * vec[0] + vec[1] * vec[1] + vec[2] * vec[2]);
    } else {
      std::vector<double> p = a.vec("pos", {0, 0, 0}), q = a.vec("quat", {1, 0, 0, 0});
      for (int k = 0; k < 3; k++) pos[k] = p[k];
      for (int k = 0; k < 4; k++) quat[k] = q[k];
      normalize4(quat);
    }
    double lp[3], lq[4];
    if (global) {
      to_local_pos(b, pos, lp);
      to_local_quat(b, quat, lq);
    } else {
      for (int k = 0; k < 3; k++) lp[k] = pos[k];
      for (int k = 0; k < 4; k++) lq[k] = quat[k];
    }
    for (int k = 0; k < 3; k++) { m.geom_pos.push_back(lp[k]); m.geom_size.push_back(size[k]); }
    for (int k = 0; k < 4; k++) m.geom_quat.push_back(lq[k]);
    // mass / inertia (solid of uniform density, exact hemispherical caps)
    double density = a.num("density", 1000), mass = 0, I[3] = {0, 0, 0};
    double r = size[0];
    if (type == GEOM_SPHERE) {
      mass = density * 4.0 / 3.0 * kPi * r * r * r;
      I[0] = I[1] = I[2] = 0.4 * mass * r * r;
      m.geom_rbound.push_back(r);
    } else if (type == GEOM_CAPSULE) {
      double h = 2 * size[1];
      double mc = density * kPi * r * r * h, ms = density * 4.0 / 3.0 * kPi * r * r * r;
      mass = mc + ms;
      I[2] = mc * r * r / 2 + ms * 0.4 * r * r;
      I[0] = I[1] = mc * (r * r / 4 + h * h / 12) + ms * (0.4 * r * r + h * h / 4 + 3 * h * r / 8);
      m.geom_rbound.push_back(r + size[1]);
    } else {
      m.geom_rbound.push_back(0);
    }
    if (const std::string* mv = a.get("mass")) {
      double target = numbers(*mv).empty() ? mass : numbers(*mv)[0];
      double sc = mass > 0 ? target / mass : 0;
      for (int k = 0; k < 3; k++) I[k] *= sc;
      mass = target;
    }
    if (b == 0) { mass = 0; I[0] = I[1] = I[2] = 0; }
    gmass.push_back(mass);
    for (int k = 0; k < 3; k++) ginert.push_back(I[k]);
    return true;
  }

  bool add_actuators(const Elem* e) {
    for (auto& c : e->kids) {
      if (c->name != "motor") { err = "actuator <" + c->name + "> not supported (motor only)"; return false; }
      AttrSource a{c.get(), &dmotor};
      std::string jn = a.str("joint", "");
      auto it = jnt_by_name.find(jn);
      if (it == jnt_by_name.end()) { err = "motor joint '" + jn + "' not found"; return false; }
      int jt = m.jnt_type[it->second];
      if (jt != JNT_SLIDE && jt != JNT_HINGE) { err = "motor on multi-dof joint not supported"; return false; }
      m.actuator_names.push_back(a.str("name", ""));
      m.actuator_trnid.push_back(it->second);
      m.actuator_gear.push_back(a.vec("gear", {1})[0]);
      std::vector<double> cr = a.vec("ctrlrange", {0, 0}), fr = a.vec("forcerange", {0, 0});
      m.actuator_ctrlrange.push_back(cr[0]); m.actuator_ctrlrange.push_back(cr[1]);
      m.actuator_forcerange.push_back(fr[0]); m.actuator_forcerange.push_back(fr[1]);
      m.actuator_ctrllimited.push_back(a.boolean("ctrllimited", 0));
      m.actuator_forcelimited.push_back(a.boolean("forcelimited", 0));
      m.actuator_gainprm.push_back(1.0);
    }
    return true;
  }

  static void collect_defaults(const Elem* d, std::map<std::string, std::string>& dj,
                               std::map<std::string, std::string>& dg, std::map<std::string, std::string>& dm) {
    for (auto& c : d->kids) {
      std::map<std::string, std::string>* t = nullptr;
      if (c->name == "joint") t = &dj;
      else if (c->name == "geom") t = &dg;
      else if (c->name == "motor") t = &dm;
      if (t)
        for (auto& kv : c->attrs) (*t)[kv.first] = kv.second;
    }
  }

  bool run(const Elem* root) {
    if (root->name != "mujoco") { err = "root element must be <mujoco>"; return false; }
    if (const std::string* nm = root->attr("model")) m.model_name = *nm;
    // defaults (MuJoCo 2.0)
    m.opt_timestep = 0.002;
    m.opt_gravity0 = 0; m.opt_gravity1 = 0; m.opt_gravity2 = -9.81;
    m.opt_integrator = 0;
    m.opt_iterations = 100;
    m.opt_tolerance = 1e-8;
    m.opt_impratio = 1;
    m.opt_cone = 0;
    m.opt_solver = 2;
    m.nconmax = 100;
    m.njmax = 500;
    m.nstack = -1;
    const Elem* world = nullptr;
    const Elem* actuator = nullptr;
    for (auto& c : root->kids) {
      if (c->name == "compiler") {
        AttrSource a{c.get(), nullptr};
        degree = a.str("angle", "degree") == "degree";
        global = a.str("coordinate", "local") == "global";
        std::string ifg = a.str("inertiafromgeom", "auto");
        if (ifg == "false") { err = "inertiafromgeom=false not supported"; return false; }
      } else if (c->name == "default") {
        for (auto& k : c->kids)
          if (k->name == "default") { err = "nested default classes not supported"; return false; }
        collect_defaults(c.get(), djoint, dgeom, dmotor);
      } else if (c->name == "option") {
        AttrSource a{c.get(), nullptr};
        m.opt_timestep = a.num("timestep", m.opt_timestep);
        std::vector<double> g = a.vec("gravity", {0, 0, -9.81});
        m.opt_gravity0 = g[0]; m.opt_gravity1 = g[1]; m.opt_gravity2 = g[2];
        std::string integ = a.str("integrator", "Euler");
        if (integ == "Euler") m.opt_integrator = 0;
        else if (integ == "RK4") m.opt_integrator = 1;
        else { err = "integrator " + integ + " not supported"; return false; }
        m.opt_iterations = (int)a.num("iterations", m.opt_iterations);
        m.opt_tolerance = a.num("tolerance", m.opt_tolerance);
        m.opt_impratio = a.num("impratio", 1);
        if (a.str("cone", "pyramidal") != "pyramidal") { err = "only pyramidal cones supported"; return false; }
        if (a.str("solver", "Newton") != "Newton") { err = "only the Newton solver is supported"; return false; }
      } else if (c->name == "size") {
        AttrSource a{c.get(), nullptr};
        m.nconmax = (int)a.num("nconmax", m.nconmax);
        m.njmax = (int)a.num("njmax", m.njmax);
        m.nstack = (int)a.num("nstack", m.nstack);
      } else if (c->name == "worldbody") {
        world = c.get();
      } else if (c->name == "actuator") {
        actuator = c.get();
      }
    }
    if (!world) { err = "missing <worldbody>"; return false; }
    // world body
    BodyTmp w{};
    w.parent = 0;
    w.gquat[0] = w.lquat[0] = 1;
    bodies.push_back(w);
    m.body_names.push_back("world");
    m.body_parentid.push_back(0);
    m.body_rootid.push_back(0);
    m.body_jntadr.push_back(-1); m.body_jntnum.push_back(0);
    m.body_dofadr.push_back(-1); m.body_dofnum.push_back(0);
    m.body_geomadr.push_back(-1); m.body_geomnum.push_back(0);
    for (int k = 0; k < 3; k++) m.body_pos.push_back(0);
    m.body_quat.insert(m.body_quat.end(), {1, 0, 0, 0});
    for (auto& c : world->kids)
      if (c->name == "geom")
        if (!add_geom(c.get(), 0)) return false;
    for (auto& c : world->kids)
      if (c->name == "body")
        if (!add_body(c.get(), 0)) return false;
    if (actuator && !add_actuators(actuator)) return false;
    finish();
    return true;
  }

  void finish() {
    m.nbody = (int)bodies.size();
    m.njnt = (int)m.jnt_type.size();
    m.ngeom = (int)m.geom_type.size();
    m.nq = (int)m.qpos0.size();
    m.nv = (int)m.dof_bodyid.size();
    m.nu = (int)m.actuator_trnid.size();
    // weld ids
    m.body_weldid.assign(m.nbody, 0);
    for (int b = 1; b < m.nbody; b++) m.body_weldid[b] = m.body_jntnum[b] ? b : m.body_weldid[m.body_parentid[b]];
    // dof parents
    m.dof_parentid.assign(m.nv, -1);
    for (int b = 1; b < m.nbody; b++) {
      int prev = -1;
      for (int p = m.body_parentid[b]; p > 0; p = m.body_parentid[p])
        if (m.body_dofnum[p]) { prev = m.body_dofadr[p] + m.body_dofnum[p] - 1; break; }
      for (int k = 0; k < m.body_dofnum[b]; k++) {
        m.dof_parentid[m.body_dofadr[b] + k] = prev;
        prev = m.body_dofadr[b] + k;
      }
    }
    // body inertia from geoms
    m.body_mass.assign(m.nbody, 0);
    m.body_ipos.assign(3 * m.nbody, 0);
    m.body_iquat.assign(4 * m.nbody, 0);
    m.body_inertia.assign(3 * m.nbody, 0);
    for (int b = 0; b < m.nbody; b++) {
      m.body_iquat[4 * b] = 1;
      if (b == 0) continue;
      double M = 0, com[3] = {0, 0, 0}, I[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      for (int g = 0; g < m.ngeom; g++)
        if (m.geom_bodyid[g] == b) {
          M += gmass[g];
          for (int k = 0; k < 3; k++) com[k] += gmass[g] * m.geom_pos[3 * g + k];
        }
      if (M < kMinVal) continue;
      for (int k = 0; k < 3; k++) com[k] /= M;
      for (int g = 0; g < m.ngeom; g++)
        if (m.geom_bodyid[g] == b) {
          double R[9], d[3];
          quat2mat(R, &m.geom_quat[4 * g]);
          for (int k = 0; k < 3; k++) d[k] = m.geom_pos[3 * g + k] - com[k];
          double dd = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
          for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) {
              double s = 0;
              for (int k = 0; k < 3; k++) s += R[3 * r + k] * ginert[3 * g + k] * R[3 * c + k];
              I[3 * r + c] += s + gmass[g] * ((r == c ? dd : 0) - d[r] * d[c]);
            }
        }
      double ev[3], V[9];
      eig3(I, ev, V);
      // sort eigenvalues descending (with their vectors), keep right-handed
      int idx[3] = {0, 1, 2};
      for (int i = 0; i < 3; i++)
        for (int j = i + 1; j < 3; j++)
          if (ev[idx[j]] > ev[idx[i]]) std::swap(idx[i], idx[j]);
      double Vs[9], evs[3];
      for (int c = 0; c < 3; c++) {
        evs[c] = ev[idx[c]];
        for (int r = 0; r < 3; r++) Vs[3 * r + c] = V[3 * r + idx[c]];
      }
      double det = Vs[0] * (Vs[4] * Vs[8] - Vs[5] * Vs[7]) - Vs[1] * (Vs[3] * Vs[8] - Vs[5] * Vs[6]) +
                   Vs[2] * (Vs[3] * Vs[7] - Vs[4] * Vs[6]);
      if (det < 0)
        for (int r = 0; r < 3; r++) Vs[3 * r + 2] = -Vs[3 * r + 2];
      m.body_mass[b] = M;
      for (int k = 0; k < 3; k++) { m.body_ipos[3 * b + k] = com[k]; m.body_inertia[3 * b + k] = evs[k]; }
      mat2quat(&m.body_iquat[4 * b], Vs);
    }
    // buffer sizing bounds
    int maxcon = 0;
    for (int g1 = 0; g1 < m.ngeom; g1++)
      for (int g2 = g1 + 1; g2 < m.ngeom; g2++) {
        int b1 = m.geom_bodyid[g1], b2 = m.geom_bodyid[g2];
        int w1 = m.body_weldid[b1], w2 = m.body_weldid[b2];
        int wp1 = m.body_weldid[m.body_parentid[w1]], wp2 = m.body_weldid[m.body_parentid[w2]];
        if (w1 == w2) continue;
        if (w1 && w2 && (w1 == wp2 || w2 == wp1)) continue;
        if (!((m.geom_contype[g1] & m.geom_conaffinity[g2]) || (m.geom_contype[g2] & m.geom_conaffinity[g1])))
          continue;
        int t1 = std::min(m.geom_type[g1], m.geom_type[g2]), t2 = std::max(m.geom_type[g1], m.geom_type[g2]);
        int n = 1;
        if ((t1 == GEOM_PLANE && t2 == GEOM_CAPSULE) || (t1 == GEOM_CAPSULE && t2 == GEOM_CAPSULE)) n = 2;
        if (t1 == GEOM_PLANE && t2 == GEOM_PLANE) n = 0;
        maxcon += n;
      }
    m.maxcon = std::min(maxcon, m.nconmax);
    int nlim = 0;
    for (int j = 0; j < m.njnt; j++)
      if (m.jnt_limited[j] && (m.jnt_type[j] == JNT_SLIDE || m.jnt_type[j] == JNT_HINGE)) nlim += 2;
    m.maxefc = std::min(m.njmax, nlim + 4 * m.maxcon);
    if (m.nstack <= 0) m.nstack = std::max(1000, 4 * m.njmax + 40 * (m.nv * m.nv + m.nq + m.nv + 6 * m.nbody));
  }
};

}  // namespace

bool compile_mjcf_string(const std::string& xml, HostModel& m, std::string& err) {
  m = HostModel();
  XmlParser p(xml);
  std::unique_ptr<Elem> root = p.parse_elem();
  if (!root) { err = "XML: " + p.err; return false; }
  Compiler c(m, err);
  if (!c.run(root.get())) return false;
  set_const(m);
  return true;
}

bool compile_mjcf_file(const std::string& path, HostModel& m, std::string& err) {
  std::ifstream f(path, std::ios::binary);
  if (!f) { err = "could not open " + path; return false; }
  std::stringstream ss;
  ss << f.rdbuf();
  return compile_mjcf_string(ss.str(), m, err);
}

// ------------------------------------------------------------ record ----
std::vector<unsigned char> write_blob(const HostModel& m) {
  std::vector<unsigned char> out(16, 0);
  memcpy(out.data(), ILQG_BLOB_MAGIC, 8);
  int32_t nfield = 0;
  auto put = [&](const char* name, int dtype, const void* data, int count) {
    ilqg_blob_field_hdr h{};
    strncpy(h.name, name, ILQG_BLOB_NAMELEN - 1);
    h.dtype = dtype;
    h.count = count;
    size_t at = out.size();
    out.resize(at + sizeof(h));
    memcpy(out.data() + at, &h, sizeof(h));
    size_t sz = (size_t)count * (dtype == ILQG_BLOB_F64 ? 8 : 4);
    at = out.size();
    out.resize(at + ((sz + 7) & ~(size_t)7), 0);
    if (sz) memcpy(out.data() + at, data, sz);
    nfield++;
  };
#define ILQG_PUT_I(nm) { int32_t v_ = m.nm; put(#nm, ILQG_BLOB_I32, &v_, 1); }
#define ILQG_PUT_F(nm) { double v_ = m.nm; put(#nm, ILQG_BLOB_F64, &v_, 1); }
#define ILQG_PUT_FA(nm, cnt) put(#nm, ILQG_BLOB_F64, m.nm.data(), (int)m.nm.size());
#define ILQG_PUT_IA(nm, cnt) { std::vector<int32_t> v_(m.nm.begin(), m.nm.end()); put(#nm, ILQG_BLOB_I32, v_.data(), (int)v_.size()); }
  ILQG_MODEL_I32_SCALARS(ILQG_PUT_I)
  ILQG_MODEL_F64_SCALARS(ILQG_PUT_F)
  ILQG_MODEL_F64_ARRAYS(ILQG_PUT_FA)
  ILQG_MODEL_I32_ARRAYS(ILQG_PUT_IA)
  memcpy(out.data() + 8, &nfield, 4);
  return out;
}

}  // namespace ilqg
