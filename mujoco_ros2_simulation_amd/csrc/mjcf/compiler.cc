// MJCF-subset compiler: XML -> mrs::Model.
//
// Covers what the reference's scenes and this repo's benchmark scenes use:
// <include>, <compiler angle/eulerseq/autolimits/inertiafromgeom>, <option> (+<flag>), <default>
// classes with childclass/class inheritance, bodies (pos, quat/axisangle/euler/xyaxes/zaxis,
// gravcomp), <inertial> (diaginertia/fullinertia), joints (hinge/slide/ball/free, range+autolimits,
// damping, stiffness, armature, frictionloss, actuatorfrcrange, springref, ref, margin, solref/solimp
// for limit and friction), <freejoint>, geoms (plane/sphere/capsule/ellipsoid/cylinder/box/mesh,
// fromto, contype/conaffinity/condim/group/priority, friction, margin, gap, solmix, solref, solimp,
// rgba, material, mass/density), <asset> meshes (OBJ/STL files or inline vertex/face, scale; meshdir)
// and materials (rgba), sites, cameras (fixed), <frame>, <replicate count sep offset euler> with sensor
// replication and zero-padded suffixes, actuators (motor/position/velocity/general with
// dampratio->kv), sensors (rangefinder, jointpos, jointvel, actuatorfrc, framepos, framequat, gyro,
// accelerometer, force, torque), <statistic>, <visual><map znear zfar>, <keyframe><key>.
//
// The reference hands MJCF to MuJoCo's compiler at src/mujoco_system_interface.cpp:310,318
// (mj_loadXML) and :398-399 (mj_parseXMLString + mj_compile).  MuJoCo's compiler is third-party
// and absent here, so the compile-time constants it derives (dof_M0, dof_invweight0,
// body_invweight0, dampratio->kv, stat.meaninertia) are restated from the MuJoCo 3.3 documentation
// and pinned by the closed-form known answers in tests/test_compiler.py.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <set>
#include <sstream>
#include <stdexcept>

#include "mesh.h"
#include "model.h"
#include "xml.h"

namespace mrs {

namespace {

constexpr double kPi = 3.14159265358979323846;
constexpr double kMinVal = 1e-15;

[[noreturn]] void fail(const XmlElement* e, const std::string& msg) {
  std::string where = e ? (" (line " + std::to_string(e->line) + ", <" + e->tag + ">)") : "";
  throw std::runtime_error("MJCF error: " + msg + where);
}
// a valid MJCF construct this compiler does not restate: rejected at load instead of ignored
[[noreturn]] void unsupported(const XmlElement* e, const std::string& msg) { fail(e, "not supported: " + msg); }

// ---------------------------------------------------------------- fp64 3D math
struct V3 { double v[3]; };

void quat_mul(double r[4], const double a[4], const double b[4]) {
  double t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                 a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                 a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                 a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  std::memcpy(r, t, sizeof t);
}
void quat_normalize(double q[4]) {
  double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < kMinVal) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  for (int i = 0; i < 4; ++i) q[i] /= n;
}
void quat2mat(double m[9], const double q[4]) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = w * w + x * x - y * y - z * z; m[1] = 2 * (x * y - w * z); m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z); m[4] = w * w - x * x + y * y - z * z; m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y); m[7] = 2 * (y * z + w * x); m[8] = w * w - x * x - y * y + z * z;
}
void rot_vec_quat(double r[3], const double v[3], const double q[4]) {
  double m[9];
  quat2mat(m, q);
  double t[3] = {m[0] * v[0] + m[1] * v[1] + m[2] * v[2], m[3] * v[0] + m[4] * v[1] + m[5] * v[2],
                 m[6] * v[0] + m[7] * v[1] + m[8] * v[2]};
  std::memcpy(r, t, sizeof t);
}
void axis_angle_quat(double q[4], const double axis[3], double angle) {
  double s = std::sin(angle / 2);
  q[0] = std::cos(angle / 2); q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}
// rotation matrix (columns = frame axes) -> quaternion (Shepperd)
void mat2quat(double q[4], const double m[9]) {
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
  if (q[0] < 0) for (int i = 0; i < 4; ++i) q[i] = -q[i];
  quat_normalize(q);
}
void cross3(double r[3], const double a[3], const double b[3]) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  std::memcpy(r, t, sizeof t);
}
double dot3(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
double norm3(const double a[3]) { return std::sqrt(dot3(a, a)); }
// quaternion rotating z-axis onto unit vector v (MuJoCo mju_quatZ2Vec semantics)
void quat_z2vec(double q[4], const double vin[3]) {
  double v[3] = {vin[0], vin[1], vin[2]};
  double n = norm3(v);
  q[0] = 1; q[1] = q[2] = q[3] = 0;
  if (n < kMinVal) return;
  for (double& x : v) x /= n;
  double z[3] = {0, 0, 1}, a[3];
  cross3(a, z, v);
  double s = norm3(a);
  if (s < 1e-10) {
    if (v[2] < 0) { q[0] = 0; q[1] = 1; }
    return;
  }
  for (double& x : a) x /= s;
  axis_angle_quat(q, a, std::atan2(s, v[2]));
}

// symmetric 3x3 eigen-decomposition (Jacobi); eigenvalues sorted descending, vecs as columns
void eig3(double eval[3], double evec[9], const double A[9]) {
  double a[9];
  std::memcpy(a, A, sizeof a);
  double v[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  for (int sweep = 0; sweep < 50; ++sweep) {
    double off = a[1] * a[1] + a[2] * a[2] + a[5] * a[5];
    if (off < 1e-30) break;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        double apq = a[p * 3 + q];
        if (std::fabs(apq) < 1e-300) continue;
        double theta = (a[q * 3 + q] - a[p * 3 + p]) / (2 * apq);
        double t = (theta >= 0 ? 1 : -1) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
        double c = 1 / std::sqrt(t * t + 1), s = t * c;
        for (int k = 0; k < 3; ++k) {  // A = A J
          double akp = a[k * 3 + p], akq = a[k * 3 + q];
          a[k * 3 + p] = c * akp - s * akq; a[k * 3 + q] = s * akp + c * akq;
        }
        for (int k = 0; k < 3; ++k) {  // A = J^T A
          double apk = a[p * 3 + k], aqk = a[q * 3 + k];
          a[p * 3 + k] = c * apk - s * aqk; a[q * 3 + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < 3; ++k) {
          double vkp = v[k * 3 + p], vkq = v[k * 3 + q];
          v[k * 3 + p] = c * vkp - s * vkq; v[k * 3 + q] = s * vkp + c * vkq;
        }
      }
  }
  int idx[3] = {0, 1, 2};
  std::sort(idx, idx + 3, [&](int i, int j) { return a[i * 4] > a[j * 4]; });
  for (int c = 0; c < 3; ++c) {
    eval[c] = a[idx[c] * 4];
    for (int r = 0; r < 3; ++r) evec[r * 3 + c] = v[r * 3 + idx[c]];
  }
  // right-handed frame
  double c0[3] = {evec[0], evec[3], evec[6]}, c1[3] = {evec[1], evec[4], evec[7]}, c2[3];
  cross3(c2, c0, c1);
  evec[2] = c2[0]; evec[5] = c2[1]; evec[8] = c2[2];
}

// ---------------------------------------------------------------- attribute parsing
std::vector<double> parse_reals(const std::string& s, const XmlElement* e, const char* key) {
  std::vector<double> out;
  const char* p = s.c_str();
  char* end = nullptr;
  for (;;) {
    while (*p && std::isspace(static_cast<unsigned char>(*p))) ++p;
    if (!*p) break;
    double v = std::strtod(p, &end);
    if (end == p) fail(e, std::string("cannot parse number in attribute '") + key + "': " + s);
    out.push_back(v);
    p = end;
  }
  return out;
}

struct DefaultClass {
  std::string name;
  DefaultClass* parent = nullptr;
  std::map<std::string, std::map<std::string, std::string>> attrs;  // tag -> key -> value
};

struct Options {
  bool degree = true;
  std::string eulerseq = "xyz";
  bool autolimits = true;
  int inertiafromgeom = 2;  // 0 false, 1 true, 2 auto
  std::string meshdir;      // <compiler meshdir / assetdir>
  int inertiagroup[2] = {0, 5};  // inertiagrouprange: geom groups that contribute to inertia
  double boundmass = 0, boundinertia = 0, settotalmass = -1;
  bool balanceinertia = false, strippath = false;
};

// a rigid frame: child = frame ∘ local
struct Frame {
  double pos[3] = {0, 0, 0};
  double quat[4] = {1, 0, 0, 0};
  void apply(double p[3], double q[4]) const {
    double r[3];
    rot_vec_quat(r, p, quat);
    for (int i = 0; i < 3; ++i) p[i] = pos[i] + r[i];
    quat_mul(q, quat, q);
  }
  Frame compose(const Frame& local) const {
    Frame f = local;
    apply(f.pos, f.quat);
    return f;
  }
};

struct GeomRec {
  std::string name;
  int type = MRS_GEOM_SPHERE, contype = 1, conaffinity = 1, condim = 3, group = 0, priority = 0;
  double size[3] = {0, 0, 0}, pos[3] = {0, 0, 0}, quat[4] = {1, 0, 0, 0};
  double friction[3] = {1, 0.005, 0.0001}, margin = 0, gap = 0, solmix = 1;
  double solref[2] = {0.02, 1}, solimp[5] = {0.9, 0.95, 0.001, 0.5, 2};
  double rgba[4] = {0.5, 0.5, 0.5, 1};
  double mass = -1, density = 1000;
  int mesh = -1;  // mesh id (type mesh)
  int matid = -1;  // material id
};
// a <light> (MuJoCo's defaults), pose in its body's frame
struct LightRec {
  double pos[3] = {0, 0, 0}, dir[3] = {0, 0, -1}, ambient[3] = {0, 0, 0}, diffuse[3] = {0.7, 0.7, 0.7},
         specular[3] = {0.3, 0.3, 0.3}, attenuation[3] = {1, 0, 0}, cutoff = 45, exponent = 10;
  int directional = 0, castshadow = 1, active = 1;
};
// a processed mesh asset: vertices in its inertial frame; pos/quat place that frame in the mesh file's
// frame; volume and unit-density principal moments for the geom's mass
struct MeshRec {
  std::string name;
  std::vector<double> vert;
  std::vector<int> face, hull;
  std::vector<std::vector<int>> poly;  // hull faces as polygons (hull_polygons)
  std::vector<double> poly_normal;
  double pos[3] = {0, 0, 0}, quat[4] = {1, 0, 0, 0};
  double volume = 0, inertia[3] = {0, 0, 0}, half[3] = {0, 0, 0}, rbound = 0;
};
struct SiteRec { std::string name; double pos[3] = {0, 0, 0}, quat[4] = {1, 0, 0, 0}; };
struct CamRec {
  std::string name;
  double pos[3] = {0, 0, 0}, quat[4] = {1, 0, 0, 0}, fovy = 45;
  int res[2] = {1, 1};
};
struct JointRec {
  std::string name;
  int type = MRS_JNT_HINGE;
  double pos[3] = {0, 0, 0}, axis[3] = {0, 0, 1};
  double range[2] = {0, 0};
  int limited = 2;  // auto
  bool range_given = false;
  double damping = 0, stiffness = 0, armature = 0, frictionloss = 0, springref = 0, ref = 0,
         margin = 0;
  double actfrcrange[2] = {0, 0};
  int actfrclimited = 2;
  bool actfrcrange_given = false;
  double solreflimit[2] = {0.02, 1}, solimplimit[5] = {0.9, 0.95, 0.001, 0.5, 2};
  double solreffriction[2] = {0.02, 1}, solimpfriction[5] = {0.9, 0.95, 0.001, 0.5, 2};
};
struct BodyRec {
  std::string name;
  int parent = -1;
  double pos[3] = {0, 0, 0}, quat[4] = {1, 0, 0, 0};
  bool has_inertial = false;
  double ipos[3] = {0, 0, 0}, iquat[4] = {1, 0, 0, 0}, mass = 0, inertia[3] = {0, 0, 0};
  double gravcomp = 0;
  std::vector<JointRec> joints;
  std::vector<GeomRec> geoms;
  std::vector<SiteRec> sites;
  std::vector<CamRec> cams;
  std::vector<LightRec> lights;
};

struct Compiler {
  Options opt;
  std::map<std::string, std::unique_ptr<DefaultClass>> classes;
  std::vector<BodyRec> bodies;
  // replicate bookkeeping: original element name -> (replica names, replica suffixes)
  std::map<std::string, std::vector<std::string>> replica_suffixes;
  Model m;
  bool extent_given = false;
  std::string basedir = ".";
  std::vector<MeshRec> meshes;
  std::map<std::string, int> mesh_ids;
  std::map<std::string, std::vector<double>> materials;  // name -> rgba
  std::map<std::string, int> material_ids, texture_ids;

  Compiler() {
    auto main = std::make_unique<DefaultClass>();
    main->name = "main";
    classes["main"] = std::move(main);
  }

  // ---- attribute lookup through the default-class chain
  const std::string* lookup(const XmlElement* e, const DefaultClass* cls, const std::string& tag,
                            const std::string& key) const {
    if (e) {
      if (auto* v = e->attr(key)) return v;
    }
    for (const DefaultClass* c = cls; c; c = c->parent) {
      auto it = c->attrs.find(tag);
      if (it == c->attrs.end()) continue;
      auto jt = it->second.find(key);
      if (jt != it->second.end()) return &jt->second;
    }
    return nullptr;
  }
  const DefaultClass* resolve_class(const XmlElement* e, const std::string& childclass) const {
    std::string name = childclass.empty() ? "main" : childclass;
    if (auto* c = e->attr("class")) name = *c;
    auto it = classes.find(name);
    if (it == classes.end()) fail(e, "unknown default class '" + name + "'");
    return it->second.get();
  }
  bool get_reals(const XmlElement* e, const DefaultClass* cls, const std::string& tag,
                 const std::string& key, double* out, int n, bool exact = false) const {
    const std::string* s = lookup(e, cls, tag, key);
    if (!s) return false;
    auto v = parse_reals(*s, e, key.c_str());
    if (exact && static_cast<int>(v.size()) != n)
      fail(e, "attribute '" + key + "' expects " + std::to_string(n) + " numbers");
    if (v.empty() || static_cast<int>(v.size()) > n)
      fail(e, "attribute '" + key + "' has a wrong number of values");
    for (size_t i = 0; i < v.size(); ++i) out[i] = v[i];
    return true;
  }
  bool get_real(const XmlElement* e, const DefaultClass* cls, const std::string& tag,
                const std::string& key, double& out) const {
    return get_reals(e, cls, tag, key, &out, 1, true);
  }
  bool get_int(const XmlElement* e, const DefaultClass* cls, const std::string& tag,
               const std::string& key, int& out) const {
    double v;
    if (!get_real(e, cls, tag, key, v)) return false;
    out = static_cast<int>(v);
    return true;
  }
  bool get_str(const XmlElement* e, const DefaultClass* cls, const std::string& tag,
               const std::string& key, std::string& out) const {
    const std::string* s = lookup(e, cls, tag, key);
    if (!s) return false;
    out = *s;
    return true;
  }
  int get_tristate(const XmlElement* e, const DefaultClass* cls, const std::string& tag,
                   const std::string& key) const {
    std::string s;
    if (!get_str(e, cls, tag, key, s)) return 2;
    if (s == "true") return 1;
    if (s == "false") return 0;
    if (s == "auto") return 2;
    fail(e, "attribute '" + key + "' must be true/false/auto");
  }

  // orientation: quat | axisangle | euler | xyaxes | zaxis (MuJoCo orientation specifiers)
  bool get_orientation(const XmlElement* e, const DefaultClass* cls, const std::string& tag,
                       double q[4]) const {
    double v[9];
    int count = 0;
    bool found = false;
    if (get_reals(e, cls, tag, "quat", v, 4, true)) {
      for (int i = 0; i < 4; ++i) q[i] = v[i];
      quat_normalize(q);
      found = true; ++count;
    }
    if (get_reals(e, cls, tag, "axisangle", v, 4, true)) {
      double ang = opt.degree ? v[3] * kPi / 180 : v[3];
      double n = norm3(v);
      if (n < kMinVal) fail(e, "axisangle axis too small");
      double ax[3] = {v[0] / n, v[1] / n, v[2] / n};
      axis_angle_quat(q, ax, ang);
      found = true; ++count;
    }
    if (get_reals(e, cls, tag, "euler", v, 3, true)) {
      q[0] = 1; q[1] = q[2] = q[3] = 0;
      for (int i = 0; i < 3; ++i) {
        double ang = opt.degree ? v[i] * kPi / 180 : v[i];
        char c = opt.eulerseq[i];
        double ax[3] = {0, 0, 0};
        ax[std::tolower(c) - 'x'] = 1;
        double r[4];
        axis_angle_quat(r, ax, ang);
        if (std::islower(static_cast<unsigned char>(c))) quat_mul(q, q, r);
        else quat_mul(q, r, q);
      }
      quat_normalize(q);
      found = true; ++count;
    }
    if (get_reals(e, cls, tag, "xyaxes", v, 6, true)) {
      double x[3] = {v[0], v[1], v[2]}, y[3] = {v[3], v[4], v[5]}, z[3];
      double nx = norm3(x);
      for (double& a : x) a /= nx;
      double d = dot3(x, y);
      for (int i = 0; i < 3; ++i) y[i] -= d * x[i];
      double ny = norm3(y);
      for (double& a : y) a /= ny;
      cross3(z, x, y);
      double mat[9] = {x[0], y[0], z[0], x[1], y[1], z[1], x[2], y[2], z[2]};
      mat2quat(q, mat);
      found = true; ++count;
    }
    if (get_reals(e, cls, tag, "zaxis", v, 3, true)) {
      quat_z2vec(q, v);
      found = true; ++count;
    }
    if (count > 1) fail(e, "multiple orientation specifiers");
    return found;
  }

  std::string elem_name(const XmlElement* e, const std::string& suffix) const {
    if (auto* n = e->attr("name")) return n->empty() ? "" : *n + suffix;
    return "";
  }

  // ---- top-level sections
  void parse_compiler(const XmlElement* e) {
    if (auto* a = e->attr("angle")) {
      if (*a == "radian") opt.degree = false;
      else if (*a == "degree") opt.degree = true;
      else fail(e, "angle must be radian or degree");
    }
    if (auto* s = e->attr("eulerseq")) {
      if (s->size() != 3) fail(e, "eulerseq must have 3 characters");
      opt.eulerseq = *s;
    }
    if (auto* a = e->attr("autolimits")) opt.autolimits = (*a == "true");
    if (auto* a = e->attr("inertiafromgeom"))
      opt.inertiafromgeom = (*a == "true") ? 1 : (*a == "false") ? 0 : 2;
    if (auto* a = e->attr("assetdir")) opt.meshdir = *a;
    if (auto* a = e->attr("meshdir")) opt.meshdir = *a;
    auto boolean = [&](const char* name, bool& out) {
      if (auto* a = e->attr(name)) {
        if (*a == "true") out = true;
        else if (*a == "false") out = false;
        else fail(e, std::string(name) + " must be true or false");
      }
    };
    auto real = [&](const char* name, double& out) {
      if (auto* a = e->attr(name)) out = parse_reals(*a, e, name).at(0);
    };
    // mass / inertia post-processing of mjCBody::Compile and mjCModel (settotalmass)
    real("boundmass", opt.boundmass);
    real("boundinertia", opt.boundinertia);
    real("settotalmass", opt.settotalmass);
    boolean("balanceinertia", opt.balanceinertia);
    boolean("strippath", opt.strippath);
    if (auto* a = e->attr("inertiagrouprange")) {
      auto v = parse_reals(*a, e, "inertiagrouprange");
      if (v.size() != 2) fail(e, "inertiagrouprange needs 2 values");
      opt.inertiagroup[0] = static_cast<int>(v[0]);
      opt.inertiagroup[1] = static_cast<int>(v[1]);
    }
    // accepted with no effect here: options of the viewer, the asset loader and the compiler's
    // threading / saving, which do not change the compiled dynamics, rays or depth
    bool unused = false;
    boolean("usethread", unused);
    boolean("saveinertial", unused);
    if (e->attr("texturedir")) {}
    // options that would change the model and are not restated: rejected rather than ignored
    for (const char* name : {"discardvisual", "fusestatic", "fitaabb", "alignfree"}) {
      bool on = false;
      boolean(name, on);
      if (on) unsupported(e, std::string("<compiler ") + name + "=\"true\"> is not supported");
    }
    if (auto* a = e->attr("coordinate"))
      if (*a != "local") unsupported(e, "<compiler coordinate=\"" + *a + "\"> is not supported");
    static const std::set<std::string> known = {
        "angle", "eulerseq", "autolimits", "inertiafromgeom", "assetdir", "meshdir", "texturedir", "boundmass",
        "boundinertia", "settotalmass", "balanceinertia", "strippath", "inertiagrouprange", "usethread",
        "saveinertial", "discardvisual", "fusestatic", "fitaabb", "alignfree", "coordinate"};
    for (auto& kv : e->attrs)
      if (!known.count(kv.first)) unsupported(e, "unknown <compiler> attribute '" + kv.first + "'");
  }

  // ---- <asset>: meshes and materials.  A mesh is processed as MuJoCo's compiler does: faces from the
  // file or the face attribute (else the convex hull's), volume / centre of mass / inertia from the
  // triangles (the hull's if the surface encloses no volume), then the vertices are re-expressed in
  // the inertial frame (centre of mass, principal axes, right-handed) and the geoms using the mesh
  // are offset by that frame.
  void parse_asset(const XmlElement* sec) {
    // textures first (materials refer to them), then everything else in document order
    for (int pass = 0; pass < 2; ++pass)
    for (auto& c : sec->children) {
      const XmlElement* e = c.get();
      if ((pass == 0) != (e->tag == "texture")) continue;
      if (e->tag == "material") {
        // [upstream mjCMaterial] rgba, texture, texrepeat, texuniform, specular, shininess, emission
        const DefaultClass* cls = resolve_class(e, "");
        double rgba[4] = {1, 1, 1, 1}, rep[2] = {1, 1}, spec = 0.5, shin = 0.5, emis = 0;
        get_reals(e, cls, "material", "rgba", rgba, 4, true);
        get_reals(e, cls, "material", "texrepeat", rep, 2, true);
        get_real(e, cls, "material", "specular", spec);
        get_real(e, cls, "material", "shininess", shin);
        get_real(e, cls, "material", "emission", emis);
        std::string tex, uni;
        int texid = -1;
        if (get_str(e, cls, "material", "texture", tex)) {
          auto it = texture_ids.find(tex);
          if (it == texture_ids.end()) fail(e, "material references unknown texture '" + tex + "'");
          texid = it->second;
        }
        get_str(e, cls, "material", "texuniform", uni);
        if (auto* n = e->attr("name")) {
          materials[*n] = std::vector<double>(rgba, rgba + 4);
          material_ids[*n] = static_cast<int>(m.mat_texid.size());
        }
        m.mat_texid.push_back(texid);
        m.mat_texuniform.push_back(uni == "true");
        m.mat_rgba.insert(m.mat_rgba.end(), rgba, rgba + 4);
        m.mat_texrepeat.insert(m.mat_texrepeat.end(), rep, rep + 2);
        m.mat_specular.push_back(spec);
        m.mat_shininess.push_back(shin);
        m.mat_emission.push_back(emis);
        continue;
      }
      if (e->tag == "texture") {
        // [upstream mjCTexture] procedural builtins only (no image files): checker, gradient, flat
        std::string type = "cube", builtin = "none", mark = "none", file;
        get_str(e, nullptr, "texture", "type", type);
        get_str(e, nullptr, "texture", "builtin", builtin);
        get_str(e, nullptr, "texture", "mark", mark);
        if (get_str(e, nullptr, "texture", "file", file) || e->attr("fileright") || e->attr("gridsize"))
          fail(e, "texture files are not supported (builtin checker / gradient / flat only)");
        double rgb1[3] = {0.8, 0.8, 0.8}, rgb2[3] = {0.5, 0.5, 0.5}, markrgb[3] = {0, 0, 0}, w = 0, h = 0;
        get_reals(e, nullptr, "texture", "rgb1", rgb1, 3, true);
        get_reals(e, nullptr, "texture", "rgb2", rgb2, 3, true);
        get_reals(e, nullptr, "texture", "markrgb", markrgb, 3, true);
        get_real(e, nullptr, "texture", "width", w);
        get_real(e, nullptr, "texture", "height", h);
        const int t = type == "2d" ? MRS_TEX_2D : type == "cube" ? MRS_TEX_CUBE : type == "skybox" ? MRS_TEX_SKYBOX : -1;
        const int b = builtin == "none" ? MRS_BUILTIN_NONE : builtin == "gradient" ? MRS_BUILTIN_GRADIENT
                      : builtin == "checker" ? MRS_BUILTIN_CHECKER : builtin == "flat" ? MRS_BUILTIN_FLAT : -1;
        const int mk = mark == "none" ? MRS_MARK_NONE : mark == "edge" ? MRS_MARK_EDGE : mark == "cross" ? MRS_MARK_CROSS : -1;
        if (t < 0 || b < 0 || mk < 0) fail(e, "unsupported texture type / builtin / mark");
        if (b == MRS_BUILTIN_NONE) fail(e, "a texture needs a builtin (texture files are not supported)");
        if (auto* n = e->attr("name")) texture_ids[*n] = static_cast<int>(m.tex_type.size());
        m.tex_type.push_back(t);
        m.tex_builtin.push_back(b);
        m.tex_mark.push_back(mk);
        m.tex_width.push_back(std::max(1, static_cast<int>(w > 0 ? w : 2)));
        m.tex_height.push_back(std::max(1, static_cast<int>(h > 0 ? h : (w > 0 ? w : 2))));
        m.tex_rgb1.insert(m.tex_rgb1.end(), rgb1, rgb1 + 3);
        m.tex_rgb2.insert(m.tex_rgb2.end(), rgb2, rgb2 + 3);
        m.tex_markrgb.insert(m.tex_markrgb.end(), markrgb, markrgb + 3);
        continue;
      }
      if (e->tag == "hfield" || e->tag == "skin" || e->tag == "model") {
        if (e->tag == "hfield") fail(e, "height fields are not supported");
        continue;
      }
      if (e->tag != "mesh") fail(e, "unsupported asset element");
      MeshRec r;
      MeshAsset a;
      std::string file;
      const bool has_file = get_str(e, nullptr, "mesh", "file", file);
      if (has_file) {
        if (opt.strippath) {  // <compiler strippath>: keep the file name only
          const size_t k = file.find_last_of("/\\");
          if (k != std::string::npos) file = file.substr(k + 1);
        }
        std::string path = file;
        if (!path.empty() && path[0] != '/') {
          std::string dir = opt.meshdir;
          if (dir.empty() || dir[0] != '/') dir = basedir + (dir.empty() ? "" : "/" + dir);
          path = dir + "/" + file;
        }
        try {
          a = load_mesh_file(path);
        } catch (const std::exception& ex) {
          fail(e, ex.what());
        }
      }
      if (auto* v = e->attr("vertex")) {
        if (has_file) fail(e, "mesh has both file and vertex");
        a.vert = parse_reals(*v, e, "vertex");
        if (a.vert.size() % 3 || a.vert.size() < 12) fail(e, "vertex needs at least 4 points (3 numbers each)");
      }
      if (auto* f = e->attr("face")) {
        auto fv = parse_reals(*f, e, "face");
        if (fv.size() % 3) fail(e, "face needs 3 vertex ids per triangle");
        a.face.clear();
        for (double x : fv) {
          if (x < 0 || x >= static_cast<double>(a.vert.size() / 3)) fail(e, "face vertex id out of range");
          a.face.push_back(static_cast<int>(x));
        }
      }
      if (a.vert.empty()) fail(e, "mesh needs a file or a vertex attribute");
      double scale[3] = {1, 1, 1};
      get_reals(e, nullptr, "mesh", "scale", scale, 3, true);
      for (size_t i = 0; i < a.vert.size(); ++i) a.vert[i] *= scale[i % 3];
      if (scale[0] * scale[1] * scale[2] < 0)  // a mirroring scale flips the winding
        for (size_t t = 0; t + 2 < a.face.size(); t += 3) std::swap(a.face[t + 1], a.face[t + 2]);
      std::vector<int> hull_face;
      try {
        convex_hull(a.vert, hull_face, r.hull);
      } catch (const std::exception& ex) {
        fail(e, ex.what());
      }
      if (a.face.empty()) a.face = hull_face;
      double vol, com[3], I[9];
      mesh_mass_properties(a.vert, a.face, vol, com, I);
      if (!(vol > 1e-12)) mesh_mass_properties(a.vert, hull_face, vol, com, I);
      if (!(vol > 1e-12)) fail(e, "mesh volume is too small");
      double ev[3], R[9];
      eig3(ev, R, I);
      mat2quat(r.quat, R);
      quat2mat(R, r.quat);  // the frame the quaternion stores exactly
      std::memcpy(r.pos, com, sizeof com);
      r.volume = vol;
      for (int k = 0; k < 3; ++k) r.inertia[k] = ev[k];
      r.vert.resize(a.vert.size());
      for (size_t i = 0; i < a.vert.size() / 3; ++i) {
        const double d[3] = {a.vert[3 * i] - com[0], a.vert[3 * i + 1] - com[1], a.vert[3 * i + 2] - com[2]};
        for (int k = 0; k < 3; ++k) {
          const double x = R[k] * d[0] + R[3 + k] * d[1] + R[6 + k] * d[2];
          r.vert[3 * i + k] = x;
          r.half[k] = std::max(r.half[k], std::fabs(x));
        }
        r.rbound = std::max(r.rbound, norm3(&r.vert[3 * i]));
      }
      r.face = a.face;
      hull_polygons(r.vert, hull_face, r.poly, r.poly_normal);
      std::string name;
      if (!get_str(e, nullptr, "mesh", "name", name)) {
        if (!has_file) fail(e, "a mesh without a file needs a name");
        name = file.substr(file.find_last_of('/') + 1);
        name = name.substr(0, name.find_last_of('.'));
      }
      r.name = name;
      if (mesh_ids.count(name)) fail(e, "repeated mesh name '" + name + "'");
      mesh_ids[name] = static_cast<int>(meshes.size());
      meshes.push_back(std::move(r));
    }
  }
  void parse_option(const XmlElement* e) {
    double v[3];
    if (auto* s = e->attr("timestep")) m.timestep = parse_reals(*s, e, "timestep").at(0);
    if (e->attr("gravity")) {
      get_reals(e, nullptr, "option", "gravity", v, 3, true);
      for (int i = 0; i < 3; ++i) m.gravity[i] = v[i];
    }
    if (auto* s = e->attr("integrator")) {
      if (*s == "Euler") m.integrator = MRS_INT_EULER;
      else if (*s == "RK4") m.integrator = MRS_INT_RK4;
      else if (*s == "implicit") m.integrator = MRS_INT_IMPLICIT;
      else if (*s == "implicitfast") m.integrator = MRS_INT_IMPLICITFAST;
      else fail(e, "unknown integrator " + *s);
    }
    if (auto* s = e->attr("solver")) {
      if (*s == "PGS") m.solver = MRS_SOL_PGS;
      else if (*s == "CG") m.solver = MRS_SOL_CG;
      else if (*s == "Newton") m.solver = MRS_SOL_NEWTON;
      else fail(e, "unknown solver " + *s);
    }
    if (auto* s = e->attr("iterations")) m.iterations = static_cast<int>(parse_reals(*s, e, "iterations").at(0));
    if (auto* s = e->attr("tolerance")) m.tolerance = parse_reals(*s, e, "tolerance").at(0);
    if (auto* s = e->attr("impratio")) {
      m.impratio = parse_reals(*s, e, "impratio").at(0);
      if (!(m.impratio > 0)) fail(e, "impratio must be positive");
    }
    if (auto* s = e->attr("ls_tolerance")) m.ls_tolerance = parse_reals(*s, e, "ls_tolerance").at(0);
    if (auto* s = e->attr("ls_iterations"))
      m.ls_iterations = static_cast<int>(parse_reals(*s, e, "ls_iterations").at(0));
    if (auto* s = e->attr("cone")) {
      if (*s == "pyramidal") m.cone = MRS_CONE_PYRAMIDAL;
      else if (*s == "elliptic") m.cone = MRS_CONE_ELLIPTIC;
      else fail(e, "unknown cone " + *s);
    }
    for (auto& c : e->children) {
      if (c->tag != "flag") continue;
      static const std::pair<const char*, int> kFlags[] = {
          {"constraint", MRS_DSBL_CONSTRAINT}, {"equality", MRS_DSBL_EQUALITY},
          {"frictionloss", MRS_DSBL_FRICTIONLOSS}, {"limit", MRS_DSBL_LIMIT},
          {"contact", MRS_DSBL_CONTACT}, {"passive", MRS_DSBL_PASSIVE},
          {"gravity", MRS_DSBL_GRAVITY}, {"clampctrl", MRS_DSBL_CLAMPCTRL},
          {"warmstart", MRS_DSBL_WARMSTART}, {"filterparent", MRS_DSBL_FILTERPARENT},
          {"actuation", MRS_DSBL_ACTUATION}, {"refsafe", MRS_DSBL_REFSAFE},
          {"sensor", MRS_DSBL_SENSOR}, {"eulerdamp", MRS_DSBL_EULERDAMP},
          {"autoreset", MRS_DSBL_AUTORESET}};
      for (auto& kv : c->attrs) {
        bool known = false;
        for (auto& f : kFlags)
          if (kv.first == f.first) {
            known = true;
            if (kv.second == "disable") m.disableflags |= f.second;
            else if (kv.second == "enable") m.disableflags &= ~f.second;
            else fail(c.get(), "flag values must be enable/disable");
          }
        if (!known) fail(c.get(), "unsupported option flag '" + kv.first + "'");
      }
    }
  }
  void parse_default(const XmlElement* e, DefaultClass* parent) {
    DefaultClass* cls;
    if (!parent) {
      cls = classes["main"].get();
      if (auto* n = e->attr("class"))
        if (*n != "main") fail(e, "top-level default class must be 'main'");
    } else {
      auto* n = e->attr("class");
      if (!n) fail(e, "nested default requires a class name");
      if (classes.count(*n)) fail(e, "repeated default class '" + *n + "'");
      auto c = std::make_unique<DefaultClass>();
      c->name = *n;
      c->parent = parent;
      cls = c.get();
      classes[*n] = std::move(c);
    }
    for (auto& c : e->children) {
      if (c->tag == "default") { parse_default(c.get(), cls); continue; }
      auto& a = cls->attrs[c->tag];
      for (auto& kv : c->attrs) a[kv.first] = kv.second;
    }
  }

  // ---- worldbody traversal
  void parse_body_children(const XmlElement* e, int body_id, const std::string& childclass,
                           const Frame& frame, const std::string& suffix) {
    for (auto& cp : e->children) {
      const XmlElement* c = cp.get();
      if (c->tag == "body") {
        parse_body(c, body_id, childclass, frame, suffix);
      } else if (c->tag == "geom") {
        bodies[body_id].geoms.push_back(parse_geom(c, childclass, frame, suffix));
      } else if (c->tag == "site") {
        bodies[body_id].sites.push_back(parse_site(c, childclass, frame, suffix));
      } else if (c->tag == "camera") {
        bodies[body_id].cams.push_back(parse_camera(c, childclass, frame, suffix));
      } else if (c->tag == "joint" || c->tag == "freejoint") {
        if (body_id == 0) fail(c, "joints cannot be attached to the world body");
        bodies[body_id].joints.push_back(parse_joint(c, childclass, frame, suffix));
      } else if (c->tag == "inertial") {
        if (body_id == 0) fail(c, "world body cannot have <inertial>");
        parse_inertial(c, bodies[body_id], frame);
      } else if (c->tag == "frame") {
        Frame local;
        get_reals(c, nullptr, "frame", "pos", local.pos, 3, true);
        get_orientation(c, nullptr, "frame", local.quat);
        std::string cc = childclass;
        if (auto* s = c->attr("childclass")) cc = *s;
        parse_body_children(c, body_id, cc, frame.compose(local), suffix);
      } else if (c->tag == "replicate") {
        parse_replicate(c, body_id, childclass, frame, suffix);
      } else if (c->tag == "light") {
        bodies[body_id].lights.push_back(parse_light(c, childclass, frame));
      } else if (c->tag == "composite" || c->tag == "plugin") {
        fail(c, "unsupported element");
      } else {
        fail(c, "unsupported element in body");
      }
    }
  }
  void parse_replicate(const XmlElement* e, int body_id, const std::string& childclass,
                       const Frame& frame, const std::string& suffix) {
    auto* cs = e->attr("count");
    if (!cs) fail(e, "replicate requires 'count'");
    int count = static_cast<int>(parse_reals(*cs, e, "count").at(0));
    if (count < 1) fail(e, "replicate count must be positive");
    std::string sep = e->attr("sep") ? *e->attr("sep") : "";
    double offset[3] = {0, 0, 0}, euler[3] = {0, 0, 0};
    get_reals(e, nullptr, "replicate", "offset", offset, 3, true);
    get_reals(e, nullptr, "replicate", "euler", euler, 3, true);
    double rq[4] = {1, 0, 0, 0};
    for (int i = 0; i < 3; ++i) {
      double ang = opt.degree ? euler[i] * kPi / 180 : euler[i];
      double ax[3] = {0, 0, 0};
      ax[std::tolower(opt.eulerseq[i]) - 'x'] = 1;
      double r[4];
      axis_angle_quat(r, ax, ang);
      if (std::islower(static_cast<unsigned char>(opt.eulerseq[i]))) quat_mul(rq, rq, r);
      else quat_mul(rq, r, rq);
    }
    int ndigits = static_cast<int>(std::to_string(count).size());
    // collect names of directly or indirectly replicated named elements for sensor replication
    std::vector<std::string> names;
    std::function<void(const XmlElement*)> collect = [&](const XmlElement* x) {
      for (auto& c : x->children) {
        if (auto* n = c->attr("name")) names.push_back(*n + suffix);
        collect(c.get());
      }
    };
    collect(e);
    Frame acc;  // accumulated replica transform: T_i = T_{i-1} ∘ (offset, R)
    for (int i = 0; i < count; ++i) {
      std::string idx = std::to_string(i);
      std::string sfx = sep + std::string(ndigits - idx.size(), '0') + idx;
      parse_body_children(e, body_id, childclass, frame.compose(acc), suffix + sfx);
      for (auto& n : names) replica_suffixes[n].push_back(sfx);
      double step_pos[3];
      rot_vec_quat(step_pos, offset, acc.quat);
      for (int k = 0; k < 3; ++k) acc.pos[k] += step_pos[k];
      quat_mul(acc.quat, acc.quat, rq);
      quat_normalize(acc.quat);
    }
  }
  void parse_body(const XmlElement* e, int parent, const std::string& parent_childclass,
                  const Frame& frame, const std::string& suffix) {
    BodyRec b;
    b.name = elem_name(e, suffix);
    b.parent = parent;
    std::string childclass = parent_childclass;
    if (auto* s = e->attr("childclass")) {
      if (!classes.count(*s)) fail(e, "unknown childclass '" + *s + "'");
      childclass = *s;
    }
    get_reals(e, nullptr, "body", "pos", b.pos, 3, true);
    get_orientation(e, nullptr, "body", b.quat);
    frame.apply(b.pos, b.quat);
    if (auto* s = e->attr("gravcomp")) b.gravcomp = parse_reals(*s, e, "gravcomp").at(0);
    if (e->attr("mocap") && *e->attr("mocap") == "true") fail(e, "mocap bodies are not supported");
    int id = static_cast<int>(bodies.size());
    bodies.push_back(b);
    parse_body_children(e, id, childclass, Frame(), suffix);
  }
  void parse_inertial(const XmlElement* e, BodyRec& b, const Frame& frame) {
    b.has_inertial = true;
    get_reals(e, nullptr, "inertial", "pos", b.ipos, 3, true);
    get_orientation(e, nullptr, "inertial", b.iquat);
    frame.apply(b.ipos, b.iquat);
    if (!get_real(e, nullptr, "inertial", "mass", b.mass)) fail(e, "inertial requires mass");
    double d[3], f[6];
    if (get_reals(e, nullptr, "inertial", "diaginertia", d, 3, true)) {
      for (int i = 0; i < 3; ++i) b.inertia[i] = d[i];
    } else if (get_reals(e, nullptr, "inertial", "fullinertia", f, 6, true)) {
      double A[9] = {f[0], f[3], f[4], f[3], f[1], f[5], f[4], f[5], f[2]}, ev[3], vec[9], q[4];
      eig3(ev, vec, A);
      mat2quat(q, vec);
      quat_mul(b.iquat, b.iquat, q);
      for (int i = 0; i < 3; ++i) b.inertia[i] = ev[i];
    } else {
      fail(e, "inertial requires diaginertia or fullinertia");
    }
  }
  JointRec parse_joint(const XmlElement* e, const std::string& childclass, const Frame& frame,
                       const std::string& suffix) {
    JointRec j;
    j.name = elem_name(e, suffix);
    if (e->tag == "freejoint") {
      j.type = MRS_JNT_FREE;
      return j;
    }
    const DefaultClass* cls = resolve_class(e, childclass);
    const std::string tag = "joint";
    std::string type;
    if (get_str(e, cls, tag, "type", type)) {
      if (type == "hinge") j.type = MRS_JNT_HINGE;
      else if (type == "slide") j.type = MRS_JNT_SLIDE;
      else if (type == "ball") j.type = MRS_JNT_BALL;
      else if (type == "free") j.type = MRS_JNT_FREE;
      else fail(e, "unknown joint type " + type);
    }
    get_reals(e, cls, tag, "pos", j.pos, 3, true);
    get_reals(e, cls, tag, "axis", j.axis, 3, true);
    double n = norm3(j.axis);
    if (n < kMinVal) fail(e, "joint axis too small");
    for (double& a : j.axis) a /= n;
    // frames rotate the joint axis and position with the body content
    double q[4] = {1, 0, 0, 0};
    frame.apply(j.pos, q);
    rot_vec_quat(j.axis, j.axis, frame.quat);
    if (get_reals(e, cls, tag, "range", j.range, 2, true)) j.range_given = true;
    j.limited = get_tristate(e, cls, tag, "limited");
    get_real(e, cls, tag, "damping", j.damping);
    get_real(e, cls, tag, "stiffness", j.stiffness);
    get_real(e, cls, tag, "armature", j.armature);
    get_real(e, cls, tag, "frictionloss", j.frictionloss);
    get_real(e, cls, tag, "springref", j.springref);
    get_real(e, cls, tag, "ref", j.ref);
    get_real(e, cls, tag, "margin", j.margin);
    if (get_reals(e, cls, tag, "actuatorfrcrange", j.actfrcrange, 2, true)) j.actfrcrange_given = true;
    j.actfrclimited = get_tristate(e, cls, tag, "actuatorfrclimited");
    get_reals(e, cls, tag, "solreflimit", j.solreflimit, 2, true);
    get_reals(e, cls, tag, "solimplimit", j.solimplimit, 5);
    get_reals(e, cls, tag, "solreffriction", j.solreffriction, 2, true);
    get_reals(e, cls, tag, "solimpfriction", j.solimpfriction, 5);
    if (j.type == MRS_JNT_HINGE || j.type == MRS_JNT_BALL) {
      if (opt.degree) {
        for (double& r : j.range) r *= kPi / 180;
        j.ref *= kPi / 180;
        j.springref *= kPi / 180;
      }
    }
    return j;
  }
  GeomRec parse_geom(const XmlElement* e, const std::string& childclass, const Frame& frame,
                     const std::string& suffix) {
    GeomRec g;
    g.name = elem_name(e, suffix);
    const DefaultClass* cls = resolve_class(e, childclass);
    const std::string tag = "geom";
    std::string type = "sphere";
    get_str(e, cls, tag, "type", type);
    if (type == "plane") g.type = MRS_GEOM_PLANE;
    else if (type == "sphere") g.type = MRS_GEOM_SPHERE;
    else if (type == "capsule") g.type = MRS_GEOM_CAPSULE;
    else if (type == "ellipsoid") g.type = MRS_GEOM_ELLIPSOID;
    else if (type == "cylinder") g.type = MRS_GEOM_CYLINDER;
    else if (type == "box") g.type = MRS_GEOM_BOX;
    else if (type == "mesh") g.type = MRS_GEOM_MESH;
    else fail(e, "unsupported geom type '" + type + "'");
    get_reals(e, cls, tag, "size", g.size, 3);
    get_int(e, cls, tag, "contype", g.contype);
    get_int(e, cls, tag, "conaffinity", g.conaffinity);
    get_int(e, cls, tag, "condim", g.condim);
    get_int(e, cls, tag, "group", g.group);
    get_int(e, cls, tag, "priority", g.priority);
    get_reals(e, cls, tag, "friction", g.friction, 3);
    get_real(e, cls, tag, "margin", g.margin);
    get_real(e, cls, tag, "gap", g.gap);
    get_real(e, cls, tag, "solmix", g.solmix);
    get_reals(e, cls, tag, "solref", g.solref, 2, true);
    get_reals(e, cls, tag, "solimp", g.solimp, 5);
    const bool rgba_given = get_reals(e, cls, tag, "rgba", g.rgba, 4, true);
    std::string material;
    if (get_str(e, cls, tag, "material", material)) {
      if (!materials.count(material)) fail(e, "geom references unknown material '" + material + "'");
      g.matid = material_ids[material];
      if (!rgba_given)
        for (int k = 0; k < 4; ++k) g.rgba[k] = materials[material][k];
    }
    get_real(e, cls, tag, "mass", g.mass);
    get_real(e, cls, tag, "density", g.density);
    if (g.condim != 1 && g.condim != 3) fail(e, "only condim 1 and 3 are supported");
    double ft[6];
    if (get_reals(e, cls, tag, "fromto", ft, 6, true)) {
      if (g.type != MRS_GEOM_CAPSULE && g.type != MRS_GEOM_CYLINDER && g.type != MRS_GEOM_BOX &&
          g.type != MRS_GEOM_ELLIPSOID)
        fail(e, "fromto requires capsule, cylinder, box or ellipsoid");
      double d[3] = {ft[3] - ft[0], ft[4] - ft[1], ft[5] - ft[2]};
      double len = norm3(d);
      if (len < kMinVal) fail(e, "fromto points coincide");
      for (int i = 0; i < 3; ++i) g.pos[i] = 0.5 * (ft[i] + ft[i + 3]);
      quat_z2vec(g.quat, d);
      if (g.type == MRS_GEOM_BOX || g.type == MRS_GEOM_ELLIPSOID) {
        g.size[1] = g.size[0];
        g.size[2] = len / 2;
      } else {
        g.size[1] = len / 2;
      }
    } else {
      get_reals(e, cls, tag, "pos", g.pos, 3, true);
      get_orientation(e, cls, tag, g.quat);
    }
    if (g.type == MRS_GEOM_MESH) {
      std::string mesh;
      if (!get_str(e, cls, tag, "mesh", mesh)) fail(e, "mesh geom needs a mesh attribute");
      auto it = mesh_ids.find(mesh);
      if (it == mesh_ids.end()) fail(e, "unknown mesh '" + mesh + "'");
      g.mesh = it->second;
      const MeshRec& r = meshes[g.mesh];
      // geom frame = declared frame o the mesh's inertial frame
      double off[3];
      rot_vec_quat(off, r.pos, g.quat);
      for (int k = 0; k < 3; ++k) g.pos[k] += off[k];
      quat_mul(g.quat, g.quat, r.quat);
      for (int k = 0; k < 3; ++k) g.size[k] = r.half[k];
    }
    frame.apply(g.pos, g.quat);
    return g;
  }
  // <light> [upstream mjCLight]: fixed mode only; pose in the body's frame (the enclosing frames applied)
  LightRec parse_light(const XmlElement* e, const std::string& childclass, const Frame& frame) {
    const DefaultClass* cls = resolve_class(e, childclass);
    const std::string tag = "light";
    LightRec l;
    get_reals(e, cls, tag, "pos", l.pos, 3, true);
    get_reals(e, cls, tag, "dir", l.dir, 3, true);
    get_reals(e, cls, tag, "ambient", l.ambient, 3, true);
    get_reals(e, cls, tag, "diffuse", l.diffuse, 3, true);
    get_reals(e, cls, tag, "specular", l.specular, 3, true);
    get_reals(e, cls, tag, "attenuation", l.attenuation, 3, true);
    get_real(e, cls, tag, "cutoff", l.cutoff);
    get_real(e, cls, tag, "exponent", l.exponent);
    std::string s;
    if (get_str(e, cls, tag, "directional", s)) l.directional = s == "true";
    if (get_str(e, cls, tag, "type", s)) {
      if (s != "directional" && s != "spot") fail(e, "light type '" + s + "' is not supported");
      l.directional = s == "directional";
    }
    if (get_str(e, cls, tag, "castshadow", s)) l.castshadow = s == "true";
    if (get_str(e, cls, tag, "active", s)) l.active = s == "true";
    if (get_str(e, cls, tag, "mode", s) && s != "fixed") fail(e, "light mode '" + s + "' is not supported (fixed only)");
    double n = std::sqrt(l.dir[0] * l.dir[0] + l.dir[1] * l.dir[1] + l.dir[2] * l.dir[2]);
    if (n < 1e-12) fail(e, "light dir is zero");
    for (int i = 0; i < 3; ++i) l.dir[i] /= n;
    double q[4] = {1, 0, 0, 0}, d[3];
    frame.apply(l.pos, q);
    rot_vec_quat(d, l.dir, frame.quat);
    for (int i = 0; i < 3; ++i) l.dir[i] = d[i];
    return l;
  }
  // lights into the model in the world frame (after set0: the bodies' qpos0 poses); a light must be
  // fixed in the world (on the world body or a body welded to it)
  void flatten_lights() {
    size_t nl = 0;
    for (const auto& bd : bodies) nl += bd.lights.size();
    // the fixed-function pipeline the colour image restates has 8 light slots (the headlight aside)
    if (nl > 8) throw std::runtime_error("MJCF error: at most 8 lights are supported");
    for (int b = 0; b < static_cast<int>(bodies.size()); ++b)
      for (const LightRec& l : bodies[b].lights) {
        if (m.body_weldid[b] != 0) throw std::runtime_error("MJCF error: lights on moving bodies are not supported");
        double p[3], d[3];
        rot_vec_quat(p, l.pos, &x0quat[4 * b]);
        for (int i = 0; i < 3; ++i) p[i] += x0pos[3 * b + i];
        rot_vec_quat(d, l.dir, &x0quat[4 * b]);
        m.light_pos.insert(m.light_pos.end(), p, p + 3);
        m.light_dir.insert(m.light_dir.end(), d, d + 3);
        m.light_ambient.insert(m.light_ambient.end(), l.ambient, l.ambient + 3);
        m.light_diffuse.insert(m.light_diffuse.end(), l.diffuse, l.diffuse + 3);
        m.light_specular.insert(m.light_specular.end(), l.specular, l.specular + 3);
        m.light_attenuation.insert(m.light_attenuation.end(), l.attenuation, l.attenuation + 3);
        m.light_cutoff.push_back(l.cutoff);
        m.light_exponent.push_back(l.exponent);
        m.light_directional.push_back(l.directional);
        m.light_castshadow.push_back(l.castshadow);
        m.light_active.push_back(l.active);
      }
  }
  SiteRec parse_site(const XmlElement* e, const std::string& childclass, const Frame& frame,
                     const std::string& suffix) {
    SiteRec s;
    s.name = elem_name(e, suffix);
    const DefaultClass* cls = resolve_class(e, childclass);
    get_reals(e, cls, "site", "pos", s.pos, 3, true);
    get_orientation(e, cls, "site", s.quat);
    frame.apply(s.pos, s.quat);
    return s;
  }
  CamRec parse_camera(const XmlElement* e, const std::string& childclass, const Frame& frame,
                      const std::string& suffix) {
    CamRec c;
    c.name = elem_name(e, suffix);
    const DefaultClass* cls = resolve_class(e, childclass);
    get_reals(e, cls, "camera", "pos", c.pos, 3, true);
    get_orientation(e, cls, "camera", c.quat);
    get_real(e, cls, "camera", "fovy", c.fovy);  // always degrees in MJCF
    std::string mode = "fixed";
    get_str(e, cls, "camera", "mode", mode);
    if (mode != "fixed") fail(e, "only camera mode=\"fixed\" is supported");
    double r[2];
    if (get_reals(e, cls, "camera", "resolution", r, 2, true)) {
      c.res[0] = static_cast<int>(r[0]);
      c.res[1] = static_cast<int>(r[1]);
    }
    frame.apply(c.pos, c.quat);
    return c;
  }

  // ---- actuators
  void parse_actuators(const XmlElement* sec) {
    for (auto& cp : sec->children) {
      const XmlElement* e = cp.get();
      const std::string& tag = e->tag;
      if (tag != "motor" && tag != "position" && tag != "velocity" && tag != "general")
        fail(e, "unsupported actuator type");
      const DefaultClass* cls = resolve_class(e, "");
      std::string joint, tendon;
      int jid, trn = MRS_TRN_JOINT;
      if (get_str(e, cls, tag, "joint", joint)) {
        jid = m.name2id(MRS_OBJ_JOINT, joint);
        if (jid < 0) fail(e, "unknown joint '" + joint + "'");
      } else if (get_str(e, cls, tag, "tendon", tendon)) {
        jid = m.name2id(MRS_OBJ_TENDON, tendon);
        if (jid < 0) fail(e, "unknown tendon '" + tendon + "'");
        trn = MRS_TRN_TENDON;
      } else {
        fail(e, "only joint and tendon transmissions are supported");
        return;
      }
      double gear[6] = {1, 0, 0, 0, 0, 0}, gain[MRS_NGAIN] = {0}, bias[MRS_NBIAS] = {0};
      get_reals(e, cls, tag, "gear", gear, 6);
      double ctrlrange[2] = {0, 0}, forcerange[2] = {0, 0};
      bool has_ctrlrange = get_reals(e, cls, tag, "ctrlrange", ctrlrange, 2, true);
      bool has_forcerange = get_reals(e, cls, tag, "forcerange", forcerange, 2, true);
      int ctrllimited = get_tristate(e, cls, tag, "ctrllimited");
      int forcelimited = get_tristate(e, cls, tag, "forcelimited");
      int gaintype = MRS_GAIN_FIXED, biastype = MRS_BIAS_NONE;
      if (tag == "motor") {
        gain[0] = 1;
      } else if (tag == "position") {
        double kp = 1, kv = 0, dampratio = 0;
        get_real(e, cls, tag, "kp", kp);
        bool has_kv = get_real(e, cls, tag, "kv", kv);
        bool has_dr = get_real(e, cls, tag, "dampratio", dampratio);
        if (has_kv && has_dr && kv != 0 && dampratio != 0) fail(e, "kv and dampratio cannot both be set");
        gain[0] = kp;
        biastype = MRS_BIAS_AFFINE;
        bias[1] = -kp;
        // positive biasprm[2] on a position-like actuator means "dampratio" until set0 converts it
        bias[2] = has_dr && dampratio > 0 ? dampratio : -kv;
      } else if (tag == "velocity") {
        double kv = 1;
        get_real(e, cls, tag, "kv", kv);
        gain[0] = kv;
        biastype = MRS_BIAS_AFFINE;
        bias[2] = -kv;
      } else {  // general
        gain[0] = 1;
        std::string s;
        if (get_str(e, cls, tag, "gaintype", s)) {
          if (s == "fixed") gaintype = MRS_GAIN_FIXED;
          else if (s == "affine") gaintype = MRS_GAIN_AFFINE;
          else fail(e, "unsupported gaintype " + s);
        }
        if (get_str(e, cls, tag, "biastype", s)) {
          if (s == "none") biastype = MRS_BIAS_NONE;
          else if (s == "affine") biastype = MRS_BIAS_AFFINE;
          else fail(e, "unsupported biastype " + s);
        }
        if (get_str(e, cls, tag, "dyntype", s) && s != "none") fail(e, "actuator dynamics are not supported");
        get_reals(e, cls, tag, "gainprm", gain, MRS_NGAIN);
        get_reals(e, cls, tag, "biasprm", bias, MRS_NBIAS);
      }
      auto resolve = [&](int tri, bool given, const double* r) {
        int v = tri == 2 ? (opt.autolimits && given ? 1 : 0) : tri;
        if (v && !(r[0] < r[1])) fail(e, "invalid range on a limited actuator");
        return v;
      };
      if (trn == MRS_TRN_TENDON && m.integrator != MRS_INT_EULER && m.integrator != MRS_INT_RK4 &&
          (biastype == MRS_BIAS_AFFINE || gaintype == MRS_GAIN_AFFINE))
        fail(e, "velocity-dependent actuators on tendons are supported with the Euler and RK4 integrators only");
      m.actuator_trntype.push_back(trn);
      m.actuator_dyntype.push_back(MRS_DYN_NONE);
      m.actuator_gaintype.push_back(gaintype);
      m.actuator_biastype.push_back(biastype);
      m.actuator_trnid.push_back(jid);
      m.actuator_trnid.push_back(-1);
      m.actuator_ctrllimited.push_back(resolve(ctrllimited, has_ctrlrange, ctrlrange));
      m.actuator_forcelimited.push_back(resolve(forcelimited, has_forcerange, forcerange));
      m.actuator_gear.insert(m.actuator_gear.end(), gear, gear + 6);
      m.actuator_gainprm.insert(m.actuator_gainprm.end(), gain, gain + MRS_NGAIN);
      m.actuator_biasprm.insert(m.actuator_biasprm.end(), bias, bias + MRS_NBIAS);
      m.actuator_ctrlrange.insert(m.actuator_ctrlrange.end(), ctrlrange, ctrlrange + 2);
      m.actuator_forcerange.insert(m.actuator_forcerange.end(), forcerange, forcerange + 2);
      m.names[MRS_OBJ_ACTUATOR].push_back(elem_name(e, ""));
      ++m.nu;
    }
  }

  // ---- sensors (with replicate-driven expansion)
  void add_sensor(int type, int objtype, int objid, int dim, const std::string& name, double cutoff) {
    m.sensor_type.push_back(type);
    m.sensor_objtype.push_back(objtype);
    m.sensor_objid.push_back(objid);
    m.sensor_dim.push_back(dim);
    m.sensor_adr.push_back(m.nsensordata);
    m.sensor_cutoff.push_back(cutoff);
    m.names[MRS_OBJ_SENSOR].push_back(name);
    m.nsensordata += dim;
    ++m.nsensor;
  }
  void parse_sensors(const XmlElement* sec) {
    for (auto& cp : sec->children) {
      const XmlElement* e = cp.get();
      const std::string& tag = e->tag;
      const DefaultClass* cls = resolve_class(e, "");
      double cutoff = 0;
      get_real(e, cls, tag, "cutoff", cutoff);
      std::string name = elem_name(e, "");
      int type, objtype, dim;
      std::string objname;
      if (tag == "rangefinder" || tag == "gyro" || tag == "accelerometer" || tag == "force" ||
          tag == "torque") {
        objtype = MRS_OBJ_SITE;
        if (!get_str(e, cls, tag, "site", objname)) fail(e, "sensor requires 'site'");
        type = tag == "rangefinder" ? MRS_SENS_RANGEFINDER
               : tag == "gyro"      ? MRS_SENS_GYRO
               : tag == "accelerometer" ? MRS_SENS_ACCELEROMETER
               : tag == "force"     ? MRS_SENS_FORCE
                                    : MRS_SENS_TORQUE;
        dim = tag == "rangefinder" ? 1 : 3;
      } else if (tag == "jointpos" || tag == "jointvel") {
        objtype = MRS_OBJ_JOINT;
        if (!get_str(e, cls, tag, "joint", objname)) fail(e, "sensor requires 'joint'");
        type = tag == "jointpos" ? MRS_SENS_JOINTPOS : MRS_SENS_JOINTVEL;
        dim = 1;
      } else if (tag == "actuatorfrc") {
        objtype = MRS_OBJ_ACTUATOR;
        if (!get_str(e, cls, tag, "actuator", objname)) fail(e, "sensor requires 'actuator'");
        type = MRS_SENS_ACTUATORFRC;
        dim = 1;
      } else if (tag == "framepos" || tag == "framequat") {
        std::string ot;
        if (!get_str(e, cls, tag, "objtype", ot) || !get_str(e, cls, tag, "objname", objname))
          fail(e, "frame sensor requires objtype and objname");
        if (ot == "site") objtype = MRS_OBJ_SITE;
        else if (ot == "body" || ot == "xbody") objtype = MRS_OBJ_BODY;
        else if (ot == "geom") objtype = MRS_OBJ_GEOM;
        else fail(e, "unsupported frame sensor objtype " + ot);
        type = tag == "framepos" ? MRS_SENS_FRAMEPOS : MRS_SENS_FRAMEQUAT;
        dim = tag == "framepos" ? 3 : 4;
      } else {
        fail(e, "unsupported sensor type");
      }
      int objid = m.name2id(objtype, objname);
      if (objid >= 0) {
        add_sensor(type, objtype, objid, dim, name, cutoff);
        continue;
      }
      // the referenced object was replicated: replicate the sensor with the same suffixes
      auto it = replica_suffixes.find(objname);
      if (it == replica_suffixes.end()) fail(e, "sensor references unknown object '" + objname + "'");
      for (const std::string& sfx : it->second) {
        int rid = m.name2id(objtype, objname + sfx);
        if (rid < 0) fail(e, "replicated object '" + objname + sfx + "' not found");
        add_sensor(type, objtype, rid, dim, name.empty() ? "" : name + sfx, cutoff);
      }
    }
  }

  void parse_keyframes(const XmlElement* sec) {
    for (auto& cp : sec->children) {
      const XmlElement* e = cp.get();
      if (e->tag != "key") fail(e, "unsupported keyframe element");
      std::vector<double> qpos = m.qpos0, qvel(m.nv, 0.0), ctrl(m.nu, 0.0);
      double time = 0;
      if (auto* s = e->attr("time")) time = parse_reals(*s, e, "time").at(0);
      auto fill = [&](const char* key, std::vector<double>& dst) {
        if (auto* s = e->attr(key)) {
          auto v = parse_reals(*s, e, key);
          if (v.size() != dst.size()) fail(e, std::string("keyframe '") + key + "' has wrong size");
          dst = v;
        }
      };
      fill("qpos", qpos);
      fill("qvel", qvel);
      fill("ctrl", ctrl);
      m.key_time.push_back(time);
      m.key_qpos.insert(m.key_qpos.end(), qpos.begin(), qpos.end());
      m.key_qvel.insert(m.key_qvel.end(), qvel.begin(), qvel.end());
      m.key_ctrl.insert(m.key_ctrl.end(), ctrl.begin(), ctrl.end());
      ++m.nkey;
    }
  }

  // ---- includes
  void expand_includes(XmlElement* e, const std::string& basedir, int depth) {
    if (depth > 20) fail(e, "include nesting too deep");
    for (size_t i = 0; i < e->children.size();) {
      XmlElement* c = e->children[i].get();
      if (c->tag != "include") { expand_includes(c, basedir, depth); ++i; continue; }
      auto* f = c->attr("file");
      if (!f) fail(c, "include requires 'file'");
      std::string path = (!f->empty() && (*f)[0] == '/') ? *f : basedir + "/" + *f;
      auto sub = xml_parse(read_file(path), path);
      if (sub->tag != "mujoco") fail(sub.get(), "included file must have a <mujoco> root");
      expand_includes(sub.get(), basedir, depth + 1);
      std::vector<std::unique_ptr<XmlElement>> kids;
      for (auto& k : sub->children) kids.push_back(std::move(k));
      e->children.erase(e->children.begin() + i);
      for (size_t k = 0; k < kids.size(); ++k)
        e->children.insert(e->children.begin() + i + k, std::move(kids[k]));
      i += kids.size();
    }
  }

  // ---- flatten the body tree into the model arrays
  void flatten() {
    m.nbody = static_cast<int>(bodies.size());
    std::vector<std::string> bnames, jnames, gnames, snames, cnames;
    for (int b = 0; b < m.nbody; ++b) {
      BodyRec& B = bodies[b];
      bnames.push_back(B.name);
      m.body_parentid.push_back(b == 0 ? 0 : B.parent);
      int root = b;
      while (root != 0 && bodies[root].parent != 0) root = bodies[root].parent;
      m.body_rootid.push_back(root);
      int depth = 0;
      for (int x = b; x != 0; x = bodies[x].parent) ++depth;
      m.body_depth.push_back(depth);
      m.max_depth = std::max(m.max_depth, depth);
      m.body_pos.insert(m.body_pos.end(), B.pos, B.pos + 3);
      quat_normalize(B.quat);
      m.body_quat.insert(m.body_quat.end(), B.quat, B.quat + 4);
      m.body_gravcomp.push_back(B.gravcomp);
      // joints and dofs
      m.body_jntadr.push_back(B.joints.empty() ? -1 : m.njnt);
      m.body_jntnum.push_back(static_cast<int>(B.joints.size()));
      m.body_dofadr.push_back(-1);
      int ndof_body = 0;
      for (size_t k = 0; k < B.joints.size(); ++k) {
        JointRec& J = B.joints[k];
        if (J.type == MRS_JNT_FREE && (k != 0 || B.parent != 0))
          fail(nullptr, "free joint must be the only joint of a top-level body ('" + B.name + "')");
        int jid = m.njnt++;
        jnames.push_back(J.name);
        m.jnt_type.push_back(J.type);
        m.jnt_qposadr.push_back(m.nq);
        m.jnt_dofadr.push_back(m.nv);
        m.jnt_bodyid.push_back(b);
        int lim = J.limited == 2 ? (opt.autolimits && J.range_given ? 1 : 0) : J.limited;
        if (lim && J.type != MRS_JNT_HINGE && J.type != MRS_JNT_SLIDE)
          fail(nullptr, "limits are supported on hinge/slide joints only ('" + J.name + "')");
        if (lim && !(J.range[0] < J.range[1])) fail(nullptr, "invalid joint range ('" + J.name + "')");
        m.jnt_limited.push_back(lim);
        int afl = J.actfrclimited == 2 ? (opt.autolimits && J.actfrcrange_given ? 1 : 0) : J.actfrclimited;
        m.jnt_actfrclimited.push_back(afl);
        m.jnt_pos.insert(m.jnt_pos.end(), J.pos, J.pos + 3);
        m.jnt_axis.insert(m.jnt_axis.end(), J.axis, J.axis + 3);
        m.jnt_stiffness.push_back(J.stiffness);
        m.jnt_range.insert(m.jnt_range.end(), J.range, J.range + 2);
        m.jnt_actfrcrange.insert(m.jnt_actfrcrange.end(), J.actfrcrange, J.actfrcrange + 2);
        m.jnt_margin.push_back(J.margin);
        m.jnt_solref.insert(m.jnt_solref.end(), J.solreflimit, J.solreflimit + 2);
        m.jnt_solimp.insert(m.jnt_solimp.end(), J.solimplimit, J.solimplimit + 5);
        int nqj = J.type == MRS_JNT_FREE ? 7 : J.type == MRS_JNT_BALL ? 4 : 1;
        int nvj = J.type == MRS_JNT_FREE ? 6 : J.type == MRS_JNT_BALL ? 3 : 1;
        // qpos0 / qpos_spring
        if (J.type == MRS_JNT_FREE) {
          double q[7] = {B.pos[0], B.pos[1], B.pos[2], B.quat[0], B.quat[1], B.quat[2], B.quat[3]};
          m.qpos0.insert(m.qpos0.end(), q, q + 7);
          m.qpos_spring.insert(m.qpos_spring.end(), q, q + 7);
        } else if (J.type == MRS_JNT_BALL) {
          double q[4] = {1, 0, 0, 0};
          m.qpos0.insert(m.qpos0.end(), q, q + 4);
          m.qpos_spring.insert(m.qpos_spring.end(), q, q + 4);
        } else {
          m.qpos0.push_back(J.ref);
          m.qpos_spring.push_back(J.springref);
        }
        if (m.body_dofadr[b] < 0) m.body_dofadr[b] = m.nv;
        for (int d = 0; d < nvj; ++d) {
          m.dof_bodyid.push_back(b);
          m.dof_jntid.push_back(jid);
          m.dof_armature.push_back(J.armature);
          m.dof_damping.push_back(J.damping);
          m.dof_frictionloss.push_back(J.frictionloss);
          m.dof_solref.insert(m.dof_solref.end(), J.solreffriction, J.solreffriction + 2);
          m.dof_solimp.insert(m.dof_solimp.end(), J.solimpfriction, J.solimpfriction + 5);
        }
        m.nq += nqj;
        m.nv += nvj;
        ndof_body += nvj;
      }
      m.body_dofnum.push_back(ndof_body);
      // geoms
      m.body_geomadr.push_back(B.geoms.empty() ? -1 : m.ngeom);
      m.body_geomnum.push_back(static_cast<int>(B.geoms.size()));
      for (GeomRec& G : B.geoms) {
        if (G.type == MRS_GEOM_PLANE && b != 0 && !B.joints.empty())
          fail(nullptr, "plane geoms must be static ('" + G.name + "')");
        gnames.push_back(G.name);
        m.geom_type.push_back(G.type);
        m.geom_contype.push_back(G.contype);
        m.geom_conaffinity.push_back(G.conaffinity);
        m.geom_condim.push_back(G.condim);
        m.geom_bodyid.push_back(b);
        m.geom_group.push_back(G.group);
        m.geom_priority.push_back(G.priority);
        m.geom_size.insert(m.geom_size.end(), G.size, G.size + 3);
        m.geom_pos.insert(m.geom_pos.end(), G.pos, G.pos + 3);
        quat_normalize(G.quat);
        m.geom_quat.insert(m.geom_quat.end(), G.quat, G.quat + 4);
        double rb = 0;
        switch (G.type) {
          case MRS_GEOM_SPHERE: rb = G.size[0]; break;
          case MRS_GEOM_CAPSULE: rb = G.size[0] + G.size[1]; break;
          case MRS_GEOM_CYLINDER: rb = std::sqrt(G.size[0] * G.size[0] + G.size[1] * G.size[1]); break;
          case MRS_GEOM_ELLIPSOID: rb = std::max(G.size[0], std::max(G.size[1], G.size[2])); break;
          case MRS_GEOM_BOX: rb = norm3(G.size); break;
          case MRS_GEOM_MESH: rb = meshes[G.mesh].rbound; break;
          default: rb = 0;
        }
        m.geom_rbound.push_back(rb);
        m.geom_dataid.push_back(G.mesh);
        m.geom_friction.insert(m.geom_friction.end(), G.friction, G.friction + 3);
        m.geom_margin.push_back(G.margin);
        m.geom_gap.push_back(G.gap);
        m.geom_solmix.push_back(G.solmix);
        m.geom_solref.insert(m.geom_solref.end(), G.solref, G.solref + 2);
        m.geom_solimp.insert(m.geom_solimp.end(), G.solimp, G.solimp + 5);
        m.geom_rgba.insert(m.geom_rgba.end(), G.rgba, G.rgba + 4);
        m.geom_matid.push_back(G.matid);
        ++m.ngeom;
      }
      for (SiteRec& S : B.sites) {
        snames.push_back(S.name);
        m.site_bodyid.push_back(b);
        m.site_pos.insert(m.site_pos.end(), S.pos, S.pos + 3);
        quat_normalize(S.quat);
        m.site_quat.insert(m.site_quat.end(), S.quat, S.quat + 4);
        ++m.nsite;
      }
      for (CamRec& C : B.cams) {
        cnames.push_back(C.name);
        m.cam_bodyid.push_back(b);
        m.cam_pos.insert(m.cam_pos.end(), C.pos, C.pos + 3);
        quat_normalize(C.quat);
        m.cam_quat.insert(m.cam_quat.end(), C.quat, C.quat + 4);
        m.cam_fovy.push_back(C.fovy);
        m.cam_resolution.push_back(C.res[0]);
        m.cam_resolution.push_back(C.res[1]);
        ++m.ncam;
      }
    }
    m.names[MRS_OBJ_BODY] = bnames;
    m.names[MRS_OBJ_JOINT] = jnames;
    m.names[MRS_OBJ_GEOM] = gnames;
    m.names[MRS_OBJ_SITE] = snames;
    m.names[MRS_OBJ_CAMERA] = cnames;
    for (auto& kv : m.names) {
      std::set<std::string> seen;
      for (auto& n : kv.second)
        if (!n.empty() && !seen.insert(n).second)
          fail(nullptr, "repeated name '" + n + "'");
    }
    // weld ids: nearest ancestor-or-self with joints (0 = welded to world)
    for (int b = 0; b < m.nbody; ++b) {
      int w = b;
      while (w != 0 && m.body_jntnum[w] == 0) w = m.body_parentid[w];
      m.body_weldid.push_back(w);
    }
    // dof parents: previous dof of the same body, else last dof of nearest ancestor with dofs
    m.dof_parentid.assign(m.nv, -1);
    for (int j = 0; j < m.nv; ++j) {
      int b = m.dof_bodyid[j];
      if (j > m.body_dofadr[b]) { m.dof_parentid[j] = j - 1; continue; }
      for (int p = m.body_parentid[b]; p != 0; p = m.body_parentid[p])
        if (m.body_dofnum[p] > 0) { m.dof_parentid[j] = m.body_dofadr[p] + m.body_dofnum[p] - 1; break; }
    }
    // mass and inertia
    for (int b = 0; b < m.nbody; ++b) {
      BodyRec& B = bodies[b];
      double ipos[3] = {0, 0, 0}, iquat[4] = {1, 0, 0, 0}, inertia[3] = {0, 0, 0}, mass = 0;
      bool from_geom = b != 0 && (opt.inertiafromgeom == 1 || (opt.inertiafromgeom == 2 && !B.has_inertial));
      if (b != 0 && !from_geom) {
        std::memcpy(ipos, B.ipos, sizeof ipos);
        std::memcpy(iquat, B.iquat, sizeof iquat);
        quat_normalize(iquat);
        std::memcpy(inertia, B.inertia, sizeof inertia);
        mass = B.mass;
      } else if (from_geom) {
        geom_inertia(B, mass, ipos, iquat, inertia);
      }
      if (b != 0) {
        // mjCBody::Compile: lower bounds, then the triangle inequality of the principal inertia
        // (balanceinertia replaces a violating triple by its mean, otherwise the model is rejected)
        mass = std::max(mass, opt.boundmass);
        for (double& v : inertia) v = std::max(v, opt.boundinertia);
        const double tol = 1e-12 * (inertia[0] + inertia[1] + inertia[2]);
        if (inertia[0] + inertia[1] < inertia[2] - tol || inertia[0] + inertia[2] < inertia[1] - tol ||
            inertia[1] + inertia[2] < inertia[0] - tol) {
          if (!opt.balanceinertia)
            fail(nullptr, "inertia of body '" + B.name + "' must satisfy A + B >= C; use 'balanceinertia' to fix");
          const double mean = (inertia[0] + inertia[1] + inertia[2]) / 3;
          inertia[0] = inertia[1] = inertia[2] = mean;
        }
      }
      m.body_mass.push_back(mass);
      m.body_ipos.insert(m.body_ipos.end(), ipos, ipos + 3);
      m.body_iquat.insert(m.body_iquat.end(), iquat, iquat + 4);
      m.body_inertia.insert(m.body_inertia.end(), inertia, inertia + 3);
      if (b != 0 && m.body_weldid[b] == b && mass < 1e-10)
        fail(nullptr, "moving body '" + B.name + "' has zero mass");
    }
    if (opt.settotalmass > 0) {
      // scale every body's mass and inertia so that the model's total mass is settotalmass
      double total = 0;
      for (int b = 1; b < m.nbody; ++b) total += m.body_mass[b];
      if (total > kMinVal) {
        const double sc = opt.settotalmass / total;
        for (int b = 1; b < m.nbody; ++b) {
          m.body_mass[b] *= sc;
          for (int i = 0; i < 3; ++i) m.body_inertia[3 * b + i] *= sc;
        }
      }
    }
    m.body_subtreemass = m.body_mass;
    for (int b = m.nbody - 1; b > 0; --b) m.body_subtreemass[m.body_parentid[b]] += m.body_subtreemass[b];
  }

  void geom_mass_inertia(const GeomRec& g, double& mass, double I[3]) const {
    const double* s = g.size;
    double vol = 0;
    I[0] = I[1] = I[2] = 0;
    switch (g.type) {
      case MRS_GEOM_SPHERE: vol = 4.0 / 3 * kPi * s[0] * s[0] * s[0]; break;
      case MRS_GEOM_CAPSULE: vol = 4.0 / 3 * kPi * s[0] * s[0] * s[0] + kPi * s[0] * s[0] * 2 * s[1]; break;
      case MRS_GEOM_CYLINDER: vol = kPi * s[0] * s[0] * 2 * s[1]; break;
      case MRS_GEOM_ELLIPSOID: vol = 4.0 / 3 * kPi * s[0] * s[1] * s[2]; break;
      case MRS_GEOM_BOX: vol = 8 * s[0] * s[1] * s[2]; break;
      case MRS_GEOM_MESH: vol = meshes[g.mesh].volume; break;
      default: vol = 0;
    }
    mass = g.mass >= 0 ? g.mass : g.density * vol;
    if (vol <= 0) return;
    double rho = mass / vol;
    switch (g.type) {
      case MRS_GEOM_SPHERE: I[0] = I[1] = I[2] = 0.4 * mass * s[0] * s[0]; break;
      case MRS_GEOM_CAPSULE: {
        double r = s[0], h = 2 * s[1];
        double ms = rho * 4.0 / 3 * kPi * r * r * r, mc = rho * kPi * r * r * h;
        I[2] = mc * r * r / 2 + ms * 2 * r * r / 5;
        I[0] = I[1] = mc * (3 * r * r + h * h) / 12 + ms * (2 * r * r / 5 + h * h / 4 + 3 * h * r / 8);
        break;
      }
      case MRS_GEOM_CYLINDER: {
        double r = s[0], h = 2 * s[1];
        I[2] = mass * r * r / 2;
        I[0] = I[1] = mass * (3 * r * r + h * h) / 12;
        break;
      }
      case MRS_GEOM_ELLIPSOID:
        I[0] = mass * (s[1] * s[1] + s[2] * s[2]) / 5;
        I[1] = mass * (s[0] * s[0] + s[2] * s[2]) / 5;
        I[2] = mass * (s[0] * s[0] + s[1] * s[1]) / 5;
        break;
      case MRS_GEOM_BOX:
        I[0] = mass * (s[1] * s[1] + s[2] * s[2]) / 3;
        I[1] = mass * (s[0] * s[0] + s[2] * s[2]) / 3;
        I[2] = mass * (s[0] * s[0] + s[1] * s[1]) / 3;
        break;
      case MRS_GEOM_MESH:  // unit-density principal moments scaled by the density
        for (int k = 0; k < 3; ++k) I[k] = rho * meshes[g.mesh].inertia[k];
        break;
      default: break;
    }
  }
  // mesh arrays of the model (after flatten: geoms reference meshes by id)
  void flatten_meshes() {
    m.nmesh = static_cast<int>(meshes.size());
    std::vector<std::string> names;
    for (const MeshRec& r : meshes) {
      names.push_back(r.name);
      m.mesh_vertadr.push_back(static_cast<int>(m.mesh_vert.size() / 3));
      m.mesh_vertnum.push_back(static_cast<int>(r.vert.size() / 3));
      m.mesh_faceadr.push_back(static_cast<int>(m.mesh_face.size() / 3));
      m.mesh_facenum.push_back(static_cast<int>(r.face.size() / 3));
      m.mesh_hulladr.push_back(static_cast<int>(m.mesh_hull.size()));
      m.mesh_hullnum.push_back(static_cast<int>(r.hull.size()));
      m.mesh_vert.insert(m.mesh_vert.end(), r.vert.begin(), r.vert.end());
      m.mesh_face.insert(m.mesh_face.end(), r.face.begin(), r.face.end());
      m.mesh_hull.insert(m.mesh_hull.end(), r.hull.begin(), r.hull.end());
      m.mesh_polyadr.push_back(static_cast<int>(m.mesh_polynum_v.size()));
      m.mesh_polynum.push_back(static_cast<int>(r.poly.size()));
      for (size_t q = 0; q < r.poly.size(); ++q) {
        m.mesh_polyvertadr.push_back(static_cast<int>(m.mesh_polyvert.size()));
        m.mesh_polynum_v.push_back(static_cast<int>(r.poly[q].size()));
        m.mesh_polyvert.insert(m.mesh_polyvert.end(), r.poly[q].begin(), r.poly[q].end());
        for (int k = 0; k < 3; ++k) m.mesh_polynormal.push_back(r.poly_normal[3 * q + k]);
      }
    }
    m.names[MRS_OBJ_MESH] = names;
  }
  void geom_inertia(const BodyRec& B, double& mass, double ipos[3], double iquat[4], double inertia[3]) {
    mass = 0;
    double com[3] = {0, 0, 0};
    std::vector<double> gm;
    auto counts = [&](const GeomRec& g) { return g.group >= opt.inertiagroup[0] && g.group <= opt.inertiagroup[1]; };
    for (auto& g : B.geoms) {
      double I[3], mg;
      geom_mass_inertia(g, mg, I);
      if (!counts(g)) mg = 0;  // inertiagrouprange: geoms of other groups carry no mass
      gm.push_back(mg);
      mass += mg;
      for (int i = 0; i < 3; ++i) com[i] += mg * g.pos[i];
    }
    if (mass <= 0) return;
    for (double& c : com) c /= mass;
    double T[9] = {0};
    for (size_t k = 0; k < B.geoms.size(); ++k) {
      const GeomRec& g = B.geoms[k];
      if (!counts(g)) continue;
      double I[3], mg, R[9];
      geom_mass_inertia(g, mg, I);
      quat2mat(R, g.quat);
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
          double v = 0;
          for (int k2 = 0; k2 < 3; ++k2) v += R[r * 3 + k2] * I[k2] * R[c * 3 + k2];
          T[r * 3 + c] += v;
        }
      double d[3] = {g.pos[0] - com[0], g.pos[1] - com[1], g.pos[2] - com[2]};
      double dd = dot3(d, d);
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) T[r * 3 + c] += mg * ((r == c ? dd : 0) - d[r] * d[c]);
    }
    double ev[3], vec[9];
    eig3(ev, vec, T);
    mat2quat(iquat, vec);
    for (int i = 0; i < 3; ++i) { ipos[i] = com[i]; inertia[i] = ev[i]; }
  }

  // ---- set0: constants that need kinematics at qpos0 (MuJoCo engine_setconst.c, restated)
  void set0() {
    const int nb = m.nbody, nv = m.nv;
    std::vector<double> xpos(3 * nb, 0), xquat(4 * nb, 0), xmat(9 * nb), xipos(3 * nb), ximat(9 * nb);
    std::vector<double> xanchor(3 * std::max(1, m.njnt)), xaxis(3 * std::max(1, m.njnt));
    xquat[0] = 1;
    quat2mat(&xmat[0], &xquat[0]);
    std::memcpy(&ximat[0], &xmat[0], 9 * sizeof(double));
    for (int b = 1; b < nb; ++b) {
      int p = m.body_parentid[b];
      double* pos = &xpos[3 * b];
      double* q = &xquat[4 * b];
      int ja = m.body_jntadr[b];
      if (m.body_jntnum[b] > 0 && m.jnt_type[ja] == MRS_JNT_FREE) {
        int a = m.jnt_qposadr[ja];
        for (int i = 0; i < 3; ++i) pos[i] = m.qpos0[a + i];
        for (int i = 0; i < 4; ++i) q[i] = m.qpos0[a + 3 + i];
        quat_normalize(q);
        for (int i = 0; i < 3; ++i) { xanchor[3 * ja + i] = pos[i]; xaxis[3 * ja + i] = 0; }
      } else {
        double r[3];
        rot_vec_quat(r, &m.body_pos[3 * b], &xquat[4 * p]);
        for (int i = 0; i < 3; ++i) pos[i] = xpos[3 * p + i] + r[i];
        quat_mul(q, &xquat[4 * p], &m.body_quat[4 * b]);
        for (int k = 0; k < m.body_jntnum[b]; ++k) {
          int j = ja + k;
          rot_vec_quat(&xanchor[3 * j], &m.jnt_pos[3 * j], q);
          for (int i = 0; i < 3; ++i) xanchor[3 * j + i] += pos[i];
          rot_vec_quat(&xaxis[3 * j], &m.jnt_axis[3 * j], q);
          // at qpos0 hinge/slide displacement is zero and ball is identity
        }
      }
      quat_normalize(q);
      quat2mat(&xmat[9 * b], q);
      double r[3], iq[4];
      rot_vec_quat(r, &m.body_ipos[3 * b], q);
      for (int i = 0; i < 3; ++i) xipos[3 * b + i] = pos[i] + r[i];
      quat_mul(iq, q, &m.body_iquat[4 * b]);
      quat2mat(&ximat[9 * b], iq);
    }
    x0pos = xpos;
    x0quat = xquat;
    // subtree com
    std::vector<double> scom(3 * nb, 0);
    for (int b = 0; b < nb; ++b)
      for (int i = 0; i < 3; ++i) scom[3 * b + i] = m.body_mass[b] * xipos[3 * b + i];
    for (int b = nb - 1; b > 0; --b)
      for (int i = 0; i < 3; ++i) scom[3 * m.body_parentid[b] + i] += scom[3 * b + i];
    for (int b = 0; b < nb; ++b)
      for (int i = 0; i < 3; ++i)
        scom[3 * b + i] = m.body_subtreemass[b] > kMinVal ? scom[3 * b + i] / m.body_subtreemass[b] : xipos[3 * b + i];
    // cdof
    std::vector<double> cdof(6 * std::max(1, nv), 0);
    for (int j = 0; j < m.njnt; ++j) {
      int b = m.jnt_bodyid[j], d = m.jnt_dofadr[j];
      const double* c = &scom[3 * m.body_rootid[b]];
      double off[3];
      for (int i = 0; i < 3; ++i) off[i] = c[i] - xanchor[3 * j + i];
      auto rot_dof = [&](double* out, const double* ax) {
        out[0] = ax[0]; out[1] = ax[1]; out[2] = ax[2];
        cross3(out + 3, ax, off);
      };
      switch (m.jnt_type[j]) {
        case MRS_JNT_HINGE: rot_dof(&cdof[6 * d], &xaxis[3 * j]); break;
        case MRS_JNT_SLIDE:
          for (int i = 0; i < 3; ++i) { cdof[6 * d + i] = 0; cdof[6 * d + 3 + i] = xaxis[3 * j + i]; }
          break;
        case MRS_JNT_FREE:
          for (int k = 0; k < 3; ++k)
            for (int i = 0; i < 6; ++i) cdof[6 * (d + k) + i] = (i == 3 + k) ? 1 : 0;
          d += 3;
          [[fallthrough]];
        case MRS_JNT_BALL:
          for (int k = 0; k < 3; ++k) {
            double ax[3] = {xmat[9 * b + k], xmat[9 * b + 3 + k], xmat[9 * b + 6 + k]};
            rot_dof(&cdof[6 * (d + k)], ax);
          }
          break;
      }
    }
    // cinert, crb, M
    std::vector<double> crb(10 * nb, 0);
    for (int b = 1; b < nb; ++b) {
      double dif[3];
      for (int i = 0; i < 3; ++i) dif[i] = xipos[3 * b + i] - scom[3 * m.body_rootid[b] + i];
      inert_com(&crb[10 * b], &m.body_inertia[3 * b], &ximat[9 * b], dif, m.body_mass[b]);
    }
    for (int b = nb - 1; b > 0; --b)
      if (m.body_parentid[b] > 0)
        for (int i = 0; i < 10; ++i) crb[10 * m.body_parentid[b] + i] += crb[10 * b + i];
    std::vector<double> M(nv * nv, 0);
    for (int i = 0; i < nv; ++i) {
      double buf[6];
      mul_inert_vec(buf, &crb[10 * m.dof_bodyid[i]], &cdof[6 * i]);
      for (int j = i; j >= 0; j = m.dof_parentid[j]) {
        double v = 0;
        for (int k = 0; k < 6; ++k) v += cdof[6 * j + k] * buf[k];
        M[i * nv + j] = M[j * nv + i] = v;
      }
      M[i * nv + i] += m.dof_armature[i];
    }
    m.dof_M0.resize(nv);
    double trace = 0;
    for (int i = 0; i < nv; ++i) { m.dof_M0[i] = M[i * nv + i]; trace += M[i * nv + i]; }
    m.stat_meaninertia = nv > 0 ? trace / nv : 1;
    // inverse of M (dense Cholesky) for invweight0
    std::vector<double>& Minv = Minv0;
    Minv.assign(nv * nv, 0);
    if (nv > 0) dense_inverse_spd(M, Minv, nv);
    m.dof_invweight0.assign(nv, 0);
    for (int j = 0; j < m.njnt; ++j) {
      int d = m.jnt_dofadr[j];
      switch (m.jnt_type[j]) {
        case MRS_JNT_FREE: {
          double t = (Minv[d * nv + d] + Minv[(d + 1) * nv + d + 1] + Minv[(d + 2) * nv + d + 2]) / 3;
          double r = (Minv[(d + 3) * nv + d + 3] + Minv[(d + 4) * nv + d + 4] + Minv[(d + 5) * nv + d + 5]) / 3;
          for (int k = 0; k < 3; ++k) { m.dof_invweight0[d + k] = t; m.dof_invweight0[d + 3 + k] = r; }
          break;
        }
        case MRS_JNT_BALL: {
          double r = (Minv[d * nv + d] + Minv[(d + 1) * nv + d + 1] + Minv[(d + 2) * nv + d + 2]) / 3;
          for (int k = 0; k < 3; ++k) m.dof_invweight0[d + k] = r;
          break;
        }
        default: m.dof_invweight0[d] = Minv[d * nv + d];
      }
    }
    // body_invweight0: mean diagonal of J M^-1 J' (translation, rotation) at the body com
    m.body_invweight0.assign(2 * nb, 0);
    for (int b = 1; b < nb; ++b) {
      if (m.body_weldid[b] == 0) continue;
      std::vector<double> J(6 * nv, 0);  // rows 0-2 translation, 3-5 rotation
      for (int j = nv - 1; j >= 0; --j) {
        // dof j affects body b if dof j's body is b or an ancestor of b
        bool affects = false;
        for (int x = b; x != 0; x = m.body_parentid[x])
          if (x == m.dof_bodyid[j]) { affects = true; break; }
        if (!affects) continue;
        double off[3];
        for (int i = 0; i < 3; ++i) off[i] = xipos[3 * b + i] - scom[3 * m.body_rootid[b] + i];
        double cr[3];
        cross3(cr, &cdof[6 * j], off);
        for (int i = 0; i < 3; ++i) {
          J[i * nv + j] = cdof[6 * j + 3 + i] + cr[i];
          J[(3 + i) * nv + j] = cdof[6 * j + i];
        }
      }
      double A[6] = {0};
      for (int r = 0; r < 6; ++r)
        for (int a = 0; a < nv; ++a)
          for (int c = 0; c < nv; ++c) A[r] += J[r * nv + a] * Minv[a * nv + c] * J[r * nv + c];
      double t = (A[0] + A[1] + A[2]) / 3, r = (A[3] + A[4] + A[5]) / 3;
      // a body that can only translate or only rotate borrows the other weight
      if (t < kMinVal) t = r;
      if (r < kMinVal) r = t;
      m.body_invweight0[2 * b] = t;
      m.body_invweight0[2 * b + 1] = r;
    }
    // statistic: extent/center when not given (bounding box of body and geom positions at qpos0)
    if (!extent_given) {
      double lo[3] = {1e30, 1e30, 1e30}, hi[3] = {-1e30, -1e30, -1e30};
      auto grow = [&](const double* p, double r) {
        for (int i = 0; i < 3; ++i) { lo[i] = std::min(lo[i], p[i] - r); hi[i] = std::max(hi[i], p[i] + r); }
      };
      for (int b = 1; b < nb; ++b) grow(&xipos[3 * b], 0);
      for (int g = 0; g < m.ngeom; ++g) {
        if (m.geom_type[g] == MRS_GEOM_PLANE) continue;
        int b = m.geom_bodyid[g];
        double r[3], p[3];
        rot_vec_quat(r, &m.geom_pos[3 * g], &xquat[4 * b]);
        for (int i = 0; i < 3; ++i) p[i] = xpos[3 * b + i] + r[i];
        grow(p, m.geom_rbound[g]);
      }
      if (lo[0] > hi[0]) { m.stat_extent = 1; }
      else {
        double d = 0;
        for (int i = 0; i < 3; ++i) {
          m.stat_center[i] = 0.5 * (lo[i] + hi[i]);
          d = std::max(d, hi[i] - lo[i]);
        }
        m.stat_extent = d > kMinVal ? d : 1;
      }
    }
  }

  static void inert_com(double res[10], const double inert[3], const double mat[9], const double dif[3],
                        double mass) {
    double full[9];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        double v = 0;
        for (int k = 0; k < 3; ++k) v += mat[r * 3 + k] * inert[k] * mat[c * 3 + k];
        full[r * 3 + c] = v;
      }
    res[0] = full[0] + mass * (dif[1] * dif[1] + dif[2] * dif[2]);
    res[1] = full[4] + mass * (dif[0] * dif[0] + dif[2] * dif[2]);
    res[2] = full[8] + mass * (dif[0] * dif[0] + dif[1] * dif[1]);
    res[3] = full[1] - mass * dif[0] * dif[1];
    res[4] = full[2] - mass * dif[0] * dif[2];
    res[5] = full[5] - mass * dif[1] * dif[2];
    res[6] = mass * dif[0]; res[7] = mass * dif[1]; res[8] = mass * dif[2];
    res[9] = mass;
  }
  static void mul_inert_vec(double r[6], const double i[10], const double v[6]) {
    r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
    r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
    r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
    r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
    r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
    r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
  }
  static void dense_inverse_spd(const std::vector<double>& A, std::vector<double>& inv, int n) {
    std::vector<double> L(n * n, 0);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j <= i; ++j) {
        double s = A[i * n + j];
        for (int k = 0; k < j; ++k) s -= L[i * n + k] * L[j * n + k];
        if (i == j) {
          if (s <= 0) throw std::runtime_error("MJCF error: mass matrix at qpos0 is not positive definite");
          L[i * n + i] = std::sqrt(s);
        } else {
          L[i * n + j] = s / L[j * n + j];
        }
      }
    for (int c = 0; c < n; ++c) {
      std::vector<double> y(n, 0);
      for (int i = 0; i < n; ++i) {
        double s = (i == c) ? 1 : 0;
        for (int k = 0; k < i; ++k) s -= L[i * n + k] * y[k];
        y[i] = s / L[i * n + i];
      }
      for (int i = n - 1; i >= 0; --i) {
        double s = y[i];
        for (int k = i + 1; k < n; ++k) s -= L[k * n + i] * inv[k * n + c];
        inv[i * n + c] = s / L[i * n + i];
      }
    }
  }

  // ---- driver
  Model compile(std::unique_ptr<XmlElement> root, const std::string& base) {
    basedir = base;
    if (root->tag != "mujoco") fail(root.get(), "root element must be <mujoco>");
    if (auto* n = root->attr("model")) m.model_name = *n;
    expand_includes(root.get(), basedir, 0);
    // pass 1: compiler, option, defaults, statistic, visual (order-independent in MJCF)
    for (auto& c : root->children) {
      if (c->tag == "compiler") parse_compiler(c.get());
    }
    for (auto& c : root->children) {
      if (c->tag == "option") parse_option(c.get());
      else if (c->tag == "default") parse_default(c.get(), nullptr);
      else if (c->tag == "statistic") {
        if (auto* s = c->attr("extent")) { m.stat_extent = parse_reals(*s, c.get(), "extent").at(0); extent_given = true; }
        if (c->attr("center")) get_reals(c.get(), nullptr, "statistic", "center", m.stat_center, 3, true);
      } else if (c->tag == "visual") {
        for (auto& v : c->children)
          if (v->tag == "map") {
            if (auto* s = v->attr("znear")) m.vis_znear = parse_reals(*s, v.get(), "znear").at(0);
            if (auto* s = v->attr("zfar")) m.vis_zfar = parse_reals(*s, v.get(), "zfar").at(0);
          } else if (v->tag == "headlight") {
            get_reals(v.get(), nullptr, "headlight", "ambient", m.vis_headlight, 3, true);
            get_reals(v.get(), nullptr, "headlight", "diffuse", m.vis_headlight + 3, 3, true);
            get_reals(v.get(), nullptr, "headlight", "specular", m.vis_headlight + 6, 3, true);
            std::string a;
            if (get_str(v.get(), nullptr, "headlight", "active", a)) m.vis_headlight[9] = a == "0" || a == "false" ? 0 : 1;
          }
      }
    }
    for (auto& c : root->children)
      if (c->tag == "asset") parse_asset(c.get());
    // pass 2: world body tree
    BodyRec world;
    world.name = "world";
    bodies.push_back(world);
    for (auto& c : root->children)
      if (c->tag == "worldbody") parse_body_children(c.get(), 0, "", Frame(), "");
    flatten();
    flatten_meshes();
    set0();
    flatten_lights();
    // pass 3: elements that reference the tree
    for (auto& c : root->children)
      if (c->tag == "tendon") parse_tendons(c.get());
    for (auto& c : root->children) {
      if (c->tag == "actuator") parse_actuators(c.get());
    }
    set0_actuators();
    for (auto& c : root->children) {
      if (c->tag == "sensor") parse_sensors(c.get());
      else if (c->tag == "keyframe") parse_keyframes(c.get());
      else if (c->tag == "equality") parse_equality(c.get());
      else if (c->tag == "contact") parse_contact(c.get());
    }
    candidate_pairs();
    return std::move(m);
  }
  std::vector<double> x0pos, x0quat;  // body poses at qpos0 (set0)
  std::vector<double> Minv0;          // M(qpos0)^-1, dense (set0)
  // <tendon><fixed> [upstream mjCTendon, fixed only]: wraps of hinge / slide joints with coefficients;
  // limited (autolimits: a range given), range, margin, solreflimit / solimplimit, frictionloss,
  // solreffriction / solimpfriction, stiffness, damping, springlength (one value, two for a dead band;
  // -1: the length at qpos_spring), tendon_invweight0 = J M(qpos0)^-1 J' [upstream mj_setConst]
  void parse_tendons(const XmlElement* sec) {
    const int nv = m.nv;
    for (auto& cp : sec->children) {
      const XmlElement* e = cp.get();
      const std::string& tag = e->tag;
      if (tag == "spatial") fail(e, "spatial tendons are not supported");
      if (tag != "fixed") fail(e, "unsupported tendon type '" + tag + "'");
      const DefaultClass* cls = resolve_class(e, "");
      double range[2] = {0, 0}, margin = 0, srl[2] = {0.02, 1}, sil[5] = {0.9, 0.95, 0.001, 0.5, 2};
      double fl = 0, srf[2] = {0.02, 1}, sif[5] = {0.9, 0.95, 0.001, 0.5, 2}, k = 0, b = 0, ls[2] = {-1, -1};
      const bool has_range = get_reals(e, cls, "tendon", "range", range, 2, true);
      get_real(e, cls, "tendon", "margin", margin);
      get_reals(e, cls, "tendon", "solreflimit", srl, 2, true);
      get_reals(e, cls, "tendon", "solimplimit", sil, 5);
      get_real(e, cls, "tendon", "frictionloss", fl);
      get_reals(e, cls, "tendon", "solreffriction", srf, 2, true);
      get_reals(e, cls, "tendon", "solimpfriction", sif, 5);
      get_real(e, cls, "tendon", "stiffness", k);
      get_real(e, cls, "tendon", "damping", b);
      double arm = 0;
      if (get_real(e, cls, "tendon", "armature", arm) && arm != 0) fail(e, "tendon armature is not supported");
      int nls = 0;
      {
        std::string sl;
        if (get_str(e, cls, "tendon", "springlength", sl)) {
          const auto v = parse_reals(sl, e, "springlength");
          if (v.empty() || v.size() > 2) fail(e, "springlength takes one or two numbers");
          nls = static_cast<int>(v.size());
          for (int i = 0; i < nls; ++i) ls[i] = v[i];
          if (nls == 2 && ls[1] == -1 && ls[0] != -1) nls = 1;
        }
      }
      int lim = get_tristate(e, cls, "tendon", "limited");
      lim = lim == 2 ? (opt.autolimits && has_range ? 1 : 0) : lim;
      if (lim && !(range[0] < range[1])) fail(e, "invalid range on a limited tendon");
      if (b != 0 && m.integrator != MRS_INT_EULER && m.integrator != MRS_INT_RK4)
        fail(e, "tendon damping is supported with the Euler and RK4 integrators only");
      const int adr = static_cast<int>(m.wrap_objid.size());
      double len_spring = 0, len0 = 0;
      std::vector<double> J(nv, 0.0);
      for (auto& wp : e->children) {
        const XmlElement* w = wp.get();
        if (w->tag != "joint") fail(w, "fixed tendons wrap joints only");
        std::string jn;
        if (!get_str(w, nullptr, "joint", "joint", jn)) fail(w, "tendon joint requires 'joint'");
        const int j = m.name2id(MRS_OBJ_JOINT, jn);
        if (j < 0) fail(w, "unknown joint '" + jn + "'");
        if (m.jnt_type[j] != MRS_JNT_HINGE && m.jnt_type[j] != MRS_JNT_SLIDE)
          fail(w, "fixed tendons need hinge or slide joints");
        double coef = 0;
        if (!get_real(w, nullptr, "joint", "coef", coef)) fail(w, "tendon joint requires 'coef'");
        m.wrap_objid.push_back(j);
        m.wrap_prm.push_back(coef);
        len_spring += coef * m.qpos_spring[m.jnt_qposadr[j]];
        len0 += coef * m.qpos0[m.jnt_qposadr[j]];
        J[m.jnt_dofadr[j]] += coef;
      }
      const int num = static_cast<int>(m.wrap_objid.size()) - adr;
      if (num == 0) fail(e, "a fixed tendon needs at least one joint");
      if (nls == 0 || ls[0] == -1) ls[0] = ls[1] = len_spring;
      else if (nls == 1) ls[1] = ls[0];
      if (ls[0] > ls[1]) fail(e, "springlength dead band must be non-decreasing");
      double iw = 0;
      for (int i = 0; i < nv; ++i)
        for (int jj = 0; jj < nv; ++jj) iw += J[i] * Minv0[i * nv + jj] * J[jj];
      m.tendon_adr.push_back(adr);
      m.tendon_num.push_back(num);
      m.tendon_limited.push_back(lim);
      m.tendon_range.insert(m.tendon_range.end(), range, range + 2);
      m.tendon_margin.push_back(margin);
      m.tendon_solref_lim.insert(m.tendon_solref_lim.end(), srl, srl + 2);
      m.tendon_solimp_lim.insert(m.tendon_solimp_lim.end(), sil, sil + 5);
      m.tendon_frictionloss.push_back(fl);
      m.tendon_solref_fri.insert(m.tendon_solref_fri.end(), srf, srf + 2);
      m.tendon_solimp_fri.insert(m.tendon_solimp_fri.end(), sif, sif + 5);
      m.tendon_stiffness.push_back(k);
      m.tendon_damping.push_back(b);
      m.tendon_lengthspring.insert(m.tendon_lengthspring.end(), ls, ls + 2);
      m.tendon_invweight0.push_back(iw);
      m.tendon_length0.push_back(len0);
      m.names[MRS_OBJ_TENDON].push_back(elem_name(e, ""));
    }
  }
  // <equality> [upstream mjCEquality]: connect, weld and joint constraints with solref / solimp /
  // active (defaults 0.02 1 / 0.9 0.95 0.001 0.5 2 / true); what MuJoCo's compiler completes at qpos0
  // is completed here: connect's anchor in body2's frame, weld's relpose when not given (its quaternion
  // all zeros), the joints' reference positions (eq_data layout: include/mrs_model.h)
  void parse_equality(const XmlElement* sec) {
    for (auto& cp : sec->children) {
      const XmlElement* e = cp.get();
      const std::string& tag = e->tag;
      const DefaultClass* cls = resolve_class(e, "");
      double sr[2] = {0.02, 1}, si[5] = {0.9, 0.95, 0.001, 0.5, 2}, data[MRS_NEQDATA] = {};
      get_reals(e, cls, "equality", "solref", sr, 2, true);
      get_reals(e, cls, "equality", "solimp", si, 5);
      get_reals(e, cls, tag, "solref", sr, 2, true);
      get_reals(e, cls, tag, "solimp", si, 5);
      int active = 1;
      std::string a;
      if (get_str(e, cls, tag, "active", a) || get_str(e, cls, "equality", "active", a)) active = a == "true";
      int type, o1, o2;
      auto body = [&](const char* key, bool required) {
        std::string n;
        if (!get_str(e, cls, tag, key, n)) {
          if (required) fail(e, std::string(tag) + " requires " + key);
          return 0;  // world
        }
        const int b = m.name2id(MRS_OBJ_BODY, n);
        if (b < 0) fail(e, "unknown body '" + n + "'");
        return b;
      };
      auto pose_of = [&](int b, double p[3], double q[4]) {
        for (int i = 0; i < 3; ++i) p[i] = x0pos[3 * b + i];
        for (int i = 0; i < 4; ++i) q[i] = x0quat[4 * b + i];
      };
      if (tag == "connect") {
        type = MRS_EQ_CONNECT;
        o1 = body("body1", true);
        o2 = body("body2", false);
        if (!get_reals(e, cls, tag, "anchor", data, 3, true)) fail(e, "connect requires anchor");
        // the same world point in body2's frame at qpos0
        double p1[3], q1[4], p2[3], q2[4], w[3], r[3], qc[4];
        pose_of(o1, p1, q1);
        pose_of(o2, p2, q2);
        rot_vec_quat(r, data, q1);
        for (int i = 0; i < 3; ++i) w[i] = p1[i] + r[i] - p2[i];
        qc[0] = q2[0]; qc[1] = -q2[1]; qc[2] = -q2[2]; qc[3] = -q2[3];
        rot_vec_quat(data + 3, w, qc);
      } else if (tag == "weld") {
        type = MRS_EQ_WELD;
        o1 = body("body1", true);
        o2 = body("body2", false);
        get_reals(e, cls, tag, "anchor", data, 3, true);
        double rp[7] = {0, 1, 0, 0, 0, 0, 0};  // MuJoCo's default: quaternion zero = from qpos0
        get_reals(e, cls, tag, "relpose", rp, 7, true);
        data[10] = 1;
        get_real(e, cls, tag, "torquescale", data[10]);
        if (rp[3] == 0 && rp[4] == 0 && rp[5] == 0 && rp[6] == 0) {
          // body2's pose in body1's frame at qpos0
          double p1[3], q1[4], p2[3], q2[4], d[3], qc[4];
          pose_of(o1, p1, q1);
          pose_of(o2, p2, q2);
          for (int i = 0; i < 3; ++i) d[i] = p2[i] - p1[i];
          qc[0] = q1[0]; qc[1] = -q1[1]; qc[2] = -q1[2]; qc[3] = -q1[3];
          rot_vec_quat(rp, d, qc);
          quat_mul(rp + 3, qc, q2);
        }
        for (int i = 0; i < 7; ++i) data[3 + i] = rp[i];
        quat_normalize(data + 6);
      } else if (tag == "joint") {
        type = MRS_EQ_JOINT;
        std::string n1, n2;
        if (!get_str(e, cls, tag, "joint1", n1)) fail(e, "joint equality requires joint1");
        o1 = m.name2id(MRS_OBJ_JOINT, n1);
        o2 = -1;
        if (get_str(e, cls, tag, "joint2", n2)) o2 = m.name2id(MRS_OBJ_JOINT, n2);
        if (o1 < 0 || (!n2.empty() && o2 < 0)) fail(e, "joint equality references an unknown joint");
        double pc[5] = {0, 1, 0, 0, 0};
        get_reals(e, cls, tag, "polycoef", pc, 5);
        for (int k : {o1, o2}) {
          if (k < 0) continue;
          if (m.jnt_type[k] != MRS_JNT_HINGE && m.jnt_type[k] != MRS_JNT_SLIDE)
            fail(e, "joint equality needs hinge or slide joints");
        }
        for (int i = 0; i < 5; ++i) data[i] = pc[i];
        data[5] = m.qpos0[m.jnt_qposadr[o1]];
        data[6] = o2 >= 0 ? m.qpos0[m.jnt_qposadr[o2]] : 0;
      } else {
        fail(e, "unsupported equality type '" + tag + "'");
        return;
      }
      if ((type == MRS_EQ_CONNECT || type == MRS_EQ_WELD) && o1 == o2) fail(e, "equality of a body with itself");
      m.eq_type.push_back(type);
      m.eq_obj1id.push_back(o1);
      m.eq_obj2id.push_back(o2);
      m.eq_active0.push_back(active);
      m.eq_solref.insert(m.eq_solref.end(), sr, sr + 2);
      m.eq_solimp.insert(m.eq_solimp.end(), si, si + 5);
      m.eq_data.insert(m.eq_data.end(), data, data + MRS_NEQDATA);
    }
  }
  // <contact>: explicit geom pairs and excluded body pairs [upstream mjCPair / mjCBodyPair].  A pair's
  // omitted attributes take the values a candidate pair of its geoms would (max condim and friction,
  // solmix-weighted solref / solimp, max margin and gap); friction has MuJoCo's 5 components, of which
  // the pyramidal / elliptic rows use the sliding one (both sliding values must agree).
  void parse_contact(const XmlElement* sec) {
    for (auto& cp : sec->children) {
      const XmlElement* e = cp.get();
      const DefaultClass* cls = resolve_class(e, "");
      if (e->tag == "exclude") {
        std::string n1, n2;
        if (!get_str(e, cls, "exclude", "body1", n1) || !get_str(e, cls, "exclude", "body2", n2))
          fail(e, "exclude requires body1 and body2");
        const int b1 = m.name2id(MRS_OBJ_BODY, n1), b2 = m.name2id(MRS_OBJ_BODY, n2);
        if (b1 < 0 || b2 < 0) fail(e, "exclude references an unknown body");
        m.exclude_body1.push_back(std::min(b1, b2));
        m.exclude_body2.push_back(std::max(b1, b2));
      } else if (e->tag == "pair") {
        std::string n1, n2;
        if (!get_str(e, cls, "pair", "geom1", n1) || !get_str(e, cls, "pair", "geom2", n2))
          fail(e, "pair requires geom1 and geom2");
        int g1 = m.name2id(MRS_OBJ_GEOM, n1), g2 = m.name2id(MRS_OBJ_GEOM, n2);
        if (g1 < 0 || g2 < 0) fail(e, "pair references an unknown geom");
        if (g1 == g2) fail(e, "pair of a geom with itself");
        if (m.geom_type[g1] > m.geom_type[g2]) std::swap(g1, g2);
        // the candidate-pair mixing of the two geoms, then the pair's own attributes on top
        double s1 = m.geom_solmix[g1], s2 = m.geom_solmix[g2], mix;
        if (s1 >= 1e-15 && s2 >= 1e-15) mix = s1 / (s1 + s2);
        else if (s1 < 1e-15 && s2 < 1e-15) mix = 0.5;
        else mix = s1 < 1e-15 ? 0 : 1;
        int dim = std::max(m.geom_condim[g1], m.geom_condim[g2]);
        double fr[5], sr[2], si[5], mg = std::max(m.geom_margin[g1], m.geom_margin[g2]);
        double gp = std::max(m.geom_gap[g1], m.geom_gap[g2]);
        const double f3[3] = {std::max(m.geom_friction[3 * g1], m.geom_friction[3 * g2]),
                              std::max(m.geom_friction[3 * g1 + 1], m.geom_friction[3 * g2 + 1]),
                              std::max(m.geom_friction[3 * g1 + 2], m.geom_friction[3 * g2 + 2])};
        fr[0] = fr[1] = f3[0]; fr[2] = f3[1]; fr[3] = fr[4] = f3[2];
        for (int i = 0; i < 2; ++i) sr[i] = mix * m.geom_solref[2 * g1 + i] + (1 - mix) * m.geom_solref[2 * g2 + i];
        for (int i = 0; i < 5; ++i) si[i] = mix * m.geom_solimp[5 * g1 + i] + (1 - mix) * m.geom_solimp[5 * g2 + i];
        get_int(e, cls, "pair", "condim", dim);
        if (dim != 1 && dim != 3) fail(e, "only condim 1 and 3 are supported");
        get_reals(e, cls, "pair", "friction", fr, 5);
        if (fr[0] != fr[1]) fail(e, "anisotropic pair friction (sliding1 != sliding2) is not supported");
        get_reals(e, cls, "pair", "solref", sr, 2, true);
        get_reals(e, cls, "pair", "solimp", si, 5);
        double srf[2] = {0, 0};
        if (get_reals(e, cls, "pair", "solreffriction", srf, 2, true) && (srf[0] != 0 || srf[1] != 0))
          fail(e, "pair solreffriction is not supported");
        get_real(e, cls, "pair", "margin", mg);
        get_real(e, cls, "pair", "gap", gp);
        m.expair_geom1.push_back(g1);
        m.expair_geom2.push_back(g2);
        m.expair_dim.push_back(dim);
        m.expair_friction.insert(m.expair_friction.end(), fr, fr + 5);
        m.expair_solref.insert(m.expair_solref.end(), sr, sr + 2);
        m.expair_solimp.insert(m.expair_solimp.end(), si, si + 5);
        m.expair_margin.push_back(mg);
        m.expair_gap.push_back(gp);
      } else {
        fail(e, "unsupported contact element");
      }
    }
  }
  // Static part of mj_collision's broad phase [upstream engine_collision_driver.c mj_collideGeoms /
  // filterBitmask]: geom pairs of different weld groups, not parent-child welds (unless the
  // filterparent flag is disabled; the world body is never filtered), with contype/conaffinity
  // compatible in either direction.  The dynamic bounding-sphere test stays per step.  Each pair is
  // ordered with the lower geom type first (the narrow phase's convention).
  void candidate_pairs() {
    m.pair_geom1.clear();
    m.pair_geom2.clear();
    if (m.disableflags & (MRS_DSBL_CONTACT | MRS_DSBL_CONSTRAINT)) {
      m.expair_geom1.clear(); m.expair_geom2.clear(); m.expair_dim.clear(); m.expair_friction.clear();
      m.expair_solref.clear(); m.expair_solimp.clear(); m.expair_margin.clear(); m.expair_gap.clear();
      return;
    }
    for (int g1 = 0; g1 < m.ngeom; ++g1)
      for (int g2 = g1 + 1; g2 < m.ngeom; ++g2) {
        const int b1 = m.geom_bodyid[g1], b2 = m.geom_bodyid[g2];
        const int w1 = m.body_weldid[b1], w2 = m.body_weldid[b2];
        if (w1 == w2) continue;
        if (!(m.disableflags & MRS_DSBL_FILTERPARENT) && w1 != 0 && w2 != 0 &&
            (w1 == m.body_weldid[m.body_parentid[w2]] || w2 == m.body_weldid[m.body_parentid[w1]]))
          continue;
        if (!((m.geom_contype[g1] & m.geom_conaffinity[g2]) || (m.geom_contype[g2] & m.geom_conaffinity[g1])))
          continue;
        // body pairs excluded (mjModel exclude signatures), or this very geom pair given explicitly:
        // mj_collision merges the dynamic pairs of a body pair with the explicit pairs of the same body
        // signature by skipping only the geom pairs the explicit list holds (mj_collideGeoms' merge
        // test over the signature's pair range) -- the bodies' other geoms still collide dynamically
        // [upstream engine_collision_driver.c; verify]
        const int lo = std::min(b1, b2), hi = std::max(b1, b2);
        bool skip = false;
        for (size_t k = 0; k < m.exclude_body1.size() && !skip; ++k)
          skip = m.exclude_body1[k] == lo && m.exclude_body2[k] == hi;
        for (size_t k = 0; k < m.expair_geom1.size() && !skip; ++k) {
          const int e1 = m.expair_geom1[k], e2 = m.expair_geom2[k];
          skip = (e1 == g1 && e2 == g2) || (e1 == g2 && e2 == g1);
        }
        if (skip) continue;
        const bool swap = m.geom_type[g1] > m.geom_type[g2];
        m.pair_geom1.push_back(swap ? g2 : g1);
        m.pair_geom2.push_back(swap ? g1 : g2);
      }
  }
  // dampratio -> kv for position-like actuators: kv = dampratio * 2 * sqrt(kp * mass) with
  // mass = sum over transmitted dofs of dof_M0 / moment^2  [upstream engine_setconst.c; verify].
  // Runs after set0() because it needs dof_M0.
  void set0_actuators() {
    for (int a = 0; a < m.nu; ++a) {
      double* gain = &m.actuator_gainprm[a * MRS_NGAIN];
      double* bias = &m.actuator_biasprm[a * MRS_NBIAS];
      if (m.actuator_biastype[a] != MRS_BIAS_AFFINE) continue;
      if (gain[0] != -bias[1] || bias[2] <= 0) continue;
      int j = m.actuator_trnid[2 * a];
      double gear = m.actuator_gear[6 * a];
      double mass = 0;
      if (m.actuator_trntype[a] == MRS_TRN_TENDON) {
        // moment gear * coef on each wrapped dof
        for (int k = m.tendon_adr[j]; k < m.tendon_adr[j] + m.tendon_num[j]; ++k) {
          const double mo = gear * m.wrap_prm[k];
          if (mo != 0) mass += m.dof_M0[m.jnt_dofadr[m.wrap_objid[k]]] / (mo * mo);
        }
      } else {
        int d = m.jnt_dofadr[j];
        if ((m.jnt_type[j] == MRS_JNT_HINGE || m.jnt_type[j] == MRS_JNT_SLIDE) && gear != 0)
          mass = m.dof_M0[d] / (gear * gear);
      }
      bias[2] = -bias[2] * 2 * std::sqrt(gain[0] * mass);
    }
  }
};

std::string dirname_of(const std::string& path) {
  auto p = path.find_last_of('/');
  return p == std::string::npos ? "." : path.substr(0, p);
}

}  // namespace

int Model::name2id(int objtype, const std::string& name) const {
  auto it = names.find(objtype);
  if (it == names.end() || name.empty()) return -1;
  for (size_t i = 0; i < it->second.size(); ++i)
    if (it->second[i] == name) return static_cast<int>(i);
  return -1;
}

const char* Model::id2name(int objtype, int id) const {
  auto it = names.find(objtype);
  if (it == names.end() || id < 0 || id >= static_cast<int>(it->second.size())) return nullptr;
  const std::string& s = it->second[id];
  return s.empty() ? nullptr : s.c_str();
}

mrs_model_view Model::view() const {
  mrs_model_view v;
  std::memset(&v, 0, sizeof v);
  v.nq = nq; v.nv = nv; v.nu = nu; v.na = na; v.nbody = nbody; v.njnt = njnt; v.ngeom = ngeom;
  v.nsite = nsite; v.ncam = ncam; v.nsensor = nsensor; v.nsensordata = nsensordata; v.nkey = nkey;
  v.nM = nv * nv; v.max_depth = max_depth; v.npair = static_cast<int>(pair_geom1.size());
  v.timestep = timestep;
  for (int i = 0; i < 3; ++i) { v.gravity[i] = gravity[i]; v.stat_center[i] = stat_center[i]; }
  v.tolerance = tolerance; v.impratio = impratio; v.integrator = integrator; v.solver = solver;
  v.iterations = iterations; v.disableflags = disableflags; v.cone = cone;
  v.ls_tolerance = ls_tolerance; v.ls_iterations = ls_iterations; v.restate = restate;
  v.stat_extent = stat_extent; v.stat_meaninertia = stat_meaninertia;
  v.vis_znear = vis_znear; v.vis_zfar = vis_zfar;
#define MRS_V(f) v.f = f.empty() ? nullptr : f.data()
  MRS_V(body_parentid); MRS_V(body_rootid); MRS_V(body_weldid); MRS_V(body_jntnum);
  MRS_V(body_jntadr); MRS_V(body_dofnum); MRS_V(body_dofadr); MRS_V(body_geomnum);
  MRS_V(body_geomadr); MRS_V(body_depth); MRS_V(body_pos); MRS_V(body_quat); MRS_V(body_ipos);
  MRS_V(body_iquat); MRS_V(body_mass); MRS_V(body_subtreemass); MRS_V(body_inertia);
  MRS_V(body_invweight0); MRS_V(body_gravcomp);
  MRS_V(jnt_type); MRS_V(jnt_qposadr); MRS_V(jnt_dofadr); MRS_V(jnt_bodyid); MRS_V(jnt_limited);
  MRS_V(jnt_actfrclimited); MRS_V(jnt_pos); MRS_V(jnt_axis); MRS_V(jnt_stiffness); MRS_V(jnt_range);
  MRS_V(jnt_actfrcrange); MRS_V(jnt_margin); MRS_V(jnt_solref); MRS_V(jnt_solimp);
  MRS_V(dof_bodyid); MRS_V(dof_jntid); MRS_V(dof_parentid); MRS_V(dof_armature); MRS_V(dof_damping);
  MRS_V(dof_frictionloss); MRS_V(dof_solref); MRS_V(dof_solimp); MRS_V(dof_invweight0); MRS_V(dof_M0);
  MRS_V(geom_type); MRS_V(geom_contype); MRS_V(geom_conaffinity); MRS_V(geom_condim);
  MRS_V(geom_bodyid); MRS_V(geom_group); MRS_V(geom_priority); MRS_V(geom_size); MRS_V(geom_pos);
  MRS_V(geom_quat); MRS_V(geom_rbound); MRS_V(geom_friction); MRS_V(geom_margin); MRS_V(geom_gap);
  MRS_V(geom_solmix); MRS_V(geom_solref); MRS_V(geom_solimp); MRS_V(geom_rgba);
  MRS_V(site_bodyid); MRS_V(site_pos); MRS_V(site_quat);
  MRS_V(cam_bodyid); MRS_V(cam_resolution); MRS_V(cam_pos); MRS_V(cam_quat); MRS_V(cam_fovy);
  MRS_V(actuator_trntype); MRS_V(actuator_dyntype); MRS_V(actuator_gaintype);
  MRS_V(actuator_biastype); MRS_V(actuator_trnid); MRS_V(actuator_ctrllimited);
  MRS_V(actuator_forcelimited); MRS_V(actuator_gear); MRS_V(actuator_gainprm);
  MRS_V(actuator_biasprm); MRS_V(actuator_ctrlrange); MRS_V(actuator_forcerange);
  MRS_V(sensor_type); MRS_V(sensor_objtype); MRS_V(sensor_objid); MRS_V(sensor_dim);
  MRS_V(sensor_adr); MRS_V(sensor_cutoff);
  MRS_V(qpos0); MRS_V(qpos_spring); MRS_V(key_time); MRS_V(key_qpos); MRS_V(key_qvel); MRS_V(key_ctrl);
  MRS_V(pair_geom1); MRS_V(pair_geom2);
  v.nmesh = nmesh;
  v.nmeshvert = static_cast<int>(mesh_vert.size() / 3);
  v.nmeshface = static_cast<int>(mesh_face.size() / 3);
  v.nmeshhull = static_cast<int>(mesh_hull.size());
  MRS_V(geom_dataid); MRS_V(mesh_vertadr); MRS_V(mesh_vertnum); MRS_V(mesh_faceadr); MRS_V(mesh_facenum);
  MRS_V(mesh_hulladr); MRS_V(mesh_hullnum); MRS_V(mesh_face); MRS_V(mesh_hull); MRS_V(mesh_vert);
  for (int i = 0; i < 10; ++i) v.vis_headlight[i] = vis_headlight[i];
  v.nlight = static_cast<int>(light_active.size());
  v.ntex = static_cast<int>(tex_type.size());
  v.nmat = static_cast<int>(mat_texid.size());
  MRS_V(light_directional); MRS_V(light_castshadow); MRS_V(light_active); MRS_V(tex_type); MRS_V(tex_builtin);
  MRS_V(tex_mark); MRS_V(tex_width); MRS_V(tex_height); MRS_V(mat_texid); MRS_V(mat_texuniform); MRS_V(geom_matid);
  MRS_V(light_pos); MRS_V(light_dir); MRS_V(light_ambient); MRS_V(light_diffuse); MRS_V(light_specular);
  MRS_V(light_attenuation); MRS_V(light_cutoff); MRS_V(light_exponent); MRS_V(tex_rgb1); MRS_V(tex_rgb2);
  MRS_V(tex_markrgb); MRS_V(mat_rgba); MRS_V(mat_texrepeat); MRS_V(mat_specular); MRS_V(mat_shininess);
  MRS_V(mat_emission);
  v.neq = static_cast<int>(eq_type.size());
  MRS_V(eq_type); MRS_V(eq_obj1id); MRS_V(eq_obj2id); MRS_V(eq_active0); MRS_V(eq_solref); MRS_V(eq_solimp);
  MRS_V(eq_data);
  v.ntendon = static_cast<int>(tendon_adr.size());
  v.nwrap = static_cast<int>(wrap_objid.size());
  MRS_V(tendon_adr); MRS_V(tendon_num); MRS_V(tendon_limited); MRS_V(wrap_objid); MRS_V(wrap_prm);
  MRS_V(tendon_range); MRS_V(tendon_margin); MRS_V(tendon_solref_lim); MRS_V(tendon_solimp_lim);
  MRS_V(tendon_frictionloss); MRS_V(tendon_solref_fri); MRS_V(tendon_solimp_fri); MRS_V(tendon_stiffness);
  MRS_V(tendon_damping); MRS_V(tendon_lengthspring); MRS_V(tendon_invweight0); MRS_V(tendon_length0);
  v.nexpair = static_cast<int>(expair_geom1.size());
  v.nexclude = static_cast<int>(exclude_body1.size());
  MRS_V(expair_geom1); MRS_V(expair_geom2); MRS_V(expair_dim); MRS_V(exclude_body1); MRS_V(exclude_body2);
  MRS_V(expair_friction); MRS_V(expair_solref); MRS_V(expair_solimp); MRS_V(expair_margin); MRS_V(expair_gap);
  v.nmeshpoly = static_cast<int>(mesh_polynum_v.size());
  v.nmeshpolyvert = static_cast<int>(mesh_polyvert.size());
  MRS_V(mesh_polyadr); MRS_V(mesh_polynum); MRS_V(mesh_polyvertadr); MRS_V(mesh_polyvert); MRS_V(mesh_polynormal);
  v.mesh_polyvertnum = mesh_polynum_v.empty() ? nullptr : mesh_polynum_v.data();
#undef MRS_V
  return v;
}

Model compile_mjcf_file(const std::string& path) {
  auto root = xml_parse(read_file(path), path);
  Compiler c;
  return c.compile(std::move(root), dirname_of(path));
}

Model compile_mjcf_string(const std::string& xml, const std::string& basedir) {
  auto root = xml_parse(xml, "<string>");
  Compiler c;
  return c.compile(std::move(root), basedir.empty() ? "." : basedir);
}

}  // namespace mrs
