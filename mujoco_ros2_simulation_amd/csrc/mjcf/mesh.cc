// Mesh assets (mesh.h): OBJ / STL loading, convex hull, mass properties.
#include "mesh.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <set>
#include <sstream>
#include <stdexcept>

namespace mrs {

namespace {

const double* P(const std::vector<double>& v, int i) { return v.data() + 3 * i; }
double dot(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
void sub(double r[3], const double a[3], const double b[3]) { for (int i = 0; i < 3; ++i) r[i] = a[i] - b[i]; }
void cross(double r[3], const double a[3], const double b[3]) {
  r[0] = a[1] * b[2] - a[2] * b[1];
  r[1] = a[2] * b[0] - a[0] * b[2];
  r[2] = a[0] * b[1] - a[1] * b[0];
}

std::string lower_ext(const std::string& path) {
  auto dot_pos = path.find_last_of('.');
  std::string e = dot_pos == std::string::npos ? "" : path.substr(dot_pos + 1);
  for (char& c : e) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return e;
}

MeshAsset load_obj(const std::string& text, const std::string& path) {
  MeshAsset m;
  std::istringstream in(text);
  std::string line;
  int lineno = 0;
  while (std::getline(in, line)) {
    ++lineno;
    std::istringstream ls(line);
    std::string tag;
    if (!(ls >> tag)) continue;
    if (tag == "v") {
      double x, y, z;
      if (!(ls >> x >> y >> z)) throw std::runtime_error(path + ":" + std::to_string(lineno) + ": bad vertex");
      m.vert.insert(m.vert.end(), {x, y, z});
    } else if (tag == "f") {
      std::vector<int> poly;
      std::string tok;
      const int nv = static_cast<int>(m.vert.size() / 3);
      while (ls >> tok) {
        int idx = std::atoi(tok.c_str());  // "a", "a/b", "a//c", "a/b/c": the position index
        if (idx < 0) idx = nv + idx + 1;
        if (idx < 1 || idx > nv) throw std::runtime_error(path + ":" + std::to_string(lineno) + ": face index out of range");
        poly.push_back(idx - 1);
      }
      if (poly.size() < 3) throw std::runtime_error(path + ":" + std::to_string(lineno) + ": face with fewer than 3 vertices");
      for (size_t k = 1; k + 1 < poly.size(); ++k) m.face.insert(m.face.end(), {poly[0], poly[k], poly[k + 1]});
    }
  }
  return m;
}

struct VertexMerger {
  MeshAsset& m;
  std::map<std::array<double, 3>, int> ids;
  int add(double x, double y, double z) {
    auto it = ids.emplace(std::array<double, 3>{x, y, z}, static_cast<int>(m.vert.size() / 3));
    if (it.second) m.vert.insert(m.vert.end(), {x, y, z});
    return it.first->second;
  }
};

MeshAsset load_stl(const std::string& text, const std::string& path) {
  MeshAsset m;
  VertexMerger merge{m, {}};
  uint32_t n = 0;
  if (text.size() >= 84) std::memcpy(&n, text.data() + 80, 4);
  if (text.size() >= 84 && text.size() == 84 + 50ull * n) {  // binary
    for (uint32_t t = 0; t < n; ++t) {
      const char* rec = text.data() + 84 + 50ull * t + 12;  // skip the facet normal
      int v[3];
      for (int k = 0; k < 3; ++k) {
        float x[3];
        std::memcpy(x, rec + 12 * k, 12);
        v[k] = merge.add(x[0], x[1], x[2]);
      }
      m.face.insert(m.face.end(), {v[0], v[1], v[2]});
    }
    return m;
  }
  std::istringstream in(text);  // ASCII: "vertex x y z" triples
  std::string tok;
  std::vector<int> tri;
  while (in >> tok) {
    if (tok != "vertex") continue;
    double x, y, z;
    if (!(in >> x >> y >> z)) throw std::runtime_error(path + ": bad STL vertex");
    tri.push_back(merge.add(x, y, z));
    if (tri.size() == 3) {
      m.face.insert(m.face.end(), tri.begin(), tri.end());
      tri.clear();
    }
  }
  if (m.face.empty()) throw std::runtime_error(path + ": no triangles in STL file");
  return m;
}

struct HullFace {
  int v[3];
  double n[3], d;
  bool alive;
};

HullFace make_face(const std::vector<double>& vert, int a, int b, int c) {
  HullFace f{{a, b, c}, {0, 0, 0}, 0, true};
  double e1[3], e2[3];
  sub(e1, P(vert, b), P(vert, a));
  sub(e2, P(vert, c), P(vert, a));
  cross(f.n, e1, e2);
  const double len = std::sqrt(dot(f.n, f.n));
  if (len > 0)
    for (double& x : f.n) x /= len;
  f.d = dot(f.n, P(vert, a));
  return f;
}

}  // namespace

MeshAsset load_mesh_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open mesh file '" + path + "'");
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string text = ss.str();
  const std::string ext = lower_ext(path);
  MeshAsset m;
  if (ext == "obj") m = load_obj(text, path);
  else if (ext == "stl") m = load_stl(text, path);
  else throw std::runtime_error("unsupported mesh file type '." + ext + "' (obj and stl are supported)");
  if (m.vert.size() < 12) throw std::runtime_error("mesh file '" + path + "' has fewer than 4 vertices");
  return m;
}

void convex_hull(const std::vector<double>& vert, std::vector<int>& hull_face, std::vector<int>& hull_vert) {
  const int n = static_cast<int>(vert.size() / 3);
  if (n < 4) throw std::runtime_error("mesh has fewer than 4 vertices");
  double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], P(vert, i)[k]); hi[k] = std::max(hi[k], P(vert, i)[k]); }
  double diag[3];
  sub(diag, hi, lo);
  const double eps = 1e-10 * std::max(std::sqrt(dot(diag, diag)), 1e-300);
  // initial tetrahedron: farthest pair along the widest axis, farthest from that line, from that plane
  int ax = 0;
  for (int k = 1; k < 3; ++k)
    if (diag[k] > diag[ax]) ax = k;
  int i0 = 0, i1 = 0;
  for (int i = 0; i < n; ++i) {
    if (P(vert, i)[ax] < P(vert, i0)[ax]) i0 = i;
    if (P(vert, i)[ax] > P(vert, i1)[ax]) i1 = i;
  }
  if (i0 == i1) throw std::runtime_error("mesh vertices coincide");
  double e01[3];
  sub(e01, P(vert, i1), P(vert, i0));
  int i2 = -1;
  double best = eps;
  for (int i = 0; i < n; ++i) {
    double d[3], c[3];
    sub(d, P(vert, i), P(vert, i0));
    cross(c, e01, d);
    const double l = std::sqrt(dot(c, c)) / std::sqrt(dot(e01, e01));
    if (l > best) { best = l; i2 = i; }
  }
  if (i2 < 0) throw std::runtime_error("mesh vertices are collinear");
  HullFace base = make_face(vert, i0, i1, i2);
  int i3 = -1;
  best = eps;
  for (int i = 0; i < n; ++i) {
    const double l = std::fabs(dot(base.n, P(vert, i)) - base.d);
    if (l > best) { best = l; i3 = i; }
  }
  if (i3 < 0) throw std::runtime_error("mesh vertices are coplanar (a mesh needs volume)");
  double centre[3] = {0, 0, 0};
  for (int id : {i0, i1, i2, i3})
    for (int k = 0; k < 3; ++k) centre[k] += 0.25 * P(vert, id)[k];
  std::vector<HullFace> faces;
  auto add_oriented = [&](int a, int b, int c) {
    HullFace f = make_face(vert, a, b, c);
    if (dot(f.n, centre) - f.d > 0) f = make_face(vert, a, c, b);
    faces.push_back(f);
  };
  add_oriented(i0, i1, i2);
  add_oriented(i0, i1, i3);
  add_oriented(i0, i2, i3);
  add_oriented(i1, i2, i3);
  for (int p = 0; p < n; ++p) {
    if (p == i0 || p == i1 || p == i2 || p == i3) continue;
    const double* x = P(vert, p);
    std::vector<int> visible;
    for (int f = 0; f < static_cast<int>(faces.size()); ++f)
      if (faces[f].alive && dot(faces[f].n, x) - faces[f].d > eps) visible.push_back(f);
    if (visible.empty()) continue;
    std::set<std::pair<int, int>> edges;
    for (int f : visible)
      for (int k = 0; k < 3; ++k) edges.emplace(faces[f].v[k], faces[f].v[(k + 1) % 3]);
    for (int f : visible) faces[f].alive = false;
    for (const auto& e : edges)
      if (!edges.count({e.second, e.first})) faces.push_back(make_face(vert, e.first, e.second, p));
  }
  hull_face.clear();
  std::set<int> used;
  for (const auto& f : faces)
    if (f.alive) {
      hull_face.insert(hull_face.end(), f.v, f.v + 3);
      used.insert(f.v, f.v + 3);
    }
  hull_vert.assign(used.begin(), used.end());
}

void hull_polygons(const std::vector<double>& vert, const std::vector<int>& hull_face,
                   std::vector<std::vector<int>>& polys, std::vector<double>& normals) {
  polys.clear();
  normals.clear();
  const size_t nt = hull_face.size() / 3;
  std::vector<double> tn(3 * nt);
  std::vector<double> ta(nt);
  for (size_t t = 0; t < nt; ++t) {
    const double *a = P(vert, hull_face[3 * t]), *b = P(vert, hull_face[3 * t + 1]), *c = P(vert, hull_face[3 * t + 2]);
    const double e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
    double n[3];
    cross(n, e1, e2);
    const double l = std::sqrt(dot(n, n));
    ta[t] = l;
    for (int k = 0; k < 3; ++k) tn[3 * t + k] = l > 0 ? n[k] / l : 0;
  }
  std::vector<int> group(nt, -1);
  for (size_t t = 0; t < nt; ++t) {
    if (group[t] >= 0 || !(ta[t] > 0)) continue;
    const int gid = static_cast<int>(polys.size());
    double nsum[3] = {0, 0, 0};
    std::vector<int> ids;
    for (size_t u = t; u < nt; ++u) {
      if (group[u] >= 0 || !(ta[u] > 0)) continue;
      if (dot(&tn[3 * t], &tn[3 * u]) < 1 - 1e-6) continue;
      group[u] = gid;
      for (int k = 0; k < 3; ++k) nsum[k] += ta[u] * tn[3 * u + k];
      for (int k = 0; k < 3; ++k) ids.push_back(hull_face[3 * u + k]);
    }
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    const double l = std::sqrt(dot(nsum, nsum));
    const double n[3] = {nsum[0] / l, nsum[1] / l, nsum[2] / l};
    // order about the centroid in the face plane (u, v, n right-handed: counter-clockwise about n)
    double cen[3] = {0, 0, 0};
    for (int i : ids)
      for (int k = 0; k < 3; ++k) cen[k] += P(vert, i)[k] / ids.size();
    double uax[3] = {P(vert, ids[0])[0] - cen[0], P(vert, ids[0])[1] - cen[1], P(vert, ids[0])[2] - cen[2]};
    const double un = dot(uax, n);
    for (int k = 0; k < 3; ++k) uax[k] -= un * n[k];
    const double ul = std::sqrt(dot(uax, uax));
    for (int k = 0; k < 3; ++k) uax[k] /= ul;
    double vax[3];
    cross(vax, n, uax);
    std::vector<std::pair<double, int>> ang;
    for (int i : ids) {
      const double d[3] = {P(vert, i)[0] - cen[0], P(vert, i)[1] - cen[1], P(vert, i)[2] - cen[2]};
      ang.push_back({std::atan2(dot(d, vax), dot(d, uax)), i});
    }
    std::sort(ang.begin(), ang.end());
    std::vector<int> loop;
    for (auto& a : ang) loop.push_back(a.second);
    // drop vertices on a straight boundary edge (their neighbours' edge passes through them)
    double ext = 0;
    for (int i : loop) {
      const double d[3] = {P(vert, i)[0] - cen[0], P(vert, i)[1] - cen[1], P(vert, i)[2] - cen[2]};
      ext = std::max(ext, std::sqrt(dot(d, d)));
    }
    std::vector<int> keep;
    const size_t nl = loop.size();
    for (size_t q = 0; q < nl; ++q) {
      const double *pa = P(vert, loop[(q + nl - 1) % nl]), *pb = P(vert, loop[q]), *pc = P(vert, loop[(q + 1) % nl]);
      const double e1[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]}, e2[3] = {pc[0] - pb[0], pc[1] - pb[1], pc[2] - pb[2]};
      double c[3];
      cross(c, e1, e2);
      if (dot(c, n) > 1e-12 * ext * ext) keep.push_back(loop[q]);
    }
    polys.push_back(keep.size() >= 3 ? keep : loop);
    for (int k = 0; k < 3; ++k) normals.push_back(n[k]);
  }
}

void mesh_mass_properties(const std::vector<double>& vert, const std::vector<int>& face, double& volume,
                          double com[3], double inertia[9]) {
  double vol = 0, c1[3] = {0, 0, 0}, C[9] = {0};
  for (size_t t = 0; t + 2 < face.size(); t += 3) {
    const double *a = P(vert, face[t]), *b = P(vert, face[t + 1]), *c = P(vert, face[t + 2]);
    double bc[3];
    cross(bc, b, c);
    const double v = dot(a, bc) / 6;
    const double s[3] = {a[0] + b[0] + c[0], a[1] + b[1] + c[1], a[2] + b[2] + c[2]};
    vol += v;
    for (int k = 0; k < 3; ++k) c1[k] += v * s[k] / 4;
    for (int r = 0; r < 3; ++r)
      for (int q = 0; q < 3; ++q)
        C[3 * r + q] += v / 20 * (a[r] * a[q] + b[r] * b[q] + c[r] * c[q] + s[r] * s[q]);
  }
  volume = vol;
  if (vol <= 0) {
    for (int k = 0; k < 3; ++k) com[k] = 0;
    std::fill(inertia, inertia + 9, 0.0);
    return;
  }
  for (int k = 0; k < 3; ++k) com[k] = c1[k] / vol;
  for (int r = 0; r < 3; ++r)
    for (int q = 0; q < 3; ++q) C[3 * r + q] -= vol * com[r] * com[q];
  const double tr = C[0] + C[4] + C[8];
  for (int r = 0; r < 3; ++r)
    for (int q = 0; q < 3; ++q) inertia[3 * r + q] = (r == q ? tr : 0) - C[3 * r + q];
}

}  // namespace mrs
