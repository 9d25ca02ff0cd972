// Mesh assets for the MJCF compiler: file loading (Wavefront OBJ, binary / ASCII STL), the convex
// hull used by collision, and the mass properties MuJoCo derives from a mesh (its compiler's mesh
// processing: volume, centre of mass, principal inertia, and the recentred/realigned vertices).
#pragma once

#include <string>
#include <vector>

namespace mrs {

struct MeshAsset {
  std::vector<double> vert;  // 3 per vertex
  std::vector<int> face;     // 3 per triangle
};

// .obj (v / f records, polygons fanned into triangles, negative indices) or .stl (binary or ASCII;
// coincident vertices merged).  Throws std::runtime_error on unreadable or malformed files.
MeshAsset load_mesh_file(const std::string& path);

// Convex hull of the vertices (incremental; coplanar or fewer than 4 distinct points throw):
// outward-oriented triangles over vertex indices, and the sorted ids of the hull's vertices.
void convex_hull(const std::vector<double>& vert, std::vector<int>& hull_face, std::vector<int>& hull_vert);

// The convex hull's faces as polygons: coplanar hull triangles (unit normals within 1e-6) merged, each
// polygon's vertices counter-clockwise about its outward unit normal, collinear boundary vertices
// dropped.  polys: vertex ids per polygon; normals: 3 per polygon.
void hull_polygons(const std::vector<double>& vert, const std::vector<int>& hull_face,
                   std::vector<std::vector<int>>& polys, std::vector<double>& normals);

// Volume, centre of mass and the inertia tensor about it (unit density) of the solid bounded by the
// triangles (divergence theorem over signed tetrahedra from the origin).
void mesh_mass_properties(const std::vector<double>& vert, const std::vector<int>& face, double& volume,
                          double com[3], double inertia[9]);

}  // namespace mrs
