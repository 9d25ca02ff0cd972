"""Generate the procedural mesh fixtures under scenes/meshes/ (data, deterministic; run once, output
committed): a bumpy sphere "statue" of 6912 triangles and a ribbed link shell of 1536 triangles, both
closed and consistently wound (outward normals), written as Wavefront OBJ.
Usage: python scripts/make_mesh_fixtures.py"""
import math
from pathlib import Path

OUT = Path(__file__).resolve().parents[1] / "scenes" / "meshes"


def write_obj(path, verts, faces, comment):
    with open(path, "w") as f:
        f.write(f"# {comment}\n")
        for v in verts:
            f.write("v %.6f %.6f %.6f\n" % v)
        for a, b, c in faces:
            f.write(f"f {a + 1} {b + 1} {c + 1}\n")


def uv_sphere(nu, nv, radius):
    """closed UV sphere: poles + (nv - 1) rings of nu vertices; 2 nu (nv - 1) triangles"""
    verts = [(0.0, 0.0, radius(0.0, 0.0))]
    for j in range(1, nv):
        th = math.pi * j / nv
        for i in range(nu):
            ph = 2 * math.pi * i / nu
            r = radius(th, ph)
            verts.append((r * math.sin(th) * math.cos(ph), r * math.sin(th) * math.sin(ph), r * math.cos(th)))
    verts.append((0.0, 0.0, -radius(math.pi, 0.0)))
    south = len(verts) - 1
    ring = lambda j, i: 1 + (j - 1) * nu + (i % nu)
    faces = [(0, ring(1, i), ring(1, i + 1)) for i in range(nu)]
    for j in range(1, nv - 1):
        for i in range(nu):
            a, b, c, d = ring(j, i), ring(j + 1, i), ring(j + 1, i + 1), ring(j, i + 1)
            faces += [(a, b, c), (a, c, d)]
    faces += [(ring(nv - 1, i), south, ring(nv - 1, i + 1)) for i in range(nu)]
    return verts, faces


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    # statue: sphere radius 0.5 with radial bumps of 4 cm; 72 x 49 -> 2 * 72 * 48 = 6912 triangles
    v, f = uv_sphere(72, 49, lambda th, ph: 0.5 + 0.04 * math.sin(5 * th) * math.cos(6 * ph))
    write_obj(OUT / "statue.obj", v, f, f"bumpy sphere, {len(v)} vertices, {len(f)} triangles (scripts/make_mesh_fixtures.py)")
    # link shell: ellipsoid-like capsule along z (half length 0.5, radius 0.5 before scaling) with 8 ribs
    def link_r(th, ph):
        return 0.5 * (1 + 0.06 * math.cos(8 * ph))
    v, f = uv_sphere(32, 25, link_r)
    v = [(x, y, 2.0 * z) for (x, y, z) in v]   # stretched along z: unit-length link before scaling
    write_obj(OUT / "link.obj", v, f, f"ribbed link shell, {len(v)} vertices, {len(f)} triangles (scripts/make_mesh_fixtures.py)")


if __name__ == "__main__":
    main()
