"""The reference's structured, stretched flat-plate meshes, restated without gmsh.

/root/reference/testcases/visc-flatplate/grids/flatplatestructstretched.geo:1-70 (the meshes of
SpatialFlow_NS_FlatPlate_LeastSquares_Roe_Struct_CDConvergence, tests/visc-flatplate/CMakeLists.txt:15-39):
  * two transfinite quadrilateral blocks: x in [-0.5, 0] ahead of the plate (Line 1, nxi = 10 points,
    progression 1.2 away from the leading edge) and x in [0, 1] along it (Line 2, nxp = 20 points,
    progression 1.1), y in [0, 1] (Lines 3, 6, 7, ny = 20 points, progression 1.4 away from the wall);
    opposite block sides carry the same distributions, so the transfinite interpolation is the tensor
    product of the edge distributions;
  * gmsh's "Transfinite Line = n Using Progression r": n points, successive intervals in ratio r from
    the line's first point, i.e. point k at L (r^k - 1)/(r^(n-1) - 1);
  * markers (Physical Line): 2 the plate (y = 0, x >= 0), 3 the bottom ahead of it (y = 0, x < 0),
    4 far field (x = -0.5 and y = 1), 5 outlet (x = 1);
  * mesh i = mesh 0 after i RefineMesh steps: every quadrilateral split into four at its edge
    midpoints (straight edges, so the midpoints are the geometric ones).
Cell and node numbering differ from gmsh's; the CDsf convergence test depends only on the geometry
(functionals are sums over the wall faces, the mesh-size parameter is 1/sqrt(nelem),
casesolvers.cpp:96)."""
import numpy as np


def _progression(n, r, length):
    k = np.arange(n, dtype=np.float64)
    return length * (r ** k - 1.0) / (r ** (n - 1) - 1.0)


def _refine(x, levels):
    for _ in range(levels):
        mid = 0.5 * (x[:-1] + x[1:])
        out = np.empty(2 * len(x) - 1)
        out[0::2] = x
        out[1::2] = mid
        x = out
    return x


def flatplate_points(level, ref=2):
    """x and y node coordinates of mesh `level` (0, 1, 2, ...)"""
    nxi, nxp, ny = 5 * ref, 10 * ref, 10 * ref
    xin = -_progression(nxi, 1.2, 0.5)[::-1]          # -0.5 .. 0, fine near x = 0
    xpl = _progression(nxp, 1.1, 1.0)                  # 0 .. 1, fine near the leading edge
    x = np.concatenate([xin[:-1], xpl])
    y = _progression(ny, 1.4, 1.0)                     # 0 .. 1, fine near the wall
    return _refine(x, level), _refine(y, level)


def write_flatplate_msh(path, level):
    """Gmsh 2.2 ASCII file of mesh `level`: boundary line elements first (physical tag = marker),
    then counter-clockwise quadrilaterals (physical surface 1), as gmsh writes the .geo's mesh"""
    x, y = flatplate_points(level)
    nx, ny = len(x), len(y)
    nid = lambda i, j: j * nx + i + 1                  # 1-based node id
    lines = []
    for i in range(nx - 1):                            # bottom: slip wall ahead of the plate, then the plate
        lines.append((3 if x[i] < 0 else 2, nid(i, 0), nid(i + 1, 0)))
    for j in range(ny - 1):                            # outlet x = 1
        lines.append((5, nid(nx - 1, j), nid(nx - 1, j + 1)))
    for i in range(nx - 1, 0, -1):                     # top y = 1 (far field)
        lines.append((4, nid(i, ny - 1), nid(i - 1, ny - 1)))
    for j in range(ny - 1, 0, -1):                     # left x = -0.5 (far field)
        lines.append((4, nid(0, j), nid(0, j - 1)))
    quads = [(nid(i, j), nid(i + 1, j), nid(i + 1, j + 1), nid(i, j + 1))
             for j in range(ny - 1) for i in range(nx - 1)]
    out = ["$MeshFormat", "2.2 0 8", "$EndMeshFormat", "$Nodes", str(nx * ny)]
    for j in range(ny):
        for i in range(nx):
            out.append("%d %.17g %.17g 0" % (nid(i, j), x[i], y[j]))
    out += ["$EndNodes", "$Elements", str(len(lines) + len(quads))]
    e = 1
    for tag, a, b in lines:
        out.append("%d 1 2 %d %d %d %d" % (e, tag, tag, a, b))
        e += 1
    for q in quads:
        out.append("%d 3 2 1 1 %d %d %d %d" % (e, *q))
        e += 1
    out.append("$EndElements")
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")
    return (nx - 1) * (ny - 1)
