#!/usr/bin/env python3
"""Cell-shape statistics of a generated NACA 0012 mesh (host only): counts of quadrangles and triangles,
triangle aspect ratio (longest edge over the height onto it) and largest angle, neighbour area ratios.
usage: python tools/mesh_quality.py hybrid NSURF NWAKE NQUAD NROWS [WALL]
       python tools/mesh_quality.py c5 SCALE"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def quality(m):
    nn = m.nnode
    tri = np.where(nn == 3)[0]
    P = m.coords[m.inpoel[tri, :3]]                        # [nt][3][2]
    e = np.stack([P[:, 1] - P[:, 0], P[:, 2] - P[:, 1], P[:, 0] - P[:, 2]], 1)
    L = np.linalg.norm(e, axis=2)
    area = 0.5 * np.abs(e[:, 0, 0] * e[:, 1, 1] - e[:, 0, 1] * e[:, 1, 0])
    lmax = L.max(1)
    aspect = lmax * lmax / (2.0 * area)                    # longest edge over its height
    c = [np.einsum("ij,ij->i", -e[:, (k + 2) % 3], e[:, k]) / (L[:, (k + 2) % 3] * L[:, k]) for k in range(3)]
    maxang = np.degrees(np.arccos(np.clip(np.min(np.stack(c, 1), 1), -1, 1)))
    F = m.intfac[m.nbface:]
    ar = m.area[F[:, 0]] / m.area[F[:, 1]]
    ar = np.maximum(ar, 1 / ar)
    pct = lambda a: {p: round(float(np.percentile(a, p)), 3) for p in (50, 90, 99, 99.9, 100)} if len(a) else {}
    return {"cells": int(m.nelem), "faces": int(m.naface), "quads": int((nn == 4).sum()), "triangles": int(len(tri)),
            "tri_aspect": pct(aspect), "tri_max_angle": pct(maxang), "neighbour_area_ratio": pct(ar)}


def main():
    import fvens_amd as fa
    kind = sys.argv[1]
    if kind == "hybrid":
        a = [int(x) for x in sys.argv[2:6]]
        ws = float(sys.argv[6]) if len(sys.argv) > 6 else 1e-5
        m = fa.UMesh.naca_hybrid(*a, 20.0, ws)
        rec = {"args": a, "wall": ws}
    else:
        from bench import c4_mesh
        m, dims = c4_mesh(fa, int(sys.argv[2]), 2)
        rec = {"dims": dims}
    rec.update(quality(m))
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
