"""Convex hulls of collision meshes (build time only).

MuJoCo collides mesh geoms through the convex hull of the mesh vertices (it runs
qhull at compile time, [3P]).  We do the same with scipy's Qhull binding: this
runs once, on the host, when a scene is compiled into an asset blob; nothing on
the step path touches scipy.

For every hull we keep
  * the hull vertices (the only points a support query can return),
  * the vertex adjacency graph (CSR) used by hill-climbing support queries,
  * the volume centroid, used as the interior reference point of MPR
    (MuJoCo re-centres meshes at their centre of mass, so its MPR starts from
    the same point).
"""

from __future__ import annotations

import dataclasses

import numpy as np
from scipy.spatial import ConvexHull


@dataclasses.dataclass
class Hull:
    vert: np.ndarray  # (n, 3) hull vertices
    face: np.ndarray  # (m, 3) triangles, indices into vert
    adj_ptr: np.ndarray  # (n + 1,) CSR row pointers of the vertex graph
    adj_idx: np.ndarray  # neighbour indices
    centroid: np.ndarray  # (3,) volume centroid
    volume: float


def convex_hull(points: np.ndarray) -> Hull:
    points = np.asarray(points, dtype=np.float64)
    # Deduplicate first: STL repeats every vertex once per incident triangle.
    points = np.unique(np.round(points, 12), axis=0)
    qh = ConvexHull(points)
    used = np.unique(qh.simplices.ravel())
    remap = -np.ones(len(points), dtype=np.int64)
    remap[used] = np.arange(len(used))
    vert = points[used]
    face = remap[qh.simplices]
    # Orient faces outward using the hull equations (normal . x + offset <= 0).
    normals = qh.equations[:, :3]
    for k in range(len(face)):
        a, b, c = vert[face[k]]
        if np.dot(np.cross(b - a, c - a), normals[k]) < 0:
            face[k] = face[k][[0, 2, 1]]
    # Vertex adjacency.
    nbr = [set() for _ in range(len(vert))]
    for a, b, c in face:
        nbr[a].update((b, c))
        nbr[b].update((a, c))
        nbr[c].update((a, b))
    adj_ptr = np.zeros(len(vert) + 1, dtype=np.int64)
    adj_ptr[1:] = np.cumsum([len(s) for s in nbr])
    adj_idx = np.concatenate([sorted(s) for s in nbr]).astype(np.int64)
    # Volume centroid via tetrahedra from an interior point.
    ref = vert.mean(axis=0)
    a = vert[face[:, 0]] - ref
    b = vert[face[:, 1]] - ref
    c = vert[face[:, 2]] - ref
    vol6 = np.einsum("ij,ij->i", a, np.cross(b, c))
    volume = vol6.sum() / 6.0
    centroid = ref + (vol6[:, None] * (a + b + c) / 4.0).sum(axis=0) / vol6.sum()
    return Hull(vert, face.astype(np.int64), adj_ptr, adj_idx, centroid, float(volume))
