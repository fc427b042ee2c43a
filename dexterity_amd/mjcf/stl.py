"""STL reader for the build-time model compiler.

The Shadow hand collision meshes are binary STL files referenced from
`shadow_hand_series_e.xml:14-199` in the reference; Adroit uses one convex mesh
(`adroit_hand.xml:44`).  Only vertices matter for collision: MuJoCo collides a
mesh geom through the convex hull of its vertices, so faces are discarded here
and the hull is rebuilt in `hull.py`.
"""

from __future__ import annotations

import struct

import numpy as np


def read_stl(path: str) -> np.ndarray:
    """Returns the (n, 3) float64 vertex array of a binary or ASCII STL file."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) >= 84:
        (ntri,) = struct.unpack("<I", data[80:84])
        if 84 + 50 * ntri == len(data):
            rec = np.dtype(
                [("n", "<f4", 3), ("v", "<f4", (3, 3)), ("attr", "<u2")]
            )
            tris = np.frombuffer(data, dtype=rec, count=ntri, offset=84)
            return tris["v"].reshape(-1, 3).astype(np.float64)
    # ASCII fallback.
    verts = []
    for line in data.decode("ascii", errors="replace").splitlines():
        tok = line.split()
        if len(tok) == 4 and tok[0] == "vertex":
            verts.append([float(t) for t in tok[1:]])
    if not verts:
        raise ValueError(f"could not parse STL file {path}")
    return np.asarray(verts, dtype=np.float64)
