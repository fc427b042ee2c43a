"""Test infrastructure (tests/, tools/ only; never the product path): the oracle's MPR
(oracle/dx_oracle.c mpr_penetration, [3P] libccd ccdMPRPenetration) restated in numpy
with the arithmetic type as a parameter.  Evaluated in fp64 it reproduces the C oracle;
evaluated in fp32 -- the precision the north star sets for the kernel -- from the geoms'
poses perturbed at the fp32 forward kinematics' resolution, it reproduces the answer the
kernel's fp32 MPR stops on at a deep overlap of two curved hulls, where fp64 MPR ends on
another portal (tests/test_gpu_parity.py _contact_lists_agree's "fp32 portal" rule,
tests/test_mpr_precision.py on the committed fixtures).
"""
import numpy as np

MPR_TOL, MPR_ITER = 1e-6, 50


def mpr(pos1, mat1, ver1, cen1, pos2, mat2, ver2, cen2, half_margin, T):
    """Penetration of convex 1 into convex 2 (a hull's vertices, or a box as [[half
    sizes]]): (depth, normal, portal, trips) or None; every operation in numpy type T
    (np.float32 or np.float64)."""
    z = T(0)
    pos1, mat1, ver1, cen1, pos2, mat2, ver2, cen2 = (np.asarray(a, dtype=T) for a in
                                                      (pos1, mat1, ver1, cen1, pos2, mat2, ver2, cen2))
    hm = T(half_margin)
    tiny = T(1e-14)

    def dot(a, b):
        return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]

    def cross(a, b):
        return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]], dtype=T)

    def normalize(a):
        n = np.sqrt(dot(a, a))
        return a / n if n > T(1e-15) else a

    def support(pos, mat, ver, d):
        ld = np.array([mat[0, 0] * d[0] + mat[1, 0] * d[1] + mat[2, 0] * d[2],
                       mat[0, 1] * d[0] + mat[1, 1] * d[1] + mat[2, 1] * d[2],
                       mat[0, 2] * d[0] + mat[1, 2] * d[1] + mat[2, 2] * d[2]], dtype=T)  # mattvec3
        if ver.shape[0] == 1:  # a box: ver holds its half sizes
            lp = np.where(ld >= z, ver[0], -ver[0])
        else:
            proj = ver[:, 0] * ld[0] + ver[:, 1] * ld[1] + ver[:, 2] * ld[2]
            lp = ver[int(np.argmax(proj))]  # first maximiser, as the serial scan
        out = np.array([mat[k, 0] * lp[0] + mat[k, 1] * lp[1] + mat[k, 2] * lp[2] for k in range(3)], dtype=T) + pos
        if hm > 0:
            n = np.sqrt(dot(d, d))
            if n > T(1e-15):
                out = out + d / n * hm
        return out

    def msup(d):
        a = support(pos1, mat1, ver1, d)
        b = support(pos2, mat2, ver2, -d)
        return (a - b, a, b)

    def iszero(x):
        return abs(x) < tiny

    P = [None] * 4
    P[0] = (cen1 - cen2, cen1, cen2)
    d = normalize(-P[0][0])
    P[1] = msup(d)
    if iszero(dot(P[1][0], d)) or dot(P[1][0], d) < z:
        return None
    d = cross(P[0][0], P[1][0])
    if iszero(dot(d, d)):
        return ("segment",)
    d = normalize(d)
    P[2] = msup(d)
    if iszero(dot(P[2][0], d)) or dot(P[2][0], d) < z:
        return None
    d = normalize(cross(P[1][0] - P[0][0], P[2][0] - P[0][0]))
    if dot(d, P[0][0]) > z:
        P[1], P[2] = P[2], P[1]
        d = -d
    for it in range(1002):
        if it > 1000:
            return None
        P[3] = msup(d)
        dt = dot(P[3][0], d)
        if iszero(dt) or dt < z:
            return None
        cont = False
        dt = dot(cross(P[1][0], P[3][0]), P[0][0])
        if dt < z and not iszero(dt):
            P[2] = P[3]
            cont = True
        if not cont:
            dt = dot(cross(P[3][0], P[2][0]), P[0][0])
            if dt < z and not iszero(dt):
                P[1] = P[3]
                cont = True
        if cont:
            d = normalize(cross(P[1][0] - P[0][0], P[2][0] - P[0][0]))
        else:
            break

    def portal_dir():
        return normalize(cross(P[2][0] - P[1][0], P[3][0] - P[1][0]))

    def reach_tol(v4, d):
        dv4 = dot(v4[0], d)
        return min(dv4 - dot(P[1][0], d), dv4 - dot(P[2][0], d), dv4 - dot(P[3][0], d)) <= T(MPR_TOL)

    def expand(v4):
        v4v0 = cross(v4[0], P[0][0])
        if dot(P[1][0], v4v0) > z:
            if dot(P[2][0], v4v0) > z:
                P[1] = v4
            else:
                P[3] = v4
        else:
            if dot(P[3][0], v4v0) > z:
                P[2] = v4
            else:
                P[1] = v4

    for it in range(10 ** 6):
        d = portal_dir()
        if dot(d, P[1][0]) >= z:
            break
        v4 = msup(d)
        if dot(v4[0], d) < z or reach_tol(v4, d) or it > MPR_ITER:
            return None
        expand(v4)
    trips = 0
    for it in range(10 ** 6):
        d = portal_dir()
        v4 = msup(d)
        trips += 1
        if reach_tol(v4, d) or it > MPR_ITER:
            # closest point of the final portal to the origin, in fp64 (the kernel's and the
            # oracle's exit)
            a, b, c = (np.asarray(P[k][0], dtype=np.float64) for k in (1, 2, 3))
            q = _closest(a, b, c)
            depth = float(np.linalg.norm(q))
            return depth, q / depth, [np.asarray(P[k][0], dtype=np.float64) for k in range(4)], trips
        expand(v4)


def _closest(a, b, c):
    """Closest point of triangle abc to the origin (Ericson 5.1.5), fp64."""
    ab, ac, ap = b - a, c - a, -a
    d1, d2 = ab @ ap, ac @ ap
    if d1 <= 0 and d2 <= 0:
        return a
    bp = -b
    d3, d4 = ab @ bp, ac @ bp
    if d3 >= 0 and d4 <= d3:
        return b
    vc = d1 * d4 - d3 * d2
    if vc <= 0 and d1 >= 0 and d3 <= 0:
        return a + d1 / (d1 - d3) * ab
    cp = -c
    d5, d6 = ab @ cp, ac @ cp
    if d6 >= 0 and d5 <= d6:
        return c
    vb = d5 * d2 - d1 * d6
    if vb <= 0 and d2 >= 0 and d6 <= 0:
        return a + d2 / (d2 - d6) * ac
    va = d3 * d6 - d5 * d4
    if va <= 0 and (d4 - d3) >= 0 and (d5 - d6) >= 0:
        return b + (d4 - d3) / ((d4 - d3) + (d5 - d6)) * (c - b)
    den = 1.0 / (va + vb + vc)
    return a + ab * (vb * den) + ac * (vc * den)


def pair_inputs(cm, d, g1, g2):
    """World pose, hull and interior point of both geoms at the oracle state d, and the
    pair's half margin."""
    def geom(g):
        if int(cm.geom_type[g]) == 6:  # box: its half sizes (support = sign(ld) * size)
            ver = np.asarray(cm.geom_size, dtype=np.float64).reshape(-1, 3)[g][None, :]
        else:
            mid = int(cm.geom_dataid[g])
            a, n = int(cm.mesh_vertadr[mid]), int(cm.mesh_vertnum[mid])
            ver = np.asarray(cm.mesh_vert, dtype=np.float64).reshape(-1, 3)[a:a + n]
        pos = d.geom_xpos.reshape(-1, 3)[g].copy()
        mat = d.geom_xmat.reshape(-1, 3, 3)[g].copy()
        cen = pos + mat @ np.asarray(cm.geom_center, dtype=np.float64).reshape(-1, 3)[g]
        return pos, mat, ver, cen

    gp = np.asarray(cm.gpair_geom).reshape(-1, 2)
    k = np.flatnonzero((gp[:, 0] == g1) & (gp[:, 1] == g2))
    margin = float(np.asarray(cm.gpair_margin)[k[0]]) if len(k) else 0.0
    return geom(g1), geom(g2), 0.5 * margin


def fp32_reproduces(cm, d, g1, g2, rec, n=100, rel=3e-7, seed=0, ang_tol=1e-4, depth_tol=1e-4):
    """Whether MPR in fp32 from the pair's poses at the oracle state d -- as computed, then
    perturbed at relative `rel` (seven-level chains of fp32 transforms) in up to n draws --
    reproduces the contact record `rec` (the kernel's: dist in rec[12], normal rec[3:6])
    within ang_tol rad and depth_tol of the depth.  Returns (ok, best angle, best depth
    error, draws)."""
    (p1, m1, v1, c1), (p2, m2, v2, c2), hm = pair_inputs(cm, d, g1, g2)
    rng = np.random.RandomState(seed)
    best = (np.inf, np.inf)
    nrm = np.asarray(rec[3:6], dtype=np.float64)
    nrm = nrm / np.linalg.norm(nrm)
    for i in range(n):
        j = (lambda a: a * (1 + rng.standard_normal(a.shape) * rel)) if i else (lambda a: a)
        res = mpr(j(p1), j(m1), v1, j(c1), j(p2), j(m2), v2, j(c2), hm, np.float32)
        if res is None or len(res) < 4:
            continue
        ang = float(np.arccos(np.clip(res[1] @ nrm, -1.0, 1.0)))
        dr = abs((2 * hm - res[0]) - rec[12]) / abs(rec[12])
        if ang + dr < best[0] + best[1]:
            best = (ang, dr)
        if ang <= ang_tol and dr <= depth_tol:
            return True, ang, dr, i + 1
    return False, best[0], best[1], n
