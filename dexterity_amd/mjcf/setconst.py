"""Compile-time constants that need the mass matrix at qpos0 ([3P] mj_setConst).

MuJoCo approximates diag(J M^-1 J^T) of every constraint row with per-object
"inverse weights" computed once at qpos0; they set the constraint regulariser R
(DESIGN.md §3.6).  This module evaluates forward kinematics and the
composite-rigid-body mass matrix once, in numpy, on the host.  It is build-time
code and deliberately simple.
"""

from __future__ import annotations

import numpy as np

from dexterity_amd.mjcf import math3d as m3

_MINVAL = 1e-15


def kinematics(A, qpos):
    nbody = int(A["nbody"][0])
    xpos = np.zeros((nbody, 3))
    xquat = np.zeros((nbody, 4))
    xquat[0] = (1, 0, 0, 0)
    xanchor = np.zeros((len(A["jnt_type"]), 3))
    xaxis = np.zeros((len(A["jnt_type"]), 3))
    for b in range(1, nbody):
        p = A["body_parent"][b]
        jn, ja = A["body_jntnum"][b], A["body_jntadr"][b]
        if jn and A["jnt_type"][ja] == 0:
            a = A["jnt_qposadr"][ja]
            xpos[b] = qpos[a : a + 3]
            xquat[b] = m3.quat_normalize(qpos[a + 3 : a + 7])
            xanchor[ja] = xpos[b]
            xaxis[ja] = m3.quat_to_mat(xquat[b])[:, 2]
            continue
        xpos[b] = xpos[p] + m3.quat_rotate(xquat[p], A["body_pos"][b])
        xquat[b] = m3.quat_mul(xquat[p], A["body_quat"][b])
        for j in range(ja, ja + jn):
            R = m3.quat_to_mat(xquat[b])
            xanchor[j] = R @ A["jnt_pos"][j] + xpos[b]
            xaxis[j] = R @ A["jnt_axis"][j]
            q = qpos[A["jnt_qposadr"][j]]
            xquat[b] = m3.quat_normalize(m3.quat_mul(xquat[b], m3.axis_angle_quat(A["jnt_axis"][j], q)))
            xpos[b] = xanchor[j] - m3.quat_to_mat(xquat[b]) @ A["jnt_pos"][j]
    xmat = np.array([m3.quat_to_mat(q) for q in xquat])
    xipos = xpos + np.einsum("bij,bj->bi", xmat, A["body_ipos"])
    ximat = np.array([xmat[b] @ m3.quat_to_mat(A["body_iquat"][b]) for b in range(nbody)])
    return xpos, xquat, xmat, xipos, ximat, xanchor, xaxis


def com_and_dofs(A, xpos, xmat, xipos, ximat, xanchor, xaxis):
    nbody = int(A["nbody"][0])
    nv = int(A["nv"][0])
    mass = A["body_mass"]
    rootid = A["body_rootid"]
    # subtree com per root body
    msum = mass.copy()
    mcom = mass[:, None] * xipos
    for b in range(nbody - 1, 0, -1):
        p = A["body_parent"][b]
        if p > 0:
            msum[p] += msum[b]
            mcom[p] += mcom[b]
    subtree_com = np.where(msum[:, None] > _MINVAL, mcom / np.maximum(msum, _MINVAL)[:, None], xipos)
    cdof = np.zeros((nv, 6))
    for d in range(nv):
        b = A["dof_bodyid"][d]
        j = A["dof_jntid"][d]
        off = subtree_com[rootid[b]] - xanchor[j]
        if A["jnt_type"][j] == 0:
            k = d - A["jnt_dofadr"][j]
            if k < 3:
                cdof[d, 3 + k] = 1.0
                continue
            ax = xmat[b][:, k - 3]
        else:
            ax = xaxis[j]
        cdof[d, :3] = ax
        cdof[d, 3:] = np.cross(ax, off)
    return subtree_com, cdof


def mass_matrix(A, qpos):
    xpos, xquat, xmat, xipos, ximat, xanchor, xaxis = kinematics(A, qpos)
    subtree_com, cdof = com_and_dofs(A, xpos, xmat, xipos, ximat, xanchor, xaxis)
    nbody = int(A["nbody"][0])
    nv = int(A["nv"][0])
    # 6x6 spatial inertia about subtree com of the root, in world orientation.
    I6 = np.zeros((nbody, 6, 6))
    for b in range(1, nbody):
        m = A["body_mass"][b]
        Rb = ximat[b]
        Ic = Rb @ np.diag(A["body_inertia"][b]) @ Rb.T
        c = xipos[b] - subtree_com[A["body_rootid"][b]]
        C = _skew(c)
        I6[b, :3, :3] = Ic + m * (C @ C.T)
        I6[b, :3, 3:] = m * C
        I6[b, 3:, :3] = m * C.T
        I6[b, 3:, 3:] = m * np.eye(3)
    crb = I6.copy()
    for b in range(nbody - 1, 0, -1):
        p = A["body_parent"][b]
        if p > 0:
            crb[p] += crb[b]
    M = np.zeros((nv, nv))
    for i in range(nv):
        f = crb[A["dof_bodyid"][i]] @ cdof[i]
        j = i
        while j >= 0:
            M[i, j] = M[j, i] = cdof[j] @ f
            j = A["dof_parentid"][j]
    M += np.diag(A["dof_armature"])
    return M, cdof, subtree_com, xipos


def _skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def body_jacobian(A, cdof, subtree_com, b, point):
    nv = int(A["nv"][0])
    jacp = np.zeros((3, nv))
    jacr = np.zeros((3, nv))
    if A["body_weldid"][b] == 0:
        return jacp, jacr
    d = A["body_dofadr"][b] + A["body_dofnum"][b] - 1 if A["body_dofnum"][b] else -1
    bb = b
    while d < 0 and bb > 0:
        bb = A["body_parent"][bb]
        d = A["body_dofadr"][bb] + A["body_dofnum"][bb] - 1 if A["body_dofnum"][bb] else -1
    off = point - subtree_com[A["body_rootid"][b]]
    while d >= 0:
        jacr[:, d] = cdof[d, :3]
        jacp[:, d] = cdof[d, 3:] + np.cross(cdof[d, :3], off)
        d = A["dof_parentid"][d]
    return jacp, jacr


def invweight0(A):
    nbody = int(A["nbody"][0])
    nv = int(A["nv"][0])
    M, cdof, subtree_com, xipos = mass_matrix(A, A["qpos0"])
    Minv = np.linalg.inv(M)
    bw = np.zeros((nbody, 2))
    for b in range(1, nbody):
        if A["body_weldid"][b] == 0:
            continue
        jp, jr = body_jacobian(A, cdof, subtree_com, b, xipos[b])
        bw[b, 0] = max(_MINVAL, np.trace(jp @ Minv @ jp.T) / 3)
        bw[b, 1] = max(_MINVAL, np.trace(jr @ Minv @ jr.T) / 3)
    dw = np.zeros(nv)
    for j in range(len(A["jnt_type"])):
        d = A["jnt_dofadr"][j]
        if A["jnt_type"][j] == 0:
            dw[d : d + 3] = max(_MINVAL, np.mean(np.diag(Minv)[d : d + 3]))
            dw[d + 3 : d + 6] = max(_MINVAL, np.mean(np.diag(Minv)[d + 3 : d + 6]))
        else:
            dw[d] = max(_MINVAL, Minv[d, d])
    nten = len(A["tendon_adr"])
    tw = np.zeros(nten)
    for t in range(nten):
        J = np.zeros(nv)
        for w in range(A["tendon_adr"][t], A["tendon_adr"][t] + A["tendon_num"][t]):
            J[A["wrap_dof"][w]] += A["wrap_coef"][w]
        tw[t] = max(_MINVAL, J @ Minv @ J)
    return bw, dw, tw
