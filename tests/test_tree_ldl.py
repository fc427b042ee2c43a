"""CPU restatement of the tree-sparse LDL^T solve of M and M + h D (dx_device.h
tree_solve, item table built by dx_api.hip dx_model_load; MuJoCo's mj_factorM /
mj_solveM [3P]).  For every shipped scene: the elimination items grouped by height
level, applied slot by slot with every slot's reads taken before its writes (what the
wave does with LDS atomics), then the two substitution chains with the kernel's
scaling, must solve a random SPD matrix with the scene's tree sparsity; and the table
must fit the kernel's DX_LDL_SLOTS, so the device takes the tree path."""
import glob
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DX_LDL_SLOTS = 16  # dx_internal.h
WAVE = 64


def ldl_slots(par):
    """Items (k, i, j) per 64-lane slot, level by level (dx_api.hip ldl_tab)."""
    nv = len(par)
    height = [0] * nv
    for k in range(nv - 1, -1, -1):
        if par[k] >= 0:
            height[par[k]] = max(height[par[k]], height[k] + 1)
    slots, ends = [], []
    for h in range(max(height) + 1):
        items = []
        for k in range(nv):
            if height[k] != h:
                continue
            i = par[k]
            while i >= 0:
                j = i
                while j >= 0:
                    items.append((k, i, j))
                    j = par[j]
                i = par[i]
        if not items:
            continue
        for s in range(0, len(items), WAVE):
            slots.append(items[s:s + WAVE])
        ends.append(len(slots) - 1)
    return slots, ends


def tree_solve(A, slots, b):
    """The kernel's arithmetic on a copy of the lower triangle of A."""
    T = np.tril(A).copy()
    for sl in slots:
        upd = [(i, j, -T[k, i] * (T[k, j] / T[k, k])) for (k, i, j) in sl]
        for i, j, v in upd:  # LDS float atomics after the slot's reads
            T[i, j] += v
    n = len(b)
    dinv = 1.0 / np.diag(T)
    u = b * dinv  # lane i: y_i / D_i
    for k in range(n - 1, -1, -1):
        for i in range(k):
            u[i] -= T[k, i] * dinv[i] * u[k]
    v = u.copy()  # lane k: w_k - sum_i A[k][i] / D_k x_i
    for i in range(n):
        for k in range(i + 1, n):
            v[k] -= T[k, i] * dinv[k] * v[i]
    return v


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(ROOT, "assets", "*.npz"))),
                         ids=lambda p: os.path.basename(p))
def test_tree_ldl_solves_tree_sparse_spd(path):
    par = [int(p) for p in np.load(path, allow_pickle=False)["dof_parentid"]]
    nv = len(par)
    slots, ends = ldl_slots(par)
    assert len(slots) <= DX_LDL_SLOTS, "the scene would fall back to the dense solver"
    # a level's dofs are never ancestors of one another, and never read its targets
    anc = [set() for _ in range(nv)]
    for k in range(nv):
        i = par[k]
        while i >= 0:
            anc[k].add(i)
            i = par[i]
    start = 0
    for e in ends:
        level = [it for sl in slots[start:e + 1] for it in sl]
        ks = {k for k, _, _ in level}
        assert all(not (anc[a] & ks) for a in ks)  # no dof of the level is another's ancestor
        assert not ({i for _, i, _ in level} & ks)  # the rows it writes are not the rows it reads
        start = e + 1
    rng = np.random.default_rng(nv)
    L = np.eye(nv)
    for k in range(nv):
        for i in anc[k]:
            L[k, i] = rng.normal(scale=0.5)
    M = L.T @ np.diag(rng.uniform(0.2, 3.0, nv)) @ L
    for _ in range(3):
        b = rng.normal(size=nv)
        d = rng.uniform(0.0, 0.5, nv)  # the Euler step's h * damping
        x = tree_solve(M + np.diag(d), slots, b)
        np.testing.assert_allclose(x, np.linalg.solve(M + np.diag(d), b), rtol=1e-9, atol=1e-9)
