"""CPU restatement of the matrix-core sweep solve (dx_device.h mfma_sweep_solve30) that
the Newton step uses for its dense Hessian solve H dir = -grad when nv <= 30 (MuJoCo's
mj_solveNewton factorises H by Cholesky [3P]; the sweep solves the same system).

The bordered 32 x 32 matrix [[A, b], [b^T, 0]] (b in row/column 31, identity padding
between) is swept two pivots at a time: the pivot rows and columns are zeroed, then
S <- S - V W V^T with V the pivot columns (-I in the pivot rows) and W the inverse 2 x 2
pivot block; column 31 then holds A^-1 b.  Run here in fp32, the kernel's arithmetic
type, on SPD systems shaped like the Newton Hessian (M + J^T D J, wide dynamic range).
"""
import numpy as np
import pytest


def sweep_solve(A, b, dtype=np.float32):
    n = len(b)
    assert n <= 30
    S = np.eye(32, dtype=dtype)
    S[:n, :n] = A
    S[31, :n] = b
    S[:n, 31] = b
    S[31, 31] = 0
    for k in range(0, 30, 2):
        if k >= n:
            break
        p00, p10, p11 = S[k, k], S[k + 1, k], S[k + 1, k + 1]
        idet = dtype(1) / (p00 * p11 - p10 * p10)
        W = np.array([[p11 * idet, -p10 * idet], [-p10 * idet, p00 * idet]], dtype=dtype)
        V = S[:, [k, k + 1]].copy()
        V[k] = [-1, 0]
        V[k + 1] = [0, -1]
        S[[k, k + 1], :] = 0
        S[:, [k, k + 1]] = 0
        S = (S - V @ (W @ V.T)).astype(dtype)
    return S[:n, 31]


def hessian_like(rng, n, nefc, spread):
    """M (SPD, inertia scale 1e-3..1) + J^T D J with D over `spread` decades."""
    X = rng.standard_normal((n, n)) * 0.03
    M = X @ X.T + np.diag(10 ** rng.uniform(-3, 0, n))
    J = rng.standard_normal((nefc, n))
    D = 10 ** rng.uniform(0, spread, nefc)
    return M + J.T @ (D[:, None] * J)


@pytest.mark.parametrize("n", [1, 2, 7, 24, 29, 30])
def test_sweep_solves_spd(n):
    rng = np.random.default_rng(n)
    for _ in range(20):
        X = rng.standard_normal((n, n + 3))
        A = X @ X.T + 0.1 * np.eye(n)
        b = rng.standard_normal(n)
        x = sweep_solve(A, b)
        ref = np.linalg.solve(A, b)
        assert np.abs(x - ref).max() <= 1e-4 * np.abs(ref).max()


@pytest.mark.parametrize("nefc", [0, 12, 40, 70])
def test_sweep_matches_cholesky_on_newton_hessians(nefc):
    """Residual of the fp32 sweep within a small factor of the fp32 Cholesky solve's
    (the kernel's previous path, mfma_chol_solve32) on Hessian-like systems."""
    rng = np.random.default_rng(100 + nefc)
    worse = []
    for _ in range(20):
        H = hessian_like(rng, 30, nefc, 4.0)
        g = rng.standard_normal(30)
        x = sweep_solve(H.astype(np.float32), g.astype(np.float32)).astype(np.float64)
        L = np.linalg.cholesky(H.astype(np.float32))
        y = np.linalg.solve(L, g.astype(np.float32))
        xc = np.linalg.solve(L.T, y).astype(np.float64)
        ref = np.linalg.solve(H, g)
        err_s = np.abs(x - ref).max() / np.abs(ref).max()
        err_c = np.abs(xc - ref).max() / np.abs(ref).max()
        worse.append(err_s / max(err_c, 1e-12))
        assert err_s < max(1e-4, 10 * err_c)
    assert np.median(worse) < 4.0


def sweep_inverse(A, dtype=np.float32):
    """dx_device.h mfma_sweep_inverse30: every pivot pair swept with its whole rows and
    columns zeroed first; the result is -A^-1."""
    n = len(A)
    S = np.eye(32, dtype=dtype)
    S[:n, :n] = A
    for k in range(0, 30, 2):
        if k >= n:
            break
        p00, p10, p11 = S[k, k], S[k + 1, k], S[k + 1, k + 1]
        idet = dtype(1) / (p00 * p11 - p10 * p10)
        W = np.array([[p11 * idet, -p10 * idet], [-p10 * idet, p00 * idet]], dtype=dtype)
        V = S[:, [k, k + 1]].copy()
        V[k] = [-1, 0]
        V[k + 1] = [0, -1]
        S[[k, k + 1], :] = 0
        S[:, [k, k + 1]] = 0
        S = (S - V @ (W @ V.T)).astype(dtype)
    return -S[:n, :n]


@pytest.mark.parametrize("n", [2, 7, 24, 30])
def test_sweep_inverse_of_mass_matrices(n):
    """The CG solver's M^-1 (one sweep per solve, then a product per iteration) equals
    the inverse, and M^-1 g agrees with the sweep solve of the same system in fp32."""
    rng = np.random.default_rng(200 + n)
    for _ in range(20):
        M = hessian_like(rng, n, 0, 0.0)
        Mi = sweep_inverse(M.astype(np.float32)).astype(np.float64)
        ref = np.linalg.inv(M)
        assert np.abs(Mi - ref).max() <= 1e-4 * np.abs(ref).max()
        assert np.abs(Mi - Mi.T).max() <= 1e-5 * np.abs(ref).max()
        g = rng.standard_normal(n)
        x = (Mi.astype(np.float32) @ g.astype(np.float32)).astype(np.float64)
        xs = sweep_solve(M.astype(np.float32), g.astype(np.float32)).astype(np.float64)
        xr = np.linalg.solve(M, g)
        assert np.abs(x - xr).max() <= max(3 * np.abs(xs - xr).max(), 1e-5 * np.abs(xr).max())
