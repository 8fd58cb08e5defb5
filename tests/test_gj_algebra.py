"""CPU restatement of the reduced camera solve's algebra (gjr_solve.hpp,
round 4): block Gauss-Jordan with Cholesky pivots, laid out by tile rows --
owner r keeps its row's live tiles (j <= r before its pivot, j > p after),
forms G_r = A_rp L_p^-T by a product with the published inverse factor (no
triangular solve), imports A_pj = L_p G_j^T at its own pivot, and ends with
x_r = L_r^-T L_r^-1 b_r, no back substitution.  This checks the dataflow the
kernel implements (which tile is updated with which G at which step) against
LAPACK; the GPU kernel itself is checked in test_gpu_parity.py
(test_reduced_solve)."""
import numpy as np
import pytest


def gj_rows(A, b, TL=16):
    n = A.shape[0]
    nT = (n + TL - 1) // TL
    N = nT * TL
    Ap = np.eye(N)
    Ap[:n, :n] = A
    bp = np.zeros(N)
    bp[:n] = b
    T = lambda i: slice(i * TL, (i + 1) * TL)  # noqa: E731
    tiles = {r: {j: Ap[T(r), T(j)].copy() for j in range(r + 1)} for r in range(nT)}  # lower part
    bb = {r: bp[T(r)].copy() for r in range(nT)}
    Linv = {}
    for p in range(nT):
        L = np.linalg.cholesky(tiles[p][p])  # the chain, with the b row and the identity as panel rows
        Li = np.linalg.inv(L)
        Linv[p] = Li
        y = Li @ bb[p]
        G = {r: tiles[r][p] @ Li.T for r in range(nT) if r != p}  # every owner, from P_p = {L_p^-1, y_p}
        for j in range(p + 1, nT):  # the pivot owner's import of its row right of the diagonal
            tiles[p][j] = L @ G[j].T
        for r in range(nT):
            if r == p:
                continue
            hi = r if r > p else nT - 1  # unpivoted: (p, r]; pivoted: (p, nT)
            for j in range(p + 1, hi + 1):
                tiles[r][j] -= G[r] @ G[j].T
            bb[r] -= G[r] @ y
            del tiles[r][p]  # column p is eliminated from every other row
    x = np.concatenate([Linv[r].T @ (Linv[r] @ bb[r]) for r in range(nT)])
    return x[:n]


@pytest.mark.parametrize("n", [1, 6, 16, 40, 300])
def test_row_distributed_gauss_jordan_matches_lapack(n):
    rng = np.random.default_rng(n)
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    S = (Q * np.logspace(0, 4, n)) @ Q.T
    S = 0.5 * (S + S.T)
    b = rng.standard_normal(n)
    x, xr = gj_rows(S, b), np.linalg.solve(S, b)
    assert np.abs(x - xr).max() <= 1e-11 * np.abs(xr).max()
