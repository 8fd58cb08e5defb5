"""numpy model of gj_solve.hpp's block Gauss-Jordan (design check, not the
kernel): the kept tiles, the mirror skip and the import, per workgroup
(column block cb, segment s) with a diagonal replica per owned column."""
import numpy as np


def gj_solve(A, b, T=16, SR=4, CB=4):
    n = A.shape[0]
    nT = (n + T - 1) // T
    nsp = nT * T
    M = np.eye(nsp)
    M[:n, :n] = np.tril(A) + np.tril(A, -1).T   # lower triangle mirrored
    bb = np.zeros(nsp)
    bb[:n] = b
    tile = lambda X, i, j: X[i * T:(i + 1) * T, j * T:(j + 1) * T]
    own = {(i, j): tile(M, i, j).copy() for i in range(nT) for j in range(nT)}
    D = {j: tile(M, j, j).copy() for j in range(nT)}
    bj = {j: bb[j * T:(j + 1) * T].copy() for j in range(nT)}    # b replicas
    ob = {i: bb[i * T:(i + 1) * T].copy() for i in range(nT)}    # b of the rows
    Ls = {}
    for p in range(nT):
        L = np.linalg.cholesky(D[p])
        Ls[p] = L
        G = {i: np.linalg.solve(L, own[(i, p)].T).T for i in range(nT)}   # A_ip L^-T
        y = np.linalg.solve(L, bj[p])
        for j in range(p + 1, nT):
            for i in range(nT):
                if i == p:
                    own[(i, j)] = L @ G[j].T          # import
                elif p < i < j:
                    continue                          # mirror, not kept
                else:
                    own[(i, j)] = own[(i, j)] - G[i] @ G[j].T
            D[j] = D[j] - G[j] @ G[j].T
            bj[j] = bj[j] - G[j] @ y
        for i in range(nT):
            if i != p:
                ob[i] = ob[i] - G[i] @ y
    x = np.concatenate([np.linalg.solve(Ls[i].T, np.linalg.solve(Ls[i], ob[i])) for i in range(nT)])
    return x[:n]


if __name__ == "__main__":
    rng = np.random.default_rng(0)
    for n in (6, 36, 300, 304, 500):
        B = rng.standard_normal((n, n + 10))
        A = B @ B.T + 0.1 * np.eye(n)
        b = rng.standard_normal(n)
        x = gj_solve(A, b)
        xr = np.linalg.solve(A, b)
        print(n, np.abs(x - xr).max() / np.abs(xr).max())
