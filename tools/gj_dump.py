"""Dev check: compare the panels a persistent GJ solve published (sfm_gj_dump)
with tools/gj_model.py's panels; prints the first deviating (panel, segment)."""
import os, sys, ctypes
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + '/structure-from-motion-_amd')
sys.path.insert(0, R + '/tools')
import numpy as np, _sfmcore as c
n, cb = (int(v) for v in sys.argv[1].split(":"))
os.environ["SFM_GJ_CB"] = str(cb)
rng = np.random.default_rng(n)
Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
A = (Q * np.logspace(0, 4, n)) @ Q.T
A = 0.5 * (A + A.T)
b = rng.standard_normal(n)
x = c.reduced_solve(A, b)
T = 16
nT = (n + 15) // 16
nsp = nT * T
nseg = (nT + 3) // 4
G = np.zeros((nT, nsp, 16)); L = np.zeros((nT, nseg, 256)); Y = np.zeros((nT, nseg, 16))
P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
rc = c._lib.sfm_gj_dump(P(G), P(L), P(Y), nT, nseg, 0)
print("dump rc", rc)
# model panels
M = np.eye(nsp); M[:n, :n] = np.tril(A) + np.tril(A, -1).T
bb = np.zeros(nsp); bb[:n] = b
tile = lambda X, i, j: X[i*T:(i+1)*T, j*T:(j+1)*T]
own = {(i, j): tile(M, i, j).copy() for i in range(nT) for j in range(nT)}
D = {j: tile(M, j, j).copy() for j in range(nT)}
bj = {j: bb[j*T:(j+1)*T].copy() for j in range(nT)}
shown = 0
for p in range(nT):
    Lm = np.linalg.cholesky(D[p])
    Gm = {i: np.linalg.solve(Lm, own[(i, p)].T).T for i in range(nT)}
    y = np.linalg.solve(Lm, bj[p])
    for s in range(nseg):
        eL = np.abs(L[p, s].reshape(16, 16) - Lm).max() / np.abs(Lm).max()
        eY = np.abs(Y[p, s] - y).max() / max(1e-300, np.abs(y).max())
        rows = [i for i in range(s*4, min(nT, s*4+4)) if i != p]
        eG = max([np.abs(G[p, i*T:(i+1)*T] - Gm[i]).max() / max(1e-300, np.abs(Gm[i]).max()) for i in rows] or [0])
        if (eL > 1e-8 or eY > 1e-8 or eG > 1e-8) and shown < 25:
            print(f"panel {p} seg {s}: L {eL:.1e} y {eY:.1e} G {eG:.1e}")
            shown += 1
    for j in range(p + 1, nT):
        for i in range(nT):
            if i == p: own[(i, j)] = Lm @ Gm[j].T
            elif p < i < j: continue
            else: own[(i, j)] = own[(i, j)] - Gm[i] @ Gm[j].T
        D[j] = D[j] - Gm[j] @ Gm[j].T
        bj[j] = bj[j] - Gm[j] @ y
print("done")
