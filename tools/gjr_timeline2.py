"""Dev probe (round 5): stamps of one row-distributed reduced solve with two
pivots per hop (gjr_solve.hpp built with -DGJR_STAMPS=1, e.g. the package in
abso/stamps), on a dense SPD n x n system.  Per owner r: when W0 reached its
critical step (ready), the row-state record R_{r-1} arrived, P_{r-2} arrived,
the recomputed pivot r - 1's chain, G_r of step r - 1, its own chain, P_r
published, and the hop of P_r to owner r + 2; T2 = A_r,r-2 from its U wave.
Usage: gjr_timeline2.py PKGDIR [n]"""
import os, sys, ctypes
os.environ["SFM_GJ_DEBUG"] = "1"
sys.path.insert(0, sys.argv[1])
import numpy as np, _sfmcore as c
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1200
rng = np.random.default_rng(n)
Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
S = (Q * np.logspace(0, 4, n)) @ Q.T
S = 0.5 * (S + S.T)
b = rng.standard_normal(n)
for _ in range(3):
    x = c.reduced_solve(S, b)
print("max rel err vs LAPACK", np.abs(x - np.linalg.solve(S, b)).max() / np.abs(x).max())
nT = (n + 15) // 16
buf = np.zeros(256 * 129 * 16, dtype=np.int64)
c._lib.sfm_gj_debug(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), ctypes.c_int64(buf.size))
d = buf[:nT * (nT + 1) * 16].reshape(nT, nT + 1, 16).astype(np.float64)
t0 = d[d > 0].min()
d = np.where(d > 0, (d - t0) * 0.01, np.nan)  # us (100 MHz)
PIN, GCRIT, CH0, CH1, PPUB, GHOLD, UDONE, GREM, PLW, GRDY, HPRDY, RIN, T2, READY, GC = range(15)
print(f"n={n} nT={nT}   (us from the first stamp)")
print("   r    T2@r-3    ready     R_in   P_r-2in  ch(r-1)0 ch(r-1)1      gc  ch(r)0  ch(r)1   P_r pub | hop->r+2  period")
g = lambda r, p, k: d[r, p, k] if 0 <= p <= nT and 0 <= r < nT else float("nan")
for r in range(nT):
    hop = g(r + 2, r, PIN) - g(r, r, PPUB) if r + 2 < nT else float("nan")
    per = g(r, r, PPUB) - g(r - 2, r - 2, PPUB) if r >= 2 else float("nan")
    print(f"{r:4d} {g(r, r-3, T2):9.2f} {g(r, r-2, READY):8.2f} {g(r, r-2, RIN):8.2f} {g(r, r-2, PIN):8.2f} "
          f"{g(r, r-1, CH0):8.2f} {g(r, r-1, CH1):8.2f} {g(r, r-1, GC):8.2f} {g(r, r, CH0):7.2f} {g(r, r, CH1):7.2f} "
          f"{g(r, r, PPUB):9.2f} | {hop:8.2f} {per:7.2f}")
fin = ["start", "prologue", "w0end", "arrived"]
for w in (0, 1, nT - 2, nT - 1):
    print(f"owner {w:3d}: " + " ".join(f"{fin[k]}={d[w, nT, k]:8.2f}" for k in range(len(fin))))
pp = d[np.arange(nT), np.arange(nT), PPUB]
print(f"P_r published: mean step {np.nanmean(np.diff(pp)):.3f} us, median {np.nanmedian(np.diff(pp)):.3f}")
