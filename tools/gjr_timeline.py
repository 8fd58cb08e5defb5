"""Dev probe (round 4): SFM_GJ_DEBUG stamps of one row-distributed persistent
reduced solve (gjr_solve.hpp) on a dense SPD n x n system, printed as the
critical path per pivot: P_{p-1} arriving at owner p, G_p published, the
chain, P_p published, and the hop to owner p + 1; with owners listed, each
one's own stamps over the steps before its pivot.
Usage: gjr_timeline.py [n [owner,owner,...]]"""
import os, sys, ctypes
os.environ["SFM_GJ_DEBUG"] = "1"
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + '/structure-from-motion-_amd')
import numpy as np, _sfmcore as c
n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
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
PIN, GCRIT, CH0, CH1, PPUB, GHOLD, UDONE, GREM, PLW, GRDY, HPRDY = range(11)
print(f"n={n} nT={nT}   (us from the first stamp)")
print("   p  P_{p-1}@p   G_p pub   chain0   chain1   P_p pub | hop->p+1   step")
prev = None
for p in range(nT):
    pin = d[p, p - 1, PIN] if p else float("nan")
    gcr = d[p, p - 1, GCRIT] if p else float("nan")
    c0, c1, pp = d[p, p, CH0], d[p, p, CH1], d[p, p, PPUB]
    hop = d[p + 1, p, PIN] - pp if p + 1 < nT else float("nan")
    step = pp - prev if prev is not None else float("nan")
    prev = pp
    print(f"{p:4d} {pin:9.2f} {gcr:9.2f} {c0:8.2f} {c1:8.2f} {pp:9.2f} | {hop:8.2f} {step:7.2f}")
fin = ["start", "prologue", "w0end", "arrived"]
for w in range(nT):
    if w < 2 or w >= nT - 2:
        print(f"owner {w:3d}: " + " ".join(f"{fin[k]}={d[w, nT, k]:8.2f}" for k in range(len(fin))))
steps = np.diff(d[np.arange(nT), np.arange(nT), PPUB])
print(f"mean step {np.nanmean(steps):.3f} us, median {np.nanmedian(steps):.3f}")
if len(sys.argv) > 2:
    for r in map(int, sys.argv[2].split(",")):
        print(f"owner {r}: step  Ppub@p   P_p@W0  pdoneOK  Hpready   G_hold  greadyW0   U0done")
        for p in range(0 if os.environ.get("GJR_ALL") else max(0, r - 8), r):
            print(f"   {p:4d} " + " ".join(f"{d[i, p, k]:8.2f}" for i, k in ((p, PPUB), (r, PIN), (r, PLW), (r, HPRDY), (r, GHOLD), (r, GRDY), (r, UDONE))))
