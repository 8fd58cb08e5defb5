"""Dev probe (round 6): SFM_GJ_DEBUG stamps of one reduced solve with the
pivot workgroup (gjr_solve.hpp, PWG) on a dense SPD n x n system: per pivot
q, when wave C had window q (stall = its wait after P_{q-1}), G_q out, the
chain, P_q out, and when wave A had owner q's window record and handed the
window on (negative slack = wave C waited for it).
Usage: gjp_timeline.py [n [reps]]"""
import os, sys, ctypes
os.environ["SFM_GJ_DEBUG"] = "1"
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + '/structure-from-motion-_amd')
import numpy as np, _sfmcore as c
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1200
rng = np.random.default_rng(n)
Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
S = (Q * np.logspace(0, 4, n)) @ Q.T
S = 0.5 * (S + S.T)
b = rng.standard_normal(n)
for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    x = c.reduced_solve(S, b)
print("max rel err vs LAPACK", np.abs(x - np.linalg.solve(S, b)).max() / np.abs(x).max())
nT = (n + 15) // 16
buf = np.zeros(256 * 129 * 16, dtype=np.int64)
c._lib.sfm_gj_debug(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), ctypes.c_int64(buf.size))
d = buf[:(nT + 1) * (nT + 1) * 16].reshape(nT + 1, nT + 1, 16).astype(np.float64)
t0 = d[d > 0].min()
d = np.where(d > 0, (d - t0) * 0.01, np.nan)  # us (100 MHz)
WIN, GPUB, CH0, CH1, PPUB, AWIN, AOUT, BPUB = range(8)
pw = d[nT]
print(f"n={n} nT={nT}   (us from the first stamp)")
print("   q   C:win  stall   G out  chain0  chain1   P out   step |  A:rec  A:out  slack")
prev = None
for q in range(nT):
    stall = pw[q, WIN] - prev if prev is not None else float("nan")
    step = pw[q, PPUB] - prev if prev is not None else float("nan")
    slack = (prev if prev is not None else pw[q, WIN]) - pw[q, AOUT]
    print(f"{q:4d} {pw[q, WIN]:7.2f} {stall:6.2f} {pw[q, GPUB]:7.2f} {pw[q, CH0]:7.2f} {pw[q, CH1]:7.2f} "
          f"{pw[q, PPUB]:7.2f} {step:6.2f} | {pw[q, AWIN]:7.2f} {pw[q, AOUT]:6.2f} {slack:6.2f}")
    prev = pw[q, PPUB]
# the look-ahead stages of the pivot workgroup: per window, when its record
# (or the link from the early stage) was in and each of its steps done
LIN, STEP = 8, 9
print("   q   rec   d4done  d3done | link  d2done   out | C:win[q-1]")
for q in range(2, min(nT, 30)):
    print(f"{q:4d} {pw[q, AWIN]:7.2f} {pw[q, STEP + 4]:7.2f} {pw[q, STEP + 3]:7.2f} | {pw[q, LIN]:6.2f} "
          f"{pw[q, STEP + 2]:7.2f} {pw[q, AOUT]:6.2f} | {pw[q - 1, WIN]:7.2f}")
steps = np.diff(pw[:nT, PPUB])
chain = pw[:nT, CH1] - pw[:nT, CH0]
print(f"mean step {np.nanmean(steps):.3f} us, median {np.nanmedian(steps):.3f}, chain median {np.nanmedian(chain):.3f}")
fin = ["start", "prologue", "w0end", "arrived"]
ends = [d[w, nT, 2] for w in range(nT)]
print(f"last P out {pw[nT - 1, PPUB]:.2f} us, last owner x {np.nanmax(ends):.2f} us, "
      f"last arrival {np.nanmax([d[w, nT, 3] for w in range(nT)]):.2f} us")
# owners: per step p, when P_p left the pivot workgroup, reached owner r's W0,
# the holder had it (pready) and published G_r,p, the remote G's of W0's
# window tiles arrived, W0 had the holder's G, U0 finished the step; W = the
# window shipped (step r - LA - 1)
PIN, GCRIT, GHOLD, UDONE, GREM, GRDY, HPRDY = 0, 1, 5, 6, 7, 9, 10
for r in [int(v) for v in (sys.argv[3].split(",") if len(sys.argv) > 3 else [])]:
    print(f"owner {r}:    p   Pout  P@W0  Hprdy  Ghold   Grem   Grdy  U0done")
    for p in range(0, min(r, nT)):
        row = [pw[p, PPUB], d[r, p, PIN], d[r, p, HPRDY], d[r, p, GHOLD], d[r, p, GREM], d[r, p, GRDY], d[r, p, UDONE]]
        print(f"        {p:4d} " + " ".join(f"{v:6.1f}" for v in row) + (f"  W {d[r, p, GCRIT]:.1f}" if not np.isnan(d[r, p, GCRIT]) else ""))
