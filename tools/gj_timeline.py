"""Dev probe: SFM_GJ_DEBUG stamps of one persistent reduced solve (dense SPD
n x n), printed as a per-pivot timeline of the critical workgroups."""
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
nT = (n + 15) // 16
nseg = (nT + 3) // 4
cb = 4 if ((nT + 3) // 4) * nseg <= 256 else 8
ncb = (nT + cb - 1) // cb
buf = np.zeros(256 * 129 * 16, dtype=np.int64)
c._lib.sfm_gj_debug(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), ctypes.c_int64(buf.size))
d = buf[:ncb * nseg * (nT + 1) * 16].reshape(ncb * nseg, nT + 1, 16).astype(np.float64)
t0 = d[d > 0].min()
d = np.where(d > 0, (d - t0) * 0.01, np.nan)  # us (100 MHz)
names = ["cst", "chain", "pub", "load0", "loaded", "gm", "phA", "phB", "w0buf", "w0gst", "w0lds", "w0drain", "agj", "acst", "amma", "abb"]
print(f"n={n} nT={nT} nseg={nseg} cb={cb} grid={ncb*nseg}")
for p in range(nT):
    cbp, sp = p // cb, p // 4
    w = cbp * nseg + sp  # the pivot-row owner
    row = d[w, p]
    other = [cbp * nseg + s for s in range(nseg) if s != sp]
    pubs = [d[o, p, 2] for o in other]
    print(f"p={p:3d} owner wg {w:3d}: " + " ".join(f"{names[k]}={row[k]:7.2f}" for k in range(16)) +
          f" | others pub max {np.nanmax(pubs) if pubs else float('nan'):8.2f}")
fin = ["start", "prologue", "finwait", "finsolved", "arrived", "epilogue"]
for w in range(ncb * nseg):
    if w < nseg or w >= (ncb - 1) * nseg:
        print(f"wg {w:3d}: " + " ".join(f"{fin[k]}={d[w, nT, k]:7.2f}" for k in range(6)))
