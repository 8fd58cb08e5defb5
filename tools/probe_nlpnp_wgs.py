"""Dev probe (round 3): multi-workgroup NonlinearPnP -- the bench's scene
(5000 points, 30 % outliers, from the PnP-RANSAC winner) and 20k / 100k
clean points, per SFM_NLPNP_WGS setting: GPU wall time per call (median of
7), kernel time (HIP events), info, and the distance from the C oracle and
from the one-workgroup result."""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R + '/structure-from-motion-_amd', R + '/oracle']
import random
import numpy as np, _sfmcore as core, sfm_synthetic as syn, oracle as O
K = syn.K_REF
x1, x2, idx, m = syn.two_view(n=1000, seed=1)
wgs = [int(a) for a in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["1", "2", "4", "5", "8", "16"])]


def scene(n, outl):
    rng = np.random.default_rng(12)
    Xw = np.column_stack([rng.uniform(-3, 3, n), rng.uniform(-2, 2, n), rng.uniform(5, 12, n)])
    u = (K @ (m["R2"] @ (Xw - m["C2"]).T)).T
    xw = u[:, :2] / u[:, 2:3] + rng.normal(0, 0.5, (n, 2))
    if outl:
        o = rng.choice(n, n * 3 // 10, replace=False)
        xw[o] = rng.uniform(0, 1000, (len(o), 2))
    return Xw, xw


for n, outl in ((5000, True), (20000, False), (100000, False)):
    Xw, xw = scene(n, outl)
    random.seed(1)
    ps = core.sample_table(n, 4, 16384)
    _, _, C0, R0, _, _ = core.pnp_ransac(Xw, xw, K, ps, 8.0)
    Co, Ro, io = O.nonlinear_pnp(Xw, xw, K, C0, R0)
    base = None
    for nb in wgs:
        os.environ["SFM_NLPNP_WGS"] = str(nb)
        core.nonlinear_pnp(Xw, xw, K, C0, R0)
        tl = []
        for _ in range(7):
            t = time.perf_counter()
            C, Rr, info = core.nonlinear_pnp(Xw, xw, K, C0, R0)
            tl.append(time.perf_counter() - t)
        core.set_call_timing(True)
        core.nonlinear_pnp(Xw, xw, K, C0, R0)
        tk = core.last_timings()[1]
        core.set_call_timing(False)
        if base is None:
            base = (C, Rr)
        print(f"n={n} wgs={nb}: call {np.median(tl)*1e3:.3f} ms kernel {tk:.3f} ms info {info} (oracle {io}) "
              f"|dC| oracle {np.abs(C - Co).max():.2e} |dR| {np.abs(Rr - Ro).max():.2e}; "
              f"vs 1 wg |dC| {np.abs(C - base[0]).max():.2e}", flush=True)
