"""Dev probe: NonlinearPnP on the bench's 5000-point scene (and 20k / 100k
points): GPU wall time per call, info, and the C oracle's result for
comparison."""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R + '/structure-from-motion-_amd', R + '/oracle']
import numpy as np, _sfmcore as core, sfm_synthetic as syn, oracle as O
K = syn.K_REF
_, _, _, m = syn.two_view(n=10, seed=6, outlier_frac=0.2)
for n in (5000, 20000, 100000):
    rng = np.random.default_rng(12)
    Xw = np.column_stack([rng.uniform(-3, 3, n), rng.uniform(-2, 2, n), rng.uniform(5, 12, n)])
    u = (K @ (m["R2"] @ (Xw - m["C2"]).T)).T
    xw = u[:, :2] / u[:, 2:3] + rng.normal(0, 0.5, (n, 2))
    C0 = m["C2"] + 0.05
    from scipy.spatial.transform import Rotation
    R0 = Rotation.from_rotvec([0.03, -0.13, 0.02]).as_matrix()
    core.nonlinear_pnp(Xw, xw, K, C0, R0)
    t = time.perf_counter()
    for _ in range(5):
        C, Rr, info = core.nonlinear_pnp(Xw, xw, K, C0, R0)
    tg = (time.perf_counter() - t) / 5
    t = time.perf_counter()
    Co, Ro, io = O.nonlinear_pnp(Xw, xw, K, C0, R0)
    tc = time.perf_counter() - t
    print(n, "gpu ms %.3f" % (tg * 1e3), "info", info, "oracle ms %.3f" % (tc * 1e3), "info", io,
          "|dC| %.2e |dR| %.2e" % (np.abs(C - Co).max(), np.abs(Rr - Ro).max()), flush=True)
