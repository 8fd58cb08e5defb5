"""Dev check: persistent GJ reduced solve accuracy for given sizes and forced
column-block widths (SFM_GJ_CB)."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + '/structure-from-motion-_amd')
import numpy as np, _sfmcore as c
for spec in sys.argv[1:]:
    n, cb = (int(v) for v in spec.split(":"))
    os.environ["SFM_GJ_CB"] = str(cb)
    rng = np.random.default_rng(n)
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    S = (Q * np.logspace(0, 4, n)) @ Q.T
    S = 0.5 * (S + S.T)
    b = rng.standard_normal(n)
    xr = np.linalg.solve(S, b)
    errs = []
    for _ in range(3):
        x = c.reduced_solve(S, b)
        errs.append(np.abs(x - xr).max() / np.abs(xr).max())
    bad = np.where(np.abs(x - xr) > 1e-9 * np.abs(xr).max())[0]
    print(f"n={n} cb={cb}: rel err {['%.2e' % e for e in errs]} bad rows {bad[:8]} ... {len(bad)} tiles {sorted(set((bad // 16).tolist()))[:20]}", flush=True)
