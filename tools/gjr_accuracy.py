"""Dev probe (round 4): accuracy of the reduced solve (sfm_reduced_solve) on
SPD systems of condition 1e4 against LAPACK, three calls each; argv[1]: the
package directory to load libsfmcore.so from (default: the repo's)."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, sys.argv[1] if len(sys.argv) > 1 else R + '/structure-from-motion-_amd')
import numpy as np, _sfmcore as c
print("lib:", c._lib._name)
for n in (40, 150, 300, 600, 1200, 1800):
    rng = np.random.default_rng(n)
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    S = (Q * np.logspace(0, 4, n)) @ Q.T
    S = 0.5 * (S + S.T)
    b = rng.standard_normal(n)
    xr = np.linalg.solve(S, b)
    errs = [float(np.abs(c.reduced_solve(S, b) - xr).max() / np.abs(xr).max()) for _ in range(3)]
    print(n, " ".join(f"{e:.2e}" for e in errs), flush=True)
