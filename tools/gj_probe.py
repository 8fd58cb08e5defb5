"""Dev probe (round 3): the persistent Gauss-Jordan reduced solve against the
multi-launch Cholesky (SFM_SOLVE=chol) -- accuracy on dense SPD systems and
the BA solve at cfg4 / cfg5 (20 fixed LM iterations, per-phase kernel times)."""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + '/structure-from-motion-_amd')
import numpy as np, _sfmcore as c, sfm_synthetic as syn


def spd(n, seed, cond=1e4):
    rng = np.random.default_rng(seed)
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    S = (Q * np.logspace(0, np.log10(cond), n)) @ Q.T
    return 0.5 * (S + S.T), rng.standard_normal(n)


def run(mode, fn):
    if mode == "chol":
        os.environ["SFM_SOLVE"] = "chol"
    else:
        os.environ.pop("SFM_SOLVE", None)
    return fn()


for n in [int(a) for a in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["6", "48", "300", "1200"])]:
    S, b = spd(n, n)
    xr = np.linalg.solve(S, b)
    for mode in ("gj", "chol"):
        t = time.perf_counter()
        x = run(mode, lambda: c.reduced_solve(S, b))
        dt = time.perf_counter() - t
        print(f"reduced_solve n={n} {mode}: rel err {np.abs(x - xr).max() / np.abs(xr).max():.2e} ({dt*1e3:.1f} ms)", flush=True)

for name in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["cfg4"]):
    p = syn.ba_problem_cfg(name, dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    res = {}
    for mode in ("gj", "chol"):
        def one():
            prob = c.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF)
            prob.solve(max_iterations=3, fixed_iterations=True)
            prob.reset()
            t = time.perf_counter()
            rep = prob.solve(max_iterations=20, fixed_iterations=True)
            dt = time.perf_counter() - t
            prob.reset()
            prob.set_timing()
            prob.solve(max_iterations=20, fixed_iterations=True)
            kt = prob.kernel_times()
            prob.reset()
            prob.set_timing(False)
            conv = prob.solve(max_iterations=100)
            prob.close()
            return rep, dt, kt, conv
        rep, dt, kt, conv = run(mode, one)
        res[mode] = rep
        print(f"{name} {mode}: {dt / 20 * 1e3:.4f} ms/step acc {rep['accepted']} cost {rep['cost']:.12e} "
              f"conv it {conv['iterations']} acc {conv['accepted']} st {conv['status']} cost {conv['cost']:.12e}",
              {k: round(v, 4) for k, v in kt.items()}, flush=True)
