"""One cfg4 (or argv[1]) BA problem, argv[2] (default 20, bench.py's
timed region) fixed LM iterations from x0, for rocprofv3 kernel-trace / PMC
runs (tools/profile_round.sh; per-iteration traffic = totals / iterations)."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("SFM_PKG") or R + '/structure-from-motion-_amd')  # SFM_PKG: an A/B build's directory
import numpy as np, _sfmcore as c, sfm_synthetic as syn
p = syn.ba_problem_cfg(sys.argv[1] if len(sys.argv) > 1 else "cfg4", dense=False)
n_it = int(sys.argv[2]) if len(sys.argv) > 2 else 20
conv = len(sys.argv) > 3 and sys.argv[3] == "conv"  # converged solve (twice: warm, then traced)
cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
prob = c.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF)
if conv:
    prob.solve(max_iterations=n_it)
    prob.reset()
rep = prob.solve(max_iterations=n_it, fixed_iterations=not conv)
print(rep["t_loop_ms"] / n_it, rep["accepted"])
print(rep)
prob.close()
