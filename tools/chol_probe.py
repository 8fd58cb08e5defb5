"""Dev probe: cfg4 (or argv[1]) BA, 20 fixed LM iterations: prints the final
cost (hex, for a bitwise comparison between reduced-solve variants) and the
per-iteration kernel times."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + '/structure-from-motion-_amd')
import numpy as np, _sfmcore as c, sfm_synthetic as syn
p = syn.ba_problem_cfg(sys.argv[1] if len(sys.argv) > 1 else "cfg4", dense=False)
cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
prob = c.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF)
prob.set_timing()
prob.solve(max_iterations=3, fixed_iterations=True)
prob.reset()
rep = prob.solve(max_iterations=20, fixed_iterations=True)
kt = prob.kernel_times()
print(float(rep["cost"]).hex(),
      rep["accepted"], round(rep["t_loop_ms"] / 20, 4), {k: round(v, 4) for k, v in kt.items()}, flush=True)
prob.close()
