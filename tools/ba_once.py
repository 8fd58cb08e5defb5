"""Dev probe: one cfg4 (or argv[1]) BA problem, 10 fixed LM iterations, for
rocprofv3 kernel-trace / PMC runs."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + '/structure-from-motion-_amd')
import numpy as np, _sfmcore as c, sfm_synthetic as syn
p = syn.ba_problem_cfg(sys.argv[1] if len(sys.argv) > 1 else "cfg4", dense=False)
cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
prob = c.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF)
rep = prob.solve(max_iterations=10, fixed_iterations=True)
print({k: round(v, 4) for k, v in prob.kernel_times().items()}, rep["t_loop_ms"] / 10)
prob.close()
