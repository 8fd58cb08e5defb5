"""Dev probe: a small BA solve (argv[1]: cfg name or 'tiny'), a few fixed
iterations, printing the report (hang / correctness triage)."""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + '/structure-from-motion-_amd')
import numpy as np, _sfmcore as c, sfm_synthetic as syn
name = sys.argv[1] if len(sys.argv) > 1 else "tiny"
p = syn.ba_problem(6, 200, 4, seed=3, dense=False) if name == "tiny" else syn.ba_problem_cfg(name, dense=False)
cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
print("built", flush=True)
prob = c.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF)
print("created", flush=True)
t = time.time()
rep = prob.solve(max_iterations=5, fixed_iterations=True)
print("solved", time.time() - t, rep, flush=True)
prob.close()
