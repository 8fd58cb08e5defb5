"""Dev probe: k_schur_sweep phase costs (SFM_SWEEP_DEBUG bits skip work:
1 off-diagonal pairs, 2 diagonal records, 4 staging).  Timing only."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + '/structure-from-motion-_amd')
import numpy as np, _sfmcore as c, sfm_synthetic as syn
p = syn.ba_problem_cfg(sys.argv[1] if len(sys.argv) > 1 else "cfg4", dense=False)
cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
for dbg in (0, 1, 2, 3, 4, 5, 7):
    os.environ["SFM_SWEEP_DEBUG"] = str(dbg)
    prob = c.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF)
    prob.set_timing()
    prob.solve(max_iterations=3, fixed_iterations=True)
    prob.reset()
    rep = prob.solve(max_iterations=10, fixed_iterations=True)
    print("dbg", dbg, "schur ms", round(prob.kernel_times()["schur_blocks"], 4), flush=True)
    prob.close()
