"""Dev probe: BA step timing with the sweep's lanes per pair (SFM_SWEEP_LPP
1 or 2) at the given configs (kernel split from HIP events)."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + '/structure-from-motion-_amd')
import numpy as np, _sfmcore as c, sfm_synthetic as syn
for name in sys.argv[1].split(","):
    p = syn.ba_problem_cfg(name, dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    for lpp in sys.argv[2].split(","):
        os.environ["SFM_SWEEP_LPP"] = lpp
        prob = c.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF)
        conv = prob.solve(max_iterations=50)
        prob.reset()
        prob.solve(max_iterations=3, fixed_iterations=True)
        prob.reset()
        r = prob.solve(max_iterations=20, fixed_iterations=True)
        prob.reset()
        prob.set_timing(True)
        prob.solve(max_iterations=20, fixed_iterations=True)
        kt = prob.kernel_times()
        prob.close()
        print(f"{name} lpp={lpp}: {r['t_loop_ms'] / 20:.4f} ms/step conv it {conv['iterations']} acc {conv['accepted']} "
              f"cost {conv['cost']:.12e} {dict((k, round(v, 4)) for k, v in kt.items())}", flush=True)
