"""Dev sweep: lanes per point of k_linearize / k_backsub_trial (env
SFM_LINEARIZE_LANES / SFM_BACKSUB_LANES) on cfg4 and cfg5, fixed 10 LM
iterations, per-kernel ms/iter (median of 3)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + "/structure-from-motion-_amd")
import numpy as np  # noqa: E402
import _sfmcore as c  # noqa: E402
import sfm_synthetic as syn  # noqa: E402

for name in ("cfg4", "cfg5"):
    p = syn.ba_problem_cfg(name, dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    prob = c.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF)
    prob.set_timing()
    for g in [int(v) for v in os.environ.get("SWEEP", "1,2,4,8").split(",")]:
        os.environ["SFM_LINEARIZE_LANES"] = str(g)
        os.environ["SFM_BACKSUB_LANES"] = str(g)
        lin, bs, tot = [], [], []
        for _ in range(3):
            prob.reset()
            rep = prob.solve(max_iterations=10, fixed_iterations=True)
            kt = prob.kernel_times()
            lin.append(kt["linearize"]); bs.append(kt["backsub_trial"]); tot.append(rep["t_loop_ms"] / 10)
        print(f"{name} lanes={g}: linearize {np.median(lin):.4f} backsub {np.median(bs):.4f} iter {np.median(tot):.4f} ms",
              flush=True)
    prob.close()
