"""sfm_ba_create's phases (SFM_CREATE_TIMING=1) for a BASELINE config,
three creates in one process (the first pays HIP's and the kernels' one-time
loads; the later ones are what a drop-in call in a running pipeline pays).
Usage: create_once.py [cfg4|cfg5] [host]  (host: SFM_PLAN_HOST=1)"""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("SFM_PKG") or R + "/structure-from-motion-_amd")  # SFM_PKG: an A/B build's directory
os.environ["SFM_CREATE_TIMING"] = "1"
if len(sys.argv) > 2 and sys.argv[2] == "host":
    os.environ["SFM_PLAN_HOST"] = "1"
import numpy as np, _sfmcore as c, sfm_synthetic as syn
p = syn.ba_problem_cfg(sys.argv[1] if len(sys.argv) > 1 else "cfg5", dense=False)
cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
for k in range(3):
    t0 = time.perf_counter()
    prob = c.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF)
    t1 = time.perf_counter()
    prob.close()
    print(f"create {k}: {1e3 * (t1 - t0):.2f} ms (close {1e3 * (time.perf_counter() - t1):.2f} ms)", file=sys.stderr,
          flush=True)
