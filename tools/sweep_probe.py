"""Dev probe: BA step and kernel split under environment variants, e.g.
  python tools/sweep_probe.py cfg5 "SFM_SWEEP_DEBUG=0" "SFM_SWEEP_DEBUG=4" "SFM_SWEEP_DEBUG=7"
(SFM_SWEEP_DEBUG bits: 1 skip the off-diagonal pairs, 2 skip the diagonal
blocks, 4 skip the staging, 8 return at once; timing only -- the results are wrong then)."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + '/structure-from-motion-_amd')
import numpy as np, _sfmcore as c, sfm_synthetic as syn
p = syn.ba_problem_cfg(sys.argv[1], dense=False)
cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
for var in sys.argv[2:]:
    saved = {}
    for kv in var.split(";"):
        k, v = kv.split("=")
        saved[k] = os.environ.get(k)
        os.environ[k] = v
    prob = c.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF)
    prob.solve(max_iterations=3, fixed_iterations=True)
    prob.reset()
    prob.set_timing(True)
    r = prob.solve(max_iterations=20, fixed_iterations=True)
    kt = prob.kernel_times()
    prob.close()
    print(f"{sys.argv[1]} [{var}]: {r['t_loop_ms'] / 20:.4f} ms/step cost {r['cost']:.12e} "
          f"{dict((k, round(v, 4)) for k, v in kt.items())}", flush=True)
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k)
        else:
            os.environ[k] = v
