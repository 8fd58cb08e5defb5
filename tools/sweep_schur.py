"""Dev probe: k_schur_sweep time per LM iteration over the sweep plan's
range count and chunk size (env SFM_SWEEP_RANGES / SFM_SWEEP_CHUNK)."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + '/structure-from-motion-_amd')
import numpy as np, _sfmcore as c, sfm_synthetic as syn
cfgs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["cfg4"]
for name in cfgs:
    p = syn.ba_problem_cfg(name, dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    nrs = [int(v) for v in os.environ.get("NRS", "8,16").split(",")]
    chs = [int(v) for v in os.environ.get("CHS", "2048,4096,8192,16384").split(",")]
    for nr in nrs:
        for ch in chs:
            os.environ["SFM_SWEEP_RANGES"] = str(nr)
            os.environ["SFM_SWEEP_CHUNK"] = str(ch)
            prob = c.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF)
            prob.set_timing()
            prob.solve(max_iterations=3, fixed_iterations=True)
            prob.reset()
            rep = prob.solve(max_iterations=10, fixed_iterations=True)
            kt = prob.kernel_times()
            print(name, "ranges", nr, "chunk", ch, "schur ms", round(kt["schur_blocks"], 4), "iter ms",
                  round(rep["t_loop_ms"] / 10, 4), "cost", rep["cost"], flush=True)
            prob.close()
