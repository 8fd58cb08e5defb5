"""k_camera_lin chunk size probe: converged cfg4 solve, linearize phase time
(k_linearize + k_camera_lin, every iteration accepted) per SFM_CAM_CHUNK."""
import os, sys, subprocess
if len(sys.argv) > 1:
    R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, R + '/structure-from-motion-_amd')
    import numpy as np, _sfmcore as c, sfm_synthetic as syn
    p = syn.ba_problem_cfg("cfg4", dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    prob = c.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF)
    prob.set_timing()
    for _ in range(2):
        prob.reset()
        rep = prob.solve(max_iterations=50)
    print(sys.argv[1], "lin ms", round(prob.kernel_times()["linearize"], 4), "loop", round(rep["t_loop_ms"] / rep["iterations"], 4),
          rep["iterations"], rep["cost"], flush=True)
    prob.close()
else:
    for ch in os.environ.get("CHUNKS", "4096 2048 1024 512").split():
        th = os.environ.get("THREADS", "256")
        for t in th.split():
            print("threads", t, flush=True)
            subprocess.run([sys.executable, __file__, ch], env=dict(os.environ, SFM_CAM_CHUNK=ch, SFM_CAMLIN_THREADS=t),
                           check=True, timeout=120)
