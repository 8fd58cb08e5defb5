"""Host phases of sfm_ba_create (SFM_CREATE_TIMING=1) without a device:
SFM_CREATE_PLAN_ONLY=1 stops create after the host planning (validation, CSR,
co-observation counts, the Schur sweep plan, camera items).  Usage:
create_probe.py [cfg4|cfg5] [repeats]"""
import ctypes, os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + "/structure-from-motion-_amd")
os.environ["SFM_CREATE_PLAN_ONLY"] = "1"
os.environ["SFM_CREATE_TIMING"] = "1"
import numpy as np
import _sfmcore as c
import sfm_synthetic as syn

name = sys.argv[1] if len(sys.argv) > 1 else "cfg5"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
p = syn.ba_problem_cfg(name, dense=False)
cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
ci = np.ascontiguousarray(p["cam_idx"], dtype=np.int32)
pi = np.ascontiguousarray(p["pt_idx"], dtype=np.int32)
obs, K, pts = c._f64(p["obs"]), c._f64(syn.K_REF), c._f64(p["X0"])
cams = c._f64(cams0)
for r in range(reps):
    h = ctypes.c_void_p()
    t0 = time.perf_counter()
    rc = c._lib.sfm_ba_create(len(cams), len(pts), len(ci), c._p(ci, c._i32), c._p(pi, c._i32), c._p(obs), c._p(K),
                              c._p(cams), c._p(pts), 0, None, ctypes.byref(h))
    print(f"rep {r}: rc {rc} host plan {1e3 * (time.perf_counter() - t0):.1f} ms", file=sys.stderr, flush=True)
