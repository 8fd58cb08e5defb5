"""Times the dense -> COO observation phase of perform_bundle_adjustment at
a BASELINE config (host only, no GPU): python tools/obs_probe.py cfg5 [threads]"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "structure-from-motion-_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import sfm_synthetic as syn  # noqa: E402
import _sfmcore as core  # noqa: E402
import BundleAdjustment as BA  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "cfg5"
nt = int(sys.argv[2]) if len(sys.argv) > 2 else 0
p = syn.ba_problem_cfg(wl, dense=False)
n_pts, n_cams = p["n_pts"], p["n_cams"]
fx = np.zeros((n_pts, n_cams))
fy = np.zeros((n_pts, n_cams))
fl = np.zeros((n_pts, n_cams), dtype=np.int64)
fx[p["pt_idx"], p["cam_idx"]] = p["obs"][:, 0]
fy[p["pt_idx"], p["cam_idx"]] = p["obs"][:, 1]
fl[p["pt_idx"], p["cam_idx"]] = 1
fwc = np.ones((n_pts, 1), dtype=np.int64)
for it in range(3):
    t0 = time.perf_counter()
    v = np.where(np.asarray(fwc).flatten() == 1)[0]
    t1 = time.perf_counter()
    got = core.dense_observations(fl, fx, fy, v, n_cams, n_threads=nt)
    t2 = time.perf_counter()
    obs = BA._observations(fwc, fx, fy, fl, n_cams)
    t3 = time.perf_counter()
    print(f"where {1e3*(t1-t0):.2f} ms  dense_observations {1e3*(t2-t1):.2f} ms  _observations {1e3*(t3-t2):.2f} ms  n={len(got[0])}")

# split: scan call vs read call
f = fl
rows = np.ascontiguousarray(v, dtype=np.int64)
for it in range(3):
    h = ctypes.c_void_p()
    no = np.zeros(1, dtype=np.int64)
    t0 = time.perf_counter()
    core._check(core._lib.sfm_dense_obs_scan(f.ctypes.data, core._DENSE_DTYPES[f.dtype], f.strides[0], f.shape[0],
                                             core._p(rows, core._i64), len(rows), int(n_cams), fx.ctypes.data_as(core._d),
                                             fy.ctypes.data_as(core._d), fx.strides[0], nt, ctypes.byref(h),
                                             core._p(no, core._i64)))
    t1 = time.perf_counter()
    n = int(no[0])
    cam, pt, ob = np.empty(n, dtype=np.int32), np.empty(n, dtype=np.int32), np.empty((n, 2))
    core._check(core._lib.sfm_dense_obs_read(h, core._p(cam, core._i32), core._p(pt, core._i32), core._p(ob)))
    t2 = time.perf_counter()
    core._lib.sfm_dense_obs_free(h)
    t3 = time.perf_counter()
    print(f"scan {1e3*(t1-t0):.2f}  read {1e3*(t2-t1):.2f}  free {1e3*(t3-t2):.2f}")
