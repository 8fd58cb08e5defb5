"""TEST INFRASTRUCTURE ONLY -- timing restatement of the reference's BA
residual (Phase 1/BundleAdjustment.py:43-110), used by bench.py's
cpu_baseline leg to price the as-shipped reference path, which cannot run on
the GPU box (the reference does not travel) nor finish at cfg4/cfg5.

It keeps the reference's loop structure call for call: one scipy Rotation
conversion and centre per camera (:79-91), then per observation a 1x4
homogeneous point, P = K [R | -R C], a projection and a divide by
(w + 1e-8) (:95-108, project_points :8-40), two residual entries appended to
a list.  Its values equal oracle.ba_residuals (tests/test_oracle.py); only
its time is used.
"""
import numpy as np
from scipy.spatial.transform import Rotation


def residuals(params, n_cams, n_pts, cam_idx, pt_idx, obs, K):
    cams = params[:6 * n_cams].reshape(n_cams, 6)
    X = params[6 * n_cams:].reshape(n_pts, 3)
    Rs, Cs = [], []
    for c in range(n_cams):
        R = Rotation.from_rotvec(cams[c, :3]).as_matrix()
        Rs.append(R)
        Cs.append(-R.T @ cams[c, 3:6])
    out = []
    for o in range(len(cam_idx)):
        R, C = Rs[cam_idx[o]], Cs[cam_idx[o]]
        Xh = np.hstack([X[pt_idx[o]].reshape(1, 3), np.ones((1, 1))])
        P = K @ np.hstack([R, -R @ C.reshape(3, 1)])
        xh = (P @ Xh.T).T
        x = xh[:, :2] / (xh[:, 2:3] + 1e-8)
        e = obs[o] - x[0]
        out.extend([e[0], e[1]])
    return np.array(out)
