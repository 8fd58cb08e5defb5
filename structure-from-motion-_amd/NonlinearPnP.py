"""Drop-in for the reference module ``NonlinearPnP``
(Phase 1/NonlinearPnP.py:5-151).

The pose refinement (scipy least_squares(method='lm', max_nfev=100) on the
2N reprojection residuals) runs as MINPACK lmdif on the MI355X (pnp.hip
k_nonlinear_pnp) over ceil(2N / 1024) workgroups (at most 64, clamped to
the resident count; a timed-out hand-off retries on one workgroup): each
workgroup keeps its ~1,024 residual rows in registers and forms its partial
block sums, the partials are all-gathered and every workgroup adds them in
the same fixed order, so each runs the same replicated lmdif control.  Every
forward-difference Jacobian (the base and the six perturbed projections in
one pass) is reduced to its 6 x 6 R factor and Q^T f by CholeskyQR2
(fixed-order block sums of J^T J, then of q^T q and q^T f with
q = J R1^-1; a shifted third pass when J is numerically rank-deficient,
reported in info's flags); MINPACK's qrfac with column pivoting, lmpar, the
trust region and the stopping tests then run on the 6 x 6 factor on one
lane.  Rotation conversions follow scipy's quaternion
formulas.  The result is the reference's minimum (cost within 1e-9, pose
within 1e-5), not bit-exact: device sin/cos and the parallel sums round
differently.
"""
import numpy as np
from scipy.spatial.transform import Rotation

import _sfmcore as _core


def NonLinearPnPLoss(X0, X, x, K):
    """
    The loss function for optimization in Non-Linear PnP (NonlinearPnP.py:5-44).

    Parameters
    ----------
    X0 : numpy.ndarray
        parameters (rotation vector (3) + translation (3))
    X : numpy.ndarray
        a set of 3D points (N x 3)
    x : numpy.ndarray
        a set of projections of these 3D points (N x 2)
    K : numpy.ndarray
        camera intrinsic matrix (3 x 3)

    Results
    -------
    error : numpy.ndarray
        reprojection errors (2*N,)
    """
    R = Rotation.from_rotvec(X0[:3]).as_matrix()
    C = -R.T @ X0[3:6]
    X_hom = np.hstack([X, np.ones((X.shape[0], 1))])
    P = K @ np.hstack([R, -R @ C.reshape(3, 1)])
    x_proj_hom = (P @ X_hom.T).T
    x_proj = x_proj_hom[:, :2] / (x_proj_hom[:, 2:3] + 1e-8)
    return (x - x_proj).flatten()


def NonLinearPnP(X, x, K, C, R):
    """
    Non-linear Perspective-n-Point (PnP): refines the camera pose by
    minimising the reprojection error.

    Parameters
    ----------
    X : numpy.ndarray
        a set of 3D points (N x 3)
    x : numpy.ndarray
        a set of projections of these 3D points (N x 2)
    K : numpy.ndarray
        camera intrinsic matrix (3 x 3)
    C : numpy.ndarray
        the center of camera (3,) - initial estimate
    R : numpy.ndarray
        the rotation matrix (3 x 3) - initial estimate

    Results
    -------
    Cnew : numpy.ndarray
        the estimated center of camera (3,)
    Rnew : numpy.ndarray
        the estimated rotation matrix (3 x 3)
    """
    X = np.array(X)
    x = np.array(x)
    K = np.array(K)
    C = np.array(C)
    R = np.array(R)
    n_points = len(X)
    if n_points < 4:  # :96-98
        return C, R
    Cn, Rn, info = _core.nonlinear_pnp(X.reshape(n_points, 3), x.reshape(n_points, 2), K, C, R, max_nfev=100)
    if info == -1:  # :119-123, the reference's except path
        msg = ("Initial guess is outside of provided bounds" if not (np.all(np.isfinite(C)) and
               np.all(np.isfinite(R))) else "Residuals are not finite in the initial point.")
        print(f"Non-linear PnP optimization failed: {msg}")
        return C, R
    return Cn, Rn


def nonlinear_PnP(K, C, R, x, X):
    """
    Alias for NonLinearPnP with different parameter order to match wrapper usage.
    """
    return NonLinearPnP(X, x, K, C, R)
