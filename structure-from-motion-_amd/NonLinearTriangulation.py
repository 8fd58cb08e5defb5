"""Drop-in for the reference module ``NonLinearTriangulation``
(Phase 1/NonLinearTriangulation.py:5-130).

The reference runs one scipy ``least_squares(method='lm', max_nfev=50)`` per
point (:100-121).  Here all points go to the GPU at once: one thread per
point runs the same MINPACK lmdif on the same 4-residual loss
(csrc/lm_small.hpp, csrc/nltri.hip), so a point's result is the one the
reference computes for it (pinned bit-for-bit by tests/golden/nltri.npz).
Points the reference's ``try/except`` leaves at ``x0`` (non-finite ``x0`` or
residuals) are copied through the same way.
"""
import numpy as np

import _sfmcore as _core


def Loss(X, x1, x2, P1, P2):
    """
    Loss function for optimization in non-linear triangulation.
    Computes reprojection error for a single 3D point (NonLinearTriangulation.py:5-50).

    Parameters
    ----------
    X : array-like
        3D point (3,)
    x1, x2 : array-like
        projections of the point in the first / second image (2,)
    P1, P2 : array-like
        projection matrices (3 x 4)

    Results
    -------
    error : numpy.ndarray
        reprojection errors (4,)
    """
    X_hom = np.array([X[0], X[1], X[2], 1])
    out = []
    for P, x in ((P1, x1), (P2, x2)):
        h = P @ X_hom
        proj = np.array([x[0], x[1]]) if abs(h[2]) < 1e-8 else h[:2] / h[2]
        out.append(x - proj)
    return np.hstack(out)


def NonLinearTriangulation(K, C1, R1, C2, R2, x1, x2, x0):
    """
    Computes the 3D position of a set of points given its projections in two images using
    non-linear triangulation. Refines 3D points using non-linear optimization.

    Parameters
    ----------
    K : array-like
        camera intrinsic matrix (3 x 3)
    C1, R1 : array-like
        center (3,) and rotation (3 x 3) of the first camera
    C2, R2 : array-like
        center (3,) and rotation (3 x 3) of the second camera
    x1, x2 : array-like
        projections of the points in the first / second image (N x 2)
    x0 : array-like
        initial estimate of 3D points from linear triangulation (N x 3)

    Results
    -------
    X : array-like
        refined 3D points (N x 3)
    """
    K = np.array(K)
    C1 = np.array(C1)
    R1 = np.array(R1)
    C2 = np.array(C2)
    R2 = np.array(R2)
    x1 = np.array(x1)
    x2 = np.array(x2)
    x0 = np.array(x0)
    n_points = len(x1)
    # P = K [R | -R C]  (NonLinearTriangulation.py:93-97), formed on the host
    t1 = -R1 @ C1.reshape(3, 1)
    P1 = K @ np.hstack([R1, t1])
    t2 = -R2 @ C2.reshape(3, 1)
    P2 = K @ np.hstack([R2, t2])
    if n_points == 0:
        return np.array([])
    x1 = x1.reshape(n_points, -1)
    x2 = x2.reshape(n_points, -1)
    if x1.shape[1] != 2 or x2.shape[1] != 2:
        # Loss's `x - proj` cannot broadcast: every point raises inside the
        # reference's try and keeps its initial estimate (:114-121)
        return np.array([x0[i] for i in range(n_points)])
    X0 = np.asarray(x0[:n_points], dtype=float)
    if X0.ndim != 2 or X0.shape[1] != 3:
        raise ValueError("NonLinearTriangulation: x0 must be N x 3 (one initial point per correspondence)")
    X, _info = _core.triangulate_nonlinear(P1, P2, x1, x2, X0, max_nfev=50)
    return X


def nonlinear_triangulation(K, C1, R1, C2, R2, x1, x2, x0):
    """
    Alias for NonLinearTriangulation with lowercase name.
    """
    return NonLinearTriangulation(K, C1, R1, C2, R2, x1, x2, x0)
