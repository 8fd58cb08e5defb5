"""Drop-in for the reference module ``PnPRANSAC`` (Phase 1/PnPRANSAC.py:6-89).

The n_max 4-point samples are drawn from the GLOBAL ``random`` instance
exactly as the reference draws them (replayed natively, state written back).
Every hypothesis' LinearPnP runs in its own GPU thread, every (hypothesis,
point) reprojection test in one wavefront per hypothesis, and the first
strictly-largest count wins (:72-76); the all-point LinearPnP fallback and
its warning (:82-87) are kept.
"""
import numpy as np

import _sfmcore as _core
from LinearPnP import LinearPnP


def PnPRANSAC(X, x, K, threshold=200, n_max=1000):
    """
    Estimates the 6-DoF camera pose with respect to a 3D object using the Perspective-n-Point (PnP) algorithm
    with Random Sample Consensus (RANSAC) to handle outliers.

    Parameters
    ----------
    X : numpy.ndarray
        a set of 3D points in the world (N x 3)
    x : numpy.ndarray
        the 2D projections of the 3D points in the image (N x 2)
    K : numpy.ndarray
        the camera intrinsic matrix (3 x 3)
    threshold : float
        threshold for inlier detection in pixels (default: 200)
    n_max : int
        maximum number of RANSAC iterations (default: 1000)

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
    n_points = len(X)
    if n_points < 4:  # :36-37
        raise ValueError("At least 4 point correspondences are required for PnP")
    n_iter = max(int(n_max), 0)
    samples = _core.sample_table(n_points, min(4, n_points), n_iter)
    best, best_count, C, R, _, _ = _core.pnp_ransac(X.reshape(n_points, 3), x.reshape(n_points, 2), K, samples,
                                                    threshold)
    if best < 0 or best_count < 4:  # :82-87
        try:
            C, R = LinearPnP(X, x, K)
            print("Warning: PnP RANSAC failed, using linear PnP on all points")
        except Exception as e:
            raise ValueError(f"PnP estimation failed: {e}")
    return C, R
