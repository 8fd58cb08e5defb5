"""Drop-in for the reference module ``LinearPnP`` (Phase 1/LinearPnP.py:3-96).

One wavefront on the MI355X builds the 2N x 12 DLT system, reduces it
(Givens QR, then Jacobi SVD of the 12 x 12 factor) and applies LinearPnP's
post-processing; for N = 4, 5 -- where the null space is 4-/2-dimensional
and np.linalg.svd's Vt[-1] is a property of LAPACK's dgesdd path -- that
path's bidiagonalisation is emulated so the same vector comes out.
"""
import numpy as np

import _sfmcore as _core


def LinearPnP(Xset, xset, K):
    """
    Estimates camera pose using linear least squares method on the 3D points and corresponding 2D projection on
    the image. Uses Direct Linear Transform (DLT) algorithm.

    Parameters
    ----------
    Xset : numpy.ndarray
        set of 3D points (N x 3)
    xset : numpy.ndarray
        set of 2D projections of 3D points on the image (N x 2)
    K : numpy.ndarray
        camera intrinsic matrix (3 x 3)

    Results
    -------
    C : numpy.ndarray
        the estimated center of camera (3,)
    R : numpy.ndarray
        the estimated rotation matrix (3 x 3)
    """
    Xset = np.array(Xset)
    xset = np.array(xset)
    K = np.array(K)
    n_points = len(Xset)
    if n_points < 4:  # :31-32
        raise ValueError("At least 4 point correspondences are required for PnP")
    C, R, _branch = _core.linear_pnp(Xset.reshape(n_points, 3), xset.reshape(n_points, 2), K)
    return C, R
