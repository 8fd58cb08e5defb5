"""Drop-in for the reference module ``LinearTriangulation``
(Phase 1/LinearTriangulation.py:3-99): one GPU thread per point solves the
4x4 DLT system (:69-81) by one-sided Jacobi SVD and dehomogenises (:84-88).
"""
import numpy as np

import _sfmcore as _core


def LinearTriangulation(K, C1, R1, C2, R2, x1, x2):
    """
    Computes the 3D position of a set of points given its projections in two images using
    linear triangulation. Uses Direct Linear Transform (DLT) algorithm.

    Parameters
    ----------
    K : array-like
        camera intrinsic matrix (3 x 3)
    C1 : array-like
        center of first camera (3,)
    R1 : array-like
        rotation matrix of first camera (3 x 3)
    C2 : array-like
        center of second camera (3,)
    R2 : array-like
        rotation matrix of second camera (3 x 3)
    x1 : array-like
        projections of a set of points in first image (N x 2)
    x2 : array-like
        projections of a set of points in second image (N x 2)

    Results
    -------
    X : array-like
        set of vectors representing the 3D positions of points in space (N x 3)
    """
    K = np.array(K)
    C1 = np.array(C1)
    R1 = np.array(R1)
    C2 = np.array(C2)
    R2 = np.array(R2)
    x1 = np.array(x1)
    x2 = np.array(x2)
    n_points = len(x1)
    # P = K [R | -R C]  (LinearTriangulation.py:44-49), formed on the host
    P1 = K @ np.hstack([R1, -R1 @ C1.reshape(3, 1)])
    P2 = K @ np.hstack([R2, -R2 @ C2.reshape(3, 1)])
    if n_points == 0:
        return np.array([])
    return _core.triangulate(P1, P2, x1.reshape(n_points, -1)[:, :2], x2.reshape(n_points, -1)[:, :2])


def linear_triangulation(K, C1, R1, C2, R2, x1, x2):
    """
    Alias for LinearTriangulation with lowercase name.
    """
    return LinearTriangulation(K, C1, R1, C2, R2, x1, x2)
