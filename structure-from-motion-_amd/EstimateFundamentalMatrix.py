"""Drop-in for the reference module ``EstimateFundamentalMatrix``
(Phase 1/EstimateFundamentalMatrix.py:3-83): same name, signature and
result; the arithmetic runs on the MI355X (libsfmcore, csrc/sfm_geom.hpp).

The reference's conventions are kept exactly, including the as-shipped
design-matrix / denormalisation mismatch (A row solves x1^T F x2 = 0, :62,
while F = T2^T F T1, :75) -- parity means parity with *that* arithmetic.
"""
import numpy as np

import _sfmcore as _core


def EstimateFundamentalMatrix(points1, points2):
    """
    Estimates the fundamental matrix from the eight randomly selected feature matches.
    Uses the 8-point algorithm with normalization (Hartley normalization).

    Parameters
    ----------
    points1 : array-like
        points for matching from image 1 (N x 2 or 8 x 2)
    points2 : array-like
        points for matching from image 2 (N x 2 or 8 x 2)

    Results
    -------
    F : array-like
         the resulting fundamental matrix (3 x 3)
    """
    points1 = np.array(points1)
    points2 = np.array(points2)
    if points1.shape[1] == 2:  # EstimateFundamentalMatrix.py:25
        if len(points1) == 8:
            # the batched 8-point kernel RANSAC uses (k_f8_points)
            return _core.f8_batch(points1.reshape(1, 8, 2), points2.reshape(1, 8, 2))[0]
        if len(points1) == 0:
            raise ValueError("EstimateFundamentalMatrix needs at least one correspondence")
        # least-squares null vector of the N x 9 design matrix (k_f8_general)
        return _core.f8_general(points1, points2)
    raise ValueError("Points must be in 2D format (N x 2)")  # :80-81
