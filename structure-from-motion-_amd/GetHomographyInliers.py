"""Drop-in for the reference module ``GetHomographyInliers``
(Phase 1/GetHomographyInliers.py:4-165).

The reference's loop (:124-157: sample 4, DLT homography, transfer error of
all N points, strict '>' update) becomes one batched evaluation on the
MI355X, exactly as GetInliersRANSAC does for F:

1. the n_max samples are drawn from the GLOBAL ``random`` instance as the
   reference draws them (n_max calls of random.sample(range(N), 4), replayed
   natively and written back), so the F-RANSAC that follows in the driver
   (Wrapper_dev.py:87-105) sees the same stream;
2. libsfmcore fits every 4-point homography (one thread each), counts the
   inliers of every hypothesis (one wavefront each, LDS tiles, ballot
   popcount) and keeps the first hypothesis with the strictly largest count.
"""
import random  # noqa: F401  (part of the reference module's star-import surface)

import numpy as np

import _sfmcore as _core


def find_homography(image1_coords, image2_coords):
    """
    Find the homography matrix between two images using Direct Linear Transform (DLT).
    Requires at least 4 point correspondences.

    :param image1_coords: Image 1 coordinates (N x 2 array).
    :type image1_coords: numpy.ndarray
    :param image2_coords: Image 2 coordinates (N x 2 array).
    :type image2_coords: numpy.ndarray
    :return: Homography matrix (3 x 3).
    :rtype: numpy.ndarray
    """
    image1_coords = np.array(image1_coords)
    image2_coords = np.array(image2_coords)
    n_points = len(image1_coords)
    if n_points < 4:  # :21-22
        raise ValueError("At least 4 point correspondences are required for homography estimation")
    p1 = image1_coords.reshape(n_points, 2)
    p2 = image2_coords.reshape(n_points, 2)
    if n_points == 4:  # the RANSAC hypothesis path (8 x 9 system)
        return _core.h4_batch(p1[None], p2[None])[0]
    return _core.homography_general(p1, p2)


def get_homography_inliers(image1_coords_org, image2_coords_org, idx, threshold=30, n_max=1000):
    """
    Get the inliers for the homography matrix using RANSAC.

    :param image1_coords_org: Coordinates of the points in the first image (N x 2).
    :type image1_coords_org: numpy.ndarray
    :param image2_coords_org: Coordinates of the points in the second image (N x 2).
    :type image2_coords_org: numpy.ndarray
    :param idx: Indices of the points.
    :type idx: numpy.ndarray
    :param threshold: Error threshold for inlier detection (default: 30 pixels).
    :type threshold: float
    :param n_max: Maximum number of RANSAC iterations (default: 1000).
    :type n_max: int, optional
    :return: Homography matrix, inlier indices
    :rtype: tuple (numpy.ndarray, numpy.ndarray)
    """
    image1_coords_org = np.array(image1_coords_org)
    image2_coords_org = np.array(image2_coords_org)
    idx = np.array(idx)
    n_points = len(image1_coords_org)
    if n_points < 4:  # :108-110, before any draw from the stream
        return None, np.array([])
    n_iter = max(int(n_max), 0)
    # n_iter draws of random.sample(range(N), 4) from the global stream,
    # replayed inside the call while the GPU scores the drawn chunks
    best, H_best, mask, _, _ = _core.ransac_h4_pyrandom(image1_coords_org.reshape(n_points, 2),
                                                        image2_coords_org.reshape(n_points, 2), n_iter, threshold)
    if best < 0:  # :159-161
        return None, np.array([])
    return H_best, idx[np.where(mask)[0]]
