"""Drop-in for the reference module ``GetInliersRANSAC``
(Phase 1/GetInliersRANSAC.py:5-121).

The reference loop (:53-92: sample 8, estimate F, score all N, strict '>'
update) becomes one batched evaluation on the MI355X:

1. the n_max samples are drawn from the GLOBAL ``random`` instance exactly as
   the reference draws them (n_max calls of random.sample(range(N), 8) in
   iteration order, replayed natively inside the C-ABI call, chunk by chunk
   while the GPU scores the chunks already drawn, the generator's state
   read and written back in place), so the stream seen by later callers
   (PnPRANSAC, the next image pair) is unchanged;
2. libsfmcore builds every hypothesis F (8 lanes each, the next chunk's
   fits riding in the current chunk's score launch), scores every
   (hypothesis, correspondence) pair (correspondences held in registers,
   hypotheses streamed through them: a packed float prefilter proves the
   outliers, the FP64 test -- the reference's decision bit for bit --
   decides the rest) and picks the first hypothesis with the strictly
   largest count -- the reference's tie rule (:85-88).
"""
import numpy as np

import _sfmcore as _core
from EstimateFundamentalMatrix import EstimateFundamentalMatrix  # noqa: F401  (re-exported as in :3)


def GetInliersRANSAC(points1, points2, index, threshold=0.06, n_max=1000):
    """
    Rejects the outliers from a set of feature matches and returns the inliner indices.

    Parameters
    ----------
    points1 : numpy.ndarray
        feature points for matching in first image
    points2 : numpy.ndarray
        feature points for matching in second image
    index : numpy.ndarray
        index of all feature matches
    threshold : float
        threshold for inlier detection (default: 0.06)
    n_max : int
        maximum number of RANSAC iterations (default: 1000)

    Results
    -------
    inlier_index : numpy.ndarray
        index of all inlier feature matches
    outlier_index : numpy.ndarray
        index of all outlier feature matches for visulaization
    F_best : numpy.ndarray
        the best fundamental matrix
    """
    # np.asarray for the points: the reference's np.array(...) (:32-34)
    # without the copy (they are only read).  index is copied as the
    # reference does: the early returns hand it back, and a caller that
    # modifies the result must not modify its own input
    points1 = np.asarray(points1)
    points2 = np.asarray(points2)
    index = np.array(index)
    n_points = len(points1)
    if n_points < 8:  # :38-40
        return np.array([]), index, None
    # :48-50 builds the homogeneous copies with np.hstack before the loop: it
    # raises for anything but a 2-D array of n_points rows, before any draw
    # (checked here, and np.hstack itself raises the reference's ValueError)
    for pts in (points1, points2):
        if pts.ndim != 2 or pts.shape[0] != n_points:
            np.hstack([pts, np.ones((n_points, 1))])
    n_iter = max(int(n_max), 0)
    if points1.shape[1] != 2 or points2.shape[1] != 2:
        # every iteration then raises inside the loop's try -- in
        # EstimateFundamentalMatrix (not N x 2, EstimateFundamentalMatrix.py:80-81)
        # or in the scoring's shapes (:67-69) -- and is skipped (:90-92), but
        # its random.sample has been drawn: n_max draws, then the sentinel (:95-96)
        if n_iter:
            _core.sample_table(n_points, 8, n_iter)
        return np.array([]), index, None
    # n_iter draws of random.sample(range(N), 8) from the global stream,
    # replayed inside the call while the GPU scores the drawn chunks
    best, F_best, split, n_in = _core.ransac_f8_dropin(points1.reshape(n_points, 2), points2.reshape(n_points, 2),
                                                       n_iter, threshold)
    if best < 0:  # :95-96 (no hypothesis with a positive count)
        return np.array([]), index, None
    # :99-106 from the library's positions: split[:n_in] is np.where(inlier_mask)[0],
    # split[n_in:] the outlier positions, ascending
    inlier_index = split[:n_in]
    if index.ndim >= 1 and len(index) == n_points:
        outlier_indices = index[split[n_in:]]
    else:  # the reference's boolean index, with its IndexError
        outlier_mask = np.ones(n_points, dtype=bool)
        outlier_mask[inlier_index] = False
        outlier_indices = index[outlier_mask]
    return inlier_index, outlier_indices, F_best


def get_inliers_ransac(points1, points2, index, threshold=0.06, n_max=1000):
    """
    Alias for GetInliersRANSAC with lowercase name.
    Returns (F_best, inlier_index) instead of (inlier_index, outlier_index, F_best)
    for compatibility with wrapper code.
    """
    inlier_index, outlier_indices, F_best = GetInliersRANSAC(points1, points2, index, threshold, n_max)
    if len(inlier_index) > 0:  # :113-121
        inlier_idx = index[inlier_index]
    else:
        inlier_idx = np.array([])
    return F_best, inlier_idx
