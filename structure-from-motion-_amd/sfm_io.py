"""Matching-file IO (reference Phase 1/Utils.py:8-64).

``get_data`` is a drop-in for the reference's ``Utils.get_data`` (same
signature, same arrays bit for bit) built on the native reader in
libsfmcore (csrc/matching_io.cpp).  ``read_matching`` returns the same data
as a COO ``MatchStore`` -- one record per (feature, image) observation --
so large scenes reach bundle adjustment without the dense
n_features x n_images matrices (800 MB each at cfg5).
"""
import numpy as np

import _sfmcore as _core


class MatchStore:
    """COO observation store: ``feature``, ``image`` (0-based), ``x``, ``y``,
    feature-major with images ascending (the row-major order of the dense
    matrices), plus a per-observation ``flag`` -- the COO form of the
    driver's ``filtered_feature_flags`` (Wrapper_dev.py:98-122)."""

    def __init__(self, n_features, n_images, feature, image, x, y):
        self.n_features = int(n_features)
        self.n_images = int(n_images)
        self.feature, self.image, self.x, self.y = feature, image, x, y
        self.flag = np.zeros(len(feature), dtype=np.uint8)
        self._row_start = np.searchsorted(feature, np.arange(self.n_features + 1))

    def __len__(self):
        return len(self.feature)

    def dense(self):
        """(feature_x, feature_y, feature_flag) exactly as get_data builds them."""
        fx = np.zeros((self.n_features, self.n_images))
        fy = np.zeros((self.n_features, self.n_images))
        ff = np.zeros((self.n_features, self.n_images), dtype=int)
        fx[self.feature, self.image] = self.x
        fy[self.feature, self.image] = self.y
        ff[self.feature, self.image] = 1
        return fx, fy, ff

    def lookup(self, rows, image):
        """Observation index of (rows[i], image), -1 where there is none."""
        rows = np.asarray(rows, dtype=np.int64)
        lo, hi = self._row_start[rows], self._row_start[rows + 1]
        out = np.full(len(rows), -1, dtype=np.int64)
        for k in np.unique(hi - lo):  # rows have few observations: vectorise per length
            sel = (hi - lo) == k
            for j in range(int(k)):
                idx = lo[sel] + j
                hit = self.image[idx] == image
                tgt = np.where(sel)[0][hit]
                out[tgt] = idx[hit]
        return out

    def set_flags(self, rows, image, value=1):
        """filtered_feature_flags[rows, image] = value, for observed entries."""
        idx = self.lookup(rows, image)
        self.flag[idx[idx >= 0]] = value

    def observations(self, filtered_world_coords, n_cameras, use_flags=True):
        """COO inputs of bundle adjustment in the reference's order
        (BundleAdjustment.py:164-169): valid points ascending, cameras
        ascending.  Returns (valid_point_indices, camera_indices,
        point_indices, points_2d) -- the same arrays the dense path gives."""
        valid = np.asarray(filtered_world_coords).flatten() == 1
        valid_point_indices = np.where(valid)[0]
        keep = valid[self.feature] & (self.image < n_cameras)
        if use_flags:
            keep &= self.flag == 1
        feat, cam = self.feature[keep], self.image[keep]
        point_indices = np.searchsorted(valid_point_indices, feat)
        points_2d = np.column_stack([self.x[keep], self.y[keep]])
        return valid_point_indices, cam.astype(np.int64), point_indices, points_2d


def read_matching(data_path, no_of_images, n_threads=0):
    """Parse data_path/matching1..(no_of_images-1).txt into a MatchStore."""
    nf, feat, img, x, y = _core.parse_matching(data_path, no_of_images, n_threads)
    return MatchStore(nf, no_of_images, feat, img, x, y)


def get_data(data_path, no_of_images):
    """
    Read data from matching files and extract features.

    :param data_path: Path to the directory containing matching files.
    :type data_path: str
    :param no_of_images: Number of images.
    :type no_of_images: int
    :return: x_features, y_features, feature_flags
    :rtype: numpy.ndarray, numpy.ndarray, numpy.ndarray
    """
    return read_matching(data_path, no_of_images).dense()
