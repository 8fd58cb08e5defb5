"""Drop-in for the reference module ``BundleAdjustment``
(Phase 1/BundleAdjustment.py:8-242).

``perform_bundle_adjustment`` keeps the reference's signature, observation
order (point-major, camera ascending, :164-169), parameterisation
([rotvec, t] per camera then points, :183-197), printed lines (:202, :236,
:241) and failure contract (any exception -> print + return the inputs
unchanged, :240-242; scipy's m < n and non-finite-x0 errors reproduced).
The solve itself is the MI355X sparse Schur-complement Levenberg-Marquardt
of libsfmcore (csrc/ba.hip) run to convergence on the reference residual.
The reference's scipy call stops at max_nfev=100 and, for any problem with
6*n_cams + 3*n_pts >= 98 parameters, returns x0 unchanged;
the drop-in's result is never worse than that and matches the converged
least-squares solution (tests/test_gpu_parity.py).
"""
import time

import numpy as np

import _sfmcore as _core


def project_points(K, C, R, X):
    """
    Project 3D points to 2D image coordinates.

    Parameters
    ----------
    K : numpy.ndarray
        Camera intrinsic matrix (3 x 3)
    C : numpy.ndarray
        Camera center (3,)
    R : numpy.ndarray
        Camera rotation matrix (3 x 3)
    X : numpy.ndarray
        3D points (N x 3)

    Returns
    -------
    x_proj : numpy.ndarray
        Projected 2D points (N x 2)
    """
    P = K @ np.hstack([R, -R @ C.reshape(3, 1)])  # :32
    return _core.project(P, np.asarray(X).reshape(-1, 3))


def bundle_adjustment_residuals(params, n_cameras, n_points, camera_indices, point_indices,
                                points_2d, K, n_cam_params=6):
    """
    Compute residuals for bundle adjustment.

    Returns
    -------
    residuals : numpy.ndarray
        Reprojection errors (2*N,), interleaved [r0x, r0y, r1x, ...]
    """
    params = np.asarray(params, dtype=np.float64)
    camera_params = params[:n_cameras * n_cam_params].reshape(n_cameras, n_cam_params)[:, :6]
    points_3d = params[n_cameras * n_cam_params:].reshape(n_points, 3)
    return _core.ba_residuals(camera_params, points_3d, camera_indices, point_indices,
                              np.asarray(points_2d).reshape(-1, 2), K)


# Wall-time split of the last perform_bundle_adjustment(_coo) call, in ms
# (measurement only; bench.py reports it as the drop-in's end-to-end time):
# observations (the dense scan of the flag matrix), cams0 (Rotation ->
# rotvec), ba_lm (the library call: create = host prep + plan + upload,
# loop, download, and the wrapper's copies), post (rotvec -> R, C and the
# points out), total.
last_timings = {}


def _observation_source(filtered_world_coords, feature_x, feature_y, filtered_feature_flags, n_cameras,
                        valid_point_indices=None):
    """Dense flags -> COO observations in the reference's order (:164-169):
    (valid_point_indices, source), the source the library's threaded scan of
    the valid rows (point-major, camera ascending, as np.where; a
    _core.DenseScan the solve reads without COO arrays), or the numpy
    expression's (camera_indices, point_indices, points_2d) for layouts the
    scanner does not read (a non-contiguous row, a flag dtype other than
    float/int/bool)."""
    if valid_point_indices is None:
        valid_point_indices = np.where(np.asarray(filtered_world_coords).flatten() == 1)[0]
    # the reference's loop indexes filtered_feature_flags[pt_idx, cam_idx] for
    # every valid point and camera (:164-166), outside its try: IndexError
    # escapes when the flag matrix is too short or too narrow
    flag_shape = np.shape(filtered_feature_flags)
    if len(flag_shape) != 2:
        raise IndexError(f"too many indices for array: array is {len(flag_shape)}-dimensional, but 2 were indexed")
    if valid_point_indices[-1] >= flag_shape[0]:
        raise IndexError(f"index {valid_point_indices[-1]} is out of bounds for axis 0 with size {flag_shape[0]}")
    if n_cameras > flag_shape[1]:
        raise IndexError(f"index {flag_shape[1]} is out of bounds for axis 1 with size {flag_shape[1]}")
    scan = _core.dense_scan(filtered_feature_flags, feature_x, feature_y, valid_point_indices, n_cameras)
    if scan is not None:
        return valid_point_indices, scan
    flags = np.asarray(filtered_feature_flags)[valid_point_indices][:, :n_cameras] == 1
    point_indices, camera_indices = np.nonzero(flags)  # row-major = point-major, camera ascending
    rows = valid_point_indices[point_indices]
    points_2d = np.column_stack([np.asarray(feature_x)[rows, camera_indices],
                                 np.asarray(feature_y)[rows, camera_indices]])
    return valid_point_indices, (camera_indices, point_indices, points_2d)


def _observations(filtered_world_coords, feature_x, feature_y, filtered_feature_flags, n_cameras):
    """(valid_point_indices, camera_indices, point_indices, points_2d) as the
    reference assembles them (:164-169)."""
    valid_point_indices, src = _observation_source(filtered_world_coords, feature_x, feature_y,
                                                   filtered_feature_flags, n_cameras)
    if isinstance(src, _core.DenseScan):
        with src:
            src = src.arrays()
    return (valid_point_indices,) + tuple(src)


def perform_bundle_adjustment(all_world_coords, filtered_world_coords, feature_x, feature_y,
                              filtered_feature_flags, R_set, C_set, K, cam_index, *,
                              max_iterations=100, function_tolerance=1e-10, parameter_tolerance=1e-12,
                              initial_lambda=1e-4):
    """
    Perform bundle adjustment to optimize camera poses and 3D points.

    Parameters
    ----------
    all_world_coords : numpy.ndarray
        All 3D points (n_features x 3)
    filtered_world_coords : numpy.ndarray
        Flag array indicating which points are valid (n_features x 1)
    feature_x : numpy.ndarray
        X coordinates of features (n_features x n_cameras)
    feature_y : numpy.ndarray
        Y coordinates of features (n_features x n_cameras)
    filtered_feature_flags : numpy.ndarray
        Flag matrix indicating which features are visible in which cameras (n_features x n_cameras)
    R_set : list
        List of rotation matrices for each camera
    C_set : list
        List of camera centers for each camera
    K : numpy.ndarray
        Camera intrinsic matrix (3 x 3)
    cam_index : int
        Current camera index (0-based); unused, as in the reference
    max_iterations, function_tolerance, parameter_tolerance, initial_lambda :
        keyword-only LM controls of the GPU solver (not in the reference)

    Returns
    -------
    R_set_opt : list
        Optimized rotation matrices
    C_set_opt : list
        Optimized camera centers
    all_world_coords_opt : numpy.ndarray
        Optimized 3D points
    """
    last_timings.clear()  # a call that returns early leaves no stale split behind
    t0 = time.perf_counter()
    valid_point_indices = np.where(np.asarray(filtered_world_coords).flatten() == 1)[0]
    if len(valid_point_indices) == 0:  # :152-153
        return R_set, C_set, all_world_coords
    vpi, src = _observation_source(filtered_world_coords, feature_x, feature_y, filtered_feature_flags, len(R_set),
                                   valid_point_indices)
    t_obs = (time.perf_counter() - t0) * 1e3
    try:
        out = _adjust(all_world_coords, vpi, src, R_set, C_set, K, max_iterations, function_tolerance,
                      parameter_tolerance, initial_lambda)
    finally:
        if isinstance(src, _core.DenseScan):
            src.close()
    last_timings["observations"] = t_obs
    last_timings["total"] = (time.perf_counter() - t0) * 1e3
    return out


def perform_bundle_adjustment_coo(all_world_coords, filtered_world_coords, store, R_set, C_set, K, *,
                                  max_iterations=100, function_tolerance=1e-10, parameter_tolerance=1e-12,
                                  initial_lambda=1e-4):
    """perform_bundle_adjustment fed from a sfm_io.MatchStore (its ``flag``
    plays filtered_feature_flags) instead of dense n_features x n_images
    matrices; same observations, order, solver, prints and failure
    behaviour."""
    last_timings.clear()  # a call that returns early leaves no stale split behind
    t0 = time.perf_counter()
    valid_point_indices = np.where(np.asarray(filtered_world_coords).flatten() == 1)[0]
    if len(valid_point_indices) == 0:
        return R_set, C_set, all_world_coords
    obs = store.observations(filtered_world_coords, len(R_set))
    t_obs = (time.perf_counter() - t0) * 1e3
    out = _adjust(all_world_coords, obs[0], obs[1:], R_set, C_set, K, max_iterations, function_tolerance,
                  parameter_tolerance, initial_lambda)
    last_timings["observations"] = t_obs
    last_timings["total"] = (time.perf_counter() - t0) * 1e3
    return out


def _adjust(all_world_coords, valid_point_indices, src, R_set, C_set, K, max_iterations, function_tolerance,
            parameter_tolerance, initial_lambda):
    """BundleAdjustment.py:156-242 from the observations: src a DenseScan or
    (camera_indices, point_indices, points_2d)."""
    dense = isinstance(src, _core.DenseScan)
    n_obs = len(src) if dense else len(src[0])
    n_cameras = len(R_set)
    n_points = len(valid_point_indices)
    last_timings.clear()
    if n_obs == 0:  # :171-172
        return R_set, C_set, all_world_coords
    t0 = time.perf_counter()
    # :183-193 for all cameras at once (the stacked conversions and products
    # give the per-camera loop's bits: the same routine per matrix)
    Rs = np.array([np.array(R) for R in R_set], dtype=np.float64).reshape(n_cameras, 3, 3)
    Cs = np.array([np.array(C) for C in C_set], dtype=np.float64).reshape(n_cameras, 3)
    cams0 = np.empty((n_cameras, 6))
    cams0[:, :3] = _core.matrix_to_rotvec(Rs)  # scipy's Rotation, its bits (csrc/rotations.cpp)
    cams0[:, 3:] = (-Rs @ Cs[:, :, None])[:, :, 0]
    t1 = time.perf_counter()
    last_timings["cams0"] = (t1 - t0) * 1e3  # :183-193, the stacked rotvec / t conversion
    pts0 = _core.gather_points(all_world_coords, valid_point_indices)  # :196-197 (host pool)
    t2 = time.perf_counter()
    last_timings["pts0"] = (t2 - t1) * 1e3
    print(f"  Bundle adjustment: {n_cameras} cameras, {n_points} points, {n_obs} observations")
    _core.require_device()  # a missing GPU is an error, never a silent "failed"
    try:
        if 2 * n_obs < 6 * n_cameras + 3 * n_points:  # scipy least_squares.py:850-852
            raise ValueError("Method 'lm' doesn't work when the number of residuals is less than the "
                             "number of variables.")
        t3 = time.perf_counter()
        opts = dict(max_iterations=max_iterations, function_tolerance=function_tolerance,
                    parameter_tolerance=parameter_tolerance, initial_lambda=initial_lambda)
        # cams0 / pts0 are this call's own arrays: solved in place (own=True)
        if dense:
            cams, pts, rep = _core.ba_lm_dense(cams0, pts0, src, K, own=True, **opts)
        else:
            camera_indices, point_indices, points_2d = src
            cams, pts, rep = _core.ba_lm(cams0, pts0, camera_indices, point_indices, points_2d, K, own=True, **opts)
        t4 = time.perf_counter()
        if rep["status"] == 6:  # the cost at x0 is not finite: least_squares.py:843-845, nothing solved
            raise ValueError("Residuals are not finite in the initial point.")
        last_timings.update(ba_lm=(t4 - t3) * 1e3, ba_lm_create=rep["t_setup_ms"],
                            ba_lm_loop=rep["t_loop_ms"], ba_lm_download=rep["t_download_ms"],
                            iterations=rep["iterations"])
        # :220-228 for all cameras at once (bitwise the per-camera loop)
        R_all = _core.rotvec_to_matrix(cams[:, :3])  # Rotation.from_rotvec(...).as_matrix(), its bits
        C_all = (-np.transpose(R_all, (0, 2, 1)) @ cams[:, 3:, None])[:, :, 0]
        R_set_opt = [R_all[i] for i in range(n_cameras)]
        C_set_opt = [C_all[i] for i in range(n_cameras)]
        if (type(all_world_coords) is np.ndarray and all_world_coords.dtype == np.float64
                and all_world_coords.shape == pts.shape):
            # every row valid (valid_point_indices = arange): the copy with
            # every row replaced is pts itself, a fresh C-order array
            all_world_coords_opt = pts
        else:
            all_world_coords_opt = all_world_coords.copy()  # :231-234
            all_world_coords_opt[valid_point_indices] = pts
        last_timings["post"] = (time.perf_counter() - t4) * 1e3
        print(f"  Bundle adjustment completed. Final cost: {rep['cost']:.6f}")
        return R_set_opt, C_set_opt, all_world_coords_opt
    except Exception as e:
        print(f"  Bundle adjustment failed: {e}")
        return R_set, C_set, all_world_coords
