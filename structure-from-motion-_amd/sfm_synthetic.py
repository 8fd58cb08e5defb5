"""Synthetic workloads for the BASELINE configs.

These generators define the inputs every parity test, fixture and bench line
uses; they are pure numpy and deterministic in their seed.

* ``two_view(...)``   -- cfg2: 5k correspondences, 40 % outliers
  (SURVEY.md §8(d) "cfg2 synthetic 2-view").
* ``ba_problem(...)`` -- cfg3/4/5: cameras on a yaw arc, each point seen by
  ``k`` distinct cameras, pixel noise 0.5, perturbed initial poses / points
  (SURVEY.md §8(d) "cfg3/4/5 synthetic BA").  Returned both as the dense
  ``perform_bundle_adjustment`` arguments (``Phase 1/BundleAdjustment.py:113``)
  and, for large configs, directly as the COO observation list the dense
  path would produce (``Phase 1/BundleAdjustment.py:164-169`` order:
  point-major, camera ascending).
"""
import numpy as np

# Intrinsics hard-coded by the reference driver (Phase 1/Wrapper_dev.py:143).
K_REF = np.array([[531.122155322710, 0.0, 407.192550839899],
                  [0.0, 531.541737503901, 313.308715048366],
                  [0.0, 0.0, 1.0]])


def rotvec_to_matrix(r):
    """Rodrigues formula, (n,3) -> (n,3,3); matches scipy Rotation.from_rotvec."""
    r = np.atleast_2d(np.asarray(r, dtype=np.float64))
    th = np.linalg.norm(r, axis=1)
    out = np.empty((len(r), 3, 3))
    small = th < 1e-6
    th2 = th * th
    with np.errstate(invalid="ignore", divide="ignore"):
        a = np.where(small, 1.0 - th2 / 6.0 + th2 * th2 / 120.0, np.sin(th) / th)
        b = np.where(small, 0.5 - th2 / 24.0 + th2 * th2 / 720.0, (1.0 - np.cos(th)) / th2)
    x, y, z = r[:, 0], r[:, 1], r[:, 2]
    I = np.eye(3)
    Kx = np.zeros((len(r), 3, 3))
    Kx[:, 0, 1], Kx[:, 0, 2] = -z, y
    Kx[:, 1, 0], Kx[:, 1, 2] = z, -x
    Kx[:, 2, 0], Kx[:, 2, 1] = -y, x
    out[:] = I + a[:, None, None] * Kx + b[:, None, None] * (Kx @ Kx)
    return out


def two_view(n=5000, outlier_frac=0.4, seed=0, noise=0.5):
    """cfg2 generator: returns (x1, x2, index, meta)."""
    rng = np.random.default_rng(seed)
    X = np.column_stack([rng.uniform(-3, 3, n), rng.uniform(-2, 2, n), rng.uniform(5, 12, n)])
    R2 = rotvec_to_matrix([0.02, -0.15, 0.01])[0]
    C2 = np.array([1.0, 0.05, 0.1])

    def proj(R, C):
        xc = (R @ (X - C).T).T
        u = (K_REF @ xc.T).T
        return u[:, :2] / u[:, 2:3]

    x1 = proj(np.eye(3), np.zeros(3)) + rng.normal(0, noise, (n, 2))
    x2 = proj(R2, C2) + rng.normal(0, noise, (n, 2))
    n_out = int(round(outlier_frac * n))
    out_idx = rng.choice(n, n_out, replace=False)
    x2[out_idx] = np.column_stack([rng.uniform(0, 800, n_out), rng.uniform(0, 600, n_out)])
    clean1 = proj(np.eye(3), np.zeros(3))
    clean2 = proj(R2, C2)
    meta = dict(X=X, R2=R2, C2=C2, outliers=np.sort(out_idx), clean1=clean1, clean2=clean2)
    return np.ascontiguousarray(x1), np.ascontiguousarray(x2), np.arange(n, dtype=np.int64), meta


BA_CONFIGS = {
    # name: (n_cams, n_pts, k obs per point)
    "tiny": (3, 30, 3),
    "small": (6, 200, 4),
    "cfg3": (6, 2000, 5),
    "cfg4": (50, 100_000, 10),
    "cfg5": (200, 500_000, 8),
}


def ba_problem(n_cams, n_pts, k, seed=3, noise=0.5, pose_noise=0.01, pt_noise=0.05,
               dense=True):
    """cfg3/4/5 generator.

    Returns a dict with the ground truth, the perturbed initial state, and the
    observation list.  With ``dense=True`` it also holds the dense
    ``feature_x/feature_y/filtered_feature_flags`` matrices that
    ``perform_bundle_adjustment`` takes (only sensible for small configs).
    """
    rng = np.random.default_rng(seed)
    k = min(k, n_cams)
    X = np.column_stack([rng.uniform(-2, 2, n_pts), rng.uniform(-2, 2, n_pts),
                         rng.uniform(4, 8, n_pts)])
    yaw = np.linspace(-0.15, 0.15, n_cams)
    C = np.column_stack([3.0 * np.sin(yaw), rng.normal(0, 0.05, n_cams), rng.normal(0, 0.05, n_cams)])
    rv = np.column_stack([rng.normal(0, 0.01, n_cams), -yaw + rng.normal(0, 0.01, n_cams),
                          rng.normal(0, 0.01, n_cams)])
    R = rotvec_to_matrix(rv)
    # each point observed by k distinct cameras (sorted ascending)
    keys = rng.random((n_pts, n_cams))
    cams = np.sort(np.argpartition(keys, k - 1, axis=1)[:, :k], axis=1).astype(np.int32)
    pt_idx = np.repeat(np.arange(n_pts, dtype=np.int32), k)
    cam_idx = cams.reshape(-1)
    Xo = X[pt_idx]
    xc = np.einsum("nij,nj->ni", R[cam_idx], Xo - C[cam_idx])
    u = xc @ K_REF.T
    obs = u[:, :2] / u[:, 2:3] + rng.normal(0, noise, (len(cam_idx), 2))
    # perturbed initialisation
    rv0 = rv + rng.normal(0, pose_noise, rv.shape)
    C0 = C + rng.normal(0, pose_noise, C.shape)
    X0 = X + rng.normal(0, pt_noise, X.shape)
    out = dict(n_cams=n_cams, n_pts=n_pts, k=k, X_true=X, R_true=R, C_true=C,
               rotvec0=rv0, R0=rotvec_to_matrix(rv0), C0=C0, X0=X0,
               cam_idx=cam_idx, pt_idx=pt_idx, obs=np.ascontiguousarray(obs))
    if dense:
        fx = np.zeros((n_pts, n_cams))
        fy = np.zeros((n_pts, n_cams))
        fl = np.zeros((n_pts, n_cams), dtype=np.int64)
        fx[pt_idx, cam_idx] = obs[:, 0]
        fy[pt_idx, cam_idx] = obs[:, 1]
        fl[pt_idx, cam_idx] = 1
        out.update(feature_x=fx, feature_y=fy, flags=fl,
                   filtered_world_coords=np.ones((n_pts, 1), dtype=np.int64))
    return out


def ba_problem_cfg(name, seed=3, dense=None):
    n_cams, n_pts, k = BA_CONFIGS[name]
    if dense is None:
        dense = n_pts * n_cams <= 2_000_000
    return ba_problem(n_cams, n_pts, k, seed=seed, dense=dense)


def rmse_from_cost(cost, n_obs):
    """Per-observation reprojection RMSE (px): sqrt(sum_o |r_o|^2 / n_obs),
    from cost = 0.5 * sum r^2 (the scipy/MINPACK cost the reference prints,
    Phase 1/BundleAdjustment.py:236)."""
    return float(np.sqrt(2.0 * cost / n_obs))
