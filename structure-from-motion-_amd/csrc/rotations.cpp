// scipy.spatial.transform.Rotation conversions for the BA drop-in's camera
// parameters (round 6): perform_bundle_adjustment converts every camera's R
// to [rotvec, t] before the solve (Phase 1/BundleAdjustment.py:183-193) and
// back after it (:220-228).  Through scipy these took ~0.6 ms of the cfg5
// call (200 cameras) for microseconds of arithmetic.  Restated here with
// scipy 1.15.3's operations in its order (its quaternion path: Markley's
// branch on the largest of the diagonal and the trace, normalise, w >= 0,
// angle 2 atan2(|v|, w) with the series below 1e-3; from_rotvec through the
// half-angle quaternion), contraction off, so the bits are scipy's
// (tests/test_abi.py compares them with scipy itself).  scipy orthogonalises
// a matrix that is not orthogonal to within its own tolerance first: a
// matrix with max |R R^T - I| above 1e-13 (scipy's bits measured equal up to
// 6e-13), or a reflection, is reported back and the caller uses scipy for
// the batch.
#include <cmath>
#include <cstdint>

#include "sfm_common.hpp"

#pragma clang fp contract(off)

namespace {

bool near_orthogonal(const double *R) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            const double d = R[3 * i] * R[3 * j] + R[3 * i + 1] * R[3 * j + 1] + R[3 * i + 2] * R[3 * j + 2];
            if (!(std::fabs(d - (i == j ? 1.0 : 0.0)) <= 1e-13)) return false;
        }
    // a reflection (det -1) is orthogonal too: scipy's business
    const double det = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                       R[2] * (R[3] * R[7] - R[4] * R[6]);
    return det > 0.5;
}

void matrix_to_rotvec(const double *R, double *w) {
    const double tr = R[0] + R[4] + R[8];
    double q[4];  // x y z w
    if (tr > R[0] && tr > R[4] && tr > R[8]) {
        q[3] = 1.0 + tr;
        q[0] = R[7] - R[5];
        q[1] = R[2] - R[6];
        q[2] = R[3] - R[1];
    } else {
        const int i = (R[0] >= R[4] && R[0] >= R[8]) ? 0 : (R[4] >= R[8] ? 1 : 2);
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        q[i] = 1.0 - tr + 2.0 * R[i * 4];
        q[j] = R[j * 3 + i] + R[i * 3 + j];
        q[k] = R[k * 3 + i] + R[i * 3 + k];
        q[3] = R[k * 3 + j] - R[j * 3 + k];
    }
    const double nq = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (double &v : q) v /= nq;
    if (q[3] < 0)
        for (double &v : q) v = -v;
    const double vn = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
    const double ang = 2.0 * std::atan2(vn, q[3]);
    double sc;
    if (ang <= 1e-3) {
        const double a2 = ang * ang;
        sc = 2.0 + a2 / 12.0 + 7.0 * a2 * a2 / 2880.0;
    } else {
        sc = ang / std::sin(ang / 2.0);
    }
    w[0] = sc * q[0];
    w[1] = sc * q[1];
    w[2] = sc * q[2];
}

void rotvec_to_matrix(const double *rv, double *R) {
    const double x = rv[0], y = rv[1], z = rv[2];
    const double ang = std::sqrt(x * x + y * y + z * z);
    double sc;
    if (ang <= 1e-3) {
        const double a2 = ang * ang;
        sc = 0.5 - a2 / 48 + a2 * a2 / 3840;
    } else {
        sc = std::sin(ang / 2) / ang;
    }
    const double qx = sc * x, qy = sc * y, qz = sc * z, qw = std::cos(ang / 2);
    const double x2 = qx * qx, y2 = qy * qy, z2 = qz * qz, w2 = qw * qw;
    const double xy = qx * qy, zw = qz * qw, xz = qx * qz, yw = qy * qw, yz = qy * qz, xw = qx * qw;
    R[0] = x2 - y2 - z2 + w2;
    R[1] = 2 * (xy - zw);
    R[2] = 2 * (xz + yw);
    R[3] = 2 * (xy + zw);
    R[4] = -x2 + y2 - z2 + w2;
    R[5] = 2 * (yz - xw);
    R[6] = 2 * (xz - yw);
    R[7] = 2 * (yz + xw);
    R[8] = -x2 - y2 + z2 + w2;
}

}  // namespace

// Rotation.from_matrix(R).as_rotvec() for n row-major 3 x 3 matrices; returns
// the number of matrices outside the orthogonality tolerance (their rotvecs
// are not written: the caller converts the batch with scipy instead)
extern "C" int64_t sfm_matrix_to_rotvec(const double *R, int64_t n, double *w) {
    if (n < 0 || (n && (!R || !w))) return -1;
    int64_t off = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (!near_orthogonal(R + 9 * i)) {
            ++off;
            continue;
        }
        matrix_to_rotvec(R + 9 * i, w + 3 * i);
    }
    return off;
}

// Rotation.from_rotvec(w).as_matrix() for n rotation vectors
extern "C" int sfm_rotvec_to_matrix(const double *w, int64_t n, double *R) {
    SFM_CHECK_ARG(n >= 0 && (n == 0 || (w && R)), "null pointer or bad size");
    for (int64_t i = 0; i < n; ++i) rotvec_to_matrix(w + 3 * i, R + 9 * i);
    return 0;
}
