// Dense visibility -> COO observations for the BA drop-in (round 4).
// perform_bundle_adjustment's interface (Phase 1/BundleAdjustment.py:113-
// 169) hands over n_features x n_cameras matrices (feature_x, feature_y,
// filtered_feature_flags) and builds the observation list with
//   flags = filtered_feature_flags[valid_point_indices][:, :n_cameras] == 1
//   point_indices, camera_indices = np.where(flags)
//   points_2d = (feature_x[rows, cam], feature_y[rows, cam])
// At cfg5 (500k points x 200 cameras, 8-byte flags) numpy's fancy-indexed
// copy of the flag matrix, the comparison and np.where took ~0.4 s, half of
// the drop-in's call.  Here the rows are scanned once by a thread pool (each
// thread a contiguous block of rows, so the output stays point-major with
// cameras ascending: np.where's row-major order), the coordinates gathered
// at the hits, and the per-thread pieces concatenated in row order.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "sfm_common.hpp"

namespace {

struct Piece {
    std::vector<int32_t> cam, pt;
    std::vector<double> xy;
};

struct DenseObs {
    std::vector<Piece> pieces;
    int64_t n = 0;
};

// a row in 64-camera words: the comparisons into a bit mask (branch-free,
// vectorised), then one visit per hit
template <class T>
void scan_rows(const char *flags, int64_t flag_row_bytes, const int64_t *rows, int64_t r0, int64_t r1, int32_t n_cams,
               const char *fx, const char *fy, int64_t xy_row_bytes, Piece &out) {
    out.cam.reserve((size_t)(r1 - r0) * 8);
    out.pt.reserve((size_t)(r1 - r0) * 8);
    out.xy.reserve((size_t)(r1 - r0) * 16);
    for (int64_t i = r0; i < r1; ++i) {
        const int64_t r = rows[i];
        const T *fr = reinterpret_cast<const T *>(flags + r * flag_row_bytes);
        const double *xr = reinterpret_cast<const double *>(fx + r * xy_row_bytes);
        const double *yr = reinterpret_cast<const double *>(fy + r * xy_row_bytes);
        for (int32_t c0 = 0; c0 < n_cams; c0 += 64) {
            const int w = std::min(64, n_cams - c0);
            uint64_t mk = 0;
            if (w == 64) {
                for (int j = 0; j < 64; ++j) mk |= (uint64_t)(fr[c0 + j] == static_cast<T>(1)) << j;
            } else {
                for (int j = 0; j < w; ++j) mk |= (uint64_t)(fr[c0 + j] == static_cast<T>(1)) << j;
            }
            while (mk) {
                const int c = c0 + __builtin_ctzll(mk);
                mk &= mk - 1;
                out.cam.push_back(c);
                out.pt.push_back((int32_t)i);
                out.xy.push_back(xr[c]);
                out.xy.push_back(yr[c]);
            }
        }
    }
}

}  // namespace

extern "C" int sfm_dense_obs_scan(const void *flags, int32_t dtype, int64_t flag_row_bytes, int64_t n_matrix_rows,
                                  const int64_t *rows, int64_t n_rows, int32_t n_cams, const double *fx,
                                  const double *fy, int64_t xy_row_bytes, int32_t n_threads, void **handle,
                                  int64_t *n_obs) {
    SFM_CHECK_ARG(handle && n_obs && (n_rows == 0 || (flags && rows && fx && fy)), "null pointer");
    SFM_CHECK_ARG(n_rows >= 0 && n_cams >= 0 && n_rows < ((int64_t)1 << 31) && n_matrix_rows >= 0, "bad sizes");
    // every row index inside the matrices (the reference's fancy index raises
    // IndexError there, BundleAdjustment.py:166; the binding raises it first)
    for (int64_t i = 0; i < n_rows; ++i)
        SFM_CHECK_ARG(rows[i] >= 0 && rows[i] < n_matrix_rows, "row index out of bounds of the flag matrix");
    SFM_CHECK_ARG(dtype >= 0 && dtype <= 4, "flag dtype: 0 f64, 1 f32, 2 i64, 3 i32, 4 u8/bool");
    int nt = n_threads > 0 ? n_threads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, (n_rows + 4095) / 4096));
    auto *h = new DenseObs();
    h->pieces.resize(nt);
    auto work = [&](int t) {
        const int64_t r0 = n_rows * t / nt, r1 = n_rows * (t + 1) / nt;
        Piece &p = h->pieces[t];
        const char *f = static_cast<const char *>(flags);
        const char *x = reinterpret_cast<const char *>(fx), *y = reinterpret_cast<const char *>(fy);
        switch (dtype) {
        case 0: scan_rows<double>(f, flag_row_bytes, rows, r0, r1, n_cams, x, y, xy_row_bytes, p); break;
        case 1: scan_rows<float>(f, flag_row_bytes, rows, r0, r1, n_cams, x, y, xy_row_bytes, p); break;
        case 2: scan_rows<int64_t>(f, flag_row_bytes, rows, r0, r1, n_cams, x, y, xy_row_bytes, p); break;
        case 3: scan_rows<int32_t>(f, flag_row_bytes, rows, r0, r1, n_cams, x, y, xy_row_bytes, p); break;
        default: scan_rows<uint8_t>(f, flag_row_bytes, rows, r0, r1, n_cams, x, y, xy_row_bytes, p); break;
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto &t : th) t.join();
    for (auto &p : h->pieces) h->n += (int64_t)p.cam.size();
    *handle = h;
    *n_obs = h->n;
    return 0;
}

extern "C" int sfm_dense_obs_read(void *handle, int32_t *cam, int32_t *pt, double *obs) {
    SFM_CHECK_ARG(handle, "null handle");
    auto *h = static_cast<DenseObs *>(handle);
    SFM_CHECK_ARG(h->n == 0 || (cam && pt && obs), "null pointer");
    std::vector<int64_t> off(h->pieces.size() + 1, 0);
    for (size_t t = 0; t < h->pieces.size(); ++t) off[t + 1] = off[t] + (int64_t)h->pieces[t].cam.size();
    auto copy = [&](size_t t) {
        const Piece &p = h->pieces[t];
        const size_t n = p.cam.size();
        if (!n) return;
        std::memcpy(cam + off[t], p.cam.data(), n * sizeof(int32_t));
        std::memcpy(pt + off[t], p.pt.data(), n * sizeof(int32_t));
        std::memcpy(obs + 2 * off[t], p.xy.data(), 2 * n * sizeof(double));
    };
    std::vector<std::thread> th;
    for (size_t t = 1; t < h->pieces.size(); ++t) th.emplace_back(copy, t);
    if (!h->pieces.empty()) copy(0);
    for (auto &t : th) t.join();
    return 0;
}

extern "C" int sfm_dense_obs_free(void *handle) {
    delete static_cast<DenseObs *>(handle);
    return 0;
}
