// Dense visibility -> COO observations for the BA drop-in (rounds 4-5).
// perform_bundle_adjustment's interface (Phase 1/BundleAdjustment.py:113-
// 169) hands over n_features x n_cameras matrices (feature_x, feature_y,
// filtered_feature_flags) and builds the observation list with
//   flags = filtered_feature_flags[valid_point_indices][:, :n_cameras] == 1
//   point_indices, camera_indices = np.where(flags)
//   points_2d = (feature_x[rows, cam], feature_y[rows, cam])
// At cfg5 (500k points x 200 cameras, 8-byte flags) numpy's fancy-indexed
// copy of the flag matrix, the comparison and np.where took ~0.4 s, half of
// the drop-in's call.  Here the rows are scanned once by the host thread
// pool (each job a contiguous block of rows, so the output stays
// point-major with cameras ascending: np.where's row-major order), the
// coordinates gathered at the hits, and the per-job pieces concatenated in
// row order -- into numpy arrays (sfm_dense_obs_read) or straight into the
// BA create's pinned upload buffer (sfm_ba_lm_dense).
//
// Round 5: the comparisons run 8-64 flags per AVX-512 instruction (run-time
// dispatch; the scalar loop otherwise), a block of rows is scanned before its
// coordinates are gathered (the gathers are then independent loads), and
// the pieces are kept across calls, so a repeated call writes into memory
// that is already mapped (first-touch page faults of the ~100 MB of pieces
// had cost more than the scan).
#include <immintrin.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "host_pool.hpp"
#include "sfm_common.hpp"

namespace {

struct Piece {
    std::vector<int32_t> cam, pt;  // grown, never shrunk: size() is capacity
    std::vector<double> xy;
    int64_t n = 0;
    void ensure(int64_t need) {
        if ((int64_t)cam.size() >= need) return;
        const size_t c = (size_t)std::max<int64_t>(need, (int64_t)cam.size() * 3 / 2);
        cam.resize(c);
        pt.resize(c);
        xy.resize(2 * c);
    }
};

struct DenseObs {
    std::vector<Piece> pieces;
    int64_t n = 0, n_rows = 0;
    int32_t n_cams = 0;
};

// the pieces of the last call, reused by the next one (one user at a time;
// a concurrent caller gets its own)
std::mutex g_pool_mu;
DenseObs *g_pool = nullptr;

constexpr int ROW_BLOCK = 32;  // rows scanned before their coordinates are gathered

// NUMA placement (round 6).  The flag and coordinate matrices were written
// by the caller's thread, so their pages sit on one node of a two-socket
// host; scan threads on the other socket read them across the socket link.
// data_node: the node holding most of 16 pages sampled over [p, p + bytes)
// (move_pages in query mode), -1 if unknown or split.
int data_node(const void *p, size_t bytes) {
    const long pg = sysconf(_SC_PAGESIZE);
    if (pg <= 0 || bytes == 0) return -1;
    constexpr int NS = 16;
    void *pages[NS];
    int status[NS];
    for (int i = 0; i < NS; ++i)
        pages[i] = reinterpret_cast<void *>((reinterpret_cast<uintptr_t>(p) + bytes / NS * i) & ~(uintptr_t)(pg - 1));
    if (syscall(SYS_move_pages, 0, (unsigned long)NS, pages, nullptr, status, 0) != 0) return -1;
    int cnt[64] = {0}, best = -1;
    for (int s : status)
        if (s >= 0 && s < 64 && ++cnt[s] > NS / 2) best = s;
    return best;
}
// the CPUs of node n this process may run on (false: none or unreadable)
bool node_cpus(int n, cpu_set_t *set) {
    char path[96];
    std::snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", n);
    FILE *fp = std::fopen(path, "r");
    if (!fp) return false;
    char buf[4096];
    const size_t len = std::fread(buf, 1, sizeof buf - 1, fp);
    std::fclose(fp);
    buf[len] = 0;
    cpu_set_t allowed;
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return false;
    CPU_ZERO(set);
    for (char *q = buf; *q;) {
        char *e;
        const long a = std::strtol(q, &e, 10);
        if (e == q) break;
        long b = a;
        if (*e == '-') b = std::strtol(e + 1, &e, 10);
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c)
            if (CPU_ISSET(c, &allowed)) CPU_SET(c, set);
        q = *e ? e + 1 : e;
    }
    return CPU_COUNT(set) > 0;
}
// the pool workers pinned to one node: each pins itself once per node (a
// thread_local record); the caller's thread is never pinned
thread_local int t_pinned = -1;

inline bool have_avx512() {
    static const bool v = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                          !std::getenv("SFM_DENSE_SCALAR");
    return v;
}

// flags[0..w) == 1 as a bit mask, w <= 64
template <class T>
inline uint64_t mask_scalar(const T *f, int w) {
    uint64_t mk = 0;
    for (int j = 0; j < w; ++j) mk |= (uint64_t)(f[j] == static_cast<T>(1)) << j;
    return mk;
}

__attribute__((target("avx512f,avx512bw"))) inline uint64_t mask512(const double *f, int w) {
    const __m512d one = _mm512_set1_pd(1.0);
    uint64_t mk = 0;
    for (int j = 0; j < w; j += 8) {
        const __mmask8 m = (__mmask8)(w - j >= 8 ? 0xFF : (1u << (w - j)) - 1);
        mk |= (uint64_t)_mm512_mask_cmp_pd_mask(m, _mm512_maskz_loadu_pd(m, f + j), one, _CMP_EQ_OQ) << j;
    }
    return mk;
}
__attribute__((target("avx512f,avx512bw"))) inline uint64_t mask512(const float *f, int w) {
    const __m512 one = _mm512_set1_ps(1.0f);
    uint64_t mk = 0;
    for (int j = 0; j < w; j += 16) {
        const __mmask16 m = (__mmask16)(w - j >= 16 ? 0xFFFF : (1u << (w - j)) - 1);
        mk |= (uint64_t)_mm512_mask_cmp_ps_mask(m, _mm512_maskz_loadu_ps(m, f + j), one, _CMP_EQ_OQ) << j;
    }
    return mk;
}
__attribute__((target("avx512f,avx512bw"))) inline uint64_t mask512(const int64_t *f, int w) {
    const __m512i one = _mm512_set1_epi64(1);
    uint64_t mk = 0;
    for (int j = 0; j < w; j += 8) {
        const __mmask8 m = (__mmask8)(w - j >= 8 ? 0xFF : (1u << (w - j)) - 1);
        mk |= (uint64_t)_mm512_mask_cmpeq_epi64_mask(m, _mm512_maskz_loadu_epi64(m, f + j), one) << j;
    }
    return mk;
}
__attribute__((target("avx512f,avx512bw"))) inline uint64_t mask512(const int32_t *f, int w) {
    const __m512i one = _mm512_set1_epi32(1);
    uint64_t mk = 0;
    for (int j = 0; j < w; j += 16) {
        const __mmask16 m = (__mmask16)(w - j >= 16 ? 0xFFFF : (1u << (w - j)) - 1);
        mk |= (uint64_t)_mm512_mask_cmpeq_epi32_mask(m, _mm512_maskz_loadu_epi32(m, f + j), one) << j;
    }
    return mk;
}
__attribute__((target("avx512f,avx512bw"))) inline uint64_t mask512(const uint8_t *f, int w) {
    const __mmask64 m = w >= 64 ? ~0ull : (1ull << w) - 1;
    return _mm512_mask_cmpeq_epi8_mask(m, _mm512_maskz_loadu_epi8(m, f), _mm512_set1_epi8(1));
}

// rows[r0, r1) into p: per block of ROW_BLOCK rows, the hits (row, camera)
// first, then their coordinates
template <class T, bool AVX, bool PF = true>
void scan_rows(const char *flags, int64_t flag_row_bytes, const int64_t *rows, int64_t r0, int64_t r1, int32_t n_cams,
               const char *fx, const char *fy, int64_t xy_row_bytes, Piece &p) {
    p.n = 0;
    std::vector<int32_t> hr, hc;
    hr.resize((size_t)ROW_BLOCK * n_cams);
    hc.resize((size_t)ROW_BLOCK * n_cams);
    for (int64_t b0 = r0; b0 < r1; b0 += ROW_BLOCK) {
        const int64_t b1 = std::min(r1, b0 + ROW_BLOCK);
        int64_t nh = 0;
        for (int64_t i = b0; i < b1; ++i) {
            const T *fr = reinterpret_cast<const T *>(flags + rows[i] * flag_row_bytes);
            for (int32_t c0 = 0; c0 < n_cams; c0 += 64) {
                const int w = std::min(64, n_cams - c0);
                uint64_t mk;
                if constexpr (AVX) mk = mask512(fr + c0, w);
                else mk = mask_scalar(fr + c0, w);
                while (mk) {
                    const int c = c0 + __builtin_ctzll(mk);
                    if (PF) {  // the coordinates' lines, requested while the block's flags are scanned
                        const int64_t off = rows[i] * xy_row_bytes + (int64_t)c * 8;
                        _mm_prefetch(fx + off, _MM_HINT_T0);
                        _mm_prefetch(fy + off, _MM_HINT_T0);
                    }
                    hc[nh] = c;
                    hr[nh++] = (int32_t)i;
                    mk &= mk - 1;
                }
            }
        }
        p.ensure(p.n + nh);
        int32_t *cam = p.cam.data() + p.n, *pt = p.pt.data() + p.n;
        double *xy = p.xy.data() + 2 * p.n;
        for (int64_t k = 0; k < nh; ++k) {
            const int64_t off = rows[hr[k]] * xy_row_bytes + (int64_t)hc[k] * 8;
            cam[k] = hc[k];
            pt[k] = hr[k];
            xy[2 * k] = *reinterpret_cast<const double *>(fx + off);
            xy[2 * k + 1] = *reinterpret_cast<const double *>(fy + off);
        }
        p.n += nh;
    }
}

template <bool AVX>
void scan_dispatch(int32_t dtype, const char *f, int64_t frb, const int64_t *rows, int64_t r0, int64_t r1, int32_t nc,
                   const char *x, const char *y, int64_t xyrb, Piece &p) {
    switch (dtype) {
    case 0: scan_rows<double, AVX>(f, frb, rows, r0, r1, nc, x, y, xyrb, p); break;
    case 1: scan_rows<float, AVX>(f, frb, rows, r0, r1, nc, x, y, xyrb, p); break;
    case 2: scan_rows<int64_t, AVX>(f, frb, rows, r0, r1, nc, x, y, xyrb, p); break;
    case 3: scan_rows<int32_t, AVX>(f, frb, rows, r0, r1, nc, x, y, xyrb, p); break;
    default: scan_rows<uint8_t, AVX>(f, frb, rows, r0, r1, nc, x, y, xyrb, p); break;
    }
}

}  // namespace

namespace sfm {

// for sfm_ba_lm_dense (ba.hip): the scan's size and its concatenation
bool dense_obs_info(void *handle, int64_t *n, int64_t *n_rows, int32_t *n_cams) {
    if (!handle) return false;
    auto *h = static_cast<DenseObs *>(handle);
    *n = h->n;
    *n_rows = h->n_rows;
    *n_cams = h->n_cams;
    return true;
}

int dense_obs_pieces(void *handle, std::vector<int64_t> &off) {
    auto *h = static_cast<DenseObs *>(handle);
    const size_t np = h->pieces.size();
    off.assign(np + 1, 0);
    for (size_t t = 0; t < np; ++t) off[t + 1] = off[t] + h->pieces[t].n;
    return (int)np;
}

// pieces [t0, t1) to their places in the concatenated arrays (off:
// dense_obs_pieces); a null destination is skipped
void dense_obs_copy_pieces(void *handle, const std::vector<int64_t> &off, int t0, int t1, int32_t *cam, int32_t *pt,
                           double *obs) {
    auto *h = static_cast<DenseObs *>(handle);
    par_for_dynamic((int64_t)(t1 - t0), [&](int64_t k) {
        const int64_t t = t0 + k;
        const Piece &p = h->pieces[t];
        if (!p.n) return;
        if (cam) std::memcpy(cam + off[t], p.cam.data(), p.n * sizeof(int32_t));
        if (pt) std::memcpy(pt + off[t], p.pt.data(), p.n * sizeof(int32_t));
        if (obs) std::memcpy(obs + 2 * off[t], p.xy.data(), 2 * p.n * sizeof(double));
    });
}

void dense_obs_copy(void *handle, int32_t *cam, int32_t *pt, double *obs) {
    std::vector<int64_t> off;
    const int np = dense_obs_pieces(handle, off);
    dense_obs_copy_pieces(handle, off, 0, np, cam, pt, obs);
}

}  // namespace sfm

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
    // jobs of >= 1024 rows, dealt dynamically to up to 16 threads (round 6:
    // 64 jobs of 4096+ rows in contiguous blocks per thread had the scan time
    // set by the slowest thread -- 7 to 16 ms at cfg5 on a shared host)
    int nj = n_threads > 0 ? n_threads : 256;
    nj = (int)std::max<int64_t>(1, std::min<int64_t>(nj, (n_rows + 1023) / 1024));
    DenseObs *h = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        if (g_pool) {
            h = g_pool;
            g_pool = nullptr;
        }
    }
    if (!h) h = new DenseObs();
    if ((int)h->pieces.size() < nj) h->pieces.resize(nj);
    for (auto &p : h->pieces) p.n = 0;
    h->n_rows = n_rows;
    h->n_cams = n_cams;
    const char *f = static_cast<const char *>(flags);
    const char *x = reinterpret_cast<const char *>(fx), *y = reinterpret_cast<const char *>(fy);
    const bool avx = have_avx512();
    // SFM_SCAN_PIN=0: no pinning (the A/B of tools/e2e_ab.py)
    static const bool pin_on = !std::getenv("SFM_SCAN_PIN") || std::atoi(std::getenv("SFM_SCAN_PIN")) != 0;
    cpu_set_t node_set;
    const int node = pin_on && n_rows ? data_node(f + rows[0] * flag_row_bytes, (size_t)flag_row_bytes * n_rows) : -1;
    const bool pin = node >= 0 && node_cpus(node, &node_set);
    const std::thread::id caller = std::this_thread::get_id();
    // SFM_TEST_SCAN_THROW=k (tests): job k throws std::bad_alloc, as a failed
    // piece allocation would (the exception contract of csrc/host_pool.hpp)
    const char *thr = std::getenv("SFM_TEST_SCAN_THROW");
    const int64_t throw_job = thr ? std::atoll(thr) : -1;
    const int rc = sfm::abi_guard("sfm_dense_obs_scan", [&] {
        sfm::par_for_dynamic(nj, [&](int64_t t) {
            if (t == throw_job) throw std::bad_alloc();
            if (pin && t_pinned != node && std::this_thread::get_id() != caller) {
                t_pinned = sched_setaffinity(0, sizeof node_set, &node_set) == 0 ? node : -2;
            }
            const int64_t r0 = n_rows * t / nj, r1 = n_rows * (t + 1) / nj;
            Piece &p = h->pieces[t];
            if (avx) scan_dispatch<true>(dtype, f, flag_row_bytes, rows, r0, r1, n_cams, x, y, xy_row_bytes, p);
            else scan_dispatch<false>(dtype, f, flag_row_bytes, rows, r0, r1, n_cams, x, y, xy_row_bytes, p);
        });
        return 0;
    });
    if (rc) {
        delete h;
        return rc;
    }
    h->n = 0;
    for (auto &p : h->pieces) h->n += p.n;
    *handle = h;
    *n_obs = h->n;
    return 0;
}

extern "C" int sfm_dense_obs_read(void *handle, int32_t *cam, int32_t *pt, double *obs) {
    SFM_CHECK_ARG(handle, "null handle");
    auto *h = static_cast<DenseObs *>(handle);
    SFM_CHECK_ARG(h->n == 0 || (cam && pt && obs), "null pointer");
    sfm::dense_obs_copy(handle, cam, pt, obs);
    return 0;
}

extern "C" int sfm_dense_obs_free(void *handle) {
    auto *h = static_cast<DenseObs *>(handle);
    if (!h) return 0;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (!g_pool) {
        g_pool = h;  // kept for the next scan
        return 0;
    }
    delete h;
    return 0;
}

// perform_bundle_adjustment's x0 points (BundleAdjustment.py:196-197: the
// valid rows of all_world_coords, 3 doubles each) gathered on the host pool:
// dst[i] = src[rows[i]] (rows null: src[i]).  numpy's fancy-indexed copy of
// 500k rows took ~3 ms of the cfg5 call on one thread.
extern "C" int sfm_gather_rows3(const double *src, int64_t src_rows, const int64_t *rows, int64_t n, double *dst) {
    SFM_CHECK_ARG(n == 0 || (src && dst), "null pointer");
    SFM_CHECK_ARG(n >= 0 && src_rows >= 0, "bad sizes");
    constexpr int NJ = 64;
    const int nj = n >= 65536 ? NJ : 1;  // small gathers: one thread; large ones dealt dynamically
    int bad[NJ] = {0};
    const int rc = sfm::abi_guard("sfm_gather_rows3", [&] {
        sfm::par_for_dynamic(nj, [&](int64_t t) {
            for (int64_t i = n * t / nj; i < n * (t + 1) / nj; ++i) {
                const int64_t r = rows ? rows[i] : i;
                if (r < 0 || r >= src_rows) {
                    bad[t] = 1;
                    continue;
                }
                dst[3 * i] = src[3 * r];
                dst[3 * i + 1] = src[3 * r + 1];
                dst[3 * i + 2] = src[3 * r + 2];
            }
        });
        return 0;
    });
    if (rc) return rc;
    for (int t = 0; t < NJ; ++t) SFM_CHECK_ARG(!bad[t], "row index out of bounds");
    return 0;
}
