// Batched RANSAC engine for gfx950, templated on the model:
//   EpiModel  fundamental matrix, 8-point samples, symmetric epipolar
//             distance (GetInliersRANSAC.py:5-106)
//   HomModel  homography, 4-point samples, transfer error
//             (GetHomographyInliers.py:88-165)
// Kernels:
//   k_fit_samples<M>   gather the K sampled correspondences and fit the 3x3
//                      model: 8 lanes per hypothesis for F (f8_points_group8),
//                      one thread per hypothesis for H.
//   k_epi_score        (F) correspondences resident in registers (a packed
//                      float copy), a workgroup's hypotheses streamed through
//                      them: packed float prefilter, survivors queued in LDS
//                      for the FP64 test one lane each (round 5).
//   k_ransac_score<M>  (H) one WAVE per hypothesis: the model is
//                      wave-uniform (scalar registers); correspondence tiles
//                      are staged once per workgroup in LDS and every wave
//                      sweeps them, one correspondence per lane; inlier
//                      count = popcount of the wave ballot (scalar unit).
//   k_ransac_select<M> one workgroup: (max count, min iteration) reduction ==
//                      the reference's strict '>' update, then the inlier
//                      mask of the winner.
#pragma once
#include <algorithm>
#include <atomic>
#include <immintrin.h>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <sched.h>
#include <thread>
#include <vector>

#include "sfm_common.hpp"
#include "sfm_geom.hpp"
#include "pyrandom.hpp"
#include "select.hpp"
#include "host_pool.hpp"

namespace sfm {

constexpr int SCORE_WAVES = 8;          // hypotheses per workgroup
constexpr int SCORE_TILE = 1024;        // correspondences per LDS tile (32 KiB)

struct EpiModel {
    static constexpr int K = 8;
    static constexpr bool GROUP_FIT = true;  // has an 8-lane fit (f8_points_group8)
    __device__ static void fit(const double (&ax)[K], const double (&ay)[K], const double (&bx)[K],
                               const double (&by)[K], double *out) {
        f8_points(ax, ay, bx, by, out);
    }
    __device__ static bool inlier(const double *f, double2 p, double2 q, double thr) {
        return epi_inlier(f, p.x, p.y, q.x, q.y, thr);
    }
    __device__ static bool inlier_fast(const double *f, double2 p, double2 q, double thr, double lo, double hi) {
        return epi_inlier_fast(f, p.x, p.y, q.x, q.y, thr, lo, hi);
    }
    using Part = EpiPart;
    __device__ static Part fast(const double *f, double2 p, double2 q, double, double lo, double hi) {
        return epi_fast(f, p.x, p.y, q.x, q.y, lo, hi);
    }
    static constexpr bool SPLIT = true;  // fast() as fast_b(fast_a()): the wave-level outlier skip
    using PartA = EpiPartA;
    __device__ static PartA fast_a(const double *f, double2 p, double2 q, double hi) {
        return epi_fast_a(f, p.x, p.y, q.x, q.y, hi);
    }
    __device__ static Part fast_b(const PartA &a, const double *f, double2 q, double lo, double hi) {
        return epi_fast_b(a, f, q.x, q.y, lo, hi);
    }
    __device__ static bool exact(const Part &r, double2, double2, const double *, double thr) {
        return epi_exact(r, thr);
    }
};

struct HomModel {
    static constexpr int K = 4;
    static constexpr bool GROUP_FIT = false;
    __device__ static void fit(const double (&ax)[K], const double (&ay)[K], const double (&bx)[K],
                               const double (&by)[K], double *out) {
        h4_points(ax, ay, bx, by, out);
    }
    __device__ static bool inlier(const double *f, double2 p, double2 q, double thr) {
        return hom_inlier(f, p.x, p.y, q.x, q.y, thr);
    }
    __device__ static bool inlier_fast(const double *f, double2 p, double2 q, double thr, double, double) {
        return hom_inlier(f, p.x, p.y, q.x, q.y, thr);
    }
    using Part = HomPart;
    __device__ static Part fast(const double *f, double2 p, double2 q, double thr, double, double) {
        return hom_fast(f, p.x, p.y, q.x, q.y, thr);
    }
    __device__ static bool exact(const Part &r, double2, double2 q, const double *, double thr) {
        return hom_exact(r, q.x, q.y, thr);
    }
    static constexpr bool SPLIT = false;
    using PartA = Part;
    __device__ static PartA fast_a(const double *, double2, double2, double) { return {}; }
    __device__ static Part fast_b(const PartA &a, const double *, double2, double, double) { return a; }
};

template <class M>
__global__ void __launch_bounds__(256) k_fit_samples(const double2 *__restrict__ x1, const double2 *__restrict__ x2,
                                                     const int32_t *__restrict__ samples, int64_t H,
                                                     double *__restrict__ out, int32_t *__restrict__ counts) {
    if constexpr (M::GROUP_FIT) {  // 8 lanes per hypothesis, as in the fused launches (same bits)
        const int64_t h = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
        if (h >= H) return;
        const int i = threadIdx.x & 7;
        if (counts && i == 0) counts[h] = 0;
        const int32_t sidx = samples[h * 8 + i];
        const double2 p = x1[sidx], q = x2[sidx];
        f8_points_group8(p.x, p.y, q.x, q.y, out + 9 * h);
        return;
    }
    const int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= H) return;
    if (counts) counts[h] = 0;  // the point-sliced score accumulates into it
    double ax[M::K], ay[M::K], bx[M::K], by[M::K];
#pragma unroll
    for (int i = 0; i < M::K; ++i) {
        const int32_t s = samples[h * M::K + i];
        const double2 p = x1[s], q = x2[s];
        ax[i] = p.x; ay[i] = p.y; bx[i] = q.x; by[i] = q.y;
    }
    M::fit(ax, ay, bx, by, out + 9 * h);
}

// fit H hypotheses whose sample rows are at rows (device-readable)
template <class M>
static int launch_fit(const double2 *d1, const double2 *d2, const int32_t *rows, int64_t H, double *dF,
                      int32_t *counts, hipStream_t s) {
    if constexpr (M::GROUP_FIT)
        hipLaunchKernelGGL(k_fit_samples<M>, dim3(ceil_div(H * 8, 256)), dim3(256), 0, s, d1, d2, rows, H, dF, counts);
    else
        hipLaunchKernelGGL(k_fit_samples<M>, dim3(ceil_div(H, 64)), dim3(64), 0, s, d1, d2, rows, H, dF, counts);
    SFM_HIP(hipGetLastError());
    return 0;
}

// samples given as coordinates (H x K x 2 each): the batch fit entry points
template <class M>
__global__ void __launch_bounds__(256) k_fit_points(const double2 *__restrict__ x1s, const double2 *__restrict__ x2s,
                                                    int64_t H, double *__restrict__ out) {
    const int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= H) return;
    double ax[M::K], ay[M::K], bx[M::K], by[M::K];
#pragma unroll
    for (int i = 0; i < M::K; ++i) {
        const double2 p = x1s[h * M::K + i], q = x2s[h * M::K + i];
        ax[i] = p.x; ay[i] = p.y; bx[i] = q.x; by[i] = q.y;
    }
    M::fit(ax, ay, bx, by, out + 9 * h);
}

// The next chunk's fit, carried by the first nfb workgroups of a score
// launch (row y = 0): 8 lanes per hypothesis (f8_points_group8), so the
// launch keeps the score's register budget, and the fit runs beside the
// score instead of between two score launches.
struct FitNext {
    const int32_t *rows;  // nh x K sample rows (pinned, zero-copy)
    int64_t nh;
    double *F;            // nh x 9
    int32_t *counts;      // zeroed when the next score is point-sliced, else null
    int nfb;              // fit workgroups (64 hypotheses each)
};
constexpr int FIT_PER_WG = 64 * SCORE_WAVES / 8;  // k_ransac_score's fit workgroups (8 lanes a hypothesis)

template <class M, int PER_WG = FIT_PER_WG>
__device__ __forceinline__ void fit_next_group(const double2 *__restrict__ x1, const double2 *__restrict__ x2,
                                               const FitNext &fn) {
    const int64_t h = (int64_t)blockIdx.x * PER_WG + (threadIdx.x >> 3);
    if (h >= fn.nh) return;
    const int i = threadIdx.x & 7;
    if (fn.counts && i == 0) fn.counts[h] = 0;
    const int32_t sidx = fn.rows[h * 8 + i];
    const double2 p = x1[sidx], q = x2[sidx];
    f8_points_group8(p.x, p.y, q.x, q.y, fn.F + 9 * h);
}

// waves per SIMD the fused launch is compiled for: the F score needs 64
// VGPRs (six waves a SIMD: its 48-KB LDS tiles allow three workgroups a CU),
// the fit's rank-2 step (with its Jacobi fallback) ~120, so the cap makes
// the fit spill (off the critical path) rather than the score lose
// occupancy (round 5: 8 could not be met, the compiler then gave the whole
// launch 126 VGPRs)
#ifndef SFM_SCORE_FIT_OCC
#define SFM_SCORE_FIT_OCC 6
#endif
// score_split bits: 1 the wave-level outlier skip after stage A, 2 the float
// prefilter ahead of it (k_epi_score)
constexpr int SCORE_SKIP_A = 1, SCORE_PRE32 = 2;

// The H score (and, before round 5, the F one): correspondence tiles staged
// in LDS, every wave sweeping them for its hypothesis, both fast decisions
// of a pass before either branch to the exact tail.
template <class M, bool FIT = false>
__global__ void __launch_bounds__(64 * SCORE_WAVES, FIT ? SFM_SCORE_FIT_OCC : 1) k_ransac_score(const double2 *__restrict__ x1,
                                                                   const double2 *__restrict__ x2,
                                                                   int64_t N, const double *__restrict__ F,
                                                                   int64_t H, double thr,
                                                                   int32_t *__restrict__ counts, int64_t slice,
                                                                   FitNext fn) {
    static_assert(!M::SPLIT, "the F model scores in k_epi_score");
    __shared__ double2 s1[SCORE_TILE];
    __shared__ double2 s2[SCORE_TILE];
    int bx = blockIdx.x;
    if (FIT) {
        if (bx < fn.nfb) {
            if (blockIdx.y == 0) fit_next_group<M>(x1, x2, fn);
            return;
        }
        bx -= fn.nfb;
    }
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t h = (int64_t)bx * SCORE_WAVES + wave;
    const bool active = h < H;
    double f[9];
    int finite = 1;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        f[k] = active ? F[9 * h + k] : 0.0;
        finite &= isfinite(f[k]) ? 1 : 0;
    }
    int cnt = 0;
    // the fast decision's band around 2 thr (epi_inlier_fast compares the
    // doubled mean)
    const double thr_lo = 2.0 * (thr >= 0 ? thr * (1.0 - 1e-4) : thr * (1.0 + 1e-4));
    const double thr_hi = 2.0 * (thr >= 0 ? thr * (1.0 + 1e-4) : thr * (1.0 - 1e-4));
    // gridDim.y > 1: this workgroup scores correspondences [y*slice, (y+1)*slice)
    const int64_t p0 = (int64_t)blockIdx.y * slice, p1 = min<int64_t>(N, p0 + slice);
    for (int64_t base = p0; base < p1; base += SCORE_TILE) {
        const int n = (int)min<int64_t>(SCORE_TILE, p1 - base);
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            s1[i] = x1[base + i];
            s2[i] = x2[base + i];
        }
        __syncthreads();
        if (active && finite) {
            // two correspondences per lane per pass: independent chains for the
            // FP64 pipe (the tile length is a multiple of 128 except the last)
            int j = 0;
            for (; j + 128 <= n; j += 128) {
                const double2 p0 = s1[j + lane], q0 = s2[j + lane];
                const double2 p1 = s1[j + 64 + lane], q1 = s2[j + 64 + lane];
                const typename M::Part r0 = M::fast(f, p0, q0, thr, thr_lo, thr_hi);
                const typename M::Part r1 = M::fast(f, p1, q1, thr, thr_lo, thr_hi);
                bool in0 = r0.in, in1 = r1.in;
                if (r0.unsure) in0 = M::exact(r0, p0, q0, f, thr);
                if (r1.unsure) in1 = M::exact(r1, p1, q1, f, thr);
                cnt += __popcll(__ballot(in0)) + __popcll(__ballot(in1));
            }
            for (; j < n; j += 64) {
                const int i = j + lane;
                bool inl = false;
                if (i < n) {
                    const double2 p = s1[i], q = s2[i];
                    inl = M::inlier_fast(f, p, q, thr, thr_lo, thr_hi);
                }
                cnt += __popcll(__ballot(inl));
            }
        }
        __syncthreads();
    }
    if (active && lane == 0) {
        if (gridDim.y == 1)
            counts[h] = cnt;
        else
            atomicAdd(counts + h, cnt);
    }
}

// The F score (round 5): the correspondences stay in registers and the
// hypotheses stream through them.  A workgroup of EPI_W waves takes hb
// hypotheses (hb <= 64) and a range of 128-pair passes; a wave holds
// EPI_SLOTS passes at a time in registers (the packed float copy
// k_stage_tiles writes: lane l of a pass has (x, x', y, y') and
// (u, u', v, v') of pairs l and 64 + l), loaded once, and runs every
// hypothesis of the workgroup over them.  Per hypothesis:
//  * its prefilter constants (epi_pre_setup: the model scaled by a power of
//    two and rounded to float, the bounds for the workgroup's coordinate
//    range) are computed once per workgroup, by lane t of wave 0 for
//    hypothesis t, and read back from LDS as broadcast pairs;
//  * the packed prefilter runs on every slot (rigorous "outlier" proofs,
//    14 instructions per 128 pairs); the pairs it leaves (cfg2: ~6 of 5000
//    a hypothesis) go to the workgroup's LDS queue, and after the loop
//    every lane takes one queued (hypothesis, pair) through the FP64 test
//    (the reference's decision bit for bit), so the rare survivors cost
//    one lane each instead of a wave-wide test; a full queue falls back to
//    the FP64 test in place;
//  * a hypothesis whose prefilter is off (pk null, SFM_SCORE_PRE=0,
//    coordinates past 2^24, a model too large or small to scale) runs the
//    round-4 FP64 test over the wave's passes, from global memory.
// Counts: a wave's in lane k of a register, the workgroup's summed in LDS,
// stored (one pass range) or added (several) per hypothesis.
// Measured, cfg2 one-shot (16384 hypotheses x 5000 pairs), same box:
// round-4 FP64 score 86 us; the round-5 first form (one wave per
// hypothesis sweeping LDS tiles of the float copy, the survivors through a
// wave-wide float test) 66.6; this form 58.5 with the wave-wide test, 55.0
// with the queue at 4 slots, 49.6 at 5 (cfg2's 40 passes in one range of 8
// waves), 51.6 at 6 (registers spill).  The instruction count bounds it:
// 20.8 M VALU per launch (5 of 9 in the prefilter) against 58 us at 4
// cycles each over 1024 SIMDs.
#ifndef SFM_EPI_SLOTS
#define SFM_EPI_SLOTS 5
#endif
constexpr int EPI_SLOTS = SFM_EPI_SLOTS;  // 128-pair passes a wave holds
constexpr int EPI_W = 8;                  // waves a workgroup
constexpr int EPI_HB_MAX = 64;            // hypotheses a workgroup (a setup lane each)
constexpr int EPI_QCAP = 4096;            // candidates a workgroup queues
#ifndef SFM_EPI_OCC
#define SFM_EPI_OCC 4
#endif
#ifndef SFM_EPI_PROBE
#define SFM_EPI_PROBE 0
#endif
#ifndef SFM_EPI_FIT_OCC
#define SFM_EPI_FIT_OCC 4
#endif

// the FP64 test of two 64-pair sets (pair a = lane, b = 64 + lane) for one
// hypothesis: the number of inliers among the 128 pairs
__device__ __forceinline__ int epi_sets_f64(const double *f, double2 pa, double2 qa, double2 pb, double2 qb, double thr,
                                            double thr_lo, double thr_hi, int score_split) {
    using M = EpiModel;
    const M::PartA sa = M::fast_a(f, pa, qa, thr_hi);
    const M::PartA sb = M::fast_a(f, pb, qb, thr_hi);
    const bool n0 = !(score_split & SCORE_SKIP_A) || __ballot(!sa.out) != 0;
    const bool n1 = !(score_split & SCORE_SKIP_A) || __ballot(!sb.out) != 0;
    if (!n0 && !n1) return 0;
    bool in0 = false, in1 = false;
    if (n0 && n1) {
        const M::Part r0 = M::fast_b(sa, f, qa, thr_lo, thr_hi);
        const M::Part r1 = M::fast_b(sb, f, qb, thr_lo, thr_hi);
        in0 = r0.in;
        in1 = r1.in;
        if (r0.unsure) in0 = M::exact(r0, pa, qa, f, thr);
        if (r1.unsure) in1 = M::exact(r1, pb, qb, f, thr);
    } else {
        const bool first = n0;  // the one set that needs stage B
        const M::Part r = M::fast_b(first ? sa : sb, f, first ? qa : qb, thr_lo, thr_hi);
        bool in = r.in;
        if (r.unsure) in = M::exact(r, first ? pa : pb, first ? qa : qb, f, thr);
        in0 = first && in;
        in1 = !first && in;
    }
    return __popcll(__ballot(in0)) + __popcll(__ballot(in1));
}

template <bool FIT = false>
__global__ void __launch_bounds__(64 * EPI_W, FIT ? SFM_EPI_FIT_OCC : SFM_EPI_OCC)
    k_epi_score(const double2 *__restrict__ x1, const double2 *__restrict__ x2, int64_t N, const double *__restrict__ F,
                int64_t H, double thr, int32_t *__restrict__ counts, int hb, FitNext fn, int score_split,
                const float4 *__restrict__ tmax, const float4 *__restrict__ pk) {
    using M = EpiModel;
    // per hypothesis, 6 quads: (flags, -, q1, q1) (q0, q0, g0, g0) (g1, g1, g2, g2)
    // (g3, g3, g4, g4) (g5, g5, g6, g6) (g7, g7, g8, g8)
    __shared__ float4 sC[EPI_HB_MAX][6];
    __shared__ int sCnt[EPI_HB_MAX];
    // the candidates the prefilter leaves, (hypothesis << 26 | pair - 128 P0)
    __shared__ uint32_t sQ[EPI_QCAP];
    __shared__ int sQn;
    int bx = blockIdx.x;
    if (FIT) {
        if (bx < fn.nfb) {
            if (blockIdx.y == 0) fit_next_group<M, 64 * EPI_W / 8>(x1, x2, fn);
            return;
        }
        bx -= fn.nfb;
    }
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t h0 = (int64_t)bx * hb;
    const int nh = (int)min<int64_t>(hb, H - h0);
    // a model in FP64 (the FP64 tests: from memory -- the scalar cache --
    // rather than held in scalar registers across the hypothesis loop)
    auto load_f = [&](int64_t h, double (&f)[9]) {
        asm volatile("" ::: "memory");
#pragma unroll
        for (int q = 0; q < 9; ++q) f[q] = F[9 * h + q];
    };
    auto band = [&](double &lo, double &hi) {  // the FP64 test's band around 2 thr
        lo = 2.0 * (thr >= 0 ? thr * (1.0 - 1e-4) : thr * (1.0 + 1e-4));
        hi = 2.0 * (thr >= 0 ? thr * (1.0 + 1e-4) : thr * (1.0 - 1e-4));
    };
    const int P = (int)((N + 127) >> 7);  // 128-pair passes (N < 2^31)
    const int P0 = (int)((int64_t)blockIdx.y * P / gridDim.y), P1 = (int)((int64_t)(blockIdx.y + 1) * P / gridDim.y);
    const bool use_pre = pk && tmax && (score_split & SCORE_PRE32);  // workgroup-uniform
    if (threadIdx.x < EPI_HB_MAX) {  // wave 0: hypothesis h0 + t's constants
        const int t = threadIdx.x;
        int flags = 0;
        EpiPre p{};
        double f[9];
        bool fin = t < nh;
#pragma unroll
        for (int q = 0; q < 9; ++q) {
            f[q] = t < nh ? F[9 * (h0 + t) + q] : 0.0;
            fin = fin && isfinite(f[q]);
        }
        // the coordinate bounds of the workgroup's passes: the wave's lanes
        // take the tiles in turn (one load latency for the usual few), then
        // a wave max
        float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
        if (use_pre) {
            const int64_t e = min<int64_t>(N, (int64_t)P1 * 128);
            for (int64_t i = (int64_t)P0 * 128 / SCORE_TILE + t; i * SCORE_TILE < e; i += 64) {
                const float4 q = tmax[i];
                b = make_float4(fmaxf(b.x, q.x), fmaxf(b.y, q.y), fmaxf(b.z, q.z), fmaxf(b.w, q.w));
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1)
                b = make_float4(fmaxf(b.x, __shfl_xor(b.x, o)), fmaxf(b.y, __shfl_xor(b.y, o)),
                                fmaxf(b.z, __shfl_xor(b.z, o)), fmaxf(b.w, __shfl_xor(b.w, o)));
        }
        if (fin) {
            flags = 1;
            if (use_pre && SFM_EPI_PROBE != 3) {
                double lo, hi;
                band(lo, hi);
                p = epi_pre_setup(f, hi, b);
                if (p.on) flags |= 2;
            }
        }
#if SFM_EPI_PROBE == 3 || SFM_EPI_PROBE == 4  // timing probes (wrong counts): no setup / setup, no loop
        flags = 0;
#endif
        sC[t][0] = make_float4(__int_as_float(flags), 0.f, p.q1, p.q1);
        sC[t][1] = make_float4(p.q0, p.q0, p.g[0], p.g[0]);
#pragma unroll
        for (int k = 0; k < 4; ++k) sC[t][2 + k] = make_float4(p.g[1 + 2 * k], p.g[1 + 2 * k], p.g[2 + 2 * k], p.g[2 + 2 * k]);
        sCnt[t] = 0;
        if (t == 0) sQn = 0;
    }
    int cntv = 0;  // lane k: this wave's count for hypothesis h0 + k
    bool first = true;
    for (int base = P0 + wave; base < P1; base += EPI_W * EPI_SLOTS) {
        // slot s: pass base + s EPI_W
        float4 A[EPI_SLOTS], B[EPI_SLOTS];
#pragma unroll
        for (int s = 0; s < EPI_SLOTS; ++s) {
            const int q = base + s * EPI_W;
            A[s] = B[s] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (use_pre && q < P1) {
                A[s] = pk[(int64_t)q * 128 + lane];
                B[s] = pk[(int64_t)q * 128 + 64 + lane];
                const int nl = (int)min<int64_t>(128, N - (int64_t)q * 128);  // pairs in the pass
                if (nl < 128) {
                    // the last, partial pass: its missing pairs repeat the pass's
                    // first one (a candidate past N is dropped by the FP64 stage)
                    const float4 A0 = pk[(int64_t)q * 128], B0 = pk[(int64_t)q * 128 + 64];
                    if (lane >= nl) {
                        A[s].x = A0.x; A[s].z = A0.z; B[s].x = B0.x; B[s].z = B0.z;
                    }
                    if (64 + lane >= nl) {
                        A[s].y = A0.x; A[s].w = A0.z; B[s].y = B0.x; B[s].w = B0.z;
                    }
                }
            }
        }
        // slots holding passes (wave-uniform)
        const int ns = min(EPI_SLOTS, (P1 - base + EPI_W - 1) / EPI_W);
        if (first) __syncthreads();  // the constants (the loads above in flight)
        first = false;
        for (int k = 0; k < nh; ++k) {
            float4 c[6];  // hypothesis k's prefilter quads (LDS broadcasts)
#pragma unroll
            for (int j = 0; j < 6; ++j) c[j] = sC[k][j];
            const int flags = __builtin_amdgcn_readfirstlane(__float_as_int(c[0].x));
            if (!(flags & 1)) continue;
#if SFM_EPI_PROBE == 2  // timing probe (wrong counts): the loop without tests
            cntv += lane == k ? flags : 0;
            continue;
#endif
            const int64_t h = h0 + k;
            int cnt = 0;
            if (flags & 2) {
                EpiPk p;
                p.q1 = epi_f2{c[0].z, c[0].w};
                p.q0 = epi_f2{c[1].x, c[1].y};
                p.g[0] = epi_f2{c[1].z, c[1].w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    p.g[1 + 2 * j] = epi_f2{c[2 + j].x, c[2 + j].y};
                    p.g[2 + 2 * j] = epi_f2{c[2 + j].z, c[2 + j].w};
                }
                uint64_t cand[EPI_SLOTS][2], any = 0;
#pragma unroll
                for (int s = 0; s < EPI_SLOTS; ++s) {
                    cand[s][0] = cand[s][1] = 0;
                    if (s >= ns) continue;
                    bool o0, o1;
                    epi_pre_test(p, A[s], B[s], o0, o1);
                    cand[s][0] = ~__ballot(o0);
                    cand[s][1] = ~__ballot(o1);
                    any |= cand[s][0] | cand[s][1];
                }
#if SFM_EPI_PROBE == 1  // timing probe (wrong counts): the prefilter alone
                cnt += any != 0;
                any = 0;
#endif
                if (any) {  // the candidates into the workgroup's queue
                    int ubits = 0;  // bit 2 s + t: the lane's pair of slot s, half t, past a full queue
#pragma unroll
                    for (int s = 0; s < EPI_SLOTS; ++s)
#pragma unroll
                        for (int t = 0; t < 2; ++t) {
                            const uint64_t cm = cand[s][t];
                            if (!cm) continue;
                            int at = 0;
                            if (lane == 0) at = atomicAdd(&sQn, __popcll(cm));
                            at = __builtin_amdgcn_readfirstlane(at);
                            const int slot =
                                at + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(cm >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)cm, 0u));
                            const bool mine = (cm >> lane) & 1;
                            const int pi = (base + s * EPI_W - P0) * 128 + 64 * t + lane;  // the workgroup's pair
                            if (mine && slot < EPI_QCAP) sQ[slot] = ((uint32_t)k << 26) | (uint32_t)pi;
                            if (mine && slot >= EPI_QCAP) ubits |= 1 << (2 * s + t);
                        }
                    // past a full queue: the FP64 test here, one of a lane's pairs a round
                    while (__ballot(ubits != 0)) {
                        bool in = false;
                        if (ubits) {
                            const int b = __builtin_ctz(ubits);
                            ubits &= ubits - 1;
                            const int64_t i = (int64_t)(base + (b >> 1) * EPI_W) * 128 + 64 * (b & 1) + lane;
                            if (i < N) {
                                double f[9], lo, hi;
                                load_f(h, f);
                                band(lo, hi);
                                in = M::inlier_fast(f, x1[i], x2[i], thr, lo, hi);
                            }
                        }
                        cnt += __popcll(__ballot(in));
                    }
                }
            } else {  // the FP64 test on every pair of the wave's passes
                double f[9], lo, hi;
                load_f(h, f);
                band(lo, hi);
                for (int s = 0; s < ns; ++s) {
                    const int64_t i = (int64_t)(base + s * EPI_W) * 128 + lane;
                    if (i - lane + 128 <= N) {
                        cnt += epi_sets_f64(f, x1[i], x2[i], x1[i + 64], x2[i + 64], thr, lo, hi, score_split);
                    } else {
                        const bool in0 = i < N && M::inlier_fast(f, x1[i], x2[i], thr, lo, hi);
                        const bool in1 = i + 64 < N && M::inlier_fast(f, x1[i + 64], x2[i + 64], thr, lo, hi);
                        cnt += __popcll(__ballot(in0)) + __popcll(__ballot(in1));
                    }
                }
            }
            cntv += lane == k ? cnt : 0;
        }
    }
    if (first) __syncthreads();  // a wave without passes still meets the barrier
    if (lane < nh && cntv) atomicAdd(&sCnt[lane], cntv);
    __syncthreads();
    {  // the queued candidates: the FP64 test, one a lane
        double lo, hi;
        band(lo, hi);
        const int qn = min(sQn, EPI_QCAP);
        for (int e = threadIdx.x; e < qn; e += 64 * EPI_W) {
            const uint32_t v = sQ[e];
            const int k = (int)(v >> 26);
            const int64_t i = (int64_t)P0 * 128 + (v & ((1u << 26) - 1));
            if (i >= N) continue;  // a repeat in the partial pass
            const double *fk = F + 9 * (h0 + k);
            double f[9];
#pragma unroll
            for (int q = 0; q < 9; ++q) f[q] = fk[q];
            if (M::inlier_fast(f, x1[i], x2[i], thr, lo, hi)) atomicAdd(&sCnt[k], 1);
        }
    }
    __syncthreads();
    if (threadIdx.x < nh) {
        const int64_t h = h0 + threadIdx.x;
        const int c = sCnt[threadIdx.x];
        if (gridDim.y == 1)
            counts[h] = c;
        else if (c)
            atomicAdd(counts + h, c);
    }
}

// the score's wave-level outlier skip (EpiModel stage A) and its float
// prefilter; SFM_SCORE_SPLIT=0 / SFM_SCORE_PRE=0 turn them off (same-box
// A/B; the tests' check that the counts do not move)
static inline int score_split_on() {
    const char *e = std::getenv("SFM_SCORE_SPLIT");
    const char *q = std::getenv("SFM_SCORE_PRE");
    return ((e && std::atoi(e) == 0) ? 0 : SCORE_SKIP_A) | ((q && std::atoi(q) == 0) ? 0 : SCORE_PRE32);
}

template <class M>
constexpr int score_threads() {
    return 64 * (M::SPLIT ? EPI_W : SCORE_WAVES);
}
// hypotheses a fit workgroup of a fused launch takes (8 lanes each)
template <class M>
constexpr int fit_per_wg() {
    return score_threads<M>() / 8;
}
static inline int64_t env_pos(const char *name, int64_t dflt) {
    const char *e = std::getenv(name);
    const long long v = e ? std::atoll(e) : 0;
    return v > 0 ? (int64_t)v : dflt;
}
// The score grid for nh hypotheses: *gx score workgroups (hypothesis
// groups) by *gy correspondence ranges; returns the launch's argument.
//  H: one hypothesis a wave, point slices (a whole number of LDS tiles)
//     for enough workgroups to put ~4 on every CU; returns the slice.
//  F: hb hypotheses a workgroup (returned) and pass ranges of about
//     EPI_W x EPI_SLOTS passes; hb from the target workgroup count
//     (SFM_EPI_WGS, default 512: one round of two workgroups a CU; cfg2,
//     16384 / 4096 / 1024 hypotheses: 44.6 / 19.2 / 11.9 us, against 47.0 /
//     22.8 / 17.2 at 1024 workgroups and 61.2 / 25.1 / 11.8 at 384), at
//     least SFM_EPI_HB_MIN (default 4), and more ranges when the
//     hypotheses alone leave the chip short.
template <class M>
static inline int64_t score_grid(int64_t nh, int64_t N, int64_t *gx, int *gy) {
    if constexpr (M::SPLIT) {
        static const int64_t target = env_pos("SFM_EPI_WGS", 512);
        static const int64_t hb_min = std::min<int64_t>(EPI_HB_MAX, env_pos("SFM_EPI_HB_MIN", 4));
        const int64_t P = (N + 127) / 128;
        // (a workgroup's passes < 2^19: its queue entries hold pair - 128 P0 in 26 bits)
        int64_t y = std::min<int64_t>(65535, std::max(ceil_div(P, (int64_t)EPI_W * EPI_SLOTS), ceil_div(P, 1 << 19)));
        const int64_t hb = std::max(hb_min, std::min<int64_t>(EPI_HB_MAX, ceil_div(nh * y, target)));
        *gx = ceil_div(nh, hb);
        if (*gx * y < target) y = std::min<int64_t>({65535, ceil_div(P, (int64_t)EPI_W), ceil_div(target, *gx)});
        *gy = (int)y;
        return hb;
    } else {
        const int64_t wg = ceil_div(nh, (int64_t)SCORE_WAVES);
        const int64_t tiles = (N + SCORE_TILE - 1) / SCORE_TILE;
        int64_t y = std::min<int64_t>(tiles, std::max<int64_t>(1, (1024 + wg - 1) / wg));
        const int64_t per = (tiles + y - 1) / y;
        y = (tiles + per - 1) / per;
        *gx = wg;
        *gy = (int)y;
        return per * SCORE_TILE;
    }
}

// grid = 1 workgroup of 1024 threads: the winner (wg_select_best), then the
// mask with 4 correspondence pairs per thread loaded before any is tested.
template <class M>
__global__ void __launch_bounds__(1024) k_ransac_select(const double2 *__restrict__ x1,
                                                        const double2 *__restrict__ x2, int64_t N,
                                                        const double *__restrict__ F,
                                                        const int32_t *__restrict__ counts, int64_t H,
                                                        double thr, int64_t *__restrict__ best_out,
                                                        double *__restrict__ F_best,
                                                        uint8_t *__restrict__ mask) {
    constexpr int NT = 1024, MU = 4;
    __shared__ int32_t sc[NT / 64];
    __shared__ int64_t sh[NT / 64];
    const int t = threadIdx.x;
    int32_t bc;
    int64_t best;
    wg_select_best<NT>(counts, H, sc, sh, bc, best);
    if (t == 0) {
        best_out[0] = best;
        best_out[1] = bc;  // its count (the shard key's high word)
    }
    if (best < 0) return;
    double f[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = F[9 * best + k];
    if (t < 9) F_best[t] = f[t];
    if (!mask) return;  // a hypothesis shard: the mask is emitted after the combine
    // the score's fast test with its exact tail: the same decisions as M::inlier
    const double thr_lo = 2.0 * (thr >= 0 ? thr * (1.0 - 1e-4) : thr * (1.0 + 1e-4));
    const double thr_hi = 2.0 * (thr >= 0 ? thr * (1.0 + 1e-4) : thr * (1.0 - 1e-4));
    for (int64_t base = t; base < N; base += (int64_t)MU * NT) {
        double2 p[MU], q[MU];
#pragma unroll
        for (int u = 0; u < MU; ++u) {
            const int64_t i = base + (int64_t)u * NT;
            p[u] = i < N ? x1[i] : make_double2(0.0, 0.0);
            q[u] = i < N ? x2[i] : make_double2(0.0, 0.0);
        }
#pragma unroll
        for (int u = 0; u < MU; ++u) {
            const int64_t i = base + (int64_t)u * NT;
            if (i < N) mask[i] = M::inlier_fast(f, p[u], q[u], thr, thr_lo, thr_hi) ? 1 : 0;
        }
    }
}

// ------------------------------------------------------------------ host
static inline float ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}


// Correspondences from the pinned host staging buffer into device memory
// with a kernel on the compute queue (two SDMA copies plus the copy-engine
// to compute handoff cost ~24 us before the first fit; this ~3 us), one
// workgroup per score tile, which also records the tile's coordinate bounds
// for the score's float prefilter: max |x|, |y|, |u|, |v| rounded up to
// float (+inf for a non-finite coordinate).  h null: d1 / d2 already hold
// the correspondences (bounds only).
constexpr int TB_THREADS = SCORE_TILE;
__device__ __forceinline__ float abs_ru(double v) {
    const double a = fabs(v);
    return a <= 3.0e38 ? __double2float_ru(a) : __builtin_inff();  // NaN -> inf
}
static __global__ void __launch_bounds__(TB_THREADS) k_stage_tiles(const double2 *__restrict__ h, int64_t N,
                                                                   double2 *__restrict__ d1, double2 *__restrict__ d2,
                                                                   float4 *__restrict__ tmax, float4 *__restrict__ pk) {
    __shared__ float4 red[TB_THREADS / 64];
    const int64_t i = (int64_t)blockIdx.x * TB_THREADS + threadIdx.x;
    float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < N) {
        double2 p, q;
        if (h) {
            p = h[i];
            q = h[N + i];
            d1[i] = p;
            d2[i] = q;
        } else {
            p = d1[i];
            q = d2[i];
        }
        m = make_float4(abs_ru(p.x), abs_ru(p.y), abs_ru(q.x), abs_ru(q.y));
        if (pk) {  // the score's packed float copy (k_epi_score)
            const int64_t b = i >> 7;
            const int r = (int)(i & 127), l = r & 63, hh = r >> 6;
            float *A = reinterpret_cast<float *>(pk + b * 128 + l), *B = reinterpret_cast<float *>(pk + b * 128 + 64 + l);
            A[hh] = (float)p.x;
            A[2 + hh] = (float)p.y;
            B[hh] = (float)q.x;
            B[2 + hh] = (float)q.y;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        m.x = fmaxf(m.x, __shfl_xor(m.x, o));
        m.y = fmaxf(m.y, __shfl_xor(m.y, o));
        m.z = fmaxf(m.z, __shfl_xor(m.z, o));
        m.w = fmaxf(m.w, __shfl_xor(m.w, o));
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float4 r = red[0];
        for (int k = 1; k < TB_THREADS / 64; ++k)
            r = make_float4(fmaxf(r.x, red[k].x), fmaxf(r.y, red[k].y), fmaxf(r.z, red[k].z), fmaxf(r.w, red[k].w));
        tmax[blockIdx.x] = r;
    }
}
static inline int64_t n_tiles(int64_t N) { return (N + SCORE_TILE - 1) / SCORE_TILE; }
static inline size_t pk_bytes(int64_t N) { return (size_t)((N + 127) / 128) * 128 * sizeof(float4); }

// Whole RANSAC on one device: upload, fit, score, select, download.
// Timings (sfm_last_timings): upload, kernels, download, score, fit, select.
template <class M>
int ransac_run(const double *x1, const double *x2, int64_t N, const int32_t *samples, int64_t H, double thr,
               int32_t *counts_out, int64_t *best_iter, double *F_best, uint8_t *best_mask, int device) {
    SFM_CHECK_ARG(N >= M::K && H >= 0, "need N >= sample size and H >= 0");
    SFM_CHECK_ARG(x1 && x2 && best_iter && F_best && best_mask && (samples || H == 0), "null pointer");
    for (int64_t i = 0; i < H * M::K; ++i)
        SFM_CHECK_ARG(samples[i] >= 0 && samples[i] < N, "sample index out of range");
    *best_iter = -1;
    if (H == 0) return 0;
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    const size_t pb = (size_t)N * sizeof(double2);
    int rc;
    if ((rc = c->buf[0].reserve(pb)) || (rc = c->buf[1].reserve(pb)) ||
        (rc = c->buf[2].reserve((size_t)H * M::K * sizeof(int32_t))) ||
        (rc = c->buf[3].reserve((size_t)H * 9 * sizeof(double))) ||
        (rc = c->buf[4].reserve((size_t)H * sizeof(int32_t))) ||
        (rc = c->buf[5].reserve(16 * sizeof(double) + (size_t)N)) ||
        (rc = c->buf[10].reserve((size_t)n_tiles(N) * sizeof(float4))) || (rc = c->buf[9].reserve(pk_bytes(N))))
        return rc;
    double2 *d1 = c->buf[0].as<double2>(), *d2 = c->buf[1].as<double2>();
    float4 *tmax = c->buf[10].as<float4>(), *pk = c->buf[9].as<float4>();
    int32_t *ds = c->buf[2].as<int32_t>(), *dcnt = c->buf[4].as<int32_t>();
    double *dF = c->buf[3].as<double>();
    int64_t *dbest = c->buf[5].as<int64_t>();
    double *dFb = c->buf[5].as<double>() + 2;
    uint8_t *dmask = reinterpret_cast<uint8_t *>(c->buf[5].as<double>() + 16);
    hipStream_t s = c->stream;
    SFM_HIP(hipEventRecord(c->ev[0], s));
    SFM_HIP(hipMemcpyAsync(d1, x1, pb, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(d2, x2, pb, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(ds, samples, (size_t)H * M::K * sizeof(int32_t), hipMemcpyHostToDevice, s));
    if (M::SPLIT) {
        hipLaunchKernelGGL(k_stage_tiles, dim3((unsigned)n_tiles(N)), dim3(TB_THREADS), 0, s, (const double2 *)nullptr,
                           N, d1, d2, tmax, pk);
        SFM_HIP(hipGetLastError());
    }
    SFM_HIP(hipEventRecord(c->ev[1], s));
    int ny;
    int64_t gx;
    const int64_t arg = score_grid<M>(H, N, &gx, &ny);
    if ((rc = launch_fit<M>(d1, d2, ds, H, dF, ny > 1 ? dcnt : nullptr, s))) return rc;
    SFM_HIP(hipEventRecord(c->ev[2], s));
    if constexpr (M::SPLIT)
        hipLaunchKernelGGL((k_epi_score<false>), dim3((unsigned)gx, ny), dim3(score_threads<M>()), 0, s, d1, d2, N, dF,
                           H, thr, dcnt, (int)arg, FitNext{}, score_split_on(), tmax, pk);
    else
        hipLaunchKernelGGL((k_ransac_score<M, false>), dim3((unsigned)gx, ny), dim3(64 * SCORE_WAVES), 0, s, d1, d2, N,
                           dF, H, thr, dcnt, arg, FitNext{});
    SFM_HIP(hipGetLastError());
    SFM_HIP(hipEventRecord(c->ev[3], s));
    hipLaunchKernelGGL(k_ransac_select<M>, dim3(1), dim3(1024), 0, s, d1, d2, N, dF, dcnt, H, thr, dbest, dFb, dmask);
    SFM_HIP(hipGetLastError());
    SFM_HIP(hipEventRecord(c->ev[4], s));
    SFM_HIP(hipMemcpyAsync(best_iter, dbest, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    SFM_HIP(hipMemcpyAsync(F_best, dFb, 9 * sizeof(double), hipMemcpyDeviceToHost, s));
    SFM_HIP(hipMemcpyAsync(best_mask, dmask, (size_t)N, hipMemcpyDeviceToHost, s));
    if (counts_out) SFM_HIP(hipMemcpyAsync(counts_out, dcnt, (size_t)H * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    SFM_HIP(hipEventRecord(c->ev[5], s));
    SFM_HIP(hipStreamSynchronize(s));
    const double t[6] = {ev_ms(c->ev[0], c->ev[1]), ev_ms(c->ev[1], c->ev[4]), ev_ms(c->ev[4], c->ev[5]),
                         ev_ms(c->ev[2], c->ev[3]), ev_ms(c->ev[1], c->ev[2]), ev_ms(c->ev[3], c->ev[4])};
    set_timings(t, 6);
    return 0;
}

// The drop-in's whole call with the samples drawn inside it: the CPython
// random stream (MT19937 state st[625], in/out) is replayed on the host in
// chunks of RP_CHUNK hypotheses into pinned memory, and each chunk's fit
// (reading the rows in place, zero-copy) and score are enqueued as soon as
// it is drawn, so the GPU works on
// chunk c while the host draws chunk c + 1 (the draw is sequential by
// construction: every hypothesis consumes a data-dependent number of MT
// outputs).  samples_out (nullable) receives the table.  Timings as
// ransac_run, plus [6] = host sampling ms.
constexpr int64_t RP_CHUNK = 4096;
static inline size_t xoff_of(int64_t N) { return ((size_t)16 * sizeof(double) + (size_t)N + 255) & ~(size_t)255; }
static inline int64_t rp_chunk() {
    static const int64_t c = [] {
        const char *e = std::getenv("SFM_RP_CHUNK");
        const long v = e ? std::atol(e) : 0;
        return v > 0 ? (int64_t)v : RP_CHUNK;
    }();
    return c;
}
// chunk sizes ramp up from RP_FIRST (doubling to rp_chunk()): the device
// waits for the first draw (the pipeline fill), and every later draw has to
// finish within the previous chunk's kernels
constexpr int64_t RP_FIRST = 1024;
static inline int64_t rp_next(int64_t h0, int64_t H) {
    static const int64_t first = [] {
        const char *e = std::getenv("SFM_RP_FIRST");
        const long v = e ? std::atol(e) : 0;
        return v > 0 ? (int64_t)v : RP_FIRST;
    }();
    static const bool ramp = std::getenv("SFM_RP_RAMP") && std::atoi(std::getenv("SFM_RP_RAMP"));
    // SFM_RP_SCHEDULE="a,b,c": explicit chunk sizes, the last one repeated
    static const std::vector<int64_t> sched = [] {
        std::vector<int64_t> v;
        if (const char *e = std::getenv("SFM_RP_SCHEDULE"))
            for (const char *q = e; *q;) {
                char *nx;
                const long x = std::strtol(q, &nx, 10);
                if (nx == q) break;
                if (x > 0) v.push_back(x);
                q = *nx ? nx + 1 : nx;
            }
        return v;
    }();
    if (!sched.empty()) {
        int64_t pos = 0;
        for (size_t k = 0;; ++k) {
            const int64_t sz = sched[std::min(k, sched.size() - 1)];
            if (pos + sz > h0) return std::min(H, pos + sz);
            pos += sz;
        }
    }
    const int64_t chunk = rp_chunk();
    if (!ramp) return std::min(H, h0 + (h0 == 0 ? std::min(first, chunk) : chunk));
    int64_t size = std::min(first, chunk), pos = 0;
    while (size < chunk && pos + size <= h0) {
        pos += size;
        size = std::min(chunk, 2 * size);
    }
    return std::min(H, h0 + size);
}

// Fit + score of the drawn chunks.  With a group fit (EpiModel) a chunk's
// score is enqueued only once the next chunk is drawn, and that launch fits
// the next chunk in extra workgroups (FitNext): only the first chunk's fit
// runs on its own.  SFM_RANSAC_FUSED=0 restores fit-then-score per chunk.
static inline bool ransac_fused() {
    static const bool on = [] {
        const char *e = std::getenv("SFM_RANSAC_FUSED");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}

template <class M>
struct ScorePipe {
    const double2 *d1, *d2;
    int64_t N;
    double thr;
    hipStream_t s;
    double *dF;      // models of hypotheses off..: dF + 9 (h - off)
    int32_t *dcnt;   // counts likewise
    int64_t off;
    const float4 *tmax, *pk;  // per-tile coordinate bounds and the packed float copy (k_stage_tiles)
    int64_t pa = 0, pb = 0;  // the fitted, not yet scored piece
    bool fused = M::GROUP_FIT && ransac_fused();
    int split = score_split_on();  // read once, on the caller's thread (the launcher thread reads no environment)

    int score(int64_t a, int64_t b, const FitNext *fn) {
        int ny;
        int64_t gx;
        const int64_t n = b - a, arg = score_grid<M>(n, N, &gx, &ny);
        const dim3 grid((unsigned)(gx + (fn ? fn->nfb : 0)), ny);
        if constexpr (M::SPLIT) {
            if (fn)
                hipLaunchKernelGGL((k_epi_score<true>), grid, dim3(score_threads<M>()), 0, s, d1, d2, N,
                                   dF + (a - off) * 9, n, thr, dcnt + (a - off), (int)arg, *fn, split, tmax, pk);
            else
                hipLaunchKernelGGL((k_epi_score<false>), grid, dim3(score_threads<M>()), 0, s, d1, d2, N,
                                   dF + (a - off) * 9, n, thr, dcnt + (a - off), (int)arg, FitNext{}, split, tmax,
                                   pk);
        } else {  // the H model (no group fit: its fits run on their own)
            hipLaunchKernelGGL((k_ransac_score<M, false>), grid, dim3(64 * SCORE_WAVES), 0, s, d1, d2, N,
                               dF + (a - off) * 9, n, thr, dcnt + (a - off), arg, FitNext{});
        }
        SFM_HIP(hipGetLastError());
        return 0;
    }
    // hypotheses [a, b), sample rows at rows (device-readable)
    int add(int64_t a, int64_t b, const int32_t *rows) {
        if (b <= a) return 0;
        int ny, rc;
        int64_t gx;
        (void)score_grid<M>(b - a, N, &gx, &ny);  // as score() will cut it
        int32_t *cz = ny > 1 ? dcnt + (a - off) : nullptr;
        if (!fused) {
            if ((rc = launch_fit<M>(d1, d2, rows, b - a, dF + (a - off) * 9, cz, s))) return rc;
            return score(a, b, nullptr);
        }
        if (pb > pa) {
            const FitNext fn{rows, b - a, dF + (a - off) * 9, cz, (int)ceil_div(b - a, fit_per_wg<M>())};
            if ((rc = score(pa, pb, &fn))) return rc;
        } else if ((rc = launch_fit<M>(d1, d2, rows, b - a, dF + (a - off) * 9, cz, s))) {
            return rc;
        }
        pa = a;
        pb = b;
        return 0;
    }
    int flush() {
        int rc = 0;
        if (pb > pa) rc = score(pa, pb, nullptr);
        pa = pb = 0;
        return rc;
    }
};

template <class M>
int ransac_run_pysample(const double *x1, const double *x2, int64_t N, uint32_t *st, int64_t H, double thr,
                        int32_t *counts_out, int64_t *best_iter, double *F_best, uint8_t *best_mask,
                        int32_t *samples_out, int device, int64_t *split = nullptr, int64_t *n_inliers = nullptr) {
    SFM_CHECK_ARG(N >= M::K && H >= 0, "need N >= sample size and H >= 0");
    SFM_CHECK_ARG(x1 && x2 && st && best_iter && F_best && (best_mask || (split && n_inliers)), "null pointer");
    if (n_inliers) *n_inliers = 0;
    SFM_CHECK_ARG(N < ((int64_t)1 << 31) && st[624] <= 624, "bad sizes / MT19937 position");
    *best_iter = -1;
    if (H == 0) return 0;
    const auto t_entry = std::chrono::steady_clock::now();
    auto since = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_entry).count(); };
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    const size_t pb = (size_t)N * sizeof(double2);
    const size_t sb = (size_t)H * M::K * sizeof(int32_t);
    const size_t sbp = (sb + 255) & ~(size_t)255;
    int rc;
    if ((rc = c->buf[0].reserve(pb)) || (rc = c->buf[1].reserve(pb)) ||
        (rc = c->buf[3].reserve((size_t)H * 9 * sizeof(double))) ||
        (rc = c->buf[4].reserve((size_t)H * sizeof(int32_t))) ||
        (rc = c->buf[10].reserve((size_t)n_tiles(N) * sizeof(float4))) || (rc = c->buf[9].reserve(pk_bytes(N))) ||
        (rc = c->pinned.reserve(sbp + xoff_of(N) + 2 * pb)))
        return rc;
    double2 *d1 = c->buf[0].as<double2>(), *d2 = c->buf[1].as<double2>();
    int32_t *dcnt = c->buf[4].as<int32_t>();
    double *dF = c->buf[3].as<double>();
    float4 *tmax = c->buf[10].as<float4>(), *pk = c->buf[9].as<float4>();
    // Zero-copy through pinned host memory: the fit kernels read each chunk's
    // sample rows straight from where the host replay wrote them, and the
    // select kernel writes (best, F, mask) back the same way, so no SDMA copy
    // (and no copy-engine/compute-queue handoff) sits between host and kernels.
    int32_t *hs = c->pinned.as<int32_t>();
    char *hout = c->pinned.as<char>() + sbp;
    // the correspondences are staged through pinned memory as well, so their
    // upload is a true async copy that overlaps the first chunk's draw (from
    // pageable memory the copy would hold the host until it lands)
    char *hx = hout + xoff_of(N);
    PySampler ps(st, N, M::K);
    double t_draw = 0, h_pre = 0;
    const int64_t hfirst = rp_next(0, H);
    int64_t *dbest = reinterpret_cast<int64_t *>(hout);
    double *dFb = reinterpret_cast<double *>(hout) + 2;
    uint8_t *dmask = reinterpret_cast<uint8_t *>(hout) + 16 * sizeof(double);
    hipStream_t s = c->stream;
    const bool tm = call_timing();
    ScorePipe<M> pipe{d1, d2, N, thr, s, dF, dcnt, 0, tmax, pk};
    // the correspondences into pinned memory and the staging kernel
    auto stage = [&]() -> int {
        std::memcpy(hx, x1, pb);
        std::memcpy(hx + pb, x2, pb);
        if (tm) SFM_HIP(hipEventRecord(c->ev[0], s));
        hipLaunchKernelGGL(k_stage_tiles, dim3((unsigned)n_tiles(N)), dim3(TB_THREADS), 0, s,
                           reinterpret_cast<const double2 *>(hx), N, d1, d2, tmax, pk);
        SFM_HIP(hipGetLastError());
        if (tm) SFM_HIP(hipEventRecord(c->ev[1], s));
        return 0;
    };
    auto draw = [&](int64_t h0, int64_t h1) {
        const auto ta = std::chrono::steady_clock::now();
        ps.draw(h0, h1, hs);
        t_draw += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count();
        if (h0 == 0) h_pre = since();
    };
    // Two host threads (round 5): the caller draws every chunk, a pool
    // worker copies the points, launches the staging kernel and enqueues
    // each chunk's fit / score as soon as its rows are drawn, so the ~4-us
    // launch calls leave the sequential draw's path (one thread had
    // interleaved them: the last launch at ~129 us after ~101 us of draws).
    // SFM_RANSAC_LAUNCHER=0, or a busy pool, keeps the one-thread order.
    // the CPUs this process may run on (taskset / cpuset), not the machine's:
    // on one CPU the launcher would only compete with the drawer
    static const bool multi_core = [] {
        cpu_set_t cs;
        CPU_ZERO(&cs);
        return sched_getaffinity(0, sizeof cs, &cs) == 0 ? CPU_COUNT(&cs) > 1 : std::thread::hardware_concurrency() > 1;
    }();
    const char *le = std::getenv("SFM_RANSAC_LAUNCHER");  // read per call (the tests flip it)
    const bool two = multi_core && !(le && std::atoi(le) == 0);
    std::atomic<int64_t> drawn{0};
    int lrc = 0;
    const bool ran = two && HostPool::get().try_run(2, [&](int t) {
        if (t == 0) {  // the launcher (a pool worker)
            if (hipSetDevice(c->device) != hipSuccess) {
                lrc = SFM_ERR_HIP;
                return;
            }
            if ((lrc = stage())) return;
            for (int64_t h0 = 0, h1; h0 < H; h0 = h1) {
                h1 = rp_next(h0, H);
                // a bounded spin, then yield (an oversubscribed host must not starve the drawer)
                for (int spin = 0; drawn.load(std::memory_order_acquire) < h1; ++spin)
                    if (spin < 20000) _mm_pause();
                    else std::this_thread::yield();
                if ((lrc = pipe.add(h0, h1, hs + h0 * M::K))) return;
            }
        } else {  // the drawer (the caller): every chunk, in the reference's order
            for (int64_t h0 = 0, h1; h0 < H; h0 = h1) {
                h1 = rp_next(h0, H);
                draw(h0, h1);
                drawn.store(h1, std::memory_order_release);
            }
        }
    });
    if (ran) {
        if (lrc) {
            set_error("RANSAC launcher thread: HIP error %d", lrc);
            return lrc;
        }
    } else {  // one thread: the first chunk's draw, then each launch after its draw
        draw(0, hfirst);
        if ((rc = stage())) return rc;
        if ((rc = pipe.add(0, hfirst, hs))) return rc;
        for (int64_t h0 = hfirst, h1; h0 < H; h0 = h1) {
            h1 = rp_next(h0, H);
            draw(h0, h1);
            if ((rc = pipe.add(h0, h1, hs + h0 * M::K))) return rc;
        }
    }
    if ((rc = pipe.flush())) return rc;
    ps.save(st);
    if (tm) SFM_HIP(hipEventRecord(c->ev[3], s));
    hipLaunchKernelGGL(k_ransac_select<M>, dim3(1), dim3(1024), 0, s, d1, d2, N, dF, dcnt, H, thr, dbest, dFb, dmask);
    SFM_HIP(hipGetLastError());
    if (tm) SFM_HIP(hipEventRecord(c->ev[4], s));
    if (counts_out) SFM_HIP(hipMemcpyAsync(counts_out, dcnt, (size_t)H * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (tm) SFM_HIP(hipEventRecord(c->ev[5], s));
    const double h_enq = since();
    SFM_HIP(hipStreamSynchronize(s));
    const double h_sync = since();
    *best_iter = *dbest;
    if (*best_iter >= 0) {
        std::memcpy(F_best, dFb, 9 * sizeof(double));
        if (best_mask) std::memcpy(best_mask, dmask, (size_t)N);
        if (split) {  // inlier positions ascending, then the outliers' (branch-free)
            int64_t ni = 0;
            for (int64_t i = 0; i < N; ++i) ni += dmask[i] != 0;
            int64_t a = 0, b = ni;
            for (int64_t i = 0; i < N; ++i) {
                const bool in = dmask[i] != 0;
                split[in ? a : b] = i;
                a += in;
                b += !in;
            }
            *n_inliers = ni;
        }
    } else if (best_mask) {
        std::memset(best_mask, 0, (size_t)N);
    }
    if (samples_out) std::memcpy(samples_out, hs, sb);
    // [7..10]: host ms from entry to the first chunk drawn, the last launch
    // enqueued, the stream drained and the return
    double t[11] = {0, 0, 0, 0, 0, 0, t_draw, h_pre, h_enq, h_sync, since()};
    if (tm) {
        t[0] = ev_ms(c->ev[0], c->ev[1]); t[1] = ev_ms(c->ev[1], c->ev[4]); t[2] = ev_ms(c->ev[4], c->ev[5]);
        t[3] = ev_ms(c->ev[1], c->ev[3]); t[5] = ev_ms(c->ev[3], c->ev[4]);
    }
    set_timings(t, 11);
    return 0;
}

// The inlier mask of one model (the winner's emit after a sharded combine).
template <class M>
__global__ void __launch_bounds__(256) k_ransac_mask(const double2 *__restrict__ x1, const double2 *__restrict__ x2,
                                                     int64_t N, const double *__restrict__ F, double thr,
                                                     uint8_t *__restrict__ mask) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    double f[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = F[k];
    mask[i] = M::inlier(f, x1[i], x2[i], thr) ? 1 : 0;
}

// Shard key of a (count, iteration) winner: the reference's strict '>'
// update keeps the max count and, among equal counts, the earliest
// iteration, which is the max of (count << 32) | (0xFFFFFFFF - iteration);
// key 0 = no hypothesis with an inlier.  Ranks combine keys with max.
static inline uint64_t shard_key(int64_t count, int64_t iter) {
    return count > 0 ? ((uint64_t)count << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)iter) : 0;
}

// One hypothesis shard [r0, r1) of an H-hypothesis RANSAC
// (GetInliersRANSAC.py:53-92 split over ranks).  The sample
// table is either given (samples: the whole H x K table) or drawn in the
// call from the CPython MT19937 state st (all H rows are drawn, in the
// reference's order, so st advances exactly as the unsharded call; only the
// shard's rows are fitted and scored).  Out: counts of the shard (nullable),
// the shard key and the shard winner's model (untouched when key = 0).
template <class M>
int ransac_run_range(const double *x1, const double *x2, int64_t N, const int32_t *samples, uint32_t *st, int64_t H,
                     int64_t r0, int64_t r1, double thr, int32_t *counts_out, uint64_t *key_out, double *F_best,
                     int device) {
    SFM_CHECK_ARG(N >= M::K && H >= 0 && H < ((int64_t)1 << 32), "need N >= sample size and 0 <= H < 2^32");
    SFM_CHECK_ARG(0 <= r0 && r0 <= r1 && r1 <= H, "need 0 <= h0 <= h1 <= H");
    SFM_CHECK_ARG(x1 && x2 && key_out && F_best && (samples || st || H == 0), "null pointer");
    SFM_CHECK_ARG(!st || (N < ((int64_t)1 << 31) && st[624] <= 624), "bad sizes / MT19937 position");
    if (samples)
        for (int64_t i = r0 * M::K; i < r1 * M::K; ++i)
            SFM_CHECK_ARG(samples[i] >= 0 && samples[i] < N, "sample index out of range");
    *key_out = 0;
    const int64_t nh = r1 - r0;
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    const size_t pb = (size_t)N * sizeof(double2);
    const size_t sb = (size_t)(st ? H : nh) * M::K * sizeof(int32_t);
    const size_t sbp = (sb + 255) & ~(size_t)255;
    int rc;
    if ((rc = c->buf[0].reserve(pb)) || (rc = c->buf[1].reserve(pb)) ||
        (rc = c->buf[3].reserve((size_t)std::max<int64_t>(nh, 1) * 9 * sizeof(double))) ||
        (rc = c->buf[4].reserve((size_t)std::max<int64_t>(nh, 1) * sizeof(int32_t))) ||
        (rc = c->buf[10].reserve((size_t)n_tiles(N) * sizeof(float4))) || (rc = c->buf[9].reserve(pk_bytes(N))) ||
        (rc = c->pinned.reserve(sbp + xoff_of(N) + 2 * pb)))
        return rc;
    double2 *d1 = c->buf[0].as<double2>(), *d2 = c->buf[1].as<double2>();
    int32_t *dcnt = c->buf[4].as<int32_t>();
    double *dF = c->buf[3].as<double>();
    float4 *tmax = c->buf[10].as<float4>(), *pk = c->buf[9].as<float4>();
    int32_t *hs = c->pinned.as<int32_t>();
    char *hout = c->pinned.as<char>() + sbp;
    char *hx = hout + xoff_of(N);
    std::memcpy(hx, x1, pb);
    std::memcpy(hx + pb, x2, pb);
    int64_t *dbest = reinterpret_cast<int64_t *>(hout);
    double *dFb = reinterpret_cast<double *>(hout) + 2;
    hipStream_t s = c->stream;
    const bool tm = call_timing();
    if (tm) SFM_HIP(hipEventRecord(c->ev[0], s));
    hipLaunchKernelGGL(k_stage_tiles, dim3((unsigned)n_tiles(N)), dim3(TB_THREADS), 0, s,
                       reinterpret_cast<const double2 *>(hx), N, d1, d2, tmax, pk);
    SFM_HIP(hipGetLastError());
    if (tm) SFM_HIP(hipEventRecord(c->ev[1], s));
    double t_draw = 0;
    // fit + score the hypotheses of the shard, hypothesis h at dF + 9 (h - r0)
    ScorePipe<M> pipe{d1, d2, N, thr, s, dF, dcnt, r0, tmax, pk};
    if (st) {
        PySampler ps(st, N, M::K);
        for (int64_t h0 = 0, h1; h0 < H; h0 = h1) {
            h1 = rp_next(h0, H);
            const auto ta = std::chrono::steady_clock::now();
            ps.draw(h0, h1, hs);
            t_draw += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count();
            const int64_t a = std::max(h0, r0), b = std::min(h1, r1);
            if ((rc = pipe.add(a, b, hs + a * M::K))) return rc;
        }
        ps.save(st);
    } else {
        std::memcpy(hs, samples + r0 * M::K, sb);
        if ((rc = pipe.add(r0, r1, hs))) return rc;
    }
    if ((rc = pipe.flush())) return rc;
    if (tm) SFM_HIP(hipEventRecord(c->ev[3], s));
    if (nh > 0) {
        hipLaunchKernelGGL(k_ransac_select<M>, dim3(1), dim3(1024), 0, s, d1, d2, N, dF, dcnt, nh, thr, dbest, dFb,
                           (uint8_t *)nullptr);
        SFM_HIP(hipGetLastError());
    }
    if (tm) SFM_HIP(hipEventRecord(c->ev[4], s));
    if (counts_out && nh)
        SFM_HIP(hipMemcpyAsync(counts_out, dcnt, (size_t)nh * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (tm) SFM_HIP(hipEventRecord(c->ev[5], s));
    SFM_HIP(hipStreamSynchronize(s));
    if (nh > 0 && dbest[0] >= 0) {
        *key_out = shard_key(dbest[1], r0 + dbest[0]);
        std::memcpy(F_best, dFb, 9 * sizeof(double));
    }
    double t[7] = {0, 0, 0, 0, 0, 0, t_draw};
    if (tm) {
        t[0] = ev_ms(c->ev[0], c->ev[1]); t[1] = ev_ms(c->ev[1], c->ev[4]); t[2] = ev_ms(c->ev[4], c->ev[5]);
        t[3] = ev_ms(c->ev[1], c->ev[3]); t[5] = ev_ms(c->ev[3], c->ev[4]);
    }
    set_timings(t, 7);
    return 0;
}

template <class M>
int ransac_mask_run(const double *x1, const double *x2, int64_t N, const double *F, double thr, uint8_t *mask,
                    int device) {
    SFM_CHECK_ARG(x1 && x2 && F && (mask || N == 0) && N >= 0, "null pointer");
    if (N == 0) return 0;
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    const size_t pb = (size_t)N * sizeof(double2);
    int rc;
    if ((rc = c->buf[0].reserve(pb)) || (rc = c->buf[1].reserve(pb)) ||
        (rc = c->buf[5].reserve(16 * sizeof(double) + (size_t)N)))
        return rc;
    double2 *d1 = c->buf[0].as<double2>(), *d2 = c->buf[1].as<double2>();
    double *dF = c->buf[5].as<double>();
    uint8_t *dm = reinterpret_cast<uint8_t *>(dF + 16);
    hipStream_t s = c->stream;
    SFM_HIP(hipMemcpyAsync(d1, x1, pb, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(d2, x2, pb, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(dF, F, 9 * sizeof(double), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_ransac_mask<M>, dim3(ceil_div(N, 256)), dim3(256), 0, s, d1, d2, N, dF, thr, dm);
    SFM_HIP(hipGetLastError());
    SFM_HIP(hipMemcpyAsync(mask, dm, (size_t)N, hipMemcpyDeviceToHost, s));
    SFM_HIP(hipStreamSynchronize(s));
    return 0;
}

}  // namespace sfm
