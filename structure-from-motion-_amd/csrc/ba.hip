// Sparse Schur-complement Levenberg-Marquardt bundle adjustment for gfx950.
//
// Replaces perform_bundle_adjustment's scipy least_squares(method='lm')
// (BundleAdjustment.py:113-242) on the reference residual
// (BundleAdjustment.py:43-110): r = obs - proj, proj = K(RX+t)[:2]/(K(RX+t)[2]+1e-8).
//
// One LM iteration = one damped solve + one trial evaluation:
//   k_linearize      (after an accepted step) thread per point: residual,
//                    analytic 2x6 / 2x3 Jacobians per observation -> J cache;
//                    point block V = sum Jp^T Jp, g_p = sum Jp^T r.
//   k_point_prep     thread per point: Vd = V + lambda*clamp(diag V) = C C^T,
//                    L = C^-T (so Vd^-1 = L L^T), q = L^T g_p,
//                    Z_o = (Jc^T Jp)_o L per observation.
//   k_camera_lin     (after linearize) workgroup per camera: U_c, g_c.
//   k_schur_sweep    S_ij = U_i [i==j] - sum_p Z_pi Z_pj^T: workgroups own
//                    camera-block rows and sweep XCD-local point ranges
//                    (a records staged in LDS, b records from L2);
//   k_schur_finish   fixed-order sum of the ranges of each camera block ->
//                    deterministic, no atomics.
//   [RCCL all-reduce of the packed partial system across ranks]
//   (assembly of S + lambda*clamp(diag U), b = -g_c + sum Z q folded into the
//    first Cholesky launch)
//   k_chol_col       one launch per 16-wide tile column: trailing update
//                    by the previous column + factor/TRSM of this one
//                    (+ folded forward solve); k_chol_backsolve.
//   (backsolve epilogue) R' = exp([dtheta]x) R, t' = t + dt; camera part of the
//                    model decrease.
//   k_backsub_trial  thread per point: dp = L L^T(-g_p - sum W^T dc),
//                    X' = X + dp, trial cost of its observations.
//   k_lm_step        the accept/reject decision and Nielsen's damping update
//                    on the device (state double-buffered by iteration
//                    parity), the accepted step's copy trial -> current.
// Per-point partial sums are finished by the last block of their kernel
// (grid_sum_last), so an iteration is linearize / camera_lin (accepted
// steps only), point_prep, schur_sweep, schur_finish, the Cholesky launches,
// backsub_trial and lm_step; the host polls the device state once per batch
// of iterations.  On a rejected step only k_point_prep onwards is repeated.
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <utility>
#include <numeric>
#include <vector>

#include "sfm_common.hpp"
#include "sfm_geom.hpp"
#include "host_pool.hpp"

// In-process rank group (N host threads, one per rank): the all-reduce is
// staged through host memory and summed in rank order (deterministic).
struct LocalGroup {
    int nranks = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    long generation = 0;
    std::vector<std::vector<double>> bufs;
    std::vector<double> result;
    int refs = 0;
    bool aborted = false;  // a rank failed: the others stop waiting and return SFM_ERR_COMM
    // In-process ranks share one GPU: their persistent solves (gj_solve.hpp)
    // run one after another (each launch waits for the previous rank's), so
    // two spinning grids never compete for the CUs.
    std::mutex solve_mu;
    hipEvent_t last_solve = nullptr;  // an event of the rank that launched last (not owned)
};

struct sfm_comm {
    ncclComm_t comm = nullptr;   // RCCL (one process per GPU)
    LocalGroup *local = nullptr; // or an in-process group
    int nranks = 1, rank = 0, device = 0;
    void *scratch = nullptr;     // sfm_ransac_combine's device words (RCCL)
    hipStream_t stream = nullptr;
};

namespace sfm {

constexpr int PT_THREADS = 128;   // per-point kernels
constexpr int PT_GROUP = 8;       // max lanes per point in k_linearize / k_backsub_trial

// sum over an aligned group of G lanes (fixed butterfly order; every lane of
// the group ends with the same total)
template <int G>
__device__ __forceinline__ double group_sum(double v) {
#pragma unroll
    for (int off = G / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__device__ __forceinline__ double clampd(double x) { return fmin(fmax(x, 1e-6), 1e32); }

// ----------------------------------------------------------- reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// block of PT_THREADS threads: reduce NV values, thread 0 writes out[0..NV)
template <int NV>
__device__ __forceinline__ void block_sum_store(double (&v)[NV], double *out) {
    __shared__ double red[PT_THREADS / 64][NV];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const double s = wave_sum(v[k]);
        if (lane == 0) red[w][k] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            double s = 0;
            for (int i = 0; i < PT_THREADS / 64; ++i) s += red[i][k];
            out[k] = s;
        }
    }
}

// Grid-wide fixed-order sum without a second launch.  Every block of
// PT_THREADS threads reduces its NV values, thread 0 stores them write-through
// (agent-scope relaxed stores = sc1) to partial[block][NV], waits for the
// stores and counts itself in with an agent-scope atomic; the block whose add
// returns nblk - 1 sums all partials in block order (sc1 loads) into
// out[0..NV) and re-arms the counter.  The same summation order as a separate
// k_finalize launch, so the result is deterministic.
// counter block of grid_sum_last: [0] top, [1 + g] blocks with blockIdx % 8 == g,
// one 128-B line each (arrivals on ONE word serialise at ~11-13 ns each:
// 1024 blocks cost ~12 us; eight group words take them in parallel)
constexpr int GS_STRIDE = 32;
constexpr int GS_WORDS = 9 * GS_STRIDE;

template <int NV, int NT = PT_THREADS>
__device__ __forceinline__ void grid_sum_last(double (&v)[NV], double *partial, unsigned *counter, double *out) {
    __shared__ double red[NT / 64][NV];
    __shared__ int last;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned nblk = gridDim.x;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const double s = wave_sum(v[k]);
        if (lane == 0) red[w][k] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            double s = 0;
            for (int i = 0; i < NT / 64; ++i) s += red[i][k];
            __hip_atomic_store(partial + (int64_t)NV * blockIdx.x + k, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // Release side.  The partials are agent-scope atomic stores (sc1,
        // written through to the coherence point), and the wait below holds
        // the arrival until they have completed; the asm's memory clobber
        // keeps the compiler from moving them past it.  A formal agent-scope
        // release (an acq_rel add or a release fence) would add buffer_wbl2,
        // a write-back of the whole XCD L2, to every block's arrival:
        // measured at cfg4, k_backsub_trial 0.042 -> 0.074 ms and
        // k_camera_lin +8 us per iteration, so it is not used.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // two-level arrival: the block counts in at its group's word; the
        // group's last arriver counts the group in at the top word
        const unsigned g = blockIdx.x % 8, ng = (nblk - g + 7) / 8, ngroups = nblk < 8 ? nblk : 8;
        int l = 0;
        if (__hip_atomic_fetch_add(counter + GS_STRIDE * (1 + g), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            ng - 1)
            l = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1;
        last = l;
    }
    __syncthreads();
    if (!last) return;
    // Acquire side: every load of the partials below is an agent-scope
    // atomic load (global_load sc1, L1 bypassed), which MI355X_MICROARCH.md
    // ("Valid forms", table row 1: one lane per storing workgroup, sc1
    // stores drained by vmcnt(0), an agent-scope add, the last adder loading
    // sc1) lists in place of an acquire fence; the fence (buffer_inv sc1)
    // would add ~1.7 us to the tail of every launch.
    // all NV sums at once: NV x GS_BATCH independent sc1 loads in flight
    // per thread, one tree -- per value the same order as summing them one by one
    __shared__ double tot[NV][NT];
    double s[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) s[k] = 0;
    constexpr int GS_BATCH = NV > 1 ? 8 : 16;  // bounded so the tail does not set the kernel's VGPR count
    for (unsigned b0 = threadIdx.x; b0 < nblk; b0 += GS_BATCH * NT) {
        double v16[NV][GS_BATCH];
#pragma unroll
        for (int u = 0; u < GS_BATCH; ++u) {
            const unsigned b = b0 + u * NT;
#pragma unroll
            for (int k = 0; k < NV; ++k)
                v16[k][u] = b < nblk ? __hip_atomic_load(partial + (int64_t)NV * b + k, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT)
                                     : 0.0;
        }
#pragma unroll
        for (int k = 0; k < NV; ++k)
#pragma unroll
            for (int u = 0; u < GS_BATCH; ++u) s[k] += v16[k][u];
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) tot[k][threadIdx.x] = s[k];
    __syncthreads();
    for (int st = NT / 2; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st)
#pragma unroll
            for (int k = 0; k < NV; ++k) tot[k][threadIdx.x] += tot[k][threadIdx.x + st];
        __syncthreads();
    }
    if (threadIdx.x < NV) out[threadIdx.x] = tot[threadIdx.x][0];
    if (threadIdx.x < 9) __hip_atomic_store(counter + GS_STRIDE * threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------ observation model
// Every Jacobian block of an observation follows from A = dr/dx_cam (2x3),
// p = R X (the rotated point) and the camera's R:
//   Jc = [A (-[p]x) | A]  (2x6, rotation perturbed on the left: R <- exp([d]x) R)
//   Jp = A R              (2x3)
//   W  = Jc^T Jp = E (A^T A R),  E = [[p]x ; I]  (6x3)
// so (r, A, p) is all an observation needs, and it is recomputed from X and
// the camera wherever it is used (no stored Jacobians).

__device__ __forceinline__ void obs_model(const double *__restrict__ Rt, const double *X, const double (&K)[9],
                                          double2 ob, double (&r)[2], double (&A)[2][3], double (&p)[3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) p[i] = Rt[3 * i] * X[0] + Rt[3 * i + 1] * X[1] + Rt[3 * i + 2] * X[2];
    const double xc0 = p[0] + Rt[9], xc1 = p[1] + Rt[10], xc2 = p[2] + Rt[11];
    double u[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) u[i] = K[3 * i] * xc0 + K[3 * i + 1] * xc1 + K[3 * i + 2] * xc2;
    const double iw = 1.0 / (u[2] + 1e-8);
    const double pu = u[0] * iw, pv = u[1] * iw;
    r[0] = ob.x - pu;
    r[1] = ob.y - pv;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        A[0][c] = -(iw * K[c] - pu * iw * K[6 + c]);
        A[1][c] = -(iw * K[3 + c] - pv * iw * K[6 + c]);
    }
}

// (A, p) of obs_model without the residual: the same expression trees, so
// the same values bit for bit (no J cache: every consumer recomputes them
// from X and the camera instead of re-reading 96 B per observation)
__device__ __forceinline__ void obs_Ap(const double *__restrict__ Rt, const double *X, const double (&K)[9],
                                       double (&A)[2][3], double (&p)[3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) p[i] = Rt[3 * i] * X[0] + Rt[3 * i + 1] * X[1] + Rt[3 * i + 2] * X[2];
    const double xc0 = p[0] + Rt[9], xc1 = p[1] + Rt[10], xc2 = p[2] + Rt[11];
    double u[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) u[i] = K[3 * i] * xc0 + K[3 * i + 1] * xc1 + K[3 * i + 2] * xc2;
    const double iw = 1.0 / (u[2] + 1e-8);
    const double pu = u[0] * iw, pv = u[1] * iw;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        A[0][c] = -(iw * K[c] - pu * iw * K[6 + c]);
        A[1][c] = -(iw * K[3 + c] - pv * iw * K[6 + c]);
    }
}

__device__ __forceinline__ void jc_of(const double (&A)[2][3], const double (&p)[3], double (&Jc)[2][6]) {
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        Jc[a][0] = A[a][1] * (-p[2]) + A[a][2] * p[1];
        Jc[a][1] = A[a][0] * p[2] + A[a][2] * (-p[0]);
        Jc[a][2] = A[a][0] * (-p[1]) + A[a][1] * p[0];
        Jc[a][3] = A[a][0];
        Jc[a][4] = A[a][1];
        Jc[a][5] = A[a][2];
    }
}

__device__ __forceinline__ double obs_cost(const double *__restrict__ Rt, const double *X, const double (&K)[9],
                                           double2 ob) {
    double xc[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) xc[i] = Rt[3 * i] * X[0] + Rt[3 * i + 1] * X[1] + Rt[3 * i + 2] * X[2] + Rt[9 + i];
    double u[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) u[i] = K[3 * i] * xc[0] + K[3 * i + 1] * xc[1] + K[3 * i + 2] * xc[2];
    const double iw = 1.0 / (u[2] + 1e-8);
    const double r0 = ob.x - u[0] * iw, r1 = ob.y - u[1] * iw;
    return 0.5 * (r0 * r0 + r1 * r1);
}

struct Kmat {
    double k[9];
};

template <int G>
__global__ void __launch_bounds__(PT_THREADS) k_linearize(int64_t np_, const int32_t *__restrict__ pstart,
                                                          const int32_t *__restrict__ cam,
                                                          const double2 *__restrict__ obs, Kmat Km,
                                                          const double *__restrict__ Rt,
                                                          const double *__restrict__ X,
                                                          double *__restrict__ Vg, double *__restrict__ partial,
                                                          unsigned *__restrict__ counter, double *__restrict__ cost_out,
                                                          int want_cost, const int *__restrict__ gate, double gtol,
                                                          unsigned *__restrict__ nbig) {
    if (gate && !*gate) return;  // device-side LM control: iteration gated off
    const int64_t gt = (int64_t)blockIdx.x * PT_THREADS + threadIdx.x;
    const int64_t p = gt / G;  // G lanes per point, striding over its observations
    const int sub = (int)(gt % G);
    double K[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) K[i] = Km.k[i];
    double acc[1] = {0.0};
    double V[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
    if (p < np_) {
        double x[3] = {X[3 * p], X[3 * p + 1], X[3 * p + 2]};
        for (int32_t o = pstart[p] + sub; o < pstart[p + 1]; o += G) {
            const double *Rt_c = Rt + 12 * cam[o];
            double r[2], A[2][3], q[3];
            obs_model(Rt_c, x, K, obs[o], r, A, q);
            double Jp[2][3];
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int c = 0; c < 3; ++c) Jp[a][c] = A[a][0] * Rt_c[c] + A[a][1] * Rt_c[3 + c] + A[a][2] * Rt_c[6 + c];
            acc[0] += 0.5 * (r[0] * r[0] + r[1] * r[1]);
            V[0] += Jp[0][0] * Jp[0][0] + Jp[1][0] * Jp[1][0];
            V[1] += Jp[0][0] * Jp[0][1] + Jp[1][0] * Jp[1][1];
            V[2] += Jp[0][0] * Jp[0][2] + Jp[1][0] * Jp[1][2];
            V[3] += Jp[0][1] * Jp[0][1] + Jp[1][1] * Jp[1][1];
            V[4] += Jp[0][1] * Jp[0][2] + Jp[1][1] * Jp[1][2];
            V[5] += Jp[0][2] * Jp[0][2] + Jp[1][2] * Jp[1][2];
#pragma unroll
            for (int i = 0; i < 3; ++i) g[i] += Jp[0][i] * r[0] + Jp[1][i] * r[1];
        }
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) V[i] = group_sum<G>(V[i]);
#pragma unroll
    for (int i = 0; i < 3; ++i) g[i] = group_sum<G>(g[i]);
    if (p < np_ && sub == 0) {
        double *vg = Vg + 9 * p;
#pragma unroll
        for (int i = 0; i < 6; ++i) vg[i] = V[i];
#pragma unroll
        for (int i = 0; i < 3; ++i) vg[6 + i] = g[i];
    }
    if (gtol > 0.0) {  // gradient_tolerance: count point-gradient entries >= gtol (an exact integer sum)
        int big = 0;
        if (p < np_ && sub == 0)
#pragma unroll
            for (int i = 0; i < 3; ++i) big += fabs(g[i]) >= gtol;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) big += __shfl_xor(big, o);
        if ((threadIdx.x & 63) == 0 && big) atomicAdd(nbig, (unsigned)big);
    }
    if (want_cost) grid_sum_last<1>(acc, partial, counter, cost_out);  // only the initial cost is used
}

// k_linearize with the cameras' Rt (96 B each) staged in LDS once per
// workgroup instead of gathered per observation (as k_backsub_trial): a
// resident grid striding over points, the next point's pstart and X loaded
// while this one is worked on, a lane's first LIN_PRE observations loaded
// together.  The per-point values are the same bits; the cost's block
// partials are summed over a different grid.
constexpr int LIN_PRE = 4;
constexpr int LIN_CL_THREADS = 256;
// the cameras' LDS stride in doubles (round 5): the
// camera reads are ds_read_b128, 16 lanes a group, 4 banks a lane; 12
// doubles (48 dwords) left the rows on 8 of the 16 bank positions (48 c mod
// 64), 14 (56 B of padding a camera) uses all 16: cfg5 LDS bank-conflict
// cycles 1.37 M -> 0.84 M per launch, 0.0179 -> 0.0174 ms.  An odd stride
// (13) spreads 8-B reads further but loses the 16-B alignment: b64 reads,
// 0.0184 ms.
#ifndef SFM_LIN_CAM_STRIDE
#define SFM_LIN_CAM_STRIDE 14
#endif
constexpr int LIN_CAM = SFM_LIN_CAM_STRIDE;
template <int G, int NT = LIN_CL_THREADS>
__global__ void __launch_bounds__(NT) k_linearize_cl(int64_t np_, int32_t nc, const int32_t *__restrict__ pstart,
                                                     const int32_t *__restrict__ cam, const double2 *__restrict__ obs,
                                                     Kmat Km, const double *__restrict__ Rt,
                                                     const double *__restrict__ X, double *__restrict__ Vg,
                                                     double *__restrict__ partial, unsigned *__restrict__ counter,
                                                     double *__restrict__ cost_out, int want_cost,
                                                     const int *__restrict__ gate, double gtol,
                                                     unsigned *__restrict__ nbig) {
    if (gate && !*gate) return;  // device-side LM control: iteration gated off
    struct Pre {
        int32_t o0, o1;
        double x[3];
    };
    auto fetch = [&](int64_t g, Pre &P) {
        const int64_t p = g / G;
        const bool live = p < np_;
        P.o0 = live ? pstart[p] : 0;
        P.o1 = live ? pstart[p + 1] : 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) P.x[i] = live ? X[3 * p + i] : 0.0;
    };
    const int64_t stride = (int64_t)gridDim.x * NT;
    Pre cur;
    fetch((int64_t)blockIdx.x * NT + threadIdx.x, cur);
    extern __shared__ __attribute__((aligned(16))) double lin_cam[];
#pragma unroll 4
    for (int i = threadIdx.x; i < 12 * nc; i += NT) lin_cam[LIN_CAM * (i / 12) + i % 12] = Rt[i];
    __syncthreads();
    double K[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) K[i] = Km.k[i];
    double acc[1] = {0.0};
    int big = 0;
    for (int64_t gt = (int64_t)blockIdx.x * NT + threadIdx.x; gt / G < np_; gt += stride) {
        const int64_t p = gt / G;
        const int sub = (int)(gt % G);
        const int32_t o0 = cur.o0, o1 = cur.o1;
        int32_t cpre[LIN_PRE];
        double2 opre[LIN_PRE];
#pragma unroll
        for (int k = 0; k < LIN_PRE; ++k) {
            const int32_t o = o0 + sub + k * G;
            cpre[k] = o < o1 ? cam[o] : 0;
            opre[k] = o < o1 ? obs[o] : make_double2(0.0, 0.0);
        }
        Pre nxt;
        fetch(gt + stride, nxt);
        const double x[3] = {cur.x[0], cur.x[1], cur.x[2]};
        double V[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
        auto add = [&](int32_t c, double2 ob) {
            const double *Rt_c = lin_cam + LIN_CAM * c;
            double r[2], A[2][3], q[3];
            obs_model(Rt_c, x, K, ob, r, A, q);
            double Jp[2][3];
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int c2 = 0; c2 < 3; ++c2)
                    Jp[a][c2] = A[a][0] * Rt_c[c2] + A[a][1] * Rt_c[3 + c2] + A[a][2] * Rt_c[6 + c2];
            acc[0] += 0.5 * (r[0] * r[0] + r[1] * r[1]);
            V[0] += Jp[0][0] * Jp[0][0] + Jp[1][0] * Jp[1][0];
            V[1] += Jp[0][0] * Jp[0][1] + Jp[1][0] * Jp[1][1];
            V[2] += Jp[0][0] * Jp[0][2] + Jp[1][0] * Jp[1][2];
            V[3] += Jp[0][1] * Jp[0][1] + Jp[1][1] * Jp[1][1];
            V[4] += Jp[0][1] * Jp[0][2] + Jp[1][1] * Jp[1][2];
            V[5] += Jp[0][2] * Jp[0][2] + Jp[1][2] * Jp[1][2];
#pragma unroll
            for (int i = 0; i < 3; ++i) g[i] += Jp[0][i] * r[0] + Jp[1][i] * r[1];
        };
#pragma unroll
        for (int k = 0; k < LIN_PRE; ++k)
            if (o0 + sub + k * G < o1) add(cpre[k], opre[k]);
        for (int32_t o = o0 + sub + LIN_PRE * G; o < o1; o += G) add(cam[o], obs[o]);
#pragma unroll
        for (int i = 0; i < 6; ++i) V[i] = group_sum<G>(V[i]);
#pragma unroll
        for (int i = 0; i < 3; ++i) g[i] = group_sum<G>(g[i]);
        if (sub == 0) {
            double *vg = Vg + 9 * p;
#pragma unroll
            for (int i = 0; i < 6; ++i) vg[i] = V[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) vg[6 + i] = g[i];
            if (gtol > 0.0)
#pragma unroll
                for (int i = 0; i < 3; ++i) big += fabs(g[i]) >= gtol;
        }
        cur = nxt;
    }
    if (gtol > 0.0) {  // gradient_tolerance: count point-gradient entries >= gtol (an exact integer sum)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) big += __shfl_xor(big, o);
        if ((threadIdx.x & 63) == 0 && big) atomicAdd(nbig, (unsigned)big);
    }
    if (want_cost) grid_sum_last<1, NT>(acc, partial, counter, cost_out);
}

// Lq layout per point (9 doubles): L00 L01 L02 L11 L12 L22 | q0 q1 q2,
// L = Cinv^T with C C^T = V + lambda clamp(diag V) (so Vd^-1 = L L^T) and
// q = L^T g_p: everything the sweep and the back substitution need of a
// point (record-free: no per-observation Schur record is written; the
// sweep rebuilds each observation's G = A^T (A R L) from X, L and the
// camera, k_schur_sweep).  A thread per point, 144 B of traffic per point.
constexpr int OBS_THREADS = 256;

__global__ void __launch_bounds__(OBS_THREADS) k_point_prep(int64_t np_, const double *__restrict__ Vg,
                                                            const double *__restrict__ lam, double *__restrict__ Lq,
                                                            const int *__restrict__ gate) {
    if (gate && !*gate) return;  // device-side LM control: iteration gated off
    // the workgroup's 9-double records go through LDS both ways: coalesced
    // global loads and stores (a thread's own 72-B record, strided across
    // the wave, touched 36 lines per load instruction)
    __shared__ double buf[9 * OBS_THREADS];
    const int64_t p0 = (int64_t)blockIdx.x * OBS_THREADS;
    const int n9 = 9 * (int)(np_ - p0 < OBS_THREADS ? np_ - p0 : OBS_THREADS);
    const int t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < 9; ++k)
        if (t + k * OBS_THREADS < n9) buf[t + k * OBS_THREADS] = Vg[9 * p0 + t + k * OBS_THREADS];
    __syncthreads();
    if (9 * t < n9) {
        const double lambda = *lam;
        double *vg = buf + 9 * t;
        const double v00 = vg[0] + lambda * clampd(vg[0]), v01 = vg[1], v02 = vg[2];
        const double v11 = vg[3] + lambda * clampd(vg[3]), v12 = vg[4];
        const double v22 = vg[5] + lambda * clampd(vg[5]);
        const double c00 = sqrt(v00), c10 = v01 / c00, c20 = v02 / c00;
        const double c11 = sqrt(v11 - c10 * c10), c21 = (v12 - c20 * c10) / c11;
        const double c22 = sqrt(v22 - c20 * c20 - c21 * c21);
        const double i00 = 1.0 / c00, i11 = 1.0 / c11, i22 = 1.0 / c22;
        const double i10 = -c10 * i00 * i11;
        const double i21 = -c21 * i11 * i22;
        const double i20 = -(c20 * i00 + c21 * i10) * i22;
        // L = Cinv^T (upper): Vd^-1 = L L^T
        const double L[3][3] = {{i00, i10, i20}, {0.0, i11, i21}, {0.0, 0.0, i22}};
        const double g0 = vg[6], g1 = vg[7], g2 = vg[8];
        double *lq = vg;  // in place: the thread's own record
        lq[0] = L[0][0]; lq[1] = L[0][1]; lq[2] = L[0][2]; lq[3] = L[1][1]; lq[4] = L[1][2]; lq[5] = L[2][2];
        lq[6] = L[0][0] * g0;
        lq[7] = L[0][1] * g0 + L[1][1] * g1;
        lq[8] = L[0][2] * g0 + L[1][2] * g1 + L[2][2] * g2;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 9; ++k)
        if (t + k * OBS_THREADS < n9) Lq[9 * p0 + t + k * OBS_THREADS] = buf[t + k * OBS_THREADS];
}

// Payload layout (doubles): S as its upper-triangle 6x6 camera blocks
// (block (i <= j) at 36 * dense index, row-major) | diagU[ns] | gc[ns] |
// bZ[ns] | cost.  Half the dense ns x ns, which is what the multi-GPU
// all-reduce moves each iteration.
__host__ __device__ __forceinline__ int64_t pay_nblk(int32_t ns) {
    const int64_t nc = (ns + 5) / 6;
    return nc * (nc + 1) / 2;
}
__host__ __device__ __forceinline__ int64_t pay_vec_base(int32_t ns) { return 36 * pay_nblk(ns); }
// element (i, j) of the symmetric S
__host__ __device__ __forceinline__ int64_t pay_index(int32_t ns, int i, int j) {
    int bi = i / 6, bj = j / 6, ri = i % 6, rj = j % 6;
    if (bi > bj) {
        const int tb = bi; bi = bj; bj = tb;
        const int tr = ri; ri = rj; rj = tr;
    }
    const int64_t nc = (ns + 5) / 6;
    return 36 * ((int64_t)bi * nc - (int64_t)bi * (bi - 1) / 2 + (bj - bi)) + ri * 6 + rj;
}
constexpr int CAMLIN = 27;  // U_c (21, upper) | g_c (6)
constexpr int ITEM_W = 42;  // 36 block + 6 bZ

// Camera items: a camera's observations (camera-major list) cut into chunks
// of <= CAM_CHUNK; BlockInfo groups the items of one camera.
constexpr int CAM_CHUNK = 4096;

struct PairItem {
    int32_t blk, k0, k1, diag;
};

struct BlockInfo {
    int32_t i, j, first_item, last_item;
};

// Camera blocks of the normal equations, once per linearisation: each item
// (a run of one camera's camera-major observations) sums U = sum Jc^T Jc (21)
// and g = sum Jc^T r (6).  A workgroup takes the items [wg_first[g],
// wg_first[g+1]) in order.  direct (every camera is one item of its own
// workgroup): the workgroup writes its camera's camlin row.  Otherwise the
// items go write-through to slab2 and the workgroup that arrives last adds
// every camera's items in order into camlin (deterministic).  Run as
// k_camera_lin, or by extra workgroups of k_schur_sweep (the CUs the sweep
// leaves idle), which then needs no launch of its own.
struct CamLinArgs {
    const PairItem *items;
    const int32_t *wg_first;
    const int32_t *cm_pt;
    const double2 *cm_obs;
    const double *X, *Rt;
    Kmat Km;
    double *slab2;
    const BlockInfo *blocks;
    int32_t nblocks, nwg, direct;
    double *camlin;
    unsigned *counter;
    const int *glin;  // gate: run only after an accepted step (LM state run_lin)
};

template <int THREADS>
__device__ __forceinline__ void camera_lin_wg(const CamLinArgs &a, int g, double (*red)[CAMLIN], int *last) {
    constexpr int NW = THREADS / 64;
    double K[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) K[i] = a.Km.k[i];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int itx = a.wg_first[g]; itx < a.wg_first[g + 1]; ++itx) {
        const PairItem it = a.items[itx];
        const double *Rc = a.Rt + 12 * it.blk;  // the item's camera
        double acc[CAMLIN];
#pragma unroll
        for (int k = 0; k < CAMLIN; ++k) acc[k] = 0.0;
        // camera-major copies of the point index and the observation (static):
        // coalesced loads, one dependent gather (X); the next observation's
        // loads are issued before this one's arithmetic
        int32_t k = it.k0 + threadIdx.x;
        double2 on = {0.0, 0.0};
        double xn[3] = {0.0, 0.0, 0.0};
        if (k < it.k1) {
            const int64_t p = a.cm_pt[k];
            on = a.cm_obs[k];
            xn[0] = a.X[3 * p]; xn[1] = a.X[3 * p + 1]; xn[2] = a.X[3 * p + 2];
        }
        for (; k < it.k1; k += THREADS) {
            const double2 ob = on;
            const double xp[3] = {xn[0], xn[1], xn[2]};
            if (k + THREADS < it.k1) {
                const int64_t p = a.cm_pt[k + THREADS];
                on = a.cm_obs[k + THREADS];
                xn[0] = a.X[3 * p]; xn[1] = a.X[3 * p + 1]; xn[2] = a.X[3 * p + 2];
            }
            double rr[2], A[2][3], q[3], Jc[2][6];
            obs_model(Rc, xp, K, ob, rr, A, q);
            jc_of(A, q, Jc);
            const double r0 = rr[0], r1 = rr[1];
            double u6[6], v6[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) { u6[i] = Jc[0][i]; v6[i] = Jc[1][i]; }
            int u = 0;
#pragma unroll
            for (int r = 0; r < 6; ++r) {
#pragma unroll
                for (int s2 = r; s2 < 6; ++s2) acc[u++] += u6[r] * u6[s2] + v6[r] * v6[s2];
                acc[21 + r] += u6[r] * r0 + v6[r] * r1;
            }
        }
#pragma unroll
        for (int e = 0; e < CAMLIN; ++e) {
            const double v = wave_sum(acc[e]);
            if (lane == 0) red[w][e] = v;
        }
        __syncthreads();
        double tot = 0.0;
        if (threadIdx.x < CAMLIN)
#pragma unroll
            for (int v = 0; v < NW; ++v) tot += red[v][threadIdx.x];
        if (threadIdx.x < CAMLIN) {
            if (a.direct)
                a.camlin[CAMLIN * it.blk + threadIdx.x] = tot;
            else
                __hip_atomic_store(a.slab2 + (int64_t)CAMLIN * itx + threadIdx.x, tot, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();  // red is reused by the next item
    }
    if (a.direct) return;
    // release as in grid_sum_last: sc1 atomic stores completed before the
    // arrival (no buffer_wbl2 on every workgroup)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        *last = __hip_atomic_fetch_add(a.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)a.nwg - 1;
    __syncthreads();
    if (!*last) return;  // sc1 loads below stand in for the acquire, as in grid_sum_last
    for (int e = threadIdx.x; e < a.nblocks * CAMLIN; e += THREADS) {
        const BlockInfo bi = a.blocks[e / CAMLIN];
        const int k = e % CAMLIN;
        double v = 0;
        for (int i0 = bi.first_item; i0 < bi.last_item; i0 += 8) {  // 8 sc1 loads in flight, summed in order
            double v8[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                v8[u] = i0 + u < bi.last_item ? __hip_atomic_load(a.slab2 + (int64_t)CAMLIN * (i0 + u) + k,
                                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                              : 0.0;
#pragma unroll
            for (int u = 0; u < 8; ++u) v += v8[u];
        }
        a.camlin[CAMLIN * bi.i + k] = v;
    }
    if (threadIdx.x == 0) *a.counter = 0u;
}

template <int THREADS>
__global__ void __launch_bounds__(THREADS) k_camera_lin(CamLinArgs a) {
    if (!*a.glin) return;  // device-side LM control: iteration gated off
    __shared__ double red[THREADS / 64][CAMLIN];
    __shared__ int last;
    camera_lin_wg<THREADS>(a, blockIdx.x, red, &last);
}

// ---------------------------------------------------------------------
// Reduced camera system S_ij = [i==j] U_i - sum_{p seen by i and j} Z_pi Z_pj^T
// as a sweep over point ranges, record-free: an observation's Schur factor
// is (p, G) with Z = E G, E = [[p]x; I], G = A^T (A R L) = M L, M = A^T A R,
// p = R X, and the pair term is S_ab = E_a (G_a G_b^T) E_b^T with
// G_a G_b^T = (G_a L^T) M_b^T = F_a M_b^T (L L^T = Vd^-1 of the shared
// point).  Both observations of a pair see the same point, so a pair needs
// only the a side's (p_a, F_a), the point's X and the b camera.
//
// The points (with their observations, point-major) are cut into NR
// ranges of equal observation count and every range into chunks.  A
// workgroup owns a fixed set of camera-block rows (a "spec": cameras i and
// nc-1-i, so every spec has the same pair work) and sweeps one range chunk
// by chunk:
//   * the chunk's observations of the spec's own cameras (the "a" side of
//     every pair) are staged in LDS one chunk ahead by two staging waves,
//     each as a slot (p_a, F_a, G_a q, X) computed from the point's X and
//     Lq and the spec's camera;
//   * every block (i, j) of the spec is owned by one lane group (2 lanes
//     per pair slot, group size proportional to the block's pair count)
//     that accumulates its 6x6 block in registers over the whole range; the
//     "b" side of a pair, M_b, is rebuilt from the slot's X and the group's
//     own camera j (registers): no global memory access in the pair loop;
//   * at the end every group reduces its slots (fixed butterfly) and writes
//     its block to slab[range][block]; k_schur_finish sums the ranges in
//     order.  Deterministic, no atomics.
constexpr int SW_THREADS = 768;

constexpr int SW_MAX_COLS = SW_THREADS / 2 - 96;  // blocks per spec (2 lanes each; a loader wave, two staging waves)
constexpr int NXCD = 8;
constexpr int SLOT_D = 18;  // staged slot (doubles): p (3) | F = G L^T (9, row-major) | G q (3) | X (3)
constexpr int SW_STAGE_WAVES = 2;  // waves that stage the next chunk (no lane group)
constexpr int SW_PAIR_WAVES = SW_THREADS / 64 - SW_STAGE_WAVES;  // the lane groups' waves (loaders among them)
constexpr int SW_STAGE_BATCH = 4;  // slots a staging lane has in flight
constexpr int SW_MAX_STAGED = 64 * SW_STAGE_WAVES * SW_STAGE_BATCH;  // slots per (chunk, spec): one staging round
constexpr int SW_STAMP_WG = 4096, SW_STAMP_EV = 68;  // SFM_SWEEP_STAMPS: workgroups, events per wave

struct SweepGroup {
    int32_t blk, lane_base, G, flags;  // flags: 1 = diagonal block, 2 = a side is the spec's second camera
    int32_t cam_b;                     // the block's column camera (the b side of every pair)
};

// an observation's (p, G) from its camera, the point X and the point's
// factor l = (L00 L01 L02 L11 L12 L22): p = R X, G = A^T (A R L)
__device__ __forceinline__ void obs_pG(const double *R, const double (&x)[3], const double (&K)[9],
                                       const double (&l)[6], double (&p)[3], double (&G)[3][3]) {
    double A[2][3];
    obs_Ap(R, x, K, A, p);
    const double L[3][3] = {{l[0], l[1], l[2]}, {0.0, l[3], l[4]}, {0.0, 0.0, l[5]}};
    double T[2][3];  // (A R) L
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        double ar[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) ar[c] = A[a][0] * R[c] + A[a][1] * R[3 + c] + A[a][2] * R[6 + c];
#pragma unroll
        for (int c = 0; c < 3; ++c) T[a][c] = ar[0] * L[0][c] + ar[1] * L[1][c] + ar[2] * L[2][c];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int c = 0; c < 3; ++c) G[i][c] = A[0][i] * T[0][c] + A[1][i] * T[1][c];
}

// the b side of a pair from its camera and the point: p = R X, the
// projection Jacobian A (2x3) and A R.  The reciprocal of the depth is
// v_rcp_f64 refined by two Newton steps (within an ulp of the division; the
// Schur sweep's Hessian only -- the residuals, the gradient and the trial
// cost use the division)
__device__ __forceinline__ void obs_pAR(const double *R, const double (&x)[3], const double (&K)[9], double (&p)[3],
                                        double (&A)[2][3], double (&ar)[2][3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) p[i] = R[3 * i] * x[0] + R[3 * i + 1] * x[1] + R[3 * i + 2] * x[2];
    const double xc0 = p[0] + R[9], xc1 = p[1] + R[10], xc2 = p[2] + R[11];
    double u[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) u[i] = K[3 * i] * xc0 + K[3 * i + 1] * xc1 + K[3 * i + 2] * xc2;
    const double wz = u[2] + 1e-8;
    double iw = __builtin_amdgcn_rcp(wz);
    iw = __builtin_fma(iw, __builtin_fma(-wz, iw, 1.0), iw);
    iw = __builtin_fma(iw, __builtin_fma(-wz, iw, 1.0), iw);
    const double pu = u[0] * iw, pv = u[1] * iw;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        A[0][c] = -(iw * K[c] - pu * iw * K[6 + c]);
        A[1][c] = -(iw * K[3 + c] - pv * iw * K[6 + c]);
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 3; ++c) ar[a][c] = A[a][0] * R[c] + A[a][1] * R[3 + c] + A[a][2] * R[6 + c];
}

// obs_pAR for a pinhole K = [[fx, 0, cx], [0, fy, cy], [0, 0, 1]] (the
// reference's calibration, checked on the host): the five structural zeros
// and the unit K[8] dropped -- 4 of the 9 products of K xc, 10 of the 12
// entries' products of A, 6 of the 18 of A R (~15 % of a pair's VALU work)
template <bool PH>
__device__ __forceinline__ void obs_pAR_k(const double *R, const double (&x)[3], const double (&K)[9],
                                          double (&p)[3], double (&A)[2][3], double (&ar)[2][3]) {
    if constexpr (!PH) {
        obs_pAR(R, x, K, p, A, ar);
    } else {
#pragma unroll
        for (int i = 0; i < 3; ++i) p[i] = R[3 * i] * x[0] + R[3 * i + 1] * x[1] + R[3 * i + 2] * x[2];
        const double xc0 = p[0] + R[9], xc1 = p[1] + R[10], xc2 = p[2] + R[11];
        const double u0 = K[0] * xc0 + K[2] * xc2, u1 = K[4] * xc1 + K[5] * xc2;
        const double wz = xc2 + 1e-8;
        double iw = __builtin_amdgcn_rcp(wz);
        iw = __builtin_fma(iw, __builtin_fma(-wz, iw, 1.0), iw);
        iw = __builtin_fma(iw, __builtin_fma(-wz, iw, 1.0), iw);
        const double pu = u0 * iw, pv = u1 * iw;
        A[0][0] = -(iw * K[0]);
        A[0][1] = 0.0;
        A[0][2] = -(iw * K[2] - pu * iw);
        A[1][0] = 0.0;
        A[1][1] = -(iw * K[4]);
        A[1][2] = -(iw * K[5] - pv * iw);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            ar[0][c] = A[0][0] * R[c] + A[0][2] * R[6 + c];
            ar[1][c] = A[1][1] * R[3 + c] + A[1][2] * R[6 + c];
        }
    }
}

// slot pieces (16 B): 0-5 p, F | 6 Gq0 Gq1 | 7 Gq2 X0 | 8 X1 X2
__device__ __forceinline__ void load_slot_a(const double2 *sl, double (&p)[3], double (&F)[3][3]) {
    const double2 v0 = sl[0], v1 = sl[1], v2 = sl[2], v3 = sl[3], v4 = sl[4], v5 = sl[5];
    p[0] = v0.x; p[1] = v0.y; p[2] = v1.x;
    F[0][0] = v1.y; F[0][1] = v2.x; F[0][2] = v2.y;
    F[1][0] = v3.x; F[1][1] = v3.y; F[1][2] = v4.x;
    F[2][0] = v4.y; F[2][1] = v5.x; F[2][2] = v5.y;
}
__device__ __forceinline__ void load_slot_x(const double2 *sl, double (&x)[3]) {
    const double2 v7 = sl[7], v8 = sl[8];
    x[0] = v7.y; x[1] = v8.x; x[2] = v8.y;
}

__device__ __forceinline__ void cross_rows(const double (&p)[3], const double (&H)[3][3], double (&X)[3][3]) {
    // X = [p]x H, [p]x = [[0,-p2,p1],[p2,0,-p0],[-p1,p0,0]]
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        X[0][c] = -p[2] * H[1][c] + p[1] * H[2][c];
        X[1][c] = p[2] * H[0][c] - p[0] * H[2][c];
        X[2][c] = -p[1] * H[0][c] + p[0] * H[1][c];
    }
}

// rows 3h..3h+2 of S_ab = E_a H E_b^T into acc[o..o+18): X = [p_a]x H (h = 0)
// or H (h = 1), row r of X E_b^T = [X [p_b]x^T | X]; the cross terms go
// into the accumulators as two fused multiply-adds each
template <int NA>
__device__ __forceinline__ void pair_rows(int h, int o, const double (&pa)[3], const double (&H)[3][3],
                                          const double (&pb)[3], double (&acc)[NA]) {
    double X[3][3];
    if (h == 0) {
        cross_rows(pa, H, X);
    } else {
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) X[i][j] = H[i][j];
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        double *a = acc + o + 6 * r;
        a[0] = __builtin_fma(pb[1], X[r][2], __builtin_fma(-pb[2], X[r][1], a[0]));
        a[1] = __builtin_fma(-pb[0], X[r][2], __builtin_fma(pb[2], X[r][0], a[1]));
        a[2] = __builtin_fma(pb[0], X[r][1], __builtin_fma(-pb[1], X[r][0], a[2]));
        a[3] += X[r][0];
        a[4] += X[r][1];
        a[5] += X[r][2];
    }
}
// a lane's share of one pair: H = G_a G_b^T = F_a M_b^T with M_b = A_b^T (A_b
// R_b), formed as (F_a (A_b R_b)^T) A_b (18 + 18 multiply-adds, not 27 + 18);
// LPP = 2: rows 3h..3h+2 (acc[0..18)); LPP = 1: the whole 6x6 block
// (acc[0..36)), H formed once
template <int LPP, bool PH = false, int NA>
__device__ __forceinline__ void pair_block(int h, const double (&pa)[3], const double (&Fa)[3][3],
                                           const double (&pb)[3], const double (&Ab)[2][3],
                                           const double (&arb)[2][3], double (&acc)[NA]) {
    double U[3][2], H[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int a = 0; a < 2; ++a) U[i][a] = Fa[i][0] * arb[a][0] + Fa[i][1] * arb[a][1] + Fa[i][2] * arb[a][2];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if constexpr (PH) {  // A_b[0][1] = A_b[1][0] = 0
            H[i][0] = U[i][0] * Ab[0][0];
            H[i][1] = U[i][1] * Ab[1][1];
            H[i][2] = U[i][0] * Ab[0][2] + U[i][1] * Ab[1][2];
        } else {
#pragma unroll
            for (int j = 0; j < 3; ++j) H[i][j] = U[i][0] * Ab[0][j] + U[i][1] * Ab[1][j];
        }
    }
    if constexpr (LPP == 2) {
        pair_rows(h, 0, pa, H, pb, acc);
    } else {
        pair_rows(0, 0, pa, H, pb, acc);
        pair_rows(1, 18, pa, H, pb, acc);
    }
}
// the diagonal block's E_a (G_a q) term: LPP = 2 rows 3h..3h+2 at acc[18..21);
// LPP = 1 all six at acc[36..42)
template <int LPP, int NA>
__device__ __forceinline__ void diag_gq(int h, const double (&pa)[3], const double (&gq)[3], double (&acc)[NA]) {
    constexpr int o = LPP == 2 ? 18 : 36;
    if (LPP == 1 || h == 0) {
        acc[o + 0] += -pa[2] * gq[1] + pa[1] * gq[2];
        acc[o + 1] += pa[2] * gq[0] - pa[0] * gq[2];
        acc[o + 2] += -pa[1] * gq[0] + pa[0] * gq[1];
    }
    if (LPP == 1 || h == 1) {
        constexpr int o2 = LPP == 2 ? 18 : 39;
        acc[o2 + 0] += gq[0]; acc[o2 + 1] += gq[1]; acc[o2 + 2] += gq[2];
    }
}

// LDS per buffer (4-B words): slots [buf_slots][2 * SLOT_D] | pairs
// [pair_cap / 2] (16-bit slot indices) | header [hdr_cap] (group pair offsets (ngroups + 1), n0, n1,
// chunk obs0); after both buffers the spec's two cameras (24 doubles).
// Chunk q uses buffer q & 1.  The list (global, list_cap words per
// (chunk, spec)) holds the slot count, then every slot's point | (row << 31).
struct SweepLds {
    int buf_slots, pair_cap, hdr_cap, list_cap;
    __device__ int words() const { return buf_slots * 2 * SLOT_D + pair_cap / 2 + hdr_cap; }
};

__device__ __forceinline__ void glds4(const void *src, void *lds) {
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void *)lds, 4, 0, 0);
}

// loader lanes (t < 64 nload): pairs and header of region qw, LDS-DMA
__device__ __forceinline__ void sweep_fetch(int t, int nload, int64_t qw, const SweepLds &L,
                                            const uint32_t *__restrict__ pairs, const int32_t *__restrict__ hdr,
                                            uint32_t *bufw) {
    const int lane = t & 63, step = 64 * nload;
    uint32_t *pw = bufw + L.buf_slots * 2 * SLOT_D;
    const int pwords = L.pair_cap / 2;
    for (int base = (t & ~63); base < pwords; base += step) glds4(pairs + qw * pwords + base + lane, pw + base);
    uint32_t *hw = pw + pwords;
    for (int base = (t & ~63); base < L.hdr_cap; base += step) glds4(hdr + qw * L.hdr_cap + base + lane, hw + base);
}

// end-of-range reduction, SW_RED_W accumulators a round: the groups' lanes
// put their accumulators in LDS (red[k][lane]), then EVERY thread of the
// workgroup takes output tasks (group, half, accumulator) and sums that
// group's slots in slot order (the order of the sequential sum before, so
// the same bits) -- independent LDS loads in flight instead of one lane per
// group walking its slots 42 times (28 us of a 92-us cfg5 workgroup)
constexpr int SW_RED_W = 21;
constexpr int SW_RED_LD = SW_THREADS + 1;  // padded row: an output task's 21 accumulators sit in different banks
// workgroup barrier ordering LDS only: outstanding global loads and stores
// stay in flight (__syncthreads drains them)
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// k_schur_sweep's chunk hand-off: wait (whole wave) until the LDS counter
// reaches target.  Bounded (200 ms of s_memrealtime): a lost hand-off raises
// the workgroup's abort word and the global error word (the host reports it)
// instead of hanging the GPU
__device__ __forceinline__ bool sw_wait(const int *c, int target, int *abort_w, int *err) {
    if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        return true;
    }
    long long t0 = -1;
    for (unsigned it = 1;; ++it) {
        __builtin_amdgcn_s_sleep(1);
        if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) break;
        if (__hip_atomic_load(abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
        if (it % 1024 == 0) {
            const long long tn = __builtin_amdgcn_s_memrealtime();
            if (t0 < 0) t0 = tn;
            else if (tn - t0 > 20000000) {
                __hip_atomic_store(abort_w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (err && (threadIdx.x & 63) == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    return true;
}
// after the wave's LDS writes (and, for a loader, its LDS-DMA: vmcnt first)
__device__ __forceinline__ void sw_signal(int *c) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The dispatch tail (round 4): nspec x nrange (spec, range) items run as
// rounds of one workgroup per CU; when the last round would be a sliver
// (cfg5: 800 items on 256 CUs, the fourth round 32 workgroups for a
// quarter of the span), the specs [w0, nspec) that would form it are cut
// per range into S chunk sub-ranges instead, S x as many short workgroups
// filling the last round.  A sub-range's partial goes to slabx, indexed by
// (range, sub-range, spec - w0, group); k_schur_finish adds those partials
// in (range, sub-range) order for the split specs' blocks.
struct SweepSplit {
    int32_t nfull, S, w0, nsplit, gmax;  // S = 0: no split (every workgroup a whole item)
    double *slabx;
};

template <int LPP, int NACC>
__device__ __forceinline__ void sweep_reduce(const double (&acc)[NACC], bool has_acc, int t, int ng,
                                             const SweepGroup *__restrict__ grps, double *__restrict__ slab_r,
                                             double *red, bool by_group = false) {
    constexpr int NH = LPP == 2 ? 2 : 1;  // output halves per group (LPP = 2: rows 3h..3h+2)
    // the spec's group table in LDS after the accumulators (one global
    // latency, not one per output task)
    SweepGroup *gtab = reinterpret_cast<SweepGroup *>(red + SW_RED_W * SW_RED_LD);
    for (int g = t; g < ng; g += SW_THREADS) gtab[g] = grps[g];
#pragma unroll
    for (int k0 = 0; k0 < NACC; k0 += SW_RED_W) {
        if (has_acc)
#pragma unroll
            for (int k = 0; k < SW_RED_W; ++k) red[k * SW_RED_LD + t] = acc[k0 + k];
        lds_barrier();
        for (int o = t; o < ng * NH * SW_RED_W; o += SW_THREADS) {
            const int g = o / (NH * SW_RED_W), hk = o % (NH * SW_RED_W), h = hk / SW_RED_W, k = hk % SW_RED_W;
            const SweepGroup gr = gtab[g];
            const int kk = k0 + k;
            const bool dg = gr.flags & 1;
            // LPP = 1: acc[0..36) the 6x6 block row-major, acc[36..42) the
            // diagonal's sum Z q; LPP = 2: acc[0..18) rows 3h..3h+2, acc[18..21) the
            // diagonal's three sum Z q entries of half h
            const int dst = LPP == 2 ? (kk < 18 ? 18 * h + kk : 36 + 3 * h + (kk - 18)) : kk;
            if (dst >= 36 && !dg) continue;
            const double *src = red + k * SW_RED_LD + gr.lane_base + h;
            double v = 0.0;
            const int n = gr.G / LPP;
            int sl = 0;
            for (; sl + 4 <= n; sl += 4) {  // four loads in flight, summed in slot order
                const double a0 = src[LPP * sl], a1 = src[LPP * (sl + 1)], a2 = src[LPP * (sl + 2)],
                             a3 = src[LPP * (sl + 3)];
                v += a0;
                v += a1;
                v += a2;
                v += a3;
            }
            for (; sl < n; ++sl) v += src[LPP * sl];
            slab_r[(int64_t)(by_group ? g : gr.blk) * ITEM_W + dst] = v;
        }
        lds_barrier();  // the slab stores need not land before the next round
    }
}

template <int LPP, bool PH = false>  // lanes per pair slot; pinhole K
__global__ void __launch_bounds__(SW_THREADS) k_schur_sweep(
    int32_t nspec, int32_t nrange, int32_t nbd, SweepLds L, const int32_t *__restrict__ rchunk,
    const int32_t *__restrict__ spec_nload, const int32_t *__restrict__ spec_goff,
    const SweepGroup *__restrict__ groups, const int16_t *__restrict__ lanegrp,
    const int32_t *__restrict__ spec_cam, const uint32_t *__restrict__ list, const uint32_t *__restrict__ pairs,
    const int32_t *__restrict__ hdr, const double *__restrict__ Xg, const double *__restrict__ Lq,
    const double *__restrict__ Rt, Kmat Km, double *__restrict__ slab, const int *__restrict__ gate, int dbg,
    int nsweep, CamLinArgs cl, long long *__restrict__ stamps, int *__restrict__ sw_err, SweepSplit sp) {
    extern __shared__ double2 sw_lds[];
    if ((int)blockIdx.x >= nsweep) {  // camera blocks of the normal equations on the CUs the sweep leaves idle
        if (!*cl.glin) return;
        double(*red)[CAMLIN] = reinterpret_cast<double(*)[CAMLIN]>(sw_lds);
        camera_lin_wg<SW_THREADS>(cl, (int)blockIdx.x - nsweep, red,
                                  reinterpret_cast<int *>(sw_lds + SW_THREADS / 64 * CAMLIN / 2 + 1));
        return;
    }
    if (gate && !*gate) return;  // device-side LM control: iteration gated off
    uint32_t *ldsw = reinterpret_cast<uint32_t *>(sw_lds);
    // the work item: a whole (spec, range), or a chunk sub-range of a split one
    int w, r, q0, q1;
    double *slab_out;
    const bool sub = sp.S > 0 && (int)blockIdx.x >= sp.nfull;
    if (!sub) {
        if (nrange >= NXCD) {  // range r on XCD r % 8 (round-robin dispatch)
            const int loc = blockIdx.x / NXCD;
            w = loc % nspec;
            r = (loc / nspec) * NXCD + (int)(blockIdx.x % NXCD);
        } else {  // 1, 2 or 4 ranges: range r on the XCDs x with x % nrange == r
            const int x = blockIdx.x % NXCD;
            w = (int)(blockIdx.x / NXCD) * (NXCD / nrange) + x / nrange;
            r = x % nrange;
            if (w >= nspec) return;  // whole workgroup
        }
        if (r >= nrange) return;  // whole workgroup
        q0 = rchunk[r];
        q1 = rchunk[r + 1];
        slab_out = slab + (int64_t)r * nbd * ITEM_W;
    } else {
        const int u = blockIdx.x - sp.nfull, v = u / NXCD, s = v % sp.S;
        r = u % NXCD;
        w = sp.w0 + v / sp.S;
        const int Q0 = rchunk[r], Q1 = rchunk[r + 1];
        q0 = Q0 + (Q1 - Q0) * s / sp.S;
        q1 = Q0 + (Q1 - Q0) * (s + 1) / sp.S;
        slab_out = sp.slabx + ((int64_t)((r * sp.S + s) * sp.nsplit + (w - sp.w0)) * sp.gmax) * ITEM_W;
    }
    const int t = threadIdx.x;
    // SFM_SWEEP_STAMPS: s_memrealtime per (workgroup, event, wave), lane 0
    long long *stw = stamps && blockIdx.x < SW_STAMP_WG && (t & 63) == 0
                         ? stamps + (int64_t)blockIdx.x * SW_STAMP_EV * (SW_THREADS / 64) + (t >> 6)
                         : nullptr;
    auto stamp = [&](int ev) {
        if (stw && ev < SW_STAMP_EV) stw[ev * (SW_THREADS / 64)] = (long long)__builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    const int nload = spec_nload[w];
    const bool loader = (t >> 6) < nload;
    const int gi = lanegrp[w * SW_THREADS + t];
    const int ng = spec_goff[w + 1] - spec_goff[w];
    SweepGroup grp = {0, 0, 2, 0, 0};
    if (gi >= 0) grp = groups[spec_goff[w] + gi];
    const int h = LPP == 2 ? (t - grp.lane_base) & 1 : 0, slot = (t - grp.lane_base) / LPP, nslot = grp.G / LPP;
    constexpr int NACC = LPP == 2 ? 21 : 42;
    const bool diag = grp.flags & 1, second = grp.flags & 2;
    const int bw = L.words();
    double *scam = reinterpret_cast<double *>(ldsw + 2 * bw);  // the spec's cameras (rows 0 and 1)
    // chunk hand-off counters: filled[b] += 1 per producer
    // wave (two stagers, nload loaders) once its part of a chunk is in buffer
    // b; freed[b] += 1 per pair wave once it is done with the chunk in b.
    // Instead of a workgroup barrier per chunk, a pair wave waits only for
    // its next chunk to be filled and a producer only for its buffer to be
    // freed, so the per-chunk spread between the lane groups (Poisson pair
    // counts) averages out over the chunks instead of adding up chunk by chunk
    int *cnt = reinterpret_cast<int *>(scam + 24);  // filled[2] | freed[2] | abort
    if (t < 5) cnt[t] = 0;
    if (t < 24) {
        const int c = spec_cam[2 * w + t / 12];
        scam[t] = c >= 0 ? Rt[12 * c + t % 12] : 0.0;
    }
    double K[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) K[i] = Km.k[i];
    const int tst = t - (SW_THREADS - 64 * SW_STAGE_WAVES);
    // a scalar branch: the two roles run different barrier sequences, and a
    // barrier inside an exec-masked (divergent) region would still execute
    if (__builtin_amdgcn_readfirstlane(t >> 6) >= SW_THREADS / 64 - SW_STAGE_WAVES) {
        // the next chunk's staging was the chunk hand-off's critical path
        // (round 6 stamps at cfg5: the pair waves waited 1.01 us a chunk for
        // it, the stagers 0.24 us for them): the staging waves issue first on
        // the SIMDs they share with pair waves (waits 0.01 / 1.79 us; the
        // sweep 0.296-0.301 -> 0.293-0.296 ms at cfg5, 0.0805 -> 0.0784 at
        // cfg4).  Ranking the pair waves by their trips in the chunk the same
        // way measured slower (cfg5 0.322-0.327 ms), not kept.
        __builtin_amdgcn_s_setprio(2);
        // staging waves (no lane group): chunk q + 1's slots into the other
        // buffer while the groups work on chunk q; SW_STAGE_BATCH slots a
        // lane per round, their list entries, then their points' X and Lq,
        // all in flight together.  The same barriers as the groups below.
        // one round a chunk: lane l stages slots l + 128 u (u < SW_STAGE_BATCH;
        // the planner caps a chunk's slots at SW_MAX_STAGED).  Software
        // pipelined over the chunks: while chunk q + 1 is written from
        // registers, the points of chunk q + 2 and the list entries of chunk
        // q + 3 are in flight, across the barrier (an LDS-only barrier: the
        // stagers' loads need not land).
        constexpr int SB = SW_STAGE_BATCH, SSTEP = 64 * SW_STAGE_WAVES;
        uint32_t e1[SB], e2[SB];
        int n1 = 0, n2 = 0;
        double gx[SB][3], gl[SB][9];
        auto load_list = [&](int qs, uint32_t(&e)[SB], int &n) {
            if (qs >= q1) {  // uniform; point 0 stands in (load_pts may still read it)
                n = 0;
#pragma unroll
                for (int u = 0; u < SB; ++u) e[u] = 0u;
                return;
            }
            // word 0: the (chunk, spec)'s slot count; the entries follow
            // (padded to list_cap > buf_slots: every load is in bounds)
            const uint32_t *lst = list + ((int64_t)qs * nspec + w) * L.list_cap;
            n = (int)lst[0];
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int sl = tst + u * SSTEP;
                e[u] = lst[1 + (sl < L.buf_slots ? sl : 0)];
            }
        };
        auto load_pts = [&](const uint32_t(&e)[SB]) {
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int64_t P = e[u] & 0x7fffffffu;
#pragma unroll
                for (int i = 0; i < 3; ++i) gx[u][i] = Xg[3 * P + i];
#pragma unroll
                for (int i = 0; i < 9; ++i) gl[u][i] = Lq[9 * P + i];
            }
        };
        auto commit = [&](const uint32_t(&e)[SB], int n, uint32_t *bw_dst) {
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int sl = tst + u * SSTEP;
                if (sl >= n) continue;
                const double *R = scam + 12 * (int)(e[u] >> 31);
                const double l[6] = {gl[u][0], gl[u][1], gl[u][2], gl[u][3], gl[u][4], gl[u][5]};
                const double x[3] = {gx[u][0], gx[u][1], gx[u][2]};
                double pa[3], G[3][3], F[3][3], gq[3];
                obs_pG(R, x, K, l, pa, G);
                // F = G L^T (L upper: L^T[k][c] = L[c][k], k >= c); G q
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    F[i][0] = G[i][0] * l[0] + G[i][1] * l[1] + G[i][2] * l[2];
                    F[i][1] = G[i][1] * l[3] + G[i][2] * l[4];
                    F[i][2] = G[i][2] * l[5];
                    gq[i] = G[i][0] * gl[u][6] + G[i][1] * gl[u][7] + G[i][2] * gl[u][8];
                }
                double2 *d = reinterpret_cast<double2 *>(bw_dst) + sl * (SLOT_D / 2);
                d[0] = make_double2(pa[0], pa[1]);
                d[1] = make_double2(pa[2], F[0][0]);
                d[2] = make_double2(F[0][1], F[0][2]);
                d[3] = make_double2(F[1][0], F[1][1]);
                d[4] = make_double2(F[1][2], F[2][0]);
                d[5] = make_double2(F[2][1], F[2][2]);
                d[6] = make_double2(gq[0], gq[1]);
                d[7] = make_double2(gq[2], x[0]);
                d[8] = make_double2(x[1], x[2]);
            }
        };
        load_list(q0, e1, n1);
        load_list(q0 + 1, e2, n2);
        load_pts(e1);
        __syncthreads();  // the cameras are in LDS
        if (q0 < q1) commit(e1, n1, ldsw);
        sw_signal(&cnt[0]);
        auto advance = [&]() {  // chunk q+2's points and chunk q+3's list in flight
            load_pts(e2);
#pragma unroll
            for (int u = 0; u < SB; ++u) e1[u] = e2[u];
            n1 = n2;
        };
        advance();
        load_list(q0 + 2, e2, n2);
        stamp(1);
        for (int q = q0; q < q1; ++q) {
            if (q + 1 < q1) {
                const int b1 = ((q - q0) & 1) ^ 1;
                // buffer b1 held chunk q - 1: every pair wave done with it
                if (sw_wait(&cnt[2 + b1], ((q + 1 - q0) >> 1) * SW_PAIR_WAVES, &cnt[4], sw_err)) {
                    commit(e1, n1, ldsw + b1 * bw);
                    sw_signal(&cnt[b1]);
                }
            }
            if (q + 2 < q1) {
                advance();
                load_list(q + 3, e2, n2);
            }
            stamp(2 + q - q0);
        }
        lds_barrier();  // every pair wave is done with the buffers sweep_reduce reuses
        const double none[NACC] = {};  // no accumulators: output tasks only
        sweep_reduce<LPP>(none, false, t, ng, groups + spec_goff[w], slab_out, reinterpret_cast<double *>(sw_lds),
                          sub);
        stamp(SW_STAMP_EV - 1);
        return;
    }
    double Rb[12];  // the group's column camera (the b side; the a camera itself for a diagonal block)
#pragma unroll
    for (int k = 0; k < 12; ++k) Rb[k] = gi >= 0 ? Rt[12 * grp.cam_b + k] : 0.0;
    double acc[NACC];
#pragma unroll
    for (int k = 0; k < NACC; ++k) acc[k] = 0.0;
    if (q0 < q1 && loader) sweep_fetch(t, nload, (int64_t)q0 * nspec + w, L, pairs, hdr, ldsw);
    __syncthreads();  // the cameras are in LDS
    stamp(1);
    const int nprod = SW_STAGE_WAVES + nload;  // producer waves of a chunk
    if (loader && q0 < q1) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA of chunk q0's pairs and header
        sw_signal(&cnt[0]);
    }
    for (int q = q0; q < q1; ++q) {
        const int cur = (q - q0) & 1;
        const uint32_t *bufw = ldsw + cur * bw;
        if (loader && q + 1 < q1) {
            // buffer cur ^ 1 held chunk q - 1: every pair wave done with it
            if (sw_wait(&cnt[2 + (cur ^ 1)], ((q + 1 - q0) >> 1) * SW_PAIR_WAVES, &cnt[4], sw_err))
                sweep_fetch(t, nload, (int64_t)(q + 1) * nspec + w, L, pairs, hdr, ldsw + (cur ^ 1) * bw);
        }
        const bool have = sw_wait(&cnt[cur], (((q - q0) >> 1) + 1) * nprod, &cnt[4], sw_err);
        if (gi >= 0 && have) {
            const double2 *buf = reinterpret_cast<const double2 *>(bufw);
            const uint32_t *pl = bufw + L.buf_slots * 2 * SLOT_D;
            const int32_t *hd = reinterpret_cast<const int32_t *>(pl + L.pair_cap / 2);
            const int n0 = hd[ng + 1], n1 = hd[ng + 2];
            if (diag) {  // S_ii: the camera's own observations, b = a; plus sum Z_a q_p
                const int a0 = second ? n0 : 0, a1 = second ? n0 + n1 : n0;
                for (int a = a0 + slot; a < a1; a += nslot) {
                    const double2 *sl = buf + a * (SLOT_D / 2);
                    double pa[3], Fa[3][3], x[3], pm[3], Aa[2][3], ara[2][3];
                    load_slot_a(sl, pa, Fa);
                    load_slot_x(sl, x);
                    obs_pAR_k<PH>(Rb, x, K, pm, Aa, ara);
                    pair_block<LPP, PH>(h, pa, Fa, pa, Aa, ara, acc);
                    const double2 v6 = sl[6], v7 = sl[7];
                    const double gq[3] = {v6.x, v6.y, v7.x};  // G_a q
                    diag_gq<LPP>(h, pa, gq, acc);
                }
            } else {
                const int k0 = hd[gi], k1 = hd[gi + 1];
                const uint16_t *pl16 = reinterpret_cast<const uint16_t *>(pl);
                for (int k = k0 + slot; k < k1; k += nslot) {
                    const double2 *sl = buf + (int)pl16[k] * (SLOT_D / 2);
                    double pa[3], Fa[3][3], x[3], pb[3], Ab[2][3], arb[2][3];
                    load_slot_a(sl, pa, Fa);
                    load_slot_x(sl, x);
                    obs_pAR_k<PH>(Rb, x, K, pb, Ab, arb);  // the b side: camera j, the same point
                    pair_block<LPP, PH>(h, pa, Fa, pb, Ab, arb, acc);
                }
            }
        }
        if (loader && q + 1 < q1) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // chunk q + 1's DMA, overlapped with chunk q
            sw_signal(&cnt[cur ^ 1]);
        }
        sw_signal(&cnt[2 + cur]);
        stamp(2 + q - q0);
    }
    // reduce the groups' slots in slot order through LDS (the staging
    // buffers are free now)
    lds_barrier();
    sweep_reduce<LPP>(acc, gi >= 0, t, ng, groups + spec_goff[w], slab_out, reinterpret_cast<double *>(sw_lds), sub);
    stamp(SW_STAMP_EV - 1);
}

// one thread per (camera block, entry) over the dense upper-triangle block
// index (blocks of ITEM_W entries, coalesced across the workgroup): fixed-
// order sum over the ranges, then U_i - S (diagonal) / -S (off-diagonal,
// mirrored), g_c and sum Z q into the payload.  (Round 4: it was one
// 64-thread workgroup per block, 42 lanes busy, one range load at a time:
// 20,100 workgroups at cfg5, 28 us.)
constexpr int FIN_THREADS = 256;
__global__ void __launch_bounds__(FIN_THREADS) k_schur_finish(int32_t ns, int32_t nbd, int32_t nrange,
                                                              const int2 *__restrict__ blkij,
                                                              const double *__restrict__ slab,
                                                              const double *__restrict__ camlin,
                                                              double *__restrict__ payload, const int *__restrict__ gate,
                                                              const int32_t *__restrict__ split_of, SweepSplit sp) {
    if (gate && !*gate) return;  // device-side LM control: iteration gated off
    const int64_t e = (int64_t)blockIdx.x * FIN_THREADS + threadIdx.x;
    if (e >= (int64_t)nbd * ITEM_W) return;
    const int b = (int)(e / ITEM_W), t = (int)(e - (int64_t)b * ITEM_W);
    const int2 ij = blkij[b];
    const bool diag = ij.x == ij.y;
    if (t >= (diag ? ITEM_W : 36)) return;
    const int si = sp.S > 0 ? split_of[b] : -1;  // (spec - w0) * gmax + group, split specs only
    // the partials in range order, eight loads in flight, summed one by one
    const double *src = si < 0 ? slab + (int64_t)b * ITEM_W + t : sp.slabx + (int64_t)si * ITEM_W + t;
    const int64_t rstr = si < 0 ? (int64_t)nbd * ITEM_W : (int64_t)sp.nsplit * sp.gmax * ITEM_W;
    const int n = si < 0 ? nrange : nrange * sp.S;
    double v = 0;
    int q = 0;
    for (; q + 8 <= n; q += 8) {
        double a8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) a8[u] = src[(q + u) * rstr];
#pragma unroll
        for (int u = 0; u < 8; ++u) v += a8[u];
    }
    for (; q < n; ++q) v += src[q * rstr];
    const int64_t base = pay_vec_base(ns);
    if (t < 36) {
        const int r = t / 6, c = t % 6;
        const int64_t row = 6 * ij.x + r;
        double *blk = payload + pay_index(ns, 6 * ij.x, 6 * ij.y);  // the block's (0, 0)
        if (diag) {
            const int lo = r < c ? r : c, hi = r < c ? c : r;
            const double u = camlin[CAMLIN * ij.x + lo * 6 - lo * (lo - 1) / 2 + (hi - lo)];
            blk[t] = u - v;
            if (r == c) payload[base + row] = u;  // diag(U)
        } else {
            blk[t] = -v;
        }
    } else {
        const int r = t - 36;
        payload[base + ns + 6 * ij.x + r] = camlin[CAMLIN * ij.x + 21 + r];  // g_c
        payload[base + 2 * ns + 6 * ij.x + r] = v;                           // sum Z q
    }
}

// --------------------------------------------------------------- Cholesky
// Blocked (NB = 16) right-looking fp64 Cholesky of the padded nsp x nsp
// reduced camera system with the forward substitution folded in (b is
// carried along); one k_chol_col launch per tile column (below), then
// k_chol_backsolve solves L^T x = y in one workgroup.
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// broadcast lane l's double to the whole wave (two v_readlane_b32 -> SGPRs)
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// ---- merged step kernel: one launch per tile column s (nT launches).
// Launch s applies column s-1's trailing update to every lower tile (r, c),
// c >= s, and factors column s in the same launch:
//   tile (r, c), c > s : A_rc -= L_r,s-1 L_c,s-1^T
//   tile (r, s), r > s : C_rs = A_rs - L_r,s-1 L_s,s-1^T, C_ss likewise
//                        (recomputed identically by every column block),
//                        wave 0 factors C_ss and, in the same chain on its
//                        other lanes, forms L_rs = C_rs L_ss^-T, written with
//                        its mirror;
//   tile (s, s)        : C_ss, factor, y_s = L_ss^-1 (b_s - L_s,s-1 y_s-1),
//                        L_ss -> D[s & 1] (read-only copy of A_ss is still
//                        in use by the other column blocks);
//   block 0 (s >= 1)   : D[(s-1) & 1] -> A's diagonal tile s-1 and
//                        b_i -= L_i,s-1 y_s-1 for rows past column s.
template <int TB>
__device__ __forceinline__ void chol_factor(double (&r)[TB], double (&dinv)[TB], int lane, int *bad) {
#pragma unroll
    for (int k = 0; k < TB; ++k) {
        const double d = readlane_f64(r[k], k);
        if (lane == 0 && !(d > 0.0)) *bad = 1;
        // 1/sqrt(d): v_rsq_f64 then two Newton steps (~1 ulp), off the
        // long IEEE sqrt + divide sequences of the serial chain
        double g = __builtin_amdgcn_rsq(d);
        g = g * (1.5 - 0.5 * d * g * g);
        g = g * (1.5 - 0.5 * d * g * g);
        dinv[k] = g;
        r[k] = (lane == k) ? d * g : r[k] * g;
#pragma unroll
        for (int j = k + 1; j < TB; ++j) r[j] -= r[k] * readlane_f64(r[k], j);
    }
}

// lane j of each 16-lane row of the wave, to the whole row: one
// v_mov_b64_dpp row_newbcast (DPP64), no SGPR round trip
template <int J>
__device__ __forceinline__ double bcast16_c(double v) {
    return __longlong_as_double(
        __builtin_amdgcn_update_dpp(0ll, __double_as_longlong(v), 0x150 + J, 0xF, 0xF, true));
}
__device__ __forceinline__ double bcast16(double v, int j) {  // j a constant after unrolling
    switch (j) {
    case 0: return bcast16_c<0>(v);   case 1: return bcast16_c<1>(v);   case 2: return bcast16_c<2>(v);
    case 3: return bcast16_c<3>(v);   case 4: return bcast16_c<4>(v);   case 5: return bcast16_c<5>(v);
    case 6: return bcast16_c<6>(v);   case 7: return bcast16_c<7>(v);   case 8: return bcast16_c<8>(v);
    case 9: return bcast16_c<9>(v);   case 10: return bcast16_c<10>(v); case 11: return bcast16_c<11>(v);
    case 12: return bcast16_c<12>(v); case 13: return bcast16_c<13>(v); case 14: return bcast16_c<14>(v);
    default: return bcast16_c<15>(v);
    }
}

// r_j += bcast_j(rk) * nrk and p_j += bcast_j(rk) * npk, two v_fmac_f64 with
// a row_newbcast:j source (DPP64).  Inline asm, so the panel updates stay in
// the pivot step that produces their operand (the compiler otherwise sinks
// them to the end and holds the 120 broadcasts in registers); NOP = 1 puts
// the two wait states a DPP read of a just-written VGPR needs in front.
template <int J, int NOP>
__device__ __forceinline__ void fmac2_bc(double &rj, double &pj, double rk, double nrk, double npk) {
    if constexpr (NOP)
        asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %2, %3 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %1, %2, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf"
                     : "+v"(rj), "+v"(pj) : "v"(rk), "v"(nrk), "v"(npk), "n"(J));
    else
        asm volatile("v_fmac_f64_dpp %0, %2, %3 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %1, %2, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf"
                     : "+v"(rj), "+v"(pj) : "v"(rk), "v"(nrk), "v"(npk), "n"(J));
}
template <int J>
__device__ __forceinline__ double bcast16_asm(double v) {  // s_nop: v may have just been written
    double d;
    asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
                 : "=v"(d) : "v"(v), "n"(J));
    return d;
}
template <int K, int... I>
__device__ __forceinline__ void chol16_updates(double (&r)[16], double (&p)[16], std::integer_sequence<int, I...>) {
    const double nrk = -r[K], npk = -p[K];
    (fmac2_bc<K + 1 + I, I == 0>(r[K + 1 + I], p[K + 1 + I], r[K], nrk, npk), ...);
}

// The same factor for TB = 16 with the broadcasts inside 16-lane DPP rows:
// every row of the wave holds C_ss (r[j] = element (li, j), li = lane & 15)
// and one row of the panel (p[j] = C_rs element (li, j)).  Step k scales
// column k by 1/L_kk and subtracts L_jk (lane j's r[k], one row_newbcast)
// times it from columns j > k, in r and p alike: the operation order of
// chol_factor, so L_ss and L_rs = C_rs L_ss^-T are bitwise the same.
template <int K>
__device__ __forceinline__ void chol16_step(double (&r)[16], double (&p)[16], double (&dinv)[16], int li,
                                            bool &nonpos) {
    const double d = bcast16_asm<K>(r[K]);
    nonpos |= !(d > 0.0);
    double g = __builtin_amdgcn_rsq(d);
    g = g * (1.5 - 0.5 * d * g * g);
    g = g * (1.5 - 0.5 * d * g * g);
    dinv[K] = g;
    r[K] = (li == K) ? d * g : r[K] * g;
    p[K] = p[K] * g;
    if constexpr (K < 15) chol16_updates<K>(r, p, std::make_integer_sequence<int, 15 - K>{});
}
template <int... K>
__device__ __forceinline__ void chol16_steps(double (&r)[16], double (&p)[16], double (&dinv)[16], int li,
                                             bool &nonpos, std::integer_sequence<int, K...>) {
    (chol16_step<K>(r, p, dinv, li, nonpos), ...);
}
__device__ __forceinline__ void chol_factor16(double (&r)[16], double (&p)[16], double (&dinv)[16], int li,
                                              int lane, int *bad) {
    bool nonpos = false;  // one store after the chain: no branch (and basic block) per pivot
    chol16_steps(r, p, dinv, li, nonpos, std::make_integer_sequence<int, 16>{});
    if (lane == 0 && nonpos) *bad = 1;
}

// element (i, j) of the damped, identity-padded system S + lambda clamp(diag U)
// read straight from the Schur payload (launch 0 assembles as it loads)
__device__ __forceinline__ double assembled(const double *__restrict__ payload, int32_t ns, double lambda, int i,
                                            int j) {
    if (i < ns && j < ns) {
        double v = payload[pay_index(ns, i, j)];
        if (i == j) v += lambda * clampd(payload[pay_vec_base(ns) + i]);
        return v;
    }
    return i == j ? 1.0 : 0.0;
}

__device__ __forceinline__ double assembled_b(const double *__restrict__ payload, int32_t ns, int i) {
    const int64_t base = pay_vec_base(ns);
    return i < ns ? -payload[base + ns + i] + payload[base + 2 * ns + i] : 0.0;
}

// One rank, no all-reduce between the sweep and the solve: launch 0 reads the
// system straight from the sweep's per-range slabs (k_schur_finish's sums, in
// its order, so bitwise the same values) and one extra workgroup writes the
// payload's vectors for the back substitution's epilogue; no finish launch.
struct SlabSrc {
    const double *slab, *camlin;  // slab == nullptr: read the finished payload
    int32_t nbd, nrange;
    SweepSplit sp;                // the dispatch tail's split (sp.S = 0: none)
    const int32_t *split_of;
};

__device__ __forceinline__ double slab_sum(const SlabSrc &q, int64_t blk, int item) {
    double v = 0;
    const int si = q.sp.S > 0 ? q.split_of[blk] : -1;
    if (si >= 0) {  // a split spec's block: every (range, sub-range) partial, in order (k_schur_finish's)
        const int64_t row = (int64_t)q.sp.nsplit * q.sp.gmax * ITEM_W;
        const double *src = q.sp.slabx + (int64_t)si * ITEM_W + item;
        const int n = q.nrange * q.sp.S;
        for (int r0 = 0; r0 < n; r0 += 8) {
            double x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = r0 + u < n ? src[(r0 + u) * row] : 0.0;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (r0 + u < n) v += x[u];
        }
        return v;
    }
    const int64_t stride = (int64_t)q.nbd * ITEM_W;
    const double *src = q.slab + blk * ITEM_W + item;
    for (int r0 = 0; r0 < q.nrange; r0 += 8) {  // 8 loads in flight, then the sum in range order
        double x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = r0 + u < q.nrange ? src[(r0 + u) * stride] : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (r0 + u < q.nrange) v += x[u];
    }
    return v;
}

__device__ __forceinline__ double cam_u(const double *__restrict__ camlin, int c, int r, int k) {
    const int lo = r < k ? r : k, hi = r < k ? k : r;
    return camlin[CAMLIN * c + lo * 6 - lo * (lo - 1) / 2 + (hi - lo)];
}

__device__ __forceinline__ double assembled_src(const SlabSrc &q, const double *__restrict__ payload, int32_t ns,
                                                double lambda, int i, int j) {
    if (!q.slab) return assembled(payload, ns, lambda, i, j);
    if (i < ns && j < ns) {
        const int64_t idx = pay_index(ns, i, j);
        const int item = (int)(idx % 36);
        const double s = slab_sum(q, idx / 36, item);
        double v = (i / 6 == j / 6) ? cam_u(q.camlin, i / 6, item / 6, item % 6) - s : -s;
        if (i == j) v += lambda * clampd(cam_u(q.camlin, i / 6, i % 6, i % 6));
        return v;
    }
    return i == j ? 1.0 : 0.0;
}

__device__ __forceinline__ double gc_src(const SlabSrc &q, int i) { return q.camlin[CAMLIN * (i / 6) + 21 + i % 6]; }
__device__ __forceinline__ double bz_src(const SlabSrc &q, int32_t ns, int i) {
    return slab_sum(q, pay_index(ns, i - i % 6, i - i % 6) / 36, 36 + i % 6);
}

__device__ __forceinline__ double assembled_b_src(const SlabSrc &q, const double *__restrict__ payload, int32_t ns,
                                                  int i) {
    if (!q.slab) return assembled_b(payload, ns, i);
    return i < ns ? -gc_src(q, i) + bz_src(q, ns, i) : 0.0;
}

template <int TB>
__global__ void __launch_bounds__(256) k_chol_col(double *__restrict__ A, int32_t nsp, int s,
                                                  double *__restrict__ D, double *__restrict__ bvec,
                                                  int *__restrict__ bad, const double *__restrict__ payload,
                                                  int32_t ns, const double *__restrict__ lam,
                                                  const int *__restrict__ gate, int dpp, SlabSrc src,
                                                  double *__restrict__ payload_out) {
    if (gate && !*gate) return;  // device-side LM control: iteration gated off
    const double lambda = s == 0 ? *lam : 0.0;
    __shared__ double Lr[TB][TB + 1], Lc[TB][TB + 1], Ct[TB][TB + 1], Cd[TB][TB + 1];
    __shared__ double yk[TB];
    const int t = threadIdx.x;
    const bool upd = s >= 1;
    const int kp = (s - 1) * TB;  // previous column's first index
    int blk = blockIdx.x;
    if (!upd && src.slab && blk == 0) {  // launch 0 from the slabs: the payload's vectors
        const int64_t base = pay_vec_base(ns);
        for (int i = t; i < ns; i += blockDim.x) {
            payload_out[base + i] = cam_u(src.camlin, i / 6, i % 6, i % 6);
            payload_out[base + ns + i] = gc_src(src, i);
            payload_out[base + 2 * ns + i] = bz_src(src, ns, i);
        }
        return;
    }
    if (!upd && src.slab) --blk;
    if (upd && blk == 0) {
        const double *Dp = D + ((s - 1) & 1) * TB * TB;
        for (int e = t; e < TB * TB; e += blockDim.x) {
            const int i = e / TB, j = e % TB;
            A[(int64_t)(kp + i) * nsp + kp + j] = i >= j ? Dp[i * TB + j] : Dp[j * TB + i];
        }
        if (t < TB) yk[t] = bvec[kp + t];
        __syncthreads();
        for (int i = (s + 1) * TB + t; i < nsp; i += blockDim.x) {
            double acc = 0;
#pragma unroll 8
            for (int m = 0; m < TB; ++m) acc += A[(int64_t)(kp + m) * nsp + i] * yk[m];  // L[i][kp+m] (mirror)
            bvec[i] -= acc;
        }
        return;
    }
    if (upd) --blk;
    int rr = 0;
    while (blk > rr) { blk -= rr + 1; ++rr; }
    const int r = s + rr, c = s + blk;  // lower tile (r, c), r >= c >= s
    const int r0 = r * TB, c0 = c * TB, s0 = s * TB;
    const bool colblk = c == s, need_d = colblk && r > s;
    // every global load of the block in one round: L_r,s-1, L_c,s-1, A_rc, A_ss
    constexpr int EPT = TB * TB / 256;  // tile elements per thread
    {
        double arc[EPT], ass[EPT];
#pragma unroll
        for (int q = 0; q < EPT; ++q) {
            const int e = t + 256 * q, i = e / TB, j = e % TB;
            Lr[i][j] = upd ? A[(int64_t)(r0 + i) * nsp + kp + j] : 0.0;
            Lc[i][j] = upd ? A[(int64_t)(c0 + i) * nsp + kp + j] : 0.0;
            if (upd) {
                arc[q] = A[(int64_t)(r0 + i) * nsp + c0 + j];
                ass[q] = need_d ? A[(int64_t)(s0 + i) * nsp + s0 + j] : 0.0;
            } else {
                arc[q] = assembled_src(src, payload, ns, lambda, r0 + i, c0 + j);
                ass[q] = need_d ? assembled_src(src, payload, ns, lambda, s0 + i, s0 + j) : 0.0;
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < EPT; ++q) {
            const int e = t + 256 * q, i = e / TB, j = e % TB;
            double v = arc[q], w = ass[q];
            if (upd) {
                double a1 = 0, a2 = 0;
#pragma unroll 8
                for (int m = 0; m < TB; ++m) {
                    a1 += Lr[i][m] * Lc[j][m];
                    a2 += Lc[i][m] * Lc[j][m];
                }
                v -= a1;
                w -= a2;
            }
            if (!colblk) {
                A[(int64_t)(r0 + i) * nsp + c0 + j] = v;
            } else {
                Ct[i][j] = v;
                if (need_d) Cd[i][j] = w;
            }
        }
        if (!colblk) return;  // trailing tile: done
    }
    // column s: C_ss (Cd, or Ct in the diagonal block) is bitwise the same in
    // every column block -- same inputs, same operation order
    if (!upd && r == s)  // launch 0: the right-hand side of the rows past tile 0
        for (int i = TB + t; i < nsp; i += blockDim.x) bvec[i] = assembled_b_src(src, payload, ns, i);
    __syncthreads();
    if (t >= 64) return;
    const int lane = t;
    double (*Cdd)[TB + 1] = (r > s) ? Cd : Ct;
    if constexpr (TB == 16) {
        if (dpp) {  // every 16-lane row: C_ss row li in rw, C_rs row li in pw
            const int li = lane & 15;
            double rw[16], pw[16], dinv[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                rw[j] = Cdd[li][j];
                pw[j] = Ct[li][j];
            }
            chol_factor16(rw, pw, dinv, li, lane, bad);
            if (r == s) {
                double y = upd ? bvec[s0 + li] : assembled_b_src(src, payload, ns, li);
                if (upd) {
                    double acc = 0;
#pragma unroll
                    for (int m = 0; m < TB; ++m) acc += Lc[li][m] * bvec[kp + m];
                    y -= acc;
                }
#pragma unroll
                for (int j = 0; j < TB; ++j) {
                    const double yj = bcast16(y, j) * dinv[j];
                    if (li == j) y = yj;
                    if (li > j) y -= rw[j] * yj;
                }
                if (lane < TB) {
                    bvec[s0 + lane] = y;
                    double *Dn = D + (s & 1) * TB * TB;
#pragma unroll
                    for (int j = 0; j < TB; ++j) Dn[lane * TB + j] = j <= lane ? rw[j] : 0.0;
                }
                return;
            }
            wave_sync_lds();
            if (lane < TB)
#pragma unroll
                for (int j = 0; j < TB; ++j) Lr[lane][j] = pw[j];
            wave_sync_lds();
            for (int e = lane; e < TB * TB; e += 64)
                A[(int64_t)(r0 + e / TB) * nsp + s0 + e % TB] = Lr[e / TB][e % TB];
            for (int e = lane; e < TB * TB; e += 64)  // mirror into the upper triangle
                A[(int64_t)(s0 + e / TB) * nsp + r0 + e % TB] = Lr[e % TB][e / TB];
            return;
        }
    }
    const int li = lane < TB ? lane : TB - 1;
    // lanes [0, TB) hold the rows of C_ss; in a panel block lanes [TB, 2 TB)
    // hold the rows of C_rs.  The right-looking factor step (scale column k
    // by 1/L_kk, subtract L_jk times it from column j > k) is also the
    // right-looking forward substitution x L_ss^T = c of a panel row, so one
    // chain factors L_ss and forms L_rs = C_rs L_ss^-T
    const bool prow = r > s && lane >= TB && lane < 2 * TB;
    double rw[TB], dinv[TB];
#pragma unroll
    for (int j = 0; j < TB; ++j) rw[j] = prow ? Ct[lane - TB][j] : Cdd[li][j];
    chol_factor<TB>(rw, dinv, lane, bad);
    if (r == s) {
        double y = upd ? bvec[s0 + li] : assembled_b_src(src, payload, ns, li);
        if (upd) {
            double acc = 0;
#pragma unroll
            for (int m = 0; m < TB; ++m) acc += Lc[li][m] * bvec[kp + m];
            y -= acc;
        }
#pragma unroll
        for (int j = 0; j < TB; ++j) {
            const double yj = readlane_f64(y, j) * dinv[j];
            if (lane == j) y = yj;
            if (lane > j) y -= rw[j] * yj;
        }
        if (lane < TB) {
            bvec[s0 + lane] = y;
            double *Dn = D + (s & 1) * TB * TB;
#pragma unroll
            for (int j = 0; j < TB; ++j) Dn[lane * TB + j] = j <= lane ? rw[j] : 0.0;
        }
        return;
    }
    wave_sync_lds();
    if (prow)
#pragma unroll
        for (int j = 0; j < TB; ++j) Lr[lane - TB][j] = rw[j];
    wave_sync_lds();
    for (int e = lane; e < TB * TB; e += 64)
        A[(int64_t)(r0 + e / TB) * nsp + s0 + e % TB] = Lr[e / TB][e % TB];
    for (int e = lane; e < TB * TB; e += 64)  // mirror into the upper triangle
        A[(int64_t)(s0 + e / TB) * nsp + r0 + e % TB] = Lr[e % TB][e / TB];
}

// L^T x = y (y already in xg from the folded forward substitution), one
// workgroup, tile rows from the bottom, with the critical path on one wave:
//   wave 0 ("chain wave") solves tile k (16-deep readlane chain, pivots as
//   reciprocals off the chain), then forms tile k's contribution to the
//   rows of tile k-1 itself (acc, kept in registers), so the next solve
//   only waits for that and for one barrier;
//   waves 1.. ("row waves", row r = t - 64) apply tile k to the rows below
//   tile k-1 one barrier later, overlapped with wave 0's next solve.
// Every operand is fetched two steps ahead by the wave that uses it, with
// branch-free clamped loads, and the barriers order LDS only (lds_barrier),
// so the loads stay in flight across them.
constexpr int SOLVE_THREADS = 512;
constexpr int SOLVE_ROWS = SOLVE_THREADS - 64;  // rows owned by the row waves per pass
constexpr int SOLVE_MAX = 4096;

// One row segment of tile k's rows per lane and register: lanes [0, TB) hold
// the diagonal tile's column (q[m] = L[k0+m][k0+lane]), lanes [TB, 2 TB) the
// block left of it (q[m] = L[k0+m][k0-TB+lane-TB], tile k's contribution to
// tile k-1): one 2 TB-wide load per row instead of two loads, and the pivot
// L[k0+li][k0+li] is q[li] of lane li (no load of its own).
template <int TB>
struct ChainOps {
    double q[TB];
};

template <int TB>
__device__ __forceinline__ void chain_fetch(ChainOps<TB> &o, const double *__restrict__ A, int32_t nsp, int kt,
                                            int lane) {
    const int kb = kt >= 0 ? kt * TB : 0;
    const int col = lane < TB ? kb + lane : (lane < 2 * TB && kb >= TB) ? kb - 2 * TB + lane : kb;
    const double *row = A + (int64_t)kb * nsp + col;
#pragma unroll
    for (int m = 0; m < TB; ++m) o.q[m] = row[(int64_t)m * nsp];
}

template <int TB>
__device__ __forceinline__ void chain_step(ChainOps<TB> &o, const double *__restrict__ A, int32_t nsp, int kt,
                                           double *x, double &acc, int lane, int li) {
    const int k0 = kt * TB;
    double d = o.q[0];
#pragma unroll
    for (int m = 1; m < TB; ++m) d = (li == m) ? o.q[m] : d;
    const double rinv = 1.0 / d;  // off the chain
    double v = x[k0 + li] - acc;
#pragma unroll
    for (int j = TB - 1; j >= 0; --j) {
        const double vj = readlane_f64(v, j) * readlane_f64(rinv, j);
        if (lane == j) v = vj;
        if (lane < j) v -= o.q[j] * vj;
    }
    if (lane < TB) x[k0 + lane] = v;
    double a = 0;  // lanes [TB, 2 TB): L[k0+m][k0-TB+lane-TB] x[k0+m] for the row lane - TB of tile k-1
#pragma unroll
    for (int m = 0; m < TB; ++m) a += o.q[m] * readlane_f64(v, m);
    acc = __shfl(a, (lane + TB) & 63);
    chain_fetch<TB>(o, A, nsp, kt - 2, lane);
    lds_barrier();
}

template <int TB>
__device__ __forceinline__ void rows_fetch(double (&l)[TB], const double *__restrict__ A, int32_t nsp, int kt,
                                           int r) {
    const int kb = kt >= 0 ? kt * TB : 0, col = r < nsp ? r : 0;
#pragma unroll
    for (int m = 0; m < TB; ++m) l[m] = A[(int64_t)(kb + m) * nsp + col];
}

template <int TB>
__device__ __forceinline__ void rows_step(double (&l)[TB], const double *__restrict__ A, int32_t nsp, int kt,
                                          double *x, int r) {
    const int k0 = kt * TB, lim = k0 - TB;  // rows of tile k-1 get tile k from the chain wave
    lds_barrier();
    if (r < lim) {
        double sacc = 0;
#pragma unroll
        for (int m = 0; m < TB; ++m) sacc += l[m] * x[k0 + m];
        x[r] -= sacc;
    }
    for (int i = r + SOLVE_ROWS; i < lim; i += SOLVE_ROWS) {  // nsp > SOLVE_ROWS only
        double sacc = 0;
#pragma unroll 8
        for (int m = 0; m < TB; ++m) sacc += A[(int64_t)(k0 + m) * nsp + i] * x[k0 + m];
        x[i] -= sacc;
    }
    rows_fetch<TB>(l, A, nsp, kt - 2, r);
}

// trial cameras + camera part of the model decrease / norms, by one
// workgroup of THREADS threads (run at the end of k_chol_backsolve, which
// holds the camera step dc in LDS).  cam_out[0..3) = {model_c, |dc|^2, |t|^2}
template <int THREADS>
__device__ __forceinline__ void camera_trial(int32_t nc, const double *dc, const double *__restrict__ payload,
                                             int32_t ns, double lambda, const double *__restrict__ Rt,
                                             double *__restrict__ Rt_new, double *__restrict__ cam_out,
                                             double (*red)[THREADS]) {
    double m = 0, dn = 0, xn = 0;
    const double *diagU = payload + pay_vec_base(ns), *gc = diagU + ns;
    for (int c = threadIdx.x; c < nc; c += THREADS) {
        const double *d = dc + 6 * c;
        double dR[9];
        rotvec_to_R(d[0], d[1], d[2], dR);
        const double *R = Rt + 12 * c;
        double *Rn = Rt_new + 12 * c;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) Rn[3 * i + j] = dR[3 * i] * R[j] + dR[3 * i + 1] * R[3 + j] + dR[3 * i + 2] * R[6 + j];
        for (int i = 0; i < 3; ++i) {
            Rn[9 + i] = R[9 + i] + d[3 + i];
            xn += R[9 + i] * R[9 + i];
        }
        for (int i = 0; i < 6; ++i) {
            m += d[i] * (lambda * clampd(diagU[6 * c + i]) * d[i] - gc[6 * c + i]);
            dn += d[i] * d[i];
        }
    }
    red[0][threadIdx.x] = m; red[1][threadIdx.x] = dn; red[2][threadIdx.x] = xn;
    __syncthreads();
    for (int s = THREADS / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s)
            for (int k = 0; k < 3; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x < 3) cam_out[threadIdx.x] = red[threadIdx.x][0];
}

struct CamTrialArgs {  // k_chol_backsolve's epilogue (nc = 0: none)
    int32_t nc, ns;
    const double *payload, *lam, *Rt;
    double *Rt_new, *cam_out;
};

#include "gj_solve.hpp"   // the persistent block Gauss-Jordan solve (one launch), segment layout
#include "gjr_solve.hpp"  // ... and its row-distributed form (default since round 4)

template <int TB>
__global__ void __launch_bounds__(SOLVE_THREADS) k_chol_backsolve(double *__restrict__ A, int32_t nsp,
                                                                  double *__restrict__ xg,
                                                                  const double *__restrict__ Dlast, CamTrialArgs ct,
                                                                  const int *__restrict__ gate) {
    if (gate && !*gate) return;  // device-side LM control: iteration gated off
    __shared__ double x[SOLVE_MAX];
    const int t = threadIdx.x;
    const int nT = nsp / TB;
    for (int i = t; i < nsp; i += SOLVE_THREADS) x[i] = xg[i];
    if (t < 64) {  // chain wave
        const int lane = t, li = lane < TB ? lane : TB - 1;
        ChainOps<TB> oa, ob;
        chain_fetch<TB>(oa, A, nsp, nT - 1, lane);
        if (lane < TB)  // the last diagonal factor is still in the step kernel's scratch
#pragma unroll
            for (int m = 0; m < TB; ++m) oa.q[m] = Dlast[m * TB + lane];
        chain_fetch<TB>(ob, A, nsp, nT - 2, lane);
        double acc = 0;
        lds_barrier();  // x staged
        int kt = nT - 1;
        for (; kt >= 1; kt -= 2) {
            chain_step<TB>(oa, A, nsp, kt, x, acc, lane, li);
            chain_step<TB>(ob, A, nsp, kt - 1, x, acc, lane, li);
        }
        if (kt == 0) chain_step<TB>(oa, A, nsp, 0, x, acc, lane, li);
    } else {  // row waves
        const int r = t - 64;
        double la[TB], lb[TB];
        rows_fetch<TB>(la, A, nsp, nT - 1, r);
        rows_fetch<TB>(lb, A, nsp, nT - 2, r);
        lds_barrier();  // x staged
        int kt = nT - 1;
        for (; kt >= 1; kt -= 2) {
            rows_step<TB>(la, A, nsp, kt, x, r);
            rows_step<TB>(lb, A, nsp, kt - 1, x, r);
        }
        if (kt == 0) rows_step<TB>(la, A, nsp, 0, x, r);
    }
    lds_barrier();
    for (int i = t; i < nsp; i += SOLVE_THREADS) xg[i] = x[i];
    if (ct.nc > 0) {
        __shared__ double red[3][SOLVE_THREADS];
        camera_trial<SOLVE_THREADS>(ct.nc, x, ct.payload, ct.ns, *ct.lam, ct.Rt, ct.Rt_new, ct.cam_out, red);
    }
}

// ------------------------------------------------- device-side LM control
// The accept/reject decision and the damping update run on the device, so
// the host can enqueue many iterations without reading anything back; each
// kernel of an iteration is gated on run_lin / run_step (set by the previous
// decision), and the host polls `done` once per batch.
struct LMState {
    double lambda, nu, cost, cost0;
    int status, accepted, iters, done;
    int run_lin, run_step, accept_now, pad;
};

// The host's view of the LM state: k_lm_step of iteration it publishes its
// decision to pinned host memory (slot it % kHostRing, seq = it + 1 written
// last, system scope), so the host can stop enqueuing iterations once the
// solve is done without draining the stream (sfm_ba_solve).
struct HostLM {
    LMState st;
    int seq, pad[3];
};
constexpr int kHostRing = 4;

// create: the camera-major copies of (point, observation) gathered on the
// device from the uploaded point-major arrays; cm_pt holds the permutation
// (camera-major position -> observation) on entry, each thread reads its own
// entry before overwriting it
__global__ void __launch_bounds__(256) k_gather_cam_major(int64_t no, const int32_t *__restrict__ pt,
                                                         const double2 *__restrict__ obs, int32_t *cm_pt,
                                                         double2 *__restrict__ cm_obs) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= no) return;
    const int32_t o = cm_pt[k];
    cm_pt[k] = pt[o];
    cm_obs[k] = obs[o];
}

__global__ void k_lm_reset(LMState *lm, double lambda0, int *bad) {
    lm->lambda = lambda0; lm->nu = 2.0; lm->cost = 0.0; lm->cost0 = 0.0;
    lm->status = 4; lm->accepted = 0; lm->iters = 0; lm->done = 0;
    lm->run_lin = 1; lm->run_step = 1; lm->accept_now = 0;
    bad[0] = 0;
}

// the cost at x0; a non-finite one (a residual is NaN / inf: scipy's
// "Residuals are not finite in the initial point", least_squares.py:843-845)
// ends the solve before its first step with status 6
__global__ void k_lm_init(LMState *lm, const double *lin_cost) {
    const double c0 = *lin_cost;
    lm->cost = lm->cost0 = c0;
    if (!isfinite(c0)) {
        lm->status = 6;
        lm->done = 1;
        lm->run_step = 0;
        lm->run_lin = 0;
    }
}

// sfm_ba_solve's host logic, verbatim: Nielsen's lambda update on the gain
// ratio of the trial step; scal = [cost_trial, model_p, dn_p, xn_p, model_c,
// dn_c, xn_c].  Returns the new state from the old one (a pure function, so
// every block of k_lm_step computes the same decision).
__device__ __forceinline__ LMState lm_decide(LMState lm, const double *__restrict__ h, int bad, int max_iterations,
                                             int fixed, double ftol, double ptol, double lambda0) {
#pragma clang fp contract(off)
    if (lm.done) { lm.accept_now = 0; return lm; }
    const double cost = lm.cost;
    const double cost_new = h[0];
    const double model = 0.5 * (h[1] + h[4]);
    const double dnorm = sqrt(h[2] + h[5]), xnorm = sqrt(h[3] + h[6]);
    const double rho = (!bad && model > 0) ? (cost - cost_new) / model : -1.0;
    lm.iters += 1;
    int done = 0;
    if (!bad && isfinite(cost_new) && rho > 1e-3) {
        lm.accept_now = 1;
        const double dcost = cost - cost_new;
        lm.cost = cost_new;
        lm.accepted += 1;
        double f = 2.0 * rho - 1.0;
        f = 1.0 - f * f * f;
        lm.lambda *= (f > 1.0 / 3.0 ? f : 1.0 / 3.0);
        lm.nu = 2.0;
        lm.run_lin = 1;
        if (!fixed) {
            if (dcost < ftol * cost_new) { lm.status = 1; done = 1; }
            else if (dnorm < ptol * (xnorm + ptol)) { lm.status = 3; done = 1; }
        }
    } else {
        lm.accept_now = 0;
        lm.lambda *= lm.nu;
        lm.nu *= 2.0;
        lm.run_lin = 0;
        if (lm.lambda > 1e32) {
            if (!fixed) { lm.status = 5; done = 1; }
            else { lm.lambda = lambda0; lm.nu = 2.0; }
        }
    }
    if (lm.iters >= max_iterations) done = 1;
    lm.done = done;
    lm.run_step = !done;
    lm.run_lin = lm.run_lin && !done;
    return lm;
}

// gradient_tolerance (orc_ba_lm's stop after a linearisation: max |g| < gtol
// over the camera and point gradients, status 2, the iteration not counted).
// k_gtol_pack moves the point count and g_c into gbuf (all-reduced across
// ranks: a sum of counts and of the per-rank g_c partials); k_gtol_check
// stops the LM state of this iteration, which gates off the rest of it.
__global__ void k_gtol_pack(int32_t nc, const double *__restrict__ camlin, unsigned *__restrict__ nbig,
                            double *__restrict__ gbuf, const int *__restrict__ gate) {
    if (!*gate) return;
    for (int i = threadIdx.x; i < 6 * nc; i += blockDim.x) gbuf[1 + i] = camlin[CAMLIN * (i / 6) + 21 + i % 6];
    if (threadIdx.x == 0) {
        gbuf[0] = (double)*nbig;
        *nbig = 0u;
    }
}

__global__ void k_gtol_check(int32_t nc, double gtol, const double *__restrict__ gbuf, LMState *__restrict__ lm,
                             const int *__restrict__ gate) {
    if (!*gate) return;  // gate = lm->run_lin: only right after a linearisation
    __shared__ int big;
    if (threadIdx.x == 0) big = 0;
    __syncthreads();
    int b = 0;
    for (int i = threadIdx.x; i < 6 * nc; i += blockDim.x) b += fabs(gbuf[1 + i]) >= gtol;
    if (b) atomicAdd(&big, b);
    __syncthreads();
    if (threadIdx.x == 0 && big == 0 && gbuf[0] == 0.0) {
        lm->status = 2;
        lm->done = 1;
        lm->run_step = 0;
        lm->run_lin = 0;
    }
}

// One launch per LM iteration end: the decision (recomputed by every block
// from the old state lm_in, written by block 0 to lm_out -- the state is
// double-buffered by iteration parity, so no block reads what another
// writes), the accepted step's copy trial -> current, and the reset of the
// next iteration's not-positive-definite flag.
__global__ void k_lm_step(const LMState *__restrict__ lm_in, LMState *__restrict__ lm_out,
                          const double *__restrict__ h, const int *__restrict__ bad_in, int *__restrict__ bad_next,
                          int max_iterations, int fixed, double ftol, double ptol, double lambda0, int64_t np_,
                          int32_t nc, double *__restrict__ X, const double *__restrict__ X2, double *__restrict__ Rt,
                          const double *__restrict__ Rt2, HostLM *__restrict__ ring, int seq) {
    const LMState lm = lm_decide(*lm_in, h, *bad_in, max_iterations, fixed, ftol, ptol, lambda0);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *lm_out = lm;
        *bad_next = 0;
        if (ring) {  // publish to the host: the state, then (system-scope release) its sequence number
            HostLM *r = ring + (seq - 1) % kHostRing;
            r->st = lm;
            __hip_atomic_store(&r->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (!lm.accept_now) return;
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = i0; i < 3 * np_; i += st) X[i] = X2[i];  // bounded grid: cheap when nothing is copied
    for (int64_t i = i0; i < 12 * (int64_t)nc; i += st) Rt[i] = Rt2[i];
}

// Lanes per point for the grouped per-point kernels (1, 2, 4 or 8; an
// environment override is read once, for tuning).
// lanes per point of the point kernels (the measured choices; the round-2..5
// switches SFM_*_LANES, SFM_BACKSUB_THREADS / _BLOCKS are retired)
constexpr int LIN_CL_LANES = 2;  // k_linearize_cl (cameras in LDS)
constexpr int LIN_LANES = 4;     // k_linearize (global cameras: more nc than the LDS stage holds)
constexpr int BS_LANES = 2;      // k_backsub_trial

// Factor + forward solve (nT launches of k_chol_col) and backward solve of
// the padded reduced camera system with tiles of tb (16 or 32) columns; A, b
// on the device, D = 2 tb^2 scratch; nsp a multiple of tb.
template <int TB>
static int launch_cholesky_t(const double *payload, int32_t ns, const double *lam, double *A, int32_t nsp, double *b,
                             double *D, int *bad, hipStream_t s, const int *gate, const CamTrialArgs &ct,
                             const SlabSrc &src, int dpp) {
    const int nT = nsp / TB;
    for (int st = 0; st < nT; ++st) {
        const int T = nT - st;
        const int extra = st >= 1 || src.slab ? 1 : 0;  // bookkeeping / payload-vector workgroup
        hipLaunchKernelGGL(k_chol_col<TB>, dim3(T * (T + 1) / 2 + extra), dim3(256), 0, s, A, nsp, st, D, b, bad,
                           payload, ns, lam, gate, dpp, st == 0 ? src : SlabSrc{nullptr, nullptr, 0, 0},
                           const_cast<double *>(payload));
        SFM_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_chol_backsolve<TB>, dim3(1), dim3(SOLVE_THREADS), 0, s, A, nsp, b,
                       D + ((nT - 1) & 1) * TB * TB, ct, gate);
    SFM_HIP(hipGetLastError());
    return 0;
}

static int launch_cholesky(const double *payload, int32_t ns, const double *lam, double *A, int32_t nsp, double *b,
                           double *D, int *bad, hipStream_t s, int tb, const int *gate, const CamTrialArgs &ct,
                           const SlabSrc &src, int dpp) {
    return tb == 32 ? launch_cholesky_t<32>(payload, ns, lam, A, nsp, b, D, bad, s, gate, ct, src, dpp)
                    : launch_cholesky_t<16>(payload, ns, lam, A, nsp, b, D, bad, s, gate, ct, src, dpp);
}

// Cholesky tile width 16.  Measured on MI355X at ns = 300: 16 -> 0.167 ms,
// 32 -> 0.267 ms (round 2; the 32 variant and its switch are retired): each
// launch is bound by its column's serial factor + TRSM chain, which grows as
// tb^2, not by the launch count.
static int chol_tile(int64_t) { return 16; }

// S + lambda diag(clamp(diag U)) x = b from the Schur payload (assembled by the
// tiled Cholesky); x -> b.
//
// Measured alternatives, not kept (MI355X, ns = 300): a single-workgroup
// solve with the lower triangle resident in one CU's registers + LDS and fp64
// MFMA trailing updates ran 0.246 ms; a single-workgroup LEFT-looking solve
// (L tiles in L2, MFMA updates from a 4-deep load ring, explicit diagonal-tile
// inverses so the TRSM and both substitutions are MFMA / mat-vec work) ran
// 0.258 ms (updates 108 us, diagonal factor + inverse chains 78 us, back
// substitution 40 us) against 0.177 ms for this multi-launch path: one CU's
// fp64 MFMA rate and its serial per-tile chains bound both.
static int launch_reduced_solve(int32_t ns, int32_t nsp, const double *payload, const double *lam, double *A,
                                double *b, double *D, int *bad, hipStream_t s, int tb, const int *gate,
                                const CamTrialArgs &ct, const SlabSrc &src = SlabSrc{nullptr, nullptr, 0, 0},
                                int dpp = 1) {
    return launch_cholesky(payload, ns, lam, A, nsp, b, D, bad, s, tb, gate, ct, src, dpp);
}

// Persistent Gauss-Jordan solve (gj_solve.hpp): the workgroup layout for
// nT tiles.  cb = 0: the grid would not fit one workgroup per CU, so the
// multi-launch Cholesky above runs instead (SFM_SOLVE=chol forces it).
struct GjPlan {
    int cb = 0, nseg = 0, ncb = 0;
    int grid() const { return cb ? ncb * nseg : 0; }
};
static GjPlan gj_plan(int nT, int ncu) {
    GjPlan g;
    if (const char *e = std::getenv("SFM_SOLVE"))
        if (std::strcmp(e, "chol") == 0) return g;
    if (nT > gj::NTMAX) return g;
    const int nseg = (nT + gj::SR - 1) / gj::SR;
    for (int cb : {gj::SR, 2 * gj::SR}) {
        const int ncb = (nT + cb - 1) / cb;
        if (ncb * nseg <= ncu) {
            g.cb = cb;
            g.nseg = nseg;
            g.ncb = ncb;
            break;
        }
    }
    return g;
}
static int device_cus(int device) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n <= 0) n = 256;
    return n;
}

// device buffers of one solver instance: panels, L / y copies, flags (zeroed
// once; epochs only grow), abort word, arrival counter
struct GjBufs {
    double *G = nullptr, *L = nullptr, *Y = nullptr;
    int *flag = nullptr, *err = nullptr;
    unsigned *arrive = nullptr;
    static size_t doubles(int nT, int nseg) {
        return (size_t)nT * nT * 16 * 16 + (size_t)nT * nseg * (256 + 16);
    }
    static size_t ints(int nT, int nseg) { return (size_t)nT * nseg + 64; }
    void carve(double *d, int *i, int nT, int nseg) {
        G = d;
        L = G + (size_t)nT * nT * 16 * 16;
        Y = L + (size_t)nT * nseg * 256;
        flag = i;
        err = i + (size_t)nT * nseg;
        arrive = reinterpret_cast<unsigned *>(i + (size_t)nT * nseg + 32);
    }
};

// SFM_SWEEP_STAMPS=1: k_schur_sweep records s_memrealtime stamps per
// (workgroup, event, wave) into a process-wide device buffer (sfm_sweep_debug
// reads it): event 0 start, 1 the first chunk staged (stagers) / the
// cameras in LDS (groups), 2 + i chunk i done, SW_STAMP_EV - 1 the end
static long long *g_sw_dbg = nullptr;
static const size_t g_sw_dbg_n = (size_t)SW_STAMP_WG * SW_STAMP_EV * (SW_THREADS / 64);
static long long *sw_dbg_ptr() {
    static const bool on = std::getenv("SFM_SWEEP_STAMPS") && std::atoi(std::getenv("SFM_SWEEP_STAMPS")) != 0;
    if (!on) return nullptr;
    if (!g_sw_dbg) {
        if (hipMalloc(&g_sw_dbg, g_sw_dbg_n * sizeof(long long)) != hipSuccess) return g_sw_dbg = nullptr;
        (void)hipMemset(g_sw_dbg, 0, g_sw_dbg_n * sizeof(long long));
    }
    return g_sw_dbg;
}
extern "C" int sfm_sweep_debug(long long *out, int64_t n) {
    SFM_CHECK_ARG(out, "null pointer");
    if (!g_sw_dbg) return 0;
    SFM_HIP(hipDeviceSynchronize());
    SFM_HIP(hipMemcpy(out, g_sw_dbg, std::min<size_t>((size_t)n, g_sw_dbg_n) * sizeof(long long), hipMemcpyDeviceToHost));
    return 0;
}

// SFM_GJ_DEBUG=1: the persistent solve records s_memrealtime stamps per
// (workgroup, panel) into a process-wide device buffer (sfm_gj_debug reads it)
static long long *g_gj_dbg = nullptr;
static size_t g_gj_dbg_n = 0;
static long long *gj_dbg_ptr() {
    static const bool on = std::getenv("SFM_GJ_DEBUG") && std::atoi(std::getenv("SFM_GJ_DEBUG")) != 0;
    if (!on) return nullptr;
    if (!g_gj_dbg) {
        g_gj_dbg_n = (size_t)256 * (gj::NTMAX + 1) * 16;
        if (hipMalloc(&g_gj_dbg, g_gj_dbg_n * sizeof(long long)) != hipSuccess) return g_gj_dbg = nullptr;
        (void)hipMemset(g_gj_dbg, 0, g_gj_dbg_n * sizeof(long long));
    }
    return g_gj_dbg;
}
extern "C" int sfm_gj_debug(long long *out, int64_t n) {
    SFM_CHECK_ARG(out, "null pointer");
    if (!g_gj_dbg) return 0;
    SFM_HIP(hipDeviceSynchronize());
    SFM_HIP(hipMemcpy(out, g_gj_dbg, std::min<size_t>((size_t)n, g_gj_dbg_n) * sizeof(long long), hipMemcpyDeviceToHost));
    return 0;
}

static int launch_gj(const GjPlan &g, int nT, int32_t ns, const double *payload, const double *lam, const GjBufs &b, int epoch, double *x, int *bad, const int *gate,
                     const CamTrialArgs &ct, hipStream_t s) {
    gj::Args a;
    a.payload = payload;
    a.ns = ns;
    a.nT = nT;
    a.cb = g.cb;
    a.nseg = g.nseg;
    a.lam = lam;
    a.gate = gate;
    a.Gp = b.G;
    a.Lp = b.L;
    a.Yp = b.Y;
    a.flag = b.flag;
    a.epoch = epoch;
    a.x = x;
    a.bad = bad;
    a.err = b.err;
    a.arrive = b.arrive;
    a.ct = ct;
    a.dbg = gj_dbg_ptr();
    hipLaunchKernelGGL(gj::k_gj_solve, dim3(g.grid()), dim3(gj::THREADS), 0, s, a);
    SFM_HIP(hipGetLastError());
    return 0;
}

// Row-distributed persistent solve (gjr_solve.hpp): one workgroup per tile
// row, all resident at once (every wait is bounded, and the host checks the
// occupancy against the grid).  tpw = 0: not applicable, the segment layout
// above (or the Cholesky) runs instead; SFM_SOLVE=gjseg / chol force those.
struct GjrPlan {
    int nT = 0, tpw = 0;
    bool ok() const { return tpw > 0; }
};
template <int TR, int TLS>
static bool gjr_resident(int nT, int ncu) {
    static int nb = -1;  // resident workgroups per CU (queried once per instantiation)
    if (nb < 0) {
        nb = 0;
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(&gjr::k_gjr_solve<TR, TLS>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, gjr::DYN_LDS) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, gjr::k_gjr_solve<TR, TLS>, gjr::THREADS, gjr::DYN_LDS) !=
                hipSuccess)
            nb = 0;
        (void)hipGetLastError();
    }
    return nb >= 1 && nT <= nb * ncu;
}
static GjrPlan gjr_plan(int nT, int ncu) {
    GjrPlan g;
    if (const char *e = std::getenv("SFM_SOLVE"))
        if (std::strcmp(e, "chol") == 0 || std::strcmp(e, "gjseg") == 0) return g;
    // tile slots per U wave: 4 or TREG in registers (up to 28 / 77 tile
    // rows), past that TREG_L + TLDS_L (the latter in LDS: up to gjr::NTMAX = 128)
    if (nT < 1 || nT > gjr::NTMAX || nT > ncu) return g;
    const int tpw = nT <= 4 * gjr::NUW ? 4 : nT <= gjr::TREG * gjr::NUW ? gjr::TREG : gjr::TREG_L + gjr::TLDS_L;
    const bool res = tpw == 4 ? gjr_resident<4, 0>(nT, ncu)
                   : tpw == gjr::TREG ? gjr_resident<gjr::TREG, 0>(nT, ncu)
                                      : gjr_resident<gjr::TREG_L, gjr::TLDS_L>(nT, ncu);
    if (!res) return g;
    g.nT = nT;
    g.tpw = tpw;
    return g;
}
// granule records (zeroed once; tags only grow) and the err / arrival words
struct GjrBufs {
    gjr::u64 *P = nullptr, *G = nullptr;
    double *Gd = nullptr;
    unsigned *Gf = nullptr;
    int *err = nullptr;
    unsigned *arrive = nullptr;
    static size_t words(int nT) {
        const size_t t = (size_t)nT * nT;
        return ((size_t)2 * nT * gjr::PBYTES + t * gjr::GBYTES + t * gjr::GDBYTES) / 8 + (t + 1) / 2;
    }
    static constexpr size_t ints = 64;
    void carve(gjr::u64 *w, int *i, int nT) {
        const size_t t = (size_t)nT * nT;
        P = w;
        G = P + (size_t)2 * nT * gjr::PBYTES / 8;
        Gd = reinterpret_cast<double *>(G + t * gjr::GBYTES / 8);
        Gf = reinterpret_cast<unsigned *>(Gd + t * gjr::GDBYTES / 8);
        err = i;
        arrive = reinterpret_cast<unsigned *>(i + 32);
    }
};
static int launch_gjr(const GjrPlan &g, int32_t ns, const double *payload, const double *lam, const GjrBufs &b,
                      unsigned tag, double *x, int *bad, const int *gate, const CamTrialArgs &ct, hipStream_t s,
                      const SlabSrc &src = SlabSrc{nullptr, nullptr, 0, 0, {}, nullptr}) {
    gjr::Args a;
    a.src = src;
    a.payload = payload;
    a.ns = ns;
    a.nT = g.nT;
    a.lam = lam;
    a.gate = gate;
    a.P = b.P;
    a.G = b.G;
    a.Gd = b.Gd;
    a.Gf = b.Gf;
    a.tag = tag;
    a.x = x;
    a.bad = bad;
    a.err = b.err;
    a.arrive = b.arrive;
    a.ct = ct;
    a.dbg = gj_dbg_ptr();
    switch (g.tpw) {
    case 4: hipLaunchKernelGGL((gjr::k_gjr_solve<4, 0>), dim3(g.nT), dim3(gjr::THREADS), gjr::DYN_LDS, s, a); break;
    case gjr::TREG:
        hipLaunchKernelGGL((gjr::k_gjr_solve<gjr::TREG, 0>), dim3(g.nT), dim3(gjr::THREADS), gjr::DYN_LDS, s, a);
        break;
    default:
        hipLaunchKernelGGL((gjr::k_gjr_solve<gjr::TREG_L, gjr::TLDS_L>), dim3(g.nT), dim3(gjr::THREADS), gjr::DYN_LDS,
                           s, a);
        break;
    }
    SFM_HIP(hipGetLastError());
    return 0;
}

// partial[block][4] = {trial cost, model_p, |dp|^2, |X|^2}
constexpr int BS_PRE = 6;  // observations per lane prefetched by k_backsub_trial
// CL: the cameras (Rt 12 | Rt_new 12 | dc 6 doubles, 240 B each) staged in
// LDS once per workgroup, so the per-observation camera reads (30 doubles,
// 240 B) are LDS reads instead of L1/L2 gathers
// 30 doubles (60 dwords) already put the 16-B camera reads on all 16 bank
// positions of a ds_read_b128 group; an odd stride (31, 33) lost the 16-B
// alignment and ran 0.051 -> 0.060 ms at cfg5 (round 5).  What conflicts
// remain (0.53 of the LDS cycles) are random cameras of a lane group
// sharing a position, inherent to the gather.
#ifndef SFM_BS_CAM_STRIDE
#define SFM_BS_CAM_STRIDE 30
#endif
constexpr int BS_CAM = SFM_BS_CAM_STRIDE;
static_assert(BS_CAM >= 30, "Rt 12 | Rt_new 12 | dc 6");
constexpr int BS_CAM_LDS_MAX = 64 * 1024;
template <int G, bool CL, int NT = PT_THREADS>
__global__ void __launch_bounds__(NT) k_backsub_trial(int64_t np_, int32_t nc, const int32_t *__restrict__ pstart,
                                                              const int32_t *__restrict__ cam,
                                                              const double2 *__restrict__ obs, Kmat Km,
                                                              const double *__restrict__ Vg,
                                                              const double *__restrict__ Lq,
                                                              const double *__restrict__ dc, const double *__restrict__ lam,
                                                              const double *__restrict__ Rt,
                                                              const double *__restrict__ Rt_new,
                                                              const double *__restrict__ X,
                                                              double *__restrict__ X_new, double *__restrict__ partial,
                                                              unsigned *__restrict__ counter, double *__restrict__ out,
                                                              const int *__restrict__ gate) {
    if (gate && !*gate) return;  // device-side LM control: iteration gated off
    const double lambda = *lam;
    double K[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) K[i] = Km.k[i];
    double acc[4] = {0, 0, 0, 0};
    // grid-stride over points (a bounded grid keeps the per-block partial
    // store + arrival count, and the last block's sum, small), software
    // pipelined: the next point's pstart, X, V / g and L are loaded while this
    // point is worked on, so an iteration waits for one round of loads (its
    // observations') instead of three in a row (pstart, then the
    // observations, then V / g and L)
    struct Pre {
        int32_t o0, o1;
        double x[3], g[3], dg[3], l[6];
    };
    auto fetch = [&](int64_t gtn, Pre &P) {
        const int64_t p = gtn / G;
        const bool live = p < np_;
        P.o0 = live ? pstart[p] : 0;
        P.o1 = live ? pstart[p + 1] : 0;
        const double *vg = Vg + 9 * (live ? p : 0);
        const double *l = Lq + 9 * (live ? p : 0);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            P.x[i] = live ? X[3 * p + i] : 0.0;
            P.g[i] = vg[6 + i];
        }
        P.dg[0] = vg[0];
        P.dg[1] = vg[3];
        P.dg[2] = vg[5];
#pragma unroll
        for (int i = 0; i < 6; ++i) P.l[i] = l[i];
    };
    const int64_t stride = (int64_t)gridDim.x * NT;
    Pre cur;
    fetch((int64_t)blockIdx.x * NT + threadIdx.x, cur);
    extern __shared__ __attribute__((aligned(16))) double bs_cam[];
    if constexpr (CL) {
        auto stage = [&](const double *__restrict__ src, int w, int off) {
            const int n = w * nc;
#pragma unroll 4
            for (int i = threadIdx.x; i < n; i += NT) {
                const int c = i / w;
                bs_cam[BS_CAM * c + off + (i - w * c)] = src[i];
            }
        };
        stage(Rt, 12, 0);
        stage(Rt_new, 12, 12);
        stage(dc, 6, 24);
        __syncthreads();
    }
    const double *const cRt = CL ? bs_cam : Rt, *const cRn = CL ? bs_cam + 12 : Rt_new,
                        *const cdc = CL ? bs_cam + 24 : dc;
    constexpr int RS = CL ? BS_CAM : 12, DS = CL ? BS_CAM : 6;
    for (int64_t gt = (int64_t)blockIdx.x * NT + threadIdx.x; gt / G < np_; gt += stride) {
    const int64_t p = gt / G;  // G lanes per point, striding over its observations
    const int sub = (int)(gt % G);
    const bool live = p < np_;
    const int32_t o0 = cur.o0, o1 = cur.o1;
    // the lane's first BS_PRE observations (camera index and measurement)
    // loaded up front, for both passes: their loads are in flight together
    // instead of one round trip per observation and pass
    int32_t cpre[BS_PRE];
    double2 opre[BS_PRE];
#pragma unroll
    for (int k = 0; k < BS_PRE; ++k) {
        const int32_t o = o0 + sub + k * G;
        cpre[k] = o < o1 ? cam[o] : 0;
        opre[k] = o < o1 ? obs[o] : make_double2(0.0, 0.0);
    }
    Pre nxt;
    fetch(gt + stride, nxt);
    // W^T dc = Jp^T (Jc dc) = R^T A^T (A (dtheta x p + dt)), summed over the point's observations
    double wt[3] = {0, 0, 0};
    const double x[3] = {cur.x[0], cur.x[1], cur.x[2]};
    auto wt_add = [&](int32_t c) {
        const double *d = cdc + DS * c;
        const double *R = cRt + RS * c;
        double A[2][3], q[3];
        obs_Ap(R, x, K, A, q);
        const double v0 = d[1] * q[2] - d[2] * q[1] + d[3];
        const double v1 = d[2] * q[0] - d[0] * q[2] + d[4];
        const double v2 = d[0] * q[1] - d[1] * q[0] + d[5];
        const double s0 = A[0][0] * v0 + A[0][1] * v1 + A[0][2] * v2;
        const double s1 = A[1][0] * v0 + A[1][1] * v1 + A[1][2] * v2;
        double w[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) w[i] = A[0][i] * s0 + A[1][i] * s1;
#pragma unroll
        for (int i = 0; i < 3; ++i) wt[i] += R[i] * w[0] + R[3 + i] * w[1] + R[6 + i] * w[2];
    };
#pragma unroll
    for (int k = 0; k < BS_PRE; ++k)
        if (o0 + sub + k * G < o1) wt_add(cpre[k]);
    for (int32_t o = o0 + sub + BS_PRE * G; o < o1; o += G) wt_add(cam[o]);
#pragma unroll
    for (int i = 0; i < 3; ++i) wt[i] = group_sum<G>(wt[i]);
    if (live) {
        const double rhs[3] = {-cur.g[0] - wt[0], -cur.g[1] - wt[1], -cur.g[2] - wt[2]};
        const double *l = cur.l;  // L upper: 00 01 02 11 12 22
        // y = L^T rhs ; dp = L y  (every lane of the group, identically)
        const double y0 = l[0] * rhs[0];
        const double y1 = l[1] * rhs[0] + l[3] * rhs[1];
        const double y2 = l[2] * rhs[0] + l[4] * rhs[1] + l[5] * rhs[2];
        const double dp[3] = {l[0] * y0 + l[1] * y1 + l[2] * y2, l[3] * y1 + l[4] * y2, l[5] * y2};
        double xn[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) xn[i] = x[i] + dp[i];
        if (sub == 0) {
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                X_new[3 * p + i] = xn[i];
                acc[1] += dp[i] * (lambda * clampd(cur.dg[i]) * dp[i] - cur.g[i]);
                acc[2] += dp[i] * dp[i];
                acc[3] += x[i] * x[i];
            }
        }
#pragma unroll
        for (int k = 0; k < BS_PRE; ++k)
            if (o0 + sub + k * G < o1) acc[0] += obs_cost(cRn + RS * cpre[k], xn, K, opre[k]);
        for (int32_t o = o0 + sub + BS_PRE * G; o < o1; o += G) acc[0] += obs_cost(cRn + RS * cam[o], xn, K, obs[o]);
    }
    cur = nxt;
    }
    grid_sum_last<4, NT>(acc, partial, counter, out);
}

// ---------------------------------------------------------------- host math
static void h_rotvec_to_R(const double *w, double *R) {
    double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    double th = std::sqrt(th2), a, b;
    if (th < 1e-6) {
        a = 1.0 - th2 / 6.0 + th2 * th2 / 120.0;
        b = 0.5 - th2 / 24.0 + th2 * th2 / 720.0;
    } else {
        a = std::sin(th) / th;
        b = (1.0 - std::cos(th)) / th2;
    }
    double x = w[0], y = w[1], z = w[2];
    R[0] = 1.0 - b * (y * y + z * z); R[1] = -a * z + b * x * y;       R[2] = a * y + b * x * z;
    R[3] = a * z + b * x * y;         R[4] = 1.0 - b * (x * x + z * z); R[5] = -a * x + b * y * z;
    R[6] = -a * y + b * x * z;        R[7] = a * x + b * y * z;         R[8] = 1.0 - b * (x * x + y * y);
}

// scipy Rotation.from_matrix(R).as_rotvec() (quaternion route, w >= 0)
static void h_R_to_rotvec(const double *R, double *w) {
    double tr = R[0] + R[4] + R[8], q[4];
    if (tr > R[0] && tr > R[4] && tr > R[8]) {
        q[3] = 1.0 + tr;
        q[0] = R[7] - R[5]; q[1] = R[2] - R[6]; q[2] = R[3] - R[1];
    } else {
        int i = (R[0] >= R[4] && R[0] >= R[8]) ? 0 : (R[4] >= R[8] ? 1 : 2);
        int j = (i + 1) % 3, k = (j + 1) % 3;
        q[i] = 1.0 - tr + 2.0 * R[i * 4];
        q[j] = R[j * 3 + i] + R[i * 3 + j];
        q[k] = R[k * 3 + i] + R[i * 3 + k];
        q[3] = R[k * 3 + j] - R[j * 3 + k];
    }
    double nq = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (double &v : q) v /= nq;
    if (q[3] < 0)
        for (double &v : q) v = -v;
    double vn = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
    double ang = 2.0 * std::atan2(vn, q[3]);
    double sc = ang <= 1e-3 ? 2.0 + ang * ang / 12.0 + 7.0 * ang * ang * ang * ang / 2880.0 : ang / std::sin(ang / 2.0);
    w[0] = sc * q[0]; w[1] = sc * q[1]; w[2] = sc * q[2];
}

}  // namespace sfm

using namespace sfm;

// ------------------------------------------------------ Schur sweep plan
// Host-side construction of k_schur_sweep's static structure (DESIGN.md
// section 4): ranges, chunks, specs (camera-row sets with their lane
// groups) and, per (chunk, spec), fixed-capacity regions so that the
// kernel computes every staging address without a dependent load: the
// staged record indices, the pair list (a slot << 16 | b offset in chunk,
// grouped by lane group, point order) and the header (group offsets, n0, n1,
// chunk obs0).
struct SweepPlan {
    int32_t nrange = 0, nspec = 0, nbd = 0, buf_slots = 0, pair_cap = 0, hdr_cap = 0, list_cap = 0, nchunk = 0;
    int32_t split_S = 0, split_w0 = 0, split_n = 0, split_gmax = 0;  // the dispatch tail's split (SweepSplit)
    std::vector<int32_t> rchunk, goff, nload, list, hdr, spec_cam, split_of;
    std::vector<int32_t> spec_row;  // per spec: (camera, j0, j1) of rows 0 and 1 (camera -1: none)
    std::vector<int32_t> cut;       // chunk first points, then np
    bool dev_lists = false;         // list / pairs / hdr are generated on the device (k_plan_lists)
    std::vector<SweepGroup> groups;
    std::vector<int16_t> lanegrp;
    std::vector<uint16_t> pairs;
    std::vector<int2> blkij;
    size_t lds_bytes() const {
        return (size_t)2 * (buf_slots * SLOT_D * 8 + (size_t)pair_cap * 2 + (size_t)hdr_cap * 4) + 24 * sizeof(double) +
               16 * sizeof(int);  // + the chunk hand-off counters (SW_SYNC)
    }
};

static int env_int(const char *name, int dflt) {
    const char *v = std::getenv(name);
    return v ? std::atoi(v) : dflt;
}

// k_backsub_trial's grid when the cameras fit its LDS stage: the resident
// workgroup count for that LDS size (every workgroup starts at once), at most
// the partial-sum slots; 0 selects the global-camera kernel
static int backsub_cl_blocks(int32_t nc, int ncu, int max_blocks) {
    constexpr int nt = 256;
    if (env_int("SFM_BACKSUB_CAM_LDS", 1) == 0) return 0;
    const size_t lds = (size_t)8 * BS_CAM * nc;
    if (nc < 1 || lds > (size_t)BS_CAM_LDS_MAX) return 0;
    int nb = 0;
    auto occ = [&](auto kern) {
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, nt, lds) != hipSuccess)
            nb = 0;
    };
    occ(k_backsub_trial<BS_LANES, true, 256>);  // the instantiation the launch picks
    (void)hipGetLastError();
    if (nb < 1) return 0;
    return std::max(1, std::min(nb * ncu, max_blocks));
}

// k_linearize_cl's grid: the resident workgroups for the cameras' LDS size
// (0: more than 64 KB of cameras, or SFM_LINEARIZE_CAM_LDS=0)
static int linearize_cl_blocks(int32_t nc, int ncu, int max_blocks) {
    if (env_int("SFM_LINEARIZE_CAM_LDS", 1) == 0) return 0;
    const size_t lds = (size_t)8 * LIN_CAM * nc;
    if (nc < 1 || lds > (size_t)BS_CAM_LDS_MAX) return 0;
    int nb = 0;
    auto occ = [&](auto kern) {
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, LIN_CL_THREADS, lds) != hipSuccess)
            nb = 0;
    };
    occ(k_linearize_cl<LIN_CL_LANES>);
    (void)hipGetLastError();
    if (nb < 1) return 0;
    return std::max(1, std::min(nb * ncu, max_blocks));
}

// camera items for camera_lin_wg from workgroup cuts (camera-major
// observation offsets, ascending, first 0, last n_obs): every item is the
// part of one camera inside one workgroup's range.  by_wg: workgroup g takes
// the items of range g (wg_first); otherwise one item per workgroup.
struct CamPlan {
    std::vector<PairItem> items;
    std::vector<BlockInfo> blocks;
    std::vector<int32_t> wg_first;
};

static void plan_camera_items(int nc, const std::vector<int32_t> &cstart, const std::vector<int32_t> &cuts, bool by_wg,
                              CamPlan &P) {
    std::vector<std::vector<int32_t>> cam_items(nc);
    P.wg_first.push_back(0);
    for (size_t g = 0; g + 1 < cuts.size(); ++g) {
        const int32_t a = cuts[g], b = cuts[g + 1];
        for (int c = 0; c < nc; ++c) {
            const int32_t k0 = std::max(a, cstart[c]), k1 = std::min(b, cstart[c + 1]);
            if (k0 >= k1) continue;
            cam_items[c].push_back((int32_t)P.items.size());
            P.items.push_back({c, k0, k1, 1});
        }
        if (by_wg) P.wg_first.push_back((int32_t)P.items.size());
    }
    if (!by_wg)
        for (size_t i = 1; i <= P.items.size(); ++i) P.wg_first.push_back((int32_t)i);
    // items are in camera-major order already (cuts ascend), so each camera's
    // items are contiguous
    for (int c = 0; c < nc; ++c)
        if (!cam_items[c].empty())
            P.blocks.push_back({c, c, cam_items[c].front(), cam_items[c].back() + 1});
}

static int32_t dense_blk(int nc, int i, int j) { return i * nc - i * (i - 1) / 2 + (j - i); }

// ------------------------------------------------- the sweep plan on the device (round 5)
// plan_sweep's passes over every point's observation pairs (the chunk
// statistics that size the LDS, the per-chunk pair counts, and the (chunk,
// spec) slot and pair lists) run as kernels over the uploaded point-major
// COO and the camera-major points, producing the host planner's arrays
// exactly (same traversal orders; SFM_PLAN_HOST=1 keeps the host passes and
// the plan digest test compares the two).  The allocation of lanes to the
// groups (a greedy over the chunk counts) stays on the host.
__device__ __forceinline__ int32_t dense_blk_d(int nc, int i, int j) { return i * nc - i * (i - 1) / 2 + (j - i); }
__device__ __forceinline__ int32_t lower_bound_d(const int32_t *__restrict__ a, int32_t lo, int32_t hi, int32_t v) {
    while (lo < hi) {
        const int32_t m = lo + ((hi - lo) >> 1);
        if (a[m] < v) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// create's CSR on the device (round 5; SFM_PLAN_HOST=1 keeps the host's):
// pstart from the point-sorted observations, cstart from the camera-sorted
// keys of the stable radix sort (csr_sort.hip: the permutation, in point
// order within a camera), the co-observation block counts (a <= b within a
// point, the diagonal included) with the duplicate-camera check
namespace sfm {
int cam_major_sort(void *temp, size_t &temp_bytes, const int32_t *cam, uint32_t *keys_out, int32_t *perm_out,
                   int64_t no, int32_t nc, hipStream_t s);
}
__global__ void __launch_bounds__(256) k_csr_pstart(int64_t no, int64_t np_, const int32_t *__restrict__ pt,
                                                    int32_t *__restrict__ pstart) {
    const int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (o > no) return;
    if (o == no) {  // the points after the last observed one
        for (int64_t i = no ? (int64_t)pt[no - 1] + 1 : 0; i <= np_; ++i) pstart[i] = (int32_t)no;
        return;
    }
    const int64_t lo = o == 0 ? 0 : (int64_t)pt[o - 1] + 1;
    for (int64_t i = lo; i <= pt[o]; ++i) pstart[i] = (int32_t)o;
}
__global__ void __launch_bounds__(256) k_csr_cstart(int64_t no, int32_t nc, const uint32_t *__restrict__ keys,
                                                    int32_t *__restrict__ cstart) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c > nc) return;
    int64_t lo = 0, hi = no;
    while (lo < hi) {
        const int64_t m = lo + ((hi - lo) >> 1);
        if (keys[m] < (uint32_t)c) lo = m + 1;
        else hi = m;
    }
    cstart[c] = (int32_t)lo;
}
__global__ void __launch_bounds__(256) k_csr_cnt(int64_t no, int32_t nc, const int32_t *__restrict__ pstart,
                                                 const int32_t *__restrict__ pt, const int32_t *__restrict__ cam,
                                                 uint32_t *__restrict__ cnt, uint32_t *__restrict__ dup) {
    const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (a >= no) return;
    const int ca = cam[a];
    const int32_t e = pstart[pt[a] + 1];
    atomicAdd(&cnt[(size_t)ca * nc + ca], 1u);
    for (int32_t b = (int32_t)a + 1; b < e; ++b) {
        const int cb = cam[b];
        if (cb == ca) atomicOr(dup, 1u);
        atomicAdd(&cnt[ca < cb ? (size_t)ca * nc + cb : (size_t)cb * nc + ca], 1u);
    }
}

// the same counts through a per-workgroup LDS histogram of the upper
// triangle (nc (nc + 1) / 2 counters, up to 160 KB), flushed with one global
// atomic per nonzero counter and workgroup: the global form's atomics all
// land on those few addresses (cfg4: 5.5 M atomics on 1,275 counters, 1.0 ms;
// cfg5 1.06 ms).  A bounded grid (CSR_CNT_WGS) keeps the flush small.
constexpr int CSR_CNT_WGS = 128;
constexpr int CNT_THREADS = 1024;  // the counting kernels: 16 waves a CU hide their dependent loads (256: 4)
__global__ void __launch_bounds__(CNT_THREADS) k_csr_cnt_lds(int64_t no, int32_t nc, const int32_t *__restrict__ pstart,
                                                     const int32_t *__restrict__ pt, const int32_t *__restrict__ cam,
                                                     uint32_t *__restrict__ cnt, uint32_t *__restrict__ dup) {
    extern __shared__ uint32_t csr_hist[];
    const int ntri = nc * (nc + 1) / 2;
    for (int i = threadIdx.x; i < ntri; i += CNT_THREADS) csr_hist[i] = 0;
    __syncthreads();
    bool twice = false;
    for (int64_t a = (int64_t)blockIdx.x * CNT_THREADS + threadIdx.x; a < no; a += (int64_t)gridDim.x * CNT_THREADS) {
        const int ca = cam[a];
        const int32_t e = pstart[pt[a] + 1];
        atomicAdd(&csr_hist[dense_blk_d(nc, ca, ca)], 1u);
        // the point's later cameras four loads at a time (one wait per four,
        // not one per camera: the loop is load-latency bound)
        for (int32_t b0 = (int32_t)a + 1; b0 < e; b0 += 4) {
            int cbv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) cbv[u] = b0 + u < e ? cam[b0 + u] : -1;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int cb = cbv[u];
                if (cb < 0) continue;
                twice |= cb == ca;
                atomicAdd(&csr_hist[ca < cb ? dense_blk_d(nc, ca, cb) : dense_blk_d(nc, cb, ca)], 1u);
            }
        }
    }
    if (twice) atomicOr(dup, 1u);
    __syncthreads();
    for (int r = 0; r < nc; ++r)
        for (int c = r + (int)threadIdx.x; c < nc; c += CNT_THREADS) {
            const uint32_t v = csr_hist[dense_blk_d(nc, r, c)];
            if (v) atomicAdd(&cnt[(size_t)r * nc + c], v);
        }
}

// the pinned staging buffer of create's uploads (grown, never shrunk; one
// user at a time)
struct PinnedStage {
    std::mutex mu;
    void *p = nullptr;
    size_t bytes = 0;
    // a second stream per device, used only under mu: the coordinates (and a
    // one-shot problem's points) go up on it while the CSR, the camera sort
    // and the planner run on the problem's stream, which waits on `ev` only
    // before the first kernel that reads them
    struct Aux {
        hipStream_t s = nullptr;
        hipEvent_t ev = nullptr;
    } aux[64];
    Aux *aux_for(int dev) {
        if (dev < 0 || dev >= 64) return nullptr;
        Aux &a = aux[dev];
        if (!a.s && hipStreamCreateWithFlags(&a.s, hipStreamNonBlocking) != hipSuccess) {
            (void)hipGetLastError();
            a.s = nullptr;
            return nullptr;
        }
        if (!a.ev && hipEventCreateWithFlags(&a.ev, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            a.ev = nullptr;
            return nullptr;
        }
        return &a;
    }
};
static PinnedStage &pinned_stage() {
    static PinnedStage *st = new PinnedStage();
    return *st;
}

// chunk q of a trial cut: the observations of points [cut[q], cend[q]); its
// largest staged-slot count (the observations of one spec's cameras) and
// pair count (off-diagonal pairs of one spec's blocks) -> out[2q], out[2q+1]
__global__ void __launch_bounds__(256) k_plan_chunkmax(int32_t nc, int32_t nspec, const int32_t *__restrict__ pstart,
                                                       const int32_t *__restrict__ pt, const int32_t *__restrict__ cam,
                                                       const int32_t *__restrict__ cut, const int32_t *__restrict__ cend,
                                                       const int32_t *__restrict__ spec_of,
                                                       const int32_t *__restrict__ spec_cam, int32_t *__restrict__ out) {
    extern __shared__ int32_t plan_sh[];
    int32_t *cc = plan_sh, *cp = plan_sh + nc, *mx = plan_sh + nc + nspec;
    const int q = blockIdx.x;
    for (int i = threadIdx.x; i < nc + nspec + 2; i += blockDim.x) plan_sh[i] = 0;
    __syncthreads();
    const int32_t o0 = pstart[cut[q]], o1 = pstart[cend[q]];
    for (int32_t a = o0 + (int32_t)threadIdx.x; a < o1; a += blockDim.x) {
        const int ca = cam[a], pnt = pt[a];
        atomicAdd(&cc[ca], 1);
        const int32_t e = pstart[pnt + 1];
        for (int32_t b0 = pstart[pnt]; b0 < e; b0 += 8) {  // eight loads, then one wait (k_plan_counts_lds)
            int cbv[8], spv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) cbv[u] = b0 + u < e ? cam[b0 + u] : -1;
#pragma unroll
            for (int u = 0; u < 8; ++u) spv[u] = cbv[u] > ca ? spec_of[ca * nc + cbv[u]] : -1;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (spv[u] >= 0) atomicAdd(&cp[spv[u]], 1);
        }
    }
    __syncthreads();
    for (int w = threadIdx.x; w < nspec; w += blockDim.x) {
        const int c0 = spec_cam[2 * w], c1 = spec_cam[2 * w + 1];
        atomicMax(&mx[0], cc[c0] + (c1 >= 0 ? cc[c1] : 0));
        atomicMax(&mx[1], cp[w]);
    }
    __syncthreads();
    if (threadIdx.x < 2) out[2 * q + threadIdx.x] = mx[threadIdx.x];
}

// The same statistics with each chunk split over gridDim.y workgroups
// (one workgroup per chunk walked up to 65,535 observations and their pairs
// on 256 threads: cfg5 0.49 ms per trial cut, cfg4 0.29, two to four trials
// per create): partial counts in LDS, added into cnt[q][nc + nspec]
// (zeroed), then k_plan_chunkmax_fin takes the two maxima per chunk.
__global__ void __launch_bounds__(256) k_plan_chunkcnt(int32_t nc, int32_t nspec, const int32_t *__restrict__ pstart,
                                                       const int32_t *__restrict__ pt, const int32_t *__restrict__ cam,
                                                       const int32_t *__restrict__ cut, const int32_t *__restrict__ cend,
                                                       const int32_t *__restrict__ spec_of, uint32_t *__restrict__ cnt) {
    extern __shared__ int32_t plan_sh[];
    int32_t *cc = plan_sh, *cp = plan_sh + nc;
    const int q = blockIdx.x;
    for (int i = threadIdx.x; i < nc + nspec; i += blockDim.x) plan_sh[i] = 0;
    __syncthreads();
    const int32_t o0 = pstart[cut[q]], o1 = pstart[cend[q]], len = o1 - o0;
    const int32_t a0 = o0 + (int32_t)((int64_t)len * blockIdx.y / gridDim.y);
    const int32_t a1 = o0 + (int32_t)((int64_t)len * (blockIdx.y + 1) / gridDim.y);
    for (int32_t a = a0 + (int32_t)threadIdx.x; a < a1; a += blockDim.x) {
        const int ca = cam[a], pnt = pt[a];
        atomicAdd(&cc[ca], 1);
        const int32_t e = pstart[pnt + 1];
        for (int32_t b0 = pstart[pnt]; b0 < e; b0 += 8) {  // eight loads, then one wait (k_plan_counts_lds)
            int cbv[8], spv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) cbv[u] = b0 + u < e ? cam[b0 + u] : -1;
#pragma unroll
            for (int u = 0; u < 8; ++u) spv[u] = cbv[u] > ca ? spec_of[ca * nc + cbv[u]] : -1;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (spv[u] >= 0) atomicAdd(&cp[spv[u]], 1);
        }
    }
    __syncthreads();
    uint32_t *row = cnt + (size_t)q * (nc + nspec);
    for (int i = threadIdx.x; i < nc + nspec; i += blockDim.x)
        if (plan_sh[i]) atomicAdd(&row[i], (uint32_t)plan_sh[i]);
}
__global__ void __launch_bounds__(256) k_plan_chunkmax_fin(int32_t nc, int32_t nspec, const uint32_t *__restrict__ cnt,
                                                           const int32_t *__restrict__ spec_cam,
                                                           int32_t *__restrict__ out) {
    __shared__ int32_t mx[2];
    if (threadIdx.x < 2) mx[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t *cc = cnt + (size_t)blockIdx.x * (nc + nspec), *cp = cc + nc;
    for (int w = threadIdx.x; w < nspec; w += blockDim.x) {
        const int c0 = spec_cam[2 * w], c1 = spec_cam[2 * w + 1];
        atomicMax(&mx[0], (int32_t)(cc[c0] + (c1 >= 0 ? cc[c1] : 0)));
        atomicMax(&mx[1], (int32_t)cp[w]);
    }
    __syncthreads();
    if (threadIdx.x < 2) out[2 * blockIdx.x + threadIdx.x] = mx[threadIdx.x];
}

// per chunk (cut: the chunks' first points, nchunk + 1 entries, the last
// np_): pairs per camera block, bq[blk][q], and observations per camera,
// cq[c][q] (32-bit counters; k_plan_narrow makes the host planner's uint16)
__global__ void __launch_bounds__(256) k_plan_counts(int64_t no, int32_t nc, int32_t nchunk,
                                                     const int32_t *__restrict__ pstart, const int32_t *__restrict__ pt,
                                                     const int32_t *__restrict__ cam, const int32_t *__restrict__ cut,
                                                     uint32_t *__restrict__ bq, uint32_t *__restrict__ cq) {
    const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (a >= no) return;
    const int32_t pnt = pt[a], ca = cam[a];
    const int q = (int)lower_bound_d(cut, 0, nchunk + 1, pnt + 1) - 1;  // last chunk starting at or before pnt
    atomicAdd(&cq[(size_t)ca * nchunk + q], 1u);
    for (int32_t b = pstart[pnt]; b < pstart[pnt + 1]; ++b) {
        const int cb = cam[b];
        if (cb > ca) atomicAdd(&bq[(size_t)dense_blk_d(nc, ca, cb) * nchunk + q], 1u);
    }
}
// k_plan_counts with a chunk's observations split over gridDim.y
// workgroups: the counts in an LDS histogram (blocks, then cameras), added
// into bq / cq once per nonzero counter and workgroup.  The global form's
// atomics of a chunk land on its nbd block counters (cfg4: 1,275 of them,
// 0.35 ms; cfg5 0.80 ms).
__global__ void __launch_bounds__(CNT_THREADS) k_plan_counts_lds(int32_t nc, int32_t nchunk, const int32_t *__restrict__ pstart,
                                                         const int32_t *__restrict__ pt, const int32_t *__restrict__ cam,
                                                         const int32_t *__restrict__ cut, uint32_t *__restrict__ bq,
                                                         uint32_t *__restrict__ cq) {
    extern __shared__ uint32_t pc_hist[];
    const int nbd = nc * (nc + 1) / 2;
    uint32_t *hb = pc_hist, *hc = pc_hist + nbd;
    for (int i = threadIdx.x; i < nbd + nc; i += CNT_THREADS) pc_hist[i] = 0;
    __syncthreads();
    const int q = blockIdx.x;
    const int32_t o0 = pstart[cut[q]], o1 = pstart[cut[q + 1]], len = o1 - o0;
    const int32_t a0 = o0 + (int32_t)((int64_t)len * blockIdx.y / gridDim.y);
    const int32_t a1 = o0 + (int32_t)((int64_t)len * (blockIdx.y + 1) / gridDim.y);
    for (int32_t a = a0 + (int32_t)threadIdx.x; a < a1; a += CNT_THREADS) {
        const int32_t pnt = pt[a], ca = cam[a];
        atomicAdd(&hc[ca], 1u);
        const int32_t e = pstart[pnt + 1];
        for (int32_t b0 = pstart[pnt]; b0 < e; b0 += 8) {  // eight loads, then one wait
            int cbv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) cbv[u] = b0 + u < e ? cam[b0 + u] : -1;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (cbv[u] > ca) atomicAdd(&hb[dense_blk_d(nc, ca, cbv[u])], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nbd + nc; i += CNT_THREADS) {
        const uint32_t v = pc_hist[i];
        if (v) atomicAdd(i < nbd ? &bq[(size_t)i * nchunk + q] : &cq[(size_t)(i - nbd) * nchunk + q], v);
    }
}
__global__ void __launch_bounds__(256) k_plan_narrow(int64_t n, const uint32_t *__restrict__ in, uint16_t *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = (uint16_t)in[i];
}

// one workgroup per (chunk q, spec w), qw = q * nspec + w: the slot list
// (count, then every slot's point | row << 31, padded with the chunk's first
// observed point), the group header (pair offsets from bq, total, n0, n1,
// first observation) and the pairs, every group's in slot order (the host's
// traversal: spec row, the camera's observations in point order, at most one
// pair per point and block).  Slots' column hits go through an LDS bit mask
// (slot x the row's block columns); one thread per group then walks the
// slots in order.
constexpr int PLAN_THREADS = 256;
__global__ void __launch_bounds__(PLAN_THREADS) k_plan_lists(
    int32_t nchunk, int32_t nspec, int32_t np_, int32_t mw, const int32_t *__restrict__ cut,
    const int32_t *__restrict__ pstart, const int32_t *__restrict__ pt, const int32_t *__restrict__ cam,
    const int32_t *__restrict__ cstart, const int32_t *__restrict__ cm_pt, const int32_t *__restrict__ spec_row,
    const int32_t *__restrict__ goff, const SweepGroup *__restrict__ groups, const uint16_t *__restrict__ bq,
    int32_t list_cap, int32_t pair_cap, int32_t hdr_cap, int32_t *__restrict__ list, uint16_t *__restrict__ pairs,
    int32_t *__restrict__ hdr) {
    extern __shared__ int32_t plan_sh[];
    int32_t *off = plan_sh;                                             // hdr_cap group offsets
    uint32_t *mask = reinterpret_cast<uint32_t *>(plan_sh + hdr_cap);   // [slot][mw] column hits
    __shared__ int32_t lo[2], nr[2], tot;
    const int q = blockIdx.x / nspec, w = blockIdx.x % nspec;
    const size_t qw = (size_t)q * nspec + w;
    const int32_t P0 = cut[q], P1 = cut[q + 1];
    const int32_t *sr = spec_row + 6 * w;  // rows: (camera, j0, j1) x 2, camera -1 = none
    if (threadIdx.x < 2) {
        const int c = sr[3 * threadIdx.x];
        int32_t l = 0, h = 0;
        if (c >= 0) {
            l = lower_bound_d(cm_pt, cstart[c], cstart[c + 1], P0);
            h = lower_bound_d(cm_pt, l, cstart[c + 1], P1);
        }
        lo[threadIdx.x] = l;
        nr[threadIdx.x] = h - l;
    }
    __syncthreads();
    const int32_t n0 = nr[0], n1 = nr[1], ns = n0 + n1;
    const int32_t o0 = pstart[P0];
    // the slot list
    int32_t *lst = list + qw * list_cap;
    const int32_t pad = pt[o0];
    for (int i = threadIdx.x; i < list_cap; i += PLAN_THREADS) {
        int32_t v = pad;
        if (i == 0) v = ns;
        else if (i - 1 < n0) v = cm_pt[lo[0] + i - 1];
        else if (i - 1 < ns) v = (int32_t)((uint32_t)cm_pt[lo[1] + i - 1 - n0] | 0x80000000u);
        lst[i] = v;
    }
    // every slot's block-column hits (the point's cameras cj > c, j0 <= cj < j1)
    for (int s = threadIdx.x; s < ns; s += PLAN_THREADS) {
        const int rr = s < n0 ? 0 : 1;
        const int c = sr[3 * rr], j0 = sr[3 * rr + 1], j1 = sr[3 * rr + 2];
        const int32_t pnt = cm_pt[lo[rr] + (rr ? s - n0 : s)];
        uint32_t *m = mask + (size_t)s * mw;
        for (int k = 0; k < mw; ++k) m[k] = 0u;
        const int32_t e = pstart[pnt + 1];
        for (int32_t b0 = pstart[pnt]; b0 < e; b0 += 8) {  // eight loads, then one wait
            int cjv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) cjv[u] = b0 + u < e ? cam[b0 + u] : -1;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int cj = cjv[u];
                if (cj <= c || cj < j0 || cj >= j1) continue;
                m[(cj - j0) >> 5] |= 1u << ((cj - j0) & 31);
            }
        }
    }
    // the group offsets: one wave, 64 groups a step (inclusive scan by shuffles)
    const int g0 = goff[w], ng = goff[w + 1] - g0;
    const int lane = threadIdx.x & 63;
    if (threadIdx.x < 64) {
        int32_t run = 0;
        for (int base = 0; base < ng; base += 64) {
            const int g = base + lane;
            int32_t v = 0;
            if (g < ng) {
                const SweepGroup G = groups[g0 + g];
                v = (G.flags & 1) ? 0 : (int32_t)bq[(size_t)G.blk * nchunk + q];
            }
            int32_t x = v;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int32_t y = __shfl_up(x, d);
                if (lane >= d) x += y;
            }
            if (g < ng) off[g] = run + x - v;
            run += __shfl(x, 63);
        }
        if (lane == 0) tot = run;
    }
    __syncthreads();
    int32_t *hd = hdr + qw * hdr_cap;
    for (int i = threadIdx.x; i < hdr_cap; i += PLAN_THREADS) {
        int32_t v = 0;
        if (i < ng) v = off[i];
        else if (i == ng) v = tot;
        else if (i == ng + 1) v = n0;
        else if (i == ng + 2) v = n1;
        else if (i == ng + 3) v = o0;
        hd[i] = v;
    }
    // the pairs: a thread per group walks the slots of its row in order
    uint16_t *pp = pairs + qw * pair_cap;
    for (int i = tot + (int)threadIdx.x; i < pair_cap; i += PLAN_THREADS) pp[i] = 0;
    for (int g = threadIdx.x; g < ng; g += PLAN_THREADS) {
        const SweepGroup G = groups[g0 + g];
        if (G.flags & 1) continue;
        const int rr = (G.flags & 2) ? 1 : 0;
        const int col = G.cam_b - sr[3 * rr + 1], wd = col >> 5;
        const uint32_t bit = 1u << (col & 31);
        const int s0 = rr ? n0 : 0, s1 = rr ? ns : n0;
        int32_t k = off[g];
        for (int s = s0; s < s1; ++s)
            if (mask[(size_t)s * mw + wd] & bit) pp[k++] = (uint16_t)s;
    }
}


// trips a slot of a group makes through its chunk share: ceil(P / s)
static inline int sweep_trips(int P, int s) { return (P + s - 1) / s; }

// slots (lanes / LPP) of the spec's off-diagonal groups, `budget` in all,
// from the exact per-chunk pair counts P[g][q] (the plan is static: the
// same points and cameras every LM iteration).  A chunk ends at a barrier,
// so its time is the largest trip count of any group in it (the diagonal
// groups' dtrip[q] included); the objective is the sum over chunks.  Greedy
// on the separable surrogate sum_g sum_q trips^6 (a soft max), one slot at a
// time to the group whose trips drop the surrogate most; the proportional
// split (slots ~ total pairs) is kept when it scores better on the true
// objective.  Returns the objective of the allocation chosen.
static int64_t sweep_alloc(const std::vector<std::vector<uint16_t>> &P, const std::vector<int> &dtrip, int budget,
                           std::vector<int> &slots) {
    const int ng = (int)P.size(), nq = (int)dtrip.size();
    // sum over chunks of the largest trip count; group-major, the division
    // ceil(P / s) as a multiply by the 32-bit reciprocal (exact: (P + s - 1)
    // s < 2^32 for 16-bit P and s <= SW_THREADS), so the chunk loop vectorises
    std::vector<int> mx(nq);
    auto objective = [&](const std::vector<int> &sl) {
        mx.assign(dtrip.begin(), dtrip.end());
        for (int g = 0; g < ng; ++g) {
            const uint64_t s = (uint64_t)sl[g], m = (((uint64_t)1 << 32) + s - 1) / s;
            const uint16_t *pg = P[g].data();
            for (int q = 0; q < nq; ++q) mx[q] = std::max(mx[q], (int)(((uint64_t)pg[q] + s - 1) * m >> 32));
        }
        int64_t f = 0;
        for (int v : mx) f += v;
        return f;
    };
    // proportional split (the round-2/3 planner): floor shares, then the
    // remaining slots to the group with the most pairs per slot
    std::vector<int64_t> tot(ng, 0);
    int64_t all = 0;
    for (int g = 0; g < ng; ++g) {
        for (int q = 0; q < nq; ++q) tot[g] += P[g][q];
        all += tot[g];
    }
    std::vector<int> prop(ng, 1);
    int sum = 0;
    for (int g = 0; g < ng; ++g) {
        prop[g] = std::max(1, (int)(all > 0 ? (double)tot[g] / all * budget : 1.0));
        sum += prop[g];
    }
    while (sum > budget) {
        auto it = std::max_element(prop.begin(), prop.end());
        *it -= 1;
        sum -= 1;
    }
    while (sum < budget && ng) {
        int best = 0;
        for (int g = 1; g < ng; ++g)
            if (tot[g] * prop[best] > tot[best] * prop[g]) best = g;
        prop[best] += 1;
        sum += 1;
    }
    // greedy on the soft max.  A group's gain depends on its per-chunk pair
    // counts only through their histogram: the distinct counts (descending)
    // with their multiplicities, so a gain costs the distinct counts above s
    // instead of every chunk (cfg5: ~100 chunks, ~15 distinct counts; the
    // greedy was 2 of the 9 ms of the cfg5 create)
    auto pw = [](int t) { const double x = t; return x * x * x * x * x * x; };
    // flat: group g's (count, multiplicity) pairs at hist[hoff[g], hoff[g + 1])
    std::vector<std::pair<int, int>> hist;
    std::vector<int> hoff(ng + 1, 0);
    hist.reserve((size_t)ng * 16);
    {
        std::vector<int> c;  // a counting pass (a sort per group cost more than the greedy)
        for (int g = 0; g < ng; ++g) {
            const uint16_t *pg = P[g].data();
            int top = 0;
            for (int q = 0; q < nq; ++q) top = std::max(top, (int)pg[q]);
            c.assign(top + 1, 0);
            for (int q = 0; q < nq; ++q) c[pg[q]]++;
            for (int v = top; v > 1; --v)  // counts <= 1 never gain
                if (c[v]) hist.push_back({v, c[v]});
            hoff[g + 1] = (int)hist.size();
        }
    }
    auto gain = [&](int g, int s) {
        double d = 0;
        for (int k = hoff[g]; k < hoff[g + 1]; ++k) {
            const auto &hm = hist[k];
            if (hm.first <= s) break;  // one trip at s and s + 1 from here down
            d += hm.second * (pw(sweep_trips(hm.first, s)) - pw(sweep_trips(hm.first, s + 1)));
        }
        return d;
    };
    // a heap of (gain, -group): the largest gain, the lowest group on ties
    // (max_element's choice); only the chosen group's gain changes
    std::vector<int> gr(ng, 1);
    std::vector<std::pair<double, int>> heap(ng);
    for (int g = 0; g < ng; ++g) heap[g] = {gain(g, 1), -g};
    std::make_heap(heap.begin(), heap.end());
    for (int used = ng; used < budget; ++used) {
        std::pop_heap(heap.begin(), heap.end());
        const int g = -heap.back().second;
        gr[g] += 1;
        heap.back() = {gain(g, gr[g]), -g};
        std::push_heap(heap.begin(), heap.end());
    }
    const int64_t fp = objective(prop), fg = ng <= budget ? objective(gr) : INT64_MAX;
    slots = fg < fp ? gr : prop;
    return std::min(fp, fg);
}

// SFM_CREATE_TIMING=1: host phase times of sfm_ba_create on stderr
struct PhaseTimer {
    bool on = env_int("SFM_CREATE_TIMING", 0) != 0;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    void tick(const char *what) {
        if (!on) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[create] %-14s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t0).count());
        t0 = t;
    }
};

// Device blocks of destroyed problems (and of the planner's scratch), kept
// for the next create on the same device.  The drop-in creates and destroys
// a problem per call; hipMalloc, and hipFree (which synchronises the
// device), cost ~6 ms of every cfg5 call.  A block is reused for a request
// of up to 1.5x less; the cache holds at most 16 GiB (oldest blocks go
// first) and is emptied for a device whose hipMalloc fails.  Every buffer a
// kernel reads before writing is memset or uploaded in create, so a reused
// block's old contents are never read: SFM_POOL_POISON=1 fills reused blocks
// with 0xFF (the tests' check of that claim).
struct DevBlockCache {
    struct Blk {
        int dev;
        size_t bytes;
        void *p;
    };
    std::mutex mu;
    std::deque<Blk> blks;  // oldest first
    size_t held = 0;
    static constexpr size_t kCap = (size_t)16 << 30;
};
static DevBlockCache &dev_cache() {
    static auto *c = new DevBlockCache();
    return *c;
}
static constexpr bool pool_on() { return true; }  // (the SFM_POOL=0 switch is retired, round 6)
static void pool_trim(int dev) {  // every cached block of dev back to the driver
    DevBlockCache &c = dev_cache();
    std::lock_guard<std::mutex> lk(c.mu);
    for (auto it = c.blks.begin(); it != c.blks.end();) {
        if (it->dev == dev) {
            (void)hipFree(it->p);
            c.held -= it->bytes;
            it = c.blks.erase(it);
        } else {
            ++it;
        }
    }
}
// a block of at least `bytes` on the current device dev; *got = its size
static hipError_t pool_malloc(void **out, size_t bytes, int dev, size_t *got) {
    *got = bytes;
    if (pool_on()) {
        DevBlockCache &c = dev_cache();
        std::unique_lock<std::mutex> lk(c.mu);
        auto best = c.blks.end();
        for (auto it = c.blks.begin(); it != c.blks.end(); ++it)
            if (it->dev == dev && it->bytes >= bytes && it->bytes <= bytes + bytes / 2 &&
                (best == c.blks.end() || it->bytes < best->bytes))
                best = it;
        if (best != c.blks.end()) {
            *out = best->p;
            *got = best->bytes;
            c.held -= best->bytes;
            c.blks.erase(best);
            lk.unlock();
            if (env_int("SFM_POOL_POISON", 0)) {
                (void)hipMemset(*out, 0xFF, *got);
                (void)hipDeviceSynchronize();
            }
            return hipSuccess;
        }
    }
    hipError_t e = hipMalloc(out, bytes);
    if (e != hipSuccess && pool_on()) {
        (void)hipGetLastError();
        pool_trim(dev);
        e = hipMalloc(out, bytes);
    }
    return e;
}
// back to the cache; the caller has synchronised every stream that used it
static void pool_free(void *p, size_t bytes, int dev) {
    if (!p) return;
    if (!pool_on()) {
        (void)hipFree(p);
        return;
    }
    DevBlockCache &c = dev_cache();
    std::lock_guard<std::mutex> lk(c.mu);
    c.blks.push_back({dev, bytes, p});
    c.held += bytes;
    while (c.held > DevBlockCache::kCap && !c.blks.empty()) {
        (void)hipFree(c.blks.front().p);
        c.held -= c.blks.front().bytes;
        c.blks.pop_front();
    }
}

// the device side of the planner: the uploaded COO and a stream; scratch
// buffers live until the object goes (released on every return path, once
// the stream has drained)
struct DevPlan {
    hipStream_t s = nullptr;
    int dev = 0;
    const int32_t *pstart = nullptr, *pt = nullptr, *cam = nullptr;
    int64_t no = 0;
    std::vector<std::pair<void *, size_t>> bufs;
    int err = 0;
    ~DevPlan() {
        if (!bufs.empty() && s) (void)hipStreamSynchronize(s);
        for (auto &b : bufs) pool_free(b.first, b.second, dev);
    }
    template <class T>
    T *scratch(size_t n) {
        void *q = nullptr;
        size_t got;
        if (pool_malloc(&q, std::max<size_t>(n, 1) * sizeof(T), dev, &got) != hipSuccess) {
            err = SFM_ERR_NOMEM;
            return nullptr;
        }
        bufs.push_back({q, got});
        return static_cast<T *>(q);
    }
    bool ok(hipError_t e) {
        if (e != hipSuccess && !err) err = SFM_ERR_HIP;
        return !err;
    }
    uint16_t *d_bq = nullptr;   // bq [blk][q] (uint16), kept for k_plan_lists
    int32_t *d_cut = nullptr;   // the final cut (nchunk + 1)
};

static void plan_sweep(int nc, int64_t np_, int64_t no, const int32_t *cam, const int32_t *pt,
                       const std::vector<int32_t> &pstart, const std::vector<int64_t> &cnt, int lpp, int ncu,
                       bool allow_split, SweepPlan &P, DevPlan *dev = nullptr) {
    PhaseTimer pt_;
    P.nbd = nc * (nc + 1) / 2;
    P.blkij.resize(P.nbd);
    for (int i = 0; i < nc; ++i)
        for (int j = i; j < nc; ++j) P.blkij[dense_blk(nc, i, j)] = make_int2(i, j);
    // specs: rows (camera c, blocks j in [j0, j1)); cameras i and nc-1-i
    // share a spec so that every spec carries about the same pair work
    struct Row { int c, j0, j1; };
    std::vector<std::vector<Row>> specs;
    if (nc - 1 <= SW_MAX_COLS) {
        for (int i = 0; i < nc / 2; ++i) specs.push_back({{i, i, nc}, {nc - 1 - i, nc - 1 - i, nc}});
        if (nc % 2) specs.push_back({{nc / 2, nc / 2, nc}});
    } else {  // long rows: split into parts of <= SW_MAX_COLS blocks
        for (int i = 0; i < nc; ++i)
            for (int j0 = i; j0 < nc; j0 += SW_MAX_COLS) specs.push_back({{i, j0, std::min(nc, j0 + SW_MAX_COLS)}});
    }
    P.nspec = (int32_t)specs.size();
    for (auto &sp : specs) {  // the a-side cameras of every spec (rows 0 and 1)
        P.spec_cam.push_back(sp[0].c);
        P.spec_cam.push_back(sp.size() > 1 ? sp[1].c : -1);
        for (size_t rr = 0; rr < 2; ++rr) {
            const bool has = rr < sp.size();
            P.spec_row.push_back(has ? sp[rr].c : -1);
            P.spec_row.push_back(has ? sp[rr].j0 : 0);
            P.spec_row.push_back(has ? sp[rr].j1 : 0);
        }
    }
    // block (i <= j) -> spec that owns it
    std::vector<int32_t> spec_of((size_t)nc * nc, -1);
    for (int w = 0; w < P.nspec; ++w)
        for (size_t rr = 0; rr < specs[w].size(); ++rr)
            for (int j = specs[w][rr].j0; j < specs[w][rr].j1; ++j) spec_of[(size_t)specs[w][rr].c * nc + j] = w;
    // per spec: the diagonal groups (their lanes are the loader waves; power
    // of two sizes) and the off-diagonal groups with their pair budget
    struct G0 { int blk, flags, slots; double work; int key, cam_b, row_cam; };
    std::vector<std::vector<G0>> sgd(P.nspec), sg(P.nspec);
    std::vector<int> sGd(P.nspec), sbudget(P.nspec);
    int max_ng = 0;
    for (int w = 0; w < P.nspec; ++w) {
        auto &gd = sgd[w], &g = sg[w];
        for (size_t rr = 0; rr < specs[w].size(); ++rr) {
            const Row &R = specs[w][rr];
            for (int j = R.j0; j < R.j1; ++j) {
                const double work = (double)cnt[(size_t)R.c * nc + j];
                G0 x = {dense_blk(nc, R.c, j), (j == R.c ? 1 : 0) | (rr == 1 ? 2 : 0), 1, work,
                        (int)(rr * nc + (j - R.j0)), j, R.c};
                (j == R.c ? gd : g).push_back(x);
            }
        }
        const int nd = (int)gd.size(), noff = (int)g.size();
        int Gd = 64, nload = 1, budget = 0;
        for (; Gd >= 2; Gd /= 2) {
            nload = std::max(1, (nd * Gd + 63) / 64);
            budget = (SW_THREADS - 64 * nload - 64 * SW_STAGE_WAVES) / lpp;  // pair slots
            if (noff <= budget) break;
        }
        sGd[w] = Gd;
        sbudget[w] = budget;
        P.nload.push_back(nload);
        max_ng = std::max(max_ng, nd + noff);
    }
    P.hdr_cap = (max_ng + 4 + 63) / 64 * 64;
    // ranges of equal observation count; chunks small enough that two
    // (chunk, spec) buffers fit the LDS and the chunk's records an XCD's L2
    // 8 ranges (one per XCD): every workgroup pays a prologue (the first
    // chunk staged, ~7 us) and the end-of-range reduction, so fewer, longer
    // workgroups win even with a partial last pass over the CUs (cfg5, 100
    // specs: 16 ranges 0.539 ms, 8 ranges 0.505 ms; cfg4: 0.145 -> 0.161 ms at 16)
    // Round 5, late: one round of workgroups, as many as fit -- the largest
    // range count with nspec x nrange <= the CU count (one sweep workgroup a
    // CU: ~150 KB of LDS).  Measured, cfg5 (100 specs) sweep + finish, rank
    // 0's shard of N (a round-5 one-off script, same box):
    //   N = 1: 8 ranges 0.330 ms, 4 0.324, 2 0.306, 1 0.557, 16 0.387
    //   N = 2: 8 0.208, 4 0.182, 2 0.168, 1 0.288
    //   N = 4: 8 0.139, 4 0.114, 2 0.102, 1 0.155
    //   N = 8: 8 0.115, 4 0.083, 2 0.075, 1 0.095
    // so 2 at every N (200 workgroups); cfg4 (25 specs) keeps 8 (its 16 had
    // measured 0.161 against 0.145 ms).  More specs than CUs: the round-4
    // model (rounds x (13.3 us + 4.7 ns per pair / workgroups), fractional
    // rounds for 8, whose dispatch tail is split).  SFM_SWEEP_RANGES
    // overrides (a multiple of 8, or 1, 2, 4).
    {
        int best = 0;
        for (int nr : {8, 4, 2, 1})
            if ((int64_t)P.nspec * nr <= ncu) {
                best = nr;
                break;
            }
        if (!best) {
            const double pairs = (double)std::accumulate(cnt.begin(), cnt.end(), int64_t(0)) - (double)no;
            double tbest = 1e300;
            best = NXCD;
            for (int nr : {8, 4, 2, 1}) {
                const double wgs = (double)P.nspec * nr;
                const double rounds = nr >= NXCD ? std::max(1.0, wgs / ncu) : std::ceil(wgs / ncu);
                const double t = rounds * (13.3 + pairs * 4.7e-3 / wgs);
                if (t < tbest * 0.97) {  // a smaller count only for a clear win
                    tbest = t;
                    best = nr;
                }
            }
        }
        const int e = env_int("SFM_SWEEP_RANGES", 0);
        P.nrange = e >= NXCD ? e / NXCD * NXCD : (e == 1 || e == 2 || e == 4) ? e : best;
    }
    // chunks as large as the LDS allows (every chunk boundary is a barrier
    // and an imbalance point): from the 16-bit cap down, scaled by the
    // overshoot until the largest (chunk, spec) fits
    int chunk_obs = 65535;
    std::vector<int64_t> cut;  // chunk first points
    int32_t *d_spec_of = nullptr, *d_scam = nullptr;  // device planner: the spec tables
    for (;;) {
        // the cuts follow from the observation counts alone; the chunks'
        // staged slots and pair counts (the LDS bound) are then counted per
        // chunk on host threads
        P.rchunk.assign(1, 0);
        cut.clear();
        std::vector<int64_t> cend;  // chunk end points
        bool ok = true;
        int64_t pcur = 0;
        for (int r = 0; r < P.nrange && ok; ++r) {
            const int64_t oend = no * (r + 1) / P.nrange;
            while (pcur < np_ && pstart[pcur] < oend) {  // one chunk
                // the chunk's end: the first point at or after oend, or the
                // first whose observations would overflow chunk_obs (the
                // first point always goes in); pstart is monotone, so two
                // binary searches instead of a walk over the points
                const int32_t o0 = pstart[pcur];
                const int32_t *ps = pstart.data();
                const int64_t a = std::lower_bound(ps + pcur + 1, ps + np_, (int32_t)std::min<int64_t>(oend, INT32_MAX)) - ps;
                const int64_t lim = (int64_t)o0 + chunk_obs;
                const int64_t j = pcur + 2 <= np_ ? std::upper_bound(ps + pcur + 2, ps + np_ + 1,
                                                                     (int32_t)std::min<int64_t>(lim, INT32_MAX)) - ps
                                                  : np_ + 1;
                const int64_t pe = std::min({a, j - 1, np_});
                if (pstart[pe] - o0 > 65535) { ok = false; break; }
                cut.push_back(pcur);
                cend.push_back(pe);
                pcur = pe;
            }
            P.rchunk.push_back((int32_t)cut.size());
        }
        // a lower bound of the trial's overshoot from the cut alone (round 6):
        // a spec's staged slots in its busiest chunk are at least its
        // observations over the chunk count, and its pair list at least the
        // 128-entry minimum.  When even that bound needs the largest shrink
        // (0.5: overshoot >= 1.96), the exact statistics would give the same
        // next size, so their pass (a device round trip) is skipped: cfg4's
        // 65,535 and 32,767 trials (overshoot 5.4 and 2.8); the plan is the
        // same (the digest tests)
        if (ok && !cut.empty() && chunk_obs > 64) {
            int64_t lb = 0;
            for (auto &sp : specs) {
                int64_t ow = 0;
                for (auto &R : sp) ow += cnt[(size_t)R.c * nc + R.c];
                lb = std::max<int64_t>(lb, ceil_div(ow, (int64_t)cut.size()));
            }
            const int bs0 = P.buf_slots, pc0 = P.pair_cap;
            P.buf_slots = std::max(8, (int)((lb + 7) / 8 * 8));
            P.pair_cap = 128;
            const double over_lb = std::max((double)lb / SW_MAX_STAGED, (double)P.lds_bytes() / (160 * 1024));
            P.buf_slots = bs0;
            P.pair_cap = pc0;
            if (0.98 / over_lb <= 0.5) {
                chunk_obs = std::max(64, (int)(chunk_obs * 0.5));
                continue;
            }
        }
        std::vector<int> cstaged(cut.size(), 0), cpmax(cut.size(), 0);
        if (ok && dev && !cut.empty()) {  // the same statistics from k_plan_chunkmax
            const size_t nk = cut.size();
            if (!d_spec_of) {
                d_spec_of = dev->scratch<int32_t>(spec_of.size());
                d_scam = dev->scratch<int32_t>(P.spec_cam.size());
                if (dev->err) return;
                dev->ok(hipMemcpyAsync(d_spec_of, spec_of.data(), spec_of.size() * 4, hipMemcpyHostToDevice, dev->s));
                dev->ok(hipMemcpyAsync(d_scam, P.spec_cam.data(), P.spec_cam.size() * 4, hipMemcpyHostToDevice, dev->s));
            }
            std::vector<int32_t> cc(2 * nk), out(2 * nk);
            for (size_t k = 0; k < nk; ++k) {
                cc[k] = (int32_t)cut[k];
                cc[nk + k] = (int32_t)cend[k];
            }
            int32_t *d_cc = dev->scratch<int32_t>(2 * nk), *d_out = dev->scratch<int32_t>(2 * nk);
            if (dev->err) return;
            dev->ok(hipMemcpyAsync(d_cc, cc.data(), 2 * nk * 4, hipMemcpyHostToDevice, dev->s));
            const int split = env_int("SFM_PLAN_CHUNK_SPLIT", std::max(1, std::min(16, (int)ceil_div(1024, (int64_t)nk))));
            if (split > 1) {
                uint32_t *d_cnt = dev->scratch<uint32_t>(nk * (size_t)(nc + P.nspec));
                if (dev->err) return;
                dev->ok(hipMemsetAsync(d_cnt, 0, nk * (size_t)(nc + P.nspec) * 4, dev->s));
                hipLaunchKernelGGL(k_plan_chunkcnt, dim3((unsigned)nk, (unsigned)split), dim3(256),
                                   (nc + P.nspec) * sizeof(int32_t), dev->s, nc, P.nspec, dev->pstart, dev->pt,
                                   dev->cam, d_cc, d_cc + nk, d_spec_of, d_cnt);
                dev->ok(hipGetLastError());
                hipLaunchKernelGGL(k_plan_chunkmax_fin, dim3((unsigned)nk), dim3(256), 0, dev->s, nc, P.nspec, d_cnt,
                                   d_scam, d_out);
            } else {
                hipLaunchKernelGGL(k_plan_chunkmax, dim3((unsigned)nk), dim3(256), (nc + P.nspec + 2) * sizeof(int32_t),
                                   dev->s, nc, P.nspec, dev->pstart, dev->pt, dev->cam, d_cc, d_cc + nk, d_spec_of,
                                   d_scam, d_out);
            }
            dev->ok(hipGetLastError());
            dev->ok(hipMemcpyAsync(out.data(), d_out, 2 * nk * 4, hipMemcpyDeviceToHost, dev->s));
            dev->ok(hipStreamSynchronize(dev->s));
            if (dev->err) return;
            for (size_t k = 0; k < nk; ++k) {
                cstaged[k] = out[2 * k];
                cpmax[k] = out[2 * k + 1];
            }
        } else if (ok)
            par_for((int64_t)cut.size(), [&](int64_t k) {
                std::vector<int32_t> ccount(nc, 0), cpairs(P.nspec, 0);
                for (int64_t pe = cut[k]; pe < cend[k]; ++pe)
                    for (int32_t a = pstart[pe]; a < pstart[pe + 1]; ++a) {
                        ccount[cam[a]]++;
                        for (int32_t b = pstart[pe]; b < pstart[pe + 1]; ++b)
                            if (cam[b] > cam[a]) cpairs[spec_of[(size_t)cam[a] * nc + cam[b]]]++;
                    }
                for (int w = 0; w < P.nspec; ++w) {
                    int st = 0;
                    for (auto &R : specs[w]) st += ccount[R.c];
                    cstaged[k] = std::max(cstaged[k], st);
                    cpmax[k] = std::max(cpmax[k], cpairs[w]);
                }
            });
        int max_staged = 0, max_pairs = 0;
        for (size_t k = 0; k < cut.size(); ++k) {
            max_staged = std::max(max_staged, cstaged[k]);
            max_pairs = std::max(max_pairs, cpmax[k]);
        }
        P.buf_slots = std::max(8, (max_staged + 7) / 8 * 8);
        P.pair_cap = std::max(128, (max_pairs + 127) / 128 * 128);  // 16-bit entries, whole 64-lane DMA rows
        P.list_cap = (P.buf_slots + 1 + 63) / 64 * 64;  // the count, then the entries
        if ((ok && max_staged <= SW_MAX_STAGED && P.lds_bytes() <= 160 * 1024) || chunk_obs <= 64) break;
        const double over = std::max((double)max_staged / SW_MAX_STAGED, (double)P.lds_bytes() / (160 * 1024));
        chunk_obs = std::max(64, (int)(chunk_obs * std::min(0.95, std::max(0.5, 0.98 / over))));
    }
    P.nchunk = (int32_t)cut.size();
    pt_.tick("plan:chunks");
    P.cut.assign(cut.begin(), cut.end());
    P.cut.push_back((int32_t)np_);
    // exact per-chunk counts: pairs per block, observations per camera
    std::vector<uint16_t> bq((size_t)P.nbd * P.nchunk, 0), cq((size_t)nc * P.nchunk, 0);
    if (dev) {  // k_plan_counts (32-bit atomics), narrowed to the planner's uint16 on the device
        const size_t nb = (size_t)P.nbd * P.nchunk, ncq = (size_t)nc * P.nchunk;
        uint32_t *b32 = dev->scratch<uint32_t>(nb + ncq);
        uint16_t *b16 = dev->scratch<uint16_t>(nb + ncq);
        dev->d_cut = dev->scratch<int32_t>(P.cut.size());
        if (dev->err) return;
        dev->ok(hipMemcpyAsync(dev->d_cut, P.cut.data(), P.cut.size() * 4, hipMemcpyHostToDevice, dev->s));
        dev->ok(hipMemsetAsync(b32, 0, (nb + ncq) * 4, dev->s));
        if (no) {
            // the LDS form while its histogram fits, split so that a
            // workgroup's pairs are several times its counters (the flush)
            const size_t hist = ((size_t)P.nbd + nc) * sizeof(uint32_t);
            static const bool big_lds =
                hipFuncSetAttribute(reinterpret_cast<const void *>(&k_plan_counts_lds),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
            const double pairs = (double)std::accumulate(cnt.begin(), cnt.end(), int64_t(0)) - (double)no;
            const int split = std::max(1, std::min(16, (int)(pairs / P.nchunk / (4.0 * (P.nbd + nc)))));
            if (hist <= (big_lds ? 160 * 1024 : 64 * 1024) && !env_int("SFM_PLAN_COUNTS_GLOBAL", 0))
                hipLaunchKernelGGL(k_plan_counts_lds, dim3((unsigned)P.nchunk, (unsigned)split), dim3(CNT_THREADS), hist,
                                   dev->s, nc, P.nchunk, dev->pstart, dev->pt, dev->cam, dev->d_cut, b32, b32 + nb);
            else
                hipLaunchKernelGGL(k_plan_counts, dim3((unsigned)ceil_div(no, 256)), dim3(256), 0, dev->s, no, nc,
                                   P.nchunk, dev->pstart, dev->pt, dev->cam, dev->d_cut, b32, b32 + nb);
            dev->ok(hipGetLastError());
        }
        hipLaunchKernelGGL(k_plan_narrow, dim3((unsigned)ceil_div((int64_t)(nb + ncq), 256)), dim3(256), 0, dev->s,
                           (int64_t)(nb + ncq), b32, b16);
        dev->ok(hipGetLastError());
        dev->ok(hipMemcpyAsync(bq.data(), b16, nb * 2, hipMemcpyDeviceToHost, dev->s));
        dev->ok(hipMemcpyAsync(cq.data(), b16 + nb, ncq * 2, hipMemcpyDeviceToHost, dev->s));
        dev->ok(hipStreamSynchronize(dev->s));
        if (dev->err) return;
        dev->d_bq = b16;
    } else
    par_for(P.nchunk, [&](int64_t q) {  // chunk q writes column q only
        const int64_t pe = q + 1 < P.nchunk ? cut[q + 1] : np_;
        for (int64_t pp = cut[q]; pp < pe; ++pp)
            for (int32_t a = pstart[pp]; a < pstart[pp + 1]; ++a) {
                cq[(size_t)cam[a] * P.nchunk + q]++;
                for (int32_t b = pstart[pp]; b < pstart[pp + 1]; ++b)
                    if (cam[b] > cam[a]) bq[(size_t)dense_blk(nc, cam[a], cam[b]) * P.nchunk + q]++;
            }
    });
    pt_.tick("plan:counts");
    // slots per group, then lanes: diagonal groups first (the loader
    // waves), then the off-diagonal groups by size.  The proportional split
    // remains for a spec with more groups than slots (the greedy needs one
    // slot per group); its power-of-two variant is retired (round 6).
    P.lanegrp.assign((size_t)P.nspec * SW_THREADS, (int16_t)-1);
    std::vector<std::vector<int>> gid_of(P.nspec);  // (row, j - j0) -> group index within spec
    int64_t f_plan = 0, f_ideal = 0;
    // the slot allocation of every spec (independent: host threads), then the
    // lane layout in spec order
    std::vector<std::vector<int>> sl_of(P.nspec);
    std::vector<int64_t> fplan_w(P.nspec, 0), fideal_w(P.nspec, 0);
    par_for_dynamic(P.nspec, [&](int64_t w) {
        const auto &gd = sgd[w], &g = sg[w];
        const int Gd = sGd[w], budget = sbudget[w];
        std::vector<int> dtrip(P.nchunk, 0);
        for (auto &x : gd)
            for (int32_t q = 0; q < P.nchunk; ++q)
                dtrip[q] = std::max(dtrip[q], sweep_trips(cq[(size_t)x.row_cam * P.nchunk + q], Gd / lpp));
        std::vector<std::vector<uint16_t>> Pg(g.size());
        for (size_t k = 0; k < g.size(); ++k)
            Pg[k].assign(bq.begin() + (size_t)g[k].blk * P.nchunk, bq.begin() + (size_t)(g[k].blk + 1) * P.nchunk);
        std::vector<int> &sl = sl_of[w];
        if (!g.empty() && (int)g.size() <= budget) {
            fplan_w[w] = sweep_alloc(Pg, dtrip, budget, sl);
        } else {  // proportional
            double tot = 0;
            for (auto &x : g) tot += x.work;
            sl.assign(g.size(), 1);
            int sum = 0;
            for (size_t k = 0; k < g.size(); ++k) {
                sl[k] = std::max(1, (int)(tot > 0 ? g[k].work / tot * budget : 1.0));
                sum += sl[k];
            }
            while (sum > budget) {
                auto it = std::max_element(sl.begin(), sl.end());
                *it -= 1;
                sum -= 1;
            }
            while (sum < budget && !g.empty()) {
                size_t best = 0;
                for (size_t k = 1; k < g.size(); ++k)
                    if (g[k].work * sl[best] > g[best].work * sl[k]) best = k;
                sl[best] += 1;
                sum += 1;
            }
        }
        for (int32_t q = 0; q < P.nchunk; ++q) {  // the balance bound: every chunk's pairs over all slots
            int64_t pq = 0;
            for (auto &v : Pg) pq += v[q];
            fideal_w[w] += std::max<int64_t>(dtrip[q], (pq + budget - 1) / std::max(1, budget));
        }
    });
    for (int w = 0; w < P.nspec; ++w) {
        f_plan += fplan_w[w];
        f_ideal += fideal_w[w];
        auto &gd = sgd[w], &g = sg[w];
        const int Gd = sGd[w], nload = P.nload[w];
        const std::vector<int> &sl = sl_of[w];
        for (size_t k = 0; k < g.size(); ++k) g[k].slots = sl[k];
        std::stable_sort(g.begin(), g.end(), [](const G0 &a, const G0 &b) { return a.slots > b.slots; });
        for (auto &x : gd) x.slots = Gd / lpp;
        g.insert(g.begin(), gd.begin(), gd.end());
        P.goff.push_back((int32_t)P.groups.size());
        gid_of[w].assign(specs[w].size() * nc, -1);
        int lane = 0;
        for (size_t k = 0; k < g.size(); ++k) {
            if (k == gd.size()) lane = 64 * nload;  // off-diagonal groups after the loader waves
            const int G = lpp * g[k].slots;
            P.groups.push_back({g[k].blk, lane, G, g[k].flags, g[k].cam_b});
            for (int l = lane; l < lane + G; ++l) P.lanegrp[(size_t)w * SW_THREADS + l] = (int16_t)k;
            gid_of[w][g[k].key] = (int)k;
            lane += G;
        }
    }
    P.goff.push_back((int32_t)P.groups.size());
    pt_.tick("plan:alloc");
    // the dispatch tail: one workgroup per CU (SW_THREADS, 168 VGPRs), so
    // items run in rounds of ncu; a short last round's specs are split per
    // range into S chunk sub-ranges (SFM_SWEEP_SPLIT=0: off).  Not with the
    // SlabSrc reads the partials in the finish's order when it is folded in.
    P.split_of.assign(P.nbd, -1);
    {
        const int per_round = ncu / NXCD;  // specs of one range group per round
        // S = 8 (SFM_SWEEP_SPLIT=0: off): cfg5 0.361 -> 0.343 ms with a full
        // round of camera workgroups (below); the first try (0.341 -> 0.362)
        // left 64 camera workgroups behind the split round, a tail of their own
        const int want = env_int("SFM_SWEEP_SPLIT", 8);
        int min_chunks = INT32_MAX;
        for (int r = 0; r < P.nrange; ++r) min_chunks = std::min(min_chunks, P.rchunk[r + 1] - P.rchunk[r]);
        const int nsplit = P.nspec % std::max(1, per_round);
        if (allow_split && want >= 2 && P.nrange == NXCD && per_round >= 1 && P.nspec > per_round && nsplit > 0) {
            const int S = std::min({want, per_round / nsplit, min_chunks});
            if (S >= 2) {
                P.split_S = S;
                P.split_n = nsplit;
                P.split_w0 = P.nspec - nsplit;
                for (int w = P.split_w0; w < P.nspec; ++w)
                    P.split_gmax = std::max(P.split_gmax, P.goff[w + 1] - P.goff[w]);
                for (int w = P.split_w0; w < P.nspec; ++w)
                    for (int g = P.goff[w]; g < P.goff[w + 1]; ++g)
                        P.split_of[P.groups[g].blk] = (w - P.split_w0) * P.split_gmax + (g - P.goff[w]);
            }
        }
    }
    if (env_int("SFM_SWEEP_VERBOSE", 0))
        std::fprintf(stderr,
                     "sweep plan: nspec %d nrange %d nchunk %d chunk_obs %d buf_slots %d pair_cap %d lds %zu B; "
                     "chunk trips (sum over specs, chunks) %lld, balance bound %lld\n",
                     P.nspec, P.nrange, P.nchunk, chunk_obs, P.buf_slots, P.pair_cap, P.lds_bytes(), (long long)f_plan,
                     (long long)f_ideal);
    const size_t nqw = (size_t)P.nchunk * P.nspec;
    if (dev && P.hdr_cap <= 1024) {  // k_plan_lists writes them into the problem's buffers
        P.dev_lists = true;
        pt_.tick("plan:lists");
        return;
    }
    P.list.assign(nqw * P.list_cap, 0);
    P.pairs.assign(nqw * P.pair_cap, 0);
    P.hdr.assign(nqw * P.hdr_cap, 0);
    par_for(P.nchunk, [&](int64_t q) {  // chunk q writes its (chunk, spec) regions only
        std::vector<std::vector<int32_t>> per_cam(nc);
        std::vector<int32_t> slot_of;  // chunk-local obs offset -> position in its camera's list
        std::vector<int32_t> gpos;     // each group's next pair position
        const int32_t o0 = pstart[cut[q]];
        const int32_t o1 = q + 1 < P.nchunk ? pstart[cut[q + 1]] : (int32_t)no;
        for (auto &v : per_cam) v.clear();
        slot_of.assign(o1 - o0, 0);
        for (int32_t o = o0; o < o1; ++o) {
            slot_of[o - o0] = (int32_t)per_cam[cam[o]].size();
            per_cam[cam[o]].push_back(o - o0);
        }
        for (int w = 0; w < P.nspec; ++w) {
            const auto &sp = specs[w];
            const size_t qw = (size_t)q * P.nspec + w;
            int32_t *lst = &P.list[qw * P.list_cap];
            const int32_t n0 = (int32_t)per_cam[sp[0].c].size();
            const int32_t n1 = sp.size() > 1 ? (int32_t)per_cam[sp[1].c].size() : 0;
            int ns_ = 1;  // the count, then every slot's point | (spec row << 31)
            for (size_t rr = 0; rr < sp.size(); ++rr)
                for (int32_t off : per_cam[sp[rr].c])
                    lst[ns_++] = (int32_t)((uint32_t)pt[o0 + off] | (rr ? 0x80000000u : 0u));
            lst[0] = n0 + n1;
            for (; ns_ < P.list_cap; ++ns_) lst[ns_] = pt[o0];  // padding: any valid point
            const int ng = P.goff[w + 1] - P.goff[w];
            // every group's pairs in this chunk are counted already (bq: a
            // block belongs to one group of one spec), so the group offsets
            // come first and the pairs go straight to their place, in the
            // traversal order (spec row, the camera's observations, the
            // point's observations)
            int32_t *hd = &P.hdr[qw * P.hdr_cap];
            uint16_t *pp = &P.pairs[qw * P.pair_cap];
            int32_t np2 = 0;
            for (int g = 0; g < ng; ++g) {
                hd[g] = np2;
                const SweepGroup &G = P.groups[P.goff[w] + g];
                if (!(G.flags & 1)) np2 += bq[(size_t)G.blk * P.nchunk + q];
            }
            hd[ng] = np2;
            gpos.assign(hd, hd + ng);
            for (size_t rr = 0; rr < sp.size(); ++rr) {
                const Row &R = sp[rr];
                const int32_t abase = rr == 0 ? 0 : n0;
                const int *gid = gid_of[w].data() + rr * nc - R.j0;
                for (int32_t off : per_cam[R.c]) {
                    const int32_t a = o0 + off, pnt = pt[a];
                    const uint16_t v = (uint16_t)(abase + slot_of[off]);
                    for (int32_t b = pstart[pnt]; b < pstart[pnt + 1]; ++b) {
                        const int cj = cam[b];
                        if (cj <= R.c || cj < R.j0 || cj >= R.j1) continue;
                        pp[gpos[gid[cj]]++] = v;
                    }
                }
            }
            hd[ng + 1] = n0;
            hd[ng + 2] = n1;
            hd[ng + 3] = o0;
        }
    });
    pt_.tick("plan:lists");
}

// ------------------------------------------------------------ problem
enum { T_LIN, T_PREP, T_SCHUR, T_COMM, T_SOLVE, T_TRIAL, T_NT };
constexpr int kEvSlots = 16;  // max iterations per batch between host polls
static const char *kTimerNames = "linearize;point_prep;schur_blocks;allreduce;cholesky;backsub_trial";

struct sfm_ba_problem {
    int device = 0;
    hipStream_t stream = nullptr;
    sfm_comm *comm = nullptr;
    int32_t nc = 0, ns = 0, nsp = 0, nT = 0, tb = 16;
    int64_t np = 0, no = 0, npairs = 0;
    uint64_t plan_digest = 0;  // SFM_PLAN_DIGEST=1: the digest of the sweep plan (sfm_ba_plan_digest)
    int32_t ndiag_items = 0, ndiag_blocks = 0;  // k_camera_lin items (one per workgroup) / cameras
    int32_t cl_fused_wg = 0, cl_fused_items = 0;  // k_schur_sweep's camera workgroups / their items
    bool cl_fused = false;                         // this solve: camera blocks inside the sweep launch
    bool chol_dpp = true, fin_fused = true;        // this solve: DPP tile factor; finish folded into the solve
    int sw_debug = 0;                              // k_schur_sweep dbg argument: 0 (the work-skipping probes are retired)
    // Schur sweep plan (k_schur_sweep): ranges, chunks, specs
    int32_t sw_nrange = 0, sw_nspec = 0, sw_nbd = 0, sw_nchunk = 0;
    SweepSplit sw_split = {};
    int32_t *d_sw_split_of = nullptr;
    SweepLds sw_L = {};
    int sw_lpp = 1;
    bool sw_pinhole = false;
    size_t sw_lds_bytes = 0;
    Kmat K;
    std::vector<double> cams0, pts0;
    // device
    int32_t *d_cam = nullptr, *d_pt = nullptr, *d_pstart = nullptr, *d_cm_pt = nullptr, *d_cstart = nullptr;
    double2 *d_cm_obs = nullptr;  // camera-major observations (with d_cm_pt: k_camera_lin)
    PairItem *d_items = nullptr, *d_fitems = nullptr;  // camera items: k_camera_lin / the sweep's camera workgroups
    BlockInfo *d_blocks = nullptr, *d_fblocks = nullptr;
    int32_t *d_wg_first = nullptr, *d_fwg_first = nullptr;
    double *d_slab = nullptr, *d_slab2 = nullptr, *d_camlin = nullptr;
    int32_t *d_sw_rchunk = nullptr, *d_sw_goff = nullptr, *d_sw_nload = nullptr, *d_sw_list = nullptr, *d_sw_hdr = nullptr;
    int32_t *d_sw_scam = nullptr;
    SweepGroup *d_sw_groups = nullptr;
    int16_t *d_sw_lanegrp = nullptr;
    uint32_t *d_sw_pairs = nullptr;
    int2 *d_sw_blkij = nullptr;
    double2 *d_obs = nullptr;
    double *d_Rt = nullptr, *d_Rt2 = nullptr, *d_X = nullptr, *d_X2 = nullptr;
    double *d_Vg = nullptr, *d_Lq = nullptr;
    double *d_payload = nullptr, *d_A = nullptr, *d_b = nullptr, *d_D = nullptr;
    double *d_partial = nullptr, *d_scal = nullptr;
    int *d_bad = nullptr;
    int *d_sw_err = nullptr;  // k_schur_sweep: a chunk hand-off timed out
    unsigned *d_count = nullptr;  // grid_sum_last arrival counters
    unsigned *d_nbig = nullptr;   // gradient_tolerance: point-gradient entries >= gtol
    double *d_gbuf = nullptr;     // gradient_tolerance: [count, g_c (6 nc)]
    double gtol = 0.0;            // this solve's gradient_tolerance (k_linearize counts when > 0)
    HostLM *h_ring = nullptr, *d_ring = nullptr;  // pinned host ring of published LM states (+ device alias)
    bool timing = false;                         // per-phase HIP events (sfm_ba_set_timing)
    int64_t payload_len = 0;
    int pt_blocks = 0;
    int bs_cl_blocks = 0;  // k_backsub_trial with the cameras in LDS: its grid (0: cameras from global)
    int lin_cl_blocks = 0;        // k_linearize_cl's grid (0: k_linearize, cameras from global)
    hipEvent_t ev[2 * T_NT] = {};
    hipEvent_t ev_it[2 * T_NT * kEvSlots] = {};  // per-iteration timing slots of a batch
    LMState *d_lm = nullptr;
    // persistent Gauss-Jordan reduced solve (gj_solve.hpp)
    GjPlan gjp;
    GjBufs gjb;
    int gj_epoch = 0;
    GjrPlan gjrp;  // the row-distributed solve (default; gjp is then unused)
    GjrBufs gjrb;
    unsigned gjr_tag = 0;
    bool gjr_fold = false;  // fold k_schur_finish into the row-distributed solve (SFM_GJR_FOLD)
    hipEvent_t ev_solve = nullptr;
    double t_acc[T_NT] = {};
    int t_iters = 0;
    std::vector<std::pair<void *, size_t>> allocs;
    ~sfm_ba_problem() {
        (void)hipSetDevice(device);
        if (ev_solve && comm && comm->local) {
            std::lock_guard<std::mutex> lk(comm->local->solve_mu);
            if (comm->local->last_solve == ev_solve) comm->local->last_solve = nullptr;
        }
        // the stream drains before its blocks and events go back to the caches
        const bool idle = stream && hipStreamSynchronize(stream) == hipSuccess;
        for (auto &a : allocs) {
            if (idle) pool_free(a.first, a.second, device);
            else (void)hipFree(a.first);
        }
        if (stream && idle) {
            kit_release(*this);
            return;
        }
        (void)hipGetLastError();
        if (h_ring) (void)hipHostFree(h_ring);
        for (auto &e : ev)
            if (e) (void)hipEventDestroy(e);
        for (auto &e : ev_it)
            if (e) (void)hipEventDestroy(e);
        if (ev_solve) (void)hipEventDestroy(ev_solve);
        if (stream) (void)hipStreamDestroy(stream);
    }
    template <class T> int alloc(T *&p, int64_t n) {
        void *q = nullptr;
        size_t bytes = (size_t)std::max<int64_t>(n, 1) * sizeof(T), got;
        if (pool_malloc(&q, bytes, device, &got) != hipSuccess) {
            set_error("hipMalloc(%zu) failed", bytes);
            return SFM_ERR_NOMEM;
        }
        allocs.push_back({q, got});
        p = reinterpret_cast<T *>(q);
        return 0;
    }
    static void kit_release(sfm_ba_problem &p);
    bool kit_acquire();
};

// A destroyed problem's stream, its 200 timing events, the solve event and
// the pinned LM ring, kept for the next create on the same device (creating
// them cost ~2-3 ms per create).
struct StreamKit {
    int dev;
    hipStream_t stream;
    hipEvent_t ev[2 * T_NT];
    hipEvent_t ev_it[2 * T_NT * kEvSlots];
    hipEvent_t ev_solve;
    HostLM *h_ring, *d_ring;
};
static std::mutex &kit_mu() {
    static auto *m = new std::mutex();
    return *m;
}
static std::vector<StreamKit> &kits() {
    static auto *v = new std::vector<StreamKit>();
    return *v;
}
void sfm_ba_problem::kit_release(sfm_ba_problem &p) {
    StreamKit k;
    k.dev = p.device;
    k.stream = p.stream;
    std::memcpy(k.ev, p.ev, sizeof k.ev);
    std::memcpy(k.ev_it, p.ev_it, sizeof k.ev_it);
    k.ev_solve = p.ev_solve;
    k.h_ring = p.h_ring;
    k.d_ring = p.d_ring;
    std::lock_guard<std::mutex> lk(kit_mu());
    kits().push_back(k);
}
bool sfm_ba_problem::kit_acquire() {
    if (!pool_on()) return false;
    std::lock_guard<std::mutex> lk(kit_mu());
    auto &v = kits();
    for (size_t i = v.size(); i-- > 0;)
        if (v[i].dev == device) {
            const StreamKit &k = v[i];
            stream = k.stream;
            std::memcpy(ev, k.ev, sizeof ev);
            std::memcpy(ev_it, k.ev_it, sizeof ev_it);
            ev_solve = k.ev_solve;
            h_ring = k.h_ring;
            d_ring = k.d_ring;
            v.erase(v.begin() + i);
            return true;
        }
    return false;
}

static int upload_state(sfm_ba_problem *p) {
    std::vector<double> Rt(12 * (size_t)p->nc);
    for (int c = 0; c < p->nc; ++c) {
        h_rotvec_to_R(&p->cams0[6 * c], &Rt[12 * c]);
        for (int i = 0; i < 3; ++i) Rt[12 * c + 9 + i] = p->cams0[6 * c + 3 + i];
    }
    SFM_HIP(hipMemcpyAsync(p->d_Rt, Rt.data(), Rt.size() * 8, hipMemcpyHostToDevice, p->stream));
    if (!p->pts0.empty())  // a one-shot problem's points went up in create
        SFM_HIP(hipMemcpyAsync(p->d_X, p->pts0.data(), p->pts0.size() * 8, hipMemcpyHostToDevice, p->stream));
    SFM_HIP(hipStreamSynchronize(p->stream));
    return 0;
}

extern "C" int sfm_comm_unique_id(char out[128]) {
    SFM_CHECK_ARG(out, "null pointer");
    static_assert(sizeof(ncclUniqueId) <= 128, "unique id size");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) {
        set_error("ncclGetUniqueId failed");
        return SFM_ERR_COMM;
    }
    std::memset(out, 0, 128);
    std::memcpy(out, &id, sizeof id);
    return 0;
}

extern "C" int sfm_comm_init(const char id[128], int nranks, int rank, int device, sfm_comm **out) {
    SFM_CHECK_ARG(id && out && nranks >= 1 && rank >= 0 && rank < nranks, "bad communicator arguments");
    SFM_HIP(hipSetDevice(device));
    auto *c = new sfm_comm();
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        set_error("ncclCommInitRank: %s", ncclGetErrorString(r));
        delete c;
        return SFM_ERR_COMM;
    }
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    *out = c;
    return 0;
}

extern "C" int sfm_comm_init_local(int nranks, sfm_comm **out) {
    SFM_CHECK_ARG(out && nranks >= 1, "bad local group arguments");
    auto *g = new LocalGroup();
    g->nranks = nranks;
    g->bufs.resize(nranks);
    g->refs = nranks;
    for (int r = 0; r < nranks; ++r) {
        out[r] = new sfm_comm();
        out[r]->local = g;
        out[r]->nranks = nranks;
        out[r]->rank = r;
    }
    return 0;
}

extern "C" int sfm_comm_destroy(sfm_comm *c) {
    if (!c) return 0;
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->local) {
        bool last;
        {
            std::lock_guard<std::mutex> lk(c->local->mu);
            last = --c->local->refs == 0;
        }
        if (last) delete c->local;
    }
    delete c;
    return 0;
}

namespace sfm {
bool dense_obs_info(void *handle, int64_t *n, int64_t *n_rows, int32_t *n_cams);  // dense_obs.cpp
void dense_obs_copy(void *handle, int32_t *cam, int32_t *pt, double *obs);
int dense_obs_pieces(void *handle, std::vector<int64_t> &off);
void dense_obs_copy_pieces(void *handle, const std::vector<int64_t> &off, int t0, int t1, int32_t *cam, int32_t *pt,
                           double *obs);
}  // namespace sfm

// sfm_ba_create; with `dense` (a sfm_dense_obs_scan handle) the
// observations come from the scan's pieces, copied straight into the pinned
// upload buffer (cam / pt / obs are then null): no COO arrays in between
static int ba_create(int32_t nc, int64_t np_, int64_t no, const int32_t *cam, const int32_t *pt, const double *obs,
                     void *dense, const double *K, const double *cams, const double *pts, int device, sfm_comm *comm,
                     sfm_ba_problem **out, bool oneshot = false) {
    SFM_CHECK_ARG(out && K && cams && (pts || np_ == 0) && (no == 0 || dense || (cam && pt && obs)), "null pointer");
    SFM_CHECK_ARG(nc >= 1 && np_ >= 0 && no >= 0, "bad sizes");
    SFM_CHECK_ARG(no < ((int64_t)1 << 31), "problem too large for int32 indexing");
    SFM_CHECK_ARG(6 * nc <= SOLVE_MAX, "at most 682 cameras (dense reduced camera system)");
    // SFM_CREATE_TIMING=1: the host phases of create on stderr (measurement)
    PhaseTimer ctm_;
    auto ctick = [&](const char *what) { ctm_.tick(what); };
    const bool ctm = ctm_.on;
    if (!dense) {  // host threads over contiguous observation ranges (the scan's output is valid by construction)
        constexpr int NB = 16;
        int bad[NB] = {0};
        par_for(NB, [&](int64_t t) {
            for (int64_t o = no * t / NB; o < no * (t + 1) / NB; ++o) {
                if (!(cam[o] >= 0 && cam[o] < nc && pt[o] >= 0 && pt[o] < np_)) bad[t] |= 1;
                if (!(o == 0 || pt[o] >= pt[o - 1])) bad[t] |= 2;
            }
        });
        int any = 0;
        for (int t = 0; t < NB; ++t) any |= bad[t];
        SFM_CHECK_ARG(!(any & 1), "observation index out of range");
        SFM_CHECK_ARG(!(any & 2), "observations must be point-major (sorted by point)");
    }
    ctick("validate");
    auto p = std::make_unique<sfm_ba_problem>();
    p->device = device;
    p->comm = comm;
    p->nc = nc;
    p->np = np_;
    p->no = no;
    p->ns = 6 * nc;
    p->tb = chol_tile(p->ns);
    p->nT = (p->ns + p->tb - 1) / p->tb;
    p->nsp = p->nT * p->tb;
    std::memcpy(p->K.k, K, sizeof p->K.k);
    // a pinhole K (the reference's calibration): the sweep drops its structural zeros
    p->sw_pinhole = K[1] == 0.0 && K[3] == 0.0 && K[6] == 0.0 && K[7] == 0.0 && K[8] == 1.0 &&
                    env_int("SFM_SWEEP_PINHOLE", 1) != 0;
    p->cams0.assign(cams, cams + 6 * (size_t)nc);
    // x0's points are kept for sfm_ba_reset; a one-shot problem (sfm_ba_lm*:
    // created, solved and destroyed in one call) uploads them from the
    // caller's array through the pinned stage instead (cfg5: the 12-MB copy
    // and a pageable upload, ~1 ms of the call)
    if (!oneshot) p->pts0.assign(pts, pts + 3 * (size_t)np_);
    bool x_up = false;
    // SFM_CREATE_PLAN_ONLY=1 (measurement, tools/create_probe.py): the host
    // planner alone, without a device; returns 1 and no problem.
    // SFM_PLAN_HOST=1: the host's CSR, counts and planner passes (the device
    // ones must produce the same plan: the digest test)
    const bool plan_only = env_int("SFM_CREATE_PLAN_ONLY", 0) != 0;
    const bool host_plan = plan_only || env_int("SFM_PLAN_HOST", 0) != 0;
    const bool want_digest = env_int("SFM_PLAN_DIGEST", 0) != 0;
    int rc;
    // point CSR (pstart), camera-major permutation (cam_obs, stable: point
    // order within a camera) and its offsets (cstart), co-observation counts
    // per camera block (cnt, the static sparsity of the reduced camera system)
    std::vector<int32_t> pstart(np_ + 1), cstart(nc + 1, 0), cam_obs;
    std::vector<int64_t> cnt((size_t)nc * nc, 0);
    int64_t tot = 0;
    if (!plan_only) {
        SFM_HIP(hipSetDevice(device));
        (void)hipGetLastError();  // launches below are checked with hipGetLastError: start clean
        if (!p->kit_acquire()) {
            SFM_HIP(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
            for (auto &e : p->ev) SFM_HIP(hipEventCreate(&e));
            for (auto &e : p->ev_it) SFM_HIP(hipEventCreate(&e));
        }
        ctick("stream");
        if ((rc = p->alloc(p->d_cam, no)) || (rc = p->alloc(p->d_pt, no)) || (rc = p->alloc(p->d_pstart, np_ + 1)) ||
            (rc = p->alloc(p->d_obs, no)) || (rc = p->alloc(p->d_cm_pt, no)) || (rc = p->alloc(p->d_cm_obs, no)) ||
            (rc = p->alloc(p->d_cstart, nc + 1)) || (rc = p->alloc(p->d_X, 3 * np_)))
            return rc;
    }
    // the COO up through a pinned staging buffer kept across calls (host
    // threads copy into it, the copy engine takes it from there: a pageable
    // hipMemcpy of the 96 MB at cfg5 ran ~10 GB/s); a concurrent create
    // finding it busy uploads from pageable memory
    std::unique_lock<std::mutex> stage_lk;
    hipEvent_t aux_ev = nullptr;  // the aux stream's uploads (the stage's coordinates and points)
    struct AuxSync {  // on every return: the aux uploads drained before the stage and the buffers go
        hipStream_t s = nullptr;
        ~AuxSync() {
            if (s) (void)hipStreamSynchronize(s);
        }
    } aux_sync;
    std::vector<int32_t> dense_cam, dense_pt;
    std::vector<double> dense_xy;
    if (dense && (plan_only || !no)) {  // no upload: the host arrays alone
        dense_cam.resize(no);
        dense_pt.resize(no);
        dense_xy.resize(2 * (size_t)no);
        if (no) dense_obs_copy(dense, dense_cam.data(), dense_pt.data(), dense_xy.data());
        cam = dense_cam.data();
        pt = dense_pt.data();
        obs = dense_xy.data();
    }
    if (!plan_only && no) {
        PinnedStage &st = pinned_stage();
        stage_lk = std::unique_lock<std::mutex>(st.mu, std::try_to_lock);
        const size_t xoff = (size_t)no * 24, need = xoff + (oneshot ? (size_t)np_ * 24 : 0);
        bool staged = false;
        if (stage_lk.owns_lock()) {
            if (st.bytes < need) {
                if (st.p) (void)hipHostFree(st.p);
                st.p = nullptr;
                st.bytes = 0;
                if (hipHostMalloc(&st.p, need, hipHostMallocDefault) == hipSuccess) st.bytes = need;
                else (void)hipGetLastError();
            }
            if (st.bytes >= need) {
                // the point / camera indices first, on the problem's stream
                // (the CSR and the planner need only them), then the
                // coordinates in batches on the aux stream: the copy engine
                // takes batch b while the host threads fill batch b + 1, and
                // the device CSR runs meanwhile (cfg5: 96 MB had gone up
                // before the CSR could start)
                char *h = static_cast<char *>(st.p);
                int32_t *hc = reinterpret_cast<int32_t *>(h), *hp = reinterpret_cast<int32_t *>(h + (size_t)no * 4);
                double *ho = reinterpret_cast<double *>(h + (size_t)no * 8);
                PinnedStage::Aux *ax = st.aux_for(device);
                const hipStream_t xs = ax ? ax->s : p->stream;
                aux_sync.s = ax ? ax->s : nullptr;
                constexpr int NBATCH = 4, NB = 16;
                std::vector<int64_t> off;
                const int npc = dense ? dense_obs_pieces(dense, off) : 0;
                if (dense) {
                    dense_obs_copy_pieces(dense, off, 0, npc, hc, hp, nullptr);
                } else {
                    par_for(2 * NB, [&](int64_t k) {
                        const int a = (int)(k / NB), t = (int)(k % NB);
                        const size_t n0 = no * t / NB, n1 = no * (t + 1) / NB;
                        std::memcpy((a ? hp : hc) + n0, (a ? pt : cam) + n0, (n1 - n0) * 4);
                    });
                }
                SFM_HIP(hipMemcpyAsync(p->d_cam, hc, no * 4, hipMemcpyHostToDevice, p->stream));
                SFM_HIP(hipMemcpyAsync(p->d_pt, hp, no * 4, hipMemcpyHostToDevice, p->stream));
                for (int b = 0; b < NBATCH; ++b) {
                    int64_t o0, o1;
                    if (dense) {
                        const int t0 = npc * b / NBATCH, t1 = npc * (b + 1) / NBATCH;
                        dense_obs_copy_pieces(dense, off, t0, t1, nullptr, nullptr, ho);
                        o0 = off[t0];
                        o1 = off[t1];
                    } else {
                        o0 = no * b / NBATCH;
                        o1 = no * (b + 1) / NBATCH;
                        par_for(NB, [&](int64_t t) {
                            const size_t n0 = o0 + (o1 - o0) * t / NB, n1 = o0 + (o1 - o0) * (t + 1) / NB;
                            std::memcpy(ho + 2 * n0, obs + 2 * n0, (n1 - n0) * 16);
                        });
                    }
                    if (o1 > o0)
                        SFM_HIP(hipMemcpyAsync(p->d_obs + o0, ho + 2 * o0, (o1 - o0) * 16, hipMemcpyHostToDevice, xs));
                }
                if (dense) {
                    cam = hc;
                    pt = hp;
                    obs = ho;
                }
                if (oneshot && np_) {
                    par_for(NB, [&](int64_t t) {
                        const size_t n0 = 3 * (size_t)np_ * t / NB, n1 = 3 * (size_t)np_ * (t + 1) / NB;
                        std::memcpy(h + xoff + n0 * 8, pts + n0, (n1 - n0) * 8);
                    });
                    SFM_HIP(hipMemcpyAsync(p->d_X, h + xoff, (size_t)np_ * 24, hipMemcpyHostToDevice, xs));
                    x_up = true;
                }
                if (ax) {
                    SFM_HIP(hipEventRecord(ax->ev, xs));
                    aux_ev = ax->ev;
                }
                staged = true;
            }
        }
        if (!staged) {
            if (stage_lk.owns_lock()) stage_lk.unlock();
            if (dense) {  // the staging buffer is busy: the pieces through pageable arrays
                dense_cam.resize(no);
                dense_pt.resize(no);
                dense_xy.resize(2 * (size_t)no);
                dense_obs_copy(dense, dense_cam.data(), dense_pt.data(), dense_xy.data());
                cam = dense_cam.data();
                pt = dense_pt.data();
                obs = dense_xy.data();
            }
            SFM_HIP(hipMemcpyAsync(p->d_cam, cam, no * 4, hipMemcpyHostToDevice, p->stream));
            SFM_HIP(hipMemcpyAsync(p->d_pt, pt, no * 4, hipMemcpyHostToDevice, p->stream));
            SFM_HIP(hipMemcpyAsync(p->d_obs, obs, no * 16, hipMemcpyHostToDevice, p->stream));
        }
        ctick("up:obs");
    }
    if (oneshot && !plan_only && !x_up && np_) {
        SFM_HIP(hipMemcpyAsync(p->d_X, pts, (size_t)np_ * 24, hipMemcpyHostToDevice, p->stream));
        SFM_HIP(hipStreamSynchronize(p->stream));  // pts is the caller's: copied before create returns
    }
    if (host_plan) {  // host threads
        constexpr int NBC = 16;
        par_for(NBC, [&](int64_t t) {  // the observations are sorted by point
            const int64_t o0 = no * t / NBC, o1 = no * (t + 1) / NBC;
            for (int64_t o = o0; o < o1; ++o) {
                const int64_t lo = o == 0 ? 0 : (int64_t)pt[o - 1] + 1;
                for (int64_t i = lo; i <= pt[o]; ++i) pstart[i] = (int32_t)o;
            }
            if (t == NBC - 1)
                for (int64_t i = no ? (int64_t)pt[no - 1] + 1 : 0; i <= np_; ++i) pstart[i] = (int32_t)no;
        });
        // a counting sort: per-range camera counts, offsets in (camera, range)
        // order, every range scatters its own observations in order
        cam_obs.resize(no);
        std::vector<int32_t> rc_cnt((size_t)NBC * nc, 0);
        par_for(NBC, [&](int64_t t) {
            int32_t *hh = rc_cnt.data() + (size_t)t * nc;
            for (int64_t o = no * t / NBC; o < no * (t + 1) / NBC; ++o) hh[cam[o]]++;
        });
        int32_t run = 0;
        for (int c = 0; c < nc; ++c) {
            cstart[c] = run;
            for (int t = 0; t < NBC; ++t) {
                const int32_t v = rc_cnt[(size_t)t * nc + c];
                rc_cnt[(size_t)t * nc + c] = run;
                run += v;
            }
        }
        cstart[nc] = run;
        par_for(NBC, [&](int64_t t) {
            int32_t *f = rc_cnt.data() + (size_t)t * nc;
            for (int64_t o = no * t / NBC; o < no * (t + 1) / NBC; ++o) cam_obs[f[cam[o]]++] = (int32_t)o;
        });
        ctick("csr");
        int dup[NBC] = {0};
        std::vector<std::vector<int64_t>> part(NBC);
        std::vector<int64_t> tpart(NBC, 0);
        par_for(NBC, [&](int64_t t) {
            auto &c = part[t];
            c.assign((size_t)nc * nc, 0);
            int64_t n = 0;
            for (int64_t i = np_ * t / NBC; i < np_ * (t + 1) / NBC; ++i)
                for (int32_t a = pstart[i]; a < pstart[i + 1]; ++a)
                    for (int32_t b = a; b < pstart[i + 1]; ++b) {
                        int ci = cam[a], cj = cam[b];
                        if (b > a && ci == cj) dup[t] = 1;
                        if (ci > cj) std::swap(ci, cj);
                        c[(size_t)ci * nc + cj]++;
                        ++n;
                    }
            tpart[t] = n;
        });
        int any = 0;
        for (int t = 0; t < NBC; ++t) {
            any |= dup[t];
            tot += tpart[t];
            for (size_t k = 0; k < cnt.size(); ++k) cnt[k] += part[t][k];
        }
        SFM_CHECK_ARG(!any, "a point is observed twice by the same camera");
        ctick("blockcounts");
        if (!plan_only) {
            hipStream_t s = p->stream;
            SFM_HIP(hipMemcpyAsync(p->d_pstart, pstart.data(), pstart.size() * 4, hipMemcpyHostToDevice, s));
            if (no) SFM_HIP(hipMemcpyAsync(p->d_cm_pt, cam_obs.data(), no * 4, hipMemcpyHostToDevice, s));
            SFM_HIP(hipMemcpyAsync(p->d_cstart, cstart.data(), cstart.size() * 4, hipMemcpyHostToDevice, s));
        }
    } else {  // on the device: the point CSR from the sorted point indices, a
              // stable radix sort of the camera indices for the permutation,
              // and the block counts with the duplicate check in one pass
        hipStream_t s = p->stream;
        DevPlan tmp;  // scratch on this problem's device and stream (the pool is per device)
        tmp.s = s;
        tmp.dev = device;
        uint32_t *keys = tmp.scratch<uint32_t>(no), *cnt32 = tmp.scratch<uint32_t>((size_t)nc * nc + 1);
        size_t tb = 0;
        if ((rc = sfm::cam_major_sort(nullptr, tb, p->d_cam, keys, p->d_cm_pt, no, nc, s))) return rc;
        void *temp = tmp.scratch<char>(tb);
        if (tmp.err) return tmp.err;
        SFM_HIP(hipMemsetAsync(cnt32, 0, ((size_t)nc * nc + 1) * 4, s));
        hipLaunchKernelGGL(k_csr_pstart, dim3((unsigned)ceil_div(no + 1, 256)), dim3(256), 0, s, no, np_, p->d_pt,
                           p->d_pstart);
        SFM_HIP(hipGetLastError());
        if (no && (rc = sfm::cam_major_sort(temp, tb, p->d_cam, keys, p->d_cm_pt, no, nc, s))) return rc;
        hipLaunchKernelGGL(k_csr_cstart, dim3((unsigned)ceil_div(nc + 1, 256)), dim3(256), 0, s, no, nc, keys,
                           p->d_cstart);
        SFM_HIP(hipGetLastError());
        if (no) {
            const size_t hist = (size_t)nc * (nc + 1) / 2 * sizeof(uint32_t);
            static const bool big_lds =
                hipFuncSetAttribute(reinterpret_cast<const void *>(&k_csr_cnt_lds),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
            if (hist <= (big_lds ? 160 * 1024 : 64 * 1024) && !env_int("SFM_CSR_CNT_GLOBAL", 0))
                hipLaunchKernelGGL(k_csr_cnt_lds, dim3((unsigned)std::min<int64_t>(CSR_CNT_WGS, ceil_div(no, CNT_THREADS))),
                                   dim3(CNT_THREADS), hist, s, no, nc, p->d_pstart, p->d_pt, p->d_cam, cnt32,
                                   cnt32 + (size_t)nc * nc);
            else
                hipLaunchKernelGGL(k_csr_cnt, dim3((unsigned)ceil_div(no, 256)), dim3(256), 0, s, no, nc,
                                   p->d_pstart, p->d_pt, p->d_cam, cnt32, cnt32 + (size_t)nc * nc);
            SFM_HIP(hipGetLastError());
        }
        std::vector<uint32_t> c32((size_t)nc * nc + 1);
        SFM_HIP(hipMemcpyAsync(pstart.data(), p->d_pstart, pstart.size() * 4, hipMemcpyDeviceToHost, s));
        SFM_HIP(hipMemcpyAsync(cstart.data(), p->d_cstart, cstart.size() * 4, hipMemcpyDeviceToHost, s));
        SFM_HIP(hipMemcpyAsync(c32.data(), cnt32, c32.size() * 4, hipMemcpyDeviceToHost, s));
        if (want_digest) {
            cam_obs.resize(no);
            if (no) SFM_HIP(hipMemcpyAsync(cam_obs.data(), p->d_cm_pt, no * 4, hipMemcpyDeviceToHost, s));
        }
        SFM_HIP(hipStreamSynchronize(s));
        SFM_CHECK_ARG(c32[(size_t)nc * nc] == 0, "a point is observed twice by the same camera");
        for (size_t k = 0; k + 1 < c32.size(); ++k) {
            cnt[k] = c32[k];
            tot += c32[k];
        }
        ctick("csr+blockcounts (device)");
    }
    // the staged copies are done once the streams have passed them (a
    // dense scan's observations live in the buffer, and plan_sweep may read
    // them on the host whichever planner runs: kept until it returns; the
    // aux stream's uploads are awaited by the problem's stream below)
    p->npairs = tot;
    // the first reader of the coordinates (and, later, of the points)
    if (aux_ev) SFM_HIP(hipStreamWaitEvent(p->stream, aux_ev, 0));
    if (!plan_only && no) {  // the camera-major copies gathered on the device (cm_pt: permutation -> points)
        hipLaunchKernelGGL(k_gather_cam_major, dim3((unsigned)ceil_div(no, 256)), dim3(256), 0, p->stream, no,
                           p->d_pt, p->d_obs, p->d_cm_pt, p->d_cm_obs);
        SFM_HIP(hipGetLastError());
    }
    SweepPlan sw;
    // lanes per pair slot: 1 (a lane forms a pair's whole 6x6 block, H once;
    // two lanes with half the rows each: cfg4 0.155 against 0.134 ms, round 3; retired)
    p->sw_lpp = 1;
    // the solves read the split partials in k_schur_finish's order (SlabSrc
    // when the finish is folded in): the sweep's dispatch tail may be split
    const bool split_ok = true;
    // the plan's passes over the observation pairs on the device
    // (SFM_PLAN_HOST=1: the host planner's threads, the same plan)
    DevPlan dev;
    const bool dev_plan = !host_plan;
    if (dev_plan) {
        dev.s = p->stream;
        dev.dev = device;
        dev.pstart = p->d_pstart;
        dev.pt = p->d_pt;
        dev.cam = p->d_cam;
        dev.no = no;
    }
    plan_sweep(nc, np_, no, cam, pt, pstart, cnt, p->sw_lpp, plan_only ? 256 : device_cus(device), split_ok, sw,
               dev_plan ? &dev : nullptr);
    if (stage_lk.owns_lock()) {
        SFM_HIP(hipStreamSynchronize(p->stream));
        stage_lk.unlock();
    }
    if (dev.err) {
        set_error("sweep plan on the device: %s", dev.err == SFM_ERR_NOMEM ? "hipMalloc failed" : "HIP error");
        return dev.err;
    }
    ctick("plan_sweep");
    if (sw.buf_slots > SW_MAX_STAGED) {  // one point with more observations in a spec's cameras than a round holds
        set_error("sweep plan: %d observations of one spec's cameras in a single point range (max %d)", sw.buf_slots,
                  SW_MAX_STAGED);
        return SFM_ERR_ARG;
    }
    // camera items (the camera blocks of the normal equations): for
    // k_camera_lin, chunks of <= CAM_CHUNK of each camera's observations, one
    // per workgroup; for the camera workgroups of k_schur_sweep, the
    // camera-major list cut into equal contiguous ranges (one per workgroup:
    // as many as the CUs the sweep leaves idle), each cut again at camera
    // boundaries
    const int cam_chunk = CAM_CHUNK;
    const int busy = sw.split_S ? NXCD * (sw.split_w0 + sw.split_n * sw.split_S) : sw.nspec * sw.nrange,
              idle = (256 - busy % 256) % 256;
    // the camera workgroups take the CUs the sweep's last round leaves idle;
    // when the dispatch tail is split there are none, and a full round of
    // them (256) beats a short one behind the split round
    p->cl_fused_wg = (int32_t)std::min<int64_t>(std::max<int64_t>(1, ceil_div(no, SW_THREADS)),
                                                sw.split_S ? 256 : idle >= 32 ? idle : 64);
    CamPlan csa, cfu;
    {
        std::vector<int32_t> cuts;
        for (int c = 0; c < nc; ++c)
            for (int32_t k = cstart[c]; k < cstart[c + 1]; k += cam_chunk) cuts.push_back(k);
        cuts.push_back((int32_t)no);
        plan_camera_items(nc, cstart, cuts, false, csa);
        cuts.clear();
        for (int g = 0; g <= p->cl_fused_wg; ++g) cuts.push_back((int32_t)(no * g / p->cl_fused_wg));
        plan_camera_items(nc, cstart, cuts, true, cfu);
    }
    p->ndiag_items = (int32_t)csa.items.size();
    p->ndiag_blocks = (int32_t)csa.blocks.size();
    p->cl_fused_items = (int32_t)cfu.items.size();
    p->sw_nrange = sw.nrange;
    p->sw_nspec = sw.nspec;
    p->sw_nbd = sw.nbd;
    p->sw_L = {sw.buf_slots, sw.pair_cap, sw.hdr_cap, sw.list_cap};
    p->sw_nchunk = sw.nchunk;
    p->sw_split = {NXCD * sw.split_w0, sw.split_S, sw.split_w0, sw.split_n, sw.split_gmax, nullptr};
    // + the end-of-range reduction: the accumulators and the group table
    p->sw_lds_bytes = std::max(sw.lds_bytes(), (size_t)SW_RED_W * SW_RED_LD * sizeof(double) +
                                                   (size_t)sw.hdr_cap * sizeof(SweepGroup));
    p->pt_blocks = std::max(1, ceil_div(np_ * PT_GROUP, PT_THREADS));
    p->payload_len = pay_vec_base(p->ns) + 3 * p->ns + 1;
    ctick("cam_items");
    // a digest of everything the planning produced, the (chunk, spec) lists
    // read back from the device (SFM_PLAN_DIGEST=1 or SFM_CREATE_TIMING=1;
    // the host and device planners must agree: tests/test_gpu_parity.py)
    const size_t nqw = (size_t)sw.nchunk * sw.nspec;
    auto plan_digest = [&](const int32_t *list, const uint16_t *pairs, const int32_t *hdr) {
        uint64_t h = 1469598103934665603ull;
        auto mix = [&](const void *d, size_t n) {
            const unsigned char *b = static_cast<const unsigned char *>(d);
            for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
        };
        auto mixv = [&](const auto &v) { mix(v.data(), v.size() * sizeof(v[0])); };
        mixv(pstart), mixv(cstart), mixv(cam_obs), mixv(cnt);
        mixv(sw.rchunk), mixv(sw.goff), mixv(sw.nload), mix(list, nqw * sw.list_cap * 4), mix(hdr, nqw * sw.hdr_cap * 4);
        mixv(sw.spec_cam), mixv(sw.split_of), mixv(sw.groups), mixv(sw.lanegrp), mix(pairs, nqw * sw.pair_cap * 2);
        mixv(sw.blkij);
        const int32_t sc[] = {sw.nrange, sw.nspec, sw.nbd, sw.buf_slots, sw.pair_cap, sw.hdr_cap, sw.list_cap,
                              sw.nchunk, sw.split_S, sw.split_w0, sw.split_n, sw.split_gmax, p->cl_fused_wg};
        mix(sc, sizeof sc);
        mixv(csa.items), mixv(csa.blocks), mixv(csa.wg_first), mixv(cfu.items), mixv(cfu.blocks), mixv(cfu.wg_first);
        return h;
    };
    if (plan_only) {
        if (want_digest)
            std::fprintf(stderr, "[create] plan digest %016llx\n",
                         (unsigned long long)plan_digest(sw.list.data(), sw.pairs.data(), sw.hdr.data()));
        return 1;
    }
    if ((rc = p->alloc(p->d_items, p->ndiag_items)) || (rc = p->alloc(p->d_blocks, p->ndiag_blocks)) ||
        (rc = p->alloc(p->d_wg_first, csa.wg_first.size())) || (rc = p->alloc(p->d_fitems, cfu.items.size())) ||
        (rc = p->alloc(p->d_fblocks, cfu.blocks.size())) || (rc = p->alloc(p->d_fwg_first, cfu.wg_first.size())) ||
        (rc = p->alloc(p->d_slab, (int64_t)ITEM_W * sw.nrange * sw.nbd)) ||
        (rc = p->alloc(p->sw_split.slabx, std::max<int64_t>(1, (int64_t)ITEM_W * sw.nrange * sw.split_S * sw.split_n *
                                                                   sw.split_gmax))) ||
        (rc = p->alloc(p->d_sw_split_of, sw.split_of.size())) ||
        (rc = p->alloc(p->d_sw_rchunk, sw.rchunk.size())) || (rc = p->alloc(p->d_sw_goff, sw.goff.size())) ||
        (rc = p->alloc(p->d_sw_nload, sw.nload.size())) ||
        (rc = p->alloc(p->d_sw_groups, sw.groups.size())) || (rc = p->alloc(p->d_sw_lanegrp, sw.lanegrp.size())) ||
        (rc = p->alloc(p->d_sw_list, (int64_t)(nqw * sw.list_cap))) ||
        (rc = p->alloc(p->d_sw_hdr, (int64_t)(nqw * sw.hdr_cap))) ||
        (rc = p->alloc(p->d_sw_pairs, (int64_t)(nqw * sw.pair_cap + 1) / 2)) ||
        (rc = p->alloc(p->d_sw_blkij, sw.blkij.size())) ||
        (rc = p->alloc(p->d_camlin, (int64_t)CAMLIN * nc)) ||
        (rc = p->alloc(p->d_slab2, (int64_t)CAMLIN * std::max<int64_t>(1, std::max(p->ndiag_items, p->cl_fused_items)))) ||
        (rc = p->alloc(p->d_Rt, 12 * (int64_t)nc)) || (rc = p->alloc(p->d_Rt2, 12 * (int64_t)nc)) ||
        (rc = p->alloc(p->d_X2, 3 * np_)) ||
        (rc = p->alloc(p->d_Vg, 9 * np_)) || (rc = p->alloc(p->d_Lq, 9 * np_)) ||
        (rc = p->alloc(p->d_sw_scam, sw.spec_cam.size())) || (rc = p->alloc(p->d_payload, p->payload_len + 8)) ||
        (rc = p->alloc(p->d_A, (int64_t)p->nsp * p->nsp)) || (rc = p->alloc(p->d_b, p->nsp)) ||
        (rc = p->alloc(p->d_D, 2 * 32 * 32)) ||
        (rc = p->alloc(p->d_partial, 4 * (int64_t)p->pt_blocks)) || (rc = p->alloc(p->d_scal, 16)) ||
        (rc = p->alloc(p->d_lm, 2)) ||
        (rc = p->alloc(p->d_bad, 4)) || (rc = p->alloc(p->d_sw_err, 1)) || (rc = p->alloc(p->d_count, 3 * GS_WORDS)) ||
        (rc = p->alloc(p->d_nbig, 1)) || (rc = p->alloc(p->d_gbuf, 6 * (int64_t)nc + 1)))
        return rc;
    p->gjrp = p->tb == 16 ? gjr_plan(p->nT, device_cus(device)) : GjrPlan{};
    p->gjp = p->tb == 16 && !p->gjrp.ok() ? gj_plan(p->nT, device_cus(device)) : GjPlan{};
    p->bs_cl_blocks = backsub_cl_blocks(nc, device_cus(device), p->pt_blocks);
    p->lin_cl_blocks = linearize_cl_blocks(nc, device_cus(device), p->pt_blocks);
    if (p->gjrp.ok()) {
        gjr::u64 *gw = nullptr;
        int *gi = nullptr;
        if ((rc = p->alloc(gw, (int64_t)GjrBufs::words(p->nT))) || (rc = p->alloc(gi, (int64_t)GjrBufs::ints)))
            return rc;
        p->gjrb.carve(gw, gi, p->nT);
        SFM_HIP(hipMemsetAsync(gw, 0, GjrBufs::words(p->nT) * sizeof(gjr::u64), p->stream));
        SFM_HIP(hipMemsetAsync(gi, 0, GjrBufs::ints * sizeof(int), p->stream));
        if (!p->ev_solve) SFM_HIP(hipEventCreateWithFlags(&p->ev_solve, hipEventDisableTiming));
    }
    if (p->gjp.cb) {
        double *gd = nullptr;
        int *gi = nullptr;
        if ((rc = p->alloc(gd, (int64_t)GjBufs::doubles(p->nT, p->gjp.nseg))) ||
            (rc = p->alloc(gi, (int64_t)GjBufs::ints(p->nT, p->gjp.nseg))))
            return rc;
        p->gjb.carve(gd, gi, p->nT, p->gjp.nseg);
        SFM_HIP(hipMemsetAsync(gi, 0, GjBufs::ints(p->nT, p->gjp.nseg) * sizeof(int), p->stream));
        if (!p->ev_solve) SFM_HIP(hipEventCreateWithFlags(&p->ev_solve, hipEventDisableTiming));
    }
    ctick("alloc");
    if (!p->h_ring) {
        SFM_HIP(hipHostMalloc((void **)&p->h_ring, kHostRing * sizeof(HostLM), hipHostMallocMapped | hipHostMallocCoherent));
        SFM_HIP(hipHostGetDevicePointer((void **)&p->d_ring, p->h_ring, 0));
    }
    std::memset((void *)p->h_ring, 0, kHostRing * sizeof(HostLM));
    hipStream_t s = p->stream;
    SFM_HIP(hipMemsetAsync(p->d_camlin, 0, (size_t)CAMLIN * nc * sizeof(double), s));
    SFM_HIP(hipMemsetAsync(p->d_count, 0, 3 * GS_WORDS * sizeof(unsigned), s));
    SFM_HIP(hipMemsetAsync(p->d_nbig, 0, sizeof(unsigned), s));
    if (p->ndiag_items) {
        SFM_HIP(hipMemcpyAsync(p->d_items, csa.items.data(), csa.items.size() * sizeof(PairItem), hipMemcpyHostToDevice, s));
        SFM_HIP(hipMemcpyAsync(p->d_blocks, csa.blocks.data(), csa.blocks.size() * sizeof(BlockInfo), hipMemcpyHostToDevice, s));
        SFM_HIP(hipMemcpyAsync(p->d_wg_first, csa.wg_first.data(), csa.wg_first.size() * 4, hipMemcpyHostToDevice, s));
        SFM_HIP(hipMemcpyAsync(p->d_fitems, cfu.items.data(), cfu.items.size() * sizeof(PairItem), hipMemcpyHostToDevice, s));
        SFM_HIP(hipMemcpyAsync(p->d_fblocks, cfu.blocks.data(), cfu.blocks.size() * sizeof(BlockInfo), hipMemcpyHostToDevice, s));
        SFM_HIP(hipMemcpyAsync(p->d_fwg_first, cfu.wg_first.data(), cfu.wg_first.size() * 4, hipMemcpyHostToDevice, s));
    }
    auto up = [&](void *dst, const void *src, size_t bytes) -> int {
        if (bytes) SFM_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
        return 0;
    };
    if ((rc = up(p->d_sw_rchunk, sw.rchunk.data(), sw.rchunk.size() * 4)) ||
        (rc = up(p->d_sw_goff, sw.goff.data(), sw.goff.size() * 4)) ||
        (rc = up(p->d_sw_nload, sw.nload.data(), sw.nload.size() * 4)) ||
        (rc = up(p->d_sw_groups, sw.groups.data(), sw.groups.size() * sizeof(SweepGroup))) ||
        (rc = up(p->d_sw_lanegrp, sw.lanegrp.data(), sw.lanegrp.size() * 2)) ||
        (rc = up(p->d_sw_scam, sw.spec_cam.data(), sw.spec_cam.size() * 4)) ||
        (rc = up(p->d_sw_blkij, sw.blkij.data(), sw.blkij.size() * sizeof(int2))) ||
        (rc = up(p->d_sw_split_of, sw.split_of.data(), sw.split_of.size() * 4)))
        return rc;
    if (sw.dev_lists) {  // the (chunk, spec) lists built on the device from the camera-major points
        int32_t *d_row = dev.scratch<int32_t>(sw.spec_row.size());
        if (dev.err) return dev.err;
        if ((rc = up(d_row, sw.spec_row.data(), sw.spec_row.size() * 4))) return rc;
        int mcols = 1;
        for (size_t w = 0; w < sw.spec_row.size() / 6; ++w)
            for (int rr = 0; rr < 2; ++rr) mcols = std::max(mcols, sw.spec_row[6 * w + 3 * rr + 2] - sw.spec_row[6 * w + 3 * rr + 1]);
        const int mw = (mcols + 31) / 32;
        const size_t lds = (size_t)sw.hdr_cap * 4 + (size_t)sw.buf_slots * mw * 4;
        SFM_HIP(hipFuncSetAttribute((const void *)k_plan_lists, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        if (nqw) {
            hipLaunchKernelGGL(k_plan_lists, dim3((unsigned)nqw), dim3(PLAN_THREADS), lds, s, sw.nchunk, sw.nspec,
                               (int32_t)np_, mw, dev.d_cut, p->d_pstart, p->d_pt, p->d_cam, p->d_cstart, p->d_cm_pt,
                               d_row, p->d_sw_goff, p->d_sw_groups, dev.d_bq, sw.list_cap, sw.pair_cap, sw.hdr_cap,
                               p->d_sw_list, reinterpret_cast<uint16_t *>(p->d_sw_pairs), p->d_sw_hdr);
            SFM_HIP(hipGetLastError());
        }
    } else if ((rc = up(p->d_sw_list, sw.list.data(), sw.list.size() * 4)) ||
               (rc = up(p->d_sw_hdr, sw.hdr.data(), sw.hdr.size() * 4)) ||
               (rc = up(p->d_sw_pairs, sw.pairs.data(), sw.pairs.size() * 2))) {
        return rc;
    }
    ctick("up:sweep");
    if (want_digest) {  // everything planned, the lists as the device holds them
        std::vector<int32_t> hl(nqw * sw.list_cap), hh(nqw * sw.hdr_cap);
        std::vector<uint16_t> hp(nqw * sw.pair_cap);
        SFM_HIP(hipMemcpyAsync(hl.data(), p->d_sw_list, hl.size() * 4, hipMemcpyDeviceToHost, s));
        SFM_HIP(hipMemcpyAsync(hh.data(), p->d_sw_hdr, hh.size() * 4, hipMemcpyDeviceToHost, s));
        SFM_HIP(hipMemcpyAsync(hp.data(), p->d_sw_pairs, hp.size() * 2, hipMemcpyDeviceToHost, s));
        SFM_HIP(hipStreamSynchronize(s));
        p->plan_digest = plan_digest(hl.data(), hp.data(), hh.data());
        if (ctm) std::fprintf(stderr, "[create] plan digest %016llx (%s lists)\n", (unsigned long long)p->plan_digest,
                              sw.dev_lists ? "device" : "host");
        ctick("digest");
    }
    if (ctm)
        std::fprintf(stderr, "[create] sweep arrays: list %.1f MB pairs %.1f MB hdr %.1f MB\n",
                     nqw * sw.list_cap * 4e-6, nqw * sw.pair_cap * 2e-6, nqw * sw.hdr_cap * 4e-6);
    SFM_HIP(hipFuncSetAttribute((const void *)k_schur_sweep<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)p->sw_lds_bytes));
    SFM_HIP(hipFuncSetAttribute((const void *)k_schur_sweep<1, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)p->sw_lds_bytes));
    SFM_HIP(hipFuncSetAttribute((const void *)k_schur_sweep<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)p->sw_lds_bytes));
    if ((rc = upload_state(p.get()))) return rc;
    ctick("upload");
    if (ctm) {
        SFM_HIP(hipStreamSynchronize(s));
        ctick("sync");
    }
    *out = p.release();
    return 0;
}

// the sweep plan's digest, computed at create with SFM_PLAN_DIGEST=1 (0
// otherwise): the device planner's lists against SFM_PLAN_HOST=1's
extern "C" int sfm_ba_plan_digest(sfm_ba_problem *p, uint64_t *out) {
    SFM_CHECK_ARG(p && out, "null pointer");
    *out = p->plan_digest;
    return 0;
}

extern "C" int sfm_ba_create(int32_t nc, int64_t np_, int64_t no, const int32_t *cam, const int32_t *pt,
                             const double *obs, const double *K, const double *cams, const double *pts, int device,
                             sfm_comm *comm, sfm_ba_problem **out) {
    return abi_guard("sfm_ba_create", [&] { return ba_create(nc, np_, no, cam, pt, obs, nullptr, K, cams, pts, device, comm, out); });
}

extern "C" int sfm_ba_reset(sfm_ba_problem *p) {
    SFM_CHECK_ARG(p, "null problem");
    SFM_HIP(hipSetDevice(p->device));
    return upload_state(p);
}

extern "C" int sfm_ba_destroy(sfm_ba_problem *p) {
    delete p;
    return 0;
}

static int local_allreduce(sfm_ba_problem *p, double *buf, int64_t n) {
    sfm_comm *c = p->comm;
    LocalGroup *g = c->local;
    std::vector<double> &mine = g->bufs[c->rank];
    mine.resize((size_t)n);
    // any failure on this rank aborts the group, so no rank waits for an
    // arrival that never comes
    auto abort_group = [&](int rc) {
        {
            std::lock_guard<std::mutex> lk(g->mu);
            g->aborted = true;
        }
        g->cv.notify_all();
        return rc;
    };
    auto aborted_err = [&]() {
        set_error("in-process all-reduce: another rank failed");
        return SFM_ERR_COMM;
    };
    if (hipMemcpyAsync(mine.data(), buf, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, p->stream) != hipSuccess ||
        hipStreamSynchronize(p->stream) != hipSuccess) {
        set_error("in-process all-reduce: device-to-host copy failed");
        return abort_group(SFM_ERR_HIP);
    }
    {
        std::unique_lock<std::mutex> lk(g->mu);
        if (g->aborted) return aborted_err();
        const long gen = g->generation;
        if (++g->arrived == g->nranks) {
            g->result.assign((size_t)n, 0.0);
            for (int r = 0; r < g->nranks; ++r)
                for (int64_t i = 0; i < n; ++i) g->result[i] += g->bufs[r][i];
            g->arrived = 0;
            g->generation++;
            g->cv.notify_all();
        } else {
            g->cv.wait(lk, [&] { return g->generation != gen || g->aborted; });
            if (g->aborted) return aborted_err();
        }
        if (hipMemcpyAsync(buf, g->result.data(), (size_t)n * sizeof(double), hipMemcpyHostToDevice, p->stream) !=
                hipSuccess ||
            hipStreamSynchronize(p->stream) != hipSuccess) {
            g->aborted = true;
            g->cv.notify_all();
            set_error("in-process all-reduce: host-to-device copy failed");
            return SFM_ERR_HIP;
        }
        // second rendezvous: nobody may overwrite `result` before all copied it
        const long gen2 = g->generation;
        if (++g->arrived == g->nranks) {
            g->arrived = 0;
            g->generation++;
            g->cv.notify_all();
        } else {
            g->cv.wait(lk, [&] { return g->generation != gen2 || g->aborted; });
            if (g->aborted) return aborted_err();
        }
    }
    return 0;
}

// RANSAC shard combine: max of the ranks' keys, then the
// winner's model (the rank whose key equals the max contributes it, the
// others zeros, summed).  Keys are unique across ranks when nonzero (the
// iteration is in the low word), so exactly one rank contributes.
extern "C" int sfm_ransac_combine(sfm_comm *c, uint64_t *key, double *model) {
    SFM_CHECK_ARG(c && key && model, "null pointer");
    if (c->local) {
        if (c->nranks == 1) return 0;
        LocalGroup *g = c->local;
        std::unique_lock<std::mutex> lk(g->mu);
        if (g->aborted) { set_error("in-process group aborted"); return SFM_ERR_COMM; }
        std::vector<double> &mine = g->bufs[c->rank];
        mine.assign(10, 0.0);
        std::memcpy(&mine[0], key, 8);
        std::memcpy(&mine[1], model, 72);
        const long gen = g->generation;
        if (++g->arrived == g->nranks) {
            uint64_t best = 0;
            int who = -1;
            for (int r = 0; r < g->nranks; ++r) {
                uint64_t k;
                std::memcpy(&k, &g->bufs[r][0], 8);
                if (k > best) { best = k; who = r; }
            }
            g->result.assign(10, 0.0);
            std::memcpy(&g->result[0], &best, 8);
            if (who >= 0) std::copy(g->bufs[who].begin() + 1, g->bufs[who].end(), g->result.begin() + 1);
            g->arrived = 0;
            g->generation++;
            g->cv.notify_all();
        } else {
            g->cv.wait(lk, [&] { return g->generation != gen || g->aborted; });
            if (g->aborted) { set_error("in-process group aborted"); return SFM_ERR_COMM; }
        }
        std::memcpy(key, &g->result[0], 8);
        if (*key != 0) std::memcpy(model, &g->result[1], 72);
        // second rendezvous: result stays intact until every rank has read it
        const long gen2 = g->generation;
        if (++g->arrived == g->nranks) {
            g->arrived = 0;
            g->generation++;
            g->cv.notify_all();
        } else {
            g->cv.wait(lk, [&] { return g->generation != gen2 || g->aborted; });
            if (g->aborted) { set_error("in-process group aborted"); return SFM_ERR_COMM; }
        }
        return 0;
    }
    // RCCL: also with a single rank, so one-GPU runs exercise the transport.
    // ONE all-gather of every rank's [key (u64 bits) | model (9 f64)] record,
    // entered by every rank whatever happened locally (a rank whose upload
    // fails contributes the neutral key 0 and reports its error after it):
    // no collective depends on a value read back on one rank only, so no
    // rank can skip one its peers are in.  Each rank then picks the largest
    // key (the reference's strict-> winner: max count, earliest iteration;
    // the ranges are disjoint, so keys of different ranks never tie unless
    // 0) and takes that rank's model bit for bit (-0.0 included): a copy,
    // not a sum.
    SFM_HIP(hipSetDevice(c->device));
    constexpr int REC = 10;
    if (!c->scratch) {
        SFM_HIP(hipMalloc(&c->scratch, sizeof(double) * REC * (c->nranks + 1)));
        SFM_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    }
    double *dmine = static_cast<double *>(c->scratch), *dall = dmine + REC;
    hipStream_t s = c->stream;
    int rc = 0;
    auto hip_ok = [&](hipError_t e) {
        if (e != hipSuccess && !rc) {
            set_error("ransac combine: %s", hipGetErrorString(e));
            rc = SFM_ERR_HIP;
        }
        return e == hipSuccess;
    };
    double h[REC];
    std::memcpy(&h[0], key, 8);
    std::memcpy(&h[1], model, 72);
    if (!hip_ok(hipMemcpyAsync(dmine, h, sizeof h, hipMemcpyHostToDevice, s)) || !hip_ok(hipStreamSynchronize(s)))
        (void)hipMemsetAsync(dmine, 0, sizeof h, s);
    const ncclResult_t nr = ncclAllGather(dmine, dall, REC, ncclDouble, c->comm, s);
    if (nr != ncclSuccess) {
        set_error("ncclAllGather(ransac keys): %s", ncclGetErrorString(nr));
        return SFM_ERR_COMM;
    }
    std::vector<double> all((size_t)REC * c->nranks);
    if (!hip_ok(hipMemcpyAsync(all.data(), dall, all.size() * sizeof(double), hipMemcpyDeviceToHost, s)) ||
        !hip_ok(hipStreamSynchronize(s)))
        return rc;
    uint64_t best = 0;
    int owner = -1;
    for (int r = 0; r < c->nranks; ++r) {
        uint64_t k;
        std::memcpy(&k, &all[(size_t)REC * r], 8);
        if (k > best) {
            best = k;
            owner = r;
        }
    }
    if (rc) return rc;
    if (owner >= 0) std::memcpy(model, &all[(size_t)REC * owner + 1], 72);
    *key = best;
    return 0;
}

static int allreduce(sfm_ba_problem *p, double *buf, int64_t n) {
    if (!p->comm) return 0;
    if (p->comm->local) return p->comm->nranks > 1 ? local_allreduce(p, buf, n) : 0;
    // RCCL: also with a single rank (an in-place no-op), so the transport
    // is exercised by the one-GPU tests
    ncclResult_t r = ncclAllReduce(buf, buf, (size_t)n, ncclDouble, ncclSum, p->comm->comm, p->stream);
    if (r != ncclSuccess) {
        set_error("ncclAllReduce: %s", ncclGetErrorString(r));
        return SFM_ERR_COMM;
    }
    return 0;
}

// camera_lin_wg's arguments: k_camera_lin's items (one per workgroup; direct
// when every camera is a single item) or the sweep's camera workgroups
static CamLinArgs camlin_args(const sfm_ba_problem *p, bool fused, const int *glin) {
    CamLinArgs a;
    a.items = fused ? p->d_fitems : p->d_items;
    a.wg_first = fused ? p->d_fwg_first : p->d_wg_first;
    a.cm_pt = p->d_cm_pt;
    a.cm_obs = p->d_cm_obs;
    a.X = p->d_X;
    a.Rt = p->d_Rt;
    a.Km = p->K;
    a.slab2 = p->d_slab2;
    a.blocks = fused ? p->d_fblocks : p->d_blocks;
    a.nblocks = p->ndiag_blocks;
    a.nwg = fused ? p->cl_fused_wg : p->ndiag_items;
    a.direct = !fused && p->ndiag_items == p->ndiag_blocks;
    a.camlin = p->d_camlin;
    a.counter = p->d_count + 2 * GS_WORDS;
    a.glin = glin;
    return a;
}

// launches one linearisation (J, V, g) and, into d_scal[8], the cost.
// want_cost: also sum the cost into d_scal[8] (the LM state takes it from
// the first linearisation only; later costs come from the accepted trials)
static int run_linearize(sfm_ba_problem *p, int par, int want_cost) {
    hipStream_t s = p->stream;
    const int *glin = &p->d_lm[par].run_lin;

    if (p->lin_cl_blocks > 0) {  // the cameras in LDS
        const int nb = std::max(1, std::min(ceil_div(p->np * LIN_CL_LANES, LIN_CL_THREADS), p->lin_cl_blocks));
        hipLaunchKernelGGL(k_linearize_cl<LIN_CL_LANES>, dim3(nb), dim3(LIN_CL_THREADS), (size_t)8 * LIN_CAM * p->nc, s,
                           p->np, p->nc, p->d_pstart, p->d_cam, p->d_obs, p->K, p->d_Rt, p->d_X, p->d_Vg, p->d_partial,
                           p->d_count, p->d_scal + 8, want_cost, glin, p->gtol, p->d_nbig);
        SFM_HIP(hipGetLastError());
        if (p->ndiag_items && !p->cl_fused) {
            const CamLinArgs cl = camlin_args(p, false, glin);
            hipLaunchKernelGGL(k_camera_lin<256>, dim3(p->ndiag_items), dim3(256), 0, s, cl);
            SFM_HIP(hipGetLastError());
        }
        return want_cost ? allreduce(p, p->d_scal + 8, 1) : 0;
    }
    const int nbl = std::max(1, ceil_div(p->np * LIN_LANES, PT_THREADS));
    hipLaunchKernelGGL(k_linearize<LIN_LANES>, dim3(nbl), dim3(PT_THREADS), 0, s, p->np, p->d_pstart, p->d_cam,
                       p->d_obs, p->K, p->d_Rt, p->d_X, p->d_Vg, p->d_partial, p->d_count, p->d_scal + 8, want_cost,
                       glin, p->gtol, p->d_nbig);
    SFM_HIP(hipGetLastError());
    if (p->ndiag_items && !p->cl_fused) {
        const CamLinArgs cl = camlin_args(p, false, glin);
        hipLaunchKernelGGL(k_camera_lin<256>, dim3(p->ndiag_items), dim3(256), 0, s, cl);
        SFM_HIP(hipGetLastError());
    }
    return want_cost ? allreduce(p, p->d_scal + 8, 1) : 0;
}

// one damped solve + trial evaluation (gated on the device LM state); leaves
// d_scal = [cost_trial, model_p, dn_p, xn_p, model_c, dn_c, xn_c] and d_bad for
// k_lm_step.  ev: this iteration's timing-event slot (nullable).
static int run_step(sfm_ba_problem *p, hipEvent_t *ev, int par) {
    hipStream_t s = p->stream;
    int rc;
    const bool timed = ev != nullptr;
    const int *gst = &p->d_lm[par].run_step;
    const double *lam = &p->d_lm[par].lambda;
    int *bad = p->d_bad + par;
    if (timed) SFM_HIP(hipEventRecord(ev[2 * T_PREP], s));
    hipLaunchKernelGGL(k_point_prep, dim3(std::max(1, ceil_div(p->np, OBS_THREADS))), dim3(OBS_THREADS), 0, s, (int64_t)p->np,
                       p->d_Vg, lam, p->d_Lq, gst);
    SFM_HIP(hipGetLastError());
    if (timed) SFM_HIP(hipEventRecord(ev[2 * T_PREP + 1], s));
    if (timed) SFM_HIP(hipEventRecord(ev[2 * T_SCHUR], s));
    const int nsweep = p->sw_split.S       ? p->sw_split.nfull + NXCD * p->sw_split.nsplit * p->sw_split.S
                       : p->sw_nrange < NXCD ? NXCD * ceil_div(p->sw_nspec, NXCD / p->sw_nrange)
                                             : NXCD * p->sw_nspec * ceil_div(p->sw_nrange, NXCD);
    const bool fused = p->cl_fused && p->ndiag_items;  // + the camera blocks (after an accepted step)
    auto sweep_k = p->sw_pinhole ? k_schur_sweep<1, true> : k_schur_sweep<1>;
    hipLaunchKernelGGL(sweep_k, dim3(nsweep + (fused ? p->cl_fused_wg : 0)), dim3(SW_THREADS),
                       p->sw_lds_bytes, s, p->sw_nspec, p->sw_nrange, p->sw_nbd, p->sw_L, p->d_sw_rchunk,
                       p->d_sw_nload, p->d_sw_goff, p->d_sw_groups, p->d_sw_lanegrp, p->d_sw_scam,
                       reinterpret_cast<const uint32_t *>(p->d_sw_list), p->d_sw_pairs, p->d_sw_hdr, p->d_X, p->d_Lq,
                       p->d_Rt, p->K, p->d_slab, gst, p->sw_debug, nsweep,
                       camlin_args(p, true, &p->d_lm[par].run_lin), sw_dbg_ptr(), p->d_sw_err, p->sw_split);
    SFM_HIP(hipGetLastError());
    // one rank: the solve's first launch sums the slabs itself (SlabSrc)
    // (the persistent solve reads the finished payload: the finish runs as its own launch)
    // (the row-distributed solve only with SFM_GJR_FOLD=1: its prologue then
    // reads 8 range slabs per element while the chain runs, cfg5 solve 0.457
    // -> 0.523 ms against the finish's 0.028 ms, round 4)
    const bool fin_fused = !p->comm && p->fin_fused && !p->gjp.cb && (!p->gjrp.ok() || p->gjr_fold);
    if (!fin_fused) {
        hipLaunchKernelGGL(k_schur_finish, dim3(ceil_div(p->sw_nbd * ITEM_W, FIN_THREADS)), dim3(FIN_THREADS), 0, s, p->ns, p->sw_nbd, p->sw_nrange,
                           p->d_sw_blkij, p->d_slab, p->d_camlin, p->d_payload, gst, p->d_sw_split_of, p->sw_split);
        SFM_HIP(hipGetLastError());
    }
    if (timed) SFM_HIP(hipEventRecord(ev[2 * T_SCHUR + 1], s));
    if (timed) SFM_HIP(hipEventRecord(ev[2 * T_COMM], s));
    if ((rc = allreduce(p, p->d_payload, p->payload_len - 1))) return rc;
    if (timed) SFM_HIP(hipEventRecord(ev[2 * T_COMM + 1], s));
    if (timed) SFM_HIP(hipEventRecord(ev[2 * T_SOLVE], s));
    // the back substitution's epilogue forms the trial cameras (k_camera_trial's work)
    const CamTrialArgs ct = {p->nc, p->ns, p->d_payload, lam, p->d_Rt, p->d_Rt2, p->d_scal + 4};
    const SlabSrc src = fin_fused ? SlabSrc{p->d_slab, p->d_camlin, p->sw_nbd, p->sw_nrange, p->sw_split, p->d_sw_split_of}
                                  : SlabSrc{nullptr, nullptr, 0, 0, {}, nullptr};
    if (p->gjp.cb || p->gjrp.ok()) {
        LocalGroup *lg = p->comm ? p->comm->local : nullptr;
        std::unique_lock<std::mutex> lk;
        if (lg) {  // in-process ranks on one GPU: one persistent solve at a time
            lk = std::unique_lock<std::mutex>(lg->solve_mu);
            if (lg->last_solve) SFM_HIP(hipStreamWaitEvent(s, lg->last_solve, 0));
        }
        if (p->gjrp.ok()) {
            if ((rc = launch_gjr(p->gjrp, p->ns, p->d_payload, lam, p->gjrb, ++p->gjr_tag, p->d_b, bad, gst, ct, s,
                                 src)))
                return rc;
        } else if ((rc = launch_gj(p->gjp, p->nT, p->ns, p->d_payload, lam, p->gjb, ++p->gj_epoch, p->d_b, bad,
                                   gst, ct, s)))
            return rc;
        if (lg) {
            SFM_HIP(hipEventRecord(p->ev_solve, s));
            lg->last_solve = p->ev_solve;
        }
    } else if ((rc = launch_reduced_solve(p->ns, p->nsp, p->d_payload, lam, p->d_A, p->d_b, p->d_D, bad, s, p->tb,
                                          gst, ct, src, p->chol_dpp)))
        return rc;
    if (timed) SFM_HIP(hipEventRecord(ev[2 * T_SOLVE + 1], s));
    if (timed) SFM_HIP(hipEventRecord(ev[2 * T_TRIAL], s));
    // grid-stride: 1024 workgroups (4 per CU); measured at cfg4 (1563 needed
    // without the stride): 512 -> 49 us, 896..1152 -> 43 us, 2048+ -> 51 us
    // with the cameras in LDS: as many workgroups as are resident at once
    // (a grid-stride kernel whose last workgroups start late ends late)
    const bool cl = p->bs_cl_blocks > 0;
    const int bst = cl ? 256 : PT_THREADS;
    const int nbb = std::max(1, std::min(ceil_div(p->np * BS_LANES, bst), cl ? p->bs_cl_blocks : 1024));
    const size_t cl_lds = cl ? (size_t)8 * BS_CAM * p->nc : 0;
    hipLaunchKernelGGL((cl ? k_backsub_trial<BS_LANES, true, 256> : k_backsub_trial<BS_LANES, false>), dim3(nbb),
                       dim3(bst), cl_lds, s, p->np, p->nc, p->d_pstart, p->d_cam, p->d_obs, p->K, p->d_Vg, p->d_Lq,
                       p->d_b, lam, p->d_Rt, p->d_Rt2, p->d_X, p->d_X2, p->d_partial, p->d_count + GS_WORDS, p->d_scal,
                       gst);
    SFM_HIP(hipGetLastError());
    if ((rc = allreduce(p, p->d_scal, 4))) return rc;
    if (timed) SFM_HIP(hipEventRecord(ev[2 * T_TRIAL + 1], s));
    return 0;
}

// Wait until iteration j's k_lm_step has published its LM state to the
// pinned ring.  A stream that stopped with an error, or drained without the
// state arriving, ends the wait with an error instead of spinning forever.
static int wait_lm_state(sfm_ba_problem *p, int j) {
    const int *seq = &p->h_ring[j % kHostRing].seq;
    for (unsigned spin = 1;; ++spin) {
        if (__atomic_load_n(seq, __ATOMIC_ACQUIRE) == j + 1) return 0;
        if (spin % 256 == 0) {
            const hipError_t q = hipStreamQuery(p->stream);
            if (q == hipErrorNotReady) {
                std::this_thread::yield();
                continue;
            }
            if (__atomic_load_n(seq, __ATOMIC_ACQUIRE) == j + 1) return 0;
            set_error("LM iteration %d: state not published (%s)", j, hipGetErrorString(q));
            return SFM_ERR_HIP;
        }
    }
}

// Per-phase HIP events in sfm_ba_solve (sfm_ba_kernel_times); off by default
// (each event record costs the stream a few microseconds).
extern "C" int sfm_ba_set_timing(sfm_ba_problem *p, int on) {
    SFM_CHECK_ARG(p, "null pointer");
    p->timing = on != 0;
    return 0;
}

extern "C" int sfm_ba_solve(sfm_ba_problem *p, const sfm_ba_opts *o, sfm_ba_report *rep) {
    SFM_CHECK_ARG(p && o, "null pointer");
    SFM_CHECK_ARG(o->max_iterations >= 0, "max_iterations < 0");
    SFM_CHECK_ARG(o->gradient_tolerance >= 0.0, "gradient_tolerance < 0");
    SFM_HIP(hipSetDevice(p->device));
    p->gtol = o->gradient_tolerance;
    // camera blocks inside the sweep launch, except when gradient_tolerance
    // needs g_c right after the linearisation
    p->cl_fused = o->gradient_tolerance == 0.0 && env_int("SFM_CAMLIN_FUSED", 1) != 0;
    // A/B switches (read per solve): DPP tile factor, finish folded into the solve
    p->chol_dpp = env_int("SFM_CHOL_DPP", 1) != 0;
    p->fin_fused = env_int("SFM_FINISH_FUSED", 1) != 0;
    p->gjr_fold = env_int("SFM_GJR_FOLD", 0) != 0;
    (void)hipGetLastError();
    const auto t0 = std::chrono::steady_clock::now();
    for (double &t : p->t_acc) t = 0;
    p->t_iters = 0;
    hipStream_t s = p->stream;
    int rc;
    // The host enqueues iteration it once it has read the published state of
    // iteration it - depth (pinned ring, no stream sync), so at most depth
    // gated-off iterations follow the one that ends the solve, and the device
    // always has the next iteration queued.
    constexpr int depth = 2;
    static_assert(depth >= 1 && depth < kHostRing, "the host ring holds the iterations in flight");
    const bool timed = p->timing;
    for (int k = 0; k < kHostRing; ++k) __atomic_store_n(&p->h_ring[k].seq, 0, __ATOMIC_RELAXED);
    hipLaunchKernelGGL(k_lm_reset, dim3(1), dim3(1), 0, s, p->d_lm, o->initial_lambda, p->d_bad);
    SFM_HIP(hipGetLastError());
    // the persistent solves' error and arrival words start clean every solve
    // (an aborted launch may have left an arrival count behind)
    if (p->gjp.cb) {
        SFM_HIP(hipMemsetAsync(p->gjb.err, 0, sizeof(int), s));
        SFM_HIP(hipMemsetAsync(p->gjb.arrive, 0, sizeof(unsigned), s));
    }
    if (p->gjrp.ok()) SFM_HIP(hipMemsetAsync(p->gjrb.err, 0, GjrBufs::ints * sizeof(int), s));
    SFM_HIP(hipMemsetAsync(p->d_sw_err, 0, sizeof(int), s));
    auto account = [&](int j) {  // per-phase event times of iteration j (complete once its state is published)
        const hipEvent_t *e = p->ev_it + (size_t)(j % kEvSlots) * 2 * T_NT;
        for (int k = 0; k < T_NT; ++k) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, e[2 * k], e[2 * k + 1]) == hipSuccess) p->t_acc[k] += ms;
        }
        p->t_iters++;
    };
    const int64_t nacc = std::max<int64_t>(3 * p->np, 12 * (int64_t)p->nc);
    int it = 0;
    for (; it < o->max_iterations; ++it) {
        if (it >= depth) {
            const int j = it - depth;
            if ((rc = wait_lm_state(p, j))) return rc;
            const LMState &st = p->h_ring[j % kHostRing].st;
            if (timed && st.iters == j + 1) account(j);
            if (st.done) break;
        }
        hipEvent_t *ev = timed ? p->ev_it + (size_t)(it % kEvSlots) * 2 * T_NT : nullptr;
        if (timed) SFM_HIP(hipEventRecord(ev[2 * T_LIN], s));
        const int par = it & 1;  // the state of iteration it lives in d_lm[par]
        if ((rc = run_linearize(p, par, it == 0))) return rc;
        if (timed) SFM_HIP(hipEventRecord(ev[2 * T_LIN + 1], s));
        if (it == 0) {
            hipLaunchKernelGGL(k_lm_init, dim3(1), dim3(1), 0, s, p->d_lm, p->d_scal + 8);
            SFM_HIP(hipGetLastError());
        }
        if (o->gradient_tolerance > 0.0) {
            const int *glin = &p->d_lm[par].run_lin;
            hipLaunchKernelGGL(k_gtol_pack, dim3(1), dim3(256), 0, s, p->nc, p->d_camlin, p->d_nbig, p->d_gbuf, glin);
            SFM_HIP(hipGetLastError());
            if ((rc = allreduce(p, p->d_gbuf, 6 * (int64_t)p->nc + 1))) return rc;
            hipLaunchKernelGGL(k_gtol_check, dim3(1), dim3(256), 0, s, p->nc, o->gradient_tolerance, p->d_gbuf,
                               p->d_lm + par, glin);
            SFM_HIP(hipGetLastError());
        }
        if ((rc = run_step(p, ev, par))) return rc;
        // bounded grid, grid-stride copy: after a rejected step nothing is copied
        hipLaunchKernelGGL(k_lm_step, dim3(std::min(ceil_div(nacc, 256), 512)), dim3(256), 0, s, p->d_lm + par,
                           p->d_lm + (par ^ 1),
                           p->d_scal, p->d_bad + par, p->d_bad + (par ^ 1), o->max_iterations, o->fixed_iterations,
                           o->function_tolerance, o->parameter_tolerance, o->initial_lambda, p->np, p->nc, p->d_X,
                           p->d_X2, p->d_Rt, p->d_Rt2, p->d_ring, it + 1);
        SFM_HIP(hipGetLastError());
    }
    // the iterations still in flight (gated off if the solve ended earlier)
    LMState h{};
    int gj_err = 0;
    SFM_HIP(hipMemcpyAsync(&h, p->d_lm + (it & 1), sizeof h, hipMemcpyDeviceToHost, s));
    if (p->gjp.cb) SFM_HIP(hipMemcpyAsync(&gj_err, p->gjb.err, sizeof gj_err, hipMemcpyDeviceToHost, s));
    if (p->gjrp.ok()) SFM_HIP(hipMemcpyAsync(&gj_err, p->gjrb.err, sizeof gj_err, hipMemcpyDeviceToHost, s));
    int sw_err = 0;
    SFM_HIP(hipMemcpyAsync(&sw_err, p->d_sw_err, sizeof sw_err, hipMemcpyDeviceToHost, s));
    SFM_HIP(hipStreamSynchronize(s));
    if (sw_err) {
        set_error("Schur sweep: a workgroup timed out waiting for a chunk hand-off");
        return SFM_ERR_HIP;
    }
    if (gj_err) {
        set_error("reduced camera solve: a workgroup of the persistent solve timed out waiting for a panel");
        return SFM_ERR_HIP;
    }
    if (timed)
        for (int j = std::max(0, it - depth); j < it && j < h.iters; ++j)
            if (p->h_ring[j % kHostRing].st.iters == j + 1) account(j);
    const auto t1 = std::chrono::steady_clock::now();
    if (rep) {
        rep->iterations = h.iters;
        rep->accepted = h.accepted;
        rep->status = h.status;
        rep->n_ranks = p->comm ? p->comm->nranks : 1;
        rep->cost0 = h.cost0;
        rep->cost = h.cost;
        rep->t_loop_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        rep->lambda = h.lambda;
    }
    return 0;
}

// Diagnostic entry: solves the SPD system S x = rhs (n x n, row-major) with
// the reduced-camera solver of sfm_ba_solve (tiled Cholesky).
// Diagnostic: the published panels of this thread's last persistent reduced
// solve (sfm_reduced_solve): G [nT][nsp][16], L [nT][nseg][256], y [nT][nseg][16].
extern "C" int sfm_gj_dump(double *G, double *L, double *Y, int32_t nT, int32_t nseg, int device) {
    SFM_CHECK_ARG(G && L && Y, "null pointer");
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    SFM_CHECK_ARG(c->buf[5].bytes >= GjBufs::doubles(nT, nseg) * sizeof(double), "no such solve");
    GjBufs b;
    b.carve(c->buf[5].as<double>(), c->buf[6].as<int>(), nT, nseg);
    SFM_HIP(hipStreamSynchronize(c->stream));
    SFM_HIP(hipMemcpy(G, b.G, (size_t)nT * nT * 256 * sizeof(double), hipMemcpyDeviceToHost));
    SFM_HIP(hipMemcpy(L, b.L, (size_t)nT * nseg * 256 * sizeof(double), hipMemcpyDeviceToHost));
    SFM_HIP(hipMemcpy(Y, b.Y, (size_t)nT * nseg * 16 * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int sfm_reduced_solve(const double *S, const double *rhs, int32_t n, double *x, int device) {
    SFM_CHECK_ARG(S && rhs && x, "null pointer");
    SFM_CHECK_ARG(n >= 1, "n < 1");
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    const int tb = chol_tile(n);
    const int32_t nsp = (n + tb - 1) / tb * tb;
    const GjrPlan gjrp = tb == 16 ? gjr_plan(nsp / 16, device_cus(device)) : GjrPlan{};
    const GjPlan gjp = tb == 16 && !gjrp.ok() ? gj_plan(nsp / 16, device_cus(device)) : GjPlan{};
    int rc;
    const size_t pb = (size_t)pay_vec_base(n);
    if ((rc = c->buf[0].reserve((pb + 3 * (size_t)n + 1) * sizeof(double))) ||
        (rc = c->buf[1].reserve((size_t)nsp * nsp * sizeof(double))) ||
        (rc = c->buf[2].reserve((size_t)nsp * sizeof(double))) ||
        (rc = c->buf[3].reserve(2 * 32 * 32 * sizeof(double))) || (rc = c->buf[4].reserve(sizeof(int))))
        return rc;
    // payload = [S (upper camera blocks), diag U = 0, g = -rhs, sum Z q = 0], lambda = 0 (last slot)
    std::vector<double> pay(pb + 3 * (size_t)n + 1, 0.0);
    for (int32_t i = 0; i < n; ++i)
        for (int32_t j = 0; j < n; ++j)
            if (i / 6 <= j / 6) pay[pay_index(n, i, j)] = S[(size_t)i * n + j];
    for (int32_t i = 0; i < n; ++i) pay[pb + n + i] = -rhs[i];
    double *d_pay = c->buf[0].as<double>();
    SFM_HIP(hipMemcpyAsync(d_pay, pay.data(), pay.size() * sizeof(double), hipMemcpyHostToDevice, c->stream));
    SFM_HIP(hipMemsetAsync(c->buf[4].p, 0, sizeof(int), c->stream));
    if (gjrp.ok()) {
        const int nT = nsp / 16;
        if ((rc = c->buf[7].reserve(GjrBufs::words(nT) * sizeof(gjr::u64))) ||
            (rc = c->buf[8].reserve(GjrBufs::ints * sizeof(int))))
            return rc;
        // records zeroed whenever the buffer or the layout changes: tags restart
        if (c->buf[7].p != c->gjr_words || c->gjr_nT != nT) {
            SFM_HIP(hipMemsetAsync(c->buf[7].p, 0, c->buf[7].bytes, c->stream));
            c->gjr_words = c->buf[7].p;
            c->gjr_nT = nT;
            c->gjr_tag = 0;
        }
        GjrBufs b;
        b.carve(c->buf[7].as<gjr::u64>(), c->buf[8].as<int>(), nT);
        SFM_HIP(hipMemsetAsync(b.err, 0, GjrBufs::ints * sizeof(int), c->stream));
        SFM_HIP(hipMemsetAsync(c->buf[2].p, 0, (size_t)nsp * sizeof(double), c->stream));
        if ((rc = launch_gjr(gjrp, n, d_pay, d_pay + pb + 3 * (size_t)n, b, ++c->gjr_tag, c->buf[2].as<double>(),
                             c->buf[4].as<int>(), nullptr, CamTrialArgs{}, c->stream)))
            return rc;
        int err = 0;
        SFM_HIP(hipMemcpyAsync(&err, b.err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        SFM_HIP(hipStreamSynchronize(c->stream));
        if (err) {
            set_error("reduced solve: the persistent solve timed out");
            return SFM_ERR_HIP;
        }
    } else if (gjp.cb) {
        const int nT = nsp / 16;
        const size_t nint = GjBufs::ints(nT, gjp.nseg);
        if ((rc = c->buf[5].reserve(GjBufs::doubles(nT, gjp.nseg) * sizeof(double))) ||
            (rc = c->buf[6].reserve(nint * sizeof(int))))
            return rc;
        // fresh flags: zero them once, epochs restart.  A regrown buffer can
        // come back at the same address, and a new layout moves the flags
        // and the arrival word: either way the old words mean nothing
        if (c->buf[6].p != c->gj_ints || c->gj_nT != nT || c->gj_nseg != gjp.nseg) {
            SFM_HIP(hipMemsetAsync(c->buf[6].p, 0, c->buf[6].bytes, c->stream));
            c->gj_ints = c->buf[6].p;
            c->gj_nT = nT;
            c->gj_nseg = gjp.nseg;
            c->gj_epoch = 0;
        }
        GjBufs b;
        b.carve(c->buf[5].as<double>(), c->buf[6].as<int>(), nT, gjp.nseg);
        SFM_HIP(hipMemsetAsync(b.err, 0, sizeof(int), c->stream));
        SFM_HIP(hipMemsetAsync(b.arrive, 0, sizeof(unsigned), c->stream));  // an aborted launch may have left a count
        SFM_HIP(hipMemsetAsync(c->buf[2].p, 0, (size_t)nsp * sizeof(double), c->stream));
        if ((rc = launch_gj(gjp, nT, n, d_pay, d_pay + pb + 3 * (size_t)n, b,
                            ++c->gj_epoch, c->buf[2].as<double>(), c->buf[4].as<int>(), nullptr, CamTrialArgs{},
                            c->stream)))
            return rc;
        int err = 0;
        SFM_HIP(hipMemcpyAsync(&err, b.err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        SFM_HIP(hipStreamSynchronize(c->stream));
        if (err) {
            set_error("reduced solve: the persistent solve timed out");
            return SFM_ERR_HIP;
        }
    } else if ((rc = launch_reduced_solve(n, nsp, d_pay, d_pay + pb + 3 * (size_t)n, c->buf[1].as<double>(),
                                          c->buf[2].as<double>(), c->buf[3].as<double>(), c->buf[4].as<int>(),
                                          c->stream, tb, nullptr, CamTrialArgs{})))
        return rc;
    int bad = 0;
    SFM_HIP(hipMemcpyAsync(x, c->buf[2].p, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    SFM_HIP(hipMemcpyAsync(&bad, c->buf[4].p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    SFM_HIP(hipStreamSynchronize(c->stream));
    if (bad) {
        set_error("reduced camera system not positive definite");
        return SFM_ERR_SOLVE;
    }
    return 0;
}

extern "C" int sfm_ba_download(sfm_ba_problem *p, double *cams, double *pts) {
    SFM_CHECK_ARG(p, "null problem");
    SFM_HIP(hipSetDevice(p->device));
    std::vector<double> Rt(12 * (size_t)p->nc);
    SFM_HIP(hipMemcpyAsync(Rt.data(), p->d_Rt, Rt.size() * 8, hipMemcpyDeviceToHost, p->stream));
    if (pts && p->np) SFM_HIP(hipMemcpyAsync(pts, p->d_X, (size_t)p->np * 24, hipMemcpyDeviceToHost, p->stream));
    SFM_HIP(hipStreamSynchronize(p->stream));
    if (cams)
        for (int c = 0; c < p->nc; ++c) {
            h_R_to_rotvec(&Rt[12 * c], cams + 6 * c);
            for (int i = 0; i < 3; ++i) cams[6 * c + 3 + i] = Rt[12 * c + 9 + i];
        }
    return 0;
}

extern "C" int sfm_ba_kernel_times(sfm_ba_problem *p, double *ms, int n, char *names, int names_len) {
    SFM_CHECK_ARG(p, "null problem");
    const int m = std::min(n, (int)T_NT);
    for (int k = 0; k < m; ++k) ms[k] = p->t_iters ? p->t_acc[k] / p->t_iters : 0.0;
    if (names && names_len > 0) {
        std::strncpy(names, kTimerNames, names_len - 1);
        names[names_len - 1] = 0;
    }
    return m;
}

static int ba_lm(int32_t nc, int64_t np_, int64_t no, const int32_t *cam, const int32_t *pt, const double *obs,
                 void *dense, const double *K, double *cams, double *pts, const sfm_ba_opts *o, sfm_ba_report *rep,
                 int device) {
    SFM_CHECK_ARG(o && cams, "null pointer");
    const auto t0 = std::chrono::steady_clock::now();
    sfm_ba_problem *p = nullptr;
    int rc = ba_create(nc, np_, no, cam, pt, obs, dense, K, cams, pts, device, nullptr, &p, true);
    if (rc) return rc;
    const auto t1 = std::chrono::steady_clock::now();
    rc = sfm_ba_solve(p, o, rep);
    const auto t2 = std::chrono::steady_clock::now();
    if (!rc) rc = sfm_ba_download(p, cams, pts);
    const auto t3 = std::chrono::steady_clock::now();
    if (rep) {
        rep->t_setup_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        rep->t_download_ms = std::chrono::duration<double, std::milli>(t3 - t2).count();
    }
    sfm_ba_destroy(p);
    return rc;
}

extern "C" int sfm_ba_lm(int32_t nc, int64_t np_, int64_t no, const int32_t *cam, const int32_t *pt,
                         const double *obs, const double *K, double *cams, double *pts, const sfm_ba_opts *o,
                         sfm_ba_report *rep, int device) {
    return abi_guard("sfm_ba_lm", [&] { return ba_lm(nc, np_, no, cam, pt, obs, nullptr, K, cams, pts, o, rep, device); });
}

// perform_bundle_adjustment from the dense scan (sfm_dense_obs_scan's
// handle, not freed here): the observations go from the scan's pieces into
// the pinned upload buffer, never through COO arrays
extern "C" int sfm_ba_lm_dense(void *obs_handle, int32_t nc, int64_t np_, const double *K, double *cams, double *pts,
                               const sfm_ba_opts *o, sfm_ba_report *rep, int device) {
    int64_t no, nrows;
    int32_t ncams;
    SFM_CHECK_ARG(dense_obs_info(obs_handle, &no, &nrows, &ncams), "null observation handle");
    SFM_CHECK_ARG(nrows == np_ && ncams <= nc, "the scan's rows / cameras do not match the problem");
    return abi_guard("sfm_ba_lm_dense",
                     [&] { return ba_lm(nc, np_, no, nullptr, nullptr, nullptr, obs_handle, K, cams, pts, o, rep, device); });
}

// Single-process multi-GPU bundle adjustment: points (with their
// observations) are split into contiguous ranges over the listed devices,
// one host thread per rank, reduced camera system summed every iteration
// through an in-process group (sfm_comm_init_local).  The same partition
// as the one-process-per-GPU RCCL path (structure-from-motion-_amd/sfm_dist.py).
extern "C" int sfm_ba_lm_multi(int32_t nc, int64_t np_, int64_t no, const int32_t *cam, const int32_t *pt,
                               const double *obs, const double *K, double *cams, double *pts, const sfm_ba_opts *o,
                               sfm_ba_report *rep, const int *devices, int n_ranks) {
    SFM_CHECK_ARG(o && cams && devices && n_ranks >= 1, "null pointer / no devices");
    for (int64_t i = 1; i < no; ++i) SFM_CHECK_ARG(pt[i] >= pt[i - 1], "observations must be point-major");
    std::vector<sfm_comm *> comms(n_ranks, nullptr);
    int rc = sfm_comm_init_local(n_ranks, comms.data());
    if (rc) return rc;
    std::vector<int> rcs(n_ranks, 0);
    std::vector<std::string> errs(n_ranks);
    std::vector<sfm_ba_report> reps(n_ranks);
    std::vector<double> cams_out(6 * (size_t)nc);
    auto worker = [&](int r) {
        const int64_t lo = np_ * r / n_ranks, hi = np_ * (r + 1) / n_ranks;
        const int64_t o0 = std::lower_bound(pt, pt + no, (int32_t)lo) - pt;
        const int64_t o1 = std::lower_bound(pt, pt + no, (int32_t)hi) - pt;
        std::vector<int32_t> lpt(pt + o0, pt + o1);
        for (auto &v : lpt) v -= (int32_t)lo;
        sfm_ba_problem *p = nullptr;
        int e = sfm_ba_create(nc, hi - lo, o1 - o0, cam + o0, lpt.data(), obs + 2 * o0, K, cams, pts + 3 * lo,
                              devices[r], comms[r], &p);
        if (!e) e = sfm_ba_solve(p, o, &reps[r]);
        if (!e) e = sfm_ba_download(p, r == 0 ? cams_out.data() : nullptr, pts + 3 * lo);
        if (p) sfm_ba_destroy(p);
        rcs[r] = e;
        if (e) {
            errs[r] = sfm_last_error();
            // a rank that fails outside the all-reduce (create, a launch)
            // releases the ranks waiting for it there
            LocalGroup *g = comms[r]->local;
            {
                std::lock_guard<std::mutex> lk(g->mu);
                g->aborted = true;
            }
            g->cv.notify_all();
        }
    };
    std::vector<std::thread> th;
    for (int r = 0; r < n_ranks; ++r) th.emplace_back(worker, r);
    for (auto &t : th) t.join();
    for (auto *c : comms) sfm_comm_destroy(c);
    // report the first rank that failed on its own (not the SFM_ERR_COMM of
    // the ranks it released)
    for (int pass = 0; pass < 2; ++pass)
        for (int r = 0; r < n_ranks; ++r)
            if (rcs[r] && (pass == 1 || rcs[r] != SFM_ERR_COMM)) {
                set_error("rank %d: %s", r, errs[r].c_str());
                return rcs[r];
            }
    std::memcpy(cams, cams_out.data(), cams_out.size() * sizeof(double));
    if (rep) *rep = reps[0];
    return 0;
}
