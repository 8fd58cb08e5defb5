// Device helper shared by the RANSAC engine and PnP RANSAC: the winner of a
// table of per-hypothesis inlier counts (Phase 1/GetInliersRANSAC.py:85,
// Phase 1/PnPRANSAC.py:72: the strict '>' update over ascending iterations).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace sfm {

// (count, iteration) winner of a RANSAC table, by one workgroup of NT
// threads: the reference's strict '>' update over ascending iterations ==
// max count, then the smallest iteration among equal positive counts.
// Every load of a pass is issued before any is used (8 counts per thread in
// flight) and the reduction runs in registers (shuffles within a wave, then
// one wave over the wave results).  Returns (count, iteration or -1) to
// every thread; sc / sh: LDS of NT / 64 entries.
__device__ __forceinline__ void sel_merge(int32_t &c1, int64_t &h1, int32_t c2, int64_t h2) {
    if (c2 > c1 || (c2 == c1 && c2 > 0 && h2 < h1)) {
        c1 = c2;
        h1 = h2;
    }
}

template <int NT>
__device__ __forceinline__ void wg_select_best(const int32_t *__restrict__ counts, int64_t H, int32_t *sc,
                                               int64_t *sh, int32_t &best_c, int64_t &best_h) {
    constexpr int CU = 8;
    const int t = threadIdx.x;
    int32_t bc = 0;
    int64_t bh = -1;
    for (int64_t base = t; base < H; base += (int64_t)CU * NT) {
        int32_t c[CU];
#pragma unroll
        for (int u = 0; u < CU; ++u) {
            const int64_t h = base + (int64_t)u * NT;
            c[u] = h < H ? counts[h] : 0;
        }
#pragma unroll
        for (int u = 0; u < CU; ++u)  // ascending h per thread: first max kept
            if (c[u] > bc) { bc = c[u]; bh = base + (int64_t)u * NT; }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const int32_t c2 = __shfl_xor(bc, off);
        const int64_t h2 = __shfl_xor(bh, off);
        sel_merge(bc, bh, c2, h2);
    }
    if ((t & 63) == 0) { sc[t >> 6] = bc; sh[t >> 6] = bh; }
    __syncthreads();
    bc = (t & 63) < NT / 64 ? sc[t & 63] : 0;
    bh = (t & 63) < NT / 64 ? sh[t & 63] : -1;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {  // every wave, so every thread has the result
        const int32_t c2 = __shfl_xor(bc, off);
        const int64_t h2 = __shfl_xor(bh, off);
        sel_merge(bc, bh, c2, h2);
    }
    best_c = bc;
    best_h = bc > 0 ? bh : -1;
}

}  // namespace sfm
