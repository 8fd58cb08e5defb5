// Microbenchmark: where the 8-point fit's ~9 us per launch goes.
//   per-launch time (50 back-to-back launches of 4096 hypotheses) with the
//   sample rows in pinned host memory (as in the product) or in HBM, and
//   per-stage timestamps (s_memrealtime, 100 MHz) of one thread per wave:
//   loads, Hartley + design matrix, null vector, rank 2 + denormalisation.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstring>
#include "../structure-from-motion-_amd/csrc/sfm_geom.hpp"

using namespace sfm;

template <bool STAMP, class IDX>
__global__ void __launch_bounds__(64) k_fit(const double2 *__restrict__ x1, const double2 *__restrict__ x2,
                                            const IDX *__restrict__ samples, int H, double *__restrict__ out,
                                            long long *__restrict__ st) {
    const int h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= H) return;
    long long t[5];
    if (STAMP) t[0] = wall_clock64();
    double ax[8], ay[8], bx[8], by[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int32_t s = (int32_t)samples[h * 8 + i];
        const double2 p = x1[s], q = x2[s];
        ax[i] = p.x; ay[i] = p.y; bx[i] = q.x; by[i] = q.y;
    }
    if (STAMP) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        t[1] = wall_clock64();
    }
    const Hartley h1 = hartley8(ax, ay), h2 = hartley8(bx, by);
    double A[8][9];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double a = h1.s * ax[i] + h1.ox, b = h1.s * ay[i] + h1.oy;
        const double c = h2.s * bx[i] + h2.ox, d = h2.s * by[i] + h2.oy;
        A[i][0] = a * c; A[i][1] = a * d; A[i][2] = a;
        A[i][3] = b * c; A[i][4] = b * d; A[i][5] = b;
        A[i][6] = c; A[i][7] = d; A[i][8] = 1.0;
    }
    if (STAMP) {
        asm volatile("" ::"v"(A[7][8]), "v"(A[7][0]));
        t[2] = wall_clock64();
    }
    double n[9];
    null_vector_8x9(A, n);
    if (STAMP) {
        asm volatile("" ::"v"(n[0]), "v"(n[8]));
        t[3] = wall_clock64();
    }
    f8_finish(n, h1, h2, out + 9 * h);
    if (STAMP) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        t[4] = wall_clock64();
        if ((threadIdx.x & 63) == 0)
            for (int k = 0; k < 4; ++k) st[(h >> 6) * 4 + k] = t[k + 1] - t[k];
    }
}

int main() {
    const int N = 5000, H = 4096, REP = 50;
    std::vector<double2> h1(N), h2(N);
    srand(7);
    for (int i = 0; i < N; ++i) {
        h1[i] = {rand() % 1200 + 0.25, rand() % 900 + 0.5};
        h2[i] = {rand() % 1200 + 0.75, rand() % 900 + 0.125};
    }
    double2 *d1, *d2;
    double *dF;
    int32_t *ds, *ps;
    long long *dst;
    hipMalloc(&d1, N * 16);
    hipMalloc(&d2, N * 16);
    hipMalloc(&dF, H * 9 * 8);
    hipMalloc(&ds, H * 8 * 4);
    hipMalloc(&dst, H / 64 * 4 * 8);
    hipHostMalloc(&ps, H * 8 * 4, hipHostMallocMapped);
    uint16_t *ps16;
    hipHostMalloc(&ps16, H * 8 * 2, hipHostMallocMapped);
    for (int i = 0; i < H * 8; ++i) ps16[i] = ps[i] = rand() % N;
    uint16_t *pdev16;
    hipHostGetDevicePointer((void **)&pdev16, ps16, 0);
    hipMemcpy(d1, h1.data(), N * 16, hipMemcpyHostToDevice);
    hipMemcpy(d2, h2.data(), N * 16, hipMemcpyHostToDevice);
    hipMemcpy(ds, ps, H * 32, hipMemcpyHostToDevice);
    int32_t *pdev;
    hipHostGetDevicePointer((void **)&pdev, ps, 0);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int32_t *rows[2] = {pdev, ds};
    const char *name[2] = {"pinned rows", "HBM rows"};
    for (int v = 0; v < 2; ++v)
        for (int pass = 0; pass < 2; ++pass) {
            hipEventRecord(e0, s);
            for (int r = 0; r < REP; ++r)
                hipLaunchKernelGGL((k_fit<false, int32_t>), dim3(H / 64), dim3(64), 0, s, d1, d2, rows[v], H, dF, dst);
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (pass) printf("%-12s %.2f us per launch\n", name[v], 1000.0 * ms / REP);
        }
    for (int pass = 0; pass < 2; ++pass) {
        hipEventRecord(e0, s);
        for (int r = 0; r < REP; ++r)
            hipLaunchKernelGGL((k_fit<false, uint16_t>), dim3(H / 64), dim3(64), 0, s, d1, d2, pdev16, H, dF, dst);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (pass) printf("%-12s %.2f us per launch\n", "pinned u16", 1000.0 * ms / REP);
    }
    const unsigned fl[2] = {hipHostMallocMapped | hipHostMallocNonCoherent, hipHostMallocMapped | hipHostMallocCoherent};
    const char *fn[2] = {"noncoherent", "coherent"};
    for (int f = 0; f < 2; ++f) {
        int32_t *pc, *pcd;
        hipHostMalloc(&pc, H * 8 * 4, fl[f]);
        memcpy(pc, ps, H * 32);
        hipHostGetDevicePointer((void **)&pcd, pc, 0);
        for (int pass = 0; pass < 2; ++pass) {
            hipEventRecord(e0, s);
            for (int r = 0; r < REP; ++r)
                hipLaunchKernelGGL((k_fit<false, int32_t>), dim3(H / 64), dim3(64), 0, s, d1, d2, pcd, H, dF, dst);
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (pass) printf("%-12s %.2f us per launch\n", fn[f], 1000.0 * ms / REP);
        }
    }
    for (int v = 0; v < 2; ++v) {
        hipLaunchKernelGGL((k_fit<true, int32_t>), dim3(H / 64), dim3(64), 0, s, d1, d2, rows[v], H, dF, dst);
        hipStreamSynchronize(s);
        std::vector<long long> hst(H / 64 * 4);
        hipMemcpy(hst.data(), dst, hst.size() * 8, hipMemcpyDeviceToHost);
        double m[4] = {0, 0, 0, 0};
        for (int w = 0; w < H / 64; ++w)
            for (int k = 0; k < 4; ++k) m[k] += hst[w * 4 + k];
        printf("%-12s stages us: loads %.2f  hartley+A %.2f  null %.2f  finish+store %.2f\n", name[v],
               m[0] / (H / 64) / 100, m[1] / (H / 64) / 100, m[2] / (H / 64) / 100, m[3] / (H / 64) / 100);
    }
    return hipGetLastError() != hipSuccess;
}
