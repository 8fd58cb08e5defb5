// Microbenchmark: back-to-back dependent launches on one stream.
//   empty kernels (1 and 192 workgroups), and a chain where each launch reads
//   a 16x16 fp64 tile written by the previous launch (on another XCD).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>

__global__ void k_empty(int *g) {
    if (g && *g == 12345) g[1] = 0;
}

__global__ void k_spin(long long cycles) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
}

__global__ void k_chain(double *a, int s) {
    // block b reads tile (s-1) and writes tile s  (tile = 256 doubles)
    const int t = threadIdx.x;
    double v = a[(s - 1) * 256 + t];
    if (blockIdx.x == 0) a[s * 256 + t] = v * 1.0000001 + 1.0;
}

int main() {
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    int *g;
    hipMalloc(&g, 64);
    hipMemset(g, 0, 64);
    double *a;
    hipMalloc(&a, 4096 * 256 * 8);
    hipMemset(a, 0, 4096 * 256 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int N = 2000;
    for (int rep = 0; rep < 2; ++rep) {
        for (int blocks : {1, 64, 192, 1024}) {
            // the device is held by a spin kernel while the host queues the
            // launches, so the events time the device-side rate only
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, st, (long long)100000000);
            hipEventRecord(e0, st);
            const auto h0 = std::chrono::steady_clock::now();
            for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, st, g);
            const auto h1 = std::chrono::steady_clock::now();
            if (rep) printf("host enqueue: %.2f us per launch\n", std::chrono::duration<double, std::micro>(h1 - h0).count() / N);
            hipEventRecord(e1, st);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep) printf("empty x%d blocks=%d: %.2f us per launch\n", N, blocks, ms * 1e3 / N);
        }
        for (int blocks : {1, 192}) {
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, st, (long long)100000000);
            hipEventRecord(e0, st);
            for (int i = 1; i < 4000; ++i) hipLaunchKernelGGL(k_chain, dim3(blocks), dim3(256), 0, st, a, i);
            hipEventRecord(e1, st);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep) printf("chain blocks=%d: %.2f us per launch\n", blocks, ms * 1e3 / 3999);
        }
        // event records between kernels
        hipEventRecord(e0, st);
        hipEvent_t ev[64];
        for (auto &e : ev) hipEventCreate(&e);
        for (int i = 0; i < 64; ++i) {
            hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, st, g);
            hipEventRecord(ev[i], st);
        }
        hipEventRecord(e1, st);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep) printf("empty + event record: %.2f us per pair\n", ms * 1e3 / 64);
        for (auto &e : ev) hipEventDestroy(e);
    }
    hipDeviceSynchronize();
    printf("DONE\n");
    return 0;
}
