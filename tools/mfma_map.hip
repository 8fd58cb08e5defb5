// Checks the fp64 MFMA lane maps used by k_chol_wg (exact integer data):
//   A operand, K-slab q: lane l holds A[l & 15][4q + (l >> 4)]
//   B operand, K-slab q: lane l holds B[4q + (l >> 4)][l & 15]
//   C/D:                 lane l, element i holds D[(l >> 4) + 4i][l & 15]
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k(const double *A, const double *B, const double *C, double *D) {
    const int l = threadIdx.x;
    d4 acc;
    for (int i = 0; i < 4; ++i) acc[i] = C[((l >> 4) + 4 * i) * 16 + (l & 15)];
    for (int q = 0; q < 4; ++q) {
        const double a = A[(l & 15) * 16 + 4 * q + (l >> 4)];
        const double b = B[(4 * q + (l >> 4)) * 16 + (l & 15)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
    for (int i = 0; i < 4; ++i) D[((l >> 4) + 4 * i) * 16 + (l & 15)] = acc[i];
}

int main() {
    double hA[256], hB[256], hC[256], hD[256], ref[256];
    for (int i = 0; i < 256; ++i) { hA[i] = (i * 7) % 11 - 5; hB[i] = (i * 5) % 13 - 6; hC[i] = i % 9; }
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            double s = hC[i * 16 + j];
            for (int k = 0; k < 16; ++k) s += hA[i * 16 + k] * hB[k * 16 + j];
            ref[i * 16 + j] = s;
        }
    double *dA, *dB, *dC, *dD;
    hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dC, 2048); hipMalloc(&dD, 2048);
    hipMemcpy(dA, hA, 2048, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, 2048, hipMemcpyHostToDevice);
    hipMemcpy(dC, hC, 2048, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
    hipMemcpy(hD, dD, 2048, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += hD[i] != ref[i];
    printf("mfma f64 16x16x4 lane maps: %s (%d mismatches)\n", bad ? "WRONG" : "ok", bad);
    return bad != 0;
}
