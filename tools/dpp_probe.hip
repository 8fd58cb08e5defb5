// Probe: does hipcc lower a 64-bit row_newbcast DPP broadcast (gfx90a+ DPP64)
// into one VALU op feeding an fp64 FMA?  Build with --save-temps and read the
// ISA; run on the box to check the lane semantics.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int J>
__device__ __forceinline__ double bcast16(double v) {
    // row_newbcast:J -- lane J of each 16-lane row to the whole row
    return __longlong_as_double(__builtin_amdgcn_update_dpp(0ll, __double_as_longlong(v), 0x150 + J, 0xF, 0xF, false));
}

__global__ void k_probe(const double *in, double *out) {
    const int l = threadIdx.x;
    double v = in[l];
    double a = in[64 + l];
    a = __builtin_fma(-v, bcast16<3>(v), a);
    out[l] = a;
    out[64 + l] = bcast16<7>(v);
}

int main() {
    double h[128], o[128];
    for (int i = 0; i < 128; ++i) h[i] = i + 0.5;
    double *d, *od;
    hipMalloc(&d, sizeof h);
    hipMalloc(&od, sizeof o);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    k_probe<<<1, 64>>>(d, od);
    hipMemcpy(o, od, sizeof o, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        const double src3 = h[(l & ~15) + 3], src7 = h[(l & ~15) + 7];
        if (o[l] != __builtin_fma(-h[l], src3, h[64 + l]) || o[64 + l] != src7) ++bad;
    }
    printf("dpp64 row_newbcast probe: %s\n", bad ? "MISMATCH" : "ok");
    return bad != 0;
}
