// Probe (round 3): the costs a persistent reduced-camera solve is built from.
//   1. dependent-instruction latencies on one wave (fp64 FMA, DPP64
//      row_newbcast FMA, rsq/rcp f64, ldexp, readlane round trip, LDS);
//   2. the 16-pivot tile factor of k_chol_col (rows of C_ss and one panel row
//      set per lane, DPP broadcasts) in variants;
//   3. a cross-workgroup hand-off (producer: sc1 stores + vmcnt(0) + sc1 flag;
//      consumer: sc1 poll, sc1 loads), ping-pong between two workgroups.
// Every spin is bounded (s_memrealtime, 20 ms) and reports a timeout.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define HC(x)                                                             \
    do {                                                                  \
        hipError_t e = (x);                                               \
        if (e != hipSuccess) {                                            \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                      \
        }                                                                 \
    } while (0)

__device__ __forceinline__ long long clk() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ int fl(double x) {  // forces x to be complete
    int lo = (int)__double_as_longlong(x), k;
    asm volatile("v_readfirstlane_b32 %0, %1\n\ts_nop 0" : "=s"(k) : "v"(lo));
    return k;
}
__device__ __forceinline__ long long rtc() { return __builtin_amdgcn_s_memrealtime(); }

// ---------------------------------------------------------------- latencies
constexpr int NL = 256;

__global__ void k_lat(const double *in, double *out, long long *cyc) {
    const int lane = threadIdx.x;
    double a = in[lane], b = in[64 + lane], c = in[128 + lane];
    long long t0, t1;
    int k = 0;
    // 0: dependent v_fma_f64
    {
        double x = a;
        t0 = clk();
#pragma unroll
        for (int i = 0; i < NL; ++i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
        k = fl(x);
        t1 = clk();
        if (lane == 0) cyc[0] = t1 - t0;
        out[lane] = x + k;
    }
    // 1: dependent v_fmac_f64_dpp row_newbcast (with the 2 wait states)
    {
        double x = a;
        t0 = clk();
#pragma unroll
        for (int i = 0; i < NL; ++i)
            asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf"
                         : "+v"(x) : "v"(b));
        k = fl(x);
        t1 = clk();
        if (lane == 0) cyc[1] = t1 - t0;
        out[64 + lane] = x + k;
    }
    // 2: dependent v_rsq_f64
    {
        double x = a * a + 1.0;
        t0 = clk();
#pragma unroll
        for (int i = 0; i < NL; ++i) asm volatile("v_rsq_f64 %0, %0" : "+v"(x));
        k = fl(x);
        t1 = clk();
        if (lane == 0) cyc[2] = t1 - t0;
        out[128 + lane] = x + k;
    }
    // 3: dependent v_rcp_f64
    {
        double x = a * a + 1.0;
        t0 = clk();
#pragma unroll
        for (int i = 0; i < NL; ++i) asm volatile("v_rcp_f64 %0, %0" : "+v"(x));
        k = fl(x);
        t1 = clk();
        if (lane == 0) cyc[3] = t1 - t0;
        out[192 + lane] = x + k;
    }
    // 4: dependent v_mul_f64
    {
        double x = a;
        t0 = clk();
#pragma unroll
        for (int i = 0; i < NL; ++i) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x) : "v"(b));
        k = fl(x);
        t1 = clk();
        if (lane == 0) cyc[4] = t1 - t0;
        out[256 + lane] = x + k;
    }
    // 5: independent v_fma_f64 issue (8 chains interleaved)
    {
        double x0 = a, x1 = b, x2 = c, x3 = a + 1, x4 = b + 1, x5 = c + 1, x6 = a + 2, x7 = b + 2;
        t0 = clk();
#pragma unroll
        for (int i = 0; i < NL / 8; ++i)
            asm volatile(
                "v_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %1, %1, %8, %9\n\tv_fma_f64 %2, %2, %8, %9\n\t"
                "v_fma_f64 %3, %3, %8, %9\n\tv_fma_f64 %4, %4, %8, %9\n\tv_fma_f64 %5, %5, %8, %9\n\t"
                "v_fma_f64 %6, %6, %8, %9\n\tv_fma_f64 %7, %7, %8, %9"
                : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                : "v"(b), "v"(c));
        const double x = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
        k = fl(x);
        t1 = clk();
        if (lane == 0) cyc[5] = t1 - t0;
        out[320 + lane] = x + k;
    }
    // 6: independent DPP fmac issue (8 chains)
    {
        double x0 = a, x1 = b, x2 = c, x3 = a + 1, x4 = b + 1, x5 = c + 1, x6 = a + 2, x7 = b + 2;
        t0 = clk();
#pragma unroll
        for (int i = 0; i < NL / 8; ++i)
            asm volatile(
                "v_fmac_f64_dpp %0, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %1, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %3, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %4, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %5, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %6, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %7, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf"
                : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                : "v"(b), "v"(c));
        const double x = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
        k = fl(x);
        t1 = clk();
        if (lane == 0) cyc[6] = t1 - t0;
        out[384 + lane] = x + k;
    }
    // 7: dependent ldexp by a constant exponent
    {
        double x = a;
        int e = 1;
        t0 = clk();
#pragma unroll
        for (int i = 0; i < NL; ++i) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(x) : "v"(e));
        k = fl(x);
        t1 = clk();
        if (lane == 0) cyc[7] = t1 - t0;
        out[448 + lane] = x + k;
    }
    // 8: LDS round trip (dependent ds_write_b64 + ds_read_b64 of another lane)
    {
        __shared__ double sh[64];
        double x = a;
        t0 = clk();
        for (int i = 0; i < 64; ++i) {
            sh[lane] = x;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
            x = sh[(lane + 1) & 63] * 1.0000001;
        }
        k = fl(x);
        t1 = clk();
        if (lane == 0) cyc[8] = (t1 - t0) * NL / 64;  // scaled to NL trips
        out[512 + lane] = x + k;
    }
    // 9: dependent v_readlane pair -> fma with SGPR operand (the readlane chain)
    {
        double x = a;
        t0 = clk();
#pragma unroll
        for (int i = 0; i < NL; ++i) {
            const int lo = __builtin_amdgcn_readlane(__double_as_longlong(x) & 0xffffffff, 5);
            const int hi = __builtin_amdgcn_readlane(__double_as_longlong(x) >> 32, 5);
            const double s = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
            x = __builtin_fma(x, b, s);
        }
        k = fl(x);
        t1 = clk();
        if (lane == 0) cyc[9] = t1 - t0;
        out[576 + lane] = x + k;
    }
}

// ---------------------------------------------------------------- tile factor
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
__device__ __forceinline__ double bcast16_asm(double v) {
    double d;
    asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
                 : "=v"(d) : "v"(v), "n"(J));
    return d;
}
template <int K, int... I>
__device__ __forceinline__ void upd(double (&r)[16], double (&p)[16], std::integer_sequence<int, I...>) {
    const double nrk = -r[K], npk = -p[K];
    (fmac2_bc<K + 1 + I, I == 0>(r[K + 1 + I], p[K + 1 + I], r[K], nrk, npk), ...);
}
template <int NEWTON, int K>
__device__ __forceinline__ void step(double (&r)[16], double (&p)[16], double (&dinv)[16], int li) {
    const double d = bcast16_asm<K>(r[K]);
    double g = __builtin_amdgcn_rsq(d);
    if constexpr (NEWTON >= 1) g = g * (1.5 - 0.5 * d * g * g);
    if constexpr (NEWTON >= 2) g = g * (1.5 - 0.5 * d * g * g);
    dinv[K] = g;
    r[K] = (li == K) ? d * g : r[K] * g;
    p[K] = p[K] * g;
    if constexpr (K < 15) upd<K>(r, p, std::make_integer_sequence<int, 15 - K>{});
}
template <int NEWTON, int... K>
__device__ __forceinline__ void steps(double (&r)[16], double (&p)[16], double (&dinv)[16], int li,
                                      std::integer_sequence<int, K...>) {
    (step<NEWTON, K>(r, p, dinv, li), ...);
}

template <int NEWTON>
__global__ void k_factor(const double *A, double *out, long long *cyc, int reps) {
    const int lane = threadIdx.x, li = lane & 15;
    double r[16], p[16], dinv[16];
    long long best = 1ll << 60;
    for (int it = 0; it < reps; ++it) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            r[j] = A[li * 16 + j];
            p[j] = A[256 + (lane >> 4) * 16 * 16 + li * 16 + j];
        }
        int k;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        k = fl(r[15]);
        const long long t0 = clk();
        steps<NEWTON>(r, p, dinv, li, std::make_integer_sequence<int, 16>{});
        double s = r[15] + p[15] + dinv[15];
        k = fl(s);
        const long long t1 = clk();
        best = (t1 - t0) < best ? (t1 - t0) : best;
        out[lane] = s + k;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        out[64 + lane * 16 + j] = r[j];
        out[64 + 1024 + lane * 16 + j] = p[j];
    }
    if (lane == 0) cyc[0] = best;
}

// ---------------------------------------------------------------- hand-off
// Workgroups 0 and `peer` ping-pong `rounds` times.  Each hop: the holder
// reads the other side's payload (NB doubles per thread, sc1 loads), adds 1
// to every element, stores its own payload (sc1), s_waitcnt vmcnt(0), a
// workgroup barrier, then one lane stores the flag (sc1).  The other side
// polls the flag (sc1 load, one lane), then a workgroup barrier.
__device__ __forceinline__ void st_sc1(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int PER>
__global__ void __launch_bounds__(256) k_pingpong(double *buf, int *flags, int peer, int rounds, long long *res) {
    const int b = blockIdx.x;
    if (b != 0 && b != peer) return;
    const int side = b == 0 ? 0 : 1;
    const int t = threadIdx.x;
    __shared__ int abort_s;
    if (t == 0) abort_s = 0;
    __syncthreads();
    double *mine = buf + side * 256 * PER, *theirs = buf + (1 - side) * 256 * PER;
    int *fl_theirs = flags + (1 - side) * 64, *fl_mine = flags + side * 64;
    const long long r0 = rtc();
    for (int it = 0; it < rounds; ++it) {
        const int want = 2 * it + side;  // hop number this side acts on
        if (want > 0) {
            if (t == 0) {
                const long long ts = rtc();
                while (__hip_atomic_load(fl_theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
                    __builtin_amdgcn_s_sleep(1);
                    if (rtc() - ts > 2000000) { abort_s = 1; break; }
                }
            }
            __syncthreads();
            if (abort_s) break;
        }
        double v[PER];
#pragma unroll
        for (int q = 0; q < PER; ++q) v[q] = want > 0 ? ld_sc1(theirs + q * 256 + t) : 0.0;
#pragma unroll
        for (int q = 0; q < PER; ++q) st_sc1(mine + q * 256 + t, v[q] + 1.0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) __hip_atomic_store(fl_mine, want + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const long long r1 = rtc();
    if (t == 0) {
        res[side * 2] = r1 - r0;
        res[side * 2 + 1] = abort_s;
    }
}

int main(int argc, char **argv) {
    double *d_in, *d_out;
    long long *d_cyc;
    HC(hipMalloc(&d_in, 8192 * 8));
    HC(hipMalloc(&d_out, 8192 * 8));
    HC(hipMalloc(&d_cyc, 64 * 8));
    std::vector<double> h(8192);
    srand(1);
    for (auto &x : h) x = 0.5 + (rand() % 1000) * 1e-3;
    // an SPD 16x16 tile at A[0..256): diag dominant
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) h[i * 16 + j] = (i == j) ? 20.0 + i : 0.1 * ((i + j) % 5) + 0.01 * (i * j % 7);
    HC(hipMemcpy(d_in, h.data(), 8192 * 8, hipMemcpyHostToDevice));
    long long cyc[64];
    k_lat<<<1, 64>>>(d_in, d_out, d_cyc);
    HC(hipDeviceSynchronize());
    k_lat<<<1, 64>>>(d_in, d_out, d_cyc);
    HC(hipDeviceSynchronize());
    HC(hipMemcpy(cyc, d_cyc, 10 * 8, hipMemcpyDeviceToHost));
    const char *nm[] = {"fma_f64 dep", "fmac_f64_dpp dep (+s_nop1)", "rsq_f64 dep", "rcp_f64 dep", "mul_f64 dep",
                        "fma_f64 indep (8 chains)", "fmac_dpp indep (8 chains)", "ldexp_f64 dep",
                        "LDS write+read dep", "readlane pair + fma dep"};
    for (int i = 0; i < 10; ++i) printf("lat %-28s %7.2f cycles/op\n", nm[i], (double)cyc[i] / NL);
    for (int nw = 0; nw <= 2; ++nw) {
        auto kf = nw == 0 ? k_factor<0> : nw == 1 ? k_factor<1> : k_factor<2>;
        kf<<<1, 64>>>(d_in, d_out, d_cyc, 20);
        HC(hipDeviceSynchronize());
        HC(hipMemcpy(cyc, d_cyc, 8, hipMemcpyDeviceToHost));
        printf("chol16 r+p factor, %d Newton: %lld cycles (%.1f per pivot)\n", nw, cyc[0], cyc[0] / 16.0);
    }
    // hand-off ping-pong
    double *buf;
    int *flags;
    long long *res;
    HC(hipMalloc(&buf, 2 * 256 * 32 * 8));
    HC(hipMalloc(&flags, 2 * 64 * 4));
    HC(hipMalloc(&res, 4 * 8));
    const int rounds = 2000;
    for (int peer : {1, 8, 3}) {
        for (int per : {1, 4, 16}) {
            HC(hipMemset(flags, 0, 2 * 64 * 4));
            HC(hipMemset(buf, 0, 2 * 256 * 32 * 8));
            auto kp = per == 1 ? k_pingpong<1> : per == 4 ? k_pingpong<4> : k_pingpong<16>;
            kp<<<16, 256>>>(buf, flags, peer, rounds, res);
            HC(hipDeviceSynchronize());
            long long hr[4];
            HC(hipMemcpy(hr, res, 32, hipMemcpyDeviceToHost));
            printf("pingpong peer=%d payload=%d KB: %.3f us per hop (abort %lld/%lld)\n", peer, per * 2,
                   hr[0] * 10e-3 / (2.0 * rounds), hr[1], hr[3]);
        }
    }
    return 0;
}
