// Row-distributed persistent block Gauss-Jordan solve of the damped reduced
// camera system (S + lambda clamp(diag U)) x = b in ONE launch (round 4).
// Replaces the reference's MINPACK dense QR step on the BA hot path
// (Phase 1/BundleAdjustment.py:205-212, via scipy lmdif); included by ba.hip
// after gj_solve.hpp (the 16-pivot DPP tile factor, elem_ref, cam_trial).
//
// The algorithm is gj_solve.hpp's block Gauss-Jordan with Cholesky pivots
// (step p: L_p = chol(A_pp), G_i = A_ip L_p^-T for every row tile i != p,
// A_ij -= G_i G_j^T for j > p, b_i -= G_i y_p; at the end x_i = L_i^-T L_i^-1
// b_i), laid out so that the critical path crosses ONE workgroup boundary per
// pivot and nothing else:
//
//  * workgroup r owns row tile r ("owner r"): the tiles A_rj of its row that
//    are still live (j <= r before its pivot: the lower triangle; j > p after
//    it: the rows above the pivot keep being eliminated), and b_r;
//  * at pivot p owner p publishes ONE record P_p = {L_p^-1, y_p} (the tile
//    factor also inverts: the identity rides as a second panel row set, so
//    L_p^-T costs no extra chain steps).  Every owner forms its own
//    G_r = A_rp L_p^-T as an MFMA product (no triangular solve), and the
//    unpivoted owners r > p publish G_r for the others' updates;
//  * owner r's wave W0 holds A_r,r-1 and A_rr: when P_{r-1} arrives it forms
//    G_r, publishes it, updates A_rr, and runs the chain for pivot r -- the
//    whole critical step inside one wave, with no LDS hand-off; the one
//    cross-workgroup hop per pivot is P_{r-1} -> owner r;
//  * G_r is only ever needed by others while r is unpivoted; the G of a
//    pivoted row updates that row alone (and its b), off every critical path.
//
// Hand-offs are data-tagged granules (MI355X_MICROARCH.md handoff-1to1,
// cdna_hip_programming.md Guideline 16 R2): every 8-byte word {tag, 32 data
// bits} is written by ONE agent-scope store and re-read by agent-scope loads
// until every tag equals this launch's tag -- no flag, no fence.  A double
// travels as two granules.  Tags grow by one every launch (host epoch), so
// no word needs re-zeroing between launches.
//
// Layout.  Tiles live in MFMA accumulators (v_mfma_f64_16x16x4f64: lane l
// element e = D[(l >> 4) + 4e][l & 15]).  A tile of owner r is held as the
// accumulator of A_rj^T: element e of lane l is A_rj(l & 15, (l >> 4) + 4e),
// which is exactly the k-block-e operand fragment of A_rj.  So:
//   G_r^T = L_p^-1 A_rp^T          A = L_p^-1 fragment, B = held A_rp
//   A_rj^T -= G_j G_r^T            A = -G_j fragment,  B = G_r fragment
//   A_rj^T  = G_j L_r^T (import)   A = G_j fragment,   B = L_r fragment
// and the product G_r^T comes out as the fragment of G_r: nothing is ever
// transposed through LDS except the diagonal tile into the chain's rows.
namespace gjr {

constexpr int TL = 16;
constexpr int NUW = 7;           // tile-holding waves U0..U6 (tile j -> U[j % NUW]); with W0 two waves a SIMD
constexpr int NW = NUW + 1;      // + W0
constexpr int THREADS = 64 * NW;
constexpr int NTMAX = 128;       // tile rows (host checks; larger systems take the Cholesky path)
constexpr int RING = 4;          // LDS ring depth of the per-step pieces
constexpr int PPAIRS = 5;        // granule pairs a lane of a pivot record: L^-1 fragment (4), y (1)
constexpr int GPAIRS = 4;        // granule pairs a lane of a published G tile
constexpr int PBYTES = PPAIRS * 64 * 16;
constexpr int GBYTES = GPAIRS * 64 * 16;
constexpr int GDBYTES = 2 * 64 * 16;  // a G tile untagged: two 16-byte rows of 64 lanes (the bulk copy)
constexpr int NB = 6;                 // bulk G tiles a U wave has in flight
constexpr long long POLL_LIMIT = 20000000;  // s_memrealtime ticks (100 MHz): 200 ms
constexpr int TREG = 11;                    // tile slots a U wave holds in registers (more would spill)
constexpr int TREG_L = 10, TLDS_L = 9;      // large systems (77 < nT <= NTMAX = 128; the slots would hold 133): 10 slots in registers, 9 in LDS
constexpr int DYN_LDS = NUW * TLDS_L * 256 * 8;  // dynamic LDS: those slots, the epilogue's scratch, and
                                                 // one workgroup per CU

typedef double d4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct Args {
    const double *payload;  // the finished (all-reduced) Schur payload
    SlabSrc src;            // one rank: the sweep's slabs read directly (k_schur_finish folded in), or none
    int32_t ns, nT;
    const double *lam;
    const int *gate;
    u64 *P;         // [2][nT] pivot records of PBYTES: write-through copy, then the L2-local copy
    u64 *G;         // [nT][nT] G_r of step p at (p, r), GBYTES each (granules: W0 of owner r + 1)
    double *Gd;     // [nT][nT] the same untagged, GDBYTES each (the U waves' bulk updates) ...
    unsigned *Gf;   // [nT][nT] ... published by a flag (= tag) behind the drained stores
    unsigned tag;   // this launch's granule tag (>= 1)
    double *x;      // [nT * 16] solution
    int *bad;       // not positive definite (the LM rejects the step)
    int *err;       // a wait timed out (the host reports an error)
    unsigned *arrive;
    CamTrialArgs ct;  // trial cameras epilogue (nc = 0: none)
    long long *dbg;   // diagnostics (nullable): [grid][nT + 1][16] s_memrealtime stamps
};

enum { DBG_PIN = 0, DBG_GCRIT, DBG_CHAIN0, DBG_CHAIN1, DBG_PPUB, DBG_GHOLD, DBG_UDONE, DBG_GREM, DBG_PLW, DBG_GRDY, DBG_HPRDY };
enum { DBG_START = 0, DBG_PROLOGUE, DBG_W0END, DBG_ARRIVED };
// row tile of workgroup b: consecutive rows on one XCD (workgroups are
// dealt round-robin over the 8 XCDs, b % 8), so the critical hop P_{r-1} ->
// owner r mostly stays inside one L2
constexpr int NXCD_ = 8;
__device__ __forceinline__ int row_of(int b, int nT) {
    const int x = b % NXCD_;
    return x * (nT / NXCD_) + min(x, nT % NXCD_) + b / NXCD_;
}
__device__ __forceinline__ int xcd_of_row(int r, int nT) {
    const int q = nT / NXCD_, m = nT % NXCD_;
    return r < m * (q + 1) ? r / (q + 1) : m + (r - m * (q + 1)) / max(q, 1);
}
__device__ __forceinline__ void stamp(const Args &a, int p, int slot) {
    if (a.dbg && (threadIdx.x & 63) == 0)
        a.dbg[((int64_t)row_of(blockIdx.x, a.nT) * (a.nT + 1) + p) * 16 + slot] = __builtin_amdgcn_s_memrealtime();
}

struct Smem {
    double PL[RING][4][64];  // L_p^-1 fragments for the holder of A_rp
    double GL[RING][4][64];  // G_r of step p for every wave's updates
    double Lf[4][64];        // L_r fragment (the imports A_rj = L_r G_j^T)
    double Dm[TL][TL + 1];   // the diagonal tile into the chain's rows; L_r rows after it
    double Li[TL][TL + 1];   // L_r^-1 (row-major)
    double bv[TL], yv[TL];
    int pready[RING], pdone[RING], gready[RING], gdone[RING];
    int lready, abort_, last;
    int *err, *bad;
};

__device__ __forceinline__ int lds_ld(const int *w) {
    return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_set(int *w, int v) {
    __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// a wave's count: ONE lane adds (called by every lane, the atomic optimiser
// would fold the wave's adds into one add of 64)
__device__ __forceinline__ void lds_add(int *w, int v) {
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local"); }
__device__ __forceinline__ void lds_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local"); }
__device__ __forceinline__ void wave_lds() { asm volatile("" ::: "memory"); }  // one wave's LDS accesses stay in order
__device__ __forceinline__ long long rtc() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void abort_solve(Smem &S) {
    lds_set(&S.abort_, 1);
    if ((threadIdx.x & 63) == 0) {
        __hip_atomic_store(S.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(S.bad, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// bounded waits: a lost hand-off (or another workgroup's abort) ends the
// solve with an error, it never hangs the GPU
__device__ __forceinline__ bool give_up(Smem &S, unsigned it, long long &t0) {
    if (lds_ld(&S.abort_)) return true;
    if (__hip_atomic_load(S.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        lds_set(&S.abort_, 1);
        return true;
    }
    const long long t = rtc();
    if (t0 < 0) t0 = t;
    else if (t - t0 > POLL_LIMIT) {
        abort_solve(S);
        return true;
    }
    return false;
}
__device__ __forceinline__ bool lds_wait(const int *w, int target, Smem &S) {
    if (lds_ld(w) >= target) {
        lds_acquire();
        return true;
    }
    long long t0 = -1;
    for (unsigned it = 1;; ++it) {
        __builtin_amdgcn_s_sleep(1);
        if (lds_ld(w) >= target) break;
        if (it % 256 == 0 && give_up(S, it, t0)) return false;
    }
    lds_acquire();
    return true;
}

// ------------------------------------------------------------- granules
// A double travels as ONE 16-byte pair of granules {lo, tag, hi, tag},
// written by one sc1 buffer store (each 8-byte half is an untorn granule) and
// polled by sc1 buffer loads; a record is PAIRS rows of 64 lanes x 16 bytes,
// so every instruction moves 1 KB contiguous.  The descriptors are built from
// kernel arguments (wave-uniform: no waterfall loops), offsets are 32-bit.
// The descriptor is rebuilt at every use from readfirstlane'd words: one the
// compiler cannot prove wave-uniform wraps every buffer op in a waterfall
// loop (cdna_hip_programming.md T20), which serialised this solve's
// hand-offs.  A store's record offset rides in the per-lane voffset
// (soffset 0): the same offset handed to the soffset through readfirstlane
// gave wrong, nondeterministic (~1e-6) solves on gfx950.  The ISA of that
// build (round 5, tools/isa_war_scan.py) shows the likely cause: the
// compiler reuses the soffset SGPR for the next record's offset, rewriting
// it with a v_readfirstlane 1-5 instructions after the record's last
// dwordx4 store.  A store wider than 8 bytes reads its operands after issue
// (LLVM's gfx950 hazard model covers only its data VGPRs, one wait state),
// so an SGPR soffset rewritten right behind it can move the store to the
// next record.  No store here reads an SGPR offset.  The polls (loads) keep
// readfirstlane'd soffsets: a load takes its address at issue -- in the
// TREG_L build 36 poll loads have their soffset rewritten 3-4 instructions
// later, and its solves are exact and bitwise repeatable (test_reduced_solve
// at n = 1800, nT = 113, instantiates it) -- and a voffset there costs VGPRs
// and spills the tile slots.
struct Buf {
    const void *base;
    int bytes;
};
struct Rs {
    Buf P, G, Gd;
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const Buf &b) {
    const u64 a = (u64)b.base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((u64)hi << 32) | lo), (short)0,
                                             __builtin_amdgcn_readfirstlane(b.bytes), 0x00020000);
}
constexpr int SC1 = 16;  // buffer op aux: sc1 (write-through stores, L2-served loads)
template <int AUX = SC1>
__device__ __forceinline__ void put_pair(const Buf &bf, int soff, int e, unsigned tag, double v, int lane) {
    const u64 b = (u64)__double_as_longlong(v);
    const u32x4 w = {(unsigned)b, tag, (unsigned)(b >> 32), tag};
    __builtin_amdgcn_raw_buffer_store_b128(w, rsrc(bf), soff + e * 1024 + lane * 16, 0, AUX);
}
template <int AUX = SC1>
__device__ __forceinline__ void put4(const Buf &rs, int soff, unsigned tag, const d4 &v, int lane) {
#pragma unroll
    for (int e = 0; e < 4; ++e) put_pair<AUX>(rs, soff, e, tag, v[e], lane);
}
__device__ __forceinline__ double dec(const u32x4 &x) {
    return __longlong_as_double((long long)(((u64)x.z << 32) | x.x));
}
// ONE wave re-reads the N pairs of NR records (all loads in flight) until
// every tag of every lane matches; false on abort / timeout
template <int NR, int N>
__device__ __forceinline__ bool sweep(const Buf &bf, const int (&soff)[NR], const bool (&need)[NR],
                                      unsigned tag, u32x4 (&x)[NR][N], int lane, Smem &S) {
    long long t0 = -1;
    for (unsigned it = 1;; ++it) {
        asm volatile("" ::: "memory");  // every pass reloads
        const __amdgpu_buffer_rsrc_t rs = rsrc(bf);
#pragma unroll
        for (int q = 0; q < NR; ++q) {
            if (need[q]) {
#pragma unroll
                for (int k = 0; k < N; ++k)
                    x[q][k] = __builtin_amdgcn_raw_buffer_load_b128(rs, k * 1024 + lane * 16, __builtin_amdgcn_readfirstlane(soff[q]), SC1);
            } else {
#pragma unroll
                for (int k = 0; k < N; ++k) x[q][k] = u32x4{0u, tag, 0u, tag};
            }
        }
        bool ok = true;
#pragma unroll
        for (int q = 0; q < NR; ++q)
#pragma unroll
            for (int k = 0; k < N; ++k) ok &= x[q][k].y == tag && x[q][k].w == tag;
        if (__all(ok)) return true;
        __builtin_amdgcn_s_sleep(1);
        if (it % 64 == 0 && give_up(S, it, t0)) return false;
    }
}
// the critical poll (owner r - 1 on this XCD): P_{r-1} from its L2-local
// copy (plain stores: the line stays in the shared L2, an sc1 load is served
// there) or from the write-through copy, per lane whichever is complete --
// the same values, so a lane may take either; the write-through copy also
// covers a workgroup placement other than round-robin
__device__ __forceinline__ bool poll_p2(const Buf &bf, int soff_wt, int soff_l2, unsigned tag, u32x4 (&x)[PPAIRS],
                                        int lane, Smem &S) {
    long long t0 = -1;
    for (unsigned it = 1;; ++it) {
        asm volatile("" ::: "memory");  // every pass reloads
        const __amdgpu_buffer_rsrc_t rs = rsrc(bf);
        u32x4 y[PPAIRS];
#pragma unroll
        for (int k = 0; k < PPAIRS; ++k)
            x[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, k * 1024 + lane * 16, __builtin_amdgcn_readfirstlane(soff_l2), SC1);
#pragma unroll
        for (int k = 0; k < PPAIRS; ++k)
            y[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, k * 1024 + lane * 16, __builtin_amdgcn_readfirstlane(soff_wt), SC1);
        bool ok = true, okw = true;
#pragma unroll
        for (int k = 0; k < PPAIRS; ++k) {
            ok &= x[k].y == tag && x[k].w == tag;
            okw &= y[k].y == tag && y[k].w == tag;
        }
        if (__all(ok || okw)) {
            if (!ok)
#pragma unroll
                for (int k = 0; k < PPAIRS; ++k) x[k] = y[k];
            return true;
        }
        __builtin_amdgcn_s_sleep(1);
        if (it % 64 == 0 && give_up(S, it, t0)) return false;
    }
}
template <int N>
__device__ __forceinline__ d4 dec4(const u32x4 (&v)[N]) {
    return d4{dec(v[0]), dec(v[1]), dec(v[2]), dec(v[3])};
}
__device__ __forceinline__ int gsoff(const Args &a, int p, int r) { return (p * a.nT + r) * GBYTES; }

// The bulk copy of G_r (step p): the U waves of every other owner read it,
// (nT - p) tiles an owner a step, so it travels untagged -- half the bytes of
// the granules, whose reads set the pace of the late owners' U waves (the
// per-CU rate of handed-off reads, MI355X_MICROARCH.md handoff-payload).
// R1 form (cdna_hip_programming.md Guideline 16): sc1 payload stores, the
// storing wave's vmcnt(0), then ONE lane's sc1 flag store; the reading wave
// polls the flags of all the tiles it needs at a step in one load and reads
// the payloads with sc1 loads after they matched.
__device__ __forceinline__ int gdoff(const Args &a, int p, int r) { return (p * a.nT + r) * GDBYTES; }
__device__ __forceinline__ void put_bulk(const Buf &bf, int off, const d4 &v, int lane) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const u64 b0 = (u64)__double_as_longlong(v[2 * h]), b1 = (u64)__double_as_longlong(v[2 * h + 1]);
        const u32x4 w = {(unsigned)b0, (unsigned)(b0 >> 32), (unsigned)b1, (unsigned)(b1 >> 32)};
        __builtin_amdgcn_raw_buffer_store_b128(w, rsrc(bf), off + h * 1024 + lane * 16, 0, SC1);
    }
}
__device__ __forceinline__ void flag_bulk(const Args &a, int p, int r) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's payload stores have completed
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(a.Gf + p * a.nT + r, a.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ d4 dec_bulk(const u32x4 (&x)[2]) {
    return d4{__longlong_as_double((long long)(((u64)x[0].y << 32) | x[0].x)),
              __longlong_as_double((long long)(((u64)x[0].w << 32) | x[0].z)),
              __longlong_as_double((long long)(((u64)x[1].y << 32) | x[1].x)),
              __longlong_as_double((long long)(((u64)x[1].w << 32) | x[1].z))};
}
// until the bulk copies of step p of this wave's tiles j = w + NUW k,
// lo < j < hi, are all published (lane k polls tile k's flag); false on abort
template <int TPW>
__device__ __forceinline__ bool wait_bulk(const Args &a, int p, int w, int lo, int hi, int lane, Smem &S) {
    static_assert(TPW <= 64, "one flag a lane");
    const int j = w + NUW * lane;
    const bool need = lane < TPW && j > lo && j < hi;
    const unsigned *f = a.Gf + p * a.nT + (need ? j : 0);
    long long t0 = -1;
    for (unsigned it = 1;; ++it) {
        const unsigned v = need ? __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : a.tag;
        if (__all(v == a.tag)) return true;
        __builtin_amdgcn_s_sleep(1);
        if (it % 64 == 0 && give_up(S, it, t0)) return false;
    }
}
// acc += sum_q A_q B_q (fp64 MFMA 16x16x4; fragment element q = k-block q)
__device__ __forceinline__ d4 mfma4(d4 acc, const d4 &a, const d4 &b) {
#pragma unroll
    for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], b[q], acc, 0, 0, 0);
    return acc;
}
__device__ __forceinline__ d4 zero4() { return d4{0.0, 0.0, 0.0, 0.0}; }

// this wave's tiles j in (lo, hi): T_k = import ? G_j L^T : T_k - G_j G_r^T,
// NB payloads in flight (after wait_bulk)
template <int TPW, bool IMPORT, class Get, class Set>
__device__ __forceinline__ void bulk_update(const Args &a, const Rs &rs, int p, int w, int lo, int hi, const d4 &m,
                                            int lane, Get &&tget, Set &&tset) {
    const __amdgpu_buffer_rsrc_t rd = rsrc(rs.Gd);
#pragma unroll
    for (int k0 = 0; k0 < TPW; k0 += NB) {
        bool nd[NB], any = false;
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            const int j = w + NUW * (k0 + q);
            nd[q] = k0 + q < TPW && j > lo && j < hi;
            any |= nd[q];
        }
        if (!any) continue;
        u32x4 x[NB][2];
#pragma unroll
        for (int q = 0; q < NB; ++q)
            if (nd[q]) {
                const int so = __builtin_amdgcn_readfirstlane(gdoff(a, p, w + NUW * (k0 + q)));
#pragma unroll
                for (int h = 0; h < 2; ++h) x[q][h] = __builtin_amdgcn_raw_buffer_load_b128(rd, h * 1024 + lane * 16, so, SC1);
            }
#pragma unroll
        for (int q = 0; q < NB; ++q)
            if (nd[q]) {
                const int k = k0 + q < TPW ? k0 + q : 0;
                if (IMPORT) tset(k, mfma4(zero4(), dec_bulk(x[q]), m));
                else tset(k, mfma4(tget(k), -dec_bulk(x[q]), m));
            }
    }
}

// (G y)(l & 15) on every lane, from the G fragment and y(l & 15): fixed order
__device__ __forceinline__ double gy(const d4 &g, double yl, int lane) {
    double s = 0.0;
#pragma unroll
    for (int e = 0; e < 4; ++e) s = fma(g[e], __shfl(yl, 4 * e + (lane >> 4)), s);
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    return s;
}

// tile A_rj of the damped, identity-padded system, held as the accumulator
// of A_rj^T: element e of lane l = A(16 r + (l & 15), 16 j + (l >> 4) + 4e)
// a strictly lower tile (j <= r - 2: no diagonal element, no damping) of the
// U waves' prologue from the payload: pay_index in 32-bit arithmetic with the
// lane's row terms hoisted, zero unless live, every load unconditional (in
// bounds) so that a group of tiles has its loads in flight together
__device__ __forceinline__ d4 load_lower(const Args &a, int r, int j, int lane) {
    const int I = TL * r + (lane & 15), nc = (a.ns + 5) / 6;
    const int ib = I / 6, ir = I - 6 * ib;
    const bool live = j <= r - 2 && I < a.ns;
    int idx[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int J = TL * j + (lane >> 4) + 4 * e, jb = J / 6, jr = J - 6 * jb;
        // J < I: block (jb, ib) of the upper block triangle; inside one
        // camera block the element (ir, jr), as the 64-bit pay_index takes it
        const int blk = 36 * (jb * nc - jb * (jb - 1) / 2 + ib - jb);
        idx[e] = live ? blk + (ib == jb ? ir * 6 + jr : jr * 6 + ir) : 0;
    }
    d4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = a.payload[idx[e]];
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (!live) v[e] = 0.0;
    return v;
}
__device__ __forceinline__ d4 load_tile(const Args &a, double lambda, int r, int j, int lane) {
    if (a.src.slab) {  // from the slabs: the finish's sums, in its order (the same bits)
        d4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e)
            v[e] = assembled_src(a.src, a.payload, a.ns, lambda, TL * r + (lane & 15), TL * j + (lane >> 4) + 4 * e);
        return v;
    }
    gj::ElemRef er[4];
    double v[4], dg[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) er[e] = gj::elem_ref(a.ns, TL * r + (lane & 15), TL * j + (lane >> 4) + 4 * e);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        v[e] = er[e].idx >= 0 ? a.payload[er[e].idx] : er[e].pad;
        dg[e] = er[e].dg >= 0 ? a.payload[er[e].dg] : 0.0;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (er[e].dg >= 0) v[e] += lambda * clampd(dg[e]);
    return d4{v[0], v[1], v[2], v[3]};
}

// uses of ring slot p % RING before step p: by the G pieces (every step but
// r) and by the L^-1 pieces for a holder (every step but r - 1 and r).
// Measured and not kept (round 4): the critical step's G kept out of the
// ring (the U waves skip step r - 1, where they have no live tile): cfg4
// 0.0848 -> 0.0834 ms but cfg5 0.301 -> 0.346 ms
__device__ __forceinline__ int g_uses(int p, int r) {
    return p / RING - (r < p && (r & (RING - 1)) == (p & (RING - 1)) ? 1 : 0);
}
__device__ __forceinline__ int p_uses(int p, int r) {
    int u = g_uses(p, r);
    if (r >= 1 && r - 1 < p && ((r - 1) & (RING - 1)) == (p & (RING - 1))) --u;
    return u;
}

// ------------------------------------------------------------------- W0
// The pivot: the chain on the diagonal tile with the b row (lane 0) and the
// identity (lanes 16..31) as panel rows -> L_r (rows), y_r, L_r^-T rows.
// Publishes P_r; leaves L_r^-1 in S.Li and the L_r fragment in S.Lf.
__device__ __forceinline__ void pivot(const Args &a, const Rs &rs, Smem &S, int r, int lane, const d4 &Td, double b) {
    const int li = lane & 15, grp = lane >> 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) S.Dm[li][grp + 4 * e] = Td[e];  // symmetric: column li = row li
    if (lane < 16) S.bv[lane] = b;
    wave_lds();
    double rw[16], pw[16], dinv[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) rw[j] = S.Dm[li][j];
#pragma unroll
    for (int j = 0; j < 16; ++j) pw[j] = grp == 0 ? (lane == 0 ? S.bv[j] : 0.0) : (grp == 1 && j == li ? 1.0 : 0.0);
    stamp(a, r, DBG_CHAIN0);
    gj::gj_factor16(rw, pw, dinv, lane, a.bad);
    stamp(a, r, DBG_CHAIN1);
    if (grp == 1)
#pragma unroll
        for (int j = 0; j < 16; ++j) S.Li[j][li] = pw[j];  // row li of L^-T = column li of L^-1
    if (lane == 0)
#pragma unroll
        for (int j = 0; j < 16; ++j) S.yv[j] = pw[j];
    wave_lds();
    d4 lv;
#pragma unroll
    for (int e = 0; e < 4; ++e) lv[e] = S.Li[li][4 * e + grp];  // L^-1(l & 15, 4e + (l >> 4))
    const double yr = S.yv[li];
    put4<0>(rs.P, (a.nT + r) * PBYTES, a.tag, lv, lane);  // the L2-local copy first (the next owner)
    put_pair<0>(rs.P, (a.nT + r) * PBYTES, 4, a.tag, yr, lane);
    put4(rs.P, r * PBYTES, a.tag, lv, lane);
    put_pair(rs.P, r * PBYTES, 4, a.tag, yr, lane);
    stamp(a, r, DBG_PPUB);
    // the L_r rows (for the import's fragment) after the publication
    if (grp == 0)
#pragma unroll
        for (int j = 0; j < 16; ++j) S.Dm[li][j] = j <= li ? rw[j] : 0.0;
    wave_lds();
#pragma unroll
    for (int e = 0; e < 4; ++e) S.Lf[e][lane] = S.Dm[li][4 * e + grp];
    lds_release();
    lds_set(&S.lready, 1);
}

// W0 of owner r: A_r,r-1 (Tm), A_rr (Td), b_r; the pivot records of every
// step (L^-1 into the ring for the holder of A_rp, y_p for b_r)
__device__ __forceinline__ bool w0_loop(const Args &a, const Rs &rs, Smem &S, int r, int lane, double lambda) {
    const int nT = a.nT, li = lane & 15;
    d4 Tm = r > 0 ? load_tile(a, lambda, r, r - 1, lane) : zero4();
    d4 Td = load_tile(a, lambda, r, r, lane);
    double b = assembled_b_src(a.src, a.payload, a.ns, TL * r + li);
    stamp(a, nT, DBG_PROLOGUE);
    d4 gc = zero4();  // G_r of the critical step: its bulk copy goes out after the pivot
    for (int p = 0; p < nT; ++p) {
        const int s = p & (RING - 1);
        double yl = 0.0;
        d4 lv = zero4();
        if (p != r) {
            const int soff[1] = {p * PBYTES};
            const bool need[1] = {true};
            u32x4 v[1][PPAIRS];
            if (p == r - 1 && xcd_of_row(p, nT) == xcd_of_row(r, nT)) {
                if (!poll_p2(rs.P, p * PBYTES, (nT + p) * PBYTES, a.tag, v[0], lane, S)) return false;
            } else if (!sweep<1, PPAIRS>(rs.P, soff, need, a.tag, v, lane, S)) {
                return false;
            }
            stamp(a, p, DBG_PIN);
            lv = dec4(v[0]);
            yl = dec(v[0][4]);
            if (p != r - 1) {  // the holder of A_rp forms G_r from L_p^-1
                if (!lds_wait(&S.pdone[s], p_uses(p, r), S)) return false;
                stamp(a, p, DBG_PLW);
#pragma unroll
                for (int e = 0; e < 4; ++e) S.PL[s][e][lane] = lv[e];
                lds_release();
                lds_set(&S.pready[s], p + 1);
            }
        }
        if (p == r - 1) {  // the critical step: G_r, its publication, A_rr, then the pivot
            const d4 g = mfma4(zero4(), lv, Tm);
            put4(rs.G, gsoff(a, p, r), a.tag, g, lane);  // owner r + 1 waits for it first
            gc = g;
            stamp(a, p, DBG_GCRIT);
            Td = mfma4(Td, -g, g);
            b -= gy(g, yl, lane);
        } else if (p == r) {
            pivot(a, rs, S, r, lane, Td, b);
            if (r > 0) {
                put_bulk(rs.Gd, gdoff(a, r - 1, r), gc, lane);
                flag_bulk(a, r - 1, r);
                // the ring piece of the critical step r - 1, after the pivot
                // record is out: no U wave has a live tile at step r - 1, they
                // only count the slot, so it leaves the critical path
                const int sc = (r - 1) & (RING - 1);
                if (!lds_wait(&S.gdone[sc], NW * g_uses(r - 1, r), S)) return false;
#pragma unroll
                for (int e = 0; e < 4; ++e) S.GL[sc][e][lane] = gc[e];
                lds_release();
                lds_set(&S.gready[sc], r);
                lds_add(&S.gdone[sc], 1);
            }
        } else {
            // G_{r-1} of this step (for A_r,r-1) first: owner r - 1 publishes
            // it as soon as it has P_p, so its round trip overlaps the holder's
            // work on G_r instead of following it (this wave reaches the next
            // step's poll, the critical one at p = r - 2, one round trip sooner)
            d4 gm = zero4();
            if (p < r) {
                const int soff[1] = {gsoff(a, p, r - 1)};
                const bool need[1] = {true};
                u32x4 v[1][GPAIRS];
                if (!sweep<1, GPAIRS>(rs.G, soff, need, a.tag, v, lane, S)) return false;
                stamp(a, p, DBG_GREM);
                gm = dec4(v[0]);
            }
            if (!lds_wait(&S.gready[s], p + 1, S)) return false;
            stamp(a, p, DBG_GRDY);
            d4 g;
#pragma unroll
            for (int e = 0; e < 4; ++e) g[e] = S.GL[s][e][lane];
            lds_release();
            lds_add(&S.gdone[s], 1);
            b -= gy(g, yl, lane);
            if (p < r) {  // A_rr and A_r,r-1
                Td = mfma4(Td, -g, g);
                Tm = mfma4(Tm, -gm, g);
            }
        }
    }
    // x_r = L_r^-T (L_r^-1 b_r)
    if (lane < 16) S.bv[lane] = b;
    wave_lds();
    double u = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) u = fma(S.Li[li][k], S.bv[k], u);
    if (lane < 16) S.yv[lane] = u;
    wave_lds();
    double x = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) x = fma(S.Li[i][li], S.yv[i], x);
    if (lane < 16) __hip_atomic_store(a.x + TL * r + lane, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    stamp(a, nT, DBG_W0END);
    return true;
}

// ------------------------------------------------------------- U waves
// U_w of owner r holds the tiles j = w + NUW k (k < TPW) other than r - 1
// and r: the lower ones from the start, the ones right of the diagonal from
// the import at its pivot.  Per step: the holder of A_rp forms G_r (and
// publishes it while r is unpivoted); every U wave applies it to its live
// tiles j in (p, hi), two tiles' remote G loads in flight at a time.
// Slots: TR in registers, TLS more in LDS (tl: this wave's [TLS][4][64]
// doubles; large systems only, the register file holds 11 a wave).
template <int TR, int TLS>
__device__ __forceinline__ bool u_loop(const Args &a, const Rs &rs, Smem &S, int r, int w, int lane, double lambda,
                                       double *tl) {
    constexpr int TPW = TR + TLS;
    const int nT = a.nT;
    d4 T[TR];
    auto tget = [&](int k) -> d4 {  // k is a constant after unrolling: the branch folds
        if (k < TR) return T[k < TR ? k : 0];
        const double *q = tl + (k - TR) * 256 + lane;
        return d4{q[0], q[64], q[128], q[192]};
    };
    auto tset = [&](int k, const d4 &v) {
        if (k < TR) {
            T[k < TR ? k : 0] = v;
            return;
        }
        double *q = tl + (k - TR) * 256 + lane;
        q[0] = v[0];
        q[64] = v[1];
        q[128] = v[2];
        q[192] = v[3];
    };
    // PG tiles at a time from the payload (their loads in flight together:
    // the late owners' U waves start their first step sooner, cfg5 0.296 ->
    // 0.290 ms) when a wave holds more than 4 tiles (with 4, cfg4, the same
    // change cost 0.081 -> 0.085 ms), else a tile at a time (and always from
    // the slabs, SlabSrc); loops that are not unrolled (all the loads at once
    // would spill), the slot chosen by selects
    if (TPW > 4 && !a.src.slab) {
#pragma unroll
        for (int kk = 0; kk < TR; ++kk) T[kk] = zero4();  // tiles right of r - 2: set by the import
        constexpr int PG = 4;
#pragma unroll 1
        for (int k0 = 0; k0 < TPW; k0 += PG) {
            if (w + NUW * k0 > r - 2) break;  // nothing live from here on
            d4 v[PG];
#pragma unroll
            for (int q = 0; q < PG; ++q) v[q] = load_lower(a, r, w + NUW * (k0 + q), lane);
#pragma unroll
            for (int q = 0; q < PG; ++q) {
                const int k = k0 + q;
#pragma unroll
                for (int kk = 0; kk < TR; ++kk)
                    if (kk == k) T[kk] = v[q];
                if (k >= TR && k < TPW) tset(k, v[q]);
            }
        }
    } else {
#pragma unroll 1
        for (int k = 0; k < TPW; ++k) {
            const int j = w + NUW * k;
            const d4 v = j <= r - 2 ? load_tile(a, lambda, r, j, lane) : zero4();
#pragma unroll
            for (int kk = 0; kk < TR; ++kk)
                if (kk == k) T[kk] = v;
            if (k >= TR) tset(k, v);
        }
    }
    for (int p = 0; p < nT; ++p) {
        const int s = p & (RING - 1);
        if (p == r) {  // the import: A_rj^T = G_j L_r^T for j > r (G_j of step r from owner j)
            bool any = false;
#pragma unroll
            for (int k = 0; k < TPW; ++k) any |= w + NUW * k > r && w + NUW * k < nT;
            if (!any) continue;
            if (!lds_wait(&S.lready, 1, S)) return false;
            d4 lf;
#pragma unroll
            for (int e = 0; e < 4; ++e) lf[e] = S.Lf[e][lane];
            if (!wait_bulk<TPW>(a, p, w, r, nT, lane, S)) return false;
            bulk_update<TPW, true>(a, rs, p, w, r, nT, lf, lane, tget, tset);
            continue;
        }
        if (p % NUW == w && p != r - 1) {  // holder of A_rp: G_r = A_rp L_p^-T
            if (!lds_wait(&S.pready[s], p + 1, S)) return false;
            stamp(a, p, DBG_HPRDY);
            d4 lv;
#pragma unroll
            for (int e = 0; e < 4; ++e) lv[e] = S.PL[s][e][lane];
            lds_release();
            lds_add(&S.pdone[s], 1);
            d4 tp = zero4();
#pragma unroll
            for (int k = 0; k < TPW; ++k)
                if (k == p / NUW) tp = tget(k);
            const d4 g = mfma4(zero4(), lv, tp);
            if (!lds_wait(&S.gdone[s], NW * g_uses(p, r), S)) return false;
#pragma unroll
            for (int e = 0; e < 4; ++e) S.GL[s][e][lane] = g[e];
            lds_release();
            lds_set(&S.gready[s], p + 1);
            stamp(a, p, DBG_GHOLD);
            if (r > p) {  // for W0 of owner r + 1 (granules) and every other owner's U waves (bulk)
                put4(rs.G, gsoff(a, p, r), a.tag, g, lane);
                put_bulk(rs.Gd, gdoff(a, p, r), g, lane);
                flag_bulk(a, p, r);
            }
        }
        const int hi = r > p ? r - 1 : nT;  // live tiles j in (p, hi); W0 holds r - 1 and r
        if (!lds_wait(&S.gready[s], p + 1, S)) return false;
        d4 g;
#pragma unroll
        for (int e = 0; e < 4; ++e) g[e] = S.GL[s][e][lane];
        lds_release();
        lds_add(&S.gdone[s], 1);
        if (!wait_bulk<TPW>(a, p, w, p, hi, lane, S)) return false;
        bulk_update<TPW, false>(a, rs, p, w, p, hi, g, lane, tget, tset);
        if (w == 0) stamp(a, p, DBG_UDONE);
    }
    return true;
}

template <int TR, int TLS>
__global__ void __launch_bounds__(THREADS) k_gjr_solve(Args a) {
    if (a.gate && !*a.gate) return;  // device-side LM control: iteration gated off
    __shared__ Smem S;
    extern __shared__ __attribute__((aligned(16))) double dyn[];  // LDS tile slots, then the epilogue's scratch
    static_assert(NUW * TLS * 256 * sizeof(double) <= DYN_LDS, "LDS tile slots");
    stamp(a, a.nT, DBG_START);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = row_of(blockIdx.x, a.nT);
    const double lambda = *a.lam;
    if (threadIdx.x < RING) S.pready[threadIdx.x] = S.pdone[threadIdx.x] = S.gready[threadIdx.x] = S.gdone[threadIdx.x] = 0;
    if (threadIdx.x == 0) {
        S.lready = S.abort_ = S.last = 0;
        S.err = a.err;
        S.bad = a.bad;
    }
    Rs rs;
    rs.P = Buf{a.P, 2 * a.nT * PBYTES};
    rs.G = Buf{a.G, a.nT * a.nT * GBYTES};
    rs.Gd = Buf{a.Gd, a.nT * a.nT * GDBYTES};
    __syncthreads();
    const int wu = __builtin_amdgcn_readfirstlane(wave);  // provably uniform: scalar record offsets
    if (wu == 0) w0_loop(a, rs, S, r, lane, lambda);
    else u_loop<TR, TLS>(a, rs, S, r, wu - 1, lane, lambda, dyn + (wu - 1) * TLS * 256);
    // every owner arrives (an aborted one too, so the count stays whole); the
    // last one forms the trial cameras unless the solve failed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // W0's x stores drained before the barrier
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add(a.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == (unsigned)a.nT - 1) {
            __hip_atomic_store(a.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            S.last = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
        }
    }
    __syncthreads();
    stamp(a, a.nT, DBG_ARRIVED);
    if (!S.last || a.ct.nc <= 0) return;
    double *dc = dyn, *red = dyn + NTMAX * TL;
    static_assert((NTMAX * TL + 3 * THREADS) * sizeof(double) <= DYN_LDS, "epilogue scratch");
    for (int i = threadIdx.x; i < 6 * a.ct.nc; i += THREADS)
        dc[i] = __hip_atomic_load(a.x + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    gj::cam_trial<THREADS>(a.ct.nc, a.ct.Rt, a.ct.Rt_new, a.ct.cam_out, *a.lam, a.payload, a.ns, dc, red,
                           a.src.slab ? a.src.camlin : nullptr);
}

}  // namespace gjr
