// Persistent block Gauss-Jordan solve of the damped reduced camera system
// (S + lambda clamp(diag U)) x = b in ONE launch (round 3).  Replaces the
// reference's MINPACK dense QR step (Phase 1/BundleAdjustment.py:205-212, via
// scipy lmdif) on the BA hot path; included by ba.hip after the assembly
// helpers (SlabSrc, assembled_src) and the 16-pivot DPP tile factor.
//
// Why Gauss-Jordan: a tiled Cholesky needs nT = nsp / 16 dependent column
// steps for the factor and as many again for the back substitution.  As one
// launch per column (k_chol_col) each step costs a kernel boundary plus a
// round of cross-XCD tile loads (~5.4 us at cfg4); the back substitution is
// a further serial chain.  Block Gauss-Jordan with Cholesky pivots
//   step p:  L_p = chol(A_pp);  G_i = A_ip L_p^-T (every row tile i != p);
//            y_p = L_p^-1 b_p;  A_ij -= G_i G_j^T (j > p);  b_i -= G_i y_p
//   end:     x_i = L_i^-T L_i^-1 b_i   (block diagonal left over)
// has no back substitution at all (its extra flops are off the critical
// path), and every step's dependency is only "column p+1 updated by panel
// p".  A_pj (j > p) is never read: the trailing matrix is symmetric, so
// L_p^-1 A_pj = G_j^T.  Rows above the pivot (already pivoted) keep being
// updated; a tile (i, j) with p < i < j (the mirror of (j, i)) is not kept
// and is imported when row i becomes pivoted: A_ij = L_i G_j^T.
//
// Work split: workgroup (cb, s) owns the column tiles [cb*CB, cb*CB + CB)
// restricted to the row tiles [s*SR, s*SR + SR) ("segment" s), plus a
// replica of the diagonal tile and of b for each of its columns.  Every
// workgroup of a column block factors each diagonal tile itself (the same
// operations on the same values, so the same bits), so the next pivot of a
// column block waits for no other workgroup unless its tile row sits in
// another segment; panels go between workgroups through global memory
// (write-through stores, one flag per (panel, segment), epoch-tagged).
//
// Waves of a workgroup (dataflow through LDS words, no workgroup barrier in
// the loop):
//   W0  the pivot chain: chol_factor16 on the diagonal replica with the
//       segment's 64 rows of the pivot column on its lanes -> L_p, G rows;
//   W1  the same chain with b_p on one lane -> y_p (and publishes L_p, y_p);
//   WL  loader: polls the flags of remote panels / tiles and stages them;
//   WP  publisher: copies this workgroup's pivots (G rows, L_p, y_p) from LDS
//       to global memory and raises their flags (off the chain waves' path);
//   U*  update waves: each owns up to TPW tiles in MFMA C-fragment layout
//       (v_mfma_f64_16x16x4f64: the VALU stays free for the chains) and
//       applies every panel; the tiles of column p+1 first (phase A, then
//       staged for the next chain), the rest after (phase B).
namespace gj {

constexpr int TL = 16;       // tile
constexpr int SR = 4;        // row tiles per segment (64 rows: W0's lanes)
constexpr int CBMAX = 8;     // column tiles per workgroup
constexpr int NUW = 8;       // update waves
constexpr int NW = 4 + NUW;  // W0, W1, WL, WP, U0..U7
constexpr int THREADS = 64 * NW;
constexpr int NCONS = NUW + 2;  // consumers of a panel's LDS buffers: the update waves, W1 and WP
constexpr int TPW = ((SR + 1) * CBMAX + NUW - 1) / NUW;  // tile slots per update wave
constexpr int LDT = TL + 1;                              // padded LDS row (doubles)
constexpr int NTMAX = 128;                               // tiles per dimension (host checks)
constexpr long long POLL_LIMIT = 20000000;               // s_memrealtime ticks (100 MHz): 200 ms
constexpr unsigned SPIN_CHECK = 1024;                    // polls between two reads of the clock

typedef double d4 __attribute__((ext_vector_type(4)));

struct Args {
    const double *payload;  // the finished (all-reduced) Schur payload
    int32_t ns, nT, cb, nseg;
    const double *lam;
    const int *gate;
    double *Gp;        // [nT][nT*16][16] published panels (G rows)
    double *Lp;        // [nT][nseg][256] L_p, one copy per producing segment
    double *Yp;        // [nT][nseg][16]
    int *flag;         // [nT][nseg] epoch of the last publication
    int epoch;
    double *x;         // [nT*16] solution
    int *bad;          // not positive definite (LM rejects the step)
    int *err;          // a poll timed out (host reports an error)
    unsigned *arrive;  // last-block arrivals (the last one runs the epilogue)
    CamTrialArgs ct;   // trial cameras epilogue (nc = 0: none)
    long long *dbg;    // diagnostics (nullable): [grid][nT][16] s_memrealtime stamps
};

// diagnostic stamps (sfm_gj_debug): slot per (workgroup, panel)
// (row nT of a workgroup: the kernel-wide phases)
enum { DBG_CST = 0, DBG_CHAIN, DBG_PUB, DBG_LOAD0, DBG_LOADED, DBG_GM, DBG_PHA, DBG_PHB,
       DBG_W0BUF, DBG_W0GST, DBG_W0LDS, DBG_W0DRAIN, DBG_AGJ, DBG_ACST, DBG_AMMA, DBG_ABB };
enum { DBG_START = 0, DBG_PROLOGUE, DBG_FINWAIT, DBG_FINSOLVED, DBG_ARRIVED, DBG_EPILOGUE };
__device__ __forceinline__ void stamp(const Args &a, int p, int slot) {
    if (a.dbg && (threadIdx.x & 63) == 0)
        a.dbg[((int64_t)blockIdx.x * (a.nT + 1) + p) * 16 + slot] = __builtin_amdgcn_s_memrealtime();
}

struct Smem {
    // Gm and Gj (adjacent) double as the prologue's staging of the tiles
    double Gm[2][SR][TL][LDT];     // panel p: G rows of the segment's row tiles
    double Gj[2][CBMAX][TL][LDT];  // panel p: G tile of each owned column's row
    double Cst[SR + 1][TL][LDT];   // column p+1 staged for the chain (own tiles | replica)
    double Ls[2][TL][LDT];         // L_p (the import A_pj = L_p G_j^T)
    double ys[2][TL];
    double bb[CBMAX][TL];          // b replica of each owned column's row tile
    double ob[SR * TL];            // b of the segment's rows (last column block)
    int gm_ok[2], ly_ok[2], gj_ok[2][CBMAX];  // = p + 1 when panel p's piece is staged
    int bb_cnt[CBMAX];  // panels applied to each b replica (W1: column p + 1; the replica's update wave: the rest)
    int cst_cnt, cst_read, abort_;
    int udone[NTMAX];  // per panel: update waves and W1 done with it (groups progress at different
                       // rates, so a single running count would not say which panels are done)
    int *err, *bad;  // global: set on an abort (the host reports it, the LM rejects the step)
};

__device__ __forceinline__ double ld_ag(const double *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ag(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int lds_ld(const int *w) {
    return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local"); }
__device__ __forceinline__ void lds_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local"); }
__device__ __forceinline__ void lds_set(int *w, int v) {  // after lds_release()
    __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_add(int *w, int v) {
    __hip_atomic_fetch_add(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ long long rtc() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void abort_solve(Smem &S) {
    lds_set(&S.abort_, 1);
    if ((threadIdx.x & 63) == 0) {
        __hip_atomic_store(S.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(S.bad, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// wait (whole wave) until the LDS word reaches target; false on abort / timeout
__device__ __forceinline__ bool lds_wait(const int *w, int target, Smem &S) {
    if (lds_ld(w) >= target) {  // the common case: no clock read, no sleep
        lds_acquire();
        return true;
    }
    long long t0 = -1;
    for (unsigned it = 1;; ++it) {
        __builtin_amdgcn_s_sleep(1);
        if (lds_ld(w) >= target) break;
        if (lds_ld(&S.abort_)) return false;
        if (it % SPIN_CHECK == 0) {  // bounded: a lost hand-off ends the solve, never hangs the GPU
            const long long t = rtc();
            if (t0 < 0) t0 = t;
            else if (t - t0 > POLL_LIMIT) {
                abort_solve(S);
                return false;
            }
        }
    }
    lds_acquire();
    return true;
}

// wait (whole wave) for a remote publication: flag >= epoch (relaxed agent
// loads; the producer's stores are write-through and drained before the flag)
__device__ __forceinline__ bool flag_wait(const int *f, int epoch, Smem &S) {
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= epoch) return true;
    long long t0 = -1;
    for (unsigned it = 1;; ++it) {
        __builtin_amdgcn_s_sleep(1);
        if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= epoch) return true;
        if (lds_ld(&S.abort_)) return false;
        if (it % (SPIN_CHECK / 8) == 0) {
            const long long t = rtc();
            if (t0 < 0) t0 = t;
            else if (t - t0 > POLL_LIMIT) {
                abort_solve(S);
                return false;
            }
        }
    }
}

// acc(r, c) += sa * sum_k Ar[r][k] Br[c][k] on fp64 MFMA 16x16x4 (lane maps
// checked by tools/mfma_map.hip: A lane l = A[l&15][4q + l>>4], B lane l =
// B[4q + l>>4][l&15], D lane l element e = D[(l>>4) + 4e][l&15])
__device__ __forceinline__ d4 mma16(d4 acc, const double (*Ar)[LDT], const double (*Br)[LDT], bool neg, int l) {
    const int r = l & 15, kq = l >> 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        double av = Ar[r][4 * q + kq];
        if (neg) av = -av;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, Br[r][4 * q + kq], acc, 0, 0, 0);
    }
    return acc;
}


// element (I, J) of S + lambda clamp(diag U) from the payload, the lower
// triangle mirrored (what a Cholesky of S reads), identity on the padding;
// the loads are issued by the caller (batched)
struct ElemRef {
    int64_t idx, dg;  // payload index of S_IJ (-1: padding), of diag U_I (-1: off-diagonal)
    double pad;       // value on the padding
};
__device__ __forceinline__ ElemRef elem_ref(int32_t ns, int I, int J) {
    if (I < J) {
        const int t = I;
        I = J;
        J = t;
    }
    ElemRef r;
    if (I < ns && J < ns) {
        r.idx = pay_index(ns, I, J);
        r.dg = I == J ? pay_vec_base(ns) + I : -1;
        r.pad = 0.0;
    } else {
        r.idx = -1;
        r.dg = -1;
        r.pad = I == J ? 1.0 : 0.0;
    }
    return r;
}

struct Geo {
    int cb, s, j0, j1, ncol, i0, i1, nrow, nT, nseg, wpg;
    __device__ int seg_of(int tile) const { return tile / SR; }
    // slot k of update wave u -> owned tile (jj, ii) (ii == SR: the replica),
    // false if none.  The owned columns are grouped by the segment of their
    // tile row (CB / SR groups), each group served by its own waves, so a
    // group whose G tiles come from a lagging workgroup never holds up the
    // tiles of the pivot column.
    __device__ __forceinline__ bool slot(int u, int k, int &jj, int &ii) const {
        const int grp = u / wpg, t = u % wpg + wpg * k, jl = t / (SR + 1);
        ii = t % (SR + 1);
        jj = grp * SR + jl;
        return jl < SR && jj < ncol && (ii == SR || ii < nrow);
    }
};

// ------------------------------------------------- the 16-pivot tile factor
// Every 16-lane row of the wave holds the rows of the diagonal tile (r[j] =
// element (li, j)) and one row of the panel (p[j]); pivot k scales column k
// by 1/L_kk and subtracts L_jk (lane j's r[k], DPP row_newbcast) times it
// from columns j > k, with v_fmac_f64_dpp's neg modifier (no negated copies).
// Unlike chol_factor16 (k_chol_col) the next pivot's 1/sqrt is started as
// soon as its column is updated and its four dependent operations (v_rsq_f64
// and one Newton step, ~1 ulp) are interleaved with the remaining updates of
// the current pivot, so the chain's latency hides under their issue.  Every
// instruction is inline asm in program order; s_nop 1 gives a DPP read of a
// just-written VGPR its two wait states.
template <int J>
__device__ __forceinline__ void gj_upd2(double &rj, double &pj, double rk, double pk) {
    asm volatile("v_fmac_f64_dpp %0, %2, -%2 row_newbcast:%4 row_mask:0xf bank_mask:0xf\n\t"
                 "v_fmac_f64_dpp %1, %2, -%3 row_newbcast:%4 row_mask:0xf bank_mask:0xf"
                 : "+v"(rj), "+v"(pj) : "v"(rk), "v"(pk), "n"(J));
}
struct NewtonState {
    double d, h, g0, a, b, c15;
};
template <int STEP>
__device__ __forceinline__ void gj_newton(NewtonState &n) {  // g1 = g0 (1.5 - (d/2) g0^2)
    if constexpr (STEP == 0) asm volatile("v_mul_f64 %0, %1, %2" : "=v"(n.a) : "v"(n.h), "v"(n.g0));
    if constexpr (STEP == 1) asm volatile("v_fma_f64 %0, -%1, %2, %3" : "=v"(n.b) : "v"(n.a), "v"(n.g0), "v"(n.c15));
    if constexpr (STEP == 2) asm volatile("v_mul_f64 %0, %1, %2" : "=v"(n.g0) : "v"(n.g0), "v"(n.b));
}
// updates of columns K+2+U.. of pivot K, the Newton steps after updates 1, 3, 5
template <int K, int U>
__device__ __forceinline__ void gj_rest(double (&r)[16], double (&p)[16], NewtonState &n) {
    if constexpr (K + 2 + U <= 15) {
        gj_upd2<K + 2 + U>(r[K + 2 + U], p[K + 2 + U], r[K], p[K]);
        if constexpr (U == 1) gj_newton<0>(n);
        if constexpr (U == 3) gj_newton<1>(n);
        if constexpr (U == 5) gj_newton<2>(n);
        gj_rest<K, U + 1>(r, p, n);
    } else {  // fewer updates than Newton steps: the rest back to back
        if constexpr (U <= 1) gj_newton<0>(n);
        if constexpr (U <= 3) gj_newton<1>(n);
        if constexpr (U <= 5) gj_newton<2>(n);
    }
}
template <int K>
__device__ __forceinline__ void gj_step(double (&r)[16], double (&p)[16], double (&dinv)[16], NewtonState &n,
                                        bool &nonpos) {
    const double g = n.g0;
    asm volatile("v_mul_f64 %0, %0, %2\n\tv_mul_f64 %1, %1, %2" : "+v"(r[K]), "+v"(p[K]) : "v"(g));
    dinv[K] = g;
    if constexpr (K < 15) {
        asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %2, -%2 row_newbcast:%4 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %1, %2, -%3 row_newbcast:%4 row_mask:0xf bank_mask:0xf"
                     : "+v"(r[K + 1]), "+v"(p[K + 1]) : "v"(r[K]), "v"(p[K]), "n"(K + 1));
        asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
                     : "=v"(n.d) : "v"(r[K + 1]), "n"(K + 1));
        asm volatile("v_rsq_f64 %0, %1" : "=v"(n.g0) : "v"(n.d));
        asm volatile("v_mul_f64 %0, %1, 0.5" : "=v"(n.h) : "v"(n.d));
        nonpos |= !(n.d > 0.0);
        gj_rest<K, 0>(r, p, n);
    }
}
template <int... K>
__device__ __forceinline__ void gj_steps(double (&r)[16], double (&p)[16], double (&dinv)[16], NewtonState &n,
                                         bool &nonpos, std::integer_sequence<int, K...>) {
    (gj_step<K>(r, p, dinv, n, nonpos), ...);
}
__device__ __forceinline__ void gj_factor16(double (&r)[16], double (&p)[16], double (&dinv)[16], int lane,
                                            int *bad) {
    NewtonState n;
    n.c15 = 1.5;
    asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:0 row_mask:0xf bank_mask:0xf" : "=v"(n.d) : "v"(r[0]));
    asm volatile("v_rsq_f64 %0, %1" : "=v"(n.g0) : "v"(n.d));
    asm volatile("v_mul_f64 %0, %1, 0.5" : "=v"(n.h) : "v"(n.d));
    bool nonpos = !(n.d > 0.0);
    gj_newton<0>(n);
    gj_newton<1>(n);
    gj_newton<2>(n);
    gj_steps(r, p, dinv, n, nonpos, std::make_integer_sequence<int, 16>{});
    if (lane == 0 && nonpos) *bad = 1;
}

// -------------------------------------------------------------- the chain
// W0 / W1: pivot p from the staged column (Cst).  W0 carries the segment's
// rows, W1 the b row; both factor the same replica (same bits).  Only LDS
// is written here (this workgroup's next pivot waits on it); WP writes the
// global copy for the other workgroups.
__device__ __forceinline__ bool chain_pivot(const Args &a, const Geo &g, Smem &S, int p, int wave, int lane) {
    const int li = lane & 15, grp = lane >> 4, buf = p & 1;
    double rw[16], pw[16], dinv[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) rw[j] = S.Cst[SR][li][j];
    if (wave == 0) {
#pragma unroll
        for (int j = 0; j < 16; ++j) pw[j] = grp < g.nrow ? S.Cst[grp][li][j] : 0.0;
    } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) pw[j] = lane == 0 ? S.bb[p - g.j0][j] : 0.0;
    }
    lds_release();
    if (lane == 0) lds_add(&S.cst_read, 1);  // Cst may be restaged (phase A of panel p)
    if (wave == 0) stamp(a, p, DBG_CST);
    gj_factor16(rw, pw, dinv, lane, a.bad);
    if (wave == 0) stamp(a, p, DBG_CHAIN);
    // panel p's buffers were last read by the consumers of panel p - 2
    if (p >= 2 && !lds_wait(&S.udone[p - 2], NCONS, S)) return false;
    if (wave == 0) {
        stamp(a, p, DBG_W0BUF);
        if (grp < g.nrow) {
#pragma unroll
            for (int j = 0; j < 16; ++j) S.Gm[buf][grp][li][j] = pw[j];
            const int tj = g.i0 + grp - g.j0;  // this row tile is an owned column's row: its G tile is local
            if (tj >= 0 && tj < g.ncol && g.i0 + grp > p)
#pragma unroll
                for (int j = 0; j < 16; ++j) S.Gj[buf][tj][li][j] = pw[j];
        }
        lds_release();
        if (lane == 0) {
            lds_set(&S.gm_ok[buf], p + 1);
            for (int gg = 0; gg < g.nrow; ++gg) {
                const int tj = g.i0 + gg - g.j0;
                if (tj >= 0 && tj < g.ncol && g.i0 + gg > p) lds_set(&S.gj_ok[buf][tj], p + 1);
            }
        }
        stamp(a, p, DBG_W0LDS);
    } else {
        if (lane < 16) {
#pragma unroll
            for (int j = 0; j < 16; ++j) S.Ls[buf][li][j] = j <= li ? rw[j] : 0.0;
        }
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < 16; ++j) S.ys[buf][j] = pw[j];
        }
        lds_release();
        if (lane == 0) lds_set(&S.ly_ok[buf], p + 1);
    }
    return true;
}

// WP: the global copy of each own pivot's pieces (write-through stores,
// read back from LDS so that every store instruction writes contiguous
// bytes), drained, then the flag; remote panels: nothing to publish
__device__ __forceinline__ void publisher(const Args &a, const Geo &g, Smem &S, int lane) {
    for (int p = 0; p < g.j1; ++p) {
        if (p >= g.j0) {
            const int buf = p & 1;
            if (!lds_wait(&S.gm_ok[buf], p + 1, S) || !lds_wait(&S.ly_ok[buf], p + 1, S)) return;
            double *dst = a.Gp + ((int64_t)p * g.nT * TL + g.i0 * TL) * TL;  // the segment's rows: contiguous
            const int nel = g.nrow * TL * TL;
#pragma unroll
            for (int k = 0; k < SR * TL * TL / 64; ++k) {
                const int e = lane + 64 * k, row = e >> 4;
                if (e < nel) st_ag(dst + e, S.Gm[buf][row >> 4][row & 15][e & 15]);
            }
            double *dl = a.Lp + ((int64_t)p * g.nseg + g.s) * 256;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int e = lane + 64 * k;
                st_ag(dl + e, S.Ls[buf][e >> 4][e & 15]);
            }
            if (lane < 16) st_ag(a.Yp + ((int64_t)p * g.nseg + g.s) * 16 + lane, S.ys[buf][lane]);
            stamp(a, p, DBG_W0GST);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) {
                __hip_atomic_store(a.flag + (int64_t)p * g.nseg + g.s, a.epoch, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                stamp(a, p, DBG_PUB);
            }
        }
        if (lane == 0) lds_add(&S.udone[p], 1);
    }
}

// b replica of owned column jj: bb -= G_j y_p (16 lanes, a row each), in
// panel order (bb_cnt: the panels applied so far), so that every workgroup
// of the column block holds the same bits
__device__ __forceinline__ bool apply_bb(Smem &S, int p, int jj, int lane) {
    const int buf = p & 1;
    if (!lds_wait(&S.bb_cnt[jj], p, S)) return false;
    if (lane < 16) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) acc = fma(S.Gj[buf][jj][lane][k], S.ys[buf][k], acc);
        S.bb[jj][lane] -= acc;
    }
    lds_release();
    if (lane == 0) lds_set(&S.bb_cnt[jj], p + 1);
    return true;
}

// W1's loop: its own pivots' chain (the b row), and for every panel p the
// b replica of column p + 1 (the next pivot reads it; the update waves keep
// the other columns' b replicas)
__device__ __forceinline__ void w1_loop(const Args &a, const Geo &g, Smem &S, int lane) {
    for (int p = 0; p < g.j1; ++p) {
        const int buf = p & 1, ja = p + 1 - g.j0;
        if (p >= g.j0) {
            if (!lds_wait(&S.cst_cnt, (p - g.j0 + 1) * (g.nrow + 1), S) || !chain_pivot(a, g, S, p, 1, lane))
                return;
        }
        if (ja >= 0 && ja < g.ncol) {
            if (!lds_wait(&S.ly_ok[buf], p + 1, S) || !lds_wait(&S.gj_ok[buf][ja], p + 1, S) ||
                !apply_bb(S, p, ja, lane))
                return;
        }
        lds_release();
        if (lane == 0) lds_add(&S.udone[p], 1);
        if (lds_ld(&S.abort_)) return;
    }
}

// ------------------------------------------------------------- the loader
// Stages remote pieces of panel p, one producing segment at a time: the
// segment's flag, then every load from it in one round (the segment's own
// G rows for a remote panel: 16 doubles a lane; the G tiles of the owned
// columns whose tile row it holds: up to SR tiles, 16 doubles a lane), then
// the LDS words.  The segment holding column p+1's tile row goes first.
__device__ __forceinline__ bool load_segment(const Args &a, const Geo &g, Smem &S, int p, int sg, bool rows,
                                             unsigned tiles, int lane) {
    const int nsp = g.nT * TL, buf = p & 1;
    if (!flag_wait(a.flag + (int64_t)p * g.nseg + sg, a.epoch, S)) return false;
    stamp(a, p, DBG_LOAD0);
    // every load in flight at once, 8 B a lane, each instruction 512 B contiguous
    const bool lrow = rows && p >= g.i0 && p < g.i1;  // row p is this segment's: the import needs L_p
    const int nre = rows ? g.nrow * TL * TL : 0;
    double vr[SR * TL * TL / 64], vt[SR][4], vl[4], vy = 0.0;
    const double *gr = a.Gp + ((int64_t)p * nsp + g.i0 * TL) * TL;
#pragma unroll
    for (int k = 0; k < SR * TL * TL / 64; ++k) {
        const int e = lane + 64 * k;
        if (e < nre) vr[k] = ld_ag(gr + e);
    }
#pragma unroll
    for (int t = 0; t < SR; ++t)
        if (tiles >> t & 1) {
            const double *src = a.Gp + ((int64_t)p * nsp + (sg * SR + t) * TL) * TL;
#pragma unroll
            for (int k = 0; k < 4; ++k) vt[t][k] = ld_ag(src + lane + 64 * k);
        }
    if (rows) {
        const double *ls = a.Lp + ((int64_t)p * g.nseg + g.s) * 256;
        if (lrow)
#pragma unroll
            for (int k = 0; k < 4; ++k) vl[k] = ld_ag(ls + lane + 64 * k);
        if (lane < 16) vy = ld_ag(a.Yp + ((int64_t)p * g.nseg + g.s) * 16 + lane);
    }
#pragma unroll
    for (int k = 0; k < SR * TL * TL / 64; ++k) {
        const int e = lane + 64 * k, row = e >> 4;
        if (e < nre) S.Gm[buf][row >> 4][row & 15][e & 15] = vr[k];
    }
#pragma unroll
    for (int t = 0; t < SR; ++t)
        if (tiles >> t & 1) {
            const int jj = sg * SR + t - g.j0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int e = lane + 64 * k;
                S.Gj[buf][jj][e >> 4][e & 15] = vt[t][k];
            }
        }
    if (rows) {
        if (lrow)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int e = lane + 64 * k;
                S.Ls[buf][e >> 4][e & 15] = vl[k];
            }
        if (lane < 16) S.ys[buf][lane] = vy;
    }
    lds_release();
    stamp(a, p, DBG_LOADED);
    if (lane == 0) {
        if (rows) {
            lds_set(&S.gm_ok[buf], p + 1);
            lds_set(&S.ly_ok[buf], p + 1);
        }
        for (int t = 0; t < SR; ++t)
            if (tiles >> t & 1) lds_set(&S.gj_ok[buf][sg * SR + t - g.j0], p + 1);
    }
    return true;
}

__device__ __forceinline__ void loader(const Args &a, const Geo &g, Smem &S, int lane) {
    const int sfirst = g.j0 / SR, slast = (g.j1 - 1) / SR;  // segments of the owned columns' tile rows
    for (int p = 0; p < g.j1; ++p) {
        if (p >= 2 && !lds_wait(&S.udone[p - 2], NCONS, S)) return;  // buffers of panel p - 2 consumed
        const bool remote = p < g.j0;
        // remote G tiles of the owned columns j > p (our own pivot's tiles in our rows come from W0)
        auto tiles_of = [&](int sg) {
            unsigned m = 0;
            for (int t = 0; t < SR; ++t) {
                const int j = sg * SR + t;
                if (j >= g.j0 && j < g.j1 && j > p && (remote || sg != g.s)) m |= 1u << t;
            }
            return m;
        };
        const int scrit = (p + 1 >= g.j0 && p + 1 < g.j1) ? (p + 1) / SR : -1;
        if (scrit >= 0) {
            const unsigned m = tiles_of(scrit);
            const bool rows = remote && scrit == g.s;
            if ((m || rows) && !load_segment(a, g, S, p, scrit, rows, m, lane)) return;
        }
        if (remote && scrit != g.s && !load_segment(a, g, S, p, g.s, true, sfirst <= g.s && g.s <= slast ? tiles_of(g.s) : 0u, lane))
            return;
        for (int sg = sfirst; sg <= slast; ++sg) {
            if (sg == scrit || (remote && sg == g.s)) continue;
            const unsigned m = tiles_of(sg);
            if (m && !load_segment(a, g, S, p, sg, false, m, lane)) return;
        }
    }
}

// ------------------------------------------------------------ update waves
__device__ __forceinline__ void store_cst(Smem &S, int ii, const d4 &acc, int l) {
#pragma unroll
    for (int e = 0; e < 4; ++e) S.Cst[ii][(l >> 4) + 4 * e][l & 15] = acc[e];
}

// apply panel p to tile (jj, ii) (ii == SR: the diagonal replica)
__device__ __forceinline__ void apply_tile(d4 &acc, const Geo &g, Smem &S, int p, int jj, int ii, int l) {
    const int buf = p & 1, j = g.j0 + jj;
    if (ii == SR) {
        acc = mma16(acc, S.Gj[buf][jj], S.Gj[buf][jj], true, l);
        return;
    }
    const int i = g.i0 + ii;
    if (i == p) {  // row p just pivoted: the kept tile becomes A_pj = L_p G_j^T
        const d4 z = {0.0, 0.0, 0.0, 0.0};
        acc = mma16(z, S.Ls[buf], S.Gj[buf][jj], false, l);
        return;
    }
    if (i > p && i < j) return;  // mirror of (j, i): not kept
    acc = mma16(acc, S.Gm[buf][ii], S.Gj[buf][jj], true, l);
}

__device__ __forceinline__ void updater(const Args &a, const Geo &g, Smem &S, int u, int lane, d4 (&acc)[TPW], bool track_ob) {
    for (int p = 0; p < g.j1; ++p) {
        const int buf = p & 1;
        if (!lds_wait(&S.gm_ok[buf], p + 1, S)) return;
        if (u == 0) stamp(a, p, DBG_GM);
        // L_p and y_p (W1 or the loader): only the import of row p and the segment's b need them
        bool ly = false, ok = true;
        auto need_ly = [&]() {
            if (!ly) {
                ok = lds_wait(&S.ly_ok[buf], p + 1, S);
                ly = true;
            }
            return ok;
        };
        // phase A: the tiles of column p + 1, staged for its pivot
        const int ja = p + 1 - g.j0;
        if (ja >= 0 && ja < g.ncol) {
#pragma unroll
            for (int k = 0; k < TPW; ++k) {
                int jj, ii;
                if (!ok || !g.slot(u, k, jj, ii) || jj != ja) continue;
                // Cst still holds column p for chain(p) (both chain waves read it)
                if (!lds_wait(&S.gj_ok[buf][jj], p + 1, S)) {
                    ok = false;
                    continue;
                }
                stamp(a, p, DBG_AGJ);
                if (p >= g.j0 && !lds_wait(&S.cst_read, 2 * (p - g.j0 + 1), S)) {
                    ok = false;
                    continue;
                }
                if (ii < SR && g.i0 + ii == p && !need_ly()) continue;
                stamp(a, p, DBG_ACST);
                apply_tile(acc[k], g, S, p, jj, ii, lane);
                store_cst(S, ii, acc[k], lane);
                stamp(a, p, DBG_AMMA);
                lds_release();
                if (lane == 0) lds_add(&S.cst_cnt, 1);
            }
        }
        if (u == 0) stamp(a, p, DBG_PHA);
        // phase B: every other owned column j > p + 1
#pragma unroll
        for (int k = 0; k < TPW; ++k) {
            int jj, ii;
            if (!ok || !g.slot(u, k, jj, ii) || g.j0 + jj <= p + 1) continue;
            if (!lds_wait(&S.gj_ok[buf][jj], p + 1, S)) {
                ok = false;
                continue;
            }
            if (ii < SR && g.i0 + ii == p && !need_ly()) continue;
            apply_tile(acc[k], g, S, p, jj, ii, lane);
            if (ii == SR && (!need_ly() || !apply_bb(S, p, jj, lane))) ok = false;
        }
        if (track_ob && u == 0 && ok && need_ly()) {  // b of the segment's rows: ob_i -= G_i y_p, i != p
            const int ti = lane >> 4;
            if (ti < g.nrow && g.i0 + ti != p) {
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < 16; ++k) s = fma(S.Gm[buf][ti][lane & 15][k], S.ys[buf][k], s);
                S.ob[lane] -= s;
            }
        }
        if (!ok) return;
        lds_release();
        if (lane == 0) lds_add(&S.udone[p], 1);
        if (u == 0) stamp(a, p, DBG_PHB);
    }
}

// trial cameras and the camera part of the model decrease from dc (LDS),
// as camera_trial (k_chol_backsolve's epilogue) with the system read from
// its source; red: 3 x NTH / 64 doubles
// (scalar arguments: a reference to the kernel's Args would put a copy of it
// on the stack of every lane)
template <int NTH>
__device__ __attribute__((noinline)) void cam_trial(int nc, const double *Rt, double *Rt_new, double *cam_out,
                                                    double lambda, const double *payload, int32_t ns,
                                                    const double *dc, double *red, const double *camlin = nullptr) {
    // diag U and g_c: the payload's vectors, or (finish folded into the solve) the camera blocks themselves
    const double *du = payload + pay_vec_base(ns), *gc = du + ns;
    double m = 0, dn = 0, xn = 0;
    constexpr int NWT = NTH / 64;
    for (int c = threadIdx.x; c < nc; c += NTH) {
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
            const double u = camlin ? cam_u(camlin, c, i, i) : du[6 * c + i];
            const double g = camlin ? camlin[CAMLIN * c + 21 + i] : gc[6 * c + i];
            m += d[i] * (lambda * clampd(u) * d[i] - g);
            dn += d[i] * d[i];
        }
    }
    // fixed order: a butterfly inside each wave, then the NW wave sums in
    // wave order (a serial sum over all THREADS values was a ~THREADS-long
    // dependent chain of LDS loads and adds on the solve's tail)
    double v[3] = {m, dn, xn};
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int k = 0; k < 3; ++k) red[k * NWT + w] = v[k];
    __syncthreads();
    if (threadIdx.x < 3) {
        double s = 0.0;
#pragma unroll
        for (int t = 0; t < NWT; ++t) s += red[threadIdx.x * NWT + t];
        cam_out[threadIdx.x] = s;
    }
}

// x_i = L_i^-T L_i^-1 b_i for the segment's row tiles (W0; a 16-lane row a
// tile, lane li holding row li and column li of L_i): both substitutions as
// 16 steps of a DPP broadcast within the row (row_newbcast), a multiply by
// the pivot's reciprocal (computed up front, off the chain) and an fma
template <int K>
__device__ __forceinline__ double bcast16(double v) {
    double r;
    asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v), "n"(K));
    return r;
}
template <int K>
__device__ __forceinline__ void fwd_step(double &v, const double (&L)[16], const double (&inv)[16], int li) {
    const double yk = bcast16<K>(v) * inv[K];
    v = li == K ? yk : li > K ? fma(-L[K], yk, v) : v;
}
template <int K>
__device__ __forceinline__ void bwd_step(double &v, const double (&Lc)[16], const double (&inv)[16], int li) {
    const double xk = bcast16<K>(v) * inv[K];
    v = li == K ? xk : li < K ? fma(-Lc[K], xk, v) : v;
}
template <int... K>
__device__ __forceinline__ void tri_solve16(double &v, const double (&L)[16], const double (&Lc)[16],
                                            const double (&inv)[16], int li, std::integer_sequence<int, K...>) {
    (fwd_step<K>(v, L, inv, li), ...);
    (bwd_step<15 - K>(v, Lc, inv, li), ...);
}
template <int... K>
__device__ __forceinline__ void bcast_all16(double d, double (&inv)[16], std::integer_sequence<int, K...>) {
    ((inv[K] = bcast16<K>(d)), ...);
}
__device__ __forceinline__ void final_solve(const double *Lp, double *x, int nseg, int s, int i0, int nrow,
                                            double v, int lane) {
    const int li = lane & 15, ti = lane >> 4;
    const bool act = ti < nrow;
    const int i = i0 + (act ? ti : 0);
    double L[16], Lc[16], inv[16];  // row li and column li of L_i
    const double *ls = Lp + ((int64_t)i * nseg + s) * 256;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        L[j] = ld_ag(ls + li * 16 + j);
        Lc[j] = ld_ag(ls + j * 16 + li);
    }
    double d = 0.0;
#pragma unroll
    for (int j = 0; j < 16; ++j) d = j == li ? L[j] : d;
    d = act ? 1.0 / d : 1.0;
    bcast_all16(d, inv, std::make_integer_sequence<int, 16>{});
    tri_solve16(v, L, Lc, inv, li, std::make_integer_sequence<int, 16>{});
    if (act) st_ag(x + i * TL + li, v);
}

__global__ void __launch_bounds__(THREADS) k_gj_solve(Args a) {
    if (a.gate && !*a.gate) return;  // device-side LM control: iteration gated off
    __shared__ Smem S;
    stamp(a, a.nT, DBG_START);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    Geo g;
    g.nT = a.nT;
    g.nseg = a.nseg;
    g.cb = blockIdx.x / a.nseg;
    g.s = blockIdx.x % a.nseg;
    g.j0 = g.cb * a.cb;
    g.j1 = min(a.nT, g.j0 + a.cb);
    g.ncol = g.j1 - g.j0;
    g.i0 = g.s * SR;
    g.i1 = min(a.nT, g.i0 + SR);
    g.nrow = g.i1 - g.i0;
    g.wpg = NUW / (a.cb / SR);
    const bool last_block = g.j1 == a.nT;
    const double lambda = *a.lam;
    // ---- prologue
    if (threadIdx.x < 2) S.gm_ok[threadIdx.x] = S.ly_ok[threadIdx.x] = 0;
    if (threadIdx.x < 2 * CBMAX) S.gj_ok[threadIdx.x / CBMAX][threadIdx.x % CBMAX] = 0;
    if (threadIdx.x < CBMAX) S.bb_cnt[threadIdx.x] = 0;
    if (threadIdx.x < NTMAX) S.udone[threadIdx.x] = 0;
    if (threadIdx.x == 0) {
        S.cst_cnt = S.cst_read = S.abort_ = 0;
        S.err = a.err;
        S.bad = a.bad;
    }
    d4 acc[TPW];
#pragma unroll
    for (int k = 0; k < TPW; ++k) acc[k] = d4{0.0, 0.0, 0.0, 0.0};
    const int u = wave - 4;
    // initial tiles, SR owned columns per pass: every thread gathers up to 8
    // elements from the payload in one round into LDS, then each update wave
    // takes its fragments (column j0's are staged for pivot j0 if j0 == 0)
    double *stage = &S.Gm[0][0][0][0];
    static_assert(offsetof(Smem, Gj) == sizeof(S.Gm) &&
                      sizeof(S.Gm) + sizeof(S.Gj) >= (SR + 1) * SR * TL * LDT * sizeof(double), "staging");
    constexpr int EPT = ((SR + 1) * SR * 256 + THREADS - 1) / THREADS;
    for (int c0 = 0; c0 < g.ncol; c0 += SR) {
        const int nc = min(SR, g.ncol - c0), nel = nc * (SR + 1) * 256;
        ElemRef er[EPT];
        double v[EPT], dg[EPT];
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const int idx = threadIdx.x + k * THREADS, q = idx >> 8, e = idx & 255;
            const int jl = q / (SR + 1), ii = q % (SR + 1);
            const bool ok = idx < nel && (ii == SR || ii < g.nrow);
            const int ti = ii == SR ? g.j0 + c0 + jl : g.i0 + ii, tj = g.j0 + c0 + jl;
            er[k] = ok ? elem_ref(a.ns, ti * TL + (e >> 4), tj * TL + (e & 15)) : ElemRef{-1, -1, 0.0};
        }
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            v[k] = er[k].idx >= 0 ? a.payload[er[k].idx] : er[k].pad;
            dg[k] = er[k].dg >= 0 ? a.payload[er[k].dg] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const int idx = threadIdx.x + k * THREADS, q = idx >> 8, e = idx & 255;
            if (er[k].dg >= 0) v[k] += lambda * clampd(dg[k]);
            if (idx < nel) stage[(q * TL + (e >> 4)) * LDT + (e & 15)] = v[k];
        }
        __syncthreads();
        if (u >= 0) {
#pragma unroll
            for (int k = 0; k < TPW; ++k) {
                int jj, ii;
                if (!g.slot(u, k, jj, ii) || jj < c0 || jj >= c0 + nc) continue;
                const double *tq = stage + ((jj - c0) * (SR + 1) + ii) * TL * LDT;
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[k][e] = tq[((lane >> 4) + 4 * e) * LDT + (lane & 15)];
                if (jj == 0 && g.j0 == 0) store_cst(S, ii, acc[k], lane);  // pivot 0 needs no panel
            }
        }
        __syncthreads();
    }
    if (wave == 1) {  // b replicas of the owned columns
        for (int e = lane; e < g.ncol * TL; e += 64) S.bb[e / TL][e % TL] = assembled_b(a.payload, a.ns, g.j0 * TL + e);
    } else if (wave == 2 && last_block) {  // b of the segment's rows
        S.ob[lane] = lane / TL < g.nrow ? assembled_b(a.payload, a.ns, g.i0 * TL + lane) : 0.0;
    }
    if (threadIdx.x == 0) S.cst_cnt = g.j0 == 0 ? g.nrow + 1 : 0;  // else staged by panel j0 - 1
    __syncthreads();
    // ---- the pivot loop, by role
    stamp(a, a.nT, DBG_PROLOGUE);
    if (wave == 0) {
        for (int p = g.j0; p < g.j1; ++p) {
            if (!lds_wait(&S.cst_cnt, (p - g.j0 + 1) * (g.nrow + 1), S) || !chain_pivot(a, g, S, p, 0, lane)) break;
            if (lds_ld(&S.abort_)) break;
        }
    } else if (wave == 1) {
        w1_loop(a, g, S, lane);
    } else if (wave == 2) {
        loader(a, g, S, lane);
    } else if (wave == 3) {
        publisher(a, g, S, lane);
    } else {
        updater(a, g, S, u, lane, acc, last_block);
    }
    // ---- the solution (last column block) and the epilogue (last arrival)
    if (!last_block) return;
    __shared__ int last_arrival;
    if (wave == 0) {
        bool ok = lds_wait(&S.udone[a.nT - 1], NCONS, S);  // every wave is done with every panel
        stamp(a, a.nT, DBG_FINWAIT);
        if (ok) final_solve(a.Lp, a.x, g.nseg, g.s, g.i0, g.nrow, S.ob[lane], lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        stamp(a, a.nT, DBG_FINSOLVED);
        if (lane == 0) {
            last_arrival = 0;
            if (ok) {
                const unsigned old = __hip_atomic_fetch_add(a.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (old == (unsigned)a.nseg - 1) {
                    last_arrival = 1;
                    __hip_atomic_store(a.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
    }
    __syncthreads();
    stamp(a, a.nT, DBG_ARRIVED);
    if (!last_arrival || a.ct.nc <= 0) return;
    double *dc = &S.Gm[0][0][0][0];  // LDS reused: x, then the reductions
    double *red = &S.Gj[0][0][0][0];
    static_assert(sizeof(S.Gj) >= 3 * THREADS * sizeof(double), "reduction scratch");
    static_assert(sizeof(S.Gm) >= 6 * (NTMAX * TL / 6) * sizeof(double), "trial step");
    for (int i = threadIdx.x; i < 6 * a.ct.nc; i += THREADS) dc[i] = ld_ag(a.x + i);
    __syncthreads();
    cam_trial<THREADS>(a.ct.nc, a.ct.Rt, a.ct.Rt_new, a.ct.cam_out, *a.lam, a.payload, a.ns, dc, red);
    stamp(a, a.nT, DBG_EPILOGUE);
}

}  // namespace gj
