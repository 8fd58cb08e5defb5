// CPython random replay, host side: MT19937 exactly as _randommodule.c's
// genrand_uint32, plus random.py (3.10) _randbelow_with_getrandbits and both
// branches of sample() (pool for n <= setsize, set rejection above).  The
// reference draws its RANSAC samples with random.sample(range(N), k) on the
// global instance (GetInliersRANSAC.py:55, GetHomographyInliers.py:126,
// PnPRANSAC.py:49); replaying that stream natively keeps every later draw
// identical.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#if defined(__x86_64__)
#include <immintrin.h>
#endif
#include <vector>

namespace sfm {

struct PyMT {
    uint32_t mt[624];
    uint32_t tmp[624];  // tempered outputs of the current state block
    int idx;
    // the twist, branch-free (mag01[y & 1] == -(y & 1) & 0x9908b0df) so the
    // two long loops vectorise
    void twist() {
        int kk;
        for (kk = 0; kk < 624 - 397; kk++) {
            const uint32_t y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
            mt[kk] = mt[kk + 397] ^ (y >> 1) ^ ((0u - (y & 0x1U)) & 0x9908b0dfU);
        }
        for (; kk < 623; kk++) {
            const uint32_t y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
            mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ ((0u - (y & 0x1U)) & 0x9908b0dfU);
        }
        const uint32_t y = (mt[623] & 0x80000000U) | (mt[0] & 0x7fffffffU);
        mt[623] = mt[396] ^ (y >> 1) ^ ((0u - (y & 0x1U)) & 0x9908b0dfU);
        idx = 0;
        temper_from(0);
    }
    void temper_from(int i0) {  // vectorisable tempering of the whole block
        for (int i = i0; i < 624; ++i) {
            uint32_t y = mt[i];
            y ^= (y >> 11);
            y ^= (y << 7) & 0x9d2c5680U;
            y ^= (y << 15) & 0xefc60000U;
            y ^= (y >> 18);
            tmp[i] = y;
        }
    }
    uint32_t next() {
        if (idx >= 624) twist();
        return tmp[idx++];
    }
    uint32_t getrandbits(int k) { return k == 0 ? 0u : next() >> (32 - k); }
    int64_t randbelow(int64_t n) {
        if (n == 0) return 0;
        const int k = 64 - __builtin_clzll((unsigned long long)n);  // n.bit_length()
        if (k > 32) return -1;  // not needed for N < 2^31
        uint32_t r = getrandbits(k);
        while ((int64_t)r >= n) r = getrandbits(k);
        return r;
    }
};

// random.sample(range(n), k) for hypotheses [h0, h1) into out[h * k ...]
struct PySampler {
    PyMT m;
    int64_t n;
    int32_t k;
    int64_t setsize;
    std::vector<int32_t> pool;
    PySampler(const uint32_t *st, int64_t n_, int32_t k_) : n(n_), k(k_) {
        for (int i = 0; i < 624; ++i) m.mt[i] = st[i];
        m.idx = (int)st[624];
        if (m.idx < 624) m.temper_from(m.idx);
        setsize = 21;
        if (k > 5) setsize += (int64_t)std::pow(4.0, std::ceil(std::log((double)k * 3) / std::log(4.0)));
    }
    void save(uint32_t *st) const {
        for (int i = 0; i < 624; ++i) st[i] = m.mt[i];
        st[624] = (uint32_t)m.idx;
    }
    void draw(int64_t h0, int64_t h1, int32_t *out) {
        if (n > setsize) {
#if defined(__x86_64__)
            static const bool simd = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl") &&
                                     __builtin_cpu_supports("avx512cd") && !std::getenv("SFM_PYRANDOM_SCALAR");
            if (simd) switch (k) {
                case 4: draw_set_512<4>(h0, h1, out); return;
                case 5: draw_set_512<5>(h0, h1, out); return;
                case 6: draw_set_512<6>(h0, h1, out); return;
                case 7: draw_set_512<7>(h0, h1, out); return;
                case 8: draw_set_512<8>(h0, h1, out); return;
                default: break;
                }
#endif
            switch (k) {
            case 4: draw_set<4>(h0, h1, out); return;
            case 5: draw_set<5>(h0, h1, out); return;
            case 6: draw_set<6>(h0, h1, out); return;
            case 7: draw_set<7>(h0, h1, out); return;
            case 8: draw_set<8>(h0, h1, out); return;
            default: break;
            }
        }
        for (int64_t h = h0; h < h1; ++h) {
            int32_t *res = out + h * k;
            if (n <= setsize) {
                pool.resize(n);
                for (int64_t i = 0; i < n; ++i) pool[i] = (int32_t)i;
                for (int32_t i = 0; i < k; ++i) {
                    const int64_t j = m.randbelow(n - i);
                    res[i] = pool[j];
                    pool[j] = pool[n - i - 1];
                }
            } else {  // set rejection; randbelow(n) with n.bit_length() hoisted
                const int sh = 32 - (64 - __builtin_clzll((unsigned long long)n));
                for (int32_t i = 0; i < k; ++i) {
                    uint32_t j;
                    for (;;) {
                        do { j = m.next() >> sh; } while ((int64_t)j >= n);
                        bool dup = false;
                        for (int32_t q = 0; q < i; ++q) dup |= (res[q] == (int32_t)j);
                        if (!dup) break;
                    }
                    res[i] = (int32_t)j;
                }
            }
        }
    }

    // Set-rejection branch for a compile-time k, restructured for
    // throughput without changing which outputs are consumed: each tempered
    // block is first compacted to its in-range values (randbelow's retries,
    // branch-free), then hypotheses are cut k at a time from the compacted
    // stream; a group holding a duplicate (about 28/n of them) re-walks its
    // values with sample()'s "j in selected" retry.  Stream positions ride
    // along so the state is left exactly after the last consumed output.
    template <int K> void draw_set(int64_t h0, int64_t h1, int32_t *out) {
        const int sh = 32 - (64 - __builtin_clzll((unsigned long long)n));
        const uint32_t nn = (uint32_t)n;
        int32_t *res = out + h0 * K;
        int32_t *const end = out + h1 * K;
        if (res >= end) return;
        int64_t base = -(int64_t)m.idx;  // stream position of tmp[0]; 0 = first output of this call
        int i0 = m.idx;
        int c = 0, p = 0;
        for (;;) {
            if (i0 >= 624) {
                m.twist();
                base += 624;
                i0 = 0;
            }
            if (p > 0) {  // carry the unfinished group to the front
                for (int q = p; q < c; ++q) {
                    vals[q - p] = vals[q];
                    at[q - p] = at[q];
                }
                c -= p;
                p = 0;
            }
            if ((int)vals.size() < c + 624) {
                vals.resize(c + 624);
                at.resize(c + 624);
            }
            uint32_t *v = vals.data();
            int64_t *a = at.data();
            for (int i = i0; i < 624; ++i) {
                const uint32_t u = m.tmp[i] >> sh;
                v[c] = u;
                a[c] = base + i;
                c += u < nn;
            }
            i0 = 624;
            while (res < end && c - p >= K) {
                const uint32_t *g = v + p;
                int dup = 0;
#pragma unroll
                for (int x = 1; x < K; ++x)
#pragma unroll
                    for (int y = 0; y < x; ++y) dup |= g[x] == g[y];
                if (!dup) {
#pragma unroll
                    for (int x = 0; x < K; ++x) res[x] = (int32_t)g[x];
                    res += K;
                    p += K;
                    continue;
                }
                int na = 0, q = p;
                for (; q < c && na < K; ++q) {
                    bool seen = false;
                    for (int y = 0; y < na; ++y) seen |= (uint32_t)res[y] == v[q];
                    if (!seen) res[na++] = (int32_t)v[q];
                }
                if (na < K) break;  // needs outputs of the next block
                res += K;
                p = q;
            }
            if (res >= end) {
                m.idx = (int)(a[p - 1] + 1 - base);
                return;
            }
        }
    }
#if defined(__x86_64__)
    // The same stream walk with AVX-512: the twist and tempering vectorise
    // under this target, each block is compacted 16 outputs at a time with
    // vpcompressd, and a group's duplicate test is one vpconflictd.  Chosen at
    // run time (draw) when the CPU has AVX-512 F/VL/CD; bit-identical output.
    template <int K> __attribute__((target("avx512f,avx512vl,avx512cd"))) void draw_set_512(int64_t h0, int64_t h1,
                                                                                         int32_t *out) {
        static_assert(K <= 8, "one 8-lane conflict test per group");
        const int sh = 32 - (64 - __builtin_clzll((unsigned long long)n));
        const __m512i vnn = _mm512_set1_epi32((int)(uint32_t)n);
        const __m512i iota = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
        const __m128i vsh = _mm_cvtsi32_si128(sh);
        static const bool cstore = std::getenv("SFM_PYRANDOM_CSTORE") && std::atoi(std::getenv("SFM_PYRANDOM_CSTORE"));
        int32_t *res = out + h0 * K;
        int32_t *const end = out + h1 * K;
        if (res >= end) return;
        int i0 = m.idx;
        int c = 0, p = 0;
        for (;;) {
            if (i0 >= 624) {
                m.twist();
                i0 = 0;
            }
            if (p > 0) {  // carry the unfinished group to the front
                std::memmove(vals.data(), vals.data() + p, (size_t)(c - p) * sizeof(uint32_t));
                std::memmove(pos.data(), pos.data() + p, (size_t)(c - p) * sizeof(int32_t));
                c -= p;
                p = 0;
            }
            if ((int)vals.size() < c + 624 + 16) {
                vals.resize(c + 624 + 16);
                pos.resize(c + 624 + 16);
            }
            uint32_t *v = vals.data();
            int32_t *a = pos.data();  // index within the current block
            // compress into a register, then one full 64-byte store (the
            // buffers carry 16 words of slack): the memory form of
            // vpcompressd is microcoded on AMD Zen cores (SFM_PYRANDOM_CSTORE=1
            // keeps it, for comparison)
            if (cstore)
                for (int i = i0; i < 624; i += 16) {
                    const __mmask16 lm = 624 - i >= 16 ? (__mmask16)0xFFFF : (__mmask16)((1u << (624 - i)) - 1);
                    const __m512i u = _mm512_srl_epi32(_mm512_maskz_loadu_epi32(lm, m.tmp + i), vsh);
                    const __mmask16 kin = _mm512_mask_cmplt_epu32_mask(lm, u, vnn);
                    _mm512_mask_compressstoreu_epi32(v + c, kin, u);
                    _mm512_mask_compressstoreu_epi32(a + c, kin, _mm512_add_epi32(_mm512_set1_epi32(i), iota));
                    c += _mm_popcnt_u32((unsigned)kin);
                }
            else
                for (int i = i0; i < 624; i += 16) {
                    const __mmask16 lm = 624 - i >= 16 ? (__mmask16)0xFFFF : (__mmask16)((1u << (624 - i)) - 1);
                    const __m512i u = _mm512_srl_epi32(_mm512_maskz_loadu_epi32(lm, m.tmp + i), vsh);
                    const __mmask16 kin = _mm512_mask_cmplt_epu32_mask(lm, u, vnn);
                    _mm512_storeu_si512(v + c, _mm512_maskz_compress_epi32(kin, u));
                    _mm512_storeu_si512(a + c, _mm512_maskz_compress_epi32(kin, _mm512_add_epi32(_mm512_set1_epi32(i), iota)));
                    c += _mm_popcnt_u32((unsigned)kin);
                }
            i0 = 624;
            while (res < end && c - p >= K) {
                const uint32_t *g = v + p;
                const __m256i gv = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(g));
                const __m256i cf = _mm256_conflict_epi32(gv);
                if (_mm256_mask_test_epi32_mask((__mmask8)((1u << K) - 1), cf, cf) == 0) {
#pragma unroll
                    for (int x = 0; x < K; ++x) res[x] = (int32_t)g[x];
                    res += K;
                    p += K;
                    continue;
                }
                int na = 0, q = p;
                for (; q < c && na < K; ++q) {
                    bool seen = false;
                    for (int y = 0; y < na; ++y) seen |= (uint32_t)res[y] == v[q];
                    if (!seen) res[na++] = (int32_t)v[q];
                }
                if (na < K) break;  // needs outputs of the next block
                res += K;
                p = q;
            }
            if (res >= end) {  // the last consumed output is in this block (see draw_set)
                m.idx = a[p - 1] + 1;
                return;
            }
        }
    }
#endif
    std::vector<uint32_t> vals;
    std::vector<int64_t> at;
    std::vector<int32_t> pos;
};

}  // namespace sfm
