// Shared host-side plumbing for libsfmcore: error reporting, per-thread /
// per-device stream + scratch buffers, HIP-event phase timers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/sfmcore.h"

namespace sfm {

void set_error(const char *fmt, ...);
void clear_error();
void set_timings(const double *t, int n);
// HIP events for sfm_last_timings in the drop-in RANSAC calls (off by
// default: each event record costs the stream a few microseconds)
bool call_timing();

#define SFM_HIP(call)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess) {                                                              \
            ::sfm::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
            return SFM_ERR_HIP;                                                              \
        }                                                                                    \
    } while (0)

#define SFM_CHECK_ARG(cond, msg)                   \
    do {                                           \
        if (!(cond)) {                             \
            ::sfm::set_error("argument: %s", msg); \
            return SFM_ERR_ARG;                    \
        }                                          \
    } while (0)

// Device scratch that only grows; freed at thread exit.
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    int reserve(size_t n) {
        if (n <= bytes) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        size_t want = n + n / 4 + 256;
        if (hipMalloc(&p, want) != hipSuccess) {
            set_error("hipMalloc(%zu) failed", want);
            return SFM_ERR_NOMEM;
        }
        bytes = want;
        return 0;
    }
    template <class T> T *as() const { return reinterpret_cast<T *>(p); }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

// Pinned host scratch that only grows (async uploads from it overlap host work).
struct HostBuf {
    void *p = nullptr;
    size_t bytes = 0;
    int reserve(size_t n) {
        if (n <= bytes) return 0;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
        size_t want = n + n / 4 + 256;
        if (hipHostMalloc(&p, want) != hipSuccess) {
            set_error("hipHostMalloc(%zu) failed", want);
            return SFM_ERR_NOMEM;
        }
        bytes = want;
        return 0;
    }
    template <class T> T *as() const { return reinterpret_cast<T *>(p); }
    ~HostBuf() {
        if (p) (void)hipHostFree(p);
    }
};

// One per (host thread, device): its own stream makes entry points reentrant.
struct ThreadCtx {
    int device = -1;
    hipStream_t stream = nullptr;
    hipEvent_t ev[8] = {};
    DevBuf buf[12];
    HostBuf pinned;
    void *gj_ints = nullptr;  // sfm_reduced_solve: the flag buffer its epochs refer to
    int gj_epoch = 0;
    int gj_nT = 0, gj_nseg = 0;  // ... and the layout they were carved with
    void *gjr_words = nullptr;   // ... the row-distributed solve's granule records (buf[7])
    unsigned gjr_tag = 0;
    int gjr_nT = 0;
    void *nl_sync = nullptr;     // sfm_nonlinear_pnp's cross-workgroup sums (zeroed once; epoch-tagged flags)
    unsigned nl_epoch = 0;
    int nl_resident = -1;        // sfm_nonlinear_pnp: workgroups resident at once (computed on first use)
    ~ThreadCtx() {
        if (stream) {
            (void)hipSetDevice(device);
            if (nl_sync) (void)hipFree(nl_sync);
            for (auto &e : ev)
                if (e) (void)hipEventDestroy(e);
            (void)hipStreamDestroy(stream);
        }
    }
};

// Selects `device` and returns this thread's context for it (nullptr on error).
ThreadCtx *thread_ctx(int device);

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

}  // namespace sfm
