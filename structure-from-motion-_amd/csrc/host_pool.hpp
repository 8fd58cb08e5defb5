// Host worker threads shared by the library's host-side passes (BA create,
// the dense observation scan): parked on a condition variable between jobs.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <exception>
#include <new>
#include <sched.h>
#include <stdexcept>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "sfm_common.hpp"

namespace sfm {

// Host threads kept across calls (round 5): create fans out ~15 times (the
// validation, the CSR, the counts, the planner's passes), and spawning and
// joining 16 threads cost ~0.3-0.5 ms each time.  Workers park on a
// condition variable; one job at a time -- a concurrent caller (in-process
// ranks creating their problems together) spawns its own threads instead.
class HostPool {
  public:
    static HostPool &get() {
        static HostPool *p = new HostPool();  // never destroyed: workers may outlive static teardown
        return *p;
    }
    // f(t) for t in [0, nt), the caller taking t = nt - 1; false if busy.
    // An exception from any f(t) (the caller's or a worker's) is held until
    // every worker has finished with f, then rethrown on the caller: no
    // worker ever runs a job whose frame has unwound.
    template <class F>
    bool try_run(int nt, F &&f) {
        std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
        if (!busy.owns_lock()) return false;
        const int nw = nt - 1;
        {
            std::lock_guard<std::mutex> lk(mu_);
            while ((int)workers_.size() < nw) {
                const int id = (int)workers_.size();
                workers_.emplace_back([this, id] { loop(id); });
                workers_.back().detach();
            }
            job_ = [&f](int t) { f(t); };
            njob_ = nw;
            remaining_ = nw;
            eptr_ = nullptr;
            ++gen_;
        }
        cv_.notify_all();
        std::exception_ptr mine;
        try {
            f(nt - 1);
        } catch (...) {
            mine = std::current_exception();
        }
        std::exception_ptr theirs;
        {
            std::unique_lock<std::mutex> lk(mu_);
            done_cv_.wait(lk, [this] { return remaining_ == 0; });
            job_ = nullptr;
            theirs = eptr_;
            eptr_ = nullptr;
        }
        if (mine) std::rethrow_exception(mine);
        if (theirs) std::rethrow_exception(theirs);
        return true;
    }

  private:
    void loop(int id) {
        uint64_t seen = 0;
        for (;;) {
            std::function<void(int)> job;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (id >= njob_) continue;
                job = job_;
            }
            std::exception_ptr e;
            try {
                job(id);
            } catch (...) {
                e = std::current_exception();
            }
            std::lock_guard<std::mutex> lk(mu_);
            if (e && !eptr_) eptr_ = e;
            if (--remaining_ == 0) done_cv_.notify_all();
        }
    }
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    std::vector<std::thread> workers_;
    std::function<void(int)> job_;
    std::exception_ptr eptr_;  // the first worker exception of the current job
    uint64_t gen_ = 0;
    int njob_ = 0, remaining_ = 0;
};

// threads for the host passes: SFM_PLAN_THREADS, else the CPUs this process
// may run on (its affinity mask, not the machine's count: under taskset or a
// cpuset more threads than CPUs would only time-slice), at most 16
inline int host_threads() {
    static const int n = [] {
        const char *s = std::getenv("SFM_PLAN_THREADS");
        const int e = s ? std::atoi(s) : 0;
        if (e > 0) return e;
        cpu_set_t cs;
        const int c = sched_getaffinity(0, sizeof cs, &cs) == 0 ? CPU_COUNT(&cs)
                                                               : (int)std::thread::hardware_concurrency();
        return std::min(16, std::max(1, c));
    }();
    return n;
}

// the planner's independent loops (per chunk, per spec) on host threads:
// f(i) for i in [0, n), contiguous blocks, up to 16 threads (SFM_PLAN_THREADS)
template <class F>
inline void par_for(int64_t n, F &&f) {
    static const int nt0 = host_threads();
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt0, n));
    if (nt == 1) {
        for (int64_t i = 0; i < n; ++i) f(i);
        return;
    }
    auto block = [&](int t) {
        for (int64_t i = n * t / nt; i < n * (t + 1) / nt; ++i) f(i);
    };
    if (HostPool::get().try_run(nt, block)) return;
    // the pool is busy: threads of our own, with the same exception contract
    std::vector<std::exception_ptr> ex(nt);
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            try {
                block(t);
            } catch (...) {
                ex[t] = std::current_exception();
            }
        });
    for (auto &x : th) x.join();
    for (auto &e : ex)
        if (e) std::rethrow_exception(e);
}

// f(i) for i in [0, n), the items dealt dynamically: each thread takes the
// next item from a shared counter.  For memory-bound passes over many items
// (the dense scan's row blocks): on a shared host a thread whose core is busy
// with another tenant's work takes fewer items instead of setting the time
// of the whole pass, as a contiguous block per thread would.
template <class F>
inline void par_for_dynamic(int64_t n, F &&f) {
    std::atomic<int64_t> next{0};
    static const int nt0 = host_threads();
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt0, n));
    par_for(nt, [&](int64_t) {
        for (int64_t i; (i = next.fetch_add(1, std::memory_order_relaxed)) < n;) f(i);
    });
}

// The C-ABI never lets a C++ exception out: a host allocation that fails
// inside an entry point (a vector of a create, a dense scan's pieces) comes
// back as SFM_ERR_NOMEM with the reason in sfm_last_error.
template <class F>
inline int abi_guard(const char *what, F &&f) {
    try {
        return f();
    } catch (const std::bad_alloc &) {
        set_error("%s: host memory allocation failed", what);
        return SFM_ERR_NOMEM;
    } catch (const std::exception &e) {
        set_error("%s: %s", what, e.what());
        return SFM_ERR_ARG;
    } catch (...) {
        set_error("%s: unknown C++ exception", what);
        return SFM_ERR_ARG;
    }
}

}  // namespace sfm
