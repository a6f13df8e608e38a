// host_pool.h -- the engine's persistent pool of host threads (LO trial
// draws and fits, graph-cut cell jobs, the refit's per-inlier angles, the
// problem setup's fills).  Header-only and free of HIP, so the CPU suite
// builds it under ThreadSanitizer and AddressSanitizer
// (tests/cpp/host_pool.cpp, tests/test_sanitizers.py).
//
// One job at a time: fn(i) for i in [0, n), handed out through an atomic
// counter to the workers and the calling thread.  Results land at their
// index, so the outcome never depends on the scheduling.  A caller that
// finds the pool busy (another gcr_solve_batch thread, or a job nested in a
// job) runs its job itself instead of queueing behind the other one.
//
// Round-5 history: begin() / end() first kept the call
// lock in a shared std::unique_lock member.  A second caller whose try-lock
// failed move-assigned its empty lock into that member, which unlocked the
// FIRST caller's mutex from the wrong thread; a third caller then started a
// job while the first still ran -- job_, n_ and pending_ overwritten, workers
// running one caller's fn with the other's n (pending_ underflowed to -4 in
// tools/stress_batch.py).  The lock is now a plain try_lock / unlock pair,
// and a thread that already owns the call (a caller between begin() and
// end(), or a worker inside a job) never try-locks the mutex again.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace gcr {

class HostPool {
public:
    using Clock = std::chrono::steady_clock;

    // n threads in all (n - 1 workers plus the caller).  `crowded`, when
    // given, counts host threads solving problems at once: while it is above
    // one the workers block instead of spinning between jobs.
    explicit HostPool(unsigned n, const std::atomic<int>* crowded = nullptr) : crowded_(crowded) {
        for (unsigned t = 1; t < n; ++t) workers_.emplace_back([this] { loop(); });
    }
    HostPool(const HostPool&) = delete;
    HostPool& operator=(const HostPool&) = delete;
    size_t threads() const { return workers_.size() + 1; }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_.store(true, std::memory_order_relaxed);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        for (auto& w : workers_) w.join();
    }

    // fn(i) for i in [0, n); the calling thread works too.  Exceptions: the
    // first one thrown by any fn(i) is rethrown here (later items are not
    // started once one has thrown).
    void parallel_for(size_t n, const std::function<void(size_t)>& fn) {
        if (n == 0) return;
        if (workers_.empty() || n == 1 || t_owner_ == this || !call_mu_.try_lock()) {
            for (size_t i = 0; i < n; ++i) fn(i);
            return;
        }
        start(n, fn);
        finish();
    }

    // fn(i) for i in [0, n) started on the workers; the caller goes on (e.g.
    // launches GPU work) and then calls end(), which helps with what is left
    // and waits.  false (nothing started) when the pool has no workers or is
    // busy: the caller then uses parallel_for.  fn must outlive end().
    bool begin(size_t n, const std::function<void(size_t)>& fn) {
        if (workers_.empty() || n == 0 || t_owner_ == this) return false;
        if (!call_mu_.try_lock()) return false;
        start(n, fn);
        return true;
    }
    void end() { finish(); }

    // diagnostics for the tests: jobs started on the workers so far
    uint64_t jobs() const { return gen_.load(std::memory_order_relaxed); }

private:
    // under call_mu_: publish the job (the gen_ release orders job_, n_,
    // next_ and pending_ before any worker's acquire of the new generation)
    void start(size_t n, const std::function<void(size_t)>& fn) {
        t_owner_ = this;
        job_ = &fn;
        n_ = n;
        next_.store(0, std::memory_order_relaxed);
        pending_.store(workers_.size(), std::memory_order_relaxed);
        {
            // published under the lock so a worker about to block cannot miss it
            std::lock_guard<std::mutex> lk(mu_);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
    }
    // the caller's share, then wait for every worker to have left the job:
    // after this no worker touches fn or anything it captured
    void finish() {
        run();
        const auto t0 = Clock::now();
        bool told = false;
        // the workers are awake (spinning or just woken) and the jobs are
        // short: wait for the stragglers by polling
        for (unsigned spin = 0; pending_.load(std::memory_order_acquire) != 0; ++spin) {
            if (spin > 4096) std::this_thread::yield();
            if (!told && (spin & 65535) == 0 && spin &&
                std::chrono::duration<double>(Clock::now() - t0).count() > 5.0) {
                fprintf(stderr, "gcr: host pool: %zu workers still in a job after 5 s\n",
                        (size_t)pending_.load(std::memory_order_acquire));
                told = true;
            }
        }
        job_ = nullptr;
        std::exception_ptr e;
        {
            std::lock_guard<std::mutex> lk(err_mu_);
            std::swap(e, err_);
        }
        t_owner_ = nullptr;
        call_mu_.unlock();
        if (e) std::rethrow_exception(e);         // the first failure, on the caller
    }
    void run() {
        try {
            for (size_t i; (i = next_.fetch_add(1, std::memory_order_relaxed)) < n_;) (*job_)(i);
        } catch (...) {
            std::lock_guard<std::mutex> lk(err_mu_);
            if (!err_) err_ = std::current_exception();
            next_.store(n_, std::memory_order_relaxed);       // stop handing out work
        }
    }
    // A worker polls for the next job for ~spin_us() after finishing one (the
    // LO rounds call the pool every ~100 us: a condition-variable wake-up of
    // 15 threads costs tens of us per call), then blocks.  GCR_POOL_SPIN_US
    // sets the window (default 300, 0 = always block); while more than one
    // thread of gcr_solve_batch is solving, workers block at once (their
    // spinning would take cores from those threads).
    int64_t spin_us() const {
        static const int64_t us = [] {
            const char* e = getenv("GCR_POOL_SPIN_US");
            return e ? std::max<int64_t>(0, atoll(e)) : (int64_t)300;
        }();
        return crowded_ && crowded_->load(std::memory_order_relaxed) > 1 ? 0 : us;
    }
    void loop() {
        t_owner_ = this;                          // a job's nested pool calls run inline
        uint64_t seen = 0;
        for (;;) {
            uint64_t g = gen_.load(std::memory_order_acquire);
            if (g == seen) {
                const auto t0 = Clock::now();
                const int64_t window = spin_us();
                unsigned k = 0;
                while (window > 0 && (g = gen_.load(std::memory_order_acquire)) == seen) {
                    if ((++k & 255) == 0 &&
                        std::chrono::duration_cast<std::chrono::microseconds>(Clock::now() - t0).count() > window)
                        break;
#if defined(__x86_64__)
                    __builtin_ia32_pause();
#endif
                }
                if (g == seen) {
                    std::unique_lock<std::mutex> lk(mu_);
                    cv_.wait(lk, [&] { return stop_.load(std::memory_order_relaxed) || gen_.load(std::memory_order_acquire) != seen; });
                    g = gen_.load(std::memory_order_acquire);
                }
            }
            if (stop_.load(std::memory_order_relaxed)) return;     // ordered by gen_'s acquire
            seen = g;
            run();
            pending_.fetch_sub(1, std::memory_order_acq_rel);
        }
    }

    static inline thread_local const HostPool* t_owner_ = nullptr;   // this thread holds a call of that pool
    const std::atomic<int>* crowded_;
    std::vector<std::thread> workers_;
    std::mutex mu_, call_mu_, err_mu_;
    std::exception_ptr err_;
    std::condition_variable cv_;
    const std::function<void(size_t)>* job_ = nullptr;
    size_t n_ = 0;
    std::atomic<size_t> next_{0};
    std::atomic<size_t> pending_{0};
    std::atomic<uint64_t> gen_{0};
    std::atomic<bool> stop_{false};
};

}  // namespace gcr
