// The round-5 host pool's begin()/end() as they were before the fix
// (test infrastructure: a regression canary for tests/test_sanitizers.py,
// never built into the engine).  Reconstructed from the fix's description
// in commit 73ef833 and csrc/host_pool.h: the call lock lived in a shared
// std::unique_lock member.  A caller whose try-lock failed move-assigned its
// empty lock into that member -- and a unique_lock's move assignment first
// unlocks the mutex the member owns, i.e. the FIRST caller's, from the wrong
// thread.  A third caller then started a job while the first one still ran.
// parallel_for and the workers are the current pool's.
#pragma once

#include <atomic>
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace prefix {

class HostPool {
public:
    explicit HostPool(unsigned n) {
        for (unsigned t = 1; t < n; ++t) workers_.emplace_back([this] { loop(); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_.store(true);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        for (auto& w : workers_) w.join();
    }
    void parallel_for(size_t n, const std::function<void(size_t)>& fn) {
        if (n == 0) return;
        if (workers_.empty() || n == 1) {
            for (size_t i = 0; i < n; ++i) fn(i);
            return;
        }
        std::unique_lock<std::mutex> call(call_mu_, std::try_to_lock);
        if (!call.owns_lock()) {
            for (size_t i = 0; i < n; ++i) fn(i);
            return;
        }
        start(n, fn);
        wait();
    }
    bool begin(size_t n, const std::function<void(size_t)>& fn) {
        if (workers_.empty() || n == 0) return false;
        call_ = std::unique_lock<std::mutex>(call_mu_, std::try_to_lock);      // the bug
        if (!call_.owns_lock()) return false;
        start(n, fn);
        return true;
    }
    void end() {
        wait();
        call_.unlock();
    }

private:
    void start(size_t n, const std::function<void(size_t)>& fn) {
        job_ = &fn;
        n_ = n;
        next_.store(0, std::memory_order_relaxed);
        pending_.store(workers_.size(), std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> lk(mu_);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
    }
    void wait() {
        run();
        for (unsigned spin = 0; pending_.load(std::memory_order_acquire) != 0; ++spin)
            if (spin > 4096) std::this_thread::yield();
        job_ = nullptr;
        if (err_) {
            std::exception_ptr e = err_;
            err_ = nullptr;
            std::rethrow_exception(e);
        }
    }
    void run() {
        try {
            for (size_t i; (i = next_.fetch_add(1)) < n_;) (*job_)(i);
        } catch (...) {
            std::lock_guard<std::mutex> lk(err_mu_);
            if (!err_) err_ = std::current_exception();
            next_.store(n_);
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            uint64_t g = gen_.load(std::memory_order_acquire);
            if (g == seen) {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_.load() || gen_.load(std::memory_order_acquire) != seen; });
                g = gen_.load(std::memory_order_acquire);
            }
            if (stop_.load()) return;
            seen = g;
            run();
            pending_.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
    std::vector<std::thread> workers_;
    std::mutex mu_, call_mu_, err_mu_;
    std::unique_lock<std::mutex> call_;
    std::exception_ptr err_;
    std::condition_variable cv_;
    const std::function<void(size_t)>* job_ = nullptr;
    size_t n_ = 0;
    std::atomic<size_t> next_{0};
    std::atomic<size_t> pending_{0};
    std::atomic<uint64_t> gen_{0};
    std::atomic<bool> stop_{false};
};

}  // namespace prefix
