// Concurrency hammer for the engine's host pool (csrc/host_pool.h), built by
// tests/test_sanitizers.py under ThreadSanitizer and, separately, under
// AddressSanitizer + UBSan.
//
// Several caller threads (the gcr_solve_batch shape: solver threads sharing
// one pool) issue short jobs at random through every entry point:
//   * parallel_for, writing one slot per index of a heap buffer;
//   * begin() ... end() with the caller doing its own nested pool call in
//     between (the LO pipeline shape), the buffer freed right after end() --
//     a worker still inside the job afterwards is a heap use-after-free
//     (ASan) or a race (TSan);
//   * jobs whose items call the pool again (nested calls run inline);
//   * jobs that throw (the first exception reaches the caller; the pool
//     stays usable).
// Every call checks that each index ran exactly once.  Exit 0 and "OK" when
// everything held.
//
// -DGCR_PREFIX_POOL builds the same hammer against the round-5 pool as it
// was before the begin/end fix (tests/cpp/host_pool_prefix.h); the test
// expects ThreadSanitizer to report it.
#include <atomic>
#include <cstdio>
#include <random>
#include <stdexcept>
#include <thread>
#include <vector>

#ifdef GCR_PREFIX_POOL
#include "host_pool_prefix.h"
using Pool = prefix::HostPool;
#else
#include "../../graph-cut-ransac_amd/csrc/host_pool.h"
using Pool = gcr::HostPool;
#endif

namespace {

std::atomic<long> g_bad{0};

void bad(const char* what, long a, long b) {
    if (g_bad.fetch_add(1) < 20) fprintf(stderr, "FAIL %s: %ld %ld\n", what, a, b);
}

void check(const std::vector<int>& hits, const char* what) {
    for (size_t i = 0; i < hits.size(); ++i)
        if (hits[i] != 1) bad(what, (long)i, hits[i]);
}

struct Boom {
    size_t at;
};

void caller(Pool& pool, unsigned seed, int reps, std::atomic<long>& calls) {
    std::mt19937 rng(seed);
    for (int r = 0; r < reps; ++r) {
        const size_t n = rng() % 70;
        const int mode = (int)(rng() % 5);
        if (mode == 0) {
            auto* hits = new std::vector<int>(n, 0);
            pool.parallel_for(n, [&](size_t i) { (*hits)[i] += 1; });
            check(*hits, "parallel_for");
            delete hits;
        } else if (mode == 1) {
            auto* hits = new std::vector<int>(n, 0);
            std::function<void(size_t)> fn = [hits](size_t i) {
                (*hits)[i] += 1;
                if (i % 7 == 0) std::this_thread::yield();
            };
            const bool async = pool.begin(n, fn);
            // the caller's own pool call between begin and end (runs inline
            // while this thread holds the pool's call)
            std::vector<int> mine(5, 0);
            pool.parallel_for(mine.size(), [&](size_t i) { mine[i] += 1; });
            check(mine, "nested in begin/end");
            if (async) pool.end();
            else pool.parallel_for(n, fn);
            check(*hits, "begin/end");
            delete hits;                     // a worker still in fn would now touch freed memory
        } else if (mode == 2) {
            std::vector<int> hits(n, 0);
            std::vector<std::vector<int>> inner(n, std::vector<int>(3, 0));
            pool.parallel_for(n, [&](size_t i) {
                hits[i] += 1;
                pool.parallel_for(3, [&](size_t k) { inner[i][k] += 1; });
            });
            check(hits, "nested outer");
            for (auto& v : inner) check(v, "nested inner");
        } else if (mode == 3) {
            if (n == 0) continue;
            const size_t at = rng() % n;
            std::vector<std::atomic<int>> hits(n);
            for (auto& h : hits) h.store(0);
            bool caught = false;
            try {
                pool.parallel_for(n, [&](size_t i) {
                    hits[i].fetch_add(1);
                    if (i == at) throw Boom{at};
                });
            } catch (const Boom& b) {
                caught = b.at == at;
            }
            if (!caught) bad("exception not rethrown", (long)at, (long)n);
            for (size_t i = 0; i < n; ++i)
                if (hits[i].load() > 1) bad("index ran twice (throwing job)", (long)i, hits[i].load());
        } else {
            // many tiny jobs back to back (the LO rounds' cadence)
            for (int k = 0; k < 8; ++k) {
                std::vector<int> hits(2 + k, 0);
                pool.parallel_for(hits.size(), [&](size_t i) { hits[i] += 1; });
                check(hits, "tiny");
            }
        }
        calls.fetch_add(1, std::memory_order_relaxed);
    }
}

}  // namespace

int main(int argc, char** argv) {
    const int callers = argc > 1 ? atoi(argv[1]) : 6;
    const int reps = argc > 2 ? atoi(argv[2]) : 400;
    const unsigned threads = argc > 3 ? (unsigned)atoi(argv[3]) : 8;
    std::atomic<long> calls{0};
    {
        Pool pool(threads);
        std::vector<std::thread> ts;
        for (int c = 0; c < callers; ++c)
            ts.emplace_back([&, c] { caller(pool, 1234u + (unsigned)c, reps, calls); });
        for (auto& t : ts) t.join();
        // the solving thread alone afterwards
        caller(pool, 99u, reps / 4, calls);
    }
    if (g_bad.load()) {
        fprintf(stderr, "host pool hammer: %ld failures\n", g_bad.load());
        return 1;
    }
    printf("OK %ld calls\n", calls.load());
    return 0;
}
