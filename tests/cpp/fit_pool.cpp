// The host fits on the engine's host pool, built by tests/test_sanitizers.py
// under AddressSanitizer + UBSan (and ThreadSanitizer).
//
// Round-5 heap corruption: fit_sift22's rectified-angle
// lambda, which a big refit spreads over the pool (SiftSystemSolver::
// for_ranges), once named a thread_local scratch vector inside its body.  A
// thread_local named in a lambda is the EXECUTING thread's instance, so every
// worker wrote the angles of its range into its own vector -- sized by that
// worker's last LO fit (14 entries), or empty -- past its end.  The caller's
// vector kept stale angles.  This program does what the engine does: LO-sized
// fits on the pool first (the workers' scratch gets small), then big refits
// whose angles go through the pool, each compared bit for bit with the same
// fit done serially.  The old code fails here with a heap-buffer-overflow
// under ASan (and wrong models without it).
#include "host_fit.h"
#include "host_pool.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

using namespace gcr;

namespace {

struct PoolSolver : SiftSystemSolver {
    HostPool* pool;
    explicit PoolSolver(HostPool* p) : pool(p) {}
    void solve(const std::vector<uint32_t>&, const std::vector<uint32_t>&, size_t, double x[3]) override {
        x[0] = x[1] = x[2] = 0.0;     // not reached: the systems below take the Gram path
        std::fprintf(stderr, "unexpected solve()\n");
    }
    // the engine's GpuSiftSolver::for_ranges: 8 ranges on the pool
    void for_ranges(size_t n, const std::function<void(size_t, size_t)>& fn) override {
        const size_t parts = n < 1024 ? 1 : 8;
        const size_t step = (n + parts - 1) / parts;
        pool->parallel_for(parts, [&](size_t p) {
            const size_t lo = p * step, hi = std::min(n, lo + step);
            if (lo < hi) fn(lo, hi);
        });
    }
};

bool same(const RectModel& a, const RectModel& b) { return std::memcmp(&a, &b, sizeof(RectModel)) == 0; }

}  // namespace

int main() {
    std::mt19937_64 rng(11);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    HostClass cls[2];
    const size_t n = 3000;
    for (int c = 0; c < 2; ++c) {
        cls[c].n = n;
        for (size_t i = 0; i < n; ++i) {
            const double th = 6.283185307179586 * U(rng);
            const double s = 1.0 + U(rng);
            cls[c].x.push_back(1000 * U(rng));
            cls[c].y.push_back(800 * U(rng));
            cls[c].a.push_back(c == 0 ? s : th);
            cls[c].c0.push_back(c == 0 ? std::cbrt(s) : std::cos(th));
            cls[c].c1.push_back(c == 0 ? 0.0 : std::sin(th));
        }
    }
    HostPool pool(8);
    PoolSolver big(&pool);
    long bad = 0, fitted = 0;
    for (int round = 0; round < 6; ++round) {
        // LO trials: 50 fits of 14 + 14 points on the pool's threads
        std::vector<RectModel> lo(50);
        std::vector<char> ok(50, 0);
        std::vector<std::vector<uint32_t>> idx(100);
        for (auto& v : idx)
            for (int k = 0; k < 14; ++k) v.push_back((uint32_t)(U(rng) * n));
        pool.parallel_for(50, [&](size_t t) {
            std::vector<uint32_t> two[2] = {idx[2 * t], idx[2 * t + 1]};
            ok[t] = fit_nonminimal(2, cls, two, lo[t], nullptr, 0) ? 1 : 0;
        });
        for (size_t t = 0; t < 50; ++t) {
            RectModel m{};
            std::vector<uint32_t> two[2] = {idx[2 * t], idx[2 * t + 1]};
            const bool o = fit_nonminimal(2, cls, two, m, nullptr, 0);
            if (o != (ok[t] != 0) || (o && !same(m, lo[t]))) ++bad;
        }
        // the final refit: a big hybrid system, angles spread over the pool
        std::vector<uint32_t> big_idx[2];
        const size_t ns = 200 + rng() % 300, no = 1030 + rng() % 500;     // >= 1024: 8 ranges
        for (size_t k = 0; k < ns; ++k) big_idx[0].push_back((uint32_t)(U(rng) * n));
        for (size_t k = 0; k < no; ++k) big_idx[1].push_back((uint32_t)(U(rng) * n));
        RectModel mp{}, ms{};
        const bool op = fit_nonminimal(2, cls, big_idx, mp, &big, 0);
        const bool os = fit_nonminimal(2, cls, big_idx, ms, nullptr, 0);
        if (op != os || (op && !same(mp, ms))) {
            ++bad;
            std::fprintf(stderr, "round %d: pooled refit differs from the serial one (phi %.17g vs %.17g)\n", round,
                         mp.phi, ms.phi);
        }
        fitted += op ? 1 : 0;
    }
    if (bad) {
        std::fprintf(stderr, "fit_pool: %ld mismatches\n", bad);
        return 1;
    }
    std::printf("OK %ld big refits\n", fitted);
    return 0;
}
