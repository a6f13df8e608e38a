// host_fit.h -- host-side model fitting for local optimisation and the final
// refit (the parts north_star keeps in host C++).  Per-feature constants come
// from the problem's precomputed SoA arrays; hypothesis-dependent angles use
// glibc, as the reference's fits do (models are never twin arithmetic).
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <type_traits>
#include <vector>

#include "fund.h"
#include "geo.h"
#include "gram.h"
#include "rect.h"

namespace gcr {

// Per-class host copy of the features plus the precomputed per-feature
// constants (same values the GPU holds):
//   scale class:       c0 = pow(s, kScalePower)      (glibc, +1/3 or -1/3)
//   orientation class: c0 = cos(theta), c1 = sin(theta)
// std::vector storage that default-initialises (no zero fill on resize): the
// feature columns are filled in parallel right after sizing
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = DefaultInitAlloc<U>;
    };
    DefaultInitAlloc() = default;
    template <class U>
    DefaultInitAlloc(const DefaultInitAlloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) {
        ::new (static_cast<void*>(p)) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};
using HVec = std::vector<double, DefaultInitAlloc<double>>;

struct HostClass {
    HVec x, y, a, c0, c1;
    size_t n = 0;
};

// Eigen ColPivHouseholderQR<MatrixX3d>::compute(A).solve(b) restated for an
// m x 3 column-major matrix (A and b are overwritten); qr3.h, blocked sums.
void colpiv_qr_solve3(std::vector<double>& A, size_t m, std::vector<double>& b, double x[3]);

// Another backend for the hybrid fit's least-squares system (the GPU refit):
// builds the ns scale rows + C(no, 2) vanishing-point pair rows of the index
// lists itself and solves them with qr3_solve; must be op-identical to the
// host path (rows as in fit_sift22, blocked sums).
struct SiftSystemSolver {
    virtual ~SiftSystemSolver() = default;
    virtual void solve(const std::vector<uint32_t>& si, const std::vector<uint32_t>& oi, size_t rows,
                       double x[3]) = 0;
    // the double-double Gram matrix of the same rows (gram.h order), ten
    // entries; false: not available here (the host computes it)
    virtual bool gram(const std::vector<uint32_t>& si, const std::vector<uint32_t>& oi, size_t rows,
                      DD g[kGramN]) { return false; }
    // fn(lo, hi) over [0, n) in disjoint ranges, possibly in parallel (the
    // per-inlier work around a big solve); the default runs it in one piece
    virtual void for_ranges(size_t n, const std::function<void(size_t, size_t)>& fn) { fn(0, n); }
};

// RectifyingHomographyEstimator::estimateModelNonminimal for the three solvers
// (rectifying_homography_estimator.h:164-227): normalisation check, then the
// minimal solver when the subset is exactly minimal, else weighted LS (+ mode).
// Hybrid systems with at least `big_rows` rows go to `big` when given.
bool fit_nonminimal(int solver, const HostClass* cls, const std::vector<uint32_t>* idx, RectModel& out,
                    SiftSystemSolver* big = nullptr, size_t big_rows = 0);

// Non-minimal homography fit (LO and final refit; geo.h): exactly 4 points ->
// the minimal solver; more -> Hartley-normalised DLT, h33 = 1, solved by the
// 8-column pivoted QR of qr3.h, denormalised and scaled to h33 = 1.
// Correspondences: c.x = x1, c.y = y1, c.a = x2, c.c0 = y2.
bool fit_h4_nonminimal(const HostClass& c, const std::vector<uint32_t>& idx, GeoModel& out);

// Non-minimal fundamental-matrix fit (LO and final refit; fund.h): exactly 7
// points -> the 7-point solver's first model; more -> normalised 8-point
// (smallest eigenvector of A^T A by cyclic Jacobi, rank-2 projection), unit
// Frobenius norm.  Blocked-order sums (qr3.h), restated by the oracle.
bool fit_f8_nonminimal(const HostClass& c, const std::vector<uint32_t>& idx, GeoModel& out);

// Cyclic Jacobi eigen-decomposition of a symmetric N x N matrix (a is
// destroyed); eigenvalues d[k] with eigenvectors in the COLUMNS of v.
template <int N>
void jacobi_eigen(double (&a)[N][N], double (&v)[N][N], double (&d)[N]);

// findWeightedMode (two_sift.hpp:354-394), libstdc++ unordered_map order.
double weighted_mode(const std::vector<double>& angles, const std::vector<double>& weights, double bin_width);

// The hybrid system's Gram matrix on the host, in gram.h's order (tiles,
// 256 lanes, halving tree, tiles in order): bit-identical to the GPU kernel.
void gram_sift_host(const HostClass& sc, const HostClass& oc, const std::vector<uint32_t>& si,
                    const std::vector<uint32_t>& oi, size_t rows, DD g[kGramN]);
// min |A x - b| from the Gram matrix of [A | b] (gram.h): column-pivoted
// Cholesky in double-double with Eigen's pivot rule and rank threshold.
void gram_solve3(const DD g[kGramN], size_t rows, double x[3]);
// GCR_REFIT=qr: big hybrid systems by Householder QR (round 2) instead
bool gram_refit_on();

// RectifyingHomography::getHomography (model.h:211-226), row-major, / H22.
void homography_of(const RectModel& m, double H[9]);

}  // namespace gcr
