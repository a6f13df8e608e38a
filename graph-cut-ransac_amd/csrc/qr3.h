// qr3.h -- least-squares solve of an m x 3 system by column-pivoted Householder
// QR (Eigen ColPivHouseholderQR<MatrixX3d>::compute(A).solve(b), the solve the
// reference's non-minimal fits call: three_sift.hpp:237, two_sift.hpp:524),
// written once against a storage backend so that the host (LO fits, small
// systems) and the GPU (the hybrid final refit's ~n_o^2/2 pair rows) run the
// same control flow and the same per-element arithmetic.
//
// Reductions use ONE fixed order, blocked_sum: rows are grouped into aligned
// blocks of kSumBlock = 1024 rows; inside a block, "lane" l (0..255) sums the
// rows base + l + 256 q (q = 0..3) of the range sequentially, and the 256 lane
// partials are combined by a halving tree (x[l] += x[l + h] for h = 128, 64,
// .., 1; the value of x[0]); block partials are summed sequentially inside
// aligned super-blocks of kSumSuper rows, then the super-block partials
// sequentially.  It is the order a 256-thread GPU workgroup produces with
// coalesced loads (one block per workgroup, the tree's two top levels through
// LDS, the rest as a wave butterfly, whose lane 0 equals the halving tree), so
// the refit's passes are bandwidth-bound.  Eigen's own order is
// packet-vectorised and unpinned (no Eigen here).  The oracle restates the
// same order (oracle/gcr_oracle.cpp), so host, GPU and oracle agree bitwise.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <limits>
#include <utility>

namespace gcr {

constexpr size_t kSumBlock = 1024;
constexpr size_t kSumLanes = 256;                // lanes of a block (rows l + 256 q)
constexpr size_t kSumSuper = 64 * kSumBlock;     // super-blocks: 64 blocks

// the block partial of block `base` (aligned) over rows [lo, hi) ∩ block.
// Lanes at or above `top` (the rows end before reaching them) hold +0.0, and
// no lane ever holds -0.0 (every lane starts at +0.0 and round-to-nearest
// sums reach zero only as +0.0), so x + acc[l + h] with l + h >= top is x
// itself: each tree level adds only the pairs whose upper lane may be
// nonzero -- the full tree's value bit for bit, at a fraction of its adds
// for short ranges (the LO trials' 105-row systems).
template <class F>
inline double block_partial(size_t base, size_t lo, size_t hi, F f) {
    if (base == 0 && hi <= kSumLanes) {
        // one row per lane (systems of at most 256 rows, e.g. the LO trials'):
        // the same lane values and halving tree without the lane loop's
        // read-modify-write (+0.0 + f, as the lane sum of one row)
        double acc[kSumLanes];
        if (hi == 0) return 0.0;
        for (size_t l = 0; l < lo; ++l) acc[l] = 0.0;
        for (size_t l = lo; l < hi; ++l) acc[l] = 0.0 + f(l);
        size_t top = hi;
        for (size_t h = kSumLanes / 2; h >= 1; h >>= 1) {
            if (top <= h) continue;
            double* __restrict d = acc;                 // [0, top - h) and [h, top) do not overlap
            const double* __restrict u = acc + h;
            const size_t n2 = top - h;
            for (size_t l = 0; l < n2; ++l) d[l] = d[l] + u[l];
            top = h;
        }
        return acc[0];
    }
    double acc[kSumLanes];
    const size_t b0 = std::max(base, lo), b1 = std::min(base + kSumBlock, hi);
    size_t top = b1 > base ? std::min(kSumLanes, b1 - base) : 0;
    for (size_t l = 0; l < top; ++l) acc[l] = 0.0;
    for (size_t i = b0; i < b1; ++i) acc[(i - base) & (kSumLanes - 1)] += f(i);   // each lane in q order
    if (top == 0) return 0.0;
    for (size_t h = kSumLanes / 2; h >= 1; h >>= 1) {
        if (top <= h) continue;
        for (size_t l = 0; l + h < top; ++l) acc[l] = acc[l] + acc[l + h];
        top = h;
    }
    return acc[0];
}

// sum_{i in [lo, hi)} f(i) in blocked order (see the file comment)
template <class F>
inline double blocked_sum(size_t lo, size_t hi, F f) {
    double total = 0.0;
    size_t i = lo;
    while (i < hi) {
        const size_t send = std::min(hi, (i / kSumSuper + 1) * kSumSuper);
        double sup = 0.0;
        while (i < send) {
            const size_t base = i / kSumBlock * kSumBlock;
            const size_t end = std::min(send, base + kSumBlock);
            sup += block_partial(base, i, end, f);
            i = end;
        }
        total += sup;
    }
    return total;
}

// Backend S stores C + 1 columns of length m: 0..C-1 = A, C = b, and provides
//   double sumsq(c, lo, hi)             blocked sum of col[c][i]^2
//   double dot(a, c, lo, hi)            blocked sum of col[a][i] * col[c][i]
//   double get(c, i); void set(c, i, v)
//   void scale(c, lo, hi, den)          col[c][i] = col[c][i] / den
//   void zero(c, lo, hi)
//   void update(c, e, lo, hi, tau, t)   col[c][i] -= (tau * col[e][i]) * t
template <int C, class S>
void qr_solve(S& st, size_t m, double x[C]) {
    constexpr size_t cols = C;
    constexpr int kB = C;                  // stored column of b
    auto sq = [](double v) { return v * v; };
    const size_t size = std::min(m, cols);
    int pc[C];                             // logical -> stored column (pivot swaps)
    double tau_k[C];
    size_t transp[C];
    double nu[C], nd[C];
    for (int k = 0; k < C; ++k) { pc[k] = k; tau_k[k] = 0.0; transp[k] = k; }
    for (size_t k = 0; k < cols; ++k) {
        nd[k] = std::sqrt(st.sumsq(pc[k], 0, m));
        nu[k] = nd[k];
    }
    const double eps = std::numeric_limits<double>::epsilon();
    double maxn = nu[0];
    for (size_t k = 1; k < cols; ++k)
        if (maxn < nu[k]) maxn = nu[k];
    const double thr_helper = sq(maxn * eps) / (double)m;
    const double downdate_thr = std::sqrt(eps);
    size_t nonzero = size;

    // H_k = I - tau v v^T applied to stored column c; v = (1, ess[k+1..m))
    auto apply_reflector = [&](int ess, size_t k, double tau, int c) {
        if (m - k == 1) {
            st.set(c, k, st.get(c, k) * (1.0 - tau));
            return;
        }
        if (tau == 0.0) return;
        double t = st.dot(ess, c, k + 1, m);
        const double ck = st.get(c, k);
        t += ck;
        st.set(c, k, ck - tau * t);
        st.update(c, ess, k + 1, m, tau, t);
    };

    for (size_t k = 0; k < size; ++k) {
        size_t big = k;
        double bign = nu[k];
        for (size_t j = k + 1; j < cols; ++j)
            if (bign < nu[j]) { bign = nu[j]; big = j; }
        if (nonzero == size && sq(bign) < thr_helper * (double)(m - k)) nonzero = k;
        transp[k] = big;
        if (k != big) {
            std::swap(pc[k], pc[big]);
            std::swap(nu[k], nu[big]);
            std::swap(nd[k], nd[big]);
        }
        const int ck = pc[k];
        const double tail = st.sumsq(ck, k + 1, m);
        const double c0 = st.get(ck, k);
        double tau, beta;
        if (tail <= std::numeric_limits<double>::min()) {
            tau = 0.0;
            beta = c0;
            st.zero(ck, k + 1, m);
        } else {
            beta = std::sqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
            st.scale(ck, k + 1, m, c0 - beta);
            tau = (beta - c0) / beta;
        }
        tau_k[k] = tau;
        st.set(ck, k, beta);
        for (size_t j = k + 1; j < cols; ++j) apply_reflector(ck, k, tau, pc[j]);
        for (size_t j = k + 1; j < cols; ++j) {
            if (nu[j] != 0.0) {
                double temp = std::fabs(st.get(pc[j], k)) / nu[j];
                temp = (1.0 + temp) * (1.0 - temp);
                temp = temp < 0.0 ? 0.0 : temp;
                const double temp2 = temp * sq(nu[j] / nd[j]);
                if (temp2 <= downdate_thr) {
                    nd[j] = std::sqrt(st.sumsq(pc[j], k + 1, m));
                    nu[j] = nd[j];
                } else {
                    nu[j] *= std::sqrt(temp);
                }
            }
        }
    }
    size_t perm[C];
    for (int k = 0; k < C; ++k) perm[k] = k;
    for (size_t k = 0; k < size; ++k) std::swap(perm[k], perm[transp[k]]);
    if (nonzero == 0) {
        for (int k = 0; k < C; ++k) x[k] = 0.0;
        return;
    }
    for (size_t k = 0; k < nonzero; ++k) apply_reflector(pc[k], k, tau_k[k], kB);
    double c[C];
    for (int k = 0; k < C; ++k) c[k] = m > (size_t)k ? st.get(kB, k) : 0.0;
    for (size_t jj = nonzero; jj-- > 0;) {
        c[jj] = c[jj] / st.get(pc[jj], jj);
        for (size_t i = 0; i < jj; ++i) c[i] -= c[jj] * st.get(pc[jj], i);
    }
    for (size_t i = 0; i < nonzero; ++i) x[perm[i]] = c[i];
    for (size_t i = nonzero; i < cols; ++i) x[perm[i]] = 0.0;
}

template <class S>
void qr3_solve(S& st, size_t m, double x[3]) { qr_solve<3>(st, m, x); }

// Host storage: C + 1 column pointers of length m (C = 3 unless given).
template <int C = 3>
struct HostQRStoreN {
    double* col[C + 1];
    double sumsq(int c, size_t lo, size_t hi) const {
        const double* p = col[c];
        return blocked_sum(lo, hi, [p](size_t i) { return p[i] * p[i]; });
    }
    double dot(int a, int c, size_t lo, size_t hi) const {
        const double* p = col[a];
        const double* q = col[c];
        return blocked_sum(lo, hi, [p, q](size_t i) { return p[i] * q[i]; });
    }
    double get(int c, size_t i) const { return col[c][i]; }
    void set(int c, size_t i, double v) { col[c][i] = v; }
    void scale(int c, size_t lo, size_t hi, double den) {
        for (size_t i = lo; i < hi; ++i) col[c][i] = col[c][i] / den;
    }
    void zero(int c, size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) col[c][i] = 0.0;
    }
    void update(int c, int e, size_t lo, size_t hi, double tau, double t) {
        for (size_t i = lo; i < hi; ++i) col[c][i] -= (tau * col[e][i]) * t;
    }
};

using HostQRStore = HostQRStoreN<3>;

}  // namespace gcr
