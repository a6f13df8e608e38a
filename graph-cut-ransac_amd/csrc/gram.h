// gram.h -- the hybrid final refit's big least-squares systems by a
// double-double Gram matrix (GCR_HD: the gfx950 kernel and the host build the
// same sums in the same order).
//
// The reference solves min |A x - b| with Eigen's colPivHouseholderQr
// (two_sift.hpp:423-579, :524), whose reduction order is unpinned.  A system
// of n_s scale rows and C(n_o, 2) vanishing-point pair rows has ~3 M rows at
// n_o = 2500; Householder QR streams its columns through HBM six times.
// Here every row is built once, on the fly, and contributes its ten products
// r_a r_b (a <= b over the columns of [A | b]) to a 4 x 4 Gram matrix
// accumulated in double-double (error-free products, accurate DW additions,
// relative error ~2^-104), and the 3 x 3 system is solved by column-pivoted
// Cholesky in double-double arithmetic, with Eigen's pivot rule (largest
// remaining column norm, first on ties) and rank threshold ((max norm eps)^2
// / rows * (rows - k)).  The normal equations square the condition number,
// which the ~2^-104 accuracy of the sums absorbs: the solution is the exact
// least-squares solution to ~1 ulp, i.e. at least as close to it as the
// Householder solve.  The oracle restates this (oracle/gcr_oracle.cpp) and
// the frozen QR pin (tests/test_frozen_pin.py) holds it to the sequential
// Householder order within 1e-6.
//
// Order (defines the sums bit for bit): rows r = 0 .. rows-1 (scale rows,
// then pair rows i < j in lexicographic order) in tiles of kGramTile rows;
// inside a tile, lane l (0..255) accumulates rows tile*kGramTile + l + 256 u
// (u increasing); the 256 lane sums are combined by the halving tree
// x[l] += x[l + h], h = 128 .. 1.  The tile sums: lane l (0..63) adds tiles
// l, l + 64, l + 128, ... in order to +0, then the halving tree h = 32 .. 1
// (one parallel combination on the device instead of a sequential chain of
// every tile).
#pragma once

#include "gcr_hd.h"

namespace gcr {

constexpr size_t kGramRows = 32768;     // hybrid systems of at least this many rows take the Gram path
constexpr size_t kGramTile = 4096;      // rows per tile
constexpr int kGramLanes = 256;         // lanes per tile
constexpr int kGramN = 10;              // products r_a r_b, a <= b, of the 4 columns of [A | b]

struct DD {
    double hi, lo;
};

GCR_HD DD dd_two_sum(double a, double b) {
    const double s = a + b;
    const double bb = s - a;
    return DD{s, (a - (s - bb)) + (b - bb)};
}
GCR_HD DD dd_fast_two_sum(double a, double b) {      // |a| >= |b| (or a == 0)
    const double s = a + b;
    return DD{s, b - (s - a)};
}
GCR_HD DD dd_two_prod(double a, double b) {
    const double p = a * b;
    return DD{p, fma_rn(a, b, -p)};
}
// AccurateDWPlusDW (Joldes, Muller, Popescu 2017, Alg. 6): relative error <= 3 u^2
GCR_HD DD dd_add(DD x, DD y) {
    const DD s = dd_two_sum(x.hi, y.hi);
    const DD t = dd_two_sum(x.lo, y.lo);
    const double c = s.lo + t.hi;
    const DD v = dd_fast_two_sum(s.hi, c);
    const double w = t.lo + v.lo;
    return dd_fast_two_sum(v.hi, w);
}
GCR_HD DD dd_neg(DD x) { return DD{-x.hi, -x.lo}; }
GCR_HD DD dd_sub(DD x, DD y) { return dd_add(x, dd_neg(y)); }
// DWTimesDW (Alg. 12 of the same paper, with FMA)
GCR_HD DD dd_mul(DD x, DD y) {
    const DD c = dd_two_prod(x.hi, y.hi);
    const double tl = x.hi * y.lo;
    const double tl2 = fma_rn(x.lo, y.hi, tl);
    return dd_fast_two_sum(c.hi, c.lo + tl2);
}
// DWDivDW (Alg. 17): one double division, two corrections
GCR_HD DD dd_div(DD x, DD y) {
    const double th = x.hi / y.hi;
    const DD r = dd_mul(y, DD{th, 0.0});
    const double ph = x.hi - r.hi;
    const double dl = x.lo - r.lo;
    const double d = ph + dl;
    const double tl = d / y.hi;
    return dd_fast_two_sum(th, tl);
}
// sqrt of a non-negative double-double: one Newton step on the double root
GCR_HD DD dd_sqrt(DD x) {
    if (!(x.hi > 0.0)) return DD{x.hi == 0.0 ? 0.0 : sqrt(x.hi), 0.0};
    const double s = sqrt(x.hi);
    const DD s2 = dd_two_prod(s, s);
    const double r = ((x.hi - s2.hi) - s2.lo) + x.lo;
    return dd_fast_two_sum(s, r / (2.0 * s));
}
GCR_HD bool dd_lt(DD a, DD b) { return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo); }

// the ten products of one row (r0, r1, r2 | r3), order 00 01 02 03 11 12 13 22 23 33
GCR_HD void gram_add_row(DD acc[kGramN], const double r[4]) {
    int k = 0;
    for (int a = 0; a < 4; ++a)
        for (int b = a; b < 4; ++b, ++k) acc[k] = dd_add(acc[k], dd_two_prod(r[a], r[b]));
}

// a pair row (r2 == +0.0) with finite r0, r1, r3: its four products with r2
// are zeros, and adding a zero double-double to a finite accumulator of
// gram_add_row leaves it bit for bit unchanged (the accumulators are
// normalised and never hold a -0.0), so only the other six are added
GCR_HD void gram_add_pair_row(DD acc[kGramN], const double r[4]) {
    acc[0] = dd_add(acc[0], dd_two_prod(r[0], r[0]));
    acc[1] = dd_add(acc[1], dd_two_prod(r[0], r[1]));
    acc[3] = dd_add(acc[3], dd_two_prod(r[0], r[3]));
    acc[4] = dd_add(acc[4], dd_two_prod(r[1], r[1]));
    acc[6] = dd_add(acc[6], dd_two_prod(r[1], r[3]));
    acc[9] = dd_add(acc[9], dd_two_prod(r[3], r[3]));
}

// pair p (0-based, lexicographic i < j over n) -> (i, j): a floating
// estimate corrected with exact integer arithmetic
GCR_HD void pair_of(uint64_t p, uint64_t n, uint64_t& i, uint64_t& j) {
    const double q = (double)(2 * n - 1);
    int64_t ii = (int64_t)((q - sqrt(q * q - 8.0 * (double)p)) * 0.5);
    if (ii < 0) ii = 0;
    if (ii > (int64_t)n - 2) ii = (int64_t)n - 2;
    while (ii > 0 && (uint64_t)ii * (2 * n - (uint64_t)ii - 1) / 2 > p) --ii;
    while ((uint64_t)ii + 2 < n && ((uint64_t)ii + 1) * (2 * n - (uint64_t)ii - 2) / 2 <= p) ++ii;
    i = (uint64_t)ii;
    j = p - i * (2 * n - i - 1) / 2 + i + 1;
}

// the halving tree over kGramLanes lane sums (lane[l * kGramN + k]) into
// lane 0
GCR_HD void gram_lane_tree(DD* lane) {
    for (int h = kGramLanes / 2; h >= 1; h >>= 1)
        for (int l = 0; l < h; ++l)
            for (int k = 0; k < kGramN; ++k)
                lane[(size_t)l * kGramN + k] = dd_add(lane[(size_t)l * kGramN + k], lane[(size_t)(l + h) * kGramN + k]);
}

// the tile sums (tiles[t * kGramN + k], nt tiles) into the matrix g, in the
// order above (host restatement of k_sift_gram's last workgroup)
constexpr int kGramTileLanes = 64;      // lanes of the tile-sum combination
inline void gram_combine_tiles(const DD* tiles, size_t nt, DD g[kGramN]) {
    DD lane[kGramTileLanes * kGramN];
    for (int l = 0; l < kGramTileLanes; ++l) {
        DD* a = lane + (size_t)l * kGramN;
        for (int k = 0; k < kGramN; ++k) a[k] = DD{0.0, 0.0};
        for (size_t t = (size_t)l; t < nt; t += kGramTileLanes)
            for (int k = 0; k < kGramN; ++k) a[k] = dd_add(a[k], tiles[t * kGramN + k]);
    }
    for (int h = kGramTileLanes / 2; h >= 1; h >>= 1)
        for (int l = 0; l < h; ++l)
            for (int k = 0; k < kGramN; ++k)
                lane[(size_t)l * kGramN + k] = dd_add(lane[(size_t)l * kGramN + k], lane[(size_t)(l + h) * kGramN + k]);
    for (int k = 0; k < kGramN; ++k) g[k] = lane[k];
}

// index of (a, b), a <= b, in the product order
GCR_HD int gram_index(int a, int b) {
    if (a > b) { const int t = a; a = b; b = t; }
    return a * 4 - (a * (a - 1)) / 2 + (b - a);
}

}  // namespace gcr
