// graphcut.h -- host graph-cut labeling for the 1-class local optimisation:
// the neighbourhood grid's edge list and a Boykov-Kolmogorov st-mincut.
//
// GCRANSAC::labeling (HDR/GCRANSAC.h:759-870) builds, per graph-cut round, an
// Energy<double,double,double> (HDR/energy.h:204-245) over the points: unary
// terms from the truncated quadratic cost of the LO model, and for
// lambda > 0 a pairwise term for every pair of points that share a cell of the
// neighbourhood grid (neighborhood/grid_neighborhood_graph.h:229-301), then
// runs BK max-flow (HDR/graph.h, graph.ti, maxflow.ti) and returns the SINK
// nodes as inliers.  The reference's own entry points build the grid over an
// empty point set (gcransac_python.cpp:60-67), so only the correspondence
// estimators (findHomography / findFundamentalMatrix, an extension here) ever
// have pairwise terms.
//
// The cut found is the minimal sink side (the nodes that can still reach the
// sink), which is unique for exact arithmetic; to stay bit-identical with the
// reference under floating-point rounding the max-flow below performs the
// reference's operations in the reference's order: arcs in sister pairs
// prepended to their tail's list, the two-queue active list, orphans at the
// front after an augmentation and at the rear during adoption, the TS/DIST
// origin heuristics.  The data layout is flat arrays with 32-bit indices (no
// pointers, no block allocator) sized once and reused across rounds.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <numeric>
#include <vector>

namespace gcr {

// Edges of the neighbourhood grid in labeling()'s order (GCRANSAC.h:821-857):
// for every point i in row order, every later point of its cell, ascending.
// The cell of a point is sum_d idx_d * cell_number^d (size_t arithmetic) with
// idx_d = floor(coord_d / cell_size_d) converted to size_t as on x86-64 (the
// 64-bit two's-complement value; 2^63 when out of range), grid_neighborhood_
// graph.h:246-267 / GridCell :70-82; cells are keyed by that index alone.
struct NeighbourEdges {
    std::vector<uint32_t> u, v;
    // the same graph by cell: cell c's points are nodes[off[c] .. off[c+1])
    // in ascending order (cells of >= 2 points only); its edges are every
    // pair of them, in labeling()'s order (a < b, by a then b)
    std::vector<uint32_t> off, nodes;
    // points outside every multi-point cell (the terminal test), ascending
    std::vector<uint32_t> singles;
    // per point: its position in nodes, or kNoPos for a single
    static constexpr uint32_t kNoPos = 0xffffffffu;
    std::vector<uint32_t> pos_of;
    // the labeling's work units for a pool (gc_schedule): job j covers
    // cells order[jobs[j].b .. jobs[j].e); range r the points
    // [ranges[r].b, ranges[r].e) of the assembly pass
    struct Job {
        uint32_t kind, b, e;
    };
    std::vector<uint32_t> order;
    std::vector<Job> jobs, ranges;
    size_t cells() const { return off.empty() ? 0 : off.size() - 1; }
};

inline uint64_t grid_axis_index(double v) {
    const double f = std::floor(v);
    if (!(f >= -9.2233720368547758e18 && f < 9.2233720368547758e18)) return (uint64_t)1 << 63;
    return (uint64_t)(int64_t)f;
}

// coords: `dims` column pointers of n values each; the explicit edge list
// (u, v) only when `with_edges` (the engine needs the cells alone)
inline void grid_edges(const double* const* coords, int dims, size_t n, const double* cell_size,
                       uint64_t cell_number, NeighbourEdges& out, bool with_edges = true) {
    out.u.clear();
    out.v.clear();
    out.off.assign(1, 0);
    out.nodes.clear();
    // (cell key, point) sorted: cells in key order, points ascending inside
    std::vector<std::pair<uint64_t, uint32_t>> kp(n);
    uint64_t kmax = 0;
    for (size_t i = 0; i < n; ++i) {
        uint64_t k = 0, off = 1;
        for (int d = 0; d < dims; ++d) {
            k += off * grid_axis_index(coords[d][i] / cell_size[d]);
            off *= cell_number;
        }
        kp[i] = {k, (uint32_t)i};
        kmax = std::max(kmax, k);
    }
    if (kmax < ((uint64_t)1 << 22) && kmax < 64 * (uint64_t)n + 4096) {
        // the usual case (coordinates inside the image): a counting sort over
        // the cell keys, stable, so points stay ascending inside a cell
        std::vector<uint32_t> start(kmax + 2, 0);
        for (size_t i = 0; i < n; ++i) ++start[kp[i].first + 1];
        for (uint64_t k = 0; k <= kmax; ++k) start[k + 1] += start[k];
        std::vector<std::pair<uint64_t, uint32_t>> sorted(n);
        for (size_t i = 0; i < n; ++i) sorted[start[kp[i].first]++] = kp[i];
        kp.swap(sorted);
    } else {
        std::sort(kp.begin(), kp.end());
    }
    std::vector<uint8_t> in_cell(n, 0);
    for (size_t s0 = 0; s0 < n;) {
        size_t e = s0;
        while (e < n && kp[e].first == kp[s0].first) ++e;
        if (e - s0 >= 2) {
            for (size_t q = s0; q < e; ++q) {
                out.nodes.push_back(kp[q].second);
                in_cell[kp[q].second] = 1;
            }
            out.off.push_back((uint32_t)out.nodes.size());
        }
        s0 = e;
    }
    out.singles.clear();
    for (size_t i = 0; i < n; ++i)
        if (!in_cell[i]) out.singles.push_back((uint32_t)i);
    out.pos_of.assign(n, NeighbourEdges::kNoPos);
    for (size_t q = 0; q < out.nodes.size(); ++q) out.pos_of[out.nodes[q]] = (uint32_t)q;
    out.order.clear();
    out.jobs.clear();
    out.ranges.clear();
    if (!with_edges) return;
    // labeling()'s order: for every point i in row order, every later point
    // of its cell, ascending
    std::vector<uint32_t> cell_of(n, UINT32_MAX), pos(n, 0);
    for (size_t c = 0; c + 1 < out.off.size(); ++c)
        for (uint32_t q = out.off[c]; q < out.off[c + 1]; ++q) {
            cell_of[out.nodes[q]] = (uint32_t)c;
            pos[out.nodes[q]] = q;
        }
    for (size_t i = 0; i < n; ++i) {
        if (cell_of[i] == UINT32_MAX) continue;
        for (uint32_t q = pos[i] + 1; q < out.off[cell_of[i] + 1]; ++q) {
            out.u.push_back((uint32_t)i);
            out.v.push_back(out.nodes[q]);
        }
    }
}

// The labeling's work units for `parts` workers drawing jobs in order (the
// host pool hands them out dynamically): a cell costs ~ 8 + k^2 (BK on a
// k-clique; measured 27 us at k = 61, ~0.15 us at k = 3).  Cells costing
// more than a job's share (total / 4 parts) get a job each, largest first;
// the remaining cells are packed in index order into jobs of about that
// share.  Any order gives the same labeling: every cell is cut on its own
// (graphcut_labeling below).  The assembly pass takes 2 parts contiguous
// point ranges (multiples of 64 points).
inline void gc_schedule(NeighbourEdges& g, size_t parts) {
    g.order.clear();
    g.jobs.clear();
    g.ranges.clear();
    const size_t nc = g.cells();
    auto cost = [&](size_t c) { const double k = g.off[c + 1] - g.off[c]; return 8.0 + k * k; };
    double total = 0.0;
    for (size_t c = 0; c < nc; ++c) total += cost(c);
    const double share = total / (double)(4 * std::max<size_t>(parts, 1)) + 1.0;
    std::vector<uint32_t> big, rest;
    for (size_t c = 0; c < nc; ++c) (cost(c) >= share ? big : rest).push_back((uint32_t)c);
    std::stable_sort(big.begin(), big.end(), [&](uint32_t a, uint32_t b) { return cost(a) > cost(b); });
    for (uint32_t c : big) {
        g.jobs.push_back({0u, (uint32_t)g.order.size(), (uint32_t)g.order.size() + 1});
        g.order.push_back(c);
    }
    double acc = 0.0;
    uint32_t b = (uint32_t)g.order.size();
    for (uint32_t c : rest) {
        g.order.push_back(c);
        acc += cost(c);
        if (acc >= share) {
            g.jobs.push_back({0u, b, (uint32_t)g.order.size()});
            b = (uint32_t)g.order.size();
            acc = 0.0;
        }
    }
    if (b < g.order.size()) g.jobs.push_back({0u, b, (uint32_t)g.order.size()});
    const size_t n = g.pos_of.size();
    const size_t per = std::max<size_t>(1024, ((n + 2 * parts - 1) / std::max<size_t>(2 * parts, 1) + 63) & ~(size_t)63);
    for (size_t i = 0; i < n; i += per) g.ranges.push_back({1u, (uint32_t)i, (uint32_t)std::min(n, i + per)});
}

// Boykov-Kolmogorov max-flow, Graph<double,double,double> semantics.
class MaxFlow {
public:
    // storage grows to the largest graph seen and is reused (no per-graph
    // allocation or vector bookkeeping: the cells are mostly 2-4 nodes)
    void reset(size_t n_nodes, size_t n_edges) {
        n_ = n_nodes;
        if (first_.size() < n_) {
            first_.resize(n_);
            parent_.resize(n_);
            next_.resize(n_);
            ts_.resize(n_);
            dist_.resize(n_);
            sink_.resize(n_);
            tr_.resize(n_);
        }
        for (size_t i = 0; i < n_; ++i) {
            first_[i] = kNone;
            parent_[i] = kNone;
            next_[i] = kNone;
            ts_[i] = 0;
            dist_[i] = 0;
            sink_[i] = 0;
            tr_[i] = 0.0;
        }
        if (head_.size() < 2 * n_edges) {
            head_.resize(2 * n_edges);
            anext_.resize(2 * n_edges);
            rcap_.resize(2 * n_edges);
        }
        na_ = 0;
    }
    // Graph::add_tweights (graph.h:405-418)
    void add_tweights(int32_t i, double cap_source, double cap_sink) {
        const double delta = tr_[i];
        if (delta > 0) cap_source += delta;
        else cap_sink -= delta;
        tr_[i] = cap_source - cap_sink;
    }
    // Graph::add_edge (graph.h:420-452): arc 2k = i -> j, arc 2k+1 = j -> i
    void add_edge(int32_t i, int32_t j, double cap, double rev_cap) {
        const int32_t a = na_;
        if ((size_t)a + 2 > head_.size()) {                  // more edges than reset() was told
            head_.resize((size_t)a + 2);
            anext_.resize((size_t)a + 2);
            rcap_.resize((size_t)a + 2);
        }
        head_[a] = j;
        anext_[a] = first_[i];
        rcap_[a] = cap;
        first_[i] = a;
        head_[a + 1] = i;
        anext_[a + 1] = first_[j];
        rcap_[a + 1] = rev_cap;
        first_[j] = a + 1;
        na_ = a + 2;
    }
    // Energy::add_term1 / add_term2 (energy.h:204-245)
    void add_term1(int32_t x, double A, double B) { add_tweights(x, B, A); }
    void add_term2(int32_t x, int32_t y, double A, double B, double C, double D) {
        add_tweights(x, D, A);
        B -= A;
        C -= D;
        if (B < 0) {
            add_tweights(x, 0, B);
            add_tweights(y, 0, -B);
            add_edge(x, y, 0, B + C);
        } else if (C < 0) {
            add_tweights(x, 0, -C);
            add_tweights(y, 0, C);
            add_edge(x, y, B + C, 0);
        } else {
            add_edge(x, y, B, C);
        }
    }
    // what_segment (graph.h:476-487) with the default SOURCE: 1 = SINK
    bool is_sink(int32_t i) const { return parent_[i] != kNone && sink_[i]; }

    // Graph::maxflow (maxflow.ti:463-597), first call (no tree reuse)
    void maxflow() {
        init();
        int32_t cur = kNone;
        while (true) {
            int32_t i = cur;
            if (i != kNone) {
                next_[i] = kNone;
                if (parent_[i] == kNone) i = kNone;
            }
            if (i == kNone) {
                i = next_active();
                if (i == kNone) break;
            }
            int32_t a;
            if (!sink_[i]) {                              // grow the source tree
                for (a = first_[i]; a != kNone; a = anext_[a])
                    if (rcap_[a] != 0.0) {
                        const int32_t j = head_[a];
                        if (parent_[j] == kNone) {
                            sink_[j] = 0;
                            parent_[j] = a ^ 1;
                            ts_[j] = ts_[i];
                            dist_[j] = dist_[i] + 1;
                            set_active(j);
                        } else if (sink_[j]) {
                            break;
                        } else if (ts_[j] <= ts_[i] && dist_[j] > dist_[i]) {
                            parent_[j] = a ^ 1;
                            ts_[j] = ts_[i];
                            dist_[j] = dist_[i] + 1;
                        }
                    }
            } else {                                      // grow the sink tree
                for (a = first_[i]; a != kNone; a = anext_[a])
                    if (rcap_[a ^ 1] != 0.0) {
                        const int32_t j = head_[a];
                        if (parent_[j] == kNone) {
                            sink_[j] = 1;
                            parent_[j] = a ^ 1;
                            ts_[j] = ts_[i];
                            dist_[j] = dist_[i] + 1;
                            set_active(j);
                        } else if (!sink_[j]) {
                            a = a ^ 1;
                            break;
                        } else if (ts_[j] <= ts_[i] && dist_[j] > dist_[i]) {
                            parent_[j] = a ^ 1;
                            ts_[j] = ts_[i];
                            dist_[j] = dist_[i] + 1;
                        }
                    }
            }
            ++time_;
            if (a != kNone) {
                next_[i] = i;                             // keep i active
                cur = i;
                augment(a);
                // adoption (maxflow.ti:560-583): the orphan list is the
                // augmentation's front insertions, i.e. their reverse order;
                // each orphan is processed with everything its processing
                // appends before the next one
                for (size_t k = aug_.size(); k-- > 0;) {
                    adopt_.clear();
                    adopt_.push_back(aug_[k]);
                    for (size_t h = 0; h < adopt_.size(); ++h) {
                        const int32_t o = adopt_[h];
                        if (sink_[o]) process_orphan<true>(o);
                        else process_orphan<false>(o);
                    }
                }
                aug_.clear();
            } else {
                cur = kNone;
            }
        }
    }

private:
    static constexpr int32_t kNone = -1, kTerminal = -2, kOrphan = -3;
    static constexpr int kInfD = 0x7fffffff;
    size_t n_ = 0;
    int32_t na_ = 0;                                          // arcs in use
    std::vector<int32_t> first_, parent_, next_;
    std::vector<int> ts_, dist_;
    std::vector<uint8_t> sink_;
    std::vector<double> tr_;
    std::vector<int32_t> head_, anext_;
    std::vector<double> rcap_;
    int32_t qf_[2] = {kNone, kNone}, ql_[2] = {kNone, kNone};
    std::vector<int32_t> aug_, adopt_;
    int time_ = 0;

    void set_active(int32_t i) {
        if (next_[i] == kNone) {
            if (ql_[1] != kNone) next_[ql_[1]] = i;
            else qf_[1] = i;
            ql_[1] = i;
            next_[i] = i;
        }
    }
    int32_t next_active() {
        while (true) {
            int32_t i = qf_[0];
            if (i == kNone) {
                qf_[0] = i = qf_[1];
                ql_[0] = ql_[1];
                qf_[1] = ql_[1] = kNone;
                if (i == kNone) return kNone;
            }
            if (next_[i] == i) qf_[0] = ql_[0] = kNone;
            else qf_[0] = next_[i];
            next_[i] = kNone;
            if (parent_[i] != kNone) return i;
        }
    }
    void init() {
        qf_[0] = ql_[0] = qf_[1] = ql_[1] = kNone;
        aug_.clear();
        time_ = 0;
        for (size_t k = 0; k < n_; ++k) {
            const int32_t i = (int32_t)k;
            next_[i] = kNone;
            ts_[i] = 0;
            if (tr_[i] > 0) {
                sink_[i] = 0;
                parent_[i] = kTerminal;
                set_active(i);
                dist_[i] = 1;
            } else if (tr_[i] < 0) {
                sink_[i] = 1;
                parent_[i] = kTerminal;
                set_active(i);
                dist_[i] = 1;
            } else {
                parent_[i] = kNone;
            }
        }
    }
    void orphan_front(int32_t i) {
        parent_[i] = kOrphan;
        aug_.push_back(i);
    }
    // maxflow.ti augment: the middle arc runs from the source tree to the sink tree
    void augment(int32_t mid) {
        double bottleneck = rcap_[mid];
        int32_t i, a;
        for (i = head_[mid ^ 1];; i = head_[a]) {
            a = parent_[i];
            if (a == kTerminal) break;
            if (bottleneck > rcap_[a ^ 1]) bottleneck = rcap_[a ^ 1];
        }
        if (bottleneck > tr_[i]) bottleneck = tr_[i];
        for (i = head_[mid];; i = head_[a]) {
            a = parent_[i];
            if (a == kTerminal) break;
            if (bottleneck > rcap_[a]) bottleneck = rcap_[a];
        }
        if (bottleneck > -tr_[i]) bottleneck = -tr_[i];
        rcap_[mid ^ 1] += bottleneck;
        rcap_[mid] -= bottleneck;
        for (i = head_[mid ^ 1];; i = head_[a]) {
            a = parent_[i];
            if (a == kTerminal) break;
            rcap_[a] += bottleneck;
            rcap_[a ^ 1] -= bottleneck;
            if (rcap_[a ^ 1] == 0.0) orphan_front(i);
        }
        tr_[i] -= bottleneck;
        if (tr_[i] == 0.0) orphan_front(i);
        for (i = head_[mid];; i = head_[a]) {
            a = parent_[i];
            if (a == kTerminal) break;
            rcap_[a ^ 1] += bottleneck;
            rcap_[a] -= bottleneck;
            if (rcap_[a] == 0.0) orphan_front(i);
        }
        tr_[i] += bottleneck;
        if (tr_[i] == 0.0) orphan_front(i);
    }
    // process_source_orphan / process_sink_orphan (maxflow.ti:326-459)
    template <bool kSink>
    void process_orphan(int32_t i) {
        int32_t a0_min = kNone;
        int d_min = kInfD;
        for (int32_t a0 = first_[i]; a0 != kNone; a0 = anext_[a0]) {
            if ((kSink ? rcap_[a0] : rcap_[a0 ^ 1]) == 0.0) continue;
            int32_t j = head_[a0];
            if ((bool)sink_[j] != kSink || parent_[j] == kNone) continue;
            int d = 0;
            while (true) {                                // origin of j
                if (ts_[j] == time_) {
                    d += dist_[j];
                    break;
                }
                const int32_t a = parent_[j];
                d++;
                if (a == kTerminal) {
                    ts_[j] = time_;
                    dist_[j] = 1;
                    break;
                }
                if (a == kOrphan) {
                    d = kInfD;
                    break;
                }
                j = head_[a];
            }
            if (d < kInfD) {
                if (d < d_min) {
                    a0_min = a0;
                    d_min = d;
                }
                for (j = head_[a0]; ts_[j] != time_; j = head_[parent_[j]]) {
                    ts_[j] = time_;
                    dist_[j] = d--;
                }
            }
        }
        parent_[i] = a0_min;
        if (a0_min != kNone) {
            ts_[i] = time_;
            dist_[i] = d_min + 1;
            return;
        }
        for (int32_t a0 = first_[i]; a0 != kNone; a0 = anext_[a0]) {
            const int32_t j = head_[a0];
            const int32_t a = parent_[j];
            if ((bool)sink_[j] != kSink || a == kNone) continue;
            if ((kSink ? rcap_[a0] : rcap_[a0 ^ 1]) != 0.0) set_active(j);
            if (a != kTerminal && a != kOrphan && head_[a] == i) {
                parent_[j] = kOrphan;                     // set_orphan_rear
                adopt_.push_back(j);
            }
        }
    }
};

// labeling() of GCRANSAC.h:759-870 for one class: r2 = squared residuals of
// the LO model, sqt = squared truncated threshold, pairwise terms over
// `edges` when lambda > 0.  Writes seg[i] = 1 for the SINK points (inliers).
//
// The pairwise terms only join points of one grid cell, so every cell is an
// independent component of the graph, and BK on the whole graph performs,
// restricted to one component, exactly the operations BK performs on that
// component alone: the component's nodes keep their relative order in the
// active queues and the orphan list, its arcs their order in the adjacency
// lists, and the TS stamps their relative order (the checks compare stamps of
// the component's own nodes, or test "stamped in this adoption").  So each
// cell is cut on its own -- in parallel through `for_cells(ncells, fn)` --
// and a point outside any multi-point cell takes the terminal test.
// (tests/test_graphcut.py checks this against the oracle's whole-graph BK.)
struct CellScratch {
    MaxFlow g;
    std::vector<int32_t> local;
    std::vector<double> tr;                  // graphcut_clique's terminal capacities
    std::vector<double> lq, lr;              // graphcut_labeling_jobs: the cell's q and r2
    std::vector<uint32_t> ln;                //   and its nodes renumbered 0 .. k-1
};

// A two-point cell in closed form: the same unary / pairwise arithmetic as
// add_term1 / add_term2 (energy.h:204-245, graph.h:405-452), then BK's
// result without running it.  With at most one s-t path (s -> i -> j -> t
// needs tr_i > 0 > tr_j) BK augments it once by f = min(arc cap, tr_i, -tr_j)
// and stops; the SINK nodes are those that still reach t in the residual
// graph: j iff -tr_j > f, i iff its arc keeps capacity (cap > f) and j is
// SINK; without a path, a node is SINK iff tr < 0, or tr == 0 and its arc
// leads to a node with tr < 0.  (Comparisons replace BK's subtractions: for
// floats, x - f > 0 exactly when x > f.)  Returns false (BK decides) when a
// term is not a number.  tests/cpp/gc_pair.cpp checks it against
// graphcut_cell_bk.
inline bool graphcut_pair(const double* q, const double* r2, double sqt, double lambda, const uint32_t* nodes,
                          uint8_t* seg) {
    const double oml = 1.0 - lambda;
    double tr[2] = {0.0, 0.0};
    // Graph::add_tweights on a node whose tr may be nonzero
    auto tweights = [&](int i, double cs, double ck) {
        const double delta = tr[i];
        if (delta > 0) cs += delta;
        else ck -= delta;
        tr[i] = cs - ck;
    };
    for (int a = 0; a < 2; ++a) {
        const uint32_t i = nodes[a];
        const double energy = 1.0 - q[i];
        if (r2[i] <= sqt) tweights(a, 0.0, oml * energy);      // add_term1(a, oml energy, 0)
        else tweights(a, oml * (1.0 - energy), 0.0);           // add_term1(a, 0, oml (1 - energy))
    }
    // add_term2(0, 1, A = e00 lambda, B = C = lambda, D = 0)
    const double e00 = 0.5 * (q[nodes[0]] + q[nodes[1]]);
    double A = e00 * lambda, B = lambda, C = lambda, D = 0.0 * lambda;
    tweights(0, D, A);
    B -= A;
    C -= D;
    double c01, c10;                                           // arc 0 -> 1, arc 1 -> 0
    if (B < 0) {
        tweights(0, 0, B);
        tweights(1, 0, -B);
        c01 = 0;
        c10 = B + C;
    } else if (C < 0) {
        tweights(0, 0, -C);
        tweights(1, 0, C);
        c01 = B + C;
        c10 = 0;
    } else {
        c01 = B;
        c10 = C;
    }
    if (tr[0] != tr[0] || tr[1] != tr[1] || c01 != c01 || c10 != c10) return false;
    bool sink[2];
    auto path = [&](int i, int j, double cap) {                // s -> i -> j -> t
        double f = cap;
        if (f > tr[i]) f = tr[i];
        if (f > -tr[j]) f = -tr[j];
        sink[j] = -tr[j] > f;
        sink[i] = cap > f && sink[j];
    };
    if (tr[0] > 0 && tr[1] < 0 && c01 != 0.0) {
        path(0, 1, c01);
    } else if (tr[1] > 0 && tr[0] < 0 && c10 != 0.0) {
        path(1, 0, c10);
    } else {
        sink[0] = tr[0] < 0 || (tr[0] == 0 && c01 != 0.0 && tr[1] < 0);
        sink[1] = tr[1] < 0 || (tr[1] == 0 && c10 != 0.0 && tr[0] < 0);
    }
    seg[nodes[0]] = sink[0] ? 1 : 0;
    seg[nodes[1]] = sink[1] ? 1 : 0;
    return true;
}

inline void graphcut_cell_bk(const double* q, const double* r2, double sqt, double lambda, const uint32_t* nodes,
                             uint32_t k, CellScratch& cs, uint8_t* seg) {
    const double oml = 1.0 - lambda;
    MaxFlow& g = cs.g;
    g.reset(k, (size_t)k * (k - 1) / 2);
    for (uint32_t a = 0; a < k; ++a) {
        const uint32_t i = nodes[a];
        const double energy = 1.0 - q[i];
        if (r2[i] <= sqt) g.add_term1((int32_t)a, oml * energy, 0.0);
        else g.add_term1((int32_t)a, 0.0, oml * (1.0 - energy));
    }
    const double e11 = 0;
    for (uint32_t a = 0; a < k; ++a)
        for (uint32_t b = a + 1; b < k; ++b) {
            const double e00 = 0.5 * (q[nodes[a]] + q[nodes[b]]);
            g.add_term2((int32_t)a, (int32_t)b, e00 * lambda, lambda, lambda, e11 * lambda);
        }
    g.maxflow();
    for (uint32_t a = 0; a < k; ++a) seg[nodes[a]] = g.is_sink((int32_t)a) ? 1 : 0;
}

// A cell in which at most one node can push flow, decided without running
// BK.  The terms are those graphcut_cell_bk builds (add_term1 per node, then
// add_term2 for every pair a < b in cell order).  With 0 < lambda < inf and
// q in [0, 1], A_ab = (0.5 (q_a + q_b)) lambda <= lambda, so every pair
// takes add_term2's last branch: node a's terminal capacity tr_a is its unary
// term minus A_ab for every later b, in order (add_tweights' two cases round
// alike: 0 - fl(A - t) == fl(t - A)), and the arcs are a -> b with
// fl(lambda - A_ab), b -> a with lambda.
// - No tr positive and none zero: BK never augments; every node is in the
//   sink tree from the start.
// - Exactly one tr_v > 0, every other tr < 0, and tr_v below every -tr_j and
//   every arc capacity out of v: BK's first active node is v (which meets a
//   sink node j) or a sink node j (which meets v), so the first augmentation
//   is s -> v -> j -> t and carries exactly tr_v.  That leaves tr_v == 0
//   (x - x), tr_j < 0 and the arc v -> j with capacity > 0 (a difference of
//   unequal floats is never zero), so no source node remains and v rejoins
//   the sink tree over a residual arc (the node that met it is processed
//   again; or, when v itself was processed, the next active sink node).
// Either way every node is SINK.  Anything else (a NaN, a zero, more
// sources, an arc or sink capacity at or below tr_v) returns false and BK
// decides.  With the default lambda (0.975) nearly every cell qualifies: an
// outlier's unary term (1 - lambda) is outweighed by its first pairwise term,
// so only a cell's last node can be a source.  tests/cpp/gc_clique.cpp
// checks it against graphcut_cell_bk.
inline bool graphcut_clique(const double* q, const double* r2, double sqt, double lambda, const uint32_t* nodes,
                            uint32_t k, CellScratch& cs, uint8_t* seg) {
    if (!(lambda > 0.0) || !(lambda <= 1.7976931348623157e308)) return false;
    const double oml = 1.0 - lambda;
    if (cs.tr.size() < 2 * (size_t)k + 4) cs.tr.resize(2 * (size_t)k + 4);
    double* tr = cs.tr.data();
    double* ql = tr + k + 4;                                 // the cell's q, contiguous
    for (uint32_t a = 0; a < k; ++a) {
        const uint32_t i = nodes[a];
        const double qi = q[i];
        if (!(qi >= 0.0 && qi <= 1.0)) return false;
        ql[a] = qi;
        const double energy = 1.0 - qi;
        // add_term1 on a fresh node: tr = 0 - ck or cs - 0
        tr[a] = (r2[i] <= sqt) ? 0.0 - oml * energy : oml * (1.0 - energy) - 0.0;
    }
    // each row's subtractions in order (b ascending); four rows side by side
    // so that their dependent chains overlap
    auto A = [&](double qa, double qb) {
        const double e00 = 0.5 * (qa + qb);
        return e00 * lambda;
    };
    // (lane-wise vector arithmetic: every lane rounds as the scalar code)
    typedef double v4 __attribute__((vector_size(32)));
    uint32_t a = 0;
    for (; a + 4 < k; a += 4) {
        const double q0 = ql[a], q1 = ql[a + 1], q2 = ql[a + 2];
        double t0 = tr[a], t1 = tr[a + 1], t2 = tr[a + 2];
        t0 = t0 - A(q0, q1);
        t0 = t0 - A(q0, q2);
        t1 = t1 - A(q1, q2);
        t0 = t0 - A(q0, ql[a + 3]);
        t1 = t1 - A(q1, ql[a + 3]);
        t2 = t2 - A(q2, ql[a + 3]);
        const v4 q4 = {q0, q1, q2, ql[a + 3]};
        v4 t4 = {t0, t1, t2, tr[a + 3]};
        for (uint32_t b = a + 4; b < k; ++b) {
            const v4 e00 = 0.5 * (q4 + ql[b]);
            t4 = t4 - e00 * lambda;
        }
        tr[a] = t4[0];
        tr[a + 1] = t4[1];
        tr[a + 2] = t4[2];
        tr[a + 3] = t4[3];
    }
    for (; a + 1 < k; ++a) {
        const double qa = ql[a];
        double t = tr[a];
        for (uint32_t b = a + 1; b < k; ++b) t = t - A(qa, ql[b]);
        tr[a] = t;
    }
    uint32_t npos = 0, v = 0;
    for (uint32_t a = 0; a < k; ++a) {
        if (!(tr[a] < 0.0)) {
            if (!(tr[a] > 0.0)) return false;               // zero or NaN
            ++npos;
            v = a;
        }
    }
    if (npos > 1) return false;
    if (npos == 1) {
        const double f = tr[v];
        if (!(f < lambda)) return false;                     // arcs v -> j, j < v
        const double qv = ql[v];
        for (uint32_t j = 0; j < k; ++j) {
            if (j == v) continue;
            if (!(f < -tr[j])) return false;
            if (j > v && !(f < lambda - A(qv, ql[j]))) return false;   // arc v -> j
        }
    }
    for (uint32_t a = 0; a < k; ++a) seg[nodes[a]] = 1;
    return true;
}

// GCR_GC_CLIQUE=0 (read once): every cell of three or more points through BK
inline bool gc_clique_on() {
    static const bool on = [] {
        const char* e = getenv("GCR_GC_CLIQUE");
        return !(e && e[0] == '0');
    }();
    return on;
}

inline void graphcut_cell(const double* q, const double* r2, double sqt, double lambda, const uint32_t* nodes,
                          uint32_t k, CellScratch& cs, uint8_t* seg) {
    if (k == 2 && graphcut_pair(q, r2, sqt, lambda, nodes, seg)) return;
    if (k > 2 && gc_clique_on() && graphcut_clique(q, r2, sqt, lambda, nodes, k, cs, seg)) return;
    graphcut_cell_bk(q, r2, sqt, lambda, nodes, k, cs, seg);
}

// q_i = std::clamp(r2_i / sqt, 0, 1), NaN passing through, as selects
inline double gc_q(double r2, double sqt) {
    const double v = r2 / sqt;
    const double lo = v < 0.0 ? 0.0 : v;
    return 1.0 < lo ? 1.0 : lo;
}
// the terminal test (a node without pairwise terms): SINK iff its terminal
// residual capacity is < 0
inline uint8_t gc_terminal(double r2, double q, double sqt, double oml) {
    const double energy = 1.0 - q;
    const double tin = 0.0 - oml * energy, tout = oml * (1.0 - energy) - 0.0;
    const double tr = (r2 <= sqt) ? tin : tout;
    return tr < 0 ? 1 : 0;
}

// One labeling over the schedule of gc_schedule, in two passes of
// concurrent jobs (for_jobs(njobs, fn) calls fn(j, scratch) for every job
// and returns when all are done).  Cell jobs cut each cell on local copies
// of its q and r2 (nodes renumbered 0 .. k-1, the cell order kept) and
// write its labels to cseg[off[c] .. off[c+1]) -- contiguous per cell, so
// concurrent jobs do not share cache lines the way writes to the cells'
// scattered points would.  Range jobs then assemble seg over contiguous point
// ranges: a cell point's label from cseg, a single point's terminal test.
// cseg holds nodes.size() bytes, seg n.
template <class ForJobs>
inline void graphcut_labeling_jobs(const double* r2, double sqt, double lambda, const NeighbourEdges& g,
                                   uint8_t* cseg, uint8_t* seg, ForJobs&& for_jobs) {
    const double oml = 1.0 - lambda;
    for_jobs(g.jobs.size(), [&](size_t j, CellScratch& cs) {
        const NeighbourEdges::Job jb = g.jobs[j];
        for (uint32_t t = jb.b; t < jb.e; ++t) {
            const uint32_t c = g.order[t];
            const uint32_t* nodes = g.nodes.data() + g.off[c];
            const uint32_t k = g.off[c + 1] - g.off[c];
            if (cs.lq.size() < k) {
                cs.lq.resize(k);
                cs.lr.resize(k);
                cs.ln.resize(k);
            }
            for (uint32_t a = 0; a < k; ++a) {
                const double v = r2[nodes[a]];
                cs.lr[a] = v;
                cs.lq[a] = gc_q(v, sqt);
                cs.ln[a] = a;
            }
            graphcut_cell(cs.lq.data(), cs.lr.data(), sqt, lambda, cs.ln.data(), k, cs, cseg + g.off[c]);
        }
    });
    for_jobs(g.ranges.size(), [&](size_t j, CellScratch&) {
        const NeighbourEdges::Job jb = g.ranges[j];
        for (uint32_t i = jb.b; i < jb.e; ++i) {
            const uint32_t p = g.pos_of[i];
            seg[i] = p != NeighbourEdges::kNoPos ? cseg[p] : gc_terminal(r2[i], gc_q(r2[i], sqt), sqt, oml);
        }
    });
}

// serial driver (tests, small problems): the terminal test for every point,
// then every multi-point cell (lambda > 0)
inline void graphcut_labeling(const double* r2, size_t n, double sqt, double lambda, const NeighbourEdges& edges,
                              std::vector<double>& q, std::vector<uint8_t>& seg) {
    const double oml = 1.0 - lambda;
    q.resize(n);
    seg.resize(n);
    for (size_t i = 0; i < n; ++i) {
        q[i] = gc_q(r2[i], sqt);
        seg[i] = gc_terminal(r2[i], q[i], sqt, oml);
    }
    if (!(lambda > 0) || edges.off.size() < 2) return;
    CellScratch cs;
    for (size_t c = 0; c + 1 < edges.off.size(); ++c)
        graphcut_cell(q.data(), r2, sqt, lambda, edges.nodes.data() + edges.off[c], edges.off[c + 1] - edges.off[c], cs,
                      seg.data());
}

}  // namespace gcr
