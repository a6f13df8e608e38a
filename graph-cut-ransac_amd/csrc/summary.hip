// summary.hip -- device-side summary of a scored block of slots (summary.h):
// the prefix-maximum chain of finished MSAC scores, iteration / hypothesis
// prefix sums, the last live hypothesis and the iteration-target locate.
//
// A block holds npos = nslots * per positions (per = hypotheses per slot: 1,
// or 3 for the 7-point fundamental matrix); position p = slot * per + q.
// inc[p] as the generators write it: 1..101 = attempts of the slot's first
// success, 102 = every attempt failed (q = 0); 0 = an extra model of the slot,
// 255 = absent (q > 0).  Live hypotheses are inc <= 101, a slot adds its
// inc[slot * per] iterations (GCRANSAC.h:293-339).  Scores are at position p,
// or at the live rank of p for compacted launches (hmap != null, k_compact).
//
// Three launches per summary, all bandwidth-trivial (a few bytes per
// position): A per part of ~1024 positions its iteration / live totals and
// last live position (one wave per part); B per part its local prefix-maximum
// chain from the bar (one wave per part, global offsets from A's totals); C
// one workgroup: the parts' maxima scanned, each part's chain filtered against
// the maximum before it, the survivors gathered into the summary (and the
// optional locate of an iteration target).
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "summary.h"

namespace gcr {
namespace {

constexpr int kPartCap = kCandCap;      // chain members kept per part

struct SumPart {
    uint32_t contrib;                   // sum of inc contributions of the part
    uint32_t live;                      // live hypotheses of the part
    int32_t last_pos;                   // last live position of the part (-1: none)
    uint32_t last_it;                   // part-relative iterations before last_pos's slot
    uint32_t ncand;                     // B: chain members kept
    uint32_t over;                      // B: chain truncated at kPartCap
    double maxv;                        // B: largest eligible value of the part (-1: none)
    uint32_t nflag;                     // B: flagged members of the part (exact.h)
    uint32_t pad;
};

struct PartCand {
    uint32_t pos;
    uint32_t it_before;                 // block-relative
    uint32_t hyps_before;               // block-relative
    uint32_t pad;
    double val;                         // its score (+inf: flagged, always a member)
    double rb;                          // the part's running maximum including it
};

// Wave scans by DPP (row shifts, then the two row broadcasts): the lanes
// exchange through the VALU's data-parallel moves instead of ds_bpermute
// round trips through the LDS (a scan step ~10 cycles instead of ~100; the
// one-wave summary k_sum_one runs three scans per 64 positions).  Integer sums
// and maxima: the results do not depend on the combination order.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_f64(double old, double v) {
    const uint64_t o = __builtin_bit_cast(uint64_t, old), u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = dpp_u32<CTRL, ROWS>((uint32_t)o, (uint32_t)u);
    const uint32_t hi = dpp_u32<CTRL, ROWS>((uint32_t)(o >> 32), (uint32_t)(u >> 32));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v, int) {
    v += dpp_u32<0x111, 0xf>(0u, v);     // row_shr:1
    v += dpp_u32<0x112, 0xf>(0u, v);     // row_shr:2
    v += dpp_u32<0x114, 0xf>(0u, v);     // row_shr:4
    v += dpp_u32<0x118, 0xf>(0u, v);     // row_shr:8
    v += dpp_u32<0x142, 0xa>(0u, v);     // row_bcast:15 into rows 1, 3
    v += dpp_u32<0x143, 0xc>(0u, v);     // row_bcast:31 into rows 2, 3
    return v;
}
__device__ __forceinline__ double dmax(double v, double o) { return v < o ? o : v; }
__device__ __forceinline__ double wave_incl_max(double v, int) {
    constexpr double ninf = -__builtin_huge_val();
    v = dmax(v, dpp_f64<0x111, 0xf>(ninf, v));
    v = dmax(v, dpp_f64<0x112, 0xf>(ninf, v));
    v = dmax(v, dpp_f64<0x114, 0xf>(ninf, v));
    v = dmax(v, dpp_f64<0x118, 0xf>(ninf, v));
    v = dmax(v, dpp_f64<0x142, 0xa>(ninf, v));
    v = dmax(v, dpp_f64<0x143, 0xc>(ninf, v));
    return v;
}
// the previous lane's value (wave_shr:1); lane 0 gets `old`
__device__ __forceinline__ double prev_lane_f64(double old, double v) { return dpp_f64<0x138, 0xf>(old, v); }
// a lane's value, wave-uniform index
__device__ __forceinline__ uint32_t lane_u32(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ double lane_f64(double v, int l) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    return __builtin_bit_cast(double, ((uint64_t)lane_u32((uint32_t)(u >> 32), l) << 32) | lane_u32((uint32_t)u, l));
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    return v;
}

__device__ __forceinline__ uint32_t contrib_of(uint32_t in) { return in <= 102 ? in : 0u; }

// MSACScoringFunction::getScore finish (MSAC_scoring_function.hpp:108-127),
// the same operations as the host's RunnerT::finish and k_select
__device__ __forceinline__ double finish_at(const ScoreOut& sc, uint32_t j, int K, uint32_t m0, uint32_t m1,
                                            double Tm0, double Tm1) {
    double sum = sc.tot[j];
    for (int c = 0; c < K; ++c) {
        const uint32_t nc = c == 0 ? sc.n0[j] : sc.n1[j];
        if (nc < (c == 0 ? m0 : m1)) return 0.0;
        const double v = c == 0 ? sc.v0[j] : sc.v1[j];
        const double msac = v / (c == 0 ? Tm0 : Tm1) + static_cast<double>(nc);
        sum -= v;
        sum += msac;
    }
    return sum;
}

struct SumArgs {
    const uint8_t* inc;
    const void* models;                 // RectModel (solvers 0-2) or GeoModel (3, 4), per position
    ScoreOut sc;
    const uint32_t* hmap;               // non-null: scores at the live rank (compacted launch)
    uint32_t npos, per, pp;             // positions, hypotheses per slot, positions per part
    uint32_t nparts;
    int solver;
    uint32_t m0, m1;
    double Tm0, Tm1;
    double bar;                         // chain members must beat it
    double tol;                         // ... or come within tol of the running maximum
                                        // (a near tie, compared in glibc by the host:
                                        // exact.h ScoreBound; 0 for the correspondences)
    uint32_t from_pos;                  // positions below are not eligible (continuation)
    uint64_t target;                    // locate: iteration target (block-relative); ~0 = none
    uint32_t cap;                       // members kept per part and per summary (<= kCandCap)
    SumPart* parts;
    PartCand* pcand;                    // nparts * kPartCap
    BlockSummary* out;
};

// ---- A: per-part totals and last live position
__global__ __launch_bounds__(64) void k_sum_parts(SumArgs a) {
    const int lane = threadIdx.x;
    const uint32_t base = blockIdx.x * a.pp, end = min(a.npos, base + a.pp);
    uint32_t contrib = 0, live = 0, last_it = 0;
    int32_t last = -1;
    for (uint32_t o = 0; base + o < end; o += 64) {
        const uint32_t p = base + o + lane;
        const uint32_t in = p < end ? a.inc[p] : 255u;
        const uint32_t c = contrib_of(in);
        const bool l = in <= 101;
        const uint32_t cs = wave_incl_sum(c, lane);
        const uint64_t bl = __ballot(l);
        if (bl) {
            const int hl = 63 - __builtin_clzll(bl);
            // iterations before that position's slot: the exclusive prefix at
            // the position minus its slot's own inc when q > 0
            const uint32_t q = (base + o + hl) % a.per;
            const uint32_t excl = lane_u32(cs - c, hl);
            const uint32_t own = q > 0 ? (uint32_t)contrib_of(a.inc[base + o + hl - q]) : 0u;
            last = (int32_t)(base + o + hl);
            last_it = contrib + excl - own;
        }
        contrib += lane_u32(cs, 63);
        live += (uint32_t)__builtin_popcountll(bl);
    }
    if (lane == 0) {
        SumPart& s = a.parts[blockIdx.x];
        s.contrib = contrib;
        s.live = live;
        s.last_pos = last;
        s.last_it = last_it;
    }
}

// ---- B: per-part prefix-maximum chain from the bar (global offsets from A)
template <class M>
__global__ __launch_bounds__(64) void k_sum_chain(SumArgs a) {
    const int lane = threadIdx.x;
    const uint32_t k = blockIdx.x;
    uint32_t coff = 0, loff = 0;
    for (uint32_t i = lane; i < k; i += 64) {
        coff += a.parts[i].contrib;
        loff += a.parts[i].live;
    }
    coff = wave_sum(coff);
    loff = wave_sum(loff);
    const uint32_t base = k * a.pp, end = min(a.npos, base + a.pp);
    const int K = a.solver == 2 ? 2 : 1;
    const M* models = static_cast<const M*>(a.models);
    double run = a.bar, pmax = -1.0;
    uint32_t nc = 0, over = 0, nflag = 0;
    for (uint32_t o = 0; base + o < end; o += 64) {
        const uint32_t p = base + o + lane;
        const uint32_t in = p < end ? a.inc[p] : 255u;
        const uint32_t c = contrib_of(in);
        const bool l = in <= 101;
        const uint32_t cs = wave_incl_sum(c, lane), ls = wave_incl_sum(l ? 1u : 0u, lane);
        const uint32_t hb = loff + ls - (l ? 1u : 0u);          // live hypotheses before p
        double val = -1.0;
        bool flagged = false;
        if (l && p >= a.from_pos) {
            const uint32_t j = a.hmap != nullptr ? hb : p;
            val = finish_at(a.sc, j, K, a.m0, a.m1, a.Tm0, a.Tm1);
            if constexpr (std::is_same<M, RectModel>::value)
                if (a.solver == 2 && !valid_model_sift22(models[p])) val = -2.0;
            // flagged decisions: its exact score is the host's to find (a
            // member whatever its twin score, never the running maximum)
            if (val > -2.0 && a.sc.fl != nullptr && a.sc.fl[j] != 0) {
                flagged = true;
                val = -1.0;
            }
        }
        const double im = wave_incl_max(val, lane);
        const double before = prev_lane_f64(run, im);
        const double bar = lane == 0 ? run : (run < before ? before : run);
        const bool cand = (val >= 0.0 && val > bar - a.tol) || flagged;
        const uint64_t bc = __ballot(cand);
        if (cand) {
            const uint32_t r = nc + (uint32_t)__builtin_popcountll(bc & ((1ull << lane) - 1ull));
            if (r < a.cap) {
                const uint32_t q = p % a.per;
                const uint32_t own = q > 0 ? contrib_of(a.inc[p - q]) : 0u;
                PartCand& pc = a.pcand[(size_t)k * kPartCap + r];
                pc.pos = p;
                pc.it_before = coff + cs - c - own;
                pc.hyps_before = hb;
                pc.val = flagged ? __builtin_huge_val() : val;
                pc.rb = (flagged || !(val > bar)) ? bar : val;      // the running maximum after it
            }
        }
        nflag += (uint32_t)__builtin_popcountll(__ballot(flagged));
        const uint32_t add = (uint32_t)__builtin_popcountll(bc);
        if (nc + add > a.cap) over = 1;
        nc = min(nc + add, a.cap);
        const double wm = lane_f64(im, 63);
        run = run < wm ? wm : run;
        pmax = pmax < wm ? wm : pmax;
        coff += lane_u32(cs, 63);
        loff += lane_u32(ls, 63);
    }
    if (lane == 0) {
        SumPart& s = a.parts[k];
        s.ncand = nc;
        s.over = over;
        s.maxv = pmax;
        s.nflag = nflag;
    }
}

template <class M>
__device__ void fill_hyp(const SumArgs& a, uint32_t p, uint64_t it_before, uint64_t hyps_before, SumHyp& h) {
    const uint32_t q = p % a.per;
    const uint32_t j = a.hmap != nullptr ? (uint32_t)hyps_before : p;
    h.pos = p;
    h.inc = a.inc[p - q];
    h.it_before = it_before;
    h.hyps_before = hyps_before;
    h.n0 = a.sc.n0[j];
    h.n1 = a.sc.n1[j];
    h.fl = a.sc.fl != nullptr ? a.sc.fl[j] : 0u;
    h.lfl = a.sc.lfl != nullptr ? a.sc.lfl[j] : 0u;
    h.v0 = a.sc.v0[j];
    h.v1 = a.sc.v1[j];
    h.tot = a.sc.tot[j];
    const double* src = reinterpret_cast<const double*>(static_cast<const M*>(a.models) + p);
    for (int i = 0; i < 9; ++i) h.m[i] = i < (int)(sizeof(M) / sizeof(double)) ? src[i] : 0.0;
}

constexpr int kSumFinalThreads = 1024;

// ---- C: the block's chain, totals, last live hypothesis and locate
template <class M>
__global__ __launch_bounds__(kSumFinalThreads) void k_sum_final(SumArgs a) {
    __shared__ uint32_t s_coff[kSumFinalThreads], s_loff[kSumFinalThreads];
    __shared__ double s_mx[kSumFinalThreads];
    __shared__ uint32_t s_g[kSumFinalThreads];
    __shared__ uint32_t s_fail, s_k0;
    __shared__ int s_lastpart;
    const int t = threadIdx.x;
    const uint32_t np = a.nparts;            // <= kSumFinalThreads (launch checks)
    const bool mine = (uint32_t)t < np;
    const bool locate = a.target != ~0ull;
    SumPart sp{0, 0, -1, 0, 0, 0, -1.0, 0, 0};
    if (mine) sp = a.parts[t];
    if (locate) { sp.ncand = 0; sp.over = 0; sp.maxv = -1.0; sp.nflag = 0; }   // chain fields: not this launch's
    s_coff[t] = sp.contrib;
    s_loff[t] = sp.live;
    s_mx[t] = sp.maxv;
    if (t == 0) { s_fail = 0xffffffffu; s_k0 = 0xffffffffu; s_lastpart = -1; }
    __syncthreads();
    // inclusive scans (Hillis-Steele): sums of contrib / live, max of maxv
    for (int d = 1; d < kSumFinalThreads; d <<= 1) {
        const uint32_t c = t >= d ? s_coff[t - d] : 0u, l = t >= d ? s_loff[t - d] : 0u;
        const double m = t >= d ? s_mx[t - d] : -1.0;
        __syncthreads();
        s_coff[t] += c;
        s_loff[t] += l;
        if (s_mx[t] < m) s_mx[t] = m;
        __syncthreads();
    }
    const uint32_t coff = s_coff[t] - sp.contrib;             // exclusive prefixes
    const double mprev = t == 0 ? -1.0 : s_mx[t - 1];
    const double mb = a.bar < mprev ? mprev : a.bar;         // the maximum before part t
    // this part's members that beat it (flagged ones always); a truncated
    // chain whose part maximum beats it, or that holds flagged members, may
    // have lost members
    uint32_t g = 0;
    if (mine) {
        for (uint32_t i = 0; i < sp.ncand; ++i) g += a.pcand[(size_t)t * kPartCap + i].val > mb - a.tol ? 1u : 0u;
        if (sp.over && (sp.maxv > mb - a.tol || sp.nflag > 0)) atomicMin(&s_fail, (uint32_t)t);
        if (sp.live > 0) atomicMax(&s_lastpart, t);
    }
    if (locate && mine && (uint64_t)coff < a.target && (uint64_t)coff + sp.contrib >= a.target)
        s_k0 = (uint32_t)t;                                  // the one part where the prefix crosses
    __syncthreads();
    const uint32_t kf = s_fail;
    const uint32_t gk = (mine && (uint32_t)t <= kf) ? g : 0u;
    s_g[t] = gk;
    __syncthreads();
    for (int d = 1; d < kSumFinalThreads; d <<= 1) {
        const uint32_t v = t >= d ? s_g[t - d] : 0u;
        __syncthreads();
        s_g[t] += v;
        __syncthreads();
    }
    const uint32_t gbase = s_g[t] - gk;
    const uint32_t total = s_g[kSumFinalThreads - 1];
    BlockSummary* out = a.out;
    if (!locate) {
        if (gk > 0) {
            uint32_t r = gbase;
            for (uint32_t i = 0; i < sp.ncand && r < a.cap; ++i) {
                const PartCand& pc = a.pcand[(size_t)t * kPartCap + i];
                if (!(pc.val > mb - a.tol)) continue;
                fill_hyp<M>(a, pc.pos, pc.it_before, pc.hyps_before, out->cand[r]);
                if (r + 1 == min(total, a.cap)) {                        // the last member emitted
                    out->resume_pos = pc.pos + 1;
                    out->resume_bar = mb < pc.rb ? pc.rb : mb;
                }
                ++r;
            }
        }
        // nothing emitted before the first lossy part: resume at its start
        if (mine && (uint32_t)t == kf && total == 0) {
            out->resume_pos = (uint32_t)t * a.pp;
            out->resume_bar = mb;
        }
    }
    if (t == kSumFinalThreads - 1) {
        out->inc_total = s_coff[kSumFinalThreads - 1];
        out->hyps_total = s_loff[kSumFinalThreads - 1];
        out->ncand = locate ? 0u : min(total, a.cap);
        out->overflow = (!locate && (kf != 0xffffffffu || total > a.cap)) ? 1u : 0u;
    }
    const int lp = s_lastpart;
    auto block_last = [&]() {
        out->has_last = lp >= 0 ? 1u : 0u;
        if (lp >= 0) {
            const SumPart s = a.parts[lp];
            fill_hyp<M>(a, (uint32_t)s.last_pos, s_coff[lp] - s.contrib + s.last_it, s_loff[lp] - 1u, out->last);
        }
    };
    if (!locate) {
        if (t == 0) {
            out->stop_found = 0;
            block_last();
        }
        return;
    }
    // ---- locate: the loop stops before the first slot whose iterations-before
    // (exclusive prefix of inc) reach the target
    if (a.target == 0) {                                     // before slot 0
        if (t == 0) {
            out->stop_found = 1;
            out->stop_slot = 0;
            out->stop_it_before = 0;
            out->stop_hyps_before = 0;
            out->has_last = 0;
        }
        return;
    }
    const uint32_t k0 = s_k0;
    if (k0 == 0xffffffffu) {                                 // the block stays below it
        if (t == 0) {
            out->stop_found = 0;
            block_last();
        }
        return;
    }
    // wave 0 walks part k0 (its prefix crosses the target inside it, or its
    // last slot reaches it and the stop is the next part's first slot)
    if (t >= 64) return;
    const int lane = t;
    const uint32_t base = k0 * a.pp, end = min(a.npos, base + a.pp);
    uint32_t run = s_coff[k0] - a.parts[k0].contrib;
    uint32_t lrun = s_loff[k0] - a.parts[k0].live;
    int32_t lastp = -1;
    uint32_t last_it = 0, last_hb = 0;
    uint32_t stop_p = 0xffffffffu, stop_it = 0, stop_hb = 0;
    for (uint32_t o = 0; base + o < end && stop_p == 0xffffffffu; o += 64) {
        const uint32_t p = base + o + lane;
        const uint32_t in = p < end ? a.inc[p] : 255u;
        const uint32_t c = contrib_of(in);
        const bool l = in <= 101;
        const uint32_t cs = wave_incl_sum(c, lane), ls = wave_incl_sum(l ? 1u : 0u, lane);
        const uint32_t excl = run + cs - c;
        const uint32_t lexcl = lrun + ls - (l ? 1u : 0u);
        const bool start = p < end && (p % a.per) == 0;
        const uint64_t hit = __ballot(start && (uint64_t)excl >= a.target);
        const uint32_t lim = hit ? (uint32_t)__builtin_ctzll(hit) : 64u;   // positions before the stop
        const uint64_t bl = __ballot(l) & (lim >= 64u ? ~0ull : ((1ull << lim) - 1ull));
        if (bl) {
            const int hl = 63 - __builtin_clzll(bl);
            const uint32_t q = (base + o + (uint32_t)hl) % a.per;
            const uint32_t own = q > 0 ? contrib_of(a.inc[base + o + hl - q]) : 0u;
            lastp = (int32_t)(base + o + (uint32_t)hl);
            last_it = lane_u32(excl, hl) - own;
            last_hb = lane_u32(lexcl, hl);
        }
        if (hit) {
            stop_p = base + o + lim;
            stop_it = lane_u32(excl, (int)lim);
            stop_hb = lane_u32(lexcl, (int)lim);
        }
        run += lane_u32(cs, 63);
        lrun += lane_u32(ls, 63);
    }
    if (lane == 0) {
        if (stop_p == 0xffffffffu) {
            stop_p = end;
            stop_it = run;
            stop_hb = lrun;
        }
        out->stop_found = 1;
        out->stop_slot = stop_p / a.per;
        out->stop_it_before = stop_it;
        out->stop_hyps_before = stop_hb;
        if (lastp < 0) {                                     // the last live one of an earlier part
            int32_t kk = (int32_t)k0 - 1;
            while (kk >= 0 && a.parts[kk].live == 0) --kk;
            if (kk >= 0) {
                const SumPart s = a.parts[kk];
                lastp = s.last_pos;
                last_it = s_coff[kk] - s.contrib + s.last_it;
                last_hb = s_loff[kk] - 1u;
            }
        }
        out->has_last = lastp >= 0 ? 1u : 0u;
        if (lastp >= 0) fill_hyp<M>(a, (uint32_t)lastp, last_it, last_hb, out->last);
    }
}

// ---- one-part summaries (npos <= pp: LO-sized and early adaptive chunks):
// A, B and C fused into one wave, no scratch round trip and one launch
// instead of three (the 1024-thread final pass alone cost ~25 us)
template <class M>
__global__ __launch_bounds__(64) void k_sum_one(SumArgs a) {
    const int lane = threadIdx.x;
    const uint32_t end = a.npos;
    const bool locate = a.target != ~0ull;
    const int K = a.solver == 2 ? 2 : 1;
    const M* models = static_cast<const M*>(a.models);
    BlockSummary* out = a.out;
    uint32_t coff = 0, loff = 0, nc = 0, over = 0;
    int32_t lastp = -1;
    uint32_t last_it = 0, last_hb = 0;
    uint32_t stop_p = 0xffffffffu, stop_it = 0, stop_hb = 0;
    double run = a.bar;
    for (uint32_t o = 0; o < end; o += 64) {
        const uint32_t p = o + lane;
        const uint32_t in = p < end ? a.inc[p] : 255u;
        const uint32_t c = contrib_of(in);
        const bool l = in <= 101;
        const uint32_t cs = wave_incl_sum(c, lane), ls = wave_incl_sum(l ? 1u : 0u, lane);
        const uint32_t excl = coff + cs - c;                   // iterations before p's slot (q = 0)
        const uint32_t hb = loff + ls - (l ? 1u : 0u);          // live hypotheses before p
        uint32_t lim = 64u;                                     // positions of this 64 before the stop
        if (locate) {
            if (stop_p == 0xffffffffu) {
                const bool start = p < end && (p % a.per) == 0;
                const uint64_t hit = __ballot(start && (uint64_t)excl >= a.target);
                if (hit) {
                    lim = (uint32_t)__builtin_ctzll(hit);
                    stop_p = o + lim;
                    stop_it = lane_u32(excl, (int)lim);
                    stop_hb = lane_u32(hb, (int)lim);
                }
            } else {
                lim = 0u;                                       // past the stop: totals only
            }
        }
        const uint64_t bl = __ballot(l) & (lim >= 64u ? ~0ull : ((1ull << lim) - 1ull));
        if (bl) {
            const int hl = 63 - __builtin_clzll(bl);
            const uint32_t q = (o + (uint32_t)hl) % a.per;
            const uint32_t own = q > 0 ? contrib_of(a.inc[o + hl - q]) : 0u;
            lastp = (int32_t)(o + (uint32_t)hl);
            last_it = lane_u32(excl, hl) - own;
            last_hb = lane_u32(hb, hl);
        }
        if (!locate) {
            double val = -1.0;
            bool flagged = false;
            if (l && p >= a.from_pos) {
                const uint32_t j = a.hmap != nullptr ? hb : p;
                val = finish_at(a.sc, j, K, a.m0, a.m1, a.Tm0, a.Tm1);
                if constexpr (std::is_same<M, RectModel>::value)
                    if (a.solver == 2 && !valid_model_sift22(models[p])) val = -2.0;
                // flagged decisions (exact.h): always a member, never the maximum
                if (val > -2.0 && a.sc.fl != nullptr && a.sc.fl[j] != 0) {
                    flagged = true;
                    val = -1.0;
                }
            }
            const double im = wave_incl_max(val, lane);
            const double before = prev_lane_f64(run, im);
            const double bar = lane == 0 ? run : (run < before ? before : run);
            const bool cand = (val >= 0.0 && val > bar - a.tol) || flagged;
            const uint64_t bc = __ballot(cand);
            if (cand) {
                const uint32_t r = nc + (uint32_t)__builtin_popcountll(bc & ((1ull << lane) - 1ull));
                if (r < a.cap) {
                    const uint32_t q = p % a.per;
                    const uint32_t own = q > 0 ? contrib_of(a.inc[p - q]) : 0u;
                    fill_hyp<M>(a, p, excl - own, hb, out->cand[r]);
                    if (r + 1 == a.cap) {                      // the last member a full summary holds
                        out->resume_pos = p + 1;
                        out->resume_bar = (flagged || !(val > bar)) ? bar : val;
                    }
                }
            }
            const uint32_t add = (uint32_t)__builtin_popcountll(bc);
            if (nc + add > a.cap) over = 1;
            nc = min(nc + add, a.cap);
            const double wm = lane_f64(im, 63);
            run = run < wm ? wm : run;
        }
        coff += lane_u32(cs, 63);
        loff += lane_u32(ls, 63);
    }
    if (lane != 0) return;
    if (!locate) {
        out->inc_total = coff;
        out->hyps_total = loff;
        out->ncand = nc;
        out->overflow = over;
        out->stop_found = 0;
    } else {
        out->inc_total = coff;
        out->hyps_total = loff;
        out->ncand = 0;
        out->overflow = 0;
        if (a.target == 0) {                                 // before slot 0
            out->stop_found = 1;
            out->stop_slot = 0;
            out->stop_it_before = 0;
            out->stop_hyps_before = 0;
            out->has_last = 0;
            return;
        }
        if (stop_p == 0xffffffffu && (uint64_t)coff >= a.target) {   // the last slot reaches it
            stop_p = end;
            stop_it = coff;
            stop_hb = loff;
        }
        out->stop_found = stop_p != 0xffffffffu ? 1u : 0u;
        if (stop_p != 0xffffffffu) {
            out->stop_slot = stop_p / a.per;
            out->stop_it_before = stop_it;
            out->stop_hyps_before = stop_hb;
        }
    }
    out->has_last = lastp >= 0 ? 1u : 0u;
    if (lastp >= 0) fill_hyp<M>(a, (uint32_t)lastp, last_it, last_hb, out->last);
}

}  // namespace

size_t summary_scratch_bytes(uint32_t npos, uint32_t per) {
    const uint32_t pp = per * (1024u / per);
    const size_t nparts = (npos + pp - 1) / pp;
    return nparts * (sizeof(SumPart) + kPartCap * sizeof(PartCand));
}

hipError_t launch_block_summary(int solver, const uint8_t* inc, const void* models, const ScoreOut& sc,
                                const uint32_t* hmap, uint32_t nslots, uint32_t per, const uint32_t m[2],
                                const double Tm[2], double bar, uint32_t from_pos, uint64_t target, void* scratch,
                                BlockSummary* out, hipStream_t stream, bool parts_ready, double tol) {
    SumArgs a{};
    a.inc = inc;
    a.models = models;
    a.sc = sc;
    a.hmap = hmap;
    a.npos = nslots * per;
    a.per = per;
    a.pp = per * (1024u / per);
    a.nparts = (a.npos + a.pp - 1) / a.pp;
    a.solver = solver;
    a.m0 = m[0];
    a.m1 = m[1];
    a.Tm0 = Tm[0];
    a.Tm1 = Tm[1];
    a.bar = bar;
    a.tol = tol >= 0.0 ? tol : 0.0;
    a.from_pos = from_pos;
    a.target = target;
    // GCR_SUMMARY_CAP=n (1 .. kCandCap): fewer members per summary, so that
    // tests exercise the overflow continuation; read per launch
    a.cap = kCandCap;
    if (const char* e = getenv("GCR_SUMMARY_CAP")) {
        const int v = atoi(e);
        if (v >= 1 && v <= kCandCap) a.cap = (uint32_t)v;
    }
    a.parts = static_cast<SumPart*>(scratch);
    a.pcand = reinterpret_cast<PartCand*>(static_cast<char*>(scratch) + (size_t)a.nparts * sizeof(SumPart));
    a.out = out;
    if (a.npos == 0 || a.nparts > (uint32_t)kSumFinalThreads) return hipErrorInvalidValue;
    const bool rect = solver <= 2;
    if (!rect) a.sc.fl = a.sc.lfl = nullptr;   // the correspondence scorers flag nothing (no libm in their residuals)
    // GCR_SUMMARY_ONE=0: one-part summaries through the three launches too
    // (read per launch: tests switch it)
    const char* e1 = getenv("GCR_SUMMARY_ONE");
    const bool one_on = !(e1 && e1[0] == '0');
    if (a.nparts == 1 && one_on) {
        if (rect) hipLaunchKernelGGL(k_sum_one<RectModel>, dim3(1), dim3(64), 0, stream, a);
        else hipLaunchKernelGGL(k_sum_one<GeoModel>, dim3(1), dim3(64), 0, stream, a);
        return hipGetLastError();
    }
    if (!parts_ready) hipLaunchKernelGGL(k_sum_parts, dim3(a.nparts), dim3(64), 0, stream, a);
    if (target == ~0ull) {
        if (rect) hipLaunchKernelGGL(k_sum_chain<RectModel>, dim3(a.nparts), dim3(64), 0, stream, a);
        else hipLaunchKernelGGL(k_sum_chain<GeoModel>, dim3(a.nparts), dim3(64), 0, stream, a);
    }
    if (rect) hipLaunchKernelGGL(k_sum_final<RectModel>, dim3(1), dim3(kSumFinalThreads), 0, stream, a);
    else hipLaunchKernelGGL(k_sum_final<GeoModel>, dim3(1), dim3(kSumFinalThreads), 0, stream, a);
    return hipGetLastError();
}

}  // namespace gcr
