// kernels.h -- launch interface of the gfx950 kernels (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

#include "exact.h"
#include "fund.h"
#include "geo.h"
#include "gram.h"
#include "rect.h"
#include "summary.h"

namespace gcr {

// One feature class resident in HBM, structure-of-arrays fp64.
//   scale class:       a = s,      c0 = pow(s, +-1/3)
//   orientation class: a = theta,  c0 = cos(theta), c1 = sin(theta)
struct DevClass {
    const double* x;
    const double* y;
    const double* a;
    const double* c0;
    const double* c1;
    uint32_t n;
    // max |x|, |y|, |a|, |c0| over the class (+inf if any is not finite):
    // the error bounds of the fundamental matrix's fp32 pre-band
    double amax[4];
};

// model type per estimator: rectification solvers 0-2, homography 3
template <int KIND>
struct ModelOf {
    using type = RectModel;
    static GCR_HD type def() { return default_model(); }
};
template <>
struct ModelOf<3> {
    using type = GeoModel;
    static GCR_HD type def() { return default_geo(); }
};
template <>
struct ModelOf<4> {                 // fundamental matrix: same 9-double POD
    using type = GeoModel;
    static GCR_HD type def() { return default_geo(); }
};

// solver 3 (homography): class 0 holds correspondences, x = x1, y = y1,
// a = x2, c0 = y2
// Scratch of the split small-batch scorer (launch_score_small): per model
// small_score_pairs(p) doubles (each 64-pair chunk's inlier values, compacted
// to the chunk's start) and small_score_pairs(p) / 64 chunk counts.
constexpr uint32_t kSplitModels = 256;         // models per split launch (kSmallScore)
constexpr size_t kSplitMaxPairs = 16384;       // pairs (every inlier value fits k_lo_fold's LDS)
struct SmallScratch {
    double* vals = nullptr;
    uint32_t* meta = nullptr;
    uint32_t cap_models = 0;
    uint32_t* arrive = nullptr;     // per model: k_lo_split's arrival counter (zero between launches)
    double* psum = nullptr;         // per chunk: its inlier values' sum in any order (k_lo_approx), optional
};

struct DevProblem {
    int solver;     // GCR_SOLVER_*
    DevClass cls[2];
    SmallScratch lo;
};

// Raw MSAC accumulators per hypothesis (host finishes the score exactly as
// MSACScoringFunction::getScore does, MSAC_scoring_function.hpp:108-127).
// fl (rectification scorers, optional): the hypothesis's pairs whose twin
// r^2 lies in the flag band of the MSAC threshold (exact.h) -- decisions the
// host rechecks with glibc; lfl (small scorer with ListBits, optional): the
// same for the list predicate.  Correspondence scorers leave them alone.
struct ScoreOut {
    uint32_t* n0;
    uint32_t* n1;
    double* v0;
    double* v1;
    double* tot;
    uint32_t* fl = nullptr;
    uint32_t* lfl = nullptr;
    // small scorer, optional: per model, `epoch` stored into done[m] (host
    // memory, coherent) after model m's results -- the host waits on these
    // flags instead of the stream's completion signal
    uint32_t* done = nullptr;
    uint32_t epoch = 0;
};

// Draw + validate + solve `nslots` outer-iteration slots [slot0, slot0+nslots).
// inc[i] = attempt index + 1 of the first success (1..101), 102 when all 101
// attempts failed (GCRANSAC.h:296-339).
hipError_t launch_generate(const DevProblem& p, uint64_t seed, uint64_t slot0, uint32_t nslots, uint8_t* inc,
                           RectModel* models, hipStream_t stream);

// Exact sequential MSAC accumulation of `nh` models over every feature;
// T[c] = (2.25 * thr_c) * thr_c.
// models with inc[i] > 101 (no model) produce zeros.  inc may be null.
// identity: every model has x0 = y0 = 0, s = 1 (true for all models of this
// fork: normalizePoints resets the transform), skips the normalisation ops.
hipError_t launch_score(const DevProblem& p, const double T[2], const RectModel* models, const uint8_t* inc,
                        uint32_t nh, bool identity, const ScoreOut& out, hipStream_t stream);

// One batch's verdict, layout-identical to gcr_batch_result (include/gcr.h).
struct BatchRecord {
    uint64_t models;
    uint64_t iterations;
    int64_t best_slot;
    double best_score;
    uint64_t best_inliers[2];
    RectModel best_model;
};

// First strict best of a scored batch, on the device: each slot's score is
// finished as MSACScoringFunction::getScore does (MSAC_scoring_function.hpp:
// 108-127: zero if some n_c < m_c, else v_c / T_c + n_c folded into the running
// sum), and the reference's update rule `best < score && isValidModel`
// (GCRANSAC.h:440-446) applied over the slots in order is the maximum score
// > 0 among valid models with the lowest slot index.
hipError_t launch_select(int solver, const ScoreOut& sc, const uint8_t* inc, const RectModel* models,
                         uint32_t nslots, uint64_t slot0, const uint32_t m[2], const double Tm[2], BatchRecord* out,
                         hipStream_t stream);

// ---- GPU least-squares refit (qr3.h backend) ----
// Rows of the hybrid non-minimal system for scale inliers si[ns] and
// orientation inliers oi[no]: ns scale rows then C(no, 2) pair rows (i < j,
// index order), written to column arrays A0, A1, A2, b of length `rows`.
hipError_t launch_sift_rows(const DevClass& sc, const DevClass& oc, const uint32_t* si, uint32_t ns,
                            const uint32_t* oi, uint32_t no, size_t rows, double* A0, double* A1, double* A2,
                            double* b, hipStream_t stream);
// The hybrid system's double-double Gram matrix in gram.h's order: tile t's
// kGramN entries at tiles[t * kGramN ..] (ceil(rows / kGramTile) tiles), and
// with fin.out set the matrix itself -- the tiles combined in gram.h's order
// by a second one-workgroup launch -- at fin.out[0 .. kGramN), then fin.epoch
// stored into fin.done (optional; coherent host memory for the host to wait on).
struct GramFinal {
    DD* out = nullptr;
    uint32_t* done = nullptr;
    uint32_t epoch = 0;
};
// hidx: the index lists (si[ns] then oi[no]) in pinned host memory, mapped;
// idx (ns + no) and lines (3 no) device scratch.
hipError_t launch_sift_gram(const DevClass& sc, const DevClass& oc, const uint32_t* hidx, uint32_t ns, uint32_t no,
                            size_t rows, uint32_t* idx, double* lines, DD* tiles, const GramFinal& fin,
                            hipStream_t stream);
// Block partials of sum_{i in [lo, hi)} a[i] * c[i] for the aligned blocks of
// kSumBlock (qr3.h) rows that intersect [lo, hi), each summed in row order;
// partials[0 .. nblocks) in block order.  Returns the block count via nblocks.
hipError_t launch_qr_partials(const double* a, const double* c, size_t lo, size_t hi, double* partials,
                              size_t* nblocks, hipStream_t stream);
// Device-resident qr_solve<3> (qr3.h) on the columns cols[0..2] | b = cols[3]
// of length m (4 <= m <= 256 * kSumSuper): the driver's decisions run in
// one-thread control kernels between the reductions, with the same fp64
// operations and blocked summation order as the host driver; one host
// synchronisation for x.  st: device scratch; partials: (m-1)/kSumBlock+1.
struct QRDevState {
    int red_a, red_c, red_on, pad0;                      // next reduction
    uint64_t red_lo, red_hi;
    int ew_op, ew_c, ew_e, pad1;                         // next element-wise step
    uint64_t ew_lo, ew_hi;
    double ew_p0, ew_p1;
    uint64_t m;
    int pc[3], transp[3], nonzero, ck, done, ddflag[3];
    double nu[3], nd[3], tau_k[3], thr_helper;
    double x[3];
};
struct QRCols {
    double* col[4];
};
enum { kQsInit = 0, kQsNorm, kQsTail, kQsRefl, kQsDd, kQsDd2, kQsBStart, kQsBRefl, kQsFinal };

// Fused device QR (launch_sift_refit_fused): qr3.h qr_solve<3> in 6 passes over the
// rows instead of ~25.  Every reduction of the sequential driver is still one
// blocked_sum over the same values in the same order, and every element-wise
// step the same per-element operation; a pass applies one step's element-wise
// operation and, from the values it just produced, every reduction the driver
// needs next (they do not depend on each other).  Passes: P0 column norms
// and step-0 tails; per step k: A(k) scales the Householder column and takes
// its dots with the remaining columns and b; U(k) applies the reflector to
// them and takes the norm-downdate and next-tail sums (no U(2): rows past the
// top of b are never read again).  A one-thread control kernel between passes
// runs the driver's scalar logic.
constexpr int kQrfMaxRed = 6;
struct QRFState {
    // the next pass (written by the control kernel)
    int mode;               // 0 none, 1 reductions only, 2 apply (scale / zero + dots), 3 update (+ sums)
    int ck, zero, write_ck; // Householder column; zero instead of scale; store the scaled column (slot 0)
    int nslot, nt;          // columns the pass reads (slots), of which slots 1 .. nt are updated (mode 3)
    int scol[4];            // stored column of each slot (slot 0 = the Householder column in modes 2 / 3)
    int nred, pad0;
    double den, tau;
    double tt[3];           // reflector multiplier of slots 1 .. nt
    uint64_t lo;            // element-wise range start (rows [lo, m))
    int ra[kQrfMaxRed], rc[kQrfMaxRed];
    uint64_t rlo[kQrfMaxRed];   // reduction r: blocked sum of slot ra * slot rc over [rlo, m)
    // driver state
    int pc[3], transp[3], nonzero, done, dob, pad1;
    double nu[3], nd[3], tau_k[3], thr_helper;
    double x[3];
};
enum { kQfStep = 1, kQfApply, kQfFinal };
// the hybrid refit's system (rows as launch_sift_rows) built inside P0 and
// solved by the same fused passes; x_out pinned, one synchronisation
hipError_t launch_sift_refit_fused(const DevClass& sc, const DevClass& oc, const uint32_t* si, uint32_t ns,
                                   const uint32_t* oi, uint32_t no, size_t m, double* const cols[4], QRFState* st,
                                   double* partials, double x_out[3], hipStream_t stream);
hipError_t launch_qr_device(double* const cols[4], size_t m, QRDevState* st, double* partials, double x_out[3],
                            hipStream_t stream);
// rows 0..2 of the four columns into out[c * 3 + i] (0 past m)
hipError_t launch_qr_top(const double* c0, const double* c1, const double* c2, const double* c3, size_t m,
                         double* out, hipStream_t stream);
// element-wise updates on [lo, hi): c = c / den; c = 0; c -= (tau * e) * t
hipError_t launch_qr_scale(double* c, size_t lo, size_t hi, double den, hipStream_t stream);
hipError_t launch_qr_zero(double* c, size_t lo, size_t hi, hipStream_t stream);
hipError_t launch_qr_update(double* c, const double* e, size_t lo, size_t hi, double tau, double t,
                            hipStream_t stream);

// Fused verify step (gcr_problem_verify_batches): the scorer generates its own
// hypotheses (slots slot0 .. slot0 + nslots) in a prologue -- exactly
// k_generate's lowest-successful-attempt rule -- writes inc / models / raw
// scores like the separate kernels, and each workgroup reduces its slots to
// their first strict best (WgBest); k_select_wg then reduces the workgroups.
struct WgBest {
    double score;        // finished MSAC score of the best slot (0 if none)
    int32_t slot;        // slot offset in the batch, -1 if none
    uint32_t n0, n1;     // its raw inlier counts
    uint32_t models;     // slots of the workgroup with a model (inc <= 101)
    uint64_t iterations; // sum of the workgroup's inc
};
// Batch chaining of the feature-major fused scorer (H = 16 launches): `pre`
// holds this batch's slots already generated by the previous launch (null:
// the launch's prologue generates them), `next` receives the next batch's
// (slots slot0 + nslots ...), generated by a dedicated wave while this batch
// is scored (null: none).  Same models and attempt counts as the prologue.
// `ahead`: the batch `next` belongs to, counted from this one (2 when
// consecutive batches alternate between two streams: batch b generates batch
// b + 2's slots, which the same stream scores next).
// `const` (optional, both or neither): the look-ahead wave also writes each
// generated slot's band and value constants (HypConst, kFmHypBytes per slot)
// and its half of the packed-fp32 pre-band record (RPairBand, kFmPairBytes
// per two slots), which the next launch's prologue copies instead of
// computing them.
constexpr size_t kFmHypBytes = 80, kFmPairBytes = 128;
struct GenChain {
    const uint8_t* pre_inc = nullptr;
    const RectModel* pre_models = nullptr;
    uint8_t* next_inc = nullptr;
    RectModel* next_models = nullptr;
    uint32_t ahead = 1;
    const void* pre_hyp = nullptr;
    const void* pre_pair = nullptr;
    void* next_hyp = nullptr;
    void* next_pair = nullptr;
};
// rec == nullptr: the launch leaves its workgroup records in `wg` (and its
// models in `models`) for a later launch_select_batches instead of reducing
// them right away
hipError_t launch_verify_fused(const DevProblem& p, const double T[2], uint64_t seed, uint64_t slot0,
                               uint32_t nslots, const uint32_t m[2], uint8_t* inc, RectModel* models,
                               const ScoreOut& out, WgBest* wg, size_t wg_cap, BatchRecord* rec,
                               hipEvent_t ev0, hipEvent_t ev1, hipStream_t stream, const GenChain& chain = {});
// Deferred selection of `count` consecutive fused batches in one launch (one
// workgroup per batch): batch i's workgroup records at wg + i * wg_stride,
// its models at models + i * nslots, its slots from slot0 + i * nslots, its
// record to rec[i].  Same reduction as the per-launch k_select_wg.
hipError_t launch_select_batches(const WgBest* wg, size_t wg_stride, const RectModel* models, uint64_t slot0,
                                 uint32_t nslots, uint32_t count, BatchRecord* rec, hipStream_t stream);
// true when launch_verify_fused at this batch size uses the chained kernel
bool verify_chains(uint32_t nslots);

// homography (solver 3) counterparts of launch_generate / launch_score /
// launch_mask / launch_select
// solver 3 (homography): one hypothesis per slot; solver 4 (fundamental
// matrix): kFModels hypotheses per slot (inc / models sized kFModels * nslots,
// see k_generate_f).  Score / mask / select dispatch on the same solver.
hipError_t launch_generate_geo(const DevProblem& p, uint64_t seed, uint64_t slot0, uint32_t nslots, uint8_t* inc,
                               GeoModel* models, hipStream_t stream);
// Hypotheses per workgroup of the batch scorers at a launch of nh (64, 16 or
// 4; GCR_SPLIT_H pins one for sweeps).
int split_h(uint32_t nh);
// launch_score_geo(compact = true) compacts in the scorer's prologue at nh
bool geo_scorer_scans(uint32_t nh);
// compact: inc covers all nh hypotheses and the launch compacts them itself
// (hmap / hcount written: in the scorer's prologue, or by k_compact first)
hipError_t launch_score_geo(const DevProblem& p, double T, const GeoModel* models, const uint8_t* inc, uint32_t nh,
                            const ScoreOut& out, hipStream_t stream, const uint32_t* hmap = nullptr,
                            const uint32_t* hcount = nullptr,
                            bool compact = false);
hipError_t launch_mask_geo(const DevProblem& p, const GeoModel& model, int rule, double T, double lambda,
                           uint8_t* mask, hipStream_t stream);
hipError_t launch_select_geo(int solver, const ScoreOut& sc, const uint8_t* inc, uint32_t nh, uint64_t slot0,
                             uint32_t m, double Tm, BatchRecord* out, hipStream_t stream,
                             const uint32_t* hmap = nullptr, const uint32_t* hcount = nullptr);
// deferred selection of `count` consecutive batches in one launch (one
// workgroup per batch): batch b's score arrays, inc, hmap at offset b * stride,
// its hcount at hcount + b, its slots from slot0 + b * nh / per, its record out[b]
hipError_t launch_select_geo_batches(int solver, const ScoreOut& sc, const uint8_t* inc, uint32_t nh, uint32_t stride,
                                     uint64_t slot0, uint32_t m, double Tm, uint32_t count, BatchRecord* out,
                                     hipStream_t stream, const uint32_t* hmap, const uint32_t* hcount);
// order-preserving list of live hypotheses (inc <= 101): map[0 .. *count)
// budget cut of a prefetched chunk: slots whose preceding increments reach
// `budget` get inc = 255 (no model)
hipError_t launch_truncate(uint8_t* inc, uint32_t n, uint64_t budget, hipStream_t stream);
hipError_t launch_sqres_geo(const DevProblem& p, const GeoModel& model, double* r2, hipStream_t stream);
hipError_t launch_compact(const uint8_t* inc, uint32_t n, uint32_t* map, uint32_t* count, hipStream_t stream);

// Low-latency scoring of a few models (LO trials, refits).  Split scorer
// (at most kSplitModels models, at most kSplitMaxPairs pairs, p.lo set):
// k_lo_resid evaluates one (model, feature) pair per thread over as many
// workgroups as the pairs need and compacts each 64-pair chunk's inlier
// values into p.lo; k_lo_fold (one 1024-thread workgroup per model) gathers
// them in feature order into LDS and folds them (fold_exact_chains).
// Otherwise one 1024-thread workgroup per model does both (k_lo_chain).
// Both count the decisions within the value-glibc bound of the thresholds
// (out.fl, out.lfl; exact.h).  Same raw accumulators as
// launch_score / launch_score_geo.  `models` points to RectModel (solvers
// 0-2) or GeoModel (3, 4), identity normalisation only; models with inc > 101
// (inc may be null) score zeros.  Bit arrays: per model small_score_pairs(p)
// / 64 words (class 0 at [0, pad0), class 1 after it, pad_c = n_c rounded up
// to 64).
size_t small_score_pairs(const DevProblem& p);
// Optional second per-pair predicate of the same launch (LO inlier lists):
// rule 0: r^2 <= T[cls]; rule 2: the 1-class labeling of k_mask with T[0] and
// lambda, into `bits` (pinned host memory mapped for the device).
struct ListBits {
    double T[2];
    int rule;
    double lambda;
    uint64_t* bits;
    uint64_t* mbits;         // optional: the MSAC inlier ballots too (r^2 <= the scoring threshold)
};
// hmodels (optional, rectification solvers): a host copy of the nm
// RectModels; with at most kArgModels of them the split scorer takes the
// models as a kernel argument instead of reading `models` (pinned host memory
// for small batches: a PCIe round trip at the start of every workgroup).
constexpr uint32_t kArgModels = 50;
hipError_t launch_score_small(const DevProblem& p, const double T[2], const void* models, const uint8_t* inc,
                              uint32_t nm, const ScoreOut& out, hipStream_t stream, const ListBits* lists = nullptr,
                              const void* hmodels = nullptr);
// The split scorer in parts (LO trials scored while the rest are still being
// fitted): stage 1 = the residual launch of models [mi_base, mi_base + nm)
// (`models` / `hmodels` point at the part's first model); stage 2 = the fold
// of models [0, nm_fold); stage 4 (instead of 2, p.lo.psum set) = their
// approximate scores (k_lo_approx: exact counts and flag counts, class sums
// in a tree order).  Only where score_small_splits() holds.
bool score_small_splits(const DevProblem& p, uint32_t nm_total);
hipError_t launch_score_small_part(const DevProblem& p, const double T[2], const void* models, uint32_t mi_base,
                                   uint32_t nm, int stage, uint32_t nm_fold, const ScoreOut& out, hipStream_t stream,
                                   const ListBits* lists, const void* hmodels);
// the exact fold (k_lo_fold) of models [src, src + nm) of the last stage-1
// launch into slots [slot, slot + nm) of `out`
hipError_t launch_lo_fold_slots(const DevProblem& p, uint32_t src, uint32_t nm, uint32_t slot, const ScoreOut& out,
                                hipStream_t stream);

// Per-feature inlier mask of one model for class `cls`: bit 0 the decision,
// bit 1 set when the pair's twin r^2 lies in the flag band of T (exact.h:
// the host rechecks it with glibc).
// rule 0: r^2 <= T (T = MSAC 2.25 thr^2 or LO (1.5 thr)^2 as passed)
// rule 2: 1-class graph-cut labeling with weight lambda, T = (1.5 thr)^2
hipError_t launch_mask(const DevProblem& p, int cls, const RectModel& model, int rule, double T, double lambda,
                       uint8_t* mask, hipStream_t stream);

// element-wise evaluation of the device math primitives (parity tests)
hipError_t launch_math(int op, const double* a, const double* b, size_t n, double* out, hipStream_t stream);
// perspective warp (examples/utils.py:92-123): M maps dst pixels to source
// coordinates (row-major 3 x 3), border: constant per-channel values (mode 0)
// or replicate (mode 1); dtype 0 = uint8, 1 = float32, channels interleaved
struct WarpMap {
    double m[9];
    float border[4];
};
hipError_t launch_warp(const void* src, int sh, int sw, int ch, int dtype, const WarpMap& M, void* dst, int dh,
                       int dw, int border_mode, hipStream_t stream);
// Summary of a scored block of `nslots` slots (summary.h, summary.hip): per =
// hypotheses per slot, positions slot * per + q; scores at the position, or
// at its live rank when hmap != null (compacted launch).  target == ~0: the
// chain of hypotheses beating `bar` (from position from_pos on), totals and
// the block's last live hypothesis; otherwise locate the first slot whose
// iterations-before reach `target` (block-relative) -- parts_ready: the
// per-part totals of an earlier summary of the same block are reused.
// tol: hypotheses within tol of the running maximum are members too (near
// ties of the score comparison, exact.h ScoreBound).
// scratch: summary_scratch_bytes(nslots * per, per) bytes of device memory.
size_t summary_scratch_bytes(uint32_t npos, uint32_t per);
hipError_t launch_block_summary(int solver, const uint8_t* inc, const void* models, const ScoreOut& sc,
                                const uint32_t* hmap, uint32_t nslots, uint32_t per, const uint32_t m[2],
                                const double Tm[2], double bar, uint32_t from_pos, uint64_t target, void* scratch,
                                BlockSummary* out, hipStream_t stream, bool parts_ready = false, double tol = 0.0);

// streaming copy of `bytes` (a multiple of 16) for the HBM peak probe
hipError_t launch_hbm_copy(const void* src, void* dst, size_t bytes, int nontemporal, hipStream_t stream);

}  // namespace gcr
