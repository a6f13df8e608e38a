// engine.cpp -- host engine behind the C ABI (include/gcr.h).
//
// GCRANSAC::run (HDR/GCRANSAC.h:192-685) is a strictly sequential loop.  The
// engine keeps its semantics exactly while moving all per-hypothesis work to
// the GPU:
//
//   * every outer-iteration slot s draws its sample from a Philox stream keyed
//     by (seed, s, attempt), so slots are independent and are generated and
//     MSAC-scored in batches (kernels.hip);
//   * the host then REPLAYS the slots in order with the reference's control
//     flow: iteration accounting (:293-339), strict best update + isValidModel
//     (:440-484), LO trigger (:467-477, :494-515), adaptive termination
//     (:286-287, :738-757), the two inlier buffers (:241-246, :460, :563-594)
//     and the final refit (:628-675).  Results are independent of batch size.
//   * local optimisation (:873-1062) runs on the host (relabel masks and the
//     50 trial scores come from GPU launches, the least-squares fits are host
//     C++); graph-cut labeling runs on the empty neighbourhood graph that every
//     Python entry point builds (gcransac_python.cpp:63-68), i.e. a per-node
//     terminal-capacity test evaluated in k_mask.
//
// An inlier buffer is represented by the model whose MSAC inliers it holds and
// its per-class sizes; index lists are materialised (k_mask) only when needed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <functional>
#include <limits>
#include <memory>
#include <new>
#include <string>
#include <vector>
#include <thread>
#include <map>
#include <mutex>
#include <atomic>
#include <exception>
#include <array>
#include <condition_variable>

#include <rccl/rccl.h>

#include <csignal>
#include <execinfo.h>
#include <unistd.h>

#include "gcr.h"
#include "host_fit.h"
#include "kernels.h"
#include "philox.h"
#include "qr3.h"
#include "graphcut.h"
#include "host_pool.h"

using namespace gcr;

namespace {

thread_local std::string g_err;

int set_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

struct HipError {
    hipError_t e;
    const char* what;
};

inline void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw HipError{e, what};
}
#define HIPC(x) hip_check((x), #x)

using Clock = std::chrono::steady_clock;
inline double ms_since(Clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

// host threads currently solving problems inside gcr_solve_batch (the pool's
// workers do not spin while several of them share the cores)
std::atomic<int> g_solving{0};


template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;
    void ensure(size_t n) {
        if (n <= cap) return;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        HIPC(hipMalloc(reinterpret_cast<void**>(&p), sizeof(T) * n));
        cap = n;
    }
    ~DevBuf() { if (p) (void)hipFree(p); }
};

template <class T>
struct PinBuf {
    T* p = nullptr;
    size_t cap = 0;
    bool coherent = false;      // fine-grained (device writes not cached in its L2s)
    void ensure(size_t n) {
        if (n <= cap) return;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        HIPC(hipHostMalloc(reinterpret_cast<void**>(&p), sizeof(T) * n,
                           coherent ? hipHostMallocCoherent : hipHostMallocDefault));
        cap = n;
    }
    ~PinBuf() { if (p) (void)hipHostFree(p); }
};

template <class T>
struct Ptr {
    T* p = nullptr;
};

// the device address of pinned (hipHostMalloc) host memory: kernels write
// small results straight into it (no copy-back launch) and read small inputs
// from it (GCR_ZEROCOPY=0: staged copies instead)
template <class T>
T* dev_view(T* host) {
    void* d = nullptr;
    HIPC(hipHostGetDevicePointer(&d, host, 0));
    return static_cast<T*>(d);
}
inline bool zerocopy_on() {
    const char* e = getenv("GCR_ZEROCOPY");              // read per call (tests switch it)
    return !(e && e[0] == '0');
}

template <class B>
void swap_buf(B& a, B& b) {
    std::swap(a.p, b.p);
    std::swap(a.cap, b.cap);
}

// Score arrays for `cap` hypotheses, device and pinned host mirrors, each set
// in one allocation laid out n0 | n1 | v0 | v1 | tot | fl | lfl
// (capacity-sized fields; fl / lfl: the flagged decisions of exact.h), so that
// a small batch comes back in one copy instead of seven (every copy is a ~5 us
// blit on the stream).
struct ScoreBufs {
    DevBuf<double> dblk;
    PinBuf<double> hblk;
    size_t cap = 0;
    Ptr<uint32_t> n0, n1, hn0, hn1, fl, lfl, hfl, hlfl;
    Ptr<double> v0, v1, tot, hv0, hv1, htot;
    void ensure(size_t n) {
        if (n <= cap) return;
        dblk.ensure(5 * n);
        hblk.ensure(5 * n);
        cap = n;
        auto carve = [n](double* b, Ptr<uint32_t>& a0, Ptr<uint32_t>& a1, Ptr<double>& b0, Ptr<double>& b1,
                         Ptr<double>& b2, Ptr<uint32_t>& f0, Ptr<uint32_t>& f1) {
            a0.p = reinterpret_cast<uint32_t*>(b);
            a1.p = a0.p + n;
            b0.p = b + n;
            b1.p = b + 2 * n;
            b2.p = b + 3 * n;
            f0.p = reinterpret_cast<uint32_t*>(b + 4 * n);
            f1.p = f0.p + n;
        };
        carve(dblk.p, n0, n1, v0, v1, tot, fl, lfl);
        carve(hblk.p, hn0, hn1, hv0, hv1, htot, hfl, hlfl);
    }
    ScoreOut dev() const { return ScoreOut{n0.p, n1.p, v0.p, v1.p, tot.p, fl.p, lfl.p}; }
    // the pinned mirror as kernels see it (results written in place)
    ScoreOut host_dev() const {
        double* b = dev_view(hblk.p);
        const ptrdiff_t d = reinterpret_cast<char*>(b) - reinterpret_cast<char*>(hblk.p);
        auto at = [d](auto* h) { return reinterpret_cast<decltype(h)>(reinterpret_cast<char*>(h) + d); };
        return ScoreOut{at(hn0.p), at(hn1.p), at(hv0.p), at(hv1.p), at(htot.p), at(hfl.p), at(hlfl.p)};
    }
    void swap(ScoreBufs& o) {
        std::swap(dblk.p, o.dblk.p); std::swap(dblk.cap, o.dblk.cap);
        std::swap(hblk.p, o.hblk.p); std::swap(hblk.cap, o.hblk.cap);
        std::swap(cap, o.cap);
        std::swap(n0, o.n0); std::swap(n1, o.n1); std::swap(hn0, o.hn0); std::swap(hn1, o.hn1);
        std::swap(v0, o.v0); std::swap(v1, o.v1); std::swap(tot, o.tot);
        std::swap(hv0, o.hv0); std::swap(hv1, o.hv1); std::swap(htot, o.htot);
        std::swap(fl, o.fl); std::swap(lfl, o.lfl); std::swap(hfl, o.hfl); std::swap(hlfl, o.hlfl);
    }
    void d2h(size_t n, hipStream_t s) {
        const size_t span = 4 * cap * sizeof(double) + (cap + n) * sizeof(uint32_t);    // n0 .. lfl[n)
        if (span <= (size_t)256 * 1024 || 2 * n >= cap) {
            HIPC(hipMemcpyAsync(hblk.p, dblk.p, span, hipMemcpyDeviceToHost, s));
            return;
        }
        HIPC(hipMemcpyAsync(hn0.p, n0.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIPC(hipMemcpyAsync(hn1.p, n1.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIPC(hipMemcpyAsync(hv0.p, v0.p, n * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPC(hipMemcpyAsync(hv1.p, v1.p, n * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPC(hipMemcpyAsync(htot.p, tot.p, n * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPC(hipMemcpyAsync(hfl.p, fl.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIPC(hipMemcpyAsync(hlfl.p, lfl.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    }
};

// Score<K> (score.hpp:11-102) with the MSAC post-processing of
// MSACScoringFunction::getScore (MSAC_scoring_function.hpp:108-127).
struct HScore {
    uint64_t n[2] = {0, 0};
    double v[2] = {0.0, 0.0};
    uint64_t total = 0;
    double sum = 0.0;
};

template <class M>
struct BufferT {             // one of temp_inner_inliers[2]
    bool has = false;
    M model{};
    uint64_t n[2] = {0, 0};  // list sizes (raw inlier counts of `model`)
    // rectification, resolved when the buffer is read (RunnerT::resolve):
    // inc 1..101: `model` is slot `slot`'s generated model with the twin phi
    // of the 2-SIFT minimal solver (the glibc phi is computed on demand);
    // exact: n are the reference's counts (false: flagged decisions, or a
    // model exact.h's bound does not cover, still to recheck)
    uint64_t slot = 0;
    uint32_t inc = 0;
    bool exact = true;
};

}  // namespace

// Device and pinned work buffers of a problem.  A context keeps one shared
// workspace that the one-shot entry points (gcr_rect_*) reuse call after call:
// allocating and freeing pinned memory per call costs milliseconds.
struct Workspace {
    DevBuf<double> feat;                // feature SoA (make_problem)
    PinBuf<double> feat_stage;          // its pinned host image (one upload)
    hipEvent_t feat_ev = nullptr;       // ... recorded after the upload
    bool feat_ev_pending = false;
    DevBuf<uint8_t> inc;
    DevBuf<RectModel> models;
    PinBuf<uint8_t> h_inc;
    PinBuf<RectModel> h_models;
    ScoreBufs sb;
    DevBuf<RectModel> lo_models;
    DevBuf<GeoModel> gmodels, lo_gmodels;     // homography (solver 3) / fundamental (4)
    DevBuf<uint32_t> hmap, hcount;            // live-hypothesis compaction (fundamental)
    PinBuf<GeoModel> h_gmodels;
    ScoreBufs lo_sb;
    DevBuf<uint8_t> mask[2];
    PinBuf<uint8_t> h_mask[2];
    DevBuf<uint8_t> mask_all;           // inlier_lists: both classes, one copy back
    DevBuf<double> r2;                  // graph-cut labeling: squared residuals of the LO model
    PinBuf<double> h_r2;
    PinBuf<RectModel> h_lorect;         // score_models: small batches' models, read in place
    PinBuf<GeoModel> h_logeo;
    DevBuf<double> lo_vals;             // launch_score_small's split scorer (DevProblem::lo)
    DevBuf<uint32_t> lo_meta;
    DevBuf<uint32_t> lo_arrive;         // ... k_lo_split's per-model arrival counters (zeroed once)
    DevBuf<double> lo_psum;             // ... per chunk inlier value sums (k_lo_approx)
    PinBuf<uint64_t> h_mbits;           // launch_score_small: MSAC inlier ballots (ListBits.mbits)
    PinBuf<uint64_t> h_lbits;           // launch_score_small: LO list bits (ListBits), written by
                                        // the kernel straight into this mapped pinned buffer
    PinBuf<uint8_t> h_mask_all;
    DevBuf<BatchRecord> recs;           // verify_batches: one record per batch
    PinBuf<BatchRecord> h_recs;         // ... and their pinned host image
    DevBuf<uint8_t> pg_inc[4];          // verify_batches: slots generated one (two, overlapped) launches ahead
    DevBuf<RectModel> pg_models[4];
    DevBuf<uint8_t> pg_hyp[4], pg_pair[4];   // their band / value constants (GenChain::next_hyp)
    DevBuf<WgBest> wg;                  // verify_batches: per-workgroup bests
    DevBuf<WgBest> vb_wg;               // verify_batches: a ring of batches' workgroup bests and
    DevBuf<RectModel> vb_models;        // models, reduced by one deferred selection launch
    // correspondence verify_batches with deferred selection: a ring of batch
    // buffer sets, each array holding every set back to back (stride nh)
    DevBuf<uint8_t> gr_inc;
    DevBuf<GeoModel> gr_models;
    DevBuf<uint32_t> gr_hmap, gr_hcount, gr_n0, gr_n1;
    DevBuf<double> gr_v0, gr_v1, gr_tot;
    hipEvent_t vb_flush = nullptr;
    hipEvent_t vb_aux = nullptr;        // verify_batches: the aux scoring stream's last batch of a ring
    DevBuf<uint32_t> rf_idx;            // GPU refit: inlier index lists
    PinBuf<uint32_t> rf_hidx;           // GPU refit: their pinned staging
    DevBuf<double> rf_A;                // GPU refit: A (3 columns) and b, column-major
    DevBuf<double> rf_part;             // GPU refit: reduction block partials
    DevBuf<QRDevState> rf_qrst;         // GPU refit: device-resident QR driver state
    DevBuf<QRFState> rf_qrf;            // GPU refit: fused-pass QR driver state
    PinBuf<double> rf_hpart;
    PinBuf<double> rf_htop;             // GPU refit: async upload ring
    DevBuf<DD> rf_gram;                 // GPU refit (Gram path): per-tile double-double sums,
    DevBuf<double> rf_lines;            //   the orientation inliers' lines,
    PinBuf<DD> rf_hgout;                //   the Gram matrix (coherent pinned memory)
    PinBuf<uint32_t> rf_gdone;          //   and its completion flag
    uint32_t gdone_epoch = 0;
    // the next chunk of slots, generated and scored on the side stream while
    // the host replays the current one (RunnerT prefetch); swapped in whole
    DevBuf<uint8_t> pf_inc;
    DevBuf<RectModel> pf_models;
    DevBuf<GeoModel> pf_gmodels;
    PinBuf<uint8_t> pf_h_inc;
    PinBuf<RectModel> pf_h_models;
    PinBuf<GeoModel> pf_h_gmodels;
    ScoreBufs pf_sb;
    DevBuf<uint32_t> pf_hmap, pf_hcount;   // verify_batches: the second batch's compaction
    hipEvent_t vb_gen[2] = {nullptr, nullptr}, vb_done[2] = {nullptr, nullptr}, vb_start = nullptr;
    std::vector<hipEvent_t> evs;        // score-kernel brackets, 2 per batch
    // summary replay (RunnerT::replay_summaries): per chunk buffer set (set 0
    // = inc / models / sb / hmap, set 1 = the pf_ arrays) its summary scratch,
    // device summary, pinned summaries of every rank, the small-scorer pair
    // buffers of a short chunk, and its completion / score-kernel events
    DevBuf<uint8_t> sum_scr[2];
    DevBuf<BlockSummary> dsum[2];
    PinBuf<BlockSummary> hsum[2];       // [0] this rank's, then the all-gathered ones
    DevBuf<BlockSummary> dall[2];       // gcr_comm: the all-gathered summaries on the device
    PinBuf<uint64_t> h_cbits[2];        // small-scored chunks: every slot's LO list bits (ListBits)
    PinBuf<uint64_t> h_cmbits[2];       // ... and its MSAC ballots (ListBits::mbits)
    // small-scored chunks: the split scorer's scratch of each chunk set.  Such
    // a chunk may run on the side stream while the replay stream scores LO
    // trials / the refit through DevProblem::lo, so they never share one.
    DevBuf<double> cs_vals[2];
    DevBuf<uint32_t> cs_meta[2];
    DevBuf<uint32_t> cs_arrive[2];
    hipEvent_t sum_done[2] = {nullptr, nullptr}, sum_k0[2] = {nullptr, nullptr}, sum_k1[2] = {nullptr, nullptr};
    bool spec_pending[2] = {false, false};   // a speculative chunk of this set may still run
    // score_models' completion flags (ScoreOut::done): the small scorer stores
    // done_epoch into lo_done[m] after model m's results; the results, list
    // bits and flags live in coherent pinned memory, so the host waits on the
    // flags instead of the stream's end-of-kernel signal (~5 us sooner)
    PinBuf<uint32_t> lo_done;
    uint32_t done_epoch = 0;
    // LO with approximate trial scores: the exact fold of a round's winner
    // (its results and completion flag), launched behind the round
    ScoreBufs lo_wb;
    PinBuf<uint32_t> lo_wdone;
    uint32_t wdone_epoch = 0;
    Workspace() {
        lo_sb.hblk.coherent = true;
        h_lbits.coherent = true;
        h_mbits.coherent = true;
        lo_done.coherent = true;
        lo_wb.hblk.coherent = true;
        lo_wdone.coherent = true;
        rf_hgout.coherent = true;
        rf_gdone.coherent = true;
    }
    ~Workspace() {
        // the pinned staging image may still be read by the problem upload
        if (feat_ev_pending && feat_ev) (void)hipEventSynchronize(feat_ev);
        for (hipEvent_t e : evs) (void)hipEventDestroy(e);
        for (hipEvent_t e : {vb_gen[0], vb_gen[1], vb_done[0], vb_done[1], vb_start, vb_flush, vb_aux, sum_done[0],
                             sum_done[1], sum_k0[0], sum_k0[1], sum_k1[0], sum_k1[1], feat_ev})
            if (e) (void)hipEventDestroy(e);
    }
};

namespace {
// GCR_EXCHANGE_LOG=1 (read per run): the summary replay logs every event that
// is a collective under gcr_comm -- a chunk's issue (the all-gather of its
// block summaries) and a re-summary (chain continuation or stop locate) --
// and every chunk collected, on the calling thread (gcr_debug_exchange_log).
// RCCL needs every rank to issue the same collectives in the same order; the
// tests compare these logs across ranks (callback path) and between the
// callback and the gcr_comm paths.  Four words per event: kind (1 issue, 2
// re-summary, 3 collect), chunk number, set | ahead << 1 (issue) or set |
// locate << 1 (re-summary), slots (issue) or owner + 1 | from_pos << 16.
thread_local std::vector<uint64_t> t_xlog;

// GCR_LO_TRACE=1 (read at load): host-side timeline of every LO round
// (lists, fits, launch, wait, pick) printed to stderr per local optimisation
const bool g_lo_trace = [] {
    const char* e = getenv("GCR_LO_TRACE");
    return e && e[0] == '1';
}();
thread_local std::vector<std::pair<const char*, Clock::time_point>> t_lot, t_run;
inline void lot(const char* tag) {
    if (g_lo_trace) t_lot.emplace_back(tag, Clock::now());
}
// ... and of the whole run (main loop, LO, final refit): "gcr RUN:"
inline void rlot(const char* tag) {
    if (g_lo_trace) t_run.emplace_back(tag, Clock::now());
}
void lot_print(const char* label, std::vector<std::pair<const char*, Clock::time_point>>& v) {
    if (!g_lo_trace || v.empty()) return;
    std::string line = label;
    const auto b = v.front().second;
    for (const auto& e : v) {
        char buf[64];
        snprintf(buf, sizeof(buf), " %s %.1f", e.first, std::chrono::duration<double, std::micro>(e.second - b).count());
        line += buf;
    }
    fprintf(stderr, "%s\n", line.c_str());
    v.clear();
}

// one step of a host spin-wait on a completion flag: a pause, or -- while
// several gcr_solve_batch threads share the cores -- a yield, so a waiting
// thread hands its core to another problem's host work
inline void spin_pause() {
    if (g_solving.load(std::memory_order_relaxed) > 1) std::this_thread::yield();
    else __builtin_ia32_pause();
}

// spin until a kernel has stored `epoch` into the coherent host flag; a
// stream that drained (or failed) without it is an error.
// A slow completion is not an error (a co-tenant process, or gcr_solve_batch's
// threads sharing the hardware queues, can delay a valid kernel): the wait
// goes on for as long as the stream runs -- as the hipStreamSynchronize it
// replaces did -- and says so once on stderr after GCR_WAIT_WARN_MS (default
// 5000; 0: never).  Errors come from hipStreamQuery.
double wait_warn_ms() {
    static const double v = [] {
        const char* e = getenv("GCR_WAIT_WARN_MS");
        return e ? atof(e) : 5000.0;
    }();
    return v;
}
void slow_wait_note(const char* what, Clock::time_point t0, bool& told) {
    if (told) return;
    const double lim = wait_warn_ms();
    if (lim > 0.0 && ms_since(t0) > lim) {
        fprintf(stderr, "gcr: %s still running after %.0f ms (waiting on)\n", what, lim);
        told = true;
    }
}

void wait_flag(const uint32_t* flag, uint32_t epoch, hipStream_t s, const char* what) {
    const auto t0 = Clock::now();
    bool told = false;
    for (uint64_t it = 1; __atomic_load_n(flag, __ATOMIC_ACQUIRE) != epoch; ++it) {
        if ((it & 4095) == 0) {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess) {
                if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == epoch) break;
                throw std::runtime_error(std::string(what) + ": completion flag missing after the stream drained");
            }
            if (q != hipErrorNotReady) HIPC(q);
            slow_wait_note(what, t0, told);
        }
        spin_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
}

// GCR_BACKTRACE=1 (read at load): SIGABRT / SIGSEGV print the native stack
// to stderr before the default action (diagnostics on the GPU box, which has
// no debugger)
void gcr_crash_handler(int sig) {
    void* fr[64];
    const int n = backtrace(fr, 64);
    const char msg[] = "gcr: fatal signal, native backtrace:\n";
    (void)!write(2, msg, sizeof(msg) - 1);
    backtrace_symbols_fd(fr, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}
[[maybe_unused]] const bool g_crash_hook = [] {
    const char* e = getenv("GCR_BACKTRACE");
    if (e && e[0] == '1') {
        signal(SIGABRT, gcr_crash_handler);
        signal(SIGSEGV, gcr_crash_handler);
    }
    return true;
}();
bool xlog_on() {
    const char* e = getenv("GCR_EXCHANGE_LOG");
    return e && e[0] == '1';
}

// A run can end with a speculative chunk of the summary replay still running
// on the side stream (RunnerT::replay_summaries leaves it in flight so the
// run returns sooner).  It writes set 0 / 1's chunk buffers and reads the
// feature SoA, so everything that reuses the workspace -- the next run's
// replay (either path), verify_batches, the debug entry points, the upload
// of the next problem into a recycled workspace -- waits for it first.
void await_spec(Workspace* w) {
    for (int k = 0; k < 2; ++k)
        if (w->spec_pending[k]) {
            HIPC(hipEventSynchronize(w->sum_done[k]));
            w->spec_pending[k] = false;
        }
}
}  // namespace

struct gcr_ctx {
    int device = 0;
    hipStream_t stream = nullptr;       // the replay's stream: LO, refit, fetched chunks (high priority)
    hipStream_t side = nullptr;         // speculative next chunks (low priority)
    hipStream_t aux = nullptr;          // verify_batches: the second scoring stream (aux_stream)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t pev0 = nullptr, pev1 = nullptr, pdone = nullptr;
    int n_cu = 256;                     // compute units (one batch-scorer workgroup each)
    Workspace shared;                   // reused by the gcr_rect_* calls
    // workspaces of destroyed problems, reused by the next gcr_problem_create
    // (their device and pinned buffers stay allocated: pinned allocations
    // cost milliseconds)
    std::mutex ws_mu;
    std::vector<std::unique_ptr<Workspace>> ws_free;
};

// A communicator rank for the hypothesis-sharded run (RCCL, one process per
// GPU): the block summaries are exchanged by ncclAllGather on the context's
// side stream (RunnerT::exchange).
struct gcr_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1;
    gcr_ctx* ctx = nullptr;
    bool aborted = false;               // ncclCommAbort'ed after an error: every later run fails
};

namespace {
// GCR_COMM_TIMEOUT_MS (read per wait): a collective's completion not seen
// within this many ms is an error (0 / unset: no limit, the RCCL default)
double comm_timeout_ms() {
    const char* e = getenv("GCR_COMM_TIMEOUT_MS");
    return e ? atof(e) : 0.0;
}

// Wait for an event behind a collective of `comm`, polling the
// communicator's asynchronous error state (a peer that failed or left makes
// RCCL report ncclRemoteError / ncclSystemError here instead of leaving the
// kernel spinning).  Throws on an error or past the time limit; the caller's
// error path then aborts the communicator (gcr_problem_run_comm).
void comm_sync(hipEvent_t ev, ncclComm_t comm, const char* what) {
    const auto t0 = Clock::now();
    const double limit = comm_timeout_ms();
    for (uint64_t it = 1;; ++it) {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) hip_check(q, what);
        if ((it & 255) == 0) {
            ncclResult_t ae = ncclSuccess;
            const ncclResult_t r = ncclCommGetAsyncError(comm, &ae);
            if (r != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress))
                throw std::runtime_error(std::string(what) + ": RCCL asynchronous error: " +
                                         ncclGetErrorString(r != ncclSuccess ? r : ae));
            if (limit > 0.0 && ms_since(t0) > limit)
                throw std::runtime_error(std::string(what) + ": no completion within GCR_COMM_TIMEOUT_MS");
            std::this_thread::yield();
        }
    }
}
}  // namespace

struct gcr_problem {
    gcr_ctx* ctx = nullptr;
    int solver = 0;
    int K = 1;
    HostClass hc[2];
    DevProblem dp{};
    std::unique_ptr<Workspace> own;     // gcr_problem_create: private buffers
    Workspace* w = nullptr;             // own.get() or &ctx->shared
    bool scales_ok = true;              // exact.h scales_in_range over the scale features
};

namespace {

// ---------------------------------------- decisions in glibc (exact.h) ----
// The kernels evaluate the detmath twins and flag every decision whose twin
// residual lies within the proven twin-glibc bound of its threshold; these
// host routines take those decisions (and every decision of a model the bound
// does not cover, scale_unsafe) in the reference's arithmetic.

// one pair's squared residual under model m in the reference's formula with
// glibc (GlibcMath: the reference's decision)
template <class M>
double host_r2(const gcr_problem* P, int cls, size_t i, const RectModel& m) {
    const HostClass& h = P->hc[cls];
    if (cls == 0) {
        const double ac = alpha_cube(m);
        return P->solver == 1 ? scale_sq_residual<true, false, M>(h.x[i], h.y[i], h.a[i], m, ac)
                              : scale_sq_residual<false, false, M>(h.x[i], h.y[i], h.a[i], m, ac);
    }
    return orient_sq_residual<false, M>(h.x[i], h.y[i], h.c0[i], h.c1[i], m, orient_const(m));
}

// ... and its value (rect.h scale_sq_value / orient_sq_value: what the
// kernels fold), vc = value_const of m
double host_value(const gcr_problem* P, int cls, size_t i, const RectModel& m, const ValueConst& vc) {
    const HostClass& h = P->hc[cls];
    if (cls == 0)
        return P->solver == 1 ? scale_sq_value<true, false>(h.x[i], h.y[i], h.a[i], m, vc.ac, vc.cut)
                              : scale_sq_value<false, false>(h.x[i], h.y[i], h.a[i], m, vc.ac, vc.cut);
    return orient_sq_value<false>(h.x[i], h.y[i], h.c0[i], h.c1[i], m, vc.c, vc.s, vc.cphi, vc.cphi2);
}

struct ExactCount {
    uint64_t models = 0;       // models whose decisions went through the host
    uint64_t pairs = 0;        // pairs decided with glibc
    uint64_t flips = 0;        // ... whose decision differs from the twin's
    double ms = 0.0;
    uint64_t near_ties = 0;    // score comparisons decided by glibc scores (exact.h ScoreBound)
    uint64_t near_flips = 0;   // ... whose outcome differs from the value comparison
};

// GCR_EXACT=0: decisions stay the twins' (no host recheck, no glibc phi):
// the A/B switch of the rechecks' cost; read per call
bool exact_on() {
    const char* e = getenv("GCR_EXACT");
    return !(e && e[0] == '0');
}

bool model_unsafe(const gcr_problem* P, const RectModel& m, double T0) {
    return P->solver <= 2 && scale_unsafe(P->solver, m.alpha, T0, P->scales_ok);
}

// The MSAC accumulators of one model with every decision in the reference's
// arithmetic (the oracle's TWIN-mode getScore): pair i of class c is an
// inlier iff its glibc r^2 under md is <= T[c] (MSAC_scoring_function.hpp:
// 53-107), and then adds -(its twin r^2 under mv) -- the value the kernels
// fold; mv differs from md only in a generated 2-SIFT model's phi.  Sums in
// feature order, class 0 then 1, the total running across classes.  Pairs in
// parallel on the host pool, the sums sequential.  `lists`: the MSAC inlier
// lists too.  `glibc_sums`: add -(the glibc r^2 under md) instead -- the
// reference's own score (the near-tie comparisons, exact.h ScoreBound).
void exact_accumulate(const gcr_problem* P, const RectModel& mv, const RectModel& md, const double T[2],
                      uint32_t n[2], double v[2], double& tot, std::vector<uint32_t>* lists, ExactCount& ec,
                      bool glibc_sums = false);

// k_mask bytes of one class (bit 0 the twin decision, bit 1 flagged) turned
// into the reference's decisions under md: flagged pairs -- every pair when
// `all` -- decided with glibc (mask_rule on the glibc r^2)
void exact_mask(const gcr_problem* P, int cls, const RectModel& md, int rule, double T, double lambda, uint8_t* mk,
                bool all, ExactCount& ec);

// The glibc phi of slot `slot`'s generated 2-SIFT model (successful attempt
// a): the reference's atan2 of the sample's vanishing point (two_sift.hpp:
// 341); the generators evaluate the twin.  The sample is redrawn on the host
// from the same Philox stream as kernels.hip attempt<2>; its h7, h8, alpha
// must equal the device model's bit for bit.
RectModel glibc_minimal_model(const gcr_problem* P, uint64_t seed, uint64_t slot, uint32_t a, const RectModel& dev);

}  // namespace

namespace {

// The GPU refit runs qr3.h's driver on the device (launch_qr_device) unless
// GCR_QR_DEVICE=0 (host-driven reductions, one synchronisation each)
constexpr size_t kQrDeviceMaxRows = (size_t)256 * kSumSuper;
bool qr_device_on() {
    const char* e = getenv("GCR_QR_DEVICE");           // read per refit (tests switch it)
    return !(e && e[0] == '0');
}
// the device driver in fused passes (launch_sift_refit_fused) unless GCR_QR_FUSED=0
// (one pass per reduction / element-wise step, launch_qr_device)
bool qr_fused_on() {
    const char* e = getenv("GCR_QR_FUSED");
    return !(e && e[0] == '0');
}

// --------------------------------------------------------- GPU refit ----
// qr3.h storage backend in HBM: element-wise steps are kernels, reductions are
// per-block partials (k_qr_partials, row order inside a block) summed here in
// block order -- blocked_sum's order exactly, so results equal the host's.
struct DevQRStore {
    // qr_solve<3> only ever reads rows 0..2 of a column on the host (pivots,
    // R entries, the reduced right-hand side).  Those rows are mirrored in a
    // host cache refreshed inside every reduction's synchronisation, and
    // writes go out asynchronously from a pinned ring, so the ~50 scalar
    // round trips of the driver collapse to one synchronisation per reduction.
    static constexpr int kTop = 3;
    static constexpr int kRing = 64;
    double* col[4];
    hipStream_t s;
    gcr_problem* P;
    size_t m = 0;                 // rows
    double cache[4][kTop] = {};
    bool valid[4][kTop] = {};
    int ring_used = 0;

    double* ring() { return P->w->rf_htop.p; }            // async upload ring
    void prepare() { P->w->rf_htop.ensure(kRing); }

    // gather rows 0..kTop-1 of every column to rf_part[off .. off + 4 kTop) on
    // the device and queue ONE copy of rf_part[0 .. off + 4 kTop) back
    // (complete after the caller's next stream synchronisation)
    void enqueue_with_top(size_t off) {
        P->w->rf_part.ensure(off + 4 * kTop);
        P->w->rf_hpart.ensure(off + 4 * kTop);
        HIPC(launch_qr_top(col[0], col[1], col[2], col[3], m, P->w->rf_part.p + off, s));
        HIPC(hipMemcpyAsync(P->w->rf_hpart.p, P->w->rf_part.p, (off + 4 * kTop) * sizeof(double),
                            hipMemcpyDeviceToHost, s));
    }
    void sync_and_take_top(size_t off) {
        HIPC(hipStreamSynchronize(s));
        ring_used = 0;                                    // every queued upload has completed
        const size_t n = std::min<size_t>(kTop, m);
        for (int c = 0; c < 4; ++c)
            for (size_t i = 0; i < (size_t)kTop; ++i) {
                valid[c][i] = i < n;
                if (i < n) cache[c][i] = P->w->rf_hpart.p[off + c * kTop + i];
            }
    }
    void invalidate(int c, size_t lo, size_t hi) {
        for (size_t i = lo; i < hi && i < (size_t)kTop; ++i) valid[c][i] = false;
    }

    double dot(int a, int c, size_t lo, size_t hi) {
        if (hi <= lo) return 0.0;
        size_t nb = (hi - 1) / kSumBlock - lo / kSumBlock + 1;
        P->w->rf_part.ensure(nb + 4 * kTop);
        P->w->rf_hpart.ensure(nb + 4 * kTop);
        HIPC(launch_qr_partials(col[a], col[c], lo, hi, P->w->rf_part.p, &nb, s));
        enqueue_with_top(nb);
        sync_and_take_top(nb);
        // block partials: sequentially inside each aligned super-block, then
        // the super-block partials sequentially (blocked_sum's order)
        const size_t blk0 = lo / kSumBlock, per = kSumSuper / kSumBlock;
        double total = 0.0, sup = 0.0;
        for (size_t b = 0; b < nb; ++b) {
            if (b > 0 && (blk0 + b) % per == 0) {
                total += sup;
                sup = 0.0;
            }
            sup += P->w->rf_hpart.p[b];
        }
        total += sup;
        return total;
    }
    double sumsq(int c, size_t lo, size_t hi) { return dot(c, c, lo, hi); }
    double get(int c, size_t i) {
        if (i < (size_t)kTop && valid[c][i]) return cache[c][i];
        if (i < (size_t)kTop) {
            enqueue_with_top(0);
            sync_and_take_top(0);
            return cache[c][i];
        }
        HIPC(hipMemcpyAsync(P->w->rf_hpart.p, col[c] + i, sizeof(double), hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        ring_used = 0;
        return P->w->rf_hpart.p[0];
    }
    void set(int c, size_t i, double v) {
        if (ring_used == kRing) {                         // never at C = 3; kept for safety
            HIPC(hipStreamSynchronize(s));
            ring_used = 0;
        }
        double* slot = ring() + ring_used++;
        *slot = v;
        HIPC(hipMemcpyAsync(col[c] + i, slot, sizeof(double), hipMemcpyHostToDevice, s));
        if (i < (size_t)kTop) {
            cache[c][i] = v;
            valid[c][i] = true;
        }
    }
    void scale(int c, size_t lo, size_t hi, double den) {
        HIPC(launch_qr_scale(col[c], lo, hi, den, s));
        invalidate(c, lo, hi);
    }
    void zero(int c, size_t lo, size_t hi) {
        HIPC(launch_qr_zero(col[c], lo, hi, s));
        invalidate(c, lo, hi);
    }
    void update(int c, int e, size_t lo, size_t hi, double tau, double t) {
        HIPC(launch_qr_update(col[c], col[e], lo, hi, tau, t, s));
        invalidate(c, lo, hi);
    }
};

// The hybrid final refit's least-squares system on the GPU: rows built in HBM
// (k_sift_rows, same arithmetic as sift_rows_host), solved by qr3_solve.
struct GpuSiftSolver final : SiftSystemSolver {
    explicit GpuSiftSolver(gcr_problem* p) : P(p) {}
    gcr_problem* P;
    void solve(const std::vector<uint32_t>& si, const std::vector<uint32_t>& oi, size_t rows, double x[3]) override {
        hipStream_t s = P->ctx->stream;
        const size_t ns = si.size(), no = oi.size();
        // reserve for the largest system this problem can produce (every
        // feature an inlier, up to 2^24 rows = 512 MB): a workspace that
        // grows with each bigger refit pays hipFree + hipMalloc (device
        // synchronisations, ~1-2 ms) inside the timed call
        const size_t all_s = P->dp.cls[0].n, all_o = P->dp.cls[1].n;
        const size_t rows_max = std::max(rows, std::min<size_t>(all_s + all_o * (all_o - (all_o > 0)) / 2, 1u << 24));
        P->w->rf_idx.ensure(all_s + all_o);
        P->w->rf_hpart.ensure(1);
        P->w->rf_A.ensure(4 * rows_max);
        double* A = P->w->rf_A.p;
        if (qr_device_on() && qr_fused_on() && rows >= 4 && rows <= kQrDeviceMaxRows) {
            // index lists through pinned memory (no synchronisation before the
            // solve), rows built inside the first fused pass, one synchronisation
            P->w->rf_hidx.ensure(all_s + all_o);
            std::memcpy(P->w->rf_hidx.p, si.data(), ns * sizeof(uint32_t));
            std::memcpy(P->w->rf_hidx.p + ns, oi.data(), no * sizeof(uint32_t));
            HIPC(hipMemcpyAsync(P->w->rf_idx.p, P->w->rf_hidx.p, (ns + no) * sizeof(uint32_t), hipMemcpyHostToDevice,
                                s));
            P->w->rf_part.ensure(kQrfMaxRed * ((rows_max - 1) / kSumBlock + 1));
            P->w->rf_hpart.ensure(3);
            P->w->rf_qrf.ensure(1);
            double* const cols[4] = {A, A + rows, A + 2 * rows, A + 3 * rows};
            HIPC(launch_sift_refit_fused(P->dp.cls[0], P->dp.cls[1], P->w->rf_idx.p, (uint32_t)ns, P->w->rf_idx.p + ns,
                                         (uint32_t)no, rows, cols, P->w->rf_qrf.p, P->w->rf_part.p, P->w->rf_hpart.p,
                                         s));
            for (int q = 0; q < 3; ++q) x[q] = P->w->rf_hpart.p[q];
            return;
        }
        HIPC(hipMemcpyAsync(P->w->rf_idx.p, si.data(), ns * sizeof(uint32_t), hipMemcpyHostToDevice, s));
        HIPC(hipMemcpyAsync(P->w->rf_idx.p + ns, oi.data(), no * sizeof(uint32_t), hipMemcpyHostToDevice, s));
        HIPC(launch_sift_rows(P->dp.cls[0], P->dp.cls[1], P->w->rf_idx.p, (uint32_t)ns, P->w->rf_idx.p + ns, (uint32_t)no,
                              rows, A, A + rows, A + 2 * rows, A + 3 * rows, s));
        HIPC(hipStreamSynchronize(s));          // index lists are pageable host vectors
        if (qr_device_on() && rows >= 4 && rows <= kQrDeviceMaxRows) {
            // the QR driver's decisions on the device, one pass per step
            // (GCR_QR_FUSED=0): one synchronisation
            P->w->rf_part.ensure((rows_max - 1) / kSumBlock + 1);
            P->w->rf_hpart.ensure(3);
            double* const cols[4] = {A, A + rows, A + 2 * rows, A + 3 * rows};
            P->w->rf_qrst.ensure(1);
            HIPC(launch_qr_device(cols, rows, P->w->rf_qrst.p, P->w->rf_part.p, P->w->rf_hpart.p, s));
            for (int q = 0; q < 3; ++q) x[q] = P->w->rf_hpart.p[q];
            return;
        }
        DevQRStore st{{A, A + rows, A + 2 * rows, A + 3 * rows}, s, P};
        st.m = rows;
        st.prepare();
        qr3_solve(st, rows, x);
        HIPC(hipStreamSynchronize(s));          // the pinned ring must outlive its uploads
    }
    // the double-double Gram matrix of the same rows (gram.h): one kernel
    // builds every row once and reduces it in its tile, a second combines
    // the tiles into the matrix, written into coherent pinned memory with a
    // completion flag the host waits on
    bool gram(const std::vector<uint32_t>& si, const std::vector<uint32_t>& oi, size_t rows, DD g[kGramN]) override {
        hipStream_t s = P->ctx->stream;
        const size_t ns = si.size(), no = oi.size();
        const size_t all_s = P->dp.cls[0].n, all_o = P->dp.cls[1].n;
        const size_t rows_max = std::max(rows, all_s + all_o * (all_o - (all_o > 0)) / 2);
        const size_t tiles_max = (rows_max + kGramTile - 1) / kGramTile, tiles = (rows + kGramTile - 1) / kGramTile;
        P->w->rf_idx.ensure(all_s + all_o);
        P->w->rf_hidx.ensure(all_s + all_o);
        P->w->rf_gram.ensure(tiles_max * kGramN);
        P->w->rf_hgout.ensure(kGramN);
        P->w->rf_gdone.ensure(1);
        GramFinal fin;
        fin.out = dev_view(P->w->rf_hgout.p);
        fin.done = dev_view(P->w->rf_gdone.p);
        fin.epoch = ++P->w->gdone_epoch;
        if (fin.epoch == 0) fin.epoch = ++P->w->gdone_epoch;
        P->w->rf_lines.ensure(3 * all_o);
        rlot("g_setup");
        // the index lists through pinned memory, read in place by the prep kernel
        std::memcpy(P->w->rf_hidx.p, si.data(), ns * sizeof(uint32_t));
        std::memcpy(P->w->rf_hidx.p + ns, oi.data(), no * sizeof(uint32_t));
        rlot("g_h2d");
        HIPC(launch_sift_gram(P->dp.cls[0], P->dp.cls[1], dev_view(P->w->rf_hidx.p), (uint32_t)ns, (uint32_t)no, rows,
                              P->w->rf_idx.p, P->w->rf_lines.p, P->w->rf_gram.p, fin, s));
        rlot("g_launch");
        wait_flag(P->w->rf_gdone.p, fin.epoch, s, "gram refit");
        rlot("g_synced");
        for (int k = 0; k < kGramN; ++k) g[k] = P->w->rf_hgout.p[k];
        (void)tiles;
        return true;
    }
    void for_ranges(size_t n, const std::function<void(size_t, size_t)>& fn) override;
};

// A small persistent pool of host threads for the LO trial fits (independent
// least-squares solves; results land at their trial index, so the outcome
// does not depend on the scheduling).  Size: GCR_HOST_THREADS, default
// min(16, hardware threads) -- one GPU's CPU share on an MI355X node; the
// 50 LO fits of a graph-cut round take 42 us on 16 threads, 70 on 8.

HostPool& host_pool() {
    static HostPool pool(
        [] {
            const char* e = getenv("GCR_HOST_THREADS");
            long n = e ? atol(e) : (long)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
            return (unsigned)std::max(1L, std::min(64L, n));
        }(),
        &g_solving);
    return pool;
}

// ---------------------------------------- decisions in glibc: bodies ----
void exact_accumulate(const gcr_problem* P, const RectModel& mv, const RectModel& md, const double T[2],
                      uint32_t n[2], double v[2], double& tot, std::vector<uint32_t>* lists, ExactCount& ec,
                      bool glibc_sums) {
    const auto t0 = Clock::now();
    thread_local std::vector<double> val;
    thread_local std::vector<uint8_t> dec;
    n[0] = n[1] = 0;
    v[0] = v[1] = 0.0;
    tot = 0.0;
    for (int c = 0; c < 2; ++c) {
        if (lists) lists[c].clear();
        if (c >= P->K) continue;
        const size_t N = P->hc[c].n;
        val.resize(N);
        dec.resize(N);
        // the caller's thread_local scratch (the pool's workers have their own)
        double* const vp = val.data();
        uint8_t* const dp = dec.data();
        std::atomic<uint64_t> flips{0};
        const ValueConst vc = value_const(mv, P->solver == 1, c == 1);
        auto body = [&](size_t lo, size_t hi) {
            uint64_t f = 0;
            for (size_t i = lo; i < hi; ++i) {
                const double rg = host_r2<GlibcMath>(P, c, i, md);
                const bool d = rg <= T[c];
                const double rv = glibc_sums ? rg : host_value(P, c, i, mv, vc);
                vp[i] = rv;
                dp[i] = d ? 1 : 0;
                f += (rv <= T[c]) != d ? 1u : 0u;
            }
            flips.fetch_add(f, std::memory_order_relaxed);
        };
        const size_t parts = N >= 4096 ? 16 : 1, step = (N + parts - 1) / parts;
        host_pool().parallel_for(parts, [&](size_t q) { body(std::min(N, q * step), std::min(N, (q + 1) * step)); });
        for (size_t i = 0; i < N; ++i)
            if (dec[i]) {
                ++n[c];
                v[c] += -val[i];
                tot += -val[i];
                if (lists) lists[c].push_back((uint32_t)i);
            }
        ec.pairs += N;
        ec.flips += flips.load();
    }
    ++ec.models;
    ec.ms += ms_since(t0);
}

void exact_mask(const gcr_problem* P, int cls, const RectModel& md, int rule, double T, double lambda, uint8_t* mk,
                bool all, ExactCount& ec) {
    const size_t N = P->hc[cls].n;
    if (!all) {
        // flags are rare: find them eight bytes at a time
        size_t i0 = 0;
        for (; i0 + 8 <= N; i0 += 8) {
            uint64_t w;
            std::memcpy(&w, mk + i0, 8);
            if (w & 0x0202020202020202ull) break;
        }
        for (size_t i = i0; i < N; ++i) {
            if (!(mk[i] & 2)) continue;
            const uint8_t d = mask_rule(host_r2<GlibcMath>(P, cls, i, md), rule, T, lambda) ? 1 : 0;
            ++ec.pairs;
            ec.flips += (mk[i] & 1) != d ? 1u : 0u;
            mk[i] = d;
        }
        return;
    }
    const auto t0 = Clock::now();
    std::atomic<uint64_t> flips{0};
    auto body = [&](size_t lo, size_t hi) {
        uint64_t f = 0;
        for (size_t i = lo; i < hi; ++i) {
            const uint8_t d = mask_rule(host_r2<GlibcMath>(P, cls, i, md), rule, T, lambda) ? 1 : 0;
            f += (mk[i] & 1) != d ? 1u : 0u;
            mk[i] = d;
        }
        flips.fetch_add(f, std::memory_order_relaxed);
    };
    const size_t parts = N >= 4096 ? 16 : 1, step = (N + parts - 1) / parts;
    host_pool().parallel_for(parts, [&](size_t q) { body(std::min(N, q * step), std::min(N, (q + 1) * step)); });
    ec.pairs += N;
    ec.flips += flips.load();
    ec.ms += ms_since(t0);
}

RectModel glibc_minimal_model(const gcr_problem* P, uint64_t seed, uint64_t slot, uint32_t a, const RectModel& dev) {
    const HostClass& sc = P->hc[0];
    const HostClass& oc = P->hc[1];
    uint32_t si[2], oi[2];
    WordStream ws0(seed, slot, a, kStreamMain, 0);
    WordStream ws1(seed, slot, a, kStreamMain, 1);
    RectModel m = default_model();
    bool ok = sample_distinct<2>(ws0, sc.n, 2, si) && sample_distinct<2>(ws1, oc.n, 2, oi);
    if (ok) {
        double sx[2], sy[2], sp[2], ox[2], oy[2], oco[2], osi[2];
        for (int j = 0; j < 2; ++j) {
            sx[j] = sc.x[si[j]];
            sy[j] = sc.y[si[j]];
            sp[j] = sc.c0[si[j]];
            ox[j] = oc.x[oi[j]];
            oy[j] = oc.y[oi[j]];
            oco[j] = oc.c0[oi[j]];
            osi[j] = oc.c1[oi[j]];
        }
        ok = valid_sample_sift22(sx, sy, ox, oy, oco, osi) && solve_sift22<GlibcMath>(sx, sy, sp, ox, oy, oco, osi, m);
    }
    if (!ok || as_u64(m.h7) != as_u64(dev.h7) || as_u64(m.h8) != as_u64(dev.h8) ||
        as_u64(m.alpha) != as_u64(dev.alpha))
        throw std::runtime_error("host redraw of a generated 2-SIFT slot disagrees with the generator");
    return m;
}

// LO trials, refits and reconciliations of at most kSmallScore models use
// launch_score_small; GCR_SMALL_SCORE=0 routes them through the batch scorers
constexpr uint32_t kSmallScore = 256;
bool small_score_on() {
    static const bool on = [] {
        const char* e = getenv("GCR_SMALL_SCORE");
        return !(e && e[0] == '0');
    }();
    return on;
}

// gcr_debug_score[_h]: GCR_DEBUG_SCORER=small scores through
// launch_score_small (read per call, so tests can compare both paths)
bool debug_small_scorer(uint32_t n) {
    const char* e = getenv("GCR_DEBUG_SCORER");
    return e && e[0] == 's' && n > 0 && n <= kSmallScore;
}

// the final refit's per-inlier host work on the host pool (the refit runs on
// the solving thread, never inside a pool job)
void GpuSiftSolver::for_ranges(size_t n, const std::function<void(size_t, size_t)>& fn) {
    const size_t parts = n < 1024 ? 1 : 8;
    const size_t step = (n + parts - 1) / parts;
    host_pool().parallel_for(parts, [&](size_t p) {
        const size_t lo = p * step, hi = std::min(n, lo + step);
        if (lo < hi) fn(lo, hi);
    });
}

// verify_batches records kernel-timing events on every n-th batch
// (GCR_TIMING_STRIDE, default 1 = every batch)
// every batch's event pair costs ~6 us of queue time (measured at the
// driver's 20-step line: stride 1 / 4 / 20 -> 0.136 / 0.130 / 0.129 ms per
// step), so by default every 4th batch is timed
uint32_t timing_stride() {
    static uint32_t v = [] {
        const char* e = getenv("GCR_TIMING_STRIDE");
        const long n = e ? atol(e) : 4;
        return (uint32_t)(n < 1 ? 1 : n);
    }();
    return v;
}

// Span timing (the fused, non-pipelined path; default): ONE event pair
// around the back-to-back scoring launches 1 .. nb-2 of a call when no
// deferred selection falls between them -- their mean duration without the
// per-batch pairs' ~6 us queue gaps (a 20-step call: 10 gaps, ~3 % of its
// time).  The first launch (it generates its own slots: no look-ahead batch
// before it) and the last (followed by the selection) are left out.
// GCR_TIMING_SPAN=0 keeps the per-batch pairs.
bool timing_span() {
    const char* e = getenv("GCR_TIMING_SPAN");
    return !(e && e[0] == '0');
}

// hybrid systems at least this tall are solved on the GPU (the host QR costs
// ~15 ns/row; the GPU path ~0.3 ms + ~15 synchronisations)
size_t gpu_refit_rows() {
    static size_t v = [] {
        const char* e = getenv("GCR_GPU_REFIT_ROWS");
        return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)32768;
    }();
    return v;
}

// ------------------------------------------------------------- problem ----
// Host SoA copy plus the per-feature constants, evaluated with glibc exactly as
// the reference evaluates them inside its solvers and residuals:
//   scale:       pow(s, kScalePower)   (three_sift.hpp:89/172, two_sift.hpp:224)
//   orientation: cos(theta), sin(theta) (math_utils.hpp:104-109, model.h:158-159)
//                as ONE glibc sincos(theta): the reference is built with GCC,
//                which fuses those adjacent cos/sin calls into sincos, and
//                sincos differs from separate sin/cos in ~0.1% of arguments.
// One parallel pass over the features (host pool, element-wise, so the split
// changes no value): the host SoA columns and constants, the pinned staging
// image of the device SoA (class c's five columns of np[c] doubles each, at
// off[c]), each column's largest finite |value| (amax: +inf if a NaN or an
// infinity occurs) and the scale-range flag of exact.h (scales_in_range).
struct FillOut {
    double amax[2][4];
    bool scales_ok;
};
FillOut fill_host_classes(int solver, const double* f0, size_t n0, const double* f1, size_t n1, HostClass* hc,
                          double* hst, const size_t np[2], const size_t off[2]) {
    const bool corr = solver == 3 || solver == 4;
    const int K = solver == 2 ? 2 : 1;
    const double kScalePower = (solver == 1) ? (-1.0 / 3.0) : (1.0 / 3.0);
    const double* src[2] = {f0, f1};
    const size_t ns[2] = {n0, K == 2 ? n1 : 0};
    FillOut res{};
    res.scales_ok = true;
    struct Part {
        int c;
        size_t lo, hi;
        double mx[4];
        bool bad[4];
        bool range;
    };
    // both classes' parts in ONE pool job (16 per large class)
    Part pr[32];
    int np_ = 0;
    double* d[2][5];
    for (int c = 0; c < 2; ++c) {
        HostClass& h = hc[c];
        const size_t n = ns[c];
        if (c >= K) {
            h = HostClass{};
            continue;
        }
        h.n = n;
        h.x.resize(n); h.y.resize(n); h.a.resize(n); h.c0.resize(n); h.c1.resize(n);
        for (int q = 0; q < 5; ++q) d[c][q] = hst + off[c] + (size_t)q * np[c];
        const size_t parts = n >= 4096 ? 16 : 1;
        const size_t step = (n + parts - 1) / parts;
        for (size_t p = 0; p < parts; ++p)
            pr[np_++] = Part{c, std::min(n, p * step), std::min(n, (p + 1) * step), {}, {}, true};
    }
    auto fill = [&](size_t pi) {
        Part& o = pr[pi];
        const int c = o.c;
        HostClass& h = hc[c];
        double* const* dd = d[c];
        for (int q = 0; q < 4; ++q) {
            o.mx[q] = 0.0;
            o.bad[q] = false;
        }
        o.range = true;
        for (size_t i = o.lo; i < o.hi; ++i) {
            double v[5];
            if (corr) {
                v[0] = src[0][4 * i];
                v[1] = src[0][4 * i + 1];
                v[2] = src[0][4 * i + 2];
                v[3] = src[0][4 * i + 3];
                v[4] = 0.0;
            } else {
                v[0] = src[c][3 * i];
                v[1] = src[c][3 * i + 1];
                v[2] = src[c][3 * i + 2];
                if (c == 0) {
                    v[3] = std::pow(v[2], kScalePower);
                    v[4] = 0.0;
                    const double sc = v[2];
                    if (sc > 0.0 && sc < HUGE_VAL && !(sc >= 0x1p-200 && sc <= 0x1p200)) o.range = false;
                } else {
                    double sn, cs;
                    ::sincos(v[2], &sn, &cs);
                    v[3] = cs;
                    v[4] = sn;
                }
            }
            h.x[i] = v[0]; h.y[i] = v[1]; h.a[i] = v[2]; h.c0[i] = v[3]; h.c1[i] = v[4];
            for (int q = 0; q < 5; ++q) dd[q][i] = v[q];
            for (int q = 0; q < 4; ++q) {
                const double a = std::fabs(v[q]);
                if (!(a < HUGE_VAL)) o.bad[q] = true;
                else if (a > o.mx[q]) o.mx[q] = a;
            }
        }
    };
    host_pool().parallel_for((size_t)np_, fill);
    for (int c = 0; c < 2; ++c) {
        for (int q = 0; q < 4; ++q) {
            double mx = 0.0;
            bool bad = false;
            for (int p = 0; p < np_; ++p)
                if (pr[p].c == c) {
                    bad = bad || pr[p].bad[q];
                    mx = std::max(mx, pr[p].mx[q]);
                }
            res.amax[c][q] = c < K ? (bad ? HUGE_VAL : mx) : 0.0;
        }
        if (c >= K) continue;
        if (c == 0 && solver <= 2)
            for (int p = 0; p < np_; ++p) res.scales_ok = res.scales_ok && (pr[p].c != 0 || pr[p].range);
        for (int q = 0; q < 5; ++q)
            for (size_t i = ns[c]; i < np[c]; ++i) d[c][q][i] = 0.0;      // pads
    }
    return res;
}

// the host classes alone (debug and host-only entry points)
void fill_host_classes(int solver, const double* f0, size_t n0, const double* f1, size_t n1, HostClass* hc) {
    const size_t n1k = solver == 2 ? n1 : 0;
    const size_t np[2] = {(n0 + 1) & ~size_t(1), (n1k + 1) & ~size_t(1)};
    const size_t off[2] = {0, 5 * np[0]};
    std::vector<double> stage(5 * (np[0] + np[1]));
    (void)fill_host_classes(solver, f0, n0, f1, n1, hc, stage.data(), np, off);
}

// GCR_VERIFY_OVERLAP=0: verify_batches keeps its scoring launches on one
// stream (A/B; the default overlaps consecutive launches on two streams)
bool verify_overlap_on() {
    const char* e = getenv("GCR_VERIFY_OVERLAP");
    return !(e && e[0] == '0');
}

// the context's second scoring stream (verify_batches' overlap), created on
// first use at the replay stream's priority
hipStream_t aux_stream(gcr_ctx* ctx) {
    if (ctx->aux == nullptr) {
        int least = 0, greatest = 0;
        HIPC(hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIPC(hipStreamCreateWithPriority(&ctx->aux, hipStreamNonBlocking, greatest));
    }
    return ctx->aux;
}

int make_problem(gcr_ctx* ctx, int solver, const double* f0, size_t n0, const double* f1, size_t n1,
                 gcr_problem** out, bool shared_workspace = false) {
    if (!ctx || !out) return set_err(GCR_EINVAL, "null context or output pointer");
    if (solver < 0 || solver > 4) return set_err(GCR_EINVAL, "unknown solver %d", solver);
    const int K = solver == 2 ? 2 : 1;
    const size_t m0 = solver == 2 ? 2 : solver == 3 ? 4 : solver == 4 ? 7 : 3;
    if (!f0 || (K == 2 && !f1)) return set_err(GCR_EINVAL, "null feature pointer");
    if (n0 < m0 || (K == 2 && n1 < 2))
        return set_err(GCR_EINTERNAL, "Data set smaller than minimal sample size for corresponding data type");
    if (n0 > 0xffffffffull || n1 > 0xffffffffull) return set_err(GCR_EINVAL, "too many features");
    auto P = std::unique_ptr<gcr_problem>(new (std::nothrow) gcr_problem());
    if (!P) return set_err(GCR_ENOMEM, "out of host memory");
    P->ctx = ctx;
    P->solver = solver;
    P->K = K;
    const size_t ns[2] = {n0, K == 2 ? n1 : 0};
    std::vector<std::pair<const char*, Clock::time_point>> st;      // GCR_LO_TRACE: "gcr SETUP:"
    if (g_lo_trace) st.emplace_back("start", Clock::now());
    // SoA, every array padded to an even length (zeros) so that 16-byte
    // LDS-DMA strips (k_score_split staging) are aligned and in bounds
    const size_t np[2] = {(ns[0] + 1) & ~size_t(1), (ns[1] + 1) & ~size_t(1)};
    const size_t total = 5 * (np[0] + np[1]);
    HIPC(hipSetDevice(ctx->device));
    if (shared_workspace) {
        P->w = &ctx->shared;
    } else {
        {
            std::lock_guard<std::mutex> lk(ctx->ws_mu);
            if (!ctx->ws_free.empty()) {
                P->own = std::move(ctx->ws_free.back());
                ctx->ws_free.pop_back();
            }
        }
        if (!P->own) P->own.reset(new Workspace());
        P->w = P->own.get();
    }
    await_spec(P->w);                   // a recycled workspace: its last speculative chunk reads feat
    // this workspace's previous upload (queued, possibly never waited for:
    // a problem created and destroyed without running) reads the staging
    // image and writes the device SoA: it must be done before either buffer
    // is reallocated below
    if (P->w->feat_ev_pending) {
        HIPC(hipEventSynchronize(P->w->feat_ev));
        P->w->feat_ev_pending = false;
    }
    P->w->feat.ensure(total);
    // the whole SoA image (pads zeroed) is staged in pinned memory and goes
    // up in ONE copy (ten pageable copies cost ~150 us of a one-shot call)
    P->w->feat_stage.ensure(total);
    if (g_lo_trace) st.emplace_back("ws", Clock::now());
    double* hst = P->w->feat_stage.p;
    const size_t off[2] = {0, 5 * np[0]};
    const FillOut fo = fill_host_classes(solver, f0, n0, f1, n1, P->hc, hst, np, off);
    if (solver <= 2) P->scales_ok = fo.scales_ok;
    if (g_lo_trace) st.emplace_back("fill", Clock::now());
    P->dp.solver = solver;
    for (int c = 0; c < 2; ++c) {
        DevClass& d = P->dp.cls[c];
        d.n = (uint32_t)ns[c];
        for (int q = 0; q < 4; ++q) d.amax[q] = fo.amax[c][q];
        if (ns[c] == 0) { d.x = d.y = d.a = d.c0 = d.c1 = nullptr; continue; }
        const double** dst[5] = {&d.x, &d.y, &d.a, &d.c0, &d.c1};
        for (int q = 0; q < 5; ++q) *dst[q] = P->w->feat.p + off[c] + (size_t)q * np[c];
    }
    // the split small-batch scorer's scratch (launch_score_small)
    P->dp.lo = SmallScratch{};
    const size_t spairs = small_score_pairs(P->dp);
    if (spairs > 0 && spairs <= kSplitMaxPairs) {
        P->w->lo_vals.ensure(spairs * kSplitModels);
        P->w->lo_meta.ensure(spairs / 64 * kSplitModels);
        P->w->lo_psum.ensure(spairs / 64 * kSplitModels);
        if (!P->w->lo_arrive.p) {
            P->w->lo_arrive.ensure(kSplitModels);
            HIPC(hipMemsetAsync(P->w->lo_arrive.p, 0, kSplitModels * sizeof(uint32_t), ctx->stream));
        }
        P->dp.lo = SmallScratch{P->w->lo_vals.p, P->w->lo_meta.p, kSplitModels, P->w->lo_arrive.p, P->w->lo_psum.p};
    }
    if (g_lo_trace) st.emplace_back("staged", Clock::now());
    // the upload stays asynchronous: the problem's kernels follow it on the
    // stream, and the side stream (speculative chunks, generation) waits on
    // its event; the next problem on this workspace waits before restaging
    // A copy kernel reads the pinned image through its device address (one
    // dispatch) instead of an SDMA copy: configs[4] batch 3 637 -> 3 976
    // problems/s (three interleaved pairs), M2 latency 0.527 -> 0.514 ms; the
    // SDMA path's runtime calls stall under the batch's 8 threads.
    // GCR_UPLOAD=sdma (read per call): hipMemcpyAsync (A/B)
    const char* eu = getenv("GCR_UPLOAD");
    if (!(eu && eu[0] == 's') && total % 2 == 0)
        HIPC(launch_hbm_copy(dev_view(hst), P->w->feat.p, total * sizeof(double), 0, ctx->stream));
    else
        HIPC(hipMemcpyAsync(P->w->feat.p, hst, total * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    if (!P->w->feat_ev) HIPC(hipEventCreateWithFlags(&P->w->feat_ev, hipEventDisableTiming));
    HIPC(hipEventRecord(P->w->feat_ev, ctx->stream));
    HIPC(hipStreamWaitEvent(ctx->side, P->w->feat_ev, 0));
    P->w->feat_ev_pending = true;
    if (g_lo_trace) {
        st.emplace_back("queued", Clock::now());
        lot_print("gcr SETUP:", st);
    }
    *out = P.release();
    return GCR_OK;
}

// ---------------------------------------------------------------- runner ----
// Estimator traits of the host engine: model type, kernels and host fits of
// the rectification solvers (0-2) and the homography (3).
struct RectTraits {
    using Model = RectModel;
    static constexpr size_t kPer = 1;
    static constexpr bool kFusedVerify = true;    // verify = one fused generate + score launch
    static Model def() { return default_model(); }
    static DevBuf<Model>& dmodels(Workspace* w) { return w->models; }
    static PinBuf<Model>& hmodels(Workspace* w) { return w->h_models; }
    static DevBuf<Model>& pf_dmodels(Workspace* w) { return w->pf_models; }
    static PinBuf<Model>& pf_hmodels(Workspace* w) { return w->pf_h_models; }
    static DevBuf<Model>& lomodels(Workspace* w) { return w->lo_models; }
    static PinBuf<Model>& hlomodels(Workspace* w) { return w->h_lorect; }
    static bool identity(const Model& m) { return identity_norm(m); }
    static bool valid(int solver, const Model& m) { return solver == 2 ? valid_model_sift22(m) : true; }
    static hipError_t generate(gcr_problem* P, uint64_t seed, uint64_t s0, uint32_t n, uint8_t* inc, Model* m,
                               hipStream_t s) {
        return launch_generate(P->dp, seed, s0, n, inc, m, s);
    }
    static hipError_t score(gcr_problem* P, const double T[2], const Model* m, const uint8_t* inc, uint32_t n,
                            bool identity, const ScoreOut& out, hipStream_t s) {
        return launch_score(P->dp, T, m, inc, n, identity, out, s);
    }
    static hipError_t mask(gcr_problem* P, int cls, const Model& m, int rule, double T, double lambda, uint8_t* mk,
                           hipStream_t s) {
        return launch_mask(P->dp, cls, m, rule, T, lambda, mk, s);
    }
    // the rectification entry points never have pairwise terms (empty grid)
    static hipError_t sqres(gcr_problem*, const Model&, double*, hipStream_t) { return hipErrorNotSupported; }
    static hipError_t score_live(gcr_problem* P, const double T[2], const Model* m, const uint8_t* inc, uint32_t nh,
                                 uint32_t, const ScoreOut& out, hipStream_t s) {
        return launch_score(P->dp, T, m, inc, nh, true, out, s);
    }
    static constexpr bool kPipe = false;   // generation is fused into the scorer
    static size_t per(gcr_problem*) { return 1; }
    struct VBufs {};
    static VBufs vbufs(gcr_problem*, int, uint32_t) { return {}; }
    static VBufs vbufs_ring(gcr_problem*, uint32_t, uint32_t, uint32_t) { return {}; }
    static uint32_t select_ring(gcr_problem*, uint32_t) { return 1; }
    static hipError_t select_ring_batches(gcr_problem*, const double*, uint64_t, uint32_t, const uint32_t*, uint32_t,
                                          BatchRecord*, hipStream_t) {
        return hipErrorNotSupported;
    }
    static hipError_t verify_gen(gcr_problem*, uint64_t, uint64_t, uint32_t, const VBufs&, hipStream_t) {
        return hipErrorNotSupported;
    }
    static hipError_t verify_score(gcr_problem*, const double*, uint64_t, uint32_t, const uint32_t*, BatchRecord*,
                                   hipEvent_t, hipEvent_t, const VBufs&, hipStream_t) {
        return hipErrorNotSupported;
    }
    // batch b of nb: chained launches (the previous launch generated this
    // batch's slots, this one generates the next batch's) when the kernel
    // at this batch size supports it (verify_chains)
    // ahead = 2 (verify_batches' two-stream overlap): batches alternate
    // between two streams, batch b chains to b + 2 (same stream) and uses
    // buffer set b & 1 for its per-slot outputs; its ring selection is left
    // to the caller (select_flush), which orders it after both streams
    static hipError_t verify(gcr_problem* P, const double Tm[2], uint64_t seed, uint64_t s0, uint32_t n,
                             const uint32_t m[2], size_t wg_cap, BatchRecord* rec, hipEvent_t e0, hipEvent_t e1,
                             hipStream_t s, uint32_t b = 0, uint32_t nb = 1, uint32_t ahead = 1) {
        GenChain ch;
        Workspace* w = P->w;
        if (nb > ahead && verify_chains(n) && chain_on()) {
            const uint32_t nbuf = 2 * ahead;
            for (uint32_t k = 0; k < nbuf; ++k) {
                w->pg_inc[k].ensure(n);
                w->pg_models[k].ensure(n);
            }
            const bool pc = preconst_on();
            if (pc)
                for (uint32_t k = 0; k < nbuf; ++k) {
                    w->pg_hyp[k].ensure((size_t)n * kFmHypBytes);
                    w->pg_pair[k].ensure((size_t)(n + 1) / 2 * kFmPairBytes);
                }
            if (b >= ahead) {
                ch.pre_inc = w->pg_inc[b % nbuf].p;
                ch.pre_models = w->pg_models[b % nbuf].p;
                if (pc) {
                    ch.pre_hyp = w->pg_hyp[b % nbuf].p;
                    ch.pre_pair = w->pg_pair[b % nbuf].p;
                }
            }
            if (b + ahead < nb) {
                ch.next_inc = w->pg_inc[(b + ahead) % nbuf].p;
                ch.next_models = w->pg_models[(b + ahead) % nbuf].p;
                if (pc) {
                    ch.next_hyp = w->pg_hyp[(b + ahead) % nbuf].p;
                    ch.next_pair = w->pg_pair[(b + ahead) % nbuf].p;
                }
            }
            ch.ahead = ahead;
        }
        const bool set1 = ahead == 2 && (b & 1);
        if (set1) {
            w->pf_inc.ensure(n);
            w->pf_sb.ensure(n);
        }
        uint8_t* const inc = set1 ? w->pf_inc.p : w->inc.p;
        const ScoreOut sb = set1 ? w->pf_sb.dev() : w->sb.dev();
        if (!defer_on()) {
            return launch_verify_fused(P->dp, Tm, seed, s0, n, m, inc, P->w->models.p, sb, P->w->wg.p, wg_cap, rec,
                                       e0, e1, s, ch);
        }
        // deferred selection: batch b leaves its workgroup bests and models in
        // ring slot b % R; one launch reduces a whole ring (one workgroup per
        // batch) after its last batch, so the per-batch reduction kernel and
        // its launch leave the chain of scoring launches
        const uint32_t R = select_ring(n);
        w->vb_wg.ensure((size_t)R * wg_cap);
        w->vb_models.ensure((size_t)R * n);
        const uint32_t k = b % R;
        hipError_t e = launch_verify_fused(P->dp, Tm, seed, s0, n, m, inc, w->vb_models.p + (size_t)k * n, sb,
                                           w->vb_wg.p + (size_t)k * wg_cap, wg_cap, nullptr, e0, e1, s, ch);
        if (e != hipSuccess || ahead != 1 || !(k == R - 1 || b + 1 == nb)) return e;
        return select_flush(P, s0 - (uint64_t)k * n, n, k + 1, wg_cap, rec - k, s);
    }
    // the deferred selection of ring batches 0 .. count - 1 (slots from s0):
    // their records to rec[0 .. count)
    static hipError_t select_flush(gcr_problem* P, uint64_t s0, uint32_t n, uint32_t count, size_t wg_cap,
                                   BatchRecord* rec, hipStream_t s) {
        return launch_select_batches(P->w->vb_wg.p, wg_cap, P->w->vb_models.p, s0, n, count, rec, s);
    }
    // true when batch b's launch directly follows a deferred selection launch
    // (verify_batches does not time those batches: their start event measured
    // ~30 us late in 2000-batch runs)
    static bool select_flush_before(uint32_t b, uint32_t n) { return b > 0 && defer_on() && b % select_ring(n) == 0; }
    // batches per deferred selection launch: up to 64, the models ring held to
    // 2^18 models (14.7 MB)
    static uint32_t select_ring(uint32_t n) { return std::max<uint32_t>(1u, std::min<uint32_t>(64u, (1u << 18) / n)); }
    // GCR_VERIFY_DEFER=0: every fused launch reduces its own batch (A/B)
    static bool defer_on() {
        const char* e = getenv("GCR_VERIFY_DEFER");
        return !(e && e[0] == '0');
    }
    static bool overlap_on() { return verify_overlap_on(); }
    // GCR_FM_PRECONST=0 (read per call): chained launches compute their
    // slots' constants in the prologue instead of copying the look-ahead
    // wave's (A/B)
    static bool preconst_on() {
        const char* e = getenv("GCR_FM_PRECONST");
        return !(e && e[0] == '0');
    }
    // GCR_VERIFY_CHAIN=0: every launch generates its own slots (A/B)
    static bool chain_on() {
        const char* e = getenv("GCR_VERIFY_CHAIN");
        return !(e && e[0] == '0');
    }
    // LO fits on the host; the final hybrid refit solves big systems on the GPU
    static bool fit(gcr_problem* P, const std::vector<uint32_t>* lists, Model& out, bool final_refit) {
        if (!final_refit) return fit_nonminimal(P->solver, P->hc, lists, out);
        GpuSiftSolver gpu(P);
        return fit_nonminimal(P->solver, P->hc, lists, out, &gpu, gpu_refit_rows());
    }
    static void output(const Model& m, double* H, gcr_rect_model* model_out) {
        homography_of(m, H);
        if (model_out) *model_out = gcr_rect_model{m.x0, m.y0, m.s, m.h7, m.h8, m.alpha, m.phi};
    }
};

struct GeoTraits {                 // homography (3) and fundamental matrix (4)
    using Model = GeoModel;
    static constexpr size_t kPer = 1;
    static constexpr bool kFusedVerify = false;   // verify = generation + scoring launches
    static Model def() { return default_geo(); }
    static DevBuf<Model>& dmodels(Workspace* w) { return w->gmodels; }
    static PinBuf<Model>& hmodels(Workspace* w) { return w->h_gmodels; }
    static DevBuf<Model>& pf_dmodels(Workspace* w) { return w->pf_gmodels; }
    static PinBuf<Model>& pf_hmodels(Workspace* w) { return w->pf_h_gmodels; }
    static DevBuf<Model>& lomodels(Workspace* w) { return w->lo_gmodels; }
    static PinBuf<Model>& hlomodels(Workspace* w) { return w->h_logeo; }
    static bool identity(const Model&) { return true; }
    static bool valid(int, const Model&) { return true; }
    static hipError_t generate(gcr_problem* P, uint64_t seed, uint64_t s0, uint32_t n, uint8_t* inc, Model* m,
                               hipStream_t s) {
        return launch_generate_geo(P->dp, seed, s0, n, inc, m, s);
    }
    static hipError_t score(gcr_problem* P, const double T[2], const Model* m, const uint8_t* inc, uint32_t n, bool,
                            const ScoreOut& out, hipStream_t s) {
        return launch_score_geo(P->dp, T[0], m, inc, n, out, s);
    }
    static hipError_t mask(gcr_problem* P, int, const Model& m, int rule, double T, double lambda, uint8_t* mk,
                           hipStream_t s) {
        return launch_mask_geo(P->dp, m, rule, T, lambda, mk, s);
    }
    static hipError_t sqres(gcr_problem* P, const Model& m, double* r2, hipStream_t s) {
        return launch_sqres_geo(P->dp, m, r2, s);
    }
    // One batch = generate (+ compact the live models of multi-model slots)
    // -> score -> first strict best, split in two halves so verify_batches
    // can pipeline them over two streams: batch b + 1 is generated on the side
    // stream while batch b is scored on the main one (the generator is
    // latency-bound at 2 waves per SIMD and co-resides with the scorer's
    // workgroups), each batch in its own buffer set (`set` 0 / 1)
    static constexpr bool kPipe = true;
    struct VBufs {
        uint8_t* inc;
        Model* models;
        uint32_t* hmap;
        uint32_t* hcount;
        ScoreOut sb;
    };
    static VBufs vbufs(gcr_problem* P, int set, uint32_t n) {
        Workspace* w = P->w;
        const size_t nh = (size_t)n * per(P);
        auto& inc = set ? w->pf_inc : w->inc;
        auto& mod = set ? w->pf_gmodels : w->gmodels;
        auto& map = set ? w->pf_hmap : w->hmap;
        auto& cnt = set ? w->pf_hcount : w->hcount;
        auto& sb = set ? w->pf_sb : w->sb;
        inc.ensure(nh);
        mod.ensure(nh);
        sb.ensure(nh);
        if (per(P) > 1) {
            map.ensure(nh);
            cnt.ensure(1);
        }
        return VBufs{inc.p, mod.p, per(P) > 1 ? map.p : nullptr, per(P) > 1 ? cnt.p : nullptr, sb.dev()};
    }
    // Multi-model slots (F) are scored compacted.  launch_score_geo compacts
    // in the feature-major scorer's prologue when it runs at H = 16
    // (split_h) and otherwise with k_compact on the scoring stream; in that
    // case verify_gen compacts instead, behind the generator on its own
    // stream, so that the pipeline's scoring stream goes straight to the
    // scorer (the ~24 us k_compact of a 14848-slot batch overlaps the
    // previous batch's scoring).  GCR_GEN_COMPACT=0 (read per call): the
    // scoring launch compacts.
    static bool gen_compacts(uint32_t nh) {
        const char* e = getenv("GCR_GEN_COMPACT");
        if (e && e[0] == '0') return false;
        return !geo_scorer_scans(nh);
    }
    static hipError_t verify_gen(gcr_problem* P, uint64_t seed, uint64_t s0, uint32_t n, const VBufs& b,
                                 hipStream_t s) {
        hipError_t e = launch_generate_geo(P->dp, seed, s0, n, b.inc, b.models, s);
        const uint32_t nh = n * (uint32_t)per(P);
        if (e == hipSuccess && b.hmap != nullptr && gen_compacts(nh))
            e = launch_compact(b.inc, nh, b.hmap, b.hcount, s);
        return e;
    }
    // rec == nullptr: score only (the ring's deferred selection reduces it)
    static hipError_t verify_score(gcr_problem* P, const double Tm[2], uint64_t s0, uint32_t n, const uint32_t m[2],
                                   BatchRecord* rec, hipEvent_t e0, hipEvent_t e1, const VBufs& b, hipStream_t s) {
        const uint32_t nh = n * (uint32_t)per(P);
        if (e0) (void)hipEventRecord(e0, s);
        hipError_t e = launch_score_geo(P->dp, Tm[0], b.models, b.inc, nh, b.sb, s, b.hmap, b.hcount,
                                        b.hmap != nullptr && !gen_compacts(nh));
        if (e != hipSuccess) return e;
        if (e1) (void)hipEventRecord(e1, s);
        if (rec == nullptr) return hipSuccess;
        return launch_select_geo(P->solver, b.sb, b.inc, nh, s0, m[0], Tm[0], rec, s, b.hmap, b.hcount);
    }
    // deferred selection (GCR_VERIFY_DEFER, default on): the pipelined
    // verify_batches scores batch b into ring set b % R and reduces a whole
    // ring of batches in one launch; R up to 64, the ring held to 2^18
    // hypotheses
    static bool defer_on() {
        const char* e = getenv("GCR_VERIFY_DEFER");
        return !(e && e[0] == '0');
    }
    static uint32_t select_ring(gcr_problem* P, uint32_t n) {
        const uint32_t nh = n * (uint32_t)per(P);
        return std::max<uint32_t>(1u, std::min<uint32_t>(64u, (1u << 18) / nh));
    }
    static VBufs vbufs_ring(gcr_problem* P, uint32_t j, uint32_t R, uint32_t n) {
        Workspace* w = P->w;
        const size_t nh = (size_t)n * per(P);
        w->gr_inc.ensure(R * nh);
        w->gr_models.ensure(R * nh);
        w->gr_n0.ensure(R * nh);
        w->gr_n1.ensure(R * nh);
        w->gr_v0.ensure(R * nh);
        w->gr_v1.ensure(R * nh);
        w->gr_tot.ensure(R * nh);
        const bool cmp = per(P) > 1;
        if (cmp) {
            w->gr_hmap.ensure(R * nh);
            w->gr_hcount.ensure(R);
        }
        const size_t o = j * nh;
        return VBufs{w->gr_inc.p + o, w->gr_models.p + o, cmp ? w->gr_hmap.p + o : nullptr,
                     cmp ? w->gr_hcount.p + j : nullptr,
                     ScoreOut{w->gr_n0.p + o, w->gr_n1.p + o, w->gr_v0.p + o, w->gr_v1.p + o, w->gr_tot.p + o}};
    }
    // one launch for the `count` batches in ring sets 0 .. count - 1
    static hipError_t select_ring_batches(gcr_problem* P, const double Tm[2], uint64_t s0_first, uint32_t n,
                                          const uint32_t m[2], uint32_t count, BatchRecord* rec, hipStream_t s) {
        const VBufs b0 = vbufs_ring(P, 0, 1, n);   // set 0 (already sized)
        const uint32_t nh = n * (uint32_t)per(P);
        return launch_select_geo_batches(P->solver, b0.sb, b0.inc, nh, nh, s0_first, m[0], Tm[0], count, rec, s,
                                         b0.hmap, b0.hcount);
    }
    static hipError_t verify(gcr_problem* P, const double Tm[2], uint64_t seed, uint64_t s0, uint32_t n,
                             const uint32_t m[2], size_t, BatchRecord* rec, hipEvent_t e0, hipEvent_t e1,
                             hipStream_t s, uint32_t = 0, uint32_t = 1) {
        const VBufs b = vbufs(P, 0, n);
        const hipError_t e = verify_gen(P, seed, s0, n, b, s);
        if (e != hipSuccess) return e;
        return verify_score(P, Tm, s0, n, m, rec, e0, e1, b, s);
    }
    static bool select_flush_before(uint32_t, uint32_t) { return false; }   // selection per batch
    // replay-path scoring of a fetched chunk: fundamental-matrix launches are
    // compacted to the live hypotheses (results in hypothesis order); the
    // host counted them (`live`), so the scorer's shape follows the live count
    static hipError_t score_live(gcr_problem* P, const double T[2], const Model* m, const uint8_t* inc, uint32_t nh,
                                 uint32_t live, const ScoreOut& out, hipStream_t s) {
        if (per(P) == 1) return launch_score_geo(P->dp, T[0], m, inc, nh, out, s);
        P->w->hmap.ensure(nh);
        P->w->hcount.ensure(1);
        hipError_t e = launch_compact(inc, nh, P->w->hmap.p, P->w->hcount.p, s);
        if (e != hipSuccess) return e;
        return launch_score_geo(P->dp, T[0], m, inc, std::max<uint32_t>(live, 1u), out, s, P->w->hmap.p,
                                P->w->hcount.p);
    }
    static size_t per(gcr_problem* P) { return P->solver == 4 ? kFModels : 1; }
    static bool fit(gcr_problem* P, const std::vector<uint32_t>* lists, Model& out, bool) {
        if (P->solver == 4) return fit_f8_nonminimal(P->hc[0], lists[0], out);
        return fit_h4_nonminimal(P->hc[0], lists[0], out);
    }
    static void output(const Model& m, double* H, gcr_rect_model*) {
        for (int k = 0; k < 9; ++k) H[k] = m.h[k];
    }
};

struct FundTraits : GeoTraits {     // up to kFModels models per sample
    static constexpr size_t kPer = kFModels;
    // summary replay: the live hypotheses of `nh` positions compacted on the
    // device (hmap / hcount), the scorer sized by nh and cut at *hcount
    static hipError_t score_compact(gcr_problem* P, const double T[2], const Model* m, const uint8_t* inc, uint32_t nh,
                                    uint32_t* hmap, uint32_t* hcount, const ScoreOut& out, hipStream_t s) {
        return launch_score_geo(P->dp, T[0], m, inc, nh, out, s, hmap, hcount, true);
    }
};

constexpr int kMaxLOSample = 64;     // largest LO sample: 7 x the largest minimal sample (7)

template <class Tr>
class RunnerT {
public:
    using Model = typename Tr::Model;
    using Buffer = BufferT<Model>;
    static constexpr size_t kP = Tr::kPer;           // hypotheses per slot
    ~RunnerT() {
        if (pf_active_) (void)hipEventSynchronize(P_->ctx->pdone);     // an exception left one in flight
    }
    RunnerT(gcr_problem* P, const gcr_params& prm) : P_(P), prm_(prm), s_(P->ctx->stream) {
        K_ = P->K;
        m_[0] = P->solver == 2 ? 2 : P->solver == 3 ? 4 : P->solver == 4 ? 7 : 3;
        m_[1] = 2;
        thr_[0] = prm.scale_residual_thresh;
        thr_[1] = prm.orientation_residual_thresh;
        for (int c = 0; c < 2; ++c) {
            Tm_[c] = (2.25 * thr_[c]) * thr_[c];            // MSAC_scoring_function.hpp:64
            const double t = 1.5 * thr_[c];                 // GCRANSAC.h:207-208
            Tlo_[c] = t * t;
        }
        Tu_ = std::max(Tm_[0], Tlo_[0]);
        N_[0] = P->hc[0].n;
        N_[1] = K_ == 2 ? P->hc[1].n : 0;
        log_prob_ = std::log(1.0 - prm.confidence);
        do_lo_ = (prm.flags & GCR_FLAG_NO_LO) == 0;
        std::memset(&st_, 0, sizeof(st_));
        if (kRect && exact_) {
            sbnd_ = score_bound(Tm_, K_);
            // any two scores of the problem: counts at most N_c, scores at most N
            const double nf0 = (double)N_[0], nf1 = (double)N_[1];
            // the best's glibc score is at least every processed hypothesis's,
            // so its value score is within 2 B of their running maximum, and a
            // near tie of it within 4 B: every comparison the reference could
            // decide differently, and every one the host compares in glibc,
            // is a chain member
            if (sbnd_.finite) chain_tol_ = 4.0 * score_dev(sbnd_, nf0, nf1, nf0 + nf1);
        }
    }

    // Shard every chunk over the communicator's ranks, the exchange by
    // ncclAllGather on the device (summary replay only)
    gcr_comm* comm_ = nullptr;
    void set_comm(gcr_comm* c) {
        rank_ = c->rank;
        world_ = c->world;
        comm_ = c;
        compact_ = false;
    }

    // Shard every fetched chunk over `world` ranks.
    void set_sharding(int rank, int world, gcr_allgather_fn fn, void* user) {
        rank_ = rank;
        world_ = world;
        xfn_ = fn;
        xuser_ = user;
        compact_ = false;         // fixed-size per-hypothesis records cross the exchange
    }

    // GCR_CHUNK_LISTS=0: small-scored chunks write no LO list bits (every
    // LO's first round launches its own masks)
    static bool chunk_lists_on() {
        const char* e = getenv("GCR_CHUNK_LISTS");         // read per run
        return !(e && e[0] == '0');
    }
    // GCR_CHUNK_MSAC=0: small-scored chunks mirror no MSAC ballots (the final
    // refit's lists of a chunk-found best come from mask launches)
    static bool chunk_msac_on() {
        const char* e = getenv("GCR_CHUNK_MSAC");          // read per run
        return !(e && e[0] == '0');
    }

    // GCR_LO_REUSE=0: the final refit always rescores the buffer model
    static bool lo_reuse_on() {
        const char* e = getenv("GCR_LO_REUSE");            // read per run
        return !(e && e[0] == '0');
    }
    static bool lo_cache_check_on() {
        const char* e = getenv("GCR_LO_CACHE_CHECK");      // read per run
        return e && e[0] == '1';
    }

    // GCR_SPEC_TRIM=0: speculate even when the chunk's best member already
    // ends the run inside it
    static bool spec_trim_on() {
        const char* e = getenv("GCR_SPEC_TRIM");           // read per run
        return !(e && e[0] == '0');
    }

    // GCR_REPLAY=slots: the per-slot replay of round 2 (every chunk's
    // per-hypothesis records copied back and walked on the host), kept as the
    // A/B reference of the summary replay
    static bool summary_replay_on() {
        const char* e = getenv("GCR_REPLAY");              // read per run (tests switch it)
        return !(e && e[0] == 's');
    }

    void replay_slots() {
        const uint64_t ones[2] = {1, 1};
        uint64_t max_iteration = iteration_number(ones);
        const uint64_t min_it = prm_.min_iteration_number, max_it = prm_.max_iteration_number;
        const uint64_t L = std::max(min_it, max_it);
        uint64_t slot = 0, chunk_begin = 0, chunk_end = 0, chunk_no = 0, last_chunk = 0;
        double replay_ms = 0;
        auto t_rep = Clock::now();
        while (min_it > it_ || it_ < std::min(max_iteration, max_it)) {
            if (slot == chunk_end) {
                replay_ms += ms_since(t_rep);
                const uint64_t B = plan_chunk(chunk_no, last_chunk, it_, L);
                last_chunk = B;
                chunk_begin = slot;
                uint64_t cnt;
                if (pf_active_ && pf_s0_ == slot && pf_B_ == B) {
                    cnt = take_prefetch(L);
                } else {
                    drain_prefetch();
                    cnt = fetch_chunk(slot, (uint32_t)B, L);
                }
                chunk_end = slot + cnt;
                ++chunk_no;
                finish_chunk(cnt);
                plan_prefetch(chunk_no, B, cnt, chunk_end);
                if (pf_pending_ && pf_trigger_ < 0) maybe_prefetch(0, max_iteration, L);
                t_rep = Clock::now();
            }
            const size_t j = slot - chunk_begin;
            bool do_lo = false;
            ++it_;
            const uint8_t inc = P_->w->h_inc.p[j * kP];
            it_ += (uint64_t)inc - 1;
            ++slot;
            // the sample's models in solver order (kP > 1: inc 0 marks an
            // extra model of the same sample, 255 an absent one)
            for (size_t q = 0; inc <= 101 && q < kP; ++q) {
                const size_t hj = j * kP + q;
                if (q > 0 && P_->w->h_inc.p[hj] != 0) break;
                // multi-model slots are scored compacted: results in order
                const size_t si = compact_ ? cursor_++ : hj;
                const Model& model = Tr::hmodels(P_->w).p[hj];
                const uint32_t rn[2] = {P_->w->sb.hn0.p[si], P_->w->sb.hn1.p[si]};
                HScore cur = kP == 1 ? chunk_sc_[j]
                                     : finish(rn, P_->w->sb.hv0.p[si], P_->w->sb.hv1.p[si], P_->w->sb.htot.p[si]);
                Buffer b = gen_buf(model, chunk_begin + j, inc, rn, kRect ? P_->w->sb.hfl.p[si] : 0u);
                if (!b.exact) resolve(b, &cur);         // flagged: the reference's score
                bufs_[off_] = b;
                ++st_.hypotheses;
                if (valid_model(model) &&
                    score_less(best_, [&] { return best_model_; }, cur, [&] { return dec_model(bufs_[off_]); })) {
                    resolve(bufs_[off_]);               // the glibc phi of a generated 2-SIFT model
                    best_model_ = bufs_[off_].model;
                    best_val_ = model;
                    off_ = 1 - off_;
                    best_ = cur;
                    bool nonmin = false;
                    for (int c = 0; c < K_; ++c) if (best_.n[c] > m_[c]) { nonmin = true; break; }
                    do_lo = (it_ > 20) && nonmin;
                    max_iteration = iteration_number(best_.n);
                }
            }
            if (do_lo_ && do_lo) {
                replay_ms += ms_since(t_rep);
                ++lo_number_;
                local_optimization(bufs_[off_]);
                max_iteration = iteration_number(best_.n);
                t_rep = Clock::now();
            }
            // past the chunk's last possible new best (and its LO): the rest
            // of the chunk is bookkeeping, the next chunk can be speculated
            if (pf_pending_ && (int64_t)j == pf_trigger_) maybe_prefetch(j + 1, max_iteration, L);
        }
        replay_ms += ms_since(t_rep);
        st_.slots = slot;
        st_.ms_replay = replay_ms;
    }

    // ---- summary replay (the default) ------------------------------------
    // Each chunk of slots is generated, scored and SUMMARISED on the device
    // (summary.h): its prefix-maximum chain of finished scores with the
    // iteration / hypothesis counts before each member, the totals, and the
    // last live hypothesis.  Only those records come back (a few KB per chunk,
    // one copy into pinned memory), and the replay walks the chain instead of
    // every slot: a strict new best (GCRANSAC.h:440-446) is always a chain
    // member, max_iteration and LO change only there (:467-483), and the loop
    // condition (:286-287) is monotone in the iteration count, so the stop
    // slot is located on the device once the last threshold is known.  A
    // hypothesis-sharded run all-gathers these fixed-size records (SURVEY.md
    // §8(e) row 2) instead of per-hypothesis data.  Chunks run on the side
    // stream (low priority) into two buffer sets, the next one issued before
    // the current one is replayed whenever the loop is certain to reach it
    // (GCR_PREFETCH=0: never), so LO / refit kernels on the replay stream do
    // not queue behind them.  Adaptive runs also issue it speculatively while
    // the current chunk's iterations stay below the stop threshold known
    // before its replay (GCR_SPECULATE=0: never): the device computes the next
    // chunk while the host replays and runs LO on this one, and a chunk the
    // loop never reaches is simply not replayed (slots are pure functions of
    // (seed, slot): results are identical).  Its completion is awaited at the
    // next run's start, not at this run's end.
    struct Chunk {
        uint64_t s0 = 0;          // first slot
        uint32_t B = 0;           // slots of the chunk
        uint32_t per = 0;         // slots per rank block
        uint64_t it_lo = 0;       // iterations before the chunk (exact, or a lower bound when issued ahead)
        int set = 0;              // buffer set
        double bar = 0.0;         // the best score when issued (members beat it)
        uint64_t no = 0;          // chunk number of the run
    };
    bool xlog_ = false;
    void xlog(uint64_t kind, uint64_t no, uint64_t a, uint64_t b) {
        if (xlog_) t_xlog.insert(t_xlog.end(), {kind, no, a, b});
    }
    uint64_t rank_slot0(const Chunk& c, int r) const { return c.s0 + (uint64_t)r * c.per; }
    uint32_t rank_nslots(const Chunk& c, int r) const {
        const uint64_t b = (uint64_t)r * c.per;
        return b >= c.B ? 0u : (uint32_t)std::min<uint64_t>(c.per, c.B - b);
    }
    DevBuf<uint8_t>& set_inc(int set) { return set ? P_->w->pf_inc : P_->w->inc; }
    DevBuf<Model>& set_models(int set) { return set ? Tr::pf_dmodels(P_->w) : Tr::dmodels(P_->w); }
    ScoreBufs& set_sb(int set) { return set ? P_->w->pf_sb : P_->w->sb; }
    DevBuf<uint32_t>& set_hmap(int set) { return set ? P_->w->pf_hmap : P_->w->hmap; }
    DevBuf<uint32_t>& set_hcount(int set) { return set ? P_->w->pf_hcount : P_->w->hcount; }

    // summary launch of this rank's block of chunk c (mode chain or locate)
    hipError_t launch_summary(const Chunk& c, double bar, uint32_t from_pos, uint64_t target, bool parts_ready,
                              BlockSummary* out, hipStream_t s) {
        Workspace* w = P_->w;
        const uint32_t n = rank_nslots(c, rank_);
        const uint32_t m32[2] = {(uint32_t)m_[0], (uint32_t)m_[1]};
        ScoreOut sc = set_sb(c.set).dev();
        if (!chunk_lists_[c.set]) sc.lfl = nullptr;      // list flags exist with the chunk's list bits only
        return launch_block_summary(P_->solver, set_inc(c.set).p, set_models(c.set).p, sc,
                                    kP > 1 ? set_hmap(c.set).p : nullptr, n, (uint32_t)kP, m32, Tm_, bar, from_pos,
                                    target, w->sum_scr[c.set].p, out, s, parts_ready, chain_tol_);
    }

    // generate + score + summarise this rank's block of chunk c on stream s
    void issue_chunk(const Chunk& c, hipStream_t s) {
        Workspace* w = P_->w;
        for (int k = 0; k < 2; ++k) {
            for (hipEvent_t* e : {&w->sum_done[k]})
                if (*e == nullptr) HIPC(hipEventCreateWithFlags(e, hipEventDisableTiming));
            for (hipEvent_t* e : {&w->sum_k0[k], &w->sum_k1[k]})
                if (*e == nullptr) HIPC(hipEventCreate(e));
        }
        const int set = c.set;
        if (lo_row_ >= 0 && lo_row_set_ == set) lo_row_ = -1;   // its list bits are about to be rewritten
        if (msac_row_ >= 0 && msac_row_set_ == set) msac_row_ = -1;
        w->hsum[set].ensure((size_t)world_ + 1);
        w->dsum[set].ensure(1);
        const uint32_t n = rank_nslots(c, rank_);
        if (n == 0) {                                     // an empty block (more ranks than slots)
            if (comm_) {                                  // it still takes part in the exchange
                HIPC(hipMemsetAsync(w->dsum[set].p, 0, sizeof(BlockSummary), s));
                exchange(set, s);
            }
            HIPC(hipEventRecord(w->sum_done[set], s));
            return;
        }
        const size_t np = (size_t)n * kP;
        set_inc(set).ensure(np);
        set_models(set).ensure(np);
        set_sb(set).ensure(np);
        w->sum_scr[set].ensure(summary_scratch_bytes((uint32_t)np, (uint32_t)kP));
        HIPC(Tr::generate(P_, prm_.seed, rank_slot0(c, rank_), n, set_inc(set).p, set_models(set).p, s));
        HIPC(hipEventRecord(w->sum_k0[set], s));
        if constexpr (kP > 1) {
            // multi-model slots: the live hypotheses compacted on the device
            // (k_compact / the scorer's prologue), scores at the live rank
            set_hmap(set).ensure(np);
            set_hcount(set).ensure(1);
            HIPC(Tr::score_compact(P_, Tm_, set_models(set).p, set_inc(set).p, (uint32_t)np, set_hmap(set).p,
                                   set_hcount(set).p, set_sb(set).dev(), s));
        } else {
            if (np <= kSmallScore && small_score_on()) {
                const size_t pairs = small_score_pairs(P_->dp);
                // every slot's LO lists (Tlo, LO rule) into pinned memory: an LO
                // triggered by one of these models starts without its own mask
                // launch and synchronisation
                ListBits lb{{Tlo_[0], Tlo_[1]}, K_ == 2 ? 0 : 2, prm_.spatial_coherence_weight, nullptr, nullptr};
                const bool cl = chunk_lists_on() && world_ == 1 && !(lb.rule == 2 && use_graph());
                if (cl) {
                    w->h_cbits[set].ensure(pairs * kSmallScore / 64);    // sized once
                    void* dptr = nullptr;
                    HIPC(hipHostGetDevicePointer(&dptr, w->h_cbits[set].p, 0));
                    lb.bits = static_cast<uint64_t*>(dptr);
                    // the MSAC ballots as well: a run whose best stays a
                    // hypothesis of this chunk takes its final-refit lists
                    // from them (no mask launches and synchronisation)
                    if (chunk_msac_on()) {
                        w->h_cmbits[set].ensure(pairs * kSmallScore / 64);
                        HIPC(hipHostGetDevicePointer(&dptr, w->h_cmbits[set].p, 0));
                        lb.mbits = static_cast<uint64_t*>(dptr);
                    }
                }
                chunk_lists_[set] = cl;
                chunk_msac_[set] = cl && lb.mbits != nullptr;
                DevProblem dpc = P_->dp;                  // this set's own split-scorer scratch
                if (dpc.lo.vals) {
                    w->cs_vals[set].ensure(pairs * kSplitModels);
                    w->cs_meta[set].ensure(pairs / 64 * kSplitModels);
                    if (!w->cs_arrive[set].p) {
                        w->cs_arrive[set].ensure(kSplitModels);
                        HIPC(hipMemsetAsync(w->cs_arrive[set].p, 0, kSplitModels * sizeof(uint32_t), s));
                    }
                    dpc.lo = SmallScratch{w->cs_vals[set].p, w->cs_meta[set].p, kSplitModels, w->cs_arrive[set].p};
                }
                HIPC(launch_score_small(dpc, Tm_, set_models(set).p, set_inc(set).p, (uint32_t)np,
                                        set_sb(set).dev(), s, cl ? &lb : nullptr));
            } else {
                chunk_lists_[set] = false;
                chunk_msac_[set] = false;
                HIPC(Tr::score(P_, Tm_, set_models(set).p, set_inc(set).p, (uint32_t)np, true, set_sb(set).dev(),
                               s));
            }
        }
        HIPC(hipEventRecord(w->sum_k1[set], s));
        const bool zc = zerocopy_on() && !comm_;          // the exchange reads the device summary
        HIPC(launch_summary(c, c.bar, 0, ~0ull, false, zc ? dev_view(w->hsum[set].p) : w->dsum[set].p, s));
        if (comm_)
            exchange(set, s);
        else if (!zc)
            HIPC(hipMemcpyAsync(w->hsum[set].p, w->dsum[set].p, sizeof(BlockSummary), hipMemcpyDeviceToHost, s));
        HIPC(hipEventRecord(w->sum_done[set], s));
        st_.launches += 5;
        st_.hypotheses_computed += np;
    }

    // gcr_comm: every rank's device summary of set `set` gathered into
    // dall[set] by ncclAllGather on stream s (the same order of collectives
    // on every rank: the replay is identical everywhere), then one copy of the
    // world records into hsum[set][1 ..]
    void exchange(int set, hipStream_t s) {
        Workspace* w = P_->w;
        w->dall[set].ensure((size_t)world_);
        const ncclResult_t r = ncclAllGather(w->dsum[set].p, w->dall[set].p, sizeof(BlockSummary), ncclUint8,
                                             comm_->comm, s);
        if (r != ncclSuccess) throw std::runtime_error(std::string("ncclAllGather: ") + ncclGetErrorString(r));
        HIPC(hipMemcpyAsync(w->hsum[set].p + 1, w->dall[set].p, (size_t)world_ * sizeof(BlockSummary),
                            hipMemcpyDeviceToHost, s));
    }

    // every rank's summary of its block (this rank's: `mine`, the others':
    // the all-gather) into `all` (world records)
    void gather_summaries(const BlockSummary& mine, BlockSummary* all) {
        if (world_ == 1) {
            all[0] = mine;
            return;
        }
        const auto t0 = Clock::now();
        if (xfn_(xuser_, &mine, all, sizeof(BlockSummary)) != 0) throw std::runtime_error("all-gather callback failed");
        st_.ms_score += ms_since(t0);
    }

    static BlockSummary empty_summary() {
        BlockSummary b;
        std::memset(&b, 0, sizeof(b));
        return b;
    }

    // chunk c's summaries of every rank into `all` (waits for this rank's)
    void collect_chunk(const Chunk& c, BlockSummary* all) {
        Workspace* w = P_->w;
        xlog(3, c.no, (uint64_t)c.set, 0);
        const auto t0 = Clock::now();
        if (comm_) comm_sync(w->sum_done[c.set], comm_->comm, "chunk all-gather");
        else HIPC(hipEventSynchronize(w->sum_done[c.set]));
        st_.ms_score += ms_since(t0);
        BlockSummary mine = empty_summary();
        if (rank_nslots(c, rank_) > 0) {
            if (!comm_) mine = w->hsum[c.set].p[0];
            float kms = 0;
            HIPC(hipEventElapsedTime(&kms, w->sum_k0[c.set], w->sum_k1[c.set]));
            st_.ms_score_kernel += kms;
        }
        if (comm_) {                                      // gathered on the device behind the summary
            for (int r = 0; r < world_; ++r) all[r] = w->hsum[c.set].p[1 + r];
            return;
        }
        gather_summaries(mine, all);
    }

    // a collective re-summary of chunk c (every rank calls it) into `all`:
    // the chain of `owner`'s block continued from (from_pos, bar), or
    // (target != null) the locate of target[rank] on every block
    void resummarise(const Chunk& c, int owner, uint32_t from_pos, double bar, const uint64_t* target,
                     BlockSummary* all) {
        Workspace* w = P_->w;
        xlog(2, c.no, (uint64_t)c.set | (target ? 2u : 0u), (uint64_t)(owner + 1) | ((uint64_t)from_pos << 16));
        if (comm_) {
            // the summary (or an empty record) on the replay stream, the
            // exchange on the side stream behind it: every collective of the
            // communicator on one stream, in the same order on every rank
            if (rank_nslots(c, rank_) > 0 && (target != nullptr || owner == rank_)) {
                HIPC(launch_summary(c, bar, target ? 0u : from_pos, target ? target[rank_] : ~0ull, target != nullptr,
                                    w->dsum[c.set].p, s_));
                st_.launches += 2;
            } else {
                HIPC(hipMemsetAsync(w->dsum[c.set].p, 0, sizeof(BlockSummary), s_));
            }
            hipStream_t side = P_->ctx->side;
            HIPC(hipEventRecord(P_->ctx->ev0, s_));
            HIPC(hipStreamWaitEvent(side, P_->ctx->ev0, 0));
            const auto t0 = Clock::now();
            exchange(c.set, side);
            HIPC(hipEventRecord(P_->ctx->ev1, side));
            comm_sync(P_->ctx->ev1, comm_->comm, "re-summary all-gather");
            st_.ms_score += ms_since(t0);
            for (int r = 0; r < world_; ++r) all[r] = w->hsum[c.set].p[1 + r];
            return;
        }
        BlockSummary mine = empty_summary();
        if (rank_nslots(c, rank_) > 0 && (target != nullptr || owner == rank_)) {
            const bool zc = zerocopy_on();
            HIPC(launch_summary(c, bar, target ? 0u : from_pos, target ? target[rank_] : ~0ull, target != nullptr,
                                zc ? dev_view(w->hsum[c.set].p) : w->dsum[c.set].p, s_));
            if (!zc)
                HIPC(hipMemcpyAsync(w->hsum[c.set].p, w->dsum[c.set].p, sizeof(BlockSummary), hipMemcpyDeviceToHost,
                                    s_));
            HIPC(hipStreamSynchronize(s_));
            st_.launches += 2;
            mine = w->hsum[c.set].p[0];
        }
        gather_summaries(mine, all);
    }

    // the model of a summarised hypothesis
    static Model model_of(const SumHyp& h) {
        Model m;
        std::memcpy(&m, h.m, sizeof(Model));
        return m;
    }

    // the hypothesis the inlier buffer holds when the loop leaves a stretch of
    // slots: the last one processed, if it came after the last new best
    // (otherwise the buffer still holds what that new best -- or its LO --
    // left there; GCRANSAC.h:460 writes every hypothesis, :440-446 flips)
    uint64_t ord_last_best_ = 0;          // ordinal + 1 of the last strict new best (0: none)
    void hold_last(const SumHyp& h, uint64_t ord, uint64_t slot) {
        const uint32_t rn[2] = {h.n0, h.n1};
        if (ord + 1 > ord_last_best_) bufs_[off_] = gen_buf(model_of(h), slot, h.inc, rn, h.fl);
    }

    void replay_summaries() {
        // speculative chunks a previous run left in flight (their pinned
        // summary buffers are rewritten below)
        await_spec(P_->w);
        xlog_ = xlog_on();
        if (xlog_) t_xlog.clear();
        const uint64_t ones[2] = {1, 1};
        uint64_t max_iteration = iteration_number(ones);
        const uint64_t min_it = prm_.min_iteration_number, max_it = prm_.max_iteration_number;
        const uint64_t L = std::max(min_it, max_it);
        auto thr = [&]() { return std::max(min_it, std::min(max_iteration, max_it)); };
        const bool ahead_ok = prefetch_on();
        Workspace* w = P_->w;
        double replay_ms = 0;
        uint64_t hyps = 0;                 // live hypotheses before the current chunk
        uint64_t next_slot = 0, chunk_no = 0, last_B = 0;
        std::vector<Chunk> q;              // issued, not yet replayed (at most 2: one per buffer set)
        int next_set = 0;
        std::vector<BlockSummary> S(world_), X(world_);
        std::vector<SumHyp> lasts(world_);
        std::vector<uint8_t> has_last(world_);
        std::vector<uint64_t> itb(world_ + 1), hb(world_ + 1), tgt(world_);
        // plan + issue the chunk after the last issued one; `it_lo`: iterations
        // before it (exact, or a lower bound: every slot adds at least one)
        const bool spec_ok = ahead_ok && speculate_on() && min_it < max_it && prm_.batch_slots == 0;
        auto issue = [&](uint64_t it_lo, bool ahead) -> bool {
            if (it_lo >= L) return false;
            Chunk c;
            c.B = (uint32_t)plan_chunk(chunk_no, last_B, it_lo, L, thr(), next_slot);
            c.s0 = next_slot;
            c.per = (uint32_t)((c.B + world_ - 1) / world_);
            c.it_lo = it_lo;
            c.set = next_set;
            c.bar = best_.sum;
            c.no = chunk_no;
            xlog(1, c.no, (uint64_t)c.set | (ahead ? 2u : 0u), c.B);
            issue_chunk(c, P_->ctx->side);
            next_set ^= 1;
            next_slot += c.B;
            last_B = c.B;
            ++chunk_no;
            q.push_back(c);
            return true;
        };
        while (min_it > it_ || it_ < std::min(max_iteration, max_it)) {
            if (q.empty() && !issue(it_, false)) break;
            const Chunk c = q.front();
            // the chunk after it goes ahead (before this one is replayed) when
            // the loop certainly reaches it: the iteration floor min_it alone
            // keeps the loop going, and every slot adds at least one iteration
            if (ahead_ok && q.size() == 1 && c.it_lo + c.B < min_it && issue(c.it_lo + c.B, true)) ++st_.prefetched_chunks;
            collect_chunk(c, S.data());
            const auto t_rep = Clock::now();
            itb[0] = it_;
            hb[0] = hyps;
            for (int r = 0; r < world_; ++r) {
                itb[r + 1] = itb[r] + S[r].inc_total;
                hb[r + 1] = hb[r] + S[r].hyps_total;
                lasts[r] = S[r].last;
                has_last[r] = S[r].has_last ? 1 : 0;
            }
            // with this chunk's totals known the next one may be certain, or
            // (adaptive runs) likely: below the threshold known before this
            // chunk's replay, which only its new bests can lower
            // A speculative chunk is skipped when this chunk's own best
            // member already brings the threshold inside it (the usual end of
            // a short run): its scoring would occupy the CUs that this
            // chunk's LO and refit kernels need (a ~85 us scorer launch held
            // the LO masks for 60-80 us).  LO rarely raises the threshold
            // again; if it does, the next chunk is issued after the replay.
            // Results are identical either way.
            uint64_t spec_thr = thr();
            if (spec_ok && spec_trim_on())
                for (int r = 0; r < world_; ++r)
                    if (S[r].ncand) {
                        const SumHyp& h = S[r].cand[S[r].ncand - 1];
                        const uint32_t rn[2] = {h.n0, h.n1};
                        const HScore sc = finish(rn, h.v0, h.v1, h.tot);
                        if (best_.sum < sc.sum)
                            spec_thr = std::min(spec_thr, std::max(min_it, iteration_number(sc.n)));
                    }
            if (ahead_ok && q.size() == 1 && (itb[world_] < min_it || (spec_ok && itb[world_] < spec_thr)) &&
                issue(itb[world_], true))
                ++st_.prefetched_chunks;
            bool stopped = false;
            // LO runs once per slot, after all of the slot's models (the
            // last new best of the slot decides, GCRANSAC.h:440-515), before
            // the next slot's loop condition
            uint64_t cur_slot = ~0ull;
            bool slot_lo = false;
            double lo_ms = 0.0;               // LO time inside this chunk's replay (reported as ms_lo)
            auto flush_lo = [&]() {
                if (do_lo_ && slot_lo) {
                    const auto t_lo = Clock::now();
                    ++lo_number_;
                    local_optimization(bufs_[off_]);
                    max_iteration = iteration_number(best_.n);
                    lo_ms += ms_since(t_lo);
                }
                slot_lo = false;
            };
            for (int r = 0; r < world_ && !stopped; ++r) {
                uint32_t k = 0;
                while (true) {
                    if (k == S[r].ncand) {
                        if (!S[r].overflow) break;
                        // more members than one summary holds: the owner
                        // continues the chain from the last one (collective)
                        resummarise(c, r, S[r].resume_pos, S[r].resume_bar, nullptr, X.data());
                        S[r] = X[r];
                        k = 0;
                        continue;
                    }
                    const SumHyp& h = S[r].cand[k++];
                    const uint64_t gslot = rank_slot0(c, r) + h.pos / kP;
                    if (gslot != cur_slot) {
                        flush_lo();
                        cur_slot = gslot;
                        const uint64_t it_before = itb[r] + h.it_before;
                        if (!(min_it > it_before || it_before < std::min(max_iteration, max_it))) {
                            stopped = true;             // the loop ends at or before this member's slot
                            break;
                        }
                        it_ = it_before + h.inc;
                    }
                    const Model model = model_of(h);
                    const uint32_t rn[2] = {h.n0, h.n1};
                    HScore cur = finish(rn, h.v0, h.v1, h.tot);
                    Buffer b = gen_buf(model, gslot, h.inc, rn, h.fl);
                    if (!b.exact) resolve(b, &cur);     // flagged: the reference's score
                    bufs_[off_] = b;
                    if (valid_model(model) &&
                        score_less(best_, [&] { return best_model_; }, cur, [&] { return dec_model(bufs_[off_]); })) {
                        resolve(bufs_[off_]);           // the glibc phi of a generated 2-SIFT model
                        best_model_ = bufs_[off_].model;
                        best_val_ = model;
                        off_ = 1 - off_;
                        best_ = cur;
                        ord_last_best_ = hb[r] + h.hyps_before + 1;
                        // its LO lists are in the chunk's list bits (small-scored chunks)
                        lo_row_ = (kP == 1 && chunk_lists_[c.set]) ? (int64_t)h.pos : -1;
                        lo_row_set_ = c.set;
                        lo_row_model_ = best_model_;
                        lo_row_lfl_ = h.lfl;
                        // ... and its MSAC lists, for the final refit
                        msac_row_ = (kP == 1 && chunk_msac_[c.set]) ? (int64_t)h.pos : -1;
                        msac_row_set_ = c.set;
                        msac_row_model_ = best_model_;
                        msac_row_fl_ = h.fl;
                        bool nonmin = false;
                        for (int cc = 0; cc < K_; ++cc) if (best_.n[cc] > m_[cc]) { nonmin = true; break; }
                        slot_lo = (it_ > 20) && nonmin;
                        max_iteration = iteration_number(best_.n);
                    }
                }
            }
            if (!stopped) flush_lo();
            // past the last member the threshold is fixed: the loop ends in
            // this chunk iff its iterations reach it
            if (!stopped && itb[world_] >= thr()) stopped = true;
            if (stopped) {
                // the first slot after the last member processed whose
                // iterations-before reach the threshold (located on every
                // rank's block, the first rank's wins).  Earlier slots passed
                // the condition under the thresholds of their time, which can
                // be higher (a better score with fewer inliers in one class
                // raises max_iteration); it_ is the count before that first
                // slot and the counts increase strictly, so target max(thr, it_)
                const uint64_t T = std::max(thr(), it_);
                for (int r = 0; r < world_; ++r) tgt[r] = T > itb[r] ? T - itb[r] : 0;
                resummarise(c, -1, 0, 0.0, tgt.data(), X.data());
                int rs = -1;
                for (int r = 0; r < world_; ++r)
                    if (X[r].stop_found) { rs = r; break; }
                if (rs < 0) throw std::runtime_error("summary replay: stop slot not located");
                it_ = itb[rs] + X[rs].stop_it_before;
                st_.slots = rank_slot0(c, rs) + X[rs].stop_slot;
                st_.hypotheses = hb[rs] + X[rs].stop_hyps_before;
                // the last hypothesis processed: before the stop in its block,
                // else the last one of an earlier block of the chunk (earlier
                // chunks were settled at their ends)
                if (X[rs].has_last) {
                    hold_last(X[rs].last, hb[rs] + X[rs].last.hyps_before, rank_slot0(c, rs) + X[rs].last.pos / kP);
                } else {
                    for (int r = rs - 1; r >= 0; --r)
                        if (has_last[r]) {
                            hold_last(lasts[r], hb[r] + lasts[r].hyps_before, rank_slot0(c, r) + lasts[r].pos / kP);
                            break;
                        }
                }
                replay_ms += ms_since(t_rep) - lo_ms;
                break;
            }
            // the whole chunk was processed
            it_ = itb[world_];
            hyps = hb[world_];
            st_.hypotheses = hyps;
            st_.slots = c.s0 + c.B;
            for (int r = world_ - 1; r >= 0; --r)
                if (has_last[r]) {
                    hold_last(lasts[r], hb[r] + lasts[r].hyps_before, rank_slot0(c, r) + lasts[r].pos / kP);
                    break;
                }
            q.erase(q.begin());
            replay_ms += ms_since(t_rep) - lo_ms;
        }
        // chunks issued ahead that the loop never reached: awaited by the
        // next run (above) or the workspace's release
        for (const Chunk& c : q) w->spec_pending[c.set] = true;
        st_.ms_replay = replay_ms;
    }

    // Full GCRANSAC::run; fills outputs, returns total inlier count.
    int run(uint8_t* mask0, uint8_t* mask1, double* H, gcr_rect_model* model_out) {
        const auto t_all = Clock::now();
        if (g_lo_trace) t_run.clear();
        rlot("start");
        await_spec(P_->w);                // either replay path reuses set 0 / 1's buffers
        if (comm_ && !summary_replay_on())
            throw std::runtime_error("GCR_REPLAY=slots exchanges per-hypothesis records: use the callback exchange");
        if (summary_replay_on()) replay_summaries();
        else replay_slots();
        rlot("loop");

        int total = 0;
        Model out_model = Tr::def();
        std::memset(mask0, 0, N_[0]);
        if (K_ == 2 && mask1) std::memset(mask1, 0, N_[1]);
        bool minimal = true;
        for (int c = 0; c < K_; ++c) if (best_.n[c] > m_[c]) minimal = false;
        if (!minimal) {
            if (do_lo_ && lo_number_ == 0) {
                ++lo_number_;
                local_optimization(bufs_[off_]);
                rlot("lo");
            }
            const auto t_ref = Clock::now();
            resolve(bufs_[0]);            // the reference's counts and models in both buffers
            resolve(bufs_[1]);
            rlot("resolved");
            bool diff = false;
            for (int c = 0; c < K_; ++c) if (bufs_[off_].n[c] != best_.n[c]) diff = true;
            if (diff) off_ = 1 - off_;
            diff = false;
            for (int c = 0; c < K_; ++c) if (bufs_[off_].n[c] != best_.n[c]) diff = true;
            // the buffer model's MSAC inlier lists come back with its score
            // when it is (re)scored here (score_models' list bits)
            const ListReq msac{{Tm_[0], Tm_[1]}, 0};
            std::vector<uint32_t> lists[2];
            bool have_lists = false;
            // the adopted LO winner's own scoring launch already gave its
            // score, raw counts and MSAC lists (the launch scores with Tm and
            // mirrored its MSAC ballots): the rescore below would repeat that
            // launch bit for bit
            const bool cached = diff && lo_cache_.valid && lo_reuse_on() &&
                                std::memcmp(&lo_cache_.model, &best_model_, sizeof(Model)) == 0;
            if (cached) {
                best_ = lo_cache_.score;
                lists[0] = lo_cache_.lists[0];
                lists[1] = lo_cache_.lists[1];
                have_lists = true;
                bufs_[off_] = Buffer{true, best_model_, {lo_cache_.raw[0], lo_cache_.raw[1]}};
                if (lo_cache_check_on()) {
                    // the rescore the cache replaces, compared bit for bit
                    HScore s;
                    uint32_t rn[2];
                    std::vector<uint32_t> rl[2];
                    const bool bits = score_models(&best_val_, 1, &s, rn, &msac, &best_model_) && !sm_lbad_[0];
                    if (bits) list_of(0, rl);
                    const bool same = std::memcmp(&s, &best_, sizeof(HScore)) == 0 && rn[0] == lo_cache_.raw[0] &&
                                      rn[1] == lo_cache_.raw[1] && (!bits || (rl[0] == lists[0] && rl[1] == lists[1]));
                    if (!same) throw std::runtime_error("LO cache differs from the refit's rescore (GCR_LO_CACHE_CHECK)");
                }
            } else if (diff) {
                HScore s;
                uint32_t rn[2];
                if (score_models(&best_val_, 1, &s, rn, &msac, &best_model_) && !sm_lbad_[0]) {
                    list_of(0, lists);
                    have_lists = true;
                }
                best_ = s;
                bufs_[off_] = Buffer{true, best_model_, {rn[0], rn[1]}};
            }
            // iteratedLeastSquaresFitting never succeeds (GCRANSAC.h:1092-1098):
            // one non-minimal fit on the buffer's inliers, kept if strictly better.
            rlot("rescored");
            // a best that is still the chunk hypothesis it was found as: its
            // MSAC lists from that chunk's ballots, when none of its decisions
            // was flagged (the same rule as its raw counts, gen_buf)
            if (!have_lists && msac_row_ >= 0 &&
                std::memcmp(&msac_row_model_, &bufs_[off_].model, sizeof(Model)) == 0 &&
                (msac_row_fl_ == 0 || !exact_) && !unsafe(bufs_[off_].model)) {
                decode_lists(P_->w->h_cmbits[msac_row_set_].p, (uint32_t)msac_row_, lists);
                have_lists = true;
                ++st_.chunk_msac_lists;
            }
            if (!have_lists) inlier_lists(bufs_[off_].model, Tm_, 0, lists);
            rlot("lists");
            Model refit;
            const auto t_fit = Clock::now();
            const bool fitted = Tr::fit(P_, lists, refit, true);
            st_.ms_refit_fit = ms_since(t_fit);
            rlot("fit");
            if (fitted) {
                HScore s;
                uint32_t rn[2];
                const bool rl = score_models(&refit, 1, &s, rn, &msac) && !sm_lbad_[0];
                rlot("refit_scored");
                const int idx = 1 - off_;
                bufs_[idx] = Buffer{true, refit, {rn[0], rn[1]}};
                if (score_less(best_, [&] { return best_model_; }, s, [&] { return refit; })) {
                    best_model_ = refit;
                    best_val_ = refit;
                    off_ = idx;
                    if (rl) list_of(0, lists);
                    else inlier_lists(bufs_[off_].model, Tm_, 0, lists);
                }
            }
            for (uint32_t i : lists[0]) mask0[i] = 1;
            if (K_ == 2 && mask1) for (uint32_t i : lists[1]) mask1[i] = 1;
            total = (int)(lists[0].size() + lists[1].size());
            out_model = best_model_;
            st_.score = best_.sum;
            st_.ms_refit = ms_since(t_ref);
            rlot("masks");
        }
        drain_prefetch();                 // the side stream idle before the workspace is reused
        rlot("end");
        lot_print("gcr RUN:", t_run);
        Tr::output(out_model, H, model_out);
        st_.iteration_number = it_;
        st_.local_optimization_number = lo_number_;
        st_.graph_cut_number = gc_number_;
        st_.exact_models = ec_.models;
        st_.exact_pairs = ec_.pairs;
        st_.exact_flips = ec_.flips;
        st_.ms_exact = ec_.ms;
        st_.near_ties = ec_.near_ties;
        st_.near_tie_flips = ec_.near_flips;
        st_.ms_total = ms_since(t_all);
        return total;
    }

    gcr_stats stats() const { return st_; }

    // gcr_debug_score_less: a and b scored by the small scorer, compared as
    // the run loop compares (bit 0 the decision, 1 a near tie, 2 value order)
    int debug_less(const Model& a, const Model& b) {
        const Model ms[2] = {a, b};
        HScore sc[2];
        uint32_t raw[4];
        score_models(ms, 2, sc, raw);
        const uint64_t nt0 = ec_.near_ties;
        const bool d = score_less(sc[0], [&] { return a; }, sc[1], [&] { return b; });
        return (d ? 1 : 0) | (ec_.near_ties > nt0 ? 2 : 0) | (sc[0].sum < sc[1].sum ? 4 : 0);
    }

    // verify_batches' two-stream overlap of the fused launches (see there):
    // chained H = 16 launches with deferred selection, at least 4 batches
    bool overlap_batches(uint32_t nslots, uint32_t nb) const {
        if constexpr (Tr::kFusedVerify)
            return nb >= 4 && Tr::overlap_on() && Tr::defer_on() && Tr::chain_on() && verify_chains(nslots);
        return false;
    }

    // One hot-path batch (bench): generate + score + first strict maximum.
    // `nb` back-to-back batches of `nslots` slots starting at slot0, each
    // generated, scored and reduced to its first strict best on the device by
    // the fused scorer (launch_verify_fused); one host synchronisation at the end.
    void verify_batches(uint64_t slot0, uint32_t nslots, uint32_t nb, gcr_batch_result* out) {
        static_assert(sizeof(BatchRecord) == sizeof(gcr_batch_result), "record layout");
        static_assert(offsetof(BatchRecord, best_model) == offsetof(gcr_batch_result, best_model), "record layout");
        const auto t0 = Clock::now();
        await_spec(P_->w);
        P_->w->inc.ensure(nslots * kP); Tr::dmodels(P_->w).ensure(nslots * kP); P_->w->sb.ensure(nslots * kP);
        // record buffers sized once for up to 4096 batches: a reallocation
        // (device + pinned) inside a timed call costs milliseconds
        constexpr uint32_t kRecMin = 4096;
        P_->w->recs.ensure(std::max(nb, kRecMin));
        P_->w->h_recs.ensure(std::max(nb, kRecMin));

        const uint32_t m32[2] = {(uint32_t)m_[0], (uint32_t)m_[1]};
        const size_t wg_cap = (nslots + 3) / 4;
        P_->w->wg.ensure(wg_cap);
        // the selections write the batch records straight into the mapped
        // pinned buffer (no D2H copy and its ~10 us on the stream at the end
        // of the call); GCR_ZEROCOPY=0 writes them to HBM and copies them
        const bool zc = zerocopy_on();
        BatchRecord* const drecs = zc ? dev_view(P_->w->h_recs.p) : P_->w->recs.p;
        // score-kernel timing events on every `stride`-th batch
        // (GCR_TIMING_STRIDE; default every 4th), at most kMaxTimed evenly
        // spaced batches per call: the event pool is created once and reused
        // (hipEventCreate inside a long queue costs more than the kernels)
        constexpr uint32_t kMaxTimed = 64;
        const uint32_t stride = std::max(timing_stride(), (nb + kMaxTimed - 1) / kMaxTimed);
        const uint32_t ntimed = (nb + stride - 1) / stride;
        while (P_->w->evs.size() < 2 * (size_t)std::max(ntimed, kMaxTimed)) {
            hipEvent_t ev;
            HIPC(hipEventCreate(&ev));
            P_->w->evs.push_back(ev);
        }
        uint32_t timed = 0;
        uint32_t span_launches = 0;              // > 0: evs[0..1] bracket that many launches
        if (Tr::kPipe && nb > 1 && pipe_on()) {
            // two-stream pipeline (Tr::verify_gen / verify_score): generation
            // of batch b on the side stream once batch b - 2 (same buffer set)
            // has been scored; scoring of batch b on s_ once it is generated
            Workspace* w = P_->w;
            for (hipEvent_t* e : {&w->vb_gen[0], &w->vb_gen[1], &w->vb_done[0], &w->vb_done[1], &w->vb_start})
                if (*e == nullptr) HIPC(hipEventCreateWithFlags(e, hipEventDisableTiming));
            if (w->vb_flush == nullptr) HIPC(hipEventCreateWithFlags(&w->vb_flush, hipEventDisableTiming));
            // deferred selection: batch b in ring set b % R, one selection
            // launch per ring (after its last batch); otherwise two buffer
            // sets and a selection launch per batch
            const bool ring = Tr::defer_on();
            const uint32_t R = ring ? Tr::select_ring(P_, nslots) : 2u;
            std::vector<typename Tr::VBufs> bufs(R);
            for (uint32_t j = 0; j < R; ++j)
                bufs[j] = ring ? Tr::vbufs_ring(P_, j, R, nslots) : Tr::vbufs(P_, (int)j, nslots);
            hipStream_t side = P_->ctx->side;
            // overlapped scoring (ring mode, one model per slot: the
            // homography): batch b scored on s_ (b even) or the aux stream
            // (b odd), so one scoring launch's last workgroups share the CUs
            // with the next one's first; a ring's selection on s_ after both;
            // one event pair around the call.  H 6.79 -> 8.77 x 10^7 hyp/s;
            // the fundamental matrix's generator (247 VGPRs) shares the CUs
            // with its scorer, which overlapping only crowds (4.34 -> 4.27)
            const bool ovl = ring && nb >= 4 && Tr::per(P_) == 1 && verify_overlap_on();
            hipStream_t aux = ovl ? aux_stream(P_->ctx) : s_;
            if (ovl) {
                if (w->vb_aux == nullptr) HIPC(hipEventCreateWithFlags(&w->vb_aux, hipEventDisableTiming));
                HIPC(hipEventRecord(P_->w->evs[0], s_));
            }
            HIPC(hipEventRecord(w->vb_start, s_));
            HIPC(hipStreamWaitEvent(side, w->vb_start, 0));
            for (uint32_t b = 0; b < nb; ++b) {
                const int e = (int)(b & 1u);
                const uint32_t k = b % R;
                const uint64_t s0 = slot0 + (uint64_t)b * nslots;
                const bool t = !ovl && b % stride == 0 && !(ring && b > 0 && k == 0) && timed < ntimed;
                hipStream_t sc = (ovl && (b & 1u)) ? aux : s_;
                // generation of batch b overlaps the scoring of batch b - 1
                // only (not further ahead), and reuses a ring set only once
                // the ring's selection has read it
                if (b >= 2) HIPC(hipStreamWaitEvent(side, w->vb_done[e], 0));
                if (ring && b >= R && k == 0) HIPC(hipStreamWaitEvent(side, w->vb_flush, 0));
                HIPC(Tr::verify_gen(P_, prm_.seed, s0, nslots, bufs[k], side));
                HIPC(hipEventRecord(w->vb_gen[e], side));
                HIPC(hipStreamWaitEvent(sc, w->vb_gen[e], 0));
                HIPC(Tr::verify_score(P_, Tm_, s0, nslots, m32, ring ? nullptr : drecs + b,
                                      t ? P_->w->evs[2 * timed] : nullptr, t ? P_->w->evs[2 * timed + 1] : nullptr,
                                      bufs[k], sc));
                HIPC(hipEventRecord(w->vb_done[e], sc));
                if (ring && (k == R - 1 || b + 1 == nb)) {
                    if (ovl) {
                        HIPC(hipEventRecord(w->vb_aux, aux));
                        HIPC(hipStreamWaitEvent(s_, w->vb_aux, 0));
                    }
                    HIPC(Tr::select_ring_batches(P_, Tm_, s0 - (uint64_t)k * nslots, nslots, m32, k + 1,
                                                 drecs + (b - k), s_));
                    HIPC(hipEventRecord(w->vb_flush, s_));
                }
                timed += t;
            }
            if (ovl) {
                HIPC(hipEventRecord(P_->w->evs[1], s_));
                span_launches = nb;
                timed = 1;
            }
        } else if (overlap_batches(nslots, nb)) {
            if constexpr (Tr::kFusedVerify) {
                // two-stream overlap of the fused launches: batch b on s_ (b
                // even) or the side stream (b odd), chained to b + 2 on the
                // same stream.  One launch's workgroups finish unevenly (one
                // per CU, ~0.76 of the launch busy on average, MEASUREMENTS
                // round 6) and the other stream's next launch takes the CUs
                // they free.  A ring's selection runs on s_ after both
                // streams' batches of the ring, and the side stream's first
                // batch after it waits for it (ring slots are reused).  One
                // event pair brackets the whole call: the per-launch time is
                // the span over the launches.
                Workspace* w = P_->w;
                hipStream_t side = aux_stream(P_->ctx);
                for (hipEvent_t* e : {&w->vb_gen[0], &w->vb_gen[1], &w->vb_start, &w->vb_flush})
                    if (*e == nullptr) HIPC(hipEventCreateWithFlags(e, hipEventDisableTiming));
                const uint32_t R = Tr::select_ring(nslots);
                HIPC(hipEventRecord(P_->w->evs[0], s_));
                HIPC(hipEventRecord(w->vb_start, s_));
                HIPC(hipStreamWaitEvent(side, w->vb_start, 0));
                bool side_wait = false;             // the side stream must wait for the last selection
                for (uint32_t b = 0; b < nb; ++b) {
                    const uint32_t k = b % R;
                    const uint64_t s0 = slot0 + (uint64_t)b * nslots;
                    hipStream_t st = (b & 1) ? side : s_;
                    if ((b & 1) && side_wait) {
                        HIPC(hipStreamWaitEvent(side, w->vb_flush, 0));
                        side_wait = false;
                    }
                    HIPC(Tr::verify(P_, Tm_, prm_.seed, s0, nslots, m32, wg_cap, drecs + b, nullptr, nullptr, st, b,
                                    nb, 2));
                    if (k == R - 1 || b + 1 == nb) {
                        HIPC(hipEventRecord(w->vb_gen[1], side));
                        HIPC(hipStreamWaitEvent(s_, w->vb_gen[1], 0));
                        HIPC(Tr::select_flush(P_, s0 - (uint64_t)k * nslots, nslots, k + 1, wg_cap, drecs + (b - k),
                                              s_));
                        HIPC(hipEventRecord(w->vb_flush, s_));
                        side_wait = true;
                    }
                }
                HIPC(hipEventRecord(P_->w->evs[1], s_));
                span_launches = nb;
                timed = 1;
            }
        } else {
            // one event pair around launches 1 .. nb-2 only where each verify
            // is the one fused generate + score launch (rectification): the
            // correspondence verify here also runs its generation kernels,
            // which would count as scoring time
            bool span = Tr::kFusedVerify && nb >= 4 && timing_span();
            for (uint32_t b = 2; span && b + 2 <= nb; ++b)
                if (Tr::select_flush_before(b, nslots)) span = false;    // a selection inside the span
            for (uint32_t b = 0; b < nb; ++b) {
                const uint64_t s0 = slot0 + (uint64_t)b * nslots;
                hipEvent_t e0 = nullptr, e1 = nullptr;
                if (span) {
                    if (b == 1) e0 = P_->w->evs[0];
                    if (b + 2 == nb) e1 = P_->w->evs[1];
                } else if (b % stride == 0 && !Tr::select_flush_before(b, nslots) && timed < ntimed) {
                    e0 = P_->w->evs[2 * timed];
                    e1 = P_->w->evs[2 * timed + 1];
                    ++timed;
                }
                HIPC(Tr::verify(P_, Tm_, prm_.seed, s0, nslots, m32, wg_cap, drecs + b, e0, e1, s_, b, nb));
            }
            if (span) {
                span_launches = nb - 2;
                timed = 1;
            }
        }
        if (!zc)
            HIPC(hipMemcpyAsync(P_->w->h_recs.p, P_->w->recs.p, nb * sizeof(BatchRecord), hipMemcpyDeviceToHost, s_));
        HIPC(hipStreamSynchronize(s_));
        std::memcpy(out, P_->w->h_recs.p, nb * sizeof(BatchRecord));
        float kms_sum = 0;
        for (uint32_t q = 0; q < timed; ++q) {
            float kms = 0;
            HIPC(hipEventElapsedTime(&kms, P_->w->evs[2 * q], P_->w->evs[2 * q + 1]));
            kms_sum += kms;
        }
        // scaled to all batches: the sampled launches' mean (span: the span's
        // time over its launches)
        const double per = span_launches ? (double)span_launches : (double)timed;
        st_.ms_score_kernel += timed ? kms_sum * (double)nb / per : 0.0;
        for (uint32_t b = 0; b < nb; ++b) st_.hypotheses += out[b].models;
        st_.launches += 2 * nb;
        st_.hypotheses_computed += (uint64_t)nslots * nb * kP;
        st_.ms_total += ms_since(t0);
    }

private:
    gcr_problem* P_;
    gcr_params prm_;
    hipStream_t s_;
    int K_;
    uint64_t m_[2];
    double thr_[2], Tm_[2], Tlo_[2];
    uint64_t N_[2];
    double log_prob_;
    bool do_lo_;
    gcr_stats st_;

    uint64_t it_ = 0;
    size_t cursor_ = 0;           // next compacted score of the current chunk
    bool compact_ = kP > 1;       // multi-model slots scored compacted (single rank)
    // one problem over several ranks (gcr_problem_run_sharded)
    int rank_ = 0, world_ = 1;
    gcr_allgather_fn xfn_ = nullptr;
    void* xuser_ = nullptr;
    HScore best_{};
    Model best_model_ = Tr::def();
    Buffer bufs_[2];
    int off_ = 0;
    uint64_t lo_number_ = 0, gc_number_ = 0;
    // the last adopted LO winner: its score, raw counts and MSAC inlier lists
    // (threshold Tm) from its own small-scorer launch, which scored it with Tm
    // and mirrored its MSAC ballots (ListReq::msac) -- any estimator, whenever
    // that launch returned bits and none of the model's MSAC decisions was
    // flagged (lo_lists_from_bits_); the final refit then need not rescore it.
    // GCR_LO_CACHE_CHECK=1 rescores anyway and requires bit-identical results.
    struct LoCache {
        bool valid = false;
        Model model{};
        HScore score{};
        uint32_t raw[2] = {0, 0};
        std::vector<uint32_t> lists[2];
    } lo_cache_;
    bool chunk_lists_[2] = {false, false};    // the set's chunk was small-scored with LO list bits
    int64_t lo_row_ = -1;                       // the last new best's row in those bits (-1: none)
    bool chunk_msac_[2] = {false, false};       // ... and also mirrored its MSAC ballots (h_cmbits)
    int64_t msac_row_ = -1;                     // the last new best's row in the MSAC bits (-1: none)
    int msac_row_set_ = 0;
    Model msac_row_model_{};
    uint32_t msac_row_fl_ = 0;                  // its flagged MSAC decisions in that launch
    int lo_row_set_ = 0;
    Model lo_row_model_{};
    bool lo_lists_from_bits_ = false;     // the current LO winner's lists came from its scoring launch
    std::vector<uint64_t> lo_msac_row_;   // its MSAC list bits (ListBits.mbits row)

    bool valid_model(const Model& m) const { return Tr::valid(P_->solver, m); }

    // ---- decisions in the reference's arithmetic (exact.h) ---------------
    // The kernels decide with the detmath twins and flag every decision within
    // the twin-glibc bound of its threshold (ScoreOut::fl / lfl, k_mask bit
    // 1, SumHyp::fl).  Every hypothesis the replay acts on -- chain members,
    // the buffers, LO winners, the refit -- is then taken in glibc: a flagged
    // score is recounted on the host (exact_score), flagged lists rechecked
    // (exact_mask), and a generated 2-SIFT model carries the glibc phi of its
    // sample (dec_of) wherever the reference would use the model.  The twin
    // phi stays the hypothesis's VALUE model (best_val_): what its MSAC sums
    // were folded with.
    static constexpr bool kRect = std::is_same<Model, RectModel>::value;
    ExactCount ec_;
    double Tu_ = 0.0;                     // the larger scale threshold (scale_unsafe)
    Model best_val_ = Tr::def();          // best_model_ as the kernels score it
    std::vector<uint8_t> sm_mbad_, sm_lbad_;  // score_models: model q's MSAC / list bits need the host
    uint32_t lo_row_lfl_ = 0;             // flagged list decisions of the lo_row_ model in its chunk bits

    const bool exact_ = exact_on();       // GCR_EXACT=0: the twins' decisions throughout (A/B)
    bool unsafe(const Model& m) const {
        if constexpr (kRect) return exact_ && model_unsafe(P_, m, Tu_);
        else return false;
    }
    // a hypothesis of a generated chunk as an inlier buffer, its decisions
    // resolved when the buffer is read
    Buffer gen_buf(const Model& m, uint64_t slot, uint32_t inc, const uint32_t rn[2], uint32_t fl) const {
        Buffer b{true, m, {rn[0], rn[1]}};
        if constexpr (kRect) {
            if (!exact_) return b;
            b.slot = slot;
            b.inc = (P_->solver == 2 && inc >= 1 && inc <= 101) ? inc : 0;
            b.exact = fl == 0 && !unsafe(m);
        }
        return b;
    }
    // the model the reference holds for a generated hypothesis (glibc phi)
    Model dec_of(const Model& m, uint64_t slot, uint32_t inc) const {
        if constexpr (kRect) {
            if (P_->solver == 2 && inc >= 1 && inc <= 101) return glibc_minimal_model(P_, prm_.seed, slot, inc - 1, m);
        }
        return m;
    }
    // the score of value model mv with decision model md's glibc decisions
    HScore exact_score(const Model& mv, const Model& md, uint32_t raw[2], std::vector<uint32_t>* lists = nullptr) {
        if constexpr (kRect) {
            uint32_t n[2];
            double v[2], tot;
            exact_accumulate(P_, mv, md, Tm_, n, v, tot, lists, ec_);
            raw[0] = n[0];
            raw[1] = K_ == 2 ? n[1] : 0;
            return finish(n, v[0], v[1], tot);
        } else {
            (void)mv; (void)md; (void)raw; (void)lists;
            throw std::logic_error("exact_score: rectification solvers only");
        }
    }
    // ---- score comparisons in the reference's arithmetic (exact.h ScoreBound)
    // The reference compares glibc scores (score.hpp:28-36 at GCRANSAC.h:440,
    // :662, :1036, :1054); the engine holds value scores within a proven
    // bound of them.  Two value scores further apart than their two bounds
    // compare the same; a closer pair is compared by its glibc scores, recounted
    // on the host (exact_accumulate, glibc sums).  The device chains keep every
    // hypothesis within chain_tol_ of the running maximum as a member, so the
    // replay sees every possible near tie.
    ScoreBound sbnd_{{0.0, 0.0}, {0.0, 0.0}, 0.0, false};
    double chain_tol_ = 0.0;              // 4 x the bound at full counts (constructor)
    struct GCache {
        Model m;
        double g;
    };
    std::vector<GCache> gcache_;
    double dev_of(const HScore& s) const { return score_dev(sbnd_, (double)s.n[0], (double)s.n[1], s.sum); }
    // the glibc score of decision model md (s: its value score; zero scores
    // -- a class below its minimal sample -- are zero in both arithmetics)
    double glibc_score(const HScore& s, const Model& md) {
        if constexpr (kRect) {
            if (s.total == 0 && s.sum == 0.0) return 0.0;
            for (const GCache& e : gcache_)
                if (std::memcmp(&e.m, &md, sizeof(Model)) == 0) return e.g;
            uint32_t n[2];
            double v[2], tot;
            exact_accumulate(P_, md, md, Tm_, n, v, tot, nullptr, ec_, true);
            const double g = finish(n, v[0], v[1], tot).sum;
            if (gcache_.size() >= 16) gcache_.erase(gcache_.begin());
            gcache_.push_back(GCache{md, g});
            return g;
        } else {
            (void)md;
            return s.sum;
        }
    }
    // the reference's `a < b` on the scores of decision models dec_a(),
    // dec_b() (evaluated only for a near tie)
    template <class FA, class FB>
    bool score_less(const HScore& a, FA&& dec_a, const HScore& b, FB&& dec_b) {
        const bool vl = a.sum < b.sum;
        if constexpr (!kRect) {
            return vl;
        } else {
            if (!exact_ || !sbnd_.finite) return vl;
            const double tol = dev_of(a) + dev_of(b);
            if (!(tol > 0.0) || !(std::fabs(b.sum - a.sum) <= tol)) return vl;
            ++ec_.near_ties;
            const Model ma = dec_a(), mb = dec_b();
            bool gl;
            if (std::memcmp(&ma, &mb, sizeof(Model)) == 0) gl = false;     // one model: equal glibc scores
            else gl = glibc_score(a, ma) < glibc_score(b, mb);
            if (gl != vl) ++ec_.near_flips;
            return gl;
        }
    }
    // the decision model of the hypothesis in an inlier buffer
    Model dec_model(Buffer b) {
        resolve(b);
        return b.model;
    }

    // buffer b with its decisions resolved: a generated model's glibc phi,
    // the reference's counts (*sc: the finished score when recounted)
    void resolve(Buffer& b, HScore* sc = nullptr) {
        if constexpr (kRect) {
            if (!b.has) return;
            const Model mv = b.model;
            if (b.inc) {
                b.model = dec_of(b.model, b.slot, b.inc);
                b.inc = 0;
            }
            if (!b.exact) {
                uint32_t raw[2];
                const HScore s = exact_score(mv, b.model, raw);
                b.n[0] = raw[0];
                b.n[1] = raw[1];
                b.exact = true;
                if (sc) *sc = s;
            }
        } else {
            (void)b; (void)sc;
        }
    }

    // neighbourhood graph (homography / fundamental matrix with a grid and
    // lambda > 0): the grid's edges are built once per run, on first use
    NeighbourEdges edges_;
    std::vector<uint8_t> gc_cseg_;
    std::vector<uint8_t> gc_seg_;
    int graph_state_ = -1;        // -1 unknown, 0 no pairwise terms, 1 edges_ built
    bool use_graph() {
        if (graph_state_ < 0) {
            graph_state_ = 0;
            if (P_->solver >= 3 && prm_.cell_number > 0 && prm_.spatial_coherence_weight > 0) {
                const HostClass& c = P_->hc[0];
                const double* cols[4] = {c.x.data(), c.y.data(), c.a.data(), c.c0.data()};
                // a cell size of 0 (image size unknown to the caller): the
                // column's extent (largest finite coordinate + 1, at least 1)
                // over the cells, as pygcransac.grid_cell_sizes computes it
                double cs[4];
                for (int d = 0; d < 4; ++d) {
                    cs[d] = prm_.cell_size[d];
                    if (cs[d] != 0.0) continue;
                    double top = 0.0;
                    bool any = false;
                    for (size_t i = 0; i < c.n; ++i) {
                        const double v = cols[d][i];
                        if (std::isfinite(v) && (!any || v > top)) {
                            top = v;
                            any = true;
                        }
                    }
                    cs[d] = (any ? std::max(1.0, top + 1.0) : 1.0) / static_cast<double>(prm_.cell_number);
                }
                grid_edges(cols, 4, c.n, cs, prm_.cell_number, edges_, false);
                gc_schedule(edges_, host_pool().threads());
                graph_state_ = edges_.cells() > 0 ? 1 : 0;
            }
        }
        return graph_state_ == 1;
    }

    HScore finish(const uint32_t rn[2], double v0, double v1, double tot) const {
        HScore s;
        s.n[0] = rn[0];
        s.n[1] = K_ == 2 ? rn[1] : 0;
        s.v[0] = v0;
        s.v[1] = K_ == 2 ? v1 : 0.0;
        s.total = s.n[0] + s.n[1];
        s.sum = tot;
        for (int c = 0; c < K_; ++c) {
            if (s.n[c] < m_[c]) return HScore{};
            const double normed = s.v[c] / Tm_[c];
            const double msac = normed + static_cast<double>(s.n[c]);
            s.sum -= s.v[c];
            s.v[c] = msac;
            s.sum += msac;
        }
        return s;
    }

    // GCRANSAC::getIterationNumber (GCRANSAC.h:738-757)
    uint64_t iteration_number(const uint64_t inl[2]) const {
        double q = 1.0;
        for (int c = 0; c < K_; ++c) {
            const double ratio = static_cast<double>(inl[c]) / static_cast<double>(N_[c]);
            q *= std::pow(ratio, static_cast<double>(m_[c]));
        }
        const double lg = std::log(1 - q);
        if (std::fabs(lg) < std::numeric_limits<double>::epsilon()) return std::numeric_limits<uint64_t>::max();
        return static_cast<uint64_t>(std::ceil(log_prob_ / lg));
    }

    // Generate [s0, s0+B), then score only the slots the loop can still reach
    // (iterations can never pass max(min_it, max_it)).  Returns slots scored.
    // One hypothesis of a sharded chunk as it crosses the exchange.
    struct HypRec {
        Model m;
        double v0, v1, tot;
        uint32_t n0, n1;
        uint32_t inc;
        uint32_t fl;
    };

    // Sharded chunk: rank r generates and scores slots [s0 + r per, s0 + (r+1) per)
    // on its own device; the all-gather gives every rank the whole chunk, so
    // every rank replays identically.
    uint64_t fetch_chunk_sharded(uint64_t s0, uint32_t B, uint64_t L) {
        const uint32_t per = (B + world_ - 1) / world_;
        const size_t nh = (size_t)per * kP;
        P_->w->inc.ensure(nh); Tr::dmodels(P_->w).ensure(nh); P_->w->sb.ensure(nh);
        P_->w->h_inc.ensure(nh); Tr::hmodels(P_->w).ensure(nh);
        auto t0 = Clock::now();
        const uint64_t my0 = s0 + (uint64_t)rank_ * per;
        HIPC(Tr::generate(P_, prm_.seed, my0, per, P_->w->inc.p, Tr::dmodels(P_->w).p, s_));
        HIPC(hipEventRecord(P_->ctx->ev0, s_));
        HIPC(Tr::score(P_, Tm_, Tr::dmodels(P_->w).p, P_->w->inc.p, (uint32_t)nh, true, P_->w->sb.dev(), s_));
        HIPC(hipEventRecord(P_->ctx->ev1, s_));
        HIPC(hipMemcpyAsync(P_->w->h_inc.p, P_->w->inc.p, nh, hipMemcpyDeviceToHost, s_));
        P_->w->sb.d2h(nh, s_);
        HIPC(hipMemcpyAsync(Tr::hmodels(P_->w).p, Tr::dmodels(P_->w).p, nh * sizeof(Model), hipMemcpyDeviceToHost,
                            s_));
        HIPC(hipStreamSynchronize(s_));
        float kms = 0;
        HIPC(hipEventElapsedTime(&kms, P_->ctx->ev0, P_->ctx->ev1));
        st_.ms_score_kernel += kms;
        st_.ms_score += ms_since(t0);
        st_.launches += 2;
        st_.hypotheses_computed += nh;
        std::vector<HypRec> send(nh), recv(nh * (size_t)world_);
        const ScoreBufs& sb = P_->w->sb;
        for (size_t i = 0; i < nh; ++i)
            send[i] = HypRec{Tr::hmodels(P_->w).p[i], sb.hv0.p[i], sb.hv1.p[i], sb.htot.p[i],
                             sb.hn0.p[i], sb.hn1.p[i], P_->w->h_inc.p[i], kRect ? sb.hfl.p[i] : 0u};
        t0 = Clock::now();
        if (xfn_(xuser_, send.data(), recv.data(), nh * sizeof(HypRec)) != 0)
            throw std::runtime_error("all-gather callback failed");
        st_.ms_score += ms_since(t0);            // the exchange is part of verification
        const size_t total = nh * (size_t)world_;
        P_->w->h_inc.ensure(total); Tr::hmodels(P_->w).ensure(total); P_->w->sb.ensure(total);
        for (size_t i = 0; i < total; ++i) {
            const HypRec& r = recv[i];
            P_->w->h_inc.p[i] = (uint8_t)r.inc;
            Tr::hmodels(P_->w).p[i] = r.m;
            P_->w->sb.hn0.p[i] = r.n0; P_->w->sb.hn1.p[i] = r.n1;
            P_->w->sb.hv0.p[i] = r.v0; P_->w->sb.hv1.p[i] = r.v1; P_->w->sb.htot.p[i] = r.tot;
            P_->w->sb.hfl.p[i] = r.fl;
        }
        const uint64_t Bw = (uint64_t)per * world_;
        uint64_t itp = it_, cnt = 0;
        while (cnt < Bw && itp < L) itp += P_->w->h_inc.p[kP * cnt++];
        if (cnt == 0) cnt = 1;
        return cnt;
    }

    // Fundamental matrix (kP models per slot, compacted to the live ones): the
    // batch scorer runs one workgroup of split_h(live) hypotheses per CU, so a
    // chunk whose live count spills a little past whole waves of workgroups
    // pays a whole extra wave (4382 live at 4096 slots: 274 workgroups on 256
    // CUs, 182 us instead of ~90).  Score only the slots that fill whole waves
    // when the last wave would be less than half full; the next chunk
    // regenerates the rest (a slot is a pure function of (seed, slot), so
    // results do not depend on the cut).  `live` returns the scored count.
    uint64_t whole_waves(uint64_t cnt, uint64_t& live) {
        const uint8_t* inc = P_->w->h_inc.p;
        auto live_of = [&](uint64_t c) {
            uint64_t l = 0;
            for (uint64_t j = 0; j < c * kP; ++j) l += inc[j] <= 101;
            return l;
        };
        live = live_of(cnt);
        const uint64_t cap = (uint64_t)split_h((uint32_t)std::min<uint64_t>(live, UINT32_MAX)) * P_->ctx->n_cu;
        const uint64_t waves = (live + cap - 1) / cap;
        if (waves < 2 || live - (waves - 1) * cap > cap / 2) return cnt;
        const uint64_t target = (waves - 1) * cap;
        uint64_t c = 0, l = 0;
        while (c < cnt) {
            uint64_t add = 0;
            for (size_t k = 0; k < kP; ++k) add += inc[c * kP + k] <= 101;
            if (l + add > target) break;
            l += add;
            ++c;
        }
        if (c == 0) return cnt;
        live = l;
        return c;
    }

    uint64_t fetch_chunk(uint64_t s0, uint32_t B, uint64_t L) {
        if (world_ > 1) return fetch_chunk_sharded(s0, B, L);
        const size_t BP = (size_t)B * kP;
        P_->w->inc.ensure(BP); Tr::dmodels(P_->w).ensure(BP); P_->w->sb.ensure(BP);
        P_->w->h_inc.ensure(BP); Tr::hmodels(P_->w).ensure(BP);
        auto t0 = Clock::now();
        HIPC(Tr::generate(P_, prm_.seed, s0, B, P_->w->inc.p, Tr::dmodels(P_->w).p, s_));
        HIPC(hipMemcpyAsync(P_->w->h_inc.p, P_->w->inc.p, BP, hipMemcpyDeviceToHost, s_));
        HIPC(hipStreamSynchronize(s_));
        st_.ms_generate += ms_since(t0);
        uint64_t itp = it_, cnt = 0;
        while (cnt < B && itp < L) itp += P_->w->h_inc.p[kP * cnt++];
        if (cnt == 0) cnt = 1;
        uint64_t live = cnt * kP;
        if (kP > 1) cnt = whole_waves(cnt, live);
        const size_t nh = cnt * kP;
        t0 = Clock::now();
        HIPC(hipEventRecord(P_->ctx->ev0, s_));
        if (kP == 1 && nh <= kSmallScore && small_score_on()) {
            // the few slots a short run needs: all pairs in parallel, one
            // wave per model (the batch scorers' chain would dominate)
            HIPC(launch_score_small(P_->dp, Tm_, Tr::dmodels(P_->w).p, P_->w->inc.p, (uint32_t)nh, P_->w->sb.dev(),
                                    s_));
        } else {
            HIPC(Tr::score_live(P_, Tm_, Tr::dmodels(P_->w).p, P_->w->inc.p, (uint32_t)nh, (uint32_t)live,
                                P_->w->sb.dev(), s_));
        }
        cursor_ = 0;
        HIPC(hipEventRecord(P_->ctx->ev1, s_));
        P_->w->sb.d2h(nh, s_);
        HIPC(hipMemcpyAsync(Tr::hmodels(P_->w).p, Tr::dmodels(P_->w).p, nh * sizeof(Model), hipMemcpyDeviceToHost,
                            s_));
        HIPC(hipStreamSynchronize(s_));
        float kms = 0;
        HIPC(hipEventElapsedTime(&kms, P_->ctx->ev0, P_->ctx->ev1));
        st_.ms_score_kernel += kms;
        st_.ms_score += ms_since(t0);
        st_.launches += 2;
        st_.hypotheses_computed += nh;
        return cnt;
    }

    // Chunk sizes: a fixed budget (min >= max) runs 65536-slot chunks; an
    // adaptive run starts with kSmallScore slots (the small-batch scorer; a
    // 0.99-confidence run at 50 % outliers needs 35-90) and grows x4; never
    // past the budget L from iteration count `it`.
    // `thr`: the loop's current stop threshold, `slots_done`: slots before
    // the chunk (summary replay; 0 = no estimate)
    uint64_t plan_chunk(uint64_t chunk_no, uint64_t last_chunk, uint64_t it, uint64_t L, uint64_t thr = ~0ull,
                        uint64_t slots_done = 0) const {
        const uint64_t min_it = prm_.min_iteration_number, max_it = prm_.max_iteration_number;
        uint64_t B;
        if (prm_.batch_slots) B = prm_.batch_slots;
        else if (min_it >= max_it) B = 65536;
        else B = chunk_no == 0 ? first_chunk() : std::min<uint64_t>(65536, last_chunk * 4);
        // adaptive runs: no more slots than the current threshold is expected
        // to need (iterations per slot so far, + 25 %), so the chunk that ends
        // the run does not compute tens of thousands of slots past the stop
        // (F at configs[3]: ~8 iterations a slot, the last 4x-grown chunk was
        // 65536 slots for ~20 000 needed).  The threshold only falls as bests
        // improve (barring rare rises, which another chunk absorbs).
        // GCR_CHUNK_CAP=0 disables.
        if (!prm_.batch_slots && min_it < max_it && slots_done > 0 && it > 0 && thr > it && chunk_cap_on()) {
            const double per = (double)it / (double)slots_done;
            const double need = (double)(thr - it) / per * 1.25 + 64.0;
            if (need < (double)B) B = std::max<uint64_t>((uint64_t)need, kSmallScore);
        }
        B = std::min<uint64_t>(B, L > it ? L - it : 0);
        B = std::min<uint64_t>(B, (uint64_t)262144 * world_);      // a block summary covers <= 2^18 slots
        return std::max<uint64_t>(B, 1);
    }

    // ---- next chunk on the side stream (north_star's side stream) ----------
    // While the host replays the rest of chunk c, the side stream generates and
    // scores chunk c + 1 into the second set of chunk buffers.  Slots are pure
    // functions of (seed, slot), so the prefetched results are exactly what a
    // fetch would return; the budget cut is applied on the device
    // (launch_truncate).  Started only past chunk c's last possible new best,
    // and only when the loop will reach chunk c + 1, so nothing is wasted and
    // no LO / refit kernel waits behind it.  One-model slots on one rank, from
    // the second chunk on.  GCR_PREFETCH=0 disables.
    bool pf_active_ = false;
    uint64_t pf_s0_ = 0, pf_B_ = 0;

    // slots of an adaptive run's first chunk: 128 (GCR_FIRST_CHUNK=n, 1 ..
    // 256).  The bench problems end within 13-83 slots; against 256, the
    // small scorer's pair launch halves (M2 / M1 / H latency to 0.99 -10 to
    // -40 us per seed, tools/lat_seeds.py, profiles/r3_fc_seeds_*.log), and
    // long runs (F) take one more, speculatively issued, chunk
    static uint64_t first_chunk() {
        const char* e = getenv("GCR_FIRST_CHUNK");           // read per run
        const long v = e ? atol(e) : 0;
        return (v >= 1 && v <= (long)kSmallScore) ? (uint64_t)v : (uint64_t)128;
    }
    static bool prefetch_on() {
        const char* e = getenv("GCR_PREFETCH");              // read per run (tests switch it)
        return !(e && e[0] == '0');
    }
    static bool speculate_on() {
        const char* e = getenv("GCR_SPECULATE");
        return !(e && e[0] == '0');
    }
    static bool chunk_cap_on() {
        const char* e = getenv("GCR_CHUNK_CAP");
        return !(e && e[0] == '0');
    }
    // GCR_VERIFY_PIPE=0: verify_batches on one stream (A/B of the pipeline)
    static bool pipe_on() {
        const char* e = getenv("GCR_VERIFY_PIPE");
        return !(e && e[0] == '0');
    }

    // At a chunk's fetch: where the replay may still find a new best (the last
    // slot whose score beats the running maximum from best_ with a valid
    // model -- an LO can only raise the bar, so no later slot can trigger
    // one).  The speculation starts after that slot, so it never competes
    // with an LO's or the final refit's kernels.
    bool pf_pending_ = false;
    int64_t pf_trigger_ = -1;
    uint64_t pf_chunk_no_ = 0, pf_chunk_B_ = 0, pf_chunk_cnt_ = 0, pf_next_s_ = 0;
    // one-model slots: every slot's finished MSAC score, computed once per
    // chunk on the host pool (the replay reads them; so does plan_prefetch)
    std::vector<HScore> chunk_sc_;
    std::vector<uint8_t> chunk_ok_;       // a model that passes isValidModel
    void finish_chunk(uint64_t cnt) {
        if (kP != 1) return;
        chunk_sc_.resize(cnt);
        chunk_ok_.resize(cnt);
        auto body = [&](size_t lo, size_t hi) {
            for (size_t j = lo; j < hi; ++j) {
                if (P_->w->h_inc.p[j] > 101) {
                    chunk_sc_[j] = HScore{};
                    chunk_ok_[j] = 0;
                    continue;
                }
                const uint32_t rn[2] = {P_->w->sb.hn0.p[j], P_->w->sb.hn1.p[j]};
                chunk_sc_[j] = finish(rn, P_->w->sb.hv0.p[j], P_->w->sb.hv1.p[j], P_->w->sb.htot.p[j]);
                chunk_ok_[j] = valid_model(Tr::hmodels(P_->w).p[j]) ? 1 : 0;
            }
        };
        const size_t parts = cnt >= 8192 ? 16 : 1;
        const size_t step = (cnt + parts - 1) / parts;
        host_pool().parallel_for(parts, [&](size_t p) { body(std::min(cnt, p * step), std::min(cnt, (p + 1) * step)); });
    }
    void plan_prefetch(uint64_t chunk_no, uint64_t B, uint64_t cnt, uint64_t s_next) {
        pf_pending_ = false;
        if (kP != 1 || world_ > 1 || chunk_no < 2 || cnt != B || !prefetch_on()) return;
        double run = best_.sum;
        int64_t trig = -1;
        for (uint64_t j = 0; j < cnt; ++j) {
            // a flagged slot may be a new best whatever its twin score (exact.h)
            const bool fl = kRect && exact_ && P_->w->sb.hfl.p[j] != 0;
            // (or a near tie of the running maximum: compared in glibc)
            if ((run - chain_tol_ < chunk_sc_[j].sum || fl) && chunk_ok_[j]) {
                if (!fl && run < chunk_sc_[j].sum) run = chunk_sc_[j].sum;
                trig = (int64_t)j;
            }
        }
        pf_pending_ = true;
        pf_trigger_ = trig;
        pf_chunk_no_ = chunk_no;
        pf_chunk_B_ = B;
        pf_chunk_cnt_ = cnt;
        pf_next_s_ = s_next;
    }

    // `from`: the first slot of the current chunk not yet replayed; it_ holds
    // the iterations up to it.  Speculates only when the loop will certainly
    // reach the next chunk (max_iteration no longer changes in this chunk).
    void maybe_prefetch(uint64_t from, uint64_t max_iteration, uint64_t L) {
        pf_pending_ = false;
        uint64_t it_end = it_;
        for (uint64_t j = from; j < pf_chunk_cnt_; ++j) it_end += P_->w->h_inc.p[j];
        const uint64_t min_it = prm_.min_iteration_number, max_it = prm_.max_iteration_number;
        if (getenv("GCR_DEBUG_PF"))
            fprintf(stderr, "pf: chunk %lu from %lu/%lu it_end %lu max_iteration %lu L %lu\n",
                    (unsigned long)pf_chunk_no_, (unsigned long)from, (unsigned long)pf_chunk_cnt_,
                    (unsigned long)it_end, (unsigned long)max_iteration, (unsigned long)L);
        if (!(min_it > it_end || it_end < std::min(max_iteration, max_it)) || it_end >= L) return;
        const uint64_t Bn = plan_chunk(pf_chunk_no_, pf_chunk_B_, it_end, L);
        if (Bn <= kSmallScore) return;
        const uint64_t s_next = pf_next_s_;
        Workspace* w = P_->w;
        w->pf_inc.ensure(Bn); Tr::pf_dmodels(w).ensure(Bn); w->pf_sb.ensure(Bn);
        w->pf_h_inc.ensure(Bn); Tr::pf_hmodels(w).ensure(Bn);
        hipStream_t s = P_->ctx->side;
        HIPC(Tr::generate(P_, prm_.seed, s_next, (uint32_t)Bn, w->pf_inc.p, Tr::pf_dmodels(w).p, s));
        HIPC(launch_truncate(w->pf_inc.p, (uint32_t)Bn, L - it_end, s));
        HIPC(hipEventRecord(P_->ctx->pev0, s));
        HIPC(Tr::score_live(P_, Tm_, Tr::pf_dmodels(w).p, w->pf_inc.p, (uint32_t)Bn, (uint32_t)Bn, w->pf_sb.dev(), s));
        HIPC(hipEventRecord(P_->ctx->pev1, s));
        HIPC(hipMemcpyAsync(w->pf_h_inc.p, w->pf_inc.p, Bn, hipMemcpyDeviceToHost, s));
        w->pf_sb.d2h(Bn, s);
        HIPC(hipMemcpyAsync(Tr::pf_hmodels(w).p, Tr::pf_dmodels(w).p, Bn * sizeof(Model), hipMemcpyDeviceToHost, s));
        HIPC(hipEventRecord(P_->ctx->pdone, s));
        pf_active_ = true;
        pf_s0_ = s_next;
        pf_B_ = Bn;
        st_.launches += 3;
        st_.hypotheses_computed += Bn;
        ++st_.prefetched_chunks;
    }

    // the prefetched chunk becomes the current one; returns its slot count
    // (the budget cut, as fetch_chunk computes it)
    uint64_t take_prefetch(uint64_t L) {
        auto t0 = Clock::now();
        HIPC(hipEventSynchronize(P_->ctx->pdone));
        pf_active_ = false;
        Workspace* w = P_->w;
        swap_buf(w->inc, w->pf_inc);
        swap_buf(Tr::dmodels(w), Tr::pf_dmodels(w));
        swap_buf(w->h_inc, w->pf_h_inc);
        swap_buf(Tr::hmodels(w), Tr::pf_hmodels(w));
        w->sb.swap(w->pf_sb);
        float kms = 0;
        HIPC(hipEventElapsedTime(&kms, P_->ctx->pev0, P_->ctx->pev1));
        st_.ms_score_kernel += kms;
        st_.ms_score += ms_since(t0);                    // the wait that remained
        cursor_ = 0;
        uint64_t itp = it_, cnt = 0;
        while (cnt < pf_B_ && itp < L) itp += w->h_inc.p[cnt++];
        return cnt == 0 ? 1 : cnt;
    }

    void drain_prefetch() {
        if (!pf_active_) return;
        HIPC(hipEventSynchronize(P_->ctx->pdone));
        pf_active_ = false;
    }

    // Score explicit host models on the GPU (LO trials, refit, reconcile).
    // Scores of n models.  With `req` (thresholds + mask rule of an
    // inlier_lists call) the small scorer also evaluates that list predicate
    // on every pair and copies the bits back with the scores: returns true
    // and list_of(q, ...) then yields model q's inlier lists without another
    // launch + synchronisation.  False: no bits (batch-scorer path).
    struct ListReq {
        double T[2];
        int rule;
        bool msac = false;        // also the MSAC ballots (mlist_of)
    };
    // `decs` (rectification): each model's decision model when it differs
    // from the one scored (a generated 2-SIFT model's glibc phi); a model with
    // flagged decisions, or one exact.h's bound does not cover, is rescored in
    // the reference's decisions on the host, and its list / MSAC bits marked
    // unusable (sm_lbad_ / sm_mbad_)
    // Parts (LO trials scored while later trials are still being fitted,
    // local_optimization): with score_parts_ok(n) a call with launch_only
    // launches the residuals of models [first, n) and returns; the next call
    // (same req, first = the models already launched) launches the rest and
    // the fold of all n, waits and finishes all n.
    bool score_parts_ok(uint32_t n) const {
        if constexpr (!kRect) {
            (void)n;
            return false;
        } else {
            return n <= kSmallScore && n <= kArgModels && small_score_on() && zerocopy_on() && done_wait_on() &&
                   lo_pipe_on() && score_small_splits(P_->dp, n);
        }
    }
    // GCR_LO_PIPE=1: LO trials scored in two parts while the second half is
    // fitted -- measured no faster on MI355X (session r5_s13: the first
    // part's residual launch reaches the GPU only with the second's), so off
    static bool lo_pipe_on() {
        const char* e = getenv("GCR_LO_PIPE");                // read per call
        return e && e[0] == '1';
    }
    bool score_models(const Model* models, uint32_t n, HScore* out, uint32_t* raw_n /* 2 per model */,
                      const ListReq* req = nullptr, const Model* decs = nullptr, uint32_t first = 0,
                      bool launch_only = false) {
        auto& lm = Tr::lomodels(P_->w);
        lm.ensure(n);
        P_->w->lo_sb.ensure(n);
        bool identity = true;
        for (uint32_t i = 0; i < n; ++i) identity = identity && Tr::identity(models[i]);
        const bool small = identity && n <= kSmallScore && small_score_on();
        // small batches: models read from pinned memory and results written
        // into the pinned mirror by the kernels (no copy launches either way)
        const bool zc = small && zerocopy_on();
        const bool parts = (first > 0 || launch_only) && zc && score_parts_ok(n);
        if ((first > 0 || launch_only) && !parts)
            throw std::logic_error("score_models: parts without score_parts_ok");
        const Model* dmodels = lm.p;
        if (zc) {
            auto& hm = Tr::hlomodels(P_->w);
            hm.ensure(kSmallScore);                  // sized once (a pinned reallocation costs milliseconds)
            std::memcpy(hm.p + first, models + first, (n - first) * sizeof(Model));
            dmodels = dev_view(hm.p);
        } else {
            HIPC(hipMemcpyAsync(lm.p, models, n * sizeof(Model), hipMemcpyHostToDevice, s_));
        }
        bool lists = false;
        if (small) {
            // a few models: all pairs in parallel, then one wave per model
            // adds its inliers in order (no ~90 us batch-scorer chain)
            const size_t pairs = small_score_pairs(P_->dp);
            // the graph-cut labeling with pairwise terms needs the residuals
            lists = req != nullptr && !(req->rule == 2 && use_graph());
            ListBits lb{{0.0, 0.0}, 0, prm_.spatial_coherence_weight, nullptr, nullptr};
            if (lists) {
                // sized once for the largest small-scorer launch (a pinned
                // reallocation costs milliseconds)
                P_->w->h_lbits.ensure(pairs * kSmallScore / 64);
                void* dptr = nullptr;
                HIPC(hipHostGetDevicePointer(&dptr, P_->w->h_lbits.p, 0));
                lb.T[0] = req->T[0];
                lb.T[1] = req->T[1];
                lb.rule = req->rule;
                lb.bits = static_cast<uint64_t*>(dptr);
                if (req->msac) {
                    // the MSAC ballots as well (the final refit's lists of an
                    // adopted LO winner, without rescoring it)
                    P_->w->h_mbits.ensure(pairs * kSmallScore / 64);
                    HIPC(hipHostGetDevicePointer(&dptr, P_->w->h_mbits.p, 0));
                    lb.mbits = static_cast<uint64_t*>(dptr);
                }
            }
            ScoreOut so = zc ? P_->w->lo_sb.host_dev() : P_->w->lo_sb.dev();
            if (parts) {
                // stage 1: the residuals of models [first, n) (from their
                // own pinned slots / kernel arguments); stage 2 (the final
                // call): the fold of all n
                if (launch_only) {
                    HIPC(launch_score_small_part(P_->dp, Tm_, dmodels + first, first, n - first, 1, 0, so, s_,
                                                 lists ? &lb : nullptr, models + first));
                    return false;
                }
                P_->w->lo_done.ensure(kSmallScore);
                so.done = dev_view(P_->w->lo_done.p);
                so.epoch = ++P_->w->done_epoch;
                if (so.epoch == 0) so.epoch = ++P_->w->done_epoch;
                HIPC(launch_score_small_part(P_->dp, Tm_, dmodels + first, first, n - first, 3, n, so, s_,
                                             lists ? &lb : nullptr, models + first));
                wait_done(P_->w->lo_done.p, n, so.epoch);
                goto scored;
            }
            if (zc && done_wait_on()) {
                P_->w->lo_done.ensure(kSmallScore);             // sized once
                so.done = dev_view(P_->w->lo_done.p);
                so.epoch = ++P_->w->done_epoch;
                if (so.epoch == 0) so.epoch = ++P_->w->done_epoch;     // 0 never marks a model done
            }
            lot("setup");
            HIPC(launch_score_small(P_->dp, Tm_, dmodels, nullptr, n, so, s_, lists ? &lb : nullptr,
                                    kRect ? static_cast<const void*>(models) : nullptr));
            lot("launched");
            if (so.done) {
                wait_done(P_->w->lo_done.p, n, so.epoch);
                goto scored;
            }
        } else {
            HIPC(Tr::score(P_, Tm_, lm.p, nullptr, n, identity, P_->w->lo_sb.dev(), s_));
        }
        if (!zc) P_->w->lo_sb.d2h(n, s_);
        HIPC(hipStreamSynchronize(s_));
    scored:
        lot("waited");
        st_.launches += 1;
        finish_small(models, n, out, raw_n, decs, lists);
        lot("finished");
        return lists;
    }

    // the scores of a small-scorer launch (lo_sb): finished, flagged
    // decisions and models exact.h does not cover recounted on the host
    // (sm_mbad_), flagged list decisions marked (sm_lbad_)
    void finish_small(const Model* models, uint32_t n, HScore* out, uint32_t* raw_n, const Model* decs, bool lists) {
        sm_mbad_.assign(n, 0);
        sm_lbad_.assign(n, 0);
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t rn[2] = {P_->w->lo_sb.hn0.p[i], P_->w->lo_sb.hn1.p[i]};
            out[i] = finish(rn, P_->w->lo_sb.hv0.p[i], P_->w->lo_sb.hv1.p[i], P_->w->lo_sb.htot.p[i]);
            raw_n[2 * i] = rn[0];
            raw_n[2 * i + 1] = K_ == 2 ? rn[1] : 0;
            if constexpr (kRect) {
                if (!exact_) continue;
                const Model& md = decs ? decs[i] : models[i];
                const bool bad = unsafe(md);
                if (P_->w->lo_sb.hfl.p[i] != 0 || bad) {
                    uint32_t raw[2];
                    out[i] = exact_score(models[i], md, raw);
                    raw_n[2 * i] = raw[0];
                    raw_n[2 * i + 1] = raw[1];
                    sm_mbad_[i] = 1;
                }
                if (lists && (P_->w->lo_sb.hlfl.p[i] != 0 || bad)) sm_lbad_[i] = 1;
            }
        }
    }

    // ---- LO trials with approximate scores (GCR_LO_APPROX=0: off) --------
    // The split scorer's residual launch plus k_lo_approx instead of the
    // exact fold: exact counts, class sums in a tree order.  A trial
    // comparison is decided on them when the bound below cannot change it;
    // a round with one that can is refolded exactly.  The round's winner is
    // folded exactly behind the round (launch_lo_fold_slots into lo_wb) and
    // its exact score replaces the approximate one before the next round's
    // comparisons -- by then the stream has run the fold.
    // GCR_LO_APPROX: 0 off, 2 every round refolded exactly (tests)
    static int lo_approx_mode() {
        const char* e = getenv("GCR_LO_APPROX");             // read per call
        return !e ? 1 : e[0] == '0' ? 0 : e[0] == '2' ? 2 : 1;
    }
    bool approx_ok(uint32_t n) const {
        if constexpr (!kRect) {
            (void)n;
            return false;
        } else {
            return n <= kSmallScore && n <= kArgModels && small_score_on() && zerocopy_on() && done_wait_on() &&
                   lo_approx_mode() != 0 && P_->dp.lo.psum != nullptr && score_small_splits(P_->dp, n);
        }
    }
    // the list bits of a small-scorer launch (ListReq), in the mapped pinned
    // buffers sized once for the largest launch
    ListBits list_bits(const ListReq& req) {
        const size_t pairs = small_score_pairs(P_->dp);
        ListBits lb{{req.T[0], req.T[1]}, req.rule, prm_.spatial_coherence_weight, nullptr, nullptr};
        P_->w->h_lbits.ensure(pairs * kSmallScore / 64);
        lb.bits = dev_view(P_->w->h_lbits.p);
        if (req.msac) {
            P_->w->h_mbits.ensure(pairs * kSmallScore / 64);
            lb.mbits = dev_view(P_->w->h_mbits.p);
        }
        return lb;
    }
    // a bound on |approximate - exact| of a finished score (value arithmetic):
    // each class sum within (n + 64) u |v| of the other order's (both within
    // (n - 1) u sum|a| of the real sum, sum|a| = |real sum| for non-positive
    // values), the total likewise, and finish()'s rounding on both sides;
    // doubled
    double approx_err(const HScore& s, double v0, double v1, double tot) const {
        constexpr double u = 0x1p-53;
        const double v[2] = {v0, v1};
        double e = 0.0, b = std::fabs(tot);
        double esum = 0.0;
        for (int c = 0; c < K_; ++c) {
            const double ec = 2.0 * ((double)s.n[c] + 64.0) * u * std::fabs(v[c]);
            const double g = 1.0 + 1.0 / Tm_[c];
            e += ec * g;
            esum += std::fabs(v[c]);
            b += (std::fabs(v[c]) + ec) * g + (double)s.n[c];
        }
        const double etot = 2.0 * ((double)(s.n[0] + s.n[1]) + 128.0) * u * esum + 2.0 * u * std::fabs(tot);
        e += etot;
        b += etot;
        return 2.0 * (e + 16.0 * u * b) + 0x1p-1000;
    }
    // score the trials approximately: out/err (err 0: exact -- a zero score,
    // or recounted on the host); returns whether list bits came back
    bool score_models_approx(const Model* models, uint32_t n, HScore* out, double* err, uint32_t* raw_n,
                             const ListReq& req) {
        auto& hm = Tr::hlomodels(P_->w);
        hm.ensure(kSmallScore);
        std::memcpy(hm.p, models, n * sizeof(Model));
        P_->w->lo_sb.ensure(n);
        const bool lists = !(req.rule == 2 && use_graph());
        const ListBits lb = lists ? list_bits(req) : ListBits{{0.0, 0.0}, 0, 0.0, nullptr, nullptr};
        ScoreOut so = P_->w->lo_sb.host_dev();
        P_->w->lo_done.ensure(kSmallScore);
        so.done = dev_view(P_->w->lo_done.p);
        so.epoch = ++P_->w->done_epoch;
        if (so.epoch == 0) so.epoch = ++P_->w->done_epoch;
        lot("setup");
        HIPC(launch_score_small_part(P_->dp, Tm_, dev_view(hm.p), 0, n, 1 | 4, n, so, s_, lists ? &lb : nullptr,
                                     models));
        lot("launched");
        wait_done(P_->w->lo_done.p, n, so.epoch);
        lot("waited");
        st_.launches += 1;
        finish_small(models, n, out, raw_n, nullptr, lists);
        for (uint32_t i = 0; i < n; ++i) {
            err[i] = 0.0;
            if (sm_mbad_[i] || out[i].total == 0) continue;        // recounted, or a zero score
            err[i] = approx_err(out[i], P_->w->lo_sb.hv0.p[i], P_->w->lo_sb.hv1.p[i], P_->w->lo_sb.htot.p[i]);
        }
        lot("finished");
        return lists;
    }
    // the exact scores of the last approximate launch's n models (a round
    // with an undecided comparison), into out
    void refold_exact(const Model* models, uint32_t n, HScore* out, uint32_t* raw_n, bool lists) {
        ScoreOut so = P_->w->lo_sb.host_dev();
        so.done = dev_view(P_->w->lo_done.p);
        so.epoch = ++P_->w->done_epoch;
        if (so.epoch == 0) so.epoch = ++P_->w->done_epoch;
        HIPC(launch_lo_fold_slots(P_->dp, 0, n, 0, so, s_));
        wait_done(P_->w->lo_done.p, n, so.epoch);
        st_.launches += 1;
        ++st_.lo_refolds;
        finish_small(models, n, out, raw_n, nullptr, lists);
    }
    // the exact fold of model q of the last approximate launch, behind it
    uint32_t win_epoch_ = 0;
    void launch_win_fold(uint32_t q) {
        P_->w->lo_wb.ensure(1);
        P_->w->lo_wdone.ensure(1);
        ScoreOut so = P_->w->lo_wb.host_dev();
        so.done = dev_view(P_->w->lo_wdone.p);
        so.epoch = ++P_->w->wdone_epoch;
        if (so.epoch == 0) so.epoch = ++P_->w->wdone_epoch;
        win_epoch_ = so.epoch;
        HIPC(launch_lo_fold_slots(P_->dp, q, 1, 0, so, s_));
    }
    HScore win_exact() {
        wait_done(P_->w->lo_wdone.p, 1, win_epoch_);
        const uint32_t rn[2] = {P_->w->lo_wb.hn0.p[0], P_->w->lo_wb.hn1.p[0]};
        return finish(rn, P_->w->lo_wb.hv0.p[0], P_->w->lo_wb.hv1.p[0], P_->w->lo_wb.htot.p[0]);
    }
    // score_less(a, b) with a, b within ea, eb of their exact scores and ma,
    // mb their decision models (b: its value model too; a_self: a's as
    // well): 1 / 0, or -1 when the bounds leave it open
    int approx_less(const HScore& a, double ea, const Model& ma, bool a_self, const HScore& b, double eb,
                    const Model& mb) {
        if (ea == 0.0 && eb == 0.0) return score_less(a, [&] { return ma; }, b, [&] { return mb; }) ? 1 : 0;
        if (a_self && std::memcmp(&ma, &mb, sizeof(Model)) == 0) {
            // one model: equal exact scores, a near tie of score_less
            if (exact_ && sbnd_.finite && dev_of(a) + dev_of(b) > 0.0) ++ec_.near_ties;
            return 0;
        }
        double tol = 0.0;
        if (exact_ && sbnd_.finite) tol = dev_of(a) + dev_of(b) + 64.0 * 0x1p-53 * (ea + eb);
        const double m = (tol + ea + eb) * (1.0 + 0x1p-40);
        const double d = b.sum - a.sum;
        if (d > m) return 1;
        if (-d > m) return 0;
        return -1;
    }

    // GCR_DONE_WAIT=0: score_models waits on the stream instead of the
    // kernels' completion flags (read per call)
    static bool done_wait_on() {
        const char* e = getenv("GCR_DONE_WAIT");
        return !(e && e[0] == '0');
    }
    // spin until the small scorer has flagged models 0 .. n-1 with `epoch`;
    // a stream that drained (or failed) without them is an error
    void wait_done(const uint32_t* done, uint32_t n, uint32_t epoch) {
        uint32_t i = 0;
        const auto t0 = Clock::now();
        bool told = false;
        for (uint64_t it = 1;; ++it) {
            while (i < n && __atomic_load_n(done + i, __ATOMIC_ACQUIRE) == epoch) ++i;
            if (i == n) break;
            if ((it & 4095) == 0) {
                const hipError_t q = hipStreamQuery(s_);
                if (q == hipSuccess) {              // drained: the flags are visible now, or never come
                    while (i < n && __atomic_load_n(done + i, __ATOMIC_ACQUIRE) == epoch) ++i;
                    if (i == n) break;
                    char msg[160];
                    snprintf(msg, sizeof(msg),
                             "small scorer: completion flag %u of %u is %u, expected %u after the stream drained", i, n,
                             __atomic_load_n(done + i, __ATOMIC_ACQUIRE), epoch);
                    throw std::runtime_error(msg);
                }
                if (q != hipErrorNotReady) HIPC(q);
                slow_wait_note("small scorer", t0, told);
            }
            spin_pause();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
    }

    // model q's inlier lists from the bits of the last score_models(req) call
    // (small scorer pair layout: class 0 at [0, pad0), class 1 after it)
    void list_of(uint32_t q, std::vector<uint32_t> lists[2], bool msac = false) const {
        decode_lists(msac ? P_->w->h_mbits.p : P_->w->h_lbits.p, q, lists);
    }
    // row q of a small-scorer bit array (pair layout: class 0 at [0, pad0),
    // class 1 after it) as inlier index lists
    void decode_lists(const uint64_t* bits, uint32_t q, std::vector<uint32_t> lists[2]) const {
        const size_t pairs = small_score_pairs(P_->dp);
        const size_t pad0 = (N_[0] + 63) & ~(size_t)63;
        const uint64_t* w = bits + q * (pairs / 64);
        for (int c = 0; c < 2; ++c) {
            lists[c].clear();
            if (c >= K_) continue;
            const uint64_t* cw = w + ((c ? pad0 : 0) >> 6);
            const size_t nw = (N_[c] + 63) / 64;
            size_t n = 0;
            for (size_t wi = 0; wi < nw; ++wi) n += (size_t)__builtin_popcountll(cw[wi]);
            lists[c].resize(n);
            uint32_t* o = lists[c].data();
            for (size_t wi = 0; wi < nw; ++wi) {
                uint64_t b = cw[wi];
                const uint32_t base = (uint32_t)(wi * 64);
                while (b) {
                    *o++ = base + (uint32_t)__builtin_ctzll(b);
                    b &= b - 1;
                }
            }
        }
    }

    // Inlier index lists of one model: rule 0 with thresholds T, or (1-class
    // LO) the graph-cut labeling (rule 2).
    void inlier_lists(const Model& model, const double T[2], int rule, std::vector<uint32_t> lists[2]) {
        if (rule == 2 && use_graph()) {
            // labeling() with pairwise terms (GCRANSAC.h:759-870): the LO
            // model's squared residuals from the GPU, the st-mincut on the host
            const size_t n = N_[0];
            P_->w->r2.ensure(n);
            P_->w->h_r2.ensure(n);
            if (zerocopy_on()) {                                 // written straight into pinned memory
                HIPC(Tr::sqres(P_, model, dev_view(P_->w->h_r2.p), s_));
            } else {
                HIPC(Tr::sqres(P_, model, P_->w->r2.p, s_));
                HIPC(hipMemcpyAsync(P_->w->h_r2.p, P_->w->r2.p, n * sizeof(double), hipMemcpyDeviceToHost, s_));
            }
            HIPC(hipStreamSynchronize(s_));
            st_.launches += 1;
            lot("gc_resid");
            lists[1].clear();
            // the cells are independent components: cut them on the host
            // pool, in the cost-balanced jobs of gc_schedule
            gc_cseg_.resize(edges_.nodes.size());
            gc_seg_.resize(n);
            graphcut_labeling_jobs(P_->w->h_r2.p, T[0], prm_.spatial_coherence_weight, edges_, gc_cseg_.data(),
                                   gc_seg_.data(), [](size_t njobs, const auto& fn) {
                                       host_pool().parallel_for(njobs, [&](size_t j) {
                                           thread_local CellScratch cs;
                                           fn(j, cs);
                                       });
                                   });
            lot("gc_cut");
            lists[0].resize(n);
            uint32_t* lp = lists[0].data();
            size_t m = 0;
            for (size_t i = 0; i < n; ++i) {
                lp[m] = (uint32_t)i;
                m += gc_seg_[i];
            }
            lists[0].resize(m);
            return;
        }
        const size_t tot = N_[0] + (K_ == 2 ? N_[1] : 0);
        P_->w->mask_all.ensure(tot);
        P_->w->h_mask_all.ensure(tot);
        // the masks written straight into pinned memory (zero-copy)
        const bool zc = zerocopy_on();
        uint8_t* mk = zc ? dev_view(P_->w->h_mask_all.p) : P_->w->mask_all.p;
        for (int c = 0; c < K_; ++c)
            HIPC(Tr::mask(P_, c, model, rule, T[c], prm_.spatial_coherence_weight, mk + (c ? N_[0] : 0), s_));
        if (!zc) HIPC(hipMemcpyAsync(P_->w->h_mask_all.p, P_->w->mask_all.p, tot, hipMemcpyDeviceToHost, s_));
        HIPC(hipStreamSynchronize(s_));
        st_.launches += K_;
        for (int c = 0; c < 2; ++c) {
            lists[c].clear();
            if (c >= K_) continue;
            uint8_t* mk = P_->w->h_mask_all.p + (c ? N_[0] : 0);
            // flagged decisions (bit 1; every scale pair of a model the bound
            // does not cover) in glibc
            if constexpr (kRect)
                if (exact_)
                    exact_mask(P_, c, model, rule, T[c], prm_.spatial_coherence_weight, mk, c == 0 && unsafe(model),
                               ec_);
            for (uint64_t i = 0; i < N_[c]; ++i)
                if (mk[i] & 1) lists[c].push_back((uint32_t)i);
        }
    }

    // graphCutLocalOptimization (GCRANSAC.h:873-1062)
    std::vector<uint8_t> drawn_;          // local_optimization: trial q's sample was drawn
    bool local_optimization(Buffer& sfb_buf) {
        const auto t0 = Clock::now();
        HScore max_score = best_;
        Model lo_model = best_model_;
        Buffer lo_buf;
        const uint64_t limit[2] = {7 * m_[0], 7 * m_[1]};
        static_assert(kMaxLOSample >= 7 * 7, "LO sample buffer");

        ++lo_number_;
        lo_lists_from_bits_ = false;
        std::vector<uint32_t> inl[2];
        std::vector<std::array<std::vector<uint32_t>, 2>> trial_samples;
        std::vector<Model> trial_fit;
        std::vector<char> trial_ok;
        std::vector<Model> trial_models;
        std::vector<HScore> trial_scores;
        std::vector<double> trial_err;        // approximate scores: their bounds (0: exact)
        std::vector<uint32_t> trial_raw;
        bool win_pending = false;             // the last winner's exact fold is still to be read
        long fold_due = -1;                   // ... and to be launched (its model index)
        bool max_self = false;                // max_score is lo_model's own value score
        const uint64_t T = prm_.max_local_optimization_number;
        // the LO lists (threshold (1.5 thr)^2, labeling rule) of the round's
        // winner come back with the trial scores, so the next round starts
        // without its own mask launch + synchronisation
        const ListReq lreq{{Tlo_[0], Tlo_[1]}, K_ == 2 ? 0 : 2, lo_reuse_on()};
        bool have_inl = false;
        if (g_lo_trace) t_lot.clear();
        while (++gc_number_ < 10) {
            bool updated = false;
            lot("round");
            auto tp = Clock::now();
            if (!have_inl) {
                if (lo_row_ >= 0 && std::memcmp(&lo_row_model_, &lo_model, sizeof(Model)) == 0 &&
                    (lo_row_lfl_ == 0 || !exact_) && !unsafe(lo_model)) {
                    // the triggering model's lists from its chunk's scoring launch
                    decode_lists(P_->w->h_cbits[lo_row_set_].p, (uint32_t)lo_row_, inl);
                } else {
                    inlier_lists(lo_model, Tlo_, lreq.rule, inl);
                }
            }
            lo_row_ = -1;
            have_inl = false;
            lot("lists");
            st_.ms_lo_lists += ms_since(tp);
            tp = Clock::now();
            uint64_t ssz[2] = {0, 0};
            bool all_deterministic = true;
            for (int c = 0; c < K_; ++c) {
                ssz[c] = std::min<uint64_t>(limit[c], inl[c].size());
                if (ssz[c] < inl[c].size()) all_deterministic = false;
            }
            const uint64_t round_id = gc_number_;
            trial_models.clear();
            // when every class uses all its inliers each trial refits the same
            // set: one trial decides the round (later ones cannot be strictly better)
            const uint64_t ntrials = all_deterministic ? std::min<uint64_t>(T, 1) : T;
            // every trial draws its sample (counter-based: independent of the
            // others) and fits it on the host worker pool; a failed draw ends
            // the round at that trial, as in the sequential loop (its fit and
            // every later trial's are discarded); the successful fits are kept
            // in trial order
            trial_samples.resize(ntrials);
            trial_fit.resize(ntrials);
            trial_ok.assign(ntrials, 0);
            drawn_.assign(ntrials, 0);
            auto draw_fit = [&](size_t trial) {
                auto& smp = trial_samples[trial];
                for (int c = 0; c < K_; ++c) {
                    if (ssz[c] < inl[c].size()) {
                        // 7 m points: 49 for the 7-point fundamental matrix
                        uint32_t pos[kMaxLOSample];
                        WordStream ws(prm_.seed, round_id, (uint32_t)trial, kStreamLO, (uint32_t)c);
                        if (!sample_distinct<kMaxLOSample>(ws, inl[c].size(), (int)ssz[c], pos)) return;
                        smp[c].resize(ssz[c]);
                        for (uint64_t q = 0; q < ssz[c]; ++q) smp[c][q] = inl[c][pos[q]];
                    } else if (m_[c] < inl[c].size()) {
                        smp[c] = inl[c];
                    } else {
                        return;
                    }
                }
                drawn_[trial] = 1;
                trial_ok[trial] = Tr::fit(P_, smp.data(), trial_fit[trial], false) ? 1 : 0;
            };
            // Pipelined with the GPU (GCR_LO_PIPE=0: off): the first half of
            // the trials is fitted, its residual launch goes out, and the
            // second half is fitted while the GPU scores the first; then the
            // second half's residuals and the fold of all.  Same models in
            // the same order, so the same scores.
            uint64_t first_half = 0;                 // trial models already launched
            const uint64_t half = (ntrials + 1) / 2;
            const bool pipe = ntrials >= 8 && score_parts_ok((uint32_t)ntrials);
            uint64_t ndrawn = 0;
            if (pipe && fold_due >= 0) {
                launch_win_fold((uint32_t)fold_due);
                fold_due = -1;
            }
            if (pipe) {
                host_pool().parallel_for(half, draw_fit);
                while (ndrawn < half && drawn_[ndrawn]) ++ndrawn;
                for (uint64_t i = 0; i < ndrawn; ++i)
                    if (trial_ok[i]) trial_models.push_back(trial_fit[i]);
                if (ndrawn == half) {                // no failed draw: the second half runs
                    auto second = [&](size_t k) { draw_fit(half + k); };
                    const bool async = host_pool().begin(ntrials - half, second);
                    if (!trial_models.empty()) {
                        trial_raw.resize(2 * ntrials);
                        trial_scores.resize(ntrials);
                        score_models(trial_models.data(), (uint32_t)trial_models.size(), trial_scores.data(),
                                     trial_raw.data(), &lreq, nullptr, 0, true);
                        first_half = trial_models.size();
                    }
                    if (async) host_pool().end();
                    else host_pool().parallel_for(ntrials - half, second);
                    while (ndrawn < ntrials && drawn_[ndrawn]) ++ndrawn;
                    for (uint64_t i = half; i < ndrawn; ++i)
                        if (trial_ok[i]) trial_models.push_back(trial_fit[i]);
                }
            } else if (fold_due >= 0) {
                // the last round's winner's exact fold goes out from the pool
                // as its first item, beside the fits (before this round's
                // launches on the stream: they follow the parallel_for)
                host_pool().parallel_for(ntrials + 1, [&](size_t i) {
                    if (i == 0) launch_win_fold((uint32_t)fold_due);
                    else draw_fit(i - 1);
                });
                fold_due = -1;
                while (ndrawn < ntrials && drawn_[ndrawn]) ++ndrawn;
                for (uint64_t i = 0; i < ndrawn; ++i)
                    if (trial_ok[i]) trial_models.push_back(trial_fit[i]);
            } else {
                host_pool().parallel_for(ntrials, draw_fit);
                while (ndrawn < ntrials && drawn_[ndrawn]) ++ndrawn;
                for (uint64_t i = 0; i < ndrawn; ++i)
                    if (trial_ok[i]) trial_models.push_back(trial_fit[i]);
            }
            lot("fits");
            st_.ms_lo_fit += ms_since(tp);
            tp = Clock::now();
            if (!trial_models.empty()) {
                const uint32_t nt = (uint32_t)trial_models.size();
                trial_scores.resize(nt);
                trial_raw.resize(2 * nt);
                const bool apx = !pipe && approx_ok(nt);
                bool bits;
                if (apx) {
                    trial_err.resize(nt);
                    bits = score_models_approx(trial_models.data(), nt, trial_scores.data(), trial_err.data(),
                                               trial_raw.data(), lreq);
                } else {
                    bits = score_models(trial_models.data(), nt, trial_scores.data(), trial_raw.data(), &lreq,
                                        nullptr, (uint32_t)first_half);
                }
                // the previous round's winner: its exact fold ran before this
                // round's launches on the stream
                if (win_pending) {
                    max_score = win_exact();
                    win_pending = false;
                }
                st_.lo_models += nt;
                st_.ms_lo_score += ms_since(tp);
                size_t win = 0;
                bool decided = false;
                if (apx) {
                    // the sequential comparisons on the approximate scores;
                    // one the bounds leave open: the round folded exactly
                    const uint64_t nt0 = ec_.near_ties, nf0 = ec_.near_flips;
                    HScore ms = max_score;
                    double me = 0.0;
                    Model mm = lo_model;
                    bool mself = max_self;
                    long w = -1;
                    decided = true;
                    for (uint32_t q = 0; q < nt; ++q) {
                        const int d = approx_less(ms, me, mm, mself, trial_scores[q], trial_err[q], trial_models[q]);
                        if (d < 0) {
                            decided = false;
                            break;
                        }
                        if (d) {
                            w = (long)q;
                            ms = trial_scores[q];
                            me = trial_err[q];
                            mm = trial_models[q];
                            mself = true;
                        }
                    }
                    if (lo_approx_mode() == 2) decided = false;
                    if (decided && w >= 0) {
                        updated = true;
                        win = (size_t)w;
                        max_score = ms;
                        max_self = true;
                        lo_model = mm;
                        lo_buf = Buffer{true, mm, {trial_raw[2 * win], trial_raw[2 * win + 1]}};
                        if (me > 0.0) {
                            fold_due = (long)win;        // launched beside the next round's fits
                            win_pending = true;
                        }
                    }
                    if (!decided) {
                        ec_.near_ties = nt0;
                        ec_.near_flips = nf0;
                        refold_exact(trial_models.data(), nt, trial_scores.data(), trial_raw.data(), bits);
                    }
                }
                for (size_t q = 0; !decided && q < nt; ++q) {
                    if (score_less(max_score, [&] { return lo_model; }, trial_scores[q],
                                   [&] { return trial_models[q]; })) {
                        updated = true;
                        win = q;
                        max_score = trial_scores[q];
                        max_self = true;
                        lo_model = trial_models[q];
                        lo_buf = Buffer{true, trial_models[q], {trial_raw[2 * q], trial_raw[2 * q + 1]}};
                    }
                }
                if (updated) lo_lists_from_bits_ = bits && lreq.msac && !sm_mbad_[win];
                if (updated && bits) {
                    // bits with flagged decisions: the next round relabels
                    // through inlier_lists (exact_mask) instead
                    if (!sm_lbad_[win]) {
                        list_of((uint32_t)win, inl);
                        have_inl = true;
                    }
                    // the MSAC lists are decoded only if the LO result is adopted
                    if (lo_lists_from_bits_) {
                        const size_t rw = small_score_pairs(P_->dp) / 64;
                        const uint64_t* src = P_->w->h_mbits.p + (size_t)win * rw;
                        lo_msac_row_.assign(src, src + rw);
                    }
                }
            }
            lot("picked");
            if (!updated) break;
        }
        if (fold_due >= 0) launch_win_fold((uint32_t)fold_due);
        if (win_pending) max_score = win_exact();
        lot_print("gcr LO:", t_lot);
        st_.ms_lo += ms_since(t0);
        if (score_less(best_, [&] { return best_model_; }, max_score, [&] { return lo_model; })) {
            best_ = max_score;
            best_model_ = lo_model;
            best_val_ = lo_model;
            sfb_buf = lo_buf;
            // lo_msac_row_ holds lo_model's MSAC list bits from its own
            // scoring launch (the round that adopted it; later rounds only
            // score other models)
            lo_cache_.valid = lo_lists_from_bits_;
            if (lo_cache_.valid) {
                lo_cache_.model = lo_model;
                lo_cache_.score = max_score;
                lo_cache_.raw[0] = lo_buf.n[0];
                lo_cache_.raw[1] = lo_buf.n[1];
                decode_lists(lo_msac_row_.data(), 0, lo_cache_.lists);
            }
            return true;
        }
        return false;
    }
};

using Runner = RunnerT<RectTraits>;
using GeoRunner = RunnerT<GeoTraits>;
using FundRunner = RunnerT<FundTraits>;

}  // namespace

// ================================================================= C ABI ====
namespace {
int guard(const std::function<int()>& fn) {
    try {
        return fn();
    } catch (const HipError& e) {
        return set_err(GCR_EHIP, "HIP error %d (%s) in %s", (int)e.e, hipGetErrorString(e.e), e.what);
    } catch (const std::bad_alloc&) {
        return set_err(GCR_ENOMEM, "out of host memory");
    } catch (const std::exception& e) {
        return set_err(GCR_EINTERNAL, "%s", e.what());
    } catch (...) {
        return set_err(GCR_EINTERNAL, "unknown error");
    }
}

int check_params(const gcr_params* p, int solver) {
    if (!p) return set_err(GCR_EINVAL, "null params");
    if (!(p->confidence > 0.0 && p->confidence < 1.0))
        return set_err(GCR_EINVAL, "confidence must be in (0, 1)");
    if (p->cell_number > 0) {
        if (solver < 3)
            return set_err(GCR_EINVAL, "a neighbourhood grid is only supported for the homography and fundamental "
                                       "matrix estimators (the rectification entry points use an empty grid)");
        for (int d = 0; d < 4; ++d)
            if (!(p->cell_size[d] >= 0.0) || !std::isfinite(p->cell_size[d]))
                return set_err(GCR_EINVAL, "neighbourhood cell sizes must be positive and finite (or 0: from the data)");
    }
    return GCR_OK;
}

void fill_stats(gcr_stats* out, const gcr_stats& st) {
    if (out) *out = st;
}
}  // namespace

// The batch entry point's solving contexts (a stream pair and a workspace
// each, with its pinned staging buffers) outlive the call: the next call on the
// device takes them back instead of creating and warming new ones (a fresh
// context's first problem pays its pinned allocations), as a persistent
// service would hold them.  Kept for the process lifetime.
namespace {
struct BatchCtxPool {
    std::mutex mu;
    std::map<int, std::vector<gcr_ctx*>> free;
};
BatchCtxPool& batch_ctx_pool() {
    static BatchCtxPool* p = new BatchCtxPool();   // never destroyed (HIP may be gone at exit)
    return *p;
}
}  // namespace

extern "C" {

const char* gcr_last_error(void) { return g_err.c_str(); }
int gcr_abi_version(void) { return GCR_ABI_VERSION; }

int gcr_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void gcr_default_params(gcr_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->scale_residual_thresh = 2.0;          // settings.h:71 default threshold
    p->orientation_residual_thresh = 2.0;
    p->spatial_coherence_weight = 0.0;       // bindings.cpp:370
    p->min_iteration_number = 10000;         // bindings.cpp:371
    p->max_iteration_number = 10000;         // bindings.cpp:372
    p->max_local_optimization_number = 50;   // bindings.cpp:373
    p->confidence = 0.95;                    // settings.h:60
    p->seed = 0;
    p->batch_slots = 0;
    p->flags = 0;
}

int gcr_create(int device, gcr_ctx** out) {
    if (!out) return set_err(GCR_EINVAL, "null output pointer");
    return guard([&]() -> int {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return set_err(GCR_ENODEV, "no HIP device available");
        if (device < 0 || device >= n) return set_err(GCR_ENODEV, "device %d out of range (%d devices)", device, n);
        auto c = std::unique_ptr<gcr_ctx>(new gcr_ctx());
        c->device = device;
        HIPC(hipSetDevice(device));
        // the replay's dependent steps (LO labeling and trial scores, the
        // refit) must not queue behind a speculative chunk's workgroups
        int least = 0, greatest = 0;
        HIPC(hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIPC(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, greatest));
        HIPC(hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, least));
        HIPC(hipEventCreate(&c->ev0));
        HIPC(hipEventCreate(&c->ev1));
        HIPC(hipEventCreate(&c->pev0));
        HIPC(hipEventCreate(&c->pev1));
        HIPC(hipEventCreateWithFlags(&c->pdone, hipEventDisableTiming));
        int cu = 0;
        if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cu > 0)
            c->n_cu = cu;
        *out = c.release();
        return GCR_OK;
    });
}

int gcr_synchronize(gcr_ctx* ctx) {
    if (!ctx) return set_err(GCR_EINVAL, "null context");
    return guard([&]() -> int {
        HIPC(hipSetDevice(ctx->device));
        HIPC(hipDeviceSynchronize());
        return GCR_OK;
    });
}

void gcr_destroy(gcr_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->pev0) (void)hipEventDestroy(ctx->pev0);
    if (ctx->pev1) (void)hipEventDestroy(ctx->pev1);
    if (ctx->pdone) (void)hipEventDestroy(ctx->pdone);
    if (ctx->side) (void)hipStreamDestroy(ctx->side);
    if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int gcr_problem_create(gcr_ctx* ctx, int solver, const double* f0, size_t n0, const double* f1, size_t n1,
                       gcr_problem** out) {
    return guard([&]() { return make_problem(ctx, solver, f0, n0, f1, n1, out); });
}

void gcr_problem_destroy(gcr_problem* prob) {
    if (!prob) return;
    (void)hipSetDevice(prob->ctx->device);
    if (prob->own) {
        std::lock_guard<std::mutex> lk(prob->ctx->ws_mu);
        if (prob->ctx->ws_free.size() < 4) prob->ctx->ws_free.push_back(std::move(prob->own));
    }
    // a workspace that is about to be freed may still have a speculative
    // chunk in flight (a recycled one is awaited by its next user)
    if (prob->own) {
        try { await_spec(prob->own.get()); } catch (...) {}
    }
    delete prob;
}

int gcr_problem_run(gcr_problem* prob, const gcr_params* params, uint8_t* mask0_out, uint8_t* mask1_out,
                    double* H_out, gcr_rect_model* model_out, gcr_stats* stats_out) {
    if (!prob) return set_err(GCR_EINVAL, "null problem");
    if (int e = check_params(params, prob->solver)) return e;
    if (!mask0_out || !H_out || (prob->K == 2 && !mask1_out)) return set_err(GCR_EINVAL, "null output buffer");
    return guard([&]() -> int {
        HIPC(hipSetDevice(prob->ctx->device));
        auto go = [&](auto&& r) {
            const int total = r.run(mask0_out, mask1_out, H_out, model_out);
            fill_stats(stats_out, r.stats());
            return total;
        };
        if (prob->solver == GCR_SOLVER_FUNDAMENTAL7) return go(FundRunner(prob, *params));
        return prob->solver == GCR_SOLVER_HOMOGRAPHY4 ? go(GeoRunner(prob, *params)) : go(Runner(prob, *params));
    });
}

int gcr_problem_run_sharded(gcr_problem* prob, const gcr_params* params, int rank, int world,
                            gcr_allgather_fn allgather, void* user, uint8_t* mask0_out, uint8_t* mask1_out,
                            double* H_out, gcr_rect_model* model_out, gcr_stats* stats_out) {
    if (!prob) return set_err(GCR_EINVAL, "null problem");
    if (int e = check_params(params, prob->solver)) return e;
    if (world < 1 || rank < 0 || rank >= world || (world > 1 && !allgather))
        return set_err(GCR_EINVAL, "bad rank/world/allgather");
    if (!mask0_out || !H_out || (prob->K == 2 && !mask1_out)) return set_err(GCR_EINVAL, "null output buffer");
    return guard([&]() -> int {
        HIPC(hipSetDevice(prob->ctx->device));
        auto go = [&](auto&& r) {
            if (world > 1) r.set_sharding(rank, world, allgather, user);
            const int total = r.run(mask0_out, mask1_out, H_out, model_out);
            fill_stats(stats_out, r.stats());
            return total;
        };
        if (prob->solver == GCR_SOLVER_FUNDAMENTAL7) return go(FundRunner(prob, *params));
        if (prob->solver == GCR_SOLVER_HOMOGRAPHY4) return go(GeoRunner(prob, *params));
        return go(Runner(prob, *params));
    });
}

int gcr_comm_unique_id(uint8_t id_out[GCR_COMM_ID_BYTES]) {
    if (!id_out) return set_err(GCR_EINVAL, "null id buffer");
    static_assert(sizeof(ncclUniqueId) == GCR_COMM_ID_BYTES, "nccl unique id size");
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return set_err(GCR_EHIP, "ncclGetUniqueId: %s", ncclGetErrorString(r));
    std::memcpy(id_out, &id, sizeof(id));
    return GCR_OK;
}

int gcr_comm_create(gcr_ctx* ctx, int rank, int world, const uint8_t id[GCR_COMM_ID_BYTES], gcr_comm** out) {
    if (!ctx || !id || !out) return set_err(GCR_EINVAL, "null argument");
    if (world < 1 || rank < 0 || rank >= world) return set_err(GCR_EINVAL, "bad rank/world");
    return guard([&]() -> int {
        HIPC(hipSetDevice(ctx->device));
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof(uid));
        auto c = std::make_unique<gcr_comm>();
        const ncclResult_t r = ncclCommInitRank(&c->comm, world, uid, rank);
        if (r != ncclSuccess) return set_err(GCR_EHIP, "ncclCommInitRank: %s", ncclGetErrorString(r));
        c->rank = rank;
        c->world = world;
        c->ctx = ctx;
        *out = c.release();
        return GCR_OK;
    });
}

namespace {
void abort_comm(gcr_comm* comm, Workspace* w) {
    if (comm->comm) (void)ncclCommAbort(comm->comm);
    comm->comm = nullptr;
    comm->aborted = true;
    (void)hipStreamSynchronize(comm->ctx->side);
    (void)hipStreamSynchronize(comm->ctx->stream);
    (void)hipGetLastError();
    for (int k = 0; k < 2; ++k) w->spec_pending[k] = false;
}
}  // namespace

void gcr_comm_destroy(gcr_comm* comm) {
    if (!comm) return;
    (void)hipSetDevice(comm->ctx->device);
    // a run can return with a speculative chunk's ncclAllGather still queued
    // on the side stream (gcr_problem_run_comm also drains it; this covers a
    // caller that destroys the communicator first)
    (void)hipStreamSynchronize(comm->ctx->side);
    if (comm->comm) (void)ncclCommDestroy(comm->comm);   // an aborted one is already gone
    delete comm;
}

int gcr_problem_run_comm(gcr_problem* prob, const gcr_params* params, gcr_comm* comm, uint8_t* mask0_out,
                         uint8_t* mask1_out, double* H_out, gcr_rect_model* model_out, gcr_stats* stats_out) {
    if (!prob || !comm) return set_err(GCR_EINVAL, "null problem or communicator");
    if (comm->ctx != prob->ctx) return set_err(GCR_EINVAL, "communicator and problem on different contexts");
    if (int e = check_params(params, prob->solver)) return e;
    if (!mask0_out || !H_out || (prob->K == 2 && !mask1_out)) return set_err(GCR_EINVAL, "null output buffer");
    if (comm->aborted) return set_err(GCR_EINVAL, "communicator was aborted after an earlier error");
    return guard([&]() -> int {
        HIPC(hipSetDevice(prob->ctx->device));
        auto go = [&](auto&& r) {
            r.set_comm(comm);
            const int total = r.run(mask0_out, mask1_out, H_out, model_out);
            // no collective of this run may outlive it: a speculative chunk
            // and its all-gather are drained before the caller can tear the
            // communicator down (every rank issued the same sequence)
            await_spec(prob->w);
            fill_stats(stats_out, r.stats());
            return total;
        };
        try {
            if (prob->solver == GCR_SOLVER_FUNDAMENTAL7) return go(FundRunner(prob, *params));
            if (prob->solver == GCR_SOLVER_HOMOGRAPHY4) return go(GeoRunner(prob, *params));
            return go(Runner(prob, *params));
        } catch (...) {
            // An error on this rank (a HIP or RCCL failure, a peer's failure
            // seen by comm_sync, bad input found mid-run): the other ranks
            // may be inside -- or about to issue -- the same collective, so
            // the communicator is aborted rather than left half-used.  That
            // ends this rank's queued collectives and tears down its
            // connections, which the peers' RCCL proxies report as an
            // asynchronous error to their own comm_sync waits, which then
            // abort their communicators in turn.  The problem's chunk sets
            // are drained and may be reused by a later single-rank run.
            abort_comm(comm, prob->w);
            throw;
        }
    });
}

int gcr_problem_verify_batches(gcr_problem* prob, const gcr_params* params, uint64_t slot0, uint32_t nslots,
                               uint32_t nbatches, gcr_batch_result* out, gcr_stats* stats_out) {
    if (!prob || !out) return set_err(GCR_EINVAL, "null problem or output");
    if (int e = check_params(params, prob->solver)) return e;
    if (nslots == 0 || nbatches == 0) return set_err(GCR_EINVAL, "nslots and nbatches must be > 0");
    return guard([&]() -> int {
        HIPC(hipSetDevice(prob->ctx->device));
        auto go = [&](auto&& r) {
            r.verify_batches(slot0, nslots, nbatches, out);
            fill_stats(stats_out, r.stats());
            return GCR_OK;
        };
        if (prob->solver == GCR_SOLVER_FUNDAMENTAL7) return go(FundRunner(prob, *params));
        return prob->solver == GCR_SOLVER_HOMOGRAPHY4 ? go(GeoRunner(prob, *params)) : go(Runner(prob, *params));
    });
}

int gcr_problem_verify_batch(gcr_problem* prob, const gcr_params* params, uint64_t slot0, uint32_t nslots,
                             gcr_batch_result* out, gcr_stats* stats_out) {
    const int rc = gcr_problem_verify_batches(prob, params, slot0, nslots, 1, out, stats_out);
    return rc < 0 ? rc : (int)out->models;
}

static int run_oneshot(gcr_ctx* ctx, int solver, const double* f0, size_t n0, const double* f1, size_t n1,
                       const gcr_params* params, uint8_t* m0, uint8_t* m1, double* H, gcr_rect_model* model,
                       gcr_stats* stats) {
    if (!ctx) return set_err(GCR_EINVAL, "null context");
    if (int e = check_params(params, solver)) return e;
    const auto t0 = Clock::now();
    gcr_problem* prob = nullptr;
    int rc = guard([&]() { return make_problem(ctx, solver, f0, n0, f1, n1, &prob, true); });
    if (rc != GCR_OK) return rc;
    const double setup = ms_since(t0);
    rc = gcr_problem_run(prob, params, m0, m1, H, model, stats);
    gcr_problem_destroy(prob);
    if (stats) {
        stats->ms_setup = setup;
        stats->ms_total += setup;
    }
    return rc;
}

int gcr_solve_batch(int device, gcr_batch_item* items, size_t n, int concurrency) {
    if (n > 0 && !items) return set_err(GCR_EINVAL, "null items");
    if (concurrency < 1) concurrency = 1;
    if ((size_t)concurrency > n) concurrency = (int)std::max<size_t>(n, 1);
    std::vector<gcr_ctx*> ctxs((size_t)concurrency, nullptr);
    {
        std::lock_guard<std::mutex> lk(batch_ctx_pool().mu);
        auto& fr = batch_ctx_pool().free[device];
        for (auto& c : ctxs)
            if (!fr.empty()) {
                c = fr.back();
                fr.pop_back();
            }
    }
    auto release = [&]() {
        std::lock_guard<std::mutex> lk(batch_ctx_pool().mu);
        auto& fr = batch_ctx_pool().free[device];
        for (auto*& c : ctxs)
            if (c) {
                if (fr.size() < 64) fr.push_back(c);
                else gcr_destroy(c);
                c = nullptr;
            }
    };
    for (auto& c : ctxs)
        if (c == nullptr)
            if (int rc = gcr_create(device, &c); rc != GCR_OK) {
                c = nullptr;
                release();
                return rc;
            }
    // Problems are handed out longest first (an estimate of each call's
    // wall time: features x a per-estimator rate, from the configs[4] bench's
    // per-kind phase sums), so the batch does not end on one long problem
    // started last while the other threads idle.  Every problem is solved
    // on its own, so the order does not change any result.
    // GCR_BATCH_ORDER=index: index order (A/B).
    std::vector<size_t> order(n);
    for (size_t i = 0; i < n; ++i) order[i] = i;
    const char* eo = getenv("GCR_BATCH_ORDER");
    if (!(eo && std::strcmp(eo, "index") == 0)) {
        auto est = [&](size_t i) {
            const gcr_batch_item& it = items[i];
            // ms per 1000 features (configs[4] mix, 8 threads per GPU)
            const double rate = it.solver == GCR_SOLVER_FUNDAMENTAL7 ? 0.68
                                : it.solver == GCR_SOLVER_HOMOGRAPHY4 ? 0.37
                                : it.solver == GCR_SOLVER_SIFT22      ? 0.29
                                                                      : 0.20;
            return 0.25 + rate * 1e-3 * (double)(it.n0 + (it.f1 ? it.n1 : 0));
        };
        std::vector<double> cost(n);
        for (size_t i = 0; i < n; ++i) cost[i] = est(i);
        std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return cost[a] > cost[b]; });
    }
    std::atomic<size_t> next{0};
    std::atomic<int> first_err{GCR_OK};
    std::mutex err_mu;
    std::string err_text;
    auto worker = [&](gcr_ctx* ctx) {
        g_solving.fetch_add(1, std::memory_order_relaxed);
        struct Leave {
            ~Leave() { g_solving.fetch_sub(1, std::memory_order_relaxed); }
        } leave;
        for (size_t k; (k = next.fetch_add(1)) < n;) {
            gcr_batch_item& it = items[order[k]];
            it.result = run_oneshot(ctx, it.solver, it.f0, it.n0, it.f1, it.n1, &it.params, it.mask0_out,
                                    it.mask1_out, it.H_out, &it.model_out, &it.stats_out);
            if (it.result < 0) {
                int expect = GCR_OK;
                if (first_err.compare_exchange_strong(expect, it.result)) {
                    std::lock_guard<std::mutex> lk(err_mu);
                    err_text = g_err;        // thread-local message of this worker
                }
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < concurrency; ++t) pool.emplace_back(worker, ctxs[(size_t)t]);
    worker(ctxs[0]);
    for (auto& th : pool) th.join();
    release();
    if (first_err.load() != GCR_OK) return set_err(first_err.load(), "%s", err_text.c_str());
    return GCR_OK;
}

int gcr_rect_scale_only(gcr_ctx* ctx, const double* features, size_t n, const gcr_params* params, int original,
                        uint8_t* mask_out, double* H_out, gcr_rect_model* model_out, gcr_stats* stats_out) {
    return run_oneshot(ctx, original ? GCR_SOLVER_SCALE3_ORIGINAL : GCR_SOLVER_SCALE3, features, n, nullptr, 0,
                       params, mask_out, nullptr, H_out, model_out, stats_out);
}

int gcr_rect_sift(gcr_ctx* ctx, const double* scale_features, size_t n_scale, const double* orientation_features,
                  size_t n_orientation, const gcr_params* params, uint8_t* scale_mask_out,
                  uint8_t* orientation_mask_out, double* H_out, gcr_rect_model* model_out, gcr_stats* stats_out) {
    return run_oneshot(ctx, GCR_SOLVER_SIFT22, scale_features, n_scale, orientation_features, n_orientation, params,
                       scale_mask_out, orientation_mask_out, H_out, model_out, stats_out);
}

int gcr_find_homography(gcr_ctx* ctx, const double* correspondences, size_t n, const gcr_params* params,
                        uint8_t* mask_out, double* H_out, gcr_stats* stats_out) {
    return run_oneshot(ctx, GCR_SOLVER_HOMOGRAPHY4, correspondences, n, nullptr, 0, params, mask_out, nullptr, H_out,
                       nullptr, stats_out);
}

int gcr_find_fundamental_matrix(gcr_ctx* ctx, const double* correspondences, size_t n, const gcr_params* params,
                                uint8_t* mask_out, double* F_out, gcr_stats* stats_out) {
    return run_oneshot(ctx, GCR_SOLVER_FUNDAMENTAL7, correspondences, n, nullptr, 0, params, mask_out, nullptr, F_out,
                       nullptr, stats_out);
}

int gcr_host_fit_f(const double* correspondences, size_t n, const uint32_t* idx, size_t k, double* F_out) {
    if (!correspondences || !idx || !F_out) return set_err(GCR_EINVAL, "bad arguments");
    return guard([&]() -> int {
        HostClass hc[2];
        fill_host_classes(GCR_SOLVER_FUNDAMENTAL7, correspondences, n, nullptr, 0, hc);
        std::vector<uint32_t> list(idx, idx + k);
        for (uint32_t i : list)
            if (i >= n) return set_err(GCR_EINVAL, "index out of range");
        GeoModel m;
        if (!fit_f8_nonminimal(hc[0], list, m)) return 0;
        for (int q = 0; q < 9; ++q) F_out[q] = m.h[q];
        return 1;
    });
}

// ------------------------------------------------------- homography debug ----
int gcr_debug_generate_h(gcr_problem* prob, uint64_t seed, uint64_t slot0, uint32_t nslots, uint8_t* inc_out,
                         double* H_out) {
    if (!prob || !inc_out || !H_out) return set_err(GCR_EINVAL, "null argument");
    if (prob->solver != GCR_SOLVER_HOMOGRAPHY4 && prob->solver != GCR_SOLVER_FUNDAMENTAL7)
        return set_err(GCR_EINVAL, "not a correspondence (homography / fundamental) problem");
    return guard([&]() -> int {
        HIPC(hipSetDevice(prob->ctx->device));
        await_spec(prob->w);
        const size_t nh = (size_t)nslots * GeoTraits::per(prob);
        prob->w->inc.ensure(nh);
        prob->w->gmodels.ensure(nh);
        hipStream_t s = prob->ctx->stream;
        HIPC(launch_generate_geo(prob->dp, seed, slot0, nslots, prob->w->inc.p, prob->w->gmodels.p, s));
        HIPC(hipMemcpyAsync(inc_out, prob->w->inc.p, nh, hipMemcpyDeviceToHost, s));
        HIPC(hipMemcpyAsync(H_out, prob->w->gmodels.p, nh * sizeof(GeoModel), hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        return GCR_OK;
    });
}

int gcr_debug_score_h(gcr_problem* prob, const gcr_params* params, const double* H, uint32_t nmodels, uint32_t* n0,
                      double* v0, double* tot) {
    if (!prob || !params || !H || !n0 || !v0 || !tot) return set_err(GCR_EINVAL, "null argument");
    if (prob->solver != GCR_SOLVER_HOMOGRAPHY4 && prob->solver != GCR_SOLVER_FUNDAMENTAL7)
        return set_err(GCR_EINVAL, "not a correspondence (homography / fundamental) problem");
    return guard([&]() -> int {
        HIPC(hipSetDevice(prob->ctx->device));
        await_spec(prob->w);
        hipStream_t s = prob->ctx->stream;
        const double thr = params->scale_residual_thresh;
        const double T = (2.25 * thr) * thr;
        prob->w->lo_gmodels.ensure(nmodels);
        prob->w->lo_sb.ensure(nmodels);
        HIPC(hipMemcpyAsync(prob->w->lo_gmodels.p, H, nmodels * sizeof(GeoModel), hipMemcpyHostToDevice, s));
        if (debug_small_scorer(nmodels)) {
            const double Tt[2] = {T, 0.0};
            HIPC(launch_score_small(prob->dp, Tt, prob->w->lo_gmodels.p, nullptr, nmodels, prob->w->lo_sb.dev(), s));
        } else {
            HIPC(launch_score_geo(prob->dp, T, prob->w->lo_gmodels.p, nullptr, nmodels, prob->w->lo_sb.dev(), s));
        }
        prob->w->lo_sb.d2h(nmodels, s);
        HIPC(hipStreamSynchronize(s));
        std::memcpy(n0, prob->w->lo_sb.hn0.p, nmodels * sizeof(uint32_t));
        std::memcpy(v0, prob->w->lo_sb.hv0.p, nmodels * sizeof(double));
        std::memcpy(tot, prob->w->lo_sb.htot.p, nmodels * sizeof(double));
        return GCR_OK;
    });
}

int gcr_debug_mask_h(gcr_problem* prob, const gcr_params* params, const double* H, int rule, uint8_t* mask_out) {
    if (!prob || !params || !H || !mask_out) return set_err(GCR_EINVAL, "null argument");
    if (prob->solver != GCR_SOLVER_HOMOGRAPHY4 && prob->solver != GCR_SOLVER_FUNDAMENTAL7)
        return set_err(GCR_EINVAL, "not a correspondence (homography / fundamental) problem");
    return guard([&]() -> int {
        HIPC(hipSetDevice(prob->ctx->device));
        await_spec(prob->w);
        hipStream_t s = prob->ctx->stream;
        const double thr = params->scale_residual_thresh;
        double T;
        if (rule == 0) T = (2.25 * thr) * thr;
        else { const double t = 1.5 * thr; T = t * t; }
        GeoModel m;
        for (int k = 0; k < 9; ++k) m.h[k] = H[k];
        const size_t n = prob->hc[0].n;
        prob->w->mask[0].ensure(n);
        HIPC(launch_mask_geo(prob->dp, m, rule == 2 ? 2 : 0, T, params->spatial_coherence_weight, prob->w->mask[0].p,
                             s));
        HIPC(hipMemcpyAsync(mask_out, prob->w->mask[0].p, n, hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        return GCR_OK;
    });
}

int gcr_host_fit_h(const double* correspondences, size_t n, const uint32_t* idx, size_t k, double* H_out) {
    if (!correspondences || !idx || !H_out) return set_err(GCR_EINVAL, "bad arguments");
    return guard([&]() -> int {
        HostClass hc[2];
        fill_host_classes(GCR_SOLVER_HOMOGRAPHY4, correspondences, n, nullptr, 0, hc);
        std::vector<uint32_t> list(idx, idx + k);
        for (uint32_t i : list)
            if (i >= n) return set_err(GCR_EINVAL, "index out of range");
        GeoModel m;
        if (!fit_h4_nonminimal(hc[0], list, m)) return 0;
        for (int q = 0; q < 9; ++q) H_out[q] = m.h[q];
        return 1;
    });
}

// ---------------------------------------------------------------- debug ----
int gcr_debug_generate(gcr_problem* prob, uint64_t seed, uint64_t slot0, uint32_t nslots, uint8_t* inc_out,
                       gcr_rect_model* models_out) {
    if (!prob || !inc_out || !models_out) return set_err(GCR_EINVAL, "null argument");
    return guard([&]() -> int {
        HIPC(hipSetDevice(prob->ctx->device));
        await_spec(prob->w);
        prob->w->inc.ensure(nslots);
        prob->w->models.ensure(nslots);
        hipStream_t s = prob->ctx->stream;
        HIPC(launch_generate(prob->dp, seed, slot0, nslots, prob->w->inc.p, prob->w->models.p, s));
        HIPC(hipMemcpyAsync(inc_out, prob->w->inc.p, nslots, hipMemcpyDeviceToHost, s));
        HIPC(hipMemcpyAsync(models_out, prob->w->models.p, nslots * sizeof(RectModel), hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        return GCR_OK;
    });
}

int gcr_debug_score(gcr_problem* prob, const gcr_params* params, const gcr_rect_model* models, uint32_t nmodels,
                    uint32_t* n0, uint32_t* n1, double* v0, double* v1, double* tot) {
    if (!prob || !params || !models) return set_err(GCR_EINVAL, "null argument");
    return guard([&]() -> int {
        HIPC(hipSetDevice(prob->ctx->device));
        await_spec(prob->w);
        hipStream_t s = prob->ctx->stream;
        double T[2];
        const double thr[2] = {params->scale_residual_thresh, params->orientation_residual_thresh};
        for (int c = 0; c < 2; ++c) T[c] = (2.25 * thr[c]) * thr[c];
        bool identity = true;
        std::vector<RectModel> hm(nmodels);
        for (uint32_t i = 0; i < nmodels; ++i) {
            hm[i] = RectModel{models[i].x0, models[i].y0, models[i].s, models[i].h7, models[i].h8, models[i].alpha,
                              models[i].phi};
            identity = identity && identity_norm(hm[i]);
        }
        prob->w->lo_models.ensure(nmodels);
        prob->w->lo_sb.ensure(nmodels);
        HIPC(hipMemcpyAsync(prob->w->lo_models.p, hm.data(), nmodels * sizeof(RectModel), hipMemcpyHostToDevice, s));
        if (identity && debug_small_scorer(nmodels)) {
            HIPC(launch_score_small(prob->dp, T, prob->w->lo_models.p, nullptr, nmodels, prob->w->lo_sb.dev(), s,
                                    nullptr, hm.data()));
        } else {
            HIPC(launch_score(prob->dp, T, prob->w->lo_models.p, nullptr, nmodels, identity, prob->w->lo_sb.dev(), s));
        }
        prob->w->lo_sb.d2h(nmodels, s);
        HIPC(hipStreamSynchronize(s));
        std::memcpy(n0, prob->w->lo_sb.hn0.p, nmodels * sizeof(uint32_t));
        std::memcpy(n1, prob->w->lo_sb.hn1.p, nmodels * sizeof(uint32_t));
        std::memcpy(v0, prob->w->lo_sb.hv0.p, nmodels * sizeof(double));
        std::memcpy(v1, prob->w->lo_sb.hv1.p, nmodels * sizeof(double));
        std::memcpy(tot, prob->w->lo_sb.htot.p, nmodels * sizeof(double));
        // flagged decisions (or a model exact.h does not cover): the
        // reference's decisions, the twin values (the oracle's TWIN mode)
        if (exact_on()) {
            ExactCount ec;
            for (uint32_t i = 0; i < nmodels; ++i)
                if (prob->w->lo_sb.hfl.p[i] != 0 || model_unsafe(prob, hm[i], T[0])) {
                    uint32_t n[2];
                    double v[2];
                    exact_accumulate(prob, hm[i], hm[i], T, n, v, tot[i], nullptr, ec);
                    n0[i] = n[0];
                    n1[i] = prob->K == 2 ? n[1] : 0;
                    v0[i] = v[0];
                    v1[i] = prob->K == 2 ? v[1] : 0.0;
                }
        }
        return GCR_OK;
    });
}

size_t gcr_debug_exchange_log(uint64_t* out, size_t cap) {
    const size_t n = t_xlog.size();
    if (out) std::memcpy(out, t_xlog.data(), std::min(n, cap) * sizeof(uint64_t));
    return n;
}

int gcr_debug_score_less(gcr_problem* prob, const gcr_params* params, const gcr_rect_model* a,
                         const gcr_rect_model* b) {
    if (!prob || !a || !b) return set_err(GCR_EINVAL, "null argument");
    if (prob->solver > 2) return set_err(GCR_EINVAL, "gcr_debug_score_less: rectification solvers only");
    if (int e = check_params(params, prob->solver)) return e;
    return guard([&]() -> int {
        HIPC(hipSetDevice(prob->ctx->device));
        await_spec(prob->w);
        Runner r(prob, *params);
        RectModel ma, mb;
        static_assert(sizeof(RectModel) == sizeof(gcr_rect_model), "model layout");
        std::memcpy(&ma, a, sizeof(ma));
        std::memcpy(&mb, b, sizeof(mb));
        return r.debug_less(ma, mb);
    });
}

int gcr_debug_mask(gcr_problem* prob, const gcr_params* params, const gcr_rect_model* model, int cls, int rule,
                   uint8_t* mask_out) {
    if (!prob || !params || !model || !mask_out) return set_err(GCR_EINVAL, "null argument");
    if (cls < 0 || cls >= prob->K) return set_err(GCR_EINVAL, "class %d out of range", cls);
    return guard([&]() -> int {
        HIPC(hipSetDevice(prob->ctx->device));
        await_spec(prob->w);
        hipStream_t s = prob->ctx->stream;
        const double thr = cls == 0 ? params->scale_residual_thresh : params->orientation_residual_thresh;
        double T;
        if (rule == 0) T = (2.25 * thr) * thr;
        else { const double t = 1.5 * thr; T = t * t; }
        const RectModel m{model->x0, model->y0, model->s, model->h7, model->h8, model->alpha, model->phi};
        const size_t n = prob->hc[cls].n;
        prob->w->mask[cls].ensure(n);
        HIPC(launch_mask(prob->dp, cls, m, rule == 2 ? 2 : 0, T, params->spatial_coherence_weight,
                         prob->w->mask[cls].p, s));
        HIPC(hipMemcpyAsync(mask_out, prob->w->mask[cls].p, n, hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        // flagged decisions in glibc (GCR_EXACT=0: the twin's)
        ExactCount ec;
        if (exact_on())
            exact_mask(prob, cls, m, rule == 2 ? 2 : 0, T, params->spatial_coherence_weight, mask_out,
                       cls == 0 && model_unsafe(prob, m, T), ec);
        for (size_t i = 0; i < n; ++i) mask_out[i] &= 1;
        return GCR_OK;
    });
}

int gcr_host_fit_nonminimal(int solver, const double* f0, size_t n0, const double* f1, size_t n1, const uint32_t* idx0,
                            size_t k0, const uint32_t* idx1, size_t k1, gcr_rect_model* model_out) {
    if (solver < 0 || solver > 2 || !f0 || !idx0 || !model_out || (solver == 2 && (!f1 || !idx1)))
        return set_err(GCR_EINVAL, "bad arguments");
    return guard([&]() -> int {
        HostClass hc[2];
        fill_host_classes(solver, f0, n0, f1, n1, hc);
        std::vector<uint32_t> lists[2];
        lists[0].assign(idx0, idx0 + k0);
        if (solver == 2) lists[1].assign(idx1, idx1 + k1);
        for (int c = 0; c < (solver == 2 ? 2 : 1); ++c)
            for (uint32_t i : lists[c])
                if (i >= hc[c].n) return set_err(GCR_EINVAL, "index out of range");
        RectModel m;
        if (!fit_nonminimal(solver, hc, lists, m)) return 0;
        *model_out = gcr_rect_model{m.x0, m.y0, m.s, m.h7, m.h8, m.alpha, m.phi};
        return 1;
    });
}

int gcr_debug_fit_nonminimal(gcr_problem* prob, const uint32_t* idx0, size_t k0, const uint32_t* idx1, size_t k1,
                              int use_gpu, gcr_rect_model* model_out) {
    if (!prob || !idx0 || !model_out || (prob->solver == 2 && !idx1)) return set_err(GCR_EINVAL, "bad arguments");
    return guard([&]() -> int {
        HIPC(hipSetDevice(prob->ctx->device));
        await_spec(prob->w);
        std::vector<uint32_t> lists[2];
        lists[0].assign(idx0, idx0 + k0);
        if (prob->solver == 2) lists[1].assign(idx1, idx1 + k1);
        for (int c = 0; c < prob->K; ++c)
            for (uint32_t i : lists[c])
                if (i >= prob->hc[c].n) return set_err(GCR_EINVAL, "index out of range");
        RectModel m;
        GpuSiftSolver gpu(prob);
        if (!fit_nonminimal(prob->solver, prob->hc, lists, m, use_gpu ? &gpu : nullptr, 0)) return 0;
        *model_out = gcr_rect_model{m.x0, m.y0, m.s, m.h7, m.h8, m.alpha, m.phi};
        return 1;
    });
}

void gcr_host_homography(const gcr_rect_model* m, double* H_out) {
    if (!m || !H_out) return;
    homography_of(RectModel{m->x0, m->y0, m->s, m->h7, m->h8, m->alpha, m->phi}, H_out);
}

double gcr_host_log(double x) { return dm::dm_log(x); }
double gcr_host_pow_m3(double t) { return dm::dm_pow_m3(t); }
double gcr_host_atan2(double y, double x) { return dm::dm_atan2(y, x); }
int gcr_host_residuals(int solver, int cls, const double* features, size_t n, const gcr_rect_model* model, int arith,
                       double* r2_out) {
    if (solver < 0 || solver > 2 || cls < 0 || cls > (solver == 2 ? 1 : 0) || !model || (n && (!features || !r2_out)))
        return set_err(GCR_EINVAL, "bad residual request");
    return guard([&]() -> int {
        gcr_problem P;
        P.solver = solver;
        P.K = solver == 2 ? 2 : 1;
        // the features as class `cls` (fill_host_classes: glibc pow / sincos)
        fill_host_classes(solver, features, cls == 0 ? n : 0, features, cls == 1 ? n : 0, P.hc);
        const RectModel m{model->x0, model->y0, model->s, model->h7, model->h8, model->alpha, model->phi};
        const ValueConst vc = value_const(m, solver == 1, cls == 1);
        for (size_t i = 0; i < n; ++i)
            r2_out[i] = arith == 0 ? host_value(&P, cls, i, m, vc) : host_r2<GlibcMath>(&P, cls, i, m);
        return GCR_OK;
    });
}
double gcr_host_math(int op, double a, double b) {
    double sn, cs;
    switch (op) {
        case 0: return dm::dm_log(a);
        case 1: return dm::dm_pow_m3(a);
        case 2: return dm::dm_atan2(a, b);
        case 3: return a / b;
        case 5: return dm::clip_angle_small(a);
        case 6: return dm::clip_angle(a);
        case 8: return dm::dm_log_fd(a);
        case 9: dm::dm_sincos(a, sn, cs); return sn;
        case 10: dm::dm_sincos(a, sn, cs); return cs;
        case 11: return dm::atan_ratio(a, b);
        default: return sqrt(a);
    }
}

int gcr_host_sample(uint64_t seed, uint64_t index, uint32_t sub, uint32_t stream, uint32_t cls, uint64_t n,
                    uint32_t m, uint32_t* out) {
    if (!out || m > 32) return set_err(GCR_EINVAL, "bad sample request");
    WordStream ws(seed, index, sub, stream, cls);
    return sample_distinct<32>(ws, n, (int)m, out) ? GCR_OK : set_err(GCR_EINTERNAL, "sample budget exhausted");
}

int gcr_debug_math(gcr_ctx* ctx, int op, const double* a, const double* b, size_t n, double* out) {
    if (!ctx || !a || !out || ((op == 2 || op == 3 || op == 11 || op == 12) && b == nullptr))
        return set_err(GCR_EINVAL, "null argument");
    return guard([&]() -> int {
        HIPC(hipSetDevice(ctx->device));
        double *da = nullptr, *db = nullptr, *dout = nullptr;
        HIPC(hipMalloc(reinterpret_cast<void**>(&da), n * sizeof(double) + 8));
        HIPC(hipMalloc(reinterpret_cast<void**>(&db), n * sizeof(double) + 8));
        HIPC(hipMalloc(reinterpret_cast<void**>(&dout), n * sizeof(double) + 8));
        HIPC(hipMemcpy(da, a, n * sizeof(double), hipMemcpyHostToDevice));
        if (b) HIPC(hipMemcpy(db, b, n * sizeof(double), hipMemcpyHostToDevice));
        HIPC(launch_math(op, da, db, n, dout, ctx->stream));
        HIPC(hipStreamSynchronize(ctx->stream));
        HIPC(hipMemcpy(out, dout, n * sizeof(double), hipMemcpyDeviceToHost));
        (void)hipFree(da);
        (void)hipFree(db);
        (void)hipFree(dout);
        return GCR_OK;
    });
}

int gcr_measure_hbm(gcr_ctx* ctx, size_t bytes, int iters, double* gbps_out) {
    if (!ctx || !gbps_out || iters < 1 || bytes < 16) return set_err(GCR_EINVAL, "invalid argument");
    bytes &= ~(size_t)15;
    return guard([&]() -> int {
        HIPC(hipSetDevice(ctx->device));
        void *src = nullptr, *dst = nullptr;
        HIPC(hipMalloc(&src, bytes));
        if (hipMalloc(&dst, bytes) != hipSuccess) {
            (void)hipFree(src);
            return set_err(GCR_ENOMEM, "hipMalloc of %zu bytes failed", bytes);
        }
        hipError_t e = hipMemsetAsync(src, 0x3f, bytes, ctx->stream);
        double best = 0.0;
        for (int it = -2; it < 2 * iters && e == hipSuccess; ++it) {      // two untimed copies first
            e = hipEventRecord(ctx->ev0, ctx->stream);
            if (e == hipSuccess) e = launch_hbm_copy(src, dst, bytes, it & 1, ctx->stream);
            if (e == hipSuccess) e = hipEventRecord(ctx->ev1, ctx->stream);
            if (e == hipSuccess) e = hipEventSynchronize(ctx->ev1);
            float ms = 0.f;
            if (e == hipSuccess) e = hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
            if (e == hipSuccess && it >= 0 && ms > 0.f) best = std::max(best, 2.0 * (double)bytes / (ms * 1e6));
        }
        (void)hipFree(src);
        (void)hipFree(dst);
        HIPC(e);
        *gbps_out = best;
        return GCR_OK;
    });
}

int gcr_warp_perspective(gcr_ctx* ctx, const void* src, int src_h, int src_w, int channels, int dtype,
                         const double M[9], int border_mode, const double border_value[4], void* dst, int dst_h,
                         int dst_w) {
    if (!ctx || !src || !M || !dst) return set_err(GCR_EINVAL, "null argument");
    if (src_h <= 0 || src_w <= 0 || dst_h < 0 || dst_w < 0) return set_err(GCR_EINVAL, "invalid image size");
    if (channels < 1 || channels > 4) return set_err(GCR_EINVAL, "channels must be 1..4, got %d", channels);
    if (dtype != 0 && dtype != 1) return set_err(GCR_EINVAL, "dtype must be 0 (uint8) or 1 (float32)");
    if (border_mode != 0 && border_mode != 1) return set_err(GCR_EINVAL, "border_mode must be 0 or 1");
    return guard([&]() -> int {
        HIPC(hipSetDevice(ctx->device));
        const size_t esz = dtype == 0 ? 1 : 4;
        const size_t sbytes = (size_t)src_h * src_w * channels * esz;
        const size_t dbytes = (size_t)dst_h * dst_w * channels * esz;
        WarpMap wm{};
        for (int i = 0; i < 9; ++i) wm.m[i] = M[i];
        for (int c = 0; c < 4; ++c) wm.border[c] = border_value ? (float)border_value[c] : 0.f;
        void *ds = nullptr, *dd = nullptr;
        HIPC(hipMalloc(&ds, sbytes));
        hipError_t e = hipMalloc(&dd, dbytes ? dbytes : 1);
        if (e == hipSuccess) e = hipMemcpyAsync(ds, src, sbytes, hipMemcpyHostToDevice, ctx->stream);
        if (e == hipSuccess)
            e = launch_warp(ds, src_h, src_w, channels, dtype, wm, dd, dst_h, dst_w, border_mode, ctx->stream);
        if (e == hipSuccess && dbytes) e = hipMemcpyAsync(dst, dd, dbytes, hipMemcpyDeviceToHost, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        (void)hipFree(ds);
        if (dd) (void)hipFree(dd);
        HIPC(e);
        return GCR_OK;
    });
}

int gcr_host_grid_edges(const double* points, size_t n, int dims, const double* cell_size, uint64_t cell_number,
                        uint32_t* edges_out, size_t cap, size_t* m_out) {
    if ((!points && n) || !cell_size || !m_out || dims < 1 || dims > 4 || (cap && !edges_out))
        return set_err(GCR_EINVAL, "invalid argument");
    return guard([&]() -> int {
        std::vector<double> cols[4];
        const double* cp[4] = {};
        for (int d = 0; d < dims; ++d) {
            cols[d].resize(n);
            for (size_t i = 0; i < n; ++i) cols[d][i] = points[i * dims + d];
            cp[d] = cols[d].data();
        }
        NeighbourEdges e;
        grid_edges(cp, dims, n, cell_size, cell_number, e);
        *m_out = e.u.size();
        for (size_t k = 0; k < e.u.size() && k < cap; ++k) {
            edges_out[2 * k] = e.u[k];
            edges_out[2 * k + 1] = e.v[k];
        }
        return GCR_OK;
    });
}

int gcr_host_bk_energy(size_t n, const double* unary, const uint32_t* edges, const double* pair, size_t m,
                       uint8_t* seg) {
    if ((!unary && n) || (m && (!edges || !pair)) || (!seg && n)) return set_err(GCR_EINVAL, "null argument");
    return guard([&]() -> int {
        MaxFlow g;
        g.reset(n, m);
        for (size_t i = 0; i < n; ++i) g.add_term1((int32_t)i, unary[2 * i], unary[2 * i + 1]);
        for (size_t k = 0; k < m; ++k) {
            if (edges[2 * k] >= n || edges[2 * k + 1] >= n || edges[2 * k] == edges[2 * k + 1])
                return set_err(GCR_EINVAL, "invalid edge %zu", k);
            g.add_term2((int32_t)edges[2 * k], (int32_t)edges[2 * k + 1], pair[4 * k], pair[4 * k + 1],
                        pair[4 * k + 2], pair[4 * k + 3]);
        }
        g.maxflow();
        for (size_t i = 0; i < n; ++i) seg[i] = g.is_sink((int32_t)i) ? 1 : 0;
        return GCR_OK;
    });
}

int gcr_host_labeling(const double* r2, size_t n, double sqt, double lambda, const double* points, int dims,
                      const double* cell_size, uint64_t cell_number, uint8_t* seg) {
    if ((!r2 && n) || (!seg && n) || (cell_number && (!points || !cell_size || dims < 1 || dims > 4)))
        return set_err(GCR_EINVAL, "invalid argument");
    return guard([&]() -> int {
        NeighbourEdges e;
        if (cell_number) {
            std::vector<double> cols[4];
            const double* cp[4] = {};
            for (int d = 0; d < dims; ++d) {
                cols[d].resize(n);
                for (size_t i = 0; i < n; ++i) cols[d][i] = points[i * dims + d];
                cp[d] = cols[d].data();
            }
            grid_edges(cp, dims, n, cell_size, cell_number, e, false);
        }
        std::vector<double> q;
        std::vector<uint8_t> sg;
        graphcut_labeling(r2, n, sqt, lambda, e, q, sg);
        std::memcpy(seg, sg.data(), n);
        return GCR_OK;
    });
}

double gcr_host_weighted_mode(const double* angles, const double* weights, size_t n, double bin_width) {
    if (n && (!angles || !weights)) return 0.0 / 0.0;
    std::vector<double> a(angles, angles + n), w(weights, weights + n);
    return weighted_mode(a, w, bin_width);
}

}  // extern "C"
