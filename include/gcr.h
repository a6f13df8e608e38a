/*
 * gcr.h -- C ABI of the MI355X-native Graph-Cut RANSAC rectification engine.
 *
 * This is the drop-in boundary for the reference's hot path.  Each entry point
 * replaces one C++ function that pygcransac's pybind11 layer binds today
 * (yuvalnis/graph-cut-ransac, src/pygcransac/include/gcransac_python.h):
 *
 *   gcr_rect_scale_only(..., original=0)  <- findRectifyingHomographyScaleOnly_
 *                                            (gcransac_python.h:7-18, .cpp:32-142)
 *   gcr_rect_scale_only(..., original=1)  <- findRectifyingHomographyScaleOnlyOriginal_
 *                                            (gcransac_python.h:20-31, .cpp:144-254)
 *   gcr_rect_sift(...)                    <- findRectifyingHomographySIFT_
 *                                            (gcransac_python.h:33-47, .cpp:256-406)
 *
 * Conventions (no C++ or torch types cross this boundary):
 *   - features are row-major N x 3 float64 arrays, exactly the flat buffers the
 *     reference copies out of numpy (bindings.cpp:12-17, 234-250);
 *   - the caller owns every buffer; masks are N bytes (0/1);
 *   - H_out is the row-major 3x3 homography model.getHomography() / H22
 *     (gcransac_python.cpp:95-104);
 *   - return value >= 0 is the total number of inliers (the reference's int
 *     return, gcransac_python.cpp:141/405), < 0 is an error code; the message is
 *     available from gcr_last_error() (thread-local).  -EINVAL maps to Python
 *     ValueError, everything else to RuntimeError.
 *   - no exceptions cross the ABI; functions are thread-safe for distinct
 *     contexts; one context per device.
 */
#ifndef GCR_H_
#define GCR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GCR_ABI_VERSION 5

/* error codes */
#define GCR_OK 0
#define GCR_EINTERNAL (-1)
#define GCR_EHIP (-5)
#define GCR_ENOMEM (-12)
#define GCR_ENODEV (-19)
#define GCR_EINVAL (-22)

/* solver kinds (types.h:43-59 estimator typedefs) */
#define GCR_SOLVER_SCALE3 0          /* RectifyingHomographyThreeSIFTSolver         */
#define GCR_SOLVER_SCALE3_ORIGINAL 1 /* RectifyingHomographyThreeSIFTSolverOriginal */
#define GCR_SOLVER_SIFT22 2          /* RectifyingHomographyTwoSIFTSolver           */
#define GCR_SOLVER_HOMOGRAPHY4 3     /* 4-point homography (upstream GC-RANSAC)     */
#define GCR_SOLVER_FUNDAMENTAL7 4    /* 7-point fundamental matrix (upstream)       */

typedef struct gcr_ctx gcr_ctx;
typedef struct gcr_problem gcr_problem;

/* Mirrors utils::Settings (settings.h:42-74) for the fields the Python entry
 * points set (gcransac_python.cpp:79-85, 191-197, 314-321), plus extensions. */
typedef struct gcr_params {
    double scale_residual_thresh;        /* settings.threshold(0)                         */
    double orientation_residual_thresh;  /* settings.threshold(1) (SIFT only)             */
    double spatial_coherence_weight;     /* lambda; binding default 0.0                   */
    uint64_t min_iteration_number;       /* binding default 10000                         */
    uint64_t max_iteration_number;       /* binding default 10000                         */
    uint64_t max_local_optimization_number; /* binding default 50                        */
    double confidence;                   /* settings.h:60 default 0.95 (not set by Python) */
    uint64_t seed;                       /* extension: Philox key (reference is unseeded) */
    uint32_t batch_slots;                /* extension: outer-iteration slots per launch, 0 = auto */
    uint32_t flags;                      /* bit 0: disable local optimisation (bench only) */
    /* extension (homography / fundamental matrix only): the neighbourhood grid
     * over (x1, y1, x2, y2) whose cells give labeling()'s pairwise terms
     * (GridNeighborhoodGraph<4>, grid_neighborhood_graph.h:229-301); cell
     * sizes in pixels, cell_number cells along every axis; 0 = the empty grid
     * of the reference's entry points (no pairwise terms).  A cell size of
     * exactly 0 (ABI 5) is taken from the data: the column's largest finite
     * coordinate + 1 (at least 1) over cell_number, as
     * pygcransac.grid_cell_sizes computes it for an unknown image size */
    double cell_size[4];
    uint32_t cell_number;
    uint32_t reserved;
} gcr_params;

#define GCR_FLAG_NO_LO 1u

/* model.h: NormalizingTransform{x0,y0,s}, RectifyingHomography{h7,h8},
 * ScaleBased{alpha}, OrientationBased{phi}. */
typedef struct gcr_rect_model {
    double x0, y0, s, h7, h8, alpha, phi;
} gcr_rect_model;

/* utils::RANSACStatistics (statistics.h:43-64) plus per-phase timings. */
typedef struct gcr_stats {
    uint64_t iteration_number;
    uint64_t local_optimization_number;
    uint64_t graph_cut_number;
    uint64_t slots;               /* outer-loop bodies executed                     */
    uint64_t hypotheses;          /* models scored in the main loop                 */
    uint64_t hypotheses_computed; /* models scored on the GPU incl. speculative     */
    uint64_t lo_models;           /* models scored inside local optimisation        */
    uint64_t launches;
    double score;                 /* statistics.score                               */
    double ms_setup, ms_generate, ms_score, ms_replay, ms_lo, ms_refit, ms_total;
    double ms_score_kernel;       /* summed HIP-event time of the scoring kernels   */
    double ms_lo_lists;           /* LO: inlier lists (GPU labeling + copy back)    */
    double ms_lo_fit;             /* LO: sample draws + least-squares fits (host)   */
    double ms_lo_score;           /* LO: scoring the trial models (GPU)             */
    double ms_refit_fit;          /* final refit: the non-minimal fit itself (system,
                                     QR, weighted mode); the rest of ms_refit is the
                                     buffer reconciliation, rescoring and lists      */
    uint64_t prefetched_chunks;   /* chunks generated + scored on the side stream
                                     while the host replayed the previous one        */
    /* decisions in the reference's arithmetic (glibc; csrc/exact.h): the kernels
     * flag every decision whose detmath residual lies within the proven
     * twin-glibc bound of its threshold, and the host takes it with glibc */
    uint64_t exact_models;        /* models rescored / relabelled on the host       */
    uint64_t exact_pairs;         /* (feature, model) decisions taken with glibc    */
    uint64_t exact_flips;         /* ... that differ from the detmath decision      */
    double ms_exact;              /* host time of those recounts                    */
    /* score comparisons in glibc (exact.h ScoreBound): two value scores closer
     * than their proven bounds are compared by their glibc scores */
    uint64_t near_ties;           /* comparisons decided in glibc                   */
    uint64_t near_tie_flips;      /* ... whose outcome differs from the values'     */
    /* LO trials are compared on approximate scores within a proven bound of
     * the exact ones; a round the bound leaves open is folded exactly */
    uint64_t lo_refolds;          /* LO rounds folded exactly for a comparison      */
    /* the final refit's inlier lists decoded from the MSAC ballots of the
     * chunk launch that found the best (1) instead of mask launches (0) */
    uint64_t chunk_msac_lists;
} gcr_stats;

/* ---- context ---------------------------------------------------------- */
const char* gcr_last_error(void);
int gcr_abi_version(void);
int gcr_device_count(void);
/* SHA-256 prefix (16 hex) of the sources the GPU code object was built from
 * (kernels.hip + device headers + build flags); profiles are keyed by it */
const char* gcr_kernel_build_id(void);
int gcr_create(int device, gcr_ctx** out);
void gcr_destroy(gcr_ctx* ctx);
/* hipDeviceSynchronize on the context's device */
int gcr_synchronize(gcr_ctx* ctx);
void gcr_default_params(gcr_params* p);

/* ---- drop-in entry points (one call = one reference call) ---------------- */
int gcr_rect_scale_only(gcr_ctx* ctx, const double* features, size_t n, const gcr_params* params, int original,
                        uint8_t* mask_out, double* H_out, gcr_rect_model* model_out, gcr_stats* stats_out);

int gcr_rect_sift(gcr_ctx* ctx, const double* scale_features, size_t n_scale, const double* orientation_features,
                  size_t n_orientation, const gcr_params* params, uint8_t* scale_mask_out,
                  uint8_t* orientation_mask_out, double* H_out, gcr_rect_model* model_out, gcr_stats* stats_out);

/* 4-point homography (an EXTENSION: this fork has no
 * homography estimator, finding 0.1 -- the entry point upstream pygcransac's
 * findHomography would bind).  correspondences: row-major N x 4 float64
 * (x1, y1, x2, y2); threshold = params->scale_residual_thresh (pixels, second
 * image); mask_out: N bytes; H_out: row-major 3x3 with H[2][2] = 1.  Returns
 * the number of inliers (0: no model, H_out untouched) or < 0 on error. */
int gcr_find_homography(gcr_ctx* ctx, const double* correspondences, size_t n, const gcr_params* params,
                        uint8_t* mask_out, double* H_out, gcr_stats* stats_out);

/* 7-point fundamental matrix (an EXTENSION like
 * gcr_find_homography -- what upstream pygcransac's findFundamentalMatrix
 * would bind).  Same buffers as gcr_find_homography; the residual is the
 * squared Sampson distance, F_out is row-major 3x3 with unit Frobenius norm
 * (x2^T F x1 = 0). */
int gcr_find_fundamental_matrix(gcr_ctx* ctx, const double* correspondences, size_t n, const gcr_params* params,
                                uint8_t* mask_out, double* F_out, gcr_stats* stats_out);

/* ---- batches of independent problems (SURVEY.md §8(b) gcr_rect_batch,
 * BASELINE configs[4]) ----------------------------------------------------- */
typedef struct gcr_batch_item {
    int solver;                  /* GCR_SOLVER_*                                   */
    const double* f0;            /* N0 x 3 features, or N0 x 4 correspondences     */
    size_t n0;
    const double* f1;            /* orientation features (SIFT22), else NULL       */
    size_t n1;
    gcr_params params;
    uint8_t* mask0_out;          /* caller-owned, n0 bytes                          */
    uint8_t* mask1_out;          /* caller-owned, n1 bytes (SIFT22), else NULL      */
    double H_out[9];
    gcr_rect_model model_out;
    gcr_stats stats_out;
    int result;                  /* inlier count (0: no model) or error code        */
} gcr_batch_item;
/* Solve n independent problems on one device.  `concurrency` host threads,
 * each with its own context (HIP stream + workspace), take problems from a
 * shared counter, longest first (estimated from the solver and the feature
 * count), so one problem's host phases (replay, LO fits, refit control)
 * overlap another's kernels and the batch does not end on a long problem
 * started last.  Results are per item; returns
 * GCR_OK, or the first error code (message in gcr_last_error()). */
int gcr_solve_batch(int device, gcr_batch_item* items, size_t n, int concurrency);

/* ---- device-resident problems (benchmarks, problem batches) -------------- */
/* Uploads the features once; runs reuse the HBM-resident copy.  f1 is the
 * orientation set for GCR_SOLVER_SIFT22 and NULL otherwise. */
int gcr_problem_create(gcr_ctx* ctx, int solver, const double* f0, size_t n0, const double* f1, size_t n1,
                       gcr_problem** out);
void gcr_problem_destroy(gcr_problem* prob);
/* full estimator call on the resident problem (same semantics as gcr_rect_*) */
int gcr_problem_run(gcr_problem* prob, const gcr_params* params, uint8_t* mask0_out, uint8_t* mask1_out,
                    double* H_out, gcr_rect_model* model_out, gcr_stats* stats_out);

/* One problem over `world` processes: every rank
 * calls this with the same problem and params.  Each fetched chunk of slots is
 * split into `world` contiguous blocks; rank r generates and scores block r
 * on its own device, and `allgather` (host memory: `bytes` from every rank
 * into recv, rank-major -- e.g. RCCL all_gather over xGMI, or gloo) hands
 * every rank the whole chunk.  The replay, LO and the final refit then run
 * identically on every rank, so all ranks return the single-rank result bit
 * for bit.  The callback returns 0 on success. */
typedef int (*gcr_allgather_fn)(void* user, const void* send, void* recv, size_t bytes);
int gcr_problem_run_sharded(gcr_problem* prob, const gcr_params* params, int rank, int world,
                            gcr_allgather_fn allgather, void* user, uint8_t* mask0_out, uint8_t* mask1_out,
                            double* H_out, gcr_rect_model* model_out, gcr_stats* stats_out);

/* The same run with the exchange inside the engine: a communicator rank
 * (RCCL over xGMI, one process per GPU) all-gathers the device-resident block
 * summaries with ncclAllGather on the context's side stream, behind the
 * summary kernel -- no host callback, no host staging of the send side, one
 * copy of the gathered records into pinned memory.  gcr_comm_unique_id on one
 * rank, the id handed to every rank (e.g. a torch.distributed broadcast),
 * then gcr_comm_create on every rank (collective). */
#define GCR_COMM_ID_BYTES 128
typedef struct gcr_comm gcr_comm;
int gcr_comm_unique_id(uint8_t id_out[GCR_COMM_ID_BYTES]);
int gcr_comm_create(gcr_ctx* ctx, int rank, int world, const uint8_t id[GCR_COMM_ID_BYTES], gcr_comm** out);
void gcr_comm_destroy(gcr_comm* comm);
int gcr_problem_run_comm(gcr_problem* prob, const gcr_params* params, gcr_comm* comm, uint8_t* mask0_out,
                         uint8_t* mask1_out, double* H_out, gcr_rect_model* model_out, gcr_stats* stats_out);

/* One pass of the hot path over one batch: draw and solve `nslots`
 * outer-iteration slots starting at `slot0`, MSAC-score every resulting model
 * against all features on the GPU, and return the best-scoring slot (first
 * strict maximum of the reference's update rule, `best < score &&
 * isValidModel`, GCRANSAC.h:440-446).  This is the throughput API of the hot
 * path: the rectification solvers' scores, inlier decisions and the 2-SIFT
 * best_model's phi are the kernels' own (the detmath twins, csrc/exact.h),
 * with no host recheck of flagged decisions or near-tie comparisons, so a
 * batch whose best is decided within the twin-glibc bounds can differ from
 * the reference's choice.  gcr_problem_run (and the pygcransac entry points)
 * take every decision, comparison and model in the reference's arithmetic.
 * Timings go to stats_out. */
typedef struct gcr_batch_result {
    uint64_t models;        /* hypotheses scored                        */
    uint64_t iterations;    /* sum of iteration increments of the batch */
    int64_t best_slot;      /* -1 if no model scored > 0                */
    double best_score;
    uint64_t best_inliers[2];
    gcr_rect_model best_model;
} gcr_batch_result;
int gcr_problem_verify_batch(gcr_problem* prob, const gcr_params* params, uint64_t slot0, uint32_t nslots,
                             gcr_batch_result* out, gcr_stats* stats_out);
/* `nbatches` consecutive batches of `nslots` slots (batch b covers slots
 * slot0 + b*nslots ...), queued back to back on the device with the per-batch
 * selection done on the GPU; out[] holds one result per batch.  One host
 * synchronisation per call.  Returns GCR_OK or an error code. */
int gcr_problem_verify_batches(gcr_problem* prob, const gcr_params* params, uint64_t slot0, uint32_t nslots,
                               uint32_t nbatches, gcr_batch_result* out, gcr_stats* stats_out);

/* ---- parity / debug hooks (used by tests; GPU required unless noted) ---- */
/* inc[i] in 1..101 (attempt of success) or 102 (no model), models[i] */
int gcr_debug_generate(gcr_problem* prob, uint64_t seed, uint64_t slot0, uint32_t nslots, uint8_t* inc_out,
                       gcr_rect_model* models_out);
/* raw MSAC accumulators for explicit models: counts, per-class sums, total */
int gcr_debug_score(gcr_problem* prob, const gcr_params* params, const gcr_rect_model* models, uint32_t nmodels,
                    uint32_t* n0, uint32_t* n1, double* v0, double* v1, double* tot);
/* The run loop's score comparison `score(a) < score(b)` (GCRANSAC.h:440) as
 * gcr_problem_run takes it: both models scored by the GPU small scorer (value
 * scores), compared directly when they are further apart than their proven
 * value-glibc bounds (csrc/exact.h ScoreBound), else by their glibc scores
 * recounted on the host.  Returns bit 0 the decision, bit 1 a near tie, bit 2
 * the value scores' own order; < 0 an error. */
int gcr_debug_score_less(gcr_problem* prob, const gcr_params* params, const gcr_rect_model* a,
                         const gcr_rect_model* b);
/* With GCR_EXCHANGE_LOG=1, the summary replay of the last run on the calling
 * thread logs every event that is a collective under gcr_comm (chunk issue,
 * re-summary) and every chunk it collected: 4 words per event (engine.cpp
 * t_xlog).  Copies min(count, cap) words to out (may be null); returns the
 * count.  No GPU needed. */
size_t gcr_debug_exchange_log(uint64_t* out, size_t cap);
/* inlier mask of one model: rule 0 = MSAC (2.25 thr^2), 1 = LO threshold
 * ((1.5 thr)^2), 2 = 1-class graph-cut labeling */
int gcr_debug_mask(gcr_problem* prob, const gcr_params* params, const gcr_rect_model* model, int cls, int rule,
                   uint8_t* mask_out);
/* the LO / final-refit fit of the given index lists on the problem's features;
 * use_gpu = 1 solves the hybrid least-squares system with the GPU refit path
 * (k_sift_rows + device QR), 0 on the host; both are bit-identical.  Returns 1
 * and the model, 0 if the fit is rejected, < 0 on error */
int gcr_debug_fit_nonminimal(gcr_problem* prob, const uint32_t* idx0, size_t k0, const uint32_t* idx1, size_t k1,
                             int use_gpu, gcr_rect_model* model_out);
/* host-only (no GPU): the LO / final-refit least-squares fit of the given index
 * lists (RectifyingHomographyEstimator::estimateModelNonminimal,
 * rectifying_homography_estimator.h:164-227); returns 1 and the model, 0 if the
 * fit is rejected, < 0 on error */
int gcr_host_fit_nonminimal(int solver, const double* f0, size_t n0, const double* f1, size_t n1, const uint32_t* idx0,
                            size_t k0, const uint32_t* idx1, size_t k1, gcr_rect_model* model_out);
/* correspondence problems (GCR_SOLVER_HOMOGRAPHY4 / _FUNDAMENTAL7): models
 * are 9 row-major doubles.  generate: homography -- inc[i] as above, H_out 9
 * per slot; fundamental -- 3 hypotheses per slot (inc_out 3 bytes, H_out 27
 * doubles per slot): inc[3s] as above, inc[3s+k] = 0 if the sample's k-th
 * model exists, 255 if not.  score: n0 / v0 / tot per model (MSAC threshold
 * 2.25 thr); mask: rules as gcr_debug_mask */
int gcr_debug_generate_h(gcr_problem* prob, uint64_t seed, uint64_t slot0, uint32_t nslots, uint8_t* inc_out,
                         double* H_out);
int gcr_debug_score_h(gcr_problem* prob, const gcr_params* params, const double* H, uint32_t nmodels, uint32_t* n0,
                      double* v0, double* tot);
int gcr_debug_mask_h(gcr_problem* prob, const gcr_params* params, const double* H, int rule, uint8_t* mask_out);
/* host-only: normalised least-squares homography of the listed
 * correspondences (the LO / final-refit fit); 1 = fitted, 0 = rejected */
int gcr_host_fit_h(const double* correspondences, size_t n, const uint32_t* idx, size_t k, double* H_out);
/* host-only: the fundamental-matrix LO / refit fit (7 points: 7-point solver's
 * first model; more: normalised 8-point with rank-2 projection) */
int gcr_host_fit_f(const double* correspondences, size_t n, const uint32_t* idx, size_t k, double* F_out);
/* host-only: RectifyingHomography::getHomography (model.h:211-226), row-major */
void gcr_host_homography(const gcr_rect_model* model, double* H_out);
/* host-only: squared residuals of one rectification model over n features of
 * class `cls` (0 scale, 1 orientation; solver 0-2), rows as the entry points
 * take them (x, y, scale | angle).  arith 0: the product's values (rect.h
 * scale_sq_value / orient_sq_value, what the kernels evaluate and fold);
 * 1: the reference's formulas in glibc (the decisions, exact.h). */
int gcr_host_residuals(int solver, int cls, const double* features, size_t n, const gcr_rect_model* model, int arith,
                       double* r2_out);
/* host-only (no GPU): the graph-cut labeling's pieces (graphcut.h).
 * grid_edges: the neighbourhood grid's edges over n points of `dims` (<= 4)
 * row-major coordinates in labeling()'s order (GCRANSAC.h:821-857,
 * grid_neighborhood_graph.h:229-301); writes min(m, cap) pairs, *m_out = m.
 * bk_energy: BK st-mincut of sum_i E_i(x_i) + sum_k E_k(x_u, x_v), unary
 * (n x 2: E(0), E(1)), pair (m x 4: E(00), E(01), E(10), E(11)), Energy::
 * add_term1 / add_term2 (energy.h:204-245); seg[i] = 1 iff SINK.
 * labeling: labeling() itself as the engine runs it -- squared residuals r2,
 * squared truncated threshold sqt, lambda, the grid over n points of `dims`
 * row-major coordinates (cell_number 0: no grid); seg[i] = 1 iff inlier. */
int gcr_host_grid_edges(const double* points, size_t n, int dims, const double* cell_size, uint64_t cell_number,
                        uint32_t* edges_out, size_t cap, size_t* m_out);
int gcr_host_bk_energy(size_t n, const double* unary, const uint32_t* edges, const double* pair, size_t m,
                       uint8_t* seg);
int gcr_host_labeling(const double* r2, size_t n, double sqt, double lambda, const double* points, int dims,
                      const double* cell_size, uint64_t cell_number, uint8_t* seg);
/* host-only: findWeightedMode (two_sift.hpp:354-394) as the fits use it */
double gcr_host_weighted_mode(const double* angles, const double* weights, size_t n, double bin_width);
/* host-only (no GPU): deterministic math and sampler used on both sides */
double gcr_host_log(double x);
double gcr_host_pow_m3(double t);
double gcr_host_atan2(double y, double x);
/* host-only: the op of gcr_debug_math below on one operand pair (ops 0-6,
 * 8-11; the host twin of each device primitive) */
double gcr_host_math(int op, double a, double b);
int gcr_host_sample(uint64_t seed, uint64_t index, uint32_t sub, uint32_t stream, uint32_t cls, uint64_t n,
                    uint32_t m, uint32_t* out);
/* device evaluation of the same primitives over arrays (GPU parity tests):
 * op 0 log(a), 1 pow_m3(a), 2 atan2(a, b), 3 a / b, 4 sqrt(a),
 * 5 clip_angle_small(a), 6 clip_angle(a), 8 round 3's log (dm_log_fd),
 * 9 / 10 sin / cos of a (dm_sincos), 11 atan(a / b) for 0 <= a <= b
 * (atan_ratio, the orientation value's);
 * op 7 (n >= 2): out[0] = the block-parallel exact in-order sum of a[0, n)
 * (k_lo_chain's fold), out[1] = the same sum by a sequential loop;
 * op 12 (7 <= n <= 8192, split h = b[0]): out[0..2] = the three chains of
 * k_lo_chain's two-class fold (a[0, h) from +0, a[h, n) from +0, a[h, n)
 * from out[0]), out[3..5] = the same by sequential loops, out[6] = cycles */
int gcr_debug_math(gcr_ctx* ctx, int op, const double* a, const double* b, size_t n, double* out);
/* perspective_warp's resampling (examples/utils.py:92-123, cv2.warpPerspective
 * with INTER_LINEAR): dst pixel (x, y) <- bilinear sample of src at
 * M (x, y, 1)^T / w, M = the dst -> src map (the inverse of the translated
 * homography), row-major.  Host buffers, channels interleaved, 1 <= channels
 * <= 4; dtype 0 = uint8 (rounded, saturated), 1 = float32.  border_mode 0 =
 * constant border_value[c], 1 = replicate the nearest edge pixel. */
int gcr_warp_perspective(gcr_ctx* ctx, const void* src, int src_h, int src_w, int channels, int dtype,
                         const double M[9], int border_mode, const double border_value[4], void* dst, int dst_h,
                         int dst_w);
/* measurement (bench.py): achievable HBM bandwidth of the device, GB/s of
 * read + write traffic of a streaming device-to-device copy of `bytes` bytes,
 * best of `iters` timed copies of each of two variants, plain and nontemporal
 * (no reference counterpart) */
int gcr_measure_hbm(gcr_ctx* ctx, size_t bytes, int iters, double* gbps_out);

#ifdef __cplusplus
}
#endif

#endif /* GCR_H_ */
