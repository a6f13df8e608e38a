// Microbenchmark: VALU issue cost per wave64 instruction class on gfx950, the
// per-class costs of bench.py's weighted VALU-issue floor (roofline.valu_issue).
//
// Each wave runs kIters x kChains independent instructions of one class (kChains
// independent register chains, so latency hides behind issue).  Round 5: every
// wave reads BOTH counters around its loop -- s_memtime (clock64, the counter
// round 4 priced in "cycles") and s_memrealtime (wall_clock64, a constant
// 100 MHz) -- so each class is priced in NANOSECONDS per instruction per SIMD
// (no clock assumption) and the s_memtime rate is measured (its MHz).
// waves_per_simd 1 / 2 / 4: one wave alone on its SIMD, or several sharing it
// (cost per instruction PER SIMD = elapsed / waves / instructions per wave).
//
// A last kernel runs a KNOWN MIX of classes in one loop; the model's
// prediction (sum of count x measured per-class cost) is printed beside the
// measured time, the validation of the per-class model (VERDICT round 4,
// item 5: within 10 %).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/valu_issue.hip -o tools/micro/valu_issue.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

constexpr int kChains = 16;
constexpr int kIters = 4096;

enum Op {
    ADD_F64, FMA_F64, MUL_F64, RCP_F64, SQRT_F64, ADD_F32, FMA_F32, PK_FMA_F32, EXP_F32, RCP_F32, ADD_U32, CNDMASK,
    CNDMASK_SGPR, CVT_F64_I32, READLANE, WRITELANE, LDEXP_F64, FRACT_F64, MOV_B32, MOV_B64, XOR_B32, CMP_EQ_U32,
    CMP_LT_F64, MAD_U64_U32, LSHL_ADD_U64, MAX_F64, DIV_SCALE_F64, DIV_FMAS_F64, DIV_FIXUP_F64, MBCNT_LO, NOP_OPS
};
const char* kName[] = {"v_add_f64", "v_fma_f64", "v_mul_f64", "v_rcp_f64", "v_sqrt_f64", "v_add_f32", "v_fma_f32",
                       "v_pk_fma_f32", "v_exp_f32", "v_rcp_f32", "v_add_u32", "v_cndmask_b32(vcc)",
                       "v_cndmask_b32(s)", "v_cvt_f64_i32", "v_readlane_b32", "v_writelane_b32", "v_ldexp_f64",
                       "v_fract_f64", "v_mov_b32", "v_mov_b64", "v_xor_b32", "v_cmp_eq_u32", "v_cmp_lt_f64",
                       "v_mad_u64_u32", "v_lshl_add_u64", "v_max_f64", "v_div_scale_f64", "v_div_fmas_f64",
                       "v_div_fixup_f64", "v_mbcnt_lo_u32_b32"};

struct Stamp {
    unsigned long long mt, rt;      // s_memtime, s_memrealtime deltas of the timed loop
    unsigned long long r0, r1;      // s_memrealtime at the loop's start and end (absolute)
    unsigned hwid, xcc;             // HW_ID (simd / cu / sh / se) and XCC_ID of the wave
};

template <int OP>
__device__ __forceinline__ void op1(double& d, float& f, unsigned& u, unsigned long long& q, double dc, float fc,
                                    unsigned t, unsigned long long sm) {
    if constexpr (OP == ADD_F64) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d) : "v"(dc));
    if constexpr (OP == FMA_F64) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d) : "v"(dc));
    if constexpr (OP == MUL_F64) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d) : "v"(dc));
    if constexpr (OP == RCP_F64) asm volatile("v_rcp_f64 %0, %0" : "+v"(d));
    if constexpr (OP == SQRT_F64) asm volatile("v_sqrt_f64 %0, %0" : "+v"(d));
    if constexpr (OP == ADD_F32) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f) : "v"(fc));
    if constexpr (OP == FMA_F32) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f) : "v"(fc));
    if constexpr (OP == PK_FMA_F32) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(d) : "v"(dc));
    if constexpr (OP == EXP_F32) asm volatile("v_exp_f32 %0, %0" : "+v"(f));
    if constexpr (OP == RCP_F32) asm volatile("v_rcp_f32 %0, %0" : "+v"(f));
    if constexpr (OP == ADD_U32) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u) : "v"(t));
    if constexpr (OP == CNDMASK) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u) : "v"(t));
    if constexpr (OP == CNDMASK_SGPR) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(u) : "v"(t), "s"(sm));
    if constexpr (OP == CVT_F64_I32) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(d) : "v"(u));
    if constexpr (OP == READLANE) {
        unsigned s;
        asm volatile("v_readlane_b32 %0, %1, 5" : "=s"(s) : "v"(f));
        u += s;
    }
    if constexpr (OP == WRITELANE) asm volatile("v_writelane_b32 %0, %1, 7" : "+v"(u) : "s"((unsigned)sm));
    if constexpr (OP == LDEXP_F64) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d) : "v"(t));
    if constexpr (OP == FRACT_F64) asm volatile("v_fract_f64 %0, %0" : "+v"(d));
    if constexpr (OP == MOV_B32) asm volatile("v_mov_b32 %0, %1" : "=v"(u) : "v"(t));
    if constexpr (OP == MOV_B64) asm volatile("v_mov_b64 %0, %1" : "=v"(q) : "v"(dc));
    if constexpr (OP == XOR_B32) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u) : "v"(t));
    if constexpr (OP == CMP_EQ_U32) {
        unsigned long long m;
        asm volatile("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(m) : "v"(u), "v"(t));
        q ^= m;
    }
    if constexpr (OP == CMP_LT_F64) {
        unsigned long long m;
        asm volatile("v_cmp_lt_f64_e64 %0, %1, %2" : "=s"(m) : "v"(d), "v"(dc));
        q ^= m;
    }
    if constexpr (OP == MAD_U64_U32) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(q) : "v"(u), "v"(t));
    if constexpr (OP == LSHL_ADD_U64) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(q) : "v"(dc));
    if constexpr (OP == MAX_F64) asm volatile("v_max_f64 %0, %0, %1" : "+v"(d) : "v"(dc));
    if constexpr (OP == DIV_SCALE_F64) asm volatile("v_div_scale_f64 %0, vcc, %0, %1, %0" : "+v"(d) : "v"(dc));
    if constexpr (OP == DIV_FMAS_F64) asm volatile("v_div_fmas_f64 %0, %0, %1, %0" : "+v"(d) : "v"(dc));
    if constexpr (OP == DIV_FIXUP_F64) asm volatile("v_div_fixup_f64 %0, %0, %1, %0" : "+v"(d) : "v"(dc));
    if constexpr (OP == MBCNT_LO) asm volatile("v_mbcnt_lo_u32_b32 %0, -1, %0" : "+v"(u));
}

// The known mix: per chain and iteration 3 f64 add, 2 f64 mul, 1 f64 fma, 2
// u32 add, 2 cndmask (vcc), 1 mov_b32, 1 xor -- 12 VALU instructions
constexpr int kMixOps[][2] = {{ADD_F64, 3}, {MUL_F64, 2}, {FMA_F64, 1}, {ADD_U32, 2}, {CNDMASK, 2},
                              {MOV_B32, 1}, {XOR_B32, 1}};
constexpr int kMixVariant = 99;
constexpr int kPairBase = 1000;      // OP + kPairBase: OP interleaved with v_add_f64

template <int OP>
__global__ void k_issue(const double* in, double* out, Stamp* st) {
    const int t = threadIdx.x;
    double d[kChains];
    float f[kChains];
    unsigned u[kChains];
    unsigned long long q[kChains];
    for (int i = 0; i < kChains; ++i) {
        d[i] = in[(t + i) & 63];
        f[i] = (float)d[i];
        u[i] = (unsigned)(t * 7 + i);
        q[i] = (unsigned long long)(t + i);
    }
    const double dc = in[1];
    const float fc = (float)in[2];
    const unsigned long long sm = (unsigned long long)(in[3] > 0.0 ? 0x5555555555555555ull : 0x3ull);
    __syncthreads();
    const unsigned long long r0 = wall_clock64();
    const unsigned long long c0 = clock64();
#pragma unroll 1
    for (int it = 0; it < kIters; ++it) {
        if constexpr (OP >= kPairBase) {
            // OP - kPairBase alternating with v_add_f64 on the other chains:
            // X(0) A(1) X(2) A(3) .. then A(0) X(1) A(2) X(3) .. (16 X, 16 A)
#pragma unroll
            for (int i = 0; i < kChains; i += 2) {
                op1<OP - kPairBase>(d[i], f[i], u[i], q[i], dc, fc, t, sm);
                op1<ADD_F64>(d[i + 1], f[i + 1], u[i + 1], q[i + 1], dc, fc, t, sm);
            }
#pragma unroll
            for (int i = 0; i < kChains; i += 2) {
                op1<ADD_F64>(d[i], f[i], u[i], q[i], dc, fc, t, sm);
                op1<OP - kPairBase>(d[i + 1], f[i + 1], u[i + 1], q[i + 1], dc, fc, t, sm);
            }
        } else if constexpr (OP == kMixVariant) {
            // the mix's instructions in a fixed order, each over all chains
            // (consecutive instructions independent, as in the single-class runs)
#define GCR_MIX1(O)                                                                    \
    _Pragma("unroll") for (int i = 0; i < kChains; ++i) op1<O>(d[i], f[i], u[i], q[i], dc, fc, t, sm);
            GCR_MIX1(ADD_F64) GCR_MIX1(ADD_U32) GCR_MIX1(MUL_F64) GCR_MIX1(CNDMASK) GCR_MIX1(ADD_F64)
            GCR_MIX1(XOR_B32) GCR_MIX1(FMA_F64) GCR_MIX1(ADD_U32) GCR_MIX1(MUL_F64) GCR_MIX1(CNDMASK)
            GCR_MIX1(ADD_F64) GCR_MIX1(MOV_B32)
#undef GCR_MIX1
        } else {
#pragma unroll
            for (int i = 0; i < kChains; ++i) op1<OP>(d[i], f[i], u[i], q[i], dc, fc, t, sm);
        }
    }
    const unsigned long long c1 = clock64();
    const unsigned long long r1 = wall_clock64();
    unsigned hwid, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    double s = 0.0;
    for (int i = 0; i < kChains; ++i) s += d[i] + (double)f[i] + (double)u[i] + (double)q[i];
    out[blockIdx.x * blockDim.x + t] = s;
    if ((t & 63) == 0) st[blockIdx.x * (blockDim.x / 64) + t / 64] = Stamp{c1 - c0, r1 - r0, r0, r1, hwid, xcc};
}

struct Cost {
    double ns;          // per instruction per SIMD (realtime)
    double cyc;         // per instruction per SIMD (s_memtime)
    double mhz;         // s_memtime rate
    double ns_span;     // per instruction per SIMD from each SIMD's own span (HW_ID): the waves that
                        // ran on it, first start to last end, over the instructions they issued
    int simds, max_wps; // SIMDs seen, the most waves any one of them ran
};

template <int OP>
Cost run(const double* in, double* out, Stamp* st, int wps, int ninst, bool print) {
    // one workgroup per CU (256 CUs), 4 * wps waves: wps waves on each SIMD
    const int threads = 256 * wps, blocks = 256;
    hipLaunchKernelGGL(k_issue<OP>, dim3(blocks), dim3(threads), 0, 0, in, out, st);
    (void)hipDeviceSynchronize();
    const int nw = blocks * threads / 64;
    static Stamp h[4096];
    (void)hipMemcpy(h, st, nw * sizeof(Stamp), hipMemcpyDeviceToHost);
    double smt = 0, srt = 0;
    for (int i = 0; i < nw; ++i) {
        smt += (double)h[i].mt;
        srt += (double)h[i].rt;
    }
    smt /= nw;
    srt /= nw;
    const double insts = (double)kIters * kChains * ninst;
    Cost c;
    c.cyc = smt / insts / wps;
    c.ns = srt * 10.0 / insts / wps;            // 100 MHz ticks -> ns
    c.mhz = smt / (srt * 10.0) * 1000.0;
    // per SIMD (xcc, se, sh, cu, simd): its waves' span and instruction count
    struct S { unsigned long long lo, hi; int n; };
    static S sim[1 << 15];
    static unsigned keys[4096];
    int nk = 0;
    for (int i = 0; i < nw; ++i) {
        const unsigned hw = h[i].hwid;
        const unsigned key = ((h[i].xcc & 15u) << 11) | (((hw >> 13) & 7u) << 8) | (((hw >> 12) & 1u) << 7) |
                             (((hw >> 8) & 15u) << 3) | ((hw >> 4) & 3u);
        if (sim[key].n == 0) {
            keys[nk++] = key;
            sim[key] = S{h[i].r0, h[i].r1, 0};
        }
        sim[key].lo = h[i].r0 < sim[key].lo ? h[i].r0 : sim[key].lo;
        sim[key].hi = h[i].r1 > sim[key].hi ? h[i].r1 : sim[key].hi;
        ++sim[key].n;
    }
    double acc = 0.0;
    int mx = 0;
    for (int k = 0; k < nk; ++k) {
        const S& e = sim[keys[k]];
        acc += (double)(e.hi - e.lo) * 10.0 / (insts * e.n);
        mx = e.n > mx ? e.n : mx;
        sim[keys[k]] = S{0, 0, 0};
    }
    c.ns_span = acc / nk;
    c.simds = nk;
    c.max_wps = mx;
    if (print)
        printf("%-20s waves/SIMD %d: %7.3f ns (%6.2f s_memtime cycles) per instruction per SIMD; s_memtime %6.0f MHz; "
               "per-SIMD span %7.3f ns (%d SIMDs, at most %d waves on one)\n",
               OP == kMixVariant ? "MIX" : (OP >= kPairBase ? "PAIR" : kName[OP % kPairBase]), wps, c.ns, c.cyc,
               c.mhz, c.ns_span, c.simds, c.max_wps);
    return c;
}

Cost g_cost[NOP_OPS];       // alone, 4 waves per SIMD
Cost g_marg[NOP_OPS];       // marginal cost inside a stream of v_add_f64 (4 waves per SIMD)

template <int OP>
void run_all(const double* in, double* out, Stamp* st) {
    for (int wps : {1, 2, 4}) {
        const Cost c = run<OP>(in, out, st, wps, 1, true);
        if (wps == 4) g_cost[OP] = c;
    }
    // marginal: (time of 16 X + 16 v_add_f64) - (time of 16 v_add_f64), per X
    const Cost p = run<OP + kPairBase>(in, out, st, 4, 2, false);
    Cost m{};
    m.ns_span = 2.0 * p.ns_span - g_cost[ADD_F64].ns_span;
    m.ns = 2.0 * p.ns - g_cost[ADD_F64].ns;
    m.cyc = 2.0 * p.cyc - g_cost[ADD_F64].cyc;
    m.mhz = p.mhz;
    g_marg[OP] = m;
    printf("%-20s marginal in a v_add_f64 stream: %7.3f ns (%6.2f s_memtime cycles) per instruction per SIMD; "
           "per-SIMD span %7.3f ns\n",
           kName[OP], m.ns, m.cyc, m.ns_span);
    if constexpr (OP + 1 < NOP_OPS) run_all<OP + 1>(in, out, st);
}

int main() {
    double *in, *out;
    Stamp* st;
    (void)hipMalloc(&in, 64 * 8);
    (void)hipMalloc(&out, 256 * 1024 * 8);
    (void)hipMalloc(&st, 4096 * sizeof(Stamp));
    double h[64];
    for (int i = 0; i < 64; ++i) h[i] = 1.0 + 1e-3 * i;
    (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    for (int w = 0; w < 20; ++w) run<ADD_F64>(in, out, st, 4, 1, false);     // warm-up (clock ramp)
    run_all<0>(in, out, st);
    // the known mix, 4 waves per SIMD: measured against the per-class model
    int n = 0;
    double pred_ns = 0.0, pred_cyc = 0.0;
    for (const auto& oc : kMixOps) {
        n += oc[1];
        pred_ns += oc[1] * g_cost[oc[0]].ns;
        pred_cyc += oc[1] * g_cost[oc[0]].cyc;
    }
    const Cost m = run<kMixVariant>(in, out, st, 4, n, true);
    printf("MIX model (alone costs): predicted %.3f ns per mix iteration per SIMD, measured %.3f (residual %+.1f %%); "
           "s_memtime cycles predicted %.2f measured %.2f\n",
           pred_ns, m.ns * n, 100.0 * (pred_ns - m.ns * n) / (m.ns * n), pred_cyc, m.cyc * n);
    double mp_ns = 0.0;
    for (const auto& oc : kMixOps) mp_ns += oc[1] * g_marg[oc[0]].ns;
    printf("MIX model (marginal costs): predicted %.3f ns per mix iteration per SIMD, measured %.3f (residual %+.1f %%)\n",
           mp_ns, m.ns * n, 100.0 * (mp_ns - m.ns * n) / (m.ns * n));
    double ps_ns = 0.0, pm_ns = 0.0;
    for (const auto& oc : kMixOps) {
        ps_ns += oc[1] * g_cost[oc[0]].ns_span;
        pm_ns += oc[1] * g_marg[oc[0]].ns_span;
    }
    printf("MIX model (per-SIMD spans): alone %.3f, marginal %.3f ns predicted, measured %.3f (residuals %+.1f %%, "
           "%+.1f %%)\n",
           ps_ns, pm_ns, m.ns_span * n, 100.0 * (ps_ns - m.ns_span * n) / (m.ns_span * n),
           100.0 * (pm_ns - m.ns_span * n) / (m.ns_span * n));
    // machine-readable: per class [alone, marginal] ns per instruction per
    // SIMD from the per-SIMD spans, and the mix [measured, alone model,
    // marginal model]; the clock the s_memtime counter ran at
    printf("JSON {");
    for (int i = 0; i < NOP_OPS; ++i)
        printf("%s\"%s\": [%.4f, %.4f]", i ? ", " : "", kName[i], g_cost[i].ns_span, g_marg[i].ns_span);
    printf(", \"MIX\": [%.4f, %.4f, %.4f], \"s_memtime_mhz\": %.0f}\n", m.ns_span * n, ps_ns, pm_ns, m.mhz);
    return 0;
}
