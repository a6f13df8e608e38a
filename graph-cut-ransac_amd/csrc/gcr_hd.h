// gcr_hd.h -- host/device qualifiers and bit helpers shared by the HIP kernels
// and the host-side engine.  Every function that must give bit-identical results
// on the CPU and on gfx950 is written once, as GCR_HD, and compiled by hipcc for
// both targets with -ffp-contract=off (no silent FMA contraction on either side).
#pragma once

#include <stdint.h>
#include <math.h>
#include <float.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GCR_HD __host__ __device__ __forceinline__
#define GCR_DEVICE __device__ __forceinline__
#else
#define GCR_HD inline
#define GCR_DEVICE inline
#endif

namespace gcr {

GCR_HD uint64_t as_u64(double x) { return __builtin_bit_cast(uint64_t, x); }
GCR_HD double as_f64(uint64_t u) { return __builtin_bit_cast(double, u); }
GCR_HD uint32_t hi32(double x) { return (uint32_t)(as_u64(x) >> 32); }
GCR_HD uint32_t lo32(double x) { return (uint32_t)as_u64(x); }

// Explicit, correctly rounded fused multiply-add on both sides (v_fma_f64 on
// gfx950, glibc fma / vfmadd on x86-64).  Only used where the algorithm asks
// for it; plain a*b+c is never contracted because of -ffp-contract=off.
GCR_HD double fma_rn(double a, double b, double c) { return __builtin_fma(a, b, c); }

GCR_HD bool is_nan(double x) { return x != x; }

}  // namespace gcr
