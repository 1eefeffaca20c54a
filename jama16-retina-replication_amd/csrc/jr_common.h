// jr_common.h — shared helpers for the libjr.so HIP sources (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <cstdlib>
#include <string>

#include "jr_error.h"

namespace jr {

// Map the last HIP launch error (if any) to JR_ERR_HIP.
int check_launch(const char* what);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Device words the library owns per (device, stream, kind) (jr_api.cpp):
// zeroed once when allocated (in order on that stream) and used only by
// launches on that stream, which run in order -- so a kernel that leaves its
// words zero again (the stream-K hand-off flags, kind 0) needs no memset
// before each launch.  A capturing stream gets a fresh private region per
// call: graph replays may run on any stream.  nullptr if allocation failed.
unsigned* stream_scratch(hipStream_t s, int kind, size_t words);

// The current device's error word (jr_api.cpp): kernels count device-side
// failures into it (vector atomics); jr_device_check() reads, reports and
// clears it.  Allocated by jr_init (or on first use outside a capture).
unsigned* device_error_word(hipStream_t s);

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Bijective XCD-aware remap of a flat workgroup id (cdna_hip_programming.md
// §5 "XCD swizzle must be bijective"): blocks b, b+8, b+16 ... are dealt to one
// XCD by the dispatcher, so consecutive remapped ids land on one XCD's L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}
// round-to-nearest-even f32 -> bf16 (NaN kept NaN by the cast path)
__device__ __forceinline__ uint16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&h);
}

// BatchNormalization(scale=False) pre-activation, in one fixed rounding
// order: every kernel that applies or differentiates it (jr_bn.hip, the
// fused BN + max-pool of jr_pool.hip) sees bit-identical values and ReLU masks.
__device__ __forceinline__ float bn_xhat(float x, float mean, float invstd) {
  return __fmul_rn(__fsub_rn(x, mean), invstd);
}
__device__ __forceinline__ float bn_pre(float x, float mean, float invstd, float beta) {
  return __fadd_rn(bn_xhat(x, mean, invstd), beta);
}

// Canonical combine of ONE channel's fused BN-statistics partials (the conv
// epilogue's / split-K reduce's per-row-group (mean, M2) of R rows each; the
// last group holds the rest of the M rows) into (mean, invstd): an aligned
// group of 8 lanes, lane j summing partials j, j+8, ... in order, shifted by
// the first partial's mean K, in fp64; an xor butterfly over the 8 lanes.
// k_stats_finalize8 (jr_conv.hip) and jr_bn_relu_apply_stats (jr_bn.hip, the
// finalize folded into the BN apply) both call this, so they give bitwise the
// same statistics.  Every lane of the group returns the result.
constexpr int kStatsLanes = 8;
constexpr int kFoldMaxP = 512;   // partials per channel that this combine (and so the fold) takes
__device__ __forceinline__ void stats_combine8(const float* __restrict__ pm, const float* __restrict__ pq, int P,
                                               int R, int M, float eps, int j, float* mean, float* invstd) {
  const double K = pm[0];
  double sn = 0, sd = 0, sq = 0;
  constexpr int U = 16;   // loads in flight per lane and array
  for (int i0 = j; i0 < P; i0 += kStatsLanes * U) {
    float vm[U], vq[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {   // clamped unconditional loads, all issued before any use
      const int ic = min(i0 + kStatsLanes * u, P - 1);
      vm[u] = pm[ic];
      vq[u] = pq[ic];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + kStatsLanes * u;
      if (i < P) {
        const double c = (double)min(max(M - i * R, 0), R);
        const double d = (double)vm[u] - K;
        sn += c;
        sd += c * d;
        sq += (double)vq[u] + c * d * d;
      }
    }
  }
#pragma unroll
  for (int o = kStatsLanes / 2; o > 0; o >>= 1) {
    sn += __shfl_xor(sn, o, kStatsLanes);
    sd += __shfl_xor(sd, o, kStatsLanes);
    sq += __shfl_xor(sq, o, kStatsLanes);
  }
  const double dm = sn > 0 ? sd / sn : 0.0;
  const double m2 = fmax(sq - sn * dm * dm, 0.0);
  *mean = (float)(K + dm);
  *invstd = (float)(1.0 / sqrt(m2 / (double)M + (double)eps));
}

// Element load/store of an activation in the path dtype.
template <typename T> struct Elt;
template <> struct Elt<float> {
  __device__ static float ld(const float* p) { return *p; }
  __device__ static void st(float* p, float v) { *p = v; }
};
template <> struct Elt<uint16_t> {
  __device__ static float ld(const uint16_t* p) { return bf2f(*p); }
  __device__ static void st(uint16_t* p, float v) { *p = f2bf(v); }
};

}  // namespace jr
