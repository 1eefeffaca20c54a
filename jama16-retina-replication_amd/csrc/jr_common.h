// jr_common.h — shared helpers for the libjr.so HIP sources (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
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
unsigned* device_error_word();
// Stream-K owner poll bound (jr_debug_set_sk_spin_limit; default 2^22).
unsigned sk_spin_limit();

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
