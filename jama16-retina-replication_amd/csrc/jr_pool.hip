// jr_pool.hip — Inception-v3 pooling ops, forward and backward, NHWC with
// channel slices so pool outputs land directly in their concat buffer.
//
//  - MaxPooling2D((3,3), strides=(2,2)) 'valid' (stem x2, mixed3, mixed8 of
//    the Keras InceptionV3 built at train.py:129-130).
//    fwd writes the window argmax (first max in scan order, uint8) so bwd is
//    a deterministic gather: every input element sums the dy of the (at most
//    2x2) windows whose argmax it is.
//  - AveragePooling2D((3,3), strides=(1,1), padding='same') (mixed0-2, 4-7,
//    9-10; a7): TF divides by the number of in-bounds taps (exclude padding).
//  - GlobalAveragePooling2D (pooling='avg', train.py:130; a9).
// All kernels move fp32x4 (or bf16x4) vectors along the channel axis.
#include "jr_common.h"

namespace jr {

template <typename T> struct P4;
template <> struct P4<float> {
  __device__ static float4 ld(const float* p) { return *reinterpret_cast<const float4*>(p); }
  __device__ static void st(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
};
template <> struct P4<uint16_t> {
  __device__ static float4 ld(const uint16_t* p) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
  }
  __device__ static void st(uint16_t* p, float4 v) {
    uint2 u;
    u.x = (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
    u.y = (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16);
    *reinterpret_cast<uint2*>(p) = u;
  }
};

__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

template <typename T>
__global__ void __launch_bounds__(256) k_maxpool_fwd(jr_pool_desc d, const T* __restrict__ x, T* y,
                                                     uint8_t* argmax) {
  const int c4 = d.c >> 2;
  const int total = d.n * d.ho * d.wo * c4;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int q = e % c4;
    const int pix = e / c4;
    const int ow = pix % d.wo;
    const int t = pix / d.wo;
    const int oh = t % d.ho;
    const int b = t / d.ho;
    float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int arg[4] = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int ih = oh * 2 + r, iw = ow * 2 + c;
        const float4 v = P4<T>::ld(x + ((int64_t)(b * d.h + ih) * d.w + iw) * d.x_c_stride + d.x_c_off + q * 4);
        const float va[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (va[j] > best[j] || (r == 0 && c == 0)) { best[j] = va[j]; arg[j] = r * 3 + c; }
      }
    }
    P4<T>::st(y + (int64_t)pix * d.y_c_stride + d.y_c_off + q * 4, make_float4(best[0], best[1], best[2], best[3]));
    if (argmax) {
      const uint32_t packed = (uint32_t)arg[0] | ((uint32_t)arg[1] << 8) | ((uint32_t)arg[2] << 16) |
                              ((uint32_t)arg[3] << 24);
      *reinterpret_cast<uint32_t*>(argmax + (int64_t)pix * d.c + q * 4) = packed;
    }
  }
}

// BN + ReLU + max-pool in one pass (the stem's conv2d_3 / conv2d_5 outputs,
// whose only reader is the max-pool): every window tap is the raw conv output
// put through bn_pre and ReLU -- and rounded to the path dtype, exactly as
// k_bn_relu_apply stores it -- before the comparison, so y and argmax are
// bitwise the two-kernel result, without writing and re-reading the
// full-resolution activation (354 / 248 MB per fp32 step).  Grouped
// (ensemble members): image b belongs to member b / ipm, whose statistics
// and beta sit st_mb / be_mb floats further (0 for one member).
template <typename T>
__global__ void __launch_bounds__(256) k_bn_relu_maxpool_fwd(jr_pool_desc d, const T* __restrict__ x,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd,
                                                             const float* __restrict__ beta, T* y, uint8_t* argmax,
                                                             int ipm, long long st_mb, long long be_mb) {
  const int c4 = d.c >> 2;
  const int total = d.n * d.ho * d.wo * c4;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int q = e % c4;
    const int pix = e / c4;
    const int ow = pix % d.wo;
    const int t = pix / d.wo;
    const int oh = t % d.ho;
    const int b = t / d.ho;
    const long long mem = b / ipm;
    float mu[4], is[4], be[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mu[j] = mean[mem * st_mb + q * 4 + j];
      is[j] = invstd[mem * st_mb + q * 4 + j];
      be[j] = beta[mem * be_mb + q * 4 + j];
    }
    float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int arg[4] = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int ih = oh * 2 + r, iw = ow * 2 + c;
        const float4 v = P4<T>::ld(x + ((int64_t)(b * d.h + ih) * d.w + iw) * d.x_c_stride + d.x_c_off + q * 4);
        const float va[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float a = fmaxf(bn_pre(va[j], mu[j], is[j], be[j]), 0.f);
          if constexpr (sizeof(T) == 2) a = bf2f(f2bf(a));
          if (a > best[j] || (r == 0 && c == 0)) { best[j] = a; arg[j] = r * 3 + c; }
        }
      }
    }
    P4<T>::st(y + (int64_t)pix * d.y_c_stride + d.y_c_off + q * 4, make_float4(best[0], best[1], best[2], best[3]));
    if (argmax) {
      const uint32_t packed = (uint32_t)arg[0] | ((uint32_t)arg[1] << 8) | ((uint32_t)arg[2] << 16) |
                              ((uint32_t)arg[3] << 24);
      *reinterpret_cast<uint32_t*>(argmax + (int64_t)pix * d.c + q * 4) = packed;
    }
  }
}

// Backward as a gather over 2x2 input cells: input rows 2a, 2a+1 and columns
// 2b, 2b+1 are covered only by the windows oh in {a-1, a}, ow in {b-1, b}, so
// one thread loads those (at most) four windows' dy and argmax once and writes
// the four input pixels of its cell -- one dy/argmax load per output pixel
// instead of the 2.25 of a thread per input pixel.  Each input pixel still sums
// its windows in (oh, ow) ascending order.
template <typename T>
__global__ void __launch_bounds__(256) k_maxpool_bwd(jr_pool_desc d, const uint8_t* __restrict__ argmax,
                                                     const T* __restrict__ dy, T* __restrict__ dx, int accumulate) {
  const int c4 = d.c >> 2;
  const int hc = (d.h + 1) >> 1, wc = (d.w + 1) >> 1;
  const int total = d.n * hc * wc * c4;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int q = e % c4;
    const int cell = e / c4;
    const int cb = cell % wc;
    const int t = cell / wc;
    const int ca = t % hc;
    const int b = t / hc;
    uint32_t am[2][2];
    float4 g[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int oh = ca - 1 + i, ow = cb - 1 + j;
        am[i][j] = 0xffffffffu;                  // position 255: matches no tap
        g[i][j] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (oh >= 0 && oh < d.ho && ow >= 0 && ow < d.wo) {
          const int64_t op = ((int64_t)b * d.ho + oh) * d.wo + ow;
          am[i][j] = *reinterpret_cast<const uint32_t*>(argmax + op * d.c + q * 4);
          g[i][j] = P4<T>::ld(dy + op * d.y_c_stride + d.y_c_off + q * 4);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const int ih = 2 * ca + u, iw = 2 * cb + v;
        if (ih >= d.h || iw >= d.w) continue;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int r = u + 2 - 2 * i, c = v + 2 - 2 * j;   // tap of (ih, iw) in window (ca-1+i, cb-1+j)
            if (r > 2 || c > 2) continue;                      // compile-time after unrolling
            const float ga[4] = {g[i][j].x, g[i][j].y, g[i][j].z, g[i][j].w};
#pragma unroll
            for (int l = 0; l < 4; ++l)
              if ((int)((am[i][j] >> (8 * l)) & 0xff) == r * 3 + c) acc[l] += ga[l];
          }
        }
        T* p = dx + ((int64_t)(b * d.h + ih) * d.w + iw) * d.x_c_stride + d.x_c_off + q * 4;
        float4 o = make_float4(acc[0], acc[1], acc[2], acc[3]);
        if (accumulate) o = f4add(o, P4<T>::ld(p));
        P4<T>::st(p, o);
      }
    }
  }
}

// Avg-pool as a sliding 3x3 box: one thread per (b, strip of kStrip rows,
// column, channel quad) keeps the three row sums around its output row in
// registers, so each input vector is loaded 3 (kStrip + 2) / kStrip times
// instead of 9 times (a thread per output was L2-bound; this is +1.2 % per
// training step).  The backward is the same box over z = dy / count
// (count = ch(oh) * cw(ow), the in-bounds taps of the output window).
#ifndef JR_POOL_STRIP
#define JR_POOL_STRIP 8
#endif
constexpr int kStrip = JR_POOL_STRIP;

// x / d for a tap count d = ch * cw in {1, 2, 3, 4, 6, 9}, bitwise the IEEE
// division without its ~10-instruction sequence: q = x * RN(1/d) and one
// fma correction, guarded for q = +-0 / +-inf / NaN (selects) and for
// |x| < 2^-100 (x / 6 subnormal: one-ulp misses there: the true division
// runs, behind a branch no lane takes on real data).
// Exhaustively verified over all 2^32 inputs per d (tools/verify_pool_div.c).
// The backward divides every dy element 3 (kStrip + 2) / kStrip times.
__device__ __forceinline__ float tap_recip(float d) {
  return d == 9.f ? 0x1.c71c72p-4f : d == 6.f ? 0x1.555556p-3f : d == 4.f ? 0.25f
       : d == 3.f ? 0x1.555556p-2f : d == 2.f ? 0.5f : 1.f;
}
__device__ __forceinline__ float pool_div(float x, float d, float r) {
  const float q = __fmul_rn(x, r);
  if (__builtin_expect(fabsf(x) < 0x1p-100f, 0)) return x / d;
  const float c = __builtin_fmaf(__builtin_fmaf(-q, d, x), r, q);
  return (q == 0.f || !__builtin_isfinite(q)) ? q : c;
}
__device__ __forceinline__ float4 pool_div4(float4 v, float d) {
#ifdef JR_POOL_TRUE_DIV   // A/B: the IEEE division sequence
  return make_float4(v.x / d, v.y / d, v.z / d, v.w / d);
#endif
  // (one guard branch per vector instead of per element measured slower:
  // bf16 backward 277 vs 265 us per step)
  const float r = tap_recip(d);
  return make_float4(pool_div(v.x, d, r), pool_div(v.y, d, r), pool_div(v.z, d, r), pool_div(v.w, d, r));
}

template <typename T, bool BWD>
__device__ __forceinline__ float4 box_row(const jr_pool_desc& d, const T* __restrict__ src, int b, int h, int w,
                                          int q) {
  // sum of the (up to) three in-bounds horizontal taps of row h around w
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  const int stride = BWD ? d.y_c_stride : d.x_c_stride;
  const int off = BWD ? d.y_c_off : d.x_c_off;
  const int ch = 1 + (h > 0) + (h < d.h - 1);
#pragma unroll
  for (int c = -1; c <= 1; ++c) {
    const int iw = w + c;
    if ((unsigned)iw >= (unsigned)d.w) continue;
    float4 v = P4<T>::ld(src + ((int64_t)(b * d.h + h) * d.w + iw) * stride + off + q * 4);
    if (BWD) {
      const float fc = (float)(ch * (1 + (iw > 0) + (iw < d.w - 1)));
      v = pool_div4(v, fc);
    }
    s = f4add(s, v);
  }
  return s;
}

template <typename T, bool BWD>
__global__ void __launch_bounds__(256) k_avgpool_box(jr_pool_desc d, const T* __restrict__ src, T* dst,
                                                     int accumulate) {
  const int c4 = d.c >> 2;
  const int nstrip = (d.h + kStrip - 1) / kStrip;
  const int total = d.n * nstrip * d.w * c4;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int q = e % c4;
    const int r1 = e / c4;
    const int w = r1 % d.w;
    const int r2 = r1 / d.w;
    const int st = r2 % nstrip;
    const int b = r2 / nstrip;
    const int h0 = st * kStrip, h1 = min(d.h, h0 + kStrip);
    const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 up = h0 > 0 ? box_row<T, BWD>(d, src, b, h0 - 1, w, q) : zero;
    float4 mid = box_row<T, BWD>(d, src, b, h0, w, q);
    for (int h = h0; h < h1; ++h) {
      const float4 dn = h + 1 < d.h ? box_row<T, BWD>(d, src, b, h + 1, w, q) : zero;
      float4 o = f4add(f4add(up, mid), dn);
      if (!BWD) {
        const float fc = (float)((1 + (h > 0) + (h < d.h - 1)) * (1 + (w > 0) + (w < d.w - 1)));
        o = pool_div4(o, fc);
      }
      const int ostride = BWD ? d.x_c_stride : d.y_c_stride;
      const int ooff = BWD ? d.x_c_off : d.y_c_off;
      T* p = dst + ((int64_t)(b * d.h + h) * d.w + w) * ostride + ooff + q * 4;
      if (BWD && accumulate) o = f4add(o, P4<T>::ld(p));
      P4<T>::st(p, o);
      up = mid;
      mid = dn;
    }
  }
}

// GAP: one thread per (b, channel quad), loop over hw in order.
template <typename T>
__global__ void k_gap_fwd(const T* __restrict__ x, int n, int hw, int c, float* y) {
  const int c4 = c >> 2;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * c4) return;
  const int b = e / c4, q = e - b * c4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int p = 0; p < hw; ++p) s = f4add(s, P4<T>::ld(x + ((int64_t)b * hw + p) * c + q * 4));
  const float f = (float)hw;
  *reinterpret_cast<float4*>(y + (int64_t)b * c + q * 4) = make_float4(s.x / f, s.y / f, s.z / f, s.w / f);
}

template <typename T>
__global__ void k_gap_bwd(const float* __restrict__ dy, int n, int hw, int c, T* dx) {
  const int c4 = c >> 2;
  const int total = n * hw * c4;
  const float f = (float)hw;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int q = e % c4;
    const int pix = e / c4;
    const int b = pix / hw;
    const float4 g = *reinterpret_cast<const float4*>(dy + (int64_t)b * c + q * 4);
    P4<T>::st(dx + (int64_t)pix * c + q * 4, make_float4(g.x / f, g.y / f, g.z / f, g.w / f));
  }
}

static int grid_for(int64_t items) {
  const int64_t b = ceil_div(items, 256);
  return (int)std::min<int64_t>(std::max<int64_t>(b, 1), 256 * 16);
}

static int check_pool(const jr_pool_desc* d, int dtype, bool maxpool) {
  if (!d) return fail(JR_ERR_INVALID, "pool: null descriptor");
  if (dtype != JR_F32 && dtype != JR_BF16) return fail(JR_ERR_INVALID, "pool: bad dtype");
  if (d->n <= 0 || d->h <= 0 || d->w <= 0 || d->c <= 0) return fail(JR_ERR_INVALID, "pool: empty tensor");
  if (d->c % 4 || d->x_c_off % 4 || d->x_c_stride % 4 || d->y_c_off % 4 || d->y_c_stride % 4)
    return fail(JR_ERR_INVALID, "pool: channels, offsets and strides must be multiples of 4");
  if (d->x_c_off < 0 || d->x_c_off + d->c > d->x_c_stride || d->y_c_off < 0 || d->y_c_off + d->c > d->y_c_stride)
    return fail(JR_ERR_INVALID, "pool: channel slice out of range");
  // element indices (pixel x channel quad) are 32-bit in the kernels: the
  // 64-bit divisions they replaced dominated the avgpool backward
  if ((int64_t)d->n * d->h * d->w * (d->c / 4) >= (1LL << 30))
    return fail(JR_ERR_UNSUPPORTED, "pool: more than 2^30 channel quads");
  if (maxpool) {
    if (d->h < 3 || d->w < 3 || d->ho != (d->h - 3) / 2 + 1 || d->wo != (d->w - 3) / 2 + 1)
      return fail(JR_ERR_INVALID, "maxpool: ho/wo must be (h-3)/2+1 (3x3 stride 2 valid)");
  } else {
    if (d->ho != d->h || d->wo != d->w) return fail(JR_ERR_INVALID, "avgpool: 'same' stride 1 needs ho=h, wo=w");
  }
  return JR_OK;
}

}  // namespace jr

using namespace jr;

JR_API int jr_maxpool3x3s2_fwd(const jr_pool_desc* d, int dtype, const void* x, void* y, uint8_t* argmax,
                               void* stream) {
  int rc = check_pool(d, dtype, true);
  if (rc) return rc;
  if (!x || !y) return fail(JR_ERR_INVALID, "maxpool_fwd: null pointer");
  const int g = grid_for((int64_t)d->n * d->ho * d->wo * (d->c / 4));
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_maxpool_fwd<float>, dim3(g), dim3(256), 0, as_stream(stream), *d, (const float*)x,
                       (float*)y, argmax);
  else
    hipLaunchKernelGGL(k_maxpool_fwd<uint16_t>, dim3(g), dim3(256), 0, as_stream(stream), *d,
                       (const uint16_t*)x, (uint16_t*)y, argmax);
  return check_launch("maxpool_fwd");
}

JR_API int jr_bn_relu_maxpool3x3s2_fwd_grouped(const jr_pool_desc* d, int dtype, int32_t images_per_member,
                                               const void* raw, const float* mean, const float* invstd,
                                               int64_t stats_member_stride, const float* beta,
                                               int64_t beta_member_stride, void* y, uint8_t* argmax, void* stream) {
  int rc = check_pool(d, dtype, true);
  if (rc) return rc;
  if (!raw || !mean || !invstd || !beta || !y) return fail(JR_ERR_INVALID, "bn_relu_maxpool_fwd: null pointer");
  if (images_per_member < 1 || d->n % images_per_member != 0 || stats_member_stride < 0 || beta_member_stride < 0)
    return fail(JR_ERR_INVALID, "bn_relu_maxpool_fwd: images_per_member must divide n; strides >= 0");
  const int g = grid_for((int64_t)d->n * d->ho * d->wo * (d->c / 4));
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_bn_relu_maxpool_fwd<float>, dim3(g), dim3(256), 0, as_stream(stream), *d,
                       (const float*)raw, mean, invstd, beta, (float*)y, argmax, images_per_member,
                       (long long)stats_member_stride, (long long)beta_member_stride);
  else
    hipLaunchKernelGGL(k_bn_relu_maxpool_fwd<uint16_t>, dim3(g), dim3(256), 0, as_stream(stream), *d,
                       (const uint16_t*)raw, mean, invstd, beta, (uint16_t*)y, argmax, images_per_member,
                       (long long)stats_member_stride, (long long)beta_member_stride);
  return check_launch("bn_relu_maxpool_fwd");
}

JR_API int jr_bn_relu_maxpool3x3s2_fwd(const jr_pool_desc* d, int dtype, const void* raw, const float* mean,
                                       const float* invstd, const float* beta, void* y, uint8_t* argmax,
                                       void* stream) {
  if (!d) return fail(JR_ERR_INVALID, "pool: null descriptor");
  return jr_bn_relu_maxpool3x3s2_fwd_grouped(d, dtype, d->n > 0 ? d->n : 1, raw, mean, invstd, 0, beta, 0, y,
                                             argmax, stream);
}

JR_API int jr_maxpool3x3s2_bwd(const jr_pool_desc* d, int dtype, const uint8_t* argmax, const void* dy,
                               void* dx, int accumulate, void* stream) {
  int rc = check_pool(d, dtype, true);
  if (rc) return rc;
  if (!argmax || !dy || !dx) return fail(JR_ERR_INVALID, "maxpool_bwd: null pointer");
  const int g = grid_for((int64_t)d->n * ((d->h + 1) / 2) * ((d->w + 1) / 2) * (d->c / 4));
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_maxpool_bwd<float>, dim3(g), dim3(256), 0, as_stream(stream), *d, argmax,
                       (const float*)dy, (float*)dx, accumulate);
  else
    hipLaunchKernelGGL(k_maxpool_bwd<uint16_t>, dim3(g), dim3(256), 0, as_stream(stream), *d, argmax,
                       (const uint16_t*)dy, (uint16_t*)dx, accumulate);
  return check_launch("maxpool_bwd");
}

JR_API int jr_avgpool3x3s1_fwd(const jr_pool_desc* d, int dtype, const void* x, void* y, void* stream) {
  int rc = check_pool(d, dtype, false);
  if (rc) return rc;
  if (!x || !y) return fail(JR_ERR_INVALID, "avgpool_fwd: null pointer");
  const int g = grid_for((int64_t)d->n * ceil_div(d->h, kStrip) * d->w * (d->c / 4));
  if (dtype == JR_F32)
    hipLaunchKernelGGL((k_avgpool_box<float, false>), dim3(g), dim3(256), 0, as_stream(stream), *d, (const float*)x,
                       (float*)y, 0);
  else
    hipLaunchKernelGGL((k_avgpool_box<uint16_t, false>), dim3(g), dim3(256), 0, as_stream(stream), *d,
                       (const uint16_t*)x, (uint16_t*)y, 0);
  return check_launch("avgpool_fwd");
}

JR_API int jr_avgpool3x3s1_bwd(const jr_pool_desc* d, int dtype, const void* dy, void* dx, int accumulate,
                               void* stream) {
  int rc = check_pool(d, dtype, false);
  if (rc) return rc;
  if (!dy || !dx) return fail(JR_ERR_INVALID, "avgpool_bwd: null pointer");
  const int g = grid_for((int64_t)d->n * ceil_div(d->h, kStrip) * d->w * (d->c / 4));
  if (dtype == JR_F32)
    hipLaunchKernelGGL((k_avgpool_box<float, true>), dim3(g), dim3(256), 0, as_stream(stream), *d, (const float*)dy,
                       (float*)dx, accumulate);
  else
    hipLaunchKernelGGL((k_avgpool_box<uint16_t, true>), dim3(g), dim3(256), 0, as_stream(stream), *d,
                       (const uint16_t*)dy, (uint16_t*)dx, accumulate);
  return check_launch("avgpool_bwd");
}

JR_API int jr_gap_fwd(int dtype, const void* x, int32_t n, int32_t hw, int32_t c, float* y, void* stream) {
  if (!x || !y || n <= 0 || hw <= 0 || c <= 0 || c % 4) return fail(JR_ERR_INVALID, "gap_fwd: bad arguments");
  const int g = (int)ceil_div((int64_t)n * (c / 4), 256);
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_gap_fwd<float>, dim3(g), dim3(256), 0, as_stream(stream), (const float*)x, n, hw, c, y);
  else if (dtype == JR_BF16)
    hipLaunchKernelGGL(k_gap_fwd<uint16_t>, dim3(g), dim3(256), 0, as_stream(stream), (const uint16_t*)x, n, hw,
                       c, y);
  else
    return fail(JR_ERR_INVALID, "gap_fwd: bad dtype");
  return check_launch("gap_fwd");
}

JR_API int jr_gap_bwd(int dtype, const float* dy, int32_t n, int32_t hw, int32_t c, void* dx, void* stream) {
  if (!dy || !dx || n <= 0 || hw <= 0 || c <= 0 || c % 4) return fail(JR_ERR_INVALID, "gap_bwd: bad arguments");
  if ((int64_t)n * hw * (c / 4) >= (1LL << 30)) return fail(JR_ERR_UNSUPPORTED, "gap_bwd: more than 2^30 channel quads");
  const int g = grid_for((int64_t)n * hw * (c / 4));
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_gap_bwd<float>, dim3(g), dim3(256), 0, as_stream(stream), dy, n, hw, c, (float*)dx);
  else if (dtype == JR_BF16)
    hipLaunchKernelGGL(k_gap_bwd<uint16_t>, dim3(g), dim3(256), 0, as_stream(stream), dy, n, hw, c,
                       (uint16_t*)dx);
  else
    return fail(JR_ERR_INVALID, "gap_bwd: bad dtype");
  return check_launch("gap_bwd");
}
