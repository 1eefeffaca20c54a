// jr_misc.hip — optimizers, dtype casts, input scaling, Brier accumulator.
//
// Optimizers replace the TF ApplyMomentum / ApplyGradientDescent ops that
// .minimize adds at train.py:147-153.  One launch updates
// the whole flat parameter buffer (21,770,401 fp32 values); each lane moves
// 16-byte vectors and the arithmetic is the unfused TF expression order.
// NOTE: hipcc contracts a*b+c into an FMA by default (-ffp-contract=fast),
// and without OCML_BASIC_ROUNDED_OPERATIONS __fmul_rn / __fadd_rn are the
// plain operators, so this file is compiled with -ffp-contract=off
// (Makefile): every multiply and add rounds on its own,
// the IEEE fp32 evaluation of TF's (Eigen, non-fused) expressions:
//   ApplyMomentum(use_nesterov): accum = accum*m + g; var -= g*lr + accum*m*lr
//   ApplyMomentum:               accum = accum*m + g; var -= accum*lr
//   ApplyGradientDescent:        var -= g*lr
#include "jr_common.h"

namespace jr {

static int grid_for(int64_t items) {
  const int64_t b = ceil_div(items, 256);
  return (int)std::min<int64_t>(std::max<int64_t>(b, 1), 256 * 32);
}

__device__ __forceinline__ float nest1(float& w, float g, float& a, float lr, float m) {
  a = __fadd_rn(__fmul_rn(a, m), g);
  w = __fsub_rn(w, __fadd_rn(__fmul_rn(g, lr), __fmul_rn(__fmul_rn(a, m), lr)));
  return w;
}

__global__ void __launch_bounds__(256) k_nesterov(float* __restrict__ w, const float* __restrict__ grad,
                                                  float* __restrict__ accum, int64_t n, float lr, float m,
                                                  float gs) {
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 wv = reinterpret_cast<float4*>(w)[i];
    float4 av = reinterpret_cast<float4*>(accum)[i];
    const float4 gv = reinterpret_cast<const float4*>(grad)[i];
    nest1(wv.x, __fmul_rn(gv.x, gs), av.x, lr, m);
    nest1(wv.y, __fmul_rn(gv.y, gs), av.y, lr, m);
    nest1(wv.z, __fmul_rn(gv.z, gs), av.z, lr, m);
    nest1(wv.w, __fmul_rn(gv.w, gs), av.w, lr, m);
    reinterpret_cast<float4*>(w)[i] = wv;
    reinterpret_cast<float4*>(accum)[i] = av;
  }
  // tail
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < (n & 3)) {
    const int64_t i = n4 * 4 + t;
    nest1(w[i], __fmul_rn(grad[i], gs), accum[i], lr, m);
  }
}

__global__ void __launch_bounds__(256) k_momentum(float* __restrict__ w, const float* __restrict__ grad,
                                                  float* __restrict__ accum, int64_t n, float lr, float m,
                                                  float gs) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float g = __fmul_rn(grad[i], gs);
    const float a = __fadd_rn(__fmul_rn(accum[i], m), g);
    accum[i] = a;
    w[i] = __fsub_rn(w[i], __fmul_rn(a, lr));
  }
}

__global__ void __launch_bounds__(256) k_sgd(float* __restrict__ w, const float* __restrict__ grad, int64_t n,
                                             float lr, float gs) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    w[i] = __fsub_rn(w[i], __fmul_rn(__fmul_rn(grad[i], gs), lr));
}

// Correctly rounded sqrt (IEEE, as Eigen's sqrt on the CPU): v_sqrt_f32 is
// within 1 ulp, so check its neighbours with exact fma residuals and step
// once (denormal inputs are scaled by 2^32 first).
__device__ __forceinline__ float sqrt_cr(float x) {
  const bool tiny = x < 0x1.0p-96f;
  const float xs = tiny ? x * 0x1.0p+32f : x;
  float s = __builtin_amdgcn_sqrtf(xs);
  const float dn = __uint_as_float(__float_as_uint(s) - 1), up = __uint_as_float(__float_as_uint(s) + 1);
  if (__builtin_fmaf(-dn, s, xs) <= 0.f) s = dn;
  else if (__builtin_fmaf(-up, s, xs) > 0.f) s = up;
  s = tiny ? s * 0x1.0p-16f : s;
  return (xs == 0.f || !(xs < __builtin_inff())) ? __builtin_sqrtf(x) : s;
}

// TF ApplyAdam (training_ops.cc ApplyAdamNonCuda, Eigen, no contraction):
//   m += (g - m) * (1 - beta1);  v += (g*g - v) * (1 - beta2);
//   var -= (m * alpha) / (sqrt(v) + epsilon),
//   alpha = lr * sqrt(1 - beta2^t) / (1 - beta1^t) (lr_t, computed on the host);
// every operation a correctly rounded _rn intrinsic in that order, so the
// update is bitwise the IEEE fp32 evaluation of TF's expression.
__global__ void __launch_bounds__(256) k_adam(float* __restrict__ w, const float* __restrict__ grad,
                                              float* __restrict__ mm, float* __restrict__ vv, int64_t n,
                                              float lr_t, float b1, float b2, float eps, float gs) {
  const float one_b1 = __fsub_rn(1.f, b1), one_b2 = __fsub_rn(1.f, b2);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float g = __fmul_rn(grad[i], gs);
    const float m0 = mm[i], v0 = vv[i];
    const float m1 = __fadd_rn(m0, __fmul_rn(__fsub_rn(g, m0), one_b1));
    const float v1 = __fadd_rn(v0, __fmul_rn(__fsub_rn(__fmul_rn(g, g), v0), one_b2));
    mm[i] = m1;
    vv[i] = v1;
    w[i] = __fsub_rn(w[i], __fdiv_rn(__fmul_rn(m1, lr_t), __fadd_rn(sqrt_cr(v1), eps)));
  }
}

__global__ void k_f32_to_bf16(const float* __restrict__ s, uint16_t* d, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    d[i] = f2bf(s[i]);
}

__global__ void k_bf16_to_f32(const uint16_t* __restrict__ s, float* d, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    d[i] = bf2f(s[i]);
}

// tf.image.convert_image_dtype(uint8 -> float32): f32(x) * f32(1/255)
template <typename T>
__global__ void k_u8_scale(const uint8_t* __restrict__ s, T* d, int64_t n) {
  const float scale = 1.0f / 255.0f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    Elt<T>::st(d + i, __fmul_rn((float)s[i], scale));
}

template <typename T>
__global__ void k_image_u8(const uint8_t* __restrict__ s, T* d, int64_t pixels, int c, int ds) {
  const float scale = 1.0f / 255.0f;
  const int64_t total = pixels * ds;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / ds;
    const int ch = (int)(i - p * ds);
    Elt<T>::st(d + i, ch < c ? __fmul_rn((float)s[p * c + ch], scale) : 0.f);
  }
}

__global__ void k_brier(const float* __restrict__ p, const float* __restrict__ y, int n, double* acc) {
  __shared__ double red[256];
  const int t = threadIdx.x;
  double s = 0.0;
  for (int i = t; i < n; i += 256) {
    const double d = (double)p[i] - (double)y[i];
    s += d * d;
  }
  red[t] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  if (t == 0) {
    acc[0] += red[0];
    acc[1] += (double)n;
  }
}

}  // namespace jr

using namespace jr;

JR_API int jr_nesterov_update(float* w, const float* grad, float* accum, int64_t n, float lr, float momentum,
                              float grad_scale, void* stream) {
  if (!w || !grad || !accum || n < 0) return fail(JR_ERR_INVALID, "nesterov: bad arguments");
  if (((uintptr_t)w | (uintptr_t)grad | (uintptr_t)accum) & 15)
    return fail(JR_ERR_INVALID, "nesterov: buffers must be 16-byte aligned");
  if (n == 0) return JR_OK;
  hipLaunchKernelGGL(k_nesterov, dim3(grid_for(std::max<int64_t>(n / 4, 4))), dim3(256), 0, as_stream(stream), w,
                     grad, accum, n, lr, momentum, grad_scale);
  return check_launch("nesterov");
}

JR_API int jr_momentum_update(float* w, const float* grad, float* accum, int64_t n, float lr, float momentum,
                              float grad_scale, void* stream) {
  if (!w || !grad || !accum || n < 0) return fail(JR_ERR_INVALID, "momentum: bad arguments");
  if (n == 0) return JR_OK;
  hipLaunchKernelGGL(k_momentum, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), w, grad, accum, n, lr,
                     momentum, grad_scale);
  return check_launch("momentum");
}

JR_API int jr_sgd_update(float* w, const float* grad, int64_t n, float lr, float grad_scale, void* stream) {
  if (!w || !grad || n < 0) return fail(JR_ERR_INVALID, "sgd: bad arguments");
  if (n == 0) return JR_OK;
  hipLaunchKernelGGL(k_sgd, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), w, grad, n, lr, grad_scale);
  return check_launch("sgd");
}

JR_API int jr_adam_update(float* w, const float* grad, float* m, float* v, int64_t n, float lr_t, float beta1,
                          float beta2, float eps, float grad_scale, void* stream) {
  if (!w || !grad || !m || !v || n < 0) return fail(JR_ERR_INVALID, "adam: bad arguments");
  if (n == 0) return JR_OK;
  hipLaunchKernelGGL(k_adam, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), w, grad, m, v, n, lr_t, beta1,
                     beta2, eps, grad_scale);
  return check_launch("adam");
}

// ---------------------------------------------------------------- bf16 filters
// One block = one 32 (c_in) x 32 (c_out) tile of one tap of one layer:
// coalesced read along c_out, bf16 HWIO write along c_out, transpose through
// LDS, bf16 W^T write along c_in (zero channels up to c8).
static __device__ __forceinline__ int wprep_tiles(int kh, int kw, int cin, int cout) {
  return kh * kw * ((((cin + 7) / 8 * 8) + 31) / 32) * ((cout + 31) / 32);
}

// Exact three-way split x = h + m + l into bf16 (JR_F32_X8P operands): the
// terms of SplitFrag in jr_conv.hip, bit for bit (RNE casts; the remainders
// are exact in fp32 and l is exact in bf16).
__device__ __forceinline__ void split3(float x, uint16_t& h, uint16_t& m, uint16_t& l) {
  h = f2bf(x);
  const float r = __fsub_rn(x, bf2f(h));
  m = f2bf(r);
  l = f2bf(__fsub_rn(r, bf2f(m)));
}

// NP = 1: bf16 copies (JR_BF16); NP = 3: h / m / l planes, plane stride =
// the layer's element count (JR_F32_X8P).
template <bool SINGLE, int NP>
__global__ void __launch_bounds__(256) k_wprep(const jr_wprep* __restrict__ table, jr_wprep one, int nl,
                                               const float* __restrict__ src, uint16_t* hwio, uint16_t* wt) {
  __shared__ float t[32][33];
  const int tile = blockIdx.x;
  jr_wprep L;
  if constexpr (SINGLE) {
    L = one;
  } else {   // last layer whose tile_start <= tile
    int lo = 0, hi = nl - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (table[mid].tile_start <= tile) lo = mid; else hi = mid - 1;
    }
    L = table[lo];
  }
  const int c8 = (L.c_in + 7) / 8 * 8;
  const int cit = (c8 + 31) / 32, cot = (L.c_out + 31) / 32;
  const int local = tile - (SINGLE ? 0 : L.tile_start);
  const int tap = local / (cit * cot), rem = local - tap * (cit * cot);
  const int ci0 = (rem / cot) * 32, co0 = (rem % cot) * 32;
  const float* s = src + L.src_off;
  const int64_t hps = (int64_t)L.kh * L.kw * L.c_in * L.c_out;
  const int64_t K = (int64_t)L.kh * L.kw * c8;
  const int64_t tps = (int64_t)L.c_out * K;
  for (int e = threadIdx.x; e < 1024; e += 256) {
    const int ci = ci0 + (e >> 5), co = co0 + (e & 31);
    float v = 0.f;
    if (ci < L.c_in && co < L.c_out) {
      const int64_t idx = ((int64_t)tap * L.c_in + ci) * L.c_out + co;
      v = s[idx];
      if (hwio) {
        if constexpr (NP == 1) {
          hwio[L.hwio_off + idx] = f2bf(v);
        } else {
          uint16_t h, m, l;
          split3(v, h, m, l);
          hwio[L.hwio_off + idx] = h;
          hwio[L.hwio_off + hps + idx] = m;
          hwio[L.hwio_off + 2 * hps + idx] = l;
        }
      }
    }
    t[e >> 5][e & 31] = v;
  }
  __syncthreads();
  if (!wt) return;
  for (int e = threadIdx.x; e < 1024; e += 256) {
    const int co = co0 + (e >> 5), ci = ci0 + (e & 31);
    if (co < L.c_out && ci < c8) {
      const int64_t o = L.wt_off + co * K + (int64_t)tap * c8 + ci;
      const float v = t[e & 31][e >> 5];
      if constexpr (NP == 1) {
        wt[o] = f2bf(v);
      } else {
        uint16_t h, m, l;
        split3(v, h, m, l);
        wt[o] = h;
        wt[o + tps] = m;
        wt[o + 2 * tps] = l;
      }
    }
  }
}

// Activation / gradient split: one thread per 4 channels of one row (c and
// the offsets multiples of 4: float4 in, three 8-byte plane stores out),
// else one per channel.  Channels [c, c_pad) of the destination get zeros.
template <bool VEC>
__global__ void __launch_bounds__(256) k_split_x8p(const float* __restrict__ src, int64_t rows, int c, int src_off,
                                                   int src_stride, uint16_t* __restrict__ dst, int c_pad, int dst_off,
                                                   int dst_stride, int64_t ps) {
  constexpr int V = VEC ? 4 : 1;
  const int per_row = (c_pad + V - 1) / V;
  const int64_t total = rows * per_row;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / per_row;
    const int ch = (int)(i - r * per_row) * V;
    uint16_t* d = dst + r * dst_stride + dst_off + ch;
    if constexpr (VEC) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ch < c) v = *reinterpret_cast<const float4*>(src + r * src_stride + src_off + ch);
      const float x[4] = {v.x, v.y, v.z, v.w};
      uint16_t h[4], m[4], l[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) split3(x[k], h[k], m[k], l[k]);
      *reinterpret_cast<uint2*>(d) = make_uint2(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16));
      *reinterpret_cast<uint2*>(d + ps) = make_uint2(m[0] | ((uint32_t)m[1] << 16), m[2] | ((uint32_t)m[3] << 16));
      *reinterpret_cast<uint2*>(d + 2 * ps) = make_uint2(l[0] | ((uint32_t)l[1] << 16), l[2] | ((uint32_t)l[3] << 16));
    } else {
      const float x = ch < c ? src[r * src_stride + src_off + ch] : 0.f;
      uint16_t h, m, l;
      split3(x, h, m, l);
      d[0] = h;
      d[ps] = m;
      d[2 * ps] = l;
    }
  }
}

JR_API int32_t jr_conv_weights_bf16_tiles(int32_t kh, int32_t kw, int32_t c_in, int32_t c_out) {
  if (kh <= 0 || kw <= 0 || c_in <= 0 || c_out <= 0) return 0;
  return kh * kw * ((((c_in + 7) / 8 * 8) + 31) / 32) * ((c_out + 31) / 32);
}

JR_API int jr_conv_weights_bf16(const float* w, int32_t kh, int32_t kw, int32_t c_in, int32_t c_out, void* w_hwio,
                                void* w_t, void* stream) {
  const int tiles = jr_conv_weights_bf16_tiles(kh, kw, c_in, c_out);
  if (!w || tiles <= 0) return fail(JR_ERR_INVALID, "conv_weights_bf16: bad arguments");
  jr_wprep one{0, 0, 0, kh, kw, c_in, c_out, 0, 0};
  hipLaunchKernelGGL((k_wprep<true, 1>), dim3(tiles), dim3(256), 0, as_stream(stream), (const jr_wprep*)nullptr, one,
                     1, w, (uint16_t*)w_hwio, (uint16_t*)w_t);
  return check_launch("conv_weights_bf16");
}

JR_API int jr_conv_weights_bf16_multi(const jr_wprep* layers, int32_t n_layers, int32_t total_tiles, const float* src,
                                      void* hwio, void* wt, void* stream) {
  if (!layers || !src || n_layers <= 0 || total_tiles < 0) return fail(JR_ERR_INVALID, "conv_weights_bf16_multi: bad arguments");
  if (total_tiles == 0) return JR_OK;
  jr_wprep none{};
  hipLaunchKernelGGL((k_wprep<false, 1>), dim3(total_tiles), dim3(256), 0, as_stream(stream), layers, none, n_layers,
                     src, (uint16_t*)hwio, (uint16_t*)wt);
  return check_launch("conv_weights_bf16_multi");
}

JR_API int jr_conv_weights_x8p(const float* w, int32_t kh, int32_t kw, int32_t c_in, int32_t c_out, void* w_hwio,
                               void* w_t, void* stream) {
  const int tiles = jr_conv_weights_bf16_tiles(kh, kw, c_in, c_out);
  if (!w || tiles <= 0) return fail(JR_ERR_INVALID, "conv_weights_x8p: bad arguments");
  jr_wprep one{0, 0, 0, kh, kw, c_in, c_out, 0, 0};
  hipLaunchKernelGGL((k_wprep<true, 3>), dim3(tiles), dim3(256), 0, as_stream(stream), (const jr_wprep*)nullptr, one,
                     1, w, (uint16_t*)w_hwio, (uint16_t*)w_t);
  return check_launch("conv_weights_x8p");
}

JR_API int jr_conv_weights_x8p_multi(const jr_wprep* layers, int32_t n_layers, int32_t total_tiles, const float* src,
                                     void* hwio, void* wt, void* stream) {
  if (!layers || !src || n_layers <= 0 || total_tiles < 0) return fail(JR_ERR_INVALID, "conv_weights_x8p_multi: bad arguments");
  if (total_tiles == 0) return JR_OK;
  jr_wprep none{};
  hipLaunchKernelGGL((k_wprep<false, 3>), dim3(total_tiles), dim3(256), 0, as_stream(stream), layers, none, n_layers,
                     src, (uint16_t*)hwio, (uint16_t*)wt);
  return check_launch("conv_weights_x8p_multi");
}

JR_API int jr_split_x8p(const float* src, int64_t rows, int32_t c, int32_t src_off, int32_t src_stride, void* dst,
                        int32_t c_pad, int32_t dst_off, int32_t dst_stride, int64_t plane_stride, void* stream) {
  if (!src || !dst || rows < 0 || c <= 0 || c_pad < c || src_off < 0 || src_off + c > src_stride || dst_off < 0 ||
      dst_off + c_pad > dst_stride || plane_stride < rows * dst_stride)
    return fail(JR_ERR_INVALID, "split_x8p: bad arguments");
  if (rows == 0) return JR_OK;
  const bool vec = c % 4 == 0 && c_pad % 4 == 0 && src_off % 4 == 0 && src_stride % 4 == 0 && dst_off % 4 == 0 &&
                   dst_stride % 4 == 0 && plane_stride % 4 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 7) == 0;
  if (vec)
    hipLaunchKernelGGL(k_split_x8p<true>, dim3(grid_for(rows * (c_pad / 4))), dim3(256), 0, as_stream(stream), src, rows,
                       c, src_off, src_stride, (uint16_t*)dst, c_pad, dst_off, dst_stride, plane_stride);
  else
    hipLaunchKernelGGL(k_split_x8p<false>, dim3(grid_for(rows * c_pad)), dim3(256), 0, as_stream(stream), src, rows, c,
                       src_off, src_stride, (uint16_t*)dst, c_pad, dst_off, dst_stride, plane_stride);
  return check_launch("split_x8p");
}

// jr_absmax_prep: per segment, the max |src| of [off, off + count) raised
// into out[seg.out * 64 + blockIdx.x % 64] (atomicMax on the bits of each
// block's max); a segment with limit > 0 whose max exceeds it counts one
// failure per such block into the device error word.  grid (blocks, nseg).
__global__ void __launch_bounds__(256) k_absmax_segs(const float* __restrict__ src, const jr_absmax_seg* __restrict__ segs,
                                                     float* out, unsigned* err) {
  const jr_absmax_seg sg = segs[blockIdx.y];
  float v = 0.f;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < sg.count; i += step)
    v = fmaxf(v, fabsf(src[sg.off + i]));
  __shared__ float s_max[4];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float b = fmaxf(fmaxf(s_max[0], s_max[1]), fmaxf(s_max[2], s_max[3]));
    atomicMax(reinterpret_cast<unsigned*>(out) + (int64_t)sg.out * 64 + (blockIdx.x & 63), __float_as_uint(b));
    if (sg.limit > 0.f && !(b <= sg.limit) && err) atomicAdd(err, 1u);
  }
}

JR_API int jr_absmax_prep(const float* src, const jr_absmax_seg* segs, int32_t nseg, float* out,
                          int64_t zero_floats, void* stream) {
  if (!src || !segs || !out || nseg <= 0 || nseg > 65535 || zero_floats < 0)
    return fail(JR_ERR_INVALID, "absmax_prep: bad arguments");
  hipStream_t s = as_stream(stream);
  if (zero_floats && hipMemsetAsync(out, 0, (size_t)zero_floats * sizeof(float), s) != hipSuccess)
    return fail(JR_ERR_HIP, "absmax_prep: memset failed");
  unsigned* err = device_error_word(s);
  if (!err) return fail(JR_ERR_HIP, "absmax_prep: no device error word (call jr_init before capturing)");
  hipLaunchKernelGGL(k_absmax_segs, dim3(64, nseg), dim3(256), 0, s, src, segs, out, err);
  return check_launch("absmax_prep");
}

JR_API int jr_cast_f32_to_bf16(const float* src, void* dst, int64_t n, void* stream) {
  if (!src || !dst || n < 0) return fail(JR_ERR_INVALID, "cast: bad arguments");
  if (n == 0) return JR_OK;
  hipLaunchKernelGGL(k_f32_to_bf16, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), src, (uint16_t*)dst, n);
  return check_launch("cast f32->bf16");
}

JR_API int jr_cast_bf16_to_f32(const void* src, float* dst, int64_t n, void* stream) {
  if (!src || !dst || n < 0) return fail(JR_ERR_INVALID, "cast: bad arguments");
  if (n == 0) return JR_OK;
  hipLaunchKernelGGL(k_bf16_to_f32, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), (const uint16_t*)src, dst,
                     n);
  return check_launch("cast bf16->f32");
}

JR_API int jr_u8_to_f32_scaled(const uint8_t* src, void* dst, int dtype, int64_t n, void* stream) {
  if (!src || !dst || n < 0) return fail(JR_ERR_INVALID, "u8_scale: bad arguments");
  if (n == 0) return JR_OK;
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_u8_scale<float>, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), src, (float*)dst, n);
  else if (dtype == JR_BF16)
    hipLaunchKernelGGL(k_u8_scale<uint16_t>, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), src,
                       (uint16_t*)dst, n);
  else
    return fail(JR_ERR_INVALID, "u8_scale: bad dtype");
  return check_launch("u8_scale");
}

JR_API int jr_image_u8_to_nhwc(const uint8_t* src, void* dst, int dtype, int64_t pixels, int32_t c,
                               int32_t dst_stride, void* stream) {
  if (!src || !dst || pixels < 0 || c <= 0 || dst_stride < c) return fail(JR_ERR_INVALID, "image_u8: bad arguments");
  if (pixels == 0) return JR_OK;
  const int64_t n = pixels * dst_stride;
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_image_u8<float>, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), src, (float*)dst,
                       pixels, c, dst_stride);
  else if (dtype == JR_BF16)
    hipLaunchKernelGGL(k_image_u8<uint16_t>, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), src,
                       (uint16_t*)dst, pixels, c, dst_stride);
  else
    return fail(JR_ERR_INVALID, "image_u8: bad dtype");
  return check_launch("image_u8");
}

JR_API int jr_brier_accumulate(const float* probs, const float* labels, int32_t n, double* acc, void* stream) {
  if (!probs || !labels || !acc || n < 0) return fail(JR_ERR_INVALID, "brier: bad arguments");
  if (n == 0) return JR_OK;
  hipLaunchKernelGGL(k_brier, dim3(1), dim3(256), 0, as_stream(stream), probs, labels, n, acc);
  return check_launch("brier");
}
