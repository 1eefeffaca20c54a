// jr_bn.hip — BatchNormalization(axis=-1, scale=False, eps) + ReLU in
// training mode, forward and backward.
//
// Replaces the FusedBatchNorm / Relu / FusedBatchNormGrad / ReluGrad TF ops of
// every Keras conv2d_bn block built at train.py:129-130.
// The reference graph is built with set_learning_phase(True) (train.py:101),
// so batch statistics are used in training AND evaluation (App. C Q1).
//
//   fwd:  mean = E[x], var = E[(x-mean)^2] (biased), invstd = 1/sqrt(var+eps)
//         y = max((x - mean) * invstd + beta, 0)
//   bwd:  dy' = dy * (y > 0)            (ReluGrad)
//         dbeta = sum dy'
//         dx = invstd * (dy' - mean(dy') - xhat * mean(dy' * xhat))
//
// Reductions are per-chunk partial sums in fp64 combined in a fixed chunk
// order (deterministic, no atomics).  All passes are HBM-streaming kernels
// with 16-byte (fp32x4) accesses along the channel axis.
#include "jr_common.h"

namespace jr {

constexpr int kMaxChunks = 1024;

// Same rounding in fwd and bwd so the ReLU mask is bit-identical.
__device__ __forceinline__ float bn_xhat(float x, float mean, float invstd) {
  return __fmul_rn(__fsub_rn(x, mean), invstd);
}
__device__ __forceinline__ float bn_pre(float x, float mean, float invstd, float beta) {
  return __fadd_rn(bn_xhat(x, mean, invstd), beta);
}

template <typename T> struct V4;
template <> struct V4<float> {
  __device__ static float4 ld(const float* p) { return *reinterpret_cast<const float4*>(p); }
  __device__ static void st(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
};
template <> struct V4<uint16_t> {
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

struct ChunkGeom {
  int64_t m;
  int c;
  int rows_per_chunk;
  int nchunks;
};

static ChunkGeom chunk_geom(int64_t m, int c) {
  ChunkGeom g;
  g.m = m;
  g.c = c;
  int64_t rpc = ceil_div(m, kMaxChunks);
  const int tpr = c / 4;                       // threads per row
  const int rpp = tpr <= 256 ? 256 / tpr : 1;  // rows per pass
  if (rpc < rpp) rpc = rpp;
  const int64_t min_rows = ceil_div(16384, c);  // >= 64 KiB of fp32 input per block
  if (rpc < min_rows) rpc = min_rows;
  g.rows_per_chunk = (int)rpc;
  g.nchunks = (int)ceil_div(m, rpc);
  return g;
}

// Per-chunk column sums.  MODE 0: (sum x, sum x^2).  MODE 1 (bwd):
// (sum dy', sum dy'*xhat).  Thread layout: q = t % tpr is a float4 column
// group, rr = t / tpr a row phase.  Partials: part[chunk][2][c] (fp64).
template <int MODE, typename T>
__global__ void __launch_bounds__(256) k_bn_reduce(const T* __restrict__ x, const T* __restrict__ dy,
                                                   int dy_off, int dy_stride, int64_t m, int c,
                                                   int rows_per_chunk, const float* __restrict__ mean,
                                                   const float* __restrict__ invstd,
                                                   const float* __restrict__ beta, double* part) {
  __shared__ double red[256 * 8];
  const int tpr = c >> 2;
  const int rpp = 256 / tpr;
  const int t = threadIdx.x;
  const int q = t % tpr, rr = t / tpr;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_chunk;
  const int64_t r1 = min(m, r0 + rows_per_chunk);
  double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
  if (rr < rpp) {
    float mu[4], is[4], be[4];
    if (MODE == 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        mu[j] = mean[q * 4 + j]; is[j] = invstd[q * 4 + j]; be[j] = beta[q * 4 + j];
      }
    }
    for (int64_t r = r0 + rr; r < r1; r += rpp) {
      const float4 xv = V4<T>::ld(x + r * c + q * 4);
      const float xa[4] = {xv.x, xv.y, xv.z, xv.w};
      if (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const double d = xa[j];
          s0[j] += d;
          s1[j] += d * d;
        }
      } else {
        const float4 gv = V4<T>::ld(dy + r * dy_stride + dy_off + q * 4);
        const float ga[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float xh = bn_xhat(xa[j], mu[j], is[j]);
          const float pre = __fadd_rn(xh, be[j]);
          const float g = pre > 0.f ? ga[j] : 0.f;
          s0[j] += (double)g;
          s1[j] += (double)g * (double)xh;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[t * 8 + j] = s0[j];
    red[t * 8 + 4 + j] = s1[j];
  }
  __syncthreads();
  if (t < tpr) {
    for (int k = 1; k < rpp; ++k) {
#pragma unroll
      for (int j = 0; j < 8; ++j) red[t * 8 + j] += red[(k * tpr + t) * 8 + j];
    }
    double* pc = part + (int64_t)blockIdx.x * 2 * c;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pc[q * 4 + j] = red[t * 8 + j];
      pc[c + q * 4 + j] = red[t * 8 + 4 + j];
    }
  }
}

// Fixed-order combine of the chunk partials: one wave per channel; lane j
// sums chunks j, j+64, ... (four loads in flight), then a fixed xor-butterfly
// adds the 64 lane sums (deterministic, independent of timing).
// MODE 0: mean, invstd.   MODE 1: k1 = sum dy'/m, k2 = sum dy'xhat/m, dbeta.
template <int MODE>
__global__ void __launch_bounds__(256) k_bn_finalize(const double* __restrict__ part, int nchunks, int c,
                                                     int64_t m, float eps, float* out0, float* out1,
                                                     float* dbeta) {
  const int lane = threadIdx.x & 63;
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= c) return;   // wave-uniform
  const double* p0 = part + k;
  const double* p1 = part + c + k;
  const int64_t st = 2 * (int64_t)c;
  double a0 = 0, a1 = 0, b0 = 0, b1 = 0;
  int i = lane;
  for (; i + 64 < nchunks; i += 128) {
    const double x0 = p0[i * st], y0 = p1[i * st], x1 = p0[(i + 64) * st], y1 = p1[(i + 64) * st];
    a0 += x0; b0 += y0; a1 += x1; b1 += y1;
  }
  if (i < nchunks) { a0 += p0[i * st]; b0 += p1[i * st]; }
  double s0 = a0 + a1, s1 = b0 + b1;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s0 += __shfl_xor(s0, o, 64);
    s1 += __shfl_xor(s1, o, 64);
  }
  if (lane != 0) return;
  const double inv_m = 1.0 / (double)m;
  if (MODE == 0) {
    const double mu = s0 * inv_m;
    double var = s1 * inv_m - mu * mu;
    if (var < 0) var = 0;
    out0[k] = (float)mu;
    out1[k] = (float)(1.0 / sqrt(var + (double)eps));
  } else {
    out0[k] = (float)(s0 * inv_m);
    out1[k] = (float)(s1 * inv_m);
    dbeta[k] = (float)s0;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) k_bn_relu_apply(const T* __restrict__ x, int64_t m, int c,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ invstd,
                                                       const float* __restrict__ beta, T* y, int y_off,
                                                       int y_stride) {
  const int c4 = c >> 2;
  const int64_t total = m * c4;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / c4;
    const int q = (int)(e - r * c4);
    const float4 xv = V4<T>::ld(x + r * c + q * 4);
    const float4 mu = *reinterpret_cast<const float4*>(mean + q * 4);
    const float4 is = *reinterpret_cast<const float4*>(invstd + q * 4);
    const float4 be = *reinterpret_cast<const float4*>(beta + q * 4);
    float4 o;
    o.x = fmaxf(bn_pre(xv.x, mu.x, is.x, be.x), 0.f);
    o.y = fmaxf(bn_pre(xv.y, mu.y, is.y, be.y), 0.f);
    o.z = fmaxf(bn_pre(xv.z, mu.z, is.z, be.z), 0.f);
    o.w = fmaxf(bn_pre(xv.w, mu.w, is.w, be.w), 0.f);
    V4<T>::st(y + r * y_stride + y_off + q * 4, o);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) k_bn_relu_bwd_apply(const T* __restrict__ dy, int dy_off, int dy_stride,
                                                           const T* __restrict__ x, int64_t m, int c,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ k1,
                                                           const float* __restrict__ k2, T* dx) {
  const int c4 = c >> 2;
  const int64_t total = m * c4;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / c4;
    const int q = (int)(e - r * c4);
    const float4 xv = V4<T>::ld(x + r * c + q * 4);
    const float4 gv = V4<T>::ld(dy + r * dy_stride + dy_off + q * 4);
    const float xa[4] = {xv.x, xv.y, xv.z, xv.w};
    const float ga[4] = {gv.x, gv.y, gv.z, gv.w};
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = q * 4 + j;
      const float is = invstd[k];
      const float xh = bn_xhat(xa[j], mean[k], is);
      const float pre = __fadd_rn(xh, beta[k]);
      const float g = pre > 0.f ? ga[j] : 0.f;
      o[j] = is * (g - k1[k] - xh * k2[k]);
    }
    V4<T>::st(dx + r * c + q * 4, make_float4(o[0], o[1], o[2], o[3]));
  }
}

static int grid_for(int64_t elems) {
  const int64_t b = ceil_div(elems, 256);
  return (int)std::min<int64_t>(std::max<int64_t>(b, 1), 256 * 16);
}

static int check_common(int dtype, int64_t m, int c) {
  if (dtype != JR_F32 && dtype != JR_BF16) return fail(JR_ERR_INVALID, "bn: bad dtype");
  if (m <= 0 || c <= 0) return fail(JR_ERR_INVALID, "bn: empty tensor");
  if (c % 4 != 0) return fail(JR_ERR_INVALID, "bn: channel count must be a multiple of 4");
  if (c / 4 > 256) return fail(JR_ERR_UNSUPPORTED, "bn: more than 1024 channels");
  return JR_OK;
}

static size_t ws_need(int64_t m, int c) {
  const ChunkGeom g = chunk_geom(m, c);
  return (size_t)g.nchunks * 2 * c * sizeof(double) + 2 * (size_t)c * sizeof(float);
}

}  // namespace jr

using namespace jr;

JR_API size_t jr_bn_workspace_size(int64_t m, int32_t c) {
  if (m <= 0 || c <= 0 || c % 4) return 0;
  return ws_need(m, c);
}

JR_API int jr_bn_stats(int dtype, const void* x, int64_t m, int32_t c, float eps, float* mean,
                       float* invstd, void* ws, size_t ws_bytes, void* stream) {
  int rc = check_common(dtype, m, c);
  if (rc) return rc;
  if (!x || !mean || !invstd) return fail(JR_ERR_INVALID, "bn_stats: null pointer");
  if (!ws || ws_bytes < ws_need(m, c)) return fail(JR_ERR_WORKSPACE, "bn_stats: workspace too small");
  const ChunkGeom g = chunk_geom(m, c);
  double* part = static_cast<double*>(ws);
  hipStream_t s = as_stream(stream);
  if (dtype == JR_F32)
    hipLaunchKernelGGL((k_bn_reduce<0, float>), dim3(g.nchunks), dim3(256), 0, s, (const float*)x,
                       (const float*)nullptr, 0, 0, m, c, g.rows_per_chunk, nullptr, nullptr, nullptr, part);
  else
    hipLaunchKernelGGL((k_bn_reduce<0, uint16_t>), dim3(g.nchunks), dim3(256), 0, s, (const uint16_t*)x,
                       (const uint16_t*)nullptr, 0, 0, m, c, g.rows_per_chunk, nullptr, nullptr, nullptr,
                       part);
  rc = check_launch("bn_stats reduce");
  if (rc) return rc;
  hipLaunchKernelGGL((k_bn_finalize<0>), dim3((int)ceil_div(c, 4)), dim3(256), 0, s, part, g.nchunks, c, m,
                     eps, mean, invstd, (float*)nullptr);
  return check_launch("bn_stats finalize");
}

JR_API int jr_bn_relu_apply(int dtype, const void* x, int64_t m, int32_t c, const float* mean,
                            const float* invstd, const float* beta, void* y, int32_t y_c_off,
                            int32_t y_c_stride, void* stream) {
  int rc = check_common(dtype, m, c);
  if (rc) return rc;
  if (!x || !mean || !invstd || !beta || !y) return fail(JR_ERR_INVALID, "bn_relu_apply: null pointer");
  if (y_c_off < 0 || y_c_off + c > y_c_stride || (y_c_off % 4) || (y_c_stride % 4))
    return fail(JR_ERR_INVALID, "bn_relu_apply: bad output slice");
  hipStream_t s = as_stream(stream);
  const int grid = grid_for(m * (c / 4));
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_bn_relu_apply<float>, dim3(grid), dim3(256), 0, s, (const float*)x, m, c, mean,
                       invstd, beta, (float*)y, y_c_off, y_c_stride);
  else
    hipLaunchKernelGGL(k_bn_relu_apply<uint16_t>, dim3(grid), dim3(256), 0, s, (const uint16_t*)x, m, c,
                       mean, invstd, beta, (uint16_t*)y, y_c_off, y_c_stride);
  return check_launch("bn_relu_apply");
}

JR_API int jr_bn_relu_bwd(int dtype, const void* dy, int32_t dy_c_off, int32_t dy_c_stride, const void* x,
                          int64_t m, int32_t c, const float* mean, const float* invstd, const float* beta,
                          void* dx, float* dbeta, void* ws, size_t ws_bytes, void* stream) {
  int rc = check_common(dtype, m, c);
  if (rc) return rc;
  if (!dy || !x || !mean || !invstd || !beta || !dx || !dbeta)
    return fail(JR_ERR_INVALID, "bn_relu_bwd: null pointer");
  if (dy_c_off < 0 || dy_c_off + c > dy_c_stride || (dy_c_off % 4) || (dy_c_stride % 4))
    return fail(JR_ERR_INVALID, "bn_relu_bwd: bad dy slice");
  if (!ws || ws_bytes < ws_need(m, c)) return fail(JR_ERR_WORKSPACE, "bn_relu_bwd: workspace too small");
  const ChunkGeom g = chunk_geom(m, c);
  double* part = static_cast<double*>(ws);
  float* k1 = reinterpret_cast<float*>(part + (size_t)g.nchunks * 2 * c);
  float* k2 = k1 + c;
  hipStream_t s = as_stream(stream);
  if (dtype == JR_F32)
    hipLaunchKernelGGL((k_bn_reduce<1, float>), dim3(g.nchunks), dim3(256), 0, s, (const float*)x,
                       (const float*)dy, dy_c_off, dy_c_stride, m, c, g.rows_per_chunk, mean, invstd, beta,
                       part);
  else
    hipLaunchKernelGGL((k_bn_reduce<1, uint16_t>), dim3(g.nchunks), dim3(256), 0, s, (const uint16_t*)x,
                       (const uint16_t*)dy, dy_c_off, dy_c_stride, m, c, g.rows_per_chunk, mean, invstd,
                       beta, part);
  rc = check_launch("bn_bwd reduce");
  if (rc) return rc;
  hipLaunchKernelGGL((k_bn_finalize<1>), dim3((int)ceil_div(c, 4)), dim3(256), 0, s, part, g.nchunks, c, m,
                     0.f, k1, k2, dbeta);
  rc = check_launch("bn_bwd finalize");
  if (rc) return rc;
  const int grid = grid_for(m * (c / 4));
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_bn_relu_bwd_apply<float>, dim3(grid), dim3(256), 0, s, (const float*)dy, dy_c_off,
                       dy_c_stride, (const float*)x, m, c, mean, invstd, beta, k1, k2, (float*)dx);
  else
    hipLaunchKernelGGL(k_bn_relu_bwd_apply<uint16_t>, dim3(grid), dim3(256), 0, s, (const uint16_t*)dy,
                       dy_c_off, dy_c_stride, (const uint16_t*)x, m, c, mean, invstd, beta, k1, k2,
                       (uint16_t*)dx);
  return check_launch("bn_bwd apply");
}
