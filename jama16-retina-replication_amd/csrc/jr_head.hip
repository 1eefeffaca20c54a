// jr_head.hip — the classification head and the loss.
//
//   logits = feat . W + b          tf.layers.dense(units)        train.py:133
//   probs  = sigmoid(logits)       tf.sigmoid(name='predictions') train.py:136
//   loss   = mean(max(z,0) - z*y + log1p(exp(-|z|)))             train.py:140-141
//            (tf.nn.sigmoid_cross_entropy_with_logits + reduce_mean)
// Softmax mode (north-star extra): probs = softmax(logits), loss =
// mean_b(-sum_u y log p).  Everything here is a few kB: one workgroup per
// sample for the dense layer, one workgroup for the loss reduction, fixed
// reduction order (deterministic).
#include "jr_common.h"

namespace jr {

constexpr int kMaxUnits = 16;

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// one block (256 threads) per sample b: logits[b][u], probs[b][u]
__global__ void __launch_bounds__(256) k_head_logits(int mode, const float* __restrict__ feat,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     int c, int units, float* logits, float* probs) {
  __shared__ float red[4][kMaxUnits];
  __shared__ float z[kMaxUnits];
  const int b = blockIdx.x, t = threadIdx.x;
  float acc[kMaxUnits];
#pragma unroll
  for (int u = 0; u < kMaxUnits; ++u) acc[u] = 0.f;
  for (int k = t; k < c; k += 256) {
    const float f = feat[(int64_t)b * c + k];
#pragma unroll
    for (int u = 0; u < kMaxUnits; ++u)
      if (u < units) acc[u] = fmaf(f, w[(int64_t)k * units + u], acc[u]);
  }
#pragma unroll
  for (int u = 0; u < kMaxUnits; ++u) {
    if (u < units) {
      const float s = warp_sum(acc[u]);
      if ((t & 63) == 0) red[t >> 6][u] = s;
    }
  }
  __syncthreads();
  if (t < units) {
    const float s = ((red[0][t] + red[1][t]) + (red[2][t] + red[3][t])) + bias[t];
    z[t] = s;
    logits[(int64_t)b * units + t] = s;
  }
  __syncthreads();
  if (t == 0) {
    if (mode == JR_HEAD_SIGMOID) {
      for (int u = 0; u < units; ++u) probs[(int64_t)b * units + u] = 1.f / (1.f + expf(-z[u]));
    } else {
      float mx = z[0];
      for (int u = 1; u < units; ++u) mx = fmaxf(mx, z[u]);
      float se = 0.f;
      for (int u = 0; u < units; ++u) se += expf(z[u] - mx);
      for (int u = 0; u < units; ++u) probs[(int64_t)b * units + u] = expf(z[u] - mx) / se;
    }
  }
}

// single block: loss = mean over elements (sigmoid) or samples (softmax)
__global__ void __launch_bounds__(256) k_head_loss(int mode, const float* __restrict__ logits,
                                                   const float* __restrict__ labels, int n, int units,
                                                   float* loss) {
  __shared__ double red[256];
  const int t = threadIdx.x;
  double s = 0.0;
  if (mode == JR_HEAD_SIGMOID) {
    for (int e = t; e < n * units; e += 256) {
      const float z = logits[e], y = labels[e];
      s += (double)(fmaxf(z, 0.f) - z * y + log1pf(expf(-fabsf(z))));
    }
  } else {
    for (int b = t; b < n; b += 256) {
      const float* zb = logits + (int64_t)b * units;
      float mx = zb[0];
      for (int u = 1; u < units; ++u) mx = fmaxf(mx, zb[u]);
      float se = 0.f;
      for (int u = 0; u < units; ++u) se += expf(zb[u] - mx);
      const float lse = mx + logf(se);
      float l = 0.f;
      for (int u = 0; u < units; ++u) l += labels[(int64_t)b * units + u] * (lse - zb[u]);
      s += (double)l;
    }
  }
  red[t] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  if (t == 0) {
    const double denom = mode == JR_HEAD_SIGMOID ? (double)n * units : (double)n;
    loss[0] = (float)(red[0] / denom);
  }
}

__device__ __forceinline__ float head_dz(int mode, const float* probs, const float* labels, int b, int u, int n,
                                         int units) {
  const float p = probs[(int64_t)b * units + u], y = labels[(int64_t)b * units + u];
  const float denom = mode == JR_HEAD_SIGMOID ? (float)n * (float)units : (float)n;
  return (p - y) / denom;
}

// dfeat[b][k] = sum_u dz[b][u] * W[k][u]
__global__ void k_head_dfeat(int mode, const float* __restrict__ w, const float* __restrict__ probs,
                             const float* __restrict__ labels, int n, int c, int units, float* dfeat) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)n * c) return;
  const int b = (int)(e / c), k = (int)(e - (int64_t)b * c);
  float s = 0.f;
  for (int u = 0; u < units; ++u) s = fmaf(head_dz(mode, probs, labels, b, u, n, units), w[(int64_t)k * units + u], s);
  dfeat[e] = s;
}

// dW[k][u] = sum_b feat[b][k] dz[b][u];  db[u] = sum_b dz[b][u]
__global__ void k_head_dw(int mode, const float* __restrict__ feat, const float* __restrict__ probs,
                          const float* __restrict__ labels, int n, int c, int units, float* dw, float* db) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < (int64_t)c * units) {
    const int k = (int)(e / units), u = (int)(e - (int64_t)k * units);
    float s = 0.f;
    for (int b = 0; b < n; ++b) s = fmaf(feat[(int64_t)b * c + k], head_dz(mode, probs, labels, b, u, n, units), s);
    dw[e] = s;
  }
  if (e < units) {
    float s = 0.f;
    for (int b = 0; b < n; ++b) s += head_dz(mode, probs, labels, b, (int)e, n, units);
    db[e] = s;
  }
}

}  // namespace jr

using namespace jr;

JR_API int jr_head_fwd(int mode, const float* feat, const float* w, const float* b, const float* labels,
                       int32_t n, int32_t c, int32_t units, float* logits, float* probs, float* loss,
                       void* stream) {
  if (mode != JR_HEAD_SIGMOID && mode != JR_HEAD_SOFTMAX) return fail(JR_ERR_INVALID, "head_fwd: bad mode");
  if (!feat || !w || !b || !logits || !probs) return fail(JR_ERR_INVALID, "head_fwd: null pointer");
  if (n <= 0 || c <= 0 || units <= 0 || units > kMaxUnits) return fail(JR_ERR_INVALID, "head_fwd: bad sizes");
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(k_head_logits, dim3(n), dim3(256), 0, s, mode, feat, w, b, c, units, logits, probs);
  int rc = check_launch("head_fwd logits");
  if (rc) return rc;
  if (labels && loss) {
    hipLaunchKernelGGL(k_head_loss, dim3(1), dim3(256), 0, s, mode, (const float*)logits, labels, n, units, loss);
    rc = check_launch("head_fwd loss");
  }
  return rc;
}

JR_API int jr_head_bwd(int mode, const float* feat, const float* w, const float* probs, const float* labels,
                       int32_t n, int32_t c, int32_t units, float* dfeat, float* dw, float* db, void* stream) {
  if (mode != JR_HEAD_SIGMOID && mode != JR_HEAD_SOFTMAX) return fail(JR_ERR_INVALID, "head_bwd: bad mode");
  if (!feat || !w || !probs || !labels || !dfeat || !dw || !db) return fail(JR_ERR_INVALID, "head_bwd: null pointer");
  if (n <= 0 || c <= 0 || units <= 0 || units > kMaxUnits) return fail(JR_ERR_INVALID, "head_bwd: bad sizes");
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(k_head_dfeat, dim3((int)ceil_div((int64_t)n * c, 256)), dim3(256), 0, s, mode, w, probs,
                     labels, n, c, units, dfeat);
  int rc = check_launch("head_bwd dfeat");
  if (rc) return rc;
  hipLaunchKernelGGL(k_head_dw, dim3((int)ceil_div((int64_t)c * units, 256)), dim3(256), 0, s, mode, feat, probs,
                     labels, n, c, units, dw, db);
  return check_launch("head_bwd dw");
}
