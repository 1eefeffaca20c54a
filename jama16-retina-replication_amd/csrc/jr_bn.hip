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
// All passes are HBM-streaming: every thread moves one 16-byte vector per
// row (4 fp32 or 8 bf16 channels) and keeps several rows in flight.
// Reductions are per-chunk partial sums in fp64 combined in a fixed chunk
// order (deterministic, no atomics).
#include "jr_common.h"

#include <algorithm>

namespace jr {

#ifndef JR_BN_MAX_CHUNKS
#define JR_BN_MAX_CHUNKS 1024
#endif
#ifndef JR_BN_BWD_ROWS
#define JR_BN_BWD_ROWS 8
#endif
constexpr int kMaxChunks = JR_BN_MAX_CHUNKS;  // partial sums per channel (finalize reads them)
#ifndef JR_BN_F32_SELECT
#define JR_BN_F32_SELECT 0
#endif
constexpr bool kF32Select = JR_BN_F32_SELECT;  // (diagnostic) fp32 reduce loads in the select form
// rows in flight per thread in the reductions (16 B per row and operand)
template <int MODE> constexpr int red_rows() { return MODE == 0 ? 16 : JR_BN_BWD_ROWS; }
#ifndef JR_BN_APP_UNROLL
#define JR_BN_APP_UNROLL 4
#endif
constexpr int kAppUnroll = JR_BN_APP_UNROLL;  // rows per thread in the elementwise passes

// Pins a loaded vector in registers at this point: hipcc otherwise sinks a
// load into the conditional block of its only use (one wait per row).
__device__ __forceinline__ void pin(uint4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }

// (bn_xhat / bn_pre: jr_common.h, shared with the fused BN + max-pool)

// One 16-byte vector of channels: 4 fp32 or 8 bf16, widened to fp32.
template <typename T> struct Vec;
template <> struct Vec<float> {
  static constexpr int N = 4;
  __device__ static void unpack(uint4 u, float* v) {
    v[0] = __uint_as_float(u.x); v[1] = __uint_as_float(u.y);
    v[2] = __uint_as_float(u.z); v[3] = __uint_as_float(u.w);
  }
  __device__ static void ld(const float* p, float* v) { unpack(*reinterpret_cast<const uint4*>(p), v); }
  __device__ static void st(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct Vec<uint16_t> {
  static constexpr int N = 8;
  __device__ static void ld(const uint16_t* p, float* v) { unpack(*reinterpret_cast<const uint4*>(p), v); }
  __device__ static void unpack(uint4 u, float* v) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ static void st(uint16_t* p, const float* v) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};

constexpr int kFoldCh = 256 / kStatsLanes;   // channels per folded apply block (32)
// rows per folded apply block (JR_BN_FOLD_ROWS, read once; A/B knob): each
// block re-combines its 32 channels' partials, so fewer rows per block means
// more parallel blocks and more redundant partial reads
static int fold_rows() {
  static const int v = [] {
    const char* e = std::getenv("JR_BN_FOLD_ROWS");
    const int r = e ? std::atoi(e) : 0;
    return r > 0 ? r : 256;
  }();
  return v;
}
// the backward's finalize folded into its apply: opt-in (JR_FOLD_BN_BWD=1,
// read once) -- measured +0.14 ms/step bf16 against k_bn_finalize8 + apply
// (profiles/r05_ab_rows_bf16.txt), same arithmetic either way
static bool fold_bwd() {
  static const bool on = [] {
    const char* e = std::getenv("JR_FOLD_BN_BWD");
    return e && e[0] == '1';
  }();
  return on;
}

// Thread layout shared by every BN kernel: a row of c channels is tpr =
// c / VW threads (one vector group q each); a 256-thread block covers rpp =
// 256 / tpr rows per pass (row phase rr).  No index division in the loops.
struct ChunkGeom {
  int rows_per_chunk;
  int nchunks;
};

static int vec_width(int dtype) { return dtype == JR_BF16 ? 8 : 4; }

static ChunkGeom chunk_geom(int64_t m, int c, int vw) {
  const int tpr = c / vw;
  const int rpp = std::max(1, 256 / tpr);
  // one unrolled batch of rows per thread at least; at most kMaxChunks chunks
  // (chunks of fewer rows -- more blocks for the 17x17 / 8x8 layers -- measured
  // slower: 1.47 -> 1.83 ms of reduce + 0.46 -> 0.65 ms of finalize per step)
#ifndef JR_BN_MIN_ROWS
#define JR_BN_MIN_ROWS 16
#endif
  // (round 2: a smaller minimum for small m only -- 4 rows per thread below
  // 32,768 rows -- measured slower too: bf16 step 11.46 vs 11.35 ms)
  const int un = JR_BN_MIN_ROWS;
  int64_t rpc = std::max<int64_t>(ceil_div(m, kMaxChunks), (int64_t)rpp * un);
  rpc = ceil_div(rpc, (int64_t)rpp * un) * rpp * un;
  ChunkGeom g;
  g.rows_per_chunk = (int)rpc;
  g.nchunks = (int)ceil_div(m, rpc);
  return g;
}

// Backward inputs of one launch over the c channels of a conv launch's raw
// output: up to kMaxSegs channel segments (the members of a fused sibling
// group, jr_bn_relu_bwd_multi), each with its own upstream gradient slice
// and its own beta / dbeta (the members' tensors are separate).  A thread's
// channel vector is fixed, so it resolves its segment once.
constexpr int kMaxSegs = 4;
struct BnSegs {
  const void* dy[kMaxSegs];
  const float* beta[kMaxSegs];
  float* dbeta[kMaxSegs];
  int dy_off[kMaxSegs], dy_stride[kMaxSegs];
  int c0[kMaxSegs + 1];   // first channel of each segment; c0[n] = c
  int n;
  // backward apply: NULL, or 64 words that receive max |dx| (atomicMax on the
  // bits of each block's max into word blockIdx.x % 64; JR_F32_X6H scales)
  float* absmax;
};

__device__ __forceinline__ int seg_of(const BnSegs& sg, int ch) {
  int s = 0;
#pragma unroll
  for (int i = 1; i < kMaxSegs; ++i) s += (i < sg.n && ch >= sg.c0[i]) ? 1 : 0;
  return s;
}

// Per-chunk column sums.  MODE 0: (sum x, sum x^2).  MODE 1 (bwd):
// (sum dy', sum dy'*xhat).  Per-thread fp64 sums over a fixed row set,
// fixed-order block combine: deterministic.  bf16 MODE 1 sums each batch of
// U rows in fp32 (fma for dy'*xhat) and adds the batch sums in fp64: the
// per-element fp64 conversions and adds of 8 channels per thread had made
// the bf16 reduce VALU-bound (bf16 step 11.22 -> 10.84 ms, interleaved A/B
// on one box; per-shape bnbench 2.65 -> 2.16 ms).  fp32 (4 channels per
// thread) gained 0.3 % from the same change and keeps per-element fp64 sums:
// its 100-step loss-curve fixture is a chaotic trajectory that any change
// of summation order moves past the per-step bar.  Loads stay packed (one uint4
// per row and operand) until used, so red_rows<MODE>() rows are in flight
// per thread: the loop is latency-bound, not bandwidth-bound, with fewer.
// Partials: part[2][c][nchunks] (fp64, chunk-contiguous for the finalize).
// (body: chunk bx of nch; k_bn_reduce runs chunk blockIdx.x of gridDim.x,
// k_bn_reduce_batch a layer's chunk of a batched launch)
template <int MODE, typename T>
__device__ __forceinline__ void bn_reduce_body(const T* __restrict__ x, int xs, const BnSegs& sg, int64_t m, int c,
                                               int rows_per_chunk, const float* __restrict__ mean,
                                               const float* __restrict__ invstd, double* part, int bx, int64_t nch) {
  constexpr int VW = Vec<T>::N;
  constexpr int U = red_rows<MODE>();
  __shared__ double red[256 * 2 * VW];
  const int tpr = c / VW;
  const int rpp = 256 / tpr;
  const int t = threadIdx.x;
  const int q = t % tpr, rr = t / tpr;
  const int64_t r0 = (int64_t)bx * rows_per_chunk;
  const int64_t r1 = min(m, r0 + rows_per_chunk);
  double s0[VW], s1[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) s0[j] = s1[j] = 0.0;
  constexpr bool kBatch32 = sizeof(T) == 2;   // bf16: fp32 sums of one batch of U rows
  float f0[VW], f1[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) f0[j] = f1[j] = 0.f;
  if (rr < rpp) {
    float mu[VW], is[VW], be[VW];
    const T* gp = nullptr;
    int dy_stride = 0;
    if (MODE == 1) {
      const int sgi = seg_of(sg, q * VW), lc = q * VW - sg.c0[sgi];
      gp = static_cast<const T*>(sg.dy[sgi]) + sg.dy_off[sgi] + lc;
      dy_stride = sg.dy_stride[sgi];
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        mu[j] = mean[q * VW + j]; is[j] = invstd[q * VW + j]; be[j] = sg.beta[sgi][lc + j];
      }
    }
    const T* xp = x + q * VW;
    for (int64_t r = r0 + rr; r < r1; r += (int64_t)rpp * U) {
      uint4 xr[U], gr[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        // Rows past the chunk add zero bits (= 0.0 in both dtypes): load the
        // chunk's last row (always valid) and zero after the load.  The
        // select form (JR_BN_F32_SELECT, the fp32 default before the pins
        // below) compiles to a FLAT load from a select of the row address
        // and a scratch copy of the zero constant, a branch and a wait per row.
        const int64_t ri = r + (int64_t)u * rpp;
        const uint4 z = make_uint4(0, 0, 0, 0);
        if constexpr (sizeof(T) == 4 && kF32Select) {
          xr[u] = ri < r1 ? *reinterpret_cast<const uint4*>(xp + ri * xs) : z;
          if (MODE == 1) gr[u] = ri < r1 ? *reinterpret_cast<const uint4*>(gp + ri * dy_stride) : z;
        } else {
          const bool in = ri < r1;
          const int64_t rc = in ? ri : r1 - 1;
          const uint4 xv = *reinterpret_cast<const uint4*>(xp + rc * xs);
          xr[u] = in ? xv : z;
          if (MODE == 1) {
            const uint4 gv = *reinterpret_cast<const uint4*>(gp + rc * dy_stride);
            gr[u] = in ? gv : z;
          }
        }
      }
      // all 2U loads in flight before the first use: without the pins hipcc
      // issued half of them one at a time, each behind vmcnt(0) (a memory
      // round trip per row: the 17^2 / 8^2 reduces took 14-16 us)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        pin(xr[u]);
        if (MODE == 1) pin(gr[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float xv[VW];
        Vec<T>::unpack(xr[u], xv);
        if (MODE == 0) {
#pragma unroll
          for (int j = 0; j < VW; ++j) {
            const double d = xv[j];
            s0[j] += d;
            s1[j] += d * d;
          }
        } else {
          float gv[VW];
          Vec<T>::unpack(gr[u], gv);
#pragma unroll
          for (int j = 0; j < VW; ++j) {
            const float xh = bn_xhat(xv[j], mu[j], is[j]);
            const float pre = __fadd_rn(xh, be[j]);
            const float g = pre > 0.f ? gv[j] : 0.f;
            if constexpr (kBatch32) {
              f0[j] += g;
              f1[j] = fmaf(g, xh, f1[j]);
            } else {
              s0[j] += (double)g;
              s1[j] += (double)g * (double)xh;
            }
          }
        }
      }
      if (MODE == 1 && kBatch32) {
#pragma unroll
        for (int j = 0; j < VW; ++j) {
          s0[j] += (double)f0[j];
          s1[j] += (double)f1[j];
          f0[j] = f1[j] = 0.f;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    red[t * 2 * VW + j] = s0[j];
    red[t * 2 * VW + VW + j] = s1[j];
  }
  __syncthreads();
  // fixed-shape tree over the row phases (log2(rpp) steps, deterministic)
  int span = 1;
  while (span < rpp) span <<= 1;
  for (int s = span >> 1; s > 0; s >>= 1) {
    if (rr < s && rr + s < rpp) {
      double* a = red + t * 2 * VW;
      const double* b = red + (t + s * tpr) * 2 * VW;
#pragma unroll
      for (int j = 0; j < 2 * VW; ++j) a[j] += b[j];
    }
    __syncthreads();
  }
  if (t < tpr) {
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      part[(int64_t)(q * VW + j) * nch + bx] = red[t * 2 * VW + j];
      part[(int64_t)(c + q * VW + j) * nch + bx] = red[t * 2 * VW + VW + j];
    }
  }
}

template <int MODE, typename T>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2)))
k_bn_reduce(const T* __restrict__ x, int xs, BnSegs sg, int64_t m, int c, int rows_per_chunk,
            const float* __restrict__ mean, const float* __restrict__ invstd, double* part) {
  bn_reduce_body<MODE, T>(x, xs, sg, m, c, rows_per_chunk, mean, invstd, part, blockIdx.x, gridDim.x);
}

// Fixed-order combine of the chunk partials: one wave per channel; lane j
// sums chunks j, j+64, ... (coalesced, eight loads in flight), then a fixed
// xor-butterfly adds the 64 lane sums (deterministic, independent of timing).
// MODE 0: mean, invstd.   MODE 1: k1 = sum dy'/m, k2 = sum dy'xhat/m, dbeta.
template <int MODE>
__global__ void __launch_bounds__(256) k_bn_finalize(const double* __restrict__ part, int nchunks, int c,
                                                     int64_t m, float eps, float* out0, float* out1, BnSegs sg) {
  const int lane = threadIdx.x & 63;
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= c) return;   // wave-uniform
  const double* p0 = part + (int64_t)k * nchunks;
  const double* p1 = part + (int64_t)(c + k) * nchunks;
  double a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
  for (int i0 = 0; i0 < nchunks; i0 += 256) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * 64 + lane;
      if (i < nchunks) { a[u] += p0[i]; b[u] += p1[i]; }
    }
  }
  double s0 = (a[0] + a[1]) + (a[2] + a[3]), s1 = (b[0] + b[1]) + (b[2] + b[3]);
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
    const int sgi = seg_of(sg, k);
    sg.dbeta[sgi][k - sg.c0[sgi]] = (float)s0;
  }
}

// Elementwise passes: block b covers rows [b*rpp*U, (b+1)*rpp*U), thread
// (q, rr) rows rr, rr+rpp, ...; per-channel constants loaded once.
// Grouped (ensemble members, blockIdx.y = member): x, y, the statistics and
// beta move by their member strides (bytes; all 0 for an ordinary launch).
template <typename T>
__global__ void __launch_bounds__(256) k_bn_relu_apply(const T* __restrict__ x, int xs, int64_t m, int c,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ invstd,
                                                       const float* __restrict__ beta, T* y, int y_off,
                                                       int y_stride, int64_t x_mb, int64_t y_mb, int64_t st_mb,
                                                       int64_t be_mb) {
  if (gridDim.y > 1) {
    const int64_t mb = blockIdx.y;
    x = reinterpret_cast<const T*>(reinterpret_cast<const char*>(x) + mb * x_mb);
    y = reinterpret_cast<T*>(reinterpret_cast<char*>(y) + mb * y_mb);
    mean = reinterpret_cast<const float*>(reinterpret_cast<const char*>(mean) + mb * st_mb);
    invstd = reinterpret_cast<const float*>(reinterpret_cast<const char*>(invstd) + mb * st_mb);
    beta = reinterpret_cast<const float*>(reinterpret_cast<const char*>(beta) + mb * be_mb);
  }
  constexpr int VW = Vec<T>::N;
  const int tpr = c / VW;
  const int rpp = 256 / tpr;
  const int t = threadIdx.x;
  const int q = t % tpr, rr = t / tpr;
  if (rr >= rpp) return;
  float mu[VW], is[VW], be[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    mu[j] = mean[q * VW + j]; is[j] = invstd[q * VW + j]; be[j] = beta[q * VW + j];
  }
  const int64_t r0 = (int64_t)blockIdx.x * rpp * kAppUnroll + rr;
  // every row's load is unconditional (rows past m re-read row m - 1) and
  // unpacked only after all were issued: a load under `if (r < m)` whose
  // bf16 unpack sat in the same branch made hipcc wait for each row in turn
  uint4 xr[kAppUnroll];
#pragma unroll
  for (int u = 0; u < kAppUnroll; ++u) {
    const int64_t r = min(r0 + (int64_t)u * rpp, m - 1);
    xr[u] = *reinterpret_cast<const uint4*>(x + r * xs + q * VW);
  }
#pragma unroll
  for (int u = 0; u < kAppUnroll; ++u) pin(xr[u]);
#pragma unroll
  for (int u = 0; u < kAppUnroll; ++u) {
    const int64_t r = r0 + (int64_t)u * rpp;
    if (r >= m) break;
    float xv[VW], o[VW];
    Vec<T>::unpack(xr[u], xv);
#pragma unroll
    for (int j = 0; j < VW; ++j) o[j] = fmaxf(bn_pre(xv[j], mu[j], is[j], be[j]), 0.f);
    Vec<T>::st(y + r * y_stride + y_off + q * VW, o);
  }
}

// The apply of a fused sibling launch's members in ONE launch
// (jr_bn_relu_apply_multi): the raw output's c channels, segment i its own
// output slice and beta; per element exactly k_bn_relu_apply's arithmetic.
struct ApplySegs {
  void* y[kMaxSegs];
  const float* beta[kMaxSegs];
  int y_off[kMaxSegs], y_stride[kMaxSegs];
  int c0[kMaxSegs + 1];
  int n;
};

template <typename T>
__global__ void __launch_bounds__(256) k_bn_relu_apply_multi(const T* __restrict__ x, int xs, int64_t m, int c,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd, ApplySegs sg) {
  constexpr int VW = Vec<T>::N;
  const int tpr = c / VW;
  const int rpp = 256 / tpr;
  const int t = threadIdx.x;
  const int q = t % tpr, rr = t / tpr;
  if (rr >= rpp) return;
  int si = 0;
#pragma unroll
  for (int i = 1; i < kMaxSegs; ++i) si += (i < sg.n && q * VW >= sg.c0[i]) ? 1 : 0;
  const int lc = q * VW - sg.c0[si];
  T* y = static_cast<T*>(sg.y[si]) + sg.y_off[si] + lc;
  const int ys = sg.y_stride[si];
  float mu[VW], is[VW], be[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    mu[j] = mean[q * VW + j]; is[j] = invstd[q * VW + j]; be[j] = sg.beta[si][lc + j];
  }
  const int64_t r0 = (int64_t)blockIdx.x * rpp * kAppUnroll + rr;
  uint4 xr[kAppUnroll];
#pragma unroll
  for (int u = 0; u < kAppUnroll; ++u) {
    const int64_t r = min(r0 + (int64_t)u * rpp, m - 1);
    xr[u] = *reinterpret_cast<const uint4*>(x + r * xs + q * VW);
  }
#pragma unroll
  for (int u = 0; u < kAppUnroll; ++u) pin(xr[u]);
#pragma unroll
  for (int u = 0; u < kAppUnroll; ++u) {
    const int64_t r = r0 + (int64_t)u * rpp;
    if (r >= m) break;
    float xv[VW], o[VW];
    Vec<T>::unpack(xr[u], xv);
#pragma unroll
    for (int j = 0; j < VW; ++j) o[j] = fmaxf(bn_pre(xv[j], mu[j], is[j], be[j]), 0.f);
    Vec<T>::st(y + r * ys, o);
  }
}

// k_bn_relu_apply with the statistics finalize folded in: block (bx, by)
// first combines the conv's single-stage partials of the 32 channels of group
// by (stats_combine8: 8 lanes per channel, bitwise what k_stats_finalize8
// writes) into LDS -- blocks with bx == 0 also store them as the layer's
// mean / invstd -- then applies BN + ReLU to rows [bx*rpb, (bx+1)*rpb) of
// those channels, thread (q, rr) one 16-byte vector q of the group and rows
// rr, rr + rpp, ... (the arithmetic of k_bn_relu_apply).
template <typename T>
__global__ void __launch_bounds__(256) k_bn_relu_apply_stats(const T* __restrict__ x, int xs, int64_t m, int c,
                                                             const float* __restrict__ pm, const float* __restrict__ pq,
                                                             int P, int R, float eps, float* mean_out,
                                                             float* invstd_out, const float* __restrict__ beta, T* y,
                                                             int y_off, int y_stride, int rpb) {
  constexpr int VW = Vec<T>::N;
  __shared__ float s_mu[kFoldCh], s_is[kFoldCh];
  const int t = threadIdx.x;
  const int c0 = blockIdx.y * kFoldCh;
  const int cg = min(kFoldCh, c - c0);
  {
    const int slot = t / kStatsLanes, j = t % kStatsLanes;
    if (slot < cg) {
      const int ch = c0 + slot;
      float mu, is;
      stats_combine8(pm + (int64_t)ch * P, pq + (int64_t)ch * P, P, R, (int)m, eps, j, &mu, &is);
      if (j == 0) {
        s_mu[slot] = mu;
        s_is[slot] = is;
        if (blockIdx.x == 0) {
          mean_out[ch] = mu;
          invstd_out[ch] = is;
        }
      }
    }
  }
  __syncthreads();
  const int tpr = cg / VW;
  const int rpp = 256 / tpr;
  const int q = t % tpr, rr = t / tpr;
  if (rr >= rpp) return;
  float mu[VW], is[VW], be[VW];
#pragma unroll
  for (int k = 0; k < VW; ++k) {
    mu[k] = s_mu[q * VW + k]; is[k] = s_is[q * VW + k]; be[k] = beta[c0 + q * VW + k];
  }
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = min(m, r0 + rpb);
  const int co = c0 + q * VW;
  for (int64_t rb = r0 + rr; rb < r1; rb += (int64_t)rpp * kAppUnroll) {
    // unconditional loads (rows past the block re-read its last row), unpacked
    // after all were issued (as in k_bn_relu_apply)
    uint4 xr[kAppUnroll];
#pragma unroll
    for (int u = 0; u < kAppUnroll; ++u) {
      const int64_t r = min(rb + (int64_t)u * rpp, r1 - 1);
      xr[u] = *reinterpret_cast<const uint4*>(x + r * xs + co);
    }
#pragma unroll
    for (int u = 0; u < kAppUnroll; ++u) pin(xr[u]);
#pragma unroll
    for (int u = 0; u < kAppUnroll; ++u) {
      const int64_t r = rb + (int64_t)u * rpp;
      if (r >= r1) break;
      float xv[VW], o[VW];
      Vec<T>::unpack(xr[u], xv);
#pragma unroll
      for (int k = 0; k < VW; ++k) o[k] = fmaxf(bn_pre(xv[k], mu[k], is[k], be[k]), 0.f);
      Vec<T>::st(y + r * y_stride + y_off + co, o);
    }
  }
}

// returns the largest |dx| this thread stored (0 if none)
template <typename T>
__device__ __forceinline__ float bn_bwd_apply_body(const BnSegs& sg, const T* __restrict__ x, int xs, int64_t m, int c,
                                                   const float* __restrict__ mean, const float* __restrict__ invstd,
                                                   const float* __restrict__ k1, const float* __restrict__ k2, T* dx,
                                                   int bx) {
  constexpr int VW = Vec<T>::N;
  const int tpr = c / VW;
  const int rpp = 256 / tpr;
  const int t = threadIdx.x;
  const int q = t % tpr, rr = t / tpr;
  if (rr >= rpp) return 0.f;
  const int sgi = seg_of(sg, q * VW), lc = q * VW - sg.c0[sgi];
  const T* dy = static_cast<const T*>(sg.dy[sgi]) + sg.dy_off[sgi] + lc;
  const int dy_stride = sg.dy_stride[sgi];
  float mu[VW], is[VW], be[VW], c1[VW], c2[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    const int k = q * VW + j;
    mu[j] = mean[k]; is[j] = invstd[k]; be[j] = sg.beta[sgi][lc + j]; c1[j] = k1[k]; c2[j] = k2[k];
  }
  const int64_t r0 = (int64_t)bx * rpp * kAppUnroll + rr;
  // unconditional loads (rows past m re-read row m - 1), unpacked after all
  // were issued (as in k_bn_relu_apply)
  uint4 xr[kAppUnroll], gr[kAppUnroll];
#pragma unroll
  for (int u = 0; u < kAppUnroll; ++u) {
    const int64_t r = min(r0 + (int64_t)u * rpp, m - 1);
    xr[u] = *reinterpret_cast<const uint4*>(x + r * xs + q * VW);
    gr[u] = *reinterpret_cast<const uint4*>(dy + r * dy_stride);
  }
#pragma unroll
  for (int u = 0; u < kAppUnroll; ++u) {
    pin(xr[u]);
    pin(gr[u]);
  }
  float amax = 0.f;
#pragma unroll
  for (int u = 0; u < kAppUnroll; ++u) {
    const int64_t r = r0 + (int64_t)u * rpp;
    if (r >= m) break;
    float xv[VW], gv[VW], o[VW];
    Vec<T>::unpack(xr[u], xv);
    Vec<T>::unpack(gr[u], gv);
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      const float xh = bn_xhat(xv[j], mu[j], is[j]);
      const float pre = __fadd_rn(xh, be[j]);
      const float g = pre > 0.f ? gv[j] : 0.f;
      o[j] = is[j] * (g - c1[j] - xh * c2[j]);
      amax = fmaxf(amax, fabsf(o[j]));
    }
    Vec<T>::st(dx + r * xs + q * VW, o);
  }
  return amax;
}

// The block's max of v into word blockIdx.x % 64 of out (atomicMax on the
// float bits: every value is >= 0).  Every thread of the block calls it.
__device__ __forceinline__ void block_absmax_to(float v, float* out) {
  __shared__ float s_max[4];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = s_max[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) b = fmaxf(b, s_max[w]);
    atomicMax(reinterpret_cast<unsigned*>(out) + (blockIdx.x & 63), __float_as_uint(b));
  }
}

template <typename T>
__global__ void __launch_bounds__(256) k_bn_relu_bwd_apply(BnSegs sg, const T* __restrict__ x, int xs, int64_t m,
                                                           int c, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ k1,
                                                           const float* __restrict__ k2, T* dx) {
  const float amax = bn_bwd_apply_body<T>(sg, x, xs, m, c, mean, invstd, k1, k2, dx, blockIdx.x);
  if (sg.absmax) block_absmax_to(amax, sg.absmax);   // (uniform: a kernel argument)
}

// Canonical combine of ONE channel's backward-reduce partials when there are
// at most kFoldMaxP of them (fp64 (sum dy', sum dy' xhat) per chunk): an
// aligned group of 8 lanes, lane j summing chunks j, j+8, ... in order, then
// an xor butterfly.  k_bn_finalize8 and k_bn_relu_bwd_apply_fold share it, so
// the folded backward is bitwise the three-launch one.
__device__ __forceinline__ void bwd_combine8(const double* __restrict__ p0, const double* __restrict__ p1, int nch,
                                             int j, double* s0, double* s1) {
  double a = 0, b = 0;
  constexpr int U = 8;
  for (int i0 = j; i0 < nch; i0 += kStatsLanes * U) {
    double va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ic = min(i0 + kStatsLanes * u, nch - 1);
      va[u] = p0[ic];
      vb[u] = p1[ic];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + kStatsLanes * u < nch) {
        a += va[u];
        b += vb[u];
      }
  }
#pragma unroll
  for (int o = kStatsLanes / 2; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, kStatsLanes);
    b += __shfl_xor(b, o, kStatsLanes);
  }
  *s0 = a;
  *s1 = b;
}

// k_bn_finalize<1> for at most kFoldMaxP chunks: 32 channels per block.
__device__ __forceinline__ void bn_finalize8_body(const double* __restrict__ part, int nchunks, int c, int64_t m,
                                                  float* k1, float* k2, const BnSegs& sg, int bx) {
  const int k = bx * (256 / kStatsLanes) + threadIdx.x / kStatsLanes, j = threadIdx.x % kStatsLanes;
  if (k >= c) return;   // (whole 8-lane groups)
  double s0, s1;
  bwd_combine8(part + (int64_t)k * nchunks, part + (int64_t)(c + k) * nchunks, nchunks, j, &s0, &s1);
  if (j != 0) return;
  const double inv_m = 1.0 / (double)m;
  k1[k] = (float)(s0 * inv_m);
  k2[k] = (float)(s1 * inv_m);
  const int sgi = seg_of(sg, k);
  sg.dbeta[sgi][k - sg.c0[sgi]] = (float)s0;
}

__global__ void __launch_bounds__(256) k_bn_finalize8(const double* __restrict__ part, int nchunks, int c, int64_t m,
                                                      float* k1, float* k2, BnSegs sg) {
  bn_finalize8_body(part, nchunks, c, m, k1, k2, sg, blockIdx.x);
}

// The backward's finalize folded into its apply: block (bx, by) combines the
// reduce's partials of the 32 channels of group by (bwd_combine8; bx == 0
// also stores dbeta), then applies the backward to rows [bx*rpb, (bx+1)*rpb)
// of those channels with the arithmetic of k_bn_relu_bwd_apply.
template <typename T>
__global__ void __launch_bounds__(256) k_bn_relu_bwd_apply_fold(BnSegs sg, const T* __restrict__ x, int xs, int64_t m,
                                                                int c, const float* __restrict__ mean,
                                                                const float* __restrict__ invstd,
                                                                const double* __restrict__ part, int nchunks, T* dx,
                                                                int rpb) {
  constexpr int VW = Vec<T>::N;
  __shared__ float s_k1[kFoldCh], s_k2[kFoldCh];
  const int t = threadIdx.x;
  const int c0 = blockIdx.y * kFoldCh;
  const int cg = min(kFoldCh, c - c0);
  {
    const int slot = t / kStatsLanes, j = t % kStatsLanes;
    if (slot < cg) {
      const int k = c0 + slot;
      double s0, s1;
      bwd_combine8(part + (int64_t)k * nchunks, part + (int64_t)(c + k) * nchunks, nchunks, j, &s0, &s1);
      if (j == 0) {
        const double inv_m = 1.0 / (double)m;
        s_k1[slot] = (float)(s0 * inv_m);
        s_k2[slot] = (float)(s1 * inv_m);
        if (blockIdx.x == 0) {
          const int sgi = seg_of(sg, k);
          sg.dbeta[sgi][k - sg.c0[sgi]] = (float)s0;
        }
      }
    }
  }
  __syncthreads();
  const int tpr = cg / VW;
  const int rpp = 256 / tpr;
  const int q = t % tpr, rr = t / tpr;
  if (rr >= rpp) return;
  const int ch = c0 + q * VW;
  const int sgi = seg_of(sg, ch), lc = ch - sg.c0[sgi];
  const T* dy = static_cast<const T*>(sg.dy[sgi]) + sg.dy_off[sgi] + lc;
  const int dy_stride = sg.dy_stride[sgi];
  float mu[VW], is[VW], be[VW], c1[VW], c2[VW];
#pragma unroll
  for (int k = 0; k < VW; ++k) {
    mu[k] = mean[ch + k]; is[k] = invstd[ch + k]; be[k] = sg.beta[sgi][lc + k];
    c1[k] = s_k1[q * VW + k]; c2[k] = s_k2[q * VW + k];
  }
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = min(m, r0 + rpb);
  for (int64_t rb = r0 + rr; rb < r1; rb += (int64_t)rpp * kAppUnroll) {
    uint4 xr[kAppUnroll], gr[kAppUnroll];
#pragma unroll
    for (int u = 0; u < kAppUnroll; ++u) {
      const int64_t r = min(rb + (int64_t)u * rpp, r1 - 1);
      xr[u] = *reinterpret_cast<const uint4*>(x + r * xs + ch);
      gr[u] = *reinterpret_cast<const uint4*>(dy + r * dy_stride);
    }
#pragma unroll
    for (int u = 0; u < kAppUnroll; ++u) {
      pin(xr[u]);
      pin(gr[u]);
    }
#pragma unroll
    for (int u = 0; u < kAppUnroll; ++u) {
      const int64_t r = rb + (int64_t)u * rpp;
      if (r >= r1) break;
      float xv[VW], gv[VW], o[VW];
      Vec<T>::unpack(xr[u], xv);
      Vec<T>::unpack(gr[u], gv);
#pragma unroll
      for (int k = 0; k < VW; ++k) {
        const float xh = bn_xhat(xv[k], mu[k], is[k]);
        const float pre = __fadd_rn(xh, be[k]);
        const float g = pre > 0.f ? gv[k] : 0.f;
        o[k] = is[k] * (g - c1[k] - xh * c2[k]);
      }
      Vec<T>::st(dx + r * xs + ch, o);
    }
  }
}

// Several independent layers' backwards in ONE set of three launches
// (jr_bn_relu_bwd_batch): layer l owns blocks [b0, b0 + blocks) of each
// launch and runs exactly the single-layer bodies on them (same chunk
// geometry, same finalize arithmetic: bitwise jr_bn_relu_bwd_multi per layer).
constexpr int kBnBatchMax = 8;
struct BnBatchLayer {
  BnSegs sg;
  const void* x;
  void* dx;
  const float* mean;
  const float* invstd;
  double* part;
  float* k1;
  float* k2;
  int64_t m;
  int c, xs, rpc, nchunks;
  int b0[3];   // first block in the reduce / finalize / apply launch
};
struct BnBatch {
  BnBatchLayer L[kBnBatchMax];
  int n;
};

// the layer owning block b of launch `which` (wave-uniform linear scan)
__device__ __forceinline__ int bn_batch_layer(const BnBatch& bt, int which, int b) {
  int l = 0;
  for (int i = 1; i < bt.n; ++i) l = b >= bt.L[i].b0[which] ? i : l;
  return l;
}

template <typename T>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) k_bn_reduce_batch(BnBatch bt) {
  const int l = bn_batch_layer(bt, 0, blockIdx.x);
  const BnBatchLayer& L = bt.L[l];
  bn_reduce_body<1, T>(static_cast<const T*>(L.x), L.xs, L.sg, L.m, L.c, L.rpc, L.mean, L.invstd, L.part,
                       blockIdx.x - L.b0[0], L.nchunks);
}

__global__ void __launch_bounds__(256) k_bn_finalize8_batch(BnBatch bt) {
  const int l = bn_batch_layer(bt, 1, blockIdx.x);
  const BnBatchLayer& L = bt.L[l];
  bn_finalize8_body(L.part, L.nchunks, L.c, L.m, L.k1, L.k2, L.sg, blockIdx.x - L.b0[1]);
}

template <typename T>
__global__ void __launch_bounds__(256) k_bn_relu_bwd_apply_batch(BnBatch bt) {
  const int l = bn_batch_layer(bt, 2, blockIdx.x);
  const BnBatchLayer& L = bt.L[l];
  bn_bwd_apply_body<T>(L.sg, static_cast<const T*>(L.x), L.xs, L.m, L.c, L.mean, L.invstd, L.k1, L.k2,
                       static_cast<T*>(L.dx), blockIdx.x - L.b0[2]);
}

static int apply_grid(int64_t m, int c, int vw) {
  const int rpp = 256 / (c / vw);
  return (int)ceil_div(m, (int64_t)rpp * kAppUnroll);
}

static int check_common(int dtype, int64_t m, int c) {
  if (dtype != JR_F32 && dtype != JR_BF16) return fail(JR_ERR_INVALID, "bn: bad dtype");
  if (m <= 0 || c <= 0) return fail(JR_ERR_INVALID, "bn: empty tensor");
  if (c % vec_width(dtype) != 0)
    return fail(JR_ERR_INVALID, "bn: channel count must be a multiple of 4 (fp32) / 8 (bf16)");
  if (c / vec_width(dtype) > 256) return fail(JR_ERR_UNSUPPORTED, "bn: more than 256 vectors per row");
  return JR_OK;
}

static int check_slice(int dtype, int off, int stride, int c) {
  const int q = vec_width(dtype);
  return off >= 0 && off + c <= stride && off % q == 0 && stride % q == 0;
}

// Partials for either dtype's geometry (the query carries no dtype).
static size_t ws_need(int64_t m, int c) {
  size_t n = 0;
  for (int vw : {4, 8})
    if (c % vw == 0) n = std::max(n, (size_t)chunk_geom(m, c, vw).nchunks);
  return n * 2 * c * sizeof(double) + 2 * (size_t)c * sizeof(float);
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
  const ChunkGeom g = chunk_geom(m, c, vec_width(dtype));
  double* part = static_cast<double*>(ws);
  hipStream_t s = as_stream(stream);
  const BnSegs none{};
  if (dtype == JR_F32)
    hipLaunchKernelGGL((k_bn_reduce<0, float>), dim3(g.nchunks), dim3(256), 0, s, (const float*)x, c, none, m, c,
                       g.rows_per_chunk, nullptr, nullptr, part);
  else
    hipLaunchKernelGGL((k_bn_reduce<0, uint16_t>), dim3(g.nchunks), dim3(256), 0, s, (const uint16_t*)x, c, none,
                       m, c, g.rows_per_chunk, nullptr, nullptr, part);
  rc = check_launch("bn_stats reduce");
  if (rc) return rc;
  hipLaunchKernelGGL((k_bn_finalize<0>), dim3((int)ceil_div(c, 4)), dim3(256), 0, s, part, g.nchunks, c, m,
                     eps, mean, invstd, none);
  return check_launch("bn_stats finalize");
}

static int bn_apply_launch(int dtype, int members, const void* x, int32_t x_c_stride, int64_t x_mb, int64_t m,
                           int32_t c, const float* mean, const float* invstd, int64_t st_mb, const float* beta,
                           int64_t be_mb, void* y, int32_t y_c_off, int32_t y_c_stride, int64_t y_mb, hipStream_t s) {
  const dim3 grid(apply_grid(m, c, vec_width(dtype)), members);
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_bn_relu_apply<float>, grid, dim3(256), 0, s, (const float*)x, x_c_stride, m, c, mean,
                       invstd, beta, (float*)y, y_c_off, y_c_stride, x_mb, y_mb, st_mb, be_mb);
  else
    hipLaunchKernelGGL(k_bn_relu_apply<uint16_t>, grid, dim3(256), 0, s, (const uint16_t*)x, x_c_stride, m, c,
                       mean, invstd, beta, (uint16_t*)y, y_c_off, y_c_stride, x_mb, y_mb, st_mb, be_mb);
  return check_launch("bn_relu_apply");
}

JR_API int jr_bn_relu_apply(int dtype, const void* x, int32_t x_c_off, int32_t x_c_stride, int64_t m, int32_t c,
                            const float* mean, const float* invstd, const float* beta, void* y, int32_t y_c_off,
                            int32_t y_c_stride, void* stream) {
  int rc = check_common(dtype, m, c);
  if (rc) return rc;
  if (!x || !mean || !invstd || !beta || !y) return fail(JR_ERR_INVALID, "bn_relu_apply: null pointer");
  if (!check_slice(dtype, x_c_off, x_c_stride, c)) return fail(JR_ERR_INVALID, "bn_relu_apply: bad input slice");
  const size_t esz = dtype == JR_BF16 ? 2 : 4;
  x = static_cast<const char*>(x) + (size_t)x_c_off * esz;
  if (!check_slice(dtype, y_c_off, y_c_stride, c)) return fail(JR_ERR_INVALID, "bn_relu_apply: bad output slice");
  return bn_apply_launch(dtype, 1, x, x_c_stride, 0, m, c, mean, invstd, 0, beta, 0, y, y_c_off, y_c_stride, 0,
                         as_stream(stream));
}

JR_API int jr_bn_relu_apply_multi(int dtype, int nseg, const jr_bn_apply_seg* segs, const void* x, int32_t x_c_off,
                                  int32_t x_c_stride, int64_t m, int32_t c, const float* mean, const float* invstd,
                                  void* stream) {
  int rc = check_common(dtype, m, c);
  if (rc) return rc;
  if (!segs || nseg < 1 || nseg > kMaxSegs) return fail(JR_ERR_INVALID, "bn_relu_apply_multi: 1..4 segments");
  if (!x || !mean || !invstd) return fail(JR_ERR_INVALID, "bn_relu_apply_multi: null pointer");
  if (!check_slice(dtype, x_c_off, x_c_stride, c)) return fail(JR_ERR_INVALID, "bn_relu_apply_multi: bad input slice");
  ApplySegs sg{};
  sg.n = nseg;
  int c0 = 0;
  for (int i = 0; i < nseg; ++i) {
    const jr_bn_apply_seg& e = segs[i];
    if (!e.y || !e.beta) return fail(JR_ERR_INVALID, "bn_relu_apply_multi: null pointer in a segment");
    if (e.c <= 0 || e.c % vec_width(dtype) || !check_slice(dtype, e.y_c_off, e.y_c_stride, e.c))
      return fail(JR_ERR_INVALID, "bn_relu_apply_multi: bad output segment");
    sg.y[i] = e.y;
    sg.beta[i] = e.beta;
    sg.y_off[i] = e.y_c_off;
    sg.y_stride[i] = e.y_c_stride;
    sg.c0[i] = c0;
    c0 += e.c;
  }
  if (c0 != c) return fail(JR_ERR_INVALID, "bn_relu_apply_multi: segment channels must sum to c");
  sg.c0[nseg] = c;
  const size_t esz = dtype == JR_BF16 ? 2 : 4;
  x = static_cast<const char*>(x) + (size_t)x_c_off * esz;
  const dim3 grid(apply_grid(m, c, vec_width(dtype)));
  hipStream_t s = as_stream(stream);
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_bn_relu_apply_multi<float>, grid, dim3(256), 0, s, (const float*)x, x_c_stride, m, c, mean,
                       invstd, sg);
  else
    hipLaunchKernelGGL(k_bn_relu_apply_multi<uint16_t>, grid, dim3(256), 0, s, (const uint16_t*)x, x_c_stride, m, c,
                       mean, invstd, sg);
  return check_launch("bn_relu_apply_multi");
}

JR_API int jr_bn_relu_apply_stats(int dtype, const void* x, int32_t x_c_off, int32_t x_c_stride, int64_t m, int32_t c,
                                  const float* part, int32_t P, int32_t R, int32_t n_total, int32_t stat_c_off,
                                  float eps, float* mean, float* invstd, const float* beta, void* y, int32_t y_c_off,
                                  int32_t y_c_stride, void* stream) {
  int rc = check_common(dtype, m, c);
  if (rc) return rc;
  if (!x || !part || !mean || !invstd || !beta || !y) return fail(JR_ERR_INVALID, "bn_relu_apply_stats: null pointer");
  if (!check_slice(dtype, x_c_off, x_c_stride, c) || !check_slice(dtype, y_c_off, y_c_stride, c))
    return fail(JR_ERR_INVALID, "bn_relu_apply_stats: bad input / output slice");
  if (P < 1 || R < 1 || (int64_t)P * R < m || stat_c_off < 0 || stat_c_off + c > n_total || m >= (1LL << 31))
    return fail(JR_ERR_INVALID, "bn_relu_apply_stats: partials inconsistent with the slice");
  const size_t esz = dtype == JR_BF16 ? 2 : 4;
  x = static_cast<const char*>(x) + (size_t)x_c_off * esz;
  const float* pm = part + (int64_t)stat_c_off * P;
  const float* pq = part + (int64_t)(n_total + stat_c_off) * P;
  // rows per block: a multiple of one pass x unroll (the 32-channel group's
  // widest pass), about JR_BN_FOLD_ROWS (each block re-combines its group's
  // partials: fewer, longer blocks read them fewer times)
  const int vw = vec_width(dtype);
  const int step = 256 / (kFoldCh / vw) * kAppUnroll;
  const int rpb = (int)std::max<int64_t>(step, (int64_t)(fold_rows() + step - 1) / step * step);
  const dim3 grid((unsigned)ceil_div(m, rpb), (unsigned)ceil_div(c, kFoldCh));
  hipStream_t s = as_stream(stream);
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_bn_relu_apply_stats<float>, grid, dim3(256), 0, s, (const float*)x, x_c_stride, m, c, pm, pq,
                       P, R, eps, mean, invstd, beta, (float*)y, y_c_off, y_c_stride, rpb);
  else
    hipLaunchKernelGGL(k_bn_relu_apply_stats<uint16_t>, grid, dim3(256), 0, s, (const uint16_t*)x, x_c_stride, m, c,
                       pm, pq, P, R, eps, mean, invstd, beta, (uint16_t*)y, y_c_off, y_c_stride, rpb);
  return check_launch("bn_relu_apply_stats");
}

JR_API int jr_bn_relu_apply_grouped(int dtype, int32_t members, const void* x, int32_t x_c_off, int32_t x_c_stride,
                                    int64_t x_member_stride, int64_t m, int32_t c, const float* mean,
                                    const float* invstd, int64_t stats_member_stride, const float* beta,
                                    int64_t beta_member_stride, void* y, int32_t y_c_off, int32_t y_c_stride,
                                    int64_t y_member_stride, void* stream) {
  int rc = check_common(dtype, m, c);
  if (rc) return rc;
  if (members < 1 || members > 65535) return fail(JR_ERR_INVALID, "bn_relu_apply_grouped: members must be 1..65535");
  if (!x || !mean || !invstd || !beta || !y) return fail(JR_ERR_INVALID, "bn_relu_apply_grouped: null pointer");
  if (x_member_stride < 0 || y_member_stride < 0 || stats_member_stride < 0 || beta_member_stride < 0)
    return fail(JR_ERR_INVALID, "bn_relu_apply_grouped: negative member stride");
  if (!check_slice(dtype, x_c_off, x_c_stride, c) || !check_slice(dtype, y_c_off, y_c_stride, c))
    return fail(JR_ERR_INVALID, "bn_relu_apply_grouped: bad input / output slice");
  const size_t esz = dtype == JR_BF16 ? 2 : 4;
  if (((x_member_stride * esz) | (y_member_stride * esz)) & 15)
    return fail(JR_ERR_INVALID, "bn_relu_apply_grouped: member strides must be 16-byte multiples");
  x = static_cast<const char*>(x) + (size_t)x_c_off * esz;
  return bn_apply_launch(dtype, members, x, x_c_stride, x_member_stride * esz, m, c, mean, invstd,
                         stats_member_stride * 4, beta, beta_member_stride * 4, y, y_c_off, y_c_stride,
                         y_member_stride * esz, as_stream(stream));
}

// The apply pass of the backward (k1, k2 from a finalize).
static int bn_bwd_apply_launch(int dtype, const BnSegs& sg, const void* x, int32_t x_c_stride, int64_t m, int32_t c,
                               const float* mean, const float* invstd, const float* k1, const float* k2, void* dx,
                               hipStream_t s) {
  const int grid = apply_grid(m, c, vec_width(dtype));
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_bn_relu_bwd_apply<float>, dim3(grid), dim3(256), 0, s, sg, (const float*)x, x_c_stride, m,
                       c, mean, invstd, k1, k2, (float*)dx);
  else
    hipLaunchKernelGGL(k_bn_relu_bwd_apply<uint16_t>, dim3(grid), dim3(256), 0, s, sg, (const uint16_t*)x,
                       x_c_stride, m, c, mean, invstd, k1, k2, (uint16_t*)dx);
  return check_launch("bn_bwd apply");
}

// The three backward launches over segments (validated by the callers).
static int bn_bwd_launch(int dtype, const BnSegs& sg, const void* x, int32_t x_c_stride, int64_t m, int32_t c,
                         const float* mean, const float* invstd, void* dx, void* ws, size_t ws_bytes,
                         hipStream_t s) {
  if (!ws || ws_bytes < ws_need(m, c)) return fail(JR_ERR_WORKSPACE, "bn_relu_bwd: workspace too small");
  const int vw = vec_width(dtype);
  const ChunkGeom g = chunk_geom(m, c, vw);
  double* part = static_cast<double*>(ws);
  float* k1 = reinterpret_cast<float*>(part + (size_t)g.nchunks * 2 * c);
  float* k2 = k1 + c;
  if (dtype == JR_F32)
    hipLaunchKernelGGL((k_bn_reduce<1, float>), dim3(g.nchunks), dim3(256), 0, s, (const float*)x, x_c_stride, sg,
                       m, c, g.rows_per_chunk, mean, invstd, part);
  else
    hipLaunchKernelGGL((k_bn_reduce<1, uint16_t>), dim3(g.nchunks), dim3(256), 0, s, (const uint16_t*)x,
                       x_c_stride, sg, m, c, g.rows_per_chunk, mean, invstd, part);
  int rc = check_launch("bn_bwd reduce");
  if (rc) return rc;
  if (g.nchunks <= kFoldMaxP) {
    if (fold_bwd() && !sg.absmax) {   // the finalize inside the apply: one kernel boundary fewer
      const int vw = vec_width(dtype);
      const int step = 256 / (kFoldCh / vw) * kAppUnroll;
      const int rpb = (int)std::max<int64_t>(step, (int64_t)(fold_rows() + step - 1) / step * step);
      const dim3 grid((unsigned)ceil_div(m, rpb), (unsigned)ceil_div(c, kFoldCh));
      if (dtype == JR_F32)
        hipLaunchKernelGGL(k_bn_relu_bwd_apply_fold<float>, grid, dim3(256), 0, s, sg, (const float*)x, x_c_stride, m,
                           c, mean, invstd, (const double*)part, g.nchunks, (float*)dx, rpb);
      else
        hipLaunchKernelGGL(k_bn_relu_bwd_apply_fold<uint16_t>, grid, dim3(256), 0, s, sg, (const uint16_t*)x,
                           x_c_stride, m, c, mean, invstd, (const double*)part, g.nchunks, (uint16_t*)dx, rpb);
      return check_launch("bn_bwd apply (fold)");
    }
    hipLaunchKernelGGL(k_bn_finalize8, dim3((int)ceil_div(c, kFoldCh)), dim3(256), 0, s, (const double*)part,
                       g.nchunks, c, m, k1, k2, sg);
  } else {
    hipLaunchKernelGGL((k_bn_finalize<1>), dim3((int)ceil_div(c, 4)), dim3(256), 0, s, part, g.nchunks, c, m, 0.f,
                       k1, k2, sg);
  }
  rc = check_launch("bn_bwd finalize");
  if (rc) return rc;
  return bn_bwd_apply_launch(dtype, sg, x, x_c_stride, m, c, mean, invstd, k1, k2, dx, s);
}

JR_API int jr_bn_relu_bwd(int dtype, const void* dy, int32_t dy_c_off, int32_t dy_c_stride, const void* x,
                          int32_t x_c_off, int32_t x_c_stride, int64_t m, int32_t c, const float* mean,
                          const float* invstd, const float* beta, void* dx, float* dbeta, void* ws, size_t ws_bytes,
                          void* stream) {
  jr_bn_seg seg{dy, dy_c_off, dy_c_stride, c, beta, dbeta};
  return jr_bn_relu_bwd_multi(dtype, 1, &seg, x, x_c_off, x_c_stride, m, c, mean, invstd, dx, ws, ws_bytes, stream);
}

// Validates the segments and slices of a backward launch set; on success
// fills sg and moves x / dx to the slice's first channel.
static int bwd_setup(int dtype, int nseg, const jr_bn_seg* segs, const void*& x, int32_t x_c_off, int32_t x_c_stride,
                     int64_t m, int32_t c, const float* mean, const float* invstd, void*& dx, BnSegs& sg) {
  int rc = check_common(dtype, m, c);
  if (rc) return rc;
  if (!segs || nseg < 1 || nseg > kMaxSegs) return fail(JR_ERR_INVALID, "bn_relu_bwd: 1..4 segments");
  if (!x || !mean || !invstd || !dx) return fail(JR_ERR_INVALID, "bn_relu_bwd: null pointer");
  if (!check_slice(dtype, x_c_off, x_c_stride, c)) return fail(JR_ERR_INVALID, "bn_relu_bwd: bad x / dx slice");
  const size_t esz = dtype == JR_BF16 ? 2 : 4;
  sg = BnSegs{};
  sg.n = nseg;
  int c0 = 0;
  for (int i = 0; i < nseg; ++i) {
    const jr_bn_seg& e = segs[i];
    if (!e.dy || !e.beta || !e.dbeta) return fail(JR_ERR_INVALID, "bn_relu_bwd: null pointer in a segment");
    if (e.c <= 0 || e.c % vec_width(dtype) != 0)
      return fail(JR_ERR_INVALID, "bn_relu_bwd: segment channels must be a positive multiple of 4 (fp32) / 8 (bf16)");
    if (!check_slice(dtype, e.dy_c_off, e.dy_c_stride, e.c)) return fail(JR_ERR_INVALID, "bn_relu_bwd: bad dy slice");
    sg.dy[i] = e.dy;
    sg.dy_off[i] = e.dy_c_off;
    sg.dy_stride[i] = e.dy_c_stride;
    sg.beta[i] = e.beta;
    sg.dbeta[i] = e.dbeta;
    sg.c0[i] = c0;
    c0 += e.c;
  }
  if (c0 != c) return fail(JR_ERR_INVALID, "bn_relu_bwd: segment channels must sum to c");
  sg.c0[nseg] = c;
  x = static_cast<const char*>(x) + (size_t)x_c_off * esz;
  dx = static_cast<char*>(dx) + (size_t)x_c_off * esz;
  return JR_OK;
}

JR_API int jr_bn_relu_bwd_multi(int dtype, int nseg, const jr_bn_seg* segs, const void* x, int32_t x_c_off,
                                int32_t x_c_stride, int64_t m, int32_t c, const float* mean, const float* invstd,
                                void* dx, void* ws, size_t ws_bytes, void* stream) {
  return jr_bn_relu_bwd_multi_absmax(dtype, nseg, segs, x, x_c_off, x_c_stride, m, c, mean, invstd, dx, ws, ws_bytes,
                                     nullptr, stream);
}

JR_API int jr_bn_relu_bwd_multi_absmax(int dtype, int nseg, const jr_bn_seg* segs, const void* x, int32_t x_c_off,
                                       int32_t x_c_stride, int64_t m, int32_t c, const float* mean,
                                       const float* invstd, void* dx, void* ws, size_t ws_bytes, float* dx_absmax,
                                       void* stream) {
  BnSegs sg;
  const int rc = bwd_setup(dtype, nseg, segs, x, x_c_off, x_c_stride, m, c, mean, invstd, dx, sg);
  if (rc) return rc;
  sg.absmax = dx_absmax;
  return bn_bwd_launch(dtype, sg, x, x_c_stride, m, c, mean, invstd, dx, ws, ws_bytes, as_stream(stream));
}

// workspace of a batched backward: each layer's ws_need, 256-byte aligned
static size_t batch_ws(int n, const jr_bn_bwd_layer* layers) {
  size_t off = 0;
  for (int l = 0; l < n; ++l) off += (ws_need(layers[l].m, layers[l].c) + 255) / 256 * 256;
  return off;
}

JR_API size_t jr_bn_relu_bwd_batch_workspace_size(int32_t n, const jr_bn_bwd_layer* layers) {
  if (n < 1 || n > kBnBatchMax || !layers) return 0;
  return batch_ws(n, layers);
}

JR_API int jr_bn_relu_bwd_batch(int dtype, int32_t n, const jr_bn_bwd_layer* layers, void* ws, size_t ws_bytes,
                                void* stream) {
  if (n < 1 || n > kBnBatchMax || !layers) return fail(JR_ERR_INVALID, "bn_relu_bwd_batch: 1..8 layers");
  if (!ws || ws_bytes < batch_ws(n, layers)) return fail(JR_ERR_WORKSPACE, "bn_relu_bwd_batch: workspace too small");
  const int vw = vec_width(dtype);
  BnBatch bt{};
  bt.n = n;
  int blocks[3] = {0, 0, 0};
  size_t off = 0;
  for (int l = 0; l < n; ++l) {
    const jr_bn_bwd_layer& e = layers[l];
    BnBatchLayer& L = bt.L[l];
    const void* x = e.x;
    void* dx = e.dx;
    const int rc = bwd_setup(dtype, e.nseg, e.segs, x, e.x_c_off, e.x_c_stride, e.m, e.c, e.mean, e.invstd, dx, L.sg);
    if (rc) return rc;
    const ChunkGeom g = chunk_geom(e.m, e.c, vw);
    if (g.nchunks > kFoldMaxP)
      return fail(JR_ERR_UNSUPPORTED, "bn_relu_bwd_batch: a layer with more than 512 reduce chunks (use jr_bn_relu_bwd_multi)");
    L.x = x;
    L.dx = dx;
    L.mean = e.mean;
    L.invstd = e.invstd;
    L.part = reinterpret_cast<double*>(static_cast<char*>(ws) + off);
    L.k1 = reinterpret_cast<float*>(L.part + (size_t)g.nchunks * 2 * e.c);
    L.k2 = L.k1 + e.c;
    L.m = e.m;
    L.c = e.c;
    L.xs = e.x_c_stride;
    L.rpc = g.rows_per_chunk;
    L.nchunks = g.nchunks;
    L.b0[0] = blocks[0];
    L.b0[1] = blocks[1];
    L.b0[2] = blocks[2];
    blocks[0] += g.nchunks;
    blocks[1] += (int)ceil_div(e.c, kFoldCh);
    blocks[2] += apply_grid(e.m, e.c, vw);
    off += (ws_need(e.m, e.c) + 255) / 256 * 256;
  }
  hipStream_t s = as_stream(stream);
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_bn_reduce_batch<float>, dim3(blocks[0]), dim3(256), 0, s, bt);
  else
    hipLaunchKernelGGL(k_bn_reduce_batch<uint16_t>, dim3(blocks[0]), dim3(256), 0, s, bt);
  int rc = check_launch("bn_bwd batch reduce");
  if (rc) return rc;
  hipLaunchKernelGGL(k_bn_finalize8_batch, dim3(blocks[1]), dim3(256), 0, s, bt);
  rc = check_launch("bn_bwd batch finalize");
  if (rc) return rc;
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_bn_relu_bwd_apply_batch<float>, dim3(blocks[2]), dim3(256), 0, s, bt);
  else
    hipLaunchKernelGGL(k_bn_relu_bwd_apply_batch<uint16_t>, dim3(blocks[2]), dim3(256), 0, s, bt);
  return check_launch("bn_bwd batch apply");
}

// ---------------------------------------------------------------------------
// The backward of a conv2d_bn layer whose output only a 3x3/2 max-pool reads
// (the stem's conv2d_3 / conv2d_5; forward: jr_bn_relu_maxpool3x3s2_fwd).
// k_maxpool_bwd_bn routes the pooled gradient to the layer's output exactly
// as k_maxpool_bwd (2x2 input cells, windows summed from +0 in (oh, ow)
// order, stored in the path dtype) and, holding each dy in registers, adds
// the BN reduce's sums (sum dy', sum dy' xhat, fp64) of its channel quad
// over every cell it visits; one partial per block and channel ([2][c][grid],
// fixed order: deterministic) replaces k_bn_reduce's second read of dy.
// k_bn_finalize and k_bn_relu_bwd_apply then run as for any layer.
template <typename T>
__global__ void __launch_bounds__(256) k_maxpool_bwd_bn(jr_pool_desc d, const uint8_t* __restrict__ argmax,
                                                        const T* __restrict__ pdy, T* __restrict__ dy,
                                                        const T* __restrict__ x, int xs, const float* __restrict__ mean,
                                                        const float* __restrict__ invstd,
                                                        const float* __restrict__ beta, double* part) {
  __shared__ double red[256][8];
  const int c4 = d.c >> 2;
  const int hc = (d.h + 1) >> 1, wc = (d.w + 1) >> 1;
  const int total = d.n * hc * wc * c4;
  const int stride = gridDim.x * blockDim.x;
  const int q = (blockIdx.x * blockDim.x + threadIdx.x) % c4;   // fixed per thread: blockDim.x % c4 == 0
  float mu[4], is[4], be[4];
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    mu[l] = mean[q * 4 + l];
    is[l] = invstd[q * 4 + l];
    be[l] = beta[q * 4 + l];
  }
  double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
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
        am[i][j] = 0xffffffffu;
        g[i][j] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (oh >= 0 && oh < d.ho && ow >= 0 && ow < d.wo) {
          const int64_t op = ((int64_t)b * d.ho + oh) * d.wo + ow;
          am[i][j] = *reinterpret_cast<const uint32_t*>(argmax + op * d.c + q * 4);
          float v[4];
          if constexpr (sizeof(T) == 4) {
            const float4 f = *reinterpret_cast<const float4*>(pdy + op * d.y_c_stride + d.y_c_off + q * 4);
            v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
          } else {
            const uint2 u = *reinterpret_cast<const uint2*>(pdy + op * d.y_c_stride + d.y_c_off + q * 4);
            v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
            v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
          }
          g[i][j] = make_float4(v[0], v[1], v[2], v[3]);
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
            const int r = u + 2 - 2 * i, c = v + 2 - 2 * j;
            if (r > 2 || c > 2) continue;
            const float ga[4] = {g[i][j].x, g[i][j].y, g[i][j].z, g[i][j].w};
#pragma unroll
            for (int l = 0; l < 4; ++l)
              if ((int)((am[i][j] >> (8 * l)) & 0xff) == r * 3 + c) acc[l] += ga[l];
          }
        }
        const int64_t pix = ((int64_t)b * d.h + ih) * d.w + iw;
        float xv[4];
        T* p = dy + pix * d.x_c_stride + d.x_c_off + q * 4;
        if constexpr (sizeof(T) == 4) {
          *reinterpret_cast<float4*>(p) = make_float4(acc[0], acc[1], acc[2], acc[3]);
          const float4 f = *reinterpret_cast<const float4*>(x + pix * xs + q * 4);
          xv[0] = f.x; xv[1] = f.y; xv[2] = f.z; xv[3] = f.w;
        } else {
          uint2 w;
          w.x = (uint32_t)f2bf(acc[0]) | ((uint32_t)f2bf(acc[1]) << 16);
          w.y = (uint32_t)f2bf(acc[2]) | ((uint32_t)f2bf(acc[3]) << 16);
          *reinterpret_cast<uint2*>(p) = w;
#pragma unroll
          for (int l = 0; l < 4; ++l) acc[l] = bf2f(f2bf(acc[l]));   // the value k_bn_reduce would read
          const uint2 xr = *reinterpret_cast<const uint2*>(x + pix * xs + q * 4);
          xv[0] = __uint_as_float(xr.x << 16); xv[1] = __uint_as_float(xr.x & 0xffff0000u);
          xv[2] = __uint_as_float(xr.y << 16); xv[3] = __uint_as_float(xr.y & 0xffff0000u);
        }
#pragma unroll
        for (int l = 0; l < 4; ++l) {
          const float xh = bn_xhat(xv[l], mu[l], is[l]);
          const float g2 = __fadd_rn(xh, be[l]) > 0.f ? acc[l] : 0.f;
          s0[l] += (double)g2;
          s1[l] += (double)g2 * (double)xh;
        }
      }
    }
  }
  const int t = threadIdx.x;
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    red[t][l] = s0[l];
    red[t][4 + l] = s1[l];
  }
  __syncthreads();
  // threads t, t + c4, t + 2 c4, ... hold the same channel quad: fixed-order sum
  if (t < c4) {
    double a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = red[t][k];
    for (int o = t + c4; o < (int)blockDim.x; o += c4)
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] += red[o][k];
    const int64_t nch = gridDim.x;
    const int qq = (blockIdx.x * blockDim.x + t) % c4;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      part[(int64_t)(qq * 4 + l) * nch + blockIdx.x] = a[l];
      part[(int64_t)(d.c + qq * 4 + l) * nch + blockIdx.x] = a[4 + l];
    }
  }
}

JR_API size_t jr_bn_relu_bwd_maxpool_workspace_size(const jr_pool_desc* d) {
  if (!d || d->c <= 0) return 0;
  return (size_t)4096 * 2 * d->c * sizeof(double) + 2 * (size_t)d->c * sizeof(float);
}

JR_API int jr_bn_relu_bwd_maxpool(int dtype, const jr_pool_desc* d, const uint8_t* argmax, const void* pooled_dy,
                                  void* dy, const void* x, int32_t x_c_stride, const float* mean,
                                  const float* invstd, const float* beta, void* dx, float* dbeta, void* ws,
                                  size_t ws_bytes, void* stream) {
  return jr_bn_relu_bwd_maxpool_absmax(dtype, d, argmax, pooled_dy, dy, x, x_c_stride, mean, invstd, beta, dx, dbeta,
                                       ws, ws_bytes, nullptr, stream);
}

JR_API int jr_bn_relu_bwd_maxpool_absmax(int dtype, const jr_pool_desc* d, const uint8_t* argmax,
                                         const void* pooled_dy, void* dy, const void* x, int32_t x_c_stride,
                                         const float* mean, const float* invstd, const float* beta, void* dx,
                                         float* dbeta, void* ws, size_t ws_bytes, float* dx_absmax, void* stream) {
  if (!d || !argmax || !pooled_dy || !dy || !x || !mean || !invstd || !beta || !dx || !dbeta)
    return fail(JR_ERR_INVALID, "bn_relu_bwd_maxpool: null pointer");
  const int32_t c = d->c;
  const int64_t m = (int64_t)d->n * d->h * d->w;
  int rc = check_common(dtype, m, c);
  if (rc) return rc;
  if (c % 4 || c / 4 > 256) return fail(JR_ERR_UNSUPPORTED, "bn_relu_bwd_maxpool: c must be a multiple of 4, <= 1024");
  if (d->h < 3 || d->w < 3 || d->ho != (d->h - 3) / 2 + 1 || d->wo != (d->w - 3) / 2 + 1)
    return fail(JR_ERR_INVALID, "bn_relu_bwd_maxpool: the pool must be 3x3 stride 2 valid");
  if (!check_slice(dtype, d->y_c_off, d->y_c_stride, c) || !check_slice(dtype, d->x_c_off, d->x_c_stride, c) ||
      !check_slice(dtype, 0, x_c_stride, c))
    return fail(JR_ERR_INVALID, "bn_relu_bwd_maxpool: bad slice");
  if (!ws || ws_bytes < jr_bn_relu_bwd_maxpool_workspace_size(d))
    return fail(JR_ERR_WORKSPACE, "bn_relu_bwd_maxpool: workspace too small");
  hipStream_t s = as_stream(stream);
  const int64_t cells = (int64_t)d->n * ((d->h + 1) / 2) * ((d->w + 1) / 2) * (c / 4);
  const int bs = 256 / (c / 4) * (c / 4);        // a whole number of channel-quad rows per block
  const int grid = (int)std::min<int64_t>(std::max<int64_t>(ceil_div(cells, bs), 1), 4096);
  double* part = static_cast<double*>(ws);
  float* k1 = reinterpret_cast<float*>(part + (size_t)grid * 2 * c);
  float* k2 = k1 + c;
  if (dtype == JR_F32)
    hipLaunchKernelGGL(k_maxpool_bwd_bn<float>, dim3(grid), dim3(bs), 0, s, *d, argmax, (const float*)pooled_dy,
                       (float*)dy, (const float*)x, x_c_stride, mean, invstd, beta, part);
  else
    hipLaunchKernelGGL(k_maxpool_bwd_bn<uint16_t>, dim3(grid), dim3(bs), 0, s, *d, argmax,
                       (const uint16_t*)pooled_dy, (uint16_t*)dy, (const uint16_t*)x, x_c_stride, mean, invstd, beta,
                       part);
  rc = check_launch("maxpool_bwd + bn reduce");
  if (rc) return rc;
  BnSegs sg{};
  sg.n = 1;
  sg.dy[0] = static_cast<const char*>(dy) + (size_t)d->x_c_off * (dtype == JR_BF16 ? 2 : 4);
  sg.dy_off[0] = 0;
  sg.dy_stride[0] = d->x_c_stride;
  sg.beta[0] = beta;
  sg.dbeta[0] = dbeta;
  sg.c0[0] = 0;
  sg.c0[1] = c;
  sg.absmax = dx_absmax;
  hipLaunchKernelGGL((k_bn_finalize<1>), dim3((int)ceil_div(c, 4)), dim3(256), 0, s, part, grid, c, m, 0.f, k1, k2,
                     sg);
  rc = check_launch("bn_bwd finalize");
  if (rc) return rc;
  return bn_bwd_apply_launch(dtype, sg, x, x_c_stride, m, c, mean, invstd, k1, k2, dx, s);
}
