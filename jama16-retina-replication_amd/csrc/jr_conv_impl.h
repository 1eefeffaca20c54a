// jr_conv_impl.h — pieces shared by the fp32 (jr_conv.hip) and bf16
// (jr_conv_bf16.hip) implicit-GEMM convolution kernels: GEMM arguments,
// output addressing, counted waits, LDS-DMA, the split-K reduce, and the
// tile-configuration tables the host planner ranks and autotunes.
#pragma once
#include "jr_common.h"

namespace jr {

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { OP_FWD = 0, OP_DGRAD = 1, OP_WGRAD = 2 };

// 64 B of zeros in global memory: the DMA source of out-of-bounds taps.
static __device__ __attribute__((aligned(64))) float g_zero_page[16];

struct ConvArgs {
  const float* A;
  const float* B;
  float* C;
  int M, N, K;                // GEMM dims (DGRAD: of this phase)
  int n, h, w, cin, cp, cout, kh, kw, sh, sw, ph, pw, ho, wo;
  int xo, xs, yo, ys;         // channel slices of x and of dy
  int c_off, c_stride;        // output addressing
  int accumulate;
  int ktiles, kt_per_split, ntn;
  long long slab_elems;       // M*N (split-K slabs)
  // DGRAD phase (py,px): taps r = r0 + sh*a (a < na), c = c0 + sw*b (b < nb);
  // m = (b, u, v) over hc x wc; ih = sh*u + py; oh = u + ey - a.
  int py, px, r0, c0, na, nb, ey, ex, hc, wc;
};

// Output element offset of GEMM row m (column 0), or -1 to drop the row.
template <int OP>
__device__ __forceinline__ long long out_row(const ConvArgs& g, int m) {
  if constexpr (OP == OP_FWD) {
    return (long long)m * g.c_stride + g.c_off;
  } else if constexpr (OP == OP_DGRAD) {
    const int hw = g.hc * g.wc;
    const int b = m / hw, rem = m - b * hw;
    const int u = rem / g.wc, v = rem - u * g.wc;
    const long long pix = ((long long)b * g.h + g.sh * u + g.py) * g.w + g.sw * v + g.px;
    return pix * g.c_stride + g.c_off;
  } else {
    if (g.cp == g.cin) return (long long)m * g.N;
    const int rc = m / g.cp, ci = m - rc * g.cp;
    if (ci >= g.cin) return -1;
    return ((long long)rc * g.cin + ci) * g.N;
  }
}

// s_waitcnt vmcnt(n) + lgkmcnt(0) for a wave-uniform runtime n (immediate
// operand: switch over the values a K-tile pipeline can need).
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7) lgkmcnt(0)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9) lgkmcnt(0)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10) lgkmcnt(0)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11) lgkmcnt(0)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); break;
  }
}

// Advance the mixed-radix counter (z, y, x) (radices ly, lx) by BK along x.
// multi (wave-uniform) = lx < BK: more than one carry is possible.
template <int BK>
__device__ __forceinline__ void adv_mixed_t(int& x, int& y, int& z, int lx, int ly, bool multi) {
  x += BK;
  if (!multi) {
    const bool c1 = x >= lx;
    x = c1 ? x - lx : x;
    y += c1 ? 1 : 0;
    const bool c2 = y == ly;
    y = c2 ? 0 : y;
    z += c2 ? 1 : 0;
  } else {
    while (x >= lx) {
      x -= lx;
      if (++y == ly) { y = 0; ++z; }
    }
  }
}
#define adv_mixed(x, y, z, lx, ly, multi) adv_mixed_t<BK>(x, y, z, lx, ly, multi)

__device__ __forceinline__ void dma16(const void* src, void* lds_chunk) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_chunk, 16, 0, 0);
}

// out[out_row(m) + n] (+)= sum_z slab[z][m][n], float4 along n (N % 16 == 0
// and channel offsets/strides % 4 == 0 keep every access 16-byte aligned);
// TO = float, or uint16_t (bf16 output, summed in f32 and rounded once).
// Block = G z-lanes x (256 / G) float4 columns: z-lane zg sums slabs zg,
// zg + G, ... and the G lane sums are added in zg order through LDS, so the
// result depends only on (M, N, splits), never on timing.  G grows when
// M*N is small and splits large (the wgrad case: a few thousand outputs, up
// to 256 slabs) so the reduce still spreads over the whole chip.
template <int OP, typename TO>
__global__ void __launch_bounds__(256) k_splitk_reduce(const float* __restrict__ slab, int splits, int G,
                                                       ConvArgs g, TO* out) {
  __shared__ float4 part[256];
  const int cols = 256 / G;
  const int t = threadIdx.x;
  const int zg = t / cols, cl = t - zg * cols;
  const int n4 = g.N >> 2;
  const long long total = (long long)g.M * n4;
  const long long zs = g.slab_elems >> 2;
  for (long long e0 = (long long)blockIdx.x * cols; e0 < total; e0 += (long long)gridDim.x * cols) {
    const long long e = e0 + cl;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < total) {
      const float4* src = reinterpret_cast<const float4*>(slab) + e;
      int z = zg;
      for (; z + 3 * G < splits; z += 4 * G) {
        const float4 a = src[z * zs], b = src[(z + G) * zs], c = src[(z + 2 * G) * zs], d = src[(z + 3 * G) * zs];
        s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
        s.x += b.x; s.y += b.y; s.z += b.z; s.w += b.w;
        s.x += c.x; s.y += c.y; s.z += c.z; s.w += c.w;
        s.x += d.x; s.y += d.y; s.z += d.z; s.w += d.w;
      }
      for (; z < splits; z += G) {
        const float4 a = src[z * zs];
        s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
      }
    }
    if (G > 1) {
      part[t] = s;
      __syncthreads();
      if (zg == 0) {
        for (int k = 1; k < G; ++k) {
          const float4 a = part[k * cols + cl];
          s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
        }
      }
      __syncthreads();
    }
    if (zg != 0 || e >= total) continue;
    const int m = (int)(e / n4), q = (int)(e - (long long)m * n4);
    const long long base = out_row<OP>(g, m);
    if (base < 0) continue;
    TO* p = out + base + q * 4;
    if constexpr (sizeof(TO) == 4) {
      float4* p4 = reinterpret_cast<float4*>(p);
      if (g.accumulate) {
        const float4 o = *p4;
        s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
      }
      *p4 = s;
    } else {   // bf16 output: accumulate in f32, round once
      uint2* p2 = reinterpret_cast<uint2*>(p);
      if (g.accumulate) {
        const uint2 o = *p2;
        s.x += bf2f(o.x & 0xffff); s.y += bf2f(o.x >> 16); s.z += bf2f(o.y & 0xffff); s.w += bf2f(o.y >> 16);
      }
      *p2 = make_uint2((uint32_t)f2bf(s.x) | ((uint32_t)f2bf(s.y) << 16),
                       (uint32_t)f2bf(s.z) | ((uint32_t)f2bf(s.w) << 16));
    }
  }
}

struct TileCfg {
  int bm, bn, wgm, bk, nbuf;
  double eff;  // relative MFMA efficiency guess used to rank padded work
};

// Candidate tiles (block BMxBN, WGM waves along M, K-tile BK).  The planner
// ranks them by padded work / eff; jr_conv2d_autotune times them instead.
// Keep in sync with launch_op's switch.
static constexpr TileCfg kCfgs[] = {
    {128, 128, 2, 16, 3, 1.00},  // 0: wave 64x64, 48 KiB LDS
    {128, 128, 2, 32, 2, 1.00},  // 1: 64 KiB
    {256, 64, 4, 16, 3, 1.00},   // 2: wave 64x64, 60 KiB
    {128, 64, 2, 16, 4, 0.92},   // 3: wave 64x32, 48 KiB
    {128, 64, 2, 32, 2, 0.92},   // 4: 48 KiB
    {128, 96, 4, 16, 3, 0.90},   // 5: wave 32x96, 42 KiB
    {256, 32, 4, 16, 4, 0.85},   // 6: wave 64x32, 72 KiB
    {64, 64, 2, 32, 3, 0.75},    // 7: wave 32x32, 48 KiB
    {128, 32, 4, 32, 3, 0.75},   // 8: wave 32x32, 60 KiB
    {64, 128, 2, 32, 2, 0.80},   // 9: wave 32x64, 48 KiB
    {128, 64, 2, 16, 2, 0.90},   // 10: wave 64x32, 24 KiB
    {128, 192, 2, 16, 3, 1.02},  // 11: wave 64x96, 60 KiB (N = 192 layers)
    {256, 96, 4, 16, 3, 1.02},   // 12: wave 64x96, 66 KiB (N = 96 layers)
    {256, 128, 2, 16, 3, 1.04},  // 13: wave 128x64, 72 KiB
};
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);

// bf16 tiles (BK in bf16 elements; MFMA v_mfma_f32_32x32x16_bf16).
static constexpr TileCfg kCfgsBf16[] = {
    {128, 128, 2, 32, 3, 1.00},  // 0: wave 64x64, 48 KiB LDS
    {128, 128, 2, 64, 2, 1.00},  // 1: 64 KiB
    {256, 128, 2, 32, 3, 1.05},  // 2: wave 128x64, 72 KiB
    {128, 64, 2, 32, 3, 0.92},   // 3: wave 64x32, 36 KiB
    {256, 64, 4, 32, 3, 1.00},   // 4: wave 64x64, 60 KiB
    {128, 192, 2, 32, 3, 1.02},  // 5: wave 64x96, 60 KiB
    {128, 96, 4, 32, 3, 0.90},   // 6: wave 32x96, 42 KiB
    {64, 64, 2, 64, 3, 0.75},    // 7: wave 32x32, 48 KiB
};
constexpr int kNumCfgsBf16 = sizeof(kCfgsBf16) / sizeof(kCfgsBf16[0]);

// bf16 GEMM launch (jr_conv_bf16.hip): tile index into kCfgsBf16, fast =
// the uniform-tap / single-carry kernel variant.
void launch_conv_bf16(int op, int tile, bool fast, const ConvArgs& a, dim3 grid, hipStream_t s);

}  // namespace jr
