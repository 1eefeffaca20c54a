// jr_conv.hip — Conv2D forward / data-grad / filter-grad as implicit GEMM on
// gfx950 MFMA (fp32: v_mfma_f32_32x32x2_f32, exact f32 at the f32 peak rate).
//
// Replaces the TF ops behind the 94 Keras Conv2D(use_bias=False) layers that
// train.py:129-130 instantiates, and their gradients created by .minimize at
// train.py:150-153 (Conv2DBackpropInput / Conv2DBackpropFilter).
//
// One GEMM  C[M][N] = sum_k A[m][k] * B[k][n]  per op, activations NHWC,
// kernels HWIO:
//   FWD    m = output pixel (b,ho,wo)  n = co  k = (r,c,ci)   A = x gather,  B = W
//   DGRAD  m = input pixel  (b,h,w)    n = ci  k = (r,c,co)   A = dy gather, B = W^T(ci,co)
//   WGRAD  m = (r,c,ci)                n = co  k = pixel      A = x gather^T, B = dy
// Tiles are staged through LDS in a k-major image ([BK][BM], [BK][BN]) so
// every MFMA operand is one conflict-free ds_read_b32 per lane; k-contiguous
// global operands are transposed on the LDS write (row pad 2 floats makes the
// transposed ds_write_b32 conflict-free), m/n-contiguous ones are written
// with ds_write_b128.  Register-staged double buffering: the next tile's
// global loads are issued before the current tile's MFMAs, written to the
// other LDS buffer after them, one barrier per K-tile.
// Split-K (grid.z) writes fp32 slabs reduced in a fixed order by a second
// kernel, so results are bitwise reproducible (no float atomics).
#include "jr_common.h"

namespace jr {

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { OP_FWD = 0, OP_DGRAD = 1, OP_WGRAD = 2 };

struct ConvArgs {
  const float* A;
  const float* B;
  float* C;
  int M, N, K;
  int n, h, w, cin, cout, kh, kw, sh, sw, ph, pw, ho, wo;
  int xo, xs, yo, ys;     // channel slices of x and of dy/y
  int c_off, c_stride;    // output addressing: C[m*c_stride + c_off + n]
  int accumulate;
  int ktiles;             // total K tiles
  int kt_per_split;
  int ntn;                // number of N tiles
  long long slab_elems;   // M*N (split-K slabs)
};

template <int OP, int BM, int BN, int WM, int WN, bool SCALAR>
__global__ void __launch_bounds__(256) k_conv_f32(ConvArgs g) {
  constexpr int BK = 16;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int WGN = BN / WN;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves per block");
  constexpr bool A_TRANS = (OP != OP_WGRAD) && !SCALAR;  // k-contiguous A
  constexpr bool B_TRANS = (OP == OP_DGRAD);             // k-contiguous B
  constexpr int LDA = BM + (A_TRANS ? 2 : 0);
  constexpr int LDB = BN + (B_TRANS ? 2 : 0);
  constexpr int ASZ = BK * LDA, BSZ = BK * LDB;
  __shared__ __attribute__((aligned(16))) float smem[2 * (ASZ + BSZ)];
  float* As0 = smem;
  float* Bs0 = smem + 2 * ASZ;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm0 = (wave / WGN) * WM;
  const int wn0 = (wave % WGN) * WN;

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = tile / g.ntn, nt = tile - mt * g.ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int kt0 = blockIdx.z * g.kt_per_split;
  const int kt1 = min(g.ktiles, kt0 + g.kt_per_split);

  // ------------------------------------------------------------------ A state
  // A_TRANS: BM/64 float4 per thread, (kq = idx&3, row = idx>>2)
  // WGRAD vector: BM/64 float4 per thread, (m4 = idx % (BM/4), kk = idx / (BM/4))
  // SCALAR: BM*BK/256 scalars per thread, (row = idx % BM, kk = idx / BM)
  constexpr int NA = SCALAR ? (BM * BK / 256) : (BM / 64);
  int a_p0[NA], a_p1[NA], a_base[NA];  // per-row precomputed geometry
  int a_kk[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int idx = tid + i * 256;
    if constexpr (SCALAR) {
      const int row = idx % BM;
      a_kk[i] = idx / BM;
      const int m = m0 + row;
      if constexpr (OP == OP_FWD) {
        if (m < g.M) {
          const int hw = g.ho * g.wo;
          const int b = m / hw, rem = m - b * hw;
          const int oh = rem / g.wo, ow = rem - oh * g.wo;
          a_p0[i] = oh * g.sh - g.ph;
          a_p1[i] = ow * g.sw - g.pw;
          a_base[i] = b * g.h * g.w;
        } else {
          a_p0[i] = -(1 << 28); a_p1[i] = 0; a_base[i] = 0;
        }
      } else {  // WGRAD scalar: m = (r,c,ci)
        if (m < g.M) {
          const int rc = m / g.cin, ci = m - rc * g.cin;
          const int r = rc / g.kw, c = rc - r * g.kw;
          a_p0[i] = r - g.ph; a_p1[i] = c - g.pw; a_base[i] = ci;
        } else {
          a_p0[i] = -(1 << 28); a_p1[i] = 0; a_base[i] = 0;
        }
      }
    } else if constexpr (A_TRANS) {
      const int row = idx >> 2;
      a_kk[i] = (idx & 3) * 4;
      const int m = m0 + row;
      if (m < g.M) {
        if constexpr (OP == OP_FWD) {
          const int hw = g.ho * g.wo;
          const int b = m / hw, rem = m - b * hw;
          const int oh = rem / g.wo, ow = rem - oh * g.wo;
          a_p0[i] = oh * g.sh - g.ph;
          a_p1[i] = ow * g.sw - g.pw;
          a_base[i] = b * g.h * g.w;
        } else {  // DGRAD: m = input pixel
          const int hw = g.h * g.w;
          const int b = m / hw, rem = m - b * hw;
          const int ih = rem / g.w, iw = rem - ih * g.w;
          a_p0[i] = ih + g.ph;
          a_p1[i] = iw + g.pw;
          a_base[i] = b * g.ho * g.wo;
        }
      } else {
        a_p0[i] = -(1 << 28); a_p1[i] = -(1 << 28); a_base[i] = 0;
      }
    } else {  // WGRAD vector: m4 fixed, kk fixed
      const int m4 = idx % (BM / 4);
      a_kk[i] = idx / (BM / 4);
      const int m = m0 + m4 * 4;
      if (m < g.M) {
        const int rc = m / g.cin, ci = m - rc * g.cin;
        const int r = rc / g.kw, c = rc - r * g.kw;
        a_p0[i] = r - g.ph; a_p1[i] = c - g.pw; a_base[i] = ci;
      } else {
        a_p0[i] = -(1 << 28); a_p1[i] = 0; a_base[i] = 0;
      }
    }
  }

  constexpr int NB_TOT = BK * BN / 4;            // float4 per B tile
  constexpr int NB = (NB_TOT + 255) / 256;

  float4 ra[SCALAR ? 1 : NA];
  float rs[SCALAR ? NA : 1];
  float4 rb[NB];

  auto load_tiles = [&](int kt) {
    const int k0 = kt * BK;
    // ---------------- A
    if constexpr (SCALAR) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int k = k0 + a_kk[i];
        float v = 0.f;
        if constexpr (OP == OP_FWD) {
          if (k < g.K) {
            const int rc = k / g.cin, ci = k - rc * g.cin;
            const int r = rc / g.kw, c = rc - r * g.kw;
            const int hi = a_p0[i] + r, wi = a_p1[i] + c;
            if ((unsigned)hi < (unsigned)g.h && (unsigned)wi < (unsigned)g.w)
              v = g.A[(long long)(a_base[i] + hi * g.w + wi) * g.xs + g.xo + ci];
          }
        } else {  // WGRAD scalar
          if (k < g.K) {
            const int hw = g.ho * g.wo;
            const int b = k / hw, rem = k - b * hw;
            const int oh = rem / g.wo, ow = rem - oh * g.wo;
            const int hi = oh * g.sh + a_p0[i], wi = ow * g.sw + a_p1[i];
            if ((unsigned)hi < (unsigned)g.h && (unsigned)wi < (unsigned)g.w)
              v = g.A[(long long)((b * g.h + hi) * g.w + wi) * g.xs + g.xo + a_base[i]];
          }
        }
        rs[i] = v;
      }
    } else if constexpr (A_TRANS) {
      const int cred = (OP == OP_FWD) ? g.cin : g.cout;
      const int rc = k0 / cred, ch0 = k0 - rc * cred;
      const int r = rc / g.kw, c = rc - r * g.kw;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (OP == OP_FWD) {
          const int hi = a_p0[i] + r, wi = a_p1[i] + c;
          if ((unsigned)hi < (unsigned)g.h && (unsigned)wi < (unsigned)g.w)
            v = *reinterpret_cast<const float4*>(
                g.A + (long long)(a_base[i] + hi * g.w + wi) * g.xs + g.xo + ch0 + a_kk[i]);
        } else {  // DGRAD
          const int hn = a_p0[i] - r, wn = a_p1[i] - c;
          bool ok;
          int oh, ow;
          if (g.sh == 1 && g.sw == 1) {
            oh = hn; ow = wn;
            ok = (unsigned)oh < (unsigned)g.ho && (unsigned)ow < (unsigned)g.wo;
          } else {
            ok = hn >= 0 && wn >= 0 && (hn % g.sh) == 0 && (wn % g.sw) == 0;
            oh = hn / g.sh; ow = wn / g.sw;
            ok = ok && oh < g.ho && ow < g.wo;
          }
          if (ok)
            v = *reinterpret_cast<const float4*>(
                g.A + (long long)(a_base[i] + oh * g.wo + ow) * g.ys + g.yo + ch0 + a_kk[i]);
        }
        ra[i] = v;
      }
    } else {  // WGRAD vector
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        const int k = k0 + a_kk[i];
        if (k < g.K) {
          const int hw = g.ho * g.wo;
          const int b = k / hw, rem = k - b * hw;
          const int oh = rem / g.wo, ow = rem - oh * g.wo;
          const int hi = oh * g.sh + a_p0[i], wi = ow * g.sw + a_p1[i];
          if ((unsigned)hi < (unsigned)g.h && (unsigned)wi < (unsigned)g.w)
            v = *reinterpret_cast<const float4*>(
                g.A + (long long)((b * g.h + hi) * g.w + wi) * g.xs + g.xo + a_base[i]);
        }
        ra[i] = v;
      }
    }
    // ---------------- B
    if constexpr (B_TRANS) {  // DGRAD: B[k=(r,c,co)][n=ci] = W[(rc*cin + ci)*cout + co]
      const int rc = k0 / g.cout, co0 = k0 - rc * g.cout;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int idx = tid + i * 256;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (idx < NB_TOT) {
          const int kq = idx & 3, col = idx >> 2;
          const int nn = n0 + col;
          if (nn < g.N)
            v = *reinterpret_cast<const float4*>(g.B + ((long long)rc * g.cin + nn) * g.cout + co0 + kq * 4);
        }
        rb[i] = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int idx = tid + i * 256;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (idx < NB_TOT) {
          const int n4 = idx % (BN / 4), kk = idx / (BN / 4);
          const int k = k0 + kk, nn = n0 + n4 * 4;
          if (k < g.K && nn < g.N) {
            if constexpr (OP == OP_FWD)
              v = *reinterpret_cast<const float4*>(g.B + (long long)k * g.N + nn);
            else  // WGRAD: dy rows
              v = *reinterpret_cast<const float4*>(g.B + (long long)k * g.ys + g.yo + nn);
          }
        }
        rb[i] = v;
      }
    }
  };

  auto store_tiles = [&](int buf) {
    float* As = As0 + buf * ASZ;
    float* Bs = Bs0 + buf * BSZ;
    if constexpr (SCALAR) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int idx = tid + i * 256;
        As[a_kk[i] * LDA + (idx % BM)] = rs[i];
      }
    } else if constexpr (A_TRANS) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int row = (tid + i * 256) >> 2;
        float* p = As + a_kk[i] * LDA + row;
        p[0] = ra[i].x; p[LDA] = ra[i].y; p[2 * LDA] = ra[i].z; p[3 * LDA] = ra[i].w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int idx = tid + i * 256;
        const int m4 = idx % (BM / 4);
        *reinterpret_cast<float4*>(As + a_kk[i] * LDA + m4 * 4) = ra[i];
      }
    }
    if constexpr (B_TRANS) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int idx = tid + i * 256;
        if (idx < NB_TOT) {
          const int kq = idx & 3, col = idx >> 2;
          float* p = Bs + kq * 4 * LDB + col;
          p[0] = rb[i].x; p[LDB] = rb[i].y; p[2 * LDB] = rb[i].z; p[3 * LDB] = rb[i].w;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int idx = tid + i * 256;
        if (idx < NB_TOT) {
          const int n4 = idx % (BN / 4), kk = idx / (BN / 4);
          *reinterpret_cast<float4*>(Bs + kk * LDB + n4 * 4) = rb[i];
        }
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (kt0 < kt1) {
    load_tiles(kt0);
    store_tiles(0);
    __syncthreads();
    const int l31 = lane & 31, lhi = lane >> 5;
    for (int kt = kt0; kt < kt1; ++kt) {
      const int cur = (kt - kt0) & 1;
      const bool more = kt + 1 < kt1;
      if (more) load_tiles(kt + 1);
      const float* As = As0 + cur * ASZ;
      const float* Bs = Bs0 + cur * BSZ;
#pragma unroll
      for (int ks = 0; ks < BK / 2; ++ks) {
        const int k = ks * 2 + lhi;
        float a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = As[k * LDA + wm0 + i * 32 + l31];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = Bs[k * LDB + wn0 + j * 32 + l31];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
      if (more) store_tiles(cur ^ 1);
      __syncthreads();
    }
  }

  // ---------------------------------------------------------------- epilogue
  const bool split = gridDim.z > 1;
  float* C = g.C;
  long long cs = g.c_stride, co = g.c_off;
  if (split) {
    C = g.C + (long long)blockIdx.z * g.slab_elems;
    cs = g.N; co = 0;
  }
  const int col = lane & 31;
  const int rbase = 4 * (lane >> 5);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn0 + j * 32 + col;
      if (n >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + rbase;
        if (m < g.M) {
          float* p = C + (long long)m * cs + co + n;
          if (!split && g.accumulate) *p += acc[i][j][r];
          else *p = acc[i][j][r];
        }
      }
    }
  }
}

// out[m*c_stride + c_off + n] (+)= sum_z slab[z][m][n]   (fixed order)
__global__ void k_splitk_reduce(const float* __restrict__ slab, int splits, long long slab_elems, int M,
                                int N, float* out, int c_off, int c_stride, int accumulate) {
  const long long total = (long long)M * N;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    float s = slab[e];
    for (int z = 1; z < splits; ++z) s += slab[z * slab_elems + e];
    const long long m = e / N, n = e - m * N;
    float* p = out + m * c_stride + c_off + n;
    if (accumulate) s += *p;
    *p = s;
  }
}

// ---------------------------------------------------------------- host side
struct TileCfg {
  int bm, bn;
};

static const TileCfg kCfgs[] = {{128, 128}, {128, 64}, {64, 64}, {128, 32}};

struct Plan {
  int cfg;      // index into kCfgs
  int mt, nt;   // tiles
  int ktiles;
  int splits;
  int kt_per_split;
  bool scalar;
};

static void gemm_dims(const jr_conv_desc* d, int op, int* M, int* N, int* K) {
  const int P = d->n * d->ho * d->wo;
  if (op == OP_FWD) { *M = P; *N = d->c_out; *K = d->kh * d->kw * d->c_in; }
  else if (op == OP_DGRAD) { *M = d->n * d->h * d->w; *N = d->c_in; *K = d->kh * d->kw * d->c_out; }
  else { *M = d->kh * d->kw * d->c_in; *N = d->c_out; *K = P; }
}

static Plan make_plan(const jr_conv_desc* d, int op) {
  int M, N, K;
  gemm_dims(d, op, &M, &N, &K);
  Plan p{};
  p.scalar = (op == OP_FWD && (d->c_in % 16) != 0) || (op == OP_WGRAD && (d->c_in % 4) != 0);
  const double eff[] = {1.0, 0.92, 0.78, 0.78};
  double best = 1e300;
  for (int c = 0; c < 4; ++c) {
    if (p.scalar && op == OP_FWD && c != 3 && c != 1) continue;  // scalar fwd: BM=128 only
    const int bm = kCfgs[c].bm, bn = kCfgs[c].bn;
    const double work = (double)ceil_div(M, bm) * bm * (double)ceil_div(N, bn) * bn / eff[c];
    if (work < best * 0.999) { best = work; p.cfg = c; }
  }
  const int bm = kCfgs[p.cfg].bm, bn = kCfgs[p.cfg].bn;
  p.mt = (int)ceil_div(M, bm);
  p.nt = (int)ceil_div(N, bn);
  p.ktiles = (int)ceil_div(K, 16);
  // split-K: fill >= ~2 waves of blocks over 256 CUs, keep >= 8 K-tiles per split
  const int tiles = p.mt * p.nt;
  int splits = 1;
  const int target = 512;
  if (tiles < target) {
    splits = (int)ceil_div(target, tiles);
    const int max_by_k = p.ktiles / 8 > 0 ? p.ktiles / 8 : 1;
    if (splits > max_by_k) splits = max_by_k;
    if (splits > 256) splits = 256;
    if (splits < 1) splits = 1;
  }
  p.kt_per_split = (int)ceil_div(p.ktiles, splits);
  p.splits = (int)ceil_div(p.ktiles, p.kt_per_split);
  return p;
}

static size_t plan_ws_bytes(const jr_conv_desc* d, int op) {
  const Plan p = make_plan(d, op);
  if (p.splits <= 1) return 0;
  int M, N, K;
  gemm_dims(d, op, &M, &N, &K);
  return (size_t)p.splits * (size_t)M * (size_t)N * sizeof(float);
}

template <int OP, int BM, int BN, int WM, int WN, bool SC>
static void launch_cfg(const ConvArgs& a, dim3 grid, hipStream_t s) {
  hipLaunchKernelGGL((k_conv_f32<OP, BM, BN, WM, WN, SC>), grid, dim3(256), 0, s, a);
}

template <int OP, bool SC>
static void launch_op(int cfg, const ConvArgs& a, dim3 grid, hipStream_t s) {
  switch (cfg) {
    case 0: launch_cfg<OP, 128, 128, 64, 64, SC>(a, grid, s); break;
    case 1: launch_cfg<OP, 128, 64, 64, 32, SC>(a, grid, s); break;
    case 2: launch_cfg<OP, 64, 64, 32, 32, SC>(a, grid, s); break;
    default: launch_cfg<OP, 128, 32, 32, 32, SC>(a, grid, s); break;
  }
}

static int validate(const jr_conv_desc* d) {
  if (!d) return fail(JR_ERR_INVALID, "conv: null descriptor");
  if (d->n <= 0 || d->h <= 0 || d->w <= 0 || d->c_in <= 0 || d->c_out <= 0 || d->kh <= 0 ||
      d->kw <= 0 || d->stride_h <= 0 || d->stride_w <= 0 || d->pad_h < 0 || d->pad_w < 0)
    return fail(JR_ERR_INVALID, "conv: non-positive dimension");
  const int ho = (d->h + 2 * d->pad_h - d->kh) / d->stride_h + 1;
  const int wo = (d->w + 2 * d->pad_w - d->kw) / d->stride_w + 1;
  if (ho != d->ho || wo != d->wo)
    return fail(JR_ERR_INVALID, "conv: ho/wo inconsistent with h,w,k,stride,pad");
  if (d->x_c_off < 0 || d->x_c_off + d->c_in > d->x_c_stride)
    return fail(JR_ERR_INVALID, "conv: input channel slice out of range");
  if (d->y_c_off < 0 || d->y_c_off + d->c_out > d->y_c_stride)
    return fail(JR_ERR_INVALID, "conv: output channel slice out of range");
  if (d->c_out % 4 != 0 || d->y_c_stride % 4 != 0 || d->y_c_off % 4 != 0)
    return fail(JR_ERR_INVALID, "conv: c_out, output stride and output offset must be multiples of 4");
  if (d->c_in % 4 == 0 && (d->x_c_off % 4 != 0 || d->x_c_stride % 4 != 0))
    return fail(JR_ERR_INVALID, "conv: input offset/stride must be multiples of 4 when c_in is");
  const long long big = (long long)d->n * d->h * d->w * d->x_c_stride;
  const long long bigo = (long long)d->n * d->ho * d->wo * d->y_c_stride;
  if (big >= (1LL << 31) * 4 || bigo >= (1LL << 31) * 4)
    return fail(JR_ERR_INVALID, "conv: tensor too large for 32-bit pixel indexing");
  return JR_OK;
}

static int run_conv(const jr_conv_desc* d, int op, int dtype, const void* A, const void* B, void* C,
                    int accumulate, void* ws, size_t ws_bytes, void* stream) {
  int rc = validate(d);
  if (rc) return rc;
  if (dtype != JR_F32) return fail(JR_ERR_UNSUPPORTED, "conv: bf16 path not built in this round");
  if (op == OP_DGRAD && d->c_out % 16 != 0)
    return fail(JR_ERR_UNSUPPORTED, "conv bwd_data: c_out must be a multiple of 16");
  if (op == OP_DGRAD && d->c_in % 4 != 0)
    return fail(JR_ERR_UNSUPPORTED, "conv bwd_data: c_in must be a multiple of 4");
  if (!A || !B || !C) return fail(JR_ERR_INVALID, "conv: null tensor pointer");
  const Plan p = make_plan(d, op);
  ConvArgs a{};
  a.A = static_cast<const float*>(A);
  a.B = static_cast<const float*>(B);
  int M, N, K;
  gemm_dims(d, op, &M, &N, &K);
  a.M = M; a.N = N; a.K = K;
  a.n = d->n; a.h = d->h; a.w = d->w; a.cin = d->c_in; a.cout = d->c_out;
  a.kh = d->kh; a.kw = d->kw; a.sh = d->stride_h; a.sw = d->stride_w;
  a.ph = d->pad_h; a.pw = d->pad_w; a.ho = d->ho; a.wo = d->wo;
  a.xo = d->x_c_off; a.xs = d->x_c_stride; a.yo = d->y_c_off; a.ys = d->y_c_stride;
  a.accumulate = accumulate;
  a.ktiles = p.ktiles;
  a.kt_per_split = p.kt_per_split;
  a.ntn = p.nt;
  a.slab_elems = (long long)M * N;
  float* out = static_cast<float*>(C);
  int c_off, c_stride;
  if (op == OP_FWD) { c_off = d->y_c_off; c_stride = d->y_c_stride; }
  else if (op == OP_DGRAD) { c_off = d->x_c_off; c_stride = d->x_c_stride; }
  else { c_off = 0; c_stride = N; }
  a.c_off = c_off; a.c_stride = c_stride;
  if (p.splits > 1) {
    const size_t need = (size_t)p.splits * (size_t)M * N * sizeof(float);
    if (!ws || ws_bytes < need) return fail(JR_ERR_WORKSPACE, "conv: workspace too small for split-K");
    a.C = static_cast<float*>(ws);
  } else {
    a.C = out;
  }
  hipStream_t s = as_stream(stream);
  dim3 grid(p.mt * p.nt, 1, p.splits);
  if (op == OP_FWD) {
    if (p.scalar) launch_op<OP_FWD, true>(p.cfg, a, grid, s);
    else launch_op<OP_FWD, false>(p.cfg, a, grid, s);
  } else if (op == OP_DGRAD) {
    launch_op<OP_DGRAD, false>(p.cfg, a, grid, s);
  } else {
    if (p.scalar) launch_op<OP_WGRAD, true>(p.cfg, a, grid, s);
    else launch_op<OP_WGRAD, false>(p.cfg, a, grid, s);
  }
  rc = check_launch("conv gemm");
  if (rc) return rc;
  if (p.splits > 1) {
    const long long total = (long long)M * N;
    const int blocks = (int)std::min<long long>(ceil_div(total, 256), 4096);
    hipLaunchKernelGGL(k_splitk_reduce, dim3(blocks), dim3(256), 0, s, (const float*)ws, p.splits,
                       (long long)M * N, M, N, out, c_off, c_stride, accumulate);
    rc = check_launch("conv split-k reduce");
  }
  return rc;
}

}  // namespace jr

using namespace jr;

JR_API size_t jr_conv2d_workspace_size(const jr_conv_desc* d, int op, int dtype) {
  (void)dtype;
  if (!d || validate(d) != JR_OK) return 0;
  return plan_ws_bytes(d, op);
}

JR_API int jr_conv2d_fwd(const jr_conv_desc* d, int dtype, const void* x, const void* w, void* y,
                         void* ws, size_t ws_bytes, void* stream) {
  return run_conv(d, OP_FWD, dtype, x, w, y, 0, ws, ws_bytes, stream);
}

JR_API int jr_conv2d_bwd_data(const jr_conv_desc* d, int dtype, const void* dy, const void* w, void* dx,
                              int accumulate, void* ws, size_t ws_bytes, void* stream) {
  return run_conv(d, OP_DGRAD, dtype, dy, w, dx, accumulate, ws, ws_bytes, stream);
}

JR_API int jr_conv2d_bwd_filter(const jr_conv_desc* d, int dtype, const void* x, const void* dy,
                                float* dw, void* ws, size_t ws_bytes, void* stream) {
  return run_conv(d, OP_WGRAD, dtype, x, dy, dw, 0, ws, ws_bytes, stream);
}
