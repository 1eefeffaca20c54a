// jr_conv.hip — Conv2D forward / data-grad / filter-grad as implicit GEMM on
// gfx950 MFMA for fp32 tensors: JR_F32 on v_mfma_f32_32x32x2_f32 (exact f32
// at the f32 peak rate), JR_F32_X8 on v_mfma_f32_32x32x16_bf16 through an
// exact three-way bf16 split of the operands (SplitFrag; 2x the f32 peak).
//
// Replaces the TF ops behind the 94 Keras Conv2D(use_bias=False) layers that
// train.py:129-130 instantiates, and their gradients created by .minimize at
// train.py:150-153 (Conv2DBackpropInput / Conv2DBackpropFilter).
//
// One GEMM  C[M][N] = sum_k A[m][k] * B[k][n]  per op, activations NHWC,
// kernels HWIO:
//   FWD    m = output pixel (b,ho,wo)  n = co  k = (r,c,ci)   A = x gather,  B = W
//   DGRAD  m = input pixel of one stride phase (b,u,v)  n = ci  k = (a,b,co)
//          A = dy gather, B = W^T; a stride-s conv is split into s*s phase
//          GEMMs (input pixels with (h%s, w%s) fixed see only the taps
//          r = r0 + s*a), so no MAC multiplies a structural zero
//   WGRAD  m = (r,c,ci)                n = co  k = pixel      A = x gather^T, B = dy
//
// Staging: every operand tile goes global -> LDS by LDS-DMA
// (global_load_lds_dwordx4, one 1 KiB wave-instruction = 64 lanes x 16 B at
// lane-linear LDS addresses, per-lane gathered source addresses; lanes whose
// tap is out of bounds point at a 64 B zero page).  Two LDS images:
//   KC  operand contiguous along k in memory (x for FWD, dy and W^T for
//       DGRAD): image [rows][BK], 16 B quads XOR-swizzled by row
//       (pq = q ^ f(row)), read with ds_read_b128 — conflict-free;
//   MC  operand contiguous along m/n (W for FWD, x and dy for WGRAD):
//       image [BK][cols], read with ds_read_b32, consecutive lanes
//       consecutive columns — conflict-free.
// MFMA k order: lane half h consumes k in [h*BK/2, (h+1)*BK/2), step s = k
// offset, identical for both images.  Double-buffered LDS, one barrier per
// K-tile: tile t+1's DMA is in flight while tile t's MFMAs run.
// Split-K (grid.z) writes fp32 slabs reduced in a fixed order by a second
// kernel, so results are bitwise reproducible (no float atomics).
// c_in % 4 != 0 (conv1, c_in = 3) is handled by virtual channel padding:
// k runs over (r, c, ci4 < 4); the input buffer must hold 4 readable
// (finite; the engine keeps them zero) channels per pixel and the weight
// rows ci4 >= c_in read as zeros.
#include "jr_conv_impl.h"

#include <array>
#include <cstdlib>
#include <type_traits>
#include <map>
#include <mutex>
#include <vector>

namespace jr {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {   // v_cvt_pk_bf16_f32 (RNE), a in the low half
  const bf16x2 r = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, r);
}

// a - b as a plain v_sub_f32: hipcc otherwise SLP-packs the pairs into
// v_pk_add_f32, which costs more than two scalar ops beside MFMAs
// (MI355X_MICROARCH.md cycle constants)
__device__ __forceinline__ float sub_f32(float a, float b) {
  float r;
  asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// The low bf16 of a packed pair as f32 (u << 16) as a plain v_lshlrev_b32:
// hipcc otherwise rewrites pk_bf16(a, b) << 16 into pk_bf16(a, 0) << 16, one
// more conversion per pair and split stage (13 VALU per pair instead of 11)
__device__ __forceinline__ float lo_bf16_f32(uint32_t u) {
  uint32_t r;
  asm("v_lshlrev_b32 %0, 16, %1" : "=v"(r) : "v"(u));
  return __uint_as_float(r);
}

// Exact three-way split of 8 fp32 values into bf16 (SplitFrag): x = h + m + l with
// h = rne(x), m = rne(x - h), l = x - h - m (the remainders are exact in
// fp32; x - h has at most 16 significant bits, x - h - m at most 8, so l is
// exact in bf16).  |m| <= 2^-8 |x|, |l| <= 2^-16 |x| (normal range).  Done
// in three stages, so each stage's VALU can hide under the MFMAs of the
// terms the previous stage made available: init = h (one cvt per pair),
// stage2 = r = x - h and m, stage3 = r - m and l.  skip = diagnostic (no
// split: the fp32 bits reinterpreted).
// bf16 products per fp32 product: 8 = hh hm mh mm hl lh ml lm, dropping only
// ll (< 2^-32 |a b|).  6 (also dropping ml + lm, up to 2^-23 |a b|: the size
// of fp32's own rounding) measured 8 % faster per step but ~1.5-2x the
// fp32 kernel's error on long reductions; 8 matches it.
constexpr int kSplitTerms = 8;

struct SplitFrag {
  float x[8];
  uint32_t hp[4], mp[4], lp[4];
  __device__ __forceinline__ void init(const float* v, bool skip) {
#pragma unroll
    for (int t = 0; t < 8; ++t) x[t] = v[t];
#pragma unroll
    for (int p = 0; p < 4; ++p) hp[p] = skip ? __float_as_uint(x[2 * p]) : pk_bf16(x[2 * p], x[2 * p + 1]);
  }
  __device__ __forceinline__ void stage2(bool skip) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (skip) { mp[p] = hp[p]; continue; }
      x[2 * p] = sub_f32(x[2 * p], lo_bf16_f32(hp[p]));
      x[2 * p + 1] = sub_f32(x[2 * p + 1], __uint_as_float(hp[p] & 0xffff0000u));
      mp[p] = pk_bf16(x[2 * p], x[2 * p + 1]);
    }
  }
  __device__ __forceinline__ void stage3(bool skip) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (skip) { lp[p] = hp[p]; continue; }
      x[2 * p] = sub_f32(x[2 * p], lo_bf16_f32(mp[p]));
      x[2 * p + 1] = sub_f32(x[2 * p + 1], __uint_as_float(mp[p] & 0xffff0000u));
      lp[p] = pk_bf16(x[2 * p], x[2 * p + 1]);
    }
  }
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  __device__ __forceinline__ bf16x8 h() const { return __builtin_bit_cast(bf16x8, (u32x4){hp[0], hp[1], hp[2], hp[3]}); }
  __device__ __forceinline__ bf16x8 m() const { return __builtin_bit_cast(bf16x8, (u32x4){mp[0], mp[1], mp[2], mp[3]}); }
  __device__ __forceinline__ bf16x8 l() const { return __builtin_bit_cast(bf16x8, (u32x4){lp[0], lp[1], lp[2], lp[3]}); }
};

// JR_F32_X6H (H6): the same three-way split
// into fp16 (11-bit significands) of the operand scaled by a power of two
// (so its largest magnitude sits in [2^14, 2^15)): x s = h + m + l with h =
// rtz(x s), m = rtz(x s - h), l = x s - h - m -- every remainder exact in
// fp32 (a truncation's tail), l at most 2 bits, exact while x s >= 2^-1
// (fp16 subnormals keep the rest down to 2^-24).  Six f16 MFMAs per
// product (hh hm mh mm hl lh); dropped: ml + lm (< 2^-32 |a b|) and ll, the
// x8 class.  acc is scaled back by 2^-(ka+kb) (exact) after the K loop.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pkrtz_f16(float a, float b) {   // v_cvt_pkrtz_f16_f32, a in the low half
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(a, b));
}

// x - (f32) f16 half of a packed pair in ONE v_fma_mix_f32 (-h * one + x, the
// f16 source converted inside the instruction): exact, since h is x
// truncated to fp16 precision and x - h is x's own low significand bits, so
// bitwise the v_cvt_f32_f16 + v_sub_f32 pair it replaces at half the VALU
// issue (the residual stages were 5 VALU per pair, now 3).  `one` is 1.0
// hidden from the optimiser (H6 prologue): with a literal 1.0 the fma folds to
// fsub and hipcc emits the cvt + sub pair again; kept compiler-visible (not
// inline asm) so the hazard pass sees a mix instruction -- its result needs
// one wait state before a VALU reads it, so every stage issues all eight
// residuals before its four packs.
__device__ __forceinline__ float sub_f16lo(float x, uint32_t h, float one) {
  return __builtin_fmaf(-(float)__builtin_bit_cast(f16x2, h)[0], one, x);
}
__device__ __forceinline__ float sub_f16hi(float x, uint32_t h, float one) {
  return __builtin_fmaf(-(float)__builtin_bit_cast(f16x2, h)[1], one, x);
}

struct SplitFrag16 {
  float x[8];
  uint32_t hp[4], mp[4], lp[4];
  __device__ __forceinline__ void init(const float* v, float scale) {
#pragma unroll
    for (int t = 0; t < 8; ++t) x[t] = v[t] * scale;
#pragma unroll
    for (int p = 0; p < 4; ++p) hp[p] = pkrtz_f16(x[2 * p], x[2 * p + 1]);
  }
  __device__ __forceinline__ void stage2(float one) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      x[2 * p] = sub_f16lo(x[2 * p], hp[p], one);
      x[2 * p + 1] = sub_f16hi(x[2 * p + 1], hp[p], one);
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) mp[p] = pkrtz_f16(x[2 * p], x[2 * p + 1]);
  }
  __device__ __forceinline__ void stage3(float one) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      x[2 * p] = sub_f16lo(x[2 * p], mp[p], one);
      x[2 * p + 1] = sub_f16hi(x[2 * p + 1], mp[p], one);
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) lp[p] = pkrtz_f16(x[2 * p], x[2 * p + 1]);
  }
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  __device__ __forceinline__ f16x8 h() const { return __builtin_bit_cast(f16x8, (u32x4){hp[0], hp[1], hp[2], hp[3]}); }
  __device__ __forceinline__ f16x8 m() const { return __builtin_bit_cast(f16x8, (u32x4){mp[0], mp[1], mp[2], mp[3]}); }
  __device__ __forceinline__ f16x8 l() const { return __builtin_bit_cast(f16x8, (u32x4){lp[0], lp[1], lp[2], lp[3]}); }
};

// DBG (diagnostic builds only, jr_conv2d_debug_time): 1 = no MFMA,
// 2 = no DMA after the first tile (results are wrong in both).
//
// Address generation.  When the reduction channel count (c_in for FWD,
// c_out for DGRAD) is a multiple of BK, a K-tile never straddles a tap, so
// the tap (r, c, channel base) is WAVE-UNIFORM: it lives in SGPRs, and each
// DMA slot keeps a 64-bit base pointer fixed for the whole K loop; per tile
// a lane only adds a scalar offset and checks its row's bounds.  Otherwise
// (conv1, c_in = 3 padded to 4) every lane keeps its own mixed-radix k
// counter (generic path).  WGRAD's A operand walks pixels along k, so its
// lanes advance (b, oh, ow) counters.
//
// Stream-K (SK, the JR_F32_X8 stream-K tile ids): the grid is a fixed
// number of blocks and the GEMM's tiles x K-tiles iterations are cut into
// equal contiguous ranges, one per block (g.sk_ipb each), so every CU gets
// the same MAC count whatever the tile count -- no wave quantization and no
// split-K slabs or reduce launch.  A block walks its range tile by tile; a
// tile cut between blocks b < b+1 < ... (b holds its FIRST K-tile at the END
// of its range, the later blocks its later K-tiles at the START of theirs)
// is handed off without any block waiting (jr_conv_impl.h sk_handoff): each
// piece is published as an fp32 partial (write-through sc1 stores, drained)
// and counted on b's word, and the block completing the count adds the
// pieces in block order (deterministic: the cut points are fixed by the
// grid, the sum order by the block order) and runs the ordinary epilogue
// (store + fused BN statistics).  No block depends on another being resident,
// so concurrent kernels on other lanes or processes cannot stall a grid.  The
// count words are per-stream library words (stream_scratch) that the
// completing block resets, so a launch needs no memset.
template <int OP, int BM, int BN, int WGM, int BK, int NBUF, bool UT, bool X8, int DBG = 0, bool SK = false,
          bool H6 = false>
__global__ void __launch_bounds__(256) k_conv(ConvArgs g) {
  constexpr int WGN = 4 / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 32, TN = WN / 32;
  static_assert(WM % 32 == 0 && WN % 32 == 0, "wave tile must be a multiple of 32x32");
  constexpr int QPR = BK / 4;                 // 16 B quads per KC row
  constexpr int RPI = 64 / QPR;               // KC rows per DMA instruction
  constexpr int SWZ = 16 / QPR;               // rows sharing one swizzle value
  constexpr int HALF = BK / 2;                // k per lane half
  constexpr bool A_KC = (OP != OP_WGRAD);
  constexpr bool B_KC = (OP == OP_DGRAD);
  constexpr int ASZ = BM * BK, BSZ = BN * BK;  // floats per image
  constexpr int A_INSTR = ASZ / 256, B_INSTR = BSZ / 256;
  constexpr int A_PW = (A_INSTR + 3) / 4, B_PW = (B_INSTR + 3) / 4;  // per wave
  static_assert(ASZ % 256 == 0 && BSZ % 256 == 0, "tile must be whole DMA instructions");
  constexpr int SMEM = NBUF * (ASZ + BSZ) > 4 * stage_floats<WN>() ? NBUF * (ASZ + BSZ) : 4 * stage_floats<WN>();
  __shared__ __attribute__((aligned(1024))) float smem[SMEM];
  JR_ST(Stamps stamp; stamp.start();)
  member_offsets(g);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // JR_F32_X6H operand scales (wave-uniform)
  float h_sa = 1.f, h_sb = 1.f, h_one = 1.f;
  if constexpr (H6) {
    asm volatile("" : "+s"(h_one));      // SplitFrag16: 1.0 the optimiser cannot fold
    h_sa = __uint_as_float(__builtin_amdgcn_readfirstlane(
        __float_as_uint(pow2_scale(g.a_max ? absmax64(g.a_max, lane) : g.a_bnd))));
    h_sb = __uint_as_float(__builtin_amdgcn_readfirstlane(
        __float_as_uint(pow2_scale(g.b_max ? absmax64(g.b_max, lane) : g.b_bnd))));
  }
  const int wm0 = (wave / WGN) * WM;
  const int wn0 = (wave % WGN) * WN;

  // SK: this block's iteration range [sk_it, sk_end) over tiles x K-tiles
  long long sk_it = 0, sk_end = 0;
  // SK: logical block lb = xcd_remap(blockIdx.x): the blocks of one XCD walk
  // adjacent iteration ranges, so a cut tile's pieces and the operand rows
  // neighbouring ranges share stay in that XCD's L2 (the decomposition, and
  // so every sum, is the same as with lb = blockIdx.x)
  const int lb = SK ? xcd_remap(blockIdx.x, gridDim.x) : 0;
  if constexpr (SK) {
    const long long W = (long long)((g.M + BM - 1) / BM) * g.ntn * g.ktiles;
    sk_it = (long long)lb * g.sk_ipb;
    sk_end = sk_it + g.sk_ipb < W ? sk_it + g.sk_ipb : W;
  }
  bool sk_first = true;
  // one iteration per (tile, K range) segment: ordinary launches run exactly one
  for (;;) {
  int tile, kt0, kt1;
  if constexpr (SK) {
    if (sk_it >= sk_end) break;
    tile = (int)(sk_it / g.ktiles);
    kt0 = (int)(sk_it - (long long)tile * g.ktiles);
    kt1 = (int)(sk_end - sk_it < (long long)(g.ktiles - kt0) ? kt0 + (sk_end - sk_it) : g.ktiles);
    sk_it += kt1 - kt0;
    if (!sk_first) __syncthreads();      // the previous segment's stage / ring reads are done
  } else {
    tile = xcd_remap(blockIdx.x, gridDim.x);
    kt0 = blockIdx.z * g.kt_per_split;
    kt1 = min(g.ktiles, kt0 + g.kt_per_split);
  }
  const int mt = tile / g.ntn, nt = tile - mt * g.ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const float* zp = g_zero_page;
  const int cred = OP == OP_FWD ? g.cp : g.cout;       // channel radix of the KC k index
  // FWD/DGRAD: UT = wave-uniform tap (host guarantees cred % BK == 0).
  // WGRAD: UT = incremental pixel walk (host guarantees BK / wo < ho: one
  // carry per radix and K-tile), else the mixed-radix loop.
  constexpr bool ut = UT && OP != OP_WGRAD;
  // WGRAD UT (round 3): every piece keeps its element offset a_off and adds
  // one of three wave-uniform deltas per K-tile by its carries (no
  // multiplies: the rebuilt address cost two v_mul_lo_u32 per piece and tile);
  // single const definitions (assigned in branches they became allocas read
  // through a per-lane select of their addresses)
  const int wq = OP == OP_WGRAD ? BK / g.wo : 0, wr = OP == OP_WGRAD ? BK - wq * g.wo : 0;
  const int dW0 = OP == OP_WGRAD ? (wq * g.sh * g.w + wr * g.sw) * g.xs : 0;
  const int dW1 = OP == OP_WGRAD ? (g.sh * g.w - g.wo * g.sw) * g.xs : 0;
  const int dW2 = OP == OP_WGRAD ? (g.h * g.w - g.ho * g.sh * g.w) * g.xs : 0;

  // ---------------------------------------------------------------- A state
  const float* a_ptr[A_PW];                 // per-slot base pointer (ut paths)
  int a_p0[A_PW], a_p1[A_PW], a_p2[A_PW];   // per-slot geometry fixed over K
  int a_s0[A_PW], a_s1[A_PW], a_s2[A_PW];   // per-lane k counters (generic / WGRAD)
  int a_off[A_PW];                          // WGRAD UT: element offset from a_ptr
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int j = wave + 4 * i;
    a_ptr[i] = zp;
    a_p0[i] = a_p1[i] = a_p2[i] = 0;
    a_s0[i] = a_s1[i] = a_s2[i] = 0;
    a_off[i] = 0;
    if (A_INSTR % 4 != 0 && j >= A_INSTR) continue;
    if constexpr (A_KC) {
      const int row = j * RPI + lane / QPR;
      const int q = (lane % QPR) ^ ((row / SWZ) % QPR);
      const int m = m0 + row;
      const int k = kt0 * BK + q * 4;
      if constexpr (OP == OP_FWD) {
        int pix = 0;
        if (m < g.M) {
          const int hw = g.ho * g.wo;
          const int b = m / hw, rem = m - b * hw;
          const int oh = rem / g.wo, ow = rem - oh * g.wo;
          a_p0[i] = oh * g.sh - g.ph;
          a_p1[i] = ow * g.sw - g.pw;
          a_p2[i] = b * g.h * g.w;
          pix = a_p2[i] + a_p0[i] * g.w + a_p1[i];
        } else {
          a_p0[i] = -(1 << 28);
        }
        a_ptr[i] = g.A + ((long long)pix * g.xs + g.xo + q * 4);
        const int rc = k / g.cp;
        a_s2[i] = k - rc * g.cp;          // ci
        a_s0[i] = rc / g.kw;              // r
        a_s1[i] = rc - a_s0[i] * g.kw;    // c
      } else {  // DGRAD: m = (b,u,v) of the phase, k = (a, bb, co)
        int pix = 0;
        if (m < g.M) {
          const int hw = g.hc * g.wc;
          const int b = m / hw, rem = m - b * hw;
          const int u = rem / g.wc, v = rem - u * g.wc;
          a_p0[i] = u + g.ey;
          a_p1[i] = v + g.ex;
          a_p2[i] = b * g.ho * g.wo;
          pix = a_p2[i] + a_p0[i] * g.wo + a_p1[i];
        } else {
          a_p0[i] = -(1 << 28);
        }
        a_ptr[i] = g.A + ((long long)pix * g.ys + g.yo + q * 4);
        const int ab = k / g.cout;
        a_s2[i] = k - ab * g.cout;        // co
        a_s0[i] = ab / g.nb;              // a
        a_s1[i] = ab - a_s0[i] * g.nb;    // bb
      }
    } else {  // WGRAD MC: m = (r,c,ci) fixed per slot, k = pixel advances
      const int flat = j * 256 + lane * 4;
      const int krow = flat / BM, col = flat - krow * BM;
      const int m = m0 + col;
      if (m < g.M) {
        const int rc = m / g.cp, ci = m - rc * g.cp;
        const int r = rc / g.kw, c = rc - r * g.kw;
        a_p0[i] = r - g.ph;
        a_p1[i] = c - g.pw;
        a_p2[i] = ci;
      } else {
        a_p0[i] = -(1 << 28);
      }
      const int pix = kt0 * BK + krow;
      const int hw = g.ho * g.wo;
      a_s0[i] = pix / hw;                       // b
      const int rem = pix - a_s0[i] * hw;
      a_s1[i] = rem / g.wo;                     // oh
      a_s2[i] = rem - a_s1[i] * g.wo;           // ow
      if (m < g.M) a_ptr[i] = g.A + ((long long)(a_p0[i] * g.w + a_p1[i]) * g.xs + g.xo + a_p2[i]);
      a_off[i] = ((a_s0[i] * g.h + a_s1[i] * g.sh) * g.w + a_s2[i] * g.sw) * g.xs;
    }
  }
  // ---------------------------------------------------------------- B state
  const float* b_ptr[B_PW];
  int b_p0[B_PW], b_s0[B_PW], b_s1[B_PW], b_s2[B_PW];
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int j = wave + 4 * i;
    b_ptr[i] = zp;
    b_p0[i] = b_s0[i] = b_s1[i] = b_s2[i] = 0;
    if (B_INSTR % 4 != 0 && j >= B_INSTR) continue;
    if constexpr (B_KC) {  // DGRAD: rows = ci, k = (a, bb, co)
      const int row = j * RPI + lane / QPR;
      const int q = (lane % QPR) ^ ((row / SWZ) % QPR);
      const int nn = n0 + row;
      b_p0[i] = nn < g.N ? nn : -1;
      b_ptr[i] = g.B + ((long long)(nn < g.N ? nn : 0) * g.cout + q * 4);
      const int k = kt0 * BK + q * 4;
      const int ab = k / g.cout;
      b_s2[i] = k - ab * g.cout;
      b_s0[i] = ab / g.nb;
      b_s1[i] = ab - b_s0[i] * g.nb;
    } else {  // MC: rows = k, cols = n
      const int flat = j * 256 + lane * 4;
      const int krow = flat / BN, col = flat - krow * BN;
      b_p0[i] = (n0 + col < g.N) ? n0 + col : -1;
      b_s0[i] = kt0 * BK + krow;          // k of this lane at tile kt0
      if constexpr (OP == OP_FWD)
        b_ptr[i] = g.B + ((long long)b_s0[i] * g.N + (n0 + col));
      else
        b_ptr[i] = g.B + ((long long)b_s0[i] * g.ys + g.yo + n0 + col);
    }
  }
  // wave-uniform tap counters of the ut paths, at tile kt0
  int t_r = 0, t_c = 0, t_ch = 0;
  if constexpr (ut) {
    const int k = kt0 * BK;
    const int rc = k / cred;
    t_ch = k - rc * cred;
    t_r = rc / (OP == OP_FWD ? g.kw : g.nb);
    t_c = rc - t_r * (OP == OP_FWD ? g.kw : g.nb);
  }

  const bool a_multi = A_KC ? (cred < BK) : (!UT && g.wo < BK);
  const bool b_multi = B_KC ? (g.cout < BK) : false;
  // DMA of one operand piece (d < A_PW: A slot d, else B slot d - A_PW) of
  // tile kt; d is a compile-time constant at every call site (unrolled), so
  // the slot dispatch folds away.
  auto issue_piece = [&](int kt, int d, float* __restrict__ As, float* __restrict__ Bs) {
    if (d < A_PW) {
      const int i = d;
      const int j = wave + 4 * i;
      if (A_INSTR % 4 != 0 && j >= A_INSTR) return;
      if constexpr (A_KC && ut) {
        long long off;                          // wave-uniform element offset of the tap
        int dr, dc;
        if constexpr (OP == OP_FWD) {
          off = (long long)(t_r * g.w + t_c) * g.xs + t_ch;
          dr = t_r; dc = t_c;
        } else {
          off = -(long long)(t_r * g.wo + t_c) * g.ys + t_ch;
          dr = -t_r; dc = -t_c;
        }
        const int hmax = OP == OP_FWD ? g.h : g.ho, wmax = OP == OP_FWD ? g.w : g.wo;
        const bool ok = (unsigned)(a_p0[i] + dr) < (unsigned)hmax && (unsigned)(a_p1[i] + dc) < (unsigned)wmax;
        dma16_ring(ok ? a_ptr[i] + off : zp, As + j * 256);
      } else {
        const float* src = zp;
        if constexpr (OP == OP_FWD) {
          const int hi = a_p0[i] + a_s0[i], wi = a_p1[i] + a_s1[i];
          const bool ok = (unsigned)hi < (unsigned)g.h && (unsigned)wi < (unsigned)g.w && a_s0[i] < g.kh;
          const float* p = g.A + ((a_p2[i] + hi * g.w + wi) * g.xs + g.xo + a_s2[i]);
          src = ok ? p : zp;
          adv_mixed(a_s2[i], a_s1[i], a_s0[i], g.cp, g.kw, a_multi);
        } else if constexpr (OP == OP_DGRAD) {
          const int oh = a_p0[i] - a_s0[i], ow = a_p1[i] - a_s1[i];
          const bool ok = (unsigned)oh < (unsigned)g.ho && (unsigned)ow < (unsigned)g.wo && a_s0[i] < g.na;
          const float* p = g.A + ((a_p2[i] + oh * g.wo + ow) * g.ys + g.yo + a_s2[i]);
          src = ok ? p : zp;
          adv_mixed(a_s2[i], a_s1[i], a_s0[i], g.cout, g.nb, a_multi);
        } else if constexpr (UT) {  // WGRAD, incremental: (image, oh, ow) += BK pixels
          const int hi = __mul24(a_s1[i], g.sh) + a_p0[i], wi = __mul24(a_s2[i], g.sw) + a_p1[i];
          const bool ok = (a_s0[i] < g.n) & ((unsigned)hi < (unsigned)g.h) & ((unsigned)wi < (unsigned)g.w);
          src = ok ? a_ptr[i] + a_off[i] : zp;
          int ow = a_s2[i] + wr;
          const bool c1 = ow >= g.wo;
          ow -= c1 ? g.wo : 0;
          int oh = a_s1[i] + wq + (c1 ? 1 : 0);
          const bool c2 = oh >= g.ho;
          oh -= c2 ? g.ho : 0;
          a_off[i] += dW0 + (c1 ? dW1 : 0) + (c2 ? dW2 : 0);
          a_s2[i] = ow;
          a_s1[i] = oh;
          a_s0[i] += c2 ? 1 : 0;
        } else {  // WGRAD
          const int hi = a_s1[i] * g.sh + a_p0[i], wi = a_s2[i] * g.sw + a_p1[i];
          const bool ok = a_s0[i] < g.n && (unsigned)hi < (unsigned)g.h && (unsigned)wi < (unsigned)g.w;
          const float* p = g.A + (((a_s0[i] * g.h + hi) * g.w + wi) * g.xs + g.xo + a_p2[i]);
          src = ok ? p : zp;
          adv_mixed(a_s2[i], a_s1[i], a_s0[i], g.wo, g.ho, a_multi);
        }
        dma16_ring(src, As + j * 256);
      }
      return;
    }
    const int i = d - A_PW;
    const int j = wave + 4 * i;
    if (B_INSTR % 4 != 0 && j >= B_INSTR) return;
    if constexpr (B_KC) {  // DGRAD: W[(r0+sh*a, c0+sw*bb)][ci][co]
      if constexpr (ut) {
        const long long off = (long long)((g.r0 + g.sh * t_r) * g.kw + (g.c0 + g.sw * t_c)) * g.cin * g.cout + t_ch;
        dma16_ring(b_p0[i] >= 0 ? b_ptr[i] + off : zp, Bs + j * 256);
      } else {
        const bool ok = b_p0[i] >= 0 && b_s0[i] < g.na;
        const int r = g.r0 + g.sh * b_s0[i], c = g.c0 + g.sw * b_s1[i];
        const float* p = g.B + (((r * g.kw + c) * g.cin + b_p0[i]) * g.cout + b_s2[i]);
        dma16_ring(ok ? p : zp, Bs + j * 256);
        adv_mixed(b_s2[i], b_s1[i], b_s0[i], g.cout, g.nb, b_multi);
      }
    } else {
      const int kbase = kt * BK;                                   // wave-uniform
      const long long off = (long long)(kbase - kt0 * BK) * (OP == OP_FWD ? g.N : g.ys);
      const int k = b_s0[i] + (kbase - kt0 * BK);
      bool ok = b_p0[i] >= 0 && k < g.K;
      const float* p = b_ptr[i] + off;
      if constexpr (OP == OP_FWD) {
        if (!ut && g.cp != g.cin) {  // virtual channel padding (c_in % 4 != 0): uniform branch
          const int rc = k / g.cp, ci = k - rc * g.cp;
          ok = ok && ci < g.cin;
          p = g.B + ((rc * g.cin + ci) * g.N + b_p0[i]);
        }
      }
      dma16_ring(ok ? p : zp, Bs + j * 256);
    }
  };
  // advance the wave-uniform tap by BK after a tile's pieces are issued
  auto advance = [&]() {
    if constexpr (ut) {   // branch-free (s_cselect) so the K loop stays one basic block
      t_ch += BK;
      const bool w1 = t_ch == cred;
      t_ch = w1 ? 0 : t_ch;
      t_c += w1 ? 1 : 0;
      const bool w2 = t_c == (OP == OP_FWD ? g.kw : g.nb);
      t_c = w2 ? 0 : t_c;
      t_r += w2 ? 1 : 0;
    }
  };
  constexpr int NPIECE = A_PW + B_PW;
  auto issue = [&](int kt, float* __restrict__ As, float* __restrict__ Bs) {
#pragma unroll
    for (int d = 0; d < NPIECE; ++d) issue_piece(kt, d, As, Bs);
    advance();
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int l31 = lane & 31, lh = lane >> 5;
  // DMA wave-instructions per K-tile used for the counted waits: the
  // minimum over the block's waves, a compile-time constant.  A wave that
  // issues one more piece per tile (A_INSTR or B_INSTR not a multiple of 4)
  // then waits for one piece of a newer tile too — safe, and it keeps the
  // K loop free of per-wave branches.
  constexpr int per_tile = A_INSTR / 4 + B_INSTR / 4;

  // One K-tile: fragments of tile kt (LDS -> VGPRs), then MFMAs from
  // registers with the DMA of tile kt+NBUF-1 (into the buffer read in
  // iteration kt-1, released by the barrier that ended it) issued piece by
  // piece between the k-steps.  The reads and the DMA go through
  // __restrict__ views of two different buffers: the noalias scopes let
  // hipcc's waitcnt pass see that the ds_reads need not wait for the LDS-DMA
  // still in flight (without them it drains every DMA first).
  auto step = [&](int kt, auto do_issue, const float* __restrict__ As, const float* __restrict__ Bs,
                  float* __restrict__ wA, float* __restrict__ wB) {
    constexpr bool DO_ISSUE = decltype(do_issue)::value;
    float af[TM][HALF], bfr[TN][HALF];
    if constexpr (DBG == 3) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int t = 0; t < HALF; ++t) af[i][t] = __builtin_amdgcn_readfirstlane(kt + t + i);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int t = 0; t < HALF; ++t) bfr[j][t] = (float)(lane + t + j);
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if constexpr (A_KC) {
          const int row = wm0 + i * 32 + l31;
          const int f = (row / SWZ) % QPR;
#pragma unroll
          for (int t = 0; t < QPR / 2; ++t) {
            const float4 v = *reinterpret_cast<const float4*>(As + row * BK + (((lh * (QPR / 2) + t) ^ f) * 4));
            af[i][4 * t + 0] = v.x; af[i][4 * t + 1] = v.y; af[i][4 * t + 2] = v.z; af[i][4 * t + 3] = v.w;
          }
        } else {
#pragma unroll
          for (int s = 0; s < HALF; ++s) af[i][s] = As[(lh * HALF + s) * BM + wm0 + i * 32 + l31];
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (B_KC) {
          const int row = wn0 + j * 32 + l31;
          const int f = (row / SWZ) % QPR;
#pragma unroll
          for (int t = 0; t < QPR / 2; ++t) {
            const float4 v = *reinterpret_cast<const float4*>(Bs + row * BK + (((lh * (QPR / 2) + t) ^ f) * 4));
            bfr[j][4 * t + 0] = v.x; bfr[j][4 * t + 1] = v.y; bfr[j][4 * t + 2] = v.z; bfr[j][4 * t + 3] = v.w;
          }
        } else {
#pragma unroll
          for (int s = 0; s < HALF; ++s) bfr[j][s] = Bs[(lh * HALF + s) * BN + wn0 + j * 32 + l31];
        }
      }
    }
    if constexpr (X8) {
      // JR_F32_X8: each lane's 8 consecutive k of a lane half are exactly the
      // A / B operand of one v_mfma_f32_32x32x16_bf16 (lane l: row l % 32,
      // k = 8 (l / 32) + 0..7 of the group), so the fp32 fragments split in
      // registers into x = h + m + l (three bf16, exact) and kSplitTerms bf16
      // MFMAs accumulate the partial products in fp32 (SplitFrag).
      constexpr int G8 = HALF / 8;
      static_assert(HALF % 8 == 0, "X8 needs BK % 16 == 0");
      // Five MFMA phases per 16-k group, each a scheduling region carrying
      // the split VALU the NEXT phase needs, so the split issues under MFMAs
      // and every region holds about as much VALU as its MFMAs can cover:
      //   (h packs: one cvt per pair)
      //   P1: hh        | A residuals, A m packs
      //   P2: mh        | B residuals, B m packs
      //   P3: hm mm     | A second residuals, A l packs
      //   P4: lh        | B second residuals, B l packs
      //   P5: hl (ml lm)
      // (three phases -- hh | all m; hm mh mm | all l; the rest -- left the
      // first one VALU-bound and the last one VALU-idle).
      int piece = 0;
      auto next_piece = [&]() {
        if constexpr (DO_ISSUE && DBG != 2) {
          if (piece < NPIECE) issue_piece(kt + NBUF - 1, piece, wA, wB);
          ++piece;
        }
      };
      auto mma = [&](int i, int j, const bf16x8& x, const bf16x8& y) {
        if constexpr (DBG == 1) {   // diagnostic: no MFMA (keeps the operands live)
          const f32x4 t = __builtin_bit_cast(f32x4, x) + __builtin_bit_cast(f32x4, y);
          acc[i][j][0] += t[0]; acc[i][j][1] += t[1]; acc[i][j][2] += t[2]; acc[i][j][3] += t[3];
        } else {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, acc[i][j], 0, 0, 0);
        }
      };
      if constexpr (H6) {
        auto mmh = [&](int i, int j, const f16x8& x, const f16x8& y) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, y, acc[i][j], 0, 0, 0);
        };
#pragma unroll
        for (int g8 = 0; g8 < G8; ++g8) {
          SplitFrag16 sa[TM], sb[TN];
#pragma unroll
          for (int i = 0; i < TM; ++i) sa[i].init(&af[i][8 * g8], h_sa);
#pragma unroll
          for (int j = 0; j < TN; ++j) sb[j].init(&bfr[j][8 * g8], h_sb);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) mmh(i, j, sa[i].h(), sb[j].h());
#pragma unroll
          for (int i = 0; i < TM; ++i) sa[i].stage2(h_one);
          next_piece();
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) mmh(i, j, sa[i].m(), sb[j].h());
#pragma unroll
          for (int j = 0; j < TN; ++j) sb[j].stage2(h_one);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              mmh(i, j, sa[i].h(), sb[j].m());
              mmh(i, j, sa[i].m(), sb[j].m());
            }
#pragma unroll
          for (int i = 0; i < TM; ++i) sa[i].stage3(h_one);
          next_piece();
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) mmh(i, j, sa[i].l(), sb[j].h());
#pragma unroll
          for (int j = 0; j < TN; ++j) sb[j].stage3(h_one);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) mmh(i, j, sa[i].h(), sb[j].l());
          next_piece();
        }
        if constexpr (DO_ISSUE && DBG != 2) {
#pragma unroll
          for (int d = 3 * G8; d < NPIECE; ++d) issue_piece(kt + NBUF - 1, d, wA, wB);
          advance();
        }
        return;
      }
#pragma unroll
      for (int g8 = 0; g8 < G8; ++g8) {
        SplitFrag sa[TM], sb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) sa[i].init(&af[i][8 * g8], DBG == 4);
#pragma unroll
        for (int j = 0; j < TN; ++j) sb[j].init(&bfr[j][8 * g8], DBG == 4);
        // (sched_barrier closes each region even when this wave has no DMA
        // piece left to issue)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) mma(i, j, sa[i].h(), sb[j].h());
#pragma unroll
        for (int i = 0; i < TM; ++i) sa[i].stage2(DBG == 4);
        next_piece();
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) mma(i, j, sa[i].m(), sb[j].h());
#pragma unroll
        for (int j = 0; j < TN; ++j) sb[j].stage2(DBG == 4);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            mma(i, j, sa[i].h(), sb[j].m());
            mma(i, j, sa[i].m(), sb[j].m());
          }
#pragma unroll
        for (int i = 0; i < TM; ++i) sa[i].stage3(DBG == 4);
        next_piece();
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) mma(i, j, sa[i].l(), sb[j].h());
#pragma unroll
        for (int j = 0; j < TN; ++j) sb[j].stage3(DBG == 4);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            mma(i, j, sa[i].h(), sb[j].l());
            if constexpr (kSplitTerms == 8) {
              mma(i, j, sa[i].m(), sb[j].l());
              mma(i, j, sa[i].l(), sb[j].m());
            }
          }
        next_piece();
      }
      if constexpr (DO_ISSUE && DBG != 2) {
#pragma unroll
        for (int d = 3 * G8; d < NPIECE; ++d) issue_piece(kt + NBUF - 1, d, wA, wB);
        advance();
      }
      return;
    }
    // MFMAs of k-step s, then DMA piece s of tile kt+NBUF-1: program order
    // places each piece's address VALU and issue under an MFMA group in
    // flight (the LDS-DMA intrinsic is a scheduling boundary for hipcc).
#pragma unroll
    for (int s = 0; s < HALF; ++s) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          if constexpr (DBG == 1) acc[i][j][s & 15] += af[i][s] * bfr[j][s];
          else acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bfr[j][s], acc[i][j], 0, 0, 0);
      if constexpr (DO_ISSUE && DBG != 2)
        if (s < NPIECE) issue_piece(kt + NBUF - 1, s, wA, wB);
    }
    if constexpr (DO_ISSUE && DBG != 2) {
#pragma unroll
      for (int d = HALF; d < NPIECE; ++d) issue_piece(kt + NBUF - 1, d, wA, wB);
      advance();
    }
  };

  // every compiler-visible load of the previous segment (hand-off pieces,
  // accumulate reads, the H6 magnitude words) retired here, once per
  // segment: otherwise hipcc's waitcnt pass, which merges that state into
  // the K loop, keeps an s_waitcnt vmcnt(0) in every K-tile (and so drains
  // the DMA ring it cannot see)
  __builtin_amdgcn_s_waitcnt(0x0F70);     // vmcnt(0)
  if (kt0 < kt1) {
    // prologue: tiles kt0 .. kt0+NBUF-2 in flight
#pragma unroll
    for (int p = 0; p < NBUF - 1; ++p)
      if (kt0 + p < kt1) issue(kt0 + p, smem + p * (ASZ + BSZ), smem + p * (ASZ + BSZ) + ASZ);
    wait_vmcnt(per_tile * min(NBUF - 2, kt1 - kt0 - 1));
    __builtin_amdgcn_s_barrier();
    JR_ST(stamp.prologue();)
    int cur = 0;
    int kt = kt0;
    // steady state: NBUF-1 tiles in flight after this iteration's issue;
    // tile kt+1 landed once at most (NBUF-2) tiles per wave are outstanding
    for (; kt < kt1 - (NBUF - 1); ++kt) {
      const int nxt = cur == 0 ? NBUF - 1 : cur - 1;
      step(kt, std::true_type{}, smem + cur * (ASZ + BSZ), smem + cur * (ASZ + BSZ) + ASZ,
           smem + nxt * (ASZ + BSZ), smem + nxt * (ASZ + BSZ) + ASZ);
      // sched_barrier keeps hipcc from sinking the register-only MFMAs below
      // the wait; one barrier: every wave's part of tile kt+1 is in LDS and
      // every wave is done reading tile kt
      __builtin_amdgcn_sched_barrier(0);
      JR_ST(const unsigned long long tw = stamp.now();)
      wait_vmcnt(per_tile * (NBUF - 2));
      __builtin_amdgcn_s_barrier();
      JR_ST(stamp.w += stamp.now() - tw;)
      __builtin_amdgcn_sched_barrier(0);
      cur = cur + 1 == NBUF ? 0 : cur + 1;
    }
    // drain: no more DMA to issue
    for (; kt < kt1; ++kt) {
      step(kt, std::false_type{}, smem + cur * (ASZ + BSZ), smem + cur * (ASZ + BSZ) + ASZ, nullptr, nullptr);
      __builtin_amdgcn_sched_barrier(0);
      JR_ST(const unsigned long long tw = stamp.now();)
      wait_vmcnt(per_tile * max(0, min(NBUF - 2, kt1 - kt - 2)));
      __builtin_amdgcn_s_barrier();
      JR_ST(stamp.w += stamp.now() - tw;)
      __builtin_amdgcn_sched_barrier(0);
      cur = cur + 1 == NBUF ? 0 : cur + 1;
    }
  }
  JR_ST(stamp.loop();)
  if constexpr (H6) {        // back from the operands' power-of-two scales (exact)
    const float ia = 1.f / h_sa, ib = 1.f / h_sb;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = acc[i][j][r] * ia * ib;
  }

  if constexpr (SK) {
    sk_first = false;
    int owner, npieces, kind;
    if (sk_cut(g, tile, kt0, kt1, &owner, &npieces, &kind) &&
        !sk_handoff<TM, TN>(g, acc, wave, lane, owner, npieces, kind, lb))
      continue;                      // another block finishes the tile
  }
  // ---------------------------------------------------------------- epilogue
  conv_epilogue<OP, WM, TM, TN, false>(g, acc, smem + wave * stage_floats<WN>(), m0 + wm0, n0 + wn0, lane);
  if constexpr (!SK) break;
  }
  JR_ST(stamp.end(g.dbg);)
}

// ---------------------------------------------------------------- host side

struct Phase {
  int py, px, r0, c0, na, nb, ey, ex, hc, wc;
};

// A config id is tile | (splits << 8): splits == 0 lets the planner pick
// the split-K factor, otherwise it is forced (autotuning explores both).
constexpr int kSplitShift = 8;
// split-K factors up to 1024: the stem filter gradients (3 tiles of M = 288,
// K = 1.4 M pixels) still gain from 256 to 512 slabs (more resident blocks)
constexpr int kMaxSplits = 1024;
static int cfg_tile(int cfg) { return cfg & ((1 << kSplitShift) - 1); }
static int cfg_splits(int cfg) { return cfg >> kSplitShift; }

struct Plan {
  int cfg;   // encoded id
  int tile;
  int M, N, K;
  int mt, nt, ktiles, splits, kt_per_split;
  // stream-K (k_conv SK): blocks and iterations (tiles x K-tiles) per block
  bool sk;
  int sk_blocks;
  long long sk_ipb;
  int sk_slot;   // floats of one block's partial (BM x BN)
};

// Channel padding of the reduction operand: 16 B DMA pieces hold 4 fp32 or
// 8 bf16 channels.
static bool bf16_operands(int dtype) { return dtype == JR_BF16 || dtype == JR_F32_X8P; }
// JR_F32_X6H shares JR_F32_X8's tiles, config ids and plans (its kernels
// differ only in the split: fp16, six products, scaled operands)
static bool x8_family(int dtype) { return dtype == JR_F32_X8 || dtype == JR_F32_X6H; }
static int chan_pad(int c, int dtype) {
  const int q = bf16_operands(dtype) ? 8 : 4;
  return (c + q - 1) / q * q;
}
// GEMM tiles of a dtype (the planner heuristic ranks these), and every
// selectable config: for JR_BF16 the halo-tiled FWD configs follow them.
static int std_count(int dtype) {
  return dtype == JR_BF16 ? kNumCfgsBf16 : dtype == JR_F32_X8P ? kNumCfgsX8P : kNumCfgs;
}
// JR_F32_X8 also selects the fp32-MFMA kernel of every fp32 tile (ids
// kNumCfgs + t): both are fp32-accurate, and on the stem's N = 32 / 64
// filter-gradient GEMMs, whose per-wave split VALU outweighs the 8-product
// MFMA gain, the fp32 MFMA is the faster one -- autotuning and the pinned
// tables choose per GEMM (the planner heuristic keeps x8).
// JR_BF16 ids: [0, 17) GEMM tiles, [17, 25) halo configs, then the wide
// (8-wave) tiles, then the stream-K grids of the GEMM tiles and of the wide
// tiles (k_conv_bf16 SK); JR_F32_X8P: [0, 17) tiles, then the wide ones (new
// ids are appended so committed tile tables keep their meaning).
static int wide_base(int dtype) {
  return dtype == JR_BF16 ? kNumCfgsBf16 + kNumHaloBf16 : dtype == JR_F32_X8P ? kNumCfgsX8P : 1 << 20;
}
static int wide_count(int dtype) {
  return dtype == JR_BF16 ? kNumCfgsBf16W : dtype == JR_F32_X8P ? kNumCfgsX8PW : 0;
}
// first stream-K id: JR_F32_X8 [28, 42) = the stream-K grid of x8 tile
// (id - 28) (k_conv SK); JR_BF16 see above
static int sk_base(int dtype) {
  return x8_family(dtype) ? 2 * kNumCfgs : dtype == JR_BF16 ? wide_base(dtype) + kNumCfgsBf16W : 1 << 20;
}
static int cfg_count(int dtype) {
  return dtype == JR_BF16 ? sk_base(dtype) + kNumCfgsBf16 + kNumCfgsBf16W
         : dtype == JR_F32_X8P ? wide_base(dtype) + kNumCfgsX8PW
         : x8_family(dtype) ? 3 * kNumCfgs
         : std_count(dtype);
}
static bool is_halo(int dtype, int tile) {
  return dtype == JR_BF16 && tile >= kNumCfgsBf16 && tile < kNumCfgsBf16 + kNumHaloBf16;
}
static bool is_wide(int dtype, int tile) { return tile >= wide_base(dtype) && tile < wide_base(dtype) + wide_count(dtype); }
static bool is_x8_f32(int dtype, int tile) { return x8_family(dtype) && tile >= kNumCfgs && tile < 2 * kNumCfgs; }
static bool is_sk(int dtype, int tile) { return tile >= sk_base(dtype) && tile < cfg_count(dtype); }
// the (non-stream-K) id whose tile a stream-K id runs
static int sk_tile(int dtype, int tile) {
  const int k = tile - sk_base(dtype);
  return dtype == JR_BF16 && k >= kNumCfgsBf16 ? wide_base(dtype) + k - kNumCfgsBf16 : k;
}
static const TileCfg& tile_cfg(int dtype, int tile) {
  if (is_sk(dtype, tile)) tile = sk_tile(dtype, tile);
  if (is_halo(dtype, tile)) return kHaloBf16[tile - kNumCfgsBf16].t;
  if (is_wide(dtype, tile)) return (dtype == JR_BF16 ? kCfgsBf16W : kCfgsX8PW)[tile - wide_base(dtype)];
  if (is_x8_f32(dtype, tile)) return kCfgs[tile - kNumCfgs];
  return (dtype == JR_BF16 ? kCfgsBf16 : dtype == JR_F32_X8P ? kCfgsX8P : kCfgs)[tile];
}
// Halo rows a BM-row tile needs: output rows it spans (bound) + kh - 1.
static int halo_rows(const jr_conv_desc* d, int bm) { return (bm + d->wo - 2) / d->wo + 1 + d->kh - 1; }
static bool halo_ok(const jr_conv_desc* d, int op, int dtype, int tile) {
  if (!is_halo(dtype, tile) || op != OP_FWD) return false;
  const HaloCfg& h = kHaloBf16[tile - kNumCfgsBf16];
  return d->kh == h.kh && d->kw == h.kw && d->stride_h == 1 && d->stride_w == 1 && d->ho == d->h &&
         d->wo == d->w && d->c_in % 32 == 0 && halo_rows(d, h.t.bm) * (d->w + d->kw - 1) < h.slots;
}

static void dgrad_phases(const jr_conv_desc* d, Phase* ph, int* nph) {
  int k = 0;
  for (int py = 0; py < d->stride_h; ++py) {
    for (int px = 0; px < d->stride_w; ++px) {
      Phase p{};
      p.py = py; p.px = px;
      p.hc = py < d->h ? (d->h - py + d->stride_h - 1) / d->stride_h : 0;
      p.wc = px < d->w ? (d->w - px + d->stride_w - 1) / d->stride_w : 0;
      p.r0 = (py + d->pad_h) % d->stride_h;
      p.c0 = (px + d->pad_w) % d->stride_w;
      p.na = p.r0 < d->kh ? (d->kh - p.r0 + d->stride_h - 1) / d->stride_h : 0;
      p.nb = p.c0 < d->kw ? (d->kw - p.c0 + d->stride_w - 1) / d->stride_w : 0;
      p.ey = (py + d->pad_h - p.r0) / d->stride_h;
      p.ex = (px + d->pad_w - p.c0) / d->stride_w;
      ph[k++] = p;
    }
  }
  *nph = k;
}

constexpr int kSkBlocks = 512;     // stream-K grid: 2 x 256 CUs
constexpr int kSkMinIters = 4;     // K-tiles per stream-K block at least

// Blocks the planner's split-K factor aims for (>= 2.5 per CU). x8 filter
// gradients aim for 384: their slabs are summed per layer on the GEMM's lane
// (the fp32 engine default), and fewer slabs measured 0.12-0.14 ms per step
// faster on two boxes (profiles/r05_ab_wsplit*_f32.txt; 320 / 1,024 slower,
// bf16 at 384 slower). JR_WGRAD_SPLIT_TARGET overrides it (A/B knob, read once).
// JR_WGRAD_SPLIT_KMAX (A/B knob, read once): x8 filter gradients aim for 384
// only where K = B.Ho.Wo is at most this, 640 above it (round 5's
// K-bounded rule: faster at 299^2 and 587^2, moved the B=16 fp32 curve
// past the round-5 bar; re-judged against the calibrated bars).
static int split_target(int dtype, int op, long long K) {
  static const int wg = [] {
    const char* e = std::getenv("JR_WGRAD_SPLIT_TARGET");
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? v : 0;
  }();
  static const long long kmax = [] {
    const char* e = std::getenv("JR_WGRAD_SPLIT_KMAX");
    const long long v = e ? std::atoll(e) : 0;
    return v > 0 ? v : 0LL;
  }();
  if (op != OP_WGRAD) return 640;
  if (wg > 0) return wg;
  if (x8_family(dtype) || dtype == JR_F32_X8P) return kmax > 0 && K > kmax ? 640 : 384;
  return 640;
}

static Plan plan_with(int dtype, int cfg, int M, int N, int K, int op) {
  Plan p{};
  p.M = M; p.N = N; p.K = K; p.cfg = cfg; p.tile = cfg_tile(cfg);
  const TileCfg& t = tile_cfg(dtype, p.tile);
  p.mt = (int)ceil_div(M, t.bm);
  p.nt = (int)ceil_div(N, t.bn);
  p.ktiles = (int)ceil_div(K, t.bk);
  const int tiles = p.mt * p.nt;
  int splits = 1;
  const int target = split_target(dtype, op, K);
  if (tiles < target) {
    splits = (int)ceil_div(target, tiles);
    const int max_by_k = std::max(1, p.ktiles / 8);
    splits = std::min(std::min(splits, max_by_k), 256);
  }
  if (cfg_splits(cfg) > 0) splits = std::min(cfg_splits(cfg), std::max(p.ktiles, 1));
  if (is_sk(dtype, p.tile)) {
    // stream-K: a fixed grid (two blocks per CU at most resident; larger
    // tiles run it in two equal rounds), at least kSkMinIters K-tiles each
    // (the config's split field picks the grid instead: 128 x s blocks, s <= 8)
    const long long grid = cfg_splits(cfg) > 0 ? 128LL * std::min(cfg_splits(cfg), 8) : kSkBlocks;
    splits = 1;
    const long long W = (long long)tiles * std::max(p.ktiles, 1);
    const long long P = std::max(1LL, std::min<long long>(grid, W / kSkMinIters));
    p.sk = true;
    p.sk_ipb = ceil_div(W, P);
    p.sk_blocks = (int)ceil_div(W, p.sk_ipb);
    p.sk_slot = t.bm * t.bn;   // two per block: the first segment's piece and the owner's last
  }
  p.kt_per_split = (int)ceil_div(std::max(p.ktiles, 1), splits);
  p.splits = (int)ceil_div(std::max(p.ktiles, 1), p.kt_per_split);
  return p;
}

static int heuristic_cfg(int dtype, int M, int N, int K) {
  double best = 1e300;
  int bc = 0;
  for (int c = 0; c < std_count(dtype); ++c) {
    const TileCfg& t = tile_cfg(dtype, c);
    const double tiles = (double)ceil_div(M, t.bm) * ceil_div(N, t.bn);
    double work = tiles * t.bm * t.bn / t.eff;
    // grids that cannot fill the 256 CUs and cannot be split along K lose
    if (tiles < 256 && ceil_div(K, t.bk) < 32) work *= 256.0 / tiles;
    if (work < best * 0.999) { best = work; bc = c; }
  }
  return bc;
}

// Autotune cache: (op, GEMM dims, conv geometry) -> best config.
typedef std::array<int, 13> TuneKey;
static std::mutex g_tune_mu;
static std::map<TuneKey, int> g_tuned;
// bumped whenever an entry of g_tuned changes value (set_config, autotune):
// a caller that bound plans (split-K slab sizes) to the overrides it applied
// re-applies them when the generation moved (jr_conv2d_config_generation)
static unsigned long long g_tune_gen = 1;
static void tune_set(const TuneKey& k, int cfg) {   // g_tune_mu held; cfg < 0 erases
  auto it = g_tuned.find(k);
  if (cfg < 0) {
    if (it != g_tuned.end()) { g_tuned.erase(it); ++g_tune_gen; }
  } else if (it == g_tuned.end() || it->second != cfg) {
    g_tuned[k] = cfg;
    ++g_tune_gen;
  }
}

static TuneKey tune_key(int dtype, int op, int M, int N, int K, const jr_conv_desc* d) {
  return TuneKey{dtype, op, M, N, K, d->h, d->w, d->kh, d->kw, d->stride_h, d->c_in, d->c_out, d->n};
}

static Plan make_plan(int dtype, int op, int M, int N, int K, const jr_conv_desc* d, int force_cfg = -1) {
  int cfg = force_cfg;
  if (cfg < 0) {
    std::lock_guard<std::mutex> lk(g_tune_mu);
    auto it = g_tuned.find(tune_key(dtype, op, M, N, K, d));
    if (it != g_tuned.end()) cfg = it->second;
  }
  // a halo config (tuned, pinned or forced) only where its geometry holds
  if (cfg < 0 || (is_halo(dtype, cfg_tile(cfg)) && !halo_ok(d, op, dtype, cfg_tile(cfg))))
    cfg = heuristic_cfg(dtype, M, N, K);
  return plan_with(dtype, cfg, M, N, K, op);
}

// z-lanes per float4 column of the split-K reduce (k_splitk_reduce and the
// deferred k_wgrad_reduce: the same G gives the same summation order)
static int reduce_lanes(const Plan& p) {
  const long long total = (long long)p.M * p.N / 4;
  int G = 1;
  while (G < 64 && G * 4 <= p.splits && total * G < 128 * 1024) G *= 2;
  return G;
}

// stream-K: one BM x BN fp32 partial slot per block (the hand-off flags are
// stream_scratch words)
static size_t plan_ws(const Plan& p) {
  if (p.sk) return 2 * (size_t)p.sk_blocks * p.sk_slot * sizeof(float);
  return p.splits > 1 ? (size_t)p.splits * (size_t)p.M * (size_t)p.N * sizeof(float) : 0;
}

// Fused BN statistics (FWD): partials of R rows each, P per column.  Without
// split-K the GEMM epilogue writes one per wave row-group (R = WM); with it,
// k_splitk_reduce_stats one per block of R rows (~512 blocks).
struct StatsReq {
  float eps;
  float* mean;
  float* invstd;
  bool defer = false;   // leave the single-stage partials in ws for jr_bn_relu_apply_stats
};

static void stats_geom(int dtype, const Plan& p, int* P, int* R) {
  const TileCfg& t = tile_cfg(dtype, p.tile);
  if (p.splits <= 1) {
    *R = t.bm / t.wgm;
    *P = p.mt * t.wgm;
    return;
  }
  const int rpp = 256 / (std::min(p.N, 1024) / 4);
  int r = std::max<int>(rpp, (int)ceil_div(p.M, 512));
  r = (int)ceil_div(r, rpp) * rpp;
  *R = r;
  *P = (int)ceil_div(p.M, r);
}

static size_t align256(size_t b) { return (b + 255) / 256 * 256; }

#ifndef JR_STATS_CHUNK
#define JR_STATS_CHUNK 4096
#endif
constexpr int kStatsChunk = JR_STATS_CHUNK;   // partials one finalize block combines

static size_t stats_ws(int dtype, const Plan& p) {
  int P, R;
  stats_geom(dtype, p, &P, &R);
  const size_t S = P > kStatsChunk ? (size_t)ceil_div(P, kStatsChunk) : 0;
  return (2 * (size_t)p.N * P + 3 * (size_t)p.N * S) * sizeof(float);
}

// Fast-path kernels (UT): FWD/DGRAD when the reduction channel radix is a
// multiple of BK (every layer but conv1 FWD at BK = 16); WGRAD when BK / wo < ho
// (one carry per radix and K-tile: the incremental pixel walk).
template <int OP, int C, int DBG, bool X8, bool SK, bool H6 = false>
static void launch_cfg(const ConvArgs& a, dim3 grid, hipStream_t s) {
  constexpr TileCfg t = kCfgs[C];
  const bool fast = OP == OP_WGRAD ? t.bk / a.wo < a.ho : (OP == OP_FWD ? a.cp : a.cout) % t.bk == 0;
  if (fast) {
    hipLaunchKernelGGL((k_conv<OP, t.bm, t.bn, t.wgm, t.bk, t.nbuf, true, X8, DBG, SK, H6>), grid, dim3(256), 0, s, a);
    return;
  }
  if constexpr (DBG == 0)
    hipLaunchKernelGGL((k_conv<OP, t.bm, t.bn, t.wgm, t.bk, t.nbuf, false, X8, 0, SK, H6>), grid, dim3(256), 0, s, a);
}

// SK: the stream-K grid (k_conv SK) of the tile
template <int OP, int DBG = 0, bool X8 = false, bool SK = false, bool H6 = false>
static void launch_op(int cfg, const ConvArgs& a, dim3 grid, hipStream_t s) {
  switch (cfg) {
    case 0: launch_cfg<OP, 0, DBG, X8, SK, H6>(a, grid, s); break;
    case 1: launch_cfg<OP, 1, DBG, X8, SK, H6>(a, grid, s); break;
    case 2: launch_cfg<OP, 2, DBG, X8, SK, H6>(a, grid, s); break;
    case 3: launch_cfg<OP, 3, DBG, X8, SK, H6>(a, grid, s); break;
    case 4: launch_cfg<OP, 4, DBG, X8, SK, H6>(a, grid, s); break;
    case 5: launch_cfg<OP, 5, DBG, X8, SK, H6>(a, grid, s); break;
    case 6: launch_cfg<OP, 6, DBG, X8, SK, H6>(a, grid, s); break;
    case 7: launch_cfg<OP, 7, DBG, X8, SK, H6>(a, grid, s); break;
    case 8: launch_cfg<OP, 8, DBG, X8, SK, H6>(a, grid, s); break;
    case 9: launch_cfg<OP, 9, DBG, X8, SK, H6>(a, grid, s); break;
    case 10: launch_cfg<OP, 10, DBG, X8, SK, H6>(a, grid, s); break;
    case 11: launch_cfg<OP, 11, DBG, X8, SK, H6>(a, grid, s); break;
    case 12: launch_cfg<OP, 12, DBG, X8, SK, H6>(a, grid, s); break;
    default: launch_cfg<OP, 13, DBG, X8, SK, H6>(a, grid, s); break;
  }
}


static int validate(const jr_conv_desc* d, int op, int dtype) {
  if (dtype != JR_F32 && dtype != JR_BF16 && dtype != JR_F32_X8 && dtype != JR_F32_X8P && dtype != JR_F32_X6H)
    return fail(JR_ERR_INVALID, "conv: bad dtype");
  const int q = bf16_operands(dtype) ? 8 : 4;   // channels per 16 B piece
  if (!d) return fail(JR_ERR_INVALID, "conv: null descriptor");
  if (op < OP_FWD || op > OP_WGRAD) return fail(JR_ERR_INVALID, "conv: bad op");
  if (d->n <= 0 || d->h <= 0 || d->w <= 0 || d->c_in <= 0 || d->c_out <= 0 || d->kh <= 0 ||
      d->kw <= 0 || d->stride_h <= 0 || d->stride_w <= 0 || d->pad_h < 0 || d->pad_w < 0)
    return fail(JR_ERR_INVALID, "conv: non-positive dimension");
  const int ho = (d->h + 2 * d->pad_h - d->kh) / d->stride_h + 1;
  const int wo = (d->w + 2 * d->pad_w - d->kw) / d->stride_w + 1;
  if (ho != d->ho || wo != d->wo || ho <= 0 || wo <= 0)
    return fail(JR_ERR_INVALID, "conv: ho/wo inconsistent with h,w,k,stride,pad");
  if (d->pad_h >= d->kh || d->pad_w >= d->kw)
    return fail(JR_ERR_INVALID, "conv: padding must be smaller than the kernel");
  const int cp = chan_pad(d->c_in, dtype);
  if (d->x_c_off < 0 || d->x_c_off + cp > d->x_c_stride)
    return fail(JR_ERR_INVALID, "conv: input channel slice (padded to 4 fp32 / 8 bf16 channels) out of range");
  if (d->y_c_off < 0 || d->y_c_off + d->c_out > d->y_c_stride)
    return fail(JR_ERR_INVALID, "conv: output channel slice out of range");
  if (d->c_out % 16 != 0)
    return fail(JR_ERR_UNSUPPORTED, "conv: c_out must be a multiple of 16");
  if (d->x_c_off % q || d->x_c_stride % q || d->y_c_off % q || d->y_c_stride % q)
    return fail(JR_ERR_INVALID, "conv: channel offsets and strides must be multiples of 4 (fp32) / 8 (bf16)");
  if (op == OP_DGRAD && d->c_in % q != 0)
    return fail(JR_ERR_UNSUPPORTED, "conv bwd_data: c_in must be a multiple of 4 (fp32) / 8 (bf16)");
  if (d->stride_h * d->stride_w > 64) return fail(JR_ERR_UNSUPPORTED, "conv: stride too large");
  const long long xin = (long long)d->n * d->h * d->w * d->x_c_stride;
  const long long yout = (long long)d->n * d->ho * d->wo * d->y_c_stride;
  const long long wsz = (long long)d->kh * d->kw * d->c_in * d->c_out;
  if (xin >= (1LL << 31) || yout >= (1LL << 31) || wsz >= (1LL << 31))
    return fail(JR_ERR_INVALID, "conv: tensor too large for 32-bit element offsets");
  return JR_OK;
}

static void fill_common(ConvArgs& a, const jr_conv_desc* d, int dtype) {
  a.n = d->n; a.h = d->h; a.w = d->w; a.cin = d->c_in; a.cp = chan_pad(d->c_in, dtype); a.cout = d->c_out;
  a.kh = d->kh; a.kw = d->kw; a.sh = d->stride_h; a.sw = d->stride_w;
  a.ph = d->pad_h; a.pw = d->pad_w; a.ho = d->ho; a.wo = d->wo;
  a.xo = d->x_c_off; a.xs = d->x_c_stride; a.yo = d->y_c_off; a.ys = d->y_c_stride;
}

// JR_F32_X6H: the magnitude bounds of the op's A and B operands (FWD x, w;
// DGRAD dy, w; WGRAD x, dy) from the descriptor
static void fill_scales(ConvArgs& a, const jr_conv_desc* d, int op, int dtype) {
  if (dtype != JR_F32_X6H) return;
  const float* xm = d->x_absmax;  const float xb = d->x_bound;
  const float* wm = d->w_absmax;  const float wb = d->w_bound;
  const float* gm = d->dy_absmax; const float gb = d->dy_bound;
  if (op == OP_FWD) { a.a_max = xm; a.a_bnd = xb; a.b_max = wm; a.b_bnd = wb; }
  else if (op == OP_DGRAD) { a.a_max = gm; a.a_bnd = gb; a.b_max = wm; a.b_bnd = wb; }
  else { a.a_max = xm; a.a_bnd = xb; a.b_max = gm; a.b_bnd = gb; }
}

#ifdef JR_STAMPS
static unsigned long long* g_dbg_stamps = nullptr;
// diagnostic builds: every following conv GEMM launch writes 8 stamps per
// block into p (ConvArgs::dbg; the caller sizes it for the grid)
JR_API int jr_debug_set_stamps(void* p) {
  g_dbg_stamps = static_cast<unsigned long long*>(p);
  return JR_OK;
}
#endif

// One GEMM (plus its split-K reduce) on the stream.
// defer (WGRAD): write the split-K slabs into ws and stop (jr_wgrad_reduce
// sums them later, batched with other layers').
// Workspace of one member of a grouped GEMM: split-K slabs, then the fused
// BN statistics partials (their two-stage combine space included).
static size_t member_ws(int dtype, const Plan& p, bool stats) {
  return align256(stats ? align256(plan_ws(p)) + stats_ws(dtype, p) : plan_ws(p));
}

// (mean, invstd) from the statistics partials [2][N][P] of R rows each
// (member stride pm bytes): P <= kFoldMaxP -- k_stats_finalize8, the
// arithmetic jr_bn_relu_apply_stats shares (st->defer: left to it); P <=
// kStatsChunk -- one 256-thread combine per channel; else two stages.
static int finalize_stats(float* stats, int sP, int sR, int M, int N, int members, long long pm, const StatsReq* st,
                          long long st_mb, hipStream_t s) {
  if (sP <= kFoldMaxP) {
    if (st->defer) return JR_OK;          // the BN apply combines them (jr_bn_relu_apply_stats)
    hipLaunchKernelGGL(k_stats_finalize8, dim3((int)ceil_div(N, 256 / kStatsLanes), 1, members), dim3(256), 0, s,
                       (const float*)stats, sP, sR, M, N, st->eps, st->mean, st->invstd, pm, st_mb);
  } else if (st->defer) {
    return fail(JR_ERR_UNSUPPORTED, "conv fwd partials: more than kFoldMaxP statistics partials cannot be deferred");
  } else if (sP <= kStatsChunk) {
    hipLaunchKernelGGL(k_stats_finalize, dim3(N, 1, members), dim3(256), 0, s, (const float*)stats,
                       (const float*)nullptr, sP, sR, M, N, sP, st->eps, st->mean, st->invstd, (float*)nullptr, pm,
                       st_mb);
  } else {   // two stages: per-chunk (mean, M2, n), then the final combine
    const int S = (int)ceil_div(sP, kStatsChunk);
    float* s2 = stats + 2 * (size_t)N * sP;
    hipLaunchKernelGGL(k_stats_finalize, dim3(N, S, members), dim3(256), 0, s, (const float*)stats,
                       (const float*)nullptr, sP, sR, M, N, kStatsChunk, st->eps, (float*)nullptr, (float*)nullptr, s2,
                       pm, st_mb);
    const int rc = check_launch("conv stats combine");
    if (rc) return rc;
    hipLaunchKernelGGL(k_stats_finalize, dim3(N, 1, members), dim3(256), 0, s, (const float*)s2,
                       (const float*)(s2 + 2 * (size_t)N * S), S, 0, M, N, S, st->eps, st->mean, st->invstd,
                       (float*)nullptr, pm, st_mb);
  }
  return check_launch("conv stats finalize");
}

// conv2d_1 as the direct kernel (jr_conv_direct.hip), its statistics
// partials at ws (member m at ws + m * wsm) and finalized as any GEMM's.
static size_t conv1_direct_ws(const jr_conv_desc* d) {
  int P, R;
  conv1_direct_partials(d, &P, &R);
  return align256((size_t)2 * d->c_out * P * sizeof(float));
}

static int run_conv1_direct(const jr_conv_desc* d, int dtype, const void* x, const void* w, void* y, void* ws,
                            size_t ws_bytes, hipStream_t s, const StatsReq* st, int members = 1, long long x_mb = 0,
                            long long w_mb = 0, long long y_mb = 0, long long st_mb = 0) {
  int P, R;
  conv1_direct_partials(d, &P, &R);
  const size_t wsm = conv1_direct_ws(d);
  if (st && (!ws || ws_bytes < wsm * members)) return fail(JR_ERR_WORKSPACE, "conv1 direct: workspace too small");
  float* stats = st ? static_cast<float*>(ws) : nullptr;
  launch_conv1_direct(d, dtype, x, w, y, stats, members, x_mb, w_mb, y_mb, (long long)wsm, s);
  int rc = check_launch("conv1 direct");
  if (rc || !st) return rc;
  const long long M = (long long)d->n * d->ho * d->wo;
  return finalize_stats(stats, P, R, (int)M, d->c_out, members, (long long)wsm, st, st_mb, s);
}

template <int OP>
static int run_gemm(int dtype, ConvArgs a, const Plan& p, void* out, void* ws, size_t ws_bytes, hipStream_t s,
                    const StatsReq* st = nullptr, bool defer = false, int members = 1, long long st_mb = 0) {
  if (p.M <= 0 || p.N <= 0) return JR_OK;
  // grouped (members > 1): every member's GEMM in one launch (blockIdx.y),
  // each with its own workspace region of member_ws bytes; a.a_mb / b_mb /
  // o_mb (operand and output strides) are the caller's
  const size_t wsm = members > 1 ? member_ws(dtype, p, st != nullptr) : 0;
  if (members > 1 && (!ws || ws_bytes < wsm * members) && (p.splits > 1 || st))
    return fail(JR_ERR_WORKSPACE, "conv grouped: workspace too small (jr_conv2d_workspace_size_grouped)");
  int sP = 0, sR = 0;
  if (st) {
    stats_geom(dtype, p, &sP, &sR);
    const size_t off = align256(plan_ws(p));
    if (!ws || ws_bytes < off + stats_ws(dtype, p)) return fail(JR_ERR_WORKSPACE, "conv: workspace too small for BN statistics");
    a.stats = reinterpret_cast<float*>(static_cast<char*>(ws) + off);
    a.stats_p = sP;
    a.s_mb = (long long)wsm;
  }
  a.M = p.M; a.N = p.N; a.K = p.K;
  JR_ST(a.dbg = g_dbg_stamps;)
  a.ktiles = p.ktiles;
  a.kt_per_split = p.kt_per_split;
  a.ntn = p.nt;
  a.slab_elems = (long long)p.M * p.N;
  if (p.splits > 1) {
    if (!ws || ws_bytes < plan_ws(p)) return fail(JR_ERR_WORKSPACE, "conv: workspace too small for split-K");
    a.C = static_cast<float*>(ws);
    a.c_mb = (long long)wsm;
  } else {
    a.C = static_cast<float*>(out);
    a.c_mb = a.o_mb;
  }
  dim3 grid(p.mt * p.nt, members, p.splits);
  if (p.sk) {
    if (!ws || ws_bytes < plan_ws(p) + (members > 1 ? (size_t)(members - 1) * wsm : 0))
      return fail(JR_ERR_WORKSPACE, "conv: workspace too small for the stream-K hand-off");
    a.sk_ipb = p.sk_ipb;
    a.sk_part = static_cast<float*>(ws);
    a.sk_mb = (long long)wsm;
    // the flags: zero at launch without a memset (every flag a block sets is
    // reset by the one block that absorbs it)
    a.sk_flags = stream_scratch(s, 0, (size_t)p.sk_blocks * members);
    if (!a.sk_flags) return fail(JR_ERR_HIP, "conv: stream-K flag words could not be allocated");
    a.sk_fmb = (long long)p.sk_blocks * sizeof(unsigned);
    // a hand-off count found past its piece count (a word not left zero) is reported here
    a.sk_err = device_error_word(s);
    if (!a.sk_err) return fail(JR_ERR_HIP, "conv: no device error word (call jr_init before capturing)");
    grid = dim3(p.sk_blocks, members, 1);
  }
  if (is_halo(dtype, p.tile)) {
    const HaloCfg& h = kHaloBf16[p.tile - kNumCfgsBf16];
    a.halo_wp = a.w + a.kw - 1;
    a.halo_nr = (h.t.bm + a.wo - 2) / a.wo + 1 + a.kh - 1;
    launch_conv_halo(p.tile - kNumCfgsBf16, a, grid, s);
  } else if (bf16_operands(dtype)) {
    // operand address mode (k_conv_bf16 AM): the tap is wave-uniform when the
    // reduction channel radix is a multiple of BK (0), else every piece walks
    // its own address with at most one carry per radix and K-tile (1), else
    // the mixed-radix loop (2: conv1's 8 channels; WGRAD on images shorter
    // than BK / wo rows)
    const TileCfg& t = tile_cfg(dtype, p.tile);
    int am;
    if (OP == OP_WGRAD) {
      am = t.bk / a.wo < a.ho ? 1 : 2;
    } else {
      const int cred = OP == OP_FWD ? a.cp : a.cout;
      am = cred % t.bk == 0 ? 0 : cred >= t.bk ? 1 : 2;
    }
    if (p.sk) {   // the stream-K grid of a standard or wide JR_BF16 tile
      const int tt = sk_tile(dtype, p.tile);
      const bool w = is_wide(dtype, tt);
      launch_conv_bf16_sk(OP, w ? tt - wide_base(dtype) : tt, w, am, a, grid, s);
    } else if (is_wide(dtype, p.tile))
      launch_conv_bf16_wide(OP, p.tile - wide_base(dtype), am, a, grid, s, dtype == JR_F32_X8P ? 3 : 1);
    else
      launch_conv_bf16(OP, p.tile, am, a, grid, s, dtype == JR_F32_X8P ? 3 : 1);
  } else if (is_x8_f32(dtype, p.tile)) {
    launch_op<OP>(p.tile - kNumCfgs, a, grid, s);     // the fp32-MFMA kernel of that tile
  } else if (p.sk && dtype == JR_F32_X6H) {
    launch_op<OP, 0, true, true, true>(p.tile - 2 * kNumCfgs, a, grid, s);   // stream-K grid, fp16 six products
  } else if (p.sk) {
    launch_op<OP, 0, true, true>(p.tile - 2 * kNumCfgs, a, grid, s);   // the stream-K grid of that x8 tile
  } else if (dtype == JR_F32_X6H) {
    launch_op<OP, 0, true, false, true>(p.tile, a, grid, s);
  } else if (dtype == JR_F32_X8) {
    launch_op<OP, 0, true>(p.tile, a, grid, s);
  } else {
    launch_op<OP>(p.tile, a, grid, s);
  }
  int rc = check_launch("conv gemm");
  if (rc) return rc;
  if (st) {
    if (p.splits > 1) {
      const dim3 rg(sP, (int)ceil_div(p.N, 1024), members);
      if (dtype == JR_BF16)
        hipLaunchKernelGGL((k_splitk_reduce_stats<uint16_t>), rg, dim3(256), 0, s, (const float*)ws, p.splits, a,
                           static_cast<uint16_t*>(out), sR);
      else
        hipLaunchKernelGGL((k_splitk_reduce_stats<float>), rg, dim3(256), 0, s, (const float*)ws, p.splits, a,
                           static_cast<float*>(out), sR);
      rc = check_launch("conv split-k reduce + stats");
      if (rc) return rc;
    }
    return finalize_stats(a.stats, sP, sR, p.M, p.N, members, (long long)wsm, st, st_mb, s);
  }
  if (members > 1) return fail(JR_ERR_UNSUPPORTED, "conv grouped: forward with BN statistics only");
  if (p.splits <= 1 || defer) return rc;
  const long long total = (long long)p.M * p.N / 4;   // float4 columns
  const int G = reduce_lanes(p);                       // z-lanes per column
  const long long cols = 256 / G;
  const int blocks = (int)std::min<long long>(ceil_div(total, cols), 8192);
  if (dtype == JR_BF16 && OP != OP_WGRAD)   // bf16 activations / activation grads; dW stays fp32
    hipLaunchKernelGGL((k_splitk_reduce<OP, uint16_t>), dim3(blocks), dim3(256), 0, s, (const float*)ws, p.splits,
                       G, a, static_cast<uint16_t*>(out));
  else
    hipLaunchKernelGGL((k_splitk_reduce<OP, float>), dim3(blocks), dim3(256), 0, s, (const float*)ws, p.splits, G,
                       a, static_cast<float*>(out));
  return check_launch("conv split-k reduce");
}

static void gemm_dims(const jr_conv_desc* d, int op, int dtype, const Phase* ph, int* M, int* N, int* K) {
  const int cp = chan_pad(d->c_in, dtype);
  if (op == OP_FWD) { *M = d->n * d->ho * d->wo; *N = d->c_out; *K = d->kh * d->kw * cp; }
  else if (op == OP_WGRAD) { *M = d->kh * d->kw * cp; *N = d->c_out; *K = d->n * d->ho * d->wo; }
  else { *M = d->n * ph->hc * ph->wc; *N = d->c_in; *K = ph->na * ph->nb * d->c_out; }
}

static Plan plan_for(const jr_conv_desc* d, int op, int dtype, const Phase* ph, int force_cfg = -1) {
  int M, N, K;
  gemm_dims(d, op, dtype, ph, &M, &N, &K);
  return make_plan(dtype, op, M, N, K, d, force_cfg);
}

// Workspace: twice the max over every candidate tile's planned split-K, so
// any tuned choice fits.
static size_t ws_bytes_for(const jr_conv_desc* d, int op, int dtype) {
  Phase ph[64];
  int nph = 1;
  if (op == OP_DGRAD) dgrad_phases(d, ph, &nph);
  size_t w = 0, sw = 0;
  for (int i = 0; i < nph; ++i) {
    if (op == OP_DGRAD && (ph[i].na == 0 || ph[i].nb == 0 || ph[i].hc == 0 || ph[i].wc == 0)) continue;
    for (int c = 0; c < cfg_count(dtype); ++c) {
      const Plan p = plan_for(d, op, dtype, op == OP_DGRAD ? &ph[i] : nullptr, c);
      w = std::max(w, plan_ws(p));
      if (op == OP_FWD) {   // fused BN statistics partials, split or not
        Plan p1 = p;
        p1.splits = 1;
        sw = std::max(sw, std::max(stats_ws(dtype, p), stats_ws(dtype, p1)));
      }
    }
  }
  // 2x: room for the autotuner's doubled split-K factors; FWD: the statistics
  // partials live behind the slabs (or, conv2d_1's direct kernel, at 0)
  if (op == OP_FWD && conv1_direct_ok(d, dtype)) sw = std::max(sw, conv1_direct_ws(d));
  return op == OP_FWD ? align256(2 * w) + sw : 2 * w;
}

// DGRAD plan of one stride phase as run_conv launches it (a phase no tap
// reaches is a K = 0 GEMM that stores zeros).  ok = false: nothing to launch.
static Plan dgrad_phase_plan(const jr_conv_desc* d, int dtype, const Phase& p, int force_cfg, bool* ok) {
  *ok = p.hc > 0 && p.wc > 0;
  if (p.na == 0 || p.nb == 0) {
    const int M = d->n * p.hc * p.wc;
    Plan pl = plan_with(dtype, heuristic_cfg(dtype, M, d->c_in, 16), M, d->c_in, 16, OP_DGRAD);
    pl.K = 0; pl.ktiles = 0; pl.splits = 1; pl.kt_per_split = 1;
    return pl;
  }
  return plan_for(d, OP_DGRAD, dtype, &p, force_cfg);
}

// Runs the op; force_cfg >= 0 overrides the plan (autotuning).
static int run_conv(const jr_conv_desc* d, int op, int dtype, const void* A, const void* B, void* C,
                    int accumulate, void* ws, size_t ws_bytes, void* stream, int force_cfg = -1,
                    int only_phase = -1, const StatsReq* st = nullptr) {
  int rc = validate(d, op, dtype);
  if (rc) return rc;
  if (!A || !B || !C) return fail(JR_ERR_INVALID, "conv: null tensor pointer");
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15)
    return fail(JR_ERR_INVALID, "conv: tensors must be 16-byte aligned");
  ConvArgs a{};
  fill_common(a, d, dtype);
  fill_scales(a, d, op, dtype);
  a.A = static_cast<const float*>(A);   // bf16 kernels reinterpret
  a.B = static_cast<const float*>(B);
  a.accumulate = accumulate;
  if (dtype == JR_F32_X8P) {   // plane strides = each operand tensor's element count (jr.h)
    const long long xe = (long long)d->n * d->h * d->w * d->x_c_stride;
    const long long ye = (long long)d->n * d->ho * d->wo * d->y_c_stride;
    const long long we = (long long)d->kh * d->kw * d->c_in * d->c_out;                  // HWIO
    const long long wt = (long long)d->c_out * d->kh * d->kw * chan_pad(d->c_in, dtype);  // W^T
    if (op == OP_FWD) { a.a_ps = xe; a.b_ps = wt; }
    else if (op == OP_DGRAD) { a.a_ps = ye; a.b_ps = we; }
    else { a.a_ps = xe; a.b_ps = ye; }
  }
  hipStream_t s = as_stream(stream);
  void* out = C;
  if (op == OP_FWD) {
    if (force_cfg < 0 && conv1_direct_ok(d, dtype)) return run_conv1_direct(d, dtype, A, B, C, ws, ws_bytes, s, st);
    a.c_off = d->y_c_off; a.c_stride = d->y_c_stride;
    return run_gemm<OP_FWD>(dtype, a, plan_for(d, op, dtype, nullptr, force_cfg), out, ws, ws_bytes, s, st);
  }
  if (op == OP_WGRAD) {
    a.c_off = 0; a.c_stride = d->c_out;
    return run_gemm<OP_WGRAD>(dtype, a, plan_for(d, op, dtype, nullptr, force_cfg), out, ws, ws_bytes, s);
  }
  Phase ph[64];
  int nph = 0;
  dgrad_phases(d, ph, &nph);
  a.c_off = d->x_c_off; a.c_stride = d->x_c_stride;
  for (int i = 0; i < nph; ++i) {
    if (only_phase >= 0 && i != only_phase) continue;
    const Phase& p = ph[i];
    bool ok;
    Plan pl = dgrad_phase_plan(d, dtype, p, force_cfg, &ok);
    if (!ok) continue;
    a.py = p.py; a.px = p.px; a.r0 = p.r0; a.c0 = p.c0; a.na = p.na; a.nb = p.nb;
    a.ey = p.ey; a.ex = p.ex; a.hc = p.hc; a.wc = p.wc;
    // no tap reaches this phase: a K = 0 GEMM stores zeros (or leaves dx)
    if ((p.na == 0 || p.nb == 0) && accumulate) continue;
    rc = run_gemm<OP_DGRAD>(dtype, a, pl, out, ws, ws_bytes, s);
    if (rc) return rc;
  }
  return JR_OK;
}

// Time every candidate config of each GEMM of this op (DGRAD: per phase) on
// the caller's buffers (outputs are overwritten) and remember the fastest.
static int autotune(const jr_conv_desc* d, int op, int dtype, const void* A, const void* B, void* C, void* ws,
                    size_t ws_bytes, void* stream, int reps) {
  int rc = validate(d, op, dtype);
  if (rc) return rc;
  Phase ph[64];
  int nph = 1;
  if (op == OP_DGRAD) dgrad_phases(d, ph, &nph);
  hipStream_t s = as_stream(stream);
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
    return fail(JR_ERR_HIP, "autotune: hipEventCreate failed");
  for (int i = 0; i < nph; ++i) {
    if (op == OP_DGRAD && (ph[i].na == 0 || ph[i].nb == 0 || ph[i].hc == 0 || ph[i].wc == 0)) continue;
    int M, N, K;
    gemm_dims(d, op, dtype, op == OP_DGRAD ? &ph[i] : nullptr, &M, &N, &K);
    const int ncfg = cfg_count(dtype);
    int best_c = heuristic_cfg(dtype, M, N, K);
    float best_t = 1e30f;
    auto time_cfg = [&](int c) -> float {
      if (is_halo(dtype, cfg_tile(c)) && !halo_ok(d, op, dtype, cfg_tile(c))) return 1e30f;
      const Plan pc = plan_with(dtype, c, M, N, K, op);
      // FWD runs with the fused BN statistics: their partials must fit too
      if ((op == OP_FWD ? align256(plan_ws(pc)) + stats_ws(dtype, pc) : plan_ws(pc)) > ws_bytes) return 1e30f;
      rc = run_conv(d, op, dtype, A, B, C, 0, ws, ws_bytes, stream, c, op == OP_DGRAD ? i : -1);  // warm-up
      if (rc) return 1e30f;
      (void)hipEventRecord(e0, s);
      for (int r = 0; r < reps && !rc; ++r)
        rc = run_conv(d, op, dtype, A, B, C, 0, ws, ws_bytes, stream, c, op == OP_DGRAD ? i : -1);
      (void)hipEventRecord(e1, s);
      if (rc) return 1e30f;
      if (hipEventSynchronize(e1) != hipSuccess) { rc = fail(JR_ERR_HIP, "autotune: event sync failed"); return 1e30f; }
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      // near-ties go to the plan with fewer split-K slab bytes (fp32 partials
      // written and re-read through HBM, which a back-to-back timing on a hot
      // L2 undercounts): more splits must win by 2 %, fewer may lose by 2 %
      const int ps = pc.splits > 1 ? pc.splits : 0;
      const int bs = best_t < 1e29f ? (plan_with(dtype, best_c, M, N, K, op).splits > 1
                                           ? plan_with(dtype, best_c, M, N, K, op).splits : 0) : 0;
      const float bar = ps > bs ? 0.98f : ps < bs ? 1.02f : 1.0f;
      if (ms < best_t * bar) { best_t = ms; best_c = c; }
      return ms;
    };
    // pass 1: every tile with the planner's split-K factor
    std::vector<float> tile_t(ncfg);
    for (int c = 0; c < ncfg && !rc; ++c) tile_t[c] = time_cfg(c);
    // pass 2: the three fastest tiles with other split-K factors
    for (int pick = 0; pick < 3 && !rc; ++pick) {
      int c = -1;
      for (int k = 0; k < ncfg; ++k)
        if (tile_t[k] < 1e29f && (c < 0 || tile_t[k] < tile_t[c])) c = k;
      if (c < 0) break;
      tile_t[c] = 1e30f;
      const Plan dp = plan_with(dtype, c, M, N, K, op);
      if (dp.sk) {   // stream-K: other grid sizes (128 x v blocks) instead of split factors
        for (int v : {2, 3, 6, 8}) {
          time_cfg(c | (v << kSplitShift));
          if (rc) break;
        }
        continue;
      }
      int prev = -1;
      for (int v : {1, dp.splits / 4, dp.splits / 2, dp.splits * 2}) {
        if (v < 1 || v == dp.splits || v == prev || v > kMaxSplits || v > dp.ktiles) continue;
        prev = v;
        time_cfg(c | (v << kSplitShift));
        if (rc) break;
      }
    }
    if (rc) break;
    std::lock_guard<std::mutex> lk(g_tune_mu);
    tune_set(tune_key(dtype, op, M, N, K, d), best_c);
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return rc;
}

// Combine statistics partials in ONE pass (each is a round trip to memory
// the writer XCDs flushed): with the shift K = mean of partial 0,
//   mu = K + sum n_i d_i / M,  M2 = sum M2_i + sum n_i d_i^2 - M (mu - K)^2,
// d_i = mean_i - K, in fp64, fixed-shape tree: deterministic.  Partial
// counts are n_i = clamp(M - i R, 0, R), or explicit (cnt != nullptr, from
// the first stage of a two-stage combine).  Block (n, s) combines partials
// [s*chunk, (s+1)*chunk) of channel n; with gridDim.y == 1 it finalizes
// (mean, invstd), else it writes one (mean, M2, count) partial per chunk.
// Single-stage statistics finalize: 32 channels per block, 8 lanes each
// (stats_combine8, jr_common.h: the arithmetic jr_bn_relu_apply_stats shares).
__global__ void __launch_bounds__(256) k_stats_finalize8(const float* __restrict__ part, int P, int R, int M, int N,
                                                         float eps, float* mean, float* invstd, long long p_mb,
                                                         long long st_mb) {
  if (gridDim.z > 1) {   // grouped: member blockIdx.z
    const long long mz = blockIdx.z;
    part = reinterpret_cast<const float*>(reinterpret_cast<const char*>(part) + mz * p_mb);
    mean = reinterpret_cast<float*>(reinterpret_cast<char*>(mean) + mz * st_mb);
    invstd = reinterpret_cast<float*>(reinterpret_cast<char*>(invstd) + mz * st_mb);
  }
  const int n = blockIdx.x * (256 / kStatsLanes) + threadIdx.x / kStatsLanes, j = threadIdx.x % kStatsLanes;
  if (n >= N) return;   // (whole 8-lane groups)
  float mu, is;
  stats_combine8(part + (long long)n * P, part + (long long)(N + n) * P, P, R, M, eps, j, &mu, &is);
  if (j == 0) {
    mean[n] = mu;
    invstd[n] = is;
  }
}

__global__ void __launch_bounds__(256) k_stats_finalize(const float* __restrict__ part, const float* __restrict__ cnt,
                                                        int P, int R, int M, int N, int chunk, float eps,
                                                        float* mean, float* invstd, float* out, long long p_mb,
                                                        long long st_mb) {
  if (gridDim.z > 1) {   // grouped: member blockIdx.z (partials / counts / out by p_mb, results by st_mb)
    const long long mz = blockIdx.z;
    part = reinterpret_cast<const float*>(reinterpret_cast<const char*>(part) + mz * p_mb);
    if (cnt) cnt = reinterpret_cast<const float*>(reinterpret_cast<const char*>(cnt) + mz * p_mb);
    if (out) out = reinterpret_cast<float*>(reinterpret_cast<char*>(out) + mz * p_mb);
    if (mean) mean = reinterpret_cast<float*>(reinterpret_cast<char*>(mean) + mz * st_mb);
    if (invstd) invstd = reinterpret_cast<float*>(reinterpret_cast<char*>(invstd) + mz * st_mb);
  }
  __shared__ double red[3][256];
  const int n = blockIdx.x, t = threadIdx.x;
  const float* pm = part + (long long)n * P;
  const float* pq = part + (long long)(N + n) * P;
  const float* pc = cnt ? cnt + (long long)n * P : nullptr;
  const int i0 = blockIdx.y * chunk, i1 = min(P, i0 + chunk);
  const double K = pm[i0];
  double sn = 0, sd = 0, sq = 0;
  for (int b = i0; b < i1; b += 256 * 8) {
    float vm[8], vq[8], vc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = b + u * 256 + t;
      const bool ok = i < i1;
      vm[u] = ok ? pm[i] : 0.f;
      vq[u] = ok ? pq[i] : 0.f;
      vc[u] = !ok ? 0.f : (pc ? pc[i] : (float)min(max(M - i * R, 0), R));
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const double d = (double)vm[u] - K, c = vc[u];
      sn += c;
      sd += c * d;
      sq += (double)vq[u] + c * d * d;
    }
  }
  red[0][t] = sn; red[1][t] = sd; red[2][t] = sq;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (t < h) {
      red[0][t] += red[0][t + h];
      red[1][t] += red[1][t + h];
      red[2][t] += red[2][t + h];
    }
    __syncthreads();
  }
  if (t != 0) return;
  const double tn = red[0][0];
  const double dm = tn > 0 ? red[1][0] / tn : 0.0;
  const double m2 = fmax(red[2][0] - tn * dm * dm, 0.0);
  if (gridDim.y == 1) {
    mean[n] = (float)(K + dm);
    invstd[n] = (float)(1.0 / sqrt(m2 / (double)M + (double)eps));
  } else {
    const int S = gridDim.y;
    out[(long long)n * S + blockIdx.y] = (float)(K + dm);
    out[(long long)(N + n) * S + blockIdx.y] = (float)m2;
    out[(long long)(2 * N + n) * S + blockIdx.y] = (float)tn;
  }
}

// Deferred filter-gradient split-K reduce: ONE launch for the slabs of many
// layers (jr_wgrad_reduce).  Block b belongs to the segment with the largest
// block0 <= b and sums `256 / G` float4 columns of it exactly as
// k_splitk_reduce does (z-lane zg adds slabs zg, zg + G, ... in order, the G
// lane sums are added in zg order), so the result is bitwise that of the
// per-layer reduce; only the launch count changes (75 -> 1 per step).
__global__ void __launch_bounds__(256) k_wgrad_reduce(const jr_wgrad_seg* __restrict__ segs, int nseg) {
  __shared__ float4 part[256];
  const int b = blockIdx.x;
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {   // wave-uniform
    const int mid = (lo + hi + 1) >> 1;
    if (segs[mid].block0 <= b) lo = mid; else hi = mid - 1;
  }
  const jr_wgrad_seg sg = segs[lo];
  const int G = sg.g, cols = 256 / G;
  const int t = threadIdx.x;
  const int zg = t / cols, cl = t - zg * cols;
  const int n4 = sg.n >> 2;
  const long long total = (long long)sg.m * n4;   // = one slab, in float4
  const long long e = (long long)(b - sg.block0) * cols + cl;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e < total) {
    const float4* src = reinterpret_cast<const float4*>(sg.slabs) + e;
    for (int z = zg; z < sg.splits; z += G) {
      const float4 a = src[z * total];
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
  }
  if (zg != 0 || e >= total) return;
  const int m = (int)(e / n4), q = (int)(e - (long long)m * n4);
  long long base = (long long)m * sg.n;            // out_row<OP_WGRAD>
  if (sg.c_pad != sg.c_in) {
    const int rc = m / sg.c_pad, ci = m - rc * sg.c_pad;
    if (ci >= sg.c_in) return;
    base = ((long long)rc * sg.c_in + ci) * sg.n;
  }
  *reinterpret_cast<float4*>(sg.dw + base + q * 4) = s;
}

}  // namespace jr

using namespace jr;

JR_API int jr_conv2d_wgrad_seg(const jr_conv_desc* d, int dtype, jr_wgrad_seg* seg) {
  int rc = validate(d, OP_WGRAD, dtype);
  if (rc) return rc;
  if (!seg) return fail(JR_ERR_INVALID, "wgrad_seg: null segment");
  const Plan p = plan_for(d, OP_WGRAD, dtype, nullptr);
  seg->m = p.M;
  seg->n = p.N;
  seg->splits = p.splits;
  seg->c_in = d->c_in;
  seg->c_pad = chan_pad(d->c_in, dtype);
  seg->g = reduce_lanes(p);
  seg->block0 = 0;
  seg->blocks = (int32_t)ceil_div((long long)p.M * p.N / 4, (long long)(256 / seg->g));
  return JR_OK;
}

JR_API int jr_conv2d_bwd_filter_slabs(const jr_conv_desc* d, int dtype, const void* x, const void* dy, float* slabs,
                                      size_t slab_bytes, void* stream) {
  int rc = validate(d, OP_WGRAD, dtype);
  if (rc) return rc;
  if (!x || !dy || !slabs) return fail(JR_ERR_INVALID, "bwd_filter_slabs: null tensor pointer");
  if (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)slabs) & 15)
    return fail(JR_ERR_INVALID, "bwd_filter_slabs: tensors must be 16-byte aligned");
  const Plan p = plan_for(d, OP_WGRAD, dtype, nullptr);
  if (p.splits <= 1) return fail(JR_ERR_INVALID, "bwd_filter_slabs: the plan has no split-K (use jr_conv2d_bwd_filter)");
  // the slab region was sized by jr_conv2d_wgrad_seg for the split count the
  // deferred reduce will sum: a plan that changed since (another caller's
  // set_config / autotune on the same geometry) would leave stale slabs in
  // that sum, so any mismatch fails loudly
  if (slab_bytes != plan_ws(p))
    return fail(JR_ERR_INVALID, "bwd_filter_slabs: the plan's split-K slab bytes differ from the segment's "
                                "(tile configuration changed since jr_conv2d_wgrad_seg); re-bind the segment");
  ConvArgs a{};
  fill_common(a, d, dtype);
  fill_scales(a, d, OP_WGRAD, dtype);
  a.A = static_cast<const float*>(x);
  a.B = static_cast<const float*>(dy);
  if (dtype == JR_F32_X8P) {
    a.a_ps = (long long)d->n * d->h * d->w * d->x_c_stride;
    a.b_ps = (long long)d->n * d->ho * d->wo * d->y_c_stride;
  }
  a.c_off = 0; a.c_stride = d->c_out;
  return run_gemm<OP_WGRAD>(dtype, a, p, nullptr, slabs, slab_bytes, as_stream(stream), nullptr, true);
}

JR_API int jr_wgrad_reduce(const jr_wgrad_seg* segs, int32_t nseg, int32_t total_blocks, void* stream) {
  if (!segs || nseg <= 0 || total_blocks <= 0) return fail(JR_ERR_INVALID, "wgrad_reduce: empty segment table");
  hipLaunchKernelGGL(k_wgrad_reduce, dim3(total_blocks), dim3(256), 0, as_stream(stream), segs, nseg);
  return check_launch("wgrad_reduce");
}

JR_API int jr_conv2d_fwd_bn_stats(const jr_conv_desc* d, int dtype, const void* x, const void* w, void* y, float eps,
                                  float* mean, float* invstd, void* ws, size_t ws_bytes, void* stream) {
  if (!mean || !invstd) return fail(JR_ERR_INVALID, "conv fwd+stats: null statistics pointer");
  const StatsReq st{eps, mean, invstd};
  return run_conv(d, OP_FWD, dtype, x, w, y, 0, ws, ws_bytes, stream, -1, -1, &st);
}

// Where the planned forward GEMM leaves its BN-statistics partials in the
// workspace ([2][N][P] fp32 (mean, M2) of R rows each, at ws + ws_offset),
// and whether they are single-stage (P <= kStatsChunk: then
// jr_conv2d_fwd_bn_partials + jr_bn_relu_apply_stats may replace
// jr_conv2d_fwd_bn_stats + jr_bn_relu_apply).  The plan is the one the next
// call of this geometry would use (pinned / tuned / planner).
JR_API int jr_conv2d_bn_partials_layout(const jr_conv_desc* d, int dtype, jr_bn_partials* out) {
  int rc = validate(d, OP_FWD, dtype);
  if (rc) return rc;
  if (!out) return fail(JR_ERR_INVALID, "bn_partials_layout: null output");
  int P = 0, R = 0;
  if (conv1_direct_ok(d, dtype)) {
    conv1_direct_partials(d, &P, &R);
    out->ws_offset = 0;
  } else {
    const Plan p = plan_for(d, OP_FWD, dtype, nullptr);
    stats_geom(dtype, p, &P, &R);
    out->ws_offset = (int64_t)align256(plan_ws(p));
  }
  out->P = P;
  out->R = R;
  out->M = d->n * d->ho * d->wo;
  out->N = d->c_out;
  out->single_stage = P <= kFoldMaxP ? 1 : 0;
  return JR_OK;
}

// jr_conv2d_fwd_bn_stats without the statistics finalize: the GEMM (and its
// split-K reduce) write y and the single-stage partials into ws
// (jr_conv2d_bn_partials_layout); jr_bn_relu_apply_stats combines them.
JR_API int jr_conv2d_fwd_bn_partials(const jr_conv_desc* d, int dtype, const void* x, const void* w, void* y,
                                     void* ws, size_t ws_bytes, void* stream) {
  float dummy = 0.f;   // (never written: the finalize is skipped)
  StatsReq st{0.f, &dummy, &dummy};
  st.defer = true;
  return run_conv(d, OP_FWD, dtype, x, w, y, 0, ws, ws_bytes, stream, -1, -1, &st);
}

// Grouped forward (ensemble members): the same conv geometry for `members`
// models in ONE launch per GEMM (blockIdx.y = member), each member with its
// own input, filter, output and BN statistics at the given element strides;
// the plan (tile, split-K) is the per-member plan, so every member's result
// is bitwise that of jr_conv2d_fwd_bn_stats on its own tensors.
JR_API size_t jr_conv2d_workspace_size_grouped(const jr_conv_desc* d, int dtype, int members) {
  if (!d || members < 1 || validate(d, OP_FWD, dtype) != JR_OK) return 0;
  return (size_t)members * align256(ws_bytes_for(d, OP_FWD, dtype));
}

JR_API int jr_conv2d_fwd_bn_stats_grouped(const jr_conv_desc* d, int dtype, int members, const void* x,
                                          int64_t x_member_stride, const void* w, int64_t w_member_stride, void* y,
                                          int64_t y_member_stride, float eps, float* mean, float* invstd,
                                          int64_t stats_member_stride, void* ws, size_t ws_bytes, void* stream) {
  int rc = validate(d, OP_FWD, dtype);
  if (rc) return rc;
  if (dtype != JR_F32 && dtype != JR_BF16 && dtype != JR_F32_X8 && dtype != JR_F32_X6H)
    return fail(JR_ERR_UNSUPPORTED, "conv grouped: dtype must be JR_F32, JR_BF16, JR_F32_X8 or JR_F32_X6H");
  if (members < 1 || members > 65535) return fail(JR_ERR_INVALID, "conv grouped: members must be 1..65535");
  if (!x || !w || !y || !mean || !invstd) return fail(JR_ERR_INVALID, "conv grouped: null pointer");
  const long long esz = dtype == JR_BF16 ? 2 : 4;
  if ((((uintptr_t)x | (uintptr_t)w | (uintptr_t)y) & 15) ||
      ((x_member_stride * esz) | (w_member_stride * esz) | (y_member_stride * esz)) & 15 ||
      x_member_stride < 0 || w_member_stride < 0 || y_member_stride < 0 || stats_member_stride < 0)
    return fail(JR_ERR_INVALID, "conv grouped: tensors and member strides must be 16-byte aligned, strides >= 0");
  if (conv1_direct_ok(d, dtype)) {   // every member's conv2d_1 in one direct launch (bitwise the single call)
    const StatsReq st{eps, mean, invstd};
    const long long wsz = dtype == JR_BF16 ? 2 : 4;
    return run_conv1_direct(d, dtype, x, w, y, ws, ws_bytes, as_stream(stream), &st, members, x_member_stride * esz,
                            w_member_stride * wsz, y_member_stride * esz, stats_member_stride * 4);
  }
  ConvArgs a{};
  fill_common(a, d, dtype);
  fill_scales(a, d, OP_FWD, dtype);
  a.A = static_cast<const float*>(x);
  a.B = static_cast<const float*>(w);
  a.accumulate = 0;
  a.a_mb = x_member_stride * esz;
  a.b_mb = w_member_stride * esz;
  a.o_mb = y_member_stride * esz;
  a.c_off = d->y_c_off; a.c_stride = d->y_c_stride;
  const StatsReq st{eps, mean, invstd};
  return run_gemm<OP_FWD>(dtype, a, plan_for(d, OP_FWD, dtype, nullptr), y, ws, ws_bytes, as_stream(stream), &st,
                          false, members, stats_member_stride * 4);
}

JR_API size_t jr_conv2d_workspace_size(const jr_conv_desc* d, int op, int dtype) {
  if (!d || validate(d, op, dtype) != JR_OK) return 0;
  return ws_bytes_for(d, op, dtype);
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

JR_API int jr_conv2d_autotune(const jr_conv_desc* d, int op, int dtype, const void* a, const void* b, void* c,
                              void* ws, size_t ws_bytes, void* stream) {
  return autotune(d, op, dtype, a, b, c, ws, ws_bytes, stream, 3);
}

JR_API int jr_conv2d_num_configs(int dtype) {
  return dtype == JR_BF16 || dtype == JR_F32 || x8_family(dtype) || dtype == JR_F32_X8P ? cfg_count(dtype) : 0;
}

// Diagnostic: time `reps` launches of one FWD GEMM (no split-K) of tile
// config `cfg` in variant dbg (0 normal, 1 no MFMA, 2 no DMA, 3 no LDS reads;
// +16 = the JR_F32_X8 kernel, whose variant 4 skips the operand split);
// returns ms via *ms.  Results of variants other than 0 / 16 are garbage.
JR_API int jr_conv2d_debug_time(const jr_conv_desc* d, int cfg, int dbg, const void* x, const void* w, void* y,
                                int reps, float* ms, void* stream) {
  int rc = validate(d, OP_FWD, JR_F32);
  if (rc) return rc;
  const bool x8 = dbg >= 16;
  if (x8) dbg -= 16;
  if (cfg < 0 || cfg >= kNumCfgs || dbg < 0 || dbg > (x8 ? 4 : 3)) return fail(JR_ERR_INVALID, "debug_time: bad cfg/dbg");
  if (dbg > 0 && chan_pad(d->c_in, JR_F32) % kCfgs[cfg].bk != 0)
    return fail(JR_ERR_UNSUPPORTED, "debug_time: variants need c_in % BK == 0");
  ConvArgs a{};
  fill_common(a, d, JR_F32);
  a.A = (const float*)x; a.B = (const float*)w; a.C = (float*)y;
  a.c_off = d->y_c_off; a.c_stride = d->y_c_stride;
  Plan p = plan_for(d, OP_FWD, JR_F32, nullptr, cfg);
  p.splits = 1; p.kt_per_split = p.ktiles;
  a.M = p.M; a.N = p.N; a.K = p.K; a.ktiles = p.ktiles; a.kt_per_split = p.kt_per_split; a.ntn = p.nt;
  hipStream_t s = as_stream(stream);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  dim3 grid(p.mt * p.nt, 1, 1);
  (void)hipEventRecord(e0, s);
  for (int r = 0; r < reps; ++r) {
    switch (dbg + (x8 ? 16 : 0)) {
      case 0: launch_op<OP_FWD, 0>(cfg, a, grid, s); break;
      case 1: launch_op<OP_FWD, 1>(cfg, a, grid, s); break;
      case 2: launch_op<OP_FWD, 2>(cfg, a, grid, s); break;
      case 3: launch_op<OP_FWD, 3>(cfg, a, grid, s); break;
      case 16: launch_op<OP_FWD, 0, true>(cfg, a, grid, s); break;
      case 17: launch_op<OP_FWD, 1, true>(cfg, a, grid, s); break;
      case 18: launch_op<OP_FWD, 2, true>(cfg, a, grid, s); break;
      case 19: launch_op<OP_FWD, 3, true>(cfg, a, grid, s); break;
      default: launch_op<OP_FWD, 4, true>(cfg, a, grid, s); break;
    }
  }
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return check_launch("debug_time");
}

JR_API int jr_conv2d_set_config(const jr_conv_desc* d, int op, int dtype, int phase, int cfg) {
  int rc = validate(d, op, dtype);
  if (rc) return rc;
  if (cfg < -1 || (cfg >= 0 && (cfg_tile(cfg) >= cfg_count(dtype) || cfg_splits(cfg) > kMaxSplits)))
    return fail(JR_ERR_INVALID, "conv set_config: bad config index");
  Phase ph[64];
  int nph = 1;
  if (op == OP_DGRAD) {
    dgrad_phases(d, ph, &nph);
    if (phase < 0 || phase >= nph) return fail(JR_ERR_INVALID, "conv set_config: bad phase");
  }
  int M, N, K;
  gemm_dims(d, op, dtype, op == OP_DGRAD ? &ph[phase] : nullptr, &M, &N, &K);
  std::lock_guard<std::mutex> lk(g_tune_mu);
  tune_set(tune_key(dtype, op, M, N, K, d), cfg);   // cfg < 0: back to the planner's choice
  return JR_OK;
}

JR_API unsigned long long jr_conv2d_config_generation(void) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  return g_tune_gen;
}

JR_API int jr_conv2d_get_config(const jr_conv_desc* d, int op, int dtype, int phase) {
  if (!d || validate(d, op, dtype) != JR_OK) return -1;
  Phase ph[64];
  int nph = 1;
  if (op == OP_DGRAD) {
    dgrad_phases(d, ph, &nph);
    if (phase < 0 || phase >= nph) return -1;
  }
  return plan_for(d, op, dtype, op == OP_DGRAD ? &ph[phase] : nullptr).cfg;
}
