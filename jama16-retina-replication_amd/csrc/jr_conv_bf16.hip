// jr_conv_bf16.hip — the bf16 implicit-GEMM convolution (configs 3 and 5 of
// BASELINE: bf16 MFMA training), v_mfma_f32_32x32x16_bf16 with fp32
// accumulation.  Same GEMM mapping, phase decomposition, split-K and host
// planning as the fp32 kernel in jr_conv.hip (which documents them); what
// differs is the operand staging:
//   * 16 B LDS-DMA pieces carry 8 bf16 channels, so channel radices are
//     padded to 8 (conv1: c_in 3 -> 8, virtual zero channels);
//   * every FWD / DGRAD operand is a KC image (k contiguous): FWD's filter is
//     the transposed bf16 copy W^T [c_out][kh*kw*c8] that
//     jr_conv_weights_bf16 writes, so B rows are k-linear; one ds_read_b128
//     is exactly one MFMA operand (8 consecutive k of one row);
//   * WGRAD's operands (x and dy, both contiguous along m / n) are MC images
//     [BK][cols] read with ds_read_b64_tr_b16, the gfx950 transposing LDS
//     read: per 16-lane group a 4 (k) x 16 (col) block arrives column-major,
//     two reads give a lane its 8 k values.
// Outputs: FWD / DGRAD write bf16 (fp32 accumulate, one rounding; split-K
// slabs stay fp32 and the reduce rounds), WGRAD writes fp32 dW.
//
// NP = 3 is JR_F32_X8P: fp32 arithmetic from operands that arrive already
// split into three bf16 planes (x = h + m + l exactly, jr_split_x8p /
// jr_conv_weights_x8p_multi).  Every DMA piece is issued once per plane
// (the same source offset in each plane, plane strides g.a_ps / g.b_ps),
// each fragment is read once per plane, and eight MFMAs per (i, j, k-step)
// accumulate hh mh hm mm lh hl ml lm (A plane x B plane) in fp32 — the
// products and per-accumulator order of the JR_F32_X8 kernel (jr_conv.hip),
// without its in-register split VALU.  Outputs are fp32 as for JR_F32.
#include "jr_conv_impl.h"

namespace jr {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// ds_read_b64_tr_b16: lane 4q+p of each 16-lane group passes the address of
// row q, columns 4p..4p+3 of the group's 4x16 block; lane i gets column i.
__device__ __forceinline__ s16x4 lds_tr(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(const_cast<uint16_t*>(p)));
}

// AM = operand address mode (host: run_gemm): 0 = wave-uniform tap (FWD /
// DGRAD with cred % BK == 0), 1 = incremental per-lane walk (one carry per
// radix per K-tile), 2 = mixed-radix loop (conv1's 8 padded channels, tiny
// images).
// SK: the stream-K grid (the scheme of jr_conv.hip k_conv SK: equal ranges of
// tiles x K-tiles per block, cut tiles finished by the block holding their
// first K-tile from the later pieces' write-through partials).
template <int OP, int BM, int BN, int WGM, int BK, int NBUF, int AM, int NP, int NW, bool SK = false>
__global__ void __launch_bounds__(NW * 64) k_conv_bf16(ConvArgs g) {
  static_assert(NP == 1 || NP == 3, "one bf16 plane, or the h / m / l planes of X8P");
  static_assert(NW == 4 || NW == 8, "4 or 8 waves per block");
  constexpr int WGN = NW / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 32, TN = WN / 32;
  static_assert(WM % 32 == 0 && WN % 32 == 0, "wave tile must be a multiple of 32x32");
  constexpr int QPR = BK / 8;                 // 16 B quads per KC row
  constexpr int RPI = 64 / QPR;               // KC rows per DMA instruction
  constexpr int SWZ = 16 / QPR;               // rows sharing one swizzle value
  constexpr int KSTEPS = BK / 16;             // MFMA k-steps per tile
  constexpr bool MC = (OP == OP_WGRAD);       // both operands MC (else both KC)
  constexpr int ASZ = BM * BK, BSZ = BN * BK;  // bf16 elements per image
  constexpr int A_INSTR = ASZ / 512, B_INSTR = BSZ / 512;
  constexpr int A_PW = (A_INSTR + NW - 1) / NW, B_PW = (B_INSTR + NW - 1) / NW;  // per wave
  static_assert(ASZ % 512 == 0 && BSZ % 512 == 0, "tile must be whole DMA instructions");
  static_assert(BK % 16 == 0 && QPR <= 8, "BK must be 16..64");
  constexpr int STAGE = NP * (ASZ + BSZ);    // one ring slot: NP A planes, then NP B planes
  constexpr int SMEM = NBUF * STAGE > 2 * NW * stage_floats<WN>() ? NBUF * STAGE : 2 * NW * stage_floats<WN>();
  static_assert(SMEM * 2 <= 160 * 1024, "LDS budget of one CU");
  __shared__ __attribute__((aligned(1024))) uint16_t smem[SMEM];

  JR_ST(Stamps stamp; stamp.start();)
  member_offsets(g);
  const uint16_t* __restrict__ gA = reinterpret_cast<const uint16_t*>(g.A);
  const uint16_t* __restrict__ gB = reinterpret_cast<const uint16_t*>(g.B);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm0 = (wave / WGN) * WM;
  const int wn0 = (wave % WGN) * WN;

  long long sk_it = 0, sk_end = 0;
  const int lb = SK ? xcd_remap(blockIdx.x, gridDim.x) : 0;   // logical block (jr_conv.hip k_conv)
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
  // the zero page's address lives in an SGPR pair for the whole kernel (hipcc
  // otherwise rematerialises it with s_getpc + two v_mov per DMA piece)
  unsigned long long zpa = reinterpret_cast<unsigned long long>(g_zero_page);
  asm volatile("" : "+s"(zpa));
  const uint16_t* zp = reinterpret_cast<const uint16_t*>(zpa);
  const int cred = OP == OP_FWD ? g.cp : g.cout;
  const long long psA = NP > 1 ? g.a_ps : 0, psB = NP > 1 ? g.b_ps : 0;
  constexpr bool ut = AM == 0 && OP != OP_WGRAD;

  // ---------------------------------------------------------------- A state
  // AM 1: pieces walk their im2col address INCREMENTALLY (round 3): a_ptr =
  // the piece's base, a_off = the element offset of its current k, advanced
  // per K-tile by one of three wave-uniform deltas chosen by the piece's
  // carries -- no multiplies, no division (the mixed-radix form rebuilt the
  // address with two v_mul_lo_u32 and ~35 more VALU per piece and tile:
  // conv5's loop issued 19 VALU per MFMA).  Needs at most one carry per
  // radix per K-tile, which the host checks.
  const int wq = OP == OP_WGRAD ? BK / g.wo : 0, wr = OP == OP_WGRAD ? BK - wq * g.wo : 0;
  constexpr bool inc_a = AM == 1;
  constexpr bool inc_b = OP == OP_DGRAD && AM == 1;
  // (single const definitions: deltas assigned in branches became allocas
  // that hipcc then read through a per-lane select of their ADDRESSES --
  // scratch and flat loads in the K loop)
  const int dA0 = OP == OP_WGRAD ? (wq * g.sh * g.w + wr * g.sw) * g.xs : BK;
  const int dA1 = OP == OP_FWD ? BK - g.cp + g.xs
                  : OP == OP_DGRAD ? BK - g.cout - g.ys
                                   : (g.sh * g.w - g.wo * g.sw) * g.xs;
  const int dA2 = OP == OP_FWD ? BK - g.cp + g.xs + (g.w - g.kw) * g.xs
                  : OP == OP_DGRAD ? BK - g.cout + (g.nb - 1 - g.wo) * g.ys
                                   : (g.h * g.w - g.ho * g.sh * g.w) * g.xs;
  const int dB1 = OP == OP_DGRAD ? BK - g.cout + g.sw * g.cin * g.cout : 0;
  const int dB2 = OP == OP_DGRAD ? BK - g.cout + (g.sh * g.kw - g.sw * (g.nb - 1)) * g.cin * g.cout : 0;
  const uint16_t* a_ptr[A_PW];
  int a_p0[A_PW], a_p1[A_PW], a_p2[A_PW];
  int a_s0[A_PW], a_s1[A_PW], a_s2[A_PW], a_off[A_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int j = wave + NW * i;
    a_ptr[i] = zp;
    a_p0[i] = a_p1[i] = a_p2[i] = 0;
    a_s0[i] = a_s1[i] = a_s2[i] = 0;
    a_off[i] = 0;
    if (A_INSTR % NW != 0 && j >= A_INSTR) continue;
    if constexpr (!MC) {
      const int row = j * RPI + lane / QPR;
      const int q = (lane % QPR) ^ ((row / SWZ) % QPR);
      const int m = m0 + row;
      const int k = kt0 * BK + q * 8;
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
        a_ptr[i] = gA + ((long long)pix * g.xs + g.xo + (ut ? q * 8 : 0));
        const int rc = k / g.cp;
        a_s2[i] = k - rc * g.cp;
        a_s0[i] = rc / g.kw;
        a_s1[i] = rc - a_s0[i] * g.kw;
        a_off[i] = (a_s0[i] * g.w + a_s1[i]) * g.xs + a_s2[i];
      } else {  // DGRAD
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
        a_ptr[i] = gA + ((long long)pix * g.ys + g.yo + (ut ? q * 8 : 0));
        const int ab = k / g.cout;
        a_s2[i] = k - ab * g.cout;
        a_s0[i] = ab / g.nb;
        a_s1[i] = ab - a_s0[i] * g.nb;
        a_off[i] = a_s2[i] - (a_s0[i] * g.wo + a_s1[i]) * g.ys;
      }
    } else {  // WGRAD MC: m = (r,c,ci) fixed per slot (8 channels), k = pixel
      const int flat = j * 512 + lane * 8;
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
      a_s0[i] = pix / hw;
      const int rem = pix - a_s0[i] * hw;
      a_s1[i] = rem / g.wo;
      a_s2[i] = rem - a_s1[i] * g.wo;
      if (m < g.M) a_ptr[i] = gA + ((long long)(a_p0[i] * g.w + a_p1[i]) * g.xs + g.xo + a_p2[i]);
      a_off[i] = ((a_s0[i] * g.h + a_s1[i] * g.sh) * g.w + a_s2[i] * g.sw) * g.xs;
    }
  }
  // ---------------------------------------------------------------- B state
  const uint16_t* b_ptr[B_PW];
  int b_p0[B_PW], b_s0[B_PW], b_s1[B_PW], b_s2[B_PW], b_off[B_PW];
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int j = wave + NW * i;
    b_ptr[i] = zp;
    b_p0[i] = b_s0[i] = b_s1[i] = b_s2[i] = b_off[i] = 0;
    if (B_INSTR % NW != 0 && j >= B_INSTR) continue;
    if constexpr (!MC) {
      const int row = j * RPI + lane / QPR;
      const int q = (lane % QPR) ^ ((row / SWZ) % QPR);
      const int nn = n0 + row;
      b_p0[i] = nn < g.N ? nn : -1;
      const int k = kt0 * BK + q * 8;
      if constexpr (OP == OP_FWD) {   // W^T [N][K]: k-linear rows
        b_s0[i] = k;
        b_ptr[i] = gB + ((long long)(nn < g.N ? nn : 0) * g.K + k);
      } else {                        // DGRAD: W[(r,c)][ci][co], rows = ci, k = (a, bb, co)
        b_ptr[i] = gB + ((long long)(nn < g.N ? nn : 0) * g.cout + (ut ? q * 8 : 0));
        const int ab = k / g.cout;
        b_s2[i] = k - ab * g.cout;
        b_s0[i] = ab / g.nb;
        b_s1[i] = ab - b_s0[i] * g.nb;
        b_off[i] = ((g.r0 + g.sh * b_s0[i]) * g.kw + g.c0 + g.sw * b_s1[i]) * g.cin * g.cout + b_s2[i];
      }
    } else {  // WGRAD MC: dy rows = k (pixels), cols = n
      const int flat = j * 512 + lane * 8;
      const int krow = flat / BN, col = flat - krow * BN;
      b_p0[i] = (n0 + col < g.N) ? n0 + col : -1;
      b_s0[i] = kt0 * BK + krow;
      b_ptr[i] = gB + ((long long)b_s0[i] * g.ys + g.yo + n0 + col);
    }
  }
  int t_r = 0, t_c = 0, t_ch = 0;
  if constexpr (ut) {
    const int k = kt0 * BK;
    const int rc = k / cred;
    t_ch = k - rc * cred;
    t_r = rc / (OP == OP_FWD ? g.kw : g.nb);
    t_c = rc - t_r * (OP == OP_FWD ? g.kw : g.nb);
  }

  constexpr bool a_multi = AM == 2;
  constexpr bool b_multi = OP == OP_DGRAD && AM == 2;

  // (every bounds test below combines with bitwise &: && made hipcc branch
  // around each operand with exec-mask saves)
  // One piece into every plane image (out-of-bounds: the zero page, all planes).
  auto put = [&](bool ok, const uint16_t* src, uint16_t* dst, long long ps, int isz) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < NP; ++p) dma16(ok ? src + p * ps : zp, dst + p * isz);
  };
  // DMA of one operand piece of tile kt (d < A_PW: A slot d, else B slot).
  auto issue_piece = [&](int kt, int d, uint16_t* __restrict__ As, uint16_t* __restrict__ Bs) __attribute__((always_inline)) {
    if (d < A_PW) {
      const int i = d;
      const int j = wave + NW * i;
      if (A_INSTR % NW != 0 && j >= A_INSTR) return;
      if constexpr (!MC && ut) {
        long long off;
        int dr, dc;
        if constexpr (OP == OP_FWD) {
          off = (long long)(t_r * g.w + t_c) * g.xs + t_ch;
          dr = t_r; dc = t_c;
        } else {
          off = -(long long)(t_r * g.wo + t_c) * g.ys + t_ch;
          dr = -t_r; dc = -t_c;
        }
        const int hmax = OP == OP_FWD ? g.h : g.ho, wmax = OP == OP_FWD ? g.w : g.wo;
        const bool ok = ((unsigned)(a_p0[i] + dr) < (unsigned)hmax) & ((unsigned)(a_p1[i] + dc) < (unsigned)wmax);
        put(ok, a_ptr[i] + off, As + j * 512, psA, ASZ);
      } else {
        bool ok;
        const uint16_t* p;
        if constexpr (OP == OP_FWD) {
          const int hi = a_p0[i] + a_s0[i], wi = a_p1[i] + a_s1[i];
          ok = ((unsigned)hi < (unsigned)g.h) & ((unsigned)wi < (unsigned)g.w) & (a_s0[i] < g.kh);
          if constexpr (inc_a) {   // (r, c, ch) += BK channels, one carry at most per radix
            p = a_ptr[i] + a_off[i];
            const bool c1 = a_s2[i] + BK >= g.cp, c2 = c1 & (a_s1[i] + 1 == g.kw);
            a_off[i] += dA0 + (c1 ? dA1 - dA0 : 0) + (c2 ? dA2 - dA1 : 0);
            a_s2[i] += c1 ? BK - g.cp : BK;
            a_s1[i] = c2 ? 0 : a_s1[i] + (c1 ? 1 : 0);
            a_s0[i] += c2 ? 1 : 0;
          } else {
            p = gA + ((a_p2[i] + hi * g.w + wi) * g.xs + g.xo + a_s2[i]);
            adv_mixed(a_s2[i], a_s1[i], a_s0[i], g.cp, g.kw, a_multi);
          }
        } else if constexpr (OP == OP_DGRAD) {
          const int oh = a_p0[i] - a_s0[i], ow = a_p1[i] - a_s1[i];
          ok = ((unsigned)oh < (unsigned)g.ho) & ((unsigned)ow < (unsigned)g.wo) & (a_s0[i] < g.na);
          if constexpr (inc_a) {   // (a, b, co) += BK output channels
            p = a_ptr[i] + a_off[i];
            const bool c1 = a_s2[i] + BK >= g.cout, c2 = c1 & (a_s1[i] + 1 == g.nb);
            a_off[i] += dA0 + (c1 ? dA1 - dA0 : 0) + (c2 ? dA2 - dA1 : 0);
            a_s2[i] += c1 ? BK - g.cout : BK;
            a_s1[i] = c2 ? 0 : a_s1[i] + (c1 ? 1 : 0);
            a_s0[i] += c2 ? 1 : 0;
          } else {
            p = gA + ((a_p2[i] + oh * g.wo + ow) * g.ys + g.yo + a_s2[i]);
            adv_mixed(a_s2[i], a_s1[i], a_s0[i], g.cout, g.nb, a_multi);
          }
        } else {  // WGRAD
          const int hi = __mul24(a_s1[i], g.sh) + a_p0[i], wi = __mul24(a_s2[i], g.sw) + a_p1[i];
          ok = (a_s0[i] < g.n) & ((unsigned)hi < (unsigned)g.h) & ((unsigned)wi < (unsigned)g.w);
          if constexpr (inc_a) {   // (image, oh, ow) += BK = wq rows + wr columns of output pixels
            p = a_ptr[i] + a_off[i];
            int ow = a_s2[i] + wr;
            const bool c1 = ow >= g.wo;
            ow -= c1 ? g.wo : 0;
            int oh = a_s1[i] + wq + (c1 ? 1 : 0);
            const bool c2 = oh >= g.ho;
            oh -= c2 ? g.ho : 0;
            a_off[i] += dA0 + (c1 ? dA1 : 0) + (c2 ? dA2 : 0);
            a_s2[i] = ow;
            a_s1[i] = oh;
            a_s0[i] += c2 ? 1 : 0;
          } else {
            p = gA + (((a_s0[i] * g.h + hi) * g.w + wi) * g.xs + g.xo + a_p2[i]);
            adv_mixed(a_s2[i], a_s1[i], a_s0[i], g.wo, g.ho, a_multi);
          }
        }
        put(ok, p, As + j * 512, psA, ASZ);
      }
      return;
    }
    const int i = d - A_PW;
    const int j = wave + NW * i;
    if (B_INSTR % NW != 0 && j >= B_INSTR) return;
    if constexpr (OP == OP_FWD) {
      const int k = b_s0[i] + (kt - kt0) * BK;
      const bool ok = (b_p0[i] >= 0) & (k < g.K);
      put(ok, b_ptr[i] + (kt - kt0) * BK, Bs + j * 512, psB, BSZ);
    } else if constexpr (OP == OP_DGRAD) {
      if constexpr (ut) {
        const long long off = (long long)((g.r0 + g.sh * t_r) * g.kw + (g.c0 + g.sw * t_c)) * g.cin * g.cout + t_ch;
        put(b_p0[i] >= 0, b_ptr[i] + off, Bs + j * 512, psB, BSZ);
      } else {
        const bool ok = (b_p0[i] >= 0) & (b_s0[i] < g.na);
        if constexpr (inc_b) {   // (a, b, co) += BK, taps r = r0 + sh a, c = c0 + sw b
          put(ok, b_ptr[i] + b_off[i], Bs + j * 512, psB, BSZ);
          const bool c1 = b_s2[i] + BK >= g.cout, c2 = c1 & (b_s1[i] + 1 == g.nb);
          b_off[i] += BK + (c1 ? dB1 - BK : 0) + (c2 ? dB2 - dB1 : 0);
          b_s2[i] += c1 ? BK - g.cout : BK;
          b_s1[i] = c2 ? 0 : b_s1[i] + (c1 ? 1 : 0);
          b_s0[i] += c2 ? 1 : 0;
        } else {
          const int r = g.r0 + g.sh * b_s0[i], c = g.c0 + g.sw * b_s1[i];
          const uint16_t* p = gB + (((r * g.kw + c) * g.cin + b_p0[i]) * g.cout + b_s2[i]);
          put(ok, p, Bs + j * 512, psB, BSZ);
          adv_mixed(b_s2[i], b_s1[i], b_s0[i], g.cout, g.nb, b_multi);
        }
      }
    } else {  // WGRAD
      const int k = b_s0[i] + (kt - kt0) * BK;
      const bool ok = (b_p0[i] >= 0) & (k < g.K);
      put(ok, b_ptr[i] + (long long)(kt - kt0) * BK * g.ys, Bs + j * 512, psB, BSZ);
    }
  };
  auto advance = [&]() __attribute__((always_inline)) {
    if constexpr (ut) {
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
  auto issue = [&](int kt, uint16_t* __restrict__ As, uint16_t* __restrict__ Bs) __attribute__((always_inline)) {
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
  // transposed-read lane roles (MC): 16-lane group g16 = lh*2 + hb
  const int hb = (lane >> 4) & 1, tq = (lane & 15) >> 2, tp = lane & 3;
  constexpr int per_tile = NP * (A_INSTR / NW + B_INSTR / NW);   // DMA instructions per wave and tile (min)

  auto step = [&](int kt, auto do_issue, const uint16_t* __restrict__ As, const uint16_t* __restrict__ Bs,
                  uint16_t* __restrict__ wA, uint16_t* __restrict__ wB) __attribute__((always_inline)) {
    constexpr bool DO_ISSUE = decltype(do_issue)::value;
    bf16x8 af[NP][TM][KSTEPS], bfr[NP][TN][KSTEPS];
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if constexpr (!MC) {
          const int row = wm0 + i * 32 + l31;
          const int f = (row / SWZ) % QPR;
          af[p][i][s] = *reinterpret_cast<const bf16x8*>(As + p * ASZ + row * BK + (((2 * s + lh) ^ f) * 8));
        } else {
          const uint16_t* q = As + p * ASZ + (16 * s + 8 * lh + tq) * BM + wm0 + i * 32 + 16 * hb + 4 * tp;
          const s16x4 lo = lds_tr(q), hi = lds_tr(q + 4 * BM);
          af[p][i][s] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (!MC) {
          const int row = wn0 + j * 32 + l31;
          const int f = (row / SWZ) % QPR;
          bfr[p][j][s] = *reinterpret_cast<const bf16x8*>(Bs + p * BSZ + row * BK + (((2 * s + lh) ^ f) * 8));
        } else {
          const uint16_t* q = Bs + p * BSZ + (16 * s + 8 * lh + tq) * BN + wn0 + j * 32 + 16 * hb + 4 * tp;
          const s16x4 lo = lds_tr(q), hi = lds_tr(q + 4 * BN);
          bfr[p][j][s] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
      }
    }
    if constexpr (NP == 3) {
      // eight products per k-step, (A plane, B plane) in the JR_F32_X8 order
      // hh mh hm mm lh hl ml lm; the DMA pieces of tile kt+NBUF-1 are spread
      // over the product groups (each piece = one DMA per plane)
      constexpr int PA[8] = {0, 1, 0, 1, 2, 0, 1, 2}, PB[8] = {0, 0, 1, 1, 0, 2, 2, 1};
      constexpr int NG = 8 * KSTEPS;
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s)
#pragma unroll
        for (int t = 0; t < 8; ++t) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[PA[t]][i][s], bfr[PB[t]][j][s], acc[i][j], 0, 0, 0);
          if constexpr (DO_ISSUE) {
            const int gi = s * 8 + t;
#pragma unroll
            for (int d = gi * NPIECE / NG; d < (gi + 1) * NPIECE / NG; ++d) issue_piece(kt + NBUF - 1, d, wA, wB);
          }
        }
      if constexpr (DO_ISSUE) advance();
      return;
    }
    // MFMAs of k-step s, then this step's share of the DMA pieces of tile
    // kt+NBUF-1 (the LDS-DMA intrinsic is a scheduling boundary for hipcc)
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][i][s], bfr[0][j][s], acc[i][j], 0, 0, 0);
      if constexpr (DO_ISSUE) {
#pragma unroll
        for (int d = s * NPIECE / KSTEPS; d < (s + 1) * NPIECE / KSTEPS; ++d) issue_piece(kt + NBUF - 1, d, wA, wB);
      }
    }
    if constexpr (DO_ISSUE) advance();
  };
  auto buf_a = [&](int b) __attribute__((always_inline)) { return smem + b * STAGE; };
  auto buf_b = [&](int b) __attribute__((always_inline)) { return smem + b * STAGE + NP * ASZ; };

  if (kt0 < kt1) {
#pragma unroll
    for (int p = 0; p < NBUF - 1; ++p)
      if (kt0 + p < kt1) issue(kt0 + p, buf_a(p), buf_b(p));
    wait_vmcnt(per_tile * min(NBUF - 2, kt1 - kt0 - 1));
    __builtin_amdgcn_s_barrier();
    JR_ST(stamp.prologue();)
    int cur = 0;
    int kt = kt0;
    for (; kt < kt1 - (NBUF - 1); ++kt) {
      const int nxt = cur == 0 ? NBUF - 1 : cur - 1;
      step(kt, std::true_type{}, buf_a(cur), buf_b(cur), buf_a(nxt), buf_b(nxt));
      __builtin_amdgcn_sched_barrier(0);
      JR_ST(const unsigned long long tw = stamp.now();)
      wait_vmcnt(per_tile * (NBUF - 2));
      __builtin_amdgcn_s_barrier();
      JR_ST(stamp.w += stamp.now() - tw;)
      __builtin_amdgcn_sched_barrier(0);
      cur = cur + 1 == NBUF ? 0 : cur + 1;
    }
    for (; kt < kt1; ++kt) {
      step(kt, std::false_type{}, buf_a(cur), buf_b(cur), nullptr, nullptr);
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

  if constexpr (SK) {
    sk_first = false;
    int owner, npieces, kind;
    if (sk_cut(g, tile, kt0, kt1, &owner, &npieces, &kind) &&
        !sk_handoff<TM, TN, NW>(g, acc, wave, lane, owner, npieces, kind, lb))
      continue;                      // another block finishes the tile
  }
  // ---------------------------------------------------------------- epilogue
  conv_epilogue<OP, WM, TM, TN, NP == 1>(g, acc, reinterpret_cast<float*>(smem) + wave * stage_floats<WN>(), m0 + wm0,
                                      n0 + wn0, lane);
  if constexpr (!SK) break;
  }
  JR_ST(stamp.end(g.dbg);)
}

template <int OP, int NP, int BM, int BN, int WGM, int BK, int NBUF, int NW, bool SK>
static void launch_cfg_t(int am, const ConvArgs& a, dim3 grid, hipStream_t s) {
  if constexpr (OP != OP_WGRAD) {
    if (am == 0) {
      hipLaunchKernelGGL((k_conv_bf16<OP, BM, BN, WGM, BK, NBUF, 0, NP, NW, SK>), grid, dim3(64 * NW), 0, s, a);
      return;
    }
  }
  if (am == 1)
    hipLaunchKernelGGL((k_conv_bf16<OP, BM, BN, WGM, BK, NBUF, 1, NP, NW, SK>), grid, dim3(64 * NW), 0, s, a);
  else
    hipLaunchKernelGGL((k_conv_bf16<OP, BM, BN, WGM, BK, NBUF, 2, NP, NW, SK>), grid, dim3(64 * NW), 0, s, a);
}

// config c of the standard (W = false) or wide (W = true) table of NP; SK:
// its stream-K grid (JR_BF16 only)
template <int OP, int C, int NP, bool W, bool SK>
static void launch_tile(int am, const ConvArgs& a, dim3 grid, hipStream_t s) {
  if constexpr (W) {
    constexpr int n = NP == 1 ? kNumCfgsBf16W : kNumCfgsX8PW;
    if constexpr (C < n) {
      constexpr TileCfg t = NP == 1 ? kCfgsBf16W[C] : kCfgsX8PW[C];
      launch_cfg_t<OP, NP, t.bm, t.bn, t.wgm, t.bk, t.nbuf, t.nw, SK>(am, a, grid, s);
    }
  } else {
    constexpr TileCfg t = NP == 1 ? kCfgsBf16[C] : kCfgsX8P[C];
    launch_cfg_t<OP, NP, t.bm, t.bn, t.wgm, t.bk, t.nbuf, t.nw, SK>(am, a, grid, s);
  }
}

template <int OP, int NP, bool W, bool SK = false>
static void launch_op_bf16(int tile, int am, const ConvArgs& a, dim3 grid, hipStream_t s) {
  static_assert(kNumCfgsBf16 == 17 && kNumCfgsX8P == 17, "keep the switch in sync with kCfgsBf16 / kCfgsX8P");
  static_assert(kNumCfgsBf16W <= 17 && kNumCfgsX8PW <= 17, "keep the switch in sync with the wide tables");
  switch (tile) {
    case 0: launch_tile<OP, 0, NP, W, SK>(am, a, grid, s); break;
    case 1: launch_tile<OP, 1, NP, W, SK>(am, a, grid, s); break;
    case 2: launch_tile<OP, 2, NP, W, SK>(am, a, grid, s); break;
    case 3: launch_tile<OP, 3, NP, W, SK>(am, a, grid, s); break;
    case 4: launch_tile<OP, 4, NP, W, SK>(am, a, grid, s); break;
    case 5: launch_tile<OP, 5, NP, W, SK>(am, a, grid, s); break;
    case 6: launch_tile<OP, 6, NP, W, SK>(am, a, grid, s); break;
    case 7: launch_tile<OP, 7, NP, W, SK>(am, a, grid, s); break;
    case 8: launch_tile<OP, 8, NP, W, SK>(am, a, grid, s); break;
    case 9: launch_tile<OP, 9, NP, W, SK>(am, a, grid, s); break;
    case 10: launch_tile<OP, 10, NP, W, SK>(am, a, grid, s); break;
    case 11: launch_tile<OP, 11, NP, W, SK>(am, a, grid, s); break;
    case 12: launch_tile<OP, 12, NP, W, SK>(am, a, grid, s); break;
    case 13: launch_tile<OP, 13, NP, W, SK>(am, a, grid, s); break;
    case 14: launch_tile<OP, 14, NP, W, SK>(am, a, grid, s); break;
    case 15: launch_tile<OP, 15, NP, W, SK>(am, a, grid, s); break;
    default: launch_tile<OP, 16, NP, W, SK>(am, a, grid, s); break;
  }
}

template <int NP, bool W, bool SK = false>
static void launch_np(int op, int tile, int am, const ConvArgs& a, dim3 grid, hipStream_t s) {
  if (op == OP_FWD) launch_op_bf16<OP_FWD, NP, W, SK>(tile, am, a, grid, s);
  else if (op == OP_DGRAD) launch_op_bf16<OP_DGRAD, NP, W, SK>(tile, am, a, grid, s);
  else launch_op_bf16<OP_WGRAD, NP, W, SK>(tile, am, a, grid, s);
}

void launch_conv_bf16(int op, int tile, int am, const ConvArgs& a, dim3 grid, hipStream_t s, int np) {
  if (np == 3) launch_np<3, false>(op, tile, am, a, grid, s);
  else launch_np<1, false>(op, tile, am, a, grid, s);
}

void launch_conv_bf16_wide(int op, int tile, int am, const ConvArgs& a, dim3 grid, hipStream_t s, int np) {
  if (np == 3) launch_np<3, true>(op, tile, am, a, grid, s);
  else launch_np<1, true>(op, tile, am, a, grid, s);
}

void launch_conv_bf16_sk(int op, int tile, bool wide, int am, const ConvArgs& a, dim3 grid, hipStream_t s) {
  if (wide) launch_np<1, true, true>(op, tile, am, a, grid, s);
  else launch_np<1, false, true>(op, tile, am, a, grid, s);
}

}  // namespace jr
