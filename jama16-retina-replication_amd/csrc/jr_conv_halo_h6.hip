// jr_conv_halo_h6.hip — JR_F32_X6H forward convolution of the stride-1,
// 'same'-padded spatial layers (1x7 / 7x1 at 17^2, 3x3 at 147^2 / 35^2 / 8^2,
// 1x3 / 3x1 at 8^2) with a HALO-TILED fp32 input operand: the fp32 sibling
// of jr_conv_halo.hip (which see for the halo image, its zero slot and the
// row-edge rule).
//
// The x6h implicit GEMM (k_conv H6) streams the im2col A operand, so every
// input pixel crosses L2 -> LDS kh*kw times per block; here a block's K loop
// runs over chunks of 16 input channels (one 64-byte slot per pixel, the
// byte geometry of the bf16 kernel's 32-channel slots): per chunk it loads
// the input rows its BM output pixels touch, with the kw - 1 halo columns,
// ONCE, plus the HWIO filter rows [tap][16 channels][BN] of every tap (n-
// contiguous, read by the fragments as the GEMM's FWD B operand is), and the
// MFMAs of all taps read their A fragments as shifted windows of the halo
// image.  Each fragment is split as SplitFrag16 (jr_conv.hip: the operand
// scaled by its power of two, three fp16 terms, six f16 MFMAs), acc scaled
// back before the shared epilogue (fused BN statistics, split-K slabs).
// Selected per layer as extra JR_F32_X6H tile ids (kHaloF32, ids 42..), so
// autotuning and the pinned tables decide where it runs.
#include "jr_conv_impl.h"

namespace jr {

typedef _Float16 f16x8h __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2h __attribute__((ext_vector_type(2)));

namespace {

__device__ __forceinline__ uint32_t pkrtz(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(a, b));
}

__device__ __forceinline__ float subv(float a, float b) {
  float r;
  asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// the exact-to-scale fp16 three-way split of 8 fp32 values (SplitFrag16)
struct Split16 {
  uint32_t hp[4], mp[4], lp[4];
  __device__ __forceinline__ void make(const float* v, float scale) {
    float x[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) x[t] = v[t] * scale;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      hp[p] = pkrtz(x[2 * p], x[2 * p + 1]);
      const f16x2h h = __builtin_bit_cast(f16x2h, hp[p]);
      x[2 * p] = subv(x[2 * p], (float)h[0]);
      x[2 * p + 1] = subv(x[2 * p + 1], (float)h[1]);
      mp[p] = pkrtz(x[2 * p], x[2 * p + 1]);
      const f16x2h m = __builtin_bit_cast(f16x2h, mp[p]);
      x[2 * p] = subv(x[2 * p], (float)m[0]);
      x[2 * p + 1] = subv(x[2 * p + 1], (float)m[1]);
      lp[p] = pkrtz(x[2 * p], x[2 * p + 1]);
    }
  }
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  __device__ __forceinline__ f16x8h h() const { return __builtin_bit_cast(f16x8h, (u32x4){hp[0], hp[1], hp[2], hp[3]}); }
  __device__ __forceinline__ f16x8h m() const { return __builtin_bit_cast(f16x8h, (u32x4){mp[0], mp[1], mp[2], mp[3]}); }
  __device__ __forceinline__ f16x8h l() const { return __builtin_bit_cast(f16x8h, (u32x4){lp[0], lp[1], lp[2], lp[3]}); }
};

}  // namespace

template <int KH, int KW, int BM, int BN, int WGM, int NBUF, int SLOTS>
__global__ void __launch_bounds__(256) k_conv_halo_h6(ConvArgs g) {
  constexpr int BK = 16;                       // channels per chunk: 4 x 16 B pieces per slot
  constexpr int TAPS = KH * KW;
  constexpr int WGN = 4 / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 32, TN = WN / 32;
  static_assert(WM % 32 == 0 && WN % 32 == 0, "wave tile must be a multiple of 32x32");
  static_assert(SLOTS % 16 == 0 && (TAPS * BN) % 16 == 0, "images must be whole DMA instructions");
  constexpr int A_INSTR = SLOTS / 16, B_INSTR = TAPS * BN / 16;
  constexpr int A_PW = (A_INSTR + 3) / 4, B_PW = (B_INSTR + 3) / 4;
  constexpr int ASZ = SLOTS * BK, BSZ = TAPS * BK * BN;    // floats
  constexpr int STAGE = ASZ + BSZ;
  constexpr int SMEM = NBUF * STAGE > 4 * stage_floats<WN>() ? NBUF * STAGE : 4 * stage_floats<WN>();
  __shared__ __attribute__((aligned(1024))) float smem[SMEM];
  constexpr int NPIECE = A_PW + B_PW;
  constexpr int per_tile = A_INSTR / 4 + B_INSTR / 4;       // DMA instructions per wave and chunk (min)

  member_offsets(g);
  const float* __restrict__ gA = g.A;
  const float* __restrict__ gB = g.B;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const float h_sa = __uint_as_float(__builtin_amdgcn_readfirstlane(
      __float_as_uint(pow2_scale(g.a_max ? absmax64(g.a_max, lane) : g.a_bnd))));
  const float h_sb = __uint_as_float(__builtin_amdgcn_readfirstlane(
      __float_as_uint(pow2_scale(g.b_max ? absmax64(g.b_max, lane) : g.b_bnd))));
  const int wm0 = (wave / WGN) * WM;
  const int wn0 = (wave % WGN) * WN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = tile / g.ntn, nt = tile - mt * g.ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int kt0 = blockIdx.z * g.kt_per_split;
  const int kt1 = min(g.ktiles, kt0 + g.kt_per_split);
  const float* zp = g_zero_page;
  const int WP = g.halo_wp;                  // w + kw - 1 slot columns
  const int gr0 = m0 / g.wo;                 // first output row (over all images) of the tile
  const int glo = gr0 - g.ph;                // input row (over all images) of halo row 0; h == ho
  const int nslots = g.halo_nr * WP;         // host: nslots < SLOTS
  const int grows = g.n * g.h;

  // ---- A: the halo image; lane piece e = 64 j + lane -> slot e / 4, LDS
  // quad e % 4 holding channel quad (e % 4) ^ swz(slot)
  const float* a_ptr[A_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int j = wave + 4 * i;
    a_ptr[i] = nullptr;
    if (A_INSTR % 4 != 0 && j >= A_INSTR) continue;
    const int e = j * 64 + lane;
    const int s = e >> 2, q = (e & 3) ^ ((s >> 2) & 3);
    if (s < nslots) {
      const int sr = s / WP, sc = s - sr * WP;
      const int G = glo + sr, iw = sc - g.pw;
      if ((unsigned)G < (unsigned)grows && (unsigned)iw < (unsigned)g.w)
        a_ptr[i] = gA + (((long long)G * g.w + iw) * g.xs + g.xo + q * 4);
    }
  }
  // ---- B: HWIO rows (tap t, channel k of the chunk), BN couts each: piece
  // e -> row e / (BN / 4), couts n0 + 4 (e % (BN / 4)) .. + 3
  const float* b_ptr[B_PW];
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int j = wave + 4 * i;
    b_ptr[i] = nullptr;
    if (B_INSTR % 4 != 0 && j >= B_INSTR) continue;
    const int e = j * 64 + lane;
    const int row = e / (BN / 4), pc = e - row * (BN / 4);
    const int t = row / BK, k = row - t * BK;
    const int n = n0 + pc * 4;
    if (n < g.N) b_ptr[i] = gB + (((long long)t * g.cin + k) * g.cout + n);
  }
  auto issue_piece = [&](int kt, int d, float* __restrict__ As, float* __restrict__ Bs) {
    if (d < A_PW) {
      const int j = wave + 4 * d;
      if (A_INSTR % 4 != 0 && j >= A_INSTR) return;
      dma16(a_ptr[d] ? a_ptr[d] + kt * BK : zp, As + j * 256);
      return;
    }
    const int i = d - A_PW;
    const int j = wave + 4 * i;
    if (B_INSTR % 4 != 0 && j >= B_INSTR) return;
    dma16(b_ptr[i] ? b_ptr[i] + (long long)kt * BK * g.cout : zp, Bs + j * 256);
  };

  // ---- A fragment geometry per 32-row group i: halo slot of tap (0, 0)
  // and the output row inside its image
  const int l31 = lane & 31, lh = lane >> 5;
  int sb[TM], ohv[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm0 + i * 32 + l31;
    if (m < g.M) {
      const int gr = m / g.wo, ow = m - gr * g.wo;
      sb[i] = (gr - gr0) * WP + ow;
      ohv[i] = gr - (gr / g.ho) * g.ho;
    } else {
      sb[i] = 0;
      ohv[i] = -(1 << 20);
    }
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto step = [&](int kt, auto do_issue, const float* __restrict__ As, const float* __restrict__ Bs,
                  float* __restrict__ wA, float* __restrict__ wB) {
    constexpr bool DO_ISSUE = decltype(do_issue)::value;
#pragma unroll
    for (int t = 0; t < TAPS; ++t) {
      const int r = t / KW, c = t - (t / KW) * KW;
      Split16 sa[TM], sbf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bool ok = KH == 1 || (unsigned)(ohv[i] + r - g.ph) < (unsigned)g.h;
        const int so = ok ? sb[i] + r * WP + c : SLOTS - 1;
        const int sw = (so >> 2) & 3;
        const float4 v0 = *reinterpret_cast<const float4*>(As + so * BK + (((2 * lh) ^ sw) * 4));
        const float4 v1 = *reinterpret_cast<const float4*>(As + so * BK + (((2 * lh + 1) ^ sw) * 4));
        const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        sa[i].make(v, h_sa);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        float v[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) v[s] = Bs[(t * BK + lh * 8 + s) * BN + wn0 + j * 32 + l31];
        sbf[j].make(v, h_sb);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          f32x16 a = acc[i][j];
          a = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[i].h(), sbf[j].h(), a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[i].m(), sbf[j].h(), a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[i].h(), sbf[j].m(), a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[i].m(), sbf[j].m(), a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[i].l(), sbf[j].h(), a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_32x32x16_f16(sa[i].h(), sbf[j].l(), a, 0, 0, 0);
          acc[i][j] = a;
        }
      if constexpr (DO_ISSUE) {
#pragma unroll
        for (int d = t * NPIECE / TAPS; d < (t + 1) * NPIECE / TAPS; ++d) issue_piece(kt + NBUF - 1, d, wA, wB);
      }
    }
  };
  auto buf_a = [&](int b) { return smem + b * STAGE; };
  auto buf_b = [&](int b) { return smem + b * STAGE + ASZ; };

  if (kt0 < kt1) {
#pragma unroll
    for (int p = 0; p < NBUF - 1; ++p)
      if (kt0 + p < kt1)
#pragma unroll
        for (int d = 0; d < NPIECE; ++d) issue_piece(kt0 + p, d, buf_a(p), buf_b(p));
    wait_vmcnt(per_tile * min(NBUF - 2, kt1 - kt0 - 1));
    __builtin_amdgcn_s_barrier();
    int cur = 0;
    int kt = kt0;
    for (; kt < kt1 - (NBUF - 1); ++kt) {
      const int nxt = cur == 0 ? NBUF - 1 : cur - 1;
      step(kt, std::true_type{}, buf_a(cur), buf_b(cur), buf_a(nxt), buf_b(nxt));
      __builtin_amdgcn_sched_barrier(0);
      wait_vmcnt(per_tile * (NBUF - 2));
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      cur = cur + 1 == NBUF ? 0 : cur + 1;
    }
    for (; kt < kt1; ++kt) {
      step(kt, std::false_type{}, buf_a(cur), buf_b(cur), nullptr, nullptr);
      __builtin_amdgcn_sched_barrier(0);
      wait_vmcnt(per_tile * max(0, min(NBUF - 2, kt1 - kt - 2)));
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      cur = cur + 1 == NBUF ? 0 : cur + 1;
    }
  }
  {   // back from the operands' power-of-two scales (exact)
    const float ia = 1.f / h_sa, ib = 1.f / h_sb;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = acc[i][j][r] * ia * ib;
  }
  conv_epilogue<OP_FWD, WM, TM, TN, false>(g, acc, smem + wave * stage_floats<WN>(), m0 + wm0, n0 + wn0, lane);
}

template <int H>
static void launch_halo_h6_t(const ConvArgs& a, dim3 grid, hipStream_t s) {
  constexpr HaloCfg c = kHaloF32[H];
  hipLaunchKernelGGL((k_conv_halo_h6<c.kh, c.kw, c.t.bm, c.t.bn, c.t.wgm, c.t.nbuf, c.slots>), grid, dim3(256), 0,
                     s, a);
}

void launch_conv_halo_h6(int h, const ConvArgs& a, dim3 grid, hipStream_t s) {
  static_assert(kNumHaloF32 == 9, "keep the switch in sync with kHaloF32");
  switch (h) {
    case 0: launch_halo_h6_t<0>(a, grid, s); break;
    case 1: launch_halo_h6_t<1>(a, grid, s); break;
    case 2: launch_halo_h6_t<2>(a, grid, s); break;
    case 3: launch_halo_h6_t<3>(a, grid, s); break;
    case 4: launch_halo_h6_t<4>(a, grid, s); break;
    case 5: launch_halo_h6_t<5>(a, grid, s); break;
    case 6: launch_halo_h6_t<6>(a, grid, s); break;
    case 7: launch_halo_h6_t<7>(a, grid, s); break;
    default: launch_halo_h6_t<8>(a, grid, s); break;
  }
}

}  // namespace jr
