// jr_conv_halo.hip — bf16 forward convolution of the stride-1, 'same'-padded
// spatial layers (1x7, 7x1, 3x3, 1x3, 3x1 at 17^2 / 35^2 / 8^2) with a
// HALO-TILED input operand.
//
// The implicit-GEMM kernel (jr_conv_bf16.hip) streams the im2col A operand:
// every K-tile is one tap's BM x BK slice, so each input pixel crosses the
// L2 -> LDS path kh*kw times per block, and a K-tile carries only a few MFMAs
// per wave against one barrier and its DMA (the 17^2 GEMMs run
// at 0.1 of the MFMA peak, bound by operand delivery).  Here a block's
// K-loop runs over channel chunks of 32: per chunk it loads the input rows
// its BM output pixels touch, with the kw - 1 halo columns, ONCE (slot
// (row, col) = input pixel (global row, col - pw), 64 B = 32 channels), plus
// the W^T rows of every tap, and the MFMAs of all kh*kw taps read A fragments
// as shifted windows of that halo image.  A output pixel whose tap falls in
// another image's row (a tile may span two images) or off the tensor reads a
// zero slot instead (the last slot of the image, never loaded with data).
//
// Per block and chunk: halo slots (rows spanned + kh - 1) x (w + kw - 1)
// against BM x kh*kw im2col rows (17^2 1x7, BM = 128: 207 vs 896), and
// 2*kh*kw MFMA k-steps per barrier instead of 2.  Same epilogue (fused BN
// statistics, staged row-vector stores) and split-K slabs as the GEMM kernel.
// Selected per layer as extra bf16 tile configurations (kHaloBf16: tile ids
// kNumCfgsBf16...), so autotuning and the pinned tables decide where it runs.
#include "jr_conv_impl.h"

namespace jr {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int KH, int KW, int BM, int BN, int WGM, int NBUF, int SLOTS>
__global__ void __launch_bounds__(256) k_conv_halo(ConvArgs g) {
  constexpr int BK = 32;                       // channels per chunk: 4 x 16 B pieces per slot
  constexpr int TAPS = KH * KW;
  constexpr int WGN = 4 / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 32, TN = WN / 32;
  static_assert(WM % 32 == 0 && WN % 32 == 0, "wave tile must be a multiple of 32x32");
  static_assert(SLOTS % 16 == 0 && (TAPS * BN) % 16 == 0, "images must be whole DMA instructions");
  constexpr int A_INSTR = SLOTS / 16, B_INSTR = TAPS * BN / 16;
  constexpr int A_PW = (A_INSTR + 3) / 4, B_PW = (B_INSTR + 3) / 4;
  constexpr int ASZ = SLOTS * BK, BSZ = TAPS * BN * BK;   // bf16 elements
  constexpr int STAGE = ASZ + BSZ;
  constexpr int SMEM = NBUF * STAGE > 8 * stage_floats<WN>() ? NBUF * STAGE : 8 * stage_floats<WN>();
  __shared__ __attribute__((aligned(1024))) uint16_t smem[SMEM];
  constexpr int NPIECE = A_PW + B_PW;
  constexpr int per_tile = A_INSTR / 4 + B_INSTR / 4;       // DMA instructions per wave and chunk (min)
  constexpr int KSTEPS = 2 * TAPS;                          // 16-channel MFMA steps per chunk

  member_offsets(g);
  const uint16_t* __restrict__ gA = reinterpret_cast<const uint16_t*>(g.A);
  const uint16_t* __restrict__ gB = reinterpret_cast<const uint16_t*>(g.B);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm0 = (wave / WGN) * WM;
  const int wn0 = (wave % WGN) * WN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = tile / g.ntn, nt = tile - mt * g.ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int kt0 = blockIdx.z * g.kt_per_split;
  const int kt1 = min(g.ktiles, kt0 + g.kt_per_split);
  const uint16_t* zp = reinterpret_cast<const uint16_t*>(g_zero_page);
  const int WP = g.halo_wp;                  // w + kw - 1 slot columns
  const int gr0 = m0 / g.wo;                 // first output row (over all images) of the tile
  const int glo = gr0 - g.ph;                // input row (over all images) of halo row 0; h == ho
  const int nslots = g.halo_nr * WP;         // host: nslots < SLOTS
  const int grows = g.n * g.h;

  // ---- A: the halo image; lane piece e = 64 j + lane -> slot e / 4, quad
  // position e % 4 holding channel quad (e % 4) ^ swz(slot)
  const uint16_t* a_ptr[A_PW];
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
        a_ptr[i] = gA + (((long long)G * g.w + iw) * g.xs + g.xo + q * 8);
    }
  }
  // ---- B: W^T [c_out][kh][kw][cp] rows (tap t, column nn) of the chunk
  const uint16_t* b_ptr[B_PW];
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int j = wave + 4 * i;
    b_ptr[i] = nullptr;
    if (B_INSTR % 4 != 0 && j >= B_INSTR) continue;
    const int e = j * 64 + lane;
    const int row = e >> 2, q = (e & 3) ^ ((row >> 2) & 3);
    const int t = row / BN, n = n0 + row - t * BN;
    if (n < g.N) b_ptr[i] = gB + ((long long)n * g.K + t * g.cp + q * 8);
  }
  auto issue_piece = [&](int kt, int d, uint16_t* __restrict__ As, uint16_t* __restrict__ Bs) {
    if (d < A_PW) {
      const int j = wave + 4 * d;
      if (A_INSTR % 4 != 0 && j >= A_INSTR) return;
      dma16(a_ptr[d] ? a_ptr[d] + kt * BK : zp, As + j * 512);
      return;
    }
    const int i = d - A_PW;
    const int j = wave + 4 * i;
    if (B_INSTR % 4 != 0 && j >= B_INSTR) return;
    dma16(b_ptr[i] ? b_ptr[i] + kt * BK : zp, Bs + j * 512);
  };

  // ---- A fragment geometry per 32-row group i: halo slot of tap (0, 0)
  // and the output row inside its image (row taps crossing the image edge
  // read the zero slot)
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

  auto step = [&](int kt, auto do_issue, const uint16_t* __restrict__ As, const uint16_t* __restrict__ Bs,
                  uint16_t* __restrict__ wA, uint16_t* __restrict__ wB) {
    constexpr bool DO_ISSUE = decltype(do_issue)::value;
#pragma unroll
    for (int t = 0; t < TAPS; ++t) {
      const int r = t / KW, c = t - (t / KW) * KW;
      int so[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bool ok = KH == 1 || (unsigned)(ohv[i] + r - g.ph) < (unsigned)g.h;
        so[i] = ok ? sb[i] + r * WP + c : SLOTS - 1;
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(As + so[i] * BK + (((2 * ks + lh) ^ ((so[i] >> 2) & 3)) * 8));
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = t * BN + wn0 + j * 32 + l31;
          bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + row * BK + (((2 * ks + lh) ^ ((row >> 2) & 3)) * 8));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        if constexpr (DO_ISSUE) {
          const int gs = 2 * t + ks;
#pragma unroll
          for (int d = gs * NPIECE / KSTEPS; d < (gs + 1) * NPIECE / KSTEPS; ++d) issue_piece(kt + NBUF - 1, d, wA, wB);
        }
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
  conv_epilogue<OP_FWD, WM, TM, TN, true>(g, acc, reinterpret_cast<float*>(smem) + wave * stage_floats<WN>(),
                                          m0 + wm0, n0 + wn0, lane);
}

template <int H>
static void launch_halo_t(const ConvArgs& a, dim3 grid, hipStream_t s) {
  constexpr HaloCfg c = kHaloBf16[H];
  hipLaunchKernelGGL((k_conv_halo<c.kh, c.kw, c.t.bm, c.t.bn, c.t.wgm, c.t.nbuf, c.slots>), grid, dim3(256), 0, s,
                     a);
}

void launch_conv_halo(int h, const ConvArgs& a, dim3 grid, hipStream_t s) {
  static_assert(kNumHaloBf16 == 8, "keep the switch in sync with kHaloBf16");
  switch (h) {
    case 0: launch_halo_t<0>(a, grid, s); break;
    case 1: launch_halo_t<1>(a, grid, s); break;
    case 2: launch_halo_t<2>(a, grid, s); break;
    case 3: launch_halo_t<3>(a, grid, s); break;
    case 4: launch_halo_t<4>(a, grid, s); break;
    case 5: launch_halo_t<5>(a, grid, s); break;
    case 6: launch_halo_t<6>(a, grid, s); break;
    default: launch_halo_t<7>(a, grid, s); break;
  }
}

}  // namespace jr
