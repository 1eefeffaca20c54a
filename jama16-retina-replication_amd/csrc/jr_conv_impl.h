// jr_conv_impl.h — pieces shared by the fp32 (jr_conv.hip) and bf16
// (jr_conv_bf16.hip) implicit-GEMM convolution kernels: GEMM arguments,
// output addressing, counted waits, LDS-DMA, the split-K reduce, and the
// tile-configuration tables the host planner ranks and autotunes.
#pragma once
#include "jr_common.h"

#include <type_traits>

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
  // FWD only: fused BatchNorm statistics partials (nullptr = none), laid out
  // stats[2][N][stats_p]: per-column (mean, M2) of each group of WM rows
  float* stats;
  int stats_p;
  // DGRAD phase (py,px): taps r = r0 + sh*a (a < na), c = c0 + sw*b (b < nb);
  // m = (b, u, v) over hc x wc; ih = sh*u + py; oh = u + ey - a.
  int py, px, r0, c0, na, nb, ey, ex, hc, wc;
  // JR_F32_X8P: element stride between the h, m and l planes of A and of B
  long long a_ps, b_ps;
  // halo-tiled FWD (jr_conv_halo.hip): halo rows per block and slot columns
  int halo_nr, halo_wp;
  // diagnostic builds only (-DJR_STAMPS, `make stamps`): per-block s_memtime /
  // s_memrealtime stamps, 8 per block (jr_debug_set_stamps); nullptr otherwise
  unsigned long long* dbg;
  // grouped launches (ensemble members, jr_conv2d_fwd_bn_stats_grouped): the
  // member is blockIdx.y of the GEMM; byte strides between consecutive
  // members of A, B, C (the output, or the member's split-K slab region),
  // the statistics partials and the final output (split-K reduce)
  long long a_mb, b_mb, c_mb, s_mb, o_mb;
  // stream-K (jr_conv.hip k_conv SK): iterations (tile-major, K-tile-minor)
  // per block, the per-owner-block hand-off counts (stream_scratch words:
  // zero at launch, and the block that completes a count resets it) and the
  // partial-tile slots (workspace, two per block); sk_fmb / sk_mb = their
  // member strides
  long long sk_ipb, sk_mb, sk_fmb;
  unsigned* sk_flags;
  float* sk_part;
  // the library's device error word (jr_device_check)
  unsigned* sk_err;
  // JR_F32_X6H: magnitude bounds of the A / B operands for their
  // power-of-two scales: 64 device floats whose max is max |operand|
  // (nullptr: the host bound a_bnd / b_bnd; 0 = 2^14, scale 1)
  const float* a_max;
  const float* b_max;
  float a_bnd, b_bnd;
};

// max of the 64 floats at p (every lane of the wave gets it)
__device__ __forceinline__ float absmax64(const float* p, int lane) {
  float v = p[lane];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// 2^k with m 2^k in [2^14, 2^15) (m = 0, inf or NaN: 1; k <= 100): the
// JR_F32_X6H operand scale for a tensor whose largest magnitude is m
__device__ __forceinline__ float pow2_scale(float m) {
  const unsigned b = __float_as_uint(m);
  const int eb = (int)((b >> 23) & 0xffu);
  if (!(m > 0.f) || eb == 255) return 1.f;
  const int biased = min(268 - eb, 227);
  return __uint_as_float((unsigned)biased << 23);
}

// Moves a grouped GEMM's operand / output pointers to member blockIdx.y
// (a no-op for ordinary launches, gridDim.y == 1).
__device__ __forceinline__ void member_offsets(ConvArgs& g) {
  if (gridDim.y > 1) {
    const long long m = blockIdx.y;
    g.A = reinterpret_cast<const float*>(reinterpret_cast<const char*>(g.A) + m * g.a_mb);
    g.B = reinterpret_cast<const float*>(reinterpret_cast<const char*>(g.B) + m * g.b_mb);
    g.C = reinterpret_cast<float*>(reinterpret_cast<char*>(g.C) + m * g.c_mb);
    if (g.stats) g.stats = reinterpret_cast<float*>(reinterpret_cast<char*>(g.stats) + m * g.s_mb);
    // JR_F32_X6H grouped: each member's 64 magnitude words follow the previous member's
    if (g.a_max) g.a_max += 64 * m;
    if (g.b_max) g.b_max += 64 * m;
    if (g.sk_flags) {
      g.sk_flags = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(g.sk_flags) + m * g.sk_fmb);
      g.sk_part = reinterpret_cast<float*>(reinterpret_cast<char*>(g.sk_part) + m * g.sk_mb);
    }
  }
}

#ifdef JR_STAMPS
// [0] realtime at start, [1] realtime at end (100 MHz), [2] cycles of the
// prologue (ring fill to the first barrier), [3] cycles of the K loop, [4]
// cycles of the epilogue, [5] cycles the loop spent in vmcnt waits +
// barriers, [6] HW_ID, [7] XCC_ID -- of wave 0 of the block
struct Stamps {
  unsigned long long r0, c0, cp, cl, w;
  __device__ __forceinline__ void start() {
    r0 = __builtin_amdgcn_s_memrealtime();
    c0 = __builtin_amdgcn_s_memtime();
    w = 0;
  }
  __device__ __forceinline__ void prologue() { cp = __builtin_amdgcn_s_memtime(); }
  __device__ __forceinline__ void loop() { cl = __builtin_amdgcn_s_memtime(); }
  __device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memtime(); }
  __device__ __forceinline__ void end(unsigned long long* dbg) {
    const unsigned long long ce = __builtin_amdgcn_s_memtime(), re = __builtin_amdgcn_s_memrealtime();
    if (dbg == nullptr || threadIdx.x != 0) return;
    unsigned long long* o = dbg + 8ull * (blockIdx.z * gridDim.x + blockIdx.x);
    o[0] = r0; o[1] = re; o[2] = cp - c0; o[3] = cl - cp; o[4] = ce - cl; o[5] = w;
    o[6] = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    o[7] = __builtin_amdgcn_s_getreg((3 << 11) | 20);    // HW_REG_XCC_ID
  }
};
#define JR_ST(x) x
#else
#define JR_ST(x)
#endif

// Input pixel (over all images) of DGRAD row m of the phase.
__device__ __forceinline__ long long dgrad_pix(const ConvArgs& g, int m) {
  const int hw = g.hc * g.wc;
  const int b = m / hw, rem = m - b * hw;
  const int u = rem / g.wc, v = rem - u * g.wc;
  return ((long long)b * g.h + g.sh * u + g.py) * g.w + g.sw * v + g.px;
}

// Output element offset of GEMM row m (column 0), or -1 to drop the row.
template <int OP>
__device__ __forceinline__ long long out_row(const ConvArgs& g, int m) {
  if constexpr (OP == OP_FWD) {
    return (long long)m * g.c_stride + g.c_off;
  } else if constexpr (OP == OP_DGRAD) {
    return dgrad_pix(g, m) * g.c_stride + g.c_off;
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
#define JR_VMCNT_CASE(k) case k: asm volatile("s_waitcnt vmcnt(" #k ") lgkmcnt(0)" ::: "memory"); break;
  switch (n) {
    JR_VMCNT_CASE(0) JR_VMCNT_CASE(1) JR_VMCNT_CASE(2) JR_VMCNT_CASE(3) JR_VMCNT_CASE(4) JR_VMCNT_CASE(5)
    JR_VMCNT_CASE(6) JR_VMCNT_CASE(7) JR_VMCNT_CASE(8) JR_VMCNT_CASE(9) JR_VMCNT_CASE(10) JR_VMCNT_CASE(11)
    JR_VMCNT_CASE(12) JR_VMCNT_CASE(13) JR_VMCNT_CASE(14) JR_VMCNT_CASE(15) JR_VMCNT_CASE(16) JR_VMCNT_CASE(17)
    JR_VMCNT_CASE(18) JR_VMCNT_CASE(19) JR_VMCNT_CASE(20) JR_VMCNT_CASE(21) JR_VMCNT_CASE(22) JR_VMCNT_CASE(23)
    JR_VMCNT_CASE(24) JR_VMCNT_CASE(25) JR_VMCNT_CASE(26) JR_VMCNT_CASE(27) JR_VMCNT_CASE(28) JR_VMCNT_CASE(29)
    JR_VMCNT_CASE(30)
    default: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); break;
  }
#undef JR_VMCNT_CASE
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

// The same LDS-DMA piece issued from inline asm, for k_conv, whose K loop
// orders every DMA against the LDS reads itself (counted wait_vmcnt +
// s_barrier per K-tile).  hipcc's waitcnt pass cannot see through the
// stream-K hand-off: with the builtin it put an s_waitcnt vmcnt(0) before
// the first LDS read of every K-tile in most stream-K kernels (168 of 518
// k_conv steady loops; the non-stream-K twins had none), draining the ring's
// prefetch each iteration; invisible to that pass, the DMA is waited for
// where the kernel waits, and with one explicit vmcnt(0) per stream-K
// segment (k_conv) no steady loop keeps a drain (490 of 490; fp32 step
// -0.8 %, profiles/r06_ab_dmaring.txt).  k_conv_bf16 keeps the builtin: its
// step was 0.5 % slower this way.  m0 is written here only (the compiler
// uses it for nothing else in these kernels: checked in the build's
// assembly), and an SALU write of m0 needs one wait state before an LDS DMA
// reads it (gfx9), hence the s_nop.
__device__ __forceinline__ void dma16_ring(const void* src, void* lds_chunk) {
  const uint32_t l = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) void*)lds_chunk);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :: "v"(src), "s"(__builtin_amdgcn_readfirstlane(l)) : "memory");
}

// ---------------------------------------------------------------- stream-K
// Hand-off of a cut tile's pieces (jr_conv.hip k_conv SK documents the
// scheme; k_conv_bf16 uses the same).  No block ever waits for another:
// every piece is published to its block's slot (write-through sc1 stores,
// drained) and then counted on the tile's word (one per owner block, the
// block holding the tile's first K-tile); the block whose count completes
// the tile adds the pieces in block order -- the owner's first -- and
// finishes the tile, the others move on.  (Round 4's owner polled for the
// later pieces: with two lanes, or two processes, sharing the CUs a grid's
// later blocks need not be resident, and owners spun until their bound --
// an error raised by jr_device_check, seen on the 2-rank one-device eval.)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sk_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// Returns true in the block that finishes the tile, with acc = the sum of
// the npieces pieces of blocks owner, owner + 1, ... in that order (each
// piece's fp32 values exactly as its block accumulated them: bitwise the
// owner-absorbs order of round 4).  kind: 1 = this is the owner's piece (its
// last segment, starting at K-tile 0), 0 = a later block's (its first
// segment).  The owner's word counts published pieces (low 16 bits) plus an
// owner bit: the owner first only probes -- when every later piece is
// already published (the usual case: later blocks publish at the START of
// their ranges, the owner reaches its piece at the END of its range) it
// finishes from its registers without publishing; otherwise it publishes and
// counts like any piece.  A count found past npieces (a word not left zero)
// goes to the device error word (jr_device_check).
template <int TM, int TN, int NW = 4>
__device__ __forceinline__ void sk_store_piece(const ConvArgs& g, const f32x16 (&acc)[TM][TN], int wave, int lane,
                                               long long slot) {
  constexpr int SLOT = NW * TM * TN * 16 * 64;              // floats per slot (BM x BN)
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const auto rs = sk_rsrc(g.sk_part + slot * SLOT);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const i32x4 v = {__float_as_int(acc[i][j][4 * q]), __float_as_int(acc[i][j][4 * q + 1]),
                         __float_as_int(acc[i][j][4 * q + 2]), __float_as_int(acc[i][j][4 * q + 3])};
        const int off = (((((wave * TM + i) * TN + j) * 4 + q) * 64) + lane) * 16;
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16);    // aux 16 = sc1 (write-through)
      }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");           // every storing wave drains
}

// acc (= the owner's piece, in registers) += pieces 1 .. npieces - 1, in
// order, from their slots; load_first: acc is first set to the owner's piece
// from its slot (a later block finishing the tile).
template <int TM, int TN, int NW = 4>
__device__ __forceinline__ void sk_sum_pieces(const ConvArgs& g, f32x16 (&acc)[TM][TN], int wave, int lane, int owner,
                                              int npieces, bool load_first) {
  constexpr int SLOT = NW * TM * TN * 16 * 64;
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // (no instruction: keeps the loads below the count)
  if (load_first) {   // the owner's piece sits in its second slot
    const auto rs = sk_rsrc(g.sk_part + (2LL * owner + 1) * SLOT);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (((((wave * TM + i) * TN + j) * 4 + q) * 64) + lane) * 16,
                                                                0, 16);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][4 * q + e] = __int_as_float(v[e]);
        }
  }
  for (int k = 1; k < npieces; ++k) {   // every later block's piece sits in its first slot
    const auto rs = sk_rsrc(g.sk_part + 2LL * (owner + k) * SLOT);
    // one accumulator row i at a time (TN x 4 loads in flight): the loaded
    // piece never holds more than TN x 16 VGPRs
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      i32x4 v[TN][4];
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)   // every load of the hand-off sc1 (write-through producers, drained)
          v[j][q] = __builtin_amdgcn_raw_buffer_load_b128(rs, (((((wave * TM + i) * TN + j) * 4 + q) * 64) + lane) * 16,
                                                          0, 16);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][4 * q + e] += __int_as_float(v[j][q][e]);
    }
  }
}

constexpr unsigned kSkOwnerBit = 1u << 16;   // low 16 bits: pieces published

// lb: the block's logical index (its iteration range; xcd_remap of blockIdx.x)
template <int TM, int TN, int NW = 4>
__device__ __forceinline__ bool sk_handoff(const ConvArgs& g, f32x16 (&acc)[TM][TN], int wave, int lane, int owner,
                                           int npieces, int kind, int lb) {
  // s_state: 0 move on, 1 finish with the owner's piece in registers, 2 finish loading every piece
  __shared__ int s_state;
  unsigned* word = g.sk_flags + owner;
  const unsigned n = (unsigned)npieces;
  int st = 0;
  if (kind == 1) {          // the owner: probe first
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned old = __hip_atomic_fetch_add(word, kSkOwnerBit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool all = (old & 0xffffu) == n - 1;
      if ((old >> 16) != 0 || (old & 0xffffu) >= n)
        __hip_atomic_fetch_add(g.sk_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (all) __hip_atomic_store(word, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_state = all ? 1 : 0;
    }
    __syncthreads();
    st = s_state;
    __syncthreads();
  }
  if (st == 0) {            // publish this piece, then count it
    sk_store_piece<TM, TN, NW>(g, acc, wave, lane, 2LL * lb + kind);
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned old = __hip_atomic_fetch_add(word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = (old & 0xffffu) + 1 == n;
      if ((old >> 17) != 0 || (old & 0xffffu) >= n)
        __hip_atomic_fetch_add(g.sk_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (last) __hip_atomic_store(word, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_state = last ? (kind == 1 ? 1 : 2) : 0;
    }
    __syncthreads();
    st = s_state;
    __syncthreads();        // every wave has read s_state before the next hand-off writes it
    if (st == 0) return false;                              // (uniform)
  }
  sk_sum_pieces<TM, TN, NW>(g, acc, wave, lane, owner, npieces, st == 2);
  return true;
}

// Where a stream-K segment [kt0, kt1) of `tile` hands off: true if the tile
// is cut (then owner / npieces / kind for sk_handoff).
__device__ __forceinline__ bool sk_cut(const ConvArgs& g, int tile, int kt0, int kt1, int* owner, int* npieces,
                                       int* kind) {
  if (kt0 == 0 && kt1 == g.ktiles) return false;
  const long long t0 = (long long)tile * g.ktiles;       // the tile's first iteration
  *owner = (int)(t0 / g.sk_ipb);
  *npieces = (int)((t0 + g.ktiles - 1) / g.sk_ipb) - *owner + 1;
  *kind = kt0 == 0 ? 1 : 0;
  return true;
}


// ---------------------------------------------------------------- epilogue
// A wave's WM x WN accumulator tile leaves 32 rows at a time through the
// wave's own LDS region [32][WN + 8] fp32 (the two 32-lane halves of a store
// are 4 rows = 32 banks apart, so they do not collide) and is written as
// 8-element row vectors per lane: 32 B fp32 or 16 B bf16, whole row segments
// per wave-instruction, and one vector read-modify-write per lane when
// accumulating into dx (per-element 2-byte bf16 stores and RMW were the
// epilogue's cost before).  FWD with g.stats (no split-K): per-column BN
// statistics of the wave's rows, as stored (bf16-rounded for bf16 outputs):
// mean and M2 = sum (v - mean)^2 (two passes over the registers), combined
// in fp64 by k_stats_finalize.
template <int WN> constexpr int stage_floats() { return 32 * (WN + 8); }

template <int OP, int WM, int TM, int TN, bool BF16K>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& g, f32x16 (&acc)[TM][TN], float* stage, int mw0,
                                              int nw0, int lane) {
  constexpr int WN = TN * 32, S = WN + 8, LPR = WN / 8, NIT = 32 * LPR / 64;
  static_assert((32 * LPR) % 64 == 0, "stage read-back must be whole wave-instructions");
  const bool split = gridDim.z > 1;
  const bool bout = BF16K && OP != OP_WGRAD && !split;
  const int l31 = lane & 31, lh = lane >> 5;
  auto row_of = [&](int r) { return (r & 3) + 8 * (r >> 2) + 4 * lh; };
  if constexpr (OP == OP_FWD) {
    if (g.stats != nullptr && !split) {
      const int P = g.stats_p;
      const int pidx = mw0 / WM;
      const int nv = min(max(g.M - mw0, 0), WM);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float v = acc[i][j][r];
            if (bout) { v = bf2f(f2bf(v)); acc[i][j][r] = v; }
            s += (mw0 + i * 32 + row_of(r) < g.M) ? v : 0.f;
          }
        s += __shfl_xor(s, 32, 64);
        const float mu = nv > 0 ? s / (float)nv : 0.f;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float d = acc[i][j][r] - mu;
            q += (mw0 + i * 32 + row_of(r) < g.M) ? d * d : 0.f;
          }
        q += __shfl_xor(q, 32, 64);
        const int n = nw0 + j * 32 + l31;
        if (lh == 0 && n < g.N) {
          g.stats[(long long)n * P + pidx] = mu;
          g.stats[(long long)(g.N + n) * P + pidx] = q;
        }
      }
    }
  }
  float* C = split ? g.C + (long long)blockIdx.z * g.slab_elems : g.C;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) stage[row_of(r) * S + j * 32 + l31] = acc[i][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // the group's row vectors leave in batches of CH: all stage reads and
    // (accumulate) all old-dx loads of a batch are issued before any use --
    // unconditional loads from clamped addresses, so one memory round trip
    // per batch instead of one per row vector (a per-vector `continue`
    // around the load made hipcc wait for each load in turn)
    constexpr int CH = NIT % 4 == 0 ? 4 : NIT % 3 == 0 ? 3 : NIT % 2 == 0 ? 2 : 1;
#pragma unroll
    for (int i0 = 0; i0 < NIT; i0 += CH) {
      float v[CH][8];
      long long off[CH];
      bool ok[CH];
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const int e = (i0 + k) * 64 + lane;
        const int row = e / LPR, c8 = (e - row * LPR) * 8;
        const float4 v0 = *reinterpret_cast<const float4*>(stage + row * S + c8);
        const float4 v1 = *reinterpret_cast<const float4*>(stage + row * S + c8 + 4);
        v[k][0] = v0.x; v[k][1] = v0.y; v[k][2] = v0.z; v[k][3] = v0.w;
        v[k][4] = v1.x; v[k][5] = v1.y; v[k][6] = v1.z; v[k][7] = v1.w;
        const int m = mw0 + i * 32 + row, n = nw0 + c8;
        ok[k] = m < g.M && n < g.N;
        const long long base = ok[k] ? (split ? (long long)m * g.N : out_row<OP>(g, m)) : 0;
        ok[k] = ok[k] && base >= 0;
        off[k] = ok[k] ? base + n : 0;     // element offset of the 8-vector in C (0: a safe dummy)
      }
      if (g.accumulate && !split) {        // uniform
        if (bout) {
          uint4 o[CH];
#pragma unroll
          for (int k = 0; k < CH; ++k)
            o[k] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(g.C) + off[k]);
#pragma unroll
          for (int k = 0; k < CH; ++k) {
            const uint32_t w[4] = {o[k].x, o[k].y, o[k].z, o[k].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              v[k][2 * q] += __uint_as_float(w[q] << 16);
              v[k][2 * q + 1] += __uint_as_float(w[q] & 0xffff0000u);
            }
          }
        } else {
          float4 o0[CH], o1[CH];
#pragma unroll
          for (int k = 0; k < CH; ++k) {
            const float4* p = reinterpret_cast<const float4*>(C + off[k]);
            o0[k] = p[0];
            o1[k] = p[1];
          }
#pragma unroll
          for (int k = 0; k < CH; ++k) {
            v[k][0] += o0[k].x; v[k][1] += o0[k].y; v[k][2] += o0[k].z; v[k][3] += o0[k].w;
            v[k][4] += o1[k].x; v[k][5] += o1[k].y; v[k][6] += o1[k].z; v[k][7] += o1[k].w;
          }
        }
      }
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        if (!ok[k]) continue;
        if (bout) {
          uint32_t w[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) w[q] = (uint32_t)f2bf(v[k][2 * q]) | ((uint32_t)f2bf(v[k][2 * q + 1]) << 16);
          *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(g.C) + off[k]) = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
          float4* p = reinterpret_cast<float4*>(C + off[k]);
          p[0] = make_float4(v[k][0], v[k][1], v[k][2], v[k][3]);
          p[1] = make_float4(v[k][4], v[k][5], v[k][6], v[k][7]);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
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

// FWD split-K reduce with fused BN statistics.  Block (b, y) owns rows
// [b*R, (b+1)*R) (so its statistics partial covers exactly those rows) of
// columns [1024 y, 1024 y + 1024), thread (q, rr) one float4 column group q
// and rows rr, rr+rpp, ...; the
// output is written as in k_splitk_reduce (bf16 rounded once).  Per thread
// shifted sums about its first value, then (count, mean, M2) combined over
// the row phases by a fixed-shape Chan tree: deterministic.
template <typename TO>
__global__ void __launch_bounds__(256) k_splitk_reduce_stats(const float* __restrict__ slab, int splits, ConvArgs g,
                                                             TO* out, int R) {
  if (gridDim.z > 1) {   // grouped: member blockIdx.z
    const long long mz = blockIdx.z;
    slab = reinterpret_cast<const float*>(reinterpret_cast<const char*>(slab) + mz * g.c_mb);
    out = reinterpret_cast<TO*>(reinterpret_cast<char*>(out) + mz * g.o_mb);
    g.stats = reinterpret_cast<float*>(reinterpret_cast<char*>(g.stats) + mz * g.s_mb);
  }
  __shared__ float s_n[256];
  __shared__ float4 s_mu[256], s_m2[256];
  const int cb = blockIdx.y * 1024;
  const int tpr = min(1024, g.N - cb) >> 2;
  const int rpp = 256 / tpr;
  const int t = threadIdx.x;
  const int q = t % tpr, rr = t / tpr;
  const int c0 = cb + q * 4;
  const int r0 = blockIdx.x * R, r1 = min(g.M, r0 + R);
  float kk[4] = {0.f, 0.f, 0.f, 0.f}, a1[4] = {0.f, 0.f, 0.f, 0.f}, a2[4] = {0.f, 0.f, 0.f, 0.f};
  int cnt = 0;
  if (rr < rpp) {
    for (int m = r0 + rr; m < r1; m += rpp) {
      const float4* src = reinterpret_cast<const float4*>(slab + (long long)m * g.N + c0);
      const long long zs = g.slab_elems >> 2;
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      int z = 0;
      for (; z + 3 < splits; z += 4) {
        const float4 a = src[z * zs], b = src[(z + 1) * zs], c = src[(z + 2) * zs], d = src[(z + 3) * zs];
        s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
        s.x += b.x; s.y += b.y; s.z += b.z; s.w += b.w;
        s.x += c.x; s.y += c.y; s.z += c.z; s.w += c.w;
        s.x += d.x; s.y += d.y; s.z += d.z; s.w += d.w;
      }
      for (; z < splits; ++z) {
        const float4 a = src[z * zs];
        s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
      }
      float v[4] = {s.x, s.y, s.z, s.w};
      TO* p = out + out_row<OP_FWD>(g, m) + c0;
      if constexpr (sizeof(TO) == 4) {
        *reinterpret_cast<float4*>(p) = s;
      } else {
        const uint16_t b0 = f2bf(v[0]), b1 = f2bf(v[1]), b2 = f2bf(v[2]), b3 = f2bf(v[3]);
        *reinterpret_cast<uint2*>(p) = make_uint2((uint32_t)b0 | ((uint32_t)b1 << 16), (uint32_t)b2 | ((uint32_t)b3 << 16));
        v[0] = bf2f(b0); v[1] = bf2f(b1); v[2] = bf2f(b2); v[3] = bf2f(b3);
      }
      if (cnt == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) kk[j] = v[j];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[j] - kk[j];
        a1[j] += d;
        a2[j] = fmaf(d, d, a2[j]);
      }
      ++cnt;
    }
  }
  float mu[4], m2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    mu[j] = cnt ? kk[j] + a1[j] / (float)cnt : 0.f;
    m2[j] = cnt ? fmaxf(a2[j] - a1[j] * a1[j] / (float)cnt, 0.f) : 0.f;
  }
  s_n[t] = (float)cnt;
  s_mu[t] = make_float4(mu[0], mu[1], mu[2], mu[3]);
  s_m2[t] = make_float4(m2[0], m2[1], m2[2], m2[3]);
  __syncthreads();
  int span = 1;
  while (span < rpp) span <<= 1;
  for (int h = span >> 1; h > 0; h >>= 1) {
    if (rr < h && rr + h < rpp) {
      const int o = t + h * tpr;
      const float na = s_n[t], nb = s_n[o], nn = na + nb;
      if (nb > 0.f) {
        const float4 ma = s_mu[t], mb = s_mu[o], qa = s_m2[t], qb = s_m2[o];
        const float fa = na / nn, fb = nb / nn, w = na * nb / nn;
        const float dx = mb.x - ma.x, dy = mb.y - ma.y, dz = mb.z - ma.z, dw = mb.w - ma.w;
        s_mu[t] = make_float4(ma.x * fa + mb.x * fb, ma.y * fa + mb.y * fb, ma.z * fa + mb.z * fb, ma.w * fa + mb.w * fb);
        s_m2[t] = make_float4(qa.x + qb.x + dx * dx * w, qa.y + qb.y + dy * dy * w, qa.z + qb.z + dz * dz * w,
                              qa.w + qb.w + dw * dw * w);
        s_n[t] = nn;
      }
    }
    __syncthreads();
  }
  if (rr == 0) {
    const int P = gridDim.x;
    const float4 a = s_mu[t], b = s_m2[t];
    const float am[4] = {a.x, a.y, a.z, a.w}, bm[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      g.stats[(long long)(c0 + j) * P + blockIdx.x] = am[j];
      g.stats[(long long)(g.N + c0 + j) * P + blockIdx.x] = bm[j];
    }
  }
}

// (mean, invstd) per channel from stats[2][N][P] partials of R rows each
// (jr_conv.hip; single-pass shifted combine in fp64, two stages when P is
// large).
__global__ void __launch_bounds__(256) k_stats_finalize8(const float* __restrict__ part, int P, int R, int M, int N,
                                                         float eps, float* mean, float* invstd, long long p_mb,
                                                         long long st_mb);
__global__ void __launch_bounds__(256) k_stats_finalize(const float* __restrict__ part, const float* __restrict__ cnt,
                                                        int P, int R, int M, int N, int chunk, float eps,
                                                        float* mean, float* invstd, float* out, long long p_mb,
                                                        long long st_mb);

struct TileCfg {
  int bm, bn, wgm, bk, nbuf;
  double eff;  // relative MFMA efficiency guess used to rank padded work
  int nw = 4;  // waves per block (256 or 512 threads)
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
    // one block per CU, wave tiles of 128 x 128 / 128 x 96: 16 / 12 MFMAs per
    // k-step against 4 DMA pieces per wave (0.25-0.33 DMA per MFMA, where the
    // 64 x 64 wave tiles issue 0.5: the per-MFMA issue budget is the bound)
    {256, 256, 2, 32, 3, 1.10},  // 8: wave 128x128, 96 KiB
    {256, 192, 2, 32, 3, 1.08},  // 9: wave 128x96, 84 KiB
    // deeper rings for the short-K-loop 17x17 / 8x8 GEMMs, whose K-tiles
    // carry few MFMAs per wave: NBUF - 2 stages stay in flight under the
    // compute of one (eff just below the same-shape tile above: the untuned
    // planner keeps its choice, autotuning / the pinned tables decide)
    {128, 64, 2, 32, 5, 0.91},   // 10: 60 KiB, 3 stages in flight
    {128, 128, 2, 32, 4, 0.99},  // 11: 64 KiB, 2 in flight
    {128, 96, 4, 32, 5, 0.89},   // 12: 70 KiB
    {128, 64, 2, 64, 3, 0.91},   // 13: 72 KiB, twice the MFMAs per K-tile
    // N = 32 GEMMs (the stem: conv1 / conv2 fwd and wgrad, conv2 / conv3
    // dgrad with N = c_in = 32), which the BN >= 64 tiles pad to twice the
    // MFMA work: four waves stacked along M, wave tile 64 x 32 / 32 x 32
    {256, 32, 4, 32, 3, 0.85},   // 14: 54 KiB
    {128, 32, 4, 32, 4, 0.80},   // 15: 40 KiB
    {256, 32, 4, 64, 3, 0.85},   // 16: 108 KiB
};
constexpr int kNumCfgsBf16 = sizeof(kCfgsBf16) / sizeof(kCfgsBf16[0]);

// JR_F32_X8P tiles: the bf16 kernel with three operand planes (h, m, l) and
// eight MFMAs per k-step, so BK = 16 (one k-step) already gives a wave
// 8 * TM * TN MFMAs per K-tile; LDS = NBUF * 3 * (BM + BN) * BK * 2 B.
static constexpr TileCfg kCfgsX8P[] = {
    {128, 128, 2, 16, 3, 1.00},  // 0: wave 64x64, 72 KiB LDS
    {128, 128, 2, 16, 4, 1.00},  // 1: 96 KiB
    {256, 128, 2, 16, 3, 1.05},  // 2: wave 128x64, 108 KiB
    {128, 64, 2, 16, 3, 0.92},   // 3: wave 64x32, 54 KiB
    {256, 64, 4, 16, 3, 1.00},   // 4: wave 64x64, 81 KiB
    {128, 192, 2, 16, 3, 1.02},  // 5: wave 64x96, 90 KiB
    {128, 96, 4, 16, 3, 0.90},   // 6: wave 32x96, 63 KiB
    {64, 64, 2, 32, 3, 0.75},    // 7: wave 32x32, 72 KiB
    {256, 256, 2, 16, 2, 1.10},  // 8: wave 128x128, 96 KiB
    {256, 192, 2, 16, 3, 1.08},  // 9: wave 128x96, 126 KiB
    {128, 64, 2, 16, 5, 0.91},   // 10: 90 KiB (deeper rings, as kCfgsBf16 10-13)
    {128, 128, 2, 16, 5, 0.99},  // 11: 120 KiB
    {128, 96, 4, 16, 4, 0.89},   // 12: 84 KiB
    {128, 64, 2, 32, 3, 0.91},   // 13: 108 KiB
    {256, 32, 4, 16, 3, 0.85},   // 14: 81 KiB (N = 32, as kCfgsBf16 14-16)
    {128, 32, 4, 16, 4, 0.80},   // 15: 60 KiB
    {256, 32, 4, 32, 2, 0.85},   // 16: 108 KiB
};
constexpr int kNumCfgsX8P = sizeof(kCfgsX8P) / sizeof(kCfgsX8P[0]);

// Wide tiles (round 3): 8 waves (512 threads, two per SIMD) on 256-row
// blocks, one block per CU.  Per K-tile a block moves (BM + BN) * BK operand
// elements through L2 -> LDS-DMA for BM * BN * BK MACs: at 128 x 128 that
// ratio needs ~2x the L2 -> LDS rate a CU sustains (~70 GB/s: the bf16 GEMMs
// ran at 0.1-0.2 of the MFMA peak and x8p at 0.57 MFMA busy), at 256 x 256
// half of it.  Two waves per SIMD hide each other's DMA issue, LDS reads and
// barrier waits.  Selectable config ids FOLLOW every older id (bf16: after
// the halo configs; x8p: after kCfgsX8P), so the committed tile tables keep
// their meaning.
static constexpr TileCfg kCfgsBf16W[] = {
    {256, 256, 2, 32, 3, 1.20, 8},   // 0: wave 128x64, 96 KiB
    {256, 192, 4, 32, 3, 1.16, 8},   // 1: wave 64x96, 84 KiB
    {256, 128, 4, 64, 2, 1.12, 8},   // 2: wave 64x64, 96 KiB
    {128, 256, 2, 64, 2, 1.12, 8},   // 3: wave 64x64, 96 KiB
    {256, 256, 2, 64, 2, 1.20, 8},   // 4: wave 128x64, 128 KiB
    {256, 192, 4, 64, 2, 1.16, 8},   // 5: wave 64x96, 112 KiB
    {256, 96, 8, 64, 2, 1.00, 8},    // 6: wave 32x96, 88 KiB
    {256, 64, 8, 64, 3, 0.95, 8},    // 7: wave 32x64, 120 KiB
};
constexpr int kNumCfgsBf16W = sizeof(kCfgsBf16W) / sizeof(kCfgsBf16W[0]);
static constexpr TileCfg kCfgsX8PW[] = {
    {256, 256, 2, 16, 3, 1.20, 8},   // 0: wave 128x64, 144 KiB
    {256, 192, 4, 16, 3, 1.16, 8},   // 1: wave 64x96, 126 KiB
    {256, 128, 4, 16, 3, 1.12, 8},   // 2: wave 64x64, 108 KiB
    {128, 256, 2, 16, 3, 1.12, 8},   // 3: wave 64x64, 108 KiB
    {256, 96, 8, 16, 4, 1.00, 8},    // 4: wave 32x96, 132 KiB
    {256, 64, 8, 16, 4, 0.95, 8},    // 5: wave 32x64, 120 KiB
    {128, 192, 4, 16, 3, 1.05, 8},   // 6: wave 32x96, 90 KiB
};
constexpr int kNumCfgsX8PW = sizeof(kCfgsX8PW) / sizeof(kCfgsX8PW[0]);

// Halo-tiled bf16 FWD configurations (jr_conv_halo.hip), bf16 tile ids
// kNumCfgsBf16 + i: for stride-1 'same' convs of exactly this kh x kw with
// c_in % 32 == 0 whose halo (output rows a BM tile spans + kh - 1) x (w + kw -
// 1) fits in slots - 1 (the last slot stays zero).  t.bk = kh*kw*32 (one
// K-tile = one 32-channel chunk of every tap), so the planner's ktiles is
// the chunk count.  LDS per stage: slots x 64 B + kh*kw x BN x 64 B.
struct HaloCfg {
  int kh, kw, slots;
  TileCfg t;
};
static constexpr HaloCfg kHaloBf16[] = {
    {1, 7, 224, {128, 64, 2, 7 * 32, 2, 1.0}},   // 0: 17^2 1x7: 9 x 23 = 207 slots; 2 x 42 KiB
    {7, 1, 256, {128, 64, 2, 7 * 32, 2, 1.0}},   // 1: 17^2 7x1: 15 x 17 = 255 slots; 2 x 44 KiB
    {3, 3, 272, {128, 96, 4, 9 * 32, 2, 1.0}},   // 2: 35^2 3x3, N = 96: 7 x 37 = 259 slots; 2 x 71 KiB
    {3, 3, 272, {128, 64, 2, 9 * 32, 2, 1.0}},   // 3: 3x3, N = 64 tiles (8^2: 19 x 10 = 190 slots); 2 x 53 KiB
    {1, 3, 176, {128, 64, 2, 3 * 32, 3, 1.0}},   // 4: 8^2 1x3: 17 x 10 = 170 slots; 3 x 23 KiB
    {3, 1, 160, {128, 64, 2, 3 * 32, 3, 1.0}},   // 5: 8^2 3x1: 19 x 8 = 152 slots; 3 x 22 KiB
    {1, 7, 224, {128, 64, 2, 7 * 32, 3, 1.0}},   // 6: as 0, three stages (126 KiB)
    {7, 1, 256, {128, 64, 2, 7 * 32, 3, 1.0}},   // 7: as 1, three stages (132 KiB)
};
constexpr int kNumHaloBf16 = sizeof(kHaloBf16) / sizeof(kHaloBf16[0]);
void launch_conv_halo(int h, const ConvArgs& a, dim3 grid, hipStream_t s);
// conv2d_1 as a direct VALU convolution (jr_conv_direct.hip): the geometry
// test, its statistics partials (P of R rows) and the launch (stats may be
// nullptr; members > 1: blockIdx.y, byte strides)
bool conv1_direct_ok(const jr_conv_desc* d, int dtype);
int conv1_direct_partials(const jr_conv_desc* d, int* P, int* R);
void launch_conv1_direct(const jr_conv_desc* d, int dtype, const void* x, const void* w, void* y, float* stats,
                         int members, long long x_mb, long long w_mb, long long y_mb, long long s_mb, hipStream_t s);

// bf16-operand GEMM launch (jr_conv_bf16.hip): tile index into kCfgsBf16
// (np = 1, JR_BF16) or kCfgsX8P (np = 3, JR_F32_X8P).
// am = operand address mode (k_conv_bf16's AM).
void launch_conv_bf16(int op, int tile, int am, const ConvArgs& a, dim3 grid, hipStream_t s, int np = 1);
// the same kernel on a wide tile: index into kCfgsBf16W (np = 1) / kCfgsX8PW (np = 3)
void launch_conv_bf16_wide(int op, int tile, int am, const ConvArgs& a, dim3 grid, hipStream_t s, int np = 1);
// the stream-K grid of a JR_BF16 tile (standard, or wide with wide = true)
void launch_conv_bf16_sk(int op, int tile, bool wide, int am, const ConvArgs& a, dim3 grid, hipStream_t s);

}  // namespace jr
