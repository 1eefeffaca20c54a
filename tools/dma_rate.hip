// Diagnostic: per-CU operand-delivery rate from L2-resident data on gfx950,
// as a function of the bytes each CU keeps in flight -- the model behind the
// conv GEMM tile / ring choices.  Not part of libjr.
//
//   hipcc -O3 --offload-arch=gfx950 tools/dma_rate.hip -o tools/dma_rate && tools/dma_rate
//
// Every wave streams 1 KiB wave-instructions (64 lanes x 16 B) from a 1 MiB
// region (L2-resident after the first pass on every XCD), keeping D of them
// in flight with a counted vmcnt:
//   mode 0: LDS-DMA (global_load_lds_dwordx4) into a per-wave LDS ring
//   mode 1: global_load_dwordx4 into registers (xor-folded, stored once)
//   mode 2: LDS-DMA with an im2col-like gather: 4 lanes per 64 B row, rows
//           taken from pixels 80 channels apart (one conv5 K-tile row set)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__device__ __forceinline__ void wait_vm(int n) {
#define C(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
  switch (n) {
    C(0) C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12) C(13) C(14) C(15)
    C(16) C(17) C(18) C(19) C(20) C(21) C(22) C(23) C(24) C(25) C(26) C(27) C(28) C(29) C(30)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
#undef C
}

constexpr int kRegion = 1 << 20;   // bytes

template <int MODE, int W, int D, int RB = 64, int RS = 160>
__global__ void __launch_bounds__(W * 64) k_stream(const char* __restrict__ src, int iters, unsigned* out) {
  __shared__ __attribute__((aligned(1024))) char ring[W * D * 1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  char* myring = ring + wave * D * 1024;
  const unsigned gw = blockIdx.x * W + wave;
  unsigned off = (gw * 7919u * 1024u) % kRegion;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int i = 0; i < iters; ++i) {
    unsigned lo;
    if (MODE == 2 || MODE == 3) {
      // 1024 / RB rows of RB bytes per instruction, rows RS bytes apart
      // (RB = 64, RS = 160: a BK = 32 bf16 K-tile row set of conv5, c_in 80)
      lo = (lane / (RB / 16)) * RS + (lane % (RB / 16)) * 16;
    } else {
      lo = lane * 16;
    }
    const char* p = src + ((off + lo) & (kRegion - 1));
    if (MODE == 3 && (wave & 1)) {   // mixed: odd waves register loads, even waves LDS-DMA
      uint4 v[D];
#pragma unroll
      for (int d = 0; d < D; ++d) v[d] = *reinterpret_cast<const uint4*>(src + ((off + lo + d * 1024u) & (kRegion - 1)));
#pragma unroll
      for (int d = 0; d < D; ++d) { acc.x ^= v[d].x; acc.y ^= v[d].y; acc.z ^= v[d].z; acc.w ^= v[d].w; }
      i += D - 1;
      off = (off + (D - 1) * 1024u) & (kRegion - 1);
    } else if (MODE == 1) {   // D independent loads in flight, then fold
      uint4 v[D];
#pragma unroll
      for (int d = 0; d < D; ++d) v[d] = *reinterpret_cast<const uint4*>(src + ((off + lo + d * 1024u) & (kRegion - 1)));
#pragma unroll
      for (int d = 0; d < D; ++d) { acc.x ^= v[d].x; acc.y ^= v[d].y; acc.z ^= v[d].z; acc.w ^= v[d].w; }
      i += D - 1;
      off = (off + (D - 1) * 1024u) & (kRegion - 1);
    } else {
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)p,
                                       (__attribute__((address_space(3))) void*)(myring + (i % D) * 1024), 16, 0, 0);
      wait_vm(D - 1);
    }
    off = (off + (MODE >= 2 ? (unsigned)(1024 / RB * RS) : 1024u)) & (kRegion - 1);
  }
  wait_vm(0);
  if (MODE == 1 || (MODE == 3 && (wave & 1))) {
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;   // keeps the loads live
  } else if (lane == 0) {
    out[gw & 1023] = *reinterpret_cast<const unsigned*>(myring);
  }
}

template <int MODE, int W, int D, int RB = 64, int RS = 160>
static void run(const char* src, unsigned* out, int bpc, int cus) {
  const int iters = 4096;
  const int grid = cus * bpc;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL((k_stream<MODE, W, D, RB, RS>), dim3(grid), dim3(W * 64), 0, 0, src, iters, out);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_stream<MODE, W, D, RB, RS>), dim3(grid), dim3(W * 64), 0, 0, src, iters, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  const double bytes = (double)grid * W * iters * 1024.0;
  const double gbs_cu = bytes / (best * 1e-3) / cus / 1e9;
  const int mode_loads = D;
  if (MODE >= 2) printf("[rows of %3d B, %4d B apart] ", RB, RS);
  printf("mode %d  waves/block %d  blocks/CU %d  in-flight/wave %2d  KiB in flight/CU %4d  %7.1f us  %6.1f GB/s per CU  %6.2f TB/s chip\n",
         MODE, W, bpc, mode_loads, W * D * bpc, best * 1e3, gbs_cu, gbs_cu * cus / 1e3);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("%s, %d CUs\n", prop.gcnArchName, cus);
  char* src;
  unsigned* out;
  CHECK(hipMalloc(&src, kRegion));
  CHECK(hipMalloc(&out, 4096 * sizeof(unsigned)));
  CHECK(hipMemset(src, 1, kRegion));
  // LDS-DMA, contiguous 1 KiB pieces
  run<0, 4, 2>(src, out, 1, cus);
  run<0, 4, 4>(src, out, 1, cus);
  run<0, 4, 8>(src, out, 1, cus);
  run<0, 4, 16>(src, out, 1, cus);
  run<0, 4, 24>(src, out, 1, cus);
  run<0, 4, 8>(src, out, 2, cus);
  run<0, 4, 16>(src, out, 2, cus);
  run<0, 8, 2>(src, out, 1, cus);
  run<0, 8, 4>(src, out, 1, cus);
  run<0, 8, 8>(src, out, 1, cus);
  run<0, 8, 16>(src, out, 1, cus);
  run<0, 8, 8>(src, out, 2, cus);
  // LDS-DMA, im2col-like 64 B row gather
  run<2, 4, 4>(src, out, 1, cus);
  run<2, 4, 8>(src, out, 1, cus);
  run<2, 4, 16>(src, out, 1, cus);
  run<2, 8, 8>(src, out, 1, cus);
  run<2, 8, 16>(src, out, 1, cus);
  // row geometry: bytes per row x row stride (aligned or not)
  run<2, 8, 8, 64, 128>(src, out, 1, cus);
  run<2, 8, 8, 64, 192>(src, out, 1, cus);
  run<2, 8, 8, 64, 256>(src, out, 1, cus);
  run<2, 8, 8, 128, 128>(src, out, 1, cus);
  run<2, 8, 8, 128, 160>(src, out, 1, cus);
  run<2, 8, 8, 128, 256>(src, out, 1, cus);
  run<2, 8, 8, 128, 384>(src, out, 1, cus);
  run<2, 8, 8, 256, 256>(src, out, 1, cus);
  run<2, 8, 8, 256, 512>(src, out, 1, cus);
  run<2, 8, 8, 256, 320>(src, out, 1, cus);
  run<2, 4, 8, 128, 256>(src, out, 2, cus);
  run<2, 4, 8, 64, 128>(src, out, 2, cus);
  // mixed: half the waves LDS-DMA, half register loads (do the two paths share the TA?)
  run<3, 8, 8, 128, 128>(src, out, 1, cus);
  run<3, 8, 8, 128, 256>(src, out, 1, cus);
  run<3, 8, 8, 64, 128>(src, out, 1, cus);
  run<3, 8, 16, 128, 256>(src, out, 1, cus);
  run<3, 4, 8, 128, 256>(src, out, 2, cus);
  // register loads with the row geometry (mode 1 is contiguous)
  // register loads
  run<1, 4, 4>(src, out, 1, cus);
  run<1, 4, 8>(src, out, 1, cus);
  run<1, 4, 16>(src, out, 1, cus);
  run<1, 8, 8>(src, out, 1, cus);
  run<1, 8, 16>(src, out, 1, cus);
  run<1, 4, 8>(src, out, 4, cus);
  CHECK(hipFree(src));
  CHECK(hipFree(out));
  return 0;
}
