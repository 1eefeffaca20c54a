// Cost of cross-stream synchronisation on MI355X (run under rocprofv3
// --kernel-trace; tools/sync_probe_gaps.py prints the gap per segment).
// Segments of 40 `scale` kernels each, separated by `tag` kernels:
//   a plain; b hipEventRecord after each; c the event attached to the kernel
//   (hipExtLaunchKernelGGL stopEvent); d ping-pong record + wait; e ping-pong
//   attached + wait; f as e with DisableSystemFence events; g as b with
//   DisableSystemFence events.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

__global__ void scale(float* x, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] *= 1.0f;
}
__global__ void tag(float* x) { if (threadIdx.x == 0) x[0] += 0.f; }

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(r_)); return 1; } } while (0)

int main() {
  const int n = 8 << 20, R = 40;
  float *x, *y;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t ev[64], fe[64];
  for (int i = 0; i < 64; ++i) {
    CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&fe[i], hipEventDisableTiming | hipEventDisableSystemFence));
  }
  const dim3 g(n / 256), blk(256);
  auto T = [&]() { hipLaunchKernelGGL(tag, dim3(1), dim3(64), 0, a, x); };
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipDeviceSynchronize());
    T();
    for (int i = 0; i < R; ++i) hipLaunchKernelGGL(scale, g, blk, 0, a, x, n);
    T();
    for (int i = 0; i < R; ++i) { hipLaunchKernelGGL(scale, g, blk, 0, a, x, n); CK(hipEventRecord(ev[i % 64], a)); }
    T();
    for (int i = 0; i < R; ++i) hipExtLaunchKernelGGL(scale, g, blk, 0, a, nullptr, ev[i % 64], 0, x, n);
    T();
    CK(hipDeviceSynchronize());
    for (int i = 0; i < R; ++i) {
      hipStream_t s = i % 2 ? b : a;
      if (i) CK(hipStreamWaitEvent(s, ev[(i - 1) % 64], 0));
      hipLaunchKernelGGL(scale, g, blk, 0, s, i % 2 ? y : x, n);
      CK(hipEventRecord(ev[i % 64], s));
    }
    CK(hipDeviceSynchronize());
    T();
    CK(hipDeviceSynchronize());
    for (int i = 0; i < R; ++i) {
      hipStream_t s = i % 2 ? b : a;
      if (i) CK(hipStreamWaitEvent(s, ev[(i - 1) % 64], 0));
      hipExtLaunchKernelGGL(scale, g, blk, 0, s, nullptr, ev[i % 64], 0, i % 2 ? y : x, n);
    }
    CK(hipDeviceSynchronize());
    T();
    CK(hipDeviceSynchronize());
    for (int i = 0; i < R; ++i) {
      hipStream_t s = i % 2 ? b : a;
      if (i) CK(hipStreamWaitEvent(s, fe[(i - 1) % 64], 0));
      hipExtLaunchKernelGGL(scale, g, blk, 0, s, nullptr, fe[i % 64], 0, i % 2 ? y : x, n);
    }
    CK(hipDeviceSynchronize());
    T();
    for (int i = 0; i < R; ++i) { hipLaunchKernelGGL(scale, g, blk, 0, a, x, n); CK(hipEventRecord(fe[i % 64], a)); }
    T();
    CK(hipDeviceSynchronize());
  }
  printf("done\n");
  return 0;
}
