// jr_api.cpp — library-level C-ABI: init, launch-error mapping, HIP graph
// capture (the error convention itself is host-only code: jr_error.cpp).
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "jr_common.h"

namespace jr {

namespace {
struct Scratch {
  unsigned* p = nullptr;
  size_t words = 0;
};
std::mutex g_scratch_mu;
std::map<std::tuple<int, hipStream_t, int>, Scratch> g_scratch;
std::vector<unsigned*> g_scratch_kept;   // outgrown / captured regions: launches in flight may still use them

unsigned* scratch_alloc(hipStream_t s, size_t words) {
  void* p = nullptr;
  if (hipMalloc(&p, words * sizeof(unsigned)) != hipSuccess) return nullptr;
  if (hipMemsetAsync(p, 0, words * sizeof(unsigned), s) != hipSuccess) return nullptr;
  return static_cast<unsigned*>(p);
}
}  // namespace

unsigned* stream_scratch(hipStream_t s, int kind, size_t words) {
  words = std::max<size_t>(words, 1);
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
    // (the zeroing memset becomes a node of the graph ahead of the kernel;
    // the kernel leaves the words zero, so every replay starts from zero;
    // hipMalloc is not a stream operation: relaxed mode lets it through)
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    void* raw = nullptr;
    const bool ok = hipMalloc(&raw, words * sizeof(unsigned)) == hipSuccess;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    unsigned* p = ok && hipMemsetAsync(raw, 0, words * sizeof(unsigned), s) == hipSuccess
                      ? static_cast<unsigned*>(raw) : nullptr;
    if (p) g_scratch_kept.push_back(p);
    return p;
  }
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  Scratch& e = g_scratch[std::make_tuple(dev, s, kind)];
  if (e.words < words) {
    const size_t n = std::max<size_t>(words, std::max<size_t>(2 * e.words, 16384));
    unsigned* p = scratch_alloc(s, n);
    if (!p) return nullptr;
    if (e.p) g_scratch_kept.push_back(e.p);
    e.p = p;
    e.words = n;
  }
  return e.p;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(JR_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return JR_OK;
}

}  // namespace jr

using namespace jr;

JR_API const char* jr_version(void) { return "libjr 0.2 gfx950 (implicit-GEMM conv: fp32 x8-split / fp32 / bf16 MFMA)"; }

JR_API int jr_init(int device) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) return fail(JR_ERR_HIP, std::string("jr_init: ") + hipGetErrorString(e));
  if (device < 0 || device >= n) return fail(JR_ERR_INVALID, "jr_init: device ordinal out of range");
  e = hipSetDevice(device);
  if (e != hipSuccess) return fail(JR_ERR_HIP, std::string("jr_init: ") + hipGetErrorString(e));
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, device);
  if (e != hipSuccess) return fail(JR_ERR_HIP, std::string("jr_init: ") + hipGetErrorString(e));
  if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0)
    return fail(JR_ERR_UNSUPPORTED, std::string("jr_init: libjr is built for gfx950, device is ") + prop.gcnArchName);
  return JR_OK;
}

JR_API int jr_graph_begin(void* stream) {
  const hipError_t e = hipStreamBeginCapture(as_stream(stream), hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) return fail(JR_ERR_HIP, std::string("graph_begin: ") + hipGetErrorString(e));
  return JR_OK;
}

JR_API int jr_graph_end(void* stream, void** graph_exec) {
  if (!graph_exec) return fail(JR_ERR_INVALID, "graph_end: null output");
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(as_stream(stream), &g);
  if (e != hipSuccess) return fail(JR_ERR_HIP, std::string("graph_end: ") + hipGetErrorString(e));
  hipGraphExec_t ex = nullptr;
  e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) return fail(JR_ERR_HIP, std::string("graph_instantiate: ") + hipGetErrorString(e));
  *graph_exec = reinterpret_cast<void*>(ex);
  return JR_OK;
}

JR_API int jr_graph_launch(void* graph_exec, void* stream) {
  if (!graph_exec) return fail(JR_ERR_INVALID, "graph_launch: null graph");
  const hipError_t e = hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(graph_exec), as_stream(stream));
  if (e != hipSuccess) return fail(JR_ERR_HIP, std::string("graph_launch: ") + hipGetErrorString(e));
  return JR_OK;
}

JR_API int jr_graph_destroy(void* graph_exec) {
  if (!graph_exec) return JR_OK;
  const hipError_t e = hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(graph_exec));
  if (e != hipSuccess) return fail(JR_ERR_HIP, std::string("graph_destroy: ") + hipGetErrorString(e));
  return JR_OK;
}
