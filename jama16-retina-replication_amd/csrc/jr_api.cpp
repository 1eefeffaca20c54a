// jr_api.cpp — library-level C-ABI: init, launch-error mapping, HIP graph
// capture (the error convention itself is host-only code: jr_error.cpp).
#include <hip/hip_runtime.h>

#include <string>

#include "jr_common.h"

namespace jr {

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
