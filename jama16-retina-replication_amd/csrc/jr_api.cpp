// jr_api.cpp — library-level C-ABI: init, launch-error mapping, the device
// error word, HIP graph capture (the error convention itself is host-only
// code: jr_error.cpp).
#include <hip/hip_runtime.h>

#include <atomic>
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
  size_t used = 0;      // the most words any launch on the stream has asked for
};
std::mutex g_scratch_mu;
std::map<std::tuple<int, hipStream_t, int>, Scratch> g_scratch;
std::vector<unsigned*> g_scratch_kept;   // outgrown regions: launches in flight may still use them
// regions handed to a capturing stream, per capture sequence id until
// jr_graph_end moves them to the graph exec that references them (freed by
// jr_graph_destroy; ADVICE r04: they used to be kept forever)
std::map<unsigned long long, std::vector<void*>> g_capture_regions;
std::map<hipGraphExec_t, std::vector<void*>> g_graph_regions;

constexpr int kMaxDevices = 64;
unsigned* g_err_word[kMaxDevices] = {};

unsigned* scratch_alloc(hipStream_t s, size_t words) {
  void* p = nullptr;
  if (hipMalloc(&p, words * sizeof(unsigned)) != hipSuccess) return nullptr;
  if (hipMemsetAsync(p, 0, words * sizeof(unsigned), s) != hipSuccess) return nullptr;
  return static_cast<unsigned*>(p);
}

bool capturing(hipStream_t s, unsigned long long* id) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long cid = 0;
  if (hipStreamGetCaptureInfo(s, &cs, &cid) != hipSuccess) return false;
  if (id) *id = cid;
  return cs != hipStreamCaptureStatusNone;
}

// allocate + zero the current device's error word (not under capture)
int err_word_init(int dev) {
  if (dev < 0 || dev >= kMaxDevices) return fail(JR_ERR_UNSUPPORTED, "libjr: device ordinal above 63");
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  if (g_err_word[dev]) return JR_OK;
  void* p = nullptr;
  if (hipMalloc(&p, sizeof(unsigned)) != hipSuccess || hipMemset(p, 0, sizeof(unsigned)) != hipSuccess)
    return fail(JR_ERR_HIP, "libjr: device error word could not be allocated");
  g_err_word[dev] = static_cast<unsigned*>(p);
  return JR_OK;
}
}  // namespace

unsigned* stream_scratch(hipStream_t s, int kind, size_t words) {
  words = std::max<size_t>(words, 1);
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  unsigned long long cid = 0;
  if (capturing(s, &cid)) {
    // (the zeroing memset becomes a node of the graph ahead of the kernel;
    // the kernel leaves the words zero, so every replay starts from zero;
    // hipMalloc is not a stream operation: relaxed mode lets it through)
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    void* raw = nullptr;
    const bool ok = hipMalloc(&raw, words * sizeof(unsigned)) == hipSuccess;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    if (!ok) return nullptr;
    g_capture_regions[cid].push_back(raw);
    return hipMemsetAsync(raw, 0, words * sizeof(unsigned), s) == hipSuccess ? static_cast<unsigned*>(raw)
                                                                              : nullptr;
  }
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  Scratch& e = g_scratch[std::make_tuple(dev, s, kind)];
  e.used = std::max(e.used, words);
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

unsigned* device_error_word(hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return nullptr;
  {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    if (g_err_word[dev]) return g_err_word[dev];
  }
  // the launch's own stream capturing: no synchronous allocation now (it would
  // break a global-mode capture); the caller reports "call jr_init first"
  if (capturing(s, nullptr)) return nullptr;
  return err_word_init(dev) == JR_OK ? g_err_word[dev] : nullptr;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(JR_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return JR_OK;
}

}  // namespace jr

using namespace jr;

JR_API const char* jr_version(void) { return "libjr 0.3 gfx950 (implicit-GEMM conv: fp32 x8-split / fp32 / bf16 MFMA)"; }

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
  return err_word_init(device);
}

JR_API int jr_device_check(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices)
    return fail(JR_ERR_HIP, "jr_device_check: no current device");
  unsigned* w = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    w = g_err_word[dev];
  }
  if (!w) return JR_OK;                 // nothing has run on this device yet
  unsigned h = 0;
  hipError_t e = hipMemcpy(&h, w, sizeof(unsigned), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return fail(JR_ERR_HIP, std::string("jr_device_check: ") + hipGetErrorString(e));
  // every hand-off word of an idle stream must be back at zero: a launch
  // whose counts completed leaves its words zero, so a word found non-zero
  // there is a stale count -- below its piece count it made a tile complete
  // early (summing unpublished slots) without tripping the in-kernel check
  // (ADVICE r05); streams with work in flight are checked at a later call
  size_t stale = 0;
  {
    std::vector<std::pair<hipStream_t, Scratch>> idle;
    {
      std::lock_guard<std::mutex> lk(g_scratch_mu);
      for (auto& kv : g_scratch)
        if (std::get<0>(kv.first) == dev && std::get<2>(kv.first) == 0 && kv.second.p && kv.second.used)
          idle.emplace_back(std::get<1>(kv.first), kv.second);
    }
    std::vector<unsigned> buf;
    for (auto& [st, sc] : idle) {
      if (hipStreamQuery(st) != hipSuccess) continue;       // busy (or not a live stream): not now
      buf.resize(sc.used);
      e = hipMemcpy(buf.data(), sc.p, sc.used * sizeof(unsigned), hipMemcpyDeviceToHost);
      if (e != hipSuccess) return fail(JR_ERR_HIP, std::string("jr_device_check: ") + hipGetErrorString(e));
      for (unsigned v : buf) stale += v != 0;
    }
  }
  if (h == 0 && stale == 0) return JR_OK;
  // repair: every launch has finished, then the hand-off words of every
  // stream of this device and the error word go back to 0
  e = hipDeviceSynchronize();
  if (e != hipSuccess) return fail(JR_ERR_HIP, std::string("jr_device_check: ") + hipGetErrorString(e));
  {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    for (auto& kv : g_scratch)
      if (std::get<0>(kv.first) == dev && std::get<2>(kv.first) == 0 && kv.second.p)
        (void)hipMemset(kv.second.p, 0, kv.second.words * sizeof(unsigned));
  }
  (void)hipMemset(w, 0, sizeof(unsigned));
  (void)hipDeviceSynchronize();
  return fail(JR_ERR_DEVICE, "device check: " + std::to_string(h) +
                                 " failure(s) counted by kernels (a stream-K hand-off count past its tile's piece "
                                 "count, or a JR_F32_X6H magnitude bound exceeded: jr_absmax_prep) and " +
                                 std::to_string(stale) +
                                 " stream-K hand-off word(s) of idle streams not left zero; the outputs of the "
                                 "launches since the last jr_device_check are invalid (hand-off words reset)");
}

JR_API int jr_debug_poison_sk_counts(void* stream, uint32_t value) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(JR_ERR_HIP, "debug_poison_sk_counts: no current device");
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  auto it = g_scratch.find(std::make_tuple(dev, as_stream(stream), 0));
  if (it == g_scratch.end() || !it->second.p) return fail(JR_ERR_INVALID, "debug_poison_sk_counts: no hand-off words on this stream yet");
  const hipError_t e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(it->second.p), (int)value, it->second.words,
                                         as_stream(stream));
  return e == hipSuccess ? JR_OK : fail(JR_ERR_HIP, std::string("debug_poison_sk_counts: ") + hipGetErrorString(e));
}

JR_API int jr_graph_begin(void* stream) {
  const hipError_t e = hipStreamBeginCapture(as_stream(stream), hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) return fail(JR_ERR_HIP, std::string("graph_begin: ") + hipGetErrorString(e));
  return JR_OK;
}

JR_API int jr_graph_end(void* stream, void** graph_exec) {
  if (!graph_exec) return fail(JR_ERR_INVALID, "graph_end: null output");
  unsigned long long cid = 0;
  const bool cap = capturing(as_stream(stream), &cid);
  std::vector<void*> regions;
  auto take_regions = [&] {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    auto it = g_capture_regions.find(cid);
    if (cap && it != g_capture_regions.end()) {
      regions.swap(it->second);
      g_capture_regions.erase(it);
    }
  };
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(as_stream(stream), &g);
  take_regions();
  if (e != hipSuccess) {
    for (void* p : regions) (void)hipFree(p);
    return fail(JR_ERR_HIP, std::string("graph_end: ") + hipGetErrorString(e));
  }
  hipGraphExec_t ex = nullptr;
  e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) {
    for (void* p : regions) (void)hipFree(p);
    return fail(JR_ERR_HIP, std::string("graph_instantiate: ") + hipGetErrorString(e));
  }
  if (!regions.empty()) {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    g_graph_regions[ex] = std::move(regions);
  }
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
  const hipGraphExec_t ex = reinterpret_cast<hipGraphExec_t>(graph_exec);
  const hipError_t e = hipGraphExecDestroy(ex);
  std::vector<void*> regions;
  {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    auto it = g_graph_regions.find(ex);
    if (it != g_graph_regions.end()) {
      regions.swap(it->second);
      g_graph_regions.erase(it);
    }
  }
  if (!regions.empty()) {
    // replays of the destroyed exec may still be in flight: hipFree waits for
    // the device before releasing
    for (void* p : regions) (void)hipFree(p);
  }
  if (e != hipSuccess) return fail(JR_ERR_HIP, std::string("graph_destroy: ") + hipGetErrorString(e));
  return JR_OK;
}

JR_API int jr_graph_regions(void* graph_exec) {
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  auto it = g_graph_regions.find(reinterpret_cast<hipGraphExec_t>(graph_exec));
  return it == g_graph_regions.end() ? 0 : (int)it->second.size();
}

JR_API int jr_event_create(void** event) {
  if (!event) return fail(JR_ERR_INVALID, "event_create: null handle pointer");
  hipEvent_t e = nullptr;
  const hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence);
  if (r != hipSuccess) return fail(JR_ERR_HIP, std::string("event_create: ") + hipGetErrorString(r));
  *event = e;
  return JR_OK;
}

JR_API int jr_event_record(void* event, void* stream) {
  const hipError_t r = hipEventRecord(reinterpret_cast<hipEvent_t>(event), as_stream(stream));
  return r == hipSuccess ? JR_OK : fail(JR_ERR_HIP, std::string("event_record: ") + hipGetErrorString(r));
}

JR_API int jr_stream_wait_event(void* stream, void* event) {
  const hipError_t r = hipStreamWaitEvent(as_stream(stream), reinterpret_cast<hipEvent_t>(event), 0);
  return r == hipSuccess ? JR_OK : fail(JR_ERR_HIP, std::string("stream_wait_event: ") + hipGetErrorString(r));
}

JR_API int jr_event_destroy(void* event) {
  const hipError_t r = hipEventDestroy(reinterpret_cast<hipEvent_t>(event));
  return r == hipSuccess ? JR_OK : fail(JR_ERR_HIP, std::string("event_destroy: ") + hipGetErrorString(r));
}
