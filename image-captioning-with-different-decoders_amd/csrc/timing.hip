// Kernel timing inside HIP graphs (bench.py's roofline): timing events whose records become
// graph nodes when the stream is being captured (hipEventRecordExternal), so the duration of a
// single kernel can be read after each replay of a captured step. Host-side only; no kernels.
#include <cxxabi.h>
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>

#include "common.h"

// 0: hipEventRecordWithFlags(External) first; 1: it was refused once, go straight to the node
static int g_record_mode = 0;

thread_local CapmiArmedEvents g_capmi_armed = {nullptr, nullptr};
thread_local const void* g_capmi_last_kernel = nullptr;

// the demangled instantiation of the last GEMM kernel this host thread launched through CAPMI_KLAUNCH, as
// rocprofv3 prints it without the return type and parameter list ("gemm_bf16_kernel<128, 64, 2, false, 2>")
extern "C" int capmi_last_launch_name(char* out, int n) {
  CAPMI_REQUIRE(out != nullptr && n > 0, CAPMI_EINVAL);
  out[0] = 0;
  CAPMI_REQUIRE(g_capmi_last_kernel != nullptr, CAPMI_EINVAL);
  // the kernel's host stub is a weak, default-visibility symbol named as the kernel: dladdr names it without the
  // runtime; the HIP runtime's own registry is the fallback
  const char* raw = nullptr;
  Dl_info info;
  if (dladdr(g_capmi_last_kernel, &info) != 0 && info.dli_sname != nullptr && info.dli_saddr == g_capmi_last_kernel)
    raw = info.dli_sname;
  hipFunction_t fn = nullptr;
  if ((raw == nullptr || raw[0] == 0) && hipGetFuncBySymbol(&fn, g_capmi_last_kernel) == hipSuccess && fn != nullptr)
    raw = hipKernelNameRef(fn);
  if (raw == nullptr || raw[0] == 0) raw = hipKernelNameRefByPtr(g_capmi_last_kernel, nullptr);
  CAPMI_REQUIRE(raw != nullptr && raw[0] != 0, CAPMI_EINVAL);
  int st = -1;
  char* dem = (raw[0] == '_' && raw[1] == 'Z') ? abi::__cxa_demangle(raw, nullptr, nullptr, &st) : nullptr;
  std::string name = (dem && st == 0) ? std::string(dem) : std::string(raw);
  free(dem);
  if (name.compare(0, 5, "void ") == 0) name = name.substr(5);
  static const std::string anon = "(anonymous namespace)::";
  if (name.compare(0, anon.size(), anon) == 0) name = name.substr(anon.size());
  // drop the parameter list: the '(' that closes the template argument list's nesting level 0
  int depth = 0;
  for (size_t i = 0; i < name.size(); ++i) {
    if (name[i] == '<') ++depth;
    else if (name[i] == '>') --depth;
    else if (name[i] == '(' && depth == 0) {
      name.resize(i);
      break;
    }
  }
  snprintf(out, (size_t)n, "%s", name.c_str());
  return 0;
}

// the next GEMM launch of this host thread records its dispatch start / end into (start, stop)
// (CAPMI_KLAUNCH, common.h); eager launches only (a stream under capture refuses it)
extern "C" int capmi_timing_arm(void* start, void* stop) {
  CAPMI_REQUIRE(start != nullptr && stop != nullptr, CAPMI_EINVAL);
  g_capmi_armed = CapmiArmedEvents{reinterpret_cast<hipEvent_t>(start), reinterpret_cast<hipEvent_t>(stop)};
  return 0;
}

// drops an armed pair no launch consumed (a launch refused by its planner); returns 1 if one was left
extern "C" int capmi_timing_disarm(void) {
  const int left = g_capmi_armed.start != nullptr ? 1 : 0;
  g_capmi_armed = CapmiArmedEvents{nullptr, nullptr};
  return left;
}

extern "C" int capmi_timing_event_create(void** event) {
  CAPMI_REQUIRE(event != nullptr, CAPMI_EINVAL);
  hipEvent_t e = nullptr;
  const hipError_t rc = hipEventCreate(&e);  // default flags: timing enabled
  if (rc != hipSuccess) return (int)rc;
  *event = e;
  return 0;
}

extern "C" int capmi_timing_event_destroy(void* event) {
  return event == nullptr ? 0 : (int)hipEventDestroy(reinterpret_cast<hipEvent_t>(event));
}

extern "C" int capmi_timing_event_record(void* event, void* stream) {
  CAPMI_REQUIRE(event != nullptr, CAPMI_EINVAL);
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  hipError_t rc = hipStreamIsCapturing(as_stream(stream), &st);
  if (rc != hipSuccess) return (int)rc;
  if (st != hipStreamCaptureStatusActive) return (int)hipEventRecord(reinterpret_cast<hipEvent_t>(event), as_stream(stream));
  if (g_record_mode == 0) {
    rc = hipEventRecordWithFlags(reinterpret_cast<hipEvent_t>(event), as_stream(stream), hipEventRecordExternal);
    if (rc == hipSuccess) return 0;
    (void)hipGetLastError();
  }
  // explicit node: append an event-record node after the capture's current dependencies and
  // make it the stream's only dependency
  hipGraph_t graph = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t ndeps = 0;
  unsigned long long id = 0;
  rc = hipStreamGetCaptureInfo_v2(as_stream(stream), &st, &id, &graph, &deps, &ndeps);
  if (rc != hipSuccess) return (int)rc;
  hipGraphNode_t node = nullptr;
  rc = hipGraphAddEventRecordNode(&node, graph, deps, ndeps, reinterpret_cast<hipEvent_t>(event));
  if (rc != hipSuccess) return (int)rc;
  rc = hipStreamUpdateCaptureDependencies(as_stream(stream), &node, 1, hipStreamSetCaptureDependencies);
  if (rc == hipSuccess) g_record_mode = 1;
  return (int)rc;
}

extern "C" int capmi_timing_elapsed_ms(void* start, void* end, float* ms) {
  CAPMI_REQUIRE(start != nullptr && end != nullptr && ms != nullptr, CAPMI_EINVAL);
  return (int)hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(start), reinterpret_cast<hipEvent_t>(end));
}
