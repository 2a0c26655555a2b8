// Kernel timing inside HIP graphs (bench.py's roofline): timing events whose records become
// graph nodes when the stream is being captured (hipEventRecordExternal), so the duration of a
// single kernel can be read after each replay of a captured step. Host-side only; no kernels.
#include "common.h"

// 0: hipEventRecordWithFlags(External) first; 1: it was refused once, go straight to the node
static int g_record_mode = 0;

thread_local CapmiArmedEvents g_capmi_armed = {nullptr, nullptr};

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
