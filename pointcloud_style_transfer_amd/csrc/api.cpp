// Library-level entry points: version and thread-local last error.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace pcst {
static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}
}  // namespace pcst

extern "C" const char* pcst_version(void) { return "pcst 0.1.0 gfx950"; }
extern "C" const char* pcst_last_error(void) { return pcst::g_last_error; }

// Stream-ordering events with device-scope fences only (hipEventDisableSystemFence): the
// sampling loop's cross-stream dependencies (kNN build on a side stream) and the bench's kernel
// timing need no host visibility of device memory, and the default system-scope release/acquire
// (an L2 writeback + invalidate at every record and wait) costs a ~10 us bubble per dependency.
extern "C" int pcst_event_create(int timing, void** event) {
  PCST_CHECK_ARG(event != nullptr, "event_create: null pointer");
  hipEvent_t e = nullptr;
  const unsigned flags = hipEventDisableSystemFence | (timing ? 0u : (unsigned)hipEventDisableTiming);
  PCST_HIP(hipEventCreateWithFlags(&e, flags), "event_create");
  *event = e;
  return PCST_OK;
}

extern "C" int pcst_event_destroy(void* event) {
  if (event) PCST_HIP(hipEventDestroy(static_cast<hipEvent_t>(event)), "event_destroy");
  return PCST_OK;
}

extern "C" int pcst_event_record(void* event, void* stream) {
  PCST_CHECK_ARG(event != nullptr, "event_record: null event");
  PCST_HIP(hipEventRecord(static_cast<hipEvent_t>(event), pcst::as_stream(stream)), "event_record");
  return PCST_OK;
}

extern "C" int pcst_stream_wait_event(void* stream, void* event) {
  PCST_CHECK_ARG(event != nullptr, "stream_wait_event: null event");
  PCST_HIP(hipStreamWaitEvent(pcst::as_stream(stream), static_cast<hipEvent_t>(event), 0),
           "stream_wait_event");
  return PCST_OK;
}

// milliseconds between two recorded timing events (synchronises with the second)
extern "C" int pcst_event_elapsed_ms(void* start, void* end, float* ms) {
  PCST_CHECK_ARG(start && end && ms, "event_elapsed_ms: null pointer");
  PCST_HIP(hipEventSynchronize(static_cast<hipEvent_t>(end)), "event_elapsed_ms: sync");
  PCST_HIP(hipEventElapsedTime(ms, static_cast<hipEvent_t>(start), static_cast<hipEvent_t>(end)),
           "event_elapsed_ms");
  return PCST_OK;
}

// Streams owned by the caller (one pair per sampling loop and host thread, so two loops on one
// device never share a queue: their cross-stream flag waits could otherwise interleave on it and
// wait on each other).  priority < 0 is the device's greatest priority, else its default.
extern "C" int pcst_stream_create(int priority, void** stream) {
  PCST_CHECK_ARG(stream != nullptr, "stream_create: null pointer");
  int least = 0, greatest = 0;
  PCST_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest), "stream_create: priority range");
  hipStream_t s = nullptr;
  PCST_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority < 0 ? greatest : least),
           "stream_create");
  *stream = s;
  return PCST_OK;
}

extern "C" int pcst_stream_destroy(void* stream) {
  if (stream) PCST_HIP(hipStreamDestroy(static_cast<hipStream_t>(stream)), "stream_destroy");
  return PCST_OK;
}
