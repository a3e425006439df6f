// Error plumbing + version query for the C-ABI library (no global mutable
// state shared between threads: the error text is thread-local).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <mutex>

#include "../../include/eegan_hip.h"
#include "common.h"

static thread_local char g_err[512];
static thread_local EeTiming g_timing;

EeTiming& ee_timing() { return g_timing; }

void ee_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int ee_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    ee_set_error("%s: %s", what, hipGetErrorString(e));
    return -(int)e;
  }
  return 0;
}

static int ee_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    ee_set_error("%s: %s", what, hipGetErrorString(e));
    return -(int)e;
  }
  return 0;
}

extern "C" {
const char* eegan_last_error(void) { return g_err; }
int eegan_abi_version(void) { return EEGAN_ABI_VERSION; }

// Launch timing (bench.py's roofline).  A record on a stream that is being
// captured becomes an external event-record node, so a replayed step graph
// re-times every bracketed launch.
int eegan_event_create(hipEvent_t* ev) { return ee_hip(hipEventCreate(ev), "hipEventCreate"); }
int eegan_event_destroy(hipEvent_t ev) { return ee_hip(hipEventDestroy(ev), "hipEventDestroy"); }
int eegan_stream_create(hipStream_t* s, int priority) {
  if (priority == 0) return ee_hip(hipStreamCreateWithFlags(s, hipStreamNonBlocking), "hipStreamCreateWithFlags");
  int least = 0, greatest = 0;
  int rc = ee_hip(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
  if (rc) return rc;
  // priority > 0: the device's highest priority; < 0: its lowest
  return ee_hip(hipStreamCreateWithPriority(s, hipStreamNonBlocking, priority > 0 ? greatest : least),
                "hipStreamCreateWithPriority");
}
int eegan_stream_destroy(hipStream_t s) { return ee_hip(hipStreamDestroy(s), "hipStreamDestroy"); }
int eegan_event_record(hipEvent_t ev, hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  int rc = ee_hip(hipStreamIsCapturing(s, &st), "hipStreamIsCapturing");
  if (rc) return rc;
  if (st == hipStreamCaptureStatusActive)
    return ee_hip(hipEventRecordWithFlags(ev, s, hipEventRecordExternal), "hipEventRecordWithFlags");
  return ee_hip(hipEventRecord(ev, s), "hipEventRecord");
}
int eegan_event_elapsed(hipEvent_t a, hipEvent_t b, float* ms) {
  return ee_hip(hipEventElapsedTime(ms, a, b), "hipEventElapsedTime");
}
int eegan_timing_arm(hipEvent_t start0, hipEvent_t stop0, hipEvent_t start1, hipEvent_t stop1) {
  g_timing.ev[0] = start0;
  g_timing.ev[1] = stop0;
  g_timing.ev[2] = start1;
  g_timing.ev[3] = stop1;
  g_timing.used = 0;
  g_timing.armed = 1;
  return 0;
}
int eegan_timing_disarm(int* kernels_timed) {
  *kernels_timed = g_timing.armed ? g_timing.used : 0;
  g_timing.armed = 0;
  g_timing.used = 0;
  return 0;
}
}
