// Probe: can HIP time kernels inside a captured graph with external event
// record nodes, and does hipExtLaunchKernel with start/stop events capture?
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

__global__ void spin(float* x, int n) {
  float v = x[threadIdx.x];
  for (int i = 0; i < n; ++i) v = v * 1.0000001f + 1e-7f;
  x[threadIdx.x] = v;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); } } while (0)

int main() {
  float* d; CK(hipMalloc(&d, 4096));
  hipStream_t s; CK(hipStreamCreate(&s));
  hipEvent_t e0, e1, e2, e3;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2)); CK(hipEventCreate(&e3));
  // eager reference
  CK(hipEventRecord(e0, s)); spin<<<1, 64, 0, s>>>(d, 1 << 20); CK(hipEventRecord(e1, s)); CK(hipStreamSynchronize(s));
  float ms = -1; CK(hipEventElapsedTime(&ms, e0, e1)); printf("eager events: %.3f ms\n", ms);
  // capture with external event records
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  CK(hipEventRecordWithFlags(e0, s, hipEventRecordExternal));
  spin<<<1, 64, 0, s>>>(d, 1 << 20);
  CK(hipEventRecordWithFlags(e1, s, hipEventRecordExternal));
  spin<<<1, 64, 0, s>>>(d, 1 << 19);
  CK(hipEventRecordWithFlags(e2, s, hipEventRecordExternal));
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int it = 0; it < 3; ++it) {
    CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s));
    float a = -1, b = -1; CK(hipEventElapsedTime(&a, e0, e1)); CK(hipEventElapsedTime(&b, e1, e2));
    printf("graph replay %d: k1 %.3f ms, k2 %.3f ms\n", it, a, b);
  }
  // external records under Global / Relaxed capture modes, fresh (never recorded) events
  for (int mode = 0; mode < 3; ++mode) {
    hipStreamCaptureMode cm = mode == 0 ? hipStreamCaptureModeGlobal : mode == 1 ? hipStreamCaptureModeThreadLocal
                                                                                  : hipStreamCaptureModeRelaxed;
    hipEvent_t f0, f1;
    CK(hipEventCreate(&f0)); CK(hipEventCreate(&f1));
    hipStream_t s2; CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipGraph_t g3; hipGraphExec_t ge3;
    CK(hipStreamBeginCapture(s2, cm));
    hipError_t r0 = hipEventRecordWithFlags(f0, s2, hipEventRecordExternal);
    spin<<<1, 64, 0, s2>>>(d, 1 << 18);
    hipError_t r1 = hipEventRecordWithFlags(f1, s2, hipEventRecordExternal);
    CK(hipStreamEndCapture(s2, &g3));
    printf("capture mode %d: record %s / %s\n", mode, hipGetErrorString(r0), hipGetErrorString(r1));
    CK(hipGraphInstantiate(&ge3, g3, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge3, s2)); CK(hipStreamSynchronize(s2));
    float a3 = -1; CK(hipEventElapsedTime(&a3, f0, f1)); printf("  elapsed %.3f ms\n", a3);
  }
  // hipExtLaunchKernel with start/stop events under capture
  hipGraph_t g2; hipGraphExec_t ge2;
  int n = 1 << 20;
  void* args[] = {&d, &n};
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  hipError_t r = hipExtLaunchKernel((const void*)spin, dim3(1), dim3(64), args, 0, s, e0, e3, 0);
  printf("hipExtLaunchKernel under capture: %s\n", hipGetErrorString(r));
  CK(hipStreamEndCapture(s, &g2));
  if (r == hipSuccess) {
    CK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge2, s)); CK(hipStreamSynchronize(s));
    float a = -1; CK(hipEventElapsedTime(&a, e0, e3)); printf("ext-launch in graph: %.3f ms\n", a);
  }
  // eager hipExtLaunchKernel
  r = hipExtLaunchKernel((const void*)spin, dim3(1), dim3(64), args, 0, s, e0, e3, 0);
  CK(hipStreamSynchronize(s));
  float a = -1; CK(hipEventElapsedTime(&a, e0, e3)); printf("ext-launch eager: %s %.3f ms\n", hipGetErrorString(r), a);
  return 0;
}
