// Fused Adam over one flat fp32 parameter buffer (all parameters of a model
// live in a single allocation, so one launch steps the whole optimizer).
//
// replaces: torch.optim.Adam(params, lr, betas=(0.0, 0.9)) of train.py:252-263
// (G+ATTR_Enhance lr 1e-4, each D lr 4e-4) and the optimizer.zero_grad()
// calls of train.py:452-459, 500-502.  Arithmetic follows torch's Adam:
//   m = lerp(m, g, 1-b1); v = b2 v + (1-b2) g^2;
//   p -= step_size * m / (sqrt(v)/sqrt(bc2) + eps),  step_size = lr / bc1.
// The step count lives on the device (a tick kernel increments it before the
// update reads it), so a captured step graph replays with the right bias
// corrections.
#include "common.h"
#include "../../include/eegan_hip.h"

namespace {

__global__ void adam_tick_kernel(double* step) { *step += 1.0; }

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long n, float b1,
                                                   float b2, float lr, float eps, float wd,
                                                   const double* __restrict__ step) {
  // bias corrections in double from the device step count, as torch's
  // python-float arithmetic does
  const double t = *step;
  const float step_size = (float)((double)lr / (1.0 - pow((double)b1, t)));
  const float bc2_sqrt = (float)sqrt(1.0 - pow((double)b2, t));
  const long n4 = n / 4;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n4; e += (long)gridDim.x * blockDim.x) {
    float4 pp = reinterpret_cast<float4*>(p)[e];
    const float4 gg = reinterpret_cast<const float4*>(g)[e];
    float4 mm = reinterpret_cast<float4*>(m)[e];
    float4 vv = reinterpret_cast<float4*>(v)[e];
    float* P = &pp.x;
    const float* G = &gg.x;
    float* Mv = &mm.x;
    float* V = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gr = G[j] + wd * P[j];
      Mv[j] = (1.f - b1) >= 0.5f ? gr - (gr - Mv[j]) * b1 : Mv[j] + (1.f - b1) * (gr - Mv[j]);
      V[j] = V[j] * b2 + (1.f - b2) * gr * gr;
      const float denom = sqrtf(V[j]) / bc2_sqrt + eps;
      P[j] = P[j] + (-step_size) * (Mv[j] / denom);
    }
    reinterpret_cast<float4*>(p)[e] = pp;
    reinterpret_cast<float4*>(m)[e] = mm;
    reinterpret_cast<float4*>(v)[e] = vv;
  }
  // tail
  for (long e = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    float gr = g[e] + wd * p[e];
    m[e] = (1.f - b1) >= 0.5f ? gr - (gr - m[e]) * b1 : m[e] + (1.f - b1) * (gr - m[e]);
    v[e] = v[e] * b2 + (1.f - b2) * gr * gr;
    const float denom = sqrtf(v[e]) / bc2_sqrt + eps;
    p[e] = p[e] + (-step_size) * (m[e] / denom);
  }
}

}  // namespace

extern "C" {

int eegan_adam(float* p, const float* g, float* m, float* v, long n, float beta1, float beta2, float lr, float eps,
               float weight_decay, double* step, hipStream_t s) {
  if ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(m) |
       reinterpret_cast<uintptr_t>(v)) & 15) {
    ee_set_error("adam: buffers must be 16-byte aligned");
    return -22;
  }
  const int blocks = (int)std::max<long>(1, std::min<long>(2048, (n / 4 + 255) / 256));
  adam_tick_kernel<<<1, 1, 0, s>>>(step);
  int rc = ee_check_launch("adam_tick");
  if (rc) return rc;
  adam_kernel<<<blocks, 256, 0, s>>>(p, g, m, v, n, beta1, beta2, lr, eps, weight_decay, step);
  return ee_check_launch("adam");
}

}  // extern "C"
