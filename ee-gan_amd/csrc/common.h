// Shared device helpers for the EE-GAN MI355X (gfx950) kernel library.
// bf16 activations are stored as raw uint16 (NHWC, channel stride "ld");
// all arithmetic accumulates in fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <algorithm>

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;

#define EE_DEV __device__ __forceinline__

EE_DEV float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
EE_DEV bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32: RNE, NaN-preserving
  return __builtin_bit_cast(bf16_t, b);
}
EE_DEV uint32_t pack2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }
EE_DEV float lo_f(uint32_t u) { return __uint_as_float(u << 16); }
EE_DEV float hi_f(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// activation codes shared with the host glue (eegan_hip/_lib.py)
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_LRELU = 2, ACT_TANH = 3, ACT_SIGMOID = 4 };

EE_DEV float act_fwd(float v, int act, float slope) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_LRELU: return v > 0.f ? v : v * slope;
    case ACT_TANH: return tanhf(v);
    case ACT_SIGMOID: return 1.f / (1.f + __expf(-v));
    default: return v;
  }
}
// derivative expressed through the activation's OUTPUT y
EE_DEV float act_dgrad_from_y(float y, int act, float slope) {
  switch (act) {
    case ACT_RELU: return y > 0.f ? 1.f : 0.f;
    case ACT_LRELU: return y > 0.f ? 1.f : slope;
    case ACT_TANH: return 1.f - y * y;
    case ACT_SIGMOID: return y * (1.f - y);
    default: return 1.f;
  }
}

EE_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
EE_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sum for blockDim.x multiple of 64 (<= 1024); `red` >= 16 floats
EE_DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  const int nw = blockDim.x >> 6;
  float t = (threadIdx.x < nw) ? red[threadIdx.x] : 0.f;
  if (w == 0) t = wave_sum(t);
  if (threadIdx.x == 0) red[0] = t;
  __syncthreads();
  float r = red[0];
  __syncthreads();
  return r;
}

static inline int ee_cdiv(long a, long b) { return (int)((a + b - 1) / b); }
static inline int ee_round_up(int a, int b) { return (a + b - 1) / b * b; }

// error reporting (thread-local, no global mutable state shared across threads)
void ee_set_error(const char* fmt, ...);
int ee_check_launch(const char* what);

#define EE_LAUNCH_CHECK(name) return ee_check_launch(name)
