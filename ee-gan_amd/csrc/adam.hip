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

// Every fused multiply-add is spelled out and contraction is off: left to
// -ffp-contract the compiler fused different products in different kernels
// (adam_kernel / adam_pack_kernel), which then disagreed in the last bit.
template <bool B1ZERO>
__device__ __forceinline__ void adam_elem(float& P, float G, float& M, float& V, float b1, float b2, float wd,
                                          float step_size, float bc2_sqrt, float eps) {
#pragma clang fp contract(off)
  const float gr = __builtin_fmaf(wd, P, G);
  // torch: exp_avg.lerp_(g, 1 - b1); at b1 = 0 (train.py:252-263's betas) the
  // lerp with weight 1 is g - (g - m) * 0 = g exactly for any finite m, so
  // the old moment is not read
  if (B1ZERO)
    M = gr;
  else
    M = (1.f - b1) >= 0.5f ? __builtin_fmaf(-(gr - M), b1, gr) : __builtin_fmaf(1.f - b1, gr - M, M);
  V = __builtin_fmaf(V, b2, ((1.f - b2) * gr) * gr);
  const float denom = sqrtf(V) / bc2_sqrt + eps;
  P = __builtin_fmaf(-step_size, M / denom, P);
}

template <bool B1ZERO>
__device__ __forceinline__ void adam4(float4& P, float4 G, float4& M, float4& V, float b1, float b2, float wd,
                                      float step_size, float bc2_sqrt, float eps) {
  adam_elem<B1ZERO>(P.x, G.x, M.x, V.x, b1, b2, wd, step_size, bc2_sqrt, eps);
  adam_elem<B1ZERO>(P.y, G.y, M.y, V.y, b1, b2, wd, step_size, bc2_sqrt, eps);
  adam_elem<B1ZERO>(P.z, G.z, M.z, V.z, b1, b2, wd, step_size, bc2_sqrt, eps);
  adam_elem<B1ZERO>(P.w, G.w, M.w, V.w, b1, b2, wd, step_size, bc2_sqrt, eps);
}

template <bool B1ZERO>
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
  const long stride = (long)gridDim.x * blockDim.x;
  float4* P4 = reinterpret_cast<float4*>(p);
  const float4* G4 = reinterpret_cast<const float4*>(g);
  float4* M4 = reinterpret_cast<float4*>(m);
  float4* V4 = reinterpret_cast<float4*>(v);
  long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  // two float4 groups per iteration: every load of both issued before the
  // arithmetic (more bytes in flight per wave)
  for (; e + stride < n4; e += 2 * stride) {
    float4 pp[2], gg[2], mm[2], vv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      pp[u] = P4[e + u * stride];
      gg[u] = G4[e + u * stride];
      if (!B1ZERO) mm[u] = M4[e + u * stride];
      vv[u] = V4[e + u * stride];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float* Pp = &pp[u].x;
      const float* Gp = &gg[u].x;
      float* Mp = &mm[u].x;
      float* Vp = &vv[u].x;
#pragma unroll
      for (int j = 0; j < 4; ++j) adam_elem<B1ZERO>(Pp[j], Gp[j], Mp[j], Vp[j], b1, b2, wd, step_size, bc2_sqrt, eps);
      P4[e + u * stride] = pp[u];
      M4[e + u * stride] = mm[u];
      V4[e + u * stride] = vv[u];
    }
  }
  for (; e < n4; e += stride) {
    float4 pp = P4[e];
    const float4 gg = G4[e];
    float4 mm;
    if (!B1ZERO) mm = M4[e];
    float4 vv = V4[e];
    float* Pp = &pp.x;
    const float* Gp = &gg.x;
    float* Mp = &mm.x;
    float* Vp = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) adam_elem<B1ZERO>(Pp[j], Gp[j], Mp[j], Vp[j], b1, b2, wd, step_size, bc2_sqrt, eps);
    P4[e] = pp;
    M4[e] = mm;
    V4[e] = vv;
  }
  // tail
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float pv = p[i], mv = m[i], vv = v[i];
    adam_elem<false>(pv, g[i], mv, vv, b1, b2, wd, step_size, bc2_sqrt, eps);
    p[i] = pv;
    m[i] = mv;
    v[i] = vv;
  }
}

// ---- Adam step fused with the bf16 weight re-pack (FlatAdam over conv weights) ----
// The separate form reads every updated conv weight back from HBM in the pack
// kernel (and launches it).  Here a workgroup owns a 64 (output channel) x 64
// (input channel) tile of one tap of one conv weight -- channels-last fp32,
// element (co, tap, ci) at p_off + (co * RS + tap) * Cin + ci -- steps it (the
// same adam_elem arithmetic as adam_kernel), keeps the new values in LDS and
// writes both packed images from there: the forward image row co, columns
// tap * Cgp(Cin) + ci (16-B runs along ci) and the data-gradient image row ci,
// columns tap * Cgp(Cout) + co (the transpose, 4-B pairs along co).  Packing
// padding (rows past Cout / Cin, the K tail) is never written: it keeps the
// zeros of the full pack that created the images.  Parameters that are not
// packed conv weights (biases, linear layers, gains, the flat buffer's
// alignment gaps) are stepped by range jobs of 4096 elements per workgroup.
// Job table (int64, 8 per job): conv {0, p_off, fwd image or 0, bwd image or 0,
// Cout, Cin, R*S, 0}, range {1, start, len, 0...}; then njobs + 1 prefix block
// offsets.
constexpr int AP_T = 64, AP_RANGE = 4096;

EE_DEV int ap_cgp(int C) { return C <= 8 ? 8 : (C + 31) / 32 * 32; }

template <bool B1ZERO>
__global__ __launch_bounds__(256) void adam_pack_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        const long* __restrict__ table, int njobs, float b1,
                                                        float b2, float lr, float eps, float wd,
                                                        const double* __restrict__ step) {
  __shared__ float buf[AP_T * (AP_T + 1)];
  const double t = *step;
  const float step_size = (float)((double)lr / (1.0 - pow((double)b1, t)));
  const float bc2_sqrt = (float)sqrt(1.0 - pow((double)b2, t));
  const long* pre = table + 8L * njobs;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pre[mid] <= blockIdx.x) lo = mid;
    else hi = mid - 1;
  }
  const long* j = table + 8L * lo;
  const long lb = (long)blockIdx.x - pre[lo];
  const int tid = threadIdx.x;
  if (j[0] == 1) {   // range job
    const long s0 = j[1] + lb * AP_RANGE, s1 = min(j[1] + j[2], s0 + AP_RANGE);
    long i0 = s0;
    if ((s0 & 3) == 0) {   // float4 body: a thread's AP_RANGE / 1024 groups, all loads before the arithmetic
      const long nq = (s1 - s0) >> 2;
      float4 pp[AP_RANGE / 1024], gg[AP_RANGE / 1024], mm[AP_RANGE / 1024], vv[AP_RANGE / 1024];
#pragma unroll
      for (int u = 0; u < AP_RANGE / 1024; ++u) {
        const long q = tid + u * 256;
        if (q < nq) {
          pp[u] = reinterpret_cast<const float4*>(p + s0)[q];
          gg[u] = reinterpret_cast<const float4*>(g + s0)[q];
          if (!B1ZERO) mm[u] = reinterpret_cast<const float4*>(m + s0)[q];
          vv[u] = reinterpret_cast<const float4*>(v + s0)[q];
        }
      }
#pragma unroll
      for (int u = 0; u < AP_RANGE / 1024; ++u) {
        const long q = tid + u * 256;
        if (q < nq) {
          adam4<B1ZERO>(pp[u], gg[u], mm[u], vv[u], b1, b2, wd, step_size, bc2_sqrt, eps);
          reinterpret_cast<float4*>(p + s0)[q] = pp[u];
          reinterpret_cast<float4*>(m + s0)[q] = mm[u];
          reinterpret_cast<float4*>(v + s0)[q] = vv[u];
        }
      }
      i0 = s0 + nq * 4;
    }
    for (long i = i0 + tid; i < s1; i += 256) {   // unaligned gaps (< 4 elements) and the tail
      float P = p[i], M = B1ZERO ? 0.f : m[i], V = v[i];
      adam_elem<B1ZERO>(P, g[i], M, V, b1, b2, wd, step_size, bc2_sqrt, eps);
      p[i] = P;
      m[i] = M;
      v[i] = V;
    }
    return;
  }
  const long off = j[1];
  bf16_t* fwd = reinterpret_cast<bf16_t*>(j[2]);
  bf16_t* bwd = reinterpret_cast<bf16_t*>(j[3]);
  const int Cout = (int)j[4], Cin = (int)j[5], RS = (int)j[6];
  const int nci = (Cin + AP_T - 1) / AP_T;
  const int it = (int)(lb % nci), tap = (int)((lb / nci) % RS), ct = (int)(lb / ((long)nci * RS));
  const int ci0 = it * AP_T, co0 = ct * AP_T;
  if ((Cin & 3) == 0) {
    // float4 along ci (offsets of the flat buffer's views are multiples of 4): 16 lanes per
    // 256-B row, a thread's four groups' loads issued before their arithmetic
    constexpr int NQ = AP_T * AP_T / 4 / 256;
    float4 pp[NQ], gg[NQ], mm[NQ], vv[NQ];
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      const int e = u * 256 + tid, r = e / (AP_T / 4), c = 4 * (e % (AP_T / 4));
      if (co0 + r < Cout && ci0 + c < Cin) {
        const long i = off + ((long)(co0 + r) * RS + tap) * Cin + ci0 + c;
        pp[u] = *reinterpret_cast<const float4*>(p + i);
        gg[u] = *reinterpret_cast<const float4*>(g + i);
        if (!B1ZERO) mm[u] = *reinterpret_cast<const float4*>(m + i);
        vv[u] = *reinterpret_cast<const float4*>(v + i);
      }
    }
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      const int e = u * 256 + tid, r = e / (AP_T / 4), c = 4 * (e % (AP_T / 4));
      float4 P4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (co0 + r < Cout && ci0 + c < Cin) {
        const long i = off + ((long)(co0 + r) * RS + tap) * Cin + ci0 + c;
        adam4<B1ZERO>(pp[u], gg[u], mm[u], vv[u], b1, b2, wd, step_size, bc2_sqrt, eps);
        *reinterpret_cast<float4*>(p + i) = pp[u];
        *reinterpret_cast<float4*>(m + i) = mm[u];
        *reinterpret_cast<float4*>(v + i) = vv[u];
        P4 = pp[u];
      }
      float* b = buf + r * (AP_T + 1) + c;
      b[0] = P4.x;
      b[1] = P4.y;
      b[2] = P4.z;
      b[3] = P4.w;
    }
  } else {
#pragma unroll 4
    for (int k = 0; k < AP_T * AP_T / 256; ++k) {
      const int e = k * 256 + tid, r = e / AP_T, c = e % AP_T;   // lanes along ci: 256-B rows
      float P = 0.f;
      if (co0 + r < Cout && ci0 + c < Cin) {
        const long i = off + ((long)(co0 + r) * RS + tap) * Cin + ci0 + c;
        P = p[i];
        float M = B1ZERO ? 0.f : m[i], V = v[i];
        adam_elem<B1ZERO>(P, g[i], M, V, b1, b2, wd, step_size, bc2_sqrt, eps);
        p[i] = P;
        m[i] = M;
        v[i] = V;
      }
      buf[r * (AP_T + 1) + c] = P;
    }
  }
  __syncthreads();
  if (fwd) {   // rows co < Cout, this tap's channel run [0, Cgp(Cin)): pairs along ci
    const int cg = ap_cgp(Cin), Kw = (RS * cg + 31) / 32 * 32, ncol = min(AP_T, cg - ci0);
    for (int e = tid; e < AP_T * AP_T / 2; e += 256) {
      const int r = e / (AP_T / 2), cp = 2 * (e % (AP_T / 2));
      if (co0 + r < Cout && cp < ncol)
        *reinterpret_cast<uint32_t*>(fwd + (long)(co0 + r) * Kw + tap * cg + ci0 + cp) =
            pack2(buf[r * (AP_T + 1) + cp], buf[r * (AP_T + 1) + cp + 1]);
    }
  }
  if (bwd) {   // rows ci < Cin, this tap's run [0, Cgp(Cout)): pairs along co
    const int cg = ap_cgp(Cout), Kw = (RS * cg + 31) / 32 * 32, ncol = min(AP_T, cg - co0);
    for (int e = tid; e < AP_T * AP_T / 2; e += 256) {
      const int c = e / (AP_T / 2), rp = 2 * (e % (AP_T / 2));
      if (ci0 + c < Cin && rp < ncol)
        *reinterpret_cast<uint32_t*>(bwd + (long)(ci0 + c) * Kw + tap * cg + co0 + rp) =
            pack2(buf[rp * (AP_T + 1) + c], buf[(rp + 1) * (AP_T + 1) + c]);
    }
  }
}

}  // namespace

extern "C" {

long eegan_adam_pack_blocks(int Cout, int Cin, int R, int S) {
  return (long)((Cout + AP_T - 1) / AP_T) * R * S * ((Cin + AP_T - 1) / AP_T);
}

long eegan_adam_range_blocks(long len) { return (len + AP_RANGE - 1) / AP_RANGE; }

int eegan_adam_pack(float* p, const float* g, float* m, float* v, float beta1, float beta2, float lr, float eps,
                    float weight_decay, double* step, const long* table, int njobs, long total_blocks,
                    hipStream_t s) {
  if (njobs <= 0 || total_blocks <= 0) {
    ee_set_error("adam_pack: empty job table");
    return -22;
  }
  adam_tick_kernel<<<1, 1, 0, s>>>(step);
  int rc = ee_check_launch("adam_tick");
  if (rc) return rc;
  if (beta1 == 0.f)
    adam_pack_kernel<true><<<(unsigned)total_blocks, 256, 0, s>>>(p, g, m, v, table, njobs, beta1, beta2, lr, eps,
                                                                  weight_decay, step);
  else
    adam_pack_kernel<false><<<(unsigned)total_blocks, 256, 0, s>>>(p, g, m, v, table, njobs, beta1, beta2, lr, eps,
                                                                   weight_decay, step);
  return ee_check_launch("adam_pack");
}

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
  if (beta1 == 0.f)
    adam_kernel<true><<<blocks, 256, 0, s>>>(p, g, m, v, n, beta1, beta2, lr, eps, weight_decay, step);
  else
    adam_kernel<false><<<blocks, 256, 0, s>>>(p, g, m, v, n, beta1, beta2, lr, eps, weight_decay, step);
  return ee_check_launch("adam");
}

}  // extern "C"
