// GlobalAttentionGeneral (word <-> feature-map attention) on bf16 MFMA.
//
// replaces miscc/DAMSM_losses.py:65-132 (GlobalAttentionGeneral.forward);
// the reference defines it but never calls it on the training path (SURVEY.md
// §2 a17), so this is API completeness, not a hot op.
//
//   logits[b][q][s] = sum_d input[b][d][q] key[b][d][s]            (q < Lq = ih*iw, s < S)
//   masked_fill(-inf) with the reference's row indexing: the mask is
//     self.mask.repeat(queryL, 1) against rows b*Lq + q, so row (b, q) reads
//     mask[(b*Lq + q) % B]  (DAMSM_losses.py:118-121, reproduced as is)
//   att = softmax over s                                            [B][S][Lq]
//   wc[b][c][q] = sum_s value[b][c][s] att[b][s][q]                 [B][cdf][Lq]
//
// Forward: one workgroup per (64 queries, b), 4 waves x 16 queries.  Both
// contractions are split-bf16 MFMAs (hi*hi + lo*hi + hi*lo, ~fp32 accuracy):
// the logits over idf in K-steps of 32 (input / key tiles staged in LDS), the
// softmax in registers (16-lane shuffles), the weighted context over s with
// att kept in LDS.  S <= 64.
// Backward (fp32 SIMT; the op is cold): per query tile, g = datt + value^T dwc,
// dlogits = att (g - <att, g>), dinput = key dlogits, and per-tile partials of
// dkey = input dlogits^T and dvalue = dwc att^T, reduced over tiles in a
// fixed order (deterministic, no atomics).
#include "common.h"
#include "../../include/eegan_hip.h"

namespace {

constexpr int GQ = 64;  // queries per workgroup
constexpr int GS = 64;  // max source length
constexpr int GK = 32;  // idf per K-step
constexpr int KLD = GK + 8;
constexpr int ALD = GS + 8;

EE_DEV bf16x8_t lds_frag(const bf16_t* p) {
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(p));
}
EE_DEV f32x4_t mfma(bf16x8_t a, bf16x8_t b, f32x4_t c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
EE_DEV float xmax16(float v) {
  v = fmaxf(v, __shfl_xor(v, 1, 64));
  v = fmaxf(v, __shfl_xor(v, 2, 64));
  v = fmaxf(v, __shfl_xor(v, 4, 64));
  v = fmaxf(v, __shfl_xor(v, 8, 64));
  return v;
}
EE_DEV float xsum16(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}

__global__ __launch_bounds__(256) void gag_fwd_kernel(const float* __restrict__ in, const float* __restrict__ key,
                                                      const float* __restrict__ val, const uint8_t* __restrict__ mask,
                                                      int B, int idf, int cdf, int Lq, int S, float* __restrict__ wc,
                                                      float* __restrict__ att) {
  __shared__ __attribute__((aligned(16))) bf16_t inh[GQ][KLD], inl[GQ][KLD];  // query x k
  __shared__ __attribute__((aligned(16))) bf16_t kh[GS][KLD], kl[GS][KLD];    // source x k
  __shared__ __attribute__((aligned(16))) bf16_t ah[GQ][ALD], al[GQ][ALD];    // att: query x source
  __shared__ float af[GS][GQ + 1];                                            // att fp32: source x query
  const int t = threadIdx.x, l = t & 63, wv = t >> 6, fr = l & 15, fq = l >> 4;
  const int b = blockIdx.y, q0 = blockIdx.x * GQ;
  f32x4_t acc[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) acc[n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < idf; k0 += GK) {
    __syncthreads();
    for (int e = t; e < GK * GQ; e += 256) {
      const int k = e / GQ, q = e % GQ;
      const float v = (k0 + k < idf && q0 + q < Lq) ? in[((long)b * idf + k0 + k) * Lq + q0 + q] : 0.f;
      const bf16_t h = f2bf(v);
      inh[q][k] = h;
      inl[q][k] = f2bf(v - bf2f(h));
    }
    for (int e = t; e < GK * GS; e += 256) {
      const int k = e / GS, s = e % GS;
      const float v = (k0 + k < idf && s < S) ? key[((long)b * idf + k0 + k) * S + s] : 0.f;
      const bf16_t h = f2bf(v);
      kh[s][k] = h;
      kl[s][k] = f2bf(v - bf2f(h));
    }
    __syncthreads();
    const bf16x8_t a_h = lds_frag(&inh[wv * 16 + fr][fq * 8]), a_l = lds_frag(&inl[wv * 16 + fr][fq * 8]);
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const bf16x8_t b_h = lds_frag(&kh[n * 16 + fr][fq * 8]), b_l = lds_frag(&kl[n * 16 + fr][fq * 8]);
      acc[n] = mfma(a_h, b_h, acc[n]);
      acc[n] = mfma(a_l, b_h, acc[n]);
      acc[n] = mfma(a_h, b_l, acc[n]);
    }
  }
  // softmax over the source: row q = 16 wv + 4 fq + r, column s = 16 n + fr
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = wv * 16 + fq * 4 + r;
    const long mrow = ((long)b * Lq + q0 + q) % B;
    float x[4], m = -INFINITY;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int s = n * 16 + fr;
      const bool off = s >= S || (mask != nullptr && mask[mrow * S + s]);
      x[n] = off ? -INFINITY : acc[n][r];
      m = fmaxf(m, x[n]);
    }
    m = xmax16(m);
    float sum = 0.f;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      x[n] = n * 16 + fr < S ? expf(x[n] - m) : 0.f;
      sum += x[n];
    }
    const float inv = 1.f / xsum16(sum);
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int s = n * 16 + fr;
      const float p = x[n] * inv;
      const bf16_t h = f2bf(p);
      ah[q][s] = h;
      al[q][s] = f2bf(p - bf2f(h));
      af[s][q] = p;
    }
  }
  __syncthreads();
  for (int e = t; e < S * GQ; e += 256) {
    const int s = e / GQ, q = e % GQ;
    if (q0 + q < Lq) att[((long)b * S + s) * Lq + q0 + q] = af[s][q];
  }
  // wc[c][q] = sum_s value[c][s] att[q][s]: rows c (A from global), columns q (B from LDS)
  const int nks = (S + 31) / 32;
  for (int ct = wv; ct * 16 < cdf; ct += 4) {
    f32x4_t o[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) o[n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int c = ct * 16 + fr;
    for (int ks = 0; ks < nks; ++ks) {
      uint32_t vh[4], vl[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v2[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int s = ks * 32 + fq * 8 + 2 * j + u;
          v2[u] = (c < cdf && s < S) ? val[((long)b * cdf + c) * S + s] : 0.f;
        }
        const bf16_t h0 = f2bf(v2[0]), h1 = f2bf(v2[1]);
        vh[j] = (uint32_t)h0 | ((uint32_t)h1 << 16);
        vl[j] = pack2(v2[0] - bf2f(h0), v2[1] - bf2f(h1));
      }
      const bf16x8_t a_h = __builtin_bit_cast(bf16x8_t, make_uint4(vh[0], vh[1], vh[2], vh[3]));
      const bf16x8_t a_l = __builtin_bit_cast(bf16x8_t, make_uint4(vl[0], vl[1], vl[2], vl[3]));
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const bf16x8_t b_h = lds_frag(&ah[n * 16 + fr][ks * 32 + fq * 8]);
        const bf16x8_t b_l = lds_frag(&al[n * 16 + fr][ks * 32 + fq * 8]);
        o[n] = mfma(a_h, b_h, o[n]);
        o[n] = mfma(a_l, b_h, o[n]);
        o[n] = mfma(a_h, b_l, o[n]);
      }
    }
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cc = ct * 16 + fq * 4 + r, q = q0 + n * 16 + fr;
        if (cc < cdf && q < Lq) wc[((long)b * cdf + cc) * Lq + q] = o[n][r];
      }
  }
}

// backward of one query tile; partial dkey / dvalue of the tile into ws
__global__ __launch_bounds__(256) void gag_bwd_tile_kernel(const float* __restrict__ in, const float* __restrict__ key,
                                                           const float* __restrict__ val,
                                                           const float* __restrict__ att,
                                                           const float* __restrict__ dwc,
                                                           const float* __restrict__ datt, int B, int idf, int cdf,
                                                           int Lq, int S, float* __restrict__ din,
                                                           float* __restrict__ pkey, float* __restrict__ pval) {
  __shared__ float pa[GS][GQ + 1];  // att (source x query)
  __shared__ float dl[GS][GQ + 1];  // dlogits
  __shared__ float rdot[4][GQ];
  const int t = threadIdx.x, lq = t & 63, wv = t >> 6;
  const int b = blockIdx.y, q0 = blockIdx.x * GQ, tile = blockIdx.x;
  const int q = q0 + lq;
  const bool qok = q < Lq;
  for (int e = t; e < GS * GQ; e += 256) {
    const int s = e / GQ, qq = e % GQ;
    pa[s][qq] = (s < S && q0 + qq < Lq) ? att[((long)b * S + s) * Lq + q0 + qq] : 0.f;
  }
  __syncthreads();
  // g[s][q] = datt[s][q] + sum_c dwc[c][q] value[c][s], s = wv + 4 i
  float g[GS / 4];
#pragma unroll
  for (int i = 0; i < GS / 4; ++i) {
    const int s = wv + 4 * i;
    g[i] = (datt != nullptr && qok && s < S) ? datt[((long)b * S + s) * Lq + q] : 0.f;
  }
  if (dwc != nullptr) {
    for (int c = 0; c < cdf; ++c) {
      const float dw = qok ? dwc[((long)b * cdf + c) * Lq + q] : 0.f;
      const float* vr = val + ((long)b * cdf + c) * S;
#pragma unroll
      for (int i = 0; i < GS / 4; ++i) {
        const int s = wv + 4 * i;
        if (s < S) g[i] += dw * vr[s];
      }
    }
  }
  float dot = 0.f;
#pragma unroll
  for (int i = 0; i < GS / 4; ++i) dot += pa[wv + 4 * i][lq] * g[i];
  rdot[wv][lq] = dot;
  __syncthreads();
  dot = rdot[0][lq] + rdot[1][lq] + rdot[2][lq] + rdot[3][lq];
#pragma unroll
  for (int i = 0; i < GS / 4; ++i) {
    const int s = wv + 4 * i;
    const float p = pa[s][lq];
    dl[s][lq] = p == 0.f ? 0.f : p * (g[i] - dot);
  }
  __syncthreads();
  // dinput[d][q] = sum_s key[d][s] dl[s][q]
  for (int d = wv; d < idf; d += 4) {
    const float* kr = key + ((long)b * idf + d) * S;
    float v = 0.f;
    for (int s = 0; s < S; ++s) v += kr[s] * dl[s][lq];
    if (qok) din[((long)b * idf + d) * Lq + q] = v;
  }
  // partials over this tile's queries: lane = source s
  const int s = lq;
  for (int d = wv; d < idf; d += 4) {
    const float* ir = in + ((long)b * idf + d) * Lq + q0;
    float v = 0.f;
    for (int qq = 0; qq < GQ && q0 + qq < Lq; ++qq) v += ir[qq] * dl[s][qq];
    if (s < S) pkey[(((long)tile * B + b) * idf + d) * S + s] = v;
  }
  for (int c = wv; c < cdf; c += 4) {
    float v = 0.f;
    if (dwc != nullptr) {
      const float* dr = dwc + ((long)b * cdf + c) * Lq + q0;
      for (int qq = 0; qq < GQ && q0 + qq < Lq; ++qq) v += dr[qq] * pa[s][qq];
    }
    if (s < S) pval[(((long)tile * B + b) * cdf + c) * S + s] = v;
  }
}

// fixed-order sum of the per-tile partials
__global__ __launch_bounds__(256) void gag_bwd_reduce_kernel(const float* __restrict__ part, int ntile, long n,
                                                             float* __restrict__ out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float v = 0.f;
  for (int k = 0; k < ntile; ++k) v += part[(long)k * n + i];
  out[i] = v;
}

bool gag_check(int B, int idf, int cdf, int Lq, int S, const char* what) {
  if (B < 1 || idf < 1 || cdf < 1 || Lq < 1 || S < 1 || S > GS) {
    ee_set_error("%s: need B, idf, cdf, queryL >= 1 and 1 <= sourceL <= %d (B=%d idf=%d cdf=%d queryL=%d sourceL=%d)",
                 what, GS, B, idf, cdf, Lq, S);
    return false;
  }
  if ((long)B * Lq >= (1L << 31)) {
    ee_set_error("%s: B * queryL too large", what);
    return false;
  }
  return true;
}

}  // namespace

extern "C" {

int eegan_gag_fwd(const float* input, const float* context_key, const float* content_value, const unsigned char* mask,
                  int B, int idf, int cdf, int queryL, int sourceL, float* weighted_context, float* attn,
                  hipStream_t s) {
  if (!gag_check(B, idf, cdf, queryL, sourceL, "gag_fwd")) return -22;
  ee_launch(gag_fwd_kernel, dim3((queryL + GQ - 1) / GQ, B), dim3(256), 0, s, input, context_key, content_value,
            (const uint8_t*)mask, B, idf, cdf, queryL, sourceL, weighted_context, attn);
  return ee_check_launch("gag_fwd");
}

long eegan_gag_workspace(int B, int idf, int cdf, int queryL, int sourceL) {
  const long ntile = (queryL + GQ - 1) / GQ;
  return ntile * B * (long)(idf + cdf) * sourceL * (long)sizeof(float);
}

int eegan_gag_bwd(const float* input, const float* context_key, const float* content_value, const float* attn,
                  const float* d_weighted_context, const float* d_attn, int B, int idf, int cdf, int queryL,
                  int sourceL, float* d_input, float* d_key, float* d_value, void* ws, hipStream_t s) {
  if (!gag_check(B, idf, cdf, queryL, sourceL, "gag_bwd")) return -22;
  const int ntile = (queryL + GQ - 1) / GQ;
  float* pkey = static_cast<float*>(ws);
  float* pval = pkey + (long)ntile * B * idf * sourceL;
  ee_launch(gag_bwd_tile_kernel, dim3(ntile, B), dim3(256), 0, s, input, context_key, content_value, attn,
            d_weighted_context, d_attn, B, idf, cdf, queryL, sourceL, d_input, pkey, pval);
  int rc = ee_check_launch("gag_bwd_tile");
  if (rc) return rc;
  const long nk = (long)B * idf * sourceL, nv = (long)B * cdf * sourceL;
  ee_launch(gag_bwd_reduce_kernel, dim3((nk + 255) / 256), dim3(256), 0, s, (const float*)pkey, ntile, nk, d_key);
  rc = ee_check_launch("gag_bwd_reduce");
  if (rc) return rc;
  ee_launch(gag_bwd_reduce_kernel, dim3((nv + 255) / 256), dim3(256), 0, s, (const float*)pval, ntile, nv, d_value);
  return ee_check_launch("gag_bwd_reduce");
}

}  // extern "C"
