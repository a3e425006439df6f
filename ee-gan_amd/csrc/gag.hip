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
// Any source length: the source is processed in chunks of 64.  Forward, two
// kernels, one workgroup per (64 queries, b), 4 waves x 16 queries:
//   stats: the logits of each chunk (split-bf16 MFMA over idf in K-steps of
//          32: hi*hi + lo*hi + hi*lo, ~fp32 accuracy), the row max and the
//          rescaled row sum carried across chunks (online softmax);
//   ctx:   per 64 output channels (blockIdx.z), each chunk's logits again,
//          normalised with the final max / sum into att (written once, by
//          channel group 0), and wc accumulated over the chunks in registers
//          (split-bf16 MFMA, att staged in LDS).
// Backward (fp32 SIMT; the op is cold), deterministic (fixed-order sums, no
// atomics): per query tile g = datt + value^T dwc, <att, g> over all chunks,
// dlogits = att (g - <att, g>) into the workspace; then dinput = key dlogits,
// dkey = input dlogits^T and dvalue = dwc att^T, one output element per thread.
#include "common.h"
#include "../../include/eegan_hip.h"

namespace {

constexpr int GQ = 64;  // queries per workgroup
constexpr int GS = 64;  // sources per chunk
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

struct GagSmem {
  bf16_t inh[GQ][KLD], inl[GQ][KLD];  // query x k
  bf16_t kh[GS][KLD], kl[GS][KLD];    // source x k
};

// logits of queries q0.. (this wave: 16 rows) x sources s0..s0+63 into acc[4]
// (row q = 16 wv + 4 fq + r, column s0 + 16 n + fr); masked / out-of-range
// columns are -inf
EE_DEV void chunk_logits(GagSmem& sm, const float* __restrict__ in, const float* __restrict__ key,
                         const uint8_t* __restrict__ mask, int B, int idf, int Lq, int S, int b, int q0, int s0,
                         f32x4_t acc[4]) {
  const int t = threadIdx.x, l = t & 63, wv = t >> 6, fr = l & 15, fq = l >> 4;
#pragma unroll
  for (int n = 0; n < 4; ++n) acc[n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < idf; k0 += GK) {
    __syncthreads();
    for (int e = t; e < GK * GQ; e += 256) {
      const int k = e / GQ, q = e % GQ;
      const float v = (k0 + k < idf && q0 + q < Lq) ? in[((long)b * idf + k0 + k) * Lq + q0 + q] : 0.f;
      const bf16_t h = f2bf(v);
      sm.inh[q][k] = h;
      sm.inl[q][k] = f2bf(v - bf2f(h));
    }
    for (int e = t; e < GK * GS; e += 256) {
      const int k = e / GS, s = e % GS;
      const float v = (k0 + k < idf && s0 + s < S) ? key[((long)b * idf + k0 + k) * S + s0 + s] : 0.f;
      const bf16_t h = f2bf(v);
      sm.kh[s][k] = h;
      sm.kl[s][k] = f2bf(v - bf2f(h));
    }
    __syncthreads();
    const bf16x8_t a_h = lds_frag(&sm.inh[wv * 16 + fr][fq * 8]), a_l = lds_frag(&sm.inl[wv * 16 + fr][fq * 8]);
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const bf16x8_t b_h = lds_frag(&sm.kh[n * 16 + fr][fq * 8]), b_l = lds_frag(&sm.kl[n * 16 + fr][fq * 8]);
      acc[n] = mfma(a_h, b_h, acc[n]);
      acc[n] = mfma(a_l, b_h, acc[n]);
      acc[n] = mfma(a_h, b_l, acc[n]);
    }
  }
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int s = s0 + n * 16 + fr;
    f32x4_t v = acc[n];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long mrow = ((long)b * Lq + q0 + wv * 16 + fq * 4 + r) % B;
      const bool off = s >= S || (mask != nullptr && mask[mrow * S + s] != 0);
      v[r] = off ? -INFINITY : v[r];
    }
    acc[n] = v;
  }
}

// row max / sum of exp over all sources -> stats[b][q] = (max, sum)
__global__ __launch_bounds__(256) void gag_stats_kernel(const float* __restrict__ in, const float* __restrict__ key,
                                                        const uint8_t* __restrict__ mask, int B, int idf, int Lq,
                                                        int S, float2* __restrict__ stats) {
  __shared__ __attribute__((aligned(16))) GagSmem sm;
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6, fr = l & 15, fq = l >> 4;
  const int b = blockIdx.y, q0 = blockIdx.x * GQ;
  float m[4], z[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) m[r] = -INFINITY, z[r] = 0.f;
  for (int s0 = 0; s0 < S; s0 += GS) {
    f32x4_t acc[4];
    chunk_logits(sm, in, key, mask, B, idf, Lq, S, b, q0, s0, acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float cm = fmaxf(fmaxf(acc[0][r], acc[1][r]), fmaxf(acc[2][r], acc[3][r]));
      cm = xmax16(cm);
      const float nm = fmaxf(m[r], cm);
      float e = 0.f;
      if (nm != -INFINITY) {
#pragma unroll
        for (int n = 0; n < 4; ++n) e += expf(acc[n][r] - nm);
      }
      e = xsum16(e);
      z[r] = (m[r] == -INFINITY ? 0.f : z[r] * expf(m[r] - nm)) + e;
      m[r] = nm;
    }
  }
  if (fr == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + wv * 16 + fq * 4 + r;
      if (q < Lq) stats[(long)b * Lq + q] = make_float2(m[r], z[r]);
    }
  }
}

// att (channel group 0 writes it) and wc for 64 output channels (blockIdx.z)
__global__ __launch_bounds__(256) void gag_ctx_kernel(const float* __restrict__ in, const float* __restrict__ key,
                                                      const float* __restrict__ val, const uint8_t* __restrict__ mask,
                                                      const float2* __restrict__ stats, int B, int idf, int cdf,
                                                      int Lq, int S, float* __restrict__ wc, float* __restrict__ att) {
  __shared__ __attribute__((aligned(16))) GagSmem sm;
  __shared__ __attribute__((aligned(16))) bf16_t ah[GQ][ALD], al[GQ][ALD];  // att chunk: query x source
  __shared__ float af[GS][GQ + 1];                                          // att chunk fp32: source x query
  const int t = threadIdx.x, l = t & 63, wv = t >> 6, fr = l & 15, fq = l >> 4;
  const int b = blockIdx.y, q0 = blockIdx.x * GQ, cg = blockIdx.z;
  float rm[4], rinv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = q0 + wv * 16 + fq * 4 + r;
    const float2 st = q < Lq ? stats[(long)b * Lq + q] : make_float2(0.f, 1.f);
    rm[r] = st.x;
    rinv[r] = 1.f / st.y;
  }
  const int c = cg * 64 + wv * 16 + fr;  // this lane's A-operand row (output channel)
  f32x4_t o[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) o[n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int s0 = 0; s0 < S; s0 += GS) {
    f32x4_t acc[4];
    chunk_logits(sm, in, key, mask, B, idf, Lq, S, b, q0, s0, acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = wv * 16 + fq * 4 + r;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int s = n * 16 + fr;
        const float p = s0 + s < S ? expf(acc[n][r] - rm[r]) * rinv[r] : 0.f;
        const bf16_t h = f2bf(p);
        ah[q][s] = h;
        al[q][s] = f2bf(p - bf2f(h));
        af[s][q] = p;
      }
    }
    __syncthreads();
    if (cg == 0) {
      const int sn = min(GS, S - s0);
      for (int e = t; e < sn * GQ; e += 256) {
        const int s = e / GQ, q = e % GQ;
        if (q0 + q < Lq) att[((long)b * S + s0 + s) * Lq + q0 + q] = af[s][q];
      }
    }
    // o[c][q] += sum_{s in chunk} value[c][s] att[q][s]: rows c (A from global), columns q (B from LDS)
#pragma unroll
    for (int ks = 0; ks < GS / 32; ++ks) {
      uint32_t vh[4], vl[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v2[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int s = s0 + ks * 32 + fq * 8 + 2 * j + u;
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
    // the next chunk's logits re-stage sm behind a barrier; ah / al / af are
    // rewritten only after it, by which point every wave has consumed them
  }
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int cc = cg * 64 + wv * 16 + fq * 4 + r, q = q0 + n * 16 + fr;
      if (cc < cdf && q < Lq) wc[((long)b * cdf + cc) * Lq + q] = o[n][r];
    }
}

// dlogits of one query tile over all sources (two passes: <att, g>, then
// att (g - <att, g>)), written to dl[b][s][q]
__global__ __launch_bounds__(256) void gag_bwd_dl_kernel(const float* __restrict__ val, const float* __restrict__ att,
                                                         const float* __restrict__ dwc, const float* __restrict__ datt,
                                                         int cdf, int Lq, int S, float* __restrict__ dl) {
  __shared__ float rdot[4][GQ];
  const int t = threadIdx.x, lq = t & 63, wv = t >> 6;
  const int b = blockIdx.y, q = blockIdx.x * GQ + lq;
  const bool qok = q < Lq;
  float dot = 0.f;
  for (int pass = 0; pass < 2; ++pass) {
    for (int s0 = 0; s0 < S; s0 += GS) {
      float g[GS / 4];
#pragma unroll
      for (int i = 0; i < GS / 4; ++i) {
        const int s = s0 + wv + 4 * i;
        g[i] = (datt != nullptr && qok && s < S) ? datt[((long)b * S + s) * Lq + q] : 0.f;
      }
      if (dwc != nullptr) {
        for (int c = 0; c < cdf; ++c) {
          const float dw = qok ? dwc[((long)b * cdf + c) * Lq + q] : 0.f;
          const float* vr = val + ((long)b * cdf + c) * S;
#pragma unroll
          for (int i = 0; i < GS / 4; ++i) {
            const int s = s0 + wv + 4 * i;
            if (s < S) g[i] += dw * vr[s];
          }
        }
      }
#pragma unroll
      for (int i = 0; i < GS / 4; ++i) {
        const int s = s0 + wv + 4 * i;
        const float p = (qok && s < S) ? att[((long)b * S + s) * Lq + q] : 0.f;
        if (pass == 0) {
          dot += p * g[i];
        } else if (qok && s < S) {
          dl[((long)b * S + s) * Lq + q] = p == 0.f ? 0.f : p * (g[i] - dot);
        }
      }
    }
    if (pass == 0) {
      rdot[wv][lq] = dot;
      __syncthreads();
      dot = rdot[0][lq] + rdot[1][lq] + rdot[2][lq] + rdot[3][lq];
    }
  }
}

// dinput[b][d][q] = sum_s key[b][d][s] dl[b][s][q]
__global__ __launch_bounds__(256) void gag_bwd_din_kernel(const float* __restrict__ key, const float* __restrict__ dl,
                                                          int idf, int Lq, int S, float* __restrict__ din) {
  const int q = blockIdx.x * 256 + threadIdx.x, d = blockIdx.y, b = blockIdx.z;
  if (q >= Lq) return;
  const float* kr = key + ((long)b * idf + d) * S;
  const float* dr = dl + (long)b * S * Lq + q;
  float v = 0.f;
  for (int s = 0; s < S; ++s) v += kr[s] * dr[(long)s * Lq];
  din[((long)b * idf + d) * Lq + q] = v;
}

// out[b][r][s] = sum_q x[b][r][q] y[b][s][q]  (dkey: x = input, y = dl; dvalue: x = dwc, y = att)
__global__ __launch_bounds__(256) void gag_bwd_rowdot_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                             int R, int Lq, int S, float* __restrict__ out) {
  const int s = blockIdx.x * 256 + threadIdx.x, r = blockIdx.y, b = blockIdx.z;
  if (s >= S) return;
  const float* xr = x + ((long)b * R + r) * Lq;
  const float* yr = y + ((long)b * S + s) * Lq;
  float v = 0.f;
  for (int q = 0; q < Lq; ++q) v += xr[q] * yr[q];
  out[((long)b * R + r) * S + s] = v;
}

__global__ void fill_zero_kernel(float* __restrict__ p, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = 0.f;
}

bool gag_check(int B, int idf, int cdf, int Lq, int S, const char* what) {
  if (B < 1 || idf < 1 || cdf < 1 || Lq < 1 || S < 1) {
    ee_set_error("%s: need B, idf, cdf, queryL, sourceL >= 1 (B=%d idf=%d cdf=%d queryL=%d sourceL=%d)", what, B, idf,
                 cdf, Lq, S);
    return false;
  }
  if ((long)B * Lq >= (1L << 31) || (long)B * S * Lq >= (1L << 40) || cdf > 65535 * 64 || idf > 65535) {
    ee_set_error("%s: sizes too large", what);
    return false;
  }
  return true;
}

}  // namespace

extern "C" {

long eegan_gag_fwd_workspace(int B, int queryL) { return (long)B * queryL * (long)sizeof(float2); }

int eegan_gag_fwd(const float* input, const float* context_key, const float* content_value, const unsigned char* mask,
                  int B, int idf, int cdf, int queryL, int sourceL, float* weighted_context, float* attn, void* ws,
                  hipStream_t s) {
  if (!gag_check(B, idf, cdf, queryL, sourceL, "gag_fwd")) return -22;
  const dim3 grid((queryL + GQ - 1) / GQ, B);
  float2* stats = static_cast<float2*>(ws);
  ee_launch(gag_stats_kernel, grid, dim3(256), 0, s, input, context_key, (const uint8_t*)mask, B, idf, queryL,
            sourceL, stats);
  int rc = ee_check_launch("gag_fwd(stats)");
  if (rc) return rc;
  ee_launch(gag_ctx_kernel, dim3(grid.x, B, (cdf + 63) / 64), dim3(256), 0, s, input, context_key, content_value,
            (const uint8_t*)mask, (const float2*)stats, B, idf, cdf, queryL, sourceL, weighted_context, attn);
  return ee_check_launch("gag_fwd(ctx)");
}

long eegan_gag_workspace(int B, int idf, int cdf, int queryL, int sourceL) {
  return (long)B * sourceL * queryL * (long)sizeof(float);
}

int eegan_gag_bwd(const float* input, const float* context_key, const float* content_value, const float* attn,
                  const float* d_weighted_context, const float* d_attn, int B, int idf, int cdf, int queryL,
                  int sourceL, float* d_input, float* d_key, float* d_value, void* ws, hipStream_t s) {
  if (!gag_check(B, idf, cdf, queryL, sourceL, "gag_bwd")) return -22;
  float* dl = static_cast<float*>(ws);
  ee_launch(gag_bwd_dl_kernel, dim3((queryL + GQ - 1) / GQ, B), dim3(256), 0, s, content_value, attn,
            d_weighted_context, d_attn, cdf, queryL, sourceL, dl);
  int rc = ee_check_launch("gag_bwd(dl)");
  if (rc) return rc;
  ee_launch(gag_bwd_din_kernel, dim3((queryL + 255) / 256, idf, B), dim3(256), 0, s, context_key, (const float*)dl,
            idf, queryL, sourceL, d_input);
  if ((rc = ee_check_launch("gag_bwd(dinput)"))) return rc;
  ee_launch(gag_bwd_rowdot_kernel, dim3((sourceL + 255) / 256, idf, B), dim3(256), 0, s, input, (const float*)dl, idf,
            queryL, sourceL, d_key);
  if ((rc = ee_check_launch("gag_bwd(dkey)"))) return rc;
  if (d_weighted_context != nullptr) {
    ee_launch(gag_bwd_rowdot_kernel, dim3((sourceL + 255) / 256, cdf, B), dim3(256), 0, s, d_weighted_context, attn,
              cdf, queryL, sourceL, d_value);
  } else {
    const long n = (long)B * cdf * sourceL;
    ee_launch(fill_zero_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d_value, n);
  }
  return ee_check_launch("gag_bwd(dvalue)");
}

}  // extern "C"
