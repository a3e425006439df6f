// DAMSM word-level matching on bf16 MFMA: the (image j, caption i) similarity
// of words_loss for n_img (this rank's) images x n_txt (all ranks') captions,
// and its backward.
//
// replaces miscc/DAMSM_losses.py:17-23 (cosine_similarity), 25-63
// (func_attention) and the per-caption loop of 272-331 (words_loss); the
// masked bidirectional cross-entropy stays in loss.hip (sim_ce).
//
// Per pair (one workgroup, 8 waves), with ctx = regions of image j
// (289 x 256) and q = words of caption i (w <= 32 valid of T):
//   S  = ctx q^T           (289 x w)    MFMA, split-bf16 (hi*hi + lo*hi + hi*lo:
//                                        the logits feed a sharp softmax, so they
//                                        are kept near fp32; 3 MFMAs per tile)
//   A1 = softmax_words(S)   A2 = softmax_regions(gamma1 A1^T)   (fp32, in registers / LDS)
//   C  = A2 ctx             (w x 256)    MFMA bf16 (A2 staged in LDS)
//   sim[j][i] = gamma3 log sum_k exp(gamma2 cos(q_k, C_k))
// Backward recomputes the pair, then forms dC, dA2 = dC ctx^T (MFMA), the two
// softmax backwards, and writes per-pair factors U = [A2^T | dS] (289 x 64) and
// V = [dC ; q] (64 x 256); dregions_j = sum_i U_ij V_ij is a separate MFMA GEMM
// over K = 64 * n_txt (fixed order: deterministic, no atomics).  dwords (only
// when the words require a gradient) = sum_j (dS_ij^T ctx_j + d cos terms) via
// per-pair fp32 partials reduced in fixed order.
//
// Operand layouts are prepared once per call (eegan_words_* prep kernels):
// ctx hi / lo [n_img][304][256] (regions x dims, rows >= 289 zero), ctx^T
// [n_img][256][320] (dims x regions, zero padded), q hi / lo [n_txt][32][256]
// (zero past the caption's length), q^T [n_txt][256][32].  Every MFMA fragment
// is then one 16-byte load.
#include "common.h"
#include "../../include/eegan_hip.h"

namespace {

constexpr float G1 = 5.f, G2 = 5.f, G3 = 10.f;  // cfg.TRAIN.SMOOTH.GAMMA1/2/3 (miscc/config.py:47-49)
constexpr int NR = 289;    // 17 x 17 regions
constexpr int NRP = 304;   // regions padded to 19 MFMA tiles
constexpr int NRK = 320;   // regions padded to 10 K-steps of 32
constexpr int ND = 256;    // embedding dim
constexpr int NW = 32;     // words per caption (padded; cfg.TEXT.WORDS_NUM = 20)
constexpr int QLD = ND + 8;    // bf16 row stride of q / dC in LDS (conflict-free b128 row reads)
constexpr int A2LD = NRK + 8;  // bf16 row stride of A2 / dS^T in LDS
constexpr int A1LD = NW + 4;   // fp32 row stride of A1 in LDS (16-byte aligned rows)
constexpr int NWV = 8;         // waves per pair workgroup (latency: more waves, shorter per-wave chains)
constexpr int PT = NWV * 64;   // threads per pair workgroup
constexpr int MS = (NRP / 16 + NWV - 1) / NWV;  // region tiles per wave (19 tiles)
constexpr int DT = (ND / 16) / NWV;             // 16-dim tiles per wave (16 tiles)

EE_DEV bf16x8_t frag(const bf16_t* p) { return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(p)); }
EE_DEV f32x4_t mfma(bf16x8_t a, bf16x8_t b, f32x4_t c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
EE_DEV float xsum16(float v) {  // sum over the 16 lanes sharing lane>>4
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}
EE_DEV float xmax16(float v) {
  v = fmaxf(v, __shfl_xor(v, 1, 64));
  v = fmaxf(v, __shfl_xor(v, 2, 64));
  v = fmaxf(v, __shfl_xor(v, 4, 64));
  v = fmaxf(v, __shfl_xor(v, 8, 64));
  return v;
}
EE_DEV float xsum_groups(float v) {  // sum over the 4 lane groups (same lane & 15)
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

struct Ws {  // workspace carve-up (byte offsets), see eegan_words_workspace
  long ctxh, ctxl, ctxT, qh, ql, qT, U, V, dq, total;
};
Ws ws_layout(int n_img, int n_txt, int bwd, int dwords) {
  Ws w;
  long o = 0;
  auto take = [&](long bytes) {
    const long r = o;
    o += (bytes + 255) / 256 * 256;
    return r;
  };
  w.ctxh = take((long)n_img * NRP * ND * 2);
  w.ctxl = take((long)n_img * NRP * ND * 2);
  w.ctxT = take((long)n_img * ND * NRK * 2);
  w.qh = take((long)n_txt * NW * ND * 2);
  w.ql = take((long)n_txt * NW * ND * 2);
  w.qT = take((long)n_txt * ND * NW * 2);
  w.U = bwd ? take((long)n_img * n_txt * NRP * 64 * 2) : 0;
  w.V = bwd ? take((long)n_img * n_txt * ND * NW * 2) : 0;
  w.dq = (bwd && dwords) ? take((long)n_img * n_txt * ND * NW * 4) : 0;
  w.total = o;
  return w;
}

struct WordsArgs {
  const float* words;   // [n_txt][256][T] fp32 (RNN_ENCODER layout)
  const long* lens;     // [n_txt]
  int n_img, n_txt, T, diag_off;
  const bf16_t *ctxh, *ctxl, *ctxT, *qh, *ql;
  float* sim;           // fwd: [n_img][n_txt], gamma3 * log-sum-exp (unmasked)
  float* att;           // fwd: A2 of pairs (j, j + diag_off): [n_img][T][289] fp32, or null
  const float* dsim;    // bwd: d loss / d sim [n_img][n_txt]
  bf16_t* U;            // bwd: [pair][304][64]  = [A2^T | dS]
  bf16_t* V;            // bwd: [pair][256][32]  = dC^T
  float* dq;            // bwd, dwords only: [i][j][256][32]
};

// ----------------------------------------------------------------- prep --
// regions fp32 [n_img][289][256] -> ctx hi/lo [n_img][304][256], ctx^T [n_img][256][320]
EE_DEV void prep_q(const float* __restrict__ words, const long* lens, int T, bf16_t* qh, bf16_t* ql, bf16_t* qT,
                   int i, int d, float (*stage)[NW + 1]);

constexpr int PREP_ROWS = 16;  // region rows per workgroup: n_img * 20 + n_txt workgroups

// one launch prepares both operands: workgroups [0, n_img * NRK / 16) the
// regions (16 region rows each), the rest one caption each
__global__ __launch_bounds__(256) void words_prep_kernel(const float* __restrict__ reg, bf16_t* ctxh, bf16_t* ctxl,
                                                         bf16_t* ctxT, int n_img, const float* __restrict__ words,
                                                         const long* lens, int T, bf16_t* qh, bf16_t* ql, bf16_t* qT) {
  __shared__ float tile[ND * (NW + 1)];  // regions: [16][ND + 4]; captions: [ND][NW + 1]
  constexpr int RB = NRK / PREP_ROWS;
  if ((int)blockIdx.x >= n_img * RB) {
    prep_q(words, lens, T, qh, ql, qT, blockIdx.x - n_img * RB, threadIdx.x,
           reinterpret_cast<float(*)[NW + 1]>(tile));
    return;
  }
  float(*rt)[ND + 4] = reinterpret_cast<float(*)[ND + 4]>(tile);
  const int j = blockIdx.x / RB, r0 = (blockIdx.x % RB) * PREP_ROWS, t = threadIdx.x;
  for (int e = t; e < PREP_ROWS * (ND / 4); e += 256) {
    const int row = e / (ND / 4), d = (e % (ND / 4)) * 4, r = r0 + row;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < NR) v = *reinterpret_cast<const float4*>(reg + ((long)j * NR + r) * ND + d);
    rt[row][d] = v.x;
    rt[row][d + 1] = v.y;
    rt[row][d + 2] = v.z;
    rt[row][d + 3] = v.w;
    if (r < NRP) {
      const float f[4] = {v.x, v.y, v.z, v.w};
      uint32_t h[2], lo[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const bf16_t h0 = f2bf(f[2 * q]), h1 = f2bf(f[2 * q + 1]);
        h[q] = (uint32_t)h0 | ((uint32_t)h1 << 16);
        lo[q] = pack2(f[2 * q] - bf2f(h0), f[2 * q + 1] - bf2f(h1));
      }
      const long o = ((long)j * NRP + r) * ND + d;
      *reinterpret_cast<uint2*>(ctxh + o) = make_uint2(h[0], h[1]);
      *reinterpret_cast<uint2*>(ctxl + o) = make_uint2(lo[0], lo[1]);
    }
  }
  __syncthreads();
  const int d = t;  // 256 threads = 256 dims: 16 regions -> 32 contiguous bytes of ctx^T
  uint32_t p[PREP_ROWS / 2];
#pragma unroll
  for (int c = 0; c < PREP_ROWS / 2; ++c) p[c] = pack2(rt[2 * c][d], rt[2 * c + 1][d]);
  uint4* dst = reinterpret_cast<uint4*>(ctxT + ((long)j * ND + d) * NRK + r0);
#pragma unroll
  for (int c = 0; c < PREP_ROWS / 8; ++c) dst[c] = make_uint4(p[4 * c], p[4 * c + 1], p[4 * c + 2], p[4 * c + 3]);
}

// words fp32 [n_txt][256][T] -> q hi/lo [n_txt][32][256], q^T (hi) [n_txt][256][32]
EE_DEV void prep_q(const float* __restrict__ words, const long* lens, int T, bf16_t* qh, bf16_t* ql, bf16_t* qT,
                   int i, int d, float (*stage)[NW + 1]) {
  const int w = max(1, min((int)lens[i], min(T, NW)));
  // the caption's [256][T] block is contiguous: stage it coalesced
  for (int e = d; e < ND * T; e += 256) stage[e / T][e % T] = words[(long)i * ND * T + e];
  __syncthreads();
  uint32_t p[16];
#pragma unroll
  for (int k2 = 0; k2 < 16; ++k2) {
    bf16_t hh[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k = 2 * k2 + u;
      const float v = k < w ? stage[d][k] : 0.f;
      hh[u] = f2bf(v);
      qh[((long)i * NW + k) * ND + d] = hh[u];
      ql[((long)i * NW + k) * ND + d] = f2bf(v - bf2f(hh[u]));
    }
    p[k2] = (uint32_t)hh[0] | ((uint32_t)hh[1] << 16);
  }
  uint4* dst = reinterpret_cast<uint4*>(qT + ((long)i * ND + d) * NW);
#pragma unroll
  for (int c = 0; c < 4; ++c) dst[c] = make_uint4(p[4 * c], p[4 * c + 1], p[4 * c + 2], p[4 * c + 3]);
}

// ---------------------------------------------------------------- pairs --
struct SmemF {   // forward part (also the first part of the backward's)
  bf16_t qh[NW][QLD], ql[NW][QLD];
  bf16_t a2[NW][A2LD];                  // A2 [k][r] (phase 2 operand); bwd: dS^T [k][r]
  float colsum[NWV][NW], colinv[NW];
  float cred[NWV][NW][3], red2[NWV][NW];
  float cs[NW], nq[NW], nc[NW];
};
struct SmemB {
  SmemF f;
  float a1[NRP][A1LD];                  // A1 [r][k] fp32
  bf16_t dc[NW][QLD];                   // dC [k][d]
};

template <bool BWD>
__global__ __launch_bounds__(PT) void words_pair_kernel(WordsArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  SmemF& sm = *reinterpret_cast<SmemF*>(smem_raw);
  SmemB& sb = *reinterpret_cast<SmemB*>(smem_raw);
  const int i = blockIdx.x, j = blockIdx.y;  // caption i (of n_txt), image j (of n_img)
  const long pair = (long)j * a.n_txt + i;
  const int t = threadIdx.x, l = t & 63, wv = t >> 6;
  const int fr = l & 15, fq = l >> 4;
  const int w = max(1, min((int)a.lens[i], min(a.T, NW)));  // words[i, :, :w] (DAMSM_losses.py:288)
  const int nn = w > 16 ? 2 : 1;                             // 16-word tiles in use

  // ---- stage caption i (hi / lo) into LDS; zero the K padding of A2 / dS^T
  {
    const uint4* sh = reinterpret_cast<const uint4*>(a.qh + (long)i * NW * ND);
    const uint4* sl = reinterpret_cast<const uint4*>(a.ql + (long)i * NW * ND);
    for (int e = t; e < NW * ND / 8; e += PT) {
      const int k = e / (ND / 8), c = (e % (ND / 8)) * 8;
      *reinterpret_cast<uint4*>(&sm.qh[k][c]) = sh[e];
      *reinterpret_cast<uint4*>(&sm.ql[k][c]) = sl[e];
    }
    for (int e = t; e < NW * (NRK - NRP) / 2; e += PT)
      *reinterpret_cast<uint32_t*>(&sm.a2[e / 8][NRP + (e % 8) * 2]) = 0u;
  }
  __syncthreads();

  // ---- phase 1: S = ctx q^T (split bf16), softmax over words, exp(gamma1 A1)
  const bf16_t* ch = a.ctxh + (long)j * NRP * ND;
  const bf16_t* cl = a.ctxl + (long)j * NRP * ND;
  f32x4_t ev[MS][2];
  float colp[2] = {0.f, 0.f};
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    const int mt = wv + NWV * s;
    ev[s][0] = ev[s][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (mt >= NRP / 16) break;  // wave-uniform
    f32x4_t acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const bf16_t* ah_p = ch + (mt * 16 + fr) * ND + fq * 8;
    const bf16_t* al_p = cl + (mt * 16 + fr) * ND + fq * 8;
#pragma unroll
    for (int kk = 0; kk < ND / 32; ++kk) {
      const bf16x8_t ah = frag(ah_p + kk * 32), al = frag(al_p + kk * 32);
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        if (n >= nn) break;
        const bf16x8_t bh = frag(&sm.qh[n * 16 + fr][kk * 32 + fq * 8]);
        const bf16x8_t bl = frag(&sm.ql[n * 16 + fr][kk * 32 + fq * 8]);
        acc[n] = mfma(ah, bh, acc[n]);
        acc[n] = mfma(al, bh, acc[n]);
        acc[n] = mfma(ah, bl, acc[n]);
      }
    }
    const bool v0 = fr < w, v1 = nn > 1 && 16 + fr < w;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = mt * 16 + fq * 4 + r;
      // softmax over the caption's words (DAMSM_losses.py:42-45)
      const float m = xmax16(fmaxf(v0 ? acc[0][r] : -INFINITY, v1 ? acc[1][r] : -INFINITY));
      const float e0 = v0 ? __expf(acc[0][r] - m) : 0.f, e1 = v1 ? __expf(acc[1][r] - m) : 0.f;
      const float inv = 1.f / xsum16(e0 + e1);
      const float a10 = e0 * inv, a11 = e1 * inv;
      if (BWD) {
        sb.a1[row][fr] = a10;
        sb.a1[row][16 + fr] = a11;
      }
      // x gamma1, softmax over the regions (DAMSM_losses.py:52-54): A1 <= 1,
      // so exp(gamma1 A1) <= e^5 needs no max shift
      const bool rv = row < NR;
      ev[s][0][r] = (rv && v0) ? __expf(G1 * a10) : 0.f;
      ev[s][1][r] = (rv && v1) ? __expf(G1 * a11) : 0.f;
      colp[0] += ev[s][0][r];
      colp[1] += ev[s][1][r];
    }
  }
  colp[0] = xsum_groups(colp[0]);
  colp[1] = xsum_groups(colp[1]);
  if (fq == 0) {
    sm.colsum[wv][fr] = colp[0];
    sm.colsum[wv][16 + fr] = colp[1];
  }
  __syncthreads();
  if (t < NW) {
    float c = 0.f;
#pragma unroll
    for (int x = 0; x < NWV; ++x) c += sm.colsum[x][t];
    sm.colinv[t] = c > 0.f ? 1.f / c : 0.f;
  }
  __syncthreads();
  {
    const float inv0 = sm.colinv[fr], inv1 = sm.colinv[16 + fr];
    const bool want_att = !BWD && a.att && i == j + a.diag_off;
#pragma unroll
    for (int s = 0; s < MS; ++s) {
      const int mt = wv + NWV * s;
      if (mt >= NRP / 16) break;
      const int row0 = mt * 16 + fq * 4;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const float inv = n ? inv1 : inv0;
        const float p0 = ev[s][n][0] * inv, p1 = ev[s][n][1] * inv, p2 = ev[s][n][2] * inv, p3 = ev[s][n][3] * inv;
        *reinterpret_cast<uint2*>(&sm.a2[n * 16 + fr][row0]) = make_uint2(pack2(p0, p1), pack2(p2, p3));
        const int k = n * 16 + fr;
        if (want_att && k < w) {
          float* dst = a.att + ((long)j * a.T + k) * NR;
          const float pv[4] = {p0, p1, p2, p3};
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (row0 + r < NR) dst[row0 + r] = pv[r];
        }
      }
    }
  }
  __syncthreads();

  // ---- phase 2: C[k][d] = sum_r A2[k][r] ctx[r][d]  (wave: 64 dims)
  const bf16_t* cT = a.ctxT + (long)j * ND * NRK;
  f32x4_t cacc[2][DT];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < DT; ++n) cacc[m][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
  for (int kk = 0; kk < NRK / 32; ++kk) {
    bf16x8_t am[2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
      if (m < nn) am[m] = frag(&sm.a2[m * 16 + fr][kk * 32 + fq * 8]);
#pragma unroll
    for (int n = 0; n < DT; ++n) {
      const bf16x8_t b = frag(cT + ((wv * DT + n) * 16 + fr) * NRK + kk * 32 + fq * 8);
#pragma unroll
      for (int m = 0; m < 2; ++m)
        if (m < nn) cacc[m][n] = mfma(am[m], b, cacc[m][n]);
    }
  }

  // ---- phase 3: cosine(q_k, C_k) over the 256 dims (DAMSM_losses.py:17-23)
  float qv[2][DT][4];
  {
    float dp[2][4], c2[2][4], q2[2][4];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dp[m][r] = c2[m][r] = q2[m][r] = 0.f;
        const int k = m * 16 + fq * 4 + r;
#pragma unroll
        for (int n = 0; n < DT; ++n) {
          const int d = (wv * DT + n) * 16 + fr;
          const float q = (m < nn && k < w) ? a.words[((long)i * ND + d) * a.T + k] : 0.f;
          const float c = m < nn ? cacc[m][n][r] : 0.f;
          qv[m][n][r] = q;
          dp[m][r] += q * c;
          c2[m][r] += c * c;
          q2[m][r] += q * q;
        }
        dp[m][r] = xsum16(dp[m][r]);
        c2[m][r] = xsum16(c2[m][r]);
        q2[m][r] = xsum16(q2[m][r]);
        if (fr == 0) {
          sm.cred[wv][k][0] = dp[m][r];
          sm.cred[wv][k][1] = q2[m][r];
          sm.cred[wv][k][2] = c2[m][r];
        }
      }
  }
  __syncthreads();
  if (t < NW) {
    float u = 0.f, q2 = 0.f, c2 = 0.f;
#pragma unroll
    for (int x = 0; x < NWV; ++x) {
      u += sm.cred[x][t][0];
      q2 += sm.cred[x][t][1];
      c2 += sm.cred[x][t][2];
    }
    sm.nq[t] = sqrtf(q2);
    sm.nc[t] = sqrtf(c2);
    sm.cs[t] = u / fmaxf(sm.nq[t] * sm.nc[t], 1e-8f);
  }
  __syncthreads();
  // row similarity = log sum_k exp(gamma2 cos_k)   (DAMSM_losses.py:315-317)
  float se = 0.f;
  for (int k = 0; k < w; ++k) se += __expf(G2 * sm.cs[k]);
  if (!BWD) {
    if (t == 0) a.sim[pair] = G3 * logf(se);
    return;
  }

  // ================================ backward ================================
  const float drow = G3 * a.dsim[pair];
  float dqc[2][DT][4];  // d loss / d q through the cosine, phase-2 layout
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = m * 16 + fq * 4 + r;
      float dcos = 0.f, cs = 0.f, nq = 1.f, nc = 1.f;
      if (m < nn && k < w) {
        cs = sm.cs[k];
        nq = sm.nq[k];
        nc = sm.nc[k];
        dcos = drow * G2 * __expf(G2 * cs) / se;
      }
      const float den = nq * nc;
#pragma unroll
      for (int n = 0; n < DT; ++n) {
        const float q = qv[m][n][r], c = m < nn ? cacc[m][n][r] : 0.f;
        float dC, dq;
        if (den > 1e-8f) {
          dC = dcos * (q / den - cs * c / (nc * nc));
          dq = dcos * (c / den - cs * q / (nq * nq));
        } else {
          dC = dcos * q / 1e-8f;
          dq = dcos * c / 1e-8f;
        }
        dqc[m][n][r] = dq;
        cacc[m][n][r] = dC;  // the accumulator now holds dC
        sb.dc[k][(wv * DT + n) * 16 + fr] = f2bf(dC);
      }
    }
  // V factor: dC^T [d][k] (4 consecutive words of one dim per lane)
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < DT; ++n) {
      const int d = (wv * DT + n) * 16 + fr;
      *reinterpret_cast<uint2*>(a.V + (pair * ND + d) * NW + m * 16 + fq * 4) =
          make_uint2(pack2(cacc[m][n][0], cacc[m][n][1]), pack2(cacc[m][n][2], cacc[m][n][3]));
    }
  __syncthreads();

  // ---- phase 4: dA2[k][r] = sum_d dC[k][d] ctx[r][d]  (wave: region tiles wv, wv+4, ...)
  f32x4_t da[MS][2];
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    da[s][0] = da[s][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int nt = wv + NWV * s;
    if (nt >= NRP / 16) break;
    const bf16_t* bp = ch + (nt * 16 + fr) * ND + fq * 8;
#pragma unroll
    for (int kk = 0; kk < ND / 32; ++kk) {
      const bf16x8_t b = frag(bp + kk * 32);
#pragma unroll
      for (int m = 0; m < 2; ++m)
        if (m < nn) da[s][m] = mfma(frag(&sb.dc[m * 16 + fr][kk * 32 + fq * 8]), b, da[s][m]);
    }
  }
  // softmax-over-regions backward: dZ = A2 (dA2 - <A2, dA2>_r); dA1 = gamma1 dZ^T
  float rd[2][4];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) rd[m][r] = 0.f;
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    const int nt = wv + NWV * s;
    if (nt >= NRP / 16) break;
    const int row = nt * 16 + fr;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int k0 = m * 16 + fq * 4;
      const float4 a1v = *reinterpret_cast<const float4*>(&sb.a1[row][k0]);
      const float a1s[4] = {a1v.x, a1v.y, a1v.z, a1v.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = k0 + r;
        const float a2 = (row < NR && m < nn && k < w) ? __expf(G1 * a1s[r]) * sm.colinv[k] : 0.f;
        rd[m][r] += a2 * da[s][m][r];
      }
    }
  }
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = xsum16(rd[m][r]);
      if (fr == 0) sm.red2[wv][m * 16 + fq * 4 + r] = v;
    }
  __syncthreads();
  // dS = A1 (dA1 - <A1, dA1>_k) per region; U factor = [A2^T | dS]; dS^T to LDS for dwords
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    const int nt = wv + NWV * s;
    if (nt >= NRP / 16) break;
    const int row = nt * 16 + fr;
    float a2v[2][4], a1v[2][4], dA1[2][4];
    float rs = 0.f;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int k0 = m * 16 + fq * 4;
      const float4 q4 = *reinterpret_cast<const float4*>(&sb.a1[row][k0]);
      const float a1s[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = k0 + r;
        const bool ok = row < NR && m < nn && k < w;
        const float a2 = ok ? __expf(G1 * a1s[r]) * sm.colinv[k] : 0.f;
        float rdot = 0.f;
#pragma unroll
        for (int x = 0; x < NWV; ++x) rdot += sm.red2[x][k];
        a2v[m][r] = a2;
        a1v[m][r] = ok ? a1s[r] : 0.f;
        dA1[m][r] = ok ? G1 * a2 * (da[s][m][r] - rdot) : 0.f;
        rs += a1v[m][r] * dA1[m][r];
      }
    }
    rs = xsum_groups(rs);
    bf16_t* u = a.U + (pair * NRP + row) * 64;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      float dS[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) dS[r] = a1v[m][r] * (dA1[m][r] - rs);
      const int k0 = m * 16 + fq * 4;
      *reinterpret_cast<uint2*>(u + k0) = make_uint2(pack2(a2v[m][0], a2v[m][1]), pack2(a2v[m][2], a2v[m][3]));
      *reinterpret_cast<uint2*>(u + 32 + k0) = make_uint2(pack2(dS[0], dS[1]), pack2(dS[2], dS[3]));
      if (a.dq) {
#pragma unroll
        for (int r = 0; r < 4; ++r) sm.a2[k0 + r][row] = f2bf(dS[r]);  // dS^T (phase 2 is done with A2)
      }
    }
  }
  if (!a.dq) return;
  __syncthreads();
  // ---- dwords: dq[k][d] = sum_r dS[r][k] ctx[r][d] + d cos / d q   (phase-2 layout)
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < DT; ++n) cacc[m][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
  for (int kk = 0; kk < NRK / 32; ++kk) {
    bf16x8_t am[2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
      if (m < nn) am[m] = frag(&sm.a2[m * 16 + fr][kk * 32 + fq * 8]);
#pragma unroll
    for (int n = 0; n < DT; ++n) {
      const bf16x8_t b = frag(cT + ((wv * DT + n) * 16 + fr) * NRK + kk * 32 + fq * 8);
#pragma unroll
      for (int m = 0; m < 2; ++m)
        if (m < nn) cacc[m][n] = mfma(am[m], b, cacc[m][n]);
    }
  }
  float* dq = a.dq + ((long)i * a.n_img + j) * ND * NW;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < DT; ++n) {
      const int d = (wv * DT + n) * 16 + fr;
      f32x4_t v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = m < nn ? cacc[m][n][r] + dqc[m][n][r] : 0.f;
      *reinterpret_cast<f32x4_t*>(dq + (long)d * NW + m * 16 + fq * 4) = v;
    }
}

// dregions[j][r][d] = sum_i sum_c U[j,i][r][c] V'[j,i][c][d],  V' = [dC ; q] (K = 64 per caption).
// Workgroup = 64 regions x 64 dims; each of its 4 waves accumulates the whole
// 64 x 64 tile (16 MFMA tiles: 8 fragment loads per 16 MFMAs) over captions
// i = wave, wave + 4, ..., and the four partial tiles are added in a fixed
// order through LDS (deterministic; no atomics).
__global__ __launch_bounds__(256) void words_dctx_kernel(const bf16_t* __restrict__ U, const bf16_t* __restrict__ V,
                                                         const bf16_t* __restrict__ qT, int n_txt,
                                                         float* __restrict__ dreg) {
  __shared__ float red[3][64][64 + 4];
  const int t = threadIdx.x, l = t & 63, wv = t >> 6, fr = l & 15, fq = l >> 4;
  const int j = blockIdx.z;
  const int r0 = blockIdx.y * 64, d0 = blockIdx.x * 64;
  f32x4_t acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bool rok[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) rok[m] = r0 + m * 16 + fr < NRP;
  const bf16x8_t zero = __builtin_bit_cast(bf16x8_t, make_uint4(0u, 0u, 0u, 0u));
  for (int i = wv; i < n_txt; i += 4) {
    const long pair = (long)j * n_txt + i;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      bf16x8_t am[4], bn[4];
#pragma unroll
      for (int m = 0; m < 4; ++m)
        am[m] = rok[m] ? frag(U + (pair * NRP + r0 + m * 16 + fr) * 64 + c * 32 + fq * 8) : zero;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int d = d0 + n * 16 + fr;
        bn[n] = c == 0 ? frag(V + (pair * ND + d) * NW + fq * 8) : frag(qT + ((long)i * ND + d) * NW + fq * 8);
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = mfma(am[m], bn[n], acc[m][n]);
    }
  }
  if (wv > 0) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wv - 1][m * 16 + fq * 4 + r][n * 16 + fr] = acc[m][n][r];
  }
  __syncthreads();
  if (wv != 0) return;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m * 16 + fq * 4 + r, col = n * 16 + fr;
        float v = acc[m][n][r];
        v += red[0][row][col];
        v += red[1][row][col];
        v += red[2][row][col];
        if (r0 + row < NR) dreg[((long)j * NR + r0 + row) * ND + d0 + col] = v;
      }
}

// dwords[i][d][k] = sum_j dq[i][j][d][k]  (fixed order over j)
__global__ void words_dq_reduce_kernel(const float* __restrict__ dq, int n_img, int T, float* __restrict__ dwords) {
  const int i = blockIdx.x;
  for (int e = threadIdx.x; e < ND * T; e += blockDim.x) {
    const int d = e / T, k = e % T;
    float s = 0.f;
    if (k < NW)
      for (int j = 0; j < n_img; ++j) s += dq[(((long)i * n_img + j) * ND + d) * NW + k];
    dwords[((long)i * ND + d) * T + k] = s;
  }
}

int prep(const float* regions, const float* words, const long* lens, int n_img, int n_txt, int T, const Ws& L,
         char* ws, hipStream_t s) {
  ee_launch(words_prep_kernel, dim3(n_img * (NRK / PREP_ROWS) + n_txt), dim3(256), 0, s, regions, (bf16_t*)(ws + L.ctxh),
            (bf16_t*)(ws + L.ctxl), (bf16_t*)(ws + L.ctxT), n_img, words, lens, T, (bf16_t*)(ws + L.qh),
            (bf16_t*)(ws + L.ql), (bf16_t*)(ws + L.qT));
  return ee_check_launch("words_prep");
}

WordsArgs make_args(const float* words, const long* lens, int n_img, int n_txt, int T, const Ws& L, char* ws) {
  WordsArgs a = {};
  a.words = words;
  a.lens = lens;
  a.n_img = n_img;
  a.n_txt = n_txt;
  a.T = T;
  a.ctxh = (const bf16_t*)(ws + L.ctxh);
  a.ctxl = (const bf16_t*)(ws + L.ctxl);
  a.ctxT = (const bf16_t*)(ws + L.ctxT);
  a.qh = (const bf16_t*)(ws + L.qh);
  a.ql = (const bf16_t*)(ws + L.ql);
  return a;
}

bool check(const void* regions, int n_img, int n_txt, int T, const char* what) {
  if (T < 1 || T > NW || n_img < 1 || n_txt < 1) {
    ee_set_error("%s: need 1 <= T <= %d and non-empty batches (T=%d, n_img=%d, n_txt=%d)", what, NW, T, n_img, n_txt);
    return false;
  }
  if ((uintptr_t)regions & 15) {
    ee_set_error("%s: regions must be 16-byte aligned fp32 [n_img][289][256]", what);
    return false;
  }
  return true;
}

}  // namespace

extern "C" {

long eegan_words_workspace(int n_img, int n_txt, int backward, int want_dwords) {
  return ws_layout(n_img, n_txt, backward, want_dwords).total;
}

int eegan_words_sim(const float* regions, const float* words, const long* cap_lens, int n_img, int n_txt, int T,
                    int diag_off, float* sim, float* att, void* ws, hipStream_t s) {
  if (!check(regions, n_img, n_txt, T, "words_sim")) return -22;
  const Ws L = ws_layout(n_img, n_txt, 0, 0);
  char* w = static_cast<char*>(ws);
  int rc = prep(regions, words, cap_lens, n_img, n_txt, T, L, w, s);
  if (rc) return rc;
  WordsArgs a = make_args(words, cap_lens, n_img, n_txt, T, L, w);
  a.sim = sim;
  a.att = att;
  a.diag_off = diag_off;
  ee_launch(words_pair_kernel<false>, dim3(n_txt, n_img), dim3(PT), (uint32_t)sizeof(SmemF), s, a);
  return ee_check_launch("words_sim");
}

int eegan_words_sim_bwd(const float* regions, const float* words, const long* cap_lens, int n_img, int n_txt, int T,
                        const float* dsim, float* dregions, float* dwords, void* ws, int prepared, hipStream_t s) {
  if (!check(regions, n_img, n_txt, T, "words_sim_bwd")) return -22;
  const Ws L = ws_layout(n_img, n_txt, 1, dwords != nullptr);
  char* w = static_cast<char*>(ws);
  int rc = prepared ? 0 : prep(regions, words, cap_lens, n_img, n_txt, T, L, w, s);
  if (rc) return rc;
  WordsArgs a = make_args(words, cap_lens, n_img, n_txt, T, L, w);
  a.dsim = dsim;
  a.U = (bf16_t*)(w + L.U);
  a.V = (bf16_t*)(w + L.V);
  a.dq = dwords ? (float*)(w + L.dq) : nullptr;
  ee_launch(words_pair_kernel<true>, dim3(n_txt, n_img), dim3(PT), (uint32_t)sizeof(SmemB), s, a);
  rc = ee_check_launch("words_sim_bwd");
  if (rc) return rc;
  ee_launch(words_dctx_kernel, dim3(ND / 64, (NRP + 63) / 64, n_img), dim3(256), 0, s, (const bf16_t*)a.U,
            (const bf16_t*)a.V, (const bf16_t*)(w + L.qT), n_txt, dregions);
  rc = ee_check_launch("words_dctx");
  if (rc || !dwords) return rc;
  ee_launch(words_dq_reduce_kernel, dim3(n_txt), dim3(256), 0, s, (const float*)a.dq, n_img, T, dwords);
  return ee_check_launch("words_dq_reduce");
}

}  // extern "C"
