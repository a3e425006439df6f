// Loss-side kernels: DAMSM sentence similarity (the word-level similarity is
// in damsm.hip), cross-entropy over the similarity matrices, hinge/mean reductions of the
// discriminator outputs, BCE-with-logits, the MA gradient penalty, class
// one-hot labels and the ATTR_Enhance 4x4 self-attention core.
//
// replaces: miscc/DAMSM_losses.py:17-63 (cosine_similarity, func_attention),
// 233-342 (sent_loss, words_loss); train.py:99-103 (prepare_class_labels),
// 336-417 (d_loss / d_loss_class / MA_gradient_penalty tail / g_loss[_class]);
// models.py:155-180 (ATTR_Enhance softmax(QK^T)/sqrt(d) V, attr_merge).
#include "common.h"
#include "../../include/eegan_hip.h"

namespace {

constexpr float GAMMA3 = 10.f;  // cfg.TRAIN.SMOOTH.GAMMA3

// ------------------------------------------ masked bidirectional CE ------
// sim[a][b] (rows a), mask[a][b] = cls[a]==cls[b] && a!=b  -> -inf.
// loss0 = CE(sim, arange), loss1 = CE(sim^T, arange). One block.
__global__ void sim_ce_kernel(const float* sim, int B, const long* cls, const long* lab, float* loss, const float* gl,
                              float* dsim) {
  extern __shared__ float sh[];
  float* lse_r = sh;       // [B]
  float* lse_c = sh + B;   // [B]
  __shared__ float red[16];
  auto masked = [&](int x, int y) { return cls && x != y && cls[x] == cls[y]; };
  for (int x = threadIdx.x; x < 2 * B; x += blockDim.x) {
    const bool row = x < B;
    const int idx = row ? x : x - B;
    float mx = -INFINITY;
    for (int y = 0; y < B; ++y) {
      const int a = row ? idx : y, b = row ? y : idx;
      if (!masked(a, b)) mx = fmaxf(mx, sim[(long)a * B + b]);
    }
    float s = 0.f;
    for (int y = 0; y < B; ++y) {
      const int a = row ? idx : y, b = row ? y : idx;
      if (!masked(a, b)) s += __expf(sim[(long)a * B + b] - mx);
    }
    (row ? lse_r : lse_c)[idx] = mx + logf(s);
  }
  __syncthreads();
  if (!dsim) {
    float l0 = 0.f, l1 = 0.f;
    for (int x = threadIdx.x; x < B; x += blockDim.x) {
      const long tx = lab ? lab[x] : x;
      l0 += lse_r[x] - sim[(long)x * B + tx];
      l1 += lse_c[x] - sim[tx * B + x];
    }
    l0 = block_sum(l0, red);
    l1 = block_sum(l1, red);
    if (threadIdx.x == 0) {
      loss[0] = l0 / B;
      loss[1] = l1 / B;
    }
  } else {
    const float g0 = gl[0] / B, g1 = gl[1] / B;
    for (int e = threadIdx.x; e < B * B; e += blockDim.x) {
      const int a = e / B, b = e % B;
      float g = 0.f;
      if (!masked(a, b)) {
        const float v = sim[e];
        g = g0 * __expf(v - lse_r[a]) + g1 * __expf(v - lse_c[b]);
      }
      if (b == (lab ? lab[a] : a)) g -= g0;
      if (a == (lab ? lab[b] : b)) g -= g1;
      dsim[e] = g;
    }
  }
}

// ------------------------------------------------------------ sent loss --
// cos[a][b] * gamma3 with norms clamped as in sent_loss (DAMSM_losses.py:253-258)
__global__ void sent_sim_kernel(const float* cnn, const float* rnn, int NB, int D, float* sim) {
  const int a = blockIdx.x;
  for (int b = threadIdx.x; b < NB; b += blockDim.x) {
    float u = 0.f, n1 = 0.f, n2 = 0.f;
    for (int k = 0; k < D; ++k) {
      const float x = cnn[(long)a * D + k], y = rnn[(long)b * D + k];
      u += x * y;
      n1 += x * x;
      n2 += y * y;
    }
    sim[(long)a * NB + b] = u / fmaxf(sqrtf(n1) * sqrtf(n2), 1e-8f) * GAMMA3;
  }
}

// norms of the rows of cnn (b < NA) and rnn (NA <= b < NA + NB): nrm[b]
__global__ void row_norm_kernel(const float* cnn, const float* rnn, int NA, int D, float* nrm) {
  const int b0 = blockIdx.x;
  const bool which = b0 >= NA;
  const int b = which ? b0 - NA : b0;
  const float* X = which ? rnn : cnn;
  __shared__ float red[16];
  float s = 0.f;
  for (int k = threadIdx.x; k < D; k += blockDim.x) s += X[(long)b * D + k] * X[(long)b * D + k];
  s = block_sum(s, red);
  if (threadIdx.x == 0) nrm[b0] = sqrtf(s);
}

// gradient of sim = gamma3 * cos wrt cnn (which=0, rows a < NA) or rnn (which=1, cols b < NB); thread per (row, k)
__global__ void sent_sim_bwd_kernel(const float* cnn, const float* rnn, int NA, int NB, int D, const float* sim,
                                    const float* nrm, const float* dsim, int which, float* out) {
  const int NX = which == 0 ? NA : NB, NY = which == 0 ? NB : NA;
  const long total = (long)NX * D;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int x = e / D, k = e % D;
    const float* X = which == 0 ? cnn : rnn;
    const float* Y = which == 0 ? rnn : cnn;
    const float nx = nrm[which == 0 ? x : NA + x];
    const float xv = X[(long)x * D + k];
    float g = 0.f;
    for (int y = 0; y < NY; ++y) {
      const float ny = nrm[which == 0 ? NA + y : y];
      const long idx = which == 0 ? (long)x * NB + y : (long)y * NB + x;
      const float ds = dsim[idx];
      const float yv = Y[(long)y * D + k];
      const float den = nx * ny;
      if (den > 1e-8f) g += GAMMA3 * ds * (yv / den - (sim[idx] / GAMMA3) * xv / (nx * nx));
      else g += GAMMA3 * ds * yv / 1e-8f;
    }
    out[e] = g;
  }
}

// ------------------------------------------------- hinge / mean on D out --
// mode 0: mean(relu(1 - x)); 1: mean(relu(1 + x)); 2: -mean(x); 3: mean(x)
__global__ void dout_reduce_kernel(const float* x, int n, int mode, float* out, const float* gout, float* dx) {
  __shared__ float red[16];
  if (!dx) {
    float s = 0.f;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
      const float v = x[k];
      s += mode == 0 ? fmaxf(1.f - v, 0.f) : mode == 1 ? fmaxf(1.f + v, 0.f) : (mode == 2 ? -v : v);
    }
    s = block_sum(s, red);
    if (threadIdx.x == 0) out[0] = s / n;
  } else {
    const float g = gout[0] / n;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
      const float v = x[k];
      dx[k] = mode == 0 ? (1.f - v > 0.f ? -g : 0.f) : mode == 1 ? (1.f + v > 0.f ? g : 0.f) : (mode == 2 ? -g : g);
    }
  }
}

// mean BCE-with-logits (F.binary_cross_entropy_with_logits, numerically stable form)
__global__ void bce_kernel(const float* x, const float* y, int n, float* out, const float* gout, float* dx) {
  __shared__ float red[16];
  if (!dx) {
    float s = 0.f;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
      const float v = x[k], t = y[k];
      s += fmaxf(v, 0.f) - v * t + log1pf(__expf(-fabsf(v)));
    }
    s = block_sum(s, red);
    if (threadIdx.x == 0) out[0] = s / n;
  } else {
    const float g = gout[0] / n;
    for (int k = threadIdx.x; k < n; k += blockDim.x) dx[k] = g * (1.f / (1.f + __expf(-x[k])) - y[k]);
  }
}

// ----------------------------------------------------- gradient penalty --
// per-sample ||[g_img, g_sent]||^2 (g_img NHWC bf16 [B][HW][ld] with C channels)
constexpr int GP_CHUNKS = 64;

// per-(chunk, sample) partial sum of squares of the image gradient (16-B pixel rows)
__global__ __launch_bounds__(256) void gp_norm_kernel(const bf16_t* gx, int ld, int HW, int C, float* ws) {
  __shared__ float red[16];
  const int b = blockIdx.y;
  const int per = (HW + GP_CHUNKS - 1) / GP_CHUNKS;
  const int p0 = blockIdx.x * per, p1 = min(HW, p0 + per);
  const int C8 = (C + 7) / 8;
  float s = 0.f;
  for (long e = threadIdx.x; e < (long)(p1 - p0) * C8; e += blockDim.x) {
    const int c0 = (int)(e % C8) * 8;
    const long p = p0 + e / C8;
    const uint4 v = *reinterpret_cast<const uint4*>(gx + ((long)b * HW + p) * ld + c0);
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float lo = c0 + 2 * j < C ? lo_f(w4[j]) : 0.f, hi = c0 + 2 * j + 1 < C ? hi_f(w4[j]) : 0.f;
      s += lo * lo + hi * hi;
    }
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) ws[b * GP_CHUNKS + blockIdx.x] = s;
}

// nrm2[b] = sum of the chunk partials (fixed order) + ||g_sent_b||^2 ; loss = 2 * mean_b(||g_b||^6)
__global__ void gp_loss_kernel(const float* ws, const float* gs, int E, int B, float* nrm2, float* out) {
  __shared__ float red[16];
  __shared__ float n2s[256];
  for (int b = 0; b < B; ++b) {
    float t = 0.f;
    for (int e = threadIdx.x; e < E; e += blockDim.x) {
      const float v = gs[(long)b * E + e];
      t += v * v;
    }
    t = block_sum(t, red);
    if (threadIdx.x == 0) {
      float sb = 0.f;
      for (int k = 0; k < GP_CHUNKS; ++k) sb += ws[b * GP_CHUNKS + k];
      nrm2[b] = sb + t;
      if (b < 256) n2s[b] = sb + t;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) {
      const float n2 = b < 256 ? n2s[b] : nrm2[b];
      s += n2 * n2 * n2;
    }
    out[0] = 2.f * s / B;
  }
}

// d/dg: 2/B * 6 ||g||^4 g * gout
__global__ void gp_bwd_kernel(const bf16_t* gx, int ld, int HW, int C, const float* gs, int E, const float* nrm2,
                              int B, const float* gout, bf16_t* dgx, int lddgx, float* dgs) {
  const int C8 = (C + 7) / 8;
  const long nimg = (long)B * HW * C8;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < nimg + (long)B * E;
       e += (long)gridDim.x * blockDim.x) {
    if (e < nimg) {
      const int c0 = (int)(e % C8) * 8;
      const long p = e / C8;
      const int b = (int)(p / HW);
      const float n2 = nrm2[b];
      const float coef = gout[0] * 12.f / B * n2 * n2;
      const uint4 v = *reinterpret_cast<const uint4*>(gx + p * ld + c0);
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
      uint32_t o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = pack2(coef * lo_f(w4[j]), coef * hi_f(w4[j]));
      bf16_t* dst = dgx + p * lddgx + c0;
      if (c0 + 8 <= C) {
        *reinterpret_cast<uint4*>(dst) = make_uint4(o[0], o[1], o[2], o[3]);
      } else {
        for (int j = 0; j < 8 && c0 + j < C; ++j) dst[j] = (bf16_t)((o[j >> 1] >> (16 * (j & 1))) & 0xffffu);
      }
    } else {
      const long q = e - nimg;
      const int b = q / E;
      const float n2 = nrm2[b];
      dgs[q] = gout[0] * 12.f / B * n2 * n2 * gs[q];
    }
  }
}

// --------------------------------------------------------- class labels --
// labels[i][(idx - 1) mod ncls] = 1   (train.py:102: idx 0 wraps to the last column)
__global__ void class_onehot_kernel(const long* ids, int B, int ncls, float* out, int* err) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < (long)B * ncls; e += (long)gridDim.x * blockDim.x) {
    const int i = e / ncls, c = e % ncls;
    long col = ids[i] - 1;
    if (col < 0) col += ncls;
    if (col < 0 || col >= ncls) {
      if (err) *err = 1;
      col = -1;
    }
    out[e] = (c == col) ? 1.f : 0.f;
  }
}

// -------------------------------------------------- ATTR_Enhance core ----
// per sample: P = softmax(q k^T) * scale (rows of 4), out = P v ; merged = sum_rows(out)
__global__ void attr_attn_kernel(const float* q, const float* k, const float* v, int B, int L, int D, float scale,
                                 float* probs, float* out, float* merged) {
  const int b = blockIdx.x;
  __shared__ float P[8][8];
  __shared__ float red[16];
  for (int x = 0; x < L; ++x)
    for (int y = 0; y < L; ++y) {
      float s = 0.f;
      for (int d = threadIdx.x; d < D; d += blockDim.x)
        s += q[((long)b * L + x) * D + d] * k[((long)b * L + y) * D + d];
      s = block_sum(s, red);
      if (threadIdx.x == 0) P[x][y] = s;
    }
  __syncthreads();
  if (threadIdx.x < L) {
    const int x = threadIdx.x;
    float mx = -INFINITY;
    for (int y = 0; y < L; ++y) mx = fmaxf(mx, P[x][y]);
    float sm = 0.f;
    for (int y = 0; y < L; ++y) sm += __expf(P[x][y] - mx);
    for (int y = 0; y < L; ++y) {
      const float pv = __expf(P[x][y] - mx) / sm * scale;
      P[x][y] = pv;
      probs[((long)b * L + x) * L + y] = pv;
    }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float m = 0.f;
    for (int x = 0; x < L; ++x) {
      float o = 0.f;
      for (int y = 0; y < L; ++y) o += P[x][y] * v[((long)b * L + y) * D + d];
      out[((long)b * L + x) * D + d] = o;
      m += o;
    }
    if (merged) merged[(long)b * D + d] = m;
  }
}

// backward given dout [B][L][D] (already including the merge broadcast):
// dv = P^T dout ; dP = dout v^T ; dlogits = scale * sm*(dP' - sum sm dP') with P = scale*sm
// dq = dlogits k ; dk = dlogits^T q
__global__ void attr_attn_bwd_kernel(const float* q, const float* k, const float* v, const float* probs,
                                     const float* dout, int B, int L, int D, float scale, float* dq, float* dk,
                                     float* dv) {
  const int b = blockIdx.x;
  __shared__ float dP[8][8], G[8][8];
  __shared__ float red[16];
  for (int x = 0; x < L; ++x)
    for (int y = 0; y < L; ++y) {
      float s = 0.f;
      for (int d = threadIdx.x; d < D; d += blockDim.x)
        s += dout[((long)b * L + x) * D + d] * v[((long)b * L + y) * D + d];
      s = block_sum(s, red);
      if (threadIdx.x == 0) dP[x][y] = s;
    }
  __syncthreads();
  if (threadIdx.x < L) {
    const int x = threadIdx.x;
    // P = scale * sm ; d sm = scale * dP ; dlogit = sm * (dsm - sum(sm * dsm))
    float dot = 0.f;
    for (int y = 0; y < L; ++y) dot += (probs[((long)b * L + x) * L + y] / scale) * scale * dP[x][y];
    for (int y = 0; y < L; ++y) {
      const float sm = probs[((long)b * L + x) * L + y] / scale;
      G[x][y] = sm * (scale * dP[x][y] - dot);
    }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    for (int x = 0; x < L; ++x) {
      float gq = 0.f, gk = 0.f, gv = 0.f;
      for (int y = 0; y < L; ++y) {
        gq += G[x][y] * k[((long)b * L + y) * D + d];
        gk += G[y][x] * q[((long)b * L + y) * D + d];
        gv += probs[((long)b * L + y) * L + x] * dout[((long)b * L + y) * D + d];
      }
      dq[((long)b * L + x) * D + d] = gq;
      dk[((long)b * L + x) * D + d] = gk;
      dv[((long)b * L + x) * D + d] = gv;
    }
  }
}

}  // namespace

extern "C" {

int eegan_sim_ce(const float* sim, int B, const long* class_ids, const long* labels, float* loss2, hipStream_t s) {
  sim_ce_kernel<<<1, 256, 2 * B * sizeof(float), s>>>(sim, B, class_ids, labels, loss2, nullptr, nullptr);
  return ee_check_launch("sim_ce");
}

int eegan_sim_ce_bwd(const float* sim, int B, const long* class_ids, const long* labels, const float* gloss2,
                     float* dsim, hipStream_t s) {
  sim_ce_kernel<<<1, 256, 2 * B * sizeof(float), s>>>(sim, B, class_ids, labels, nullptr, gloss2, dsim);
  return ee_check_launch("sim_ce_bwd");
}

int eegan_sent_sim(const float* cnn, const float* rnn, int na, int nb, int D, float* sim, hipStream_t s) {
  sent_sim_kernel<<<na, 64, 0, s>>>(cnn, rnn, nb, D, sim);
  return ee_check_launch("sent_sim");
}

int eegan_sent_sim_bwd(const float* cnn, const float* rnn, int na, int nb, int D, const float* sim, const float* dsim,
                       float* nrm_ws, float* dcnn, float* drnn, hipStream_t s) {
  row_norm_kernel<<<na + nb, 64, 0, s>>>(cnn, rnn, na, D, nrm_ws);
  if (dcnn) sent_sim_bwd_kernel<<<ee_cdiv((long)na * D, 256), 256, 0, s>>>(cnn, rnn, na, nb, D, sim, nrm_ws, dsim, 0, dcnn);
  if (drnn) sent_sim_bwd_kernel<<<ee_cdiv((long)nb * D, 256), 256, 0, s>>>(cnn, rnn, na, nb, D, sim, nrm_ws, dsim, 1, drnn);
  return ee_check_launch("sent_sim_bwd");
}

int eegan_dout_reduce(const float* x, int n, int mode, float* out, hipStream_t s) {
  dout_reduce_kernel<<<1, 256, 0, s>>>(x, n, mode, out, nullptr, nullptr);
  return ee_check_launch("dout_reduce");
}

int eegan_dout_reduce_bwd(const float* x, int n, int mode, const float* gout, float* dx, hipStream_t s) {
  dout_reduce_kernel<<<1, 256, 0, s>>>(x, n, mode, nullptr, gout, dx);
  return ee_check_launch("dout_reduce_bwd");
}

int eegan_bce_logits(const float* x, const float* target, int n, float* out, hipStream_t s) {
  bce_kernel<<<1, 256, 0, s>>>(x, target, n, out, nullptr, nullptr);
  return ee_check_launch("bce");
}

int eegan_bce_logits_bwd(const float* x, const float* target, int n, const float* gout, float* dx, hipStream_t s) {
  bce_kernel<<<1, 256, 0, s>>>(x, target, n, nullptr, gout, dx);
  return ee_check_launch("bce_bwd");
}

long eegan_gp_loss_workspace(int B) { return (long)B * GP_CHUNKS * sizeof(float); }

int eegan_gp_loss(const uint16_t* gx, int ld, int B, int HW, int C, const float* gs, int E, float* nrm2, float* out,
                  float* ws, hipStream_t s) {
  if ((ld % 8) || ((uintptr_t)gx & 15)) {
    ee_set_error("gp_loss: image gradient rows must be 16-byte aligned, ld %% 8 == 0 (ld %d)", ld);
    return -22;
  }
  gp_norm_kernel<<<dim3(GP_CHUNKS, B), 256, 0, s>>>(gx, ld, HW, C, ws);
  int rc = ee_check_launch("gp_norm");
  if (rc) return rc;
  gp_loss_kernel<<<1, 256, 0, s>>>(ws, gs, E, B, nrm2, out);
  return ee_check_launch("gp_loss");
}

int eegan_gp_loss_bwd(const uint16_t* gx, int ld, int B, int HW, int C, const float* gs, int E, const float* nrm2,
                      const float* gout, uint16_t* dgx, int lddgx, float* dgs, hipStream_t s) {
  if ((ld % 8) || (lddgx % 8)) {
    ee_set_error("gp_loss_bwd: channel strides must be multiples of 8");
    return -22;
  }
  const long work = (long)B * HW * ((C + 7) / 8) + (long)B * E;
  const int blocks = (int)std::min<long>(8192, (work + 255) / 256);
  gp_bwd_kernel<<<blocks, 256, 0, s>>>(gx, ld, HW, C, gs, E, nrm2, B, gout, dgx, lddgx, dgs);
  return ee_check_launch("gp_bwd");
}

int eegan_class_onehot(const long* ids, int B, int ncls, float* out, int* err, hipStream_t s) {
  class_onehot_kernel<<<ee_cdiv((long)B * ncls, 256), 256, 0, s>>>(ids, B, ncls, out, err);
  return ee_check_launch("class_onehot");
}

int eegan_attr_attn(const float* q, const float* k, const float* v, int B, int L, int D, float scale, float* probs,
                    float* out, float* merged, hipStream_t s) {
  if (L > 8) {
    ee_set_error("attr_attn: L > 8");
    return -22;
  }
  attr_attn_kernel<<<B, 256, 0, s>>>(q, k, v, B, L, D, scale, probs, out, merged);
  return ee_check_launch("attr_attn");
}

int eegan_attr_attn_bwd(const float* q, const float* k, const float* v, const float* probs, const float* dout, int B,
                        int L, int D, float scale, float* dq, float* dk, float* dv, hipStream_t s) {
  attr_attn_bwd_kernel<<<B, 256, 0, s>>>(q, k, v, probs, dout, B, L, D, scale, dq, dk, dv);
  return ee_check_launch("attr_attn_bwd");
}

}  // extern "C"
