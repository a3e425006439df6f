// SyncBN statistics + fused BN-apply / affine_ssa modulation / activation.
//
// replaces: sync_batchnorm/batchnorm.py:48-125 (_SynchronizedBatchNorm:
// F.batch_norm on one device, sum/ssum -> mean/inv_std across replicas),
// models.py:69-86 (affine_ssa: (gamma*m+1)*BN(x) + beta*m), the ReLU /
// LeakyReLU that follow it (models.py:115-118, 28, 38) and the nearest-2x
// upsample in front of every SAGB block (models.py:219).
//
// Layout: x NHWC bf16 [N][H][W][ld]; statistics fp32; per-(sample,channel)
// modulation gamma/beta fp32 [N][C]; spatial mask fp32 [N][Ho*Wo].
#include "common.h"
#include "../../include/eegan_hip.h"

namespace {

constexpr int NT = 256;

// ------------------------------------------------------------- statistics --
// per-block partial (sum, sumsq) per channel -> ws[block][2][C]
__global__ __launch_bounds__(NT) void bn_partial_kernel(const bf16_t* __restrict__ x, long P, int C, int ld,
                                                        long rows_per_block, float* __restrict__ ws) {
  extern __shared__ float sh[];  // [rows][C8*8] x2
  const int C8 = (C + 7) / 8;
  const int rows = NT / C8;
  const int t = threadIdx.x;
  const int row = t / C8, cg = t - row * C8;
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  const long p0 = blockIdx.x * rows_per_block;
  const long p1 = min(P, p0 + rows_per_block);
  if (row < rows) {
    const int c = cg * 8;
    const bool vec = (ld % 8) == 0;
    for (long p = p0 + row; p < p1; p += rows) {
      const bf16_t* src = x + p * ld + c;
      if (vec) {
        uint4 v = *reinterpret_cast<const uint4*>(src);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float a = lo_f(w4[j]), b = hi_f(w4[j]);
          s[2 * j] += a;
          q[2 * j] += a * a;
          s[2 * j + 1] += b;
          q[2 * j + 1] += b * b;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (c + j < C) {
            const float a = bf2f(src[j]);
            s[j] += a;
            q[j] += a * a;
          }
      }
    }
  }
  const int W8 = C8 * 8;
  float* ss = sh;
  float* sq = sh + rows * W8;
  if (row < rows) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ss[row * W8 + cg * 8 + j] = s[j];
      sq[row * W8 + cg * 8 + j] = q[j];
    }
  }
  __syncthreads();
  for (int c = t; c < C; c += NT) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rows; ++r) {
      a += ss[r * W8 + c];
      b += sq[r * W8 + c];
    }
    ws[(long)blockIdx.x * 2 * C + c] = a;
    ws[(long)blockIdx.x * 2 * C + C + c] = b;
  }
}

__global__ void bn_reduce_kernel(const float* __restrict__ ws, int nblk, int C, double* __restrict__ sums) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= 2 * C) return;
  double acc = 0.0;
  for (int b = 0; b < nblk; ++b) acc += (double)ws[(long)b * 2 * C + c];
  sums[c] = acc;
}

// stats[0..C) mean, [C..2C) inv_std, [2C..3C) 1 if d(inv_std)/d(var) != 0
__global__ void bn_finalize_kernel(const double* __restrict__ sums, int C, double count, double sum_scale, float eps,
                                   float mom, int clamp_mode, float* __restrict__ rmean, float* __restrict__ rvar,
                                   float* __restrict__ stats) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  // sum_scale: replication factor of the statistics tensor (4 when x is read
  // through the nearest-2x upsample: every low-res element appears 4 times)
  const double s1 = sums[c] * sum_scale, s2 = sums[C + c] * sum_scale;
  const double mean = s1 / count;
  double sumvar = s2 - s1 * mean;
  if (sumvar < 0) sumvar = 0;
  const double var_b = sumvar / count;
  float istd, vg = 1.f;
  if (clamp_mode) {  // batchnorm.py:125  clamp(var, eps) ** -0.5
    if (var_b < eps) {
      istd = (float)(1.0 / sqrt((double)eps));
      vg = 0.f;
    } else {
      istd = (float)(1.0 / sqrt(var_b));
    }
  } else {           // F.batch_norm: 1/sqrt(var + eps)
    istd = (float)(1.0 / sqrt(var_b + (double)eps));
  }
  stats[c] = (float)mean;
  stats[C + c] = istd;
  stats[2 * C + c] = vg;
  if (rmean) {
    const double unb = count > 1 ? sumvar / (count - 1) : sumvar;
    rmean[c] = (float)((1.0 - mom) * rmean[c] + mom * mean);
    rvar[c] = (float)((1.0 - mom) * rvar[c] + mom * unb);
  }
}

// ---------------------------------------------------------------- apply --
struct ModArgs {
  const bf16_t* x;
  int N, H, W, C, ldx;  // physical input grid
  int up2;              // output grid = (H<<up2, W<<up2)
  const float* stats;   // mean / istd
  int mode;             // 0 affine BN (w,b per channel, optional), 1 ssa
  const float* w;
  const float* b;
  const float* gam;     // [N][C]
  const float* bet;     // [N][C]
  const float* mask;    // [N][Ho*Wo]
  int act;
  float slope;
};

EE_DEV void mod_coeffs(const ModArgs& a, int n, int c, float m, float& mul, float& add) {
  // t = act(xhat * mul + add)
  if (a.mode == 0) {
    mul = a.w ? a.w[c] : 1.f;
    add = a.b ? a.b[c] : 0.f;
  } else {
    const float g = a.gam[(long)n * a.C + c], be = a.bet[(long)n * a.C + c];
    mul = g * m + 1.f;
    add = be * m;
  }
}

__global__ __launch_bounds__(NT) void bnmod_fwd_kernel(ModArgs a, bf16_t* __restrict__ y, int ldy) {
  const int Ho = a.H << a.up2, Wo = a.W << a.up2;
  const int C8 = (a.C + 7) / 8;
  const long total = (long)a.N * Ho * Wo * C8;
  for (long e = blockIdx.x * (long)NT + threadIdx.x; e < total; e += (long)gridDim.x * NT) {
    const int cg = e % C8;
    const long p = e / C8;
    const int ox = p % Wo;
    const long t = p / Wo;
    const int oy = t % Ho;
    const int n = t / Ho;
    const long ip = ((long)n * a.H + (oy >> a.up2)) * a.W + (ox >> a.up2);
    const int c0 = cg * 8;
    const float m = a.mode == 1 ? a.mask[(long)n * Ho * Wo + (long)oy * Wo + ox] : 0.f;
    float xv[8];
    if ((a.ldx % 8) == 0) {
      uint4 v = *reinterpret_cast<const uint4*>(a.x + ip * a.ldx + c0);
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xv[2 * j] = lo_f(w4[j]);
        xv[2 * j + 1] = hi_f(w4[j]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[j] = (c0 + j < a.C) ? bf2f(a.x[ip * a.ldx + c0 + j]) : 0.f;
    }
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = min(c0 + j, a.C - 1);
      float mul, add;
      mod_coeffs(a, n, c, m, mul, add);
      const float xh = (xv[j] - a.stats[c]) * a.stats[a.C + c];
      o[j] = act_fwd(xh * mul + add, a.act, a.slope);
    }
    bf16_t* dst = y + p * ldy + c0;
    if ((ldy % 8) == 0 && c0 + 8 <= ldy) {
      *reinterpret_cast<uint4*>(dst) = make_uint4(pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7]));
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (c0 + j < a.C) dst[j] = f2bf(o[j]);
    }
  }
}

// ------------------------------------------------------ backward, pass 1 --
// grid: (chunks, N). Each block reduces a pixel range of ONE sample into
// ws[n][chunk][4][C]:  S0 = sum g*m*xhat, S1 = sum g*m (ssa: dgamma/dbeta
// partials; affine: sum g*xhat / sum g), S2 = sum dxhat, S3 = sum dxhat*xhat.
// dmask[n][pix] = sum_c g*(gam*xhat + bet)  (ssa only).
__global__ __launch_bounds__(NT) void bnmod_bwd_reduce_kernel(ModArgs a, const bf16_t* __restrict__ dt, int lddt,
                                                              int pix_per_chunk, float* __restrict__ ws,
                                                              float* __restrict__ dmask) {
  extern __shared__ float sh[];
  const int C = a.C;
  const int C8 = (C + 7) / 8;
  const int rows = NT / C8;
  const int t = threadIdx.x;
  const int row = t / C8, cg = t - row * C8;
  const int n = blockIdx.y;
  const int Ho = a.H << a.up2, Wo = a.W << a.up2;
  const long HWo = (long)Ho * Wo;
  const long q0 = (long)blockIdx.x * pix_per_chunk;
  const long q1 = min(HWo, q0 + pix_per_chunk);
  float acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
  const int c0 = cg * 8;
  float* red = sh;                 // [rows][C8] for dmask
  // base of the pixel loop must be block-uniform for the dmask reduction
  for (long qb = q0; qb < q1; qb += rows) {
    const long q = qb + row;
    float dm = 0.f;
    if (row < rows && q < q1) {
      const int oy = q / Wo, ox = q - (long)oy * Wo;
      const long ip = ((long)n * a.H + (oy >> a.up2)) * a.W + (ox >> a.up2);
      const long op = (long)n * HWo + q;
      const float m = a.mode == 1 ? a.mask[op] : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        if (c < C) {
          const float xv = bf2f(a.x[ip * a.ldx + c]);
          const float gv = bf2f(dt[op * lddt + c]);
          const float xh = (xv - a.stats[c]) * a.stats[C + c];
          float mul, add;
          mod_coeffs(a, n, c, m, mul, add);
          const float tv = xh * mul + add;
          float g = gv;
          if (a.act == ACT_RELU) g = tv > 0.f ? g : 0.f;
          else if (a.act == ACT_LRELU) g = tv > 0.f ? g : g * a.slope;
          const float dxh = g * mul;
          if (a.mode == 1) {
            acc[0][j] += g * m * xh;
            acc[1][j] += g * m;
            dm += g * (a.gam[(long)n * C + c] * xh + a.bet[(long)n * C + c]);
          } else {
            acc[0][j] += g * xh;
            acc[1][j] += g;
          }
          acc[2][j] += dxh;
          acc[3][j] += dxh * xh;
        }
      }
    }
    if (a.mode == 1 && dmask) {
      if (row < rows) red[row * C8 + cg] = dm;
      __syncthreads();
      if (t < rows && qb + t < q1) {
        float s = 0.f;
        for (int i = 0; i < C8; ++i) s += red[t * C8 + i];
        dmask[(long)n * HWo + qb + t] = s;
      }
      __syncthreads();
    }
  }
  // reduce acc over rows -> ws
  float* sacc = sh + rows * C8;  // [rows][4][C8*8]
  const int W8 = C8 * 8;
  if (row < rows) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) sacc[(row * 4 + i) * W8 + c0 + j] = acc[i][j];
  }
  __syncthreads();
  float* out = ws + ((long)n * gridDim.x + blockIdx.x) * 4 * C;
  for (int e = t; e < 4 * C; e += NT) {
    const int i = e / C, c = e - i * C;
    float s = 0.f;
    for (int r = 0; r < rows; ++r) s += sacc[(r * 4 + i) * W8 + c];
    out[e] = s;
  }
}

// sum the chunks: dparam0/dparam1 ([C] for affine (summed over n), [N][C] for ssa),
// chan[0..C) = sum dxhat, chan[C..2C) = sum dxhat*xhat (double)
__global__ void bnmod_bwd_sums_kernel(const float* __restrict__ ws, int N, int nchunk, int C, int mode,
                                      float* __restrict__ d0, float* __restrict__ d1, double* __restrict__ chan) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  for (int n = 0; n < N; ++n) {
    double p0 = 0, p1 = 0;
    for (int k = 0; k < nchunk; ++k) {
      const float* w = ws + ((long)n * nchunk + k) * 4 * C;
      p0 += w[c];
      p1 += w[C + c];
      s2 += w[2 * C + c];
      s3 += w[3 * C + c];
    }
    if (mode == 1) {
      if (d0) d0[(long)n * C + c] = (float)p0;
      if (d1) d1[(long)n * C + c] = (float)p1;
    }
    s0 += p0;
    s1 += p1;
  }
  if (mode == 0) {
    if (d0) d0[c] = (float)s0;
    if (d1) d1[c] = (float)s1;
  }
  chan[c] = s2;
  chan[C + c] = s3;
}

// ------------------------------------------------------ backward, pass 2 --
// dx (physical input grid) = istd * (dxhat - mean(dxhat) - xhat*mean(dxhat*xhat)), summed
// over the 2x2 children when the forward upsampled.
__global__ __launch_bounds__(NT) void bnmod_bwd_dx_kernel(ModArgs a, const bf16_t* __restrict__ dt, int lddt,
                                                          const double* __restrict__ chan, double count,
                                                          bf16_t* __restrict__ dx, int lddx) {
  const int C8 = (a.C + 7) / 8;
  const int Ho = a.H << a.up2, Wo = a.W << a.up2;
  const long total = (long)a.N * a.H * a.W * C8;
  const int nch = a.up2 ? 4 : 1;
  for (long e = blockIdx.x * (long)NT + threadIdx.x; e < total; e += (long)gridDim.x * NT) {
    const int cg = e % C8;
    const long ip = e / C8;
    const int ix = ip % a.W;
    const long tt = ip / a.W;
    const int iy = tt % a.H;
    const int n = tt / a.H;
    const int c0 = cg * 8;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = 0.f;
    for (int ch = 0; ch < nch; ++ch) {
      const int oy = (iy << a.up2) + (ch >> 1), ox = (ix << a.up2) + (ch & 1);
      const long op = ((long)n * Ho + oy) * Wo + ox;
      const float m = a.mode == 1 ? a.mask[op] : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        if (c < a.C) {
          const float xv = bf2f(a.x[ip * a.ldx + c]);
          const float gv = bf2f(dt[op * lddt + c]);
          const float mean = a.stats[c], istd = a.stats[a.C + c], vg = a.stats[2 * a.C + c];
          const float xh = (xv - mean) * istd;
          float mul, add;
          mod_coeffs(a, n, c, m, mul, add);
          const float tv = xh * mul + add;
          float g = gv;
          if (a.act == ACT_RELU) g = tv > 0.f ? g : 0.f;
          else if (a.act == ACT_LRELU) g = tv > 0.f ? g : g * a.slope;
          const float dxh = g * mul;
          const float m1 = (float)(chan[c] / count), m2 = (float)(chan[a.C + c] / count);
          o[j] += istd * (dxh - m1 - vg * xh * m2);
        }
      }
    }
    bf16_t* dst = dx + ip * lddx + c0;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (c0 + j < a.C) dst[j] = f2bf(o[j]);
  }
}

int grid_for(long work, int per_block = NT) {
  long b = (work + per_block - 1) / per_block;
  return (int)std::max<long>(1, std::min<long>(b, 8192));
}

ModArgs make_args(const eegan_bnmod_desc* d) {
  ModArgs a = {};
  a.x = d->x;
  a.N = d->N;
  a.H = d->H;
  a.W = d->W;
  a.C = d->C;
  a.ldx = d->ldx;
  a.up2 = d->up2;
  a.stats = d->stats;
  a.mode = d->mode;
  a.w = d->w;
  a.b = d->b;
  a.gam = d->gam;
  a.bet = d->bet;
  a.mask = d->mask;
  a.act = d->act;
  a.slope = d->slope;
  return a;
}

int bwd_chunks(const eegan_bnmod_desc* d, int& ppc) {
  const long HWo = (long)(d->H << d->up2) * (d->W << d->up2);
  // aim at ~1024 blocks overall, >= 64 pixels each
  int chunks = std::max(1, std::min<int>(ee_cdiv(HWo, 64), ee_cdiv(1024, d->N)));
  ppc = ee_cdiv(HWo, chunks);
  chunks = ee_cdiv(HWo, ppc);
  return chunks;
}

}  // namespace

extern "C" {

long eegan_bn_stats_workspace(long P, int C) {
  const int C8 = (C + 7) / 8;
  const int rows = NT / C8;
  long rpb = std::max<long>(rows * 16, (P + 1023) / 1024);
  const long nblk = (P + rpb - 1) / rpb;
  return nblk * 2 * C * (long)sizeof(float);
}

int eegan_bn_stats(const uint16_t* x, long P, int C, int ld, float* ws, double* sums, hipStream_t stream) {
  const int C8 = (C + 7) / 8;
  if (C8 > NT) {
    ee_set_error("bn_stats: C=%d too large", C);
    return -22;
  }
  const int rows = NT / C8;
  long rpb = std::max<long>(rows * 16, (P + 1023) / 1024);
  const int nblk = (int)std::max<long>(1, (P + rpb - 1) / rpb);
  const size_t shm = 2 * rows * C8 * 8 * sizeof(float);
  bn_partial_kernel<<<nblk, NT, shm, stream>>>(x, P, C, ld, rpb, ws);
  int rc = ee_check_launch("bn_partial");
  if (rc) return rc;
  bn_reduce_kernel<<<ee_cdiv(2 * C, 256), 256, 0, stream>>>(ws, nblk, C, sums);
  return ee_check_launch("bn_reduce");
}

int eegan_bn_finalize(const double* sums, int C, double count, double sum_scale, float eps, float momentum,
                      int clamp_mode, float* running_mean, float* running_var, float* stats, hipStream_t stream) {
  bn_finalize_kernel<<<ee_cdiv(C, 256), 256, 0, stream>>>(sums, C, count, sum_scale, eps, momentum, clamp_mode,
                                                           running_mean, running_var, stats);
  return ee_check_launch("bn_finalize");
}

int eegan_bnmod_fwd(const eegan_bnmod_desc* d, uint16_t* y, int ldy, hipStream_t stream) {
  ModArgs a = make_args(d);
  const long work = (long)d->N * (d->H << d->up2) * (d->W << d->up2) * ((d->C + 7) / 8);
  bnmod_fwd_kernel<<<grid_for(work), NT, 0, stream>>>(a, y, ldy);
  return ee_check_launch("bnmod_fwd");
}

long eegan_bnmod_bwd_workspace(const eegan_bnmod_desc* d) {
  int ppc;
  const int chunks = bwd_chunks(d, ppc);
  return (long)d->N * chunks * 4 * d->C * (long)sizeof(float);
}

int eegan_bnmod_bwd(const eegan_bnmod_desc* d, const uint16_t* dt, int lddt, float* ws, float* dparam0,
                    float* dparam1, float* dmask, double* chan, hipStream_t stream) {
  ModArgs a = make_args(d);
  int ppc;
  const int chunks = bwd_chunks(d, ppc);
  const int C8 = (d->C + 7) / 8;
  if (C8 > NT) {
    ee_set_error("bnmod_bwd: C too large");
    return -22;
  }
  const int rows = NT / C8;
  const size_t shm = (rows * C8 + rows * 4 * C8 * 8) * sizeof(float);
  dim3 grid(chunks, d->N);
  bnmod_bwd_reduce_kernel<<<grid, NT, shm, stream>>>(a, dt, lddt, ppc, ws, dmask);
  int rc = ee_check_launch("bnmod_bwd_reduce");
  if (rc) return rc;
  bnmod_bwd_sums_kernel<<<ee_cdiv(d->C, 64), 64, 0, stream>>>(ws, d->N, chunks, d->C, d->mode, dparam0, dparam1,
                                                               chan);
  return ee_check_launch("bnmod_bwd_sums");
}

int eegan_bnmod_bwd_dx(const eegan_bnmod_desc* d, const uint16_t* dt, int lddt, const double* chan, double count,
                       uint16_t* dx, int lddx, hipStream_t stream) {
  ModArgs a = make_args(d);
  const long work = (long)d->N * d->H * d->W * ((d->C + 7) / 8);
  bnmod_bwd_dx_kernel<<<grid_for(work), NT, 0, stream>>>(a, dt, lddt, chan, count, dx, lddx);
  return ee_check_launch("bnmod_bwd_dx");
}

}  // extern "C"
