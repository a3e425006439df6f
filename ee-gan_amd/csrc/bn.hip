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
#include <stdlib.h>
#include <string.h>

#include "common.h"
#include "../../include/eegan_hip.h"

namespace {

constexpr int NT = 256;

// ------------------------------------------------------------- statistics --
// per-block partial (sum, sumsq) per channel -> ws[block][2][C]
template <int SU = 4>   // pixels' loads in flight per thread (summed in pixel order for any count)
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
    long p = p0 + row;
    if (vec) {
      // SU pixels' loads in flight per thread, summed in pixel order (as one at a time)
      for (; p < p1; p += SU * rows) {
        uint4 v[SU];
#pragma unroll
        for (int u = 0; u < SU; ++u)
          if (p + u * rows < p1) v[u] = *reinterpret_cast<const uint4*>(x + (p + u * rows) * ld + c);
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          if (p + u * rows >= p1) break;
          const uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float a = lo_f(w4[j]), b = hi_f(w4[j]);
            s[2 * j] += a;
            q[2 * j] += a * a;
            s[2 * j + 1] += b;
            q[2 * j + 1] += b * b;
          }
        }
      }
    }
    for (; p < p1; p += rows) {
      const bf16_t* src = x + p * ld + c;
      {
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

// BN finalize parameters (the statistics of one BN call)
struct FinArgs {
  const double* sums;   // [2C] sum, sum of squares (after any cross-rank all-reduce)
  double count, sum_scale;
  float eps, mom;
  int clamp_mode;
  float* rmean;         // running statistics (null: not tracked)
  float* rvar;
  float* stats;         // out: [3C] mean, inv_std, d(inv_std)/d(var) != 0
};

// mean / inv_std / variance-gradient flag of channel c (bit-identical wherever it runs);
// `commit` writes stats[] and updates the running statistics (once per channel per call)
EE_DEV void bn_finalize_channel(const FinArgs& f, int C, int c, float& mean_o, float& istd_o, bool commit) {
  // sum_scale: replication factor of the statistics tensor (4 when x is read
  // through the nearest-2x upsample: every low-res element appears 4 times)
  const double s1 = f.sums[c] * f.sum_scale, s2 = f.sums[C + c] * f.sum_scale;
  const double mean = s1 / f.count;
  double sumvar = s2 - s1 * mean;
  if (sumvar < 0) sumvar = 0;
  const double var_b = sumvar / f.count;
  float istd, vg = 1.f;
  if (f.clamp_mode) {  // batchnorm.py:125  clamp(var, eps) ** -0.5
    if (var_b < f.eps) {
      istd = (float)(1.0 / sqrt((double)f.eps));
      vg = 0.f;
    } else {
      istd = (float)(1.0 / sqrt(var_b));
    }
  } else {           // F.batch_norm: 1/sqrt(var + eps)
    istd = (float)(1.0 / sqrt(var_b + (double)f.eps));
  }
  mean_o = (float)mean;
  istd_o = istd;
  if (!commit) return;
  f.stats[c] = (float)mean;
  f.stats[C + c] = istd;
  f.stats[2 * C + c] = vg;
  if (f.rmean) {
    const double unb = f.count > 1 ? sumvar / (f.count - 1) : sumvar;
    f.rmean[c] = (float)((1.0 - f.mom) * f.rmean[c] + f.mom * mean);
    f.rvar[c] = (float)((1.0 - f.mom) * f.rvar[c] + f.mom * unb);
  }
}

// stats[0..C) mean, [C..2C) inv_std, [2C..3C) 1 if d(inv_std)/d(var) != 0
__global__ void bn_finalize_kernel(FinArgs f, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float m, i;
  bn_finalize_channel(f, C, c, m, i, true);
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
  int wsh;              // log2 of the output width when it is a power of two, else -1
  float nslope;         // the activation's slope below 0: 1 (none), 0 (relu), slope (lrelu)
};

// Blocks cover (pixel chunk, sample); a thread owns 8 consecutive channels
// (one 16-byte NHWC load) for every pixel it visits, so the per-channel
// statistics / modulation parameters of its sample stay in registers.  The
// arithmetic runs on channel pairs (float2: packed v_pk_* fp32 instructions,
// half the VALU issue of scalar code), pixel coordinates by shifts when the
// output width is a power of two (no integer division per pixel), offsets in
// 32 bits (host-checked).
typedef float f2_t __attribute__((ext_vector_type(2)));

struct ChanParams {
  f2_t mean[4], istd[4], pm[4], pa[4];  // mode 0: w, b ; mode 1: gam[n], bet[n]
};

EE_DEV f2_t splat2(float v) { return f2_t{v, v}; }

// The block's channel parameters are staged once through LDS: prm[4][W8] = mean,
// istd, pm, pa (mode 0: w, b; mode 1: gam[n], bet[n]) for channels 0..W8 (those
// >= C repeat channel C-1).  Loading them per thread (8 channels x 4 values,
// every thread of every block on the same few hundred bytes) cost as much as
// the pixel loads on the small-image layers.  FIN: mean / istd straight from
// the sums (the forward's fused finalize); `commit` also writes stats[] and
// the running statistics (block (0, 0) only).
EE_DEV void stage_params(const ModArgs& a, int n, float* prm, int W8, const FinArgs* fin = nullptr,
                         bool commit = false) {
  for (int c = threadIdx.x; c < W8; c += NT) {
    const int cc = min(c, a.C - 1);
    float mean, istd;
    if (fin) {
      bn_finalize_channel(*fin, a.C, cc, mean, istd, commit && c < a.C);
    } else {
      mean = a.stats[cc];
      istd = a.stats[a.C + cc];
    }
    prm[c] = mean;
    prm[W8 + c] = istd;
    if (a.mode == 0) {
      prm[2 * W8 + c] = a.w ? a.w[cc] : 1.f;
      prm[3 * W8 + c] = a.b ? a.b[cc] : 0.f;
    } else {
      prm[2 * W8 + c] = a.gam[(long)n * a.C + cc];
      prm[3 * W8 + c] = a.bet[(long)n * a.C + cc];
    }
  }
}

EE_DEV void lds8(const float* p, f2_t (&d)[4]) {
  const float4 lo = *reinterpret_cast<const float4*>(p), hi = *reinterpret_cast<const float4*>(p + 4);
  d[0] = f2_t{lo.x, lo.y};
  d[1] = f2_t{lo.z, lo.w};
  d[2] = f2_t{hi.x, hi.y};
  d[3] = f2_t{hi.z, hi.w};
}

// a thread's 8 channels c0.. from the staged table
EE_DEV void load_params(const float* prm, int W8, int c0, ChanParams& q) {
  lds8(prm + c0, q.mean);
  lds8(prm + W8 + c0, q.istd);
  lds8(prm + 2 * W8 + c0, q.pm);
  lds8(prm + 3 * W8 + c0, q.pa);
}

EE_DEV void unpack8(uint4 v, f2_t (&f)[4]) {
  const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) f[j] = f2_t{lo_f(w4[j]), hi_f(w4[j])};
}

// zero the channels >= nv of a padded row's last chunk (padding may hold anything)
EE_DEV void clip8(f2_t (&f)[4], int nv) {
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (j >= nv) f[j >> 1][j & 1] = 0.f;
}

// act(v) for none / relu / lrelu: v > 0 ? v : v * nslope
EE_DEV f2_t act2(f2_t v, float ns) {
  const f2_t vs = v * splat2(ns);
  return f2_t{v.x > 0.f ? v.x : vs.x, v.y > 0.f ? v.y : vs.y};
}
// g * act'(t)
EE_DEV f2_t gact2(f2_t g, f2_t t, float ns) {
  const f2_t gs = g * splat2(ns);
  return f2_t{t.x > 0.f ? g.x : gs.x, t.y > 0.f ? g.y : gs.y};
}

EE_DEV void store8(bf16_t* dst, const f2_t (&o)[4], int nvalid) {
  if (nvalid >= 8) {
    *reinterpret_cast<uint4*>(dst) =
        make_uint4(pack2(o[0].x, o[0].y), pack2(o[1].x, o[1].y), pack2(o[2].x, o[2].y), pack2(o[3].x, o[3].y));
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j < nvalid) dst[j] = f2bf(o[j >> 1][j & 1]);
  }
}

// input-grid pixel (relative to the sample) of output pixel q
EE_DEV int in_pix(const ModArgs& a, int q, int Wo) {
  if (!a.up2) return q;
  int oy, ox;
  if (a.wsh >= 0) {
    oy = q >> a.wsh;
    ox = q & (Wo - 1);
  } else {
    oy = (unsigned)q / (unsigned)Wo;
    ox = q - oy * Wo;
  }
  return (oy >> 1) * a.W + (ox >> 1);
}

// grid (chunks, N): output pixels [chunk*ppc, ...) of sample n.  FUNR pixels
// per thread per iteration: their loads are all issued before any arithmetic
// (a single 16-byte load per iteration left these kernels latency-bound).
constexpr int FUNR_DEFAULT = 2;

// FIN: the statistics come from the sums (the finalize kernel folded in: every block
// recomputes its channels' mean / inv_std while staging them, block (0, 0) also writes
// stats[] and the running statistics -- one launch less per BN call on the generator's
// serial chain).  Dynamic LDS: 4 * W8 floats (stage_params).
template <bool FIN, int FUNR = FUNR_DEFAULT>
__global__ __launch_bounds__(NT, 6) void bnmod_fwd_kernel(ModArgs a, bf16_t* __restrict__ y, int ldy, int ppc,
                                                       FinArgs fin) {
  extern __shared__ float prm[];  // [4][W8]
  const int C8 = (a.C + 7) / 8, rows = NT / C8, W8 = C8 * 8;
  stage_params(a, blockIdx.y, prm, W8, FIN ? &fin : nullptr, FIN && blockIdx.x == 0 && blockIdx.y == 0);
  __syncthreads();
  const int row = threadIdx.x / C8, cg = threadIdx.x - row * C8;
  if (row >= rows) return;
  const int n = blockIdx.y, c0 = cg * 8, nv = a.C - c0;
  const int Ho = a.H << a.up2, Wo = a.W << a.up2;
  const int HWo = Ho * Wo;  // per-sample pixel counts fit 32 bits
  const int q1 = min(HWo, ((int)blockIdx.x + 1) * ppc);
  ChanParams P;
  load_params(prm, W8, c0, P);
  const bf16_t* xs = a.x + (unsigned)(n * a.H * a.W) * (unsigned)a.ldx + c0;
  bf16_t* ys = y + (unsigned)(n * HWo) * (unsigned)ldy + c0;
  const float* ms = a.mask + (long)n * HWo;
  const float ns = a.nslope;
  for (int qb = (int)blockIdx.x * ppc + row; qb < q1; qb += FUNR * rows) {
    uint4 xr[FUNR];
    float mr[FUNR];
#pragma unroll
    for (int u = 0; u < FUNR; ++u) {
      const int q = qb + u * rows;
      if (q < q1) {
        xr[u] = *reinterpret_cast<const uint4*>(xs + (unsigned)in_pix(a, q, Wo) * (unsigned)a.ldx);
        mr[u] = a.mode == 1 ? ms[q] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < FUNR; ++u) {
      const int q = qb + u * rows;
      if (q >= q1) break;
      f2_t xv[4], o[4];
      unpack8(xr[u], xv);
      const f2_t m2 = splat2(mr[u]);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const f2_t xh = (xv[k] - P.mean[k]) * P.istd[k];
        const f2_t mul = a.mode == 1 ? P.pm[k] * m2 + splat2(1.f) : P.pm[k];
        const f2_t add = a.mode == 1 ? P.pa[k] * m2 : P.pa[k];
        o[k] = act2(xh * mul + add, ns);
      }
      store8(ys + (unsigned)q * (unsigned)ldy, o, nv);
    }
  }
}

// ------------------------------------------------------ backward, pass 1 --
constexpr int RU_DEFAULT = 2;

// sum of v over the C8 consecutive lanes that hold one pixel's channel groups
// (C8 a power of two <= 64; every lane of the group gets the same bits, summed
// in the butterfly order xor 1, 2, 4, ...): DPP within 16-lane rows, no LDS trips
template <int CTRL>
EE_DEV float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
EE_DEV float group_sum(float v, int c8) {
  if (c8 >= 2) v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]: lane ^ 1
  if (c8 >= 4) v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]: lane ^ 2
  if (c8 >= 8) v += dpp_f<0x141>(v);   // row_half_mirror: the other quad of 8
  if (c8 >= 16) v += dpp_f<0x140>(v);  // row_mirror: the other half-row
  if (c8 >= 32) v += __shfl_xor(v, 16);
  if (c8 >= 64) v += __shfl_xor(v, 32);
  return v;
}

// grid: (chunks, N). Each block reduces a pixel range of ONE sample into
// ws[n][chunk][4][C]:  S0 = sum g*m*xhat, S1 = sum g*m (ssa: dgamma/dbeta
// partials; affine: sum g*xhat / sum g), S2 = sum dxhat, S3 = sum dxhat*xhat,
// with g the gradient behind the activation and dxhat = g * mul.
// dmask[n][pix] = sum_c g*(gam*xhat + bet)  (ssa only).
// The loop accumulates A = sum g*m*xhat, B = sum g*m, G = sum g, D = sum g*xhat
// (ssa; affine: D and G only) and the block's tail forms, with its sample's
// per-channel pm (ssa: gam[n], affine: w): S2 = pm*B + G, S3 = pm*A + D
// (affine: S0 = D, S1 = G, S2 = pm*G, S3 = pm*D) -- dxhat = g*(pm*m + 1).
// RU pixels' loads per thread are issued before their arithmetic; at <= 128
// VGPRs four blocks fit a CU, so the ~1024-block grid runs in one round.
template <int RU = RU_DEFAULT>
__global__ __launch_bounds__(NT, 4) void bnmod_bwd_reduce_kernel(ModArgs a, const bf16_t* __restrict__ dt, int lddt,
                                                              int pix_per_chunk, float* __restrict__ ws,
                                                              float* __restrict__ dmask, int knock) {
  // knock (diagnostic knock-outs, EEGAN_BN knock=bits; results wrong): 1 no pixel loads,
  // 2 no cross-row tail (zeros written), 4 no channel parameters (constants)
  extern __shared__ float sh[];
  const int C = a.C;
  const int C8 = (C + 7) / 8;
  const int rows = NT / C8;
  const int t = threadIdx.x;
  const int row = t / C8, cg = t - row * C8;
  const int n = blockIdx.y;
  const int Ho = a.H << a.up2, Wo = a.W << a.up2;
  const int HWo = Ho * Wo;  // per-sample pixel counts fit 32 bits
  const int q0 = (int)blockIdx.x * pix_per_chunk;
  const int q1 = min(HWo, q0 + pix_per_chunk);
  const bool ssa = a.mode == 1;
  f2_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[i][k] = splat2(0.f);
  const int c0 = cg * 8, nv = C - c0;
  const int W8 = C8 * 8, RS = 4 * W8 + 1;
  float* prm = sh;                 // [4][W8] channel parameters (stage_params)
  float* red = sh + 4 * W8;        // [rows][C8] for dmask
  float* sacc = red + rows * C8;   // [rows][RS] row partials
  ChanParams P;
  const bool live = row < rows;
  if (!(knock & 4)) stage_params(a, n, prm, W8);
  __syncthreads();
  if (live && !(knock & 4)) load_params(prm, W8, c0, P);
  if (knock & 4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) P.mean[k] = P.pm[k] = P.pa[k] = splat2(0.f), P.istd[k] = splat2(1.f);
  }
  // a pixel's C8 channel groups are C8 consecutive lanes of one wave when C8 is a
  // power of two <= 64: its dmask is then a DPP / shuffle reduction (no barriers)
  const bool wave_red = (C8 & (C8 - 1)) == 0 && C8 <= 64;
  const bf16_t* xs = a.x + (unsigned)(n * a.H * a.W) * (unsigned)a.ldx + c0;
  const bf16_t* gs = dt + (unsigned)(n * HWo) * (unsigned)lddt + c0;
  const float* ms = a.mask + (long)n * HWo;
  const float ns = a.nslope;
  // base of the pixel loop must be block-uniform for the dmask reduction
  for (int qb = q0; qb < q1; qb += RU * rows) {
    uint4 xc[RU], gc[RU];
    float mc[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int q = qb + u * rows + row;
      if (live && q < q1) {
        if (knock & 1) {
          xc[u] = gc[u] = make_uint4(0x3f803f80u, 0, 0, 0);
          mc[u] = 0.5f;
        } else {
          xc[u] = *reinterpret_cast<const uint4*>(xs + (unsigned)in_pix(a, q, Wo) * (unsigned)a.ldx);
          gc[u] = *reinterpret_cast<const uint4*>(gs + (unsigned)q * (unsigned)lddt);
          mc[u] = ssa ? ms[q] : 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int q = qb + u * rows + row;
      f2_t dm2 = splat2(0.f);
      if (live && q < q1) {
        f2_t xv[4], gv[4];
        unpack8(xc[u], xv);
        unpack8(gc[u], gv);
        if (nv < 8) {
          clip8(xv, nv);
          clip8(gv, nv);
        }
        const f2_t m2 = splat2(mc[u]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const f2_t xh = (xv[k] - P.mean[k]) * P.istd[k];
          const f2_t mul = ssa ? P.pm[k] * m2 + splat2(1.f) : P.pm[k];
          const f2_t add = ssa ? P.pa[k] * m2 : P.pa[k];
          const f2_t g = gact2(gv[k], xh * mul + add, ns);
          const f2_t gx = g * xh;
          if (ssa) {
            const f2_t gm = g * m2;
            acc[0][k] += gm * xh;
            acc[1][k] += gm;
            dm2 += P.pm[k] * gx;
            dm2 += P.pa[k] * g;
          }
          acc[2][k] += g;
          acc[3][k] += gx;
        }
      }
      if (ssa && dmask) {
        float dm = dm2.x + dm2.y;
        if (wave_red) {
          dm = group_sum(dm, C8);
          if (cg == 0 && live && q < q1) dmask[(long)n * HWo + q] = dm;
        } else {
          if (live) red[row * C8 + cg] = dm;
          __syncthreads();
          const int qt = qb + u * rows + t;
          if (t < rows && qt < q1) {
            float s = 0.f;
            for (int i = 0; i < C8; ++i) s += red[t * C8 + i];
            dmask[(long)n * HWo + qt] = s;
          }
          __syncthreads();
        }
      }
    }
  }
  // reduce acc over rows -> ws: every row's partials through LDS (a row stride of
  // 4 * W8 + 1 floats spreads a wave's rows over the banks), then one thread per
  // output sums the rows in order and forms S0..S3.
  if (knock & 2) {
    float* out = ws + ((long)n * gridDim.x + blockIdx.x) * 4 * C;
    const float z = acc[0][0].x + acc[3][3].y;   // keep the loop live
    for (int c = t; c < 4 * C; c += NT) out[c] = z;
    return;
  }
  if (live) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) sacc[row * RS + i * W8 + c0 + j] = acc[i][j >> 1][j & 1];
  }
  __syncthreads();
  float* out = ws + ((long)n * gridDim.x + blockIdx.x) * 4 * C;
  for (int c = t; c < C; c += NT) {
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < rows; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) s[i] += sacc[r * RS + i * W8 + c];
    const float pm = knock & 4 ? 0.f : prm[2 * W8 + c];
    if (ssa) {
      out[c] = s[0];
      out[C + c] = s[1];
      out[2 * C + c] = fmaf(pm, s[1], s[2]);
      out[3 * C + c] = fmaf(pm, s[0], s[3]);
    } else {
      out[c] = s[3];
      out[C + c] = s[2];
      out[2 * C + c] = pm * s[2];
      out[3 * C + c] = pm * s[3];
    }
  }
}

// per-sample chunk sums tmp[n][4C] (double, deterministic column reduce) ->
// dparam0/dparam1 ([C] for affine (summed over n), [N][C] for ssa),
// chan[0..C) = sum dxhat, chan[C..2C) = sum dxhat*xhat
__global__ void bnmod_bwd_sums_kernel(const double* __restrict__ tmp, int N, int C, int mode, float* __restrict__ d0,
                                      float* __restrict__ d1, double* __restrict__ chan) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= 4 * C) return;
  const int i = j / C, c = j - i * C;
  double s = 0;
  // 16 samples' loads in flight before their sums (the sums stay in sample order)
  for (int n0 = 0; n0 < N; n0 += 16) {
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = tmp[(long)min(n0 + u, N - 1) * 4 * C + j];   // unconditional loads
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (n0 + u >= N) break;
      s += v[u];
      if (mode == 1 && i < 2) {
        float* d = i == 0 ? d0 : d1;
        if (d) d[(long)(n0 + u) * C + c] = (float)v[u];
      }
    }
  }
  if (i >= 2) chan[(i - 2) * C + c] = s;
  else if (mode == 0) {
    float* d = i == 0 ? d0 : d1;
    if (d) d[c] = (float)s;
  }
}

// ------------------------------------------------------ backward, pass 2 --
// The dx pass keeps round 4's scalar form: a packed-fp32 rewrite (v_pk_*, 32-bit
// offsets, four blocks per CU) was 15-25 % faster in isolation but made the
// generator's backward on two streams (Gen.forward_branched) non-deterministic
// run to run -- identical forward, the block-5 conv_c1 gradient different in ~1
// of 5 repetitions under a concurrent lane (tools/gen_determinism.py; the scalar
// form: 0 of 117) -- and the cause was not found, so it is not shipped.
struct ChanParamsS {
  float mean[8], istd[8], pm[8], pa[8];  // mode 0: w, b ; mode 1: gam[n], bet[n]
};

EE_DEV void lds8_s(const float* p, float (&d)[8]) {
  const float4 lo = *reinterpret_cast<const float4*>(p), hi = *reinterpret_cast<const float4*>(p + 4);
  d[0] = lo.x, d[1] = lo.y, d[2] = lo.z, d[3] = lo.w, d[4] = hi.x, d[5] = hi.y, d[6] = hi.z, d[7] = hi.w;
}

EE_DEV void coeffs_s(const ModArgs& a, const ChanParamsS& q, int j, float m, float& mul, float& add) {
  if (a.mode == 0) {
    mul = q.pm[j];
    add = q.pa[j];
  } else {
    mul = q.pm[j] * m + 1.f;
    add = q.pa[j] * m;
  }
}

EE_DEV void unpack8_s(uint4 v, float (&f)[8]) {
  const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = lo_f(w4[j]);
    f[2 * j + 1] = hi_f(w4[j]);
  }
}

EE_DEV void store8_s(bf16_t* dst, const float (&o)[8], int nvalid) {
  if (nvalid >= 8) {
    *reinterpret_cast<uint4*>(dst) = make_uint4(pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7]));
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j < nvalid) dst[j] = f2bf(o[j]);
  }
}

// dx (physical input grid) = istd * (dxhat - mean(dxhat) - xhat*mean(dxhat*xhat)), summed
// over the 2x2 children when the forward upsampled.  grid (chunks, N) over
// input pixels of sample n.
// DXU input pixels x NCH (1, or the 4 upsampled) output children per iteration, loads first
template <int DXU, int NCH>
EE_DEV void bwd_dx_body(const ModArgs& a, const bf16_t* __restrict__ dt, int lddt, bf16_t* __restrict__ dx, int lddx,
                        int ppc, const ChanParamsS& P, const float (&vg)[8], const float (&m1)[8], const float (&m2)[8],
                        int n, int c0, int nv, int row, int rows, int q1) {
  const int Ho = a.H << a.up2, Wo = a.W << a.up2;
  const int HW = a.H * a.W;
  for (int qb = (int)blockIdx.x * ppc + row; qb < q1; qb += DXU * rows) {
    uint4 xr[DXU], gr[DXU][NCH];
    float mr[DXU][NCH];
#pragma unroll
    for (int u = 0; u < DXU; ++u) {
      const int q = qb + u * rows;
      if (q < q1) {
        const int iy = (unsigned)q / (unsigned)a.W, ix = q - iy * a.W;
        xr[u] = *reinterpret_cast<const uint4*>(a.x + ((long)n * HW + q) * a.ldx + c0);
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
          {
            const int oy = (iy << a.up2) + (ch >> 1), ox = (ix << a.up2) + (ch & 1);
            const long op = ((long)n * Ho + oy) * Wo + ox;
            gr[u][ch] = *reinterpret_cast<const uint4*>(dt + op * lddt + c0);
            mr[u][ch] = a.mode == 1 ? a.mask[op] : 0.f;
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < DXU; ++u) {
      const int q = qb + u * rows;
      if (q >= q1) break;
      float xh[8], o[8];
      unpack8_s(xr[u], xh);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xh[j] = (xh[j] - P.mean[j]) * P.istd[j];
        o[j] = 0.f;
      }
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        float gv[8];
        unpack8_s(gr[u][ch], gv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float mul, add;
          coeffs_s(a, P, j, mr[u][ch], mul, add);
          const float tv = xh[j] * mul + add;
          float g = gv[j];
          if (a.act == ACT_RELU) g = tv > 0.f ? g : 0.f;
          else if (a.act == ACT_LRELU) g = tv > 0.f ? g : g * a.slope;
          o[j] += P.istd[j] * (g * mul - m1[j] - vg[j] * xh[j] * m2[j]);
        }
      }
      store8_s(dx + ((long)n * HW + q) * lddx + c0, o, nv);
    }
  }
}

template <int DXU1 = 4>
__global__ __launch_bounds__(NT) void bnmod_bwd_dx_kernel(ModArgs a, const bf16_t* __restrict__ dt, int lddt,
                                                          const double* __restrict__ chan, double count,
                                                          bf16_t* __restrict__ dx, int lddx, int ppc) {
  // dynamic LDS [7][W8]: stage_params' four rows, then vg, mean(dxhat), mean(dxhat*xhat)
  extern __shared__ float prm[];
  const int C8 = (a.C + 7) / 8, rows = NT / C8, W8 = C8 * 8;
  stage_params(a, blockIdx.y, prm, W8);
  for (int c = threadIdx.x; c < W8; c += NT) {
    const int cc = min(c, a.C - 1);
    prm[4 * W8 + c] = a.stats[2 * a.C + cc];
    prm[5 * W8 + c] = (float)(chan[cc] / count);
    prm[6 * W8 + c] = (float)(chan[a.C + cc] / count);
  }
  __syncthreads();
  const int row = threadIdx.x / C8, cg = threadIdx.x - row * C8;
  if (row >= rows) return;
  const int n = blockIdx.y, c0 = cg * 8, nv = a.C - c0;
  const int q1 = min(a.H * a.W, ((int)blockIdx.x + 1) * ppc);
  ChanParamsS P;
  float vg[8], m1[8], m2[8];
  lds8_s(prm + c0, P.mean);
  lds8_s(prm + W8 + c0, P.istd);
  lds8_s(prm + 2 * W8 + c0, P.pm);
  lds8_s(prm + 3 * W8 + c0, P.pa);
  lds8_s(prm + 4 * W8 + c0, vg);
  lds8_s(prm + 5 * W8 + c0, m1);
  lds8_s(prm + 6 * W8 + c0, m2);
  if (a.up2) bwd_dx_body<DXU1 / 2, 4>(a, dt, lddt, dx, lddx, ppc, P, vg, m1, m2, n, c0, nv, row, rows, q1);
  else bwd_dx_body<DXU1, 1>(a, dt, lddt, dx, lddx, ppc, P, vg, m1, m2, n, c0, nv, row, rows, q1);
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
  const int Wo = d->W << d->up2;
  a.wsh = (Wo & (Wo - 1)) == 0 ? __builtin_ctz((unsigned)Wo) : -1;
  a.nslope = d->act == ACT_RELU ? 0.f : d->act == ACT_LRELU ? d->slope : 1.f;
  return a;
}

// Grid knobs for sweeps (tools/bn_bench.py): EEGAN_BN="fwd_target=1536,fwd_prow=8,
// dx_target=2048,dx_prow=8,bwd_target=1024,bwd_minpix=64,stats_blocks=1024" (unset keys
// keep these defaults; *_prow: the fewest pixel rows a block walks) and the pixels a
// thread keeps in flight: fwd_u (2 | 4), red_u (2 | 4), dx_u (4 | 8), stats_u (4 | 8).
static int bn_knob(const char* key, int dflt) {
  const char* v = getenv("EEGAN_BN");
  if (!v) return dflt;
  const size_t n = strlen(key);
  for (const char* p = v; p && *p;) {
    if (!strncmp(p, key, n) && p[n] == '=') return atoi(p + n + 1);
    p = strchr(p, ',');
    if (p) ++p;
  }
  return dflt;
}

// chunks of a per-sample pixel range: ~`target` blocks overall (whole rounds of
// resident blocks: the forward holds 6 blocks per CU -> 1536, the dx pass 4 ->
// 2048 = two rounds), >= 8 pixel rows per block
int pix_chunks(int N, long HW, int C, int& ppc, int target = 2048, int prow = 8) {
  const int rows = NT / ((C + 7) / 8);
  ppc = (int)std::max<long>((long)rows * prow, (HW * N + target - 1) / target);
  return std::max(1, ee_cdiv(HW, ppc));
}

bool vec_ok(const eegan_bnmod_desc* d, int ld, const void* p, const char* what) {
  if ((d->ldx % 8) || (ld % 8) || ((uintptr_t)d->x & 15) || ((uintptr_t)p & 15) || (d->C + 7) / 8 > NT) {
    ee_set_error("%s: bf16 rows must be 16-byte aligned with channel strides multiple of 8 (ldx %d, ld %d, C %d)",
                 what, d->ldx, ld, d->C);
    return false;
  }
  if (d->act != ACT_NONE && d->act != ACT_RELU && d->act != ACT_LRELU) {
    ee_set_error("%s: activation %d (none / relu / leaky relu only)", what, d->act);
    return false;
  }
  // element offsets of one sample's rows are 32-bit in the kernels
  const long HWo = (long)(d->H << d->up2) * (d->W << d->up2);
  if ((long)d->N * HWo * std::max(ld, d->ldx) >= (1L << 31)) {
    ee_set_error("%s: tensor of %ld elements exceeds the kernels' 32-bit offsets", what,
                 (long)d->N * HWo * std::max(ld, d->ldx));
    return false;
  }
  return true;
}

// the forward's staged channel parameters (stage_params)
size_t fwd_shm(const eegan_bnmod_desc* d) { return 4 * ((d->C + 7) / 8) * 8 * sizeof(float); }

int bwd_chunks(const eegan_bnmod_desc* d, int& ppc) {
  const long HWo = (long)(d->H << d->up2) * (d->W << d->up2);
  // aim at ~1024 blocks overall, >= 64 pixels each
  int chunks = std::max(1, std::min<int>(ee_cdiv(HWo, bn_knob("bwd_minpix", 64)),
                                         ee_cdiv(bn_knob("bwd_target", 1024), d->N)));
  ppc = ee_cdiv(HWo, chunks);
  chunks = ee_cdiv(HWo, ppc);
  return chunks;
}

}  // namespace

extern "C" {

long eegan_bn_stats_workspace(long P, int C) {
  const int C8 = (C + 7) / 8;
  const int rows = NT / C8;
  const long sb = bn_knob("stats_blocks", 1024);
  long rpb = std::max<long>(rows * 16, (P + sb - 1) / sb);
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
  const long sb = bn_knob("stats_blocks", 1024);
  long rpb = std::max<long>(rows * 16, (P + sb - 1) / sb);
  const int nblk = (int)std::max<long>(1, (P + rpb - 1) / rpb);
  const size_t shm = 2 * rows * C8 * 8 * sizeof(float);
  if (bn_knob("stats_u", 4) >= 8)
    bn_partial_kernel<8><<<nblk, NT, shm, stream>>>(x, P, C, ld, rpb, ws);
  else
    bn_partial_kernel<><<<nblk, NT, shm, stream>>>(x, P, C, ld, rpb, ws);
  int rc = ee_check_launch("bn_partial");
  if (rc) return rc;
  launch_colsum<double, double>(ws, nblk, 2 * C, 2 * C, 0, sums, 0, 1, 0, stream);
  return ee_check_launch("bn_reduce");
}

int eegan_bn_finalize(const double* sums, int C, double count, double sum_scale, float eps, float momentum,
                      int clamp_mode, float* running_mean, float* running_var, float* stats, hipStream_t stream) {
  const FinArgs f{sums, count, sum_scale, eps, momentum, clamp_mode, running_mean, running_var, stats};
  bn_finalize_kernel<<<ee_cdiv(C, 256), 256, 0, stream>>>(f, C);
  return ee_check_launch("bn_finalize");
}

int eegan_bnmod_fwd(const eegan_bnmod_desc* d, uint16_t* y, int ldy, hipStream_t stream) {
  ModArgs a = make_args(d);
  if (!vec_ok(d, ldy, y, "bnmod_fwd")) return -22;
  int ppc;
  const int chunks = pix_chunks(d->N, (long)(d->H << d->up2) * (d->W << d->up2), d->C, ppc,
                                bn_knob("fwd_target", 1536), bn_knob("fwd_prow", 8));
  // pixels whose loads a thread issues before their arithmetic (same results for any count)
  if (bn_knob("fwd_u", FUNR_DEFAULT) >= 4)
    bnmod_fwd_kernel<false, 4><<<dim3(chunks, d->N), NT, fwd_shm(d), stream>>>(a, y, ldy, ppc, FinArgs{});
  else
    bnmod_fwd_kernel<false><<<dim3(chunks, d->N), NT, fwd_shm(d), stream>>>(a, y, ldy, ppc, FinArgs{});
  return ee_check_launch("bnmod_fwd");
}

int eegan_bnmod_fwd_fin(const eegan_bnmod_desc* d, const double* sums, double count, double sum_scale, float eps,
                        float momentum, int clamp_mode, float* running_mean, float* running_var, uint16_t* y,
                        int ldy, hipStream_t stream) {
  ModArgs a = make_args(d);
  if (!vec_ok(d, ldy, y, "bnmod_fwd_fin")) return -22;
  if (!d->stats) {
    ee_set_error("bnmod_fwd_fin: the descriptor's stats buffer (written here) is missing");
    return -22;
  }
  int ppc;
  const int chunks = pix_chunks(d->N, (long)(d->H << d->up2) * (d->W << d->up2), d->C, ppc,
                                bn_knob("fwd_target", 1536), bn_knob("fwd_prow", 8));
  const FinArgs f{sums, count, sum_scale, eps, momentum, clamp_mode, running_mean, running_var,
                  const_cast<float*>(d->stats)};
  if (bn_knob("fwd_u", FUNR_DEFAULT) >= 4)
    bnmod_fwd_kernel<true, 4><<<dim3(chunks, d->N), NT, fwd_shm(d), stream>>>(a, y, ldy, ppc, f);
  else
    bnmod_fwd_kernel<true><<<dim3(chunks, d->N), NT, fwd_shm(d), stream>>>(a, y, ldy, ppc, f);
  return ee_check_launch("bnmod_fwd_fin");
}

long eegan_bnmod_bwd_workspace(const eegan_bnmod_desc* d) {
  int ppc;
  const int chunks = bwd_chunks(d, ppc);
  // chunk partials (fp32) + per-sample sums (fp64)
  return (long)d->N * chunks * 4 * d->C * (long)sizeof(float) + (long)d->N * 4 * d->C * (long)sizeof(double);
}

int eegan_bnmod_bwd(const eegan_bnmod_desc* d, const uint16_t* dt, int lddt, float* ws, float* dparam0,
                    float* dparam1, float* dmask, double* chan, hipStream_t stream) {
  ModArgs a = make_args(d);
  if (!vec_ok(d, lddt, dt, "bnmod_bwd")) return -22;
  int ppc;
  const int chunks = bwd_chunks(d, ppc);
  const int C8 = (d->C + 7) / 8;
  if (C8 > NT) {
    ee_set_error("bnmod_bwd: C too large");
    return -22;
  }
  const int rows = NT / C8;
  const size_t shm = (4 * C8 * 8 + rows * C8 + rows * (4 * C8 * 8 + 1)) * sizeof(float);
  dim3 grid(chunks, d->N);
  // pixels per thread with their loads in flight together; the per-thread pixel order, hence
  // every partial sum, is the same for any count
  if (bn_knob("red_u", RU_DEFAULT) >= 4)
    bnmod_bwd_reduce_kernel<4><<<grid, NT, shm, stream>>>(a, dt, lddt, ppc, ws, dmask, bn_knob("knock", 0));
  else
    bnmod_bwd_reduce_kernel<><<<grid, NT, shm, stream>>>(a, dt, lddt, ppc, ws, dmask, bn_knob("knock", 0));
  int rc = ee_check_launch("bnmod_bwd_reduce");
  if (rc) return rc;
  double* tmp = reinterpret_cast<double*>(ws + (long)d->N * chunks * 4 * d->C);
  launch_colsum<double, double>(ws, chunks, 4L * d->C, 4L * d->C, (long)chunks * 4 * d->C, tmp, 4L * d->C, d->N, 0,
                                stream);
  rc = ee_check_launch("bnmod_bwd_colsum");
  if (rc) return rc;
  bnmod_bwd_sums_kernel<<<ee_cdiv(4 * d->C, 256), 256, 0, stream>>>(tmp, d->N, d->C, d->mode, dparam0, dparam1, chan);
  return ee_check_launch("bnmod_bwd_sums");
}

int eegan_bnmod_bwd_dx(const eegan_bnmod_desc* d, const uint16_t* dt, int lddt, const double* chan, double count,
                       uint16_t* dx, int lddx, hipStream_t stream) {
  ModArgs a = make_args(d);
  if (!vec_ok(d, lddt, dt, "bnmod_bwd_dx") || !vec_ok(d, lddx, dx, "bnmod_bwd_dx")) return -22;
  int ppc;
  const int chunks = pix_chunks(d->N, (long)d->H * d->W, d->C, ppc, bn_knob("dx_target", 2048),
                                bn_knob("dx_prow", 8));
  const size_t dx_shm = 7 * ((d->C + 7) / 8) * 8 * sizeof(float);
  if (bn_knob("dx_u", 4) >= 8)
    bnmod_bwd_dx_kernel<8><<<dim3(chunks, d->N), NT, dx_shm, stream>>>(a, dt, lddt, chan, count, dx, lddx, ppc);
  else
    bnmod_bwd_dx_kernel<><<<dim3(chunks, d->N), NT, dx_shm, stream>>>(a, dt, lddt, chan, count, dx, lddx, ppc);
  return ee_check_launch("bnmod_bwd_dx");
}

}  // extern "C"
