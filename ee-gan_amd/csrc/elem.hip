// Memory-bound elementwise / pooling / resize / layout kernels (NHWC bf16).
//
// replaces: LeakyReLU/ReLU/Tanh/Sigmoid backward (models.py:28-30,38,
// 115-118,269-271), F.avg_pool2d(x, 2) (models.py:284), nearest-2x upsample
// (models.py:134,219), `shortcut + gamma * residual` (models.py:122,142,278),
// cond.repeat + torch.cat (models.py:302-304,327-331), F.interpolate
// bilinear (models.py:220 align_corners=True; DAMSM.py:173 align_corners=False),
// torch.sigmoid (models.py:221,232), max/avg pooling of Inception-v3
// (DAMSM.py:181-218) and the fc -> view(B, 8*ngf, 4, 4) reshape (models.py:228-230).
#include "common.h"
#include "../../include/eegan_hip.h"

namespace {

constexpr int NT = 256;

int grid_for(long work) {
  long b = (work + NT - 1) / NT;
  return (int)std::max<long>(1, std::min<long>(b, 16384));
}

#define GRID_LOOP(e, total) for (long e = blockIdx.x * (long)NT + threadIdx.x; e < (total); e += (long)gridDim.x * NT)

struct V8 {
  float v[8];
};

EE_DEV V8 load8(const bf16_t* p, int nvalid, bool vec) {
  V8 r;
  if (vec && nvalid >= 8) {
    uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r.v[2 * j] = lo_f(w[j]);
      r.v[2 * j + 1] = hi_f(w[j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) r.v[j] = j < nvalid ? bf2f(p[j]) : 0.f;
  }
  return r;
}

EE_DEV void store8(bf16_t* p, const V8& r, int nvalid, bool vec) {
  if (vec && nvalid >= 8) {
    *reinterpret_cast<uint4*>(p) = make_uint4(pack2(r.v[0], r.v[1]), pack2(r.v[2], r.v[3]), pack2(r.v[4], r.v[5]),
                                              pack2(r.v[6], r.v[7]));
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j < nvalid) p[j] = f2bf(r.v[j]);
  }
}

// dx = dy * act'(y)
__global__ void act_bwd_kernel(const bf16_t* dy, int lddy, const bf16_t* y, int ldy, long P, int C, int act,
                               float slope, bf16_t* dx, int lddx) {
  const int C8 = (C + 7) / 8;
  const bool vec = (lddy % 8 == 0) && (ldy % 8 == 0) && (lddx % 8 == 0);
  GRID_LOOP(e, P * C8) {
    const long p = e / C8;
    const int c0 = (int)(e % C8) * 8;
    const int nv = min(8, C - c0);
    V8 g = load8(dy + p * lddy + c0, nv, vec);
    V8 yy = load8(y + p * ldy + c0, nv, vec);
#pragma unroll
    for (int j = 0; j < 8; ++j) g.v[j] *= act_dgrad_from_y(yy.v[j], act, slope);
    store8(dx + p * lddx + c0, g, nv, vec);
  }
}

// out = (x ? x : 0) + alpha * (gamma ? *gamma : 1) * y
__global__ void scale_add_kernel(const bf16_t* x, int ldx, const bf16_t* y, int ldy, const float* gamma, float alpha,
                                 long P, int C, bf16_t* out, int ldo) {
  const int C8 = (C + 7) / 8;
  const bool vec = (ldx % 8 == 0) && (ldy % 8 == 0) && (ldo % 8 == 0);
  const float s = alpha * (gamma ? *gamma : 1.f);
  GRID_LOOP(e, P * C8) {
    const long p = e / C8;
    const int c0 = (int)(e % C8) * 8;
    const int nv = min(8, C - c0);
    V8 b = load8(y + p * ldy + c0, nv, vec);
    if (x) {
      V8 a = load8(x + p * ldx + c0, nv, vec);
#pragma unroll
      for (int j = 0; j < 8; ++j) b.v[j] = a.v[j] + s * b.v[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) b.v[j] *= s;
    }
    store8(out + p * ldo + c0, b, nv, vec);
  }
}

// torch.cat(parts, 1) of NHWC bf16 activations in one launch (every part's
// channel count a multiple of 8, so each 16-B output chunk has one source)
constexpr int CAT_MAX = 8;
struct CatParts {
  const bf16_t* p[CAT_MAX];
  int ld[CAT_MAX];
  int c0[CAT_MAX + 1];
  int n;
};

__global__ void cat_channels_kernel(const CatParts parts, long P, bf16_t* out, int ldo) {
  const int C8 = parts.c0[parts.n] / 8;
  GRID_LOOP(e, P * C8) {
    const long p = e / C8;
    const int c = (int)(e % C8) * 8;
    int j = 0;
    while (j + 1 < parts.n && parts.c0[j + 1] <= c) ++j;
    const uint4 v = *reinterpret_cast<const uint4*>(parts.p[j] + p * parts.ld[j] + (c - parts.c0[j]));
    *reinterpret_cast<uint4*>(out + p * ldo + c) = v;
  }
}

// partial sums of x*y (or x when y == null) per block -> ws[block]
__global__ __launch_bounds__(NT) void dot_partial_kernel(const bf16_t* x, int ldx, const bf16_t* y, int ldy, long P,
                                                         int C, float* ws) {
  __shared__ float red[16];
  const int C8 = (C + 7) / 8;
  float acc = 0.f;
  GRID_LOOP(e, P * C8) {
    const long p = e / C8;
    const int c0 = (int)(e % C8) * 8;
    const int nv = min(8, C - c0);
    V8 a = load8(x + p * ldx + c0, nv, (ldx % 8) == 0);
    if (y) {
      V8 b = load8(y + p * ldy + c0, nv, (ldy % 8) == 0);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += a.v[j] * b.v[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += a.v[j];
    }
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) ws[blockIdx.x] = acc;
}

// ScaleAdd backward in one pass over g: out = (r ? r : 0) + s * g (the
// residual-branch gradient; r = a second gradient summed into it) and the
// per-block partials of <g, h> (the gain's gradient)
__global__ __launch_bounds__(NT) void scale_dot_partial_kernel(const bf16_t* g, int ldg, const bf16_t* h, int ldh,
                                                               const float* gamma, float alpha, long P, int C,
                                                               const bf16_t* r, int ldr, bf16_t* out, int ldo,
                                                               float* ws, int act, float slope) {
  __shared__ float red[16];
  const int C8 = (C + 7) / 8;
  const bool vec = (ldg % 8 == 0) && (ldh % 8 == 0) && (ldo % 8 == 0) && (!r || ldr % 8 == 0);
  const float s = alpha * (gamma ? *gamma : 1.f);
  float acc = 0.f;
  GRID_LOOP(e, P * C8) {
    const long p = e / C8;
    const int c0 = (int)(e % C8) * 8;
    const int nv = min(8, C - c0);
    V8 a = load8(g + p * ldg + c0, nv, vec);
    V8 b = load8(h + p * ldh + c0, nv, vec);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      acc += a.v[j] * b.v[j];
      a.v[j] *= act ? s * act_dgrad_from_y(b.v[j], act, slope) : s;
    }
    if (r) {
      V8 c = load8(r + p * ldr + c0, nv, vec);
#pragma unroll
      for (int j = 0; j < 8; ++j) a.v[j] += c.v[j];
    }
    store8(out + p * ldo + c0, a, nv, vec);
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) ws[blockIdx.x] = acc;
}

// ScaleAdd's backward with the residual branch's activation gated, under create_graph
// (the gradient penalty through resD): out = (r ? r : 0) + s * act'(q) * a and, when ws
// is given, the per-block partials of <act'(q) * a, b>.  q = the activation output h
// whose derivative gates (piecewise constant: no gradient flows into it)
__global__ __launch_bounds__(NT) void scale_gate_kernel(const bf16_t* a_, int lda, const bf16_t* q_, int ldq,
                                                        const bf16_t* b_, int ldb, const float* gamma, float alpha,
                                                        long P, int C, const bf16_t* r, int ldr, bf16_t* out, int ldo,
                                                        float* ws, int act, float slope) {
  __shared__ float red[16];
  const int C8 = (C + 7) / 8;
  const bool vec = (lda % 8 == 0) && (ldq % 8 == 0) && (ldo % 8 == 0) && (!r || ldr % 8 == 0) &&
                   (!ws || ldb % 8 == 0);
  const float s = alpha * (gamma ? *gamma : 1.f);
  float acc = 0.f;
  GRID_LOOP(e, P * C8) {
    const long p = e / C8;
    const int c0 = (int)(e % C8) * 8;
    const int nv = min(8, C - c0);
    V8 a = load8(a_ + p * lda + c0, nv, vec);
    const V8 q = load8(q_ + p * ldq + c0, nv, vec);
    V8 b;
    if (ws) b = load8(b_ + p * ldb + c0, nv, vec);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float m = act_dgrad_from_y(q.v[j], act, slope);
      if (ws) acc += (a.v[j] * m) * b.v[j];
      a.v[j] *= s * m;
    }
    if (r) {
      V8 c = load8(r + p * ldr + c0, nv, vec);
#pragma unroll
      for (int j = 0; j < 8; ++j) a.v[j] += c.v[j];
    }
    store8(out + p * ldo + c0, a, nv, vec);
  }
  if (ws) {   // block-uniform
    acc = block_sum(acc, red);
    if (threadIdx.x == 0) ws[blockIdx.x] = acc;
  }
}

__global__ void dot_final_kernel(const float* ws, int n, float scale, float* out, int accumulate) {
  __shared__ float red[16];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += ws[i];
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) out[0] = accumulate ? out[0] + acc * scale : acc * scale;
}

// per-channel sum over pixels: out[c] = sum_p x[p][c]  (fp32), two-stage
__global__ __launch_bounds__(NT) void chansum_partial_kernel(const bf16_t* x, int ld, long P, int C, long rpb,
                                                             float* ws) {
  extern __shared__ float sh[];
  const int C8 = (C + 7) / 8;
  const int rows = NT / C8;
  const int t = threadIdx.x, row = t / C8, cg = t - row * C8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const long p0 = blockIdx.x * rpb, p1 = min(P, p0 + rpb);
  if (row < rows)
    for (long p = p0 + row; p < p1; p += rows) {
      V8 a = load8(x + p * ld + cg * 8, min(8, C - cg * 8), (ld % 8) == 0);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += a.v[j];
    }
  const int W8 = C8 * 8;
  if (row < rows)
#pragma unroll
    for (int j = 0; j < 8; ++j) sh[row * W8 + cg * 8 + j] = s[j];
  __syncthreads();
  for (int c = t; c < C; c += NT) {
    float a = 0.f;
    for (int r = 0; r < rows; ++r) a += sh[r * W8 + c];
    ws[(long)blockIdx.x * C + c] = a;
  }
}

// 2x2 average pool (stride 2) and its adjoint
__global__ void avgpool2_kernel(const bf16_t* x, int N, int H, int W, int C, int ld, bf16_t* y, int ldy) {
  const int Ho = H / 2, Wo = W / 2, C8 = (C + 7) / 8;
  const bool vec = (ld % 8 == 0) && (ldy % 8 == 0);
  GRID_LOOP(e, (long)N * Ho * Wo * C8) {
    const int c0 = (int)(e % C8) * 8;
    const long p = e / C8;
    const int ox = p % Wo;
    const long t = p / Wo;
    const int oy = t % Ho, n = t / Ho;
    const int nv = min(8, C - c0);
    V8 acc = {};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long ip = ((long)n * H + 2 * oy + (k >> 1)) * W + 2 * ox + (k & 1);
      V8 a = load8(x + ip * ld + c0, nv, vec);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc.v[j] += a.v[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc.v[j] *= 0.25f;
    store8(y + p * ldy + c0, acc, nv, vec);
  }
}

// mode 0: dx[hi] = dy[lo] * 0.25 (avgpool2 adjoint); mode 1: y[hi] = x[lo] (nearest up2)
__global__ void up2_kernel(const bf16_t* x, int N, int H, int W, int C, int ld, float scale, bf16_t* y, int ldy) {
  const int Ho = H * 2, Wo = W * 2, C8 = (C + 7) / 8;
  const bool vec = (ld % 8 == 0) && (ldy % 8 == 0);
  GRID_LOOP(e, (long)N * Ho * Wo * C8) {
    const int c0 = (int)(e % C8) * 8;
    const long p = e / C8;
    const int ox = p % Wo;
    const long t = p / Wo;
    const int oy = t % Ho, n = t / Ho;
    const int nv = min(8, C - c0);
    V8 a = load8(x + (((long)n * H + oy / 2) * W + ox / 2) * ld + c0, nv, vec);
#pragma unroll
    for (int j = 0; j < 8; ++j) a.v[j] *= scale;
    store8(y + p * ldy + c0, a, nv, vec);
  }
}

// nearest-up2 adjoint: y[lo] = sum of the 2x2 children of x[hi]
__global__ void sumpool2_kernel(const bf16_t* x, int N, int H, int W, int C, int ld, bf16_t* y, int ldy) {
  const int Ho = H / 2, Wo = W / 2, C8 = (C + 7) / 8;
  const bool vec = (ld % 8 == 0) && (ldy % 8 == 0);
  GRID_LOOP(e, (long)N * Ho * Wo * C8) {
    const int c0 = (int)(e % C8) * 8;
    const long p = e / C8;
    const int ox = p % Wo;
    const long t = p / Wo;
    const int oy = t % Ho, n = t / Ho;
    const int nv = min(8, C - c0);
    V8 acc = {};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long ip = ((long)n * H + 2 * oy + (k >> 1)) * W + 2 * ox + (k & 1);
      V8 a = load8(x + ip * ld + c0, nv, vec);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc.v[j] += a.v[j];
    }
    store8(y + p * ldy + c0, acc, nv, vec);
  }
}

// out[n,y,x,0:C] = feat ; out[n,y,x,C:C+E] = cond[n,:]
__global__ void cat_tile_kernel(const bf16_t* feat, int ldf, const float* cond, int N, int HW, int C, int E,
                                bf16_t* out, int ldo) {
  const int CT = C + E;
  GRID_LOOP(e, (long)N * HW * CT) {
    const int c = e % CT;
    const long p = e / CT;
    const int n = p / HW;
    out[p * ldo + c] = c < C ? feat[p * ldf + c] : f2bf(cond[(long)n * E + (c - C)]);
  }
}

// backward: dfeat = dout[..., :C];  dcond[n,e] = sum_hw dout[n,hw,C+e]
__global__ void cat_tile_bwd_kernel(const bf16_t* dout, int ldo, int N, int HW, int C, int E, bf16_t* dfeat,
                                    int ldf, float* dcond) {
  const long tf = dfeat ? (long)N * HW * C : 0;
  GRID_LOOP(e, tf + (long)N * E) {
    if (e < tf) {
      const int c = e % C;
      const long p = e / C;
      dfeat[p * ldf + c] = dout[p * ldo + c];
    } else {
      const long q = e - tf;
      const int ee = q % E, n = q / E;
      float s = 0.f;
      for (int hw = 0; hw < HW; ++hw) s += bf2f(dout[((long)n * HW + hw) * ldo + C + ee]);
      if (dcond) dcond[q] = s;
    }
  }
}

// bilinear (PyTorch semantics) on NHWC; src/dst either bf16 or fp32
EE_DEV void bil_coord(int o, int in_size, int out_size, int align, int& i0, int& i1, float& l1) {
  float src;
  if (align) {  // PyTorch: scale = (in-1)/(out-1) in fp32, src = scale * o
    const float scale = out_size > 1 ? (float)(in_size - 1) / (float)(out_size - 1) : 0.f;
    src = scale * (float)o;
  } else {
    const float scale = (float)in_size / (float)out_size;
    src = ((float)o + 0.5f) * scale - 0.5f;
    if (src < 0.f) src = 0.f;
  }
  i0 = (int)src;
  if (i0 > in_size - 1) i0 = in_size - 1;
  i1 = i0 < in_size - 1 ? i0 + 1 : i0;
  l1 = src - (float)i0;
}

EE_DEV float rd(const void* base, long idx, int f32) {
  return f32 ? reinterpret_cast<const float*>(base)[idx] : bf2f(reinterpret_cast<const bf16_t*>(base)[idx]);
}
EE_DEV void wr(void* base, long idx, int f32, float v) {
  if (f32) reinterpret_cast<float*>(base)[idx] = v;
  else reinterpret_cast<bf16_t*>(base)[idx] = f2bf(v);
}

// post: 0 none, 1 sigmoid
__global__ void bilinear_fwd_kernel(const void* x, int x_f32, int N, int H, int W, int C, int ld, int Ho, int Wo,
                                    int align, int post, void* y, int y_f32, int ldy) {
  GRID_LOOP(e, (long)N * Ho * Wo * C) {
    const int c = e % C;
    const long p = e / C;
    const int ox = p % Wo;
    const long t = p / Wo;
    const int oy = t % Ho, n = t / Ho;
    int y0, y1, x0, x1;
    float ly, lx;
    bil_coord(oy, H, Ho, align, y0, y1, ly);
    bil_coord(ox, W, Wo, align, x0, x1, lx);
    const long b = (long)n * H;
    const float v00 = rd(x, ((b + y0) * W + x0) * ld + c, x_f32), v01 = rd(x, ((b + y0) * W + x1) * ld + c, x_f32);
    const float v10 = rd(x, ((b + y1) * W + x0) * ld + c, x_f32), v11 = rd(x, ((b + y1) * W + x1) * ld + c, x_f32);
    float v = (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
    if (post == 1) v = 1.f / (1.f + __expf(-v));
    wr(y, p * ldy + c, y_f32, v);
  }
}

// first output index whose sample pair (i0, i1) can touch input i, and one past the last
EE_DEV void bil_range(int i, int in_size, int out_size, int align, int& lo, int& hi) {
  int y0, y1;
  float l;
  float scale = align ? (out_size > 1 ? (float)(in_size - 1) / (float)(out_size - 1) : 0.f)
                      : (float)in_size / (float)out_size;
  int o = scale > 0.f ? (int)((float)(i - 1) / scale) - 2 : 0;
  o = max(0, min(out_size - 1, o));
  while (o > 0) {
    bil_coord(o - 1, in_size, out_size, align, y0, y1, l);
    if (y0 < i - 1) break;
    --o;
  }
  while (o < out_size) {
    bil_coord(o, in_size, out_size, align, y0, y1, l);
    if (y0 >= i - 1) break;
    ++o;
  }
  lo = o;
  while (o < out_size) {
    bil_coord(o, in_size, out_size, align, y0, y1, l);
    if (y0 > i) break;
    ++o;
  }
  hi = o;
}

// adjoint as a gather (deterministic, no atomics): every input element sums
// the weighted output gradients of the output pixels that sampled it; dy is
// pre-scaled by the sigmoid derivative when post == 1 (y = sigmoid output).
// dx32 is [N][H][W][C] fp32.
__global__ void bilinear_bwd_kernel(const void* dy, int dy_f32, const void* y, int y_f32, int lddy, int N, int H,
                                    int W, int C, int Ho, int Wo, int align, int post, float* dx32) {
  GRID_LOOP(e, (long)N * H * W * C) {
    const int c = e % C;
    const long p = e / C;
    const int ix = p % W;
    const long t = p / W;
    const int iy = t % H, n = t / H;
    int oy0, oy1, ox0, ox1;
    bil_range(iy, H, Ho, align, oy0, oy1);
    bil_range(ix, W, Wo, align, ox0, ox1);
    float acc = 0.f;
    for (int oy = oy0; oy < oy1; ++oy) {
      int y0, y1;
      float ly;
      bil_coord(oy, H, Ho, align, y0, y1, ly);
      const float wy = (y0 == iy ? 1.f - ly : 0.f) + (y1 == iy ? ly : 0.f);
      if (wy == 0.f) continue;
      for (int ox = ox0; ox < ox1; ++ox) {
        int x0, x1;
        float lx;
        bil_coord(ox, W, Wo, align, x0, x1, lx);
        const float wx = (x0 == ix ? 1.f - lx : 0.f) + (x1 == ix ? lx : 0.f);
        if (wx == 0.f) continue;
        const long op = ((long)n * Ho + oy) * Wo + ox;
        float g = rd(dy, op * lddy + c, dy_f32);
        if (post == 1) {
          const float sg = rd(y, op * lddy + c, y_f32);
          g *= sg * (1.f - sg);
        }
        acc += g * (wy * wx);
      }
    }
    dx32[e] = acc;
  }
}

// fp32 [P][C] -> out (bf16 or f32) with stride
__global__ void convert_kernel(const float* x, long P, int C, void* y, int y_f32, int ldy) {
  GRID_LOOP(e, P * C) {
    const int c = e % C;
    const long p = e / C;
    wr(y, p * ldy + c, y_f32, x[e]);
  }
}

// NCHW fp32 <-> NHWC bf16
__global__ void nchw_to_nhwc_kernel(const float* x, int N, int C, int HW, bf16_t* y, int ldy) {
  GRID_LOOP(e, (long)N * C * HW) {
    const int c = e % C;
    const long p = e / C;
    const int hw = p % HW, n = p / HW;
    y[p * ldy + c] = f2bf(x[((long)n * C + c) * HW + hw]);
  }
}
__global__ void nhwc_to_nchw_kernel(const bf16_t* x, int ldx, int N, int C, int HW, float* y) {
  GRID_LOOP(e, (long)N * C * HW) {
    const int hw = e % HW;
    const long t = e / HW;
    const int c = t % C, n = t / C;
    y[e] = bf2f(x[((long)n * HW + hw) * ldx + c]);
  }
}

// fc output [N][C*16] (channel-major 4x4) <-> NHWC [N][16][ld]
__global__ void fc_to_nhwc_kernel(const void* x, int x_f32, int N, int C, int HW, bf16_t* y, int ldy, int reverse,
                                  void* xr, int xr_f32) {
  GRID_LOOP(e, (long)N * C * HW) {
    const int c = e % C;
    const long p = e / C;
    const int hw = p % HW, n = p / HW;
    const long src = ((long)n * C + c) * HW + hw;
    if (!reverse) y[p * ldy + c] = f2bf(rd(x, src, x_f32));
    else wr(xr, src, xr_f32, bf2f(y[p * ldy + c]));
  }
}

// 3x3 / stride-2 max pool (no padding) with argmax (0..8) and its adjoint
// 3x3 / stride-2 max pool over 8-channel groups; arg[p][c] = winning tap (first max, NaN wins)
__global__ void maxpool3s2_kernel(const bf16_t* x, int N, int H, int W, int C, int ld, int Ho, int Wo, bf16_t* y,
                                  int ldy, uint8_t* arg) {
  const int C8 = (C + 7) / 8;
  const bool vec = (ld % 8 == 0) && (ldy % 8 == 0);
  GRID_LOOP(e, (long)N * Ho * Wo * C8) {
    const int c0 = (int)(e % C8) * 8;
    const long p = e / C8;
    const int ox = p % Wo;
    const long t = p / Wo;
    const int oy = t % Ho, n = t / Ho;
    const int nv = min(8, C - c0);
    V8 best;
    int bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best.v[j] = -INFINITY;
      bi[j] = 0;
    }
    for (int k = 0; k < 9; ++k) {
      const int iy = 2 * oy + k / 3, ix = 2 * ox + k % 3;
      const V8 a = load8(x + (((long)n * H + iy) * W + ix) * ld + c0, nv, vec);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if ((a.v[j] > best.v[j] || a.v[j] != a.v[j]) && best.v[j] == best.v[j]) {
          best.v[j] = a.v[j];
          bi[j] = k;
        }
    }
    store8(y + p * ldy + c0, best, nv, vec);
    for (int j = 0; j < nv; ++j) arg[p * C + c0 + j] = (uint8_t)bi[j];
  }
}

__global__ void maxpool3s2_bwd_kernel(const bf16_t* dy, int lddy, const uint8_t* arg, int N, int H, int W, int C,
                                      int Ho, int Wo, bf16_t* dx, int lddx) {
  const int C8 = (C + 7) / 8;
  const bool vec = (lddy % 8 == 0) && (lddx % 8 == 0);
  GRID_LOOP(e, (long)N * H * W * C8) {
    const int c0 = (int)(e % C8) * 8;
    const long p = e / C8;
    const int ix = p % W;
    const long t = p / W;
    const int iy = t % H, n = t / H;
    const int nv = min(8, C - c0);
    V8 s;
#pragma unroll
    for (int j = 0; j < 8; ++j) s.v[j] = 0.f;
    const int oy_lo = max(0, (iy - 1) / 2), oy_hi = min(Ho - 1, iy / 2);
    const int ox_lo = max(0, (ix - 1) / 2), ox_hi = min(Wo - 1, ix / 2);
    for (int oy = oy_lo; oy <= oy_hi; ++oy)
      for (int ox = ox_lo; ox <= ox_hi; ++ox) {
        const int dyy = iy - 2 * oy, dxx = ix - 2 * ox;
        if (dyy < 0 || dyy > 2 || dxx < 0 || dxx > 2) continue;
        const int k = dyy * 3 + dxx;
        const long op = ((long)n * Ho + oy) * Wo + ox;
        const V8 g = load8(dy + op * lddy + c0, nv, vec);
        const uint8_t* ar = arg + op * C + c0;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j < nv && ar[j] == k) s.v[j] += g.v[j];
      }
    store8(dx + p * lddx + c0, s, nv, vec);
  }
}

// 3x3 / stride-1 / pad-1 average pool with count_include_pad (self-adjoint)
__global__ void avgpool3s1_kernel(const bf16_t* x, int N, int H, int W, int C, int ld, bf16_t* y, int ldy) {
  const int C8 = (C + 7) / 8;
  const bool vec = (ld % 8 == 0) && (ldy % 8 == 0);
  GRID_LOOP(e, (long)N * H * W * C8) {
    const int c0 = (int)(e % C8) * 8;
    const long p = e / C8;
    const int ox = p % W;
    const long t = p / W;
    const int oy = t % H, n = t / H;
    const int nv = min(8, C - c0);
    V8 acc = {};
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int iy = oy + dy, ix = ox + dx;
        if (iy < 0 || iy >= H || ix < 0 || ix >= W) continue;
        V8 a = load8(x + (((long)n * H + iy) * W + ix) * ld + c0, nv, vec);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc.v[j] += a.v[j];
      }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc.v[j] *= (1.f / 9.f);
    store8(y + p * ldy + c0, acc, nv, vec);
  }
}

// global average pool: y[n][c] (fp32 or bf16) = mean_hw x ;  adjoint: dx = dy / HW
__global__ void gap_kernel(const bf16_t* x, int ld, int N, int HW, int C, void* y, int y_f32) {
  GRID_LOOP(e, (long)N * C) {
    const int c = e % C, n = e / C;
    float s = 0.f;
    for (int i = 0; i < HW; ++i) s += bf2f(x[((long)n * HW + i) * ld + c]);
    wr(y, e, y_f32, s / (float)HW);
  }
}
__global__ void gap_bwd_kernel(const void* dy, int dy_f32, int N, int HW, int C, bf16_t* dx, int lddx) {
  GRID_LOOP(e, (long)N * HW * C) {
    const int c = e % C;
    const long p = e / C;
    const int n = p / HW;
    dx[p * lddx + c] = f2bf(rd(dy, (long)n * C + c, dy_f32) / (float)HW);
  }
}

__global__ void fill_kernel(float* x, long n, float v) {
  GRID_LOOP(e, n) x[e] = v;
}

}  // namespace

extern "C" {

int eegan_act_bwd(const uint16_t* dy, int lddy, const uint16_t* y, int ldy, long P, int C, int act, float slope,
                  uint16_t* dx, int lddx, hipStream_t s) {
  act_bwd_kernel<<<grid_for(P * ((C + 7) / 8)), NT, 0, s>>>(dy, lddy, y, ldy, P, C, act, slope, dx, lddx);
  return ee_check_launch("act_bwd");
}

int eegan_scale_add(const uint16_t* x, int ldx, const uint16_t* y, int ldy, const float* gamma, float alpha, long P,
                    int C, uint16_t* out, int ldo, hipStream_t s) {
  scale_add_kernel<<<grid_for(P * ((C + 7) / 8)), NT, 0, s>>>(x, ldx, y, ldy, gamma, alpha, P, C, out, ldo);
  return ee_check_launch("scale_add");
}

int eegan_cat_channels(const uint16_t* const* parts, const int* lds, const int* Cs, int n, long P, uint16_t* out,
                       int ldo, hipStream_t s) {
  if (n < 1 || n > CAT_MAX || (ldo % 8) || ((uintptr_t)out & 15)) {
    ee_set_error("cat_channels: %d parts (1..%d), ldo %d", n, CAT_MAX, ldo);
    return -22;
  }
  CatParts cp{};
  cp.n = n;
  for (int i = 0; i < n; ++i) {
    if ((Cs[i] % 8) || (lds[i] % 8) || ((uintptr_t)parts[i] & 15)) {
      ee_set_error("cat_channels: part %d needs C, ld multiples of 8 and 16-B alignment", i);
      return -22;
    }
    cp.p[i] = parts[i];
    cp.ld[i] = lds[i];
    cp.c0[i + 1] = cp.c0[i] + Cs[i];
  }
  cat_channels_kernel<<<grid_for(P * (cp.c0[n] / 8)), NT, 0, s>>>(cp, P, out, ldo);
  return ee_check_launch("cat_channels");
}

long eegan_dot_workspace(void) { return 1024 * sizeof(float); }

int eegan_dot(const uint16_t* x, int ldx, const uint16_t* y, int ldy, long P, int C, float scale, float* ws,
              float* out, int accumulate, hipStream_t s) {
  const int blocks = std::min(1024, grid_for(P * ((C + 7) / 8)));
  dot_partial_kernel<<<blocks, NT, 0, s>>>(x, ldx, y, ldy, P, C, ws);
  int rc = ee_check_launch("dot_partial");
  if (rc) return rc;
  dot_final_kernel<<<1, 1024, 0, s>>>(ws, blocks, scale, out, accumulate);
  return ee_check_launch("dot_final");
}

int eegan_scale_dot(const uint16_t* g, int ldg, const uint16_t* h, int ldh, const float* gamma, float alpha, long P,
                    int C, uint16_t* out, int ldo, float* ws, float* dot_out, int accumulate, int act, float slope,
                    hipStream_t s) {
  const int blocks = std::min(1024, grid_for(P * ((C + 7) / 8)));
  scale_dot_partial_kernel<<<blocks, NT, 0, s>>>(g, ldg, h, ldh, gamma, alpha, P, C, nullptr, 0, out, ldo, ws, act,
                                                 slope);
  int rc = ee_check_launch("scale_dot_partial");
  if (rc) return rc;
  dot_final_kernel<<<1, 1024, 0, s>>>(ws, blocks, 1.f, dot_out, accumulate);
  return ee_check_launch("dot_final");
}

int eegan_scale_dot_res(const uint16_t* g, int ldg, const uint16_t* h, int ldh, const float* gamma, float alpha, long P,
                        int C, const uint16_t* r, int ldr, uint16_t* out, int ldo, float* ws, float* dot_out,
                        int accumulate, hipStream_t s) {
  const int blocks = std::min(1024, grid_for(P * ((C + 7) / 8)));
  scale_dot_partial_kernel<<<blocks, NT, 0, s>>>(g, ldg, h, ldh, gamma, alpha, P, C, r, ldr, out, ldo, ws, 0, 0.f);
  int rc = ee_check_launch("scale_dot_partial");
  if (rc) return rc;
  dot_final_kernel<<<1, 1024, 0, s>>>(ws, blocks, 1.f, dot_out, accumulate);
  return ee_check_launch("dot_final");
}

int eegan_scale_gate(const uint16_t* a, int lda, const uint16_t* q, int ldq, int act, float slope, const float* gamma,
                     float alpha, long P, int C, const uint16_t* r, int ldr, const uint16_t* b, int ldb, uint16_t* out,
                     int ldo, float* ws, float* dot_out, int accumulate, hipStream_t s) {
  if (dot_out && (!ws || !b)) {
    ee_set_error("scale_gate: the dot needs b and a workspace");
    return -22;
  }
  const int blocks = std::min(1024, grid_for(P * ((C + 7) / 8)));
  scale_gate_kernel<<<blocks, NT, 0, s>>>(a, lda, q, ldq, b, ldb, gamma, alpha, P, C, r, ldr, out, ldo,
                                          dot_out ? ws : nullptr, act, slope);
  int rc = ee_check_launch("scale_gate");
  if (rc || !dot_out) return rc;
  dot_final_kernel<<<1, 1024, 0, s>>>(ws, blocks, 1.f, dot_out, accumulate);
  return ee_check_launch("dot_final");
}

long eegan_chansum_workspace(long P, int C) {
  const int rows = NT / ((C + 7) / 8);
  const long rpb = std::max<long>(rows * 8, (P + 511) / 512);
  return ((P + rpb - 1) / rpb) * (long)C * sizeof(float);
}

int eegan_chansum(const uint16_t* x, int ld, long P, int C, float* ws, float* out, int accumulate, hipStream_t s) {
  const int C8 = (C + 7) / 8;
  if (C8 > NT) {
    ee_set_error("chansum: C too large");
    return -22;
  }
  const int rows = NT / C8;
  const long rpb = std::max<long>(rows * 8, (P + 511) / 512);
  const int nblk = (int)std::max<long>(1, (P + rpb - 1) / rpb);
  chansum_partial_kernel<<<nblk, NT, rows * C8 * 8 * sizeof(float), s>>>(x, ld, P, C, rpb, ws);
  int rc = ee_check_launch("chansum_partial");
  if (rc) return rc;
  launch_colsum<float, float>(ws, nblk, C, C, 0, out, 0, 1, accumulate, s);
  return ee_check_launch("chansum_final");
}

int eegan_avgpool2(const uint16_t* x, int N, int H, int W, int C, int ld, uint16_t* y, int ldy, hipStream_t s) {
  avgpool2_kernel<<<grid_for((long)N * (H / 2) * (W / 2) * ((C + 7) / 8)), NT, 0, s>>>(x, N, H, W, C, ld, y, ldy);
  return ee_check_launch("avgpool2");
}

int eegan_upsample2(const uint16_t* x, int N, int H, int W, int C, int ld, float scale, uint16_t* y, int ldy,
                    hipStream_t s) {
  up2_kernel<<<grid_for((long)N * H * W * 4 * ((C + 7) / 8)), NT, 0, s>>>(x, N, H, W, C, ld, scale, y, ldy);
  return ee_check_launch("upsample2");
}

int eegan_sumpool2(const uint16_t* x, int N, int H, int W, int C, int ld, uint16_t* y, int ldy, hipStream_t s) {
  sumpool2_kernel<<<grid_for((long)N * (H / 2) * (W / 2) * ((C + 7) / 8)), NT, 0, s>>>(x, N, H, W, C, ld, y, ldy);
  return ee_check_launch("sumpool2");
}

int eegan_cat_tile(const uint16_t* feat, int ldf, const float* cond, int N, int HW, int C, int E, uint16_t* out,
                   int ldo, hipStream_t s) {
  cat_tile_kernel<<<grid_for((long)N * HW * (C + E)), NT, 0, s>>>(feat, ldf, cond, N, HW, C, E, out, ldo);
  return ee_check_launch("cat_tile");
}

int eegan_cat_tile_bwd(const uint16_t* dout, int ldo, int N, int HW, int C, int E, uint16_t* dfeat, int ldf,
                       float* dcond, hipStream_t s) {
  const long work = (dfeat ? (long)N * HW * C : 0) + (long)N * E;
  cat_tile_bwd_kernel<<<grid_for(work), NT, 0, s>>>(dout, ldo, N, HW, C, E, dfeat, ldf, dcond);
  return ee_check_launch("cat_tile_bwd");
}

int eegan_bilinear(const void* x, int x_f32, int N, int H, int W, int C, int ld, int Ho, int Wo, int align_corners,
                   int post, void* y, int y_f32, int ldy, hipStream_t s) {
  bilinear_fwd_kernel<<<grid_for((long)N * Ho * Wo * C), NT, 0, s>>>(x, x_f32, N, H, W, C, ld, Ho, Wo,
                                                                      align_corners, post, y, y_f32, ldy);
  return ee_check_launch("bilinear");
}

int eegan_bilinear_bwd(const void* dy, int dy_f32, const void* y, int y_f32, int lddy, int N, int H, int W, int C,
                       int Ho, int Wo, int align_corners, int post, float* dx32, hipStream_t s) {
  bilinear_bwd_kernel<<<grid_for((long)N * H * W * C), NT, 0, s>>>(dy, dy_f32, y, y_f32, lddy, N, H, W, C, Ho, Wo,
                                                                      align_corners, post, dx32);
  return ee_check_launch("bilinear_bwd");
}

int eegan_convert(const float* x, long P, int C, void* y, int y_f32, int ldy, hipStream_t s) {
  convert_kernel<<<grid_for(P * C), NT, 0, s>>>(x, P, C, y, y_f32, ldy);
  return ee_check_launch("convert");
}

int eegan_nchw_to_nhwc(const float* x, int N, int C, int HW, uint16_t* y, int ldy, hipStream_t s) {
  nchw_to_nhwc_kernel<<<grid_for((long)N * C * HW), NT, 0, s>>>(x, N, C, HW, y, ldy);
  return ee_check_launch("nchw_to_nhwc");
}

int eegan_nhwc_to_nchw(const uint16_t* x, int ldx, int N, int C, int HW, float* y, hipStream_t s) {
  nhwc_to_nchw_kernel<<<grid_for((long)N * C * HW), NT, 0, s>>>(x, ldx, N, C, HW, y);
  return ee_check_launch("nhwc_to_nchw");
}

int eegan_fc_to_nhwc(const void* x, int x_f32, int N, int C, int HW, uint16_t* y, int ldy, hipStream_t s) {
  fc_to_nhwc_kernel<<<grid_for((long)N * C * HW), NT, 0, s>>>(x, x_f32, N, C, HW, y, ldy, 0, nullptr, 0);
  return ee_check_launch("fc_to_nhwc");
}

int eegan_nhwc_to_fc(const uint16_t* y, int ldy, int N, int C, int HW, void* x, int x_f32, hipStream_t s) {
  fc_to_nhwc_kernel<<<grid_for((long)N * C * HW), NT, 0, s>>>(nullptr, 0, N, C, HW, const_cast<uint16_t*>(y), ldy, 1,
                                                               x, x_f32);
  return ee_check_launch("nhwc_to_fc");
}

int eegan_maxpool3s2(const uint16_t* x, int N, int H, int W, int C, int ld, uint16_t* y, int ldy, uint8_t* arg,
                     hipStream_t s) {
  const int Ho = (H - 3) / 2 + 1, Wo = (W - 3) / 2 + 1;
  maxpool3s2_kernel<<<grid_for((long)N * Ho * Wo * ((C + 7) / 8)), NT, 0, s>>>(x, N, H, W, C, ld, Ho, Wo, y, ldy, arg);
  return ee_check_launch("maxpool3s2");
}

int eegan_maxpool3s2_bwd(const uint16_t* dy, int lddy, const uint8_t* arg, int N, int H, int W, int C, uint16_t* dx,
                         int lddx, hipStream_t s) {
  const int Ho = (H - 3) / 2 + 1, Wo = (W - 3) / 2 + 1;
  maxpool3s2_bwd_kernel<<<grid_for((long)N * H * W * ((C + 7) / 8)), NT, 0, s>>>(dy, lddy, arg, N, H, W, C, Ho, Wo, dx, lddx);
  return ee_check_launch("maxpool3s2_bwd");
}

int eegan_avgpool3s1(const uint16_t* x, int N, int H, int W, int C, int ld, uint16_t* y, int ldy, hipStream_t s) {
  avgpool3s1_kernel<<<grid_for((long)N * H * W * ((C + 7) / 8)), NT, 0, s>>>(x, N, H, W, C, ld, y, ldy);
  return ee_check_launch("avgpool3s1");
}

int eegan_global_avgpool(const uint16_t* x, int ld, int N, int HW, int C, void* y, int y_f32, hipStream_t s) {
  gap_kernel<<<grid_for((long)N * C), NT, 0, s>>>(x, ld, N, HW, C, y, y_f32);
  return ee_check_launch("global_avgpool");
}

int eegan_global_avgpool_bwd(const void* dy, int dy_f32, int N, int HW, int C, uint16_t* dx, int lddx, hipStream_t s) {
  gap_bwd_kernel<<<grid_for((long)N * HW * C), NT, 0, s>>>(dy, dy_f32, N, HW, C, dx, lddx);
  return ee_check_launch("global_avgpool_bwd");
}

// device time stamp (100 MHz constant clock) for phase timing inside captured graphs
__global__ void stamp_kernel(unsigned long long* slot) {
  if (threadIdx.x == 0) *slot = wall_clock64();
}

int eegan_stamp(unsigned long long* slot, hipStream_t s) {
  stamp_kernel<<<1, 64, 0, s>>>(slot);
  return ee_check_launch("stamp");
}

int eegan_fill_f32(float* x, long n, float v, hipStream_t s) {
  fill_kernel<<<grid_for(n), NT, 0, s>>>(x, n, v);
  return ee_check_launch("fill_f32");
}

}  // extern "C"
