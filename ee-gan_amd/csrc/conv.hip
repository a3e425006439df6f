// Implicit-GEMM direct convolutions for gfx950 (bf16 MFMA 16x16x32, fp32 acc).
//
// Activations are NHWC bf16 with a channel stride `ld` (== C, or C rounded up
// to 8 for C >= 8).  No im2col is materialised: every B-operand tile is
// gathered straight from the activation tensor into LDS.
//
//   FWD  : y[p, co]  = sum_{r,s,c} x[gather_fwd(p,r,s), c] * W[co,r,s,c]
//   BWDD : dx[p, ci] = sum_{r,s,co} dy[gather_bwd(p,r,s), co] * W[co,ci,r,s]
//   WGRAD: dW[co, (r,s,c)] = sum_p dy[p, co] * x[gather_fwd(p,r,s), c]
//
// GEMM orientation: MFMA rows = output channels (A operand = packed weights),
// MFMA cols = pixels (B operand = gathered activations), so every lane of the
// accumulator owns 4 consecutive channels of one pixel -> 8-byte NHWC stores.
// Replaces every nn.Conv2d of models.py:14-403 and DAMSM.py.
#include "common.h"
#include "../../include/eegan_hip.h"

namespace {

constexpr int BK = 32;       // K per LDS stage (= one 16x16x32 MFMA)
constexpr int LDS_PAD = 8;   // bf16 elements of row padding (16 B)
constexpr int KROW = BK + LDS_PAD;

enum { MODE_FWD = 0, MODE_BWDD = 1 };

struct ConvArgs {
  const bf16_t* src;   // FWD: x ; BWDD: dy
  const bf16_t* wp;    // packed weights [rows_pad][Kpad]
  const float* bias;   // per output channel (FWD) or null
  const bf16_t* res;   // residual (FWD): out = res + gamma * act(acc + bias)
  const float* gamma;  // device scalar
  void* out;
  int ldres, ldo, out_f32, act;
  float slope;
  // source tensor (x for FWD, dy for BWDD)
  int N, IH, IW, lds_src;  // logical grid of the source (FWD up2: physical IH/2 x IW/2)
  int up2;
  // pixel grid of the GEMM columns
  int OH, OW;
  int R, S, st, ph, pw;
  int Cg, Cvalid;  // gathered channels (padded to 8 when vectorised) / valid channels
  int Mrows;       // valid output channels
  int P;           // N*OH*OW
  int K, Kpad;     // R*S*Cg, round_up(K, BK)
};

// ---------------------------------------------------------------- gathers --
template <int MODE>
EE_DEV bool gather_addr(const ConvArgs& a, int n, int oy, int ox, int r, int s, long& off) {
  if (MODE == MODE_FWD) {
    const int iy = oy * a.st - a.ph + r, ix = ox * a.st - a.pw + s;
    if ((unsigned)iy >= (unsigned)a.IH || (unsigned)ix >= (unsigned)a.IW) return false;
    const int PH = a.IH >> a.up2, PW = a.IW >> a.up2;
    off = ((long)(n * PH + (iy >> a.up2)) * PW + (ix >> a.up2)) * a.lds_src;
    return true;
  } else {
    const int ty = oy + a.ph - r, tx = ox + a.pw - s;
    if (ty < 0 || tx < 0) return false;
    const int qy = ty / a.st, qx = tx / a.st;
    if (qy * a.st != ty || qx * a.st != tx) return false;
    if (qy >= a.IH || qx >= a.IW) return false;
    off = ((long)(n * a.IH + qy) * a.IW + qx) * a.lds_src;
    return true;
  }
}

// load an 8-element k-chunk of the gathered operand for one pixel
template <int MODE, bool VEC>
EE_DEV uint4 gather_chunk(const ConvArgs& a, bool pvalid, int n, int oy, int ox, int k) {
  uint4 v = make_uint4(0, 0, 0, 0);
  if (!pvalid) return v;
  if (VEC) {
    if (k >= a.K) return v;
    const int rs = k / a.Cg, c = k - rs * a.Cg;
    const int r = rs / a.S, s = rs - r * a.S;
    long off;
    if (!gather_addr<MODE>(a, n, oy, ox, r, s, off)) return v;
    v = *reinterpret_cast<const uint4*>(a.src + off + c);
    if (c + 8 > a.Cvalid) {  // zero the padded channels (their storage is undefined)
      uint32_t* w = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c0 = c + 2 * j;
        if (c0 >= a.Cvalid) w[j] = 0;
        else if (c0 + 1 >= a.Cvalid) w[j] &= 0xffffu;
      }
    }
    return v;
  } else {
    uint16_t e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      e[j] = 0;
      const int kk = k + j;
      if (kk < a.K) {
        const int rs = kk / a.Cg, c = kk - rs * a.Cg;
        const int r = rs / a.S, s = rs - r * a.S;
        long off;
        if (gather_addr<MODE>(a, n, oy, ox, r, s, off)) e[j] = a.src[off + c];
      }
    }
    v.x = e[0] | ((uint32_t)e[1] << 16);
    v.y = e[2] | ((uint32_t)e[3] << 16);
    v.z = e[4] | ((uint32_t)e[5] << 16);
    v.w = e[6] | ((uint32_t)e[7] << 16);
    return v;
  }
}

EE_DEV bf16x8_t as_frag(uint4 v) { return __builtin_bit_cast(bf16x8_t, v); }

// ------------------------------------------------------- FWD / BWDD kernel --
template <int MODE, bool VEC, int TCO, int TPIX, int WCO>
__global__ __launch_bounds__(256) void conv_igemm_kernel(ConvArgs a) {
  constexpr int WPIX = 4 / WCO;
  constexpr int WT_CO = TCO / WCO, WT_PIX = TPIX / WPIX;
  constexpr int FI = WT_CO / 16, FJ = WT_PIX / 16;
  constexpr int A_CHUNKS = TCO * (BK / 8);     // 16-B chunks per A stage
  constexpr int B_CHUNKS = TPIX * (BK / 8);
  constexpr int A_PER = (A_CHUNKS + 255) / 256;
  constexpr int B_PER = B_CHUNKS / 256;
  static_assert(B_CHUNKS % 256 == 0, "pixel tile");

  __shared__ __attribute__((aligned(16))) bf16_t lds_a[2][TCO * KROW];
  __shared__ __attribute__((aligned(16))) bf16_t lds_b[2][TPIX * KROW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = wave / WPIX, wj = wave % WPIX;
  const int pix0 = blockIdx.x * TPIX, co0 = blockIdx.y * TCO;

  // per-thread fixed B rows (pixels) and k-chunk
  const int b_kc = tid & 3;
  int b_n[B_PER], b_y[B_PER], b_x[B_PER];
  bool b_ok[B_PER];
#pragma unroll
  for (int i = 0; i < B_PER; ++i) {
    const int row = (tid >> 2) + i * 64;
    const int p = pix0 + row;
    b_ok[i] = p < a.P;
    const int pp = b_ok[i] ? p : 0;
    const int hw = a.OH * a.OW;
    b_n[i] = pp / hw;
    const int rem = pp - b_n[i] * hw;
    b_y[i] = rem / a.OW;
    b_x[i] = rem - b_y[i] * a.OW;
  }

  uint4 ra[A_PER], rb[B_PER];
  auto load_stage = [&](int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int ch = tid + i * 256;
      if (ch < A_CHUNKS) {
        const int row = ch >> 2, kc = ch & 3;
        ra[i] = *reinterpret_cast<const uint4*>(a.wp + (long)(co0 + row) * a.Kpad + k0 + kc * 8);
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i)
      rb[i] = gather_chunk<MODE, VEC>(a, b_ok[i], b_n[i], b_y[i], b_x[i], k0 + b_kc * 8);
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int ch = tid + i * 256;
      if (ch < A_CHUNKS) {
        const int row = ch >> 2, kc = ch & 3;
        *reinterpret_cast<uint4*>(&lds_a[buf][row * KROW + kc * 8]) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int row = (tid >> 2) + i * 64;
      *reinterpret_cast<uint4*>(&lds_b[buf][row * KROW + b_kc * 8]) = rb[i];
    }
  };

  f32x4_t acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = a.Kpad / BK;
  load_stage(0);
  store_stage(0);
  __syncthreads();
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load_stage(kt + 1);
    bf16x8_t fa[FI], fb[FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i)
      fa[i] = as_frag(*reinterpret_cast<const uint4*>(&lds_a[buf][(wi * WT_CO + i * 16 + fr) * KROW + fk]));
#pragma unroll
    for (int j = 0; j < FJ; ++j)
      fb[j] = as_frag(*reinterpret_cast<const uint4*>(&lds_b[buf][(wj * WT_PIX + j * 16 + fr) * KROW + fk]));
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    if (kt + 1 < nk) store_stage(buf ^ 1);
    __syncthreads();
  }

  // ------------------------------------------------------------ epilogue --
  const float gam = a.res ? *a.gamma : 1.f;
#pragma unroll
  for (int i = 0; i < FI; ++i) {
    const int co = co0 + wi * WT_CO + i * 16 + (lane >> 4) * 4;
    if (co >= a.Mrows) continue;
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = (a.bias && co + r < a.Mrows) ? a.bias[co + r] : 0.f;
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int p = pix0 + wj * WT_PIX + j * 16 + fr;
      if (p >= a.P) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = act_fwd(acc[i][j][r] + bv[r], a.act, a.slope);
      if (a.res) {
        const bf16_t* rp = a.res + (long)p * a.ldres + co;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (co + r < a.Mrows) v[r] = bf2f(rp[r]) + gam * v[r];
      }
      if (a.out_f32) {
        float* op = reinterpret_cast<float*>(a.out) + (long)p * a.ldo + co;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (co + r < a.Mrows) op[r] = v[r];
      } else {
        bf16_t* op = reinterpret_cast<bf16_t*>(a.out) + (long)p * a.ldo + co;
        if (co + 4 <= a.Mrows && ((a.ldo & 3) == 0)) {
          *reinterpret_cast<uint2*>(op) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (co + r < a.Mrows) op[r] = f2bf(v[r]);
        }
      }
    }
  }
}

// ---------------------------------------------------------- WGRAD kernel --
struct WgradArgs {
  ConvArgs g;          // gather geometry of x (MODE_FWD), K = R*S*Cg
  const bf16_t* dy;    // [P][lddy]
  int lddy, Cout;
  float* ws;           // [nsplit][Cout][K]
  int p_per_split;
};

constexpr int TRP = 4;  // row padding (elements) for transposed-read tiles

template <bool VECX, bool VECDY, int TCO, int TK, int WCO>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradArgs w) {
  constexpr int WKK = 4 / WCO;
  constexpr int WT_CO = TCO / WCO, WT_K = TK / WKK;
  constexpr int FI = WT_CO / 16, FJ = WT_K / 16;
  constexpr int DROW = TCO + TRP, XROW = TK + TRP;
  constexpr int D_CHUNKS = BK * TCO / 8, X_CHUNKS = BK * TK / 8;
  constexpr int D_PER = (D_CHUNKS + 255) / 256, X_PER = (X_CHUNKS + 255) / 256;

  __shared__ __attribute__((aligned(16))) bf16_t lds_d[2][BK * DROW];
  __shared__ __attribute__((aligned(16))) bf16_t lds_x[2][BK * XROW];

  const ConvArgs& a = w.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = wave / WKK, wj = wave % WKK;
  const int co0 = blockIdx.y * TCO, kb0 = blockIdx.x * TK;
  const int p_begin = blockIdx.z * w.p_per_split;
  const int p_end = min(a.P, p_begin + w.p_per_split);
  const int hw = a.OH * a.OW;

  uint2 rd[D_PER][2];
  uint4 rx[X_PER];
  auto load_stage = [&](int p0) {
#pragma unroll
    for (int i = 0; i < D_PER; ++i) {
      const int ch = tid + i * 256;
      if (ch < D_CHUNKS) {
        const int pr = ch / (TCO / 8), cc = ch % (TCO / 8);
        const int p = p0 + pr, co = co0 + cc * 8;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (p < p_end) {
          const bf16_t* src = w.dy + (long)p * w.lddy + co;
          if (VECDY && co + 8 <= w.Cout) {
            v = *reinterpret_cast<const uint4*>(src);
          } else {
            uint16_t e[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) e[j] = (co + j < w.Cout) ? src[j] : 0;
            v = make_uint4(e[0] | ((uint32_t)e[1] << 16), e[2] | ((uint32_t)e[3] << 16),
                           e[4] | ((uint32_t)e[5] << 16), e[6] | ((uint32_t)e[7] << 16));
          }
        }
        rd[i][0] = make_uint2(v.x, v.y);
        rd[i][1] = make_uint2(v.z, v.w);
      }
    }
#pragma unroll
    for (int i = 0; i < X_PER; ++i) {
      const int ch = tid + i * 256;
      if (ch < X_CHUNKS) {
        const int pr = ch / (TK / 8), kc = ch % (TK / 8);
        const int p = p0 + pr;
        const bool ok = p < p_end;
        const int pp = ok ? p : 0;
        const int n = pp / hw, rem = pp - n * hw;
        const int y = rem / a.OW, x = rem - y * a.OW;
        rx[i] = gather_chunk<MODE_FWD, VECX>(a, ok, n, y, x, kb0 + kc * 8);
      }
    }
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int i = 0; i < D_PER; ++i) {
      const int ch = tid + i * 256;
      if (ch < D_CHUNKS) {
        const int pr = ch / (TCO / 8), cc = ch % (TCO / 8);
        uint2* dst = reinterpret_cast<uint2*>(&lds_d[buf][pr * DROW + cc * 8]);
        dst[0] = rd[i][0];
        dst[1] = rd[i][1];
      }
    }
#pragma unroll
    for (int i = 0; i < X_PER; ++i) {
      const int ch = tid + i * 256;
      if (ch < X_CHUNKS) {
        const int pr = ch / (TK / 8), kc = ch % (TK / 8);
        uint2* dst = reinterpret_cast<uint2*>(&lds_x[buf][pr * XROW + kc * 8]);
        dst[0] = make_uint2(rx[i].x, rx[i].y);
        dst[1] = make_uint2(rx[i].z, rx[i].w);
      }
    }
  };

  f32x4_t acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp4 = (li & 3) * 4;
  typedef __attribute__((address_space(3))) s16x4_t lds_s4;
  auto tr_frag = [&](const bf16_t* base, int row_stride, int col) -> bf16x8_t {
    const bf16_t* p0 = base + (8 * g + q) * row_stride + col + pp4;
    const bf16_t* p1 = p0 + 4 * row_stride;
    s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p0));
    s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p1));
    typedef __attribute__((ext_vector_type(8))) short s16x8_t;
    s16x8_t v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  };

  if (p_begin < p_end) {
    load_stage(p_begin);
    store_stage(0);
    __syncthreads();
    int buf = 0;
    for (int p0 = p_begin; p0 < p_end; p0 += BK) {
      const bool more = p0 + BK < p_end;
      if (more) load_stage(p0 + BK);
      bf16x8_t fa[FI], fb[FJ];
#pragma unroll
      for (int i = 0; i < FI; ++i) fa[i] = tr_frag(lds_d[buf], DROW, wi * WT_CO + i * 16);
#pragma unroll
      for (int j = 0; j < FJ; ++j) fb[j] = tr_frag(lds_x[buf], XROW, wj * WT_K + j * 16);
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      if (more) store_stage(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }
  float* ws = w.ws + (long)blockIdx.z * w.Cout * a.K;
#pragma unroll
  for (int i = 0; i < FI; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + wi * WT_CO + i * 16 + g * 4 + r;
      if (co >= w.Cout) continue;
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int k = kb0 + wj * WT_K + j * 16 + li;
        if (k < a.K) ws[(long)co * a.K + k] = acc[i][j][r];
      }
    }
  }
}

// sum the split slabs and scatter into the torch layout [Cout][Cin][R][S] (fp32)
__global__ void wgrad_reduce_kernel(const float* ws, int nsplit, int Cout, int Cin, int R, int S,
                                    int Cg, int K, float* dw, int accumulate) {
  const long total = (long)Cout * Cin * R * S;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int s = e % S;
    long t = e / S;
    const int r = t % R;
    t /= R;
    const int c = t % Cin;
    const int co = t / Cin;
    const long k = (long)(r * S + s) * Cg + c;
    float acc = 0.f;
    for (int z = 0; z < nsplit; ++z) acc += ws[((long)z * Cout + co) * K + k];
    dw[e] = accumulate ? dw[e] + acc : acc;
  }
}

// ------------------------------------------------------- weight packing --
// FWD pack:  out[co][(r*S+s)*Cg + c] = W[co][c][r][s] * scale[co]   (zero pad)
// BWDD pack: out[ci][(r*S+s)*Cg + co] = W[co][ci][r][s]
__global__ void pack_weights_kernel(const float* w, const float* scale, int Cout, int Cin, int R, int S,
                                    int transposed, int Cg, int rows_pad, int Kpad, bf16_t* out) {
  const long total = (long)rows_pad * Kpad;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int row = e / Kpad, k = e % Kpad;
    float v = 0.f;
    const int rs = k / Cg, c = k - rs * Cg;
    if (rs < R * S) {
      const int r = rs / S, s = rs - r * S;
      if (!transposed) {
        if (row < Cout && c < Cin) v = w[(((long)row * Cin + c) * R + r) * S + s] * (scale ? scale[row] : 1.f);
      } else {
        if (row < Cin && c < Cout) v = w[(((long)c * Cin + row) * R + r) * S + s] * (scale ? scale[c] : 1.f);
      }
    }
    out[e] = f2bf(v);
  }
}

// ------------------------------------------------------------ dispatch --
int gather_channels(int C, int ld) { return (C >= 8 && (ld % 8) == 0) ? ee_round_up(C, 8) : C; }
bool vec_ok(int C, int ld) { return C >= 8 && (ld % 8) == 0 && ld >= ee_round_up(C, 8); }

template <int MODE, bool VEC>
int launch_igemm(const ConvArgs& a, hipStream_t s) {
  const int rows = a.Mrows;
  if (rows > 64) {
    dim3 grid(ee_cdiv(a.P, 128), ee_cdiv(rows, 128));
    conv_igemm_kernel<MODE, VEC, 128, 128, 2><<<grid, 256, 0, s>>>(a);
  } else if (rows > 32) {
    dim3 grid(ee_cdiv(a.P, 128), ee_cdiv(rows, 64));
    conv_igemm_kernel<MODE, VEC, 64, 128, 2><<<grid, 256, 0, s>>>(a);
  } else if (rows > 16) {
    dim3 grid(ee_cdiv(a.P, 256), ee_cdiv(rows, 32));
    conv_igemm_kernel<MODE, VEC, 32, 256, 1><<<grid, 256, 0, s>>>(a);
  } else {
    dim3 grid(ee_cdiv(a.P, 256), ee_cdiv(rows, 16));
    conv_igemm_kernel<MODE, VEC, 16, 256, 1><<<grid, 256, 0, s>>>(a);
  }
  return ee_check_launch(MODE == MODE_FWD ? "conv_fwd" : "conv_bwd_data");
}

}  // namespace

extern "C" {

long eegan_conv_packed_elems(int Cout, int Cin, int R, int S, int transposed, int Cg) {
  const int rows = transposed ? Cin : Cout;
  return (long)ee_round_up(rows, 128) * ee_round_up(R * S * Cg, BK);
}

int eegan_conv_gather_channels(int C, int ld) { return gather_channels(C, ld); }

int eegan_conv_pack_weights(const float* w, const float* scale, int Cout, int Cin, int R, int S,
                            int transposed, int Cg, bf16_t* out, hipStream_t stream) {
  const int rows = transposed ? Cin : Cout;
  const int rows_pad = ee_round_up(rows, 128), Kpad = ee_round_up(R * S * Cg, BK);
  const long total = (long)rows_pad * Kpad;
  const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
  pack_weights_kernel<<<blocks, 256, 0, stream>>>(w, scale, Cout, Cin, R, S, transposed, Cg, rows_pad, Kpad, out);
  return ee_check_launch("pack_weights");
}

static void fill_geom(ConvArgs& a, const eegan_conv_desc* d) {
  a.R = d->R;
  a.S = d->S;
  a.st = d->stride;
  a.ph = d->pad_h;
  a.pw = d->pad_w;
}

int eegan_conv_fwd(const eegan_conv_desc* d, const bf16_t* x, const bf16_t* wpack, const float* bias, int act,
                   float slope, const bf16_t* res, int ldres, const float* gamma, void* y, int y_f32,
                   hipStream_t stream) {
  ConvArgs a = {};
  a.src = x;
  a.wp = wpack;
  a.bias = bias;
  a.res = res;
  a.ldres = ldres;
  a.gamma = gamma;
  a.out = y;
  a.ldo = d->ldy;
  a.out_f32 = y_f32;
  a.act = act;
  a.slope = slope;
  a.N = d->N;
  a.IH = d->H;
  a.IW = d->W;
  a.lds_src = d->ldx;
  a.up2 = d->up2;
  a.OH = d->Ho;
  a.OW = d->Wo;
  fill_geom(a, d);
  a.Cvalid = d->C;
  a.Cg = gather_channels(d->C, d->ldx);
  a.Mrows = d->K;
  a.P = d->N * d->Ho * d->Wo;
  a.K = d->R * d->S * a.Cg;
  a.Kpad = ee_round_up(a.K, BK);
  if (a.P == 0) return 0;
  if (res && !gamma) {
    ee_set_error("conv_fwd: residual without gamma");
    return -22;
  }
  return vec_ok(d->C, d->ldx) ? launch_igemm<MODE_FWD, true>(a, stream) : launch_igemm<MODE_FWD, false>(a, stream);
}

int eegan_conv_bwd_data(const eegan_conv_desc* d, const bf16_t* dy, const bf16_t* wpackT, void* dx, int lddx,
                        int dx_f32, hipStream_t stream) {
  if (d->up2) {
    ee_set_error("conv_bwd_data: up2 inputs take the hi-res gradient + sum-pool path");
    return -22;
  }
  ConvArgs a = {};
  a.src = dy;
  a.wp = wpackT;
  a.out = dx;
  a.ldo = lddx;
  a.out_f32 = dx_f32;
  a.act = ACT_NONE;
  a.N = d->N;
  a.IH = d->Ho;  // source grid = dy grid
  a.IW = d->Wo;
  a.lds_src = d->ldy;
  a.up2 = 0;
  a.OH = d->H;   // GEMM pixels = input pixels
  a.OW = d->W;
  fill_geom(a, d);
  a.Cvalid = d->K;
  a.Cg = gather_channels(d->K, d->ldy);
  a.Mrows = d->C;
  a.P = d->N * d->H * d->W;
  a.K = d->R * d->S * a.Cg;
  a.Kpad = ee_round_up(a.K, BK);
  if (a.P == 0) return 0;
  return vec_ok(d->K, d->ldy) ? launch_igemm<MODE_BWDD, true>(a, stream) : launch_igemm<MODE_BWDD, false>(a, stream);
}

static void wgrad_plan(const eegan_conv_desc* d, int& TCO, int& TK, int& nsplit, int& pps, int& K) {
  const int Cg = gather_channels(d->C, d->ldx);
  K = d->R * d->S * Cg;
  TCO = d->K > 64 ? 128 : (d->K > 16 ? 64 : 16);
  TK = 128;
  const int P = d->N * d->Ho * d->Wo;
  const int tiles = ee_cdiv(d->K, TCO) * ee_cdiv(K, TK);
  int want = std::max(1, 1024 / std::max(tiles, 1));
  const int maxsplit = std::max(1, ee_cdiv(P, 256));
  nsplit = std::min(want, maxsplit);
  pps = ee_round_up(ee_cdiv(P, nsplit), BK);
  nsplit = ee_cdiv(P, pps);
}

long eegan_conv_wgrad_workspace(const eegan_conv_desc* d) {
  int TCO, TK, nsplit, pps, K;
  wgrad_plan(d, TCO, TK, nsplit, pps, K);
  return (long)nsplit * d->K * K * (long)sizeof(float);
}

int eegan_conv_bwd_weight(const eegan_conv_desc* d, const bf16_t* x, const bf16_t* dy, float* ws, float* dw,
                          int accumulate, hipStream_t stream) {
  int TCO, TK, nsplit, pps, K;
  wgrad_plan(d, TCO, TK, nsplit, pps, K);
  WgradArgs w = {};
  ConvArgs& a = w.g;
  a.src = x;
  a.N = d->N;
  a.IH = d->H;
  a.IW = d->W;
  a.lds_src = d->ldx;
  a.up2 = d->up2;
  a.OH = d->Ho;
  a.OW = d->Wo;
  fill_geom(a, d);
  a.Cvalid = d->C;
  a.Cg = gather_channels(d->C, d->ldx);
  a.P = d->N * d->Ho * d->Wo;
  a.K = K;
  w.dy = dy;
  w.lddy = d->ldy;
  w.Cout = d->K;
  w.ws = ws;
  w.p_per_split = pps;
  if (a.P > 0) {
    dim3 grid(ee_cdiv(K, TK), ee_cdiv(d->K, TCO), nsplit);
    const bool vx = vec_ok(d->C, d->ldx);
    const bool vd = (d->ldy % 8) == 0;
#define WG_LAUNCH(VX, VD)                                                              \
  if (TCO == 128) conv_wgrad_kernel<VX, VD, 128, 128, 2><<<grid, 256, 0, stream>>>(w); \
  else if (TCO == 64) conv_wgrad_kernel<VX, VD, 64, 128, 2><<<grid, 256, 0, stream>>>(w); \
  else conv_wgrad_kernel<VX, VD, 16, 128, 1><<<grid, 256, 0, stream>>>(w);
    if (vx && vd) { WG_LAUNCH(true, true) }
    else if (vx) { WG_LAUNCH(true, false) }
    else if (vd) { WG_LAUNCH(false, true) }
    else { WG_LAUNCH(false, false) }
#undef WG_LAUNCH
    int rc = ee_check_launch("conv_wgrad");
    if (rc) return rc;
  } else {
    nsplit = 0;
  }
  const long total = (long)d->K * d->C * d->R * d->S;
  const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
  wgrad_reduce_kernel<<<blocks, 256, 0, stream>>>(ws, nsplit, d->K, d->C, d->R, d->S, a.Cg, K, dw, accumulate);
  return ee_check_launch("wgrad_reduce");
}

}  // extern "C"
