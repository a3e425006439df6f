// Prototype: 3x3 stride-1 pad-1 implicit-GEMM conv with an LDS halo tile
// (diagnostic probe, not part of libeegan_hip.so).  One workgroup owns TCO
// output channels x a TH x TW pixel tile of one image.  Per 32-channel input
// slice the (TH+2) x (TW+2) source halo is staged ONCE in LDS (LDS-DMA) and
// serves all 9 taps; the weights stream per tap through a 3-slot ring.  K
// order: slice-major, tap inner.
#include "../../ee-gan_amd/csrc/common.h"

namespace {

typedef __attribute__((ext_vector_type(4))) int rsrc_t;
typedef __attribute__((address_space(3))) void lds_void_t;
constexpr unsigned OOB = 0x80000000u;

EE_DEV rsrc_t make_rsrc(const void* p, long bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  rsrc_t r;
  r.x = (int)(uint32_t)a;
  r.y = (int)((a >> 32) & 0xffffu);
  r.z = (int)min(bytes, 0x7fffffffL);
  r.w = 0x00020000;
  return r;
}
EE_DEV int swz_b128(int b) { return (0x1320 >> (b * 4)) & 3; }
EE_DEV bf16x8_t as_frag(uint4 v) { return __builtin_bit_cast(bf16x8_t, v); }

#pragma clang diagnostic ignored "-Winline-asm"
EE_DEV void dma16(rsrc_t rsrc, int lds_addr, unsigned voff) {
  lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(lds_addr), "v"(voff), "s"(rsrc)
               : "memory", "m0");
}
template <int N>
EE_DEV void wait_vmcnt_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

struct HaloArgs {
  const bf16_t* src;  // NHWC [N][H][W][ld]
  const bf16_t* wp;   // packed [rows_pad][Kw], Kw = 9 * Cgp
  const float* bias;
  bf16_t* out;        // NHWC [N][H][W][ldo]
  int N, H, W, ld, C, Cgp, K, Kw, ldo, act;
  float slope;
  long src_bytes, w_bytes;
  int knock;   // diagnostics: 1 no DMA in the loop, 2 no epilogue, 4 no MFMA, 8 no barrier/wait
};

// halo pixel h's 16-B chunk q lives in LDS slot h*4 + (q ^ g(h)), g(h) = (h >> 1) & 2:
// conflict-free ds_read_b128 for any 16 consecutive halo pixels (every tap shift)
EE_DEV int hswz(int h) { return (h >> 1) & 2; }

template <int MODE, int TCO, int WCO, int WPX, int TH, int TW>
__global__ __launch_bounds__(64 * WCO * WPX, (64 * WCO * WPX <= 256 ? 2 : 1)) void halo_conv_kernel(HaloArgs a) {
  constexpr int NT = 64 * WCO * WPX;
  constexpr int WT_CO = TCO / WCO, FI = WT_CO / 16;
  constexpr int WROWS = TH / WPX, CB = TW / 16, FJ = WROWS * CB;
  constexpr int HW_ = TW + 2, HP = (TH + 2) * HW_, HCH = HP * 4;
  constexpr int HOPS = (HCH + NT - 1) / NT;            // halo DMA ops per thread per slice
  constexpr int HBUF = HOPS * NT * 16;                  // bytes per halo buffer
  constexpr int WOPS = TCO * 4 >= NT ? TCO * 4 / NT : 1;  // weight DMA ops per thread per tap
  constexpr int WBUF = TCO * 64;                        // bytes per weight stage
  constexpr int RING = 3;
  static_assert((WOPS * NT == TCO * 4 || (TCO * 4 < NT && TCO * 4 % 64 == 0)) && FI >= 1 && FJ >= 1, "tile");
  static_assert(HOPS <= 7, "halo ops must be issued (one per tap) before the last two taps of a slice");
  __shared__ __attribute__((aligned(16))) char lds[2 * HBUF + RING * WBUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wave / WPX, wj = wave % WPX;
  const int tiles_x = a.W / TW, tiles_y = a.H / TH;
  int b = blockIdx.x;
  const int tx = b % tiles_x;
  b /= tiles_x;
  const int ty = b % tiles_y;
  const int n = b / tiles_y;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int co0 = blockIdx.y * TCO;
  const int nslice = a.Cgp / 32;
  const int lds0 = (int)(uintptr_t)(lds_void_t*)lds;
  const int hb0 = lds0, wb0 = lds0 + 2 * HBUF;
  const bool w_wave = TCO * 4 >= NT || tid < TCO * 4;   // wave-uniform: waves that stage weight pieces

  const rsrc_t rs_src = make_rsrc(a.src, a.src_bytes);
  const rsrc_t rs_w = make_rsrc(a.wp, a.w_bytes);

  // this thread's halo pieces: byte offset of its chunk at slice 0 (OOB outside the image)
  unsigned hoff[HOPS];
  int hq[HOPS];
#pragma unroll
  for (int i = 0; i < HOPS; ++i) {
    const int L = i * NT + tid;
    const int h = L >> 2;
    const int q = (L & 3) ^ hswz(h);
    const int hy = h / HW_, hx = h - hy * HW_;
    const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
    hq[i] = q;
    hoff[i] = (h < HP && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
                  ? (unsigned)((((n * a.H + iy) * a.W + ix) * a.ld + q * 8) * 2)
                  : OOB;
  }
  // weight pieces: row, chunk
  unsigned woff[WOPS];
#pragma unroll
  for (int i = 0; i < WOPS; ++i) {
    const int L = i * NT + tid;
    const int row = L >> 2;
    const int q = (L & 3) ^ swz_b128((row >> 2) & 3);
    woff[i] = (unsigned)(((co0 + row) * a.Kw + q * 8) * 2);
  }

  auto issue_halo = [&](int cs, int buf, int i) {
    const int c = cs * 32 + hq[i] * 8;
    const unsigned off = (hoff[i] != OOB && c < a.C) ? hoff[i] + cs * 64 : OOB;
    dma16(rs_src, hb0 + buf * HBUF + (i * NT + wave * 64) * 16, off);
  };
  auto issue_w = [&](int step) {   // step = cs * 9 + tap
    const int cs = step / 9, t = step - cs * 9;
    const int kw = t * a.Cgp + cs * 32;
    if (!w_wave) return;
#pragma unroll
    for (int i = 0; i < WOPS; ++i)
      dma16(rs_w, wb0 + (step % RING) * WBUF + (i * NT + wave * 64) * 16, woff[i] + kw * 2);
  };

  f32x4_t acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nsteps = nslice * 9;
  // prologue: halo of slice 0, weights of steps 0 and 1
#pragma unroll
  for (int i = 0; i < HOPS; ++i) issue_halo(0, 0, i);
  issue_w(0);
  if (nsteps > 1) issue_w(1);

  const int fr = lane & 15, fq = lane >> 4;
  for (int step = 0; step < nsteps; ++step) {
    const int cs = step / 9, t = step - cs * 9;
    // ops issued after weights(step): weights(step + 1) [WOPS] and, when step - 1 was a
    // halo-issuing tap (taps 0..HOPS-1 of a slice issue one op each for the next slice),
    // one halo op
    const int tprev = (step - 1) % 9;
    const bool halo_prev = step >= 1 && tprev < HOPS && (step - 1) / 9 + 1 < nslice;
    if (step + 1 < nsteps) {
      if (w_wave) {
        if (halo_prev) wait_vmcnt_barrier<WOPS + 1>();
        else wait_vmcnt_barrier<WOPS>();
      } else {
        if (halo_prev) wait_vmcnt_barrier<1>();
        else wait_vmcnt_barrier<0>();
      }
    } else {
      wait_vmcnt_barrier<0>();
    }
    if (step + 2 < nsteps) issue_w(step + 2);
    if (t < HOPS && cs + 1 < nslice) {
#pragma unroll
      for (int i = 0; i < HOPS; ++i)   // static register index (no scratch for a dynamic one)
        if (i == t) issue_halo(cs + 1, (cs + 1) & 1, i);
    }
    const int ta = t / 3, tb = t - ta * 3;
    const int oyh = MODE == 0 ? ta : 2 - ta, oxh = MODE == 0 ? tb : 2 - tb;
    const char* wbase = lds + 2 * HBUF + (step % RING) * WBUF;
    const char* hbase = lds + (cs & 1) * HBUF;
    bf16x8_t fa[FI], fb[FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int row = wi * WT_CO + i * 16 + fr;
      fa[i] = as_frag(*reinterpret_cast<const uint4*>(wbase + (row * 4 + (fq ^ swz_b128((row >> 2) & 3))) * 16));
    }
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int r = wj * WROWS + j / CB, col = (j % CB) * 16 + fr;
      const int h = (r + oyh) * HW_ + col + oxh;
      fb[j] = as_frag(*reinterpret_cast<const uint4*>(hbase + (h * 4 + (fq ^ hswz(h))) * 16));
    }
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
  }

  // epilogue: 4 consecutive channels of one pixel per lane (8-byte stores)
  float bv[FI][4];
#pragma unroll
  for (int i = 0; i < FI; ++i) {
    const int co = co0 + wi * WT_CO + i * 16 + fq * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) bv[i][q] = (a.bias && co + q < a.K) ? a.bias[co + q] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const int r = wj * WROWS + j / CB, col = (j % CB) * 16 + fr;
    const long p = ((long)n * a.H + oy0 + r) * a.W + ox0 + col;
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int co = co0 + wi * WT_CO + i * 16 + fq * 4;
      if (co + 4 > a.K) continue;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = act_fwd(acc[i][j][q] + bv[i][q], a.act, a.slope);
      *reinterpret_cast<uint2*>(a.out + p * a.ldo + co) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    }
  }
}


// v2: weights staged G taps at a time (G = 9: a whole slice, G = 3: one filter
// row) into a ring of D + 1 stages, one barrier per stage; inside a stage the
// next tap's fragments are read while the current tap's MFMAs run.  KNOCK
// (diagnostics, compile time): 1 no DMA after the prologue, 2 no epilogue.
template <int MODE, int TCO, int WCO, int WPX, int TH, int TW, int G, int D, int KNOCK, int STAGE = 0>
__global__ __launch_bounds__(64 * WCO * WPX, (64 * WCO * WPX <= 256 ? 2 : 1)) void halo2_conv_kernel(HaloArgs a) {
  constexpr int NT = 64 * WCO * WPX;
  constexpr int WT_CO = TCO / WCO, FI = WT_CO / 16;
  constexpr int WROWS = TH / WPX, CB = TW / 16, FJ = WROWS * CB;
  constexpr int HW_ = TW + 2, HP = (TH + 2) * HW_, HCH = HP * 4;
  constexpr int HOPS = (HCH + NT - 1) / NT;
  constexpr int HBUF = HOPS * NT * 16;
  constexpr int WCH = G * TCO * 4;                      // weight chunks per stage
  constexpr int WOPS = (WCH + NT - 1) / NT;
  constexpr int WBUF = WOPS * NT * 16;
  constexpr int R = D + 1, SPS = 9 / G;
  static_assert(9 % G == 0 && FI >= 1 && FJ >= 1, "tile");
  __shared__ __attribute__((aligned(16))) char lds[2 * HBUF + R * WBUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wave / WPX, wj = wave % WPX;
  const int tiles_x = a.W / TW, tiles_y = a.H / TH;
  int b = blockIdx.x;
  const int tx = b % tiles_x;
  b /= tiles_x;
  const int ty = b % tiles_y;
  const int n = b / tiles_y;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int co0 = blockIdx.y * TCO;
  const int nslice = a.Cgp / 32;
  const int lds0 = (int)(uintptr_t)(lds_void_t*)lds;
  const int hb0 = lds0, wb0 = lds0 + 2 * HBUF;
  const rsrc_t rs_src = make_rsrc(a.src, a.src_bytes);
  const rsrc_t rs_w = make_rsrc(a.wp, a.w_bytes);

  unsigned hoff[HOPS];
  int hq[HOPS];
#pragma unroll
  for (int i = 0; i < HOPS; ++i) {
    const int L = i * NT + tid;
    const int h = L >> 2;
    const int q = (L & 3) ^ hswz(h);
    const int hy = h / HW_, hx = h - hy * HW_;
    const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
    hq[i] = q;
    hoff[i] = (h < HP && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
                  ? (unsigned)((((n * a.H + iy) * a.W + ix) * a.ld + q * 8) * 2)
                  : OOB;
  }
  // weight stage image: [tap g][row][4 chunks swizzled]; this thread's piece i: tap, row, chunk
  unsigned woff[WOPS];
  int wtap[WOPS];
#pragma unroll
  for (int i = 0; i < WOPS; ++i) {
    const int L = i * NT + tid;
    const int g = L / (TCO * 4), rem = L - g * (TCO * 4);
    const int row = rem >> 2;
    const int q = (rem & 3) ^ swz_b128((row >> 2) & 3);
    wtap[i] = g;
    woff[i] = L < WCH ? (unsigned)(((co0 + row) * a.Kw + q * 8) * 2) : OOB;
  }
  auto issue_halo = [&](int cs) {
#pragma unroll
    for (int i = 0; i < HOPS; ++i) {
      const int c = cs * 32 + hq[i] * 8;
      const unsigned off = (hoff[i] != OOB && c < a.C) ? hoff[i] + cs * 64 : OOB;
      dma16(rs_src, hb0 + (cs & 1) * HBUF + (i * NT + wave * 64) * 16, off);
    }
  };
  auto issue_w = [&](int st) {   // stage st = slice * SPS + group
    const int cs = st / SPS, g0 = (st - cs * SPS) * G;
#pragma unroll
    for (int i = 0; i < WOPS; ++i) {
      const int kw = (g0 + wtap[i]) * a.Cgp + cs * 32;
      dma16(rs_w, wb0 + (st % R) * WBUF + (i * NT + wave * 64) * 16, woff[i] == OOB ? OOB : woff[i] + kw * 2);
    }
  };

  f32x4_t acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nst = nslice * SPS;
  // prologue: halo(0), weights(0 .. D-1); halo(c + 1) is issued at the first stage of slice c,
  // BEFORE that stage's weight prefetch, so a stage's wait only counts weight pieces
  issue_halo(0);
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (d < nst) issue_w(d);
  const int fr = lane & 15, fq = lane >> 4;

  auto rd = [&](int st, int t, bf16x8_t (&fa)[FI], bf16x8_t (&fb)[FJ]) {
    const int cs = st / SPS, tap = (st - cs * SPS) * G + t;
    const int ta = tap / 3, tb = tap - ta * 3;
    const int oyh = MODE == 0 ? ta : 2 - ta, oxh = MODE == 0 ? tb : 2 - tb;
    const char* wbase = lds + 2 * HBUF + (st % R) * WBUF + t * TCO * 64;
    const char* hbase = lds + (cs & 1) * HBUF;
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int row = wi * WT_CO + i * 16 + fr;
      fa[i] = as_frag(*reinterpret_cast<const uint4*>(wbase + (row * 4 + (fq ^ swz_b128((row >> 2) & 3))) * 16));
    }
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int r = wj * WROWS + j / CB, col = (j % CB) * 16 + fr;
      const int h = (r + oyh) * HW_ + col + oxh;
      fb[j] = as_frag(*reinterpret_cast<const uint4*>(hbase + (h * 4 + (fq ^ hswz(h))) * 16));
    }
  };
  for (int st = 0; st < nst; ++st) {
    // weights(st) landed: younger pieces are weights(st+1 .. st+D-1) (halo pieces are older)
    if (KNOCK & 1) {
      wait_vmcnt_barrier<0>();
    } else if (st + D - 1 < nst) {
      wait_vmcnt_barrier<(D - 1) * WOPS>();
    } else {
      wait_vmcnt_barrier<0>();
    }
    const int cs = st / SPS;
    if (!(KNOCK & 1)) {
      if (st == cs * SPS && cs + 1 < nslice) issue_halo(cs + 1);
      if (st + D < nst) issue_w(st + D);
    }
    bf16x8_t fa[2][FI], fb[2][FJ];
    rd(st, 0, fa[0], fb[0]);
#pragma unroll
    for (int t = 0; t < G; ++t) {
      if (t + 1 < G) rd(st, t + 1, fa[(t + 1) & 1], fb[(t + 1) & 1]);
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t & 1][i], fb[t & 1][j], acc[i][j], 0, 0, 0);
    }
  }
  if (KNOCK & 2) {   // keep every MFMA alive, store nothing
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (sum == 1234.5f) a.out[0] = 1;
    return;
  }
  float bv[FI][4];
#pragma unroll
  for (int i = 0; i < FI; ++i) {
    const int co = co0 + wi * WT_CO + i * 16 + fq * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) bv[i][q] = (a.bias && co + q < a.K) ? a.bias[co + q] : 0.f;
  }
  if (STAGE) {
    // bf16 tile through LDS: [pixel][TCO] rows, 16-B chunk c of pixel p at c ^ (p & (NCK - 1)),
    // then whole 16-B chunks per lane, consecutive lanes along a pixel's channels
    constexpr int NCK = TCO / 8, TPIX = TH * TW;
    static_assert(TPIX * TCO * 2 <= 2 * HBUF + R * WBUF, "staged tile exceeds LDS");
    __syncthreads();
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int p = (wj * WROWS + j / CB) * TW + (j % CB) * 16 + fr;
#pragma unroll
      for (int i = 0; i < FI; ++i) {
        const int cl = wi * WT_CO + i * 16 + fq * 4;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = act_fwd(acc[i][j][q] + bv[i][q], a.act, a.slope);
        *reinterpret_cast<uint2*>(lds + p * TCO * 2 + (((cl >> 3) ^ (p & (NCK - 1))) << 4) + (cl & 4) * 2) =
            make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < TPIX * NCK / NT; ++k) {
      const int item = k * NT + tid;
      const int p = item / NCK, c = item % NCK;
      const uint4 v = *reinterpret_cast<const uint4*>(lds + p * TCO * 2 + ((c ^ (p & (NCK - 1))) << 4));
      const int r = p / TW, col = p % TW;
      const long gp = ((long)n * a.H + oy0 + r) * a.W + ox0 + col;
      if (co0 + c * 8 + 8 <= a.K) *reinterpret_cast<uint4*>(a.out + gp * a.ldo + co0 + c * 8) = v;
    }
    return;
  }
  if (STAGE) {
    // bf16 tile through LDS: [pixel][TCO] rows, 16-B chunk c of pixel p at c ^ (p & (NCK - 1)),
    // then whole 16-B chunks per lane, consecutive lanes along a pixel's channels
    constexpr int NCK = TCO / 8, TPIX = TH * TW;
    static_assert(TPIX * TCO * 2 <= 2 * HBUF + R * WBUF, "staged tile exceeds LDS");
    __syncthreads();
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int p = (wj * WROWS + j / CB) * TW + (j % CB) * 16 + fr;
#pragma unroll
      for (int i = 0; i < FI; ++i) {
        const int cl = wi * WT_CO + i * 16 + fq * 4;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = act_fwd(acc[i][j][q] + bv[i][q], a.act, a.slope);
        *reinterpret_cast<uint2*>(lds + p * TCO * 2 + (((cl >> 3) ^ (p & (NCK - 1))) << 4) + (cl & 4) * 2) =
            make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < TPIX * NCK / NT; ++k) {
      const int item = k * NT + tid;
      const int p = item / NCK, c = item % NCK;
      const uint4 v = *reinterpret_cast<const uint4*>(lds + p * TCO * 2 + ((c ^ (p & (NCK - 1))) << 4));
      const int r = p / TW, col = p % TW;
      const long gp = ((long)n * a.H + oy0 + r) * a.W + ox0 + col;
      if (co0 + c * 8 + 8 <= a.K) *reinterpret_cast<uint4*>(a.out + gp * a.ldo + co0 + c * 8) = v;
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const int r = wj * WROWS + j / CB, col = (j % CB) * 16 + fr;
    const long p = ((long)n * a.H + oy0 + r) * a.W + ox0 + col;
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int co = co0 + wi * WT_CO + i * 16 + fq * 4;
      if (co + 4 > a.K) continue;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = act_fwd(acc[i][j][q] + bv[i][q], a.act, a.slope);
      *reinterpret_cast<uint2*>(a.out + p * a.ldo + co) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    }
  }
}
}  // namespace

extern "C" int halo_conv(int variant, int mode, const bf16_t* src, const bf16_t* wp, const float* bias, bf16_t* out,
                         int N, int H, int W, int ld, int C, int Cgp, int K, int Kw, int ldo, int act, float slope,
                         long src_bytes, long w_bytes, int knock, hipStream_t s) {
  HaloArgs a{src, wp, bias, out, N, H, W, ld, C, Cgp, K, Kw, ldo, act, slope, src_bytes, w_bytes, knock};
#define L(MODE, TCO, WCO, WPX, TH, TW)                                                                        \
  do {                                                                                                       \
    if (H % TH || W % TW) return -22;                                                                        \
    dim3 grid(N * (H / TH) * (W / TW), (K + TCO - 1) / TCO);                                                 \
    halo_conv_kernel<MODE, TCO, WCO, WPX, TH, TW><<<grid, 64 * WCO * WPX, 0, s>>>(a);                        \
  } while (0)
#define L2(MODE, TCO, WCO, WPX, TH, TW, G, D, KN)                                                             \
  do {                                                                                                       \
    if (H % TH || W % TW) return -22;                                                                        \
    dim3 grid(N * (H / TH) * (W / TW), (K + TCO - 1) / TCO);                                                 \
    halo2_conv_kernel<MODE, TCO, WCO, WPX, TH, TW, G, D, KN><<<grid, 64 * WCO * WPX, 0, s>>>(a);             \
  } while (0)
#define L3(MODE, TCO, WCO, WPX, TH, TW, G, D, KN)                                                             \
  do {                                                                                                       \
    if (H % TH || W % TW) return -22;                                                                        \
    dim3 grid(N * (H / TH) * (W / TW), (K + TCO - 1) / TCO);                                                 \
    halo2_conv_kernel<MODE, TCO, WCO, WPX, TH, TW, G, D, KN, 1><<<grid, 64 * WCO * WPX, 0, s>>>(a);          \
  } while (0)
#define V2(MODE, KN)                                                                                         \
  do {                                                                                                       \
    if (variant == 10) L2(MODE, 64, 1, 4, 8, 32, 9, 1, KN);                                                  \
    else if (variant == 11) L2(MODE, 128, 2, 2, 8, 32, 3, 2, KN);                                            \
    else if (variant == 12) L2(MODE, 64, 2, 2, 8, 32, 9, 1, KN);                                             \
    else if (variant == 13) L2(MODE, 128, 2, 4, 16, 32, 3, 2, KN);                                           \
    else if (variant == 20) L3(MODE, 128, 2, 4, 16, 32, 3, 2, KN);                                           \
    else if (variant == 21) L3(MODE, 64, 1, 8, 16, 32, 9, 1, KN);                                            \
    else if (variant == 22) L3(MODE, 64, 1, 8, 16, 32, 3, 2, KN);                                            \
    else if (variant == 23) L3(MODE, 64, 1, 4, 8, 32, 9, 1, KN);                                             \
    else if (variant == 24) L3(MODE, 64, 1, 4, 8, 32, 3, 1, KN);                                             \
    else if (variant == 25) L3(MODE, 128, 2, 2, 8, 32, 1, 2, KN);                                            \
    else if (variant == 26) L3(MODE, 64, 2, 2, 8, 32, 3, 1, KN);                                             \
    else return -22;                                                                                         \
  } while (0)
  if (variant >= 10) {
    if (mode == 0) {
      if (knock == 0) V2(0, 0); else if (knock == 1) V2(0, 1); else if (knock == 2) V2(0, 2); else V2(0, 3);
    } else {
      if (knock == 0) V2(1, 0); else if (knock == 1) V2(1, 1); else if (knock == 2) V2(1, 2); else V2(1, 3);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  if (mode == 0) {
    if (variant == 0) L(0, 128, 2, 2, 8, 32);
    else if (variant == 1) L(0, 64, 1, 4, 8, 32);
    else if (variant == 2) L(0, 64, 1, 8, 16, 32);
    else if (variant == 3) L(0, 128, 2, 4, 16, 32);
    else return -22;
  } else {
    if (variant == 0) L(1, 128, 2, 2, 8, 32);
    else if (variant == 1) L(1, 64, 1, 4, 8, 32);
    else if (variant == 2) L(1, 64, 1, 8, 16, 32);
    else if (variant == 3) L(1, 128, 2, 4, 16, 32);
    else return -22;
  }
#undef L
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
