// Implicit-GEMM direct convolutions for gfx950 (bf16 MFMA 16x16x32, fp32 acc).
//
// Activations are NHWC bf16 with a channel stride `ld` (a multiple of 8:
// 3-channel images are stored with ld = 8).  No im2col is materialised:
// every B-operand tile is gathered straight from the activation tensor into LDS.
//
//   FWD  : y[p, co]  = sum_{r,s,c} x[gather_fwd(p,r,s), c] * W[co,r,s,c]
//   BWDD : dx[p, ci] = sum_{r,s,co} dy[gather_bwd(p,r,s), co] * W[co,ci,r,s]
//   WGRAD: dW[co, (r,s,c)] = sum_p dy[p, co] * x[gather_fwd(p,r,s), c]
//
// FWD/BWDD: MFMA rows = output channels (A = packed weights), MFMA columns =
// pixels (B = gathered activations), so each accumulator lane owns 4
// consecutive channels of one pixel -> 8-byte NHWC stores.  The K axis is
// (tap, channel) with every tap's channel run padded to a multiple of 32, so
// the tap and channel offset of each 32-deep K step are block-uniform: the
// gather does no per-element index arithmetic.  A stride-s backward-data
// pass is split into s^2 parity classes of input pixels; each class only
// visits the kernel taps that reach it (a 4x4/s2 bwd-data does 1/4 of the
// naive MFMA work).  Small grids are split along K (fp32 partial slab +
// a reduce kernel that applies the epilogue).
// Replaces every nn.Conv2d of models.py:14-403 and DAMSM.py.
#include <stdlib.h>
#include <string.h>

#include "common.h"
#include "../../include/eegan_hip.h"

namespace {

constexpr int BK = 32;       // K per LDS stage (= one 16x16x32 MFMA)
constexpr int LDS_PAD = 8;   // bf16 elements of row padding (16 B)
constexpr int KROW = BK + LDS_PAD;

enum { MODE_FWD = 0, MODE_BWDD = 1 };

EE_DEV bf16x8_t as_frag(uint4 v) { return __builtin_bit_cast(bf16x8_t, v); }

// zero the channels >= cvalid of an 8-channel chunk starting at channel c
EE_DEV uint4 mask_chunk(uint4 v, int c, int cvalid) {
  if (c + 8 > cvalid) {
    uint32_t* w = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c0 = c + 2 * j;
      if (c0 >= cvalid) w[j] = 0;
      else if (c0 + 1 >= cvalid) w[j] &= 0xffffu;
    }
  }
  return v;
}

// out = res_scale * res + gamma * v with one explicit rounding order, so the
// direct, LDS-staged and split-K epilogues agree bit for bit (left to
// -ffp-contract the compiler fuses either product, differently per site)
EE_DEV float res_combine(float rs, float r, float g, float v) { return __builtin_fmaf(g, v, rs * r); }

struct ConvArgs {
  const bf16_t* src;   // FWD: x ; BWDD: dy
  const bf16_t* wp;    // packed weights [rows_pad][Kw], K = (tap, channel padded to Cgp)
  const float* bias;   // per output channel or null
  const bf16_t* res;   // residual: out = res + gamma * act(acc + bias)
  const float* gamma;  // device scalar
  void* out;
  float* part;         // split-K partial slab [nsplit][P][Mrows] or null
  int ldres, ldo, out_f32, act;
  float slope;
  int N, IH, IW, lds_src, up2;  // source grid (LOGICAL; FWD up2: physical IH/2 x IW/2)
  int OH, OW;                   // full pixel grid of the GEMM columns
  int R, S, st, ph, pw;
  int Cgp, Cvalid;              // per-tap K run (multiple of 32) / valid gathered channels
  int Mrows, Kw;                // output channels / packed-weight row stride
  int P;                        // N*OH*OW
  int ncls, nsplit;             // parity classes (BWDD stride>1), K splits
  // BWDD only: multiply dx by act'(gate) of the activation `gate_act` expressed
  // through its output (the activated conv input x): the producer's activation
  // backward fused into this data gradient (x has no other non-gating consumer)
  const bf16_t* gate;
  int ldgate, gate_act;
  float gate_slope;
  // residual read at half resolution (nearest-2x: pixel (y>>1, x>>1)) and
  // scaled: out = res_scale * res + gamma * act(acc).  BWDD: a 2x2
  // average-pool's adjoint fused into the data gradient (resD's shortcut)
  int res_up2;
  float res_scale;
  int gate_vec;  // same for the activation gate
  int red_vec4;  // split-K reduce: 4-channel vector path (host-checked alignment)
  int res_vec;  // res rows 8-byte aligned (ldres % 4 == 0, aligned base): vector residual loads
  int wide;     // conv_fast_kernel pairs: one 64-channel stage of whole 128-B lines per K-step pair
  int stage_epi;  // conv_fast_kernel: LDS-staged epilogue (unsplit bf16 output, 16-B aligned rows; host-checked)
  int* ctr;       // conv_fast_kernel split-K: per-tile arrival counters (zero on entry and exit) -> in-kernel finish
  int tp;         // planner objective (eegan_conv_desc.plan): 1 = throughput (host only)
  // conv_fast_kernel XCD raster (xcd_g > 0): a 1-D grid of round_up(gx * gy * gz, 8) blocks; the
  // blocks one XCD runs (id % 8 equal) take a contiguous range of the logical tile order, which
  // walks groups of xcd_g co-tile rows (pixel tiles inside a group), z outermost -- so an XCD's
  // blocks share a few weight-row tiles and a run of pixel tiles in its own L2 instead of every
  // XCD reading every weight tile (round-robin dispatch of the x-fastest 3-D grid)
  int xcd_g, gx, gy, gz;
};

// K step kt, 8-channel chunk kc -> kernel tap and channel.  Normal mode: the
// step is one tap's 32-channel slice (block-uniform).  Packed mode (Cgp == 8,
// inputs with <= 8 channels): the step covers 4 consecutive taps of 8 channels,
// chunk kc being tap 4*kt + kc.  `kw` is the column in the packed weight row.
struct TapPos {
  int r, s, ta, tb, c, kw;
  bool ok;
};

template <int MODE>
EE_DEV TapPos tap_pos(const ConvArgs& a, int kt, int kc, int nc, int TS, int ntaps, int r0, int s0) {
  TapPos t;
  int tap, c;
  if (a.Cgp == 8) {
    tap = kt * 4 + kc;
    c = 0;
  } else {
    tap = kt / nc;
    c = (kt - tap * nc) * BK + kc * 8;
  }
  t.ok = tap < ntaps;
  if (!t.ok) tap = 0;
  t.ta = tap / TS;
  t.tb = tap - t.ta * TS;
  t.r = (MODE == MODE_FWD) ? t.ta : r0 + a.st * t.ta;
  t.s = (MODE == MODE_FWD) ? t.tb : s0 + a.st * t.tb;
  t.c = c;
  t.kw = (t.r * a.S + t.s) * a.Cgp + c;
  return t;
}

EE_DEV int k_steps(const ConvArgs& a, int ntaps) { return a.Cgp == 8 ? (ntaps + 3) / 4 : ntaps * (a.Cgp / BK); }

// Epilogue shared by the GEMM kernels: fragment (i, j) of wave (wi, wj) holds 4
// consecutive output channels of one pixel -> bias, activation, residual,
// 8-byte NHWC store (or the fp32 split-K slab).
template <int MODE, int FI, int FJ, int WT_CO, int WT_PIX>
EE_DEV void igemm_epilogue(const ConvArgs& a, const f32x4_t (&acc)[FI][FJ], int pix0, int co0, int wi, int wj,
                           int lane, int split, int Pc, int CH, int CW, int qy, int qx, int stc) {
  const int fr = lane & 15;
  const float gam = (a.res && a.gamma) ? *a.gamma : 1.f;
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const int pc = pix0 + wj * WT_PIX + j * 16 + fr;
    if (pc >= Pc) continue;
    long p = pc;
    long rpix = pc;  // residual pixel (half resolution when res_up2)
    if (MODE == MODE_BWDD && a.ncls > 1) {
      const int hw = CH * CW;
      const int n = pc / hw, rem = pc - n * hw;
      const int yy = rem / CW, xx = rem - yy * CW;
      const int y = qy + stc * yy, x = qx + stc * xx;
      p = ((long)n * a.OH + y) * a.OW + x;
      if (a.res_up2) rpix = ((long)n * (a.OH >> 1) + (y >> 1)) * (a.OW >> 1) + (x >> 1);
    } else if (a.res_up2) {
      // 32-bit index math, once per pixel (P < 2^31 is checked on the host)
      const unsigned hw = (unsigned)a.OH * (unsigned)a.OW;
      const unsigned n = (unsigned)pc / hw, rem = (unsigned)pc - n * hw;
      const unsigned y = rem / (unsigned)a.OW, x = rem - y * (unsigned)a.OW;
      rpix = ((long)n * (a.OH >> 1) + (y >> 1)) * (a.OW >> 1) + (x >> 1);
    }
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int co = co0 + wi * WT_CO + i * 16 + (lane >> 4) * 4;
      if (co >= a.Mrows) continue;
      if (a.nsplit > 1) {
        float* dst = a.part + ((long)split * a.P + p) * a.Mrows + co;
        if ((a.Mrows & 3) == 0) {   // one 16-B store (slab rows 16-B aligned): 4x fewer store issues
          *reinterpret_cast<f32x4_t*>(dst) = acc[i][j];
          continue;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (co + r < a.Mrows) dst[r] = acc[i][j][r];
        continue;
      }
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float bv = (a.bias && co + r < a.Mrows) ? a.bias[co + r] : 0.f;
        v[r] = act_fwd(acc[i][j][r] + bv, a.act, a.slope);
      }
      if (MODE == MODE_BWDD && a.gate) {
        const bf16_t* gp = a.gate + p * a.ldgate + co;
        if (a.gate_vec && co + 4 <= a.Mrows) {
          const uint2 gv = *reinterpret_cast<const uint2*>(gp);
          const float gg[4] = {lo_f(gv.x), hi_f(gv.x), lo_f(gv.y), hi_f(gv.y)};
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] *= act_dgrad_from_y(gg[r], a.gate_act, a.gate_slope);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (co + r < a.Mrows) v[r] *= act_dgrad_from_y(bf2f(gp[r]), a.gate_act, a.gate_slope);
        }
      }
      if (a.res) {
        const bf16_t* rp = a.res + (a.res_up2 ? rpix : p) * a.ldres + co;
        if (a.res_vec && co + 4 <= a.Mrows) {  // 8-byte aligned rows (host-checked): one load
          const uint2 rv = *reinterpret_cast<const uint2*>(rp);
          const float rr[4] = {lo_f(rv.x), hi_f(rv.x), lo_f(rv.y), hi_f(rv.y)};
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = res_combine(a.res_scale, rr[r], gam, v[r]);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (co + r < a.Mrows) v[r] = res_combine(a.res_scale, bf2f(rp[r]), gam, v[r]);
        }
      }
      if (a.out_f32) {
        float* op = reinterpret_cast<float*>(a.out) + p * a.ldo + co;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (co + r < a.Mrows) op[r] = v[r];
      } else {
        bf16_t* op = reinterpret_cast<bf16_t*>(a.out) + p * a.ldo + co;
        if (co + 4 <= a.Mrows) {
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

// LDS-staged form of igemm_epilogue for conv_fast_kernel (unsplit, bf16 out,
// Mrows % 8 == 0, output / gate / residual rows 16-B aligned: host-checked).
// Straight from the MFMA layout every store writes 16 pixels x 32 B, a quarter
// or half of each pixel's line, the rest coming from other stores and waves
// (stride-2 classes: from other workgroups) -- measured 30-47 % of the tile
// kernels' time on 64..128-channel shapes.  Here the fp32 tile goes through
// the (then idle) LDS ring and every thread finishes 8 channels of one pixel:
// 16-B loads of the gate / residual runs, one 16-B store, consecutive threads
// along the pixel's row.  Same arithmetic and order as igemm_epilogue, so
// bit-identical.  The staged image is [pixel][TCO / 4 fp32 chunks], chunk index
// XOR (pixel & 7): conflict-free ds_write_b128 (8 pixels per lane group) and
// ds_read_b128 at 8-channel runs.
template <int MODE, int TCO, int TPIX, int FI, int FJ, int WT_CO, int WT_PIX>
EE_DEV void staged_epilogue(const ConvArgs& a, const f32x4_t (&acc)[FI][FJ], float4* st, int pix0, int co0, int wi,
                            int wj, int lane, int tid, int Pc, int CH, int CW, int qy, int qx, int stc) {
  constexpr int NCK = TCO / 4, SWM = NCK >= 8 ? 7 : NCK - 1, E = TCO / 8, ITEMS = TPIX * E;
  constexpr int NIT = (ITEMS + 255) / 256;
  const int fr = lane & 15, fq = lane >> 4;
  // gate / residual runs of this thread's items loaded first: their latency overlaps the staging
  uint4 gpre[NIT], rpre[NIT];
  long ppre[NIT];
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int item = k * 256 + tid;
    gpre[k] = rpre[k] = make_uint4(0, 0, 0, 0);
    ppre[k] = -1;
    if (ITEMS % 256 && item >= ITEMS) continue;
    const int pix = item / E, e = item % E;
    const int pc = pix0 + pix, co = co0 + 8 * e;
    if (pc >= Pc || co >= a.Mrows) continue;
    long p = pc, rpix = pc;
    if (MODE == MODE_BWDD && a.ncls > 1) {
      const int hw = CH * CW;
      const int n = pc / hw, rem = pc - n * hw;
      const int yy = rem / CW, xx = rem - yy * CW;
      const int y = qy + stc * yy, x = qx + stc * xx;
      p = ((long)n * a.OH + y) * a.OW + x;
      if (a.res_up2) rpix = ((long)n * (a.OH >> 1) + (y >> 1)) * (a.OW >> 1) + (x >> 1);
    } else if (a.res_up2) {
      const unsigned hw = (unsigned)a.OH * (unsigned)a.OW;
      const unsigned n = (unsigned)pc / hw, rem = (unsigned)pc - n * hw;
      const unsigned y = rem / (unsigned)a.OW, x = rem - y * (unsigned)a.OW;
      rpix = ((long)n * (a.OH >> 1) + (y >> 1)) * (a.OW >> 1) + (x >> 1);
    }
    ppre[k] = p;
    if (MODE == MODE_BWDD && a.gate) gpre[k] = *reinterpret_cast<const uint4*>(a.gate + p * a.ldgate + co);
    if (a.res) rpre[k] = *reinterpret_cast<const uint4*>(a.res + (a.res_up2 ? rpix : p) * a.ldres + co);
  }
  __syncthreads();  // every wave's last ring reads are done
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int pix = wj * WT_PIX + j * 16 + fr;
      const int c = (wi * WT_CO + i * 16) / 4 + fq;
      st[pix * NCK + (c ^ (pix & SWM))] = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
  __syncthreads();
  const float gam = (a.res && a.gamma) ? *a.gamma : 1.f;
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int item = k * 256 + tid;
    if (ppre[k] < 0) continue;
    const int pix = item / E, e = item % E;
    const int co = co0 + 8 * e;
    const float4 lo = st[pix * NCK + ((2 * e) ^ (pix & SWM))];
    const float4 hi = st[pix * NCK + ((2 * e + 1) ^ (pix & SWM))];
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    const long p = ppre[k];
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = act_fwd(v[r] + ((a.bias && co + r < a.Mrows) ? a.bias[co + r] : 0.f), a.act, a.slope);
    if (MODE == MODE_BWDD && a.gate) {
      const uint4 gv = gpre[k];
      const uint32_t gw[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[2 * r] *= act_dgrad_from_y(lo_f(gw[r]), a.gate_act, a.gate_slope);
        v[2 * r + 1] *= act_dgrad_from_y(hi_f(gw[r]), a.gate_act, a.gate_slope);
      }
    }
    if (a.res) {
      const uint4 rv = rpre[k];
      const uint32_t rw[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[2 * r] = res_combine(a.res_scale, lo_f(rw[r]), gam, v[2 * r]);
        v[2 * r + 1] = res_combine(a.res_scale, hi_f(rw[r]), gam, v[2 * r + 1]);
      }
    }
    *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.out) + p * a.ldo + co) =
        make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
  }
}

// split-K reduction + epilogue: out[p][co] = res + gamma*act(sum_z part[z][p][co] + bias).
//
// 4 consecutive channels of one pixel: the residual / gate / bias loads are
// issued first, then the 16-byte slab loads 8 splits at a time (one memory
// round trip for the usual 8-way split), summed in split order (bit-identical
// to the scalar path); 32-bit index math (the host enables this path only for
// P * Mrows < 2^31)
EE_DEV void splitk_item4(const ConvArgs& a, unsigned p, unsigned co, float gam) {
  const unsigned total4 = (unsigned)(((long)a.P * a.Mrows) >> 2);
  const unsigned i = (p * (unsigned)a.Mrows + co) >> 2;
  uint2 gv = make_uint2(0, 0), rv = make_uint2(0, 0);
  if (a.gate) gv = *reinterpret_cast<const uint2*>(a.gate + (long)p * a.ldgate + co);
  if (a.res) {
    long rpix = p;
    if (a.res_up2) {
      const unsigned hw = (unsigned)a.OH * (unsigned)a.OW;
      const unsigned n = p / hw, rem = p - n * hw;
      const unsigned y = rem / (unsigned)a.OW, x = rem - y * (unsigned)a.OW;
      rpix = ((long)n * (a.OH >> 1) + (y >> 1)) * (a.OW >> 1) + (x >> 1);
    }
    rv = *reinterpret_cast<const uint2*>(a.res + rpix * a.ldres + co);
  }
  f32x4_t bv = {0.f, 0.f, 0.f, 0.f};
  if (a.bias) bv = f32x4_t{a.bias[co], a.bias[co + 1], a.bias[co + 2], a.bias[co + 3]};
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  const f32x4_t* src = reinterpret_cast<const f32x4_t*>(a.part) + i;
  int z = 0;
  for (; z + 8 <= a.nsplit; z += 8) {
    f32x4_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = src[(long)(z + k) * total4];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k];   // split order, as the scalar path
  }
  for (; z < a.nsplit; ++z) acc += src[(long)z * total4];
  float v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = act_fwd(acc[r] + bv[r], a.act, a.slope);
  if (a.gate) {
    const float gg[4] = {lo_f(gv.x), hi_f(gv.x), lo_f(gv.y), hi_f(gv.y)};
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] *= act_dgrad_from_y(gg[r], a.gate_act, a.gate_slope);
  }
  if (a.res) {
    const float rr[4] = {lo_f(rv.x), hi_f(rv.x), lo_f(rv.y), hi_f(rv.y)};
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = res_combine(a.res_scale, rr[r], gam, v[r]);
  }
  if (a.out_f32) {
    *reinterpret_cast<f32x4_t*>(reinterpret_cast<float*>(a.out) + (long)p * a.ldo + co) = {v[0], v[1], v[2], v[3]};
  } else {
    *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(a.out) + (long)p * a.ldo + co) =
        make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
  }
}

EE_DEV void splitk_item1(const ConvArgs& a, long p, int co, float gam) {
  const long total = (long)a.P * a.Mrows, e = p * a.Mrows + co;
  float v = 0.f;
  for (int z = 0; z < a.nsplit; ++z) v += a.part[(long)z * total + e];
  v = act_fwd(v + (a.bias ? a.bias[co] : 0.f), a.act, a.slope);
  if (a.gate) v *= act_dgrad_from_y(bf2f(a.gate[p * a.ldgate + co]), a.gate_act, a.gate_slope);
  if (a.res) {
    long rpix = p;
    if (a.res_up2) {
      const unsigned hw = (unsigned)a.OH * (unsigned)a.OW;
      const unsigned n = (unsigned)p / hw, rem = (unsigned)p - n * hw;
      const unsigned y = rem / (unsigned)a.OW, x = rem - y * (unsigned)a.OW;
      rpix = ((long)n * (a.OH >> 1) + (y >> 1)) * (a.OW >> 1) + (x >> 1);
    }
    v = res_combine(a.res_scale, bf2f(a.res[rpix * a.ldres + co]), gam, v);
  }
  if (a.out_f32) reinterpret_cast<float*>(a.out)[p * a.ldo + co] = v;
  else reinterpret_cast<bf16_t*>(a.out)[p * a.ldo + co] = f2bf(v);
}

template <int MODE>  // MODE only tags the kernel name (profiles tell fwd / bwd-data apart)
__global__ void conv_splitk_reduce_kernel(ConvArgs a) {
  const long total = (long)a.P * a.Mrows;
  const float gam = (a.res && a.gamma) ? *a.gamma : 1.f;
  if (a.red_vec4) {
    const unsigned total4 = (unsigned)(total >> 2), M = (unsigned)a.Mrows;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += gridDim.x * blockDim.x) {
      const unsigned e = i * 4, p = e / M, co = e - p * M;
      splitk_item4(a, p, co, gam);
    }
    return;
  }
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long p = e / a.Mrows;
    splitk_item1(a, p, (int)(e - p * a.Mrows), gam);
  }
}

// ------------------------------------------------------- FWD / BWDD kernel --
template <int MODE, int TCO, int TPIX, int WCO>
__global__ __launch_bounds__(256) void conv_igemm_kernel(ConvArgs a) {
  constexpr int WPIX = 4 / WCO;
  constexpr int WT_CO = TCO / WCO, WT_PIX = TPIX / WPIX;
  constexpr int FI = WT_CO / 16, FJ = WT_PIX / 16;
  constexpr int A_CHUNKS = TCO * (BK / 8);
  constexpr int B_CHUNKS = TPIX * (BK / 8);
  constexpr int A_PER = (A_CHUNKS + 255) / 256;
  constexpr int B_PER = B_CHUNKS / 256;
  static_assert(B_CHUNKS % 256 == 0, "pixel tile");
  static_assert(FI >= 1 && FJ >= 1, "wave tile");

  __shared__ __attribute__((aligned(16))) bf16_t lds_a[2][TCO * KROW];
  __shared__ __attribute__((aligned(16))) bf16_t lds_b[2][TPIX * KROW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = wave / WPIX, wj = wave % WPIX;
  const int cls = blockIdx.z % a.ncls, split = blockIdx.z / a.ncls;
  const int co0 = blockIdx.y * TCO;

  // ---- parity class (BWDD with stride > 1): input pixels (qy + st*i, qx + st*j)
  int qy = 0, qx = 0, CH = a.OH, CW = a.OW, stc = 1;
  int r0 = 0, s0 = 0, TR = a.R, TS = a.S, dqy = 0, dqx = 0;
  if (MODE == MODE_BWDD) {
    if (a.ncls > 1) {
      qy = cls / a.st;
      qx = cls - qy * a.st;
      CH = (a.OH - qy + a.st - 1) / a.st;
      CW = (a.OW - qx + a.st - 1) / a.st;
      stc = a.st;
    }
    r0 = (qy + a.ph) % a.st;
    s0 = (qx + a.pw) % a.st;
    TR = r0 < a.R ? (a.R - r0 + a.st - 1) / a.st : 0;
    TS = s0 < a.S ? (a.S - s0 + a.st - 1) / a.st : 0;
    dqy = (qy + a.ph - r0) / a.st;
    dqx = (qx + a.pw - s0) / a.st;
  }
  const int Pc = a.N * CH * CW;
  const int pix0 = blockIdx.x * TPIX;
  if (pix0 >= Pc) return;  // block-uniform
  const int nc = a.Cgp / BK;
  const int ntaps = TR * TS;
  const int nk_all = k_steps(a, ntaps);
  const int kchunk = (nk_all + a.nsplit - 1) / a.nsplit;
  const int kt0 = min(nk_all, split * kchunk), kt1 = min(nk_all, kt0 + kchunk);

  // ---- per-thread B rows (pixels) and k-chunk
  const int b_kc = tid & 3;
  int b_n[B_PER], b_y[B_PER], b_x[B_PER];
  bool b_ok[B_PER];
#pragma unroll
  for (int i = 0; i < B_PER; ++i) {
    const int p = pix0 + (tid >> 2) + i * 64;
    b_ok[i] = p < Pc;
    const int pp = b_ok[i] ? p : 0;
    const int hw = CH * CW;
    const int n = pp / hw;
    const int rem = pp - n * hw;
    const int yy = rem / CW;
    const int xx = rem - yy * CW;
    b_n[i] = n;
    if (MODE == MODE_FWD) {
      b_y[i] = yy * a.st - a.ph;
      b_x[i] = xx * a.st - a.pw;
    } else {
      b_y[i] = yy + dqy;  // oh = yy + dqy - tap_a
      b_x[i] = xx + dqx;
    }
  }
  const int PH = a.IH >> a.up2, PW = a.IW >> a.up2;

  uint4 ra[A_PER], rb[B_PER];
  auto load_stage = [&](int kt) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int ch = tid + i * 256;
      if (ch < A_CHUNKS) {
        const int row = ch >> 2, kc = ch & 3;
        const TapPos tp = tap_pos<MODE>(a, kt, kc, nc, TS, ntaps, r0, s0);
        ra[i] = *reinterpret_cast<const uint4*>(a.wp + (long)(co0 + row) * a.Kw + tp.kw);
      }
    }
    const TapPos tp = tap_pos<MODE>(a, kt, b_kc, nc, TS, ntaps, r0, s0);
    const int c = tp.c;
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (b_ok[i] && tp.ok && c < a.Cvalid) {
        long off = -1;
        if (MODE == MODE_FWD) {
          const int iy = b_y[i] + tp.r, ix = b_x[i] + tp.s;
          if ((unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW)
            off = ((long)(b_n[i] * PH + (iy >> a.up2)) * PW + (ix >> a.up2)) * a.lds_src;
        } else {
          const int oy = b_y[i] - tp.ta, ox = b_x[i] - tp.tb;
          if ((unsigned)oy < (unsigned)a.IH && (unsigned)ox < (unsigned)a.IW)
            off = ((long)(b_n[i] * a.IH + oy) * a.IW + ox) * a.lds_src;
        }
        if (off >= 0) v = mask_chunk(*reinterpret_cast<const uint4*>(a.src + off + c), c, a.Cvalid);
      }
      rb[i] = v;
    }
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

  const int fr = lane & 15, fk = (lane >> 4) * 8;
  if (kt0 < kt1) {
    load_stage(kt0);
    store_stage(0);
    __syncthreads();
    int buf = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) load_stage(kt + 1);
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
      if (more) store_stage(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  igemm_epilogue<MODE, FI, FJ, WT_CO, WT_PIX>(a, acc, pix0, co0, wi, wj, lane, split, Pc, CH, CW, qy, qx, stc);
}

// ------------------------------------- FWD / BWDD, pipelined LDS-DMA kernel --
// Same GEMM as conv_igemm_kernel, but both operand tiles go global -> LDS by
// buffer_load ... lds (16 B per lane, no VGPR staging) into a STAGES-deep ring:
// STAGES-1 K-steps are in flight while one is multiplied, one raw s_barrier per
// K-step, counted vmcnt waits (never 0 inside the steady state).  The LDS image
// is lane-linear (64-B rows of 32 bf16), so the bank-conflict swizzle is
// applied to the SOURCE chunk: LDS slot q of row r holds K-chunk
// q ^ swz_b128((r>>2)&3).
// Out-of-range taps / channels use an out-of-bounds buffer offset, which the
// hardware bounds check turns into zeros.  Requires C % 8 == 0 (whole 16-B
// chunks valid or invalid) and TCO >= 64.
constexpr unsigned OOB = 0x80000000u;
constexpr int CONV_STAGES = 4;

typedef __attribute__((address_space(3))) void lds_void_t;

// XOR swizzle of the 16-B chunk of 64-B LDS rows read as MFMA fragments by
// ds_read_b128 (lane l: row l & 15, chunk l >> 4).  gfx950 services a b128 read
// in four 16-lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, (+32): with the
// row-block permutation 0,2,3,1 every group covers the 64 banks exactly once
// (the plain (r>>2)&3 swizzle is 2-way conflicted in every group).
EE_DEV int swz_b128(int b) { return (0x1320 >> (b * 4)) & 3; }

typedef __attribute__((ext_vector_type(4))) int rsrc_t;

// Raw buffer resource (V#) for byte range [p, p + bytes): bounds-checked, so an
// offset >= bytes (OOB) reads zeros.  Built by hand so it can feed inline asm.
EE_DEV rsrc_t make_rsrc(const void* p, long bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  rsrc_t r;
  r.x = (int)(uint32_t)a;
  r.y = (int)((a >> 32) & 0xffffu);  // stride 0
  r.z = (int)min(bytes, 0x7fffffffL);
  r.w = 0x00020000;
  return r;
}

// One 16-B-per-lane LDS-DMA piece: lane l's 16 bytes from rsrc+voff land at
// LDS byte (lds_dst + 16 l).  Issued by inline asm on purpose: the compiler's
// waitcnt pass treats a builtin LDS-DMA as an LDS store that aliases every
// later ds_read and inserts s_waitcnt vmcnt(0) in front of them, which drains
// the whole ring every K-step.  Ordering is ours: counted waits + barrier
// (wait_vmcnt_barrier) before a stage is read.
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is ours to clobber in these kernels
EE_DEV void lds_dma16(rsrc_t rsrc, const void* lds_dst, unsigned voff) {
  const int m0 = __builtin_amdgcn_readfirstlane((int)(uintptr_t)(lds_void_t*)lds_dst);
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0), "v"(voff), "s"(rsrc)
               : "memory", "m0");
}

// all but this wave's N youngest LDS-DMA pieces landed, then the workgroup
// barrier (every wave's pieces of the stage landed); one asm block so no LDS
// read can be scheduled between the wait and the barrier
template <int N>
EE_DEV void wait_vmcnt_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

template <int MODE, int TCO, int TPIX>
__global__ __launch_bounds__(256, 2) void conv_glds_kernel(ConvArgs a, long src_bytes, long w_bytes) {
  constexpr int S = CONV_STAGES;
  constexpr int WCO = TCO >= 64 ? 2 : 1, WPIX = 4 / WCO;
  constexpr int WT_CO = TCO / WCO, WT_PIX = TPIX / WPIX;
  constexpr int FI = WT_CO / 16, FJ = WT_PIX / 16;
  constexpr int A_TOT = TCO * 4, B_TOT = TPIX * 4;     // 16-B chunks per K-step
  constexpr int A_INS = (A_TOT + 255) / 256, B_INS = B_TOT / 256;
  constexpr int STAGE = (TCO + TPIX) * BK;             // bf16 elements per stage
  static_assert(B_INS >= 1 && FI >= 1 && FJ >= 1, "tile");

  __shared__ __attribute__((aligned(16))) bf16_t lds[S * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = wave / WPIX, wj = wave % WPIX;
  const int cls = blockIdx.z % a.ncls, split = blockIdx.z / a.ncls;
  const int co0 = blockIdx.y * TCO;
  const bool a_wave = A_TOT >= 256 || tid < A_TOT;      // waves that stage weight chunks

  int qy = 0, qx = 0, CH = a.OH, CW = a.OW, stc = 1;
  int r0 = 0, s0 = 0, TR = a.R, TS = a.S, dqy = 0, dqx = 0;
  if (MODE == MODE_BWDD) {
    if (a.ncls > 1) {
      qy = cls / a.st;
      qx = cls - qy * a.st;
      CH = (a.OH - qy + a.st - 1) / a.st;
      CW = (a.OW - qx + a.st - 1) / a.st;
      stc = a.st;
    }
    r0 = (qy + a.ph) % a.st;
    s0 = (qx + a.pw) % a.st;
    TR = r0 < a.R ? (a.R - r0 + a.st - 1) / a.st : 0;
    TS = s0 < a.S ? (a.S - s0 + a.st - 1) / a.st : 0;
    dqy = (qy + a.ph - r0) / a.st;
    dqx = (qx + a.pw - s0) / a.st;
  }
  const int Pc = a.N * CH * CW;
  const int pix0 = blockIdx.x * TPIX;
  if (pix0 >= Pc) return;  // block-uniform
  const int nc = a.Cgp / BK;
  const int ntaps = TR * TS;
  const int nk_all = k_steps(a, ntaps);
  const int kchunk = (nk_all + a.nsplit - 1) / a.nsplit;
  const int kt0 = min(nk_all, split * kchunk), kt1 = min(nk_all, kt0 + kchunk);
  const int nk = kt1 - kt0;

  // this thread's 16-B chunk of every staged row: rows i*64 + tid/4, K-chunk swizzled
  const int rsub = tid >> 2;
  const int kc = (tid & 3) ^ swz_b128((tid >> 4) & 3);
  int b_n[B_INS], b_y[B_INS], b_x[B_INS];
  bool b_ok[B_INS];
#pragma unroll
  for (int i = 0; i < B_INS; ++i) {
    const int p = pix0 + i * 64 + rsub;
    b_ok[i] = p < Pc;
    const int pp = b_ok[i] ? p : 0;
    const int hw = CH * CW;
    const int n = pp / hw;
    const int rem = pp - n * hw;
    const int yy = rem / CW;
    const int xx = rem - yy * CW;
    b_n[i] = n;
    if (MODE == MODE_FWD) {
      b_y[i] = yy * a.st - a.ph;
      b_x[i] = xx * a.st - a.pw;
    } else {
      b_y[i] = yy + dqy;
      b_x[i] = xx + dqx;
    }
  }
  const int PH = a.IH >> a.up2, PW = a.IW >> a.up2;
  const rsrc_t rs_src = make_rsrc(a.src, src_bytes);
  const rsrc_t rs_w = make_rsrc(a.wp, w_bytes);

  auto issue = [&](int kt, int buf) {
    const TapPos tp = tap_pos<MODE>(a, kt, kc, nc, TS, ntaps, r0, s0);
    bf16_t* base = lds + buf * STAGE;
    if (a_wave) {
#pragma unroll
      for (int i = 0; i < A_INS; ++i) {
        const unsigned off = (unsigned)(((co0 + i * 64 + rsub) * a.Kw + tp.kw) * 2);
        lds_dma16(rs_w, base + (i * 256 + wave * 64) * 8, off);
      }
    }
    const int c = tp.c;
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      unsigned off = OOB;
      if (b_ok[i] && tp.ok && c < a.Cvalid) {
        if (MODE == MODE_FWD) {
          const int iy = b_y[i] + tp.r, ix = b_x[i] + tp.s;
          if ((unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW)
            off = (unsigned)((((b_n[i] * PH + (iy >> a.up2)) * PW + (ix >> a.up2)) * a.lds_src + c) * 2);
        } else {
          const int oy = b_y[i] - tp.ta, ox = b_x[i] - tp.tb;
          if ((unsigned)oy < (unsigned)a.IH && (unsigned)ox < (unsigned)a.IW)
            off = (unsigned)((((b_n[i] * a.IH + oy) * a.IW + ox) * a.lds_src + c) * 2);
        }
      }
      lds_dma16(rs_src, base + TCO * BK + (i * 256 + wave * 64) * 8, off);
    }
  };

  f32x4_t acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // packed-tap mode with < 8 valid channels: the staged chunks carry the
  // tensor's padding channels, zero them in the B fragments (element e = channel e)
  uint4 bmask = make_uint4(~0u, ~0u, ~0u, ~0u);
  if (a.Cvalid < 8) {
    uint32_t* m = reinterpret_cast<uint32_t*>(&bmask);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      m[j] = (2 * j < a.Cvalid ? 0xffffu : 0u) | (2 * j + 1 < a.Cvalid ? 0xffff0000u : 0u);
  }

  // C % 8 != 0 (get_mask's 100-channel gradients): the chunk straddling Cvalid
  // carries the tensor's padding channels (never written, may hold any bits);
  // its lanes AND them away per K-step (block-uniform switch)
  const bool rag = (a.Cvalid & 7) && a.Cgp != 8;
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int st = 0; st < S - 1; ++st)
    if (st < nk) issue(kt0 + st, st);
  for (int it = 0; it < nk; ++it) {
    if (it + S - 2 < nk) {
      if (a_wave) wait_vmcnt_barrier<(S - 2) * (A_INS + B_INS)>();
      else wait_vmcnt_barrier<(S - 2) * B_INS>();
    } else {
      wait_vmcnt_barrier<0>();
    }
    if (it + S - 1 < nk) issue(kt0 + it + S - 1, (it + S - 1) % S);
    const bf16_t* base = lds + (it % S) * STAGE;
    bf16x8_t fa[FI], fb[FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int row = wi * WT_CO + i * 16 + fr;
      fa[i] = as_frag(*reinterpret_cast<const uint4*>(base + row * BK + ((fq ^ swz_b128((row >> 2) & 3)) * 8)));
    }
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int row = wj * WT_PIX + j * 16 + fr;
      uint4 v = *reinterpret_cast<const uint4*>(base + TCO * BK + row * BK + ((fq ^ swz_b128((row >> 2) & 3)) * 8));
      v.x &= bmask.x;
      v.y &= bmask.y;
      v.z &= bmask.z;
      v.w &= bmask.w;
      if (rag) v = mask_chunk(v, ((kt0 + it) % nc) * BK + 8 * fq, a.Cvalid);
      fb[j] = as_frag(v);
    }
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
  }
  igemm_epilogue<MODE, FI, FJ, WT_CO, WT_PIX>(a, acc, pix0, co0, wi, wj, lane, split, Pc, CH, CW, qy, qx, stc);
}

// ------------------------------- FWD / BWDD, pipelined kernel, hoisted gathers --
// conv_glds_kernel with the per-K-step index arithmetic hoisted out of the loop
// (the loop was issue-bound on integer address math: ~100 VALU per K-step,
// several of them quarter-rate multiplies).  Each thread's B rows carry a byte
// offset of the row's tap-(0,0) source pixel and a bitmask of the taps that land
// inside the source image; a K-step is (tap, 32-channel slice), walked by
// uniform counters, so a gather offset is base + uniform tap offset, selected
// against the mask bit (3-5 VALU per 16-B piece).  Weight pieces use a constant
// per-thread voffset and the K position as soffset.  Normal-mode operands only
// (C % 8 == 0, C > 8), no fused upsample, <= 32 taps per parity class.
EE_DEV void lds_dma16s(rsrc_t rsrc, int lds_addr, unsigned voff, int soff) {
  // the operands are wave-uniform by construction; readfirstlane makes the
  // compiler keep them in SGPRs whatever it can prove
  lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
  soff = __builtin_amdgcn_readfirstlane(soff);
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(lds_addr), "v"(voff), "s"(rsrc),
               "s"(soff)
               : "memory", "m0");
}

// Split-K finished inside conv_fast_kernel (a.ctr set; host-checked: Mrows % 4 == 0, the
// vector reduce's alignment, slab < 2 GB): every split stores its fp32 partial tile with
// sc1 16-B stores (written through, not parked in its XCD's L2); every storing wave waits
// for its stores (vmcnt 0), the workgroup barriers, one lane adds 1 to the tile's counter
// (agent-scope atomic) -- the workgroup whose add returns nsplit - 1 arrived last.  It
// resets the counter, reads every split's partial back with sc1 loads (L1/L2 bypassed:
// the hand-off form of MI355X_MICROARCH.md's cross-workgroup table, no fences), sums them
// in split order 0..nsplit-1 and applies the epilogue exactly as splitk_item4: the same
// bits as the separate reduce launch, which it replaces (one launch boundary and its
// dispatch latency less per split conv).  The other splits exit.
EE_DEV void out_pixel(const ConvArgs& a, int pc, int CH, int CW, int qy, int qx, int stc, bool cls_map, long& p,
                      long& rpix) {
  p = pc;
  rpix = pc;
  if (cls_map) {
    const int hw = CH * CW;
    const int n = pc / hw, rem = pc - n * hw;
    const int yy = rem / CW, xx = rem - yy * CW;
    const int y = qy + stc * yy, x = qx + stc * xx;
    p = ((long)n * a.OH + y) * a.OW + x;
    if (a.res_up2) rpix = ((long)n * (a.OH >> 1) + (y >> 1)) * (a.OW >> 1) + (x >> 1);
  } else if (a.res_up2) {
    const unsigned hw = (unsigned)a.OH * (unsigned)a.OW;
    const unsigned n = (unsigned)pc / hw, rem = (unsigned)pc - n * hw;
    const unsigned y = rem / (unsigned)a.OW, x = rem - y * (unsigned)a.OW;
    rpix = ((long)n * (a.OH >> 1) + (y >> 1)) * (a.OW >> 1) + (x >> 1);
  }
}

constexpr int SC1 = 16;   // buffer-op cache policy: sc1 (gfx950)

template <int MODE, int TCO, int TPIX, int FI, int FJ, int WT_CO, int WT_PIX>
EE_DEV void splitk_fused_finish(const ConvArgs& a, const f32x4_t (&acc)[FI][FJ], int pix0, int co0, int wi, int wj,
                                int lane, int tid, int split, int tile, int Pc, int CH, int CW, int qy, int qx,
                                int stc) {
  const bool cls_map = MODE == MODE_BWDD && a.ncls > 1;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(a.part, (short)0, (int)((long)a.nsplit * a.P * a.Mrows * 4), 0x00020000);
  const int fr = lane & 15;
  const unsigned zoff = (unsigned)split * (unsigned)a.P * (unsigned)a.Mrows;
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const int pc = pix0 + wj * WT_PIX + j * 16 + fr;
    if (pc >= Pc) continue;
    long p, rpix;
    out_pixel(a, pc, CH, CW, qy, qx, stc, cls_map, p, rpix);
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int co = co0 + wi * WT_CO + i * 16 + (lane >> 4) * 4;
      if (co >= a.Mrows) continue;
      __builtin_amdgcn_raw_buffer_store_b128(acc[i][j], rs, (zoff + (unsigned)p * (unsigned)a.Mrows + co) * 4u, 0,
                                             SC1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __shared__ int s_last;
  __syncthreads();
  if (tid == 0) {
    int* c = a.ctr + tile;
    // The partials were stored with sc1 (written through to memory, not parked in this
    // XCD's L2) and every wave waited for them (vmcnt(0) + barrier) before this ticket,
    // and the last arriver reads them back with sc1 loads: the hand-off of
    // cdna_hip_programming.md §6 Guideline 16 (sc1 form), which needs no release /
    // acquire fence -- an agent-scope acq_rel here writes back and invalidates the
    // whole XCD L2 per block (3-8x slower).
    const int old = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == a.nsplit - 1;
    if (old == a.nsplit - 1) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;
  // the last split: 4 channels of one pixel per item, the slab row of each split read back
  constexpr int CQ = TCO / 4, ITEMS = TPIX * CQ;
  const float gam = (a.res && a.gamma) ? *a.gamma : 1.f;
  const unsigned zstride = (unsigned)a.P * (unsigned)a.Mrows * 4u;
  for (int item = tid; item < ITEMS; item += 256) {
    const int pc = pix0 + item / CQ, co = co0 + 4 * (item % CQ);
    if (pc >= Pc || co >= a.Mrows) continue;
    long p, rpix;
    out_pixel(a, pc, CH, CW, qy, qx, stc, cls_map, p, rpix);
    uint2 gv = make_uint2(0, 0), rv = make_uint2(0, 0);
    if (MODE == MODE_BWDD && a.gate) gv = *reinterpret_cast<const uint2*>(a.gate + p * a.ldgate + co);
    if (a.res) rv = *reinterpret_cast<const uint2*>(a.res + (a.res_up2 ? rpix : p) * a.ldres + co);
    f32x4_t bv = {0.f, 0.f, 0.f, 0.f};
    if (a.bias) bv = f32x4_t{a.bias[co], a.bias[co + 1], a.bias[co + 2], a.bias[co + 3]};
    const unsigned off = ((unsigned)p * (unsigned)a.Mrows + co) * 4u;
    f32x4_t sum = {0.f, 0.f, 0.f, 0.f};
    int z = 0;
    for (; z + 8 <= a.nsplit; z += 8) {
      f32x4_t v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + (unsigned)(z + k) * zstride, 0, SC1);
#pragma unroll
      for (int k = 0; k < 8; ++k) sum += v[k];   // split order, as the reduce kernel
    }
    for (; z < a.nsplit; ++z) sum += __builtin_amdgcn_raw_buffer_load_b128(rs, off + (unsigned)z * zstride, 0, SC1);
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = act_fwd(sum[r] + bv[r], a.act, a.slope);
    if (MODE == MODE_BWDD && a.gate) {
      const float gg[4] = {lo_f(gv.x), hi_f(gv.x), lo_f(gv.y), hi_f(gv.y)};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] *= act_dgrad_from_y(gg[r], a.gate_act, a.gate_slope);
    }
    if (a.res) {
      const float rr[4] = {lo_f(rv.x), hi_f(rv.x), lo_f(rv.y), hi_f(rv.y)};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = res_combine(a.res_scale, rr[r], gam, v[r]);
    }
    if (a.out_f32) {
      *reinterpret_cast<f32x4_t*>(reinterpret_cast<float*>(a.out) + p * a.ldo + co) = {v[0], v[1], v[2], v[3]};
    } else {
      *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(a.out) + p * a.ldo + co) =
          make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    }
  }
}

template <int MODE, int TCO, int TPIX, int KS = 1, int S = CONV_STAGES, int VAR = 0>
__global__ __launch_bounds__(256, 2) void conv_fast_kernel(ConvArgs a, long src_bytes, long w_bytes) {
  constexpr int WCO = TCO >= 64 ? 2 : 1, WPIX = 4 / WCO;
  constexpr int WT_CO = TCO / WCO, WT_PIX = TPIX / WPIX;
  constexpr int FI = WT_CO / 16, FJ = WT_PIX / 16;
  constexpr int A_TOT = TCO * 4, B_TOT = TPIX * 4;     // 16-B chunks per K-step
  constexpr int A_INS = (A_TOT + 255) / 256, B_INS = B_TOT / 256;
  constexpr int STAGE = (TCO + TPIX) * BK;             // bf16 elements per stage
  static_assert(B_INS >= 1 && FI >= 1 && FJ >= 1, "tile");

  __shared__ __attribute__((aligned(16))) bf16_t lds[S * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wave / WPIX, wj = wave % WPIX;
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (a.xcd_g) {   // XCD raster (ConvArgs::xcd_g): block-uniform remap, exits before any barrier
    const int nb = a.gx * a.gy * a.gz, nbp = (nb + 7) & ~7, id = blockIdx.x;
    const int L = (id & 7) * (nbp >> 3) + (id >> 3);
    if (L >= nb) return;
    const int nbz = a.gx * a.gy;
    bz = L / nbz;
    const int r = L - bz * nbz, gsz = a.xcd_g * a.gx, grp = r / gsz, first = grp * a.xcd_g;
    const int gh = min(a.gy - first, a.xcd_g), rr = r - grp * gsz;
    by = first + rr % gh;
    bx = rr / gh;
  }
  const int cls = bz % a.ncls, split = bz / a.ncls;
  const int co0 = by * TCO;
  const bool a_wave = A_TOT >= 256 || tid < A_TOT;

  int qy = 0, qx = 0, CH = a.OH, CW = a.OW, stc = 1;
  int r0 = 0, s0 = 0, TR = a.R, TS = a.S, dqy = 0, dqx = 0;
  if (MODE == MODE_BWDD) {
    if (a.ncls > 1) {
      qy = cls / a.st;
      qx = cls - qy * a.st;
      CH = (a.OH - qy + a.st - 1) / a.st;
      CW = (a.OW - qx + a.st - 1) / a.st;
      stc = a.st;
    }
    r0 = (qy + a.ph) % a.st;
    s0 = (qx + a.pw) % a.st;
    TR = r0 < a.R ? (a.R - r0 + a.st - 1) / a.st : 0;
    TS = s0 < a.S ? (a.S - s0 + a.st - 1) / a.st : 0;
    dqy = (qy + a.ph - r0) / a.st;
    dqx = (qx + a.pw - s0) / a.st;
  }
  const int Pc = a.N * CH * CW;
  const int pix0 = bx * TPIX;
  if (pix0 >= Pc) return;  // block-uniform
  const int nc = a.Cgp / BK;
  const int nk_all = TR * TS * nc;
  const int kchunk = (nk_all + a.nsplit - 1) / a.nsplit;
  const int kt0 = min(nk_all, split * kchunk), kt1 = min(nk_all, kt0 + kchunk);
  const int nk = kt1 - kt0;

  const int rsub = tid >> 2;
  const int kc8 = ((tid & 3) ^ swz_b128((tid >> 4) & 3)) * 8;  // swizzled 8-channel chunk of this thread
  const int ld2 = a.lds_src * 2;
  // wide pair stages: 128-B rows (8 chunks), this thread's row tid / 8 (+ 32 i) and
  // physical chunk tid & 7 holding logical chunk (tid & 7) ^ ((row >> 1) & 7)
  constexpr bool WIDE_OK = VAR == 2 && KS == 2 && TCO >= 64;
  const bool wide = WIDE_OK && a.wide;
  const int wrow = tid >> 3;
  const int wkc8 = ((tid & 7) ^ ((wrow >> 1) & 7)) * 8;
  auto pix_state = [&](int p, int kcb, int& pbo, unsigned& vmo) {
    const bool ok = p < Pc;
    const int pp = ok ? p : 0;
    const int hw = CH * CW;
    const int n = pp / hw;
    const int rem = pp - n * hw;
    const int yy = rem / CW;
    const int xx = rem - yy * CW;
    int y0, x0;
    if (MODE == MODE_FWD) {
      y0 = yy * a.st - a.ph;
      x0 = xx * a.st - a.pw;
    } else {
      y0 = yy + dqy;
      x0 = xx + dqx;
    }
    unsigned m = 0;
    for (int ta = 0; ta < TR; ++ta) {
      const int iy = MODE == MODE_FWD ? y0 + ta : y0 - ta;
      if ((unsigned)iy >= (unsigned)a.IH) continue;
      for (int tb = 0; tb < TS; ++tb) {
        const int ix = MODE == MODE_FWD ? x0 + tb : x0 - tb;
        if ((unsigned)ix < (unsigned)a.IW) m |= 1u << (ta * TS + tb);
      }
    }
    vmo = ok ? m : 0u;
    pbo = ((n * a.IH + y0) * a.IW + x0) * ld2 + kcb * 2;
  };
  int pb[B_INS];
  unsigned vm[B_INS];
  unsigned aoff[A_INS];
  constexpr int B_INW = WIDE_OK ? TPIX / 32 : 1, A_INW = WIDE_OK ? TCO / 32 : 1;  // 16-B chunks / 256 threads
  int pbw[B_INW];
  unsigned vmw[B_INW], aoffw[A_INW];
  if (!wide) {
#pragma unroll
    for (int i = 0; i < B_INS; ++i) pix_state(pix0 + i * 64 + rsub, kc8, pb[i], vm[i]);
#pragma unroll
    for (int i = 0; i < A_INS; ++i) aoff[i] = (unsigned)(((co0 + i * 64 + rsub) * a.Kw + kc8) * 2);
  } else {
#pragma unroll
    for (int i = 0; i < B_INW; ++i) pix_state(pix0 + i * 32 + wrow, wkc8, pbw[i], vmw[i]);
#pragma unroll
    for (int i = 0; i < A_INW; ++i) aoffw[i] = (unsigned)(((co0 + i * 32 + wrow) * a.Kw + wkc8) * 2);
  }

  const rsrc_t rs_src = make_rsrc(a.src, src_bytes);
  const rsrc_t rs_w = make_rsrc(a.wp, w_bytes);
  const int lds0 = (int)(uintptr_t)(lds_void_t*)lds;

  // uniform K-step walker: tap (ta, tb), 32-channel slice cs
  int w_t = nc > 0 ? kt0 / nc : 0;
  int w_cs = kt0 - w_t * nc;
  int w_ta = TS > 0 ? w_t / TS : 0;
  int w_tb = w_t - w_ta * TS;
  const int IW = a.IW;
  auto issue = [&](int buf) {
    const int t = w_ta * TS + w_tb;
    const int c = w_cs * BK;
    int toff, kw;
    if (MODE == MODE_FWD) {
      toff = (w_ta * IW + w_tb) * ld2 + c * 2;
      kw = (w_ta * a.S + w_tb) * a.Cgp + c;
    } else {
      toff = c * 2 - (w_ta * IW + w_tb) * ld2;
      kw = ((r0 + a.st * w_ta) * a.S + s0 + a.st * w_tb) * a.Cgp + c;
    }
    const int cv = a.Cvalid - c;  // chunk valid iff kc8 < cv
    const int base = lds0 + buf * (STAGE * 2);
    if (a_wave) {
#pragma unroll
      for (int i = 0; i < A_INS; ++i) lds_dma16s(rs_w, base + (i * 256 + wave * 64) * 16, aoff[i], kw * 2);
    }
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      const bool ok = ((vm[i] >> t) & 1u) && kc8 < cv;
      const unsigned off = ok ? (unsigned)(pb[i] + toff) : OOB;
      lds_dma16s(rs_src, base + TCO * BK * 2 + (i * 256 + wave * 64) * 16, off, 0);
    }
    if (++w_cs == nc) {
      w_cs = 0;
      if (++w_tb == TS) {
        w_tb = 0;
        ++w_ta;
      }
    }
  };

  // one wide stage = ring slots (sp, sp + 1): A rows then B rows of 128 B, the
  // pair's two 32-channel slices side by side
  auto issue_wide = [&](int sp) {
    const int t = w_ta * TS + w_tb;
    const int c = w_cs * BK;
    int toff, kw;
    if (MODE == MODE_FWD) {
      toff = (w_ta * IW + w_tb) * ld2 + c * 2;
      kw = (w_ta * a.S + w_tb) * a.Cgp + c;
    } else {
      toff = c * 2 - (w_ta * IW + w_tb) * ld2;
      kw = ((r0 + a.st * w_ta) * a.S + s0 + a.st * w_tb) * a.Cgp + c;
    }
    const int cv = a.Cvalid - c;
    const int base = lds0 + sp * (STAGE * 2);
#pragma unroll
    for (int i = 0; i < A_INW; ++i) lds_dma16s(rs_w, base + (i * 256 + wave * 64) * 16, aoffw[i], kw * 2);
#pragma unroll
    for (int i = 0; i < B_INW; ++i) {
      const bool ok = ((vmw[i] >> t) & 1u) && wkc8 < cv;
      const unsigned off = ok ? (unsigned)(pbw[i] + toff) : OOB;
      lds_dma16s(rs_src, base + TCO * 2 * BK * 2 + (i * 256 + wave * 64) * 16, off, 0);
    }
    w_cs += 2;  // both slices of this tap (even slice count per tap)
    if (w_cs == nc) {
      w_cs = 0;
      if (++w_tb == TS) {
        w_tb = 0;
        ++w_ta;
      }
    }
  };
  f32x4_t acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  // KS K-steps per barrier: stages it .. it+KS-1 are multiplied while stages up
  // to it+S-1 are in flight; the KS stages issued after the barrier reuse the
  // slots multiplied in the previous iteration
  constexpr int YNG = S - 2 * KS;  // stages allowed in flight at the wait
  static_assert(YNG >= 0, "stages");
  if (wide) {
#pragma unroll
    for (int st = 0; st < S - KS; st += 2)   // (S - KS) / 2 wide stages: slots (st, st + 1)
      if (st < nk) issue_wide(st);
  } else {
#pragma unroll
    for (int st = 0; st < S - KS; ++st)
      if (st < nk) issue(st);
  }
  // C % 8 != 0: the 16-B chunk straddling Cvalid carries the row's padding
  // channels (never written, any bits): ANDed away in the B fragments of the
  // K-step's slice (block-uniform switch; chunks past the row read the next
  // pixel's finite channels against zero weights, as for any Cvalid < Cgp)
  const bool rag = (a.Cvalid & 7) != 0;
  auto rag_mask = [&](uint4 v, int kt) {
    return rag ? mask_chunk(v, (kt % nc) * BK + 8 * fq, a.Cvalid) : v;
  };
  auto rd_frags_wide = [&](int sp, int half, bf16x8_t (&fa_)[FI], bf16x8_t (&fb_)[FJ], int kt) {
    const bf16_t* base = lds + sp * STAGE;
    const int q = 4 * half + fq;
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int row = wi * WT_CO + i * 16 + fr;
      fa_[i] = as_frag(*reinterpret_cast<const uint4*>(base + row * 2 * BK + ((q ^ ((row >> 1) & 7)) * 8)));
    }
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int row = wj * WT_PIX + j * 16 + fr;
      fb_[j] = as_frag(rag_mask(*reinterpret_cast<const uint4*>(base + TCO * 2 * BK + row * 2 * BK +
                                                        ((q ^ ((row >> 1) & 7)) * 8)), kt));
    }
  };
  auto rd_frags = [&](int stage, bf16x8_t (&fa_)[FI], bf16x8_t (&fb_)[FJ], int kt) {
    const bf16_t* base = lds + stage * STAGE;
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int row = wi * WT_CO + i * 16 + fr;
      fa_[i] = as_frag(*reinterpret_cast<const uint4*>(base + row * BK + ((fq ^ swz_b128((row >> 2) & 3)) * 8)));
    }
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int row = wj * WT_PIX + j * 16 + fr;
      fb_[j] = as_frag(rag_mask(
          *reinterpret_cast<const uint4*>(base + TCO * BK + row * BK + ((fq ^ swz_b128((row >> 2) & 3)) * 8)), kt));
    }
  };
  int it0 = 0;
  if (VAR == 2 && KS == 2) {
    // straight-line pairs: the second stage's fragment reads interleaved with
    // the first stage's MFMAs (sched_group_barrier), so their LDS latency hides
    for (; it0 + 1 < nk; it0 += 2) {
      if (it0 + S - 2 <= nk) {
        if (a_wave) wait_vmcnt_barrier<YNG * (A_INS + B_INS)>();
        else wait_vmcnt_barrier<YNG * B_INS>();
      } else {
        wait_vmcnt_barrier<0>();
      }
      bf16x8_t fa0[FI], fb0[FJ], fa1[FI], fb1[FJ];
      if (wide) {
        if (it0 + S - 2 < nk) issue_wide((it0 + S - 2) % S);
        rd_frags_wide(it0 % S, 0, fa0, fb0, kt0 + it0);
        rd_frags_wide(it0 % S, 1, fa1, fb1, kt0 + it0 + 1);
      } else {
        if (it0 + S - 2 < nk) issue((it0 + S - 2) % S);
        if (it0 + S - 1 < nk) issue((it0 + S - 1) % S);
        rd_frags(it0 % S, fa0, fb0, kt0 + it0);
        rd_frags((it0 + 1) % S, fa1, fb1, kt0 + it0 + 1);
      }
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa0[i], fb0[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1[i], fb1[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int r = 0; r < FI + FJ; ++r) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
      for (int r = 0; r < FI + FJ; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * FI * FJ - (FI + FJ), 0);
    }
  }
  for (int it = it0; it < nk; it += KS) {
    if (it + S - KS <= nk) {
      if (a_wave) wait_vmcnt_barrier<YNG * (A_INS + B_INS)>();
      else wait_vmcnt_barrier<YNG * B_INS>();
    } else {
      wait_vmcnt_barrier<0>();
    }
#pragma unroll
    for (int k = 0; k < KS; ++k)
      if (it + S - KS + k < nk) issue((it + S - KS + k) % S);
    bf16x8_t fa[KS][FI], fb[KS][FJ];
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      if (it + k >= nk) break;
      const bf16_t* base = lds + ((it + k) % S) * STAGE;
#pragma unroll
      for (int i = 0; i < FI; ++i) {
        const int row = wi * WT_CO + i * 16 + fr;
        fa[k][i] = as_frag(*reinterpret_cast<const uint4*>(base + row * BK + ((fq ^ swz_b128((row >> 2) & 3)) * 8)));
      }
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int row = wj * WT_PIX + j * 16 + fr;
        fb[k][j] = as_frag(rag_mask(
            *reinterpret_cast<const uint4*>(base + TCO * BK + row * BK + ((fq ^ swz_b128((row >> 2) & 3)) * 8)), kt0 + it + k));
      }
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      if (it + k >= nk) break;
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[k][i], fb[k][j], acc[i][j], 0, 0, 0);
    }
  }
  static_assert(TPIX * TCO * 4 <= S * STAGE * 2, "staged epilogue tile exceeds the LDS ring");
  if (a.stage_epi) {
    staged_epilogue<MODE, TCO, TPIX, FI, FJ, WT_CO, WT_PIX>(a, acc, reinterpret_cast<float4*>(lds), pix0, co0, wi, wj,
                                                            lane, tid, Pc, CH, CW, qy, qx, stc);
    return;
  }
  if (a.ctr) {   // split-K finished here (block-uniform)
    const int tile = a.xcd_g ? (cls * a.gy + by) * a.gx + bx
                             : (cls * (int)gridDim.y + (int)blockIdx.y) * (int)gridDim.x + (int)blockIdx.x;
    splitk_fused_finish<MODE, TCO, TPIX, FI, FJ, WT_CO, WT_PIX>(a, acc, pix0, co0, wi, wj, lane, tid, split, tile, Pc,
                                                                CH, CW, qy, qx, stc);
    return;
  }
  igemm_epilogue<MODE, FI, FJ, WT_CO, WT_PIX>(a, acc, pix0, co0, wi, wj, lane, split, Pc, CH, CW, qy, qx, stc);
}

// ------------------------------------ 3x3 stride-1 convs: LDS halo tiles --
// FWD / BWDD of 3x3 / stride-1 / pad-1 convs (resD conv_r[1] models.py:270,
// the SAGB / Cum 3x3 convs models.py:104-143 incl. the nearest-2x upsample, the
// data gradients of all of them).  The tile kernels gather every source pixel
// once per tap (9x through L2 -> LDS, 64 B pieces), which bounds them at the
// per-CU LDS-DMA rate.  Here one workgroup owns 64 output channels x a TH x 32
// pixel tile of one image; per 32-channel input slice it stages the
// (TH + 2) x 34 source halo ONCE (LDS-DMA; out-of-image pixels read zeros
// through the buffer bounds check) together with all 9 taps' 64 x 32 weight
// slabs, double-buffered per slice, so one barrier covers 9 taps x 16 MFMAs
// per wave and the next tap's fragments are read while the current tap's
// MFMAs run.  Halo pixel h = (hy, hx)'s 16-B chunk q sits in LDS slot h * 4 +
// (q ^ ((hx >> 1) & 2)): conflict-free ds_read_b128 for any 16 consecutive
// pixels of a halo row, i.e. at every tap shift, and a tap's row shift is an
// immediate offset.  BWDD reads the mirrored tap (2 - r, 2 - s) of the same
// halo with the transposed pack.  Epilogue through LDS (fp32 tile, 16-B runs of 8
// channels): bias, activation, gate, residual exactly as staged_epilogue.
// K order: slice-major, tap inner (the tile kernels: tap-major) -- a different
// fp32 summation order, deterministic.
constexpr int HALO_TW = 32, HALO_TCO = 64;
// Diagnostic builds only (tools/gpu_halo_knock.sh compiles copies of the library
// with -DEEGAN_HALO_KNOCK=bits): 1 = no operand loads, 2 = no output stores,
// 4 = no MFMAs.  The shipped library is built with 0.
#ifndef EEGAN_HALO_KNOCK
#define EEGAN_HALO_KNOCK 0
#endif

EE_DEV int halo_swz(int hx) { return (hx >> 1) & 2; }

// RAG: Cvalid % 8 != 0 -- the 16-B chunk straddling Cvalid carries the row's padding
// channels (any bits): masked in the B fragments of that slice (as the tile kernels'
// rag_mask).  Output rows Mrows % 8 != 0: the straddling chunk's valid channels are
// stored one by one, nothing past Mrows is written.
template <int MODE, int TH, int WPX, bool RAG = false, int NBUF = 2>
__global__ __launch_bounds__(64 * WPX, NBUF == 1 ? (TH == 4 ? 3 : 2) : 1) void conv_halo3_kernel(ConvArgs a, long src_bytes,
                                                                               long w_bytes) {
  constexpr int NT = 64 * WPX, TW = HALO_TW, TCO = HALO_TCO, FI = TCO / 16;
  constexpr int WROWS = TH / WPX, CB = TW / 16, FJ = WROWS * CB;
  constexpr int HW2 = TW + 2, HP = (TH + 2) * HW2, HOPS = (HP * 4 + NT - 1) / NT, HBUF = HOPS * NT * 16;
  constexpr int WCH = 9 * TCO * 4, WOPS = (WCH + NT - 1) / NT, WBUF = WOPS * NT * 16;
  constexpr int TPIX = TH * TW, NCK = TCO / 4;
  // NBUF = 1: one slice buffer, two workgroups per CU (one's loads under the other's MFMAs)
  constexpr int LDSB = NBUF * (HBUF + WBUF) > TPIX * TCO * 4 ? NBUF * (HBUF + WBUF) : TPIX * TCO * 4;
  static_assert(WROWS >= 1 && (NBUF == 1 || NBUF == 2), "halo tile");
  __shared__ __attribute__((aligned(16))) char lds[LDSB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wj = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_x = a.OW / TW, tiles_y = a.OH / TH;
  int b = blockIdx.x;
  const int tx = b % tiles_x;
  b /= tiles_x;
  const int ty = b % tiles_y;
  const int n = b / tiles_y;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int co0 = blockIdx.y * TCO;
  const int nslice = a.Cgp / BK;
  const int lds0 = (int)(uintptr_t)(lds_void_t*)lds;
  const rsrc_t rs_src = make_rsrc(a.src, src_bytes);
  const rsrc_t rs_w = make_rsrc(a.wp, w_bytes);
  const int PH = a.IH >> a.up2, PW = a.IW >> a.up2;   // physical source grid (FWD up2: half resolution)

  // this thread's halo pieces (slice 0 offsets; OOB outside the image) and their channel chunk
  unsigned hoff[HOPS];
  int hq[HOPS];
#pragma unroll
  for (int i = 0; i < HOPS; ++i) {
    const int L = i * NT + tid, h = L >> 2;
    const int hy = h / HW2, hx = h - hy * HW2, q = (L & 3) ^ halo_swz(hx);
    const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;   // logical source pixel (pad 1)
    hq[i] = q;
    hoff[i] = (h < HP && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW)
                  ? (unsigned)((((n * PH + (iy >> a.up2)) * PW + (ix >> a.up2)) * a.lds_src + q * 8) * 2)
                  : OOB;
  }
  // weight pieces: stage image [tap][row][4 chunks, swizzled as the tile kernels' rows]
  unsigned woff[WOPS];
#pragma unroll
  for (int i = 0; i < WOPS; ++i) {
    const int L = i * NT + tid, t = L / (TCO * 4), rem = L - t * (TCO * 4);
    const int row = rem >> 2, q = (rem & 3) ^ swz_b128((row >> 2) & 3);
    woff[i] = L < WCH ? (unsigned)(((co0 + row) * a.Kw + t * a.Cgp + q * 8) * 2) : OOB;
  }
  auto issue = [&](int cs) {   // slice cs: halo into buffer cs & 1, weights into buffer cs & 1
    if (EEGAN_HALO_KNOCK & 1) return;
    const int buf = NBUF == 2 ? cs & 1 : 0;
#pragma unroll
    for (int i = 0; i < HOPS; ++i) {
      const bool ok = hoff[i] != OOB && cs * BK + hq[i] * 8 < a.Cvalid;
      // soffset is wave-uniform (s_ register); an out-of-range lane's OOB voffset stays out of range with it
      lds_dma16s(rs_src, lds0 + buf * HBUF + (i * NT + wj * 64) * 16, ok ? hoff[i] : OOB, cs * 64);
    }
#pragma unroll
    for (int i = 0; i < WOPS; ++i)
      lds_dma16s(rs_w, lds0 + NBUF * HBUF + buf * WBUF + (i * NT + wj * 64) * 16, woff[i], cs * 64);
  };

  f32x4_t acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  // fragment addresses: a per-slice base register + an immediate for every tap.  Weights:
  // row i * 16 + fr of tap t at woff + t * 4096 + i * 1024 (the chunk swizzle of rows
  // i * 16 + fr is i-independent).  Halo: pixel column hx's swizzle depends on hx only (and
  // is the same for hx + 16), so B fragment j = (row jr, 16-column block jc) at tap shift
  // (oyh, oxh) is fhoff[oxh] + (oyh + jr) * HW2 * 64 + jc * 1024: 3 base registers.
  const int fwoff = NBUF * HBUF + fr * 64 + ((fq ^ swz_b128((fr >> 2) & 3)) << 4);
  int fhoff[3];
#pragma unroll
  for (int sx = 0; sx < 3; ++sx)
    fhoff[sx] = ((wj * WROWS * HW2 + fr + sx) << 6) + ((fq ^ halo_swz(fr + sx)) << 4);
  uint4 rmsk = make_uint4(~0u, ~0u, ~0u, ~0u);   // RAG: this lane's chunk mask in the current slice
  auto rd = [&](int cs, int t, bf16x8_t (&fa)[FI], bf16x8_t (&fb)[FJ]) {
    const int ta = t / 3, tb = t - ta * 3;
    const int oyh = MODE == MODE_FWD ? ta : 2 - ta, oxh = MODE == MODE_FWD ? tb : 2 - tb;
    const char* wbase = lds + (NBUF == 2 ? cs & 1 : 0) * WBUF + fwoff;
    const char* hbase = lds + (NBUF == 2 ? cs & 1 : 0) * HBUF;
#pragma unroll
    for (int i = 0; i < FI; ++i)
      fa[i] = as_frag(*reinterpret_cast<const uint4*>(wbase + t * TCO * 64 + i * 1024));
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      uint4 v = *reinterpret_cast<const uint4*>(hbase + fhoff[oxh] + (oyh + j / CB) * HW2 * 64 + (j % CB) * 1024);
      if (RAG) v = make_uint4(v.x & rmsk.x, v.y & rmsk.y, v.z & rmsk.z, v.w & rmsk.w);
      fb[j] = as_frag(v);
    }
  };
  issue(0);
  for (int cs = 0; cs < nslice; ++cs) {
    wait_vmcnt_barrier<0>();   // slice cs landed; every wave is done with slice cs - 1's buffers
    if (NBUF == 2 && cs + 1 < nslice) issue(cs + 1);
    if (RAG) rmsk = mask_chunk(make_uint4(~0u, ~0u, ~0u, ~0u), cs * BK + 8 * fq, a.Cvalid);
    bf16x8_t fa[2][FI], fb[2][FJ];
    rd(cs, 0, fa[0], fb[0]);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      // tap t + 1's fragments are requested before tap t's MFMAs (the compiler sinks each
      // read to its first use; pinning them ahead with scheduling fences measured the same,
      // within 1 %: the LDS latency is not what bounds this loop)
      if (t + 1 < 9) rd(cs, t + 1, fa[(t + 1) & 1], fb[(t + 1) & 1]);
      if (EEGAN_HALO_KNOCK & 4) continue;
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t & 1][i], fb[t & 1][j], acc[i][j], 0, 0, 0);
    }
    if (NBUF == 1 && cs + 1 < nslice) {
      __syncthreads();   // every wave is done with the one buffer
      issue(cs + 1);
    }
  }
  // epilogue: the gate / residual runs of this thread's items are loaded first, so their
  // latency overlaps the LDS staging; fp32 tile [pixel][16 chunks of 4 channels], chunk c
  // of pixel p at c ^ (p & 15)
  constexpr int NIT = TPIX * (TCO / 8) / NT;
  uint4 gpre[NIT], rpre[NIT];
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int item = k * NT + tid, p = item / (TCO / 8), e = item % (TCO / 8);
    const int co = co0 + 8 * e;
    const int y = oy0 + p / TW, x = ox0 + p % TW;
    const long gp = ((long)n * a.OH + y) * a.OW + x;
    gpre[k] = rpre[k] = make_uint4(0, 0, 0, 0);
    if (co < a.Mrows) {
      if (MODE == MODE_BWDD && a.gate) gpre[k] = *reinterpret_cast<const uint4*>(a.gate + gp * a.ldgate + co);
      if (a.res) {
        const long rp = a.res_up2 ? ((long)n * (a.OH >> 1) + (y >> 1)) * (a.OW >> 1) + (x >> 1) : gp;
        rpre[k] = *reinterpret_cast<const uint4*>(a.res + rp * a.ldres + co);
      }
    }
  }
  __syncthreads();
  float4* st = reinterpret_cast<float4*>(lds);
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const int p = (wj * WROWS + j / CB) * TW + (j % CB) * 16 + fr;
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int c = i * 4 + fq;
      st[p * NCK + (c ^ (p & 15))] = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
  }
  __syncthreads();
  const float gam = (a.res && a.gamma) ? *a.gamma : 1.f;
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int item = k * NT + tid, p = item / (TCO / 8), e = item % (TCO / 8);
    const int co = co0 + 8 * e;
    if (co >= a.Mrows) continue;
    const float4 lo = st[p * NCK + ((2 * e) ^ (p & 15))];
    const float4 hi = st[p * NCK + ((2 * e + 1) ^ (p & 15))];
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    const int y = oy0 + p / TW, x = ox0 + p % TW;
    const long gp = ((long)n * a.OH + y) * a.OW + x;
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = act_fwd(v[r] + ((a.bias && co + r < a.Mrows) ? a.bias[co + r] : 0.f), a.act, a.slope);
    if (MODE == MODE_BWDD && a.gate) {
      const uint4 gv = gpre[k];
      const uint32_t gw[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[2 * r] *= act_dgrad_from_y(lo_f(gw[r]), a.gate_act, a.gate_slope);
        v[2 * r + 1] *= act_dgrad_from_y(hi_f(gw[r]), a.gate_act, a.gate_slope);
      }
    }
    if (a.res) {
      const uint4 rv = rpre[k];
      const uint32_t rw[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[2 * r] = res_combine(a.res_scale, lo_f(rw[r]), gam, v[2 * r]);
        v[2 * r + 1] = res_combine(a.res_scale, hi_f(rw[r]), gam, v[2 * r + 1]);
      }
    }
    bf16_t* dst = reinterpret_cast<bf16_t*>(a.out) + gp * a.ldo + co;
    if (co + 8 > a.Mrows) {   // the output row's last, partial chunk
      for (int r = 0; r < a.Mrows - co; ++r) dst[r] = f2bf(v[r]);
      continue;
    }
    const uint4 o = make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
    if (!(EEGAN_HALO_KNOCK & 2) || o.x == 0x7fc17fc1u) *reinterpret_cast<uint4*>(dst) = o;
  }
}


// ------------------- 3x3 stride-1 convs on 64 input channels: resident weights --
// conv_halo3_kernel for the 64-channel inputs (D256's 64-ch 128^2 resD conv, the
// generator's 64-ch layers and their data gradients), where its per-slice
// weight slabs (9 taps x 64 x 32, 37 KB) outweigh the halo (13 KB) 3 : 1.  Here
// a workgroup stages ALL 9 x 64 x 64 weights of its output-channel tile once
// (72 KB, resident for its lifetime) and walks TPB horizontally consecutive
// 4 x 32-pixel tiles; per tile only the 6 x 34 source halo moves, as whole
// 128-B lines (64 channels of a pixel = one line, against the half-line 64-B
// pieces of 32-channel slices), double-buffered: tile k + 1's halo streams in
// under tile k's 144 MFMAs per wave, its fragment reads interleaved one per
// MFMA gap (one wave per SIMD: nothing else hides a read the compiler would
// sink to its first use).  The epilogue runs on the MFMA fragments: bias,
// activation (none / relu / leaky relu, branch-free), the gate and residual
// tiles -- LDS-DMA'd beside the next halo, so no compiler-counted load waits on
// the in-flight halo -- then bf16 through LDS for 16-B row stores.  LDS: 72 KB
// weights + 2 x 28 KB halo buffers + 2 x 16 KB gate / residual tiles = 160 KB,
// one workgroup per CU.
// Swizzles (brute-forced over gfx950's b128 / b64 lane groups): halo and weight
// rows (128 B) hold 16-B chunk q at slot q ^ (r & 6) -- conflict-free
// ds_read_b128 for any 16 consecutive rows, both 32-channel halves, so a
// fragment read is a base register (tap column shift x half) + an immediate;
// the 128-pixel gate / residual / output tiles hold chunk q of pixel p at
// q ^ ((p >> 1) & 7) -- conflict-free ds_read_b64 of a fragment's 4 channels
// and ds_read_b128 of a store's 8.  K order as conv_halo3_kernel (32-channel half
// outer, tap inner) and the same epilogue arithmetic: the same bits.
// Host-checked: Cgp == Cvalid == 64, Mrows % 64 == 0, act / gate_act in {none,
// relu, lrelu}, 16-B aligned rows.
#ifndef HALO_R_PIN
#define HALO_R_PIN 1
#endif
EE_DEV int tile_swz(int p) { return (p >> 1) & 7; }

template <int MODE>
__global__ __launch_bounds__(256, 1) void conv_halo3r_kernel(ConvArgs a, long src_bytes, long w_bytes, int tpb,
                                                             int knock) {
  constexpr int NT = 256, TH = 4, TW = HALO_TW, TCO = HALO_TCO, FI = TCO / 16, CB = TW / 16, FJ = CB;
  constexpr int HW2 = TW + 2, HP = (TH + 2) * HW2, HOPS = (HP * 8 + NT - 1) / NT, HBUF = HOPS * NT * 16;
  constexpr int WSL = 9 * TCO * 8, WOPS = WSL / NT, WBYTES = WSL * 16;
  constexpr int TPIX = TH * TW, GRB = TPIX * TCO * 2, NIT = GRB / 16 / NT;
  constexpr int GOFF = WBYTES + 2 * HBUF, ROFF = GOFF + GRB;
  static_assert(WSL % NT == 0 && NIT == 4 && GRB <= HBUF && ROFF + GRB <= 163840, "halo3r tile");
  __shared__ __attribute__((aligned(16))) char lds[ROFF + GRB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wj = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_x = a.OW / TW, tiles_y = a.OH / TH, ntiles = a.N * tiles_x * tiles_y;
  const int t0 = blockIdx.x * tpb, t1 = min(ntiles, t0 + tpb);
  const int co0 = blockIdx.y * TCO;
  const int lds0 = (int)(uintptr_t)(lds_void_t*)lds;
  const rsrc_t rs_src = make_rsrc(a.src, src_bytes);
  const rsrc_t rs_w = make_rsrc(a.wp, w_bytes);
  const bool has_gate = MODE == MODE_BWDD && a.gate, has_res = a.res != nullptr;
  const rsrc_t rs_g = make_rsrc(has_gate ? (const void*)a.gate : a.src, 0x7fffffffL);
  const rsrc_t rs_r = make_rsrc(has_res ? (const void*)a.res : a.src, 0x7fffffffL);
  const int PH = a.IH >> a.up2, PW = a.IW >> a.up2;

  // weights once: slot L = (tap, row, chunk q) holds source chunk q ^ (row & 6)
#pragma unroll
  for (int i = 0; i < WOPS; ++i) {
    const int L = i * NT + tid, t = L / (TCO * 8), rem = L - t * (TCO * 8);
    const int row = rem >> 3, q = (rem & 7) ^ (row & 6);
    lds_dma16s(rs_w, lds0 + (i * NT + wj * 64) * 16, (unsigned)(((co0 + row) * a.Kw + t * 64 + q * 8) * 2), 0);
  }
  auto tile_origin = [&](int tile, int& n, int& oy0, int& ox0) {
    int b = tile;
    const int tx = b % tiles_x;
    b /= tiles_x;
    const int ty = b % tiles_y;
    n = b / tiles_y;
    oy0 = ty * TH;
    ox0 = tx * TW;
  };
  auto issue_halo = [&](int tile, int buf) {
    int n, oy0, ox0;
    tile_origin(tile, n, oy0, ox0);
#pragma unroll
    for (int i = 0; i < HOPS; ++i) {
      const int L = i * NT + tid, h = L >> 3;
      const int hy = h / HW2, hx = h - hy * HW2, q = (L & 7) ^ (hx & 6);
      const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
      const unsigned off = (h < HP && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW)
                               ? (unsigned)((((n * PH + (iy >> a.up2)) * PW + (ix >> a.up2)) * a.lds_src + q * 8) * 2)
                               : OOB;
      lds_dma16s(rs_src, lds0 + WBYTES + buf * HBUF + (i * NT + wj * 64) * 16, off, 0);
    }
  };
  // the tile's gate / residual chunks: slot L = (pixel p, chunk q) holds chunk q ^ tile_swz(p)
  auto issue_gr = [&](int tile) {
    int n, oy0, ox0;
    tile_origin(tile, n, oy0, ox0);
#pragma unroll
    for (int j = 0; j < NIT; ++j) {
      const int L = j * NT + tid, p = L >> 3, q = (L & 7) ^ tile_swz(p);
      const int y = oy0 + p / TW, x = ox0 + p % TW;
      const int dst = (j * NT + wj * 64) * 16;
      if (has_gate)
        lds_dma16s(rs_g, lds0 + GOFF + dst, (unsigned)((((n * a.OH + y) * a.OW + x) * a.ldgate + co0 + q * 8) * 2), 0);
      if (has_res) {
        const int rp = a.res_up2 ? (n * (a.OH >> 1) + (y >> 1)) * (a.OW >> 1) + (x >> 1) : (n * a.OH + y) * a.OW + x;
        lds_dma16s(rs_r, lds0 + ROFF + dst, (unsigned)((rp * a.ldres + co0 + q * 8) * 2), 0);
      }
    }
  };

  const int fr = lane & 15, fq = lane >> 4;
  // A fragment (row i * 16 + fr, chunk kh * 4 + fq) of tap t: wbase[kh] + t * 8192 + i * 2048
  int wbase[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) wbase[kh] = fr * 128 + (((kh * 4 + fq) ^ (fr & 6)) << 4);
  // B fragment (halo row wj + oyh, column block j, tap column shift sx, half kh):
  // hbase[sx][kh] + oyh * HW2 * 128 + j * 2048 (columns c and c + 16 share the swizzle)
  int hbase[3][2];
#pragma unroll
  for (int sx = 0; sx < 3; ++sx)
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
      hbase[sx][kh] = (wj * HW2 + fr + sx) * 128 + (((kh * 4 + fq) ^ ((fr + sx) & 6)) << 4);
  // fragment (i, j) = 4 channels i * 16 + 4 fq .. of pixel wj * 32 + j * 16 + fr: its 8-B
  // piece in the 128-pixel tiles
  int tslot[FI][FJ];
  float bias[FI][4];
#pragma unroll
  for (int i = 0; i < FI; ++i) {
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int p = wj * TW + j * 16 + fr, c = 2 * i + (fq >> 1);
      tslot[i][j] = p * 128 + ((c ^ tile_swz(p)) << 4) + (fq & 1) * 8;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[i][r] = a.bias ? a.bias[co0 + i * 16 + fq * 4 + r] : 0.f;
  }
  const bool relu = a.act == ACT_RELU;
  const float sl1 = a.act == ACT_LRELU ? a.slope : 1.f;
  const float gneg = a.gate_act == ACT_RELU ? 0.f : a.gate_act == ACT_LRELU ? a.gate_slope : 1.f;
  const float gam = (has_res && a.gamma) ? *a.gamma : 1.f;
  const float rsc = a.res_scale;

  if (t0 < t1) issue_halo(t0, 0);
  for (int tile = t0, k = 0; tile < t1; ++tile, ++k) {
    int n, oy0, ox0;
    tile_origin(tile, n, oy0, ox0);
    const int buf = k & 1;
    // tile k's halo landed (and at k = 0 the weights): every older piece of this wave but
    // the previous tile's NIT output stores, then the barrier for every wave's pieces;
    // past it every wave is done with tile k - 1 (its buffers and gate / residual tiles)
    if (k == 0) wait_vmcnt_barrier<0>();
    else wait_vmcnt_barrier<NIT>();
    issue_gr(tile);
    const bool more = tile + 1 < t1 && !(knock & 1);
    if (more) issue_halo(tile + 1, buf ^ 1);

    f32x4_t acc[FI][FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const char* hb = lds + WBYTES + buf * HBUF;
    auto rd = [&](int kh, int t, bf16x8_t (&fa)[FI], bf16x8_t (&fb)[FJ]) {
      const int ta = t / 3, tb = t - ta * 3;
      const int oyh = MODE == MODE_FWD ? ta : 2 - ta, oxh = MODE == MODE_FWD ? tb : 2 - tb;
#pragma unroll
      for (int i = 0; i < FI; ++i)
        fa[i] = as_frag(*reinterpret_cast<const uint4*>(lds + wbase[kh] + t * (TCO * 128) + i * 2048));
#pragma unroll
      for (int j = 0; j < FJ; ++j)
        fb[j] = as_frag(*reinterpret_cast<const uint4*>(hb + hbase[oxh][kh] + oyh * (HW2 * 128) + j * 2048));
    };
    // 18 K-steps (channel half kh outer, tap inner); step s + 1's 6 fragment reads are
    // interleaved one per MFMA gap with step s's 8 MFMAs
    {
      bf16x8_t fa[2][FI], fb[2][FJ];
      rd(0, 0, fa[0], fb[0]);
      if (HALO_R_PIN) __builtin_amdgcn_sched_group_barrier(0x100, FI + FJ, 0);   // step 0's reads first
#pragma unroll
      for (int s = 0; s < 18; ++s) {
        if (s + 1 < 18) rd((s + 1) / 9, (s + 1) % 9, fa[(s + 1) & 1], fb[(s + 1) & 1]);
#pragma unroll
        for (int i = 0; i < FI; ++i)
#pragma unroll
          for (int j = 0; j < FJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s & 1][i], fb[s & 1][j], acc[i][j], 0, 0, 0);
        if (HALO_R_PIN) {
#pragma unroll
          for (int m = 0; m < FI * FJ; ++m) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
            if (s + 1 < 18 && m < FI + FJ) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // one DS read
          }
        }
      }
    }
    if (knock & 2) {   // diagnostics: no epilogue (one store keeps the MFMAs live)
      if (acc[0][0][0] == 1234.5f) a.part[tid] = acc[0][1][1] + acc[1][0][2];
      continue;
    }
    // the gate / residual pieces landed (the next halo's HOPS pieces may still fly) and
    // every wave is done reading this tile's halo buffer, which now takes the bf16 output
    if (more) wait_vmcnt_barrier<HOPS>();
    else wait_vmcnt_barrier<0>();
    char* ob = lds + WBYTES + buf * HBUF;
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = acc[i][j][r] + bias[i][r];
          v[r] = x > 0.f ? x : (relu ? 0.f : x * sl1);   // act_fwd for none / relu / lrelu
        }
        if (has_gate) {
          const uint2 gv = *reinterpret_cast<const uint2*>(lds + GOFF + tslot[i][j]);
          const float gy[4] = {lo_f(gv.x), hi_f(gv.x), lo_f(gv.y), hi_f(gv.y)};
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] *= gy[r] > 0.f ? 1.f : gneg;   // act_dgrad_from_y
        }
        if (has_res) {
          const uint2 rv = *reinterpret_cast<const uint2*>(lds + ROFF + tslot[i][j]);
          const float ry[4] = {lo_f(rv.x), hi_f(rv.x), lo_f(rv.y), hi_f(rv.y)};
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = res_combine(rsc, ry[r], gam, v[r]);
        }
        *reinterpret_cast<uint2*>(ob + tslot[i][j]) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NIT; ++j) {
      const int L = j * NT + tid, p = L >> 3, e = L & 7;
      const uint4 o = *reinterpret_cast<const uint4*>(ob + p * 128 + ((e ^ tile_swz(p)) << 4));
      const long gp = ((long)n * a.OH + oy0 + p / TW) * a.OW + ox0 + p % TW;
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.out) + gp * a.ldo + co0 + 8 * e) = o;
    }
  }
}

// ----------------------------- 4x4 / stride-2 forward convs on 32 channels --
// FWD of the first resD block's 4x4 / stride-2 / pad-1 conv of every D (32 -> 64
// channels, models.py:267; D256 at 256^2, N = 32: the largest conv of the D256
// lane).  The tile kernels gather every input pixel once per overlapping 4x4
// window (16 taps through L2, 64-B pieces).  Here a persistent workgroup keeps
// its wave's 16 output channels x 16 taps of weights in VGPRs (one A fragment
// per tap, loaded once) and walks 2 x 32-pixel output tiles, staging each
// tile's 6 x 66-pixel input halo ONCE in LDS by LDS-DMA (out-of-image pixels
// read zeros through the buffer bounds check).  Stride-2 taps read every other
// halo column, so each halo row is stored as its even- then its odd-column
// plane (33 pixels each): a tap's 16 consecutive output pixels are 16
// consecutive plane pixels, chunk-swizzled q ^ ((idx >> 1) & 2) -> conflict-free
// ds_read_b128 (brute-forced over all rows, planes and tap shifts).  Single
// halo buffer (28 KB); two workgroups per CU hide each other's loads.  K
// order = the tile kernels' (tap-major, one 32-channel step per tap): the same
// MFMA sequence per output, bit-identical results.  Epilogue through LDS
// (fp32 tile, 16-B runs of 8 channels): bias and activation.
constexpr int S2F_TH = 2, S2F_TW = 32;

EE_DEV int s2f_swz(int idx) { return (idx >> 1) & 2; }

__global__ __launch_bounds__(256, 2) void conv_s2fwd_kernel(ConvArgs a, long src_bytes) {
  constexpr int NT = 256, TH = S2F_TH, TW = S2F_TW, HC = 2 * TW + 2, PL = TW + 1, HR = 2 * TH + 2;
  constexpr int HP = HR * HC, HOPS = (HP * 4 + NT - 1) / NT, HBUF = HOPS * NT * 16;
  constexpr int TPIX = TH * TW, FJ = TPIX / 16, NCK = 16, NIT = TPIX * 8 / NT;
  static_assert(TPIX * 64 * 4 <= HBUF && NIT * NT == TPIX * 8, "s2fwd tile");
  __shared__ __attribute__((aligned(16))) char lds[HBUF];

  const int tid = threadIdx.x, lane = tid & 63, fr = lane & 15, fq = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_x = a.OW / TW, tiles_y = a.OH / TH, ntiles = a.N * tiles_y * tiles_x;
  const int lds0 = (int)(uintptr_t)(lds_void_t*)lds;
  const rsrc_t rs_src = make_rsrc(a.src, src_bytes);

  // this wave's weights: rows 16 w + fr, tap t's 32 channels, chunk fq (rows past Mrows are zero in the pack)
  bf16x8_t wa[16];
#pragma unroll
  for (int t = 0; t < 16; ++t)
    wa[t] = as_frag(*reinterpret_cast<const uint4*>(a.wp + (long)(16 * w + fr) * a.Kw + t * BK + fq * 8));
  // this thread's halo pieces: slot L >> 2 = (row hy, plane p, index idx) <-> column 2 idx + p
  int hpk[HOPS];
#pragma unroll
  for (int i = 0; i < HOPS; ++i) {
    const int L = i * NT + tid, slot = L >> 2;
    const int hy = slot / HC, rem = slot - hy * HC, pl = rem >= PL, idx = rem - pl * PL;
    const int q = (L & 3) ^ s2f_swz(idx);
    hpk[i] = slot < HP ? (hy << 16) | ((2 * idx + pl) << 4) | q : -1;
  }
  const int PH = a.IH, PW = a.IW;
  const int fbase[2] = {(fr << 6) + ((fq ^ s2f_swz(fr)) << 4), ((fr + 1) << 6) + ((fq ^ s2f_swz(fr + 1)) << 4)};
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    int b = t;
    const int tx = b % tiles_x;
    b /= tiles_x;
    const int ty = b % tiles_y, n = b / tiles_y;
    const int oy0 = ty * TH, ox0 = tx * TW;
#pragma unroll
    for (int i = 0; i < HOPS; ++i) {
      const int hy = hpk[i] >> 16, hx = (hpk[i] >> 4) & 0xfff, q = hpk[i] & 15;
      const int iy = 2 * oy0 - 1 + hy, ix = 2 * ox0 - 1 + hx;
      const bool ok = hpk[i] >= 0 && (unsigned)iy < (unsigned)PH && (unsigned)ix < (unsigned)PW;
      const unsigned off = ok ? (unsigned)((((n * PH + iy) * PW + ix) * a.lds_src + q * 8) * 2) : OOB;
      lds_dma16s(rs_src, lds0 + (i * NT + (tid & ~63)) * 16, off, 0);
    }
    wait_vmcnt_barrier<0>();
    f32x4_t acc[FJ];
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 16; ++tap) {
      const int r = tap >> 2, sx = tap & 3;
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        // plane index fr + (sx >> 1) + 16 jc: its swizzle is jc-independent, so every read is one of
        // two base registers + an immediate
        const int jr = j / (TW / 16), jc = j % (TW / 16);
        const int imm = ((2 * jr + r) * HC + (sx & 1) * PL + jc * 16) * 64;
        const bf16x8_t fb = as_frag(*reinterpret_cast<const uint4*>(lds + fbase[sx >> 1] + imm));
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[tap], fb, acc[j], 0, 0, 0);
      }
    }
    __syncthreads();   // every wave is done with the halo: the fp32 tile goes through the same LDS
    float4* st = reinterpret_cast<float4*>(lds);
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int p = (j / (TW / 16)) * TW + (j % (TW / 16)) * 16 + fr, c = w * 4 + fq;
      st[p * NCK + (c ^ (p & 15))] = make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int item = k * NT + tid, p = item / 8, e = item % 8, co = 8 * e;
      const float4 lo = st[p * NCK + ((2 * e) ^ (p & 15))];
      const float4 hi = st[p * NCK + ((2 * e + 1) ^ (p & 15))];
      float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = act_fwd(v[r] + (a.bias ? a.bias[co + r] : 0.f), a.act, a.slope);
      const long gp = ((long)n * a.OH + oy0 + p / TW) * a.OW + ox0 + p % TW;
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.out) + gp * a.ldo + co) =
          make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
    }
    __syncthreads();   // the staged tile is read before the next halo lands on it
  }
}

// ---------------------------------------------------------- WGRAD kernel --
struct WgradArgs {
  const bf16_t* x;     // [N][IH>>up2][IW>>up2][ldx]
  const bf16_t* dy;    // [P][lddy]
  float* ws;           // [nsplit][Cout][K]
  int N, IH, IW, ldx, up2;
  int OH, OW, R, S, st, ph, pw;
  int Cg, Cin, K;      // K = R*S*Cg, Cg = round_up(Cin, 8)
  int lddy, Cout, P, p_per_split;
  float* dw;           // nsplit == 1: epilogue writes the torch layout directly
  int accumulate;
  int quad;            // split slab in co-quad order [Cout/4][K][4] (Cout % 4 == 0): one 16-B store per lane
  int stage;           // unsplit dW through LDS: 16-B read-add-write runs along Cin (Cin % 4 == 0, host-checked)
  int xcd_remap;       // conv_wgrad_fast / glds kernels: blocks of one (co tile, split) on one XCD (grid size % 8 == 0)
};

// split-slab column (co, (tap, c)) -> channels-last weight layout [Cout][R][S][Cin]
// (unit stride along c, so a fragment row's 16 lanes store 64 contiguous bytes);
// padded channels dropped
struct WgradMap {
  int K, Cg, Cin, RS;
  EE_DEV long operator()(long col) const {  // col < Cout*K < 2^31
    const int ci = (int)col;
    const int co = ci / K, k = ci - co * K;
    const int tap = k / Cg, c = k - tap * Cg;
    return c < Cin ? ((long)co * RS + tap) * Cin + c : -1;
  }
};

// Split-slab reduce of co-quad slabs (WgradArgs::quad: [nsplit][Cout/4][K][4]):
// thread (k, quad) sums its four columns as one 16-B load per split and writes
// the four dW entries (each a coalesced run along k across the wave).  Row
// groups, chunking and the final group order are colsum_rows_kernel's, per
// column, so the sums are bit-identical to the row-major slab's reduce.
template <int COLS, int RG>
__global__ __launch_bounds__(COLS * RG) void wgrad_quad_reduce_kernel(const float* __restrict__ in, int nrows,
                                                                      long stride, float* __restrict__ out,
                                                                      int accumulate, WgradMap map) {
  __shared__ f32x4_t sh[RG][COLS];
  const int lane = threadIdx.x % COLS, g = threadIdx.x / COLS;
  const int k = blockIdx.x * COLS + lane, c4 = blockIdx.y;
  const bool ok = k < map.K;
  const f32x4_t* src = reinterpret_cast<const f32x4_t*>(in) + ((long)c4 * map.K + k);
  const long st4 = stride / 4;
  f32x4_t s = {0.f, 0.f, 0.f, 0.f};
  if (ok) {
    int r = g;
    // 8 rows' loads per round trip, summed in row order (colsum_rows_kernel's)
    for (; r + 7 * RG < nrows; r += 8 * RG) {
      f32x4_t a[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] = src[(long)(r + k * RG) * st4];
#pragma unroll
      for (int k = 0; k < 8; ++k) s += a[k];
    }
    for (; r < nrows; r += RG) s += src[(long)r * st4];
  }
  if (RG > 1) {
    sh[g][lane] = s;
    __syncthreads();
  }
  if (g == 0 && ok) {
    f32x4_t t = s;
    if (RG > 1) {
      t = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
      for (int i = 0; i < RG; ++i) t += sh[i][lane];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long o = map((long)(c4 * 4 + j) * map.K + k);
      if (o >= 0) out[o] = accumulate ? out[o] + t[j] : t[j];
    }
  }
}

constexpr int TRP = 4;  // row padding (elements) for transposed-read tiles

// dW tile epilogue: lane (g, li) of fragment (i, j) holds dW[co0 + ... + 4g + r][kb0 + ... + li];
// written straight into torch's layout when unsplit, else into the split slab
template <int FI, int FJ, int WT_CO, int WT_K>
EE_DEV void wgrad_epilogue(const WgradArgs& w, const f32x4_t (&acc)[FI][FJ], int co0, int kb0, int wi, int wj,
                           int lane, int split = -1) {
  if (split < 0) split = blockIdx.z;
  const int g = lane >> 4, li = lane & 15;
  if (w.dw) {
    // one fragment row block at a time: all 4*FJ old values are loaded before any
    // is added, so accumulation costs one memory round trip per block, not per element
    const WgradMap map{w.K, w.Cg, w.Cin, w.R * w.S};
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      long o[4][FJ];
      float old[4][FJ];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wi * WT_CO + i * 16 + g * 4 + r;
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
          const int k = kb0 + wj * WT_K + j * 16 + li;
          o[r][j] = (co < w.Cout && k < w.K) ? map((long)co * w.K + k) : -1;
          old[r][j] = (w.accumulate && o[r][j] >= 0) ? w.dw[o[r][j]] : 0.f;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
          if (o[r][j] >= 0) w.dw[o[r][j]] = old[r][j] + acc[i][j][r];
    }
    return;
  }
  float* ws = w.ws + (long)split * w.Cout * w.K;
  if (w.quad) {
    // lane (g, li) holds co = ...+ 4g + r, r = 0..3: one co quad at one k -> 16 contiguous bytes
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int co = co0 + wi * WT_CO + i * 16 + g * 4;
      if (co >= w.Cout) continue;
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int k = kb0 + wj * WT_K + j * 16 + li;
        if (k < w.K) *reinterpret_cast<f32x4_t*>(ws + ((long)(co >> 2) * w.K + k) * 4) = acc[i][j];
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < FI; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + wi * WT_CO + i * 16 + g * 4 + r;
      if (co >= w.Cout) continue;
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int k = kb0 + wj * WT_K + j * 16 + li;
        if (k < w.K) ws[(long)co * w.K + k] = acc[i][j][r];
      }
    }
  }
}

// Unsplit dW epilogue through the idle LDS ring: the fp32 tile is written as
// [co][k] with the 16-B chunk index XOR 4 * ((co >> 2) & (TK / 16 - 1)) (conflict-free
// ds_write_b32 for the fragments' 4-row lane groups, conflict-free ds_read_b128
// along k; the XOR stays inside the row's TK / 4 chunks), then every thread owns 4 consecutive k of one output channel: one
// 16-B load of the old dW (when accumulating), one 16-B store -- instead of
// four dword loads and stores per fragment row.  Same fp32 additions: bit-
// identical to wgrad_epilogue.
template <int TCO, int TK, int FI, int FJ, int WT_CO, int WT_K>
EE_DEV void wgrad_epilogue_staged(const WgradArgs& w, const f32x4_t (&acc)[FI][FJ], int co0, int kb0, int wi,
                                  int wj, int lane, int tid, float* st, int split) {
  static_assert(TK % 16 == 0 && TCO % 16 == 0, "tile");
  const int g = lane >> 4, li = lane & 15;
  constexpr int CM = TK / 16 - 1;   // XOR masks stay inside the row's TK / 4 chunks
  auto phys = [](int row, int k) { return row * TK + ((((k >> 2) ^ (4 * ((row >> 2) & CM))) << 2) | (k & 3)); };
  __syncthreads();   // every wave's last ring reads are done
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wi * WT_CO + i * 16 + g * 4 + r, k = wj * WT_K + j * 16 + li;
        st[phys(row, k)] = acc[i][j][r];
      }
  __syncthreads();
  const WgradMap map{w.K, w.Cg, w.Cin, w.R * w.S};
  constexpr int K4 = TK / 4, ITEMS = TCO * K4;
#pragma unroll 4
  for (int item = tid; item < ITEMS; item += 256) {
    const int row = item / K4, k = (item - row * K4) * 4;
    const int co = co0 + row, kk = kb0 + k;
    if (co >= w.Cout || kk >= w.K) continue;
    if (!w.dw) {   // split: this split's row-major slab [Cout][K] (K % 4 == 0, 16-B aligned)
      *reinterpret_cast<f32x4_t*>(w.ws + ((long)split * w.Cout + co) * w.K + kk) =
          *reinterpret_cast<const f32x4_t*>(st + phys(row, k));
      continue;
    }
    const long o = map((long)co * w.K + kk);
    if (o < 0) continue;   // padding channels (Cin % 4 == 0: a run is all valid or all padding)
    f32x4_t v = *reinterpret_cast<const f32x4_t*>(st + phys(row, k));
    f32x4_t* dst = reinterpret_cast<f32x4_t*>(w.dw + o);
    if (w.accumulate) {
      const f32x4_t old = *dst;
      v = old + v;
    }
    *dst = v;
  }
}

template <int TCO, int TK, int WCO>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradArgs w) {
  constexpr int WKK = 4 / WCO;
  constexpr int WT_CO = TCO / WCO, WT_K = TK / WKK;
  constexpr int FI = WT_CO / 16, FJ = WT_K / 16;
  constexpr int DROW = TCO + TRP, XROW = TK + TRP;
  constexpr int D_CHUNKS = BK * TCO / 8, X_CHUNKS = BK * TK / 8;
  constexpr int D_PER = (D_CHUNKS + 255) / 256, X_PER = (X_CHUNKS + 255) / 256;

  __shared__ __attribute__((aligned(16))) bf16_t lds_d[2][BK * DROW];
  __shared__ __attribute__((aligned(16))) bf16_t lds_x[2][BK * XROW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = wave / WKK, wj = wave % WKK;
  const int co0 = blockIdx.y * TCO, kb0 = blockIdx.x * TK;
  const int p_begin = blockIdx.z * w.p_per_split;
  const int p_end = min(w.P, p_begin + w.p_per_split);
  const int hw = w.OH * w.OW;
  const int PH = w.IH >> w.up2, PW = w.IW >> w.up2;

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
        if (p < p_end && co < w.Cout) v = mask_chunk(*reinterpret_cast<const uint4*>(w.dy + (long)p * w.lddy + co), co, w.Cout);
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
        const int k = kb0 + kc * 8;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (p < p_end && k < w.K) {
          const int n = p / hw, rem = p - n * hw;
          const int oy = rem / w.OW, ox = rem - oy * w.OW;
          const int tap = k / w.Cg, c = k - tap * w.Cg;
          const int r = tap / w.S, s = tap - r * w.S;
          const int iy = oy * w.st - w.ph + r, ix = ox * w.st - w.pw + s;
          if (c < w.Cin && (unsigned)iy < (unsigned)w.IH && (unsigned)ix < (unsigned)w.IW) {
            const long off = ((long)(n * PH + (iy >> w.up2)) * PW + (ix >> w.up2)) * w.ldx + c;
            v = mask_chunk(*reinterpret_cast<const uint4*>(w.x + off), c, w.Cin);
          }
        }
        rx[i] = v;
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
  wgrad_epilogue<FI, FJ, WT_CO, WT_K>(w, acc, co0, kb0, wi, wj, lane);
}

// XOR swizzle of the 16-B chunk index for [32 pixel][NCH chunk] LDS images
// read with ds_read_b64_tr_b16 (two 4-row blocks 8 rows apart per 32-lane
// half): conflict-free for NCH = 4, 8, 16 (exhaustive bank check).
template <int NCH>
EE_DEV int tr_swz(int row) {
  if (NCH == 16) return ((row & 3) << 1) ^ (((row >> 3) & 1) << 3);
  if (NCH == 8) return (row & 3) ^ (((row >> 3) & 1) << 2);
  return (row & 3) ^ (((row >> 3) & 1) << 1);
}

// Pipelined weight gradient: dy [32 pixel][TCO] and the gathered x [32 pixel][TK]
// K-steps go global -> LDS by buffer_load ... lds into a 4-deep ring (as
// conv_glds_kernel), fragments by transposed reads of the swizzled images.
// Padding channels of dy / x only reach dW rows / columns that are dropped;
// halo taps and pixels past the split read as zeros (bounds-checked offsets).
template <int TCO, int TK>
__global__ __launch_bounds__(256, 2) void conv_wgrad_glds_kernel(WgradArgs w, long x_bytes, long dy_bytes) {
  constexpr int S = CONV_STAGES;
  constexpr int WCO = TCO >= 64 ? 2 : 1, WKK = 4 / WCO;
  constexpr int WT_CO = TCO / WCO, WT_K = TK / WKK;
  constexpr int FI = WT_CO / 16, FJ = WT_K / 16;
  constexpr int DCH = TCO / 8, XCH = TK / 8;           // 16-B chunks per pixel row
  constexpr int D_TOT = BK * DCH, X_TOT = BK * XCH;    // chunks per K-step
  constexpr int D_INS = (D_TOT + 255) / 256, X_INS = X_TOT / 256;
  constexpr int STAGE = BK * (TCO + TK);
  static_assert(X_INS >= 1 && FI >= 1 && FJ >= 1, "tile");

  __shared__ __attribute__((aligned(16))) bf16_t lds[S * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = wave / WKK, wj = wave % WKK;
  // XCD remap as conv_wgrad_fast_kernel's (WgradArgs::xcd_remap): a (co tile, split)'s k
  // tiles share one XCD's L2 -- they all read the same dy and x rows (with an up2 source,
  // each x pixel serves 4 output pixels x 9 taps)
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (w.xcd_remap) {
    const int gx = gridDim.x, gy = gridDim.y;
    const int total = gx * gy * gridDim.z;
    const int lin = bx + gx * (by + gy * bz);
    const int logical = (lin & 7) * (total >> 3) + (lin >> 3);
    bx = logical % gx;
    const int t = logical / gx;
    by = t % gy;
    bz = t / gy;
  }
  const int co0 = by * TCO, kb0 = bx * TK;
  const int p_begin = bz * w.p_per_split;
  const int p_end = min(w.P, p_begin + w.p_per_split);
  const int nk = p_begin < p_end ? (p_end - p_begin + BK - 1) / BK : 0;
  const int PH = w.IH >> w.up2, PW = w.IW >> w.up2;
  const int hw = w.OH * w.OW;
  // waves that stage no dy chunk (TCO = 32) count fewer loads per K-step
  const bool d_wave = D_TOT >= 256 || tid < D_TOT;
  const rsrc_t rs_x = make_rsrc(w.x, x_bytes);
  const rsrc_t rs_d = make_rsrc(w.dy, dy_bytes);

  // dy chunks: fixed pixel row / channel per thread
  int d_row[D_INS], d_co[D_INS];
#pragma unroll
  for (int i = 0; i < D_INS; ++i) {
    const int idx = i * 256 + tid;
    d_row[i] = idx / DCH;
    d_co[i] = co0 + (((idx % DCH) ^ tr_swz<DCH>(d_row[i])) * 8);
  }
  // x chunks: fixed (tap, channel) and pixel row per thread; pixel tracked incrementally
  int x_row[X_INS], x_r[X_INS], x_s[X_INS], x_c[X_INS], x_n[X_INS], x_oy[X_INS], x_ox[X_INS];
  bool x_kok[X_INS];
#pragma unroll
  for (int i = 0; i < X_INS; ++i) {
    const int idx = i * 256 + tid;
    x_row[i] = idx / XCH;
    const int k = kb0 + (((idx % XCH) ^ tr_swz<XCH>(x_row[i])) * 8);
    x_kok[i] = k < w.K;
    const int tap = k / w.Cg;
    x_c[i] = k - tap * w.Cg;
    x_r[i] = tap / w.S;
    x_s[i] = tap - x_r[i] * w.S;
    const int p = p_begin + x_row[i];
    x_n[i] = p / hw;
    const int rem = p - x_n[i] * hw;
    x_oy[i] = rem / w.OW;
    x_ox[i] = rem - x_oy[i] * w.OW;
  }

  auto issue = [&](int step, int buf) {
    const int pb = p_begin + step * BK;
    bf16_t* base = lds + buf * STAGE;
    if (d_wave) {
#pragma unroll
      for (int i = 0; i < D_INS; ++i) {
        const int p = pb + d_row[i];
        const unsigned off = (p < p_end && d_co[i] < w.Cout) ? (unsigned)(((long)p * w.lddy + d_co[i]) * 2) : OOB;
        lds_dma16(rs_d, base + (i * 256 + wave * 64) * 8, off);
      }
    }
#pragma unroll
    for (int i = 0; i < X_INS; ++i) {
      unsigned off = OOB;
      if (pb + x_row[i] < p_end && x_kok[i]) {
        const int iy = x_oy[i] * w.st - w.ph + x_r[i], ix = x_ox[i] * w.st - w.pw + x_s[i];
        if ((unsigned)iy < (unsigned)w.IH && (unsigned)ix < (unsigned)w.IW)
          off = (unsigned)(((((long)x_n[i] * PH + (iy >> w.up2)) * PW + (ix >> w.up2)) * w.ldx + x_c[i]) * 2);
      }
      lds_dma16(rs_x, base + BK * TCO + (i * 256 + wave * 64) * 8, off);
      // advance this row's pixel by one K-step
      x_ox[i] += BK;
      while (x_ox[i] >= w.OW) {
        x_ox[i] -= w.OW;
        if (++x_oy[i] == w.OH) {
          x_oy[i] = 0;
          ++x_n[i];
        }
      }
    }
  };

  f32x4_t acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, li = lane & 15, q = li >> 2, pq = li & 3;
  typedef __attribute__((address_space(3))) s16x4_t lds_s4;
  // transposed fragment: rows (pixels) 8g+q and 8g+q+4, columns col + 4*pq .. +3
  auto tr_frag = [&](const bf16_t* img, int nch_shift, int col, auto swz) -> bf16x8_t {
    const int ch = (col >> 3) + (pq >> 1);
    const int r0 = 8 * g + q, r1 = r0 + 4;
    const bf16_t* p0 = img + (r0 << nch_shift) * 8 + ((ch ^ swz(r0)) * 8) + 4 * (pq & 1);
    const bf16_t* p1 = img + (r1 << nch_shift) * 8 + ((ch ^ swz(r1)) * 8) + 4 * (pq & 1);
    s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p0));
    s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p1));
    typedef __attribute__((ext_vector_type(8))) short s16x8_t;
    s16x8_t v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  };
  constexpr int DSH = DCH == 16 ? 4 : DCH == 8 ? 3 : 2;
  constexpr int XSH = XCH == 16 ? 4 : 3;
  auto dswz = [](int r) { return tr_swz<DCH>(r); };
  auto xswz = [](int r) { return tr_swz<XCH>(r); };

#pragma unroll
  for (int st = 0; st < S - 1; ++st)
    if (st < nk) issue(st, st);
  for (int it = 0; it < nk; ++it) {
    if (it + S - 2 < nk) {
      if (d_wave) wait_vmcnt_barrier<(S - 2) * (D_INS + X_INS)>();
      else wait_vmcnt_barrier<(S - 2) * X_INS>();
    } else {
      wait_vmcnt_barrier<0>();
    }
    if (it + S - 1 < nk) issue(it + S - 1, (it + S - 1) % S);
    const bf16_t* base = lds + (it % S) * STAGE;
    bf16x8_t fa[FI], fb[FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i) fa[i] = tr_frag(base, DSH, wi * WT_CO + i * 16, dswz);
#pragma unroll
    for (int j = 0; j < FJ; ++j) fb[j] = tr_frag(base + BK * TCO, XSH, wj * WT_K + j * 16, xswz);
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
  }
  wgrad_epilogue<FI, FJ, WT_CO, WT_K>(w, acc, co0, kb0, wi, wj, lane, bz);
}

// Weight gradient with the per-K-step index math hoisted (cf. conv_fast_kernel):
// power-of-two output grids, no fused upsample.  A K-step is 32 consecutive
// pixels starting at a multiple of 32, so with OW and OH*OW powers of two each
// thread's pixel is (n0 + dn, oy0 + dy, ox0 + dx) with (dn, dy, dx) fixed per
// thread and (n0, oy0, ox0) uniform shifts of the step's first pixel: a gather
// offset is a per-thread constant plus a uniform term, its bounds test two
// compares against uniform-shifted constants.  Rows past the split end read dy
// as zeros (their x rows are finite activations, so the products vanish).
template <int TCO, int TK, int KS = 1>
__global__ __launch_bounds__(256, 2) void conv_wgrad_fast_kernel(WgradArgs w, long x_bytes, long dy_bytes, int lw,
                                                                 int lhw) {
  constexpr int S = CONV_STAGES;
  constexpr int WCO = TCO >= 64 ? 2 : 1, WKK = 4 / WCO;
  constexpr int WT_CO = TCO / WCO, WT_K = TK / WKK;
  constexpr int FI = WT_CO / 16, FJ = WT_K / 16;
  constexpr int DCH = TCO / 8, XCH = TK / 8;           // 16-B chunks per pixel row
  constexpr int D_TOT = BK * DCH, X_TOT = BK * XCH;    // chunks per K-step
  constexpr int D_INS = (D_TOT + 255) / 256, X_INS = X_TOT / 256;
  constexpr int STAGE = BK * (TCO + TK);
  static_assert(X_INS >= 1 && FI >= 1 && FJ >= 1, "tile");

  __shared__ __attribute__((aligned(16))) bf16_t lds[S * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wave / WKK, wj = wave % WKK;
  // logical tile: with xcd_remap the linear block id's XCD (id % 8) owns a
  // contiguous run of logical tiles, k tiles fastest, so every k tile of one
  // (co tile, split) -- which all read the same pixels of x and dy -- shares
  // one XCD's L2 (round-robin dispatch spread them over the 8 XCDs: each XCD
  // re-fetched the same rows from HBM)
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (w.xcd_remap) {
    const int gx = gridDim.x, gy = gridDim.y;
    const int total = gx * gy * gridDim.z;
    const int lin = bx + gx * (by + gy * bz);
    const int logical = (lin & 7) * (total >> 3) + (lin >> 3);
    bx = logical % gx;
    const int t = logical / gx;
    by = t % gy;
    bz = t / gy;
  }
  const int co0 = by * TCO, kb0 = bx * TK;
  const int p_begin = bz * w.p_per_split;
  const int p_end = min(w.P, p_begin + w.p_per_split);
  const int nk = p_begin < p_end ? (p_end - p_begin + BK - 1) / BK : 0;
  const bool d_wave = D_TOT >= 256 || tid < D_TOT;
  const rsrc_t rs_x = make_rsrc(w.x, x_bytes);
  const rsrc_t rs_d = make_rsrc(w.dy, dy_bytes);
  const int lds0 = (int)(uintptr_t)(lds_void_t*)lds;

  // dy chunks: pixel row d_row of the step, channel d_co
  int d_row[D_INS];
  unsigned d_off[D_INS];
#pragma unroll
  for (int i = 0; i < D_INS; ++i) {
    const int idx = i * 256 + tid;
    d_row[i] = idx / DCH;
    const int co = co0 + (((idx % DCH) ^ tr_swz<DCH>(d_row[i])) * 8);
    d_off[i] = co < w.Cout ? (unsigned)((d_row[i] * w.lddy + co) * 2) : OOB;
    if (co >= w.Cout) d_row[i] = BK;  // never valid
  }
  // x chunks: fixed (tap, channel), pixel = step start + (dn, dy, dx)
  int x_q[X_INS], x_cy[X_INS], x_cx[X_INS];
  bool x_kok[X_INS];
  const int OW = w.OW, HW = w.OH * w.OW;
#pragma unroll
  for (int i = 0; i < X_INS; ++i) {
    const int idx = i * 256 + tid;
    const int row = idx / XCH;
    const int k = kb0 + (((idx % XCH) ^ tr_swz<XCH>(row)) * 8);
    x_kok[i] = k < w.K;
    const int tap = k / w.Cg, c = k - tap * w.Cg;
    const int r = tap / w.S, s = tap - r * w.S;
    x_kok[i] = x_kok[i] && c < w.Cin;
    // decomposition of `row` relative to a 32-aligned step start
    const int dn = HW < BK ? row >> lhw : 0;
    const int rr = HW < BK ? row & (HW - 1) : row;
    const int dy = OW < BK ? rr >> lw : 0;
    const int dx = OW < BK ? rr & (OW - 1) : rr;
    x_cy[i] = dy * w.st - w.ph + r;
    x_cx[i] = dx * w.st - w.pw + s;
    x_q[i] = ((dn * w.IH + x_cy[i]) * w.IW + x_cx[i]) * w.ldx + c;
  }

  auto issue = [&](int step, int buf) {
    const int p0 = p_begin + step * BK;
    const int base = lds0 + buf * (STAGE * 2);
    const int drem = p_end - p0;
    if (d_wave) {
#pragma unroll
      for (int i = 0; i < D_INS; ++i) {
        const unsigned off = d_row[i] < drem ? d_off[i] : OOB;
        lds_dma16s(rs_d, base + (i * 256 + wave * 64) * 16, off, p0 * w.lddy * 2);
      }
    }
    const int n0 = p0 >> lhw, rem = p0 & (HW - 1);
    const int uy = (rem >> lw) * w.st, ux = (rem & (OW - 1)) * w.st;
    const int ubase = ((n0 * w.IH + uy) * w.IW + ux) * w.ldx;
#pragma unroll
    for (int i = 0; i < X_INS; ++i) {
      const bool ok = x_kok[i] && (unsigned)(uy + x_cy[i]) < (unsigned)w.IH &&
                      (unsigned)(ux + x_cx[i]) < (unsigned)w.IW;
      const unsigned off = ok ? (unsigned)((ubase + x_q[i]) * 2) : OOB;
      lds_dma16s(rs_x, base + BK * TCO * 2 + (i * 256 + wave * 64) * 16, off, 0);
    }
  };

  f32x4_t acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, li = lane & 15, q = li >> 2, pq = li & 3;
  typedef __attribute__((address_space(3))) s16x4_t lds_s4;
  auto tr_frag = [&](const bf16_t* img, int nch_shift, int col, auto swz) -> bf16x8_t {
    const int ch = (col >> 3) + (pq >> 1);
    const int r0 = 8 * g + q, r1 = r0 + 4;
    const bf16_t* p0 = img + (r0 << nch_shift) * 8 + ((ch ^ swz(r0)) * 8) + 4 * (pq & 1);
    const bf16_t* p1 = img + (r1 << nch_shift) * 8 + ((ch ^ swz(r1)) * 8) + 4 * (pq & 1);
    s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p0));
    s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p1));
    typedef __attribute__((ext_vector_type(8))) short s16x8_t;
    s16x8_t v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  };
  constexpr int DSH = DCH == 16 ? 4 : DCH == 8 ? 3 : 2;
  constexpr int XSH = XCH == 16 ? 4 : 3;
  auto dswz = [](int r) { return tr_swz<DCH>(r); };
  auto xswz = [](int r) { return tr_swz<XCH>(r); };

  // KS pixel steps per barrier (as conv_fast_kernel)
  constexpr int YNG = S - 2 * KS;
  static_assert(YNG >= 0, "stages");
#pragma unroll
  for (int st = 0; st < S - KS; ++st)
    if (st < nk) issue(st, st);
  int it0 = 0;
  if (KS == 2) {
    // straight-line pairs, second stage's fragment reads interleaved with the
    // first stage's MFMAs (as conv_fast_kernel)
    for (; it0 + 1 < nk; it0 += 2) {
      if (it0 + S - 2 <= nk) {
        if (d_wave) wait_vmcnt_barrier<YNG * (D_INS + X_INS)>();
        else wait_vmcnt_barrier<YNG * X_INS>();
      } else {
        wait_vmcnt_barrier<0>();
      }
      if (it0 + S - 2 < nk) issue(it0 + S - 2, (it0 + S - 2) % S);
      if (it0 + S - 1 < nk) issue(it0 + S - 1, (it0 + S - 1) % S);
      bf16x8_t fa0[FI], fb0[FJ], fa1[FI], fb1[FJ];
      const bf16_t* b0 = lds + (it0 % S) * STAGE;
      const bf16_t* b1 = lds + ((it0 + 1) % S) * STAGE;
#pragma unroll
      for (int i = 0; i < FI; ++i) fa0[i] = tr_frag(b0, DSH, wi * WT_CO + i * 16, dswz);
#pragma unroll
      for (int j = 0; j < FJ; ++j) fb0[j] = tr_frag(b0 + BK * TCO, XSH, wj * WT_K + j * 16, xswz);
#pragma unroll
      for (int i = 0; i < FI; ++i) fa1[i] = tr_frag(b1, DSH, wi * WT_CO + i * 16, dswz);
#pragma unroll
      for (int j = 0; j < FJ; ++j) fb1[j] = tr_frag(b1 + BK * TCO, XSH, wj * WT_K + j * 16, xswz);
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa0[i], fb0[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1[i], fb1[j], acc[i][j], 0, 0, 0);
      // each transposed fragment is two ds_read_b64_tr_b16
#pragma unroll
      for (int r = 0; r < 2 * (FI + FJ); ++r) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
      for (int r = 0; r < FI + FJ; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * FI * FJ - (FI + FJ), 0);
    }
  }
  for (int it = it0; it < nk; it += KS) {
    if (it + S - KS <= nk) {
      if (d_wave) wait_vmcnt_barrier<YNG * (D_INS + X_INS)>();
      else wait_vmcnt_barrier<YNG * X_INS>();
    } else {
      wait_vmcnt_barrier<0>();
    }
#pragma unroll
    for (int k = 0; k < KS; ++k)
      if (it + S - KS + k < nk) issue(it + S - KS + k, (it + S - KS + k) % S);
    bf16x8_t fa[KS][FI], fb[KS][FJ];
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      if (it + k >= nk) break;
      const bf16_t* base = lds + ((it + k) % S) * STAGE;
#pragma unroll
      for (int i = 0; i < FI; ++i) fa[k][i] = tr_frag(base, DSH, wi * WT_CO + i * 16, dswz);
#pragma unroll
      for (int j = 0; j < FJ; ++j) fb[k][j] = tr_frag(base + BK * TCO, XSH, wj * WT_K + j * 16, xswz);
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      if (it + k >= nk) break;
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[k][i], fb[k][j], acc[i][j], 0, 0, 0);
    }
  }
  static_assert(TCO * TK * 4 <= S * STAGE * 2, "staged dW tile exceeds the LDS ring");
  if (w.stage) {
    wgrad_epilogue_staged<TCO, TK, FI, FJ, WT_CO, WT_K>(w, acc, co0, kb0, wi, wj, lane, tid,
                                                       reinterpret_cast<float*>(lds), bz);
    return;
  }
  wgrad_epilogue<FI, FJ, WT_CO, WT_K>(w, acc, co0, kb0, wi, wj, lane, bz);
}

// ------------------------------------------------------- weight packing --
// fp32 conv weights live channels-last, W[Cout][R][S][Cin] (torch's
// channels_last memory format of the (Cout, Cin, R, S) parameter), so the
// forward image is a padded copy of each row and the weight gradient is
// written with unit stride along Cin.
// FWD pack:  out[co][(r*S+s)*Cgp + c] = W[co][r][s][c] * scale[co]   (zero padded)
// BWDD pack: out[ci][(r*S+s)*Cgp + co] = W[co][r][s][ci] * scale[co]
__global__ void pack_weights_kernel(const float* w, const float* scale, int Cout, int Cin, int R, int S,
                                    int transposed, int Cgp, int rows_pad, int Kw, bf16_t* out) {
  const long total = (long)rows_pad * Kw;
  const int RS = R * S;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int row = e / Kw, k = e % Kw;
    const int rs = k / Cgp, c = k - rs * Cgp;
    float v = 0.f;
    if (rs >= RS) {
      // zero columns padding the row to whole 32-deep K steps
    } else if (!transposed) {
      if (row < Cout && c < Cin) v = w[((long)row * RS + rs) * Cin + c] * (scale ? scale[row] : 1.f);
    } else {
      if (row < Cin && c < Cout) v = w[((long)c * RS + rs) * Cin + row] * (scale ? scale[c] : 1.f);
    }
    out[e] = f2bf(v);
  }
}

// Batched re-pack after an optimizer step: one launch for every conv weight of a
// model (fwd and bwd-data images).  `table` (device, int64): njobs rows of
// {w, scale, out, Cout, Cin, R, S, transposed}, then njobs+1 prefix offsets of
// BLOCKS per job (pack_multi_blocks).  Forward image: one block per output row
// (w[co] is already the row's (tap, c) order: a padded copy, 8 columns = one
// 16-byte store per thread); bwd-data image: per tap, a 64x64 (ci, co) tile
// transposed through LDS, so the fp32 reads are 256-byte runs along ci and the
// bf16 writes 128-byte runs along co.
constexpr int PK_T = 64;  // bwd-image tile: input channels (rows) x output channels (columns)

EE_HOST_DEV_INLINE int pk_cgp(int C) { return C <= 8 ? 8 : (C + BK - 1) / BK * BK; }

__global__ __launch_bounds__(256) void pack_weights_multi_kernel(const long* __restrict__ table, int njobs) {
  __shared__ float buf[PK_T * (PK_T + 1)];
  const long* pre = table + 8L * njobs;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pre[mid] <= blockIdx.x) lo = mid;
    else hi = mid - 1;
  }
  const long* j = table + 8L * lo;
  const int lb = (int)(blockIdx.x - pre[lo]);
  const float* w = reinterpret_cast<const float*>(j[0]);
  const float* scale = reinterpret_cast<const float*>(j[1]);
  bf16_t* out = reinterpret_cast<bf16_t*>(j[2]);
  const int Cout = (int)j[3], Cin = (int)j[4], RS = (int)(j[5] * j[6]), tr = (int)j[7];
  const int t = threadIdx.x;
  if (!tr) {
    // ---- forward image: row co = lb, out[co][tap*Cgp + c] = w[co][tap][c]
    const int Cgp = pk_cgp(Cin), Kw = (RS * Cgp + BK - 1) / BK * BK;
    bf16_t* orow = out + (long)lb * Kw;  // Kw % 32 == 0: 16-byte aligned 8-column groups
    const bool live = lb < Cout;
    const float sc = (live && scale) ? scale[lb] : 1.f;
    const float* src = w + (long)lb * RS * Cin;
    for (int k = t * 8; k < Kw; k += 256 * 8) {
      const int tap = k / Cgp, c = k - tap * Cgp;  // Cgp % 8 == 0: the group stays in one tap
      float v[8];
      const float* sp = src + tap * Cin + c;
      if (live && tap < RS && c + 8 <= Cin && ((uintptr_t)sp & 15) == 0) {  // two 16-byte loads
        const float4 a0 = reinterpret_cast<const float4*>(sp)[0], a1 = reinterpret_cast<const float4*>(sp)[1];
        v[0] = a0.x * sc; v[1] = a0.y * sc; v[2] = a0.z * sc; v[3] = a0.w * sc;
        v[4] = a1.x * sc; v[5] = a1.y * sc; v[6] = a1.z * sc; v[7] = a1.w * sc;
      } else {
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = (live && tap < RS && c + u < Cin) ? sp[u] * sc : 0.f;
      }
      *reinterpret_cast<uint4*>(orow + k) =
          make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
    }
  } else {
    // ---- bwd-data image: out[ci][tap*Cgp + co] = w[co][tap][ci] * scale[co];
    // block lb -> (ci tile, tap, co tile)
    const int Cgp = pk_cgp(Cout), Kw = (RS * Cgp + BK - 1) / BK * BK;
    const int nco = (Cgp + PK_T - 1) / PK_T;
    const int cot = lb % nco, tap = (lb / nco) % RS, cit = lb / (nco * RS);
    const int ci0 = cit * PK_T, co0 = cot * PK_T;
#pragma unroll
    for (int r = 0; r < PK_T * PK_T / 256; ++r) {
      const int e = r * 256 + t, co = e / PK_T, i = e % PK_T;  // lanes run along ci
      float v = 0.f;
      if (co0 + co < Cout && ci0 + i < Cin)
        v = w[((long)(co0 + co) * RS + tap) * Cin + ci0 + i] * (scale ? scale[co0 + co] : 1.f);
      buf[co * (PK_T + 1) + i] = v;
    }
    __syncthreads();
    const int ncol = min(PK_T, Cgp - co0);  // never past this tap's Cgp columns
#pragma unroll
    for (int r = 0; r < PK_T * PK_T / 2 / 256; ++r) {
      const int e = r * 256 + t, row = e / (PK_T / 2), cp = 2 * (e % (PK_T / 2));  // lanes run along co
      if (cp < ncol) {
        bf16_t* op = out + (long)(ci0 + row) * Kw + tap * Cgp + co0 + cp;
        *reinterpret_cast<uint32_t*>(op) = pack2(buf[cp * (PK_T + 1) + row], buf[(cp + 1) * (PK_T + 1) + row]);
      }
    }
    if (tap != RS - 1 || cot != nco - 1) return;  // one block per row tile zeroes the K tail
    const int tail = Kw - RS * Cgp;
    for (int e = t; e < PK_T * tail; e += 256) {
      const int row = e / tail, k = RS * Cgp + e - row * tail;
      out[(long)(ci0 + row) * Kw + k] = 0;
    }
  }
}

// ------------------------------------------------------------ thin convs --
// 3x3 stride-1 convs with <= 32 output rows: the stem conv_img (3 -> ndf) of
// models.py:313/330/348, get_image (ngf -> 3) of models.py:25-32, the
// 32-channel convs of the 256x256 stage, and their data gradients (which are
// again 3x3 stride-1 convs with <= 32 output rows).  These are all big-image,
// few-channel shapes on which the tile kernels spend their time in
// prologue / epilogue / barriers.  Here a wave keeps the whole packed weight
// slab (NT x NKS A fragments) in VGPRs for its lifetime and streams groups of
// 16 output pixels: each B fragment (8 channels of one tap of one pixel, 16 B)
// is loaded straight from global memory into the lane that feeds it to the
// MFMA -- no LDS, no barriers.  Blocks own contiguous pixel ranges and the
// blocks of one XCD own adjacent ranges, so the 3x3 halo re-reads hit that
// XCD's L2.  K layout = the packed weight row: NKS == 3 is the packed mode
// (Cgp == 8, 4 taps x 8 channels per K step), otherwise tap-major 32-channel
// slices.
template <int MODE, int NT, int NKS, int GPI>
__global__ __launch_bounds__(256) void conv_thin_kernel(ConvArgs a, int iters_per_block, int src_bytes) {
  constexpr bool PACKED = (NKS == 3);
  constexpr int NC = PACKED ? 1 : NKS / 9;
  const int lane = threadIdx.x & 63, kg = lane >> 4, col = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (b & 7) * (nb >> 3) + (b >> 3);  // XCD-contiguous logical block (nb % 8 == 0)
  // OOB offsets read zeros: padding taps, image borders and tail pixels need no branches
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, (short)0, src_bytes, 0x00020000);
  bf16x8_t fa[NT][NKS];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      fa[t][ks] = as_frag(*reinterpret_cast<const uint4*>(a.wp + (long)(16 * t + col) * a.Kw + 32 * ks + 8 * kg));
  float bia[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = 16 * t + 4 * kg + r;
      bia[t][r] = (a.bias && co < a.Mrows) ? a.bias[co] : 0.f;
    }
  // per-lane tap geometry of every K step (block-invariant)
  int t_dy[NKS], t_dx[NKS], t_c[NKS];
  bool t_ok[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const int tap = PACKED ? 4 * ks + kg : ks / NC;
    const int c = PACKED ? 0 : (ks % NC) * 32 + 8 * kg;
    t_ok[ks] = tap < 9 && c < a.Cvalid;  // chunks past the valid channels are never read
    const int r = tap / 3, s = tap - 3 * (tap / 3);
    t_dy[ks] = MODE == MODE_FWD ? r - a.ph : a.ph - r;
    t_dx[ks] = MODE == MODE_FWD ? s - a.pw : a.pw - s;
    t_c[ks] = c;
  }
  const int PH = a.IH >> a.up2, PW = a.IW >> a.up2, hw = a.OH * a.OW;
  // packed mode: every chunk starts at channel 0, so one lane mask zeroes the
  // channels >= Cvalid (other modes require Cvalid % 8 == 0).  Applied with
  // ANDs after all loads were issued: a branch per load would make the
  // compiler drain vmcnt after every load.
  const uint4 cmask = mask_chunk(make_uint4(~0u, ~0u, ~0u, ~0u), 0, PACKED ? a.Cvalid : 8);
  const bool rows16 = (a.OW & 15) == 0;  // a 16-pixel group never wraps a row: scalar decomposition
  const int it0 = lb * iters_per_block, it_end = it0 + iters_per_block;
  // issue the loads of iteration `it` (iterations past the end load zeros)
  auto load = [&](uint4 (&bv)[GPI][NKS], int (&pp)[GPI], int it) {
#pragma unroll
    for (int g = 0; g < GPI; ++g) {
      const int base = (it * GPI + g) * 16;
      int n, y, x;
      if (rows16) {
        const int n0 = base / hw, rem = base - n0 * hw;
        const int y0 = rem / a.OW;
        n = n0;
        y = y0;
        x = rem - y0 * a.OW + col;
      } else {
        const int p = min(base + col, a.P - 1);
        n = p / hw;
        const int rem = p - n * hw;
        y = rem / a.OW;
        x = rem - y * a.OW;
      }
      pp[g] = (it < it_end && base + col < a.P) ? base + col : -1;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const int iy = y + t_dy[ks], ix = x + t_dx[ks];
        const bool ok = pp[g] >= 0 && t_ok[ks] && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
        const int off = (((n * PH + (iy >> a.up2)) * PW + (ix >> a.up2)) * a.lds_src + t_c[ks]) * 2;
        bv[g][ks] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? off : 0x80000000, 0, 0));
      }
    }
  };
  auto compute = [&](uint4 (&bv)[GPI][NKS], const int (&pp)[GPI]) {
#pragma unroll
    for (int g = 0; g < GPI; ++g) {
      if (PACKED) {
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          bv[g][ks].x &= cmask.x;
          bv[g][ks].y &= cmask.y;
          bv[g][ks].z &= cmask.z;
          bv[g][ks].w &= cmask.w;
        }
      }
      f32x4_t acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t][ks], as_frag(bv[g][ks]), acc[t], 0, 0, 0);
      if (pp[g] < 0) continue;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int co = 16 * t + 4 * kg;
        if (co >= a.Mrows) continue;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = act_fwd(acc[t][r] + bia[t][r], a.act, a.slope);
        bf16_t* op = reinterpret_cast<bf16_t*>(a.out) + (long)pp[g] * a.ldo + co;
        if (co + 4 <= a.Mrows) {
          *reinterpret_cast<uint2*>(op) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (co + r < a.Mrows) op[r] = f2bf(v[r]);
        }
      }
    }
  };
  // two register stages: the loads of the wave's next iteration are in flight
  // while this one's MFMAs and stores run (unconditional, zero-filled past the end)
  uint4 b0[GPI][NKS], b1[GPI][NKS];
  int p0[GPI], p1[GPI];
  int it = it0 + wv;
  load(b0, p0, it);
  for (; it < it_end; it += 8) {
    load(b1, p1, it + 4);
    compute(b0, p0);
    if (it + 4 >= it_end) break;
    load(b0, p0, it + 8);
    compute(b1, p1);
  }
}

// LDS-tiled variant of conv_thin_kernel for OW % 64 == 0 (the 64..256-wide
// images): a block stages an (8 + 2) x (64 + 2)-pixel input halo tile in LDS
// by LDS-DMA and reads every tap's B fragment from there, instead of gathering
// each pixel nine times through L2 (which bounds the direct kernel at the L2
// gather rate, ~28 B/clk per CU).  No staging registers, so 3 blocks fit a CU
// and overlap one block's halo fill with the others' MFMAs; persistent blocks
// walk XCD-contiguous tile ranges.  64-B pixel rows use the chunk swizzle
// c ^ ((pix >> 1) & 2), conflict-free for ds_read_b128 windows of 16 pixels at
// any start (tap shifts); the DMA lanes fetch in swizzled order.
template <int MODE, int NT, int NKS>
__global__ __launch_bounds__(256, 3) void conv_thin_lds_kernel(ConvArgs a, int src_bytes, int tiles_per_block) {
  constexpr bool PACKED = (NKS == 3);
  constexpr int NCH = PACKED ? 1 : 4;  // 16-B chunks per staged pixel
  constexpr int TW = 64, TH = 8, PWT = TW + 2, NPIX = (TH + 2) * PWT, NCHUNK = NPIX * NCH;
  constexpr int NDMA = (NCHUNK + 255) / 256;  // DMA pieces per thread (tail lanes fill padding)
  __shared__ uint4 tile[NDMA * 256];
  const int tid = threadIdx.x, lane = tid & 63, kg = lane >> 4, col = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (b & 7) * (nb >> 3) + (b >> 3);
  const rsrc_t rsv = make_rsrc(a.src, src_bytes);
  bf16x8_t fa[NT][NKS];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      fa[t][ks] = as_frag(*reinterpret_cast<const uint4*>(a.wp + (long)(16 * t + col) * a.Kw + 32 * ks + 8 * kg));
  float bia[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = 16 * t + 4 * kg + r;
      bia[t][r] = (a.bias && co < a.Mrows) ? a.bias[co] : 0.f;
    }
  // tile origin relative to the output tile: FWD reads rows y - ph .. y - ph + 2,
  // BWDD (stride 1) reads dy rows y + ph - 2 .. y + ph
  const int org_y = MODE == MODE_FWD ? -a.ph : a.ph - 2, org_x = MODE == MODE_FWD ? -a.pw : a.pw - 2;
  int t_off[NKS], t_ch[NKS];
  bool t_ok[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const int tap = PACKED ? 4 * ks + kg : ks;
    const int r = tap / 3, s = tap - 3 * (tap / 3);
    t_ok[ks] = tap < 9;
    t_off[ks] = (MODE == MODE_FWD ? r : 2 - r) * PWT + (MODE == MODE_FWD ? s : 2 - s);
    t_ch[ks] = PACKED ? 0 : kg;
  }
  // packed mode stages whole 8-channel pixels; channels >= Cvalid are zeroed
  // when the fragments are read (the DMA cannot mask)
  const uint4 cmask = mask_chunk(make_uint4(~0u, ~0u, ~0u, ~0u), 0, PACKED ? a.Cvalid : 8);
  const int PH = a.IH >> a.up2, PWp = a.IW >> a.up2;
  const int tiles_x = a.OW / TW, tiles_y = (a.OH + TH - 1) / TH, tiles = a.N * tiles_x * tiles_y;
  const int t0 = lb * tiles_per_block, t1 = min(t0 + tiles_per_block, tiles);
  for (int tt = t0; tt < t1; ++tt) {
    const int n = tt / (tiles_x * tiles_y), rem = tt - n * tiles_x * tiles_y;
    const int y0 = (rem / tiles_x) * TH, x0 = (rem - (rem / tiles_x) * tiles_x) * TW;
    __syncthreads();  // the previous tile's fragment reads are done
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int sl = i * 256 + wv * 64 + lane;  // LDS slot this lane's piece lands in
      const int pix = sl / NCH, phys = sl - pix * NCH;
      const int ch = NCH == 4 ? (phys ^ ((pix >> 1) & 2)) : 0;
      const int pr = pix / PWT, pq = pix - pr * PWT;
      const int iy = y0 + org_y + pr, ix = x0 + org_x + pq;
      const bool ok = sl < NCHUNK && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
      const int off = (((n * PH + (iy >> a.up2)) * PWp + (ix >> a.up2)) * a.lds_src + ch * 8) * 2;
      lds_dma16(rsv, &tile[i * 256 + wv * 64], ok ? (unsigned)off : 0x80000000u);
    }
    wait_vmcnt_barrier<0>();
#pragma unroll 1
    for (int j = 0; j < TH / 4; ++j) {
      const int rr = wv * (TH / 4) + j;
#pragma unroll 2
      for (int g = 0; g < TW / 16; ++g) {
        const int q = 16 * g + col;
        uint4 bv[NKS];
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const int pix = rr * PWT + q + t_off[ks];
          bv[ks] = tile[pix * NCH + (NCH == 4 ? (t_ch[ks] ^ ((pix >> 1) & 2)) : 0)];
        }
        f32x4_t acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          uint4 v = bv[ks];
          if (PACKED) {
            v.x &= cmask.x;
            v.y &= cmask.y;
            v.z &= cmask.z;
            v.w &= cmask.w;
          }
          if (!t_ok[ks]) v = make_uint4(0, 0, 0, 0);
#pragma unroll
          for (int t = 0; t < NT; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t][ks], as_frag(v), acc[t], 0, 0, 0);
        }
        const int y = y0 + rr;
        if (y >= a.OH) continue;
        const long p = ((long)n * a.OH + y) * a.OW + x0 + q;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int co = 16 * t + 4 * kg;
          if (co >= a.Mrows) continue;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = act_fwd(acc[t][r] + bia[t][r], a.act, a.slope);
          bf16_t* op = reinterpret_cast<bf16_t*>(a.out) + p * a.ldo + co;
          if (co + 4 <= a.Mrows) {
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
}

// ------------------------------------------------------------ 1x1 convs --
// Pointwise convs (and their data gradients, again pointwise) with <= 256
// padded input channels: resD's learned shortcut conv_s (models.py:274) at
// every resolution, get_mask's 100 -> 1 projection (models.py:39).  A plain
// streaming GEMM over pixels: the tile kernels spend one LDS ring fill, one
// barrier-paced K-step or two and an epilogue per 64..256-pixel tile on these
// 1..8-K-step shapes (35 TFLOP/s, 1.6 TB/s at C32 -> K64).  Here a wave keeps
// its 16 NT output rows' weights (NT x NKS A fragments) in VGPRs and streams
// 16-pixel groups, each B fragment (8 channels of one pixel, 16 B) loaded
// straight into the lane that feeds it to the MFMA, the next groups' loads in
// flight during this group's MFMAs and stores; blockIdx.y picks the 16 NT-row
// slice of the output channels.  K order = the packed row (32-channel steps),
// as the tile kernels: bit-identical to their unsplit result.  Epilogue = theirs.
template <int MODE, int NT, int NKS, int GPI>
__global__ __launch_bounds__(256) void conv_1x1_kernel(ConvArgs a, int iters_per_block, int src_bytes) {
  const int lane = threadIdx.x & 63, kg = lane >> 4, col = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (b & 7) * (nb >> 3) + (b >> 3);  // XCD-contiguous logical block (nb % 8 == 0)
  const int co0 = blockIdx.y * 16 * NT;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, (short)0, src_bytes, 0x00020000);
  bf16x8_t fa[NT][NKS];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      fa[t][ks] = as_frag(*reinterpret_cast<const uint4*>(a.wp + (long)(co0 + 16 * t + col) * a.Kw + 32 * ks + 8 * kg));
  // chunks at or past the valid channels read zeros (OOB offset); the one
  // straddling Cvalid is masked after the loads were issued
  const int ld2 = a.lds_src * 2;
  int c_off[NKS];
  uint4 cm[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const int c = 32 * ks + 8 * kg;
    c_off[ks] = c < a.Cvalid ? c * 2 : -1;
    cm[ks] = mask_chunk(make_uint4(~0u, ~0u, ~0u, ~0u), c, a.Cvalid);
  }
  const int it0 = lb * iters_per_block, it_end = it0 + iters_per_block;
  auto load = [&](uint4 (&bv)[GPI][NKS], int it) {
#pragma unroll
    for (int g = 0; g < GPI; ++g) {
      const int p = (it * GPI + g) * 16 + col;
      const bool pok = it < it_end && p < a.P;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const int off = (pok && c_off[ks] >= 0) ? p * ld2 + c_off[ks] : (int)0x80000000;
        bv[g][ks] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      }
    }
  };
  auto compute = [&](uint4 (&bv)[GPI][NKS], int it) {
#pragma unroll
    for (int g = 0; g < GPI; ++g) {
      f32x4_t acc[NT][1];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t][0] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        uint4 v = bv[g][ks];
        v.x &= cm[ks].x;
        v.y &= cm[ks].y;
        v.z &= cm[ks].z;
        v.w &= cm[ks].w;
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[t][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t][ks], as_frag(v), acc[t][0], 0, 0, 0);
      }
      const int pix0 = (it * GPI + g) * 16;
      if (it < it_end && pix0 < a.P)
        igemm_epilogue<MODE, NT, 1, 16 * NT, 16>(a, acc, pix0, co0, 0, 0, lane, 0, a.P, a.OH, a.OW, 0, 0, 1);
    }
  };
  uint4 b0[GPI][NKS], b1[GPI][NKS];
  int it = it0 + wv;
  load(b0, it);
  for (; it < it_end; it += 8) {
    load(b1, it + 4);
    compute(b0, it);
    if (it + 4 >= it_end) break;
    load(b0, it + 8);
    compute(b1, it + 4);
  }
}

// ------------------------------------------ stride-2 backward-data, halo --
// Data gradient of the 4x4 / stride-2 / pad-1 convs with <= 32 input channels:
// resD.conv_r[0] of every discriminator's first block (models.py:267, fin =
// ndf, at the D's full resolution).  The tile kernels run it as four parity
// classes, each re-gathering its 2x2 taps of dy through L2 (16 gathers of every
// dy pixel over the classes; 0.74 TB/s).  Here one workgroup owns a TH x TW tile
// of the class grid for ALL four classes: the (TH + 2) x (TW + 2) dy halo they
// share is staged once in LDS by LDS-DMA, and wave w computes class
// (w >> 1, w & 1) from it, its 2x2-tap weight slab (NT x 4 NC A fragments)
// held in VGPRs.  K order = the tile kernels' (tap-major, 32-channel slices),
// so the fp32 sums are bit-identical to the unsplit tile kernel's.
// Epilogue: a class's pixels are every other dx pixel, so storing straight
// from the MFMA layout writes 32-B pieces at a 128-B stride (measured: the
// stores took 60 % of the kernel).  Instead each class row pair lands as fp32
// in an LDS staging image of two dx rows x 2 TW pixels, and the workgroup
// writes it out as whole 16-B runs of 8 channels (gate and residual applied
// there, in fp32, then rounded once -- as the tile kernels' epilogue).
// Class (qy, qx) with pad 1: first tap r0 = (qy + 1) & 1, dy row = i + qy - ta.
constexpr int S2B_TH = 4, S2B_TW = 32;

template <int NT, int NC>
__global__ __launch_bounds__(256, 2) void conv_s2bwd_lds_kernel(ConvArgs a, int src_bytes, int tiles_per_block) {
  constexpr int NCH = NC * 4;  // 16-B chunks per staged dy pixel
  constexpr int TH = S2B_TH, TW = S2B_TW, PWT = TW + 2, NPIX = (TH + 2) * PWT, NCHUNK = NPIX * NCH;
  constexpr int NDMA = (NCHUNK + 255) / 256;
  constexpr int NKS = 4 * NC;  // 2 x 2 taps x NC 32-channel slices
  constexpr int SPX = 2 * 2 * TW;  // staged dx pixels per class row (2 dx rows x 2 TW columns)
  constexpr int NSB = NC >= 4 ? 1 : 2;  // staging buffers (one at 128 K channels: 2 workgroups per CU)
  __shared__ uint4 tile[NDMA * 256];
  __shared__ float4 stage[NSB][SPX * 8];  // [buffer][pixel][8 fp32 chunks of 4 channels], chunk-swizzled
  const int tid = threadIdx.x, lane = tid & 63, kg = lane >> 4, col = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qy = wv >> 1, qx = wv & 1;
  const int r0 = (qy + 1) & 1, s0 = (qx + 1) & 1;
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (b & 7) * (nb >> 3) + (b >> 3);  // XCD-contiguous logical block (nb % 8 == 0)
  const rsrc_t rsv = make_rsrc(a.src, src_bytes);
  auto swz = [](int pix, int c) {
    return NCH == 16 ? c ^ (pix & 15) : NCH == 8 ? c ^ ((pix >> 1) & 7) : c ^ ((pix >> 1) & 2);
  };
  const int co0 = blockIdx.y * 32;  // this workgroup's 32-row slice of the input channels
  bf16x8_t fa[NT][NKS];
  int t_off[NKS], t_ch[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const int tap = ks / NC, cs = ks - tap * NC, ta = tap >> 1, tb = tap & 1;
    const int r = r0 + 2 * ta, s = s0 + 2 * tb;
#pragma unroll
    for (int t = 0; t < NT; ++t)
      fa[t][ks] = as_frag(*reinterpret_cast<const uint4*>(a.wp + (long)(co0 + 16 * t + col) * a.Kw +
                                                          (r * 4 + s) * a.Cgp + 32 * cs + 8 * kg));
    t_off[ks] = (qy - ta + 1) * PWT + (qx - tb + 1);
    t_ch[ks] = cs * 4 + kg;
  }
  const float gam = (a.res && a.gamma) ? *a.gamma : 1.f;
  const int C8 = min(32, a.Mrows - co0) >> 3;  // 8-channel output runs of the slice (Mrows % 8 == 0, host-checked)
  const int CH = a.OH >> 1, CW = a.OW >> 1;
  const int tiles_x = CW / TW, tiles_y = CH / TH, tiles = a.N * tiles_x * tiles_y;
  const int t0 = lb * tiles_per_block, t1 = min(t0 + tiles_per_block, tiles);
  int sb = 0;
  for (int tt = t0; tt < t1; ++tt) {
    const int n = tt / (tiles_x * tiles_y), rem = tt - n * tiles_x * tiles_y;
    const int i0 = (rem / tiles_x) * TH, j0 = (rem - (rem / tiles_x) * tiles_x) * TW;
    __syncthreads();  // the previous tile's fragment reads are done
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int sl = i * 256 + wv * 64 + lane;  // LDS slot this lane's piece lands in
      const int pix = sl / NCH, phys = sl - pix * NCH;
      const int pr = pix / PWT, pq = pix - pr * PWT;
      const int iy = i0 - 1 + pr, ix = j0 - 1 + pq;
      const bool ok = sl < NCHUNK && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
      const int off = (((n * a.IH + iy) * a.IW + ix) * a.lds_src + swz(pix, phys) * 8) * 2;
      lds_dma16(rsv, &tile[i * 256 + wv * 64], ok ? (unsigned)off : 0x80000000u);
    }
    wait_vmcnt_barrier<0>();
#pragma unroll 1
    for (int rr = 0; rr < TH; ++rr) {
      f32x4_t acc[TW / 16][NT];
#pragma unroll
      for (int g = 0; g < TW / 16; ++g) {
        const int q = 16 * g + col;
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[g][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const int pix = rr * PWT + q + t_off[ks];
          const bf16x8_t v = as_frag(tile[pix * NCH + swz(pix, t_ch[ks])]);
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[g][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t][ks], v, acc[g][t], 0, 0, 0);
        }
      }
      // stage: lane (col, kg) of tile t holds channels 16 t + 4 kg .. + 3 of dx pixel
      // (row qy, column 2 (16 g + col) + qx); 4-channel chunk index 4 t + kg
#pragma unroll
      for (int g = 0; g < TW / 16; ++g)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int sp = qy * 2 * TW + 2 * (16 * g + col) + qx;
          stage[sb][sp * 8 + ((4 * t + kg) ^ ((sp >> 1) & 7))] =
              make_float4(acc[g][t][0], acc[g][t][1], acc[g][t][2], acc[g][t][3]);
        }
      __syncthreads();
      const int y0 = 2 * (i0 + rr), x0 = 2 * j0;
#pragma unroll
      for (int k = 0; k < (SPX * 4 + 255) / 256; ++k) {
        const int item = tid + 256 * k, sp = item >> 2, e = item & 3;
        if (sp >= SPX || e >= C8) continue;
        const float4 lo = stage[sb][sp * 8 + ((2 * e) ^ ((sp >> 1) & 7))];
        const float4 hi = stage[sb][sp * 8 + ((2 * e + 1) ^ ((sp >> 1) & 7))];
        float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        const int y = y0 + sp / (2 * TW), x = x0 + sp % (2 * TW);
        const long p = ((long)n * a.OH + y) * a.OW + x;
        if (a.gate) {
          const uint4 gv = *reinterpret_cast<const uint4*>(a.gate + p * a.ldgate + co0 + 8 * e);
          const uint32_t gw[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[2 * j] *= act_dgrad_from_y(lo_f(gw[j]), a.gate_act, a.gate_slope);
            v[2 * j + 1] *= act_dgrad_from_y(hi_f(gw[j]), a.gate_act, a.gate_slope);
          }
        }
        if (a.res) {
          const long rp = a.res_up2 ? ((long)n * (a.OH >> 1) + (y >> 1)) * (a.OW >> 1) + (x >> 1) : p;
          const uint4 rv = *reinterpret_cast<const uint4*>(a.res + rp * a.ldres + co0 + 8 * e);
          const uint32_t rw[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[2 * j] = res_combine(a.res_scale, lo_f(rw[j]), gam, v[2 * j]);
            v[2 * j + 1] = res_combine(a.res_scale, hi_f(rw[j]), gam, v[2 * j + 1]);
          }
        }
        *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.out) + p * a.ldo + co0 + 8 * e) =
            make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
      }
      // the next row pair stages into the other buffer (one barrier per row pair), or
      // waits until this copy-out has read the single one
      if (NSB == 2) sb ^= 1;
      else __syncthreads();
    }
  }
}

// ---------------------------------------------------- thin weight gradient --
// dW of 3x3 stride-1 pad-1 convs with <= 8 output channels and 32 or 64
// (padded) input channels: get_image (ngf * {1, 2} -> 3, models.py:25-32),
// whose weight gradient reduces over every pixel of a 256x256 / 128x128 batch
// into only 3 x 9 x Cin values -- a shape the tile kernels split into ~100-170
// narrow pieces.  Here M = output channels (one 16-row MFMA tile), N = (tap,
// 16-channel block) = 9 * CGB tiles dealt round-robin to the 4 waves, K =
// pixels: each block stages 4 output rows x 64 pixels of dy and the
// (4 + 2) x (64 + 2) x halo in LDS, and both operands are read K-major with the
// gfx950 transposing ds_read_b64_tr_b16.  The K order inside a 32-pixel step
// is permuted (lane group g takes pixels 4g..4g+3 and 16+4g..16+4g+3) so every
// 32-lane half reads 8 consecutive pixels of a 32-B channel plane:
// conflict-free.  One partial per block goes to the split slab; the column
// reduce of the generic path maps it into the channels-last dW.
constexpr int WTH_H = 4, WTH_W = 64, WTH_PW = WTH_W + 2, WTH_XPIX = (WTH_H + 2) * WTH_PW;
typedef __attribute__((ext_vector_type(4))) short s16x4_tr;

EE_DEV s16x4_tr lds_tr16(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_tr*)(p));
}
EE_DEV bf16x8_t tr_pair(s16x4_tr lo, s16x4_tr hi) {
  typedef __attribute__((ext_vector_type(8))) short s16x8_tr;
  const s16x8_tr v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, v);
}

template <int CGB>  // 16-channel blocks of the padded Cin (2: 32 channels, 4: 64)
__global__ __launch_bounds__(256) void conv_wgrad_thin_kernel(WgradArgs w, int x_bytes, int dy_bytes,
                                                              int tiles_per_block) {
  constexpr int NT = 9 * CGB, NTW = (NT + 3) / 4;  // N tiles, per wave
  constexpr int XCH = WTH_XPIX * CGB * 2;           // 16-B chunks of the x halo
  constexpr int XLD = (XCH + 255) / 256;            // per thread
  __shared__ __attribute__((aligned(16))) bf16_t xs[CGB * WTH_XPIX * 16];  // [cb][pixel][16 ch]
  __shared__ __attribute__((aligned(16))) bf16_t dys[WTH_H * WTH_W * 8];   // [pixel][8 ch]
  const int tid = threadIdx.x, lane = tid & 63, kg = lane >> 4, li = lane & 15, q = li >> 2, pq = li & 3;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (b & 7) * (nb >> 3) + (b >> 3);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)w.x, (short)0, x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)w.dy, (short)0, dy_bytes, 0x00020000);
  f32x4_t acc[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int tiles_x = w.OW / WTH_W, tiles_y = w.OH / WTH_H, tiles = w.N * tiles_x * tiles_y;
  const int t0 = lb * tiles_per_block, t1 = min(t0 + tiles_per_block, tiles);
  for (int tt = t0; tt < t1; ++tt) {
    const int n = tt / (tiles_x * tiles_y), rem = tt - n * tiles_x * tiles_y;
    const int y0 = (rem / tiles_x) * WTH_H, x0 = (rem - (rem / tiles_x) * tiles_x) * WTH_W;
    uint4 xv[XLD];
#pragma unroll
    for (int i = 0; i < XLD; ++i) {
      const int e = tid + 256 * i;
      const int pix = e / (2 * CGB), ch = e - pix * (2 * CGB);
      const int pr = pix / WTH_PW, pc = pix - pr * WTH_PW;
      const int iy = y0 + pr - 1, ix = x0 + pc - 1;
      const bool ok = e < XCH && (unsigned)iy < (unsigned)w.IH && (unsigned)ix < (unsigned)w.IW;
      const int off = (((n * w.IH + iy) * w.IW + ix) * w.ldx + ch * 8) * 2;
      xv[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rx, ok ? off : 0x80000000, 0, 0));
    }
    const int dr = tid >> 6, dc = tid & 63;
    const int doff = ((((n * w.OH + y0 + dr) * w.OW) + x0 + dc) * w.lddy + 8 * (int)blockIdx.y) * 2;
    const uint4 dv = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rd, doff, 0, 0));
    __syncthreads();  // previous tile's reads done
#pragma unroll
    for (int i = 0; i < XLD; ++i) {
      const int e = tid + 256 * i;
      if (e < XCH) {
        const int pix = e / (2 * CGB), ch = e - pix * (2 * CGB);
        *reinterpret_cast<uint4*>(&xs[((ch >> 1) * WTH_XPIX + pix) * 16 + (ch & 1) * 8]) = xv[i];
      }
    }
    *reinterpret_cast<uint4*>(&dys[tid * 8]) = dv;
    __syncthreads();
#pragma unroll 1
    for (int rr = 0; rr < WTH_H; ++rr) {
#pragma unroll
      for (int kc = 0; kc < 2; ++kc) {
        const int p1 = 32 * kc + 4 * kg + q, p2 = p1 + 16;  // this lane's pixel rows of the two reads
        // A = dy^T: rows are output channels; lanes with pq >= 2 (channels 8..15,
        // past the staged 8) re-read channels 0..7, landing in unused rows >= 8
        const int cA = 4 * (pq & 1);
        const bf16x8_t fa =
            tr_pair(lds_tr16(&dys[(rr * WTH_W + p1) * 8 + cA]), lds_tr16(&dys[(rr * WTH_W + p2) * 8 + cA]));
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          const int t = wv + 4 * j;
          if (t < NT) {  // wave-uniform
            const int tap = t / CGB, cb = t - tap * CGB;
            const int r = tap / 3, s = tap - 3 * r;
            const int xp = cb * WTH_XPIX + (rr + r) * WTH_PW + s;
            const bf16x8_t fb =
                tr_pair(lds_tr16(&xs[(xp + p1) * 16 + 4 * pq]), lds_tr16(&xs[(xp + p2) * 16 + 4 * pq]));
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[j], 0, 0, 0);
          }
        }
      }
    }
  }
  float* slab = w.ws + (long)b * w.Cout * w.K;
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int t = wv + 4 * j;
    if (t >= NT) continue;
    const int tap = t / CGB, cb = t - tap * CGB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = 4 * kg + i, cog = 8 * (int)blockIdx.y + co;   // this block's 8-channel group
      if (co < 8 && cog < w.Cout) slab[cog * w.K + tap * (16 * CGB) + cb * 16 + li] = acc[j][i];
    }
  }
}

// Weight gradient of 3x3 / stride-1 / pad-1 convs with 32 or 64 input channels and
// output channels in 32-channel tiles (the generator's 32/64-channel 128^2 / 256^2
// layers, D256's 64-channel 128^2 resD conv): conv_wgrad_thin_kernel's halo staging
// for full MFMA tiles.  A block walks `tiles_per_block` 4 x 32-pixel tiles; per tile
// the 6 x 34 x CI source halo and the 128-pixel x 32-channel dy tile are staged in
// LDS once ([16-channel block][pixel][16 ch], transposed reads conflict-free), and
// each of the 9 taps reads its B fragments from the SAME halo at a column / row
// shift -- the tile kernels gather every x pixel once per tap through L2.  Wave w
// owns output-channel fragment w & 1 and input-channel fragment(s) of w >> 1 for all
// 9 taps (A = dy^T shared by the taps); K = pixels, each 32-pixel step read in the
// thin kernel's permuted order (rows 4 kg + q and + 16).  One fp32 partial per
// block into the split slab [nsplit][Cout][9 * CI], reduced in split order.
template <int CI>
__global__ __launch_bounds__(256) void conv_wgrad_halo3_kernel(WgradArgs w, int x_bytes, int dy_bytes,
                                                               int tiles_per_block) {
  // 32 input channels: wave w = output fragment w & 1 x input fragment w >> 1; 64: both
  // output fragments x input fragment w -- A and B fragment reads per MFMA 10 / 9 at 32
  // channels, 11 / 18 at 64
  constexpr int TH = 4, TW = 32, PW = TW + 2, XPIX = (TH + 2) * PW, CB = CI / 16;
  constexpr int NCO = CI >= 64 ? 2 : 1, NF = CI >= 64 ? CI / 64 : 1;
  constexpr int XCH = XPIX * CI / 8, XLD = (XCH + 255) / 256;   // 16-B chunks of the halo, per thread
  constexpr int DCH = TH * TW * 4, DLD = DCH / 256;              // of the dy tile (32 channels)
  __shared__ __attribute__((aligned(16))) bf16_t xs[CB * XPIX * 16];   // [cb][pixel][16 ch]
  __shared__ __attribute__((aligned(16))) bf16_t dys[2 * TH * TW * 16];  // [cb][pixel][16 ch]
  const int tid = threadIdx.x, lane = tid & 63, kg = lane >> 4, li = lane & 15, q = li >> 2, pq = li & 3;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cf0 = CI >= 64 ? 0 : (wv & 1), nf0 = CI >= 64 ? wv * NF : (wv >> 1);   // this wave's fragments
  const int nb = gridDim.x, b = blockIdx.x;
  const int lb = (b & 7) * (nb >> 3) + (b >> 3);   // a block's consecutive tiles share one XCD (nb % 8 == 0)
  const int co0 = blockIdx.y * 32;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)w.x, (short)0, x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)w.dy, (short)0, dy_bytes, 0x00020000);
  f32x4_t acc[NCO][NF][9];
#pragma unroll
  for (int c = 0; c < NCO; ++c)
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int t = 0; t < 9; ++t) acc[c][f][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int tiles_x = w.OW / TW, tiles_y = w.OH / TH, tiles = w.N * tiles_x * tiles_y;
  const int t0 = lb * tiles_per_block, t1 = min(t0 + tiles_per_block, tiles);
  for (int tt = t0; tt < t1; ++tt) {
    const int n = tt / (tiles_x * tiles_y), rem = tt - n * tiles_x * tiles_y;
    const int y0 = (rem / tiles_x) * TH, x0 = (rem - (rem / tiles_x) * tiles_x) * TW;
    uint4 xv[XLD], dv[DLD];
#pragma unroll
    for (int i = 0; i < XLD; ++i) {
      const int e = tid + 256 * i;
      const int pix = e / (CI / 8), ch = e - pix * (CI / 8);
      const int pr = pix / PW, pc = pix - pr * PW;
      const int iy = y0 + pr - 1, ix = x0 + pc - 1;
      const bool ok = e < XCH && (unsigned)iy < (unsigned)w.IH && (unsigned)ix < (unsigned)w.IW;
      const int off = (((n * w.IH + iy) * w.IW + ix) * w.ldx + ch * 8) * 2;
      xv[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rx, ok ? off : 0x80000000, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < DLD; ++i) {
      const int e = tid + 256 * i, pix = e >> 2, ch = e & 3;
      const int off = ((((n * w.OH + y0 + pix / TW) * w.OW) + x0 + pix % TW) * w.lddy + co0 + ch * 8) * 2;
      dv[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rd, off, 0, 0));
    }
    __syncthreads();   // the previous tile's fragment reads are done
#pragma unroll
    for (int i = 0; i < XLD; ++i) {
      const int e = tid + 256 * i;
      if (e < XCH) {
        const int pix = e / (CI / 8), ch = e - pix * (CI / 8);
        *reinterpret_cast<uint4*>(&xs[((ch >> 1) * XPIX + pix) * 16 + (ch & 1) * 8]) = xv[i];
      }
    }
#pragma unroll
    for (int i = 0; i < DLD; ++i) {
      const int e = tid + 256 * i, pix = e >> 2, ch = e & 3;
      *reinterpret_cast<uint4*>(&dys[((ch >> 1) * (TH * TW) + pix) * 16 + (ch & 1) * 8]) = dv[i];
    }
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < TH; ++rr) {
      const int p1 = 4 * kg + q, p2 = p1 + 16;
      bf16x8_t fa[NCO];
#pragma unroll
      for (int c = 0; c < NCO; ++c) {
        const bf16_t* da = &dys[((cf0 + c) * (TH * TW) + rr * TW) * 16 + 4 * pq];
        fa[c] = tr_pair(lds_tr16(da + p1 * 16), lds_tr16(da + p2 * 16));
      }
#pragma unroll
      for (int f = 0; f < NF; ++f) {
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int ta = t / 3, tb = t - 3 * ta;
          const bf16_t* xb = &xs[((nf0 + f) * XPIX + (rr + ta) * PW + tb) * 16 + 4 * pq];
          const bf16x8_t fb = tr_pair(lds_tr16(xb + p1 * 16), lds_tr16(xb + p2 * 16));
#pragma unroll
          for (int c = 0; c < NCO; ++c)
            acc[c][f][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[c], fb, acc[c][f][t], 0, 0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NCO; ++c) {
    float* slab = w.ws + ((long)b * w.Cout + co0 + 16 * (cf0 + c)) * w.K;
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) slab[(4 * kg + j) * w.K + t * CI + 16 * (nf0 + f) + li] = acc[c][f][t][j];
  }
}

// ------------------------------------------------------------ dispatch --
int cgp_of(int C) { return C <= 8 ? 8 : ee_round_up(C, BK); }
int kw_of(int R, int S, int Cgp) { return ee_round_up(R * S * Cgp, BK); }

struct Plan {
  int tco, tpix, nsplit, blocks;
};

// Planner / kernel-path knobs for A/B tests and sweeps, all in one variable:
// EEGAN_CONV="thin=0,wide=0,target=256" (key = the knob's name below; unset
// keys keep their defaults).  Read per launch on the host.
static int knob(const char* key, int dflt) {
  const char* v = getenv("EEGAN_CONV");
  if (!v) return dflt;
  const size_t n = strlen(key);
  for (const char* p = v; p && *p;) {
    if (!strncmp(p, key, n) && p[n] == '=') return atoi(p + n + 1);
    p = strchr(p, ',');
    if (p) ++p;
  }
  return dflt;
}

Plan plan_igemm(const ConvArgs& a, int Pc_max) {
  // tuning knobs (benchmark sweeps only): grid target, min K-steps per split,
  // and whether 64-row tiles are tried before splitting K
  // throughput objective (eegan_conv_desc.plan = 1, a stream beside the critical chain):
  // a smaller grid target -- larger tiles, and no split-K partials / reduce launch once
  // the grid reaches it
  // 1024 (four workgroups per CU) over 512: +0.6 / +0.7 % in-process on the replayed step
  // (profiles/r06n_target_ab.txt; 1536 / 2048 -0.1 %) -- the small-grid 3x3 launches
  // (512-channel 16^2, 256-channel 8^2 ...) are latency-bound per K step, two splits halve that
  const int target = a.tp ? knob("tp_target", 128) : knob("target", 1024);
  const int mink = knob("mink", 16);
  const int small_co = knob("smallco", 1);
  const int rows = a.Mrows;
  Plan p;
  p.tco = rows > 64 ? 128 : rows > 32 ? 64 : rows > 16 ? 32 : 16;
  int co_t = ee_cdiv(rows, p.tco);
  p.tpix = (p.tco <= 32) ? 256 : 128;
  if ((long)ee_cdiv(Pc_max, p.tpix) * co_t * a.ncls < target) p.tpix = 64;
  if (small_co && p.tco == 128 && (long)ee_cdiv(Pc_max, p.tpix) * co_t * a.ncls < target) {
    p.tco = 64;
    co_t = ee_cdiv(rows, p.tco);
  }
  p.blocks = ee_cdiv(Pc_max, p.tpix) * co_t * a.ncls;
  // split K until the grid covers the chip twice, keeping >= mink K-steps per split
  int taps = a.R * a.S;
  if (a.ncls > 1) taps = ee_cdiv(a.R, a.st) * ee_cdiv(a.S, a.st);
  const int nk = a.Cgp == 8 ? (taps + 3) / 4 : taps * (a.Cgp / BK);
  p.nsplit = 1;
  while (p.blocks * p.nsplit < target && nk / (p.nsplit * 2) >= mink && p.nsplit < 64) p.nsplit *= 2;
  return p;
}

// 3x3 stride-1 convs with <= 32 output rows take conv_thin_kernel.  Returns
// 0 when the shape is not eligible (the tile kernels run), else the launch rc.
template <int MODE>
int try_thin(const ConvArgs& a, hipStream_t s, long src_bytes) {
  if (!knob("thin", 1) || src_bytes >= 0x7fffffffL) return 0;
  if (a.R != 3 || a.S != 3 || a.st != 1 || a.ncls != 1 || a.res || a.gate || a.out_f32 || a.Mrows > 32) return 0;
  if ((a.ldo & 3) || ((uintptr_t)a.out & 7) || (a.lds_src & 7) || ((uintptr_t)a.src & 15)) return 0;
  const int nt = a.Mrows > 16 ? 2 : 1, slices = ee_cdiv(a.Mrows, 32);
  const int nks = a.Cgp == 8 ? 3 : a.Cgp == 32 ? 9 : (a.Cgp == 64 && nt == 1) ? 18 : 0;
  if (!nks || (nks > 3 && (a.Cvalid & 7))) return 0;
  const int gpi = nks == 3 ? 2 : 1;
  const long iters = ((a.P + 15L) / 16 + gpi - 1) / gpi;
  const int nb = ee_round_up((int)std::min<long>((iters + 3) / 4, 1024), 8);
  const int ipb = (int)((iters + nb - 1) / nb);
  if (nks <= 9 && a.OW % 64 == 0 && a.ph <= 1 && a.pw <= 1 && knob("thin_lds", 1)) {
    const int tiles = a.N * (a.OW / 64) * ((a.OH + 7) / 8);
    const int nbl = ee_round_up(std::min(tiles, nks == 3 ? 2048 : 768), 8), tpb = (tiles + nbl - 1) / nbl;
#define TL(NT, NKS) ee_launch(conv_thin_lds_kernel<MODE, NT, NKS>, dim3(nbl), dim3(256), 0, s, a, (int)src_bytes, tpb)
    if (nks == 3) { if (nt == 1) TL(1, 3); else TL(2, 3); }
    else { if (nt == 1) TL(1, 9); else TL(2, 9); }
#undef TL
    const int rc = ee_check_launch(MODE == MODE_FWD ? "conv_fwd(thin-lds)" : "conv_bwd_data(thin-lds)");
    return rc ? rc : 1;
  }
#define TH(NT, NKS, G) ee_launch(conv_thin_kernel<MODE, NT, NKS, G>, dim3(nb), dim3(256), 0, s, a, ipb, (int)src_bytes)
  if (nks == 3) { if (nt == 1) TH(1, 3, 2); else TH(2, 3, 2); }
  else if (nks == 9) { if (nt == 1) TH(1, 9, 1); else TH(2, 9, 1); }
  else TH(1, 18, 1);
#undef TH
  const int rc = ee_check_launch(MODE == MODE_FWD ? "conv_fwd(thin)" : "conv_bwd_data(thin)");
  return rc ? rc : 1;
}

// 4x4 / stride-2 / pad-1 forward convs, 32 -> 64 channels, bias / activation only, on
// whole 2 x 32 output tiles take conv_s2fwd_kernel (0: not eligible, else the launch rc)
int try_s2fwd(const ConvArgs& a, hipStream_t s, long src_bytes) {
  if (!knob("s2f", 1) || src_bytes >= 0x7fffffffL) return 0;
  if (a.R != 4 || a.S != 4 || a.st != 2 || a.ph != 1 || a.pw != 1 || a.ncls != 1 || a.nsplit != 1 || a.up2) return 0;
  if (a.Cgp != BK || a.Cvalid != BK || a.Mrows != 64 || a.Kw != 16 * BK) return 0;
  if (a.res || a.gate || a.out_f32 || (a.ldo & 7) || ((uintptr_t)a.out & 15)) return 0;
  if ((a.lds_src & 7) || ((uintptr_t)a.src & 15)) return 0;
  if (a.OW % S2F_TW || a.OH % S2F_TH || a.IH != 2 * a.OH || a.IW != 2 * a.OW) return 0;
  const long tiles = (long)a.N * (a.OH / S2F_TH) * (a.OW / S2F_TW);
  if (tiles >= 0x7fffffffL) return 0;
  // persistent: two workgroups per CU (VGPR-bound: 64 of a wave's registers hold its weights,
  // loaded once per workgroup)
  const unsigned grid = (unsigned)std::min<long>(tiles, 2 * 256);
  ee_launch(conv_s2fwd_kernel, dim3(grid), dim3(256), 0, s, a, src_bytes);
  const int rc = ee_check_launch("conv_fwd(s2-halo)");
  return rc ? rc : 1;
}

// 3x3 / stride-1 / pad-1 convs with >= 32 output rows on grids of whole 8 x 32
// tiles take conv_halo3_kernel (0: not eligible, else the launch rc)
template <int MODE>
int try_halo3(const ConvArgs& a, hipStream_t s, long src_bytes, long w_bytes) {
  if (!knob("halo", 1) || src_bytes >= 0x7fffffffL || w_bytes >= 0x7fffffffL) return 0;
  if (a.R != 3 || a.S != 3 || a.st != 1 || a.ph != 1 || a.pw != 1 || a.ncls != 1 || a.nsplit != 1) return 0;
  if (MODE == MODE_BWDD && a.up2) return 0;
  // >= 32 rows: at 32 the 64-row tile idles half its MFMAs, and still beats the tile
  // kernels by 17-19 % (fetch-bound; 3x3 64 -> 32 at 256^2 143 -> 118 us)
  if (a.Mrows < 32 || a.Cgp % BK || a.out_f32) return 0;
  if ((a.Cvalid & 7) && MODE != MODE_BWDD) return 0;   // ragged inputs: data gradients only (get_mask's 100-ch)
  if ((a.lds_src & 7) || ((uintptr_t)a.src & 15) || (a.ldo & 7) || ((uintptr_t)a.out & 15)) return 0;
  if (a.gate && ((a.ldgate & 7) || ((uintptr_t)a.gate & 15))) return 0;
  if (a.res && ((a.ldres & 7) || ((uintptr_t)a.res & 15))) return 0;
  if (a.OW % HALO_TW || a.OH % 8 || a.OH != a.IH || a.OW != a.IW) return 0;
  const int co_t = ee_cdiv(a.Mrows, HALO_TCO);
  const auto simple_act = [](int act) { return act == ACT_NONE || act == ACT_RELU || act == ACT_LRELU; };
  if (a.Cgp == 64 && a.Cvalid == 64 && a.Mrows % HALO_TCO == 0 && simple_act(a.act) &&
      (MODE == MODE_FWD || !a.gate || simple_act(a.gate_act)) && knob("halo_r", 1)) {
    // 64-channel inputs: resident weights, TPB consecutive tiles per workgroup -- one
    // workgroup per CU (its 160 KB of LDS), up to 16 tiles each (tools/conv_bench.py: D256
    // b0 at N = 32 fwd / bwdd 54 / 58 us at 16 tiles vs 56 / 62 at 8; 64-ch 128^2 N = 16
    // 28 / 29 us at 8 vs 30 / 32 at 4)
    const long tiles = (long)a.N * (a.OH / 4) * (a.OW / HALO_TW);
    int tpb = knob("halo_r_tpb", 0);
    if (tpb <= 0) {
      const long t = tiles * co_t / 256;
      tpb = t < 1 ? 1 : t > 16 ? 16 : (int)t;
    }
    const dim3 grid((unsigned)ee_cdiv(tiles, (long)tpb), co_t);
    ee_launch(conv_halo3r_kernel<MODE>, grid, dim3(256), 0, s, a, src_bytes, w_bytes, tpb, knob("halo_r_knock", 0));
    const int rc = ee_check_launch(MODE == MODE_FWD ? "conv_fwd(halo3r)" : "conv_bwd_data(halo3r)");
    return rc ? rc : 1;
  }
  const long tiles16 = a.OH % 16 ? 0 : (long)a.N * (a.OH / 16) * (a.OW / HALO_TW) * co_t;
  const int big = knob("halo_th", 0);   // 16 / 8: force the tile height (tests, sweeps)
  const bool th16 = big == 16 || (big != 8 && tiles16 >= 256);
  if (th16 && !tiles16) return 0;
  const dim3 grid16((unsigned)(tiles16 / co_t), co_t), grid8((unsigned)((long)a.N * (a.OH / 8) * (a.OW / HALO_TW)), co_t);
  // default: three single-buffered 4-row workgroups per CU (52 KB of LDS each): one's slice
  // loads, first-slice wait and epilogue run under the others' MFMAs, and other lanes' kernels
  // still fit beside them.  Per kernel it wins on small-spatial / few-slice layers (3x3 256-ch
  // 32^2 28.5 -> 24.8 us, D256 b0 60.7 -> 58.0) and loses on others (128-ch 64^2 24.4 -> 29.0);
  // on the replayed step +0.8 / +0.9 % against two 8-row workgroups per CU (halo_nb=1), which
  // was +0.4 / +0.6 % against the double-buffered one-workgroup-per-CU forms (halo_nb=2)
  const int nb = knob("halo_nb", 3);
  const dim3 grid4((unsigned)((long)a.N * (a.OH / 4) * (a.OW / HALO_TW)), co_t);
  if constexpr (MODE == MODE_BWDD) {
    if (a.Cvalid & 7) {
      if (big == 16) ee_launch(conv_halo3_kernel<MODE, 16, 8, true>, grid16, dim3(512), 0, s, a, src_bytes, w_bytes);
      else if (big == 8) ee_launch(conv_halo3_kernel<MODE, 8, 4, true>, grid8, dim3(256), 0, s, a, src_bytes, w_bytes);
      else ee_launch(conv_halo3_kernel<MODE, 4, 4, true, 1>, grid4, dim3(256), 0, s, a, src_bytes, w_bytes);
      const int rc = ee_check_launch("conv_bwd_data(halo3)");
      return rc ? rc : 1;
    }
  }
  if (!big && nb == 3)
    ee_launch(conv_halo3_kernel<MODE, 4, 4, false, 1>, grid4, dim3(256), 0, s, a, src_bytes, w_bytes);
  else if (!big && nb == 1)
    ee_launch(conv_halo3_kernel<MODE, 8, 4, false, 1>, grid8, dim3(256), 0, s, a, src_bytes, w_bytes);
  else if (th16) ee_launch(conv_halo3_kernel<MODE, 16, 8>, grid16, dim3(512), 0, s, a, src_bytes, w_bytes);
  else ee_launch(conv_halo3_kernel<MODE, 8, 4>, grid8, dim3(256), 0, s, a, src_bytes, w_bytes);
  const int rc = ee_check_launch(MODE == MODE_FWD ? "conv_fwd(halo3)" : "conv_bwd_data(halo3)");
  return rc ? rc : 1;
}

// 4x4 / stride-2 / pad-1 data gradients with <= 32 input channels take
// conv_s2bwd_lds_kernel (0: not eligible, else the launch rc as try_thin)
int try_s2bwd(const ConvArgs& a, hipStream_t s, long src_bytes) {
  if (!knob("s2b", 1) || src_bytes >= 0x7fffffffL) return 0;
  if (a.R != 4 || a.S != 4 || a.st != 2 || a.ph != 1 || a.pw != 1 || a.ncls != 4 || a.up2 || a.Mrows > 64) return 0;
  if ((a.Cgp != 32 && a.Cgp != 64 && a.Cgp != 128) || a.Cvalid != a.Cgp || (a.lds_src & 7) ||
      ((uintptr_t)a.src & 15))
    return 0;
  if (a.Mrows > 32 && !knob("s2b64", 1)) return 0;
  // LDS-staged epilogue: bf16 output, 16-B runs of 8 channels (output / gate / residual rows 16-B aligned)
  if (a.out_f32 || a.bias || a.act != ACT_NONE || (a.Mrows & 7) || (a.ldo & 7) || ((uintptr_t)a.out & 15)) return 0;
  if (a.gate && ((a.ldgate & 7) || ((uintptr_t)a.gate & 15))) return 0;
  if (a.res && ((a.ldres & 7) || ((uintptr_t)a.res & 15))) return 0;
  if ((a.OH & 1) || (a.OW & 1) || (a.OW / 2) % S2B_TW || (a.OH / 2) % S2B_TH) return 0;
  if ((long)a.N * a.OH * a.OW >= 0x7fffffffL) return 0;
  const int tiles = a.N * (a.OW / 2 / S2B_TW) * (a.OH / 2 / S2B_TH);
  const int nbl = ee_round_up(std::min(tiles, knob("s2b_blocks", 512)), 8);
  const int tpb = (tiles + nbl - 1) / nbl;
  const int nt = a.Mrows > 16 ? 2 : 1, slices = ee_cdiv(a.Mrows, 32);
  ConvArgs a2 = a;
#define SB(NT, NC) \
  ee_launch(conv_s2bwd_lds_kernel<NT, NC>, dim3(nbl, slices), dim3(256), 0, s, a2, (int)src_bytes, tpb)
  if (a.Cgp == 128) { if (nt == 2) SB(2, 4); else SB(1, 4); }
  else if (a.Cgp == 64) { if (nt == 2) SB(2, 2); else SB(1, 2); }
  else { if (nt == 2) SB(2, 1); else SB(1, 1); }
#undef SB
  const int rc = ee_check_launch("conv_bwd_data(s2-halo)");
  return rc ? rc : 1;
}

// 1x1 stride-1 convs with <= 256 packed K columns take conv_1x1_kernel
// (0: not eligible, else the launch rc as try_thin)
template <int MODE>
int try_1x1(const ConvArgs& a, hipStream_t s, long src_bytes) {
  if (!knob("1x1", 1) || src_bytes >= 0x7fffffffL) return 0;
  if (a.R != 1 || a.S != 1 || a.st != 1 || a.ph || a.pw || a.ncls != 1 || a.up2 || a.Kw > 256) return 0;
  if ((a.lds_src & 7) || ((uintptr_t)a.src & 15)) return 0;
  const int nks = a.Kw / BK;
  // measured (tools/conv_bench.py): ahead of the tile kernels for one K-step
  // (<= 128 rows), two K-steps at <= 64 rows and single-tile rows (<= 16);
  // behind them from 64 -> 128 channels up (one B fragment per 8 MFMAs, 2
  // waves per SIMD at NT = 8; or the input re-read per 64-row slice)
  if (!(nks == 1 || (nks == 2 && a.Mrows <= 64) || a.Mrows <= 16)) return 0;
  const int nt_max = nks <= 2 ? 8 : nks == 4 ? 4 : 2;
  int nt = 1;
  while (nt < nt_max && 16 * nt < a.Mrows) nt *= 2;
  const int rowblocks = ee_cdiv(a.Mrows, 16 * nt);
  constexpr int G1 = 1;  // groups per wave iteration (larger: more loads in flight, but the
  const int gpi = G1;    // epilogue unrolled per group costs VGPRs: 247 at NT = 4, GPI = 4)
  const long iters = ((a.P + 15L) / 16 + gpi - 1) / gpi;
  const int cap = std::max(64, knob("1x1_blocks", 1024) / rowblocks);
  const int nb = ee_round_up((int)std::min<long>((iters + 3) / 4, cap), 8);
  const int ipb = (int)((iters + nb - 1) / nb);
  const dim3 grid(nb, rowblocks);
#define P1(NT, NKS, G) ee_launch(conv_1x1_kernel<MODE, NT, NKS, G>, grid, dim3(256), 0, s, a, ipb, (int)src_bytes)
  switch (nks * 16 + nt) {
    case 16 + 1: P1(1, 1, G1); break;
    case 16 + 2: P1(2, 1, G1); break;
    case 16 + 4: P1(4, 1, G1); break;
    case 16 + 8: P1(8, 1, G1); break;
    case 32 + 1: P1(1, 2, G1); break;
    case 32 + 2: P1(2, 2, G1); break;
    case 32 + 4: P1(4, 2, G1); break;
    case 32 + 8: P1(8, 2, G1); break;
    case 64 + 1: P1(1, 4, 1); break;
    case 64 + 2: P1(2, 4, 1); break;
    case 64 + 4: P1(4, 4, 1); break;
    case 128 + 1: P1(1, 8, 1); break;
    case 128 + 2: P1(2, 8, 1); break;
    default: return 0;
  }
#undef P1
  const int rc = ee_check_launch(MODE == MODE_FWD ? "conv_fwd(1x1)" : "conv_bwd_data(1x1)");
  return rc ? rc : 1;
}

template <int MODE>
int launch_igemm(ConvArgs a, int Pc_max, float* part_ws, hipStream_t s, long src_bytes, int* ctr = nullptr,
                 int ctr_n = 0) {
  if (const int th = try_thin<MODE>(a, s, src_bytes)) return th > 0 ? 0 : th;
  if (const int pw = try_1x1<MODE>(a, s, src_bytes)) return pw > 0 ? 0 : pw;
  if (MODE == MODE_BWDD)
    if (const int sb = try_s2bwd(a, s, src_bytes)) return sb > 0 ? 0 : sb;
  if (MODE == MODE_FWD)
    if (const int sf = try_s2fwd(a, s, src_bytes)) return sf > 0 ? 0 : sf;
  if (const int hl = try_halo3<MODE>(a, s, src_bytes, (long)ee_round_up(a.Mrows, 128) * a.Kw * 2))
    return hl > 0 ? 0 : hl;
  Plan p = plan_igemm(a, Pc_max);
  a.nsplit = p.nsplit;
  a.part = p.nsplit > 1 ? part_ws : nullptr;
  {
    // wide pair stages (whole 128-B lines: 64 channels per pixel / weight row): an
    // even number of 32-channel slices per tap and every split starting on a pair
    const int nc = a.Cgp / BK;
    int taps_max = a.R * a.S;
    if (MODE == MODE_BWDD && a.st > 1) taps_max = ee_cdiv(a.R, a.st) * ee_cdiv(a.S, a.st);
    const int nk_max = taps_max * nc;
    const int kchunk = ee_cdiv(nk_max, p.nsplit);
    a.wide = p.tco >= 64 && nc % 2 == 0 && kchunk % 2 == 0 && knob("wide", 1);
  }
  // LDS-staged epilogue (conv_fast_kernel): unsplit bf16 output with 16-B aligned rows
  a.stage_epi = p.nsplit == 1 && !a.out_f32 && a.Mrows % 8 == 0 && a.ldo % 8 == 0 && ((uintptr_t)a.out & 15) == 0 &&
                (!a.gate || (a.ldgate % 8 == 0 && ((uintptr_t)a.gate & 15) == 0)) &&
                (!a.res || (a.ldres % 8 == 0 && ((uintptr_t)a.res & 15) == 0)) && knob("stage_epi", 1);
  if (p.nsplit > 1 && !part_ws) {
    ee_set_error("conv: split-K workspace missing");
    return -22;
  }
  dim3 grid(ee_cdiv(Pc_max, p.tpix), ee_cdiv(a.Mrows, p.tco), a.ncls * p.nsplit);
  const long total = (long)a.P * a.Mrows;
  if (p.nsplit > 1) {
    const uintptr_t oal = a.out_f32 ? 15 : 7;
    // red_vec4=0 forces the scalar reduce (A/B and bit-identity tests)
    a.red_vec4 = a.Mrows % 4 == 0 && total < 0x7fffffffL && a.ldo % 4 == 0 && ((uintptr_t)a.out & oal) == 0 &&
                 ((uintptr_t)a.part & 15) == 0 && (!a.gate || a.gate_vec) && (!a.res || a.res_vec) &&
                 knob("red_vec4", 1);
  }
  const long w_bytes = (long)ee_round_up(a.Mrows, 128) * a.Kw * 2;
  if (p.nsplit > 1 && a.red_vec4 && ctr && (long)grid.x * grid.y * a.ncls <= ctr_n &&
      (long)p.nsplit * total * 4 < 0x7fffffffL && knob("splitk_fused", 0))
    a.ctr = ctr;   // conv_fast_kernel finishes the split itself (below: only when `fast`)
  dim3 fgrid = grid;   // conv_fast_kernel's grid: the XCD raster when it applies
  {
    const long nb = (long)grid.x * grid.y * grid.z;
    const int xcd = knob("xcd", 1);
    if (xcd && nb >= knob("xcd_minb", 64) && nb < (1L << 30)) {
      // rows per group G ~ sqrt(S * B / A), S = blocks per XCD; per tile the weight rows carry
      // TCO * taps * C and the pixel tile ~ TPIX * st^2 * C unique bytes (taps re-read pixels)
      const int S_ = (int)(((nb + 7) & ~7L) / 8);
      const double ab = (double)p.tco * a.R * a.S / ((double)p.tpix * a.st * a.st);
      int G = xcd > 1 ? xcd : (int)(sqrt((double)S_ / ab) + 0.5);
      G = std::max(1, std::min(G, (int)grid.y));
      a.xcd_g = G;
      a.gx = grid.x;
      a.gy = grid.y;
      a.gz = grid.z;
      fgrid = dim3((unsigned)((nb + 7) & ~7L), 1, 1);
    }
  }
#define GL(TC, TP) ee_launch(conv_glds_kernel<MODE, TC, TP>, grid, dim3(256), 0, s, a, src_bytes, w_bytes)
#define FA(TC, TP) ee_launch(conv_fast_kernel<MODE, TC, TP, 2, 4, 2>, fgrid, dim3(256), 0, s, a, src_bytes, w_bytes)
#define IG(TC, TP, WC) ee_launch(conv_igemm_kernel<MODE, TC, TP, WC>, grid, dim3(256), 0, s, a)
  // glds: channel chunks fetched whole (C % 8 != 0 masked in the fragments; the
  // fast kernel needs whole valid chunks)
  const bool glds = ((a.Cvalid % 8) == 0 || a.Cgp == 8 || knob("glds_ragged", 1)) &&
                    src_bytes < 0x7fffffffL && w_bytes < 0x7fffffffL;
  int tr_ = a.R, ts_ = a.S;
  if (MODE == MODE_BWDD && a.st > 1) tr_ = ee_cdiv(a.R, a.st), ts_ = ee_cdiv(a.S, a.st);
  const bool fast = glds && a.Cgp % BK == 0 && !a.up2 && tr_ * ts_ <= 32 && knob("fast", 1);
  if (!fast) a.ctr = nullptr;
  if (fast) {
    if (p.tco == 128) { if (p.tpix == 128) FA(128, 128); else FA(128, 64); }
    else if (p.tco == 64) { if (p.tpix == 128) FA(64, 128); else FA(64, 64); }
    else if (p.tco == 32) { if (p.tpix == 256) FA(32, 256); else FA(32, 64); }
    else { if (p.tpix == 256) FA(16, 256); else FA(16, 64); }
  }
  else if (glds) {
    if (p.tco == 128) { if (p.tpix == 128) GL(128, 128); else GL(128, 64); }
    else if (p.tco == 64) { if (p.tpix == 128) GL(64, 128); else GL(64, 64); }
    else if (p.tco == 32) { if (p.tpix == 256) GL(32, 256); else GL(32, 64); }
    else { if (p.tpix == 256) GL(16, 256); else GL(16, 64); }
  }
  else if (p.tco == 128) { if (p.tpix == 128) IG(128, 128, 2); else IG(128, 64, 2); }
  else if (p.tco == 64) { if (p.tpix == 128) IG(64, 128, 2); else IG(64, 64, 2); }
  else if (p.tco == 32) { if (p.tpix == 256) IG(32, 256, 1); else IG(32, 64, 1); }
  else { if (p.tpix == 256) IG(16, 256, 1); else IG(16, 64, 1); }
#undef IG
#undef GL
#undef FA
  int rc = ee_check_launch(MODE == MODE_FWD ? "conv_fwd" : "conv_bwd_data");
  if (rc || a.nsplit == 1 || a.ctr) return rc;
  const long work = a.red_vec4 ? total / 4 : total;
  ee_launch(conv_splitk_reduce_kernel<MODE>, dim3((int)std::min<long>((work + 255) / 256, 4096)), dim3(256), 0, s, a);
  return ee_check_launch("conv_splitk_reduce");
}

long part_bytes(const ConvArgs& a, int Pc_max) {
  Plan p = plan_igemm(a, Pc_max);
  return p.nsplit > 1 ? (long)p.nsplit * a.P * a.Mrows * (long)sizeof(float) : 0;
}

void fill_fwd(ConvArgs& a, const eegan_conv_desc* d) {
  a = ConvArgs{};
  a.N = d->N;
  a.IH = d->H;
  a.IW = d->W;
  a.lds_src = d->ldx;
  a.up2 = d->up2;
  a.OH = d->Ho;
  a.OW = d->Wo;
  a.R = d->R;
  a.S = d->S;
  a.st = d->stride;
  a.ph = d->pad_h;
  a.pw = d->pad_w;
  a.Cgp = cgp_of(d->C);
  a.Cvalid = d->C;
  a.Mrows = d->K;
  a.Kw = kw_of(d->R, d->S, a.Cgp);
  a.P = d->N * d->Ho * d->Wo;
  a.ncls = 1;
  a.nsplit = 1;
  a.res_scale = 1.f;
  a.tp = d->plan == 1;
}

void fill_bwdd(ConvArgs& a, const eegan_conv_desc* d) {
  a = ConvArgs{};
  a.N = d->N;
  a.IH = d->Ho;  // source grid = dy grid
  a.IW = d->Wo;
  a.lds_src = d->ldy;
  a.up2 = 0;
  a.OH = d->H;   // GEMM pixels = input pixels
  a.OW = d->W;
  a.R = d->R;
  a.S = d->S;
  a.st = d->stride;
  a.ph = d->pad_h;
  a.pw = d->pad_w;
  a.Cgp = cgp_of(d->K);
  a.Cvalid = d->K;
  a.Mrows = d->C;
  a.Kw = kw_of(d->R, d->S, a.Cgp);
  a.P = d->N * d->H * d->W;
  a.ncls = d->stride > 1 ? d->stride * d->stride : 1;
  a.nsplit = 1;
  a.res_scale = 1.f;
  a.tp = d->plan == 1;
}

int bwdd_pc_max(const eegan_conv_desc* d) {
  if (d->stride == 1) return d->N * d->H * d->W;
  return d->N * ee_cdiv(d->H, d->stride) * ee_cdiv(d->W, d->stride);
}

bool ld_ok(int ld, const void* p) { return (ld % 8) == 0 && ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" {

long eegan_conv_packed_elems(int Cout, int Cin, int R, int S, int transposed) {
  const int rows = transposed ? Cin : Cout;
  const int Cgp = cgp_of(transposed ? Cout : Cin);
  return (long)ee_round_up(rows, 128) * kw_of(R, S, Cgp);
}

int eegan_conv_pack_weights(const float* w, const float* scale, int Cout, int Cin, int R, int S, int transposed,
                            bf16_t* out, hipStream_t stream) {
  const int rows = transposed ? Cin : Cout;
  const int Cgp = cgp_of(transposed ? Cout : Cin);
  const int rows_pad = ee_round_up(rows, 128), Kw = kw_of(R, S, Cgp);
  const long total = (long)rows_pad * Kw;
  const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
  pack_weights_kernel<<<blocks, 256, 0, stream>>>(w, scale, Cout, Cin, R, S, transposed, Cgp, rows_pad, Kw, out);
  return ee_check_launch("pack_weights");
}

long eegan_conv_pack_multi_blocks(int Cout, int Cin, int R, int S, int transposed) {
  if (!transposed) return ee_round_up(Cout, 128);
  return (long)(ee_round_up(Cin, 128) / PK_T) * R * S * ee_cdiv(pk_cgp(Cout), PK_T);
}

int eegan_conv_pack_weights_multi(const long* table, int njobs, long total_blocks, hipStream_t stream) {
  if (njobs <= 0 || total_blocks <= 0) return 0;
  pack_weights_multi_kernel<<<(unsigned)total_blocks, 256, 0, stream>>>(table, njobs);
  return ee_check_launch("pack_weights_multi");
}

long eegan_conv_fwd_workspace(const eegan_conv_desc* d) {
  ConvArgs a;
  fill_fwd(a, d);
  return part_bytes(a, a.P);
}

long eegan_conv_bwd_data_workspace(const eegan_conv_desc* d) {
  ConvArgs a;
  fill_bwdd(a, d);
  return part_bytes(a, bwdd_pc_max(d));
}

int eegan_conv_fwd(const eegan_conv_desc* d, const bf16_t* x, const bf16_t* wpack, const float* bias, int act,
                   float slope, const bf16_t* res, int ldres, const float* gamma, void* y, int y_f32, float* ws,
                   hipStream_t stream) {
  ConvArgs a;
  fill_fwd(a, d);
  a.src = x;
  a.wp = wpack;
  a.bias = bias;
  a.res = res;
  a.ldres = ldres;
  a.res_vec = res && (ldres % 4) == 0 && ((uintptr_t)res & 7) == 0;
  a.gamma = gamma;
  a.out = y;
  a.ldo = d->ldy;
  a.out_f32 = y_f32;
  a.act = act;
  a.slope = slope;
  if (a.P == 0) return 0;
  if (res && !gamma) {
    ee_set_error("conv_fwd: residual without gamma");
    return -22;
  }
  if (!ld_ok(d->ldx, x)) {
    ee_set_error("conv_fwd: input channel stride %d must be a multiple of 8 (16-B aligned rows)", d->ldx);
    return -22;
  }
  return launch_igemm<MODE_FWD>(a, a.P, ws, stream, (long)d->N * (d->H >> d->up2) * (d->W >> d->up2) * d->ldx * 2,
                                d->splitk_ctr, d->splitk_ctr_n);
}

int eegan_conv_bwd_data(const eegan_conv_desc* d, const bf16_t* dy, const bf16_t* wpackT, void* dx, int lddx,
                        int dx_f32, float* ws, hipStream_t stream) {
  return eegan_conv_bwd_data_gated(d, dy, wpackT, dx, lddx, dx_f32, nullptr, 0, 0, 0.f, ws, stream);
}

int eegan_conv_bwd_data_gated(const eegan_conv_desc* d, const bf16_t* dy, const bf16_t* wpackT, void* dx, int lddx,
                              int dx_f32, const bf16_t* gate, int ldgate, int gate_act, float gate_slope, float* ws,
                              hipStream_t stream) {
  return eegan_conv_bwd_data_ex(d, dy, wpackT, dx, lddx, dx_f32, gate, ldgate, gate_act, gate_slope, nullptr, 0, 0,
                                1.f, ws, stream);
}

int eegan_conv_bwd_data_ex(const eegan_conv_desc* d, const bf16_t* dy, const bf16_t* wpackT, void* dx, int lddx,
                           int dx_f32, const bf16_t* gate, int ldgate, int gate_act, float gate_slope,
                           const bf16_t* res, int ldres, int res_up2, float res_scale, float* ws,
                           hipStream_t stream) {
  if (d->up2) {
    ee_set_error("conv_bwd_data: up2 inputs take the hi-res gradient + sum-pool path");
    return -22;
  }
  ConvArgs a;
  fill_bwdd(a, d);
  a.src = dy;
  a.wp = wpackT;
  a.out = dx;
  a.ldo = lddx;
  a.out_f32 = dx_f32;
  a.act = ACT_NONE;
  a.gate = gate;
  a.ldgate = ldgate;
  a.gate_act = gate_act;
  a.gate_slope = gate_slope;
  a.gate_vec = gate && (ldgate % 4) == 0 && ((uintptr_t)gate & 7) == 0;
  a.res = res;
  a.ldres = ldres;
  a.res_vec = res && (ldres % 4) == 0 && ((uintptr_t)res & 7) == 0;
  a.res_up2 = res_up2;
  a.res_scale = res_scale;
  if (res_up2 && ((d->H & 1) || (d->W & 1))) {
    ee_set_error("conv_bwd_data: half-resolution residual needs an even input grid");
    return -22;
  }
  if (a.P == 0) return 0;
  if (!ld_ok(d->ldy, dy)) {
    ee_set_error("conv_bwd_data: dy channel stride %d must be a multiple of 8", d->ldy);
    return -22;
  }
  return launch_igemm<MODE_BWDD>(a, bwdd_pc_max(d), ws, stream, (long)d->N * d->Ho * d->Wo * d->ldy * 2,
                                 d->splitk_ctr, d->splitk_ctr_n);
}

static long wgrad_x_bytes(const eegan_conv_desc* d) {
  return (long)d->N * (d->H >> d->up2) * (d->W >> d->up2) * d->ldx * 2;
}
static long wgrad_dy_bytes(const eegan_conv_desc* d) { return (long)d->N * d->Ho * d->Wo * d->ldy * 2; }
// the pipelined kernel addresses its operands with 32-bit buffer offsets
// <= 16 output channels (get_image / get_mask heads, models.py:25-41) also take the
// pipelined kernels, as a 32-row tile whose rows >= Cout load zeros and are never
// stored (knob wgrad_small=0: the register-staged conv_wgrad_kernel<16, ...>)
static bool wgrad_glds_ok(const eegan_conv_desc* d) {
  return (d->K > 16 || (d->C % 8 == 0 && knob("wgrad_small", 1))) && wgrad_x_bytes(d) < 0x7fffffffL &&
         wgrad_dy_bytes(d) < 0x7fffffffL;
}

// blocks of conv_wgrad_thin_kernel for this shape, or 0 when it does not apply
static int wgrad_thin_blocks(const eegan_conv_desc* d) {
  if (!knob("thin", 1)) return 0;
  if (d->R != 3 || d->S != 3 || d->stride != 1 || d->pad_h != 1 || d->pad_w != 1 || d->up2) return 0;
  const int cg = ee_round_up(d->C, 8);
  // output channels in 8-channel groups on blockIdx.y (each group re-reads the x halo)
  if (d->K > knob("wgrad_thin_maxk", 8) || (cg != 32 && cg != 64) || d->Wo % WTH_W || d->Ho % WTH_H) return 0;
  if (wgrad_x_bytes(d) >= 0x7fffffffL || wgrad_dy_bytes(d) >= 0x7fffffffL) return 0;
  const int tiles = d->N * (d->Ho / WTH_H) * (d->Wo / WTH_W);
  if (tiles < 8) return 0;
  return ee_round_up(std::min(tiles, 512), 8);
}

// 4 x 32-pixel tiles of conv_wgrad_halo3_kernel for this shape, or 0 when it does not apply
static int wgrad_halo_tiles(const eegan_conv_desc* d) {
  if (!knob("wgrad_halo", 1) || wgrad_thin_blocks(d)) return 0;
  if (d->R != 3 || d->S != 3 || d->stride != 1 || d->pad_h != 1 || d->pad_w != 1 || d->up2) return 0;
  // (128 input channels measured behind the tile path: D256's 128-ch 64^2 75 vs 50 us)
  if ((d->C != 32 && d->C != 64) || d->K % 32 || d->Wo % 32 || d->Ho % 4 || d->Ho != d->H || d->Wo != d->W) return 0;
  if (wgrad_x_bytes(d) >= 0x7fffffffL || wgrad_dy_bytes(d) >= 0x7fffffffL) return 0;
  return d->N * (d->Ho / 4) * (d->Wo / 32);
}

static void wgrad_plan(const eegan_conv_desc* d, int& TCO, int& TK, int& nsplit, int& pps, int& K) {
  const int Cg = ee_round_up(d->C, 8);
  K = d->R * d->S * Cg;
  if (const int ht = wgrad_halo_tiles(d)) {
    // ~`wgrad_halo_blocks` blocks over the output-channel tiles, a multiple of 8 per tile (XCD-contiguous walks)
    const int co_t = d->K / 32;
    const int want = std::max(8, (d->plan == 1 ? knob("tp_wgrad_halo_blocks", 256) : knob("wgrad_halo_blocks", 512)) /
                                     co_t);
    pps = ee_cdiv(ht, std::min(want, ht));   // tiles per block
    nsplit = ee_round_up(ee_cdiv(ht, pps), 8);
    TCO = 32;
    TK = 0;
    return;
  }
  if (const int tb = wgrad_thin_blocks(d)) {
    TCO = 16;
    TK = 64;
    nsplit = tb;
    pps = 0;
    return;
  }
  TCO = d->K > 64 ? 128 : d->K > 32 ? 64 : wgrad_glds_ok(d) ? 32 : d->K > 16 ? 64 : 16;
  TK = K > 64 ? 128 : 64;
  const int P = d->N * d->Ho * d->Wo;
  const int tiles = ee_cdiv(d->K, TCO) * ee_cdiv(K, TK);
  // ~2 blocks per CU, >= 16 K-steps (512 pixels) per split: the fp32 slab
  // (nsplit x Cout x K) is written once and read once by the column reduce
  // knobs for sweeps: grid target (blocks) and minimum pixels per split
  int want = std::max(1, (d->plan == 1 ? knob("tp_wgrad_target", 256) : knob("wgrad_target", 512)) /
                            std::max(tiles, 1));
  const int maxsplit = std::max(1, ee_cdiv(P, knob("wgrad_minp", 512)));
  nsplit = std::min(want, maxsplit);
  pps = ee_round_up(ee_cdiv(P, nsplit), BK);
  nsplit = ee_cdiv(P, pps);
  // many-split grids: a split count that makes the grid a multiple of 8, so the
  // fast kernel can keep each split's k tiles on one XCD (WgradArgs::xcd_remap)
  if (nsplit >= 8 && (tiles * nsplit) % 8 && knob("wgrad_split8", 1)) {
    for (int ns = nsplit + 1; ns < nsplit + 16 && ns <= maxsplit; ++ns) {
      const int pp = ee_round_up(ee_cdiv(P, ns), BK), n2 = ee_cdiv(P, pp);
      if ((tiles * n2) % 8 == 0) {
        pps = pp;
        nsplit = n2;
        break;
      }
    }
  }
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
  if (!ld_ok(d->ldx, x) || !ld_ok(d->ldy, dy)) {
    ee_set_error("conv_bwd_weight: channel strides (%d, %d) must be multiples of 8", d->ldx, d->ldy);
    return -22;
  }
  WgradArgs w = {};
  w.x = x;
  w.dy = dy;
  w.ws = ws;
  w.N = d->N;
  w.IH = d->H;
  w.IW = d->W;
  w.ldx = d->ldx;
  w.up2 = d->up2;
  w.OH = d->Ho;
  w.OW = d->Wo;
  w.R = d->R;
  w.S = d->S;
  w.st = d->stride;
  w.ph = d->pad_h;
  w.pw = d->pad_w;
  w.Cg = ee_round_up(d->C, 8);
  w.Cin = d->C;
  w.K = K;
  w.lddy = d->ldy;
  w.Cout = d->K;
  w.P = d->N * d->Ho * d->Wo;
  w.p_per_split = pps;
  if (nsplit == 1 && w.P > 0) {
    w.dw = dw;
    w.accumulate = accumulate;
    // wgrad_stage_epi: 0 off, 1 unsplit dW only, 2 (default) also the row-major split slabs
    w.stage = d->C % 4 == 0 && ((uintptr_t)dw & 15) == 0 && knob("wgrad_stage_epi", 2);
  }
  if (w.P > 0 && wgrad_halo_tiles(d)) {
    w.dw = nullptr;   // always through the slab (one partial per block)
    const dim3 grid(nsplit, d->K / 32);
    if (d->C == 32)
      ee_launch(conv_wgrad_halo3_kernel<32>, grid, dim3(256), 0, stream, w, (int)wgrad_x_bytes(d),
                (int)wgrad_dy_bytes(d), pps);
    else
      ee_launch(conv_wgrad_halo3_kernel<64>, grid, dim3(256), 0, stream, w, (int)wgrad_x_bytes(d),
                (int)wgrad_dy_bytes(d), pps);
    const int rc = ee_check_launch("conv_wgrad(halo3)");
    if (rc) return rc;
  } else if (w.P > 0 && wgrad_thin_blocks(d)) {
    const int tiles = d->N * (d->Ho / WTH_H) * (d->Wo / WTH_W);
    const dim3 grid(nsplit, ee_cdiv(d->K, 8));
    if (w.Cg == 32)
      ee_launch(conv_wgrad_thin_kernel<2>, grid, dim3(256), 0, stream, w, (int)wgrad_x_bytes(d),
                (int)wgrad_dy_bytes(d), ee_cdiv(tiles, nsplit));
    else
      ee_launch(conv_wgrad_thin_kernel<4>, grid, dim3(256), 0, stream, w, (int)wgrad_x_bytes(d),
                (int)wgrad_dy_bytes(d), ee_cdiv(tiles, nsplit));
    const int rc = ee_check_launch("conv_wgrad(thin)");
    if (rc) return rc;
  } else if (w.P > 0) {
    // co-quad slabs where they measured ahead (K > 1024; at K <= 1024 the quad reduce has too few blocks)
    w.quad = nsplit > 1 && d->K % 4 == 0 && ((uintptr_t)ws & 15) == 0 && K > knob("wgrad_quad_mink", 1024) &&
             knob("wgrad_quad", 1);
    // split slabs through the LDS-staged epilogue too (row-major, 16-B stores) where not co-quad
    if (nsplit > 1 && !w.quad)
      w.stage = ((uintptr_t)ws & 15) == 0 && knob("wgrad_stage_epi", 2) >= 2;
    dim3 grid(ee_cdiv(K, TK), ee_cdiv(d->K, TCO), nsplit);
    // (measured ahead on the many-split shapes: 3x3 128-ch 64^2 51 -> 35 us, 4x4/s2 64->128 50 -> 32 us;
    // behind on the few-split deep layers, profiles/r03_wgrad_xcd.txt)
    w.xcd_remap = grid.x > 1 && grid.z >= 8 && ((long)grid.x * grid.y * grid.z) % 8 == 0 &&
                  knob("wgrad_xcd", 1);
    const long x_bytes = wgrad_x_bytes(d), dy_bytes = wgrad_dy_bytes(d);
#define WG(TC, TKK, WC) ee_launch(conv_wgrad_kernel<TC, TKK, WC>, grid, dim3(256), 0, stream, w)
#define WL(TC, TKK) ee_launch(conv_wgrad_glds_kernel<TC, TKK>, grid, dim3(256), 0, stream, w, x_bytes, dy_bytes)
#define WF(TC, TKK) \
  ee_launch(conv_wgrad_fast_kernel<TC, TKK, 2>, grid, dim3(256), 0, stream, w, x_bytes, dy_bytes, lw, lhw)
    const int OW = d->Wo, HW = d->Ho * d->Wo;
    const bool pow2 = OW > 0 && (OW & (OW - 1)) == 0 && (HW & (HW - 1)) == 0;
    if (wgrad_glds_ok(d) && pow2 && !d->up2 && knob("fast", 1)) {
      const int lw = __builtin_ctz(OW), lhw = __builtin_ctz(HW);
      if (TCO == 128) { if (TK == 128) WF(128, 128); else WF(128, 64); }
      else if (TCO == 64) { if (TK == 128) WF(64, 128); else WF(64, 64); }
      else { if (TK == 128) WF(32, 128); else WF(32, 64); }
    }
    else if (wgrad_glds_ok(d)) {
      if (TCO == 128) { if (TK == 128) WL(128, 128); else WL(128, 64); }
      else if (TCO == 64) { if (TK == 128) WL(64, 128); else WL(64, 64); }
      else { if (TK == 128) WL(32, 128); else WL(32, 64); }
    }
    else if (TCO == 128) { if (TK == 128) WG(128, 128, 2); else WG(128, 64, 2); }
    else if (TCO == 64) { if (TK == 128) WG(64, 128, 2); else WG(64, 64, 2); }
    else { if (TK == 128) WG(16, 128, 1); else WG(16, 64, 1); }
#undef WG
#undef WL
#undef WF
    int rc = ee_check_launch("conv_wgrad");
    if (rc || w.dw) return rc;
  } else {
    nsplit = 0;
  }
  const long cols = (long)d->K * K;
  if (w.quad) {
    const WgradMap map{K, w.Cg, d->C, d->R * d->S};
    const unsigned c4 = (unsigned)(d->K / 4);
    if (nsplit <= 8)
      ee_launch(wgrad_quad_reduce_kernel<256, 1>, dim3(ee_cdiv(K, 256), c4), dim3(256), 0, stream, ws, nsplit, cols,
                dw, accumulate, map);
    else if (nsplit <= 128)
      ee_launch(wgrad_quad_reduce_kernel<32, 8>, dim3(ee_cdiv(K, 32), c4), dim3(256), 0, stream, ws, nsplit, cols, dw,
                accumulate, map);
    else
      ee_launch(wgrad_quad_reduce_kernel<32, 32>, dim3(ee_cdiv(K, 32), c4), dim3(1024), 0, stream, ws, nsplit, cols,
                dw, accumulate, map);
  } else
    launch_colsum<float, float>(ws, nsplit, cols, cols, 0, dw, 0, 1, accumulate, stream,
                                WgradMap{K, w.Cg, d->C, d->R * d->S});
  return ee_check_launch("wgrad_reduce");
}

}  // extern "C"
