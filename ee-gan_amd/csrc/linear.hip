// fp32 strided GEMM for the small-M Linear layers of the step:
//   C[i][j] = alpha * sum_k A(i,k) B(k,j) (+ bias[j]) -> act, (+ beta * C)
// A(i,k) = A[i*sai + k*sak], B(k,j) = B[k*sbk + j*sbj]; arbitrary strides
// cover y = x W^T, dx = dy W and dW = dy^T x without transposes.
//
// replaces: nn.Linear forward/backward of models.py:51-60 (affine_ssa
// fc_gamma/fc_beta), 150-152 (ATTR_Enhance Q/K/V), 188 (Gen.fc), 321
// (DiscCond.class_linear) and DAMSM.py:163 (emb_cnn_code).  M is the batch
// (<= a few hundred rows), so these run in fp32 (the f32 VALU rate is ample).
#include "common.h"
#include "../../include/eegan_hip.h"

namespace {

// 16x16 output tile per 256-thread block (one output per thread).  Each K
// chunk of 256 is staged into LDS with every thread issuing all its loads at
// once (the operands are tiny; these GEMMs are latency-, not throughput-bound),
// with the lane order chosen so the unit-stride axis of each operand is the
// coalesced one.
constexpr int T = 16, KC = 256;

// One 16x16 tile (i0, j0) of C = act(alpha * A B + bias) [* act'(gate)] (+ beta * C).
// `gate` (optional) multiplies by the derivative of `gate_act` expressed
// through that activation's output: dh = (dy W2) * relu'(h) in one pass.
EE_DEV void gemm_tile(float (&As)[T][KC + 1], float (&Bs)[KC][T + 1], const float* __restrict__ A, long sai,
                      long sak, const float* __restrict__ B, long sbk, long sbj, float* __restrict__ C, long ldc,
                      int M, int N, int K, const float* __restrict__ bias, int act, float alpha, float beta,
                      const float* __restrict__ gate, long ldg, int gate_act, int i0, int j0) {
  const int t = threadIdx.x, ti = t / T, tj = t % T;
  const bool a_k_fast = sak == 1, b_j_fast = sbj == 1;
  float acc = 0.f;
  for (int k0 = 0; k0 < K; k0 += KC) {
    const int kc = min(KC, K - k0);
    float av[T], bv[T];
#pragma unroll
    for (int r = 0; r < T; ++r) {
      const int e = t + 256 * r;  // 0 .. 4095 over the 16 x 256 tile
      int ii, kk;
      if (a_k_fast) { ii = e / KC; kk = e % KC; } else { kk = e / T; ii = e % T; }
      const int gi = i0 + ii;
      av[r] = (gi < M && kk < kc) ? A[gi * sai + (long)(k0 + kk) * sak] : 0.f;
      int jj, kb;
      if (b_j_fast) { kb = e / T; jj = e % T; } else { jj = e / KC; kb = e % KC; }
      const int gj = j0 + jj;
      bv[r] = (gj < N && kb < kc) ? B[(long)(k0 + kb) * sbk + gj * sbj] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < T; ++r) {
      const int e = t + 256 * r;
      if (a_k_fast) As[e / KC][e % KC] = av[r]; else As[e % T][e / T] = av[r];
      if (b_j_fast) Bs[e / T][e % T] = bv[r]; else Bs[e % KC][e / KC] = bv[r];
    }
    __syncthreads();
#pragma unroll 8
    for (int k = 0; k < kc; ++k) acc += As[ti][k] * Bs[k][tj];
    __syncthreads();
  }
  const int gi = i0 + ti, gj = j0 + tj;
  if (gi < M && gj < N) {
    float v = alpha * acc + (bias ? bias[gj] : 0.f);
    v = act_fwd(v, act, 0.2f);
    if (gate) v *= act_dgrad_from_y(gate[gi * ldg + gj], gate_act, 0.2f);
    float* dst = C + gi * ldc + gj;
    *dst = beta != 0.f ? beta * *dst + v : v;
  }
}

__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ A, long sai, long sak,
                                                       const float* __restrict__ B, long sbk, long sbj,
                                                       float* __restrict__ C, long ldc, int M, int N, int K,
                                                       const float* __restrict__ bias, int act, float alpha,
                                                       float beta) {
  __shared__ float As[T][KC + 1];
  __shared__ float Bs[KC][T + 1];
  gemm_tile(As, Bs, A, sai, sak, B, sbk, sbj, C, ldc, M, N, K, bias, act, alpha, beta, nullptr, 0, 0,
            blockIdx.y * T, blockIdx.x * T);
}

// Grouped form: up to GMAX independent small GEMMs in one launch (the 28
// affine_ssa MLPs of the generator run as 2 forward + 6 backward launches
// instead of ~200).  Descriptors travel by value in the kernel arguments;
// block b finds its GEMM through the tile prefix sums.
constexpr int GMAX = 32;
struct GemmDev {
  const float *A, *B, *bias, *gate;
  float* C;
  int sai, sak, sbk, sbj, ldc, ldg, M, N, K, act, gate_act;
  float alpha, beta;
};
struct GemmGroup {
  GemmDev d[GMAX];
  int tile0[GMAX + 1];
  int n;
};

__global__ __launch_bounds__(256) void gemm_f32_grouped_kernel(const GemmGroup grp) {
  __shared__ float As[T][KC + 1];
  __shared__ float Bs[KC][T + 1];
  const int b = blockIdx.x;
  int g = 0;
  while (g + 1 < grp.n && grp.tile0[g + 1] <= b) ++g;
  const GemmDev& d = grp.d[g];
  const int tl = b - grp.tile0[g], tn = (d.N + T - 1) / T;
  const int ti = tl / tn, tj = tl - ti * tn;
  gemm_tile(As, Bs, d.A, d.sai, d.sak, d.B, d.sbk, d.sbj, d.C, d.ldc, d.M, d.N, d.K, d.bias, d.act, d.alpha,
            d.beta, d.gate, d.ldg, d.gate_act, ti * T, tj * T);
}

// column sums: out[j] (+)= sum_i X[i*ld + j]   (Linear bias gradient)
__global__ void colsum_kernel(const float* X, long ld, int M, int N, float* out, int accumulate) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= N) return;
  float s = 0.f;
  for (int i = 0; i < M; ++i) s += X[i * ld + j];
  out[j] = accumulate ? out[j] + s : s;
}

// dx = dy * act'(y) for fp32 tensors
__global__ void act_bwd_f32_kernel(const float* dy, const float* y, long n, int act, float slope, float* dx) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x)
    dx[e] = dy[e] * act_dgrad_from_y(y[e], act, slope);
}

}  // namespace

extern "C" {

int eegan_gemm_f32(const float* A, long sai, long sak, const float* B, long sbk, long sbj, float* C, long ldc, int M,
                   int N, int K, const float* bias, int act, float alpha, float beta, hipStream_t s) {
  if (M == 0 || N == 0) return 0;
  dim3 grid(ee_cdiv(N, T), ee_cdiv(M, T));
  ee_launch(gemm_f32_kernel, grid, dim3(256), 0, s, A, sai, sak, B, sbk, sbj, C, ldc, M, N, K, bias, act, alpha, beta);
  return ee_check_launch("gemm_f32");
}

int eegan_gemm_f32_grouped(const eegan_gemm_desc* descs, int n, hipStream_t s) {
  for (int g0 = 0; g0 < n; g0 += GMAX) {
    GemmGroup grp{};
    grp.n = std::min(GMAX, n - g0);
    int tiles = 0;
    for (int i = 0; i < grp.n; ++i) {
      const eegan_gemm_desc& e = descs[g0 + i];
      const long strides[6] = {e.sai, e.sak, e.sbk, e.sbj, e.ldc, e.ldg};
      for (long v : strides)
        if (v < 0 || v > 0x7fffffffL) {
          ee_set_error("gemm_f32_grouped: stride %ld out of range", v);
          return -22;
        }
      GemmDev& d = grp.d[i];
      d = GemmDev{e.A, e.B, e.bias, e.gate, e.C, (int)e.sai, (int)e.sak, (int)e.sbk, (int)e.sbj, (int)e.ldc,
                  (int)e.ldg, e.M, e.N, e.K, e.act, e.gate_act, e.alpha, e.beta};
      grp.tile0[i] = tiles;
      tiles += ee_cdiv(std::max(e.M, 0), T) * ee_cdiv(std::max(e.N, 0), T);
    }
    grp.tile0[grp.n] = tiles;
    if (tiles == 0) continue;
    ee_launch(gemm_f32_grouped_kernel, dim3(tiles), dim3(256), 0, s, grp);
    const int rc = ee_check_launch("gemm_f32_grouped");
    if (rc) return rc;
  }
  return 0;
}

int eegan_colsum_f32(const float* X, long ld, int M, int N, float* out, int accumulate, hipStream_t s) {
  colsum_kernel<<<ee_cdiv(N, 256), 256, 0, s>>>(X, ld, M, N, out, accumulate);
  return ee_check_launch("colsum_f32");
}

int eegan_act_bwd_f32(const float* dy, const float* y, long n, int act, float slope, float* dx, hipStream_t s) {
  const int blocks = (int)std::min<long>(4096, (n + 255) / 256);
  act_bwd_f32_kernel<<<std::max(blocks, 1), 256, 0, s>>>(dy, y, n, act, slope, dx);
  return ee_check_launch("act_bwd_f32");
}

}  // extern "C"
