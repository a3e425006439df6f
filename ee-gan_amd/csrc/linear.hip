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

constexpr int TM = 32, TN = 64, TKK = 16;

__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* A, long sai, long sak, const float* B, long sbk,
                                                       long sbj, float* C, long ldc, int M, int N, int K,
                                                       const float* bias, int act, float alpha, float beta) {
  __shared__ float As[TKK][TM + 1];
  __shared__ float Bs[TKK][TN + 1];
  const int tx = threadIdx.x % 16, ty = threadIdx.x / 16;  // 16 x 16 threads, each 2 (i) x 4 (j)
  const int i0 = blockIdx.y * TM, j0 = blockIdx.x * TN;
  float acc[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  for (int k0 = 0; k0 < K; k0 += TKK) {
    for (int e = threadIdx.x; e < TKK * TM; e += 256) {
      const int kk = e % TKK, ii = e / TKK;
      const int gi = i0 + ii, gk = k0 + kk;
      As[kk][ii] = (gi < M && gk < K) ? A[gi * sai + gk * sak] : 0.f;
    }
    for (int e = threadIdx.x; e < TKK * TN; e += 256) {
      const int jj = e % TN, kk = e / TN;
      const int gj = j0 + jj, gk = k0 + kk;
      Bs[kk][jj] = (gj < N && gk < K) ? B[gk * sbk + gj * sbj] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < TKK; ++kk) {
      const float a0 = As[kk][ty * 2], a1 = As[kk][ty * 2 + 1];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float b = Bs[kk][tx + 16 * q];
        acc[0][q] += a0 * b;
        acc[1][q] += a1 * b;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int gi = i0 + ty * 2 + p;
    if (gi >= M) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int gj = j0 + tx + 16 * q;
      if (gj >= N) continue;
      float v = alpha * acc[p][q] + (bias ? bias[gj] : 0.f);
      v = act_fwd(v, act, 0.2f);
      float* dst = C + gi * ldc + gj;
      *dst = beta != 0.f ? beta * *dst + v : v;
    }
  }
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
  dim3 grid(ee_cdiv(N, TN), ee_cdiv(M, TM));
  gemm_f32_kernel<<<grid, 256, 0, s>>>(A, sai, sak, B, sbk, sbj, C, ldc, M, N, K, bias, act, alpha, beta);
  return ee_check_launch("gemm_f32");
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
