// FID leg (reference metrics/FID/inception.py:115-147, fid_score.py:110-228):
// the Inception input transform and the activation statistics on the GPU.
//
//  * eegan_fid_preprocess: InceptionV3.forward's input handling
//    (inception.py:131-138): F.upsample(bilinear, align_corners=True) of the
//    NCHW fp32 [0, 1] batch to 299 x 299, then the per-channel affine
//    x * (std_c / 0.5) + (mean_c - 0.5) / 0.5, written as the NHWC bf16
//    activation the HIP Inception trunk reads -- one pass, fp32 math.
//  * eegan_fid_stats: mu = mean of the pool_3 activations, sigma =
//    np.cov(rowvar=False) = (X - mu)^T (X - mu) / (N - 1), both fp64 (the
//    reference's pred_arr is a float64 array, fid_score.py:183,
//    calculate_statistic_one 126-127).  Column sums run in a fixed order
//    (one thread per column, rows in order), sigma tiles of 64 x 64 over the
//    upper triangle with fp64 FMAs from LDS-staged centred rows, mirrored:
//    deterministic and exactly symmetric.  The Frechet distance (scipy sqrtm,
//    fid_score.py:189-228) stays on the host as in the reference.
#include "common.h"
#include "../../include/eegan_hip.h"

namespace {

__global__ __launch_bounds__(256) void fid_preprocess_kernel(const float* __restrict__ x, int N, int H, int W, int Ho,
                                                             int Wo, float s0, float s1, float s2, float b0, float b1,
                                                             float b2, uint16_t* __restrict__ y, int ldy) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * Ho * Wo) return;
  const int ox = (int)(i % Wo);
  const long t = i / Wo;
  const int oy = (int)(t % Ho), n = (int)(t / Ho);
  // align_corners=True: src = dst * (in - 1) / (out - 1)
  const float ry = Ho > 1 ? (float)(H - 1) / (float)(Ho - 1) : 0.f;
  const float rx = Wo > 1 ? (float)(W - 1) / (float)(Wo - 1) : 0.f;
  const float fy = ry * oy, fx = rx * ox;
  const int y0 = (int)fy, x0 = (int)fx;
  const int y1 = y0 + (y0 < H - 1), x1 = x0 + (x0 < W - 1);
  const float ly = fy - y0, lx = fx - x0;
  const float hy = 1.f - ly, hx = 1.f - lx;
  uint16_t* o = y + i * ldy;
  const float sc[3] = {s0, s1, s2}, sh[3] = {b0, b1, b2};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float* p = x + ((long)n * 3 + c) * H * W;
    const float v = hy * (hx * p[(long)y0 * W + x0] + lx * p[(long)y0 * W + x1]) +
                    ly * (hx * p[(long)y1 * W + x0] + lx * p[(long)y1 * W + x1]);
    o[c] = f2bf(v * sc[c] + sh[c]);
  }
  for (int c = 3; c < ldy; ++c) o[c] = 0;
}

// mu[d] = (sum_n x[n][d]) / N, rows in order
__global__ __launch_bounds__(256) void fid_mean_kernel(const float* __restrict__ x, int N, int D,
                                                       double* __restrict__ mu) {
  const int d = blockIdx.x * 256 + threadIdx.x;
  if (d >= D) return;
  double s = 0.0;
  for (int n = 0; n < N; ++n) s += (double)x[(long)n * D + d];
  mu[d] = s / (double)N;
}

constexpr int CT = 64;  // sigma tile
constexpr int CR = 16;  // rows staged per step

// sigma tile (ti, tj), ti <= tj (upper triangle): 16 x 16 threads, 4 x 4 each
__global__ __launch_bounds__(256) void fid_cov_kernel(const float* __restrict__ x, int N, int D,
                                                      const double* __restrict__ mu, const int2* __restrict__ tiles,
                                                      double* __restrict__ sigma) {
  __shared__ double a[CR][CT], b[CR][CT];
  const int2 tl = tiles[blockIdx.x];
  const int i0 = tl.x * CT, j0 = tl.y * CT;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  double acc[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) acc[u][v] = 0.0;
  for (int n0 = 0; n0 < N; n0 += CR) {
    __syncthreads();
    for (int e = threadIdx.x; e < CR * CT; e += 256) {
      const int r = e / CT, c = e % CT, n = n0 + r;
      const int di = i0 + c, dj = j0 + c;
      a[r][c] = (n < N && di < D) ? (double)x[(long)n * D + di] - mu[di] : 0.0;
      b[r][c] = (n < N && dj < D) ? (double)x[(long)n * D + dj] - mu[dj] : 0.0;
    }
    __syncthreads();
#pragma unroll 4
    for (int r = 0; r < CR; ++r) {
      double av[4], bv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) av[u] = a[r][ty + 16 * u], bv[u] = b[r][tx + 16 * u];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] = fma(av[u], bv[v], acc[u][v]);
    }
  }
  const double inv = 1.0 / (double)(N - 1);
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = i0 + ty + 16 * u, j = j0 + tx + 16 * v;
      if (i < D && j < D) {
        const double s = acc[u][v] * inv;
        sigma[(long)i * D + j] = s;
        sigma[(long)j * D + i] = s;   // the mirrored element: the same value, computed once
      }
    }
}

}  // namespace

extern "C" {

int eegan_fid_preprocess(const float* x, int N, int H, int W, int Ho, int Wo, const float* scale3,
                         const float* shift3, uint16_t* y, int ldy, hipStream_t s) {
  if (N < 1 || H < 1 || W < 1 || Ho < 1 || Wo < 1 || ldy < 3) {
    ee_set_error("fid_preprocess: bad sizes");
    return -22;
  }
  const long n = (long)N * Ho * Wo;
  ee_launch(fid_preprocess_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, N, H, W, Ho, Wo, scale3[0],
            scale3[1], scale3[2], shift3[0], shift3[1], shift3[2], y, ldy);
  return ee_check_launch("fid_preprocess");
}

long eegan_fid_stats_workspace(int D) {
  const long t = (D + CT - 1) / CT;
  return t * (t + 1) / 2 * (long)sizeof(int2);
}

int eegan_fid_stats(const float* act, int N, int D, double* mu, double* sigma, void* ws, hipStream_t s) {
  if (N < 2 || D < 1) {
    ee_set_error("fid_stats: need N >= 2 samples and D >= 1 (N=%d D=%d)", N, D);
    return -22;
  }
  ee_launch(fid_mean_kernel, dim3((D + 255) / 256), dim3(256), 0, s, act, N, D, mu);
  int rc = ee_check_launch("fid_mean");
  if (rc) return rc;
  // upper-triangle tile list (host-built, copied with the launch's stream order)
  const int t = (D + CT - 1) / CT;
  const long nt = (long)t * (t + 1) / 2;
  int2* host = (int2*)malloc(nt * sizeof(int2));
  if (!host) {
    ee_set_error("fid_stats: host allocation");
    return -12;
  }
  long k = 0;
  for (int i = 0; i < t; ++i)
    for (int j = i; j < t; ++j) host[k++] = make_int2(i, j);
  hipError_t e = hipMemcpyAsync(ws, host, nt * sizeof(int2), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);   // the pageable source must outlive the copy
  free(host);
  if (e != hipSuccess) {
    ee_set_error("fid_stats: tile list copy: %s", hipGetErrorString(e));
    return -(int)e;
  }
  ee_launch(fid_cov_kernel, dim3((unsigned)nt), dim3(256), 0, s, act, N, D, (const double*)mu, (const int2*)ws, sigma);
  return ee_check_launch("fid_cov");
}

}  // extern "C"
