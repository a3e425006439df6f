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
    o[c] = f2bf(__builtin_fmaf(v, sc[c], sh[c]));
  }
  for (int c = 3; c < ldy; ++c) o[c] = 0;
}

// ---- generator samples -> Inception input (test.py:244-304 + fid_score.py:98-128)
// The reference saves every generated 256 px image with
// vutils.save_image(img, normalize=True, scale_each=True) (miscc/utils.py:11-15):
// per image x <- (clamp(x, lo, hi) - lo) * (1 / max(hi - lo, 1e-5)) with lo / hi
// the image's min / max (torchvision norm_ip, on the GPU tensor: torch's CUDA
// division by a scalar multiplies by its fp32 reciprocal), then
// uint8(clamp(x * 255 + 0.5, 0, 255)); fid_score.py reads the files back
// through PIL, Resize((299, 299)) (PIL bilinear, uint8 out) and ToTensor, and
// InceptionV3 resizes 299 -> 299 (identity) and renormalises.  Here the same
// arithmetic runs on the device without the JPEG file in between: min / max per
// image, then PIL's two fixed-point passes (host-computed 22-bit weights, the
// input pipeline's kernels' arithmetic) on the quantised pixels, written as the
// NHWC bf16 Inception input.

// per-image min / max over the 3 channels of the NHWC bf16 image (ld channels per pixel)
__global__ __launch_bounds__(1024) void fid_minmax_kernel(const uint16_t* __restrict__ img, int HW, int ld,
                                                          float* __restrict__ mm) {
  __shared__ float slo[16], shi[16];
  const uint16_t* p = img + (long)blockIdx.x * HW * ld;
  float lo = __builtin_huge_valf(), hi = -__builtin_huge_valf();
  for (int i = threadIdx.x; i < HW; i += 1024) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = bf2f(p[(long)i * ld + c]);
      lo = fminf(lo, v);
      hi = fmaxf(hi, v);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, o));
    hi = fmaxf(hi, __shfl_xor(hi, o));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) slo[w] = lo, shi[w] = hi;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 16; ++k) lo = fminf(lo, slo[k]), hi = fmaxf(hi, shi[k]);
    lo = fminf(lo, slo[0]);
    hi = fmaxf(hi, shi[0]);
    mm[2 * blockIdx.x] = lo;
    mm[2 * blockIdx.x + 1] = hi;
  }
}

// save_image's uint8 of one value (separate fp32 roundings, as torch's elementwise kernels)
#pragma clang fp contract(off)
EE_DEV int fid_q8(float v, float lo, float hi, float inv) {
  v = fminf(fmaxf(v, lo), hi);
  v = (v - lo) * inv;
  v = v * 255.f + 0.5f;
  v = fminf(fmaxf(v, 0.f), 255.f);
  return (int)v;   // .to(torch.uint8): truncation
}
#pragma clang fp contract(on)

constexpr int FID_PB = 22;  // PIL's PRECISION_BITS

EE_DEV uint8_t fid_clip8(int v) {
  if (v >= (1 << FID_PB << 8)) return 255;
  if (v <= 0) return 0;
  return (uint8_t)(v >> FID_PB);
}

EE_DEV float fid_inv(float lo, float hi) {
  const float d = (float)fmax((double)hi - (double)lo, 1e-5);   // python floats, then fp32
  return 1.f / d;
}

// horizontal PIL pass: quantised image rows (H x W) -> tmp [N][H][Wo][3] uint8
__global__ __launch_bounds__(256) void fid_samples_hpass_kernel(const uint16_t* __restrict__ img, int H, int W, int ld,
                                                                const float* __restrict__ mm, int Wo,
                                                                const int* __restrict__ coef,
                                                                const int* __restrict__ bounds, int ksize,
                                                                uint8_t* __restrict__ tmp) {
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= H * Wo) return;
  const int n = blockIdx.y;
  const int y = pix / Wo, x = pix - y * Wo;
  const float lo = mm[2 * n], hi = mm[2 * n + 1], inv = fid_inv(lo, hi);
  const int xmin = bounds[2 * x], xn = bounds[2 * x + 1];
  const int* k = coef + x * ksize;
  const uint16_t* row = img + ((long)n * H + y) * W * ld + (long)xmin * ld;
  int s0 = 1 << (FID_PB - 1), s1 = s0, s2 = s0;
  for (int t = 0; t < xn; ++t) {
    const int w = k[t];
    const uint16_t* q = row + (long)t * ld;
    s0 += fid_q8(bf2f(q[0]), lo, hi, inv) * w;
    s1 += fid_q8(bf2f(q[1]), lo, hi, inv) * w;
    s2 += fid_q8(bf2f(q[2]), lo, hi, inv) * w;
  }
  uint8_t* o = tmp + (((long)n * H + y) * Wo + x) * 3;
  o[0] = fid_clip8(s0);
  o[1] = fid_clip8(s1);
  o[2] = fid_clip8(s2);
}

// vertical PIL pass -> uint8 -> ToTensor (/ 255) -> x * scale + shift -> NHWC bf16 (optional uint8 copy)
__global__ __launch_bounds__(256) void fid_samples_vpass_kernel(const uint8_t* __restrict__ tmp, int H, int Ho, int Wo,
                                                                const int* __restrict__ coef,
                                                                const int* __restrict__ bounds, int ksize, float s0_,
                                                                float s1_, float s2_, float b0, float b1, float b2,
                                                                uint16_t* __restrict__ y, int ldy,
                                                                uint8_t* __restrict__ u8) {
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= Ho * Wo) return;
  const int n = blockIdx.y;
  const int oy = pix / Wo, x = pix - oy * Wo;
  const int ymin = bounds[2 * oy], yn = bounds[2 * oy + 1];
  const int* k = coef + oy * ksize;
  const uint8_t* col = tmp + (((long)n * H + ymin) * Wo + x) * 3;
  const long rs = 3L * Wo;
  int a0 = 1 << (FID_PB - 1), a1 = a0, a2 = a0;
  for (int t = 0; t < yn; ++t) {
    const int w = k[t];
    a0 += (int)col[t * rs] * w;
    a1 += (int)col[t * rs + 1] * w;
    a2 += (int)col[t * rs + 2] * w;
  }
  const uint8_t v[3] = {fid_clip8(a0), fid_clip8(a1), fid_clip8(a2)};
  const float sc[3] = {s0_, s1_, s2_}, sh[3] = {b0, b1, b2};
  const long p = ((long)n * Ho + oy) * Wo + x;
  uint16_t* o = y + p * ldy;
#pragma unroll
  for (int c = 0; c < 3; ++c) o[c] = f2bf(__builtin_fmaf((float)v[c] / 255.0f, sc[c], sh[c]));
  for (int c = 3; c < ldy; ++c) o[c] = 0;
  if (u8) {
    u8[3 * p] = v[0];
    u8[3 * p + 1] = v[1];
    u8[3 * p + 2] = v[2];
  }
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

long eegan_fid_samples_workspace(int N, int H, int Wo) { return 2L * N * 4 + ((long)N * H * Wo * 3 + 15) / 16 * 16; }

int eegan_fid_samples(const uint16_t* img, int N, int H, int W, int ld, int Ho, int Wo, const int* hcoef,
                      const int* hbounds, int hksize, const int* vcoef, const int* vbounds, int vksize,
                      const float* scale3, const float* shift3, uint16_t* y, int ldy, uint8_t* u8_out, void* ws,
                      hipStream_t s) {
  if (N < 1 || H < 1 || W < 1 || Ho < 1 || Wo < 1 || ld < 3 || ldy < 3 || hksize < 1 || vksize < 1) {
    ee_set_error("fid_samples: bad sizes");
    return -22;
  }
  float* mm = (float*)ws;
  uint8_t* tmp = (uint8_t*)ws + 2L * N * 4;
  ee_launch(fid_minmax_kernel, dim3(N), dim3(1024), 0, s, img, H * W, ld, mm);
  int rc = ee_check_launch("fid_minmax");
  if (rc) return rc;
  ee_launch(fid_samples_hpass_kernel, dim3((H * Wo + 255) / 256, N), dim3(256), 0, s, img, H, W, ld,
            (const float*)mm, Wo, hcoef, hbounds, hksize, tmp);
  rc = ee_check_launch("fid_samples_hpass");
  if (rc) return rc;
  ee_launch(fid_samples_vpass_kernel, dim3((Ho * Wo + 255) / 256, N), dim3(256), 0, s, (const uint8_t*)tmp, H, Ho,
            Wo, vcoef, vbounds, vksize, scale3[0], scale3[1], scale3[2], shift3[0], shift3[1], shift3[2], y, ldy,
            u8_out);
  return ee_check_launch("fid_samples_vpass");
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
