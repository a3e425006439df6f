// Device-side image transform of the training input pipeline.
//
// Replaces the per-image PIL work of TextDataset.get_imgs
// (reference datasets.py:391-424) under train.py's transform
// (train.py:269-272): Resize(304) -> RandomCrop(256) -> RandomHorizontalFlip
// -> Resize(64) / Resize(128) of the crop -> ToTensor + Normalize(0.5, 0.5).
//
// Resize is PIL's bilinear resample (what torchvision's Resize calls on a PIL
// image), reproduced bit for bit: a support-scaled triangle filter whose
// per-output weights the host computes exactly as PIL does (double precision,
// normalised, rounded to 22-bit fixed point) and passes in; each pass sums
// uint8 pixels x int32 weights from 2^21 and clips (v >> 22) to uint8; the
// horizontal pass runs first and its output is stored as uint8 before the
// vertical pass reads it (PIL's ImagingResampleInner order).  The crop and the
// flip only select / mirror output pixels, so only the 256 x 256 window of the
// 304-px image is computed: the horizontal pass for the 256 crop columns on
// the source rows the crop rows' vertical supports touch, the vertical pass
// for the 256 crop rows (written mirrored when flipped).  The 64 / 128 scales
// are resized from the (flipped) uint8 crop, as the reference resizes the
// transformed PIL image.  Normalisation is torch's ((x / 255) - 0.5) / 0.5 in
// fp32 (IEEE division, as ToTensor + Normalize on the CPU).
//
// Memory-bound byte work: one thread per output pixel (3 channels), images
// on blockIdx.y; no MFMA.
#include "common.h"
#include "../../include/eegan_hip.h"

namespace {

constexpr int PB = 22;  // PIL's PRECISION_BITS (32 - 8 - 2)

EE_DEV uint8_t clip8(int v) {
  if (v >= (1 << PB << 8)) return 255;
  if (v <= 0) return 0;
  return (uint8_t)(v >> PB);
}

EE_DEV float norm_u8(uint8_t u) {
  const float v = (float)u / 255.0f;  // ToTensor
  return (v - 0.5f) / 0.5f;           // Normalize((0.5,)*3, (0.5,)*3)
}

// horizontal pass of the 304-px resize, crop columns only:
// tmp[img][r][c][3] for source rows row0 + r (r < nrows), crop column c < 256
__global__ __launch_bounds__(256) void pipe_hpass_kernel(const uint8_t* __restrict__ src,
                                                        const eegan_img_job* __restrict__ jobs,
                                                        const int* __restrict__ coef, const int* __restrict__ bounds,
                                                        uint8_t* __restrict__ tmp, long tmp_img_bytes, int crop) {
  const eegan_img_job j = jobs[blockIdx.y];
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= j.nrows * crop) return;
  const int r = pix / crop, c = pix - r * crop;
  const int xmin = bounds[j.hbound_off + 2 * c], xn = bounds[j.hbound_off + 2 * c + 1];
  const int* k = coef + j.hcoef_off + c * j.hksize;
  const uint8_t* row = src + j.src_off + (long)(j.row0 + r) * j.src_stride + 3L * xmin;
  int s0 = 1 << (PB - 1), s1 = s0, s2 = s0;
  for (int x = 0; x < xn; ++x) {
    const int w = k[x];
    s0 += (int)row[3 * x] * w;
    s1 += (int)row[3 * x + 1] * w;
    s2 += (int)row[3 * x + 2] * w;
  }
  uint8_t* o = tmp + blockIdx.y * tmp_img_bytes + ((long)r * crop + c) * 3;
  o[0] = clip8(s0);
  o[1] = clip8(s1);
  o[2] = clip8(s2);
}

// vertical pass of the 304-px resize for the crop rows -> the uint8 crop
// (mirrored when flipped) and, optionally, the normalised 256-px outputs
__global__ __launch_bounds__(256) void pipe_vpass_kernel(const uint8_t* __restrict__ tmp, long tmp_img_bytes,
                                                        const eegan_img_job* __restrict__ jobs,
                                                        const int* __restrict__ coef, const int* __restrict__ bounds,
                                                        uint8_t* __restrict__ crop_u8, int crop, float* __restrict__ out_f32,
                                                        uint16_t* __restrict__ out_bf16, int ld_bf16) {
  const eegan_img_job j = jobs[blockIdx.y];
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= crop * crop) return;
  const int y = pix / crop, c = pix - y * crop;
  const int ymin = bounds[j.vbound_off + 2 * y], yn = bounds[j.vbound_off + 2 * y + 1];
  const int* k = coef + j.vcoef_off + y * j.vksize;
  const uint8_t* col = tmp + blockIdx.y * tmp_img_bytes + ((long)(ymin - j.row0) * crop + c) * 3;
  const long rs = 3L * crop;
  int s0 = 1 << (PB - 1), s1 = s0, s2 = s0;
  for (int t = 0; t < yn; ++t) {
    const int w = k[t];
    s0 += (int)col[t * rs] * w;
    s1 += (int)col[t * rs + 1] * w;
    s2 += (int)col[t * rs + 2] * w;
  }
  const uint8_t v0 = clip8(s0), v1 = clip8(s1), v2 = clip8(s2);
  const int x = j.flip ? crop - 1 - c : c;
  const long p = (long)blockIdx.y * crop * crop + (long)y * crop + x;
  uint8_t* o = crop_u8 + 3 * p;
  o[0] = v0;
  o[1] = v1;
  o[2] = v2;
  if (out_f32) {  // NCHW fp32, the reference's tensors
    const long plane = (long)crop * crop;
    float* f = out_f32 + (long)blockIdx.y * 3 * plane + (long)y * crop + x;
    f[0] = norm_u8(v0);
    f[plane] = norm_u8(v1);
    f[2 * plane] = norm_u8(v2);
  }
  if (out_bf16) {  // NHWC bf16, channel stride ld_bf16 (>= 3; padding channels zeroed)
    uint16_t* b = out_bf16 + p * ld_bf16;
    b[0] = f2bf(norm_u8(v0));
    b[1] = f2bf(norm_u8(v1));
    b[2] = f2bf(norm_u8(v2));
    for (int q = 3; q < ld_bf16; ++q) b[q] = 0;
  }
}

// Resize(s) of the uint8 crop (crop x crop -> s x s), the same coefficient
// table for every image.  HPASS: crop rows x s columns into tmp; else the
// vertical pass from tmp to the s x s outputs.
template <bool HPASS>
__global__ __launch_bounds__(256) void pipe_scale_kernel(const uint8_t* __restrict__ in, int in_w, long in_img_bytes,
                                                        const int* __restrict__ coef, const int* __restrict__ bounds,
                                                        int ksize, int out_w, int out_h, uint8_t* __restrict__ tmp,
                                                        float* __restrict__ out_f32, uint16_t* __restrict__ out_bf16,
                                                        int ld_bf16) {
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= out_w * out_h) return;
  const int y = pix / out_w, c = pix - y * out_w;
  const uint8_t* img = in + blockIdx.y * in_img_bytes;
  int s0 = 1 << (PB - 1), s1 = s0, s2 = s0;
  if (HPASS) {
    const int xmin = bounds[2 * c], xn = bounds[2 * c + 1];
    const int* k = coef + c * ksize;
    const uint8_t* row = img + ((long)y * in_w + xmin) * 3;
    for (int x = 0; x < xn; ++x) {
      const int w = k[x];
      s0 += (int)row[3 * x] * w;
      s1 += (int)row[3 * x + 1] * w;
      s2 += (int)row[3 * x + 2] * w;
    }
    uint8_t* o = tmp + (long)blockIdx.y * out_w * out_h * 3 + (long)pix * 3;
    o[0] = clip8(s0);
    o[1] = clip8(s1);
    o[2] = clip8(s2);
    return;
  }
  const int ymin = bounds[2 * y], yn = bounds[2 * y + 1];
  const int* k = coef + y * ksize;
  const uint8_t* col = img + ((long)ymin * in_w + c) * 3;
  const long rs = 3L * in_w;
  for (int t = 0; t < yn; ++t) {
    const int w = k[t];
    s0 += (int)col[t * rs] * w;
    s1 += (int)col[t * rs + 1] * w;
    s2 += (int)col[t * rs + 2] * w;
  }
  const uint8_t v0 = clip8(s0), v1 = clip8(s1), v2 = clip8(s2);
  const long plane = (long)out_w * out_h;
  if (out_f32) {
    float* f = out_f32 + (long)blockIdx.y * 3 * plane + pix;
    f[0] = norm_u8(v0);
    f[plane] = norm_u8(v1);
    f[2 * plane] = norm_u8(v2);
  }
  if (out_bf16) {
    uint16_t* b = out_bf16 + ((long)blockIdx.y * plane + pix) * ld_bf16;
    b[0] = f2bf(norm_u8(v0));
    b[1] = f2bf(norm_u8(v1));
    b[2] = f2bf(norm_u8(v2));
    for (int q = 3; q < ld_bf16; ++q) b[q] = 0;
  }
  if (tmp) {  // the uint8 image itself (tests / chaining)
    uint8_t* o = tmp + ((long)blockIdx.y * plane + pix) * 3;
    o[0] = v0;
    o[1] = v1;
    o[2] = v2;
  }
}

}  // namespace

extern "C" {

long eegan_pipe_workspace(int B, int crop, int max_rows, int nscales, const int* scales) {
  long ws = (long)B * max_rows * crop * 3;       // horizontal pass of the 304-px resize
  ws = (ws + 255) / 256 * 256;
  ws += (long)B * crop * crop * 3;                // the uint8 crop
  ws = (ws + 255) / 256 * 256;
  long mx = 0;
  for (int i = 0; i < nscales; ++i) mx = std::max(mx, (long)crop * scales[i] * 3);
  ws += (long)B * mx;                             // horizontal pass of a scale resize
  return (ws + 255) / 256 * 256;
}

int eegan_pipe_transform(const uint8_t* src, const eegan_img_job* jobs, int B, int max_rows, int crop,
                         const int* coef, const int* bounds, int nscales, const eegan_scale_table* scales,
                         float* const* out_f32, uint16_t* const* out_bf16, int ld_bf16, uint8_t* crop_u8_out,
                         void* ws, hipStream_t s) {
  if (B <= 0 || crop <= 0 || max_rows <= 0 || nscales < 1 || nscales > 4 || (out_bf16 && ld_bf16 < 3) ||
      scales[nscales - 1].size != crop) {
    ee_set_error("pipe_transform: bad sizes (B %d crop %d rows %d scales %d ld %d)", B, crop, max_rows, nscales,
                 ld_bf16);
    return -22;
  }
  uint8_t* w = (uint8_t*)ws;
  const long tmp_img = (long)max_rows * crop * 3;
  uint8_t* tmp = w;
  long off = ((long)B * tmp_img + 255) / 256 * 256;
  uint8_t* cropbuf = crop_u8_out ? crop_u8_out : w + off;
  off += ((long)B * crop * crop * 3 + 255) / 256 * 256;
  uint8_t* stmp = w + off;
  ee_launch(pipe_hpass_kernel, dim3(ee_cdiv((long)max_rows * crop, 256), B), dim3(256), 0, s, src, jobs, coef, bounds,
            tmp, tmp_img, crop);
  int rc = ee_check_launch("pipe_hpass");
  if (rc) return rc;
  // the largest scale (== crop) is written by the vertical pass itself
  const int last = nscales - 1;
  ee_launch(pipe_vpass_kernel, dim3(ee_cdiv((long)crop * crop, 256), B), dim3(256), 0, s, tmp, tmp_img, jobs, coef,
            bounds, cropbuf, crop, out_f32 ? out_f32[last] : nullptr, out_bf16 ? out_bf16[last] : nullptr, ld_bf16);
  if ((rc = ee_check_launch("pipe_vpass"))) return rc;
  for (int i = 0; i < last; ++i) {
    const eegan_scale_table& t = scales[i];
    ee_launch(pipe_scale_kernel<true>, dim3(ee_cdiv((long)crop * t.size, 256), B), dim3(256), 0, s, cropbuf, crop,
              (long)crop * crop * 3, t.hcoef, t.hbounds, t.ksize, t.size, crop, stmp, (float*)nullptr,
              (uint16_t*)nullptr, 0);
    if ((rc = ee_check_launch("pipe_scale_h"))) return rc;
    ee_launch(pipe_scale_kernel<false>, dim3(ee_cdiv((long)t.size * t.size, 256), B), dim3(256), 0, s, stmp, t.size,
              (long)crop * t.size * 3, t.vcoef, t.vbounds, t.ksize, t.size, t.size, (uint8_t*)nullptr,
              out_f32 ? out_f32[i] : nullptr, out_bf16 ? out_bf16[i] : nullptr, ld_bf16);
    if ((rc = ee_check_launch("pipe_scale_v"))) return rc;
  }
  return 0;
}

}  // extern "C"
