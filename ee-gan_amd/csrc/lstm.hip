// Frozen DAMSM text encoder (RNN_ENCODER, DAMSM.py:30-115) in eval mode:
// embedding gather + bidirectional single-layer LSTM over each caption's own
// length.  Replaces nn.Embedding + pack_padded_sequence + nn.LSTM +
// pad_packed_sequence (DAMSM.py:91-105) without the host sync on
// cap_lens.tolist() (DAMSM.py:94): lengths are read on the device.
//
// Input projections x_t W_ih^T + b for all t are one fp32 GEMM per direction
// (eegan_gemm_f32); this file holds the gather and the recurrence.
#include "common.h"
#include "../../include/eegan_hip.h"

namespace {

__global__ void embed_kernel(const long* ids, long n, const float* table, int E, float* out) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n * E; e += (long)gridDim.x * blockDim.x) {
    const long r = e / E;
    out[e] = table[ids[r] * E + (e % E)];
  }
}

// grid (B, 2 directions), block 4H threads (one gate row each).
// xproj: [dir][B][T][4H] (bias included); whhT: [dir][H][4H] (transposed W_hh)
// words: [B][2H][Tout] (zero-filled by the caller); sent: [B][2H]
__global__ void lstm_seq_kernel(const float* xproj, const float* whhT, const long* lens, int B, int T, int H,
                                int Tout, float* words, float* sent) {
  extern __shared__ float sh[];
  float* h = sh;            // [H]
  float* gates = sh + H;    // [4H]
  const int b = blockIdx.x, dir = blockIdx.y, r = threadIdx.x;
  const int G = 4 * H;
  int L = (int)lens[b];
  if (L > T) L = T;
  if (r < H) h[r] = 0.f;
  float c = 0.f;
  __syncthreads();
  const float* W = whhT + (long)dir * H * G;
  const float* X = xproj + ((long)dir * B + b) * T * G;
  for (int s = 0; s < L; ++s) {
    const int t = dir == 0 ? s : L - 1 - s;
    float g = X[(long)t * G + r];
    for (int k = 0; k < H; ++k) g += W[(long)k * G + r] * h[k];
    gates[r] = g;
    __syncthreads();
    if (r < H) {
      const float ig = 1.f / (1.f + __expf(-gates[r]));
      const float fg = 1.f / (1.f + __expf(-gates[H + r]));
      const float gg = tanhf(gates[2 * H + r]);
      const float og = 1.f / (1.f + __expf(-gates[3 * H + r]));
      c = fg * c + ig * gg;
      const float hv = og * tanhf(c);
      h[r] = hv;
      if (t < Tout) words[((long)b * 2 * H + dir * H + r) * Tout + t] = hv;
    }
    __syncthreads();
  }
  if (r < H) sent[(long)b * 2 * H + dir * H + r] = h[r];
}

}  // namespace

extern "C" {

int eegan_embedding(const long* ids, long n, const float* table, int E, float* out, hipStream_t s) {
  const int blocks = (int)std::max<long>(1, std::min<long>(4096, (n * E + 255) / 256));
  embed_kernel<<<blocks, 256, 0, s>>>(ids, n, table, E, out);
  return ee_check_launch("embedding");
}

int eegan_lstm_bidir(const float* xproj, const float* whhT, const long* lens, int B, int T, int H, int Tout,
                     float* words, float* sent, hipStream_t s) {
  if (4 * H > 1024) {
    ee_set_error("lstm: 4H=%d > 1024", 4 * H);
    return -22;
  }
  (void)hipMemsetAsync(words, 0, (size_t)B * 2 * H * Tout * sizeof(float), s);
  lstm_seq_kernel<<<dim3(B, 2), 4 * H, 5 * H * sizeof(float), s>>>(xproj, whhT, lens, B, T, H, Tout, words, sent);
  return ee_check_launch("lstm_bidir");
}

}  // extern "C"
