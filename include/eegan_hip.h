/*
 * eegan_hip.h -- C ABI of libeegan_hip.so, the MI355X (gfx950) kernel library
 * behind EE-GAN's data-parallel G+D training step.
 *
 * Conventions
 *  - Activations: NHWC, bf16 stored as uint16_t, channel stride `ld`
 *    (ld == C for C < 8, else ld % 8 == 0 and ld >= round_up(C, 8)).
 *  - Parameters / statistics / losses: fp32.
 *  - Every entry point is asynchronous on the `hipStream_t` it is given,
 *    never allocates or frees (the caller owns all memory, including
 *    workspaces sized by the *_workspace queries; the eegan_peer_* region
 *    calls are the one exception, since IPC needs a whole allocation), keeps no global mutable
 *    state (safe to call concurrently from several threads/devices) and
 *    returns 0 or a negative error code; eegan_last_error() then returns a
 *    thread-local description.
 *  - "replaces" names the reference (qikizh/EE-GAN) code each entry point
 *    stands in for (file:line under the reference root).
 */
#ifndef EEGAN_HIP_H
#define EEGAN_HIP_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EEGAN_ABI_VERSION 17  /* 2: fp32 conv weights channels-last; 3: eegan_scale_dot act gate;
                                4: rectangular (local x global) DAMSM words / sentence blocks on MFMA;
                                5: GlobalAttentionGeneral (eegan_gag_*), words backward reuses the forward's prep;
                                6: device input pipeline (eegan_pipe_*);
                                7: GlobalAttentionGeneral for any source length (eegan_gag_fwd workspace);
                                8: FID leg (eegan_fid_*);
                                9: SyncBN peer-write all-reduce (eegan_peer_*);
                                10: FID generator-sample input (eegan_fid_samples);
                                11: BN forward with the finalize folded in (eegan_bnmod_fwd_fin);
                                12: ScaleAdd double backward in one pass (eegan_scale_dot_res);
                                13: split-K counters in the conv descriptor, for the in-kernel split-K finish;
                                14: per-region peer wait bound (eegan_peer_set_wait);
                                15: planner objective in the conv descriptor (eegan_conv_desc.plan);
                                16: gated ScaleAdd backward under create_graph (eegan_scale_gate);
                                17: Adam fused with the conv weight re-pack (eegan_adam_pack) */

const char* eegan_last_error(void);
int eegan_abi_version(void);

/* launch timing for the benchmark's roofline: timing events; a record on a
 * capturing stream becomes an external event-record graph node */
int eegan_event_create(hipEvent_t* ev);
int eegan_event_destroy(hipEvent_t ev);
int eegan_event_record(hipEvent_t ev, hipStream_t s);
int eegan_event_elapsed(hipEvent_t start, hipEvent_t stop, float* ms);
/* a private non-blocking stream (torch's pool streams are recycled round-robin, so two
 * torch.cuda.Stream() objects can be the same HIP stream; lanes that must stay distinct use these) */
int eegan_stream_create(hipStream_t* s, int priority);  /* 0 default, > 0 highest, < 0 lowest */
int eegan_stream_destroy(hipStream_t s);
/* arm per-dispatch timing for the next op on this host thread: its first
 * (up to two) kernels launch through hipExtLaunchKernel with (start_i, stop_i),
 * stamped at the dispatch's begin and end; disarm returns how many were used */
int eegan_timing_arm(hipEvent_t start0, hipEvent_t stop0, hipEvent_t start1, hipEvent_t stop1);
int eegan_timing_disarm(int* kernels_timed);

/* ------------------------------------------------------------------ conv --
 * replaces: every nn.Conv2d / nn.Linear forward+backward of models.py:14-403
 * (conv1x1/conv3x3/conv4x4 helpers 14-23, SAGB c1/c2/c_sc 97-103, Cum_Block
 * 132-137, get_image/get_mask 25-41, resD 267-274, DiscSent/DiscCond 296-321,
 * Dis* conv_img 343/361/381) and DAMSM.py CNN_ENCODER's Inception convs.
 * A Linear(in, out) is the 1x1 conv over an (N,1,1,in) tensor. */
typedef struct eegan_conv_desc {
  int N, H, W, C, ldx;  /* input; (H, W) is the LOGICAL grid (physical H/2 x W/2 when up2) */
  int K, R, S;          /* output channels, kernel height/width */
  int stride, pad_h, pad_w;
  int up2;              /* 1: input is nearest-2x upsampled on the fly (F.interpolate(x, 2)) */
  int Ho, Wo, ldy;      /* output grid and channel stride */
  /* optional (ABI 13): zero-initialised int counters the forward / data-gradient kernels may use to
   * finish a split-K launch inside the kernel (the last-arriving split of each output tile sums the
   * partials in split order and applies the epilogue -- no separate reduce launch); every counter
   * used is zero again when the launch completes.  Launches that may run concurrently need disjoint
   * arrays (one per stream).  NULL: split-K launches reduce in a second kernel. */
  int* splitk_ctr;
  int splitk_ctr_n;
  /* optional (ABI 15): the planner's objective for this call.  0: latency -- split K until the grid
   * covers the chip twice (512 workgroups), smaller pixel tiles for small grids (a conv on the step's
   * critical chain); 1: throughput -- a grid target of 128 workgroups (128 / 256 for weight
   * gradients), so larger tiles and no split-K partials or reduce launch wherever the grid already
   * reaches it (a conv on a stream that runs beside others and is not on the critical chain: fewer
   * CU-cycles and HBM bytes per FLOP).  Same arithmetic either way except the split-K summation
   * order.  The workspace queries honour it: query and launch with the same descriptor. */
  int plan;
} eegan_conv_desc;

/* elements of the packed bf16 weight image (rows padded to 128, each tap's channel run to 32) */
long eegan_conv_packed_elems(int Cout, int Cin, int R, int S, int transposed);
/* fp32 conv weights are channels-last: W[Cout][R][S][Cin] (torch.channels_last storage of the
 * (Cout, Cin, R, S) nn.Conv2d weight).  W (x optional per-Cout scale) -> packed bf16.
 * transposed=0: forward image [Cout][R][S][Cin_32]; 1: bwd-data image [Cin][R][S][Cout_32] */
int eegan_conv_pack_weights(const float* w, const float* scale, int Cout, int Cin, int R, int S,
                            int transposed, uint16_t* out, hipStream_t stream);
/* every conv weight of one optimizer re-packed in ONE launch after its Adam step
 * (the per-weight packs above, batched).  `table` is device memory, int64:
 * njobs rows {w, scale, out, Cout, Cin, R, S, transposed} followed by njobs+1
 * prefix offsets of the blocks each job takes (eegan_conv_pack_multi_blocks);
 * `total_blocks` = the last offset. */
long eegan_conv_pack_multi_blocks(int Cout, int Cin, int R, int S, int transposed);
int eegan_conv_pack_weights_multi(const long* table, int njobs, long total_blocks, hipStream_t s);
/* split-K partial-slab bytes the call needs (0 when the grid is large enough) */
long eegan_conv_fwd_workspace(const eegan_conv_desc* d);
long eegan_conv_bwd_data_workspace(const eegan_conv_desc* d);
/* y = res + gamma * act(conv(x, W) + bias)   (res/gamma optional; act: 0 none,1 relu,2 lrelu,3 tanh,4 sigmoid)
 * x channel stride must be a multiple of 8 (16-byte rows) */
int eegan_conv_fwd(const eegan_conv_desc* d, const uint16_t* x, const uint16_t* wpack, const float* bias,
                   int act, float slope, const uint16_t* res, int ldres, const float* gamma, void* y,
                   int y_f32, float* ws, hipStream_t stream);
/* dx (logical input grid, channel stride lddx) = conv_transpose(dy, W); stride-s passes run as
 * s*s parity classes that visit only their valid taps */
int eegan_conv_bwd_data(const eegan_conv_desc* d, const uint16_t* dy, const uint16_t* wpackT, void* dx,
                        int lddx, int dx_f32, float* ws, hipStream_t stream);
/* the same, times act'(gate) of activation gate_act expressed through its output `gate` (the activated
 * conv input, channel stride ldgate): the producing layer's activation backward (models.py:262-288
 * LeakyReLU, Inception BasicConv2d ReLU) fused into this data gradient */
int eegan_conv_bwd_data_gated(const eegan_conv_desc* d, const uint16_t* dy, const uint16_t* wpackT, void* dx,
                              int lddx, int dx_f32, const uint16_t* gate, int ldgate, int gate_act,
                              float gate_slope, float* ws, hipStream_t stream);
/* gated (gate may be NULL) plus a residual: dx = res_scale * res + [gated] conv_transpose(dy, W); res_up2
 * reads res at half resolution (pixel (y/2, x/2)): with res_scale 1/4 the 2x2 average pool's adjoint, so
 * resD's shortcut (avg_pool2d, models.py:280-285) and first residual conv (267) share one input gradient */
int eegan_conv_bwd_data_ex(const eegan_conv_desc* d, const uint16_t* dy, const uint16_t* wpackT, void* dx,
                           int lddx, int dx_f32, const uint16_t* gate, int ldgate, int gate_act, float gate_slope,
                           const uint16_t* res, int ldres, int res_up2, float res_scale, float* ws,
                           hipStream_t stream);
/* dW[Cout][R][S][Cin] (fp32, channels-last like W) = sum_pixels dy x im2col(x); split-K slabs in ws */
long eegan_conv_wgrad_workspace(const eegan_conv_desc* d);
int eegan_conv_bwd_weight(const eegan_conv_desc* d, const uint16_t* x, const uint16_t* dy, float* ws, float* dw,
                          int accumulate, hipStream_t stream);

/* ----------------------------------------------------- SyncBN / modulation --
 * replaces: sync_batchnorm/batchnorm.py:48-125 (statistics, running buffers,
 * clamp(var,eps) multi-replica formula), models.py:69-86 (affine_ssa) and the
 * ReLU/LeakyReLU after every BN (models.py:28,38,115,118); the nearest-2x
 * upsample of models.py:219 is folded in via up2. */
long eegan_bn_stats_workspace(long P, int C);
/* sums[0..C) = sum x, sums[C..2C) = sum x^2 (fp64) over P pixels */
int eegan_bn_stats(const uint16_t* x, long P, int C, int ld, float* ws, double* sums, hipStream_t stream);
/* stats[3C] = (mean, inv_std, var-grad flag) of sums*sum_scale over `count` elements
 * (sum_scale = 4 when the normalised tensor is the nearest-2x upsample of x);
 * updates running buffers (nullable) */
int eegan_bn_finalize(const double* sums, int C, double count, double sum_scale, float eps, float momentum,
                      int clamp_mode, float* running_mean, float* running_var, float* stats, hipStream_t stream);

typedef struct eegan_bnmod_desc {
  const uint16_t* x;  /* input (physical grid N x H x W, channel stride ldx) */
  int N, H, W, C, ldx;
  int up2;            /* output grid is (2H, 2W) */
  const float* stats; /* from eegan_bn_finalize */
  int mode;           /* 0: affine BN  t = act(xhat*w + b)   1: affine_ssa t = act((gam*m+1)*xhat + bet*m) */
  const float* w;     /* [C] (mode 0, nullable) */
  const float* b;     /* [C] (mode 0, nullable) */
  const float* gam;   /* [N][C] (mode 1) */
  const float* bet;   /* [N][C] (mode 1) */
  const float* mask;  /* [N][Ho*Wo] fp32 (mode 1) */
  int act;            /* 0 none, 1 relu, 2 lrelu */
  float slope;
} eegan_bnmod_desc;

int eegan_bnmod_fwd(const eegan_bnmod_desc* d, uint16_t* y, int ldy, hipStream_t stream);
/* eegan_bn_finalize + eegan_bnmod_fwd in one launch (replaces the pair at sync_batchnorm/batchnorm.py:
 * 48-78 + models.py:69-86): the statistics are computed from sums[2C] (same arguments as
 * eegan_bn_finalize) and written to d->stats (with the running statistics) for the backward */
int eegan_bnmod_fwd_fin(const eegan_bnmod_desc* d, const double* sums, double count, double sum_scale, float eps,
                        float momentum, int clamp_mode, float* running_mean, float* running_var, uint16_t* y,
                        int ldy, hipStream_t stream);
long eegan_bnmod_bwd_workspace(const eegan_bnmod_desc* d);
/* pass 1: dparam0/1 = (dw, db) [C] (mode 0) or (dgam, dbet) [N][C] (mode 1); dmask [N][Ho*Wo];
 * chan[2C] (fp64) = (sum dxhat, sum dxhat*xhat) -- all-reduce these across ranks for SyncBN */
int eegan_bnmod_bwd(const eegan_bnmod_desc* d, const uint16_t* dt, int lddt, float* ws, float* dparam0,
                    float* dparam1, float* dmask, double* chan, hipStream_t stream);
/* pass 2: dx on the physical input grid (2x2 children summed when up2) */
int eegan_bnmod_bwd_dx(const eegan_bnmod_desc* d, const uint16_t* dt, int lddt, const double* chan, double count,
                       uint16_t* dx, int lddx, hipStream_t stream);

/* ------------------------------------------------------------ elementwise --
 * replaces: activation backward (models.py:28-30,38,115-118,269-271),
 * F.avg_pool2d(x,2) (models.py:284), nearest upsample (models.py:134,219),
 * shortcut + gamma*residual (models.py:122,142,278), cond.repeat+cat
 * (models.py:302-304,327-331), F.interpolate bilinear (models.py:220,
 * DAMSM.py:173), sigmoid (models.py:221,232), Inception pools (DAMSM.py:181-218),
 * Gen.fc view (models.py:228-230). */
int eegan_act_bwd(const uint16_t* dy, int lddy, const uint16_t* y, int ldy, long P, int C, int act, float slope,
                  uint16_t* dx, int lddx, hipStream_t s);
int eegan_scale_add(const uint16_t* x, int ldx, const uint16_t* y, int ldy, const float* gamma, float alpha, long P,
                    int C, uint16_t* out, int ldo, hipStream_t s);
/* out[:, c0_i : c0_i + Cs[i]] = parts[i] for n <= 8 NHWC parts of P pixels (channel counts, strides multiples
 * of 8): the Inception branch concat (torchvision Inception3 torch.cat(outputs, 1)) in one launch */
int eegan_cat_channels(const uint16_t* const* parts, const int* lds, const int* Cs, int n, long P, uint16_t* out,
                       int ldo, hipStream_t s);
/* ScaleAdd backward (models.py:122,142,278 first-order): out = alpha*gamma*g [* act'(h)] and
 * dot_out (+)= <g, h>, one pass over g; act != 0 folds the backward of the activation that produced h
 * (resD's second LeakyReLU); ws = eegan_dot_workspace() bytes */
int eegan_scale_dot(const uint16_t* g, int ldg, const uint16_t* h, int ldh, const float* gamma, float alpha, long P,
                    int C, uint16_t* out, int ldo, float* ws, float* dot_out, int accumulate, int act, float slope,
                    hipStream_t stream);
/* The gradient penalty's double backward through ScaleAdd (models.py:278 under create_graph): out = r +
 * alpha*gamma*g (the two gradients of the first backward's (g, gamma*g) summed) and dot_out (+)= <g, h>
 * (gamma's gradient, h = the first backward's g), one pass; ws = eegan_dot_workspace() bytes */
int eegan_scale_dot_res(const uint16_t* g, int ldg, const uint16_t* h, int ldh, const float* gamma, float alpha, long P,
                        int C, const uint16_t* r, int ldr, uint16_t* out, int ldo, float* ws, float* dot_out,
                        int accumulate, hipStream_t stream);
/* ScaleAdd backward with the residual branch's activation folded in, under create_graph (the gradient
 * penalty through resD, models.py:270-278; ABI 16): out = r + alpha*gamma*act'(q)*a with q the activation
 * output that gates (r optional) and, with dot_out, dot_out (+)= <act'(q)*a, b>; first backward:
 * a = g, q = h (gamma*g*act'(h), no dot); second backward: a = gg_h, q = h, r = gg_res, b = g (gamma's
 * gradient).  ws = eegan_dot_workspace() bytes (unused without dot_out) */
int eegan_scale_gate(const uint16_t* a, int lda, const uint16_t* q, int ldq, int act, float slope, const float* gamma,
                     float alpha, long P, int C, const uint16_t* r, int ldr, const uint16_t* b, int ldb, uint16_t* out,
                     int ldo, float* ws, float* dot_out, int accumulate, hipStream_t s);
long eegan_dot_workspace(void);
int eegan_dot(const uint16_t* x, int ldx, const uint16_t* y, int ldy, long P, int C, float scale, float* ws,
              float* out, int accumulate, hipStream_t s);
long eegan_chansum_workspace(long P, int C);
int eegan_chansum(const uint16_t* x, int ld, long P, int C, float* ws, float* out, int accumulate, hipStream_t s);
int eegan_avgpool2(const uint16_t* x, int N, int H, int W, int C, int ld, uint16_t* y, int ldy, hipStream_t s);
int eegan_upsample2(const uint16_t* x, int N, int H, int W, int C, int ld, float scale, uint16_t* y, int ldy,
                    hipStream_t s);
int eegan_sumpool2(const uint16_t* x, int N, int H, int W, int C, int ld, uint16_t* y, int ldy, hipStream_t s);
int eegan_cat_tile(const uint16_t* feat, int ldf, const float* cond, int N, int HW, int C, int E, uint16_t* out,
                   int ldo, hipStream_t s);
int eegan_cat_tile_bwd(const uint16_t* dout, int ldo, int N, int HW, int C, int E, uint16_t* dfeat, int ldf,
                       float* dcond, hipStream_t s);
int eegan_bilinear(const void* x, int x_f32, int N, int H, int W, int C, int ld, int Ho, int Wo, int align_corners,
                   int post, void* y, int y_f32, int ldy, hipStream_t s);
int eegan_bilinear_bwd(const void* dy, int dy_f32, const void* y, int y_f32, int lddy, int N, int H, int W, int C,
                       int Ho, int Wo, int align_corners, int post, float* dx32, hipStream_t s);
int eegan_convert(const float* x, long P, int C, void* y, int y_f32, int ldy, hipStream_t s);
int eegan_nchw_to_nhwc(const float* x, int N, int C, int HW, uint16_t* y, int ldy, hipStream_t s);
int eegan_nhwc_to_nchw(const uint16_t* x, int ldx, int N, int C, int HW, float* y, hipStream_t s);
int eegan_fc_to_nhwc(const void* x, int x_f32, int N, int C, int HW, uint16_t* y, int ldy, hipStream_t s);
int eegan_nhwc_to_fc(const uint16_t* y, int ldy, int N, int C, int HW, void* x, int x_f32, hipStream_t s);
int eegan_maxpool3s2(const uint16_t* x, int N, int H, int W, int C, int ld, uint16_t* y, int ldy, uint8_t* arg,
                     hipStream_t s);
int eegan_maxpool3s2_bwd(const uint16_t* dy, int lddy, const uint8_t* arg, int N, int H, int W, int C, uint16_t* dx,
                         int lddx, hipStream_t s);
int eegan_avgpool3s1(const uint16_t* x, int N, int H, int W, int C, int ld, uint16_t* y, int ldy, hipStream_t s);
int eegan_global_avgpool(const uint16_t* x, int ld, int N, int HW, int C, void* y, int y_f32, hipStream_t s);
int eegan_global_avgpool_bwd(const void* dy, int dy_f32, int N, int HW, int C, uint16_t* dx, int lddx, hipStream_t s);
int eegan_fill_f32(float* x, long n, float v, hipStream_t s);
/* *slot = the device's 100 MHz wall clock when the stream reaches this point (a one-thread kernel, so it
 * can sit in a captured graph; diagnostics: tools/stamp_phases.py) */
int eegan_stamp(unsigned long long* slot, hipStream_t s);

/* ------------------------------------------------------------------ linear --
 * replaces: nn.Linear of models.py:51-60,150-152,188,321 and DAMSM.py:163 (fp32) */
int eegan_gemm_f32(const float* A, long sai, long sak, const float* B, long sbk, long sbj, float* C, long ldc, int M,
                   int N, int K, const float* bias, int act, float alpha, float beta, hipStream_t s);
int eegan_colsum_f32(const float* X, long ld, int M, int N, float* out, int accumulate, hipStream_t s);
/* n independent eegan_gemm_f32 problems in ceil(n / 32) launches; `gate` (optional, row stride ldg)
 * multiplies each result by act'(gate) of activation gate_act (e.g. dh = (dy W2) * relu'(h)).
 * replaces: the 28 affine_ssa fc_gamma / fc_beta MLPs of models.py:51-60 batched per step */
typedef struct {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  const float* gate;
  long sai, sak, sbk, sbj, ldc, ldg;
  int M, N, K, act, gate_act;
  float alpha, beta;
} eegan_gemm_desc;
int eegan_gemm_f32_grouped(const eegan_gemm_desc* descs, int n, hipStream_t s);
int eegan_act_bwd_f32(const float* dy, const float* y, long n, int act, float slope, float* dx, hipStream_t s);

/* ------------------------------------------------------------------ losses --
 * replaces: miscc/DAMSM_losses.py:17-63 (cosine_similarity, func_attention),
 * 233-342 (sent_loss, words_loss); train.py:99-103, 336-417; models.py:155-180 */
/* Word-level DAMSM similarity (csrc/damsm.hip; replaces DAMSM_losses.py:17-63 and the per-caption loop of
 * words_loss, 272-331): sim[j][i] = gamma3 * log sum_k exp(gamma2 cos(word_ik, attn-context_jk)) for every
 * (image j < n_img, caption i < n_txt) -- a data-parallel rank passes its own images and ALL ranks' captions
 * (B_local x B_global block).  regions fp32 [n_img][289][256] (16-B aligned), words fp32 [n_txt][256][T]
 * (T <= 32), cap_lens int64 [n_txt].  att (optional): the attention maps of the pairs (j, j + diag_off),
 * [n_img][T][289].  Workspace bytes from eegan_words_workspace (backward: 1 for the _bwd call, want_dwords:
 * dwords != NULL).  dregions [n_img][289][256] and dwords [n_txt][256][T] are overwritten, deterministically.
 * prepared = 1: ws is the (backward-sized) workspace a preceding eegan_words_sim call on the same inputs
 * prepared its operands in, so the backward skips that pass. */
long eegan_words_workspace(int n_img, int n_txt, int backward, int want_dwords);
int eegan_words_sim(const float* regions, const float* words, const long* cap_lens, int n_img, int n_txt, int T,
                    int diag_off, float* sim, float* att, void* ws, hipStream_t s);
int eegan_words_sim_bwd(const float* regions, const float* words, const long* cap_lens, int n_img, int n_txt, int T,
                        const float* dsim, float* dregions, float* dwords, void* ws, int prepared, hipStream_t s);
/* loss2 = (CE(sim, labels), CE(sim^T, labels)) with same-class off-diagonal entries masked to -inf
 * (labels == NULL means arange(B), the reference's match_labels) */
int eegan_sim_ce(const float* sim, int B, const long* class_ids, const long* labels, float* loss2, hipStream_t s);
int eegan_sim_ce_bwd(const float* sim, int B, const long* class_ids, const long* labels, const float* gloss2,
                     float* dsim, hipStream_t s);
/* sentence cosine block sim[a][b] = gamma3 cos(cnn_a, rnn_b), a < na (this rank's images), b < nb (all
 * ranks' captions) (DAMSM_losses.py:246-258); nrm_ws holds na + nb floats */
int eegan_sent_sim(const float* cnn, const float* rnn, int na, int nb, int D, float* sim, hipStream_t s);
int eegan_sent_sim_bwd(const float* cnn, const float* rnn, int na, int nb, int D, const float* sim, const float* dsim,
                       float* nrm_ws, float* dcnn, float* drnn, hipStream_t s);
/* GlobalAttentionGeneral.forward (DAMSM_losses.py:65-132; defined, never called by the reference step):
 * input [B][idf][queryL] (queryL = ih*iw), context_key [B][idf][sourceL], content_value [B][cdf][sourceL],
 * mask (optional) uint8 [B][sourceL], row (b, q) masked by mask[(b*queryL + q) % B] exactly like the
 * reference's mask.repeat(queryL, 1); any sourceL (chunks of 64, online softmax statistics in
 * ws: eegan_gag_fwd_workspace bytes).  weighted_context [B][cdf][queryL], attn [B][sourceL][queryL].
 * Backward: d_weighted_context / d_attn may be NULL (no gradient); d_input [B][idf][queryL], d_key, d_value
 * overwritten; ws of eegan_gag_workspace bytes; deterministic. */
long eegan_gag_fwd_workspace(int B, int queryL);
int eegan_gag_fwd(const float* input, const float* context_key, const float* content_value, const unsigned char* mask,
                  int B, int idf, int cdf, int queryL, int sourceL, float* weighted_context, float* attn, void* ws,
                  hipStream_t s);
long eegan_gag_workspace(int B, int idf, int cdf, int queryL, int sourceL);
int eegan_gag_bwd(const float* input, const float* context_key, const float* content_value, const float* attn,
                  const float* d_weighted_context, const float* d_attn, int B, int idf, int cdf, int queryL,
                  int sourceL, float* d_input, float* d_key, float* d_value, void* ws, hipStream_t s);
/* mode 0 mean(relu(1-x)), 1 mean(relu(1+x)), 2 -mean(x), 3 mean(x) */
int eegan_dout_reduce(const float* x, int n, int mode, float* out, hipStream_t s);
int eegan_dout_reduce_bwd(const float* x, int n, int mode, const float* gout, float* dx, hipStream_t s);
int eegan_bce_logits(const float* x, const float* target, int n, float* out, hipStream_t s);
int eegan_bce_logits_bwd(const float* x, const float* target, int n, const float* gout, float* dx, hipStream_t s);
/* MA gradient penalty: out = 2 * mean_b ||[g_img_b, g_sent_b]||^6 */
long eegan_gp_loss_workspace(int B);
int eegan_gp_loss(const uint16_t* gx, int ld, int B, int HW, int C, const float* gs, int E, float* nrm2, float* out,
                  float* ws, hipStream_t s);
int eegan_gp_loss_bwd(const uint16_t* gx, int ld, int B, int HW, int C, const float* gs, int E, const float* nrm2,
                      const float* gout, uint16_t* dgx, int lddgx, float* dgs, hipStream_t s);
/* labels[i][(id_i - 1) mod ncls] = 1 (bit-exact with train.py:99-103; *err set if an id is out of range) */
int eegan_class_onehot(const long* ids, int B, int ncls, float* out, int* err, hipStream_t s);
int eegan_attr_attn(const float* q, const float* k, const float* v, int B, int L, int D, float scale, float* probs,
                    float* out, float* merged, hipStream_t s);
int eegan_attr_attn_bwd(const float* q, const float* k, const float* v, const float* probs, const float* dout, int B,
                        int L, int D, float scale, float* dq, float* dk, float* dv, hipStream_t s);

/* ------------------------------------------------------------ text encoder --
 * replaces: RNN_ENCODER.forward (DAMSM.py:88-115) in eval mode: nn.Embedding,
 * pack_padded_sequence/nn.LSTM(bidirectional)/pad_packed_sequence, with the
 * caption lengths read on the device (no cap_lens.tolist() host sync). */
int eegan_embedding(const long* ids, long n, const float* table, int E, float* out, hipStream_t s);
/* xproj [2][B][T][4H] = x W_ih^T + b_ih + b_hh per direction; whhT [2][H][4H];
 * words [B][2H][Tout] (zero padded past each length), sent [B][2H] = [h_fwd(last), h_bwd(first)] */
int eegan_lstm_bidir(const float* xproj, const float* whhT, const long* lens, int B, int T, int H, int Tout,
                     float* words, float* sent, hipStream_t s);

/* ---------------------------------------------------------- input pipeline --
 * replaces: the per-image PIL work of TextDataset.get_imgs (datasets.py:391-424) under train.py's
 * transform (train.py:269-272): Resize(304) -> RandomCrop(256) -> RandomHorizontalFlip -> Resize(64) /
 * Resize(128) -> ToTensor + Normalize(0.5, 0.5), for a batch of decoded RGB uint8 images (3 bytes per
 * pixel, bounding-box crop applied through src_off / the coefficient tables).  PIL's bilinear resample
 * bit for bit: the host supplies PIL's 22-bit fixed-point weights (eegan_hip/pipeline.py), the kernels
 * sum from 2^21, clip (>> 22) to uint8 and store the horizontal pass as uint8 before the vertical pass.
 *
 * One job per image (device memory, B entries): the horizontal pass reads source rows
 * [row0, row0 + nrows) of the bbox crop (relative to src_off) for the `crop` crop columns; hbounds
 * (xmin, count) and hcoef (hksize per column) give each crop column's support in bbox-crop columns;
 * vbounds / vcoef (vksize per row) each crop row's support in bbox-crop rows.  flip mirrors the crop.
 * scales[]: the output sizes, ascending, the last equal to `crop` (its tables unused); every smaller
 * scale is PIL's Resize of the uint8 crop with the given tables (device pointers, same for all images).
 * Outputs per scale (either may be NULL): out_f32[i] NCHW fp32 [B][3][s][s]; out_bf16[i] NHWC bf16
 * [B][s][s][ld_bf16] (channels 3.. zeroed).  crop_u8_out (optional) receives the uint8 crops
 * [B][crop][crop][3].  ws: eegan_pipe_workspace bytes. */
typedef struct {
  long src_off;   /* byte offset of the bbox crop's pixel (0, 0) in src */
  int src_stride; /* bytes per source row */
  int row0, nrows;
  int flip;
  int hcoef_off, hbound_off, hksize;
  int vcoef_off, vbound_off, vksize;
} eegan_img_job;
typedef struct {
  int size, ksize;
  const int* hcoef;
  const int* hbounds;
  const int* vcoef;
  const int* vbounds;
} eegan_scale_table;
long eegan_pipe_workspace(int B, int crop, int max_rows, int nscales, const int* scales);
int eegan_pipe_transform(const uint8_t* src, const eegan_img_job* jobs, int B, int max_rows, int crop,
                         const int* coef, const int* bounds, int nscales, const eegan_scale_table* scales,
                         float* const* out_f32, uint16_t* const* out_bf16, int ld_bf16, uint8_t* crop_u8_out,
                         void* ws, hipStream_t s);

/* ------------------------------------------------------------------- FID leg --
 * replaces: InceptionV3.forward's input handling (metrics/FID/inception.py:131-138) and the activation
 * statistics of fid_score.py:110-127 (np.mean / np.cov of the float64 pool_3 activations).
 * preprocess: x NCHW fp32 [N][3][H][W] in [0, 1] -> bilinear (align_corners=True) to Ho x Wo, then
 * x * scale3[c] + shift3[c] (host arrays of 3), written NHWC bf16 with channel stride ldy (>= 3, padding zeroed).
 * stats: act fp32 [N][D] -> mu fp64 [D], sigma fp64 [D][D] (divisor N - 1), deterministic; ws of
 * eegan_fid_stats_workspace bytes; synchronises the stream once (tile list upload). */
int eegan_fid_preprocess(const float* x, int N, int H, int W, int Ho, int Wo, const float* scale3,
                         const float* shift3, uint16_t* y, int ldy, hipStream_t s);
/* samples: the generator's 256 px images as fid_score.py sees them after test.py saved them
 * (test.py:244-304, miscc/utils.py:11-15: vutils.save_image(normalize=True, scale_each=True) -> uint8 file ->
 * PIL Resize((299, 299)) -> ToTensor, fid_score.py:106-113) and InceptionV3 renormalised them, without the file:
 * img NHWC bf16 [N][H][W][ld] -> per-image min/max normalise, uint8 quantise, PIL bilinear H x W -> Ho x Wo with
 * the host-computed 22-bit weights (hcoef/hbounds along W, vcoef/vbounds along H, PIL Resample.c layout),
 * x / 255 * scale3[c] + shift3[c] -> y NHWC bf16 [N][Ho][Wo][ldy]; u8_out (optional) [N][Ho][Wo][3] the resized
 * uint8 image.  ws: eegan_fid_samples_workspace(N, H, Wo) bytes. */
long eegan_fid_samples_workspace(int N, int H, int Wo);
int eegan_fid_samples(const uint16_t* img, int N, int H, int W, int ld, int Ho, int Wo, const int* hcoef,
                      const int* hbounds, int hksize, const int* vcoef, const int* vbounds, int vksize,
                      const float* scale3, const float* shift3, uint16_t* y, int ldy, uint8_t* u8_out, void* ws,
                      hipStream_t s);
long eegan_fid_stats_workspace(int D);
int eegan_fid_stats(const float* act, int N, int D, double* mu, double* sigma, void* ws, hipStream_t s);

/* ------------------------------------------------ SyncBN peer-write reduce --
 * replaces: the statistics exchange of _SynchronizedBatchNorm (sync_batchnorm/batchnorm.py:90-111, through
 * SyncMaster / SlavePipe of sync_batchnorm/comm.py:18-137) for ranks in separate processes: a one-shot
 * all-reduce of a small fp64 message by vector stores into every rank's IPC-mapped region, then a local
 * fixed-order sum (identical bits on every rank).  One region per rank and stream lane:
 *   region_bytes(cap)        bytes of a region holding messages of up to `cap` doubles (ranks <= 16);
 *   alloc(bytes, &base, h)   uncached device allocation, zeroed; h receives its 64-byte IPC handle;
 *   open(h, &base) / close   map / unmap a peer's region; free releases an own region;
 *   allreduce_f64(t, n, cap, rank, world, bases, s)  in-place sum of t[0..n) over the ranks; bases = host
 *                            array of `world` region pointers (own at [rank]); every wait is bounded;
 *   set_wait(own, seconds)   the bound of every wait on this region (default 30 s);
 *   status(own, reset, &timed_out)  nonzero timed_out: a wait gave up (1 + the missing rank). */
long eegan_peer_region_bytes(int cap);
int eegan_peer_alloc(long bytes, void** base, void* handle);
int eegan_peer_open(const void* handle, void** base);
int eegan_peer_close(void* base);
int eegan_peer_free(void* base);
int eegan_peer_allreduce_f64(double* t, int n, int cap, int rank, int world, void* const* bases, hipStream_t s);
int eegan_peer_set_wait(void* own, int seconds);
int eegan_peer_status(void* own, int reset, int* timed_out);

/* -------------------------------------------------------------------- adam --
 * replaces: torch.optim.Adam(betas=(0.0, 0.9)) of train.py:252-263 on one flat buffer.
 * `step` is a device double: incremented on the stream, then read for the bias
 * corrections (graph-replay safe). */
int eegan_adam(float* p, const float* g, float* m, float* v, long n, float beta1, float beta2, float lr, float eps,
               float weight_decay, double* step, hipStream_t s);
/* The same Adam step fused with the re-pack of the optimizer's conv weights (ABI 17; replaces
 * eegan_adam + eegan_conv_pack_weights_multi after each step): `table` is device memory, int64, 8 per
 * job -- conv weight {0, element offset in p, forward image or 0, data-gradient image or 0, Cout, Cin,
 * R*S, 0} (the weight channels-last [Cout][R][S][Cin], unscaled; the images as
 * eegan_conv_pack_weights writes them, created by it: padding is never rewritten) or element range
 * {1, start, len, 0, 0, 0, 0, 0} -- every element of p in exactly one job -- then njobs + 1 prefix
 * offsets of the blocks each job takes (eegan_adam_pack_blocks / eegan_adam_range_blocks).  Bit-identical
 * to eegan_adam followed by the pack. */
long eegan_adam_pack_blocks(int Cout, int Cin, int R, int S);
long eegan_adam_range_blocks(long len);
int eegan_adam_pack(float* p, const float* g, float* m, float* v, float beta1, float beta2, float lr, float eps,
                    float weight_decay, double* step, const long* table, int njobs, long total_blocks, hipStream_t s);

#ifdef __cplusplus
}
#endif
#endif /* EEGAN_HIP_H */
