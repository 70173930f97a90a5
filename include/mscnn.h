/*
 * mscnn.h — C ABI of the fused residual-CNN kernels (libmsenv.so).
 *
 * Replaces, for the shipped CNNResidualPolicy (minesweeper/models/cnn_residual.py:7-96),
 * the PyTorch op chain conv3x3 -> GroupNorm(C/16 groups) -> [+residual] -> ReLU
 * -> [Dropout2d] of one stem / half-block (cnn_residual.py:10-26, 50-54) with
 * one MFMA implicit-GEMM kernel per sample-workgroup, and its backward.
 *
 * Layouts: activations NHWC [N][H*W][C]; conv weights [9][COUT][CIN]
 * (tap-major, tap = 3*(dy+1) + (dx+1)); per-channel params f32. COUT = 96.
 * Activations, weights and their gradients are 16-bit, of the type `dtype` names:
 * MC_DTYPE_BF16 (bf16 autocast) or MC_DTYPE_F16 (fp16 autocast, the reference's own
 * training precision, ppo.py:25); every sum and statistic is f32 either way.
 * Below, "bf16" means that 16-bit type.
 * All pointers are device pointers; `stream` is a hipStream_t (void*).
 * Returns 0 on success, MS_EINVAL / MS_EHIP (msenv.h) otherwise.
 */
#ifndef MSCNN_H
#define MSCNN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MC_DTYPE_BF16 0
#define MC_DTYPE_F16 1

/* Observation codes (the rollout buffer's layout; no reference counterpart: the reference
 * buffer stores the f32 one-hot obs, buffers.py:24-36). The obs [N][10][A] f32 of the env
 * (env.py:172-192) is one byte per cell: 0 = hidden (all planes 0), 1 + k = revealed with k
 * adjacent mines (planes 0 and 1 + k). mc_obs_encode writes the codes (u8 [N][A], may be
 * NULL; exact for every obs the env writes) and/or the stem input (16-bit [N][A][cin_pad],
 * cin_pad = 16: the 10 planes' values cast to 16 bits, channels 10..15 zero; may be NULL) of an
 * f32 obs in one pass; mc_codes_to_nhwc expands codes to the stem input. */
int mc_obs_encode(const float* obs, uint8_t* codes, uint16_t* nhwc, int64_t n, int32_t a, int32_t cin_pad,
                  int32_t dtype, void* stream);
int mc_codes_to_nhwc(const uint8_t* codes, uint16_t* nhwc, int64_t n, int32_t a, int32_t cin_pad, int32_t dtype,
                     void* stream);

/* Forward of one fused layer:
 *   y   = conv3x3(x, w) + bias                       (saved to ysave, bf16)
 *   out = relu(GN(y) * gamma + beta [+ res]) [* dmask[n][c]]
 * cin in {16, 96} (the stem's 10 input planes are zero-padded to 16).
 * res (bf16 [N][P][96]), dmask (f32 [N][96], 0 or 1/(1-p)), ysave and stats
 * (f32 [N][6][2] = mean, rstd per group) may be NULL. relu_mask (u8 [N][P][12],
 * may be NULL) receives out > 0 as bits: bit j of byte (n, p, c8) is channel 8*c8 + j;
 * the backward reads it instead of out (1/16 of the bytes). */
int mc_conv_gn_fwd(const uint16_t* x, const uint16_t* w, const float* bias, const float* gamma,
                   const float* beta, const uint16_t* res, const float* dmask, uint16_t* out,
                   uint16_t* ysave, float* stats, uint8_t* relu_mask, int32_t n, int32_t h, int32_t w_,
                   int32_t cin, float eps, int32_t dtype, void* stream);

/* Backward of one fused layer (the forward above with the same n, h, w, cin).
 * Inputs: dout = dL/d(out); out (or its relu_mask; the other may be NULL), ysave, stats
 * from the forward; x = the forward's
 * input; wT = the conv weight re-laid out as bf16 [9][cin][96] (tap, ci, co), or
 * NULL when no input gradient is wanted (the stem: its input is the observation).
 * addend (bf16 [N][P][cin], may be NULL) is added to dx (the block input's skip
 * gradient). Outputs:
 *   dy     bf16 [N][P][96]  dL/dy, the conv-output gradient (also a workspace);
 *   dz     bf16 [N][P][96]  dL/d(pre-ReLU sum) = the residual gradient, or NULL;
 *   dx     bf16 [N][P][cin] conv input gradient (+ addend), NULL iff wT is NULL;
 *   dw     f32 [9][96][cin] weight gradient (tap, co, ci);
 *   dgn    f32 [3][96]      d gamma, d beta, d bias.
 * work: f32 scratch of at least mc_conv_gn_bwd_workspace(...) floats.
 * Replaces autograd through cnn_residual.py:10-26, 50-54 (conv/GN/ReLU/Dropout2d). */
int mc_conv_gn_bwd(const uint16_t* dout, const uint16_t* out, const uint8_t* relu_mask,
                   const uint16_t* ysave, const float* stats,
                   const float* gamma, const float* dmask, const uint16_t* x, const uint16_t* wT,
                   const uint16_t* addend, uint16_t* dy, uint16_t* dz, uint16_t* dx, float* dw, float* dgn,
                   float* work, int64_t work_floats, int32_t n, int32_t h, int32_t w_, int32_t cin,
                   int32_t dtype, void* stream);

/* f32 elements of scratch mc_conv_gn_bwd needs for these sizes. */
int64_t mc_conv_gn_bwd_workspace(int32_t n, int32_t h, int32_t w_, int32_t cin);

/* Weight gradient alone (mc_conv_gn_bwd's second half): dw f32 [9][96][cin] (tap, co, ci) =
 * sum over samples and pixels of dy[n][p][co] * x[n][p + shift(tap)][ci]. work: at least
 * mc_conv_gn_bwd_workspace(n, h, w_, cin) floats. Deterministic (fixed-order partial sums). */
int mc_conv_wgrad(const uint16_t* dy, const uint16_t* x, float* dw, float* work, int64_t work_floats, int32_t n,
                  int32_t h, int32_t w_, int32_t cin, int32_t dtype, void* stream);

/* mc_conv_wgrad of a 96-channel layer whose input x is the output of a previous layer's
 * GroupNorm + ReLU (+ Dropout2d) without a residual -- a block's conv1 output, cnn_residual.py:
 * 15-18 -- recomputed from that layer's saved y instead of read: x = 16-bit(max(y * a + b, 0) * d)
 * with a = gamma * rstd, b = beta - mean * a per (sample, channel) from its stats [N][6][2] and
 * affine parameters, d = dmask [N][96] (NULL: 1), rounded as the forward epilogue rounds, so dw
 * is bitwise mc_conv_wgrad's on the saved x. The trunk forward then need not write x at all.
 * 16x16 boards (k_wgrad_c96, whatever mc_set_variant chose for mc_conv_wgrad) only; MS_EINVAL
 * otherwise. */
int mc_conv_wgrad_gn(const uint16_t* dy, const uint16_t* y, const float* stats, const float* gamma, const float* beta,
                     const float* dmask, float* dw, float* work, int64_t work_floats, int32_t n, int32_t h, int32_t w_,
                     int32_t dtype, void* stream);

/* ---------------------------------------------------------------------------------------
 * The whole residual stack in one launch per direction (csrc/mscnn_trunk.hip). Replaces,
 * for `blocks` residual blocks of 96 channels (cnn_residual.py:7-27, 55-56), the per-layer
 * launches above: a sample's activations stay in the workgroup's LDS from layer to layer,
 * and only what the backward or the caller needs is written to HBM. Boards of at most 512
 * cells. Outputs are bitwise those of the per-layer entry points on the same inputs, except the
 * forward without saves (ysave / stats / relu_mask all NULL: the rollout's) on boards of <= 256
 * cells, which runs the ping-pong kernel k_trunk_fwd_pp: the conv bias and the GroupNorm sums
 * are accumulated in another f32 order, so its outputs agree to 16-bit rounding
 * (tests/test_trunk_gpu.py PP_TOL).
 *
 * Forward: layers[0 .. 2*blocks-1] in execution order (conv1, conv2 of block 0, ...); x0
 * (16-bit [N][P][96]) is block 0's input. Per layer (host array of device pointers):
 *   w       16-bit [9][96][96] (tap, co, ci), as mc_conv_gn_fwd's;
 *   bias, gamma, beta f32 [96];
 *   dmask   f32 [N][96] Dropout2d scale after the ReLU (conv1 layers only) or NULL;
 *   out, ysave (16-bit [N][P][96]), stats (f32 [N][6][2]), relu_mask (u8 [N][P][12]):
 *           as mc_conv_gn_fwd's, each may be NULL except the last layer's out.
 * work: mc_trunk_fwd_workspace(n, h, w_) bytes, needed when a block output (the out of a
 * conv2 layer other than the last) is NULL: it then waits there as the next block's residual. */
#define MC_TRUNK_MAX_LAYERS 16
typedef struct mc_fwd_layer {
  const uint16_t* w;
  const float* bias;
  const float* gamma;
  const float* beta;
  const float* dmask;
  uint16_t* out;
  uint16_t* ysave;
  float* stats;
  uint8_t* relu_mask;
} mc_fwd_layer;
int64_t mc_trunk_fwd_workspace(int32_t n, int32_t h, int32_t w_);
int mc_trunk_fwd(const uint16_t* x0, const mc_fwd_layer* layers, int32_t nlayers, void* work, int64_t work_bytes,
                 int32_t n, int32_t h, int32_t w_, float eps, int32_t dtype, void* stream);
/* mc_trunk_fwd that also writes pooled (f32 [N][96], NULL: not computed) = the last layer's
 * output averaged over the P pixels (the value head's AdaptiveAvgPool2d(1), cnn_residual.py:
 * 65), summed in f32 on chip (k_trunk_fwd / k_trunk_fwd2: from the last output tile in LDS;
 * k_trunk_fwd_pp: from the last layer's accumulators): no second pass over the features. */
int mc_trunk_fwd_pooled(const uint16_t* x0, const mc_fwd_layer* layers, int32_t nlayers, void* work,
                        int64_t work_bytes, float* pooled, int32_t n, int32_t h, int32_t w_, float eps, int32_t dtype,
                        void* stream);

/* Backward of the stem's GroupNorm + the residual stack: layers[0] = the stem (no input
 * gradient: wT NULL), layers[2b+1] / [2b+2] = conv1 / conv2 of block b (wT = the 16-bit
 * [9][96 ci][96 co] dgrad operand). Per layer the forward's ysave, stats, relu_mask, its
 * gamma and dmask (or NULL); dy (16-bit [N][P][96], out) receives dL/dy for mc_conv_wgrad.
 * dout = dL/d(out of the last layer). dgn (f32 [nlayers][3][96], out) = d gamma, d beta,
 * d bias per layer. work: mc_trunk_bwd_workspace(nlayers, n, h, w_) bytes. */
typedef struct mc_bwd_layer {
  const uint16_t* ysave;
  const float* stats;
  const float* gamma;
  const uint8_t* relu_mask;
  const float* dmask;
  const uint16_t* wT;
  uint16_t* dy;
} mc_bwd_layer;
int64_t mc_trunk_bwd_workspace(int32_t nlayers, int32_t n, int32_t h, int32_t w_);
int mc_trunk_bwd(const uint16_t* dout, const mc_bwd_layer* layers, int32_t nlayers, float* dgn, void* work,
                 int64_t work_bytes, int32_t n, int32_t h, int32_t w_, int32_t dtype, void* stream);

/* Policy + belief heads (cnn_residual.py:57-64, 85-96): per head
 *   logit[m] = w2 . relu(W1 f[m] + b1) + b2      over rows m of f (bf16 [M][96], NHWC trunk features).
 * w1: bf16 [nh*96][96] (policy rows first, then mine), b1/w2: f32 [nh*96], b2: f32 [nh].
 * out_m == NULL computes the policy head only (nh = 1). Logits are f32 [M]. */
int mc_heads_fwd(const uint16_t* f, const uint16_t* w1, const float* b1, const float* w2, const float* b2,
                 float* out_p, float* out_m, int64_t M, int32_t dtype, void* stream);

/* Backward of both heads. dlp/dlm: f32 [M] logit gradients (dlm may be NULL = 0).
 * w1pT: ignored, may be NULL (round 2's policy W1^T copy; the kernel now reads W1 transposed
 * from its own LDS image). df (bf16 [M][96]) = policy-head input
 * gradient (the mine head reads f.detach()) + gadd[m / P] (f32 [M/P][96], may be NULL).
 * dw1: f32 [192][96], db1, dw2: f32 [192]. work: mc_heads_bwd_workspace(M) floats. */
int mc_heads_bwd(const uint16_t* f, const float* dlp, const float* dlm, const uint16_t* w1, const uint16_t* w1pT,
                 const float* b1, const float* w2, const float* gadd, int32_t P, uint16_t* df, float* dw1,
                 float* db1, float* dw2, float* work, int64_t work_floats, int64_t M, int32_t dtype,
                 void* stream);
int64_t mc_heads_bwd_workspace(int64_t M);

/* Thread-local message of the last failing mc_* call. */
const char* mc_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* MSCNN_H */
