/* msppo.h — the PPO minibatch loss of minesweeper/ppo.py:33-87 as two HIP passes (C ABI).
 *
 * Replaces, per minibatch, the chain of PyTorch element-wise / reduction kernels between the
 * model's outputs and the scalar loss (ppo.py:33-87: masked log-softmax, gather, clipped ratio,
 * clipped value loss, entropy, pos-weighted belief BCE, calibration MSE) and its autograd
 * backward. One wavefront per minibatch row; every sum over rows runs in a fixed order
 * (per-workgroup partials, then one workgroup), so results are deterministic.
 *
 * Element types: logits / mine logits / labels / old_logp / advantages / values / returns are
 * f32; masks are bytes (0 / 1, torch.bool storage); actions int64; the value prediction is f32,
 * bf16 or fp16 (vpred_dtype: MP_F32, MC_DTYPE_BF16 or MC_DTYPE_F16 of mscnn.h).
 */
#ifndef MSPPO_H
#define MSPPO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MP_F32 (-1)

/* Outputs of mc_ppo_loss_fwd, f32 [8] (ppo.py:33-87; ms_amd/ppo.py ppo_losses):
 *   [0] policy_loss = -mean(min(r A, clamp(r, 1 - clip_eps, 1 + clip_eps) A))      (ppo.py:36-44)
 *   [1] value_loss  = 0.5 mean(max((v - R)^2, (V + clamp(v - V, +-clip_eps_v) - R)^2))  (:46-50)
 *   [2] entropy     = mean(-sum softmax * log_softmax)                                (:52)
 *   [3] aux_bce     = sum(BCEwithLogits(lf, y, pos_weight) * valid) * world / count   (:58-77)
 *   [4] aux_calib   = sum((sigmoid(lf) - y)^2 * valid) * world / count               (:78-81)
 *   [5] loss        = [0] + vf_coef [1] - ent_coef [2] + aux_mine_weight [3] + aux_mine_calib_weight [4]  (:54, 77, 81)
 *   [6], [7]        0 */
typedef struct {
  const float* logits;         /* [M][A] policy logits (masked cells are filled with mask_fill) */
  const uint8_t* action_mask;  /* [M][A] 1 = legal action */
  const int64_t* actions;      /* [M] taken action, 0 <= a < A */
  const float* old_logp;       /* [M] */
  const float* advantages;     /* [M] */
  const float* values;         /* [M] rollout value estimates (the value clip's centre) */
  const float* returns;        /* [M] */
  const void* vpred;           /* [M] value predictions of the model, vpred_dtype */
  const float* mine;           /* [M][A] belief logits, or NULL: no belief losses ([3], [4] = 0) */
  const float* labels;         /* [M][A] mine labels 0 / 1 (with mine) */
  const uint8_t* valid;        /* [M][A] cells the belief losses count, or NULL: every cell */
  const float* counts;         /* [2] (sum labels * valid, sum valid) over the GLOBAL minibatch */
  int32_t vpred_dtype;         /* MP_F32, MC_DTYPE_BF16, MC_DTYPE_F16 */
  int32_t mine_round;          /* MP_F32: none; else the 16-bit autocast type that the reference
                                  rounds the mine logits, pos_weight and calibration sigmoid to */
  float clip_eps, clip_eps_v, vf_coef, ent_coef, aux_mine_weight, aux_mine_calib_weight;
  float mask_fill;             /* the masked_fill value: -1e9 (f32 logits) or -1e4 (16-bit logits) */
  float world;                 /* data-parallel ranks (the belief losses' count is global) */
  int64_t M;                   /* rows of this rank's minibatch */
  int32_t A;                   /* actions per row = board cells, 1 ..= 512 */
} mc_ppo_loss_args;

/* floats of workspace the two passes share (per-row softmax statistics + partial sums) */
int64_t mc_ppo_loss_workspace(int64_t M);

/* Forward: out f32 [8] as above (device memory); work keeps what the backward needs. */
int mc_ppo_loss_fwd(const mc_ppo_loss_args* a, float* out, float* work, int64_t work_floats, void* stream);

/* Backward of sum_k gout[k] out[k] (gout f32 [8] on the device, e.g. the GradScaler's scale in
 * gout[5]): dlogits f32 [M][A] (0 at masked cells), dvpred [M] in vpred_dtype, dmine f32 [M][A]
 * (with mine; rounded through the 16-bit type as autocast's casts do when mine_round is set). */
int mc_ppo_loss_bwd(const mc_ppo_loss_args* a, const float* gout, const float* work, int64_t work_floats,
                    float* dlogits, void* dvpred, float* dmine, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MSPPO_H */
