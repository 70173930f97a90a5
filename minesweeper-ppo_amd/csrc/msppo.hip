// msppo.hip — the PPO minibatch loss (minesweeper/ppo.py:33-87) and its backward as HIP passes
// (C ABI include/msppo.h).
//
// PyTorch runs the loss as ~40 element-wise / reduction launches over [M, A] f32 tensors
// (masked_fill, log_softmax, gather, softmax * logp, BCE, sigmoid, ...) plus their autograd
// backward, ~3 ms per 32,768-row minibatch (profiles/r05/ppo_minibatch_by_aten_op.txt). Here one
// wavefront owns a row: the row's A logits (and belief logits) sit in registers (NQ = A / 64 per
// lane), the softmax statistics are wave reductions, and the per-row terms go to fixed-order
// partial sums -- one streaming read of the row data forward, one read + the gradient writes
// backward (HBM-bound, ~4.5 KB a row each way).
//
//   k_ppo_loss_fwd  per row: x = masked logits; max, log-sum-exp, entropy; log pi(a); ratio and
//                   the clipped surrogate; the clipped value loss; the pos-weighted BCE and the
//                   calibration error of the belief logits over the valid cells. Per-row (max,
//                   log-sum, entropy) go to the workspace for the backward; per-workgroup sums of
//                   the five terms to partial rows.
//   k_ppo_loss_fin  one workgroup: the partial rows summed in a fixed order, the means / scales of
//                   ppo.py, and the weighted loss.
//   k_ppo_loss_bwd  per row: the gradient of sum_k gout[k] out[k] by the same case split as
//                   PyTorch's autograd (torch.minimum / maximum give a tie half the gradient each,
//                   clamp passes it on its closed range), in the 16-bit roundings autocast's casts
//                   apply when the reference's belief logits are 16-bit.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>

#include "../../include/msenv.h"
#include "../../include/mscnn.h"
#include "../../include/msppo.h"
#include "mscnn_common.h"

namespace {

using namespace mc;

constexpr int NTERM = 5;        // policy, value, entropy, bce, calibration sums
constexpr int PSTRIDE = 8;      // floats per partial row
constexpr int RSTRIDE = 4;      // floats per row statistics: max, log-sum, entropy, (pad)
constexpr int MAX_GRID = 2048;  // workgroups (4 rows in flight each); fixed, so sums never depend on the device
constexpr int MAX_A = 512;

inline int loss_grid(int64_t M) {
  const int64_t g = (M + 3) / 4;
  return (int)(g < MAX_GRID ? g : MAX_GRID);
}

// x rounded to the 16-bit autocast type (dt = MC_DT_*), or unchanged (dt = MP_F32)
__device__ __forceinline__ float rnd16(float x, int dt) {
  if (dt == MC_DT_BF16) return (float)(__bf16)x;
  if (dt == MC_DT_F16) return (float)(_Float16)x;
  return x;
}

__device__ __forceinline__ float ld_val(const void* p, int dt, int64_t i) {
  if (dt == MC_DT_BF16) return (float)reinterpret_cast<const __bf16*>(p)[i];
  if (dt == MC_DT_F16) return (float)reinterpret_cast<const _Float16*>(p)[i];
  return reinterpret_cast<const float*>(p)[i];
}

__device__ __forceinline__ void st_val(void* p, int dt, int64_t i, float v) {
  if (dt == MC_DT_BF16) reinterpret_cast<__bf16*>(p)[i] = (__bf16)v;
  else if (dt == MC_DT_F16) reinterpret_cast<_Float16*>(p)[i] = (_Float16)v;
  else reinterpret_cast<float*>(p)[i] = v;
}

// butterfly reductions: every lane ends with the same value (each step adds a pair in the same order)
__device__ __forceinline__ float bfly_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float bfly_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + expf(-x)); }

// pos_weight of ppo.py:70 from the global (sum labels * valid, sum valid): (neg + 1e-6) / (pos + 1e-6),
// held in the mine logits' type (ppo.py:71) when those are 16-bit
__device__ __forceinline__ float pos_weight(const mc_ppo_loss_args& a) {
  const float pos = a.counts[0], cnt = a.counts[1];
  return rnd16((cnt - pos + 1e-6f) / (pos + 1e-6f), a.mine_round);
}

struct RowPolicy {
  int64_t act;
  float lpa, ratio, adv;
};

// log pi(a) and the ratio of row r (ppo.py:38-41), from its max and log-sum
__device__ __forceinline__ RowPolicy row_policy(const mc_ppo_loss_args& a, int64_t r, float mx, float ls) {
  RowPolicy o;
  int64_t act = a.actions[r];
  act = act < 0 ? 0 : (act >= a.A ? a.A - 1 : act);
  const int64_t ja = r * a.A + act;
  const float xa = a.action_mask[ja] ? a.logits[ja] : a.mask_fill;
  o.act = act;
  o.lpa = (xa - mx) - ls;
  o.ratio = expf(o.lpa - a.old_logp[r]);
  o.adv = a.advantages[r];
  return o;
}

template <int NQ>
__global__ __launch_bounds__(256) void k_ppo_loss_fwd(mc_ppo_loss_args a, float* __restrict__ part,
                                                       float* __restrict__ rows) {
  __shared__ float sp[4][NTERM];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int A = a.A;
  const float lo = 1.0f - a.clip_eps, hi = 1.0f + a.clip_eps;
  const float pw = a.mine ? pos_weight(a) : 1.0f;
  float acc[NTERM] = {0.f, 0.f, 0.f, 0.f, 0.f};  // lane 0: this wave's running sums, rows in order
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < a.M; r += (int64_t)gridDim.x * 4) {
    const float* lr = a.logits + r * A;
    const uint8_t* mr = a.action_mask + r * A;
    float x[NQ];
    float mx = -INFINITY;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int j = lane + 64 * q;
      x[q] = -INFINITY;
      if (j < A) x[q] = mr[j] ? lr[j] : a.mask_fill;  // masked_fill(~mask, neg_inf) (ppo.py:33-36)
      mx = fmaxf(mx, x[q]);
    }
    mx = bfly_max(mx);
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (lane + 64 * q < A) s += expf(x[q] - mx);
    const float ls = logf(bfly_sum(s));
    float h = 0.f;  // entropy -sum p log p (ppo.py:52)
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (lane + 64 * q < A) {
        const float lp = (x[q] - mx) - ls;
        h -= expf(lp) * lp;
      }
    h = bfly_sum(h);
    const RowPolicy po = row_policy(a, r, mx, ls);
    const float s1 = po.ratio * po.adv, s2 = fminf(fmaxf(po.ratio, lo), hi) * po.adv;  // ppo.py:42-44
    const float vp = ld_val(a.vpred, a.vpred_dtype, r), V = a.values[r], R = a.returns[r];
    const float vc = V + fminf(fmaxf(vp - V, -a.clip_eps_v), a.clip_eps_v);  // ppo.py:46-50
    const float v1 = (vp - R) * (vp - R), v2 = (vc - R) * (vc - R);
    float bce = 0.f, cal = 0.f;
    if (a.mine) {  // ppo.py:58-81 over the valid cells; the count and pos_weight are global
      const float* lm = a.mine + r * A;
      const float* yr = a.labels + r * A;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int j = lane + 64 * q;
        if (j < A && (!a.valid || a.valid[r * A + j])) {
          const float y = yr[j], lf = rnd16(lm[j], a.mine_round);
          const float lsig = fminf(lf, 0.f) - log1pf(expf(-fabsf(lf)));  // log sigmoid(lf)
          bce += (1.f - y) * lf - lsig * ((pw - 1.f) * y + 1.f);
          const float d = rnd16(sigmoidf(lf), a.mine_round) - y;
          cal += d * d;
        }
      }
      bce = bfly_sum(bce);
      cal = bfly_sum(cal);
    }
    if (lane == 0) {
      acc[0] += -fminf(s1, s2);
      acc[1] += fmaxf(v1, v2);
      acc[2] += h;
      acc[3] += bce;
      acc[4] += cal;
      float* rs = rows + r * RSTRIDE;
      rs[0] = mx;
      rs[1] = ls;
      rs[2] = h;
    }
  }
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < NTERM; ++k) sp[wave][k] = acc[k];
  __syncthreads();
  if (threadIdx.x < PSTRIDE)
    part[(size_t)blockIdx.x * PSTRIDE + threadIdx.x] =
        threadIdx.x < NTERM ? (sp[0][threadIdx.x] + sp[1][threadIdx.x]) + (sp[2][threadIdx.x] + sp[3][threadIdx.x]) : 0.f;
}

__global__ __launch_bounds__(256) void k_ppo_loss_fin(mc_ppo_loss_args a, const float* __restrict__ part, int G,
                                                      float* __restrict__ out) {
  __shared__ float sm[NTERM][256];
  float s[NTERM] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int g = threadIdx.x; g < G; g += 256)
#pragma unroll
    for (int k = 0; k < NTERM; ++k) s[k] += part[(size_t)g * PSTRIDE + k];
#pragma unroll
  for (int k = 0; k < NTERM; ++k) sm[k][threadIdx.x] = s[k];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
#pragma unroll
      for (int k = 0; k < NTERM; ++k) sm[k][threadIdx.x] += sm[k][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float inv_m = 1.0f / (float)a.M;  // mean = sum * (1 / M)
    const float pol = sm[0][0] * inv_m, val = 0.5f * (sm[1][0] * inv_m), ent = sm[2][0] * inv_m;
    float bce = 0.f, cal = 0.f;
    if (a.mine) {
      const float scale = a.world / fmaxf(a.counts[1], 1.0f);  // empty valid set -> 0 (ppo.py:82-87)
      bce = sm[3][0] * scale;
      cal = sm[4][0] * scale;
    }
    float loss = pol + a.vf_coef * val - a.ent_coef * ent;  // ppo.py:54, 77, 81 in that order
    if (a.mine && a.aux_mine_weight > 0.f) loss = loss + a.aux_mine_weight * bce;
    if (a.mine && a.aux_mine_calib_weight > 0.f) loss = loss + a.aux_mine_calib_weight * cal;
    out[0] = pol;
    out[1] = val;
    out[2] = ent;
    out[3] = bce;
    out[4] = cal;
    out[5] = loss;
    out[6] = 0.f;
    out[7] = 0.f;
  }
}

template <int NQ>
__global__ __launch_bounds__(256) void k_ppo_loss_bwd(mc_ppo_loss_args a, const float* __restrict__ gout,
                                                       const float* __restrict__ rows, float* __restrict__ dlogits,
                                                       void* __restrict__ dvpred, float* __restrict__ dmine) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int A = a.A;
  const float lo = 1.0f - a.clip_eps, hi = 1.0f + a.clip_eps;
  const float inv_m = 1.0f / (float)a.M;
  // d loss / d out[k] folded into each term's coefficient (out[5] is the weighted sum of out[0..4])
  const float g5 = gout[5];
  const float c_pol = gout[0] + g5, c_val = gout[1] + g5 * a.vf_coef, c_ent = gout[2] - g5 * a.ent_coef;
  const float c_bce = gout[3] + (a.aux_mine_weight > 0.f ? g5 * a.aux_mine_weight : 0.f);
  const float c_cal = gout[4] + (a.aux_mine_calib_weight > 0.f ? g5 * a.aux_mine_calib_weight : 0.f);
  const float pw = a.mine ? pos_weight(a) : 1.0f;
  const float scale = a.mine ? a.world / fmaxf(a.counts[1], 1.0f) : 0.f;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < a.M; r += (int64_t)gridDim.x * 4) {
    const float* rs = rows + r * RSTRIDE;
    const float mx = rs[0], ls = rs[1], h = rs[2];
    const RowPolicy po = row_policy(a, r, mx, ls);
    // -mean(minimum(s1, s2)): the tie (ratio inside the clip range) gives each side half; s2's
    // clamp passes its half only on [lo, hi]
    const float s1 = po.ratio * po.adv, s2 = fminf(fmaxf(po.ratio, lo), hi) * po.adv;
    const float inr = (po.ratio >= lo && po.ratio <= hi) ? 1.f : 0.f;
    const float w = s1 < s2 ? 1.f : (s1 > s2 ? inr : 0.5f * (1.f + inr));
    const float G = -c_pol * inv_m * po.adv * w * po.ratio;  // d loss / d log pi(a)
    const float E = c_ent * inv_m;                           // d loss / d H_row
    const float* lr = a.logits + r * A;
    const uint8_t* mr = a.action_mask + r * A;
    float* dl = dlogits + r * A;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int j = lane + 64 * q;
      if (j < A) {
        float d = 0.f;  // masked_fill's backward: 0 at masked cells
        if (mr[j]) {
          const float lp = (lr[j] - mx) - ls, p = expf(lp);
          // log_softmax: G (delta_ja - p_j); entropy: dH/dx_j = -p_j (log p_j + H)
          d = (j == po.act ? G : 0.f) - G * p - E * (p * (lp + h));
        }
        dl[j] = d;
      }
    }
    if (lane == 0) {  // 0.5 mean(maximum(v1, v2)); the clamp passes on [-clip_v, clip_v]
      const float vp = ld_val(a.vpred, a.vpred_dtype, r), V = a.values[r], R = a.returns[r];
      const float dvv = vp - V;
      const float vc = V + fminf(fmaxf(dvv, -a.clip_eps_v), a.clip_eps_v);
      const float v1 = (vp - R) * (vp - R), v2 = (vc - R) * (vc - R);
      const float d1 = 2.f * (vp - R), d2 = (dvv >= -a.clip_eps_v && dvv <= a.clip_eps_v) ? 2.f * (vc - R) : 0.f;
      const float dv = v1 > v2 ? d1 : (v1 < v2 ? d2 : 0.5f * (d1 + d2));
      st_val(dvpred, a.vpred_dtype, r, c_val * 0.5f * inv_m * dv);
    }
    if (a.mine) {
      const float* lm = a.mine + r * A;
      const float* yr = a.labels + r * A;
      float* dm = dmine + r * A;
      const int mr16 = a.mine_round;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int j = lane + 64 * q;
        if (j < A) {
          const float vm = (!a.valid || a.valid[r * A + j]) ? 1.f : 0.f;
          const float y = yr[j], lf = rnd16(lm[j], mr16);
          // BCE with pos_weight: ((pw y + 1 - y) sigmoid(x) - pw y) per unit gradient
          float gb = c_bce * scale * vm * (((pw * y + 1.f - y) * sigmoidf(lf)) - pw * y);
          const float sg = rnd16(sigmoidf(lf), mr16);
          float gs = rnd16(c_cal * scale * vm * (2.f * (sg - y)), mr16);  // d calib / d sigmoid, cast back
          gs = rnd16(gs * (1.f - sg) * sg, mr16);                         // sigmoid's backward in its type
          gb = rnd16(gb, mr16);
          dm[j] = rnd16(gb + gs, mr16);
        }
      }
    }
  }
}

bool args_ok(const mc_ppo_loss_args* a, const char* what) {
  const char* bad = nullptr;
  if (!a) bad = "null args";
  else if (!a->logits || !a->action_mask || !a->actions || !a->old_logp || !a->advantages || !a->values ||
           !a->returns || !a->vpred) bad = "null row tensor";
  else if (a->M <= 0 || a->A <= 0 || a->A > MAX_A) bad = "M must be >= 1 and A in 1..512";
  else if (a->vpred_dtype != MP_F32 && a->vpred_dtype != MC_DT_BF16 && a->vpred_dtype != MC_DT_F16) bad = "vpred_dtype";
  else if (a->mine_round != MP_F32 && a->mine_round != MC_DT_BF16 && a->mine_round != MC_DT_F16) bad = "mine_round";
  else if (a->mine && (!a->labels || !a->counts)) bad = "mine logits need labels and counts";
  if (bad) {
    snprintf(g_err, sizeof g_err, "%s: bad argument (%s)", what, bad);
    return false;
  }
  return true;
}

int launched(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof g_err, "%s launch: %s", what, hipGetErrorString(e));
    return MS_EHIP;
  }
  return MS_OK;
}

}  // namespace

extern "C" {

int64_t mc_ppo_loss_workspace(int64_t M) {
  if (M <= 0) return -1;
  return (int64_t)MAX_GRID * PSTRIDE + M * RSTRIDE;
}

int mc_ppo_loss_fwd(const mc_ppo_loss_args* a, float* out, float* work, int64_t work_floats, void* stream) {
  if (!args_ok(a, "mc_ppo_loss_fwd")) return MS_EINVAL;
  if (!out || !work || work_floats < mc_ppo_loss_workspace(a->M)) {
    snprintf(g_err, sizeof g_err, "mc_ppo_loss_fwd: bad argument (out / workspace)");
    return MS_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  const int G = loss_grid(a->M);
  float* part = work;
  float* rows = work + (size_t)MAX_GRID * PSTRIDE;
  if (a->A <= 128) hipLaunchKernelGGL(k_ppo_loss_fwd<2>, dim3(G), dim3(256), 0, s, *a, part, rows);
  else if (a->A <= 256) hipLaunchKernelGGL(k_ppo_loss_fwd<4>, dim3(G), dim3(256), 0, s, *a, part, rows);
  else hipLaunchKernelGGL(k_ppo_loss_fwd<8>, dim3(G), dim3(256), 0, s, *a, part, rows);
  if (int rc = launched("k_ppo_loss_fwd")) return rc;
  hipLaunchKernelGGL(k_ppo_loss_fin, dim3(1), dim3(256), 0, s, *a, part, G, out);
  return launched("k_ppo_loss_fin");
}

int mc_ppo_loss_bwd(const mc_ppo_loss_args* a, const float* gout, const float* work, int64_t work_floats,
                    float* dlogits, void* dvpred, float* dmine, void* stream) {
  if (!args_ok(a, "mc_ppo_loss_bwd")) return MS_EINVAL;
  if (!gout || !work || work_floats < mc_ppo_loss_workspace(a->M) || !dlogits || !dvpred || (a->mine && !dmine)) {
    snprintf(g_err, sizeof g_err, "mc_ppo_loss_bwd: bad argument (gout / workspace / outputs)");
    return MS_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  const int G = loss_grid(a->M);
  const float* rows = work + (size_t)MAX_GRID * PSTRIDE;
  if (a->A <= 128) hipLaunchKernelGGL(k_ppo_loss_bwd<2>, dim3(G), dim3(256), 0, s, *a, gout, rows, dlogits, dvpred, dmine);
  else if (a->A <= 256) hipLaunchKernelGGL(k_ppo_loss_bwd<4>, dim3(G), dim3(256), 0, s, *a, gout, rows, dlogits, dvpred, dmine);
  else hipLaunchKernelGGL(k_ppo_loss_bwd<8>, dim3(G), dim3(256), 0, s, *a, gout, rows, dlogits, dvpred, dmine);
  return launched("k_ppo_loss_bwd");
}

}  // extern "C"
