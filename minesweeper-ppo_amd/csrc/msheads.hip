// msheads.hip — the policy and belief ("mine") heads of CNNResidualPolicy on MFMA.
//
// Reference (minesweeper/models/cnn_residual.py:57-64, 85-96): each head is
//   Conv1x1(96, 96) -> ReLU -> Conv1x1(96, 1)
// over the trunk features f; the policy head's output is the per-cell logit
// (index r*W + c), the mine head runs on f.detach(). On NHWC features
// f [M = N*H*W][96] a 1x1 conv is a GEMM over rows, so both heads together are
// h = relu(f . W1^T + b1) (W1 = [policy W1; mine W1], 192 x 96), logit = h . w2 + b2.
//
// k_heads_fwd: per 128-row tile, H^T[c][px] on v_mfma_f32_32x32x16_bf16 (A = W1
//   rows from LDS, B = f rows loaded straight from HBM), bias + ReLU + the w2 dot
//   product in registers (the channel sum is in-lane plus one lane^32 add), one f32
//   logit per row and head. f is read once for both heads; h never reaches HBM.
// k_heads_bwd: per 64-row tile (two workgroups per CU: 78.8 KB of LDS each), recompute
//   H[px][c] (A = f tile in LDS, B = W1),
//   dh = dlogit * w2 * (h > 0) written to an LDS image (bf16), then
//     df^T = W1p^T . dh_p^T  (policy only: the mine head sees f.detach(); W1p^T read from
//                             the W1 image with ds_read_b64_tr_b16),
//     dW1 += dh^T . f        (K = the tile's pixels; both operands K-major via
//                             ds_read_b64_tr_b16 from the LDS images),
//     dw2 += h^T . dlogit, db1 += sum dh  (in-lane accumulators);
//   per-workgroup partials are summed by k_heads_reduce.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>

#include "../../include/msenv.h"
#include "../../include/mscnn.h"
#include "mscnn_common.h"

namespace {

using namespace mc;

constexpr int C = 96;        // trunk channels
constexpr int NH = 192;      // both heads' hidden channels
constexpr int WP = 104;      // padded weight row (elements): conflict-free ds_read_b128
constexpr int TR = 128;      // rows per tile
constexpr int PART = NH * C + 2 * NH;  // per-workgroup partial: dW1 | dw2 | db1

template <typename E>
struct HeadFwdParams {
  const E* f;
  const E* w1;  // [nh][96]
  const float* b1;
  const float* w2;
  const float* b2;
  float* out_p;
  float* out_m;
  int64_t M;
};

template <typename E, bool MINE>
__global__ __launch_bounds__(256, 2) void k_heads_fwd(HeadFwdParams<E> p) {
  typedef typename EV<E>::v8 E8;
  constexpr int NT = MINE ? 6 : 3;
  __shared__ __attribute__((aligned(16))) E sW[NT * 32 * WP];
  __shared__ __attribute__((aligned(16))) float sB1[NT * 32], sW2[NT * 32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  for (int i = tid; i < NT * 32 * 12; i += 256) {
    const int c = i / 12, k8 = i - c * 12;
    *reinterpret_cast<u32x4*>(&sW[c * WP + k8 * 8]) = *reinterpret_cast<const u32x4*>(&p.w1[c * C + k8 * 8]);
  }
  for (int i = tid; i < NT * 32; i += 256) {
    sB1[i] = p.b1[i];
    sW2[i] = p.w2[i];
  }
  const float b2p = p.b2[0], b2m = MINE ? p.b2[1] : 0.f;
  __syncthreads();
  const int64_t ntiles = (p.M + TR - 1) / TR;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int zo = opaque0();
    const int64_t row = tile * TR + wave * 32 + l32;
    const bool valid = row < p.M;
    // f rows: unconditional loads from a clamped row (a guarded load sits in its own exec
    // branch); rows past M are computed and not stored
    const int64_t rowc = valid ? row : p.M - 1;
    E8 b[6];
#pragma unroll
    for (int ks = 0; ks < 6; ++ks)
      b[ks] = __builtin_bit_cast(E8, *reinterpret_cast<const u32x4*>(&p.f[rowc * C + ks * 16 + 8 * hh]));
    f32x16 acc[NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[ct][i] = 0.f;
    // W1 operands double-buffered across k steps, order pinned (reads of k+1, MFMAs of k)
    E8 A[2][NT];
    auto ld = [&](int ks, E8 (&a)[NT]) {
#pragma unroll
      for (int ct = 0; ct < NT; ++ct)
        a[ct] = *reinterpret_cast<const E8*>(&sW[(ct * 32 + l32) * WP + ks * 16 + 8 * hh + zo]);
    };
    ld(0, A[0]);
    __builtin_amdgcn_sched_group_barrier(0x020, 6, 0);  // the six f loads first, together
    __builtin_amdgcn_sched_group_barrier(0x100, NT, 0);
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) {
      if (ks + 1 < 6) {
        ld(ks + 1, A[(ks + 1) & 1]);
        __builtin_amdgcn_sched_group_barrier(0x100, NT, 0);
      }
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) acc[ct] = mfma32(A[ks & 1][ct], b[ks], acc[ct]);
      __builtin_amdgcn_sched_group_barrier(0x008, NT, 0);
    }
    // acc[ct][r] = H^T[c = ct*32 + 8*(r>>2) + 4*hh + (r&3)][px = l32]
    float s[2] = {0.f, 0.f};
#pragma unroll
    for (int ct = 0; ct < NT; ++ct)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c0 = ct * 32 + 8 * g + 4 * hh;
        const float4 bb = *reinterpret_cast<const float4*>(&sB1[c0 + zo]);
        const float4 ww = *reinterpret_cast<const float4*>(&sW2[c0 + zo]);
        s[ct / 3] += fmaxf(acc[ct][4 * g + 0] + bb.x, 0.f) * ww.x + fmaxf(acc[ct][4 * g + 1] + bb.y, 0.f) * ww.y +
                     fmaxf(acc[ct][4 * g + 2] + bb.z, 0.f) * ww.z + fmaxf(acc[ct][4 * g + 3] + bb.w, 0.f) * ww.w;
      }
    s[0] += __shfl_xor(s[0], 32);
    if (MINE) s[1] += __shfl_xor(s[1], 32);
    if (valid && hh == 0) {
      p.out_p[row] = s[0] + b2p;
      if (MINE) p.out_m[row] = s[1] + b2m;
    }
  }
}

// ------------------------------------------------------------------------------------
template <typename E>
struct HeadBwdParams {
  const E* f;
  const float* dlp;
  const float* dlm;
  const E* w1;   // [192][96]
  const E* w1pT; // unused (round 2's policy W1^T copy)
  const float* b1;
  const float* w2;
  const float* gadd;  // [M / P][96] or null: added to df (the value head's pooled gradient / P)
  E* df;
  float* part;        // [gridDim][PART]
  int64_t M;
  int P;
  int exp;            // MC_WSX builds: timing experiments (HBX_* bits; results wrong)
};
// timing experiments of k_heads_bwd (libmsenv_wsx.so, mc_set_heads_exp; tools/heads_bwd_exp.py):
// each bit removes one part so its cost can be read off the launch time
#ifdef MC_WSX
#define HBX(bit) ((p.exp & (bit)) != 0)
#else
#define HBX(bit) false
#endif
[[maybe_unused]] constexpr int HBX_NO_DF_STORE = 1, HBX_NO_DW1 = 2, HBX_NO_H = 4, HBX_NO_FLOAD = 8,
                               HBX_NO_DH_WRITE = 16, HBX_NO_DF = 32;

// f tile [128][96]: 16-B chunk ch of row r at chunk ch ^ ((r >> 2) & 3)
__device__ __forceinline__ int sf_off(int r, int col) {
  return r * C + 8 * ((col >> 3) ^ ((r >> 2) & 3)) + (col & 7);
}
// dh image [128][192]: chunk ch of row r at ch ^ (((r >> 1) & 1) << 2 | (r >> 2) & 3)
__device__ __forceinline__ int sd_off(int r, int col) {
  return r * NH + 8 * ((col >> 3) ^ ((((r >> 1) & 1) << 2) | ((r >> 2) & 3))) + (col & 7);
}

// k_heads_bwd LDS (78.8 KB: two workgroups per CU). 64-row tiles; the policy W1^T operand
// of df is read from the W1 image by transposing LDS reads, so no W1^T copy is kept.
constexpr int TRB = 64;  // rows per backward tile
template <typename E>
struct HeadLds {
  E w[NH * WP];     // W1 rows [c][k]
  E f[TRB * C];     // swizzled f tile
  E dh[TRB * NH];   // swizzled dh image; after the tile loop: the dw2 / db1 combine
  float dl[2][TRB];
  float b1[NH], w2[NH];
};
static_assert(sizeof(HeadLds<__bf16>) <= 80 * 1024, "two k_heads_bwd workgroups per CU");

// one wave's share of a 64-row tile: H recompute for px-tile pt (wave & 1) and head hd
// (wave >> 1: 0 policy, 1 mine), its dh columns, df for px-tile pt and k-tiles [KT0, KT0+NKT),
// and dW1 tiles [T0, T0+NTW) of the 18 (6 c-tiles x 3 k-tiles)
template <typename E, int T0, int NTW, int KT0, int NKT>
__device__ __forceinline__ void heads_bwd_body(const HeadBwdParams<E>& p, HeadLds<E>& L) {
  typedef typename EV<E>::v8 E8;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int pt = wave & 1, hd = wave >> 1;
  f32x16 dwacc[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) dwacc[t][i] = 0.f;
  float dw2acc[3], db1acc[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) dw2acc[j] = db1acc[j] = 0.f;

  const int64_t ntiles = (p.M + TRB - 1) / TRB;
  constexpr int NFC = TRB * 12 / 256;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t base = tile * TRB;
    const int zo = opaque0();
    // ---- stage f tile and the two logit gradients (unconditional loads from clamped rows) ----
    {
      u32x4 v[NFC];
#pragma unroll
      for (int i = 0; i < NFC; ++i) {
        const int c = tid + 256 * i + zo, r = c / 12, ch = c - r * 12;
        const int64_t row = base + r < p.M ? base + r : p.M - 1;
        v[i] = HBX(HBX_NO_FLOAD) ? u32x4{(uint32_t)c, 0u, 0u, 0u} : *reinterpret_cast<const u32x4*>(&p.f[row * C + ch * 8]);
      }
      const int64_t rowd = base + (tid & (TRB - 1)) < p.M ? base + (tid & (TRB - 1)) : p.M - 1;
      const float d0 = p.dlp[rowd];
      const float d1 = p.dlm ? p.dlm[rowd] : 0.f;
#pragma unroll
      for (int i = 0; i < NFC; ++i) {
        const int c = tid + 256 * i + zo, r = c / 12, ch = c - r * 12;
        if (base + r >= p.M) v[i] = u32x4{0u, 0u, 0u, 0u};
        *reinterpret_cast<u32x4*>(&L.f[sf_off(r, ch * 8)]) = v[i];
      }
      if (tid < TRB) {
        const bool ok = base + tid < p.M;
        L.dl[0][tid] = ok ? d0 : 0.f;
        L.dl[1][tid] = ok ? d1 : 0.f;
      }
    }
    __syncthreads();
    // ---- recompute H[px][c] for px-tile pt and this head's three c-tiles; dh -> LDS ----
    {
      f32x16 acc[3];
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
      const int ra = pt * 32 + l32 + zo;
#pragma unroll 1
      for (int ks = 0; ks < (HBX(HBX_NO_H) ? 0 : 6); ++ks) {
        const E8 a = *reinterpret_cast<const E8*>(&L.f[sf_off(ra, ks * 16 + 8 * hh)]);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const E8 b = *reinterpret_cast<const E8*>(&L.w[((3 * hd + j) * 32 + l32) * WP + ks * 16 + 8 * hh + zo]);
          acc[j] = mfma32(a, b, acc[j]);
        }
      }
      // acc[j][r] = H[px = pt*32 + 8*(r>>2) + 4*hh + (r&3)][c = (3*hd + j)*32 + l32]
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int c = (3 * hd + j) * 32 + l32;
        const float b1c = L.b1[c + zo], w2c = L.w2[c + zo];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int pr = pt * 32 + 8 * (r >> 2) + 4 * hh + (r & 3) + zo;
          const float dl = L.dl[hd][pr];
          const float hv = fmaxf(acc[j][r] + b1c, 0.f);
          dw2acc[j] += hv * dl;
          const float dh = hv > 0.f ? dl * w2c : 0.f;
          db1acc[j] += dh;
          if (!HBX(HBX_NO_DH_WRITE)) L.dh[sd_off(pr, c)] = (E)dh;
        }
      }
    }
    __syncthreads();
    // ---- df^T[k][px] = sum_c W1p[c][k] dh[px][c] (policy channels only), px-tile pt ----
    {
      f32x16 acc2[NKT];
      const int rb = pt * 32 + l32 + zo;
      const int64_t row = base + rb;
      if (p.gadd) {  // (uniform) the accumulators start at gadd[m / P] (rows past M: row M-1, discarded)
        const float* ga = p.gadd + ((row < p.M ? row : p.M - 1) / p.P) * C;
#pragma unroll
        for (int u = 0; u < NKT; ++u)
#pragma unroll
          for (int gg = 0; gg < 4; ++gg) {
            const float4 a4 = *reinterpret_cast<const float4*>(&ga[(KT0 + u) * 32 + 8 * gg + 4 * hh]);
            acc2[u][4 * gg + 0] = a4.x;
            acc2[u][4 * gg + 1] = a4.y;
            acc2[u][4 * gg + 2] = a4.z;
            acc2[u][4 * gg + 3] = a4.w;
          }
      } else {
#pragma unroll
        for (int u = 0; u < NKT; ++u)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc2[u][i] = 0.f;
      }
#pragma unroll 1
      for (int ks = 0; ks < (HBX(HBX_NO_DF) ? 0 : 6); ++ks) {
        const E8 b = *reinterpret_cast<const E8*>(&L.dh[sd_off(rb, ks * 16 + 8 * hh)]);
        const int r0 = ks * 16 + 8 * (g >> 1) + q + zo;  // W1 rows (K = c), transposed read
#pragma unroll
        for (int u = 0; u < NKT; ++u) {
          const int col = (KT0 + u) * 32 + 16 * (g & 1) + 4 * pp;
          const E8 a = cat8(lds_tr4(&L.w[r0 * WP + col]), lds_tr4(&L.w[(r0 + 4) * WP + col]));
          acc2[u] = mfma32(a, b, acc2[u]);
        }
      }
      // acc2[u][r] = df[px = rb][k = (KT0+u)*32 + 8*(r>>2) + 4*hh + (r&3)]: 8-B stores (staging
      // them in LDS for 16-B stores needs the f region, i.e. dW1 first: 3.26 ms, spills)
      if (row < p.M && !HBX(HBX_NO_DF_STORE)) {
        typedef typename EV<E>::v4 E4;
#pragma unroll
        for (int u = 0; u < NKT; ++u)
#pragma unroll
          for (int gg = 0; gg < 4; ++gg) {
            const int k0 = (KT0 + u) * 32 + 8 * gg + 4 * hh;
            *reinterpret_cast<E4*>(&p.df[row * C + k0]) =
                E4{(E)acc2[u][4 * gg + 0], (E)acc2[u][4 * gg + 1], (E)acc2[u][4 * gg + 2], (E)acc2[u][4 * gg + 3]};
          }
      }
    }

    // ---- dW1[c][k] += sum_px dh[px][c] f[px][k] over the tile's 64 rows ----
#pragma unroll 1
    for (int kk = 0; kk < (HBX(HBX_NO_DW1) ? 0 : TRB / 16); ++kk) {
      const int r0 = kk * 16 + 8 * (g >> 1) + q + zo;
      E8 av[6], bv[3];
#pragma unroll
      for (int ct = T0 / 3; ct <= (T0 + NTW - 1) / 3; ++ct) {
        const int col = ct * 32 + 16 * (g & 1) + 4 * pp;
        av[ct] = cat8(lds_tr4(&L.dh[sd_off(r0, col)]), lds_tr4(&L.dh[sd_off(r0 + 4, col)]));
      }
#pragma unroll
      for (int kt = 0; kt < 3; ++kt) {
        const int col = kt * 32 + 16 * (g & 1) + 4 * pp;
        bv[kt] = cat8(lds_tr4(&L.f[sf_off(r0, col)]), lds_tr4(&L.f[sf_off(r0 + 4, col)]));
      }
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        const int tt = T0 + t;
        dwacc[t] = mfma32(av[tt / 3], bv[tt % 3], dwacc[t]);
      }
    }
    __syncthreads();  // f / dh images are re-staged by the next tile
  }
  // ---- partials ----
  float* part = p.part + (size_t)blockIdx.x * PART;
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const int tt = T0 + t, ct = tt / 3, kt = tt % 3;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = ct * 32 + 8 * (r >> 2) + 4 * hh + (r & 3);
      part[c * C + kt * 32 + l32] = dwacc[t][r];
    }
  }
  // dw2 / db1: the two waves of a head (px-tiles 0 and 1) combine in LDS (the dh region,
  // free after the tile loop's last barrier)
  float* red = reinterpret_cast<float*>(L.dh);  // [2][NH]
  for (int i = tid; i < 2 * NH; i += 256) red[i] = 0.f;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    atomicAdd(&red[(3 * hd + j) * 32 + l32], dw2acc[j]);
    atomicAdd(&red[NH + (3 * hd + j) * 32 + l32], db1acc[j]);
  }
}

template <typename E>
__global__ __launch_bounds__(256, 2) void k_heads_bwd(HeadBwdParams<E> p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  HeadLds<E>& L = *reinterpret_cast<HeadLds<E>*>(smem);
  const int tid = threadIdx.x;
  for (int i = tid; i < NH * 12; i += 256) {
    const int c = i / 12, k8 = i - c * 12;
    *reinterpret_cast<u32x4*>(&L.w[c * WP + k8 * 8]) = *reinterpret_cast<const u32x4*>(&p.w1[c * C + k8 * 8]);
  }
  for (int i = tid; i < NH; i += 256) {
    L.b1[i] = p.b1[i];
    L.w2[i] = p.w2[i];
  }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // 18 dW1 tiles split 5/5/4/4; the 6 df tiles (2 px x 3 k) split 2/2/1/1
  switch (wave) {
    case 0: heads_bwd_body<E, 0, 5, 0, 2>(p, L); break;
    case 1: heads_bwd_body<E, 5, 5, 0, 2>(p, L); break;
    case 2: heads_bwd_body<E, 10, 4, 2, 1>(p, L); break;
    default: heads_bwd_body<E, 14, 4, 2, 1>(p, L); break;
  }
  __syncthreads();
  const float* red = reinterpret_cast<const float*>(L.dh);  // the dw2 / db1 combine of the bodies
  float* part = p.part + (size_t)blockIdx.x * PART;
  for (int i = tid; i < NH; i += 256) {
    part[NH * C + i] = red[i];
    part[NH * C + NH + i] = red[NH + i];
  }
}

// Sum of the G partials, deterministic (as k_reduce in mscnn_bwd.hip): a 256-thread block covers
// 64 outputs with 4 slices over g (slice s sums g = s, s + 4, ... on four independent
// accumulators, so a thread keeps four loads in flight), combined in fixed order through LDS.
// One thread per output over all G serially kept ~74 blocks on the GPU: 123 us per call.
constexpr int HR_S = 4, HR_IB = 256 / HR_S;
__global__ __launch_bounds__(256) void k_heads_reduce(const float* __restrict__ part, int G, float* __restrict__ dw1,
                                                      float* __restrict__ dw2, float* __restrict__ db1) {
  __shared__ float sp[HR_S][HR_IB];
  const int li = threadIdx.x % HR_IB, sl = threadIdx.x / HR_IB;
  const int i = blockIdx.x * HR_IB + li;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (i < PART) {
    int g = sl;
    for (; g + 3 * HR_S < G; g += 4 * HR_S) {
      a0 += part[(size_t)g * PART + i];
      a1 += part[(size_t)(g + HR_S) * PART + i];
      a2 += part[(size_t)(g + 2 * HR_S) * PART + i];
      a3 += part[(size_t)(g + 3 * HR_S) * PART + i];
    }
    for (; g < G; g += HR_S) a0 += part[(size_t)g * PART + i];
  }
  sp[sl][li] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (sl == 0 && i < PART) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < HR_S; ++k) s += sp[k][li];
    if (i < NH * C) dw1[i] = s;
    else if (i < NH * C + NH) dw2[i - NH * C] = s;
    else db1[i - NH * C - NH] = s;
  }
}

int bwd_grid(int64_t M) {  // two k_heads_bwd workgroups per CU
  const int64_t ntiles = (M + TRB - 1) / TRB;
  const int cap = 2 * num_cus();
  return (int)(ntiles < cap ? ntiles : cap);
}

int check(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof g_err, "%s launch: %s", what, hipGetErrorString(e));
    return MS_EHIP;
  }
  return MS_OK;
}

template <typename E>
int run_heads_fwd(const uint16_t* f, const uint16_t* w1, const float* b1, const float* w2, const float* b2,
                  float* out_p, float* out_m, int64_t M, hipStream_t s) {
  HeadFwdParams<E> p;
  p.f = reinterpret_cast<const E*>(f);
  p.w1 = reinterpret_cast<const E*>(w1);
  p.b1 = b1;
  p.w2 = w2;
  p.b2 = b2;
  p.out_p = out_p;
  p.out_m = out_m;
  p.M = M;
  const int64_t ntiles = (M + TR - 1) / TR;
  const int cap = 2 * num_cus();
  const int grid = (int)(ntiles < cap ? ntiles : cap);
  if (out_m) hipLaunchKernelGGL((k_heads_fwd<E, true>), dim3(grid), dim3(256), 0, s, p);
  else hipLaunchKernelGGL((k_heads_fwd<E, false>), dim3(grid), dim3(256), 0, s, p);
  return check("k_heads_fwd");
}

#ifdef MC_WSX
int g_heads_exp = 0;
#endif

template <typename E>
int run_heads_bwd(const uint16_t* f, const float* dlp, const float* dlm, const uint16_t* w1, const uint16_t* w1pT,
                  const float* b1, const float* w2, const float* gadd, int32_t P, uint16_t* df, float* dw1, float* db1,
                  float* dw2, float* work, int64_t M, int grid, hipStream_t s) {
  HeadBwdParams<E> p;
  p.f = reinterpret_cast<const E*>(f);
  p.dlp = dlp;
  p.dlm = dlm;
  p.w1 = reinterpret_cast<const E*>(w1);
  p.w1pT = reinterpret_cast<const E*>(w1pT);
  p.b1 = b1;
  p.w2 = w2;
  p.gadd = gadd;
  p.df = reinterpret_cast<E*>(df);
  p.part = work;
  p.M = M;
  p.P = P;
  p.exp = 0;
#ifdef MC_WSX
  p.exp = g_heads_exp;
#endif
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_heads_bwd<E>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)sizeof(HeadLds<E>));
    attr = true;
  }
  hipLaunchKernelGGL(k_heads_bwd<E>, dim3(grid), dim3(256), sizeof(HeadLds<E>), s, p);
  int rc = check("k_heads_bwd");
  if (rc) return rc;
  hipLaunchKernelGGL(k_heads_reduce, dim3((PART + HR_IB - 1) / HR_IB), dim3(256), 0, s, (const float*)work, grid, dw1,
                     dw2, db1);
  return check("k_heads_reduce");
}

}  // namespace

extern "C" {

#ifdef MC_WSX
// timing experiments only (tools/heads_bwd_exp.py): HBX_* bits of the next k_heads_bwd launches
void mc_set_heads_exp(int32_t e) { g_heads_exp = e; }
#endif

int mc_heads_fwd(const uint16_t* f, const uint16_t* w1, const float* b1, const float* w2, const float* b2,
                 float* out_p, float* out_m, int64_t M, int32_t dtype, void* stream) {
  if (!f || !w1 || !b1 || !w2 || !b2 || !out_p || M <= 0) {
    snprintf(g_err, sizeof g_err, "mc_heads_fwd: bad argument");
    return MS_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MC_DT_BF16) return run_heads_fwd<__bf16>(f, w1, b1, w2, b2, out_p, out_m, M, s);
  if (dtype == MC_DT_F16) return run_heads_fwd<_Float16>(f, w1, b1, w2, b2, out_p, out_m, M, s);
  snprintf(g_err, sizeof g_err, "mc_heads_fwd: dtype %d unsupported (0 bf16, 1 f16)", dtype);
  return MS_EINVAL;
}

int64_t mc_heads_bwd_workspace(int64_t M) {
  if (M <= 0) return -1;
  return (int64_t)bwd_grid(M) * PART;
}

int mc_heads_bwd(const uint16_t* f, const float* dlp, const float* dlm, const uint16_t* w1, const uint16_t* w1pT,
                 const float* b1, const float* w2, const float* gadd, int32_t P, uint16_t* df, float* dw1,
                 float* db1, float* dw2, float* work, int64_t work_floats, int64_t M, int32_t dtype, void* stream) {
  if (!f || !dlp || !w1 || !b1 || !w2 || !df || !dw1 || !db1 || !dw2 || !work || M <= 0 ||
      (gadd && P <= 0)) {
    snprintf(g_err, sizeof g_err, "mc_heads_bwd: bad argument");
    return MS_EINVAL;
  }
  const int grid = bwd_grid(M);
  if (work_floats < (int64_t)grid * PART) {
    snprintf(g_err, sizeof g_err, "mc_heads_bwd: workspace too small");
    return MS_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MC_DT_BF16) return run_heads_bwd<__bf16>(f, dlp, dlm, w1, w1pT, b1, w2, gadd, P, df, dw1, db1, dw2, work, M, grid, s);
  if (dtype == MC_DT_F16)
    return run_heads_bwd<_Float16>(f, dlp, dlm, w1, w1pT, b1, w2, gadd, P, df, dw1, db1, dw2, work, M, grid, s);
  snprintf(g_err, sizeof g_err, "mc_heads_bwd: dtype %d unsupported (0 bf16, 1 f16)", dtype);
  return MS_EINVAL;
}

}  // extern "C"
