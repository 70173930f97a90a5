// mscnn_bwd.hip — backward of the fused residual-CNN layer (gfx950 MFMA).
//
// Forward (mscnn.hip, reference chain minesweeper/models/cnn_residual.py:10-26, 50-54):
//   y = conv3x3(x, w) + bias;  z = GN(y) * gamma + beta [+ res];  out = relu(z) [* dmask]
// Backward, per layer, in two persistent kernels:
//   k_bwd_data  (one workgroup per sample at a time, 2 workgroups per CU)
//     pass 1: dz = (out > 0) * dout * dmask  and the per-channel sums (out > 0 read
//             as the forward's ReLU bitmask, 1/16 of out's bytes, when one is given)
//             S1 = sum dz, S2 = sum dz*yhat, S3 = sum yhat (yhat = (y - mean) * rstd);
//     pass 2: dy = rstd*gamma*dz - rstd*mean_g(gamma*dz) - rstd*yhat*mean_g(gamma*dz*yhat)
//             (GroupNorm backward), kept in an LDS tile and stored for k_wgrad;
//     dgrad : dx[q] = sum_tap dy[q - s(tap)] . W[tap]^T on v_mfma_f32_32x32x16_bf16
//             (A = 32 pixels x 16 co read from the dy tile by per-lane shifted row
//             addresses, out-of-board rows pointing at a zero row; B = W^T[tap] [ci][co]),
//             + the skip-gradient addend, one bf16 store.
//     d gamma = sum S2, d beta = sum S1, d bias = sum dy come out of the same sums.
//   k_wgrad (XCD-aware grid: the 3 workgroups that split ci of one sample group sit on
//            one XCD so the dy they all read is shared in its L2)
//     dW[tap][co][ci] = sum_{n,p} dy[n][p][co] * x[n][p + s(tap)][ci]: a GEMM whose K is
//     every pixel of every sample; both operands are read K-major with
//     ds_read_b64_tr_b16 straight from the NHWC tiles (dy [P][96], x [halo][32]).
// Per-workgroup partials are summed by k_reduce (deterministic, no atomics).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/msenv.h"
#include "../../include/mscnn.h"
#include "mscnn_common.h"

namespace {

using namespace mc;

constexpr int DCP = 104;       // dy tile row stride (elements): conflict-free ds_read_b128 row reads
constexpr int PG = 21;         // pixel groups of the element-wise passes: thread = (pg, c8)
constexpr int NC8 = COUT / 8;  // 16-byte chunks per 96-channel pixel row

template <typename E>
struct BwdDataParams {
  const E* dout;
  const E* out;
  const uint8_t* rmask;  // ReLU bitmask of the forward (replaces the sign test on out), or NULL
  const E* y;
  const float* stats;
  const float* gamma;
  const float* dmask;
  const E* wT;
  const E* addend;
  E* dy;
  E* dz;
  E* dx;
  float* part;  // [gridDim][3][96]
  int N, H, W;
};

__host__ __device__ inline int dtile_bytes(int P) { return ((P + 1) * DCP * 2 + 15) & ~15; }
__host__ __device__ constexpr int red_bytes() {  // sRed [PG][3][96] f32, aliased by sW [96][DCP] bf16
  return PG * 3 * COUT * 4 > COUT * DCP * 2 ? PG * 3 * COUT * 4 : COUT * DCP * 2;
}
__host__ __device__ inline int bwd_data_lds(int P) { return dtile_bytes(P) + red_bytes() + 6 * COUT * 4; }

// RM: the ReLU decisions come from the forward's bitmask (p.rmask), else from out
template <typename E, int NPT, bool DGRAD, int NCH, bool RM>
__global__ __launch_bounds__(256, NPT <= 2 ? 2 : 1) void k_bwd_data(BwdDataParams<E> p) {
  // no contraction: every expression rounds the same way in the per-layer and the one-launch
  // kernels (explicit fmaf where a fused multiply-add is wanted), so they agree bitwise
#pragma clang fp contract(off)
  typedef typename EV<E>::v8 E8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int H = p.H, W = p.W, P = H * W;
  E* sD = reinterpret_cast<E*>(smem);  // [P+1][DCP] (row P = 0); later [P][96] dx staging
  float* sRed = reinterpret_cast<float*>(smem + dtile_bytes(P));
  E* sW = reinterpret_cast<E*>(sRed);  // W^T[tap] as [ci][DCP]
  float* sCo = reinterpret_cast<float*>(smem + dtile_bytes(P) + red_bytes());  // [3][96]
  float* sTmp = sCo + 3 * COUT;                                                 // [2][96]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const float inv_cnt = 1.0f / (16.0f * (float)P);
  float acc_g = 0.f, acc_b = 0.f, acc_bias = 0.f;  // tid < 96: running sums for channel tid

  for (int i = tid; i < DCP / 8; i += 256) *reinterpret_cast<u32x4*>(&sD[P * DCP + 8 * i]) = u32x4{0u, 0u, 0u, 0u};
  int qr[NPT], qc[NPT];
#pragma unroll
  for (int t = 0; t < NPT; ++t) {
    const int q = (wave * NPT + t) * 32 + l32;
    qr[t] = q < P ? q / W : -1000;  // an invalid pixel never lands on the board
    qc[t] = q < P ? q - qr[t] * W : -1000;
  }

  for (int n = blockIdx.x; n < p.N; n += gridDim.x) {
    // loop-variant thread coordinates: keep the per-chunk address math inside the loop
    // (hoisted out of it, a few dozen 64-bit addresses would be spilled)
    const int tid = threadIdx.x + opaque0();
    const int pg = tid / NC8, c8 = tid - pg * NC8;
    const bool gact = tid < PG * NC8;
    const int grp = c8 >> 1;
    // ---------------- pass 1: dz and per-channel sums ----------------
    float dm[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) dm[j] = 1.f;
    float mean = 0.f, rstd = 0.f;
    if (gact) {
      if (p.dmask) {
#pragma unroll
        for (int j = 0; j < 8; ++j) dm[j] = p.dmask[(size_t)n * COUT + c8 * 8 + j];
      }
      mean = p.stats[((size_t)n * NGRP + grp) * 2];
      rstd = p.stats[((size_t)n * NGRP + grp) * 2 + 1];
    }
    // y stays in registers for pass 2; dz goes to its slot of the dy tile (rewritten in place)
    u32x4 yr[NCH];
    float s1[8], s2[8], s3[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s1[j] = s2[j] = s3[j] = 0.f;
    constexpr int LB = RM ? 7 : 4;  // chunks whose loads are in flight together
#pragma unroll
    for (int i0 = 0; i0 < NCH; i0 += LB) {
      u32x4 dv[LB], ov[LB];
      uint32_t mv[LB];
#pragma unroll
      for (int u = 0; u < LB; ++u) {
        const int i = i0 + u, px = pg + PG * i;
        if (i < NCH) yr[i] = u32x4{0u, 0u, 0u, 0u};
        mv[u] = 0u;
        if (i < NCH && gact && px < P) {
          const size_t o = ((size_t)n * P + px) * COUT + c8 * 8;
          dv[u] = *reinterpret_cast<const u32x4*>(&p.dout[o]);
          if (RM) mv[u] = p.rmask[((size_t)n * P + px) * NC8 + c8];
          else ov[u] = *reinterpret_cast<const u32x4*>(&p.out[o]);
          yr[i] = *reinterpret_cast<const u32x4*>(&p.y[o]);
        }
      }
#pragma unroll
      for (int u = 0; u < LB; ++u) {
        const int i = i0 + u, px = pg + PG * i;
        if (i < NCH && gact && px < P) {
          const E8 d8 = __builtin_bit_cast(E8, dv[u]);
          const E8 y8 = __builtin_bit_cast(E8, yr[i]);
          uint32_t pos = mv[u];
          if (!RM) {
            const E8 o8 = __builtin_bit_cast(E8, ov[u]);
#pragma unroll
            for (int j = 0; j < 8; ++j) pos |= ((float)o8[j] > 0.f ? 1u : 0u) << j;
          }
          E8 z8;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float d = (float)d8[j] * dm[j];
            z8[j] = (E)(((pos >> j) & 1u) ? d : 0.f);
            const float zf = (float)z8[j];
            const float yh = ((float)y8[j] - mean) * rstd;
            s1[j] += zf;
            s2[j] = __builtin_fmaf(zf, yh, s2[j]);
            s3[j] += yh;
          }
          *reinterpret_cast<u32x4*>(&sD[px * DCP + c8 * 8]) = __builtin_bit_cast(u32x4, z8);
        }
      }
    }
    // tap 0's W^T: loaded here, its latency hidden behind the channel reductions
    constexpr int NWC = (COUT * NC8 + 255) / 256;  // 16-B chunks of one W^T tap per thread
    u32x4 wr[NWC];
    if (DGRAD) {
#pragma unroll
      for (int k = 0; k < NWC; ++k) {
        const int c = tid + 256 * k;
        if (k < COUT * NC8 / 256 || c < COUT * NC8) wr[k] = reinterpret_cast<const u32x4*>(p.wT)[c];
      }
    }
    if (gact) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sRed[(pg * 3 + 0) * COUT + c8 * 8 + j] = s1[j];
        sRed[(pg * 3 + 1) * COUT + c8 * 8 + j] = s2[j];
        sRed[(pg * 3 + 2) * COUT + c8 * 8 + j] = s3[j];
      }
    }
    __syncthreads();
    float S1 = 0.f, S2 = 0.f, S3 = 0.f, gam = 0.f, cmean = 0.f, crstd = 0.f;
    if (tid < COUT) {
      for (int g = 0; g < PG; ++g) {
        S1 += sRed[(g * 3 + 0) * COUT + tid];
        S2 += sRed[(g * 3 + 1) * COUT + tid];
        S3 += sRed[(g * 3 + 2) * COUT + tid];
      }
      gam = p.gamma[tid];
      cmean = p.stats[((size_t)n * NGRP + (tid >> 4)) * 2];
      crstd = p.stats[((size_t)n * NGRP + (tid >> 4)) * 2 + 1];
      sTmp[tid] = gam * S1;
      sTmp[COUT + tid] = gam * S2;
      acc_g += S2;
      acc_b += S1;
    }
    __syncthreads();
    if (tid < COUT) {
      const int g0 = (tid >> 4) * 16;
      float m1 = 0.f, m2 = 0.f;
      for (int k = 0; k < 16; ++k) {
        m1 += sTmp[g0 + k];
        m2 += sTmp[COUT + g0 + k];
      }
      m1 *= inv_cnt;
      m2 *= inv_cnt;
      sCo[tid] = crstd * gam;
      sCo[COUT + tid] = -crstd * crstd * m2;
      sCo[2 * COUT + tid] = crstd * (crstd * m2 * cmean - m1);
      acc_bias += crstd * (gam * S1 - (float)P * m1 - m2 * S3);
    }
    __syncthreads();

    // tap 0's W^T goes to sW (free now: the sums are read) before pass 2 issues its
    // stores: a load consumed behind those stores would wait for all of them
    if (DGRAD) {
#pragma unroll
      for (int k = 0; k < NWC; ++k) {
        const int c = tid + 256 * k;
        if (k < COUT * NC8 / 256 || c < COUT * NC8) {
          const int ci = c / NC8, k8 = c - ci * NC8;
          *reinterpret_cast<u32x4*>(&sW[ci * DCP + k8 * 8]) = wr[k];
        }
      }
    }
    // ---------------- pass 2: dy (GroupNorm backward) -> LDS tile + HBM ----------------
    if (gact) {
      float A[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) A[j] = sCo[c8 * 8 + j];
      const float Bg = sCo[COUT + c8 * 8], Cg = sCo[2 * COUT + c8 * 8];
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int px = pg + PG * i;
        if (px < P) {
          const u32x4 zv = *reinterpret_cast<const u32x4*>(&sD[px * DCP + c8 * 8]);
          // dz is stored here rather than in pass 1: a store there would sit between the
          // next chunk batch's loads and their use, and vmcnt would drain it each batch
          if (p.dz) *reinterpret_cast<u32x4*>(&p.dz[((size_t)n * P + px) * COUT + c8 * 8]) = zv;
          const E8 z8 = __builtin_bit_cast(E8, zv);
          const E8 y8 = __builtin_bit_cast(E8, yr[i]);
          E8 d8;
#pragma unroll
          for (int j = 0; j < 8; ++j) d8[j] = (E)__builtin_fmaf(A[j], (float)z8[j], __builtin_fmaf(Bg, (float)y8[j], Cg));
          const u32x4 v = __builtin_bit_cast(u32x4, d8);
          *reinterpret_cast<u32x4*>(&sD[px * DCP + c8 * 8]) = v;
          *reinterpret_cast<u32x4*>(&p.dy[((size_t)n * P + px) * COUT + c8 * 8]) = v;
        }
      }
    }
    if (!DGRAD) continue;  // (uniform) the stem's input needs no gradient
    __syncthreads();

    // ---------------- dgrad: dx = sum_tap shift(dy) . W^T[tap] ----------------
    f32x16 acc[NPT][3];
#pragma unroll
    for (int t = 0; t < NPT; ++t)
#pragma unroll
      for (int ct = 0; ct < 3; ++ct)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[t][ct][i] = 0.f;
    for (int tap = 0; tap < 9; ++tap) {
      if (tap + 1 < 9) {
        const u32x4* ws = reinterpret_cast<const u32x4*>(p.wT + (size_t)(tap + 1) * COUT * COUT);
#pragma unroll
        for (int k = 0; k < NWC; ++k) {
          const int c = tid + 256 * k;
          if (k < COUT * NC8 / 256 || c < COUT * NC8) wr[k] = ws[c];  // the first 4 chunks are always full
        }
      }
      const int dr = tap / 3 - 1, dc = tap % 3 - 1;
      int aoff[NPT];
#pragma unroll
      for (int t = 0; t < NPT; ++t) {
        const int sr = qr[t] - dr, sc = qc[t] - dc;
        const bool v = (unsigned)sr < (unsigned)H && (unsigned)sc < (unsigned)W;
        aoff[t] = (v ? sr * W + sc : P) * DCP + 8 * hh;
      }
      // 6 ci steps, operands double-buffered: step k+1's LDS reads are issued before
      // step k's MFMAs
      auto ld = [&](int k0, E8 (&a)[NPT], E8 (&b)[3]) {
#pragma unroll
        for (int ct = 0; ct < 3; ++ct)
          b[ct] = *reinterpret_cast<const E8*>(&sW[(ct * 32 + l32) * DCP + k0 + 8 * hh]);
#pragma unroll
        for (int t = 0; t < NPT; ++t) a[t] = *reinterpret_cast<const E8*>(&sD[aoff[t] + k0]);
      };
      auto mm = [&](const E8 (&a)[NPT], const E8 (&b)[3]) {
#pragma unroll
        for (int t = 0; t < NPT; ++t)
#pragma unroll
          for (int ct = 0; ct < 3; ++ct) acc[t][ct] = mfma32(a[t], b[ct], acc[t][ct]);
      };
      E8 a0[NPT], b0[3], a1[NPT], b1[3];
      ld(0, a0, b0);
      __builtin_amdgcn_sched_group_barrier(0x100, NPT + 3, 0);  // pinned order: reads(k+1), MFMAs(k)
#pragma unroll
      for (int k0 = 0; k0 < COUT; k0 += 32) {
        ld(k0 + 16, a1, b1);
        __builtin_amdgcn_sched_group_barrier(0x100, NPT + 3, 0);
        mm(a0, b0);
        __builtin_amdgcn_sched_group_barrier(0x008, 3 * NPT, 0);
        if (k0 + 32 < COUT) {
          ld(k0 + 32, a0, b0);
          __builtin_amdgcn_sched_group_barrier(0x100, NPT + 3, 0);
        }
        mm(a1, b1);
        __builtin_amdgcn_sched_group_barrier(0x008, 3 * NPT, 0);
      }
      __syncthreads();  // sW (and, after the last tap, sD) fully read
      if (tap + 1 < 9) {
#pragma unroll
        for (int k = 0; k < NWC; ++k) {
          const int c = tid + 256 * k;
          if (k < COUT * NC8 / 256 || c < COUT * NC8) {
            const int ci = c / NC8, k8 = c - ci * NC8;
            *reinterpret_cast<u32x4*>(&sW[ci * DCP + k8 * 8]) = wr[k];
          }
        }
        __syncthreads();
      }
    }
    // ---------------- epilogue: dx (+ addend) via a [P][96] staging image ----------------
#pragma unroll
    for (int t = 0; t < NPT; ++t)
#pragma unroll
      for (int ct = 0; ct < 3; ++ct)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int px = (wave * NPT + t) * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
          if (px < P) sD[px * COUT + ct * 32 + l32] = (E)acc[t][ct][i];
        }
    __syncthreads();
    if (gact) {
      u32x4 ad[NCH];  // all addend loads in flight before the first dependent store
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int px = pg + PG * i;
        ad[i] = u32x4{0u, 0u, 0u, 0u};
        if (p.addend && px < P) ad[i] = *reinterpret_cast<const u32x4*>(&p.addend[((size_t)n * P + px) * COUT + c8 * 8]);
      }
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int px = pg + PG * i;
        if (px < P) {
          const E8 a8 = __builtin_bit_cast(E8, *reinterpret_cast<const u32x4*>(&sD[px * COUT + c8 * 8]));
          const E8 r8 = __builtin_bit_cast(E8, ad[i]);
          E8 s8;
#pragma unroll
          for (int j = 0; j < 8; ++j) s8[j] = (E)pin_f32((float)a8[j] + (float)r8[j]);
          *reinterpret_cast<u32x4*>(&p.dx[((size_t)n * P + px) * COUT + c8 * 8]) = __builtin_bit_cast(u32x4, s8);
        }
      }
    }
    // the next sample's pass 1 writes dz into sD while a slower wave may still be reading its
    // dx chunks here: an LDS-only barrier (the dx stores stay in flight)
    lds_barrier();
  }
  if (tid < COUT) {
    p.part[((size_t)blockIdx.x * 3 + 0) * COUT + tid] = acc_g;
    p.part[((size_t)blockIdx.x * 3 + 1) * COUT + tid] = acc_b;
    p.part[((size_t)blockIdx.x * 3 + 2) * COUT + tid] = acc_bias;
  }
}

// ------------------------------------------------------------------------------------
template <typename E>
struct WgradParams {
  const E* dy;
  const E* x;
  float* part;  // [G][9][96][CIN]
  int N, H, W, G;
  // x recomputed from a GroupNorm layer's saved y (k_wgrad_c96 only; gn_stats == null: x is x):
  // x = 16-bit(max(y * a + b, 0) * d), a = gamma * rstd, b = beta - mean * a, d = dmask or 1,
  // every step rounded as the forward epilogue that produced x rounds it (mc_conv_wgrad_gn)
  const float* gn_stats;  // [N][6][2] (mean, rstd)
  const float* gn_gamma;
  const float* gn_beta;
  const float* gn_dmask;  // [N][96] or null
};

__host__ __device__ inline int wgrad_lds(int H, int W) {
  const int P = H * W, Ppad = (P + 15) & ~15;
  return Ppad * COUT * 2 + (H + 2) * (W + 2) * 32 * 2;
}

// One wave's share of the 27 (tap, co-tile) 32x32 tiles of a 32-wide ci slice: tiles
// [T0, T0+NT) in tap-major order, so a wave touches at most 3 taps.
// PF (16x16 boards, 96 channels): the next sample's dy and x slice are loaded into
// registers (12 + 4 16-B chunks per thread) while this sample's MFMAs run, and written
// to LDS after the trailing barrier, so the load round trip leaves the critical path.
// SG: the next step's NR LDS reads spread over this step's NT MFMAs by sched_group_barrier, so
// every MFMA's operands were read one step (NT MFMAs) earlier
template <int NR, int NT, int T = 0>
__device__ __forceinline__ void pin_reads_mfma() {
  if constexpr (T < NT) {
    constexpr int r = (NR * (T + 1)) / NT - (NR * T) / NT;
    if constexpr (r > 0) __builtin_amdgcn_sched_group_barrier(0x100, r, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    pin_reads_mfma<NR, NT, T + 1>();
  }
}

template <typename E, int CIN, int T0, int NT, bool PF, bool SG>
__device__ __forceinline__ void wgrad_body(const WgradParams<E>& p, E* sDY, E* sX, int gid, int ci0) {
  typedef typename EV<E>::v8 E8;
  constexpr int TAP0 = T0 / 3, TAP1 = (T0 + NT - 1) / 3, NTAP = TAP1 - TAP0 + 1;
  constexpr int XC = CIN < 32 ? CIN : 32;  // real channels of the slice (the stem's 16 + 16 zero)
  constexpr int XCH = XC / 8;
  const int H = p.H, W = p.W, P = H * W, Ppad = (P + 15) & ~15, WP = W + 2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int col = 16 * (g & 1) + 4 * pp;  // tr-read column of this lane within a 32-wide block
  const int rowoff = 8 * (g >> 1) + q;    // tr-read row (pixel) offset within a 16-deep k step
  const float invW = 1.0f / (float)W;
  int tapoff[NTAP];
#pragma unroll
  for (int j = 0; j < NTAP; ++j) {
    const int tap = TAP0 + j;
    tapoff[j] = ((tap / 3 - 1) * WP + (tap % 3 - 1)) * 32;
  }
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  constexpr int NDY = PF ? 256 * NC8 / 256 : 1, NXS = PF ? 256 * XCH / 256 : 1;
  u32x4 rdy[NDY], rx[NXS];
  auto prefetch = [&](int n) {  // PF: P == 256, W == 16
    if (n < p.N) {
      const u32x4* dys = reinterpret_cast<const u32x4*>(p.dy + (size_t)n * 256 * COUT);
#pragma unroll
      for (int k = 0; k < NDY; ++k) rdy[k] = dys[tid + 256 * k];
#pragma unroll
      for (int k = 0; k < NXS; ++k) {
        const int c = tid + 256 * k, px = c / XCH, kk = c - px * XCH;
        rx[k] = *reinterpret_cast<const u32x4*>(&p.x[((size_t)n * 256 + px) * CIN + ci0 + kk * 8]);
      }
    }
  };
  if (PF) prefetch(gid);
  for (int n = gid; n < p.N; n += p.G) {
    if (PF) {
#pragma unroll
      for (int k = 0; k < NDY; ++k) *reinterpret_cast<u32x4*>(&sDY[(tid + 256 * k) * 8]) = rdy[k];
#pragma unroll
      for (int k = 0; k < NXS; ++k) {
        const int c = tid + 256 * k, px = c / XCH, kk = c - px * XCH;
        const int r = px >> 4, cc = px & 15;
        *reinterpret_cast<u32x4*>(&sX[((r + 1) * 18 + cc + 1) * 32 + kk * 8]) = rx[k];
      }
      __syncthreads();
      prefetch(n + p.G);
      asm volatile("" ::: "memory");  // the prefetch is issued before the MFMA loop
    } else {
      const u32x4* dys = reinterpret_cast<const u32x4*>(p.dy + (size_t)n * P * COUT);
#pragma unroll 4
      for (int c = tid; c < P * NC8; c += 256) *reinterpret_cast<u32x4*>(&sDY[c * 8]) = dys[c];
#pragma unroll 2
      for (int c = tid; c < P * XCH; c += 256) {
        const int px = c / XCH, k = c - px * XCH;
        const int r = px / W, cc = px - r * W;
        *reinterpret_cast<u32x4*>(&sX[((r + 1) * WP + cc + 1) * 32 + k * 8]) =
            *reinterpret_cast<const u32x4*>(&p.x[((size_t)n * P + px) * CIN + ci0 + k * 8]);
      }
      __syncthreads();
    }
    if (PF) {
      // 16 pixel steps, operands double-buffered: step k+1's LDS reads are issued
      // before step k's MFMAs
      auto ld = [&](int k0, E8 (&a)[3], E8 (&b)[NTAP]) {
#pragma unroll
        for (int cot = 0; cot < 3; ++cot) {
          const E* base = sDY + (k0 + rowoff) * COUT + cot * 32 + col;
          a[cot] = cat8(lds_tr4(base), lds_tr4(base + 4 * COUT));
        }
        const int px0 = k0 + rowoff, px1 = px0 + 4;
        const int h0 = ((px0 >> 4) + 1) * 18 + (px0 & 15) + 1, h1 = ((px1 >> 4) + 1) * 18 + (px1 & 15) + 1;
#pragma unroll
        for (int j = 0; j < NTAP; ++j)
          b[j] = cat8(lds_tr4(sX + h0 * 32 + tapoff[j] + col), lds_tr4(sX + h1 * 32 + tapoff[j] + col));
      };
      auto mm = [&](const E8 (&a)[3], const E8 (&b)[NTAP]) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int tt = T0 + t;
          acc[t] = mfma32(a[tt % 3], b[tt / 3 - TAP0], acc[t]);
        }
      };
      E8 a0[3], b0[NTAP], a1[3], b1[NTAP];
      constexpr int NR = 6 + 2 * NTAP;
      ld(0, a0, b0);
      if constexpr (SG) __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
      for (int k0 = 0; k0 < 256; k0 += 32) {
        ld(k0 + 16, a1, b1);
        mm(a0, b0);
        if constexpr (SG) pin_reads_mfma<NR, NT>();
        if (k0 + 32 < 256) {
          ld(k0 + 32, a0, b0);
          mm(a1, b1);
          if constexpr (SG) pin_reads_mfma<NR, NT>();
        } else {
          mm(a1, b1);
          if constexpr (SG) pin_reads_mfma<0, NT>();
        }
      }
    } else
    for (int k0 = 0; k0 < Ppad; k0 += 16) {
      E8 a[3];
#pragma unroll
      for (int cot = 0; cot < 3; ++cot) {
        const E* base = sDY + (k0 + rowoff) * COUT + cot * 32 + col;
        a[cot] = cat8(lds_tr4(base), lds_tr4(base + 4 * COUT));
      }
      int h[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int px = k0 + rowoff + 4 * s;
        const int r = (int)(((float)px + 0.5f) * invW);
        h[s] = px < P ? (r + 1) * WP + (px - r * W) + 1 : W + 3;  // beyond P: dy rows are 0
      }
      E8 b[NTAP];
#pragma unroll
      for (int j = 0; j < NTAP; ++j)
        b[j] = cat8(lds_tr4(sX + h[0] * 32 + tapoff[j] + col), lds_tr4(sX + h[1] * 32 + tapoff[j] + col));
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int tt = T0 + t;
        acc[t] = mfma32(a[tt % 3], b[tt / 3 - TAP0], acc[t]);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int tt = T0 + t, tap = tt / 3, cot = tt % 3;
    const int ci = lane & 31;
    if (ci < XC) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = cot * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        p.part[(((size_t)gid * 9 + tap) * COUT + co) * CIN + ci0 + ci] = acc[t][r];
      }
    }
  }
}

template <typename E, int CIN, bool PF, bool SG>
__global__ __launch_bounds__(256, 2) void k_wgrad(WgradParams<E> p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NCI = CIN / 32 > 0 ? CIN / 32 : 1;
  const int P = p.H * p.W, Ppad = (P + 15) & ~15;
  E* sDY = reinterpret_cast<E*>(smem);  // [Ppad][96], rows >= P zero
  E* sX = sDY + Ppad * COUT;                  // [(H+2)(W+2)][32] zero-halo ci slice
  const int tid = threadIdx.x;
  for (int i = P * NC8 + tid; i < Ppad * NC8; i += 256) *reinterpret_cast<u32x4*>(&sDY[i * 8]) = u32x4{0u, 0u, 0u, 0u};
  for (int i = tid; i < (p.H + 2) * (p.W + 2) * 4; i += 256) *reinterpret_cast<u32x4*>(&sX[i * 8]) = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  // XCD-aware: block b runs on XCD b % 8; the NCI slices of group gid share that XCD
  const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
  const int cig = j % NCI, gid = (j / NCI) * 8 + xcd;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  switch (wave) {
    case 0: wgrad_body<E, CIN, 0, 7, PF, SG>(p, sDY, sX, gid, cig * 32); break;
    case 1: wgrad_body<E, CIN, 7, 7, PF, SG>(p, sDY, sX, gid, cig * 32); break;
    case 2: wgrad_body<E, CIN, 14, 7, PF, SG>(p, sDY, sX, gid, cig * 32); break;
    default: wgrad_body<E, CIN, 21, 6, PF, SG>(p, sDY, sX, gid, cig * 32); break;
  }
}

// k_wgrad_c96 (16x16 boards, 96 -> 96 channels; mc_set_variant(MC_VAR_WGRAD, 3)): one 512-thread
// workgroup per CU owns all 81 (tap, co tile, ci tile) 32x32 tiles, so a sample's dy and x cross
// HBM and LDS once (k_wgrad's three ci-slice workgroups read dy three times and write 192 KB of
// LDS per sample; this one 48 KB of x, and its dy arrives by LDS-DMA, double-buffered, while the
// previous sample's MFMAs run). Wave w owns tap w for every (co tile, ci tile) -- 9 tiles, B
// operands x[tap w][ci tile 0..2] -- plus one or two tiles of tap 8 (ci tile m(w)); 21/20/20/20
// tiles per SIMD. Partials [G][9][96][96] as k_wgrad's, same k_reduce.
constexpr int WC_DY = 256 * COUT;       // elements of one dy buffer
constexpr int WC_SX = 18 * 18 * COUT;   // zero-halo x image, 96 channels a pixel
constexpr int WC_CO = 3 * COUT;          // floats of the GroupNorm-apply coefficients (a | b | d)
constexpr int WC_LDS = (2 * WC_DY + WC_SX) * 2 + WC_CO * 4;  // 160,512 + 1,152 B
static_assert(WC_LDS <= 160 * 1024, "k_wgrad_c96 LDS");

// One full-wave LDS-DMA of 1 KiB (16 B a lane, lane-linear at LDS byte address m0v) issued from
// inline asm: as a builtin, the compiler makes every later LDS read wait for it (vmcnt(0) in
// front of the MFMA loop, the prefetch serialised); the kernel waits for it explicitly
__device__ __forceinline__ void dma16_asm(const void* src, uint32_t m0v) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0v) : "memory", "m0");
}

template <int WV>
struct WgcTiles {
  static constexpr int NT = WV == 0 ? 11 : 10;        // tiles
  static constexpr int M8 = WV <= 1 ? 0 : (WV <= 4 ? 1 : 2);  // ci tile of this wave's tap-8 tiles
  static constexpr int co(int t) { return t < 9 ? t % 3 : (WV == 0 ? t - 9 : (WV == 1 ? 2 : (WV - 2) % 3)); }
  static constexpr int b(int t) { return t < 9 ? t / 3 : 3; }  // B operand: 0..2 tap WV ci tile b, 3 tap 8
  static constexpr int tap(int bi) { return bi < 3 ? WV : 8; }
  static constexpr int cis(int bi) { return bi < 3 ? bi : M8; }
};

template <typename E, int WV, bool GN>
__device__ __forceinline__ void wgc_body(const WgradParams<E>& p, E* sDY, E* sX, float* sCo, int gid) {
  typedef typename EV<E>::v8 E8;
  using T = WgcTiles<WV>;
  // GN: waves 6 and 7 (threads 384 .. 479: channel c = tid - 384) fetch sample n's mean / rstd /
  // dmask with its prefetch and write a | b | d to sCo after their MFMA loop; sCo is read by
  // put_x after the barrier that frees sX (its previous reader, the last put_x, is a barrier back)
  constexpr bool CO = GN && WV >= 6;
  const int cc = threadIdx.x - 384;
  const bool cact = CO && cc < COUT;
  float cg = 0.f, cbt = 0.f, cm = 0.f, cr = 0.f, cdm = 1.f;
  if (cact) {
    cg = p.gn_gamma[cc];
    cbt = p.gn_beta[cc];
  }
  constexpr int NT = T::NT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int col = 16 * (g & 1) + 4 * pp;  // tr-read column of this lane within a 32-wide block
  const int rowoff = 8 * (g >> 1) + q;    // tr-read pixel offset within a 16-deep k step
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
  u32x4 rx[6];
  // sample n's dy -> sDY[buf] by LDS-DMA (this wave's 6 KiB: six full-wave 1-KiB instructions,
  // lane-linear destinations) and its x -> registers (6 16-B chunks a thread)
  auto issue = [&](int n, int buf) {
    if (n < p.N) {
      const E* src = p.dy + (size_t)n * WC_DY;
      const int ln = lane + opaque0();
      const uint32_t dst = (uint32_t)(size_t)((__attribute__((address_space(3))) E*)(sDY + buf * WC_DY)) + WV * 6 * 1024;
#pragma unroll
      for (int k = 0; k < 6; ++k) dma16_asm(src + ((WV * 6 + k) * 64 + ln) * 8, dst + k * 1024);
      const u32x4* xs = reinterpret_cast<const u32x4*>(p.x + (size_t)n * WC_DY);
#pragma unroll
      for (int k = 0; k < 6; ++k) rx[k] = xs[tid + 512 * k];
      if (cact) {
        cm = p.gn_stats[((size_t)n * NGRP + (cc >> 4)) * 2];
        cr = p.gn_stats[((size_t)n * NGRP + (cc >> 4)) * 2 + 1];
        if (p.gn_dmask) cdm = p.gn_dmask[(size_t)n * COUT + cc];
      }
    }
  };
  auto put_co = [&]() {  // (the forward's coefficients, same operations: a, then b from a)
#pragma clang fp contract(off)  // b = beta - (mean * a) rounded twice, as the forward computes it
    if (cact) {
      const float a = cg * cr;
      sCo[cc] = a;
      sCo[COUT + cc] = cbt - cm * a;
      sCo[2 * COUT + cc] = cdm;
    }
  };
  auto put_x = [&]() {
    if constexpr (GN) {
      // chunks k and k + 3 of a thread hold the same 8 channels (512 = 42 * 12 + 8, so chunk k's
      // channel group is (tid + 8k) mod 12): one read of their coefficients serves both. The
      // forward epilogue's z = max(y a + b + 0, 0), x = 16-bit(z d); the "+ 0" only turns a -0 into
      // +0, which the max and the weight gradient's sums cannot tell apart, so it is left out
#pragma clang fp contract(off)
#pragma unroll
      for (int j3 = 0; j3 < 3; ++j3) {
        const int kk = (tid + 512 * j3) % 12;
        f32x4 a4[2], b4[2], d4[2];
#pragma unroll
        for (int h4 = 0; h4 < 2; ++h4) {
          a4[h4] = *reinterpret_cast<const f32x4*>(&sCo[kk * 8 + 4 * h4]);
          b4[h4] = *reinterpret_cast<const f32x4*>(&sCo[COUT + kk * 8 + 4 * h4]);
          d4[h4] = *reinterpret_cast<const f32x4*>(&sCo[2 * COUT + kk * 8 + 4 * h4]);
        }
#pragma unroll
        for (int k = j3; k < 6; k += 3) {
          const int c = tid + 512 * k, px = c / 12;
          const E8 y8 = __builtin_bit_cast(E8, rx[k]);
          E8 o8;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float z = fmaxf(__builtin_fmaf((float)y8[j], a4[j >> 2][j & 3], b4[j >> 2][j & 3]), 0.f);
            o8[j] = (E)pin_f32(z * d4[j >> 2][j & 3]);
          }
          *reinterpret_cast<u32x4*>(&sX[(((px >> 4) + 1) * 18 + (px & 15) + 1) * COUT + kk * 8]) =
              __builtin_bit_cast(u32x4, o8);
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int c = tid + 512 * k, px = c / 12, kk = c - px * 12;
        *reinterpret_cast<u32x4*>(&sX[(((px >> 4) + 1) * 18 + (px & 15) + 1) * COUT + kk * 8]) = rx[k];
      }
    }
  };
  int buf = 0;
  issue(gid, 0);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (a builtin, so that the compiler's own count sees it)
  if constexpr (GN) {
    put_co();
    __syncthreads();  // sCo complete
  }
  put_x();
  __syncthreads();
  for (int n = gid; n < p.N; n += p.G, buf ^= 1) {
    issue(n + p.G, buf ^ 1);
    asm volatile("" ::: "memory");  // the prefetch is issued before the MFMA loop
    const E* D = sDY + buf * WC_DY;
    auto ld = [&](int k0, E8 (&a)[3], E8 (&b)[4]) {
#pragma unroll
      for (int cot = 0; cot < 3; ++cot) {
        const E* base = D + (k0 + rowoff) * COUT + cot * 32 + col;
        a[cot] = cat8(lds_tr4(base), lds_tr4(base + 4 * COUT));
      }
      const int px0 = k0 + rowoff, px1 = px0 + 4;
      const int h0 = ((px0 >> 4) + 1) * 18 + (px0 & 15) + 1, h1 = ((px1 >> 4) + 1) * 18 + (px1 & 15) + 1;
#pragma unroll
      for (int bi = 0; bi < 4; ++bi) {
        const int tap = T::tap(bi), toff = ((tap / 3 - 1) * 18 + (tap % 3 - 1)) * COUT + T::cis(bi) * 32 + col;
        b[bi] = cat8(lds_tr4(sX + h0 * COUT + toff), lds_tr4(sX + h1 * COUT + toff));
      }
    };
    auto mm = [&](const E8 (&a)[3], const E8 (&b)[4]) {
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma32(a[T::co(t)], b[T::b(t)], acc[t]);
    };
    if constexpr (NT == 10) {
      // operands double-buffered: step k+1's 14 reads spread between step k's MFMAs
      E8 a0[3], b0[4], a1[3], b1[4];
      ld(0, a0, b0);
      __builtin_amdgcn_sched_group_barrier(0x100, 14, 0);
#pragma unroll
      for (int k0 = 0; k0 < 256; k0 += 32) {
        ld(k0 + 16, a1, b1);
        mm(a0, b0);
        pin_reads_mfma<14, NT>();
        if (k0 + 32 < 256) {
          ld(k0 + 32, a0, b0);
          mm(a1, b1);
          pin_reads_mfma<14, NT>();
        } else {
          mm(a1, b1);
          pin_reads_mfma<0, NT>();
        }
      }
    } else {
      // wave 0 (11 tiles): one step's operands live at a time (176 accumulators and the x
      // prefetch leave no room for two); its SIMD partner covers the read latency
#pragma unroll
      for (int k0 = 0; k0 < 256; k0 += 16) {
        E8 a[3], b[4];
        ld(k0, a, b);
        mm(a, b);
        __builtin_amdgcn_sched_group_barrier(0x100, 14, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, NT, 0);
      }
    }
    if constexpr (CO) {  // sample n + G's coefficients (its loads were issued with the prefetch)
      if (n + p.G < p.N) put_co();
    }
    __syncthreads();  // sX and sDY[buf] are free; sCo holds sample n + G's coefficients
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's DMA and x loads have landed
    if (n + p.G < p.N) put_x();
    __syncthreads();  // sX and sDY[buf ^ 1] (every wave's DMA) complete
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int tap = T::tap(T::b(t)), ci = T::cis(T::b(t)) * 32 + (lane & 31), cot = T::co(t);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = cot * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      p.part[(((size_t)gid * 9 + tap) * COUT + co) * 96 + ci] = acc[t][r];
    }
  }
}

template <typename E, bool GN>
__global__ __launch_bounds__(512, 1) void k_wgrad_c96(WgradParams<E> p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  E* sDY = reinterpret_cast<E*>(smem);  // [2][256][96]
  E* sX = sDY + 2 * WC_DY;              // [18 * 18][96], zero halo
  float* sCo = reinterpret_cast<float*>(sX + WC_SX);  // [3][96] (GN)
  for (int i = threadIdx.x; i < WC_SX / 8; i += 512) *reinterpret_cast<u32x4*>(&sX[i * 8]) = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  const int gid = blockIdx.x;
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
    case 0: wgc_body<E, 0, GN>(p, sDY, sX, sCo, gid); break;
    case 1: wgc_body<E, 1, GN>(p, sDY, sX, sCo, gid); break;
    case 2: wgc_body<E, 2, GN>(p, sDY, sX, sCo, gid); break;
    case 3: wgc_body<E, 3, GN>(p, sDY, sX, sCo, gid); break;
    case 4: wgc_body<E, 4, GN>(p, sDY, sX, sCo, gid); break;
    case 5: wgc_body<E, 5, GN>(p, sDY, sX, sCo, gid); break;
    case 6: wgc_body<E, 6, GN>(p, sDY, sX, sCo, gid); break;
    default: wgc_body<E, 7, GN>(p, sDY, sX, sCo, gid); break;
  }
}

// out[i] = sum_g part[g * n + i], deterministic: a 256-thread block covers 256 / S outputs
// with S slices over g (slice s sums g = s, s + S, ... on four independent accumulators,
// so a thread keeps four loads in flight), slices combined in fixed order through LDS.
// S = 4 for the weight partials (n = 82,944, G = 168), 16 for the 288 GroupNorm sums.
template <int S>
__global__ __launch_bounds__(256) void k_reduce(const float* __restrict__ part, int G, int64_t n, float* __restrict__ out) {
  constexpr int IB = 256 / S;
  __shared__ float sp[S][IB];
  const int li = threadIdx.x % IB, s = threadIdx.x / IB;
  const int64_t i = (int64_t)blockIdx.x * IB + li;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (i < n) {
    int g = s;
    for (; g + 3 * S < G; g += 4 * S) {
      a0 += part[(int64_t)g * n + i];
      a1 += part[(int64_t)(g + S) * n + i];
      a2 += part[(int64_t)(g + 2 * S) * n + i];
      a3 += part[(int64_t)(g + 3 * S) * n + i];
    }
    for (; g < G; g += S) a0 += part[(int64_t)g * n + i];
  }
  sp[s][li] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (s == 0 && i < n) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < S; ++k) t += sp[k][li];
    out[i] = t;
  }
}

void launch_reduce(const float* part, int G, int64_t n, float* out, hipStream_t s) {
  if (n >= 16384) hipLaunchKernelGGL(k_reduce<4>, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, s, part, G, n, out);
  else hipLaunchKernelGGL(k_reduce<16>, dim3((unsigned)((n + 15) / 16)), dim3(256), 0, s, part, G, n, out);
}

// ------------------------------------------------------------------------------------
struct Plan {
  bool c96 = false;  // k_wgrad_c96 (16x16 boards, 96 channels; the default there)
  int grid_d, grid_w, G;
  int64_t gn_part, w_part;
};

// force_c96: mc_conv_wgrad_gn, which only k_wgrad_c96 implements (the forward that skipped the
// conv1 outputs may have run under another weight-gradient variant: ADVICE r05)
Plan make_plan(int n, int h, int w, int cin, bool force_c96 = false) {
  Plan pl;
  const int ncu = num_cus();
  pl.grid_d = n < 2 * ncu ? n : 2 * ncu;
  const int nci = cin == 96 ? 3 : 1;
  int J = (2 * ncu) / (8 * nci);
  if (J < 1) J = 1;
  pl.G = 8 * J;
  pl.grid_w = 8 * nci * J;
  int gmax = pl.G;
  // 16x16 boards, 96 channels, variant 3: k_wgrad_c96, one workgroup (partial row) per CU
  if (cin == 96 && h == 16 && w == 16) {
    if (ncu > gmax) gmax = ncu;
    pl.c96 = force_c96 || g_variant[MCV_WGRAD] == 0 || g_variant[MCV_WGRAD] == 3;
    if (pl.c96) pl.G = pl.grid_w = n < ncu ? n : ncu;
  }
  pl.gn_part = (int64_t)pl.grid_d * 3 * COUT;
  pl.w_part = (int64_t)gmax * 9 * COUT * cin;  // the same workspace whichever k_wgrad runs
  return pl;
}

template <typename K>
void set_lds_attr(K kernel) {
  (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

template <typename E, int NPT, bool DGRAD, int NCH, bool RM>
void launch_bwd_data_t(const BwdDataParams<E>& p, int grid, size_t lds, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    set_lds_attr(k_bwd_data<E, NPT, DGRAD, NCH, RM>);
    attr = true;
  }
  hipLaunchKernelGGL((k_bwd_data<E, NPT, DGRAD, NCH, RM>), dim3(grid), dim3(256), lds, s, p);
}

template <typename E, int NPT, bool DGRAD, int NCH>
void launch_bwd_data(const BwdDataParams<E>& p, int grid, size_t lds, hipStream_t s) {
  if (p.rmask) launch_bwd_data_t<E, NPT, DGRAD, NCH, true>(p, grid, lds, s);
  else launch_bwd_data_t<E, NPT, DGRAD, NCH, false>(p, grid, lds, s);
}

// grid: in, the per-sample kernel's grid; out, the workgroups launched (= partial rows in p.part)
template <typename E, bool DGRAD>
int dispatch_bwd_data(const BwdDataParams<E>& p, int& grid, hipStream_t s) {
  const int P = p.H * p.W;
  const size_t lds = (size_t)bwd_data_lds(P);
  if (lds > 160 * 1024) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_bwd: board %dx%d needs %zu B LDS", p.H, p.W, lds);
    return MS_EINVAL;
  }
  if (P <= 128) launch_bwd_data<E, 1, DGRAD, 13>(p, grid, lds, s);
  else if (P <= 256) launch_bwd_data<E, 2, DGRAD, 13>(p, grid, lds, s);
  else if (P <= 384) launch_bwd_data<E, 3, DGRAD, 25>(p, grid, lds, s);
  else if (P <= 512) launch_bwd_data<E, 4, DGRAD, 25>(p, grid, lds, s);
  else {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_bwd: %d pixels > 512 unsupported", P);
    return MS_EINVAL;
  }
  return MS_OK;
}

template <typename E, int CIN, bool PF, bool SG>
void launch_wgrad_t(const WgradParams<E>& p, int grid, size_t lds, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    set_lds_attr(k_wgrad<E, CIN, PF, SG>);
    attr = true;
  }
  hipLaunchKernelGGL((k_wgrad<E, CIN, PF, SG>), dim3(grid), dim3(256), lds, s, p);
}

template <typename E, int CIN>
void launch_wgrad(const WgradParams<E>& p, int grid, size_t lds, hipStream_t s) {
  // 16x16 boards with 96 channels: the register prefetch of the next sample's dy and x slice
  if constexpr (CIN == 96) {
    if (p.H == 16 && p.W == 16) {
      if (g_variant[MCV_WGRAD] == 2) return launch_wgrad_t<E, CIN, true, true>(p, grid, lds, s);
      return launch_wgrad_t<E, CIN, true, false>(p, grid, lds, s);
    }
  }
  launch_wgrad_t<E, CIN, false, false>(p, grid, lds, s);
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof g_err, "%s launch: %s", what, hipGetErrorString(e));
    return MS_EHIP;
  }
  return MS_OK;
}

struct GnApply {  // mc_conv_wgrad_gn: x recomputed from a layer's y (all null: x is given)
  const float *stats = nullptr, *gamma = nullptr, *beta = nullptr, *dmask = nullptr;
};

template <typename E, bool GN>
void launch_wgrad_c96(const WgradParams<E>& wp, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_wgrad_c96<E, GN>, hipFuncAttributeMaxDynamicSharedMemorySize, WC_LDS);
    attr = true;
  }
  hipLaunchKernelGGL((k_wgrad_c96<E, GN>), dim3(grid), dim3(512), (size_t)WC_LDS, s, wp);
}

template <typename E>
int run_wgrad(const Plan& pl, const uint16_t* dy, const uint16_t* x, float* dw, float* work, int32_t n, int32_t h,
              int32_t w_, int32_t cin, hipStream_t s, const GnApply& gn = GnApply()) {
  WgradParams<E> wp;
  wp.dy = reinterpret_cast<const E*>(dy);
  wp.x = reinterpret_cast<const E*>(x);
  wp.gn_stats = gn.stats;
  wp.gn_gamma = gn.gamma;
  wp.gn_beta = gn.beta;
  wp.gn_dmask = gn.dmask;
  wp.part = work + pl.gn_part;
  wp.N = n;
  wp.H = h;
  wp.W = w_;
  wp.G = pl.G;
  const size_t lds = (size_t)wgrad_lds(h, w_);
  if (pl.c96) {
    if (gn.stats) launch_wgrad_c96<E, true>(wp, pl.grid_w, s);
    else launch_wgrad_c96<E, false>(wp, pl.grid_w, s);
  } else if (cin == 96) launch_wgrad<E, 96>(wp, pl.grid_w, lds, s);
  else launch_wgrad<E, 16>(wp, pl.grid_w, lds, s);
  int rc;
  if ((rc = check_launch("k_wgrad"))) return rc;
  const int64_t nw = (int64_t)9 * COUT * cin;
  launch_reduce((const float*)(work + pl.gn_part), pl.G, nw, dw, s);
  return check_launch("k_reduce");
}

template <typename E>
int run_bwd(const uint16_t* dout, const uint16_t* out, const uint8_t* relu_mask, const uint16_t* ysave,
            const float* stats, const float* gamma, const float* dmask, const uint16_t* x, const uint16_t* wT,
            const uint16_t* addend, uint16_t* dy, uint16_t* dz, uint16_t* dx, float* dw, float* dgn, float* work,
            int32_t n, int32_t h, int32_t w_, int32_t cin, hipStream_t s) {
  const Plan pl = make_plan(n, h, w_, cin);
  BwdDataParams<E> bp;
  bp.dout = reinterpret_cast<const E*>(dout);
  bp.out = reinterpret_cast<const E*>(out);
  bp.rmask = relu_mask;
  bp.y = reinterpret_cast<const E*>(ysave);
  bp.stats = stats;
  bp.gamma = gamma;
  bp.dmask = dmask;
  bp.wT = reinterpret_cast<const E*>(wT);
  bp.addend = reinterpret_cast<const E*>(addend);
  bp.dy = reinterpret_cast<E*>(dy);
  bp.dz = reinterpret_cast<E*>(dz);
  bp.dx = reinterpret_cast<E*>(dx);
  bp.part = work;
  bp.N = n;
  bp.H = h;
  bp.W = w_;
  int grid_d = pl.grid_d;
  int rc = wT ? dispatch_bwd_data<E, true>(bp, grid_d, s) : dispatch_bwd_data<E, false>(bp, grid_d, s);
  if (rc) return rc;
  if ((rc = check_launch("k_bwd_data"))) return rc;
  launch_reduce((const float*)work, grid_d, (int64_t)3 * COUT, dgn, s);
  if ((rc = check_launch("k_reduce"))) return rc;
  return run_wgrad<E>(pl, dy, x, dw, work, n, h, w_, cin, s);
}

}  // namespace

extern "C" {


int64_t mc_conv_gn_bwd_workspace(int32_t n, int32_t h, int32_t w_, int32_t cin) {
  if (n <= 0 || h <= 0 || w_ <= 0 || (cin != 16 && cin != 96)) return -1;
  const Plan pl = make_plan(n, h, w_, cin);
  return pl.gn_part + pl.w_part;
}

int mc_conv_wgrad(const uint16_t* dy, const uint16_t* x, float* dw, float* work, int64_t work_floats, int32_t n,
                  int32_t h, int32_t w_, int32_t cin, int32_t dtype, void* stream) {
  if (!dy || !x || !dw || !work || n <= 0 || h <= 0 || w_ <= 0 || (cin != 16 && cin != 96)) {
    snprintf(g_err, sizeof g_err, "mc_conv_wgrad: bad argument");
    return MS_EINVAL;
  }
  const Plan pl = make_plan(n, h, w_, cin);
  if (work_floats < pl.gn_part + pl.w_part) {
    snprintf(g_err, sizeof g_err, "mc_conv_wgrad: workspace %lld < %lld floats", (long long)work_floats,
             (long long)(pl.gn_part + pl.w_part));
    return MS_EINVAL;
  }
  if (wgrad_lds(h, w_) > 160 * 1024) {
    snprintf(g_err, sizeof g_err, "mc_conv_wgrad: board %dx%d too large", h, w_);
    return MS_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MC_DT_BF16) return run_wgrad<__bf16>(pl, dy, x, dw, work, n, h, w_, cin, s);
  if (dtype == MC_DT_F16) return run_wgrad<_Float16>(pl, dy, x, dw, work, n, h, w_, cin, s);
  snprintf(g_err, sizeof g_err, "mc_conv_wgrad: dtype %d unsupported (0 bf16, 1 f16)", dtype);
  return MS_EINVAL;
}

int mc_conv_wgrad_gn(const uint16_t* dy, const uint16_t* y, const float* stats, const float* gamma, const float* beta,
                     const float* dmask, float* dw, float* work, int64_t work_floats, int32_t n, int32_t h, int32_t w_,
                     int32_t dtype, void* stream) {
  if (!dy || !y || !stats || !gamma || !beta || !dw || !work || n <= 0 || h <= 0 || w_ <= 0) {
    snprintf(g_err, sizeof g_err, "mc_conv_wgrad_gn: bad argument");
    return MS_EINVAL;
  }
  const Plan pl = make_plan(n, h, w_, 96, true);
  if (!pl.c96) {
    snprintf(g_err, sizeof g_err, "mc_conv_wgrad_gn: needs k_wgrad_c96 (16x16 boards with 96 channels)");
    return MS_EINVAL;
  }
  if (work_floats < pl.gn_part + pl.w_part) {
    snprintf(g_err, sizeof g_err, "mc_conv_wgrad_gn: workspace %lld < %lld floats", (long long)work_floats,
             (long long)(pl.gn_part + pl.w_part));
    return MS_EINVAL;
  }
  GnApply gn;
  gn.stats = stats;
  gn.gamma = gamma;
  gn.beta = beta;
  gn.dmask = dmask;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MC_DT_BF16) return run_wgrad<__bf16>(pl, dy, y, dw, work, n, h, w_, 96, s, gn);
  if (dtype == MC_DT_F16) return run_wgrad<_Float16>(pl, dy, y, dw, work, n, h, w_, 96, s, gn);
  snprintf(g_err, sizeof g_err, "mc_conv_wgrad_gn: dtype %d unsupported (0 bf16, 1 f16)", dtype);
  return MS_EINVAL;
}

int mc_conv_gn_bwd(const uint16_t* dout, const uint16_t* out, const uint8_t* relu_mask, const uint16_t* ysave,
                   const float* stats,
                   const float* gamma, const float* dmask, const uint16_t* x, const uint16_t* wT,
                   const uint16_t* addend, uint16_t* dy, uint16_t* dz, uint16_t* dx, float* dw, float* dgn,
                   float* work, int64_t work_floats, int32_t n, int32_t h, int32_t w_, int32_t cin,
                   int32_t dtype, void* stream) {
  if (!dout || (!out && !relu_mask) || !ysave || !stats || !gamma || !x || !dy || !dw || !dgn || !work || n <= 0 || h <= 0 ||
      w_ <= 0) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_bwd: bad argument");
    return MS_EINVAL;
  }
  if (cin != 16 && cin != 96) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_bwd: cin %d unsupported (16 or 96)", cin);
    return MS_EINVAL;
  }
  if ((wT == nullptr) != (dx == nullptr) || (wT && cin != 96) || (addend && !wT)) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_bwd: dx needs wT (and cin 96); addend needs dx");
    return MS_EINVAL;
  }
  const Plan pl = make_plan(n, h, w_, cin);
  if (work_floats < pl.gn_part + pl.w_part) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_bwd: workspace %lld < %lld floats", (long long)work_floats,
             (long long)(pl.gn_part + pl.w_part));
    return MS_EINVAL;
  }
  if (wgrad_lds(h, w_) > 160 * 1024) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_bwd: board %dx%d too large", h, w_);
    return MS_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MC_DT_BF16)
    return run_bwd<__bf16>(dout, out, relu_mask, ysave, stats, gamma, dmask, x, wT, addend, dy, dz, dx, dw, dgn, work, n, h,
                           w_, cin, s);
  if (dtype == MC_DT_F16)
    return run_bwd<_Float16>(dout, out, relu_mask, ysave, stats, gamma, dmask, x, wT, addend, dy, dz, dx, dw, dgn, work, n,
                             h, w_, cin, s);
  snprintf(g_err, sizeof g_err, "mc_conv_gn_bwd: dtype %d unsupported (0 bf16, 1 f16)", dtype);
  return MS_EINVAL;
}

}  // extern "C"
