// mscnn_trunk.hip — the whole residual stack in one launch per direction (gfx950 MFMA).
//
// Reference chain (minesweeper/models/cnn_residual.py:7-27, 55-56): `blocks` x
//   a1  = Dropout2d(ReLU(GN1(conv1(x))))
//   out = ReLU(GN2(conv2(a1)) + x)
// mscnn.hip / mscnn_bwd.hip run one launch per conv layer: every layer reads its input and
// residual from HBM and writes its output back, and every layer backward reads dout and writes
// dx, so the activations make one HBM round trip per layer and direction. Here one persistent
// workgroup (4 waves) carries a sample through ALL the layers, and a layer's output goes
// straight into the LDS tile the next layer's implicit GEMM reads:
//
//   k_trunk_fwd  per sample: stage block 0's input once; per layer: 9-tap implicit GEMM on
//                v_mfma_f32_32x32x16 (the per-layer kernel's tap loop), GroupNorm statistics,
//                y -> LDS, epilogue (affine, residual, ReLU, dropout) written IN PLACE over the
//                input tile (the layouts coincide: [P+1][104] padded rows), stored to HBM only
//                where the backward or the caller needs it (y, out, ReLU bits, statistics).
//                The block input needed by conv2's residual is re-read from the block output
//                the workgroup wrote two layers earlier (L2 / Infinity Cache); without saved
//                outputs (no-grad forward) it goes to a per-workgroup slot of the workspace.
//   k_trunk_bwd  per sample, layers in reverse: GroupNorm backward (pass 1: dz and channel
//                sums; pass 2: dy to LDS and to HBM for the weight gradient), then the data
//                gradient dx = sum_tap shift(dy) . W^T on the MFMA, staged in LDS where the
//                NEXT layer's pass 1 reads it as its dout. The skip gradient of a block (dz of
//                its conv2) is added where the block input's gradient is formed, two layers
//                later: it waits in registers (boards of <= 256 cells: each lane keeps the 48
//                channels of its pixels that it writes as dx) or in a per-workgroup slot of
//                the workspace (larger boards, no registers to spare). The stem's GroupNorm
//                backward closes the chain (its input needs no gradient). d gamma / d beta /
//                d bias per layer accumulate per workgroup (fixed sample order) and are summed
//                over workgroups by k_reduce: deterministic.
//
// Every arithmetic step is the per-layer kernels' (same accumulation order, same roundings to
// the 16-bit type at the same points), so the outputs are bitwise those of the per-layer path
// (tests/test_trunk_gpu.py). The weight gradients stay per-layer launches (mc_conv_wgrad).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <type_traits>

#include "../../include/msenv.h"
#include "../../include/mscnn.h"
#include "mscnn_common.h"

namespace {

using namespace mc;

constexpr int CINP = COUT + 8;  // padded pixel row (elements): conflict-free ds_read_b128 row reads
constexpr int C8 = COUT / 8;    // 16-B chunks per pixel row
constexpr int MAXL = MC_TRUNK_MAX_LAYERS;

template <typename E>
struct TFLayer {
  const E* wt;          // [9][96][96] (tap, co, ci)
  const float* bias;    // [96]
  const float* gamma;   // [96]
  const float* beta;    // [96]
  const float* dmask;   // [N][96] Dropout2d scale (0 or 1/(1-p)) after the ReLU, or NULL
  E* out;               // [N][P][96] or NULL
  E* ysave;             // [N][P][96] or NULL
  float* stats;         // [N][6][2] (mean, rstd) or NULL
  uint8_t* rmask;       // [N][P][12] ReLU bits or NULL
};

#ifdef MC_DIAG
#define TSTAMP(k)                                               \
  do {                                                          \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    dacc[k] += t_ - tlast;                                      \
    tlast = t_;                                                 \
  } while (0)
#else
#define TSTAMP(k) do { } while (0)
#endif

template <typename E>
struct TrunkFwdParams {
  const E* x0;  // [N][P][96] block 0's input
  E* ws;        // [grid][P][96]: block outputs that are not kept (residual of the next block)
  unsigned long long* diag;  // MC_DIAG builds: per-wave phase cycle totals [grid][4][8]
#ifdef MC_DIAG
  int dflags;  // timing experiments only: bit 0 drops the epilogue's global stores
#endif
  float* pooled;  // [N][96] or null: the last layer's output averaged over the pixels
  int NL, N, H, W;
  float eps;
  TFLayer<E> L[MAXL];
};

// The value head's global average pool (cnn_residual.py:65, AdaptiveAvgPool2d(1)) of the
// last layer's output tile while it is still in LDS: threads c + 96 h (h = 0, 1) sum channel c
// over pixel half h on four interleaved f32 accumulators, the halves combine in fixed order
// through sTmp ([2][96] f32), and the sum is scaled by 1 / P. Every thread of the workgroup
// calls it (one barrier); out == null stores nothing.
template <typename E>
__device__ __forceinline__ void pool_tile(const E* sX, float* sTmp, int P, int tid, float* out) {
  if (tid < 2 * COUT) {
    const int c = tid % COUT, h = tid / COUT, half = (P + 1) >> 1;
    const int p1 = h ? P : half;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int px = h ? half : 0;
    for (; px + 3 < p1; px += 4) {
      a0 += (float)sX[px * CINP + c];
      a1 += (float)sX[(px + 1) * CINP + c];
      a2 += (float)sX[(px + 2) * CINP + c];
      a3 += (float)sX[(px + 3) * CINP + c];
    }
    for (; px < p1; ++px) a0 += (float)sX[px * CINP + c];
    sTmp[h * COUT + c] = (a0 + a1) + (a2 + a3);
  }
  __syncthreads();
  if (out && tid < COUT) out[tid] = (sTmp[tid] + sTmp[COUT + tid]) * (1.0f / (float)P);
}

__host__ __device__ inline int tf_region(int P) { return ((P + 1) * CINP + 7) & ~7; }
__host__ __device__ inline size_t tf_lds(int P) {
  return (size_t)tf_region(P) * 2 + (size_t)COUT * CINP * 2 + WAVES * NGRP * 4 + 3 * COUT * 4;
}

// 16-B chunk k of this thread's share of a [P][96] tile: c = tid + 256k, pixel c / 12, chunk c % 12
template <typename E, int NWC>
__device__ __forceinline__ void load_wtap(const E* wt, int tap, int tid, u32x4 (&v)[NWC]) {
  const u32x4* ws = reinterpret_cast<const u32x4*>(wt + (size_t)tap * COUT * COUT);
#pragma unroll
  for (int k = 0; k < NWC; ++k) {
    const int i = tid + 256 * k;
    if (k < COUT * C8 / 256 || i < COUT * C8) v[k] = ws[i];  // the first 4 chunks are always full
  }
}
template <typename E, int NWC>
__device__ __forceinline__ void store_wtap(E* sW, int tid, const u32x4 (&v)[NWC]) {
#pragma unroll
  for (int k = 0; k < NWC; ++k) {
    const int i = tid + 256 * k;
    if (k < COUT * C8 / 256 || i < COUT * C8) {
      const int r = i / C8, c = i - r * C8;
      *reinterpret_cast<u32x4*>(&sW[r * CINP + c * 8]) = v[k];
    }
  }
}

// LDS: sX [P+1][104] (row P zero): the layer's input tile; after its conv the same bytes hold y,
// then the layer's output (the next layer's input). sW [96][104]: one weight tap.
// f32 sRed [4][6] (statistics exchange), sAB [3][96] (scale, shift, dropout scale).
template <typename E, int NPT, bool FULL>
__global__ __launch_bounds__(256, NPT <= 2 ? 2 : 1) void k_trunk_fwd(TrunkFwdParams<E> p) {
  // no contraction: every expression rounds the same way in the per-layer and the one-launch
  // kernels (explicit fmaf where a fused multiply-add is wanted), so they agree bitwise
#pragma clang fp contract(off)
  typedef typename EV<E>::v8 E8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NEC = (NPT * 128 * C8 + 255) / 256;  // 16-B chunks of a sample tile per thread
  constexpr int NWC = (COUT * C8 + 255) / 256;       // 16-B chunks of a weight tap per thread
  const int H = p.H, W = p.W, P = H * W;
  E* sX = reinterpret_cast<E*>(smem);
  E* sW = sX + tf_region(P);
  float* sRed = reinterpret_cast<float*>(sW + COUT * CINP);
  float* sAB = sRed + WAVES * NGRP;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const float inv_cnt = 1.0f / (16.0f * (float)P);

  int qr[NPT], qc[NPT];  // this lane's output pixel of each 32-pixel tile
#pragma unroll
  for (int t = 0; t < NPT; ++t) {
    const int q = (wave * NPT + t) * 32 + l32;
    qr[t] = q < P ? q / W : -1000;  // a pixel past P reads the zero row at every tap
    qc[t] = q < P ? q - qr[t] * W : -1000;
  }
  u32x4 wr[NWC];
#ifdef MC_DIAG
  unsigned long long dacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif

  for (int n = blockIdx.x; n < p.N; n += gridDim.x) {
    const size_t so = (size_t)n * P * COUT;  // this sample's offset in every [N][P][96] tensor
    {  // stage block 0's input and layer 0's tap-0 weights
      const int tid = threadIdx.x + opaque0();
      u32x4 xin[NEC];
      const u32x4* xs = reinterpret_cast<const u32x4*>(p.x0 + so);
#pragma unroll
      for (int k = 0; k < NEC; ++k) {
        const int i = tid + 256 * k;
        if (FULL || i < P * C8) xin[k] = xs[i];
      }
      load_wtap<E, NWC>(p.L[0].wt, 0, tid, wr);
      for (int i = tid; i < C8; i += 256) *reinterpret_cast<u32x4*>(&sX[P * CINP + i * 8]) = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int k = 0; k < NEC; ++k) {
        const int i = tid + 256 * k;
        if (FULL || i < P * C8) {
          const int px = i / C8, c8 = i - px * C8;
          *reinterpret_cast<u32x4*>(&sX[px * CINP + c8 * 8]) = xin[k];
        }
      }
      store_wtap<E, NWC>(sW, tid, wr);
    }
    __syncthreads();

    for (int l = 0; l < p.NL; ++l) {
      // loop-variant thread coordinates: the per-chunk address math and the taps' row offsets
      // are recomputed per layer instead of hoisted out of this loop (they would be spilled)
      const int tid = threadIdx.x + opaque0();
#pragma unroll
      for (int t = 0; t < NPT; ++t) asm volatile("" : "+v"(qr[t]), "+v"(qc[t]));
      const E* wt = p.L[l].wt;
      float biasv[3];
#pragma unroll
      for (int ct = 0; ct < 3; ++ct) biasv[ct] = p.L[l].bias[ct * 32 + l32];

      f32x16 acc[NPT][3];
#pragma unroll
      for (int t = 0; t < NPT; ++t)
#pragma unroll
        for (int ct = 0; ct < 3; ++ct)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[t][ct][i] = 0.f;

      TSTAMP(0);
      for (int tap = 0; tap < 9; ++tap) {
        if (tap + 1 < 9) load_wtap<E, NWC>(wt, tap + 1, tid, wr);
        const int dr = tap / 3 - 1, dc = tap % 3 - 1;
        int aoff[NPT];
#pragma unroll
        for (int t = 0; t < NPT; ++t) {
          const int sr = qr[t] + dr, sc = qc[t] + dc;
          const bool v = (unsigned)sr < (unsigned)H && (unsigned)sc < (unsigned)W;
          aoff[t] = (v ? sr * W + sc : P) * CINP + 8 * hh;
        }
        // 6 k steps, operands double-buffered, order pinned: step k+1's LDS reads before step k's MFMAs
        constexpr int KS = COUT / 16;
        E8 A[2][NPT], B[2][3];
        auto ld = [&](int ks, E8 (&a)[NPT], E8 (&b)[3]) {
#pragma unroll
          for (int ct = 0; ct < 3; ++ct)
            b[ct] = *reinterpret_cast<const E8*>(&sW[(ct * 32 + l32) * CINP + ks * 16 + 8 * hh]);
#pragma unroll
          for (int t = 0; t < NPT; ++t) a[t] = *reinterpret_cast<const E8*>(&sX[aoff[t] + ks * 16]);
        };
        ld(0, A[0], B[0]);
        __builtin_amdgcn_sched_group_barrier(0x100, NPT + 3, 0);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          if (ks + 1 < KS) {
            ld(ks + 1, A[(ks + 1) & 1], B[(ks + 1) & 1]);
            __builtin_amdgcn_sched_group_barrier(0x100, NPT + 3, 0);
          }
#pragma unroll
          for (int t = 0; t < NPT; ++t)
#pragma unroll
            for (int ct = 0; ct < 3; ++ct) acc[t][ct] = mfma32(A[ks & 1][t], B[ks & 1][ct], acc[t][ct]);
          __builtin_amdgcn_sched_group_barrier(0x008, 3 * NPT, 0);
        }
        __syncthreads();  // sW (and after the last tap sX) fully read
        if (tap + 1 < 9) {
          store_wtap<E, NWC>(sW, tid, wr);
          __syncthreads();
        }
      }
      TSTAMP(1);
      // the next layer's tap-0 weights: loaded now, written to sW (free) after the statistics
      const bool more = l + 1 < p.NL;
      if (more) load_wtap<E, NWC>(p.L[l + 1].wt, 0, tid, wr);

      // ---------------- GroupNorm statistics (two-pass, as the per-layer kernel) ----------------
      float gmean[NGRP], grstd[NGRP];
      for (int pass = 0; pass < 2; ++pass) {
        float part[3];
#pragma unroll
        for (int ct = 0; ct < 3; ++ct) {
          const float mu = pass ? gmean[2 * ct + (l32 >> 4)] : 0.f;
          float v[NPT * 16];
#pragma unroll
          for (int t = 0; t < NPT; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int px = (wave * NPT + t) * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
              const float d = acc[t][ct][i] + biasv[ct] - mu;
              v[t * 16 + i] = (FULL || px < P) ? (pass ? d * d : d) : 0.f;
            }
#pragma unroll
          for (int w2 = NPT * 8; w2 >= 1; w2 >>= 1)
#pragma unroll
            for (int i = 0; i < w2; ++i) v[i] += v[i + w2];
          part[ct] = row_sum16(v[0]);
        }
        float gs[3][2];
#pragma unroll
        for (int ct = 0; ct < 3; ++ct) {
          gs[ct][0] = readlane_f(part[ct], 15) + readlane_f(part[ct], 47);
          gs[ct][1] = readlane_f(part[ct], 31) + readlane_f(part[ct], 63);
        }
        if (lane == 0) {
#pragma unroll
          for (int ct = 0; ct < 3; ++ct) {
            sRed[wave * NGRP + 2 * ct] = gs[ct][0];
            sRed[wave * NGRP + 2 * ct + 1] = gs[ct][1];
          }
        }
        __syncthreads();
#pragma unroll
        for (int g = 0; g < NGRP; ++g) {
          float tot = 0.f;
#pragma unroll
          for (int w = 0; w < WAVES; ++w) tot += sRed[w * NGRP + g];
          if (pass == 0) gmean[g] = tot * inv_cnt;
          else grstd[g] = rsqrtf(tot * inv_cnt + p.eps);
        }
        __syncthreads();  // sRed reused by the next pass
      }
      TSTAMP(2);
      float* stats = p.L[l].stats;
      if (stats && tid < NGRP) {
        float m = 0.f, r = 0.f;
#pragma unroll
        for (int g = 0; g < NGRP; ++g)
          if (g == tid) {
            m = gmean[g];
            r = grstd[g];
          }
        stats[((size_t)n * NGRP + tid) * 2 + 0] = m;
        stats[((size_t)n * NGRP + tid) * 2 + 1] = r;
      }
      // y -> LDS over the (fully read) input tile, in the tile's padded layout
#pragma unroll
      for (int ct = 0; ct < 3; ++ct)
#pragma unroll
        for (int t = 0; t < NPT; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int px = (wave * NPT + t) * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
            if (FULL || px < P) sX[px * CINP + ct * 32 + l32] = (E)pin_f32(acc[t][ct][i] + biasv[ct]);
          }
      if (more) store_wtap<E, NWC>(sW, tid, wr);
      if (tid < COUT) {  // z = y * scale + shift (+ res), then ReLU, then * dropout scale
        const int g = tid >> 4;
        float mu = 0.f, rs = 0.f;
#pragma unroll
        for (int gg = 0; gg < NGRP; ++gg)
          if (gg == g) {
            mu = gmean[gg];
            rs = grstd[gg];
          }
        const float a = p.L[l].gamma[tid] * rs;
        sAB[tid] = a;
        sAB[COUT + tid] = p.L[l].beta[tid] - mu * a;
        const float* dmask = p.L[l].dmask;
        sAB[2 * COUT + tid] = dmask ? dmask[(size_t)n * COUT + tid] : 1.0f;
      }
      __syncthreads();
      TSTAMP(3);

      // ---------------- epilogue: 16-B chunks of [px][co], written in place ----------------
      // residual (conv2 of block b): the block input = block 0's input, or block b-1's output
      const E* res = nullptr;
      if (l & 1) {
        if (l == 1) res = p.x0 + so;
        else res = p.L[l - 2].out ? p.L[l - 2].out + so : p.ws + (size_t)blockIdx.x * P * COUT;
      }
      E* out = p.L[l].out ? p.L[l].out + so : nullptr;
      if (!out && (l & 1) && more) out = p.ws + (size_t)blockIdx.x * P * COUT;  // the next block's residual
      E* ysave = p.L[l].ysave ? p.L[l].ysave + so : nullptr;
      uint8_t* rmask = p.L[l].rmask ? p.L[l].rmask + (size_t)n * P * C8 : nullptr;
#ifdef MC_DIAG
      if (p.dflags & 1) {
        out = nullptr;
        ysave = nullptr;
        rmask = nullptr;
      }
#endif
      float ca[3][8], cb[3][8], cd[3][8];
#pragma unroll
      for (int j3 = 0; j3 < 3; ++j3) {
        const int cg = ((tid % C8) + 4 * j3) % C8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          ca[j3][j] = sAB[cg * 8 + j];
          cb[j3][j] = sAB[COUT + cg * 8 + j];
          cd[j3][j] = sAB[2 * COUT + cg * 8 + j];
        }
      }
      // residual chunks are loaded RB at a time, all of a batch before its first store (a load
      // issued after a store waits for that store too: vmcnt counts both)
      constexpr int RB = (NEC + 1) / 2;
      u32x4 rq[RB];
#pragma unroll
      for (int k = 0; k < NEC; ++k) {
        const int c = tid + 256 * k;
        if (k % RB == 0) {
#pragma unroll
          for (int u = 0; u < RB; ++u) {
            const int cu = tid + 256 * (k + u);
            rq[u] = u32x4{0u, 0u, 0u, 0u};
            if (res && k + u < NEC && (FULL || cu < P * C8)) rq[u] = *reinterpret_cast<const u32x4*>(&res[(size_t)cu * 8]);
          }
        }
        if (FULL || c < P * C8) {
          const int px = c / C8, c8 = c - px * C8;
          E* sp = &sX[px * CINP + c8 * 8];
          const u32x4 yv = *reinterpret_cast<const u32x4*>(sp);
          if (ysave) *reinterpret_cast<u32x4*>(&ysave[(size_t)c * 8]) = yv;
          const E8 y8 = __builtin_bit_cast(E8, yv);
          const E8 r8 = __builtin_bit_cast(E8, rq[k % RB]);
          E8 o8;
          uint32_t mb = 0u;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float z = fmaxf(__builtin_fmaf((float)y8[j], ca[k % 3][j], cb[k % 3][j]) + (float)r8[j], 0.f);
            o8[j] = (E)pin_f32(z * cd[k % 3][j]);
            mb |= ((float)o8[j] > 0.f ? 1u : 0u) << j;
          }
          const u32x4 ov = __builtin_bit_cast(u32x4, o8);
          if (out) *reinterpret_cast<u32x4*>(&out[(size_t)c * 8]) = ov;
          if (rmask) rmask[c] = (uint8_t)mb;
          *reinterpret_cast<u32x4*>(sp) = ov;  // the next layer's input
        }
      }
      __syncthreads();  // the tile and sAB are complete / free
      TSTAMP(4);
    }
    if (p.pooled) pool_tile(sX, sAB, P, threadIdx.x, p.pooled + (size_t)n * COUT);  // (uniform)
  }
#ifdef MC_DIAG
  if (p.diag && (threadIdx.x & 63) == 0)
    for (int k = 0; k < 8; ++k) p.diag[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + k] = dacc[k];
#endif
}

// k_trunk_fwd2 (boards of <= 256 cells): one 512-thread workgroup per CU runs TWO samples, one per
// 4-wave team, through the same code in lockstep: the teams share each weight tap, which is staged
// once for both into a double buffer, so a tap costs one barrier instead of two and its hand-off
// overlaps the MFMAs (k_trunk_fwd: one sample per 256-thread workgroup, two workgroups per CU, one
// weight buffer each). Per-sample arithmetic is k_trunk_fwd's, so the outputs are bitwise equal.
// LDS: sX [2 teams][P+1][104] | sW [2 taps][96][104] | sRed [2][4][6] | sAB [2][3][96].
__host__ __device__ inline size_t tf2_lds(int P) {
  return (size_t)2 * tf_region(P) * 2 + (size_t)2 * COUT * CINP * 2 + 2 * WAVES * NGRP * 4 + 2 * 3 * COUT * 4;
}
constexpr int NWC2 = (COUT * C8 + 511) / 512;  // 16-B chunks of a weight tap per thread of 512
template <typename E>
__device__ __forceinline__ void load_wtap2(const E* wt, int tap, int tid, u32x4 (&v)[NWC2]) {
  const u32x4* ws = reinterpret_cast<const u32x4*>(wt + (size_t)tap * COUT * COUT);
#pragma unroll
  for (int k = 0; k < NWC2; ++k) {
    const int i = tid + 512 * k;
    if (k < COUT * C8 / 512 || i < COUT * C8) v[k] = ws[i];
  }
}
template <typename E>
__device__ __forceinline__ void store_wtap2(E* sW, int tid, const u32x4 (&v)[NWC2]) {
#pragma unroll
  for (int k = 0; k < NWC2; ++k) {
    const int i = tid + 512 * k;
    if (k < COUT * C8 / 512 || i < COUT * C8) {
      const int r = i / C8, c = i - r * C8;
      *reinterpret_cast<u32x4*>(&sW[r * CINP + c * 8]) = v[k];
    }
  }
}
template <typename E, int NPT, bool FULL>
__global__ __launch_bounds__(512, 1) void k_trunk_fwd2(TrunkFwdParams<E> p) {
  // no contraction: every expression rounds the same way in the per-layer and the one-launch
  // kernels (explicit fmaf where a fused multiply-add is wanted), so they agree bitwise
#pragma clang fp contract(off)
  typedef typename EV<E>::v8 E8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NEC = (NPT * 128 * C8 + 255) / 256;  // 16-B chunks of a sample tile per thread
  const int H = p.H, W = p.W, P = H * W;
  const int team = threadIdx.x >> 8;
  E* sX = reinterpret_cast<E*>(smem) + team * tf_region(P);
  E* sW0 = reinterpret_cast<E*>(smem) + 2 * tf_region(P);  // weight tap t in buffer t & 1
  float* sRed = reinterpret_cast<float*>(sW0 + 2 * COUT * CINP) + team * WAVES * NGRP;
  float* sAB = reinterpret_cast<float*>(sW0 + 2 * COUT * CINP) + 2 * WAVES * NGRP + team * 3 * COUT;
  const int lane = threadIdx.x & 63, wave = (threadIdx.x >> 6) & 3;
  const int l32 = lane & 31, hh = lane >> 5;
  const float inv_cnt = 1.0f / (16.0f * (float)P);

  int qr[NPT], qc[NPT];  // this lane's output pixel of each 32-pixel tile
#pragma unroll
  for (int t = 0; t < NPT; ++t) {
    const int q = (wave * NPT + t) * 32 + l32;
    qr[t] = q < P ? q / W : -1000;  // a pixel past P reads the zero row at every tap
    qc[t] = q < P ? q - qr[t] * W : -1000;
  }
  u32x4 wr[NWC2];
#ifdef MC_DIAG
  unsigned long long dacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif

  // team t of workgroup b takes samples 2 (b + k G) + t; an odd N leaves team 1 of the last pair
  // without one: it runs sample N - 1 alongside team 0 (every barrier is the workgroup's) and stores
  // nothing
  for (int pair = blockIdx.x; 2 * pair < p.N; pair += gridDim.x) {
    const bool valid = 2 * pair + team < p.N;
    const int n = valid ? 2 * pair + team : p.N - 1;
    const size_t so = (size_t)n * P * COUT;  // this sample's offset in every [N][P][96] tensor
    E* wsl = p.ws + ((size_t)blockIdx.x * 2 + team) * P * COUT;  // this team's workspace slot
    {  // stage block 0's input and layer 0's tap-0 weights
      const int tid = (threadIdx.x & 255) + opaque0();
      const int wid = threadIdx.x + opaque0();
      u32x4 xin[NEC];
      const u32x4* xs = reinterpret_cast<const u32x4*>(p.x0 + so);
#pragma unroll
      for (int k = 0; k < NEC; ++k) {
        const int i = tid + 256 * k;
        if (FULL || i < P * C8) xin[k] = xs[i];
      }
      load_wtap2<E>(p.L[0].wt, 0, wid, wr);
      for (int i = tid; i < C8; i += 256) *reinterpret_cast<u32x4*>(&sX[P * CINP + i * 8]) = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int k = 0; k < NEC; ++k) {
        const int i = tid + 256 * k;
        if (FULL || i < P * C8) {
          const int px = i / C8, c8 = i - px * C8;
          *reinterpret_cast<u32x4*>(&sX[px * CINP + c8 * 8]) = xin[k];
        }
      }
      store_wtap2<E>(sW0, wid, wr);
    }
    __syncthreads();

    for (int l = 0; l < p.NL; ++l) {
      // loop-variant thread coordinates: the per-chunk address math and the taps' row offsets
      // are recomputed per layer instead of hoisted out of this loop (they would be spilled)
      const int tid = (threadIdx.x & 255) + opaque0();
      const int wid = threadIdx.x + opaque0();
#pragma unroll
      for (int t = 0; t < NPT; ++t) asm volatile("" : "+v"(qr[t]), "+v"(qc[t]));
      const E* wt = p.L[l].wt;
      float biasv[3];
#pragma unroll
      for (int ct = 0; ct < 3; ++ct) biasv[ct] = p.L[l].bias[ct * 32 + l32];

      f32x16 acc[NPT][3];
#pragma unroll
      for (int t = 0; t < NPT; ++t)
#pragma unroll
        for (int ct = 0; ct < 3; ++ct)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[t][ct][i] = 0.f;

      TSTAMP(0);
      for (int tap = 0; tap < 9; ++tap) {
        if (tap + 1 < 9) load_wtap2<E>(wt, tap + 1, wid, wr);
        const E* sW = sW0 + (tap & 1) * COUT * CINP;
        const int dr = tap / 3 - 1, dc = tap % 3 - 1;
        int aoff[NPT];
#pragma unroll
        for (int t = 0; t < NPT; ++t) {
          const int sr = qr[t] + dr, sc = qc[t] + dc;
          const bool v = (unsigned)sr < (unsigned)H && (unsigned)sc < (unsigned)W;
          aoff[t] = (v ? sr * W + sc : P) * CINP + 8 * hh;
        }
        // 6 k steps, operands double-buffered, order pinned: step k+1's LDS reads before step k's MFMAs
        constexpr int KS = COUT / 16;
        E8 A[2][NPT], B[2][3];
        auto ld = [&](int ks, E8 (&a)[NPT], E8 (&b)[3]) {
#pragma unroll
          for (int ct = 0; ct < 3; ++ct)
            b[ct] = *reinterpret_cast<const E8*>(&sW[(ct * 32 + l32) * CINP + ks * 16 + 8 * hh]);
#pragma unroll
          for (int t = 0; t < NPT; ++t) a[t] = *reinterpret_cast<const E8*>(&sX[aoff[t] + ks * 16]);
        };
        ld(0, A[0], B[0]);
        __builtin_amdgcn_sched_group_barrier(0x100, NPT + 3, 0);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          if (ks + 1 < KS) {
            ld(ks + 1, A[(ks + 1) & 1], B[(ks + 1) & 1]);
            __builtin_amdgcn_sched_group_barrier(0x100, NPT + 3, 0);
          }
#pragma unroll
          for (int t = 0; t < NPT; ++t)
#pragma unroll
            for (int ct = 0; ct < 3; ++ct) acc[t][ct] = mfma32(A[ks & 1][t], B[ks & 1][ct], acc[t][ct]);
          __builtin_amdgcn_sched_group_barrier(0x008, 3 * NPT, 0);
        }
        // tap + 1 into the other buffer (last read by tap - 1, before the previous barrier)
        if (tap + 1 < 9) store_wtap2<E>(sW0 + ((tap + 1) & 1) * COUT * CINP, wid, wr);
        lds_barrier();  // tap + 1 visible; this tap's buffer (and after the last tap sX) fully read
      }
      TSTAMP(1);
      // the next layer's tap-0 weights: loaded now, written to sW (free) after the statistics
      const bool more = l + 1 < p.NL;
      if (more) load_wtap2<E>(p.L[l + 1].wt, 0, wid, wr);

      // ---------------- GroupNorm statistics (two-pass, as the per-layer kernel) ----------------
      float gmean[NGRP], grstd[NGRP];
      for (int pass = 0; pass < 2; ++pass) {
        float part[3];
#pragma unroll
        for (int ct = 0; ct < 3; ++ct) {
          const float mu = pass ? gmean[2 * ct + (l32 >> 4)] : 0.f;
          float v[NPT * 16];
#pragma unroll
          for (int t = 0; t < NPT; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int px = (wave * NPT + t) * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
              const float d = acc[t][ct][i] + biasv[ct] - mu;
              v[t * 16 + i] = (FULL || px < P) ? (pass ? d * d : d) : 0.f;
            }
#pragma unroll
          for (int w2 = NPT * 8; w2 >= 1; w2 >>= 1)
#pragma unroll
            for (int i = 0; i < w2; ++i) v[i] += v[i + w2];
          part[ct] = row_sum16(v[0]);
        }
        float gs[3][2];
#pragma unroll
        for (int ct = 0; ct < 3; ++ct) {
          gs[ct][0] = readlane_f(part[ct], 15) + readlane_f(part[ct], 47);
          gs[ct][1] = readlane_f(part[ct], 31) + readlane_f(part[ct], 63);
        }
        if (lane == 0) {
#pragma unroll
          for (int ct = 0; ct < 3; ++ct) {
            sRed[wave * NGRP + 2 * ct] = gs[ct][0];
            sRed[wave * NGRP + 2 * ct + 1] = gs[ct][1];
          }
        }
        __syncthreads();
#pragma unroll
        for (int g = 0; g < NGRP; ++g) {
          float tot = 0.f;
#pragma unroll
          for (int w = 0; w < WAVES; ++w) tot += sRed[w * NGRP + g];
          if (pass == 0) gmean[g] = tot * inv_cnt;
          else grstd[g] = rsqrtf(tot * inv_cnt + p.eps);
        }
        __syncthreads();  // sRed reused by the next pass
      }
      TSTAMP(2);
      float* stats = p.L[l].stats;
      if (stats && valid && tid < NGRP) {
        float m = 0.f, r = 0.f;
#pragma unroll
        for (int g = 0; g < NGRP; ++g)
          if (g == tid) {
            m = gmean[g];
            r = grstd[g];
          }
        stats[((size_t)n * NGRP + tid) * 2 + 0] = m;
        stats[((size_t)n * NGRP + tid) * 2 + 1] = r;
      }
      // y -> LDS over the (fully read) input tile, in the tile's padded layout
#pragma unroll
      for (int ct = 0; ct < 3; ++ct)
#pragma unroll
        for (int t = 0; t < NPT; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int px = (wave * NPT + t) * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
            if (FULL || px < P) sX[px * CINP + ct * 32 + l32] = (E)pin_f32(acc[t][ct][i] + biasv[ct]);
          }
      if (more) store_wtap2<E>(sW0, wid, wr);  // buffer 0: last read by tap 8
      if (tid < COUT) {  // z = y * scale + shift (+ res), then ReLU, then * dropout scale
        const int g = tid >> 4;
        float mu = 0.f, rs = 0.f;
#pragma unroll
        for (int gg = 0; gg < NGRP; ++gg)
          if (gg == g) {
            mu = gmean[gg];
            rs = grstd[gg];
          }
        const float a = p.L[l].gamma[tid] * rs;
        sAB[tid] = a;
        sAB[COUT + tid] = p.L[l].beta[tid] - mu * a;
        const float* dmask = p.L[l].dmask;
        sAB[2 * COUT + tid] = dmask ? dmask[(size_t)n * COUT + tid] : 1.0f;
      }
      __syncthreads();
      TSTAMP(3);

      // ---------------- epilogue: 16-B chunks of [px][co], written in place ----------------
      // residual (conv2 of block b): the block input = block 0's input, or block b-1's output
      const E* res = nullptr;
      if (l & 1) {
        if (l == 1) res = p.x0 + so;
        else res = !valid ? p.x0 + so : (p.L[l - 2].out ? p.L[l - 2].out + so : wsl);
      }
      // a team without a sample stores nothing (its residuals come from x0: any valid address;
      // with saved outputs there is no workspace)
      E* out = !valid ? nullptr : (p.L[l].out ? p.L[l].out + so : ((l & 1) && more ? wsl : nullptr));
      E* ysave = p.L[l].ysave && valid ? p.L[l].ysave + so : nullptr;
      uint8_t* rmask = p.L[l].rmask && valid ? p.L[l].rmask + (size_t)n * P * C8 : nullptr;
#ifdef MC_DIAG
      if (p.dflags & 1) {
        out = nullptr;
        ysave = nullptr;
        rmask = nullptr;
      }
#endif
      float ca[3][8], cb[3][8], cd[3][8];
#pragma unroll
      for (int j3 = 0; j3 < 3; ++j3) {
        const int cg = ((tid % C8) + 4 * j3) % C8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          ca[j3][j] = sAB[cg * 8 + j];
          cb[j3][j] = sAB[COUT + cg * 8 + j];
          cd[j3][j] = sAB[2 * COUT + cg * 8 + j];
        }
      }
      // residual chunks are loaded RB at a time, all of a batch before its first store (a load
      // issued after a store waits for that store too: vmcnt counts both)
      constexpr int RB = (NEC + 1) / 2;
      u32x4 rq[RB];
#pragma unroll
      for (int k = 0; k < NEC; ++k) {
        const int c = tid + 256 * k;
        if (k % RB == 0) {
#pragma unroll
          for (int u = 0; u < RB; ++u) {
            const int cu = tid + 256 * (k + u);
            rq[u] = u32x4{0u, 0u, 0u, 0u};
            if (res && k + u < NEC && (FULL || cu < P * C8)) rq[u] = *reinterpret_cast<const u32x4*>(&res[(size_t)cu * 8]);
          }
        }
        if (FULL || c < P * C8) {
          const int px = c / C8, c8 = c - px * C8;
          E* sp = &sX[px * CINP + c8 * 8];
          const u32x4 yv = *reinterpret_cast<const u32x4*>(sp);
          if (ysave) *reinterpret_cast<u32x4*>(&ysave[(size_t)c * 8]) = yv;
          const E8 y8 = __builtin_bit_cast(E8, yv);
          const E8 r8 = __builtin_bit_cast(E8, rq[k % RB]);
          E8 o8;
          uint32_t mb = 0u;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float z = fmaxf(__builtin_fmaf((float)y8[j], ca[k % 3][j], cb[k % 3][j]) + (float)r8[j], 0.f);
            o8[j] = (E)pin_f32(z * cd[k % 3][j]);
            mb |= ((float)o8[j] > 0.f ? 1u : 0u) << j;
          }
          const u32x4 ov = __builtin_bit_cast(u32x4, o8);
          if (out) *reinterpret_cast<u32x4*>(&out[(size_t)c * 8]) = ov;
          if (rmask) rmask[c] = (uint8_t)mb;
          *reinterpret_cast<u32x4*>(sp) = ov;  // the next layer's input
        }
      }
      __syncthreads();  // the tile and sAB are complete / free
      TSTAMP(4);
    }
    if (p.pooled)  // (uniform) the invalid team of an odd N stores nothing
      pool_tile(sX, sAB, P, threadIdx.x & 255, valid ? p.pooled + (size_t)n * COUT : nullptr);
  }
#ifdef MC_DIAG
  if (p.diag && (threadIdx.x & 63) == 0 && team == 0)
    for (int k = 0; k < 8; ++k) p.diag[((size_t)blockIdx.x * 4 + wave) * 8 + k] = dacc[k];
#endif
}

// ------------------------------------------------------------------------------------
// k_trunk_fwd_pp (boards of <= 256 cells, <= 10 layers): the forward of k_trunk_fwd2 re-scheduled
// so that the matrix pipe never waits for the GroupNorm / epilogue work. Two 4-wave teams per
// 512-thread workgroup (one per CU), one sample each, run PING-PONG: while team A runs the 9 taps
// of a layer on the MFMA, team B runs the statistics and epilogue of its previous layer on the
// VALU, then they swap. A half-period is 9 intervals, one per tap of the MFMA team, each closed by
// one workgroup barrier; the epilogue team cuts its work into the same 9 intervals:
//   P0 GroupNorm pass 1 (sums) | P1 pass 2 (squared deviations) | P2 scale / shift / dropout
//   coefficients | P3 .. P8 the epilogue, one (channel tile, pixel tile) piece per interval.
// Differences to k_trunk_fwd2 that make the epilogue cheap enough to hide:
//  * swapped MFMA operands: D[co][px] = W[co] . X[px], so a lane holds ONE pixel and 4-channel
//    runs of the output; the epilogue works on the accumulators in place (no y -> LDS pass, no
//    chunk re-read) and writes 8-byte pieces: the next layer's tile (ds_write_b64), y / out
//    (global 8-B stores) and the ReLU bits (12 bytes a pixel after one lane exchange);
//  * the accumulators start from the conv bias (y = b + sum, staged bias table in LDS);
//  * tiles and weight taps are 192-B rows with the 16-B chunk index XOR-ed by (row >> 2) & 3
//    (conflict-free ds_read_b128 without padding), so two sample tiles and a 3-slot weight ring
//    fit: taps arrive by LDS-DMA two intervals ahead (global_load_lds gathers the swizzle), waited
//    with a counted vmcnt by the issuing wave, never behind the epilogue's stores;
//  * the next sample's input is gathered into the tile by LDS-DMA during the last layer's
//    statistics, and the value head's average pool is reduced from registers.
// The weight stream repeats each layer's taps for the second team (L0 L0 L1 L1 ...: position
// s = 9 h + tap of half-period h holds layer (h >> 1) % NL, tap s % 9, ring slot s % 3 = tap % 3).
// Arithmetic per element is k_trunk_fwd2's; the f32 sums run in another order (statistics over
// the lanes of a pixel-major layout), so results agree with the per-layer kernels to rounding
// (tests/test_trunk_gpu.py), not bitwise.
constexpr int PPRS = COUT * 2;           // tile / tap row bytes (12 chunks of 16 B, swizzled)
constexpr int PP_TAPB = COUT * PPRS;     // one weight tap: 18,432 B = 18 LDS-DMA pieces of 1 KiB
constexpr int PP_TAPP = PP_TAPB / 1024;
constexpr int PP_MAXL = 10;
constexpr int PP_SLOTS = 3;
constexpr int PP_RED = 2 * 2 * WAVES * 8;  // sRed [team][pass][wave][8] f32

__host__ __device__ inline int pp_tile(int P) { return ((P + 1) * PPRS + 15) & ~15; }
__host__ __device__ inline size_t pp_lds(int P) {
  return 2 * (size_t)pp_tile(P) + PP_SLOTS * PP_TAPB + (PP_MAXL * COUT + PP_RED + 2 * 3 * COUT + 2 * WAVES * COUT) * 4;
}
// byte offset of 16-B chunk c of row r in a swizzled [rows][192 B] image
__device__ __forceinline__ int pp_swz(int r, int c) { return r * PPRS + ((c ^ ((r >> 2) & 3)) << 4); }

__device__ __forceinline__ uint32_t pp_lds_addr(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)(p);
}
// one full-wave LDS-DMA, 16 B a lane, lane-linear at LDS byte address m0v, from a wave-uniform
// base plus this lane's 32-bit byte offset (inline asm: the compiler puts no waits on LDS reads)
__device__ __forceinline__ void pp_dma(const void* base, uint32_t off, uint32_t m0v) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(off), "s"(base), "s"(m0v)
               : "memory", "m0");
}
template <int N>
__device__ __forceinline__ void pp_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 15) | ((N >> 4) << 14));
}

// per-lane coordinates, re-derived at the top of every phase from an opaque thread index: nothing
// computed from them is hoisted out of the half-period loop (it would stay live across both
// phases and spill)
struct PPLane {
  int ttid, lane, l32, hh;
};
__device__ __forceinline__ PPLane pp_lane() {
  const int tid = (int)threadIdx.x + opaque0();
  return PPLane{tid & 255, tid & 63, tid & 31, (tid >> 5) & 1};
}

template <typename E, int NPT, bool FULL, bool SAVE>
__global__ __launch_bounds__(512, 1) void k_trunk_fwd_pp(TrunkFwdParams<E> p) {
#pragma clang fp contract(off)
  typedef typename EV<E>::v8 E8;
  typedef typename EV<E>::v4 E4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int H = p.H, W = p.W, P = H * W, NL = p.NL;
  const int tb = pp_tile(P);
  const int team = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 8);
  const int wave = __builtin_amdgcn_readfirstlane(((int)threadIdx.x >> 6) & 3);
  unsigned char* sTile = smem + team * tb;
  unsigned char* sRing = smem + 2 * tb;
  float* sBias = reinterpret_cast<float*>(sRing + PP_SLOTS * PP_TAPB);  // [NL][96]
  float* sRed = sBias + PP_MAXL * COUT;                                  // [2 team][2 pass][4 wave][8]
  float* sRedT = sRed + team * 2 * WAVES * 8;                            // this team's [2][4][8]
  float* sAB = sRed + PP_RED + team * 3 * COUT;                          // this team's [3][96]
  float* sPool = sRed + PP_RED + 2 * 3 * COUT + team * WAVES * COUT;     // this team's [4][96]
  const uint32_t ring0 = __builtin_amdgcn_readfirstlane(pp_lds_addr(sRing));
  const uint32_t tile0 = __builtin_amdgcn_readfirstlane(pp_lds_addr(sTile));
#ifdef MC_DIAG
  // per wave: 0 MFMA-phase issue + taps, 1 its vmcnt waits + barriers, 2 P0-P2 work, 3 their barrier
  // waits, 4 epilogue pieces, 5 their barrier waits, 6 active MFMA intervals, 7 active pieces
  unsigned long long dacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif

  // samples: pair k of this workgroup = blockIdx.x + k * grid; team A takes 2 pair, team B 2 pair + 1
  const int npairs = (p.N + 1) >> 1;
  const int nA = (npairs - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int lastpair = (int)blockIdx.x + (nA - 1) * (int)gridDim.x;
  const int nB = 2 * lastpair + 1 < p.N ? nA : nA - 1;
  const int nS = team ? nB : nA;
  // half-periods: team h & 1 runs its taps, the other its epilogue
  const int HP = 2 * nA * NL + 1;
  // weight-DMA pieces of a tap: the 4 tap waves take pieces wave + 4 i (4-5 each)
  constexpr int DW = WAVES, DI = (PP_TAPP + DW - 1) / DW, DMIN = PP_TAPP / DW;
  const int dw = wave;
  auto sample_of = [&](int k) { return 2 * ((int)blockIdx.x + k * (int)gridDim.x) + team; };

  // x0 of sample n into this team's tile, gathered by LDS-DMA (pieces wave, wave + 4, ...)
  auto issue_x0 = [&](int n, int lane) {
    const E* src = p.x0 + (size_t)n * P * COUT;
    const int npc = (P * PPRS + 1023) >> 10;
    for (int j = wave; j < npc; j += WAVES) {
      const int q = j * 1024 + lane * 16;
      if (q < P * PPRS) {
        const int r = q / PPRS, cs = (q - r * PPRS) >> 4;
        pp_dma(src, (uint32_t)(r * PPRS + ((cs ^ ((r >> 2) & 3)) << 4)), tile0 + j * 1024);
      }
    }
  };
  // weight stream position s, this wave's pieces j = wave + 4 i: layer ((s / 9) >> 1) % NL, tap
  // s % 9, ring slot s % 3; piece j of a slot holds LDS bytes [j KiB, j KiB + 1 KiB): row co, chunk
  // slot cs hold source chunk cs ^ ((co >> 2) & 3) of the [96][96] tap
  auto woffs = [&](int lane, uint32_t (&wo)[DI]) {
#pragma unroll
    for (int i = 0; i < DI; ++i) {
      const int j = dw + DW * i, q = j * 1024 + lane * 16, co = q / PPRS, cs = (q - co * PPRS) >> 4;
      wo[i] = (uint32_t)(co * PPRS + ((cs ^ ((co >> 2) & 3)) << 4));
    }
  };
  auto issue_w = [&](int s, const uint32_t (&wo)[DI]) {
    const int hs = s / 9, ts = s - hs * 9, ls = (hs >> 1) % NL;
    const E* base = p.L[ls].wt + (size_t)ts * COUT * COUT;
    const uint32_t sb = ring0 + (uint32_t)((s % PP_SLOTS) * PP_TAPB);
#pragma unroll
    for (int i = 0; i < DI; ++i) {
      const int j = dw + DW * i;
      if (j < PP_TAPP) pp_dma(base, wo[i], sb + j * 1024);
    }
  };
  // the same for a tap whose base pointer and ring slot are known (the MFMA phase's: no divisions)
  auto issue_wb = [&](const E* base, uint32_t sb, const uint32_t (&wo)[DI]) {
#pragma unroll
    for (int i = 0; i < DI; ++i) {
      const int j = dw + DW * i;
      if (j < PP_TAPP) pp_dma(base, wo[i], sb + j * 1024);
    }
  };

  // ---------------- prologue ----------------
  {
    const PPLane ln = pp_lane();
    for (int i = threadIdx.x; i < 2 * 12; i += 512) {  // the zero row P of both tiles
      const int tm = i / 12, c = i - tm * 12;
      *reinterpret_cast<u32x4*>(smem + tm * tb + P * PPRS + c * 16) = u32x4{0u, 0u, 0u, 0u};
    }
    for (int i = threadIdx.x; i < NL * COUT; i += 512) sBias[i] = p.L[i / COUT].bias[i % COUT];
    if (nS > 0) issue_x0(sample_of(0), ln.lane);
    uint32_t wo[DI];
    woffs(ln.lane, wo);
    issue_w(team, wo);  // stream positions 0 (team A's waves) and 1 (team B's)
    pp_wait_vm<0>();
    __syncthreads();
  }

  f32x16 acc[NPT][3];
  int pool_n = -1;  // sample whose pooled sums wait in sPool
  for (int h = 0; h < HP; ++h) {
    const int m = h & 1, j = h >> 1;
    if (team == m) {
      // ======================= MFMA phase: step j of this team =======================
#ifdef MC_DIAG
      if (p.dflags & 8) __builtin_amdgcn_s_setprio(0);  // experiment: the epilogue team prioritised
      else if (!(p.dflags & 4)) __builtin_amdgcn_s_setprio(1);  // 4: no priorities
#else
      __builtin_amdgcn_s_setprio(1);
#endif
      const PPLane ln = pp_lane();
      uint32_t wo[DI];
      woffs(ln.lane, wo);
      const bool act_rt = j < nS * NL;
      const int l = act_rt ? j % NL : 0;
      // the weight stream's layers this half-period (h >> 1) and next ((h + 1) >> 1), mod NL
      const E* wcur = p.L[(h >> 1) % NL].wt;
      const E* wnext = p.L[((h + 1) >> 1) % NL].wt;
      if (pool_n >= 0) {  // the previous sample's pooled mean (sPool complete since the last barrier)
        if (ln.ttid < COUT) {
          const int c = ln.ttid;
          p.pooled[(size_t)pool_n * COUT + c] =
              ((sPool[c] + sPool[COUT + c]) + (sPool[2 * COUT + c] + sPool[3 * COUT + c])) * (1.0f / (float)P);
        }
        pool_n = -1;
      }
      // weight A-operand rows co = ct * 32 + l32: chunk 2 ks ^ vw (even ks at wa0 + 32 ks, odd ks at
      // wa1 + 32 (ks - 1)); this lane's output pixel per 32-pixel tile (past P: the zero row)
      const int vw = ((ln.l32 >> 2) & 3) ^ ln.hh;
      const int wa0 = ln.l32 * PPRS + (vw << 4), wa1 = ln.l32 * PPRS + ((vw ^ 2) << 4);
      int qr[NPT], qc[NPT];
#pragma unroll
      for (int t = 0; t < NPT; ++t) {
        const int q = (wave * NPT + t) * 32 + ln.l32;
        qr[t] = q < P ? q / W : -1000;
        qc[t] = q < P ? q - qr[t] * W : -1000;
      }
      // (specialised on act: the compiler's vmcnt bookkeeping must not see a path on which the
      // epilogue's loads are still pending, or it waits for vmcnt(0) -- the weight DMAs -- every tap)
      auto taps = [&](auto ACT) {
      constexpr bool act = decltype(ACT)::value;
      if (act) {  // the accumulators start from the conv bias (channel ct * 32 + 8 (i >> 2) + 4 hh + (i & 3))
#pragma unroll
        for (int ct = 0; ct < 3; ++ct)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 b4 = *reinterpret_cast<const f32x4*>(&sBias[l * COUT + ct * 32 + 8 * g + 4 * ln.hh]);
#pragma unroll
            for (int t = 0; t < NPT; ++t)
#pragma unroll
              for (int e = 0; e < 4; ++e) acc[t][ct][4 * g + e] = b4[e];
          }
      }
#pragma nounroll
      for (int tap3 = 0; tap3 < 9; tap3 += 3)
#pragma unroll
        for (int ts = 0; ts < 3; ++ts) {
          const int tap = tap3 + ts;
          const int s = 9 * h + tap;
          const bool iss = s + 2 < 9 * HP;
          // position s + 2: tap + 2 of this phase's layer, or tap - 7 of the next phase's; slot (tap + 2) % 3
          if (iss)
            issue_wb(tap + 2 < 9 ? wcur + (size_t)(tap + 2) * COUT * COUT : wnext + (size_t)(tap - 7) * COUT * COUT,
                     ring0 + (uint32_t)(((ts + 2) % PP_SLOTS) * PP_TAPB), wo);
          if (act) {
            const int dr = tap / 3 - 1, dc = tap % 3 - 1;
            int xa0[NPT], xa1[NPT];
#pragma unroll
            for (int t = 0; t < NPT; ++t) {
              const int sr = qr[t] + dr, sc = qc[t] + dc;
              const bool v = (unsigned)sr < (unsigned)H && (unsigned)sc < (unsigned)W;
              const int r = v ? sr * W + sc : P;
              const int xv = ((r >> 2) & 3) ^ ln.hh;
              xa0[t] = r * PPRS + (xv << 4);
              xa1[t] = r * PPRS + ((xv ^ 2) << 4);
            }
            const unsigned char* sw = sRing + ts * PP_TAPB;  // slot s % 3 = tap % 3
            constexpr int KS = COUT / 16;
            E8 A[2][3], B[2][NPT];
            auto ld = [&](int ks, E8 (&a)[3], E8 (&b)[NPT]) {
              const int wo = (ks & 1) ? wa1 + 32 * (ks - 1) : wa0 + 32 * ks;
#pragma unroll
              for (int ct = 0; ct < 3; ++ct) a[ct] = *reinterpret_cast<const E8*>(sw + wo + ct * 32 * PPRS);
#pragma unroll
              for (int t = 0; t < NPT; ++t)
                b[t] = *reinterpret_cast<const E8*>(sTile + ((ks & 1) ? xa1[t] + 32 * (ks - 1) : xa0[t] + 32 * ks));
            };
            ld(0, A[0], B[0]);
            __builtin_amdgcn_sched_group_barrier(0x100, NPT + 3, 0);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
              if (ks + 1 < KS) {
                ld(ks + 1, A[(ks + 1) & 1], B[(ks + 1) & 1]);
                __builtin_amdgcn_sched_group_barrier(0x100, NPT + 3, 0);
              }
#pragma unroll
              for (int ct = 0; ct < 3; ++ct)
#pragma unroll
                for (int t = 0; t < NPT; ++t) acc[t][ct] = mfma32(A[ks & 1][ct], B[ks & 1][t], acc[t][ct]);
              __builtin_amdgcn_sched_group_barrier(0x008, 3 * NPT, 0);
            }
          }
          TSTAMP(0);
#ifdef MC_DIAG
          dacc[6] += act ? 1 : 0;
#endif
          // position s + 1 must have landed: issued by this wave one interval ago (tap >= 1), or by
          // the other team at its last tap (it waits for it at the top of its epilogue phase)
          if (tap >= 1) {
            if (iss) pp_wait_vm<DMIN>();  // this interval's pieces may stay in flight
            else pp_wait_vm<0>();
          }
          lds_barrier();
          TSTAMP(1);
        }
      };
      if (act_rt) taps(std::true_type{});
      else taps(std::false_type{});
#ifdef MC_DIAG
      if (p.dflags & 8) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
#else
      __builtin_amdgcn_s_setprio(0);
#endif
    } else {
      // =================== epilogue phase: step jp of this team ===================
      const int jp = m ? j : j - 1;
      const bool act_rt = jp >= 0 && jp < nS * NL;
      auto post = [&](auto ACT) {
      constexpr bool act = decltype(ACT)::value;
      const int k = act ? jp / NL : 0, l = act ? jp % NL : 0;
      const int n = act ? sample_of(k) : 0;
      const size_t so = (size_t)n * P * COUT;
      const bool last = l == NL - 1;
      const float inv_cnt = 1.0f / (16.0f * (float)P);
      // ---- P0: GroupNorm sums; the residual, the GN parameters, the next sample's input in flight ----
      pp_wait_vm<0>();  // weight pieces this wave issued at its last tap (the MFMA team's tap 0 needs them)
      // the residual (block input) of a conv2 layer: gathered at P0 by LDS-DMA into this wave's own
      // pixel rows of the tile (the taps have read them; coalesced 16-B chunks), read back per piece
      // as 8-byte pieces in the accumulators' layout (each lane then overwrites what it read)
      const E* res = nullptr;
      float gmv = 0.f, btv = 0.f, dmv = 1.f;
      {
        const PPLane ln = pp_lane();
        if (act) {
          if (l & 1) res = l == 1 ? p.x0 + so : (p.L[l - 2].out ? p.L[l - 2].out + so : p.ws + ((size_t)blockIdx.x * 2 + team) * P * COUT);
#ifdef MC_DIAG
          if (p.dflags & 2) res = nullptr;
#endif
          if (res) {
#pragma unroll
            for (int t = 0; t < NPT; ++t) {
              const int r0 = (wave * NPT + t) * 32;
#pragma unroll
              for (int kk = 0; kk < 6; ++kk) {
                const int qb = r0 * PPRS + kk * 1024 + ln.lane * 16;
                if (qb < P * PPRS) {
                  const int r = qb / PPRS, cs = (qb - r * PPRS) >> 4;
                  pp_dma(res, (uint32_t)(r * PPRS + ((cs ^ ((r >> 2) & 3)) << 4)), tile0 + r0 * PPRS + kk * 1024);
                }
              }
            }
          }
          if (ln.ttid < COUT) {
            gmv = p.L[l].gamma[ln.ttid];
            btv = p.L[l].beta[ln.ttid];
            if (p.L[l].dmask) dmv = p.L[l].dmask[(size_t)n * COUT + ln.ttid];
          }
          float s6[NGRP];
#pragma unroll
          for (int ct = 0; ct < 3; ++ct)
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
              float v = 0.f;
#pragma unroll
              for (int t = 0; t < NPT; ++t) {
                const int px = (wave * NPT + t) * 32 + ln.l32;
                float u = 0.f;
#pragma unroll
                for (int i = 0; i < 8; ++i) u += acc[t][ct][8 * hf + i];
                v += (FULL || px < P) ? u : 0.f;
              }
              s6[2 * ct + hf] = wave_sum(v);
            }
          if (ln.lane == 0) {
#pragma unroll
            for (int g = 0; g < NGRP; ++g) sRedT[wave * 8 + g] = s6[g];
          }
        }
      }
      TSTAMP(2);
      lds_barrier();
      TSTAMP(3);
      // ---- P1: means, GroupNorm squared deviations ----
      if (act) {
        const PPLane ln = pp_lane();
        float s6[NGRP];
#pragma unroll
        for (int ct = 0; ct < 3; ++ct)
#pragma unroll
          for (int hf = 0; hf < 2; ++hf) {
            const int g = 2 * ct + hf;
            const float mu = ((sRedT[g] + sRedT[8 + g]) + (sRedT[16 + g] + sRedT[24 + g])) * inv_cnt;
            float v = 0.f;
#pragma unroll
            for (int t = 0; t < NPT; ++t) {
              const int px = (wave * NPT + t) * 32 + ln.l32;
              float u = 0.f;
#pragma unroll
              for (int i = 0; i < 8; ++i) {
                const float d = acc[t][ct][8 * hf + i] - mu;
                u = __builtin_fmaf(d, d, u);
              }
              v += (FULL || px < P) ? u : 0.f;
            }
            s6[g] = wave_sum(v);
          }
        if (ln.lane == 0) {
#pragma unroll
          for (int g = 0; g < NGRP; ++g) sRedT[32 + wave * 8 + g] = s6[g];
        }
      }
      TSTAMP(2);
      lds_barrier();
      TSTAMP(3);
      // ---- P2: scale / shift / dropout coefficients per channel (threads c < 96: group c >> 4) ----
      pp_wait_vm<0>();  // residual, GN parameters, the next sample's input
      if (act) {
        const PPLane ln = pp_lane();
        if (ln.ttid < COUT) {
          const int g = ln.ttid >> 4;
          const float mu = ((sRedT[g] + sRedT[8 + g]) + (sRedT[16 + g] + sRedT[24 + g])) * inv_cnt;
          const float rs = rsqrtf(((sRedT[32 + g] + sRedT[40 + g]) + (sRedT[48 + g] + sRedT[56 + g])) * inv_cnt + p.eps);
          const float a = gmv * rs;
          sAB[ln.ttid] = a;
          sAB[COUT + ln.ttid] = btv - mu * a;
          sAB[2 * COUT + ln.ttid] = dmv;
          float* stats = p.L[l].stats;
          if (SAVE && (ln.ttid & 15) == 0) {
            stats[((size_t)n * NGRP + g) * 2 + 0] = mu;
            stats[((size_t)n * NGRP + g) * 2 + 1] = rs;
          }
        }
      }
      TSTAMP(2);
      lds_barrier();
      TSTAMP(3);
      // ---- P3 .. P8: the epilogue, piece q = (ct, t) per interval (NPT = 1: P6 .. P8 idle) ----
      E* out = nullptr;
      E* ysave = nullptr;
      uint8_t* rmask = nullptr;
      bool pool_here = false;
      if (act) {
        out = p.L[l].out ? p.L[l].out + so
                         : ((l & 1) && !last ? p.ws + ((size_t)blockIdx.x * 2 + team) * P * COUT : nullptr);
        ysave = SAVE ? p.L[l].ysave + so : nullptr;  // SAVE: every layer has ysave, stats, relu_mask
        rmask = SAVE ? p.L[l].rmask + (size_t)n * P * C8 : nullptr;
        pool_here = last && p.pooled;
#ifdef MC_DIAG
        if (p.dflags & 1) {
          if (!last) out = nullptr;
        }
#endif
      }
      // the next sample's input, gathered by LDS-DMA into this wave's own pixel rows once its last
      // pixel tile is staged (the epilogue stages y / out through those rows)
      const bool x0next = act && last && k + 1 < nS;
      // the pieces, specialised on the value head's pool (the last layer only)
      auto pieces = [&](auto POOL) {
      constexpr bool pool = decltype(POOL)::value;
      uint32_t rw[3];      // ReLU bits of the current pixel tile, per channel tile
      u32x2 ohold[3][4];   // SAVE: the tile's outputs wait here while y passes through its rows
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        if (q < 3 * NPT && act) {
          const int t = q / 3, ct = q % 3;  // pixel tile t, channel tile ct
          const PPLane ln = pp_lane();
          const int px = (wave * NPT + t) * 32 + ln.l32;
          const bool pv = FULL || px < P;
          uint32_t word = 0u;
          float pl[16];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int co = ct * 32 + 8 * g + 4 * ln.hh;
            const f32x4 ca = *reinterpret_cast<const f32x4*>(&sAB[co]);
            const f32x4 cb = *reinterpret_cast<const f32x4*>(&sAB[COUT + co]);
            const f32x4 cd = *reinterpret_cast<const f32x4*>(&sAB[2 * COUT + co]);
            // this lane's 8 bytes of pixel px, chunk ct * 4 + g: the residual (conv2) in, then y
            // (SAVE: staged for the coalesced store below, the output kept in registers meanwhile)
            // or the output itself out
            unsigned char* slot = sTile + pp_swz(px, ct * 4 + g) + ln.hh * 8;
            E4 rh;
#pragma unroll
            for (int e = 0; e < 4; ++e) rh[e] = (E)0.f;
            if (res && pv) rh = *reinterpret_cast<const E4*>(slot);
            E4 yh, oh;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              yh[e] = (E)acc[t][ct][4 * g + e];
              const float z = fmaxf(__builtin_fmaf((float)yh[e], ca[e], cb[e]) + (float)rh[e], 0.f);
              oh[e] = (E)pin_f32(z * cd[e]);
            }
            uint32_t nib = 0u;  // ReLU bits of the 16-bit outputs
#pragma unroll
            for (int e = 0; e < 4; ++e) nib |= ((float)oh[e] > 0.f ? 1u : 0u) << e;
            word |= nib << (8 * g + 4 * ln.hh);
            if (SAVE) ohold[ct][g] = __builtin_bit_cast(u32x2, oh);
            if (pv) *reinterpret_cast<u32x2*>(slot) = __builtin_bit_cast(u32x2, SAVE ? yh : oh);
            if (pool) {
#pragma unroll
              for (int e = 0; e < 4; ++e) pl[4 * g + e] = pv ? (float)oh[e] : 0.f;
            }
          }
          rw[ct] = word;
          if (pool) {  // this piece's sums over the wave's pixels -> sPool (lanes 31, 63; tile 1 adds)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              float v = row_sum16(pl[i]);
              v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x142, 0xA, 0xf, false));
              pl[i] = v;
            }
            if (ln.l32 == 31) {
#pragma unroll
              for (int g = 0; g < 4; ++g) {
                f32x4* sp = reinterpret_cast<f32x4*>(&sPool[wave * COUT + ct * 32 + 8 * g + 4 * ln.hh]);
                const f32x4 v4{pl[4 * g], pl[4 * g + 1], pl[4 * g + 2], pl[4 * g + 3]};
                *sp = t == 0 ? v4 : *sp + v4;
              }
            }
          }
          if (ct == 2) {
            // pixel tile t complete. Its 32 rows (6 KiB, contiguous in the tile) leave as 16-B chunks
            // in row order -- one 1-KiB coalesced store per wave instruction -- instead of 8-B
            // pieces at 192-B strides: y first (SAVE), then the outputs (block outputs / residual slot)
            const int r0 = (wave * NPT + t) * 32;
            auto flush = [&](E* dst) {
#pragma unroll
              for (int kk = 0; kk < 6; ++kk) {
                const int gi = kk * 64 + ln.lane, r = r0 + gi / 12, c = gi - (gi / 12) * 12;
                const u32x4 v = *reinterpret_cast<const u32x4*>(sTile + pp_swz(r, c));
                if (FULL || r < P) *reinterpret_cast<u32x4*>(dst + (size_t)r * COUT + c * 8) = v;
              }
            };
            if (SAVE) {
              flush(ysave);
#pragma unroll
              for (int c2 = 0; c2 < 3; ++c2)
#pragma unroll
                for (int g = 0; g < 4; ++g)
                  if (pv) *reinterpret_cast<u32x2*>(sTile + pp_swz(px, c2 * 4 + g) + ln.hh * 8) = ohold[c2][g];
            }
            if (out) flush(out);
            if (SAVE) {  // ReLU bits: byte ct * 4 + g = low nibble (hh 0) | high nibble (hh 1)
              uint32_t b3[3];
#pragma unroll
              for (int c2 = 0; c2 < 3; ++c2) b3[c2] = rw[c2] | (uint32_t)__shfl_xor((int)rw[c2], 32);
              if (ln.hh == 0 && pv) {
                uint32_t* rp = reinterpret_cast<uint32_t*>(rmask + (size_t)px * C8);
                rp[0] = b3[0];
                rp[1] = b3[1];
                rp[2] = b3[2];
              }
            }
            if (x0next) {  // this wave's rows of the next sample's input (all its reads of them done)
              const E* src = p.x0 + (size_t)sample_of(k + 1) * P * COUT;
#pragma unroll
              for (int kk = 0; kk < 6; ++kk) {
                const int qb = (r0 * PPRS) + kk * 1024 + ln.lane * 16;
                if (qb < P * PPRS) {
                  const int r = qb / PPRS, cs = (qb - r * PPRS) >> 4;
                  pp_dma(src, (uint32_t)(r * PPRS + ((cs ^ ((r >> 2) & 3)) << 4)), tile0 + r0 * PPRS + kk * 1024);
                }
              }
            }
          }
        }
        if (q == 5 && x0next) pp_wait_vm<0>();  // the next sample's input has landed (its taps follow)
        if (q == 5 && pool && act) pool_n = n;
        TSTAMP(4);
#ifdef MC_DIAG
        dacc[7] += (q < 3 * NPT && act) ? 1 : 0;
#endif
        lds_barrier();
        TSTAMP(5);
      }
      };
      if (pool_here) pieces(std::true_type{});
      else pieces(std::false_type{});
      };
      if (act_rt) post(std::true_type{});
      else post(std::false_type{});
    }
  }
  if (pool_n >= 0) {  // the last sample's pooled mean (sPool complete: the last barrier)
    const PPLane ln = pp_lane();
    if (ln.ttid < COUT) {
      const int c = ln.ttid;
      p.pooled[(size_t)pool_n * COUT + c] =
          ((sPool[c] + sPool[COUT + c]) + (sPool[2 * COUT + c] + sPool[3 * COUT + c])) * (1.0f / (float)P);
    }
  }
#ifdef MC_DIAG
  if (p.diag && (threadIdx.x & 63) == 0)
    for (int q = 0; q < 8; ++q) p.diag[((size_t)blockIdx.x * 8 + (threadIdx.x >> 6)) * 8 + q] = dacc[q];
#endif
}

// ------------------------------------------------------------------------------------
template <typename E>
struct TBLayer {
  const E* y;              // ysave of the forward
  const float* stats;      // [N][6][2]
  const float* gamma;      // [96]
  const uint8_t* rmask;    // [N][P][12] ReLU bits of the forward
  const float* dmask;      // [N][96] or NULL
  const E* wT;             // [9][96 ci][96 co]; NULL for layer 0 (no input gradient)
  E* dy;                   // [N][P][96] out: dL/dy (the weight gradient's operand)
};

template <typename E>
struct TrunkBwdParams {
  const E* dout;  // [N][P][96] gradient of the last layer's output
  E* ws;          // [grid][P][96]: a block's skip gradient between its conv2 and its input
  float* part;    // [VG][NL][3][96] d gamma, d beta, d bias per partial row
  unsigned long long* diag;  // MC_DIAG builds: per-wave phase cycle totals [grid][4][8]
#ifdef MC_DIAG
  int dflags;  // timing experiments only: bit 0 drops pass 2's global stores (dy, skip slot)
#endif
  int NL, N, H, W;
  int VG;         // partial rows: the per-layer kernel's grid (min(N, 2 x CUs)), so the sums match it
  TBLayer<E> L[MAXL + 1];
};

constexpr int DCP = CINP;  // dy tile row stride (elements)
constexpr int PG = 21;     // pixel groups of the element-wise passes: thread = (pg, c8)

__host__ __device__ inline int tb_dtile_bytes(int P) { return ((P + 1) * DCP * 2 + 15) & ~15; }
__host__ __device__ constexpr int tb_red_bytes() {  // sRed [PG][3][96] f32, aliased by sW [96][DCP]
  return PG * 3 * COUT * 4 > COUT * DCP * 2 ? PG * 3 * COUT * 4 : COUT * DCP * 2;
}
__host__ __device__ inline size_t tb_lds(int P) { return (size_t)tb_dtile_bytes(P) + tb_red_bytes() + 5 * COUT * 4; }

// Layer i of p.L (forward order: 0 = the stem, 2b+1 / 2b+2 = conv1 / conv2 of block b):
//   dout_i = dgrad_{i+1} (+ dz_{i+2} when i is even: the block input's skip gradient)
//   pass 1: dz = (out_i > 0) * dout_i * dmask; sums S1 = sum dz, S2 = sum dz*yhat, S3 = sum yhat
//   pass 2: dy = rstd*gamma*dz - rstd*mean_g(gamma*dz) - rstd*yhat*mean_g(gamma*dz*yhat)
//   dgrad (i > 0): dx = sum_tap shift(dy) . W^T[tap], staged in the tile for layer i-1
template <typename E, int NPT, int NCH>
__global__ __launch_bounds__(256, NPT <= 2 ? 2 : 1) void k_trunk_bwd(TrunkBwdParams<E> p) {
  // no contraction: every expression rounds the same way in the per-layer and the one-launch
  // kernels (explicit fmaf where a fused multiply-add is wanted), so they agree bitwise
#pragma clang fp contract(off)
  typedef typename EV<E>::v8 E8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int H = p.H, W = p.W, P = H * W;
  E* sD = reinterpret_cast<E*>(smem);  // [P+1][DCP] (row P = 0): dx -> dz -> dy of each layer
  float* sRed = reinterpret_cast<float*>(smem + tb_dtile_bytes(P));
  E* sW = reinterpret_cast<E*>(sRed);  // W^T[tap] as [ci][DCP]
  float* sCo = reinterpret_cast<float*>(smem + tb_dtile_bytes(P) + tb_red_bytes());  // [3][96]
  float* sTmp = sCo + 3 * COUT;                                                       // [2][96]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l32 = lane & 31, hh = lane >> 5;
  const float inv_cnt = 1.0f / (16.0f * (float)P);
  // HOLD: the skip gradient dz of a conv2 stays in registers until the dx of the block's conv1
  // (the next layer down) is written, in the dx lane layout: pixel (wave NPT + t) 32 + l32,
  // channels ct 32 + 8 g + 4 hh + 0..3 -- 4 x 16-bit each, 48 VGPRs at NPT = 2. Otherwise it
  // makes a round trip through the workgroup's workspace slot (L2 / Infinity Cache)
  constexpr bool HOLD = NPT <= 2;
  u32x2 zk[HOLD ? NPT : 1][3][4];

  for (int i = threadIdx.x; i < DCP / 8; i += 256) *reinterpret_cast<u32x4*>(&sD[P * DCP + 8 * i]) = u32x4{0u, 0u, 0u, 0u};
  int qr[NPT], qc[NPT];
#pragma unroll
  for (int t = 0; t < NPT; ++t) {
    const int q = (wave * NPT + t) * 32 + l32;
    qr[t] = q < P ? q / W : -1000;
    qc[t] = q < P ? q - qr[t] * W : -1000;
  }
  constexpr int NWC = (COUT * C8 + 255) / 256;  // 16-B chunks of one W^T tap per thread
#ifdef MC_DIAG
  unsigned long long dacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif

  // partial row vb takes samples vb, vb + VG, ... in order, as workgroup vb of the per-layer
  // kernel does; a workgroup runs rows blockIdx.x, blockIdx.x + gridDim.x, ... (VG >= gridDim.x)
  for (int vb = blockIdx.x; vb < p.VG; vb += gridDim.x)
  for (int n = vb; n < p.N; n += p.VG) {
    const size_t so = (size_t)n * P * COUT;
    E* wsl = p.ws + (size_t)blockIdx.x * P * COUT;  // this workgroup's skip-gradient slot

    for (int li = p.NL - 1; li >= 0; --li) {
      // loop-variant thread coordinates: the per-chunk address math and the taps' row offsets
      // are recomputed per layer instead of hoisted out of this loop (they would be spilled)
      const int tid = threadIdx.x + opaque0();
#pragma unroll
      for (int t = 0; t < NPT; ++t) asm volatile("" : "+v"(qr[t]), "+v"(qc[t]));
      const int pg = tid / C8, c8 = tid - pg * C8;
      const bool gact = tid < PG * C8;
      const int grp = c8 >> 1;
      const bool top = li == p.NL - 1;
      const bool addd = !HOLD && !(li & 1) && li + 2 < p.NL;  // dout += the skip gradient dz_{li+2}
      const bool keep_dz = !(li & 1) && li >= 2;              // dz of a conv2: the skip gradient of layer li-2
      const bool addz = HOLD && (li & 1) && li + 1 < p.NL;    // dx += the held dz_{li+1} (layer li-1's dout)
      float* pp = p.part + ((size_t)vb * p.NL + li) * 3 * COUT;
      float acc_g = 0.f, acc_b = 0.f, acc_bias = 0.f;  // tid < 96: this partial row's running sums
      if (tid < COUT && n != vb) {
        acc_g = pp[tid];
        acc_b = pp[COUT + tid];
        acc_bias = pp[2 * COUT + tid];
      }
      const float* stats = p.L[li].stats;
      // ---------------- pass 1: dz and per-channel sums ----------------
      float dm[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) dm[j] = 1.f;
      float mean = 0.f, rstd = 0.f;
      if (gact) {
        const float* dmask = p.L[li].dmask;
        if (dmask) {
#pragma unroll
          for (int j = 0; j < 8; ++j) dm[j] = dmask[(size_t)n * COUT + c8 * 8 + j];
        }
        mean = stats[((size_t)n * NGRP + grp) * 2];
        rstd = stats[((size_t)n * NGRP + grp) * 2 + 1];
      }
      const E* yp = p.L[li].y + so;
      const uint8_t* rmp = p.L[li].rmask + (size_t)n * P * C8;
      u32x4 yr[NCH];
      float s1[8], s2[8], s3[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) s1[j] = s2[j] = s3[j] = 0.f;
      constexpr int LB = 7;  // chunks whose loads are in flight together
#pragma unroll
      for (int i0 = 0; i0 < NCH; i0 += LB) {
        u32x4 dv[LB];  // dout (top layer) or the skip gradient (addd): never both
        uint32_t mv[LB];
#pragma unroll
        for (int u = 0; u < LB; ++u) {
          const int i = i0 + u, px = pg + PG * i;
          if (i < NCH) yr[i] = u32x4{0u, 0u, 0u, 0u};
          mv[u] = 0u;
          dv[u] = u32x4{0u, 0u, 0u, 0u};
          if (i < NCH && gact && px < P) {
            const size_t o = (size_t)px * COUT + c8 * 8;
            if (top) dv[u] = *reinterpret_cast<const u32x4*>(&p.dout[so + o]);
            else if (addd) dv[u] = *reinterpret_cast<const u32x4*>(&wsl[o]);
            mv[u] = rmp[px * C8 + c8];
            yr[i] = *reinterpret_cast<const u32x4*>(&yp[o]);
          }
        }
#pragma unroll
        for (int u = 0; u < LB; ++u) {
          const int i = i0 + u, px = pg + PG * i;
          if (i < NCH && gact && px < P) {
            E* sp = &sD[px * DCP + c8 * 8];
            E8 d8;
            if (top) {
              d8 = __builtin_bit_cast(E8, dv[u]);
            } else {
              d8 = __builtin_bit_cast(E8, *reinterpret_cast<const u32x4*>(sp));  // dgrad of layer li+1
              if (addd) {  // + the skip gradient, rounded as the per-layer kernel's dx (+ addend) store
                const E8 a8 = __builtin_bit_cast(E8, dv[u]);
#pragma unroll
                for (int j = 0; j < 8; ++j) d8[j] = (E)pin_f32((float)d8[j] + (float)a8[j]);
              }
            }
            const E8 y8 = __builtin_bit_cast(E8, yr[i]);
            const uint32_t pos = mv[u];
            const u32x4 dw = __builtin_bit_cast(u32x4, d8);
            E8 z8;
            if constexpr (std::is_same_v<E, _Float16>) {
              // fp16: every f16 -> f32 widening folded into a v_fma_mix (exact conversion, one
              // rounding each, so the values are the generic path's bit for bit): d * dmask + (-0)
              // is the product with its sign of zero, 1 * y - mean the difference, and the sums
              // take the rounded dz straight from its packed pair (zf + s1, zf * yh + s2)
#pragma unroll
              for (int w = 0; w < 4; ++w) {
                const int j0 = 2 * w, j1 = 2 * w + 1;
                const float d0 = fmix_lo(dm[j0], dw[w], -0.0f), d1 = fmix_hi(dm[j1], dw[w], -0.0f);
                const f16x2 zh = {(E)(((pos >> j0) & 1u) ? d0 : 0.f), (E)(((pos >> j1) & 1u) ? d1 : 0.f)};
                const uint32_t zp = __builtin_bit_cast(uint32_t, zh);
                const float yh0 = fmix_lo(1.0f, yr[i][w], -mean) * rstd, yh1 = fmix_hi(1.0f, yr[i][w], -mean) * rstd;
                s1[j0] = fmix_lo(1.0f, zp, s1[j0]);
                s1[j1] = fmix_hi(1.0f, zp, s1[j1]);
                s2[j0] = fmix_lo(yh0, zp, s2[j0]);
                s2[j1] = fmix_hi(yh1, zp, s2[j1]);
                s3[j0] += yh0;
                s3[j1] += yh1;
                z8[j0] = zh[0];
                z8[j1] = zh[1];
              }
            } else {
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
            }
            *reinterpret_cast<u32x4*>(sp) = __builtin_bit_cast(u32x4, z8);
          }
        }
      }
      TSTAMP(0);
      // tap 0's W^T: loaded here, its latency hidden behind the channel reductions
      const E* wT = p.L[li].wT;
      const bool dgrad = li > 0;
      u32x4 wr[NWC];
      if (dgrad) {
#pragma unroll
        for (int k = 0; k < NWC; ++k) {
          const int c = tid + 256 * k;
          if (k < COUT * C8 / 256 || c < COUT * C8) wr[k] = reinterpret_cast<const u32x4*>(wT)[c];
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
      if (HOLD && keep_dz) {  // dz is complete in the tile; pass 2 overwrites it two barriers on
#pragma unroll
        for (int t = 0; t < (HOLD ? NPT : 1); ++t) {
          const int px = (wave * NPT + t) * 32 + l32;
          if (px < P) {
#pragma unroll
            for (int ct = 0; ct < 3; ++ct)
#pragma unroll
              for (int g = 0; g < 4; ++g) zk[t][ct][g] = *reinterpret_cast<const u32x2*>(&sD[px * DCP + ct * 32 + 8 * g + 4 * hh]);
          }
        }
      }
      float S1 = 0.f, S2 = 0.f, S3 = 0.f, gam = 0.f, cmean = 0.f, crstd = 0.f;
      if (tid < COUT) {
        for (int g = 0; g < PG; ++g) {
          S1 += sRed[(g * 3 + 0) * COUT + tid];
          S2 += sRed[(g * 3 + 1) * COUT + tid];
          S3 += sRed[(g * 3 + 2) * COUT + tid];
        }
        gam = p.L[li].gamma[tid];
        cmean = stats[((size_t)n * NGRP + (tid >> 4)) * 2];
        crstd = stats[((size_t)n * NGRP + (tid >> 4)) * 2 + 1];
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
        pp[tid] = acc_g;
        pp[COUT + tid] = acc_b;
        pp[2 * COUT + tid] = acc_bias;
      }
      __syncthreads();

      TSTAMP(1);
      // tap 0's W^T goes to sW (free now: the sums are read) before pass 2 issues its stores
      if (dgrad) {
#pragma unroll
        for (int k = 0; k < NWC; ++k) {
          const int c = tid + 256 * k;
          if (k < COUT * C8 / 256 || c < COUT * C8) {
            const int ci = c / C8, k8 = c - ci * C8;
            *reinterpret_cast<u32x4*>(&sW[ci * DCP + k8 * 8]) = wr[k];
          }
        }
      }
      // ---------------- pass 2: dy (GroupNorm backward) -> LDS tile + HBM ----------------
      E* dyp = p.L[li].dy + so;
      if (gact) {
        float A[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) A[j] = sCo[c8 * 8 + j];
        const float Bg = sCo[COUT + c8 * 8], Cg = sCo[2 * COUT + c8 * 8];
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
          const int px = pg + PG * i;
          if (px < P) {
            E* sp = &sD[px * DCP + c8 * 8];
            const u32x4 zv = *reinterpret_cast<const u32x4*>(sp);
#ifdef MC_DIAG
            if (!HOLD && keep_dz && !(p.dflags & 1)) *reinterpret_cast<u32x4*>(&wsl[(size_t)px * COUT + c8 * 8]) = zv;
#else
            if (!HOLD && keep_dz) *reinterpret_cast<u32x4*>(&wsl[(size_t)px * COUT + c8 * 8]) = zv;
#endif
            const E8 z8 = __builtin_bit_cast(E8, zv);
            const E8 y8 = __builtin_bit_cast(E8, yr[i]);
            E8 d8;
            if constexpr (std::is_same_v<E, _Float16>) {  // the same two fmas, each one v_fma_mix
#pragma unroll
              for (int w = 0; w < 4; ++w) {
                d8[2 * w] = (E)fmix_lo(A[2 * w], zv[w], fmix_lo(Bg, yr[i][w], Cg));
                d8[2 * w + 1] = (E)fmix_hi(A[2 * w + 1], zv[w], fmix_hi(Bg, yr[i][w], Cg));
              }
            } else {
#pragma unroll
              for (int j = 0; j < 8; ++j) d8[j] = (E)__builtin_fmaf(A[j], (float)z8[j], __builtin_fmaf(Bg, (float)y8[j], Cg));
            }
            const u32x4 v = __builtin_bit_cast(u32x4, d8);
            *reinterpret_cast<u32x4*>(sp) = v;
#ifdef MC_DIAG
            if (!(p.dflags & 1))
#endif
            *reinterpret_cast<u32x4*>(&dyp[(size_t)px * COUT + c8 * 8]) = v;
          }
        }
      }
      if (!dgrad) {  // (uniform) the stem's input needs no gradient
        TSTAMP(2);
        continue;
      }
      __syncthreads();
      TSTAMP(2);

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
          const u32x4* ws = reinterpret_cast<const u32x4*>(wT + (size_t)(tap + 1) * COUT * COUT);
#pragma unroll
          for (int k = 0; k < NWC; ++k) {
            const int c = tid + 256 * k;
            if (k < COUT * C8 / 256 || c < COUT * C8) wr[k] = ws[c];
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
        auto ld = [&](int k0, E8 (&a)[NPT], E8 (&b)[3]) {
#pragma unroll
          for (int ct = 0; ct < 3; ++ct)
            b[ct] = *reinterpret_cast<const E8*>(&sW[(ct * 32 + l32) * DCP + k0 + 8 * hh]);
#pragma unroll
          for (int t = 0; t < NPT; ++t) a[t] = *reinterpret_cast<const E8*>(&sD[aoff[t] + k0]);
        };
        // swapped operands: D[ci][px] = W^T[ci] . dy[px], so a lane holds one pixel and 4-channel runs
        // of dx (each element the same products in the same order as D[px][ci])
        auto mm = [&](const E8 (&a)[NPT], const E8 (&b)[3]) {
#pragma unroll
          for (int t = 0; t < NPT; ++t)
#pragma unroll
            for (int ct = 0; ct < 3; ++ct) acc[t][ct] = mfma32(b[ct], a[t], acc[t][ct]);
        };
        E8 a0[NPT], b0[3], a1[NPT], b1[3];
        ld(0, a0, b0);
        __builtin_amdgcn_sched_group_barrier(0x100, NPT + 3, 0);
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
            if (k < COUT * C8 / 256 || c < COUT * C8) {
              const int ci = c / C8, k8 = c - ci * C8;
              *reinterpret_cast<u32x4*>(&sW[ci * DCP + k8 * 8]) = wr[k];
            }
          }
          __syncthreads();
        }
      }
      TSTAMP(3);
      // dx -> the tile (16-bit, as the per-layer kernel's dx store): layer li-1's dout; lane = pixel,
      // channels ct * 32 + 8 g + 4 hh + 0..3 as one 8-byte write. addz: + the held skip gradient,
      // rounded as pass 1's addend path (the per-layer kernel's dx (+ addend) store)
#pragma unroll
      for (int t = 0; t < NPT; ++t) {
        const int px = (wave * NPT + t) * 32 + l32;
        if (px < P) {
#pragma unroll
          for (int ct = 0; ct < 3; ++ct)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              typename EV<E>::v4 d4;
#pragma unroll
              for (int e = 0; e < 4; ++e) d4[e] = (E)acc[t][ct][4 * g + e];
              if (addz) {
                if constexpr (std::is_same_v<E, _Float16>) {  // 1 * dx + dz, both widened in one v_fma_mix
                  const u32x2 dp = __builtin_bit_cast(u32x2, d4), zp = zk[HOLD ? t : 0][ct][g];
#pragma unroll
                  for (int e = 0; e < 4; ++e) d4[e] = (E)((e & 1) ? fmix2_hi(dp[e >> 1], zp[e >> 1]) : fmix2_lo(dp[e >> 1], zp[e >> 1]));
                } else {
                  const typename EV<E>::v4 z4 = __builtin_bit_cast(typename EV<E>::v4, zk[HOLD ? t : 0][ct][g]);
#pragma unroll
                  for (int e = 0; e < 4; ++e) d4[e] = (E)pin_f32((float)d4[e] + (float)z4[e]);
                }
              }
              *reinterpret_cast<u32x2*>(&sD[px * DCP + ct * 32 + 8 * g + 4 * hh]) = __builtin_bit_cast(u32x2, d4);
            }
        }
      }
      __syncthreads();
      TSTAMP(4);
    }
  }
#ifdef MC_DIAG
  if (p.diag && (threadIdx.x & 63) == 0)
    for (int k = 0; k < 8; ++k) p.diag[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + k] = dacc[k];
#endif
}

// out[i] = sum_g part[g * n + i] in fixed order (k_reduce of mscnn_bwd.hip, small n)
__global__ __launch_bounds__(256) void k_reduce_rows(const float* __restrict__ part, int G, int n, float* __restrict__ out) {
  constexpr int S = 16, IB = 256 / S;
  __shared__ float sp[S][IB];
  const int li = threadIdx.x % IB, s = threadIdx.x / IB;
  const int i = blockIdx.x * IB + li;
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

int trunk_grid(int n, size_t lds) {
  const int per_cu = lds <= 80 * 1024 ? 2 : 1;
  const int cap = per_cu * num_cus();
  return n < cap ? n : cap;
}
// k_trunk_fwd2 (P <= 256): one 512-thread workgroup per CU, two samples each
inline bool fwd_two(int P) { return P <= 256; }
// which forward for P <= 256 cells: MCV_TRUNK_FWD variant 0 (default) = k_trunk_fwd_pp for the no-grad
// forward (the rollout's; 5-6 % faster, same-box A/B, profiles/r06/trunk_fwd_pp_ab.txt) and
// k_trunk_fwd2 for the saving forward (bitwise the per-layer kernels, and 5 % faster there);
// variant 1 = k_trunk_fwd2 always, variant 2 = k_trunk_fwd_pp always
inline bool fwd_pp(int P, int nl, bool save) {
  if (P > 256 || nl > PP_MAXL) return false;
  const int v = g_variant[MCV_TRUNK_FWD];
  return v == 2 || (v == 0 && !save);
}
int trunk_grid2(int n) {
  const int pairs = (n + 1) / 2, cap = num_cus();
  return pairs < cap ? pairs : cap;
}
// workspace slots of the forward: one per sample in flight (either kernel)
int64_t fwd_slots(int n, int P) {
  const int64_t one = trunk_grid(n, tf_lds(P)), two = fwd_two(P) ? 2 * (int64_t)trunk_grid2(n) : 0;
  return one > two ? one : two;
}
// the backward's partial rows: mscnn_bwd.hip make_plan's grid_d
int trunk_vgrid(int n) { return n < 2 * num_cus() ? n : 2 * num_cus(); }

template <typename K>
void lds_attr_once(K kernel, bool& done) {
  if (!done) {
    (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    done = true;
  }
}

int launched(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof g_err, "%s launch: %s", what, hipGetErrorString(e));
    return MS_EHIP;
  }
  return MS_OK;
}

#ifdef MC_DIAG
unsigned long long* g_trunk_diag[2] = {nullptr, nullptr};
int g_trunk_dflags = 0;
#endif

template <typename E, int NPT, bool FULL>
int launch_trunk_fwd(const TrunkFwdParams<E>& p, hipStream_t s) {
  static bool attr = false;
  lds_attr_once(k_trunk_fwd<E, NPT, FULL>, attr);
  const size_t lds = tf_lds(p.H * p.W);
  hipLaunchKernelGGL((k_trunk_fwd<E, NPT, FULL>), dim3(trunk_grid(p.N, lds)), dim3(256), lds, s, p);
  return launched("k_trunk_fwd");
}

template <typename E, int NPT, bool FULL, bool SAVE>
int launch_trunk_fwd_pp_k(const TrunkFwdParams<E>& p, hipStream_t s) {
  static bool attr = false;
  lds_attr_once(k_trunk_fwd_pp<E, NPT, FULL, SAVE>, attr);
  hipLaunchKernelGGL((k_trunk_fwd_pp<E, NPT, FULL, SAVE>), dim3(trunk_grid2(p.N)), dim3(512), pp_lds(p.H * p.W), s, p);
  return launched("k_trunk_fwd_pp");
}
// SAVE: every layer has ysave, stats and relu_mask (the training forward); otherwise none has
template <typename E, int NPT, bool FULL>
int launch_trunk_fwd_pp(const TrunkFwdParams<E>& p, hipStream_t s) {
  return p.L[0].ysave ? launch_trunk_fwd_pp_k<E, NPT, FULL, true>(p, s) : launch_trunk_fwd_pp_k<E, NPT, FULL, false>(p, s);
}

template <typename E, int NPT, bool FULL>
int launch_trunk_fwd2(const TrunkFwdParams<E>& p, hipStream_t s) {
  static bool attr = false;
  lds_attr_once(k_trunk_fwd2<E, NPT, FULL>, attr);
  hipLaunchKernelGGL((k_trunk_fwd2<E, NPT, FULL>), dim3(trunk_grid2(p.N)), dim3(512), tf2_lds(p.H * p.W), s, p);
  return launched("k_trunk_fwd2");
}

template <typename E>
int run_trunk_fwd(const uint16_t* x0, const mc_fwd_layer* layers, int nl, void* work, int n, int h, int w,
                  float eps, float* pooled, hipStream_t s) {
  TrunkFwdParams<E> p;
  memset(&p, 0, sizeof p);
  p.x0 = reinterpret_cast<const E*>(x0);
  p.ws = reinterpret_cast<E*>(work);
  p.pooled = pooled;
  p.NL = nl;
  p.N = n;
  p.H = h;
  p.W = w;
  p.eps = eps;
#ifdef MC_DIAG
  p.diag = g_trunk_diag[0];
  p.dflags = g_trunk_dflags;
#endif
  for (int l = 0; l < nl; ++l) {
    const mc_fwd_layer& a = layers[l];
    p.L[l].wt = reinterpret_cast<const E*>(a.w);
    p.L[l].bias = a.bias;
    p.L[l].gamma = a.gamma;
    p.L[l].beta = a.beta;
    p.L[l].dmask = a.dmask;
    p.L[l].out = reinterpret_cast<E*>(a.out);
    p.L[l].ysave = reinterpret_cast<E*>(a.ysave);
    p.L[l].stats = a.stats;
    p.L[l].rmask = a.relu_mask;
  }
  const int P = h * w;
  // same-box A/B (profiles/r05/trunk_fwd2_ab.txt): the two-sample kernel is 3 % faster on the
  // no-grad forward at 16x16 and 2-6 % at 9x9; on the saving forward at 16x16 it was level while
  // every conv1 output was stored, and is 0.4 ms a minibatch faster since they are recomputed in
  // the weight gradient instead (profiles/r05/trunk_fwd2_save_ab.txt)
  bool uniform = true;  // k_trunk_fwd_pp: saves on every layer or on none
  for (int l = 0; l < nl; ++l)
    uniform &= (layers[l].ysave != nullptr) == (layers[0].ysave != nullptr) &&
               (layers[l].stats != nullptr) == (layers[0].ysave != nullptr) &&
               (layers[l].relu_mask != nullptr) == (layers[0].ysave != nullptr);
  if (fwd_pp(P, nl, layers[0].ysave != nullptr) && uniform) {
    if (P == 256) return launch_trunk_fwd_pp<E, 2, true>(p, s);
    if (P == 128) return launch_trunk_fwd_pp<E, 1, true>(p, s);
    return P < 128 ? launch_trunk_fwd_pp<E, 1, false>(p, s) : launch_trunk_fwd_pp<E, 2, false>(p, s);
  }
  if (fwd_two(P)) {
    if (P == 256) return launch_trunk_fwd2<E, 2, true>(p, s);
    return P <= 128 ? launch_trunk_fwd2<E, 1, false>(p, s) : launch_trunk_fwd2<E, 2, false>(p, s);
  }
  // k_trunk_fwd (one sample per 256-thread workgroup): boards of more than 256 cells
  const int npt = ((P + 31) / 32 + WAVES - 1) / WAVES;
  switch (npt) {
    case 1: return launch_trunk_fwd<E, 1, false>(p, s);
    case 2: return launch_trunk_fwd<E, 2, false>(p, s);
    case 3: return launch_trunk_fwd<E, 3, false>(p, s);
    default: return launch_trunk_fwd<E, 4, false>(p, s);
  }
}

template <typename E, int NPT, int NCH>
int launch_trunk_bwd(const TrunkBwdParams<E>& p, int grid, hipStream_t s) {
  static bool attr = false;
  lds_attr_once(k_trunk_bwd<E, NPT, NCH>, attr);
  hipLaunchKernelGGL((k_trunk_bwd<E, NPT, NCH>), dim3(grid), dim3(256), tb_lds(p.H * p.W), s, p);
  return launched("k_trunk_bwd");
}

template <typename E>
int run_trunk_bwd(const uint16_t* dout, const mc_bwd_layer* layers, int nl, float* dgn, void* work, int n, int h,
                  int w, hipStream_t s) {
  const int P = h * w;
  const int grid = trunk_grid(n, tb_lds(P));
  TrunkBwdParams<E> p;
  memset(&p, 0, sizeof p);
  p.dout = reinterpret_cast<const E*>(dout);
  p.ws = reinterpret_cast<E*>(work);
  p.part = reinterpret_cast<float*>(reinterpret_cast<unsigned char*>(work) + (size_t)grid * P * COUT * 2);
  p.VG = trunk_vgrid(n);
#ifdef MC_DIAG
  p.diag = g_trunk_diag[1];
  p.dflags = g_trunk_dflags;
#endif
  p.NL = nl;
  p.N = n;
  p.H = h;
  p.W = w;
  for (int l = 0; l < nl; ++l) {
    const mc_bwd_layer& a = layers[l];
    p.L[l].y = reinterpret_cast<const E*>(a.ysave);
    p.L[l].stats = a.stats;
    p.L[l].gamma = a.gamma;
    p.L[l].rmask = a.relu_mask;
    p.L[l].dmask = a.dmask;
    p.L[l].wT = reinterpret_cast<const E*>(a.wT);
    p.L[l].dy = reinterpret_cast<E*>(a.dy);
  }
  int rc;
  if (P <= 128) rc = launch_trunk_bwd<E, 1, 13>(p, grid, s);
  else if (P <= 256) rc = launch_trunk_bwd<E, 2, 13>(p, grid, s);
  else if (P <= 384) rc = launch_trunk_bwd<E, 3, 25>(p, grid, s);
  else rc = launch_trunk_bwd<E, 4, 25>(p, grid, s);
  if (rc) return rc;
  const int nout = nl * 3 * COUT;
  hipLaunchKernelGGL(k_reduce_rows, dim3((unsigned)((nout + 15) / 16)), dim3(256), 0, s, p.part, p.VG, nout, dgn);
  return launched("k_reduce_rows");
}

bool trunk_shape_ok(int n, int h, int w, int nl, int max_nl, const char* what) {
  if (n <= 0 || h <= 0 || w <= 0 || nl <= 0 || nl > max_nl) {
    snprintf(g_err, sizeof g_err, "%s: bad sizes (n %d, board %dx%d, %d layers; at most %d)", what, n, h, w, nl, max_nl);
    return false;
  }
  if (h * w > 512 || w > 64) {
    snprintf(g_err, sizeof g_err, "%s: board %dx%d unsupported (at most 512 cells)", what, h, w);
    return false;
  }
  return true;
}

}  // namespace

extern "C" {

#ifdef MC_DIAG
// diagnostics only (not in mscnn.h): per-wave phase cycle totals of the next trunk launches
void mc_set_trunk_diag(unsigned long long* fwd, unsigned long long* bwd) {
  g_trunk_diag[0] = fwd;
  g_trunk_diag[1] = bwd;
}
void mc_set_trunk_dflags(int f) { g_trunk_dflags = f; }
#endif

int64_t mc_trunk_fwd_workspace(int32_t n, int32_t h, int32_t w_) {
  if (n <= 0 || h <= 0 || w_ <= 0 || h * w_ > 512) return -1;
  const int P = h * w_;
  return fwd_slots(n, P) * P * COUT * 2;
}

int mc_trunk_fwd(const uint16_t* x0, const mc_fwd_layer* layers, int32_t nlayers, void* work, int64_t work_bytes,
                 int32_t n, int32_t h, int32_t w_, float eps, int32_t dtype, void* stream) {
  return mc_trunk_fwd_pooled(x0, layers, nlayers, work, work_bytes, nullptr, n, h, w_, eps, dtype, stream);
}

int mc_trunk_fwd_pooled(const uint16_t* x0, const mc_fwd_layer* layers, int32_t nlayers, void* work,
                        int64_t work_bytes, float* pooled, int32_t n, int32_t h, int32_t w_, float eps, int32_t dtype,
                        void* stream) {
  if (!trunk_shape_ok(n, h, w_, nlayers, MAXL, "mc_trunk_fwd")) return MS_EINVAL;
  if (!x0 || !layers || (nlayers & 1)) {
    snprintf(g_err, sizeof g_err, "mc_trunk_fwd: bad argument (x0, layers, or an odd layer count %d)", nlayers);
    return MS_EINVAL;
  }
  for (int l = 0; l < nlayers; ++l) {
    const mc_fwd_layer& a = layers[l];
    if (!a.w || !a.bias || !a.gamma || !a.beta) {
      snprintf(g_err, sizeof g_err, "mc_trunk_fwd: layer %d lacks weights or GroupNorm parameters", l);
      return MS_EINVAL;
    }
    if ((l & 1) && a.dmask) {
      snprintf(g_err, sizeof g_err, "mc_trunk_fwd: layer %d is a conv2 (no dropout)", l);
      return MS_EINVAL;
    }
  }
  if (!layers[nlayers - 1].out) {
    snprintf(g_err, sizeof g_err, "mc_trunk_fwd: the last layer's out is required");
    return MS_EINVAL;
  }
  const int64_t need = mc_trunk_fwd_workspace(n, h, w_);
  bool need_ws = false;
  for (int l = 1; l + 2 < nlayers; l += 2) need_ws |= layers[l].out == nullptr;
  if (need_ws && (!work || work_bytes < need)) {
    snprintf(g_err, sizeof g_err, "mc_trunk_fwd: workspace %lld < %lld bytes", (long long)work_bytes, (long long)need);
    return MS_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MC_DT_BF16) return run_trunk_fwd<__bf16>(x0, layers, nlayers, work, n, h, w_, eps, pooled, s);
  if (dtype == MC_DT_F16) return run_trunk_fwd<_Float16>(x0, layers, nlayers, work, n, h, w_, eps, pooled, s);
  snprintf(g_err, sizeof g_err, "mc_trunk_fwd: dtype %d unsupported (0 bf16, 1 f16)", dtype);
  return MS_EINVAL;
}

int64_t mc_trunk_bwd_workspace(int32_t nlayers, int32_t n, int32_t h, int32_t w_) {
  if (n <= 0 || h <= 0 || w_ <= 0 || h * w_ > 512 || nlayers <= 0 || nlayers > MAXL + 1) return -1;
  const int P = h * w_;
  const int64_t grid = trunk_grid(n, tb_lds(P));
  return grid * P * COUT * 2 + (int64_t)trunk_vgrid(n) * nlayers * 3 * COUT * 4;
}

int mc_trunk_bwd(const uint16_t* dout, const mc_bwd_layer* layers, int32_t nlayers, float* dgn, void* work,
                 int64_t work_bytes, int32_t n, int32_t h, int32_t w_, int32_t dtype, void* stream) {
  if (!trunk_shape_ok(n, h, w_, nlayers, MAXL + 1, "mc_trunk_bwd")) return MS_EINVAL;
  if (!dout || !layers || !dgn || !work || !(nlayers & 1)) {
    snprintf(g_err, sizeof g_err, "mc_trunk_bwd: bad argument (dout, layers, dgn, work, or an even layer count %d)",
             nlayers);
    return MS_EINVAL;
  }
  for (int l = 0; l < nlayers; ++l) {
    const mc_bwd_layer& a = layers[l];
    if (!a.ysave || !a.stats || !a.gamma || !a.relu_mask || !a.dy || ((l == 0) != (a.wT == nullptr))) {
      snprintf(g_err, sizeof g_err, "mc_trunk_bwd: layer %d: ysave, stats, gamma, relu_mask, dy required; wT iff l > 0", l);
      return MS_EINVAL;
    }
    if (l > 0 && !(l & 1) && a.dmask) {
      snprintf(g_err, sizeof g_err, "mc_trunk_bwd: layer %d is a conv2 (no dropout)", l);
      return MS_EINVAL;
    }
  }
  const int64_t need = mc_trunk_bwd_workspace(nlayers, n, h, w_);
  if (work_bytes < need) {
    snprintf(g_err, sizeof g_err, "mc_trunk_bwd: workspace %lld < %lld bytes", (long long)work_bytes, (long long)need);
    return MS_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MC_DT_BF16) return run_trunk_bwd<__bf16>(dout, layers, nlayers, dgn, work, n, h, w_, s);
  if (dtype == MC_DT_F16) return run_trunk_bwd<_Float16>(dout, layers, nlayers, dgn, work, n, h, w_, s);
  snprintf(g_err, sizeof g_err, "mc_trunk_bwd: dtype %d unsupported (0 bf16, 1 f16)", dtype);
  return MS_EINVAL;
}

}  // extern "C"
