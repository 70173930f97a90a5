// mscnn.hip — fused conv3x3 + GroupNorm + residual + ReLU + dropout (gfx950 MFMA).
//
// Reference op chain (minesweeper/models/cnn_residual.py:10-26, 50-54):
//   y = Conv2d(C, 96, 3, padding=1)(x); y = GroupNorm(6, 96)(y); [y += residual]; y = ReLU(y);
//   [y = Dropout2d(p)(y)]
// PyTorch runs this as ~8 kernels per layer (MIOpen conv with NCHW<->NHWC
// transposes, bf16<->f32 casts, 4 GroupNorm kernels, elementwise), 70 % of the
// PPO-update time being glue (profiles/r01/ppo_minibatch_kernel_stats.csv).
//
// Here: one persistent workgroup (4 waves) per sample at a time. The sample's
// NHWC bf16 input tile (with a zero halo) sits in LDS; the conv is an implicit
// GEMM out[px][co] = sum_{tap,ci} x[px+tap][ci] * w[tap][co][ci] on
// v_mfma_f32_32x32x16_bf16 (A = 32 pixels x 16 ci read straight from the halo
// tile, B = 16 ci x 32 co from the tap's LDS-staged weights). Each wave owns
// NPT 32-pixel tiles x all 96 output channels, so a whole GroupNorm group
// (16 channels x all pixels of the sample) lives in the workgroup: mean and
// variance (two-pass) are reduced with DPP row sums + an LDS exchange across
// the 4 waves, and normalisation, affine, residual, ReLU and the dropout scale
// are applied in the epilogue before a single bf16 store.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/msenv.h"
#include "../../include/mscnn.h"
#include "mscnn_common.h"

namespace mc {

thread_local char g_err[256] = "";
int g_variant[MCV_COUNT] = {0, 0, 0, 0};

int num_cus() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0, v = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    ncu = v > 0 ? v : 256;
  }
  return ncu;
}

}  // namespace mc

namespace {

using namespace mc;

template <typename E>
struct FwdParams {
  const E* x;
  const E* wt;
  const float* bias;
  const float* gamma;
  const float* beta;
  const E* res;
  const float* dmask;
  E* out;
  E* ysave;
  float* stats;
  uint8_t* rmask;  // optional ReLU bitmask [N][P][12]: bit j of byte (px, c8) = out[px][8*c8 + j] > 0
  int N, H, W;
  float eps;
  unsigned long long* diag;  // MC_DIAG builds: per-workgroup phase cycle totals [grid][8]
};

// LDS layout (bf16 elements):
//   region0: sX[P+1][CINP] input tile, row P = zeros (every out-of-board tap read of
//            every lane points there: no halo, no masking); after the conv the same
//            bytes hold sO[P][96] (y staged for the coalesced epilogue);
//   sW[COUT][CINP]: the weights of one tap (single buffer: ~75 KB in all, so two
//            workgroups share a CU and cover one another's barriers and epilogues);
//   f32 sRed[WAVES][NGRP], sGB[2][COUT] (gamma, beta), sAB[3][COUT].
template <int CIN>
constexpr int cinp() { return CIN + 8; }  // +16 B per pixel row: conflict-free ds_read_b128

template <int CIN>
__host__ __device__ inline int region0_elems(int H, int W) {
  const int a = (H * W + 1) * cinp<CIN>(), b = H * W * COUT;
  return ((a > b ? a : b) + 7) & ~7;
}

#ifdef MC_DIAG
#define FSTAMP(k)                                      \
  do {                                                 \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    dacc[k] += t_ - tlast;                             \
    tlast = t_;                                        \
  } while (0)
#else
#define FSTAMP(k) do { } while (0)
#endif

// (macros rather than lambdas: captured register arrays would be demoted to scratch)
#define MC_LOAD_IN(n_, v_)                                                              \
  do {                                                                                  \
    const u32x4* xs_ = reinterpret_cast<const u32x4*>(p.x + (size_t)(n_) * P * CIN);   \
    _Pragma("unroll") for (int k_ = 0; k_ < NPF; ++k_) {                                \
      const int i_ = tid + 256 * k_;                                                    \
      if ((FULL && k_ < C8) || i_ < P * C8) v_[k_] = xs_[i_]; /* FULL: P = 256 */      \
    }                                                                                   \
  } while (0)
#define MC_LOAD_W(tap_, v_)                                                             \
  do {                                                                                  \
    const u32x4* ws_ = reinterpret_cast<const u32x4*>(p.wt + (size_t)(tap_) * COUT * CIN); \
    _Pragma("unroll") for (int k_ = 0; k_ < NWC; ++k_) {                                \
      const int i_ = tid + 256 * k_;                                                    \
      if (k_ < COUT * C8 / 256 || i_ < COUT * C8) v_[k_] = ws_[i_]; /* static: full */ \
    }                                                                                   \
  } while (0)
#define MC_STORE_W(v_)                                                                  \
  do {                                                                                  \
    _Pragma("unroll") for (int k_ = 0; k_ < NWC; ++k_) {                                \
      const int i_ = tid + 256 * k_;                                                    \
      if (k_ < COUT * C8 / 256 || i_ < COUT * C8) {                                    \
        const int co_ = i_ / C8, c8_ = i_ - co_ * C8;                                   \
        *reinterpret_cast<u32x4*>(&sW[co_ * CINP + c8_ * 8]) = v_[k_];                  \
      }                                                                                 \
    }                                                                                   \
  } while (0)

// Two workgroups per CU (~75 KB of LDS each) cover one another's barriers and epilogues;
// nothing is held in registers across phases.
template <typename E, int CIN, int NPT, bool FULL>
__global__ __launch_bounds__(256, NPT <= 2 ? 2 : 1) void k_conv_gn_fwd(FwdParams<E> p) {
  // no contraction: every expression rounds the same way in the per-layer and the one-launch
  // kernels (explicit fmaf where a fused multiply-add is wanted), so they agree bitwise
#pragma clang fp contract(off)
  typedef typename EV<E>::v8 E8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int CINP = cinp<CIN>();
  constexpr int C8 = CIN / 8;
  constexpr int NPF = (NPT * 128 * C8 + 255) / 256;  // 16-B input chunks per thread
  constexpr int NWC = (COUT * C8 + 255) / 256;        // 16-B weight chunks per thread and tap
  const int H = p.H, W = p.W, P = H * W;
  E* sX = reinterpret_cast<E*>(smem);
  E* sO = sX;
  E* sW = sX + region0_elems<CIN>(H, W);
  float* sRed = reinterpret_cast<float*>(sW + COUT * CINP);
  float* sGB = sRed + WAVES * NGRP;  // [gamma | beta]
  float* sAB = sGB + 2 * COUT;        // per sample: [scale | shift | dropout scale]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;

  for (int i = tid; i < COUT; i += 256) {
    sGB[i] = p.gamma[i];
    sGB[COUT + i] = p.beta[i];
  }
  int qr[NPT], qc[NPT];  // this lane's output pixel of each 32-pixel tile
#pragma unroll
  for (int t = 0; t < NPT; ++t) {
    const int q = (wave * NPT + t) * 32 + l32;
    qr[t] = q < P ? q / W : -1000;  // a pixel past P reads the zero row at every tap
    qc[t] = q < P ? q - qr[t] * W : -1000;
  }
  u32x4 wr[NWC];
  u32x4 xin[NPF];
  constexpr int NEC = (NPT * 128 * (COUT / 8) + 255) / 256;  // 16-B output chunks per thread
#ifdef MC_DIAG
  unsigned long long dacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif
  for (int n = blockIdx.x; n < p.N; n += gridDim.x) {
    // loop-variant copy of tid: keeps the per-chunk address math inside the loop instead of
    // hoisting a dozen 64-bit addresses out of it (they would be spilled)
    const int tid = threadIdx.x + opaque0();
    // ---- stage the input tile (the zero row is re-written: the epilogue reuses region0) ----
    MC_LOAD_IN(n, xin);
    for (int i = tid; i < C8; i += 256) *reinterpret_cast<u32x4*>(&sX[P * CINP + i * 8]) = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < NPF; ++k) {
      const int i = tid + 256 * k;
      if ((FULL && k < C8) || i < P * C8) {  // FULL: P = 256, every chunk in range
        const int px = i / C8, c8 = i - px * C8;
        *reinterpret_cast<u32x4*>(&sX[px * CINP + c8 * 8]) = xin[k];
      }
    }
    MC_LOAD_W(0, wr);
    MC_STORE_W(wr);
    __syncthreads();
    FSTAMP(0);  // stage input + tap-0 weights

    f32x16 acc[NPT][3];
#pragma unroll
    for (int t = 0; t < NPT; ++t)
#pragma unroll
      for (int ct = 0; ct < 3; ++ct)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[t][ct][i] = 0.f;

    for (int tap = 0; tap < 9; ++tap) {
      if (tap + 1 < 9) MC_LOAD_W(tap + 1, wr);
      const int dr = tap / 3 - 1, dc = tap % 3 - 1;
      int aoff[NPT];
#pragma unroll
      for (int t = 0; t < NPT; ++t) {
        const int sr = qr[t] + dr, sc = qc[t] + dc;
        const bool v = (unsigned)sr < (unsigned)H && (unsigned)sc < (unsigned)W;
        aoff[t] = (v ? sr * W + sc : P) * CINP + 8 * hh;
      }
      // k steps with double-buffered operands, order pinned: step k+1's LDS reads are
      // issued before step k's MFMAs (left alone, the scheduler reuses one operand set
      // and waits on every read)
      constexpr int KS = CIN / 16;
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
          for (int ct = 0; ct < 3; ++ct)
            acc[t][ct] = mfma32(A[ks & 1][t], B[ks & 1][ct], acc[t][ct]);
        __builtin_amdgcn_sched_group_barrier(0x008, 3 * NPT, 0);
      }
      __syncthreads();  // sW (and after the last tap sX) fully read
      if (tap + 1 < 9) {
        MC_STORE_W(wr);
        __syncthreads();
      }
    }

    FSTAMP(1);  // 9 taps
    // ---------------- epilogue A: bias, GroupNorm statistics, y -> LDS ----------------
    float biasv[3];
#pragma unroll
    for (int ct = 0; ct < 3; ++ct) biasv[ct] = p.bias[ct * 32 + l32];
    float gmean[NGRP], grstd[NGRP];
    const float inv_cnt = 1.0f / (16.0f * (float)P);
    for (int pass = 0; pass < 2; ++pass) {
      float part[3];
#pragma unroll
      for (int ct = 0; ct < 3; ++ct) {
        const float mu = pass ? gmean[2 * ct + (l32 >> 4)] : 0.f;
        float v[NPT * 16];  // pairwise tree below: a serial += chain is NPT*16 dependent adds
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
      float gs[3][2];  // readlanes in converged control flow (see note in the stats exchange)
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
    FSTAMP(2);  // GroupNorm statistics
    if (p.stats && tid < NGRP) {
      float m = 0.f, r = 0.f;
#pragma unroll
      for (int g = 0; g < NGRP; ++g)
        if (g == tid) {
          m = gmean[g];
          r = grstd[g];
        }
      p.stats[((size_t)n * NGRP + tid) * 2 + 0] = m;
      p.stats[((size_t)n * NGRP + tid) * 2 + 1] = r;
    }
#pragma unroll
    for (int ct = 0; ct < 3; ++ct)
#pragma unroll
      for (int t = 0; t < NPT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int px = (wave * NPT + t) * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
          if (FULL || px < P) sO[px * COUT + ct * 32 + l32] = (E)pin_f32(acc[t][ct][i] + biasv[ct]);
        }
    FSTAMP(3);  // y -> LDS
    if (tid < COUT) {  // z = y * scale + shift (+ res), then ReLU, then * dropout scale
      const int g = tid >> 4;
      float mu = 0.f, rs = 0.f;
#pragma unroll
      for (int gg = 0; gg < NGRP; ++gg)
        if (gg == g) {
          mu = gmean[gg];
          rs = grstd[gg];
        }
      const float a = sGB[tid] * rs;
      sAB[tid] = a;
      sAB[COUT + tid] = sGB[COUT + tid] - mu * a;
      sAB[2 * COUT + tid] = p.dmask ? p.dmask[(size_t)n * COUT + tid] : 1.0f;
    }
    __syncthreads();

    // ---------------- epilogue B: coalesced 16-B chunks of [px][co] ----------------
    // chunk c = tid + 256k covers channels ((tid + 4k) mod 12) * 8 ..+8: three channel
    // groups per thread, their scale / shift / dropout scale kept in registers
    float ca[3][8], cb[3][8], cd[3][8];
#pragma unroll
    for (int j3 = 0; j3 < 3; ++j3) {
      const int cg = ((tid % (COUT / 8)) + 4 * j3) % (COUT / 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ca[j3][j] = sAB[cg * 8 + j];
        cb[j3][j] = sAB[COUT + cg * 8 + j];
        cd[j3][j] = sAB[2 * COUT + cg * 8 + j];
      }
    }
    // residual chunks are loaded RB at a time, all of a batch before its first store: a
    // load issued after a store waits for that store too (vmcnt counts both), so one
    // load per chunk would drain the stores once per chunk
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
          if (p.res && k + u < NEC && ((FULL && k + u < NEC) || cu < P * (COUT / 8)))
            rq[u] = *reinterpret_cast<const u32x4*>(&p.res[(size_t)n * P * COUT + (size_t)cu * 8]);
        }
      }
      if ((FULL && k < NEC) || c < P * (COUT / 8)) {
        const size_t o = (size_t)n * P * COUT + (size_t)c * 8;
        const u32x4 yv = *reinterpret_cast<const u32x4*>(&sO[c * 8]);
        if (p.ysave) *reinterpret_cast<u32x4*>(&p.ysave[o]) = yv;
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
        *reinterpret_cast<u32x4*>(&p.out[o]) = __builtin_bit_cast(u32x4, o8);
        if (p.rmask) p.rmask[(size_t)n * P * (COUT / 8) + c] = (uint8_t)mb;
      }
    }
    FSTAMP(4);  // scale/shift + outputs issued
    __syncthreads();  // region0 is re-staged with the next input
    FSTAMP(5);
  }
#ifdef MC_DIAG
  if (p.diag && threadIdx.x == 0)
    for (int k = 0; k < 8; ++k) p.diag[blockIdx.x * 8 + k] = dacc[k];
#endif
}

template <typename E, int CIN, int NPT, bool FULL>
int launch_fwd(const FwdParams<E>& p, hipStream_t s) {
  constexpr int CINP = cinp<CIN>();
  const size_t lds = (size_t)region0_elems<CIN>(p.H, p.W) * 2 + (size_t)COUT * CINP * 2 + WAVES * NGRP * 4 +
                     5 * COUT * 4;
  if (lds > 160 * 1024) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_fwd: board %dx%d needs %zu B LDS", p.H, p.W, lds);
    return MS_EINVAL;
  }
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_conv_gn_fwd<E, CIN, NPT, FULL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr_set = true;
  }
  const int per_cu = lds <= 80 * 1024 ? 2 : 1;
  const int cap = per_cu * num_cus();
  const int grid = p.N < cap ? p.N : cap;
  hipLaunchKernelGGL((k_conv_gn_fwd<E, CIN, NPT, FULL>), dim3(grid), dim3(256), lds, s, p);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_fwd launch: %s", hipGetErrorString(e));
    return MS_EHIP;
  }
  return MS_OK;
}

template <typename E, int CIN>
int dispatch_fwd(const FwdParams<E>& p, hipStream_t s) {
  const int P = p.H * p.W;
  const int tiles = (P + 31) / 32;
  const int npt = (tiles + WAVES - 1) / WAVES;
  if (P == 256) return launch_fwd<E, CIN, 2, true>(p, s);
  switch (npt) {
    case 1: return launch_fwd<E, CIN, 1, false>(p, s);
    case 2: return launch_fwd<E, CIN, 2, false>(p, s);
    case 3: return launch_fwd<E, CIN, 3, false>(p, s);
    case 4: return launch_fwd<E, CIN, 4, false>(p, s);
    default:
      snprintf(g_err, sizeof g_err, "mc_conv_gn_fwd: %d pixels > 512 unsupported", P);
      return MS_EINVAL;
  }
}

}  // namespace


// ---------------------------------------------------------------------------------------
// Observation codes: the one-hot obs of a cell (env.py:172-192: plane 0 = revealed, plane
// 1 + k = revealed with k adjacent mines; all zero before the board's first click) is one
// byte, 0 = hidden, 1 + k = revealed with k. The rollout buffer stores codes [N][A]
// (A bytes per sample instead of 40 A), and the trunk's input [N][A][cin_pad] 16-bit is
// expanded from them; exact for every obs the env writes. k_obs_encode's stem input is the
// planes' own values cast to 16 bits (exact for any f32 input that 16 bits hold).
template <typename E>
__device__ __forceinline__ void store_onehot16(E* dst, uint32_t code, int cin_pad) {
  // channels 0..cin_pad-1 (16): 1 at channel 0 and 1 + k when code = 1 + k > 0
  typedef typename EV<E>::v8 E8;
  E8 lo, hi;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    lo[j] = (E)((j == 0 && code) || (code && (uint32_t)j == code) ? 1.0f : 0.0f);
    hi[j] = (E)(code && (uint32_t)(j + 8) == code ? 1.0f : 0.0f);
  }
  *reinterpret_cast<E8*>(dst) = lo;
  if (cin_pad > 8) *reinterpret_cast<E8*>(dst + 8) = hi;
}

template <typename E>
__global__ __launch_bounds__(256) void k_obs_encode(const float* __restrict__ obs, uint8_t* __restrict__ codes,
                                                    E* __restrict__ nhwc, int64_t n, int a, int cin_pad) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // cell of the [n][a] grid
  if (i >= n * a) return;
  const int64_t sm = i / a;
  const int c = (int)(i - sm * a);
  const float* o = obs + sm * 10 * a + c;
  float v[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) v[k] = o[(int64_t)k * a];  // coalesced per plane
  uint32_t code = 0u;
  if (v[0] != 0.f) {
#pragma unroll
    for (int k = 0; k < 9; ++k)
      if (v[1 + k] != 0.f) code = 1u + (uint32_t)k;
  }
  if (codes) codes[i] = (uint8_t)code;
  if (nhwc) {  // the planes' own values (exact for any input, not only one-hot env obs)
    typedef typename EV<E>::v8 E8;
    E8 lo, hi;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      lo[j] = (E)v[j];
      hi[j] = (E)(j < 2 ? v[8 + j] : 0.0f);
    }
    *reinterpret_cast<E8*>(nhwc + i * cin_pad) = lo;
    *reinterpret_cast<E8*>(nhwc + i * cin_pad + 8) = hi;
  }
}

template <typename E>
__global__ __launch_bounds__(256) void k_codes_to_nhwc(const uint8_t* __restrict__ codes, E* __restrict__ nhwc,
                                                       int64_t cells, int cin_pad) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= cells) return;
  store_onehot16(nhwc + i * cin_pad, (uint32_t)codes[i], cin_pad);
}

#ifdef MC_DIAG
unsigned long long* g_fwd_diag = nullptr;
#endif

namespace {

template <typename E>
int run_fwd(const uint16_t* x, const uint16_t* w, const float* bias, const float* gamma, const float* beta,
            const uint16_t* res, const float* dmask, uint16_t* out, uint16_t* ysave, float* stats, uint8_t* relu_mask,
            int32_t n, int32_t h, int32_t w_, int32_t cin, float eps, hipStream_t s) {
  FwdParams<E> p;
  p.x = reinterpret_cast<const E*>(x);
  p.wt = reinterpret_cast<const E*>(w);
  p.bias = bias;
  p.gamma = gamma;
  p.beta = beta;
  p.res = reinterpret_cast<const E*>(res);
  p.dmask = dmask;
  p.out = reinterpret_cast<E*>(out);
  p.ysave = reinterpret_cast<E*>(ysave);
  p.stats = stats;
  p.rmask = relu_mask;
  p.N = n;
  p.H = h;
  p.W = w_;
  p.eps = eps;
  p.diag = nullptr;
#ifdef MC_DIAG
  p.diag = g_fwd_diag;
#endif
  return cin == 16 ? dispatch_fwd<E, 16>(p, s) : dispatch_fwd<E, 96>(p, s);
}

}  // namespace

extern "C" {

const char* mc_last_error(void) { return g_err; }

int mc_set_variant(int32_t kernel, int32_t variant) {
  static const int vmax[MCV_COUNT] = {1, 1, 3, 2};  // fwd, data backward, weight gradient, trunk fwd
  if (kernel < 0 || kernel >= MCV_COUNT || variant < 0 || variant > vmax[kernel]) {
    snprintf(g_err, sizeof g_err, "mc_set_variant: bad kernel %d / variant %d", kernel, variant);
    return MS_EINVAL;
  }
  g_variant[kernel] = variant;
  return MS_OK;
}

int mc_obs_encode(const float* obs, uint8_t* codes, uint16_t* nhwc, int64_t n, int32_t a, int32_t cin_pad,
                  int32_t dtype, void* stream) {
  if (!obs || (!codes && !nhwc) || n <= 0 || a <= 0 || a > 255 * 255 || (nhwc && cin_pad != 16)) {
    snprintf(g_err, sizeof g_err, "mc_obs_encode: bad argument");
    return MS_EINVAL;
  }
  const unsigned grid = (unsigned)((n * a + 255) / 256);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MC_DT_BF16)
    hipLaunchKernelGGL(k_obs_encode<__bf16>, dim3(grid), dim3(256), 0, s, obs, codes, reinterpret_cast<__bf16*>(nhwc), n, a, cin_pad);
  else if (dtype == MC_DT_F16)
    hipLaunchKernelGGL(k_obs_encode<_Float16>, dim3(grid), dim3(256), 0, s, obs, codes, reinterpret_cast<_Float16*>(nhwc), n, a, cin_pad);
  else {
    snprintf(g_err, sizeof g_err, "mc_obs_encode: dtype %d unsupported (0 bf16, 1 f16)", dtype);
    return MS_EINVAL;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof g_err, "mc_obs_encode launch: %s", hipGetErrorString(e));
    return MS_EHIP;
  }
  return MS_OK;
}

int mc_codes_to_nhwc(const uint8_t* codes, uint16_t* nhwc, int64_t n, int32_t a, int32_t cin_pad, int32_t dtype,
                     void* stream) {
  if (!codes || !nhwc || n <= 0 || a <= 0 || cin_pad != 16) {
    snprintf(g_err, sizeof g_err, "mc_codes_to_nhwc: bad argument");
    return MS_EINVAL;
  }
  const int64_t cells = n * a;
  const unsigned grid = (unsigned)((cells + 255) / 256);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MC_DT_BF16)
    hipLaunchKernelGGL(k_codes_to_nhwc<__bf16>, dim3(grid), dim3(256), 0, s, codes, reinterpret_cast<__bf16*>(nhwc), cells, cin_pad);
  else if (dtype == MC_DT_F16)
    hipLaunchKernelGGL(k_codes_to_nhwc<_Float16>, dim3(grid), dim3(256), 0, s, codes, reinterpret_cast<_Float16*>(nhwc), cells, cin_pad);
  else {
    snprintf(g_err, sizeof g_err, "mc_codes_to_nhwc: dtype %d unsupported (0 bf16, 1 f16)", dtype);
    return MS_EINVAL;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof g_err, "mc_codes_to_nhwc launch: %s", hipGetErrorString(e));
    return MS_EHIP;
  }
  return MS_OK;
}

#ifdef MC_DIAG
// diagnostics only (not in mscnn.h): per-workgroup phase cycle totals of the next forwards
void mc_set_fwd_diag(unsigned long long* d) { g_fwd_diag = d; }
#endif

int mc_conv_gn_fwd(const uint16_t* x, const uint16_t* w, const float* bias, const float* gamma, const float* beta,
                   const uint16_t* res, const float* dmask, uint16_t* out, uint16_t* ysave, float* stats,
                   uint8_t* relu_mask, int32_t n, int32_t h, int32_t w_, int32_t cin, float eps, int32_t dtype,
                   void* stream) {
  if (!x || !w || !bias || !gamma || !beta || !out || n <= 0 || h <= 0 || w_ <= 0) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_fwd: bad argument");
    return MS_EINVAL;
  }
  if (cin != 16 && cin != 96) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_fwd: cin %d unsupported (16 or 96)", cin);
    return MS_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MC_DT_BF16) return run_fwd<__bf16>(x, w, bias, gamma, beta, res, dmask, out, ysave, stats, relu_mask, n, h, w_, cin, eps, s);
  if (dtype == MC_DT_F16) return run_fwd<_Float16>(x, w, bias, gamma, beta, res, dmask, out, ysave, stats, relu_mask, n, h, w_, cin, eps, s);
  snprintf(g_err, sizeof g_err, "mc_conv_gn_fwd: dtype %d unsupported (0 bf16, 1 f16)", dtype);
  return MS_EINVAL;
}

}  // extern "C"
