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
int g_variant[MCV_COUNT] = {0, 0, 0};

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
  int exp;                   // MC_DIAG builds: WS timing experiments (WSX_* bits; results wrong)
};

// MC_DIAG-only timing experiments of the wave-specialised forward (mc_set_fwd_exp): each bit
// removes one component so that its cost shows in the kernel time. Outputs are garbage.
enum { WSX_NO_MFMA = 1, WSX_NO_MEM = 2, WSX_NO_WSTREAM = 4, WSX_NO_STATS = 8 };
#if defined(MC_DIAG) || defined(MC_WSX)
#define WSX(bit) ((p.exp & (bit)) != 0)
#else
#define WSX(bit) false
#endif

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
          if (FULL || px < P) sO[px * COUT + ct * 32 + l32] = (E)(acc[t][ct][i] + biasv[ct]);
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
          const float z = fmaxf((float)y8[j] * ca[k % 3][j] + cb[k % 3][j] + (float)r8[j], 0.f);
          o8[j] = (E)(z * cd[k % 3][j]);
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

// ---------------------------------------------------------------------------------------
// Wave-specialised forward, boards of P <= 256 pixels: ONE 512-thread workgroup per CU.
//   waves 0-3, the conv waves: the implicit GEMM of sample it, transposed (D[co][px] =
//     W[co][k] . X^T[k][px], so a lane holds one pixel and four consecutive channels per
//     register quad, and the accumulators start at the bias), its GroupNorm statistics and
//     y -> LDS; they also stream the conv weights tap by tap through a two-slot LDS ring
//     (tap g+1 written while tap g is read; loads issued one tap ahead);
//   waves 4-7, the memory waves: the epilogue of sample it-1 (affine, residual, ReLU, dropout;
//     y, out and ReLU-bit stores) and the staging of sample it+1's input.
// Two sample regions alternate: the conv waves read x(it) from region it&1 and leave y(it)
// there; the memory waves read y(it-1) from the other region, then stage x(it+1) over it.
// Each SIMD holds one conv and one memory wave, so the MFMA phase of one sample runs beside the
// HBM phase of its neighbours (round 3's SQ counters showed the two independent 256-thread
// workgroups per CU lining their phases up instead). Every wave passes the same 11 barriers per
// iteration (loop top, 8 between taps, 2 for the statistics): the memory waves' work is laid
// over the first taps' segments, their loads issued six segments before use.
constexpr int YS = COUT + 8;  // y staging row stride (elements): 2-way ds_write_b64, conflict-free b128 reads
constexpr int WS_FLOATS = COUT + 2 * COUT + 2 * 3 * COUT + 2 * WAVES * NGRP + 4;  // + 2 group-barrier counters

template <int CIN>
__host__ __device__ inline int ws_region_elems(int P) {
  const int a = (P + 1) * cinp<CIN>(), b = P * YS;
  return ((a > b ? a : b) + 7) & ~7;
}
template <int CIN>
__host__ __device__ inline size_t ws_lds_bytes(int P) {
  return (size_t)2 * ws_region_elems<CIN>(P) * 2 + (size_t)2 * COUT * cinp<CIN>() * 2 + (size_t)WS_FLOATS * 4;
}

// MC_DIAG builds: per segment (the stretch after each of the 11 barriers) the s_memtime ticks a
// wave spent working and then waiting at the next barrier, for conv wave 0 and memory wave 4:
// diag[(workgroup * 2 + role) * 24 + k] = work of segment k, [.. + 12 + k] = wait before barrier k+1.
#ifdef MC_DIAG
#define WS_DIAG_DECL                                  \
  unsigned long long dwork[11], dwait[11];             \
  for (int k_ = 0; k_ < 11; ++k_) dwork[k_] = dwait[k_] = 0ull; \
  unsigned long long tprev = __builtin_amdgcn_s_memtime()
#define WS_BAR(seg)                                          \
  do {                                                       \
    const unsigned long long t0_ = __builtin_amdgcn_s_memtime(); \
    lds_barrier();                                           \
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime(); \
    dwork[(seg)] += t0_ - tprev;                             \
    dwait[(seg)] += t1_ - t0_;                               \
    tprev = t1_;                                             \
  } while (0)
#define WS_GBAR(seg, cnt, tgt)                               \
  do {                                                       \
    const unsigned long long t0_ = __builtin_amdgcn_s_memtime(); \
    grp_bar((cnt), (tgt), lane);                             \
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime(); \
    dwork[(seg)] += t0_ - tprev;                             \
    dwait[(seg)] += t1_ - t0_;                               \
    tprev = t1_;                                             \
  } while (0)
#define WS_DIAG_OUT(role)                                                                   \
  do {                                                                                      \
    if (p.diag && (threadIdx.x & 255) == 0)                                                 \
      for (int k_ = 0; k_ < 11; ++k_) {                                                     \
        p.diag[((size_t)blockIdx.x * 2 + (role)) * 24 + k_] = dwork[k_];                    \
        p.diag[((size_t)blockIdx.x * 2 + (role)) * 24 + 12 + k_] = dwait[k_];               \
      }                                                                                     \
  } while (0)
#else
#define WS_DIAG_DECL do { } while (0)
#define WS_BAR(seg) lds_barrier()
#define WS_GBAR(seg, cnt, tgt) grp_bar((cnt), (tgt), lane)
#define WS_DIAG_OUT(role) do { } while (0)
#endif

// GB: the roles sync inside an iteration with their own LDS-counter barriers (grp_bar) and meet
// at one s_barrier per iteration; without GB every wave passes all 11 s_barriers.
template <typename E, int CIN, int NPT, bool FULL, bool GB>
__global__ __launch_bounds__(512, 1) void k_conv_gn_fwd_ws(FwdParams<E> p) {
  typedef typename EV<E>::v8 E8;
  typedef typename EV<E>::v4 E4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int CINP = cinp<CIN>(), C8 = CIN / 8, KS = CIN / 16;
  constexpr int NWC = (COUT * C8 + 255) / 256;        // 16-B weight chunks per conv thread and tap
  constexpr int NXC = (NPT * 128 * C8 + 255) / 256;   // 16-B input chunks per memory thread
  constexpr int NEC = NPT * 128 * (COUT / 8) / 256;   // 16-B output chunks per memory thread (6 NPT)
  constexpr int EPS = NEC / 3;                        // of them per epilogue segment (one c8 each)
  const int H = p.H, W = p.W, P = H * W;
  const int REG = ws_region_elems<CIN>(P);
  E* sReg = reinterpret_cast<E*>(smem);  // [2][REG]
  E* sRing = sReg + 2 * REG;             // [2][COUT][CINP]
  float* sBias = reinterpret_cast<float*>(sRing + 2 * COUT * CINP);
  float* sGB = sBias + COUT;           // gamma | beta
  float* sCoef = sGB + 2 * COUT;       // [2][scale | shift | dropout scale][COUT]
  float* sRed = sCoef + 6 * COUT;      // [2 passes][WAVES][NGRP]
  unsigned* sCnt = reinterpret_cast<unsigned*>(sRed + 2 * WAVES * NGRP);  // conv | memory grp_bar counters
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const int G = gridDim.x;
  const int cnt = p.N > (int)blockIdx.x ? (p.N - 1 - (int)blockIdx.x) / G + 1 : 0;

  if (wave < WAVES) {
    // =============================== conv waves ===============================
    const int ctid = threadIdx.x;
    const int l32 = lane & 31, hh = lane >> 5;
    WS_DIAG_DECL;
    for (int i = ctid; i < COUT; i += 256) {
      sBias[i] = p.bias[i];
      sGB[i] = p.gamma[i];
      sGB[COUT + i] = p.beta[i];
    }
    if (ctid < 2) sCnt[ctid] = 0u;
    unsigned gbt = 0u;  // GB: this role's barriers passed x 4
#define CONV_BAR(seg)                      \
  do {                                     \
    if (GB) WS_GBAR(seg, &sCnt[0], gbt += 4u); \
    else WS_BAR(seg);                      \
  } while (0)
    // Weight taps are prefetched WPF taps ahead into WPF register sets (set = tap mod WPF, static in
    // the unrolled tap loop): the conv waves' weight loads share the CU's vector-memory path with
    // the memory waves' HBM streams and queue behind them, so one tap of cover (~1.2k cycles of
    // MFMA) is not enough.
    constexpr int WPF = 3;
    static_assert(9 % WPF == 0, "tap sets repeat per sample");
    u32x4 wr[WPF][NWC];
    // every load unconditional (a clamped chunk index for the partial last chunk): the waitcnt
    // pass then sees the same number of loads per tap and waits only for the set it stores,
    // instead of vmcnt(0) behind a conditionally skipped load
    auto wload = [&](int tap, u32x4 (&w)[NWC]) {
      const u32x4* ws = reinterpret_cast<const u32x4*>(p.wt + (size_t)tap * COUT * CIN);
#pragma unroll
      for (int k = 0; k < NWC; ++k) {
        const int i = ctid + 256 * k;
        w[k] = ws[i < COUT * C8 ? i : COUT * C8 - 1];
      }
    };
    auto wstore = [&](int slot, const u32x4 (&w)[NWC]) {
      E* sw = sRing + slot * COUT * CINP;
#pragma unroll
      for (int k = 0; k < NWC; ++k) {
        const int i = ctid + 256 * k;
        if (k < COUT * C8 / 256 || i < COUT * C8) {
          const int co = i / C8, c8 = i - co * C8;
          *reinterpret_cast<u32x4*>(&sw[co * CINP + c8 * 8]) = w[k];
        }
      }
    };
    wload(0, wr[0]);
    wstore(0, wr[0]);
#pragma unroll
    for (int k = 1; k <= WPF; ++k) wload(k % 9, wr[k % WPF]);
    int qr[NPT], qc[NPT];
    bool qv[NPT];
#pragma unroll
    for (int t = 0; t < NPT; ++t) {
      const int q = (wave * NPT + t) * 32 + l32;
      qv[t] = FULL || q < P;
      qr[t] = qv[t] ? q / W : -1000;  // a pixel past P reads the zero row at every tap
      qc[t] = qv[t] ? q - qr[t] * W : -1000;
    }
    const float inv_cnt = 1.0f / (16.0f * (float)P);
    const int total = 9 * cnt;  // weight taps streamed by this workgroup
    for (int it = 0; it <= cnt; ++it) {
      const bool conv = it < cnt;
      const int n = (int)blockIdx.x + it * G;
      const E* sX = sReg + (it & 1) * REG;
      float dmv = 1.f;
      WS_BAR(10);  // A: x(it) staged, tap 0 in its slot
      f32x16 acc[NPT][3];
      if (conv) {
        if (p.dmask && ctid < COUT) dmv = p.dmask[(size_t)n * COUT + ctid];  // used after the taps
#pragma unroll
        for (int ct = 0; ct < 3; ++ct)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4 b4 = *reinterpret_cast<const f32x4*>(&sBias[ct * 32 + 8 * j + 4 * hh]);
#pragma unroll
            for (int t = 0; t < NPT; ++t)
#pragma unroll
              for (int e = 0; e < 4; ++e) acc[t][ct][4 * j + e] = b4[e];
          }
      }
#pragma unroll 1
      for (int t3 = 0; t3 < 9; t3 += WPF)
#pragma unroll
      for (int u = 0; u < WPF; ++u) {  // (the register set index (tap + 1) mod WPF is static)
        const int tap = t3 + u;
        if (tap) CONV_BAR(tap - 1);  // T_tap: the ring slot of this tap is written, the other one free
        if (!conv) continue;
        const int g = it * 9 + tap;
        // set (tap+1) mod WPF holds tap (g+1) mod 9; refill it with tap g+1+WPF
        if (!WSX(WSX_NO_WSTREAM)) {
          if (g + 1 < total) wstore((g + 1) & 1, wr[(u + 1) % WPF]);
          wload((tap + 1 + WPF) % 9, wr[(u + 1) % WPF]);  // (past the last tap: unused, harmless)
        }
        if (WSX(WSX_NO_MFMA)) continue;
        const E* sW = sRing + (g & 1) * COUT * CINP;
        const int dr = tap / 3 - 1, dc = tap % 3 - 1;
        int aoff[NPT];
#pragma unroll
        for (int t = 0; t < NPT; ++t) {
          const int sr = qr[t] + dr, sc = qc[t] + dc;
          const bool v = (unsigned)sr < (unsigned)H && (unsigned)sc < (unsigned)W;
          aoff[t] = (v ? sr * W + sc : P) * CINP + 8 * hh;
        }
        E8 A[2][3], B[2][NPT];  // A: weights (32 co x 16 k), B: input (16 k x 32 px)
        auto ld = [&](int ks, E8 (&a)[3], E8 (&b)[NPT]) {
#pragma unroll
          for (int ct = 0; ct < 3; ++ct)
            a[ct] = *reinterpret_cast<const E8*>(&sW[(ct * 32 + l32) * CINP + ks * 16 + 8 * hh]);
#pragma unroll
          for (int t = 0; t < NPT; ++t) b[t] = *reinterpret_cast<const E8*>(&sX[aoff[t] + ks * 16]);
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
            for (int ct = 0; ct < 3; ++ct) acc[t][ct] = mfma32(A[ks & 1][ct], B[ks & 1][t], acc[t][ct]);
          __builtin_amdgcn_sched_group_barrier(0x008, 3 * NPT, 0);
        }
      }
      // ---- GroupNorm statistics: group 2 ct + half = registers 8 half .. 8 half + 7 of tile ct ----
      float gmean[NGRP], grstd[NGRP];
      if (conv && !WSX(WSX_NO_STATS)) {
#pragma unroll
        for (int ct = 0; ct < 3; ++ct)
#pragma unroll
          for (int hf = 0; hf < 2; ++hf) {
            float v[NPT * 8];
#pragma unroll
            for (int t = 0; t < NPT; ++t)
#pragma unroll
              for (int i = 0; i < 8; ++i) v[t * 8 + i] = qv[t] ? acc[t][ct][8 * hf + i] : 0.f;
#pragma unroll
            for (int w2 = NPT * 4; w2 >= 1; w2 >>= 1)
#pragma unroll
              for (int i = 0; i < w2; ++i) v[i] += v[i + w2];
            const float s = wave_sum(v[0]);
            if (lane == 0) sRed[wave * NGRP + 2 * ct + hf] = s;
          }
      }
      CONV_BAR(8);  // S1: every conv wave's reads of x(it) done; pass-1 sums posted
      if (conv) {
#pragma unroll
        for (int g = 0; g < NGRP; ++g) {
          float tot = 0.f;
#pragma unroll
          for (int w = 0; w < WAVES; ++w) tot += sRed[w * NGRP + g];
          gmean[g] = tot * inv_cnt;
        }
        // y -> LDS over x(it): four consecutive channels per register quad, one 8-B write each
        E* sY = sReg + (it & 1) * REG;
#pragma unroll
        for (int t = 0; t < NPT; ++t) {
          const int px = (wave * NPT + t) * 32 + l32;
          if (qv[t]) {
#pragma unroll
            for (int ct = 0; ct < 3; ++ct)
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                E4 q4;
#pragma unroll
                for (int e = 0; e < 4; ++e) q4[e] = (E)acc[t][ct][4 * j + e];
                *reinterpret_cast<E4*>(&sY[px * YS + ct * 32 + 8 * j + 4 * hh]) = q4;
              }
          }
        }
#pragma unroll
        for (int ct = 0; ct < 3; ++ct)
#pragma unroll
          for (int hf = 0; hf < 2; ++hf) {
            const float mu = gmean[2 * ct + hf];
            float v[NPT * 8];
#pragma unroll
            for (int t = 0; t < NPT; ++t)
#pragma unroll
              for (int i = 0; i < 8; ++i) {
                const float d = acc[t][ct][8 * hf + i] - mu;
                v[t * 8 + i] = qv[t] ? d * d : 0.f;
              }
#pragma unroll
            for (int w2 = NPT * 4; w2 >= 1; w2 >>= 1)
#pragma unroll
              for (int i = 0; i < w2; ++i) v[i] += v[i + w2];
            const float s = wave_sum(v[0]);
            if (lane == 0) sRed[WAVES * NGRP + wave * NGRP + 2 * ct + hf] = s;
          }
      }
      CONV_BAR(9);  // S2: pass-2 sums posted
      if (conv) {
#pragma unroll
        for (int g = 0; g < NGRP; ++g) {
          float tot = 0.f;
#pragma unroll
          for (int w = 0; w < WAVES; ++w) tot += sRed[WAVES * NGRP + w * NGRP + g];
          grstd[g] = rsqrtf(tot * inv_cnt + p.eps);
        }
        if (ctid < COUT) {  // per-channel coefficients of the memory waves' epilogue
          const int g = ctid >> 4;
          float mu = 0.f, rs = 0.f;
#pragma unroll
          for (int gg = 0; gg < NGRP; ++gg)
            if (gg == g) {
              mu = gmean[gg];
              rs = grstd[gg];
            }
          float* co = sCoef + (it & 1) * 3 * COUT;
          const float a = sGB[ctid] * rs;
          co[ctid] = a;
          co[COUT + ctid] = sGB[COUT + ctid] - mu * a;
          co[2 * COUT + ctid] = dmv;
          if (p.stats && ctid < NGRP) {
            float m = 0.f, r = 0.f;
#pragma unroll
            for (int gg = 0; gg < NGRP; ++gg)
              if (gg == ctid) {
                m = gmean[gg];
                r = grstd[gg];
              }
            p.stats[((size_t)n * NGRP + ctid) * 2 + 0] = m;
            p.stats[((size_t)n * NGRP + ctid) * 2 + 1] = r;
          }
        }
      }
    }
    WS_DIAG_OUT(0);
#undef CONV_BAR
  } else {
    // =============================== memory waves ===============================
    const int mtid0 = threadIdx.x - 256;
    unsigned gbt = 0u;
    WS_DIAG_DECL;
    u32x4 xr[NXC];   // the next input tile but one, in flight
    u32x4 rq[NEC];   // the residual of the sample whose epilogue runs next
#pragma unroll
    for (int k = 0; k < NEC; ++k) rq[k] = u32x4{0u, 0u, 0u, 0u};
    for (int it = -1; it <= cnt; ++it) {
      // loop-variant thread id: the per-chunk address math stays inside the loop (hoisted, the
      // chunks' 64-bit addresses spill on boards with runtime guards)
      const int mtid = mtid0 + opaque0();
      auto xload = [&](int n) {
        const u32x4* xs = reinterpret_cast<const u32x4*>(p.x + (size_t)n * P * CIN);
  #pragma unroll
        for (int k = 0; k < NXC; ++k) {
          const int i = mtid + 256 * k;
          if ((FULL && (k + 1) * 256 <= NPT * 128 * C8) || i < P * C8) xr[k] = xs[i];
        }
      };
      auto xstore = [&](int region) {
        E* sx = sReg + region * REG;
  #pragma unroll
        for (int k = 0; k < NXC; ++k) {
          const int i = mtid + 256 * k;
          if ((FULL && (k + 1) * 256 <= NPT * 128 * C8) || i < P * C8) {
            const int px = i / C8, c8 = i - px * C8;
            *reinterpret_cast<u32x4*>(&sx[px * CINP + c8 * 8]) = xr[k];
          }
        }
        if (mtid <= C8) *reinterpret_cast<u32x4*>(&sx[P * CINP + mtid * 8]) = u32x4{0u, 0u, 0u, 0u};  // zero row
      };
      auto rload = [&](int n) {
        const u32x4* rs = reinterpret_cast<const u32x4*>(p.res + (size_t)n * P * COUT);
  #pragma unroll
        for (int k = 0; k < NEC; ++k) {
          const int c = mtid + 256 * k;
          rq[k] = u32x4{0u, 0u, 0u, 0u};
          if (FULL || c < P * (COUT / 8)) rq[k] = rs[c];
        }
      };
      // epilogue segment j of sample n (its y in region rg): the chunks k = j + 3u share one
      // channel octet cg, whose scale / shift / dropout scale are read once
      auto epi = [&](int n, int rg, int j) {
        const E* sY = sReg + rg * REG;
        const float* co = sCoef + rg * 3 * COUT;
        const int cg = (mtid % (COUT / 8) + 4 * j) % (COUT / 8);
        float ca[8], cb[8], cd[8];
  #pragma unroll
        for (int h4 = 0; h4 < 2; ++h4) {
          const f32x4 a4 = *reinterpret_cast<const f32x4*>(&co[cg * 8 + 4 * h4]);
          const f32x4 b4 = *reinterpret_cast<const f32x4*>(&co[COUT + cg * 8 + 4 * h4]);
          const f32x4 d4 = *reinterpret_cast<const f32x4*>(&co[2 * COUT + cg * 8 + 4 * h4]);
  #pragma unroll
          for (int e = 0; e < 4; ++e) {
            ca[4 * h4 + e] = a4[e];
            cb[4 * h4 + e] = b4[e];
            cd[4 * h4 + e] = d4[e];
          }
        }
  #pragma unroll
        for (int u = 0; u < EPS; ++u) {
          const int k = j + 3 * u, c = mtid + 256 * k;
          if (FULL || c < P * (COUT / 8)) {
            const int px = c / (COUT / 8);
            const size_t o = (size_t)n * P * COUT + (size_t)c * 8;
            const u32x4 yv = *reinterpret_cast<const u32x4*>(&sY[px * YS + cg * 8]);
            if (p.ysave) *reinterpret_cast<u32x4*>(&p.ysave[o]) = yv;
            const E8 y8 = __builtin_bit_cast(E8, yv);
            const E8 r8 = __builtin_bit_cast(E8, rq[k]);
            E8 o8;
            uint32_t mb = 0u;
  #pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float z = fmaxf((float)y8[e] * ca[e] + cb[e] + (float)r8[e], 0.f);
              o8[e] = (E)(z * cd[e]);
              mb |= ((float)o8[e] > 0.f ? 1u : 0u) << e;
            }
            *reinterpret_cast<u32x4*>(&p.out[o]) = __builtin_bit_cast(u32x4, o8);
            if (p.rmask) p.rmask[(size_t)n * P * (COUT / 8) + c] = (uint8_t)mb;
          }
        }
      };
      if (it < 0) {  // prologue: x(0) into region 0, both zero rows, x(1) in flight
        if (cnt > 0) {
          xload((int)blockIdx.x);
          xstore(0);
          if (mtid <= C8) *reinterpret_cast<u32x4*>(&sReg[REG + P * CINP + mtid * 8]) = u32x4{0u, 0u, 0u, 0u};
        }
        if (cnt > 1) xload((int)blockIdx.x + G);
        continue;
      }
      const int np = (int)blockIdx.x + (it - 1) * G;  // the sample whose epilogue runs now
      const bool ep = it >= 1;
      const int rg = (it + 1) & 1;                    // its y; then x(it+1) is staged there
      if (GB) {  // one s_barrier per iteration; the memory waves' own hand-off by grp_bar
        WS_BAR(10);  // A: y(it-1) and its coefficients posted, x(it) read by nobody yet
        if (WSX(WSX_NO_MEM)) {
          WS_GBAR(0, &sCnt[1], gbt += 4u);
          continue;
        }
        if (ep) {
          epi(np, rg, 0);
          epi(np, rg, 1);
          epi(np, rg, 2);
        }
        WS_GBAR(0, &sCnt[1], gbt += 4u);  // every memory wave's reads of y(it-1) done
        if (it + 1 < cnt) xstore(rg);
        if (it + 2 < cnt) xload((int)blockIdx.x + (it + 2) * G);
        if (it < cnt && p.res) rload((int)blockIdx.x + it * G);
        continue;
      }
      WS_BAR(10);  // A
      if (ep) epi(np, rg, 0);
      WS_BAR(0);  // T1
      if (ep) epi(np, rg, 1);
      WS_BAR(1);  // T2
      if (ep) epi(np, rg, 2);
      WS_BAR(2);  // T3: every memory wave's reads of y(it-1) done
      WS_BAR(3);  // T4
      if (it + 1 < cnt) xstore(rg);
      WS_BAR(4);  // T5
      if (it + 2 < cnt) xload((int)blockIdx.x + (it + 2) * G);
      if (it < cnt && p.res) rload((int)blockIdx.x + it * G);
      WS_BAR(5);  // T6
      WS_BAR(6);  // T7
      WS_BAR(7);  // T8
      WS_BAR(8);  // S1
      WS_BAR(9);  // S2
    }
    WS_DIAG_OUT(1);
  }
}

template <typename E, int CIN, int NPT, bool FULL, bool GB>
int launch_fwd_ws_t(const FwdParams<E>& p, hipStream_t s) {
  const size_t lds = ws_lds_bytes<CIN>(p.H * p.W);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_conv_gn_fwd_ws<E, CIN, NPT, FULL, GB>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  const int cap = num_cus();
  const int grid = p.N < cap ? p.N : cap;
  hipLaunchKernelGGL((k_conv_gn_fwd_ws<E, CIN, NPT, FULL, GB>), dim3(grid), dim3(512), lds, s, p);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_fwd launch: %s", hipGetErrorString(e));
    return MS_EHIP;
  }
  return MS_OK;
}

template <typename E, int CIN, int NPT, bool FULL>
int launch_fwd_ws(const FwdParams<E>& p, hipStream_t s) {
  return g_variant[MCV_FWD] == 3 ? launch_fwd_ws_t<E, CIN, NPT, FULL, true>(p, s)
                                 : launch_fwd_ws_t<E, CIN, NPT, FULL, false>(p, s);
}

// ---------------------------------------------------------------------------------------
// Wave-specialised forward with channel-split conv waves (variant 4; boards of P <= 256 pixels):
// ONE 448-thread workgroup per CU, 3 conv waves + 4 memory waves.
//   Conv wave c owns output channels 32c .. 32c+31 for ALL pixels of the sample: NT <= 8 pixel
//   tiles of one v_mfma_f32_32x32x16 channel tile (transposed, D[co][px]: a lane holds one pixel,
//   A = the wave's 32 weight rows of the tap, read once per k step for all NT tiles; B = the
//   input tile). Its weight rows stream into its OWN three-slot LDS ring by LDS-DMA
//   (global_load_lds_dwordx4, two taps ahead, counted vmcnt), so the nine taps need no barrier;
//   its two GroupNorm groups lie wholly inside it, so the statistics are wave reductions. One
//   conv-only grp_bar per sample: every conv wave's reads of x(it) are done before y(it)
//   overwrites them. (Round 4's first WS form split pixels across 4 conv waves that shared one
//   weight ring: 11 syncs per sample, each exposing the slowest wave; conv alone ran at 45 % of
//   its MFMA time.)
//   Memory waves: the epilogue of sample it-1, x(it+1) staging and the loads, as k_conv_gn_fwd_ws;
//   they also load the dropout scales and store the statistics, so the conv waves issue no
//   vector-memory instruction but their LDS-DMA (exact vmcnt counts).
// LDS: two sample regions (x as [P+1][XS] with row P zero; CIN = 96: unpadded rows, 16-B chunks
// XOR-swizzled by (row >> 2) & 3 -- conflict-free B reads and y writes, and room for the rings;
// then y as [P][96], same swizzle), 3 x 3 weight slots [32][CINP], f32 bias / gamma / beta,
// 2 parities of scale / shift and statistics.
template <int CIN>
struct W3 {
  static constexpr int XS = CIN == 96 ? 96 : 24;  // x row stride (elements)
  static constexpr bool SWZ = CIN == 96;
  static constexpr int CINP = CIN;                // weight slot row (elements; CIN = 96: swizzled like x)
  static constexpr int SLOT = 32 * CINP;          // weight slot (elements)
  static constexpr int SCH = SLOT / 8;            // 16-B chunks per slot
  static constexpr int NGL = SCH / 64;            // LDS-DMA instructions per slot (whole waves)
  static_assert(SCH % 64 == 0, "every LDS-DMA instruction of a slot runs on all 64 lanes");
  static constexpr int FLOATS = 3 * COUT + 2 * 2 * COUT + 2 * 2 * NGRP + 2 * COUT + 4;
};
template <int CIN>
__host__ __device__ inline int w3_region_elems(int P) {
  const int a = (P + 1) * W3<CIN>::XS, b = P * COUT;
  return ((a > b ? a : b) + 7) & ~7;
}
template <int CIN>
__host__ __device__ inline size_t w3_lds_bytes(int P) {
  return (size_t)2 * w3_region_elems<CIN>(P) * 2 + (size_t)9 * W3<CIN>::SLOT * 2 + (size_t)W3<CIN>::FLOATS * 4;
}
// element offset of 16-B chunk c of row r in a swizzled [rows][12-chunk] image
template <bool SWZ>
__device__ __forceinline__ int w3_chunk(int r, int c) {
  return SWZ ? (c ^ ((r >> 2) & 3)) : c;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <typename E, int CIN, int NT, bool FULL, bool DB>
__global__ __launch_bounds__(448, 1) void k_conv_gn_fwd_ws3(FwdParams<E> p) {
  typedef typename EV<E>::v8 E8;
  typedef typename EV<E>::v4 E4;
  typedef W3<CIN> L3;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int XS = L3::XS, CINP = L3::CINP, C8 = CIN / 8, KS = CIN / 16;
  constexpr int NXC = (NT * 32 * C8 + 255) / 256;  // 16-B input chunks per memory thread
  constexpr int NEC = (NT * 32 * 12 + 255) / 256;  // 16-B output chunks per memory thread
  const int H = p.H, W = p.W, P = H * W;
  const int REG = w3_region_elems<CIN>(P);
  E* sReg = reinterpret_cast<E*>(smem);                 // [2][REG]
  E* sRing = sReg + 2 * REG;                            // [3 waves][3 slots][32][CINP]
  float* sBias = reinterpret_cast<float*>(sRing + 9 * L3::SLOT);
  float* sGB = sBias + COUT;                            // gamma | beta
  float* sCoef = sGB + 2 * COUT;                        // [2 parities][scale | shift][COUT]
  float* sStat = sCoef + 4 * COUT;                      // [2 parities][NGRP][mean, rstd]
  float* sDm = sStat + 4 * NGRP;                        // [2 parities][COUT] dropout scales
  unsigned* sCnt = reinterpret_cast<unsigned*>(sDm + 2 * COUT);  // conv | memory grp_bar
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const int G = gridDim.x;
  const int cnt = p.N > (int)blockIdx.x ? (p.N - 1 - (int)blockIdx.x) / G + 1 : 0;

  if (wave < 3) {
    // =============================== conv wave `wave` ===============================
    const int c = wave;  // channel tile
    const int l32 = lane & 31, hh = lane >> 5;
    E* myRing = sRing + c * 3 * L3::SLOT;
    // LDS-DMA of tap `tap` (this wave's 32 rows) into slot `slot`: NGL wave-instructions of 1 KiB,
    // lane-linear destinations, every lane active (a partial last instruction under a divergent
    // branch was tail-merged by hipcc into one DMA with a readfirstlane'd, wrong M0); the swizzle
    // is applied on the per-lane SOURCE chunk: LDS position pc of row r holds chunk pc ^ s(r)
    auto dma = [&](int tap, int slot) {
      const E* wsrc = p.wt + ((size_t)tap * COUT + 32 * c) * CIN;
      const int ln = lane + opaque0();  // (the per-lane source offsets stay in the loop: no spill)
#pragma unroll
      for (int k = 0; k < L3::NGL; ++k) {
        const int q = k * 64 + ln;
        const int r = q / C8, pc = q - r * C8;
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(wsrc + r * CIN + w3_chunk<L3::SWZ>(r, pc) * 8),
            (__attribute__((address_space(3))) void*)(myRing + slot * L3::SLOT + k * 512), 16, 0, 0);
      }
    };
    // each tile's pixel as (row << 16) | (col & 0xffff), one register a tile; a pixel past P is
    // (-1000, -1000) and reads the zero row at every tap
    int qrc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int q = t * 32 + l32;
      const bool v = FULL || q < P;
      const int r = v ? q / W : -1000;
      qrc[t] = (r << 16) | ((v ? q - r * W : -1000) & 0xffff);
    }
    auto qv = [&](int t) { return FULL || t * 32 + l32 < P; };
    const float inv_cnt = 1.0f / (16.0f * (float)P);
    unsigned gbt = 0u;
    dma(0, 0);
    dma(1, 1);
    for (int it = 0; it <= cnt; ++it) {
      const bool conv = it < cnt;
      const E* sX = sReg + (it & 1) * REG;
      lds_barrier();  // A: x(it) staged; y(it-1) and its coefficients posted
      if (!conv) continue;
      f32x16 acc[NT];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(&sBias[32 * c + 8 * j + 4 * hh]);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[t][4 * j + e] = b4[e];
      }
      for (int tap = 0; tap < 9; ++tap) {
        const int g = it * 9 + tap;
        wait_vmcnt<L3::NGL>();   // tap g's DMA (issued two taps ago) has landed; g+1's may fly
        dma((tap + 2) % 9, (g + 2) % 3);  // into the slot tap g-1 used (its reads are done)
        const E* sW = myRing + (g % 3) * L3::SLOT;
        const int dr = tap / 3 - 1, dc = tap % 3 - 1;
        int xrow[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int sr = (qrc[t] >> 16) + dr, sc = ((qrc[t] << 16) >> 16) + dc;
          const bool v = (unsigned)sr < (unsigned)H && (unsigned)sc < (unsigned)W;
          xrow[t] = v ? sr * W + sc : P;
        }
        auto lda = [&](int ks) {
          return *reinterpret_cast<const E8*>(&sW[l32 * CINP + w3_chunk<L3::SWZ>(l32, 2 * ks + hh) * 8]);
        };
        auto ldb = [&](int ks, int t) {
          return *reinterpret_cast<const E8*>(&sX[xrow[t] * XS + w3_chunk<L3::SWZ>(xrow[t], 2 * ks + hh) * 8]);
        };
        if constexpr (DB) {
          // B double-buffered: all of step ks+1's operands are read ahead of step ks's NT MFMAs
          // (one counted lgkmcnt per step instead of one per MFMA)
          E8 A[2], B[2][NT];
          A[0] = lda(0);
#pragma unroll
          for (int t = 0; t < NT; ++t) B[0][t] = ldb(0, t);
          __builtin_amdgcn_sched_group_barrier(0x100, NT + 1, 0);  // (its own group: step 0's reads)
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            if (ks + 1 < KS) {
              A[(ks + 1) & 1] = lda(ks + 1);
#pragma unroll
              for (int t = 0; t < NT; ++t) B[(ks + 1) & 1][t] = ldb(ks + 1, t);
              __builtin_amdgcn_sched_group_barrier(0x100, NT + 1, 0);
            }
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = mfma32(A[ks & 1], B[ks & 1][t], acc[t]);
            __builtin_amdgcn_sched_group_barrier(0x008, NT, 0);
          }
        } else {
          // B single-buffered and rotating: tile t's operand of k step ks+1 is read right after
          // tile t's MFMA of step ks has taken it, NT-1 MFMAs ahead of its use (32 VGPRs, not 64)
          E8 A[2], B[NT];
          A[0] = lda(0);
#pragma unroll
          for (int t = 0; t < NT; ++t) B[t] = ldb(0, t);
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            if (ks + 1 < KS) A[(ks + 1) & 1] = lda(ks + 1);
#pragma unroll
            for (int t = 0; t < NT; ++t) {
              acc[t] = mfma32(A[ks & 1], B[t], acc[t]);
              if (ks + 1 < KS) B[t] = ldb(ks + 1, t);
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              if (ks + 1 < KS) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
          }
        }
      }
      grp_bar(&sCnt[0], gbt += 3u, lane);  // every conv wave's reads of x(it) done
      // ---- GroupNorm statistics of groups 2c, 2c+1 (registers 8 hf .. 8 hf + 7): in-wave ----
      // (eight running sums over the tiles, then a tree: no copy of the accumulators)
      float mu[2], rs[2];
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          v[i] = 0.f;
#pragma unroll
          for (int t = 0; t < NT; ++t) v[i] += qv(t) ? acc[t][8 * hf + i] : 0.f;
        }
        mu[hf] = wave_sum(((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]))) * inv_cnt;
      }
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          v[i] = 0.f;
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const float d = acc[t][8 * hf + i] - mu[hf];
            v[i] += qv(t) ? d * d : 0.f;
          }
        }
        rs[hf] = rsqrtf(wave_sum(((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]))) * inv_cnt + p.eps);
      }
      // ---- y -> LDS over x(it): four consecutive channels per register quad, one 8-B write ----
      E* sY = sReg + (it & 1) * REG;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int px = t * 32 + l32;
        if (qv(t)) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            E4 q4;
#pragma unroll
            for (int e = 0; e < 4; ++e) q4[e] = (E)acc[t][4 * j + e];
            *reinterpret_cast<E4*>(&sY[px * COUT + w3_chunk<true>(px, 4 * c + j) * 8 + 4 * hh]) = q4;
          }
        }
      }
      if (lane < 32) {  // this wave's 32 channels: scale and shift; its 2 groups' statistics
        const int ch = 32 * c + lane, hf = lane >> 4;
        const float m = hf ? mu[1] : mu[0], r = hf ? rs[1] : rs[0];
        float* co = sCoef + (it & 1) * 2 * COUT;
        const float a = sGB[ch] * r;
        co[ch] = a;
        co[COUT + ch] = sGB[COUT + ch] - m * a;
        if ((lane & 15) == 0) {
          sStat[(it & 1) * 2 * NGRP + (2 * c + hf) * 2 + 0] = m;
          sStat[(it & 1) * 2 * NGRP + (2 * c + hf) * 2 + 1] = r;
        }
      }
    }
    wait_vmcnt<0>();  // no LDS-DMA may outlive the workgroup's LDS
  } else {
    // =============================== memory waves ===============================
    const int mtid0 = threadIdx.x - 192;
    for (int i = mtid0; i < COUT; i += 256) {
      sBias[i] = p.bias[i];
      sGB[i] = p.gamma[i];
      sGB[COUT + i] = p.beta[i];
    }
    if (mtid0 < 2) sCnt[mtid0] = 0u;
    unsigned gbt = 0u;
    u32x4 xr[NXC];   // the next input tile but one, in flight
    u32x4 rq[NEC];   // the residual of the sample whose epilogue runs next
    float dmv = 1.f; // its dropout scale of channel mtid (< 96), posted to sDm before the barrier
#pragma unroll
    for (int k = 0; k < NEC; ++k) rq[k] = u32x4{0u, 0u, 0u, 0u};
    for (int it = -1; it <= cnt; ++it) {
      const int mtid = mtid0 + opaque0();  // (loop-variant: the address math stays in the loop)
      auto xload = [&](int n) {
        const u32x4* xs = reinterpret_cast<const u32x4*>(p.x + (size_t)n * P * CIN);
#pragma unroll
        for (int k = 0; k < NXC; ++k) {
          const int i = mtid + 256 * k;
          if ((FULL && (k + 1) * 256 <= NT * 32 * C8) || i < P * C8) xr[k] = xs[i];
        }
      };
      auto xstore = [&](int region) {
        E* sx = sReg + region * REG;
#pragma unroll
        for (int k = 0; k < NXC; ++k) {
          const int i = mtid + 256 * k;
          if ((FULL && (k + 1) * 256 <= NT * 32 * C8) || i < P * C8) {
            const int px = i / C8, c8 = i - px * C8;
            *reinterpret_cast<u32x4*>(&sx[px * XS + w3_chunk<L3::SWZ>(px, c8) * 8]) = xr[k];
          }
        }
        if (mtid < XS / 8) *reinterpret_cast<u32x4*>(&sx[P * XS + mtid * 8]) = u32x4{0u, 0u, 0u, 0u};
      };
      auto rload = [&](int n) {
        if (p.res) {
          const u32x4* rs = reinterpret_cast<const u32x4*>(p.res + (size_t)n * P * COUT);
#pragma unroll
          for (int k = 0; k < NEC; ++k) {
            const int cc = mtid + 256 * k;
            rq[k] = u32x4{0u, 0u, 0u, 0u};
            if (FULL || cc < P * (COUT / 8)) rq[k] = rs[cc];
          }
        }
        dmv = (p.dmask && mtid < COUT) ? p.dmask[(size_t)n * COUT + mtid] : 1.f;
      };
      if (it < 0) {  // prologue: x(0) into region 0, both zero rows, x(1) in flight
        if (cnt > 0) {
          xload((int)blockIdx.x);
          xstore(0);
          if (mtid < XS / 8) *reinterpret_cast<u32x4*>(&sReg[REG + P * XS + mtid * 8]) = u32x4{0u, 0u, 0u, 0u};
        }
        if (cnt > 1) xload((int)blockIdx.x + G);
        continue;
      }
      const int np = (int)blockIdx.x + (it - 1) * G;  // the sample whose epilogue runs now
      const int rg = (it + 1) & 1;                    // its y (and coefficients); then x(it+1) goes there
      if (it >= 1 && mtid < COUT) sDm[rg * COUT + mtid] = dmv;  // (loaded at the end of iteration it-1)
      lds_barrier();  // A
      if (it >= 1) {
        const E* sY = sReg + rg * REG;
        const float* co = sCoef + rg * 2 * COUT;
        const float* dmp = sDm + rg * COUT;
        if (p.stats && mtid < 2 * NGRP) p.stats[(size_t)np * 2 * NGRP + mtid] = sStat[rg * 2 * NGRP + mtid];
#pragma unroll
        for (int j = 0; j < 3; ++j) {  // the chunks k = j + 3u share one channel octet cg
          const int cg = (mtid % 12 + 4 * j) % 12;
          float ca[8], cb[8], cd[8];
#pragma unroll
          for (int h4 = 0; h4 < 2; ++h4) {
            const f32x4 a4 = *reinterpret_cast<const f32x4*>(&co[cg * 8 + 4 * h4]);
            const f32x4 b4 = *reinterpret_cast<const f32x4*>(&co[COUT + cg * 8 + 4 * h4]);
            const f32x4 d4 = *reinterpret_cast<const f32x4*>(&dmp[cg * 8 + 4 * h4]);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              ca[4 * h4 + e] = a4[e];
              cb[4 * h4 + e] = b4[e];
              cd[4 * h4 + e] = d4[e];
            }
          }
#pragma unroll
          for (int u = 0; u * 3 + j < NEC; ++u) {
            const int k = j + 3 * u, cc = mtid + 256 * k;
            if (FULL || cc < P * (COUT / 8)) {
              const int px = cc / 12;
              const size_t o = (size_t)np * P * COUT + (size_t)cc * 8;
              const u32x4 yv = *reinterpret_cast<const u32x4*>(&sY[px * COUT + w3_chunk<true>(px, cg) * 8]);
              if (p.ysave) *reinterpret_cast<u32x4*>(&p.ysave[o]) = yv;
              const E8 y8 = __builtin_bit_cast(E8, yv);
              const E8 r8 = __builtin_bit_cast(E8, rq[k]);
              E8 o8;
              uint32_t mb = 0u;
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const float z = fmaxf((float)y8[e] * ca[e] + cb[e] + (float)r8[e], 0.f);
                o8[e] = (E)(z * cd[e]);
                mb |= ((float)o8[e] > 0.f ? 1u : 0u) << e;
              }
              *reinterpret_cast<u32x4*>(&p.out[o]) = __builtin_bit_cast(u32x4, o8);
              if (p.rmask) p.rmask[(size_t)np * P * (COUT / 8) + cc] = (uint8_t)mb;
            }
          }
        }
      }
      grp_bar(&sCnt[1], gbt += 4u, lane);  // every memory wave's reads of y(it-1) done
      asm volatile("" ::: "memory");
      if (it + 1 < cnt) xstore(rg);
      if (it + 2 < cnt) xload((int)blockIdx.x + (it + 2) * G);
      if (it < cnt) rload((int)blockIdx.x + it * G);
    }
  }
}

template <typename E, int CIN, int NT, bool FULL, bool DB>
int launch_fwd_ws3(const FwdParams<E>& p, hipStream_t s) {
  const size_t lds = w3_lds_bytes<CIN>(p.H * p.W);
  if (lds > 160 * 1024) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_fwd: board %dx%d needs %zu B LDS", p.H, p.W, lds);
    return MS_EINVAL;
  }
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_conv_gn_fwd_ws3<E, CIN, NT, FULL, DB>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  const int cap = num_cus();
  const int grid = p.N < cap ? p.N : cap;
  hipLaunchKernelGGL((k_conv_gn_fwd_ws3<E, CIN, NT, FULL, DB>), dim3(grid), dim3(448), lds, s, p);
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
  if (P <= 256 && g_variant[MCV_FWD] == 4) {
    if (P == 256) return launch_fwd_ws3<E, CIN, 8, true, false>(p, s);
    if (P > 128) return launch_fwd_ws3<E, CIN, 8, false, false>(p, s);
    return launch_fwd_ws3<E, CIN, 4, false, false>(p, s);
  }
  if (P <= 256 && g_variant[MCV_FWD] == 5) {
    if (P == 256) return launch_fwd_ws3<E, CIN, 8, true, true>(p, s);
    if (P > 128) return launch_fwd_ws3<E, CIN, 8, false, true>(p, s);
    return launch_fwd_ws3<E, CIN, 4, false, true>(p, s);
  }
  if (P <= 256 && g_variant[MCV_FWD] >= 2) {  // measured slower than the per-sample kernel so far
    if (P == 256) return launch_fwd_ws<E, CIN, 2, true>(p, s);
    if (P > 128) return launch_fwd_ws<E, CIN, 2, false>(p, s);
    return launch_fwd_ws<E, CIN, 1, false>(p, s);
  }
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
#if defined(MC_DIAG) || defined(MC_WSX)
int g_fwd_exp = 0;
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
  p.exp = 0;
#ifdef MC_DIAG
  p.diag = g_fwd_diag;
#endif
#if defined(MC_DIAG) || defined(MC_WSX)
  p.exp = g_fwd_exp;
#endif
  return cin == 16 ? dispatch_fwd<E, 16>(p, s) : dispatch_fwd<E, 96>(p, s);
}

}  // namespace

extern "C" {

const char* mc_last_error(void) { return g_err; }

int mc_set_variant(int32_t kernel, int32_t variant) {
  if (kernel < 0 || kernel >= MCV_COUNT || variant < 0 || variant > 5) {
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
#if defined(MC_DIAG) || defined(MC_WSX)
// timing experiments only (tools/fwd_ws_exp.py): WSX_* bits of the next wave-specialised forwards
void mc_set_fwd_exp(int32_t e) { g_fwd_exp = e; }
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
