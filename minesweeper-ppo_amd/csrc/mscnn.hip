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

struct FwdParams {
  const __bf16* x;
  const __bf16* wt;
  const float* bias;
  const float* gamma;
  const float* beta;
  const __bf16* res;
  const float* dmask;
  __bf16* out;
  __bf16* ysave;
  float* stats;
  uint8_t* rmask;  // optional ReLU bitmask [N][P][12]: bit j of byte (px, c8) = out[px][8*c8 + j] > 0
  int N, H, W;
  float eps;
  int stagger;               // start delay of the upper half of the grid, 10-ns ticks (0 = none)
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

// s_waitcnt vmcnt(n) for a wave-uniform n (the immediate must be a constant)
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
#define MC_VMW(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    MC_VMW(0) MC_VMW(1) MC_VMW(2) MC_VMW(3) MC_VMW(4) MC_VMW(5) MC_VMW(6) MC_VMW(7) MC_VMW(8) MC_VMW(9)
    MC_VMW(10) MC_VMW(11) MC_VMW(12) MC_VMW(13) MC_VMW(14) MC_VMW(15) MC_VMW(16) MC_VMW(17) MC_VMW(18)
    MC_VMW(19) MC_VMW(20) MC_VMW(21) MC_VMW(22) MC_VMW(23) MC_VMW(24) MC_VMW(25) MC_VMW(26) MC_VMW(27)
    MC_VMW(28) MC_VMW(29) MC_VMW(30) MC_VMW(31) MC_VMW(32) MC_VMW(33) MC_VMW(34) MC_VMW(35) MC_VMW(36)
#undef MC_VMW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// One weight tap [96][96] global -> LDS by LDS-DMA (global_load_lds_dwordx4: each
// wave-instruction writes 1 KiB lane-linearly). The LDS image is unpadded with 16-B
// chunk ch of row co stored at ch ^ ((co >> 2) & 3) (conflict-free B reads); the
// swizzle is applied on the SOURCE address. 18 wave-instructions per tap, split
// over the 4 waves (5/5/4/4).
#define MC_GLDS_W(T_, dst_)                                                                      \
  do {                                                                                           \
    for (int j_ = wave; j_ < 18; j_ += 4) {                                                      \
      const int o_ = 1024 * j_ + 16 * lane;                                                      \
      const int co_ = o_ / 192, ch_ = ((o_ % 192) >> 4) ^ ((co_ >> 2) & 3);                    \
      glds16(p.wt + ((size_t)(T_) * COUT + co_) * COUT + ch_ * 8,                               \
             reinterpret_cast<unsigned char*>(dst_) + 1024 * j_);                                \
    }                                                                                            \
  } while (0)

// global_load_lds_dwordx4 through inline asm: hipcc does not track it, so it inserts no
// vmcnt(0) before the next LDS read (the builtin makes it drain the DMA there); the
// kernel retires it with counted waits (wait_vmcnt). M0 is saved and restored in the
// statement (cdna_hip_programming.md, LDS-DMA recipe).
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_dst) {
  const unsigned dst = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds_dst;
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(dst))
               : "memory");
}

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
#define MC_STORE_W(buf_, v_)                                                            \
  do {                                                                                  \
    __bf16* d_ = sW + (buf_) * COUT * CINP;                                             \
    _Pragma("unroll") for (int k_ = 0; k_ < NWC; ++k_) {                                \
      const int i_ = tid + 256 * k_;                                                    \
      if (k_ < COUT * C8 / 256 || i_ < COUT * C8) {                                    \
        const int co_ = i_ / C8, c8_ = i_ - co_ * C8;                                   \
        *reinterpret_cast<u32x4*>(&d_[co_ * CINP + c8_ * 8]) = v_[k_];                  \
      }                                                                                 \
    }                                                                                   \
  } while (0)

// PF = true: one workgroup per CU with the registers to prefetch the next sample's
// input and this sample's residual, double-buffered weight taps (one barrier per
// tap). PF = false: two workgroups per CU, nothing held across phases.
template <int CIN, int NPT, bool FULL, bool PF>
__global__ __launch_bounds__(256, PF ? 1 : (NPT <= 2 ? 2 : 1)) void k_conv_gn_fwd(FwdParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int CINP = cinp<CIN>();
  constexpr int C8 = CIN / 8;
  constexpr int NPF = (NPT * 128 * C8 + 255) / 256;  // 16-B input chunks per thread
  constexpr int NWC = (COUT * C8 + 255) / 256;        // 16-B weight chunks per thread and tap
  const int H = p.H, W = p.W, P = H * W;
  __bf16* sX = reinterpret_cast<__bf16*>(smem);
  __bf16* sO = sX;
  __bf16* sW = sX + region0_elems<CIN>(H, W);
  // GL: the PF path's weight taps arrive by LDS-DMA into a ring of 3 unpadded buffers,
  // two taps ahead of the MFMAs (raw barriers + counted vmcnt keep them in flight)
#ifdef MC_FWD_GL
  constexpr bool GL = PF && CIN == 96;
#else
  constexpr bool GL = false;  // measured slower (2.87 vs 2.50 ms): per-CU LDS-DMA rate, see DESIGN.md §5
#endif
  float* sRed = reinterpret_cast<float*>(sW + (GL ? 3 * COUT * COUT : (PF ? 2 : 1) * COUT * CINP));
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
  u32x4 rv[PF ? NEC : 1];
  if (PF && (int)blockIdx.x < p.N) MC_LOAD_IN(blockIdx.x, xin);
  int gi = 0;  // GL: running tap count -> ring slot gi % 3
  const int nglds = (18 - wave + 3) / 4;  // this wave's LDS-DMA instructions per tap
  if (GL && (int)blockIdx.x < p.N) {
    MC_GLDS_W(0, sW);
    MC_GLDS_W(1, sW + COUT * COUT);
  }
  if (p.stagger != 0) {
    // the two workgroups that share a CU run the same phase sequence; delaying one by
    // about half a sample period lets its MFMA phase overlap the other's HBM epilogue
    // (stagger > 0: the upper half of the grid waits; < 0: the odd blocks)
    const bool late = p.stagger > 0 ? (int)blockIdx.x >= (int)gridDim.x / 2 : (blockIdx.x & 1) != 0;
    const unsigned long long ticks = (unsigned long long)(p.stagger > 0 ? p.stagger : -p.stagger);
    if (late) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    }
  }
#ifdef MC_DIAG
  unsigned long long dacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif
  for (int n = blockIdx.x; n < p.N; n += gridDim.x) {
    // loop-variant copy of tid: keeps the per-chunk address math inside the loop instead of
    // hoisting a dozen 64-bit addresses out of it (they would be spilled)
    const int tid = threadIdx.x + opaque0();
    // ---- stage the input tile (the zero row is re-written: the epilogue reuses region0) ----
#ifndef MC_EXP_NO_IN
    if (!PF) MC_LOAD_IN(n, xin);  // PF: prefetched during the previous sample's last tap
#else
    for (int k = 0; k < NPF; ++k) xin[k] = u32x4{1u, 2u, 3u, (unsigned)n};
#endif
    for (int i = tid; i < C8; i += 256) *reinterpret_cast<u32x4*>(&sX[P * CINP + i * 8]) = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < NPF; ++k) {
      const int i = tid + 256 * k;
      if ((FULL && k < C8) || i < P * C8) {  // FULL: P = 256, every chunk in range
        const int px = i / C8, c8 = i - px * C8;
        *reinterpret_cast<u32x4*>(&sX[px * CINP + c8 * 8]) = xin[k];
      }
    }
    if (!GL) {
      MC_LOAD_W(0, wr);
      MC_STORE_W(0, wr);
    }
    const int nn = n + gridDim.x;
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
#ifndef MC_EXP_NO_WLOAD
      if (!GL && tap + 1 < 9) MC_LOAD_W(tap + 1, wr);
#endif
      if (GL) MC_GLDS_W((tap + 2) % 9, sW + ((gi + 2) % 3) * COUT * COUT);  // next sample's taps 0/1 at 7/8
      if (PF && tap == 8) {
        // vmcnt retires in issue order: these are issued after the last weight wait,
        // in the order they are consumed (residual in this epilogue, input next sample)
#pragma unroll
        for (int k = 0; k < (PF ? NEC : 0); ++k) {
          const int c = tid + 256 * k;
          rv[k] = u32x4{0u, 0u, 0u, 0u};
          if (p.res && c < P * (COUT / 8)) rv[k] = *reinterpret_cast<const u32x4*>(&p.res[(size_t)n * P * COUT + c * 8]);
        }
        if (nn < p.N) MC_LOAD_IN(nn, xin);
      }
      const __bf16* sWt = GL ? sW + (gi % 3) * COUT * COUT : sW + (PF ? (tap & 1) : 0) * COUT * CINP;
      const int dr = tap / 3 - 1, dc = tap % 3 - 1;
      int aoff[NPT];
#pragma unroll
      for (int t = 0; t < NPT; ++t) {
        const int sr = qr[t] + dr, sc = qc[t] + dc;
        const bool v = (unsigned)sr < (unsigned)H && (unsigned)sc < (unsigned)W;
        aoff[t] = (v ? sr * W + sc : P) * CINP + 8 * hh;
      }
#ifdef MC_EXP_NO_MFMA
      if (p.N < 0)
#endif
      if constexpr (PF) {
        // all of this tap's LDS operand reads first (in k-step order), then the MFMAs:
        // with one wave per SIMD nothing else hides a read -> use latency
        constexpr int KS = CIN / 16;
        bf16x8 bq[KS][3], aq[KS][NPT];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
          for (int ct = 0; ct < 3; ++ct)
            bq[ks][ct] = GL ? *reinterpret_cast<const bf16x8*>(
                                  &sWt[(ct * 32 + l32) * COUT + 8 * ((2 * ks + hh) ^ (((ct * 32 + l32) >> 2) & 3))])
                            : *reinterpret_cast<const bf16x8*>(&sWt[(ct * 32 + l32) * CINP + ks * 16 + 8 * hh]);
#pragma unroll
          for (int t = 0; t < NPT; ++t) aq[ks][t] = *reinterpret_cast<const bf16x8*>(&sX[aoff[t] + ks * 16]);
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
          for (int t = 0; t < NPT; ++t)
#pragma unroll
            for (int ct = 0; ct < 3; ++ct)
              acc[t][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq[ks][t], bq[ks][ct], acc[t][ct], 0, 0, 0);
      } else {
        // k steps with double-buffered operands, order pinned: step k+1's LDS reads are
        // issued before step k's MFMAs (left alone, the scheduler reuses one operand set
        // and waits on every read)
        constexpr int KS = CIN / 16;
        bf16x8 A[2][NPT], B[2][3];
        auto ld = [&](int ks, bf16x8 (&a)[NPT], bf16x8 (&b)[3]) {
#pragma unroll
          for (int ct = 0; ct < 3; ++ct)
            b[ct] = *reinterpret_cast<const bf16x8*>(&sWt[(ct * 32 + l32) * CINP + ks * 16 + 8 * hh]);
#pragma unroll
          for (int t = 0; t < NPT; ++t) a[t] = *reinterpret_cast<const bf16x8*>(&sX[aoff[t] + ks * 16]);
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
              acc[t][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[ks & 1][t], B[ks & 1][ct], acc[t][ct], 0, 0, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 3 * NPT, 0);
        }
      }
      if (GL) {
        // retire this wave's DMA of tap g+1 (issued a tap ago); the one of g+2 and, on
        // the last tap, the residual / next-input loads stay in flight
        // (exact only when every chunk guard holds; otherwise count 0 = wait for more)
        const int extra = (tap == 8 && FULL) ? ((p.res ? NEC : 0) + (nn < p.N ? NPF : 0)) : 0;
        wait_vmcnt(nglds + extra);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        ++gi;
      } else if (PF) {
#ifndef MC_EXP_NO_WLOAD
        if (tap + 1 < 9) MC_STORE_W((tap + 1) & 1, wr);  // that buffer was last read in tap-1
#endif
        __syncthreads();
      } else {
        __syncthreads();  // sW (and after the last tap sX) fully read
#ifndef MC_EXP_NO_WLOAD
        if (tap + 1 < 9) {
          MC_STORE_W(0, wr);
          __syncthreads();
        }
#endif
      }
    }

    FSTAMP(1);  // 9 taps
    // ---------------- epilogue A: bias, GroupNorm statistics, y -> LDS ----------------
    float biasv[3];
#pragma unroll
    for (int ct = 0; ct < 3; ++ct) biasv[ct] = p.bias[ct * 32 + l32];
    float gmean[NGRP], grstd[NGRP];
    const float inv_cnt = 1.0f / (16.0f * (float)P);
#ifdef MC_EXP_NO_STATS
    for (int pass = 0; pass < 0; ++pass) {
#else
    for (int pass = 0; pass < 2; ++pass) {
#endif
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
          if (FULL || px < P) sO[px * COUT + ct * 32 + l32] = (__bf16)(acc[t][ct][i] + biasv[ct]);
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
#ifdef MC_EXP_NO_EPI
    if (p.N < 0)
#endif
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
      if (!PF && k % RB == 0) {
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
        const bf16x8 y8 = __builtin_bit_cast(bf16x8, yv);
        const bf16x8 r8 = __builtin_bit_cast(bf16x8, PF ? rv[PF ? k : 0] : rq[k % RB]);
        bf16x8 o8;
        uint32_t mb = 0u;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float z = fmaxf((float)y8[j] * ca[k % 3][j] + cb[k % 3][j] + (float)r8[j], 0.f);
          o8[j] = (__bf16)(z * cd[k % 3][j]);
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
  if (GL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the workgroup
#ifdef MC_DIAG
  if (p.diag && threadIdx.x == 0)
    for (int k = 0; k < 8; ++k) p.diag[blockIdx.x * 8 + k] = dacc[k];
#endif
}

template <int CIN, int NPT, bool FULL, bool PF>
int launch_fwd(const FwdParams& p, hipStream_t s) {
  constexpr int CINP = cinp<CIN>();
#ifdef MC_FWD_GL
  constexpr bool GL = PF && CIN == 96;
#else
  constexpr bool GL = false;
#endif
  const size_t lds = (size_t)region0_elems<CIN>(p.H, p.W) * 2 +
                     (size_t)(GL ? 3 * COUT * COUT : (PF ? 2 : 1) * COUT * CINP) * 2 + WAVES * NGRP * 4 + 5 * COUT * 4;
  if (lds > 160 * 1024) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_fwd: board %dx%d needs %zu B LDS", p.H, p.W, lds);
    return MS_EINVAL;
  }
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_conv_gn_fwd<CIN, NPT, FULL, PF>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr_set = true;
  }
  const int per_cu = (!PF && lds <= 80 * 1024) ? 2 : 1;
  const int cap = per_cu * num_cus();
  const int grid = p.N < cap ? p.N : cap;
  hipLaunchKernelGGL((k_conv_gn_fwd<CIN, NPT, FULL, PF>), dim3(grid), dim3(256), lds, s, p);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_fwd launch: %s", hipGetErrorString(e));
    return MS_EHIP;
  }
  return MS_OK;
}

// ------------------------------------------------------------------------------------
// Resident-weight forward for 96 -> 96 layers on boards of <= 256 cells.
//
// The per-sample kernel above re-stages every tap's weights (9 x 18 KiB) through LDS
// for every sample, behind two barriers per tap. Here the output channels are split
// in two halves of 48 (three whole GroupNorm groups): a workgroup owns one half, so
// its 9 x 48 x 96 weights (84 KiB) stay in LDS for the whole launch and a sample's
// 864-deep contraction runs with no barrier at all. The two halves of one sample are
// launched on one XCD (blocks b and b + 8), so the second read of the input tile is an
// L2 hit. One workgroup per CU, one wave per SIMD: each wave owns MT 16-pixel tiles x
// 48 channels on v_mfma_f32_16x16x32_bf16 (A = pixels x 32 ci from the tap-shifted
// input tile, B = 32 ci x 16 co from the resident weights), and the next sample's input
// and this sample's residual are loaded into registers while the MFMAs run.
// LDS: sW [9][48][104] | sX [P+1][104] (row P = zeros; after the MFMAs the same bytes
// hold y as sO [P][48] for the coalesced epilogue) | sRed [2][4][3] | sGB [3][48]
// (gamma, beta, this sample's dropout scale).
constexpr int RW_CH = 48;   // output channels per workgroup
constexpr int RW_CIP = 104; // padded ci row (elements): conflict-light ds_read_b128

__host__ __device__ inline size_t rw_lds_bytes(int P) {
  return (size_t)9 * RW_CH * RW_CIP * 2 + (size_t)(P + 1) * RW_CIP * 2 + 24 * 4 + 3 * RW_CH * 4;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MT, bool FULL>
__global__ __launch_bounds__(256, 1) void k_conv_gn_fwd_rw(FwdParams p) {
  constexpr int CI = 96, CIP = RW_CIP, CH = RW_CH;
  constexpr int NXC = 3 * MT;      // 16-B input chunks per thread (P <= 64 * MT pixels, 12 per pixel)
  constexpr int NRC = 3 * MT / 2;  // 16-B residual / output chunks per thread (6 per pixel)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int H = p.H, W = p.W, P = H * W;
  __bf16* sW = reinterpret_cast<__bf16*>(smem);
  __bf16* sX = sW + 9 * CH * CIP;
  __bf16* sO = sX;
  float* sRed = reinterpret_cast<float*>(sX + (P + 1) * CIP);
  float* sGB = sRed + 24;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, kq = lane >> 4;
  const int b = blockIdx.x, h = (b >> 3) & 1, pr = (b & 7) + 8 * (b >> 4), npairs = (int)gridDim.x >> 1;
  const int co0 = CH * h;

  for (int i = tid; i < 9 * CH * 12; i += 256) {  // this half's weights, once
    const int row = i / 12, c8 = i - row * 12;      // row = tap * 48 + co
    const int tap = row / CH, co = row - tap * CH;
    *reinterpret_cast<u32x4*>(&sW[row * CIP + c8 * 8]) =
        *reinterpret_cast<const u32x4*>(&p.wt[((size_t)tap * COUT + co0 + co) * CI + c8 * 8]);
  }
  for (int i = tid; i < CIP / 8; i += 256) *reinterpret_cast<u32x4*>(&sX[P * CIP + i * 8]) = u32x4{0u, 0u, 0u, 0u};
  for (int i = tid; i < CH; i += 256) {
    sGB[i] = p.gamma[co0 + i];
    sGB[CH + i] = p.beta[co0 + i];
  }
  int qr[MT], qc[MT];  // this lane's A-row pixel of each m-tile
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int q = (wave * MT + m) * 16 + l16;
    qr[m] = q < P ? q / W : -1000;
    qc[m] = q < P ? q - qr[m] * W : -1000;
  }
  float biasv[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) biasv[t] = p.bias[co0 + 16 * t + l16];
  const float inv_cnt = 1.0f / (16.0f * (float)P);

  u32x4 xin[NXC], rv[NRC];
  // chunk guards vanish when the board fills the tiles exactly (16x16 with MT = 4), which
  // lets the compiler count vmcnt exactly instead of draining before each LDS write
#define RW_IN(c_) (FULL || (c_) < P * 12)
#define RW_OUT(c_) (FULL || (c_) < P * 6)
  // a missing residual reads x instead (same shape) and is scaled by 0: no branch around loads
  const __bf16* rsrc = p.res ? p.res : p.x;
  const float rsc = p.res ? 1.0f : 0.0f;
  int n = pr;
  {
    const u32x4* xs = reinterpret_cast<const u32x4*>(p.x + (size_t)(n < p.N ? n : 0) * P * CI);
#pragma unroll
    for (int k = 0; k < NXC; ++k) {
      const int c = tid + 256 * k;
      if (RW_IN(c)) xin[k] = xs[c];
    }
  }
#ifdef MC_DIAG
  unsigned long long dacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif
  for (; n < p.N; n += npairs) {
    const int tid = threadIdx.x + opaque0();  // loop-variant: keeps address math in the loop
    // ---- stage the input tile ----
#pragma unroll
    for (int k = 0; k < NXC; ++k) {
      const int c = tid + 256 * k;
      if (RW_IN(c)) {
        const int px = c / 12, c8 = c - px * 12;
        *reinterpret_cast<u32x4*>(&sX[px * CIP + c8 * 8]) = xin[k];
      }
    }
    lds_barrier();
    FSTAMP(0);
    // ---- in flight during the MFMAs: this sample's residual, the next sample's input ----
    const int nn = n + npairs < p.N ? n + npairs : n;  // past the end: a harmless re-read
    // issue order = use order (vmcnt retires in order): dropout scale, residual, next input
    const float dmv = (p.dmask && tid < CH) ? p.dmask[(size_t)n * COUT + co0 + tid] : 1.0f;
#pragma unroll
    for (int k = 0; k < NRC; ++k) {
      const int c = tid + 256 * k;
      if (RW_OUT(c)) {
        const int px = c / 6, ch = c - px * 6;
        rv[k] = *reinterpret_cast<const u32x4*>(&rsrc[((size_t)n * P + px) * COUT + co0 + ch * 8]);
      }
    }
    {
      const u32x4* xs = reinterpret_cast<const u32x4*>(p.x + (size_t)nn * P * CI);
#pragma unroll
      for (int k = 0; k < NXC; ++k) {
        const int c = tid + 256 * k;
        if (RW_IN(c)) xin[k] = xs[c];
      }
    }
    // keep these loads here: the scheduler would otherwise sink them below the MFMAs,
    // and the epilogue's waits would then drain them
    asm volatile("" ::: "memory");
    // ---- implicit GEMM: [pixels] x [48 co], K = 9 taps x 96 ci = 27 steps of 32 ----
    // operands double-buffered in registers: step s+1's LDS reads are issued before
    // step s's MFMAs, so their latency hides behind the matrix pipe
    f32x4 acc[MT][3];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int t = 0; t < 3; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 opA[2][MT], opB[2][3];
#define RW_LOAD(s_, buf_)                                                                              \
  do {                                                                                                 \
    const int tap_ = (s_) / 3, ks_ = (s_) % 3, dr_ = tap_ / 3 - 1, dc_ = tap_ % 3 - 1;                \
    _Pragma("unroll") for (int t_ = 0; t_ < 3; ++t_) opB[buf_][t_] =                                 \
        *reinterpret_cast<const bf16x8*>(sW + (tap_ * CH + 16 * t_ + l16) * CIP + 8 * kq + 32 * ks_);  \
    _Pragma("unroll") for (int m_ = 0; m_ < MT; ++m_) {                                               \
      const int sr_ = qr[m_] + dr_, sc_ = qc[m_] + dc_;                                              \
      const bool v_ = (unsigned)sr_ < (unsigned)H && (unsigned)sc_ < (unsigned)W;                    \
      opA[buf_][m_] = *reinterpret_cast<const bf16x8*>(&sX[(v_ ? sr_ * W + sc_ : P) * CIP + 8 * kq + 32 * ks_]); \
    }                                                                                                  \
  } while (0)
    RW_LOAD(0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, MT + 3, 0);
#pragma unroll
    for (int st = 0; st < 27; ++st) {
      if (st + 1 < 27) RW_LOAD(st + 1, (st + 1) & 1);
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int t = 0; t < 3; ++t)
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(opA[st & 1][m], opB[st & 1][t], acc[m][t], 0, 0, 0);
      // pin the schedule: all of step st+1's LDS reads, then step st's MFMAs (the reads'
      // latency runs under 3*MT MFMAs instead of being waited for between MFMA triplets)
      if (st + 1 < 27) __builtin_amdgcn_sched_group_barrier(0x100, MT + 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 3 * MT, 0);
    }
#undef RW_LOAD
    FSTAMP(1);
    // ---- GroupNorm statistics (n-tile t = group 3h + t), two passes ----
    // acc[m][t][r] = y[px = (wave*MT + m)*16 + 4*kq + r][co = co0 + 16t + l16] - bias
    float gmean[3] = {0.f, 0.f, 0.f}, grstd[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        float v[MT * 4];
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int px = (wave * MT + m) * 16 + 4 * kq + r;
            const float d = acc[m][t][r] + biasv[t] - (pass ? gmean[t] : 0.f);
            v[m * 4 + r] = px < P ? (pass ? d * d : d) : 0.f;
          }
#pragma unroll
        for (int w2 = MT * 2; w2 >= 1; w2 >>= 1)
#pragma unroll
          for (int i = 0; i < w2; ++i) v[i] += v[i + w2];
        const float rs = row_sum16(v[0]);
        const float tot = readlane_f(rs, 15) + readlane_f(rs, 31) + readlane_f(rs, 47) + readlane_f(rs, 63);
        if (lane == 0) sRed[pass * 12 + wave * 3 + t] = tot;
      }
      if (pass == 1) {
        if (tid < CH) sGB[2 * CH + tid] = dmv;
        // y (bf16) -> sO for the coalesced epilogue; every wave is past its MFMAs (barrier above)
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int t = 0; t < 3; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int px = (wave * MT + m) * 16 + 4 * kq + r;
              if (px < P) sO[px * CH + 16 * t + l16] = (__bf16)(acc[m][t][r] + biasv[t]);
            }
      }
      lds_barrier();
      FSTAMP(2 + pass);
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const float s = sRed[pass * 12 + t] + sRed[pass * 12 + 3 + t] + sRed[pass * 12 + 6 + t] + sRed[pass * 12 + 9 + t];
        if (pass == 0) gmean[t] = s * inv_cnt;
        else grstd[t] = rsqrtf(s * inv_cnt + p.eps);
      }
    }
    if (p.stats && tid < 3) {
      float m = 0.f, r = 0.f;
#pragma unroll
      for (int t = 0; t < 3; ++t)
        if (t == tid) {
          m = gmean[t];
          r = grstd[t];
        }
      p.stats[((size_t)n * NGRP + 3 * h + tid) * 2 + 0] = m;
      p.stats[((size_t)n * NGRP + 3 * h + tid) * 2 + 1] = r;
    }
    // ---- epilogue: 16-B chunks of [px][48]: y (saved) and out ----
#pragma unroll
    for (int k = 0; k < NRC; ++k) {
      const int c = tid + 256 * k;
      if (RW_OUT(c)) {
        const int px = c / 6, ch = c - px * 6, g = ch >> 1;
        const size_t o = ((size_t)n * P + px) * COUT + co0 + ch * 8;
        const u32x4 yv = *reinterpret_cast<const u32x4*>(&sO[px * CH + ch * 8]);
        if (p.ysave) *reinterpret_cast<u32x4*>(&p.ysave[o]) = yv;
        const bf16x8 y8 = __builtin_bit_cast(bf16x8, yv);
        const bf16x8 r8 = __builtin_bit_cast(bf16x8, rv[k]);
        float mu = 0.f, rs = 0.f;
#pragma unroll
        for (int gg = 0; gg < 3; ++gg)
          if (gg == g) {
            mu = gmean[gg];
            rs = grstd[gg];
          }
        bf16x8 o8;
        uint32_t mb = 0u;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int cl = ch * 8 + j;
          const float a = sGB[cl] * rs;
          const float sh = sGB[CH + cl] - mu * a;
          const float dm = sGB[2 * CH + cl];
          const float z = fmaxf((float)y8[j] * a + sh + (float)r8[j] * rsc, 0.f);
          o8[j] = (__bf16)(z * dm);
          mb |= ((float)o8[j] > 0.f ? 1u : 0u) << j;
        }
        *reinterpret_cast<u32x4*>(&p.out[o]) = __builtin_bit_cast(u32x4, o8);
        if (p.rmask) p.rmask[((size_t)n * P + px) * (COUT / 8) + co0 / 8 + ch] = (uint8_t)mb;
      }
    }
    FSTAMP(4);
    lds_barrier();  // sO (= sX) fully read before the next input tile lands
    FSTAMP(5);
  }
#ifdef MC_DIAG
  if (p.diag && threadIdx.x == 0)
    for (int k = 0; k < 8; ++k) p.diag[blockIdx.x * 8 + k] = dacc[k];
#endif
#undef RW_IN
#undef RW_OUT
}

template <int MT, bool FULL>
int launch_fwd_rw(const FwdParams& p, hipStream_t s) {
  const size_t lds = rw_lds_bytes(p.H * p.W);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_conv_gn_fwd_rw<MT, FULL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr_set = true;
  }
  // sample pairs (blocks b, b + 8: one XCD), a multiple of 8, one workgroup per CU
  int npairs = (num_cus() / 2) & ~7;
  if (npairs < 8) npairs = 8;
  const int need = (p.N + 7) & ~7;
  if (need < npairs) npairs = need;
  hipLaunchKernelGGL((k_conv_gn_fwd_rw<MT, FULL>), dim3(2 * npairs), dim3(256), lds, s, p);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_fwd launch: %s", hipGetErrorString(e));
    return MS_EHIP;
  }
  return MS_OK;
}

template <int CIN>
int dispatch_fwd(const FwdParams& p, hipStream_t s) {
  const int P = p.H * p.W;
  const int tiles = (P + 31) / 32;
  const int npt = (tiles + WAVES - 1) / WAVES;
  // MC_FWD_RW=1 selects the resident-weight kernel for 96-channel layers on <= 256 cells
  // (measured equal to the per-sample kernel at the PPO minibatch)
  const bool rw = getenv("MC_FWD_RW") ? atoi(getenv("MC_FWD_RW")) != 0 : false;
  if (CIN == 96 && rw && P <= 256 && rw_lds_bytes(P) <= 160 * 1024)
    return P == 256 ? launch_fwd_rw<4, true>(p, s) : (P <= 128 ? launch_fwd_rw<2, false>(p, s) : launch_fwd_rw<4, false>(p, s));
  // MC_FWD_PF=1 selects the one-workgroup-per-CU prefetching variant (A/B measurements)
  static const bool pf = getenv("MC_FWD_PF") ? atoi(getenv("MC_FWD_PF")) != 0 : false;
  if (P == 256) return pf ? launch_fwd<CIN, 2, true, true>(p, s) : launch_fwd<CIN, 2, true, false>(p, s);
  switch (npt) {
    case 1: return pf ? launch_fwd<CIN, 1, false, true>(p, s) : launch_fwd<CIN, 1, false, false>(p, s);
    case 2: return pf ? launch_fwd<CIN, 2, false, true>(p, s) : launch_fwd<CIN, 2, false, false>(p, s);
    case 3: return launch_fwd<CIN, 3, false, false>(p, s);
    case 4: return launch_fwd<CIN, 4, false, false>(p, s);
    default:
      snprintf(g_err, sizeof g_err, "mc_conv_gn_fwd: %d pixels > 512 unsupported", P);
      return MS_EINVAL;
  }
}

}  // namespace

#ifdef MC_DIAG
unsigned long long* g_fwd_diag = nullptr;
#endif

extern "C" {

const char* mc_last_error(void) { return g_err; }

#ifdef MC_DIAG
// diagnostics only (not in mscnn.h): per-workgroup phase cycle totals of the next forwards
void mc_set_fwd_diag(unsigned long long* d) { g_fwd_diag = d; }
#endif

int mc_conv_gn_fwd(const uint16_t* x, const uint16_t* w, const float* bias, const float* gamma, const float* beta,
                   const uint16_t* res, const float* dmask, uint16_t* out, uint16_t* ysave, float* stats,
                   uint8_t* relu_mask, int32_t n, int32_t h, int32_t w_, int32_t cin, float eps, void* stream) {
  if (!x || !w || !bias || !gamma || !beta || !out || n <= 0 || h <= 0 || w_ <= 0) {
    snprintf(g_err, sizeof g_err, "mc_conv_gn_fwd: bad argument");
    return MS_EINVAL;
  }
  FwdParams p;
  p.x = reinterpret_cast<const __bf16*>(x);
  p.wt = reinterpret_cast<const __bf16*>(w);
  p.bias = bias;
  p.gamma = gamma;
  p.beta = beta;
  p.res = reinterpret_cast<const __bf16*>(res);
  p.dmask = dmask;
  p.out = reinterpret_cast<__bf16*>(out);
  p.ysave = reinterpret_cast<__bf16*>(ysave);
  p.stats = stats;
  p.rmask = relu_mask;
  p.N = n;
  p.H = h;
  p.W = w_;
  p.eps = eps;
  static const int stagger = getenv("MC_FWD_STAGGER") ? atoi(getenv("MC_FWD_STAGGER")) : 0;
  p.stagger = stagger;
  p.diag = nullptr;
#ifdef MC_DIAG
  p.diag = g_fwd_diag;
#endif
  hipStream_t s = (hipStream_t)stream;
  if (cin == 16) return dispatch_fwd<16>(p, s);
  if (cin == 96) return dispatch_fwd<96>(p, s);
  snprintf(g_err, sizeof g_err, "mc_conv_gn_fwd: cin %d unsupported (16 or 96)", cin);
  return MS_EINVAL;
}

}  // extern "C"
