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
// k_heads_bwd: one workgroup per CU streams 64-row f tiles through an LDS-DMA ring (below);
//   per tile it recomputes H, writes dh = dlogit * w2 * (h > 0) to an LDS image, then
//     df^T = W1p^T . dh_p^T  (policy only: the mine head sees f.detach(); W1p^T read from
//                             the W1 image with ds_read_b64_tr_b16),
//     dW1 += dh^T . f        (K = the tile's pixels; both operands K-major via
//                             ds_read_b64_tr_b16 from the LDS images),
//     dw2 += h^T . dlogit, db1 += sum dh  (in-lane accumulators);
//   per-workgroup partials are summed by k_heads_reduce in fixed order (deterministic).
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
  const float* b1;
  const float* w2;
  const float* gadd;  // [M / P][96] or null: added to df (the value head's pooled gradient / P)
  E* df;
  float* part;        // [gridDim][PART]
  int64_t M;
  int P;
  unsigned long long* diag;  // MC_DIAG builds: per-wave phase cycle totals [grid][4 waves][8]
};

#ifdef MC_DIAG
#define HSTAMP(k)                                               \
  do {                                                          \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    dacc[k] += t_ - tlast;                                      \
    tlast = t_;                                                 \
  } while (0)
#else
#define HSTAMP(k) do { } while (0)
#endif

// f tile [64][96]: 16-B chunk ch of row r at chunk ch ^ ((r >> 2) & 3)
__device__ __forceinline__ int sf_off(int r, int col) {
  return r * C + 8 * ((col >> 3) ^ ((r >> 2) & 3)) + (col & 7);
}
// dh image [64][192]: chunk ch of row r at ch ^ (((r >> 1) & 1) << 2 | (r >> 2) & 3)
__device__ __forceinline__ int sd_off(int r, int col) {
  return r * NH + 8 * ((col >> 3) ^ ((((r >> 1) & 1) << 2) | ((r >> 2) & 3))) + (col & 7);
}

// k_heads_bwd: one 256-thread workgroup per CU streams 64-row tiles through an NS-slot LDS ring
// filled by LDS-DMA (global_load_lds: no VGPRs), so NS - 1 tiles (~58 KB) are in flight per CU
// while the current one is computed; round 3/4's form (two workgroups per CU, each staging its
// next tile through registers only after the current one) had at most 24 KB in flight per CU and
// ran its staging alone at 1.1 TB/s (profiles/r04/heads_bwd_exp.txt). Per tile, wave w =
// (px-tile pt = w & 1, head hd = w >> 1):
//   H^T[c][px] = W1[c] . f[px] for its head's 96 channels and px-tile (A = W1 rows, B = f rows),
//   dh = dlogit * w2 * (h > 0) -> LDS image (8-B writes: four channels of a pixel per lane),
//   dw2 += h . dlogit, db1 += dh in-lane (lane = pixel, reduced over lanes once at the end);
//   df^T[k][px] = sum_c W1p[c][k] dh[px][c] (policy channels only: the mine head reads f.detach())
//     for k-tiles {0, 1} (w < 2) or {2} (w >= 2), staged in LDS and stored as 16-B rows;
//   dW1[c][k] += sum_px dh[px][c] f[px][k] for dW1 tiles 4 / 4 / 5 / 5 of the 18 (6 c x 3 k):
//   46 / 46 / 44 / 44 MFMAs per wave and tile.
// Ring protocol: at the top of local iteration i each wave issues its 4 DMA instructions of tile
// i + NS - 1 into the slot tile i - 1 left, then waits (counted vmcnt) for its own DMAs of tile i
// and meets the others (lds_barrier): every wave's share of tile i has landed. Per iteration a
// wave issues exactly D = 4 DMAs and S = 3 df stores, so after tile i's DMAs it has issued
// (NS - 1) D + min(i, NS - 1) S more vector-memory instructions; near the end (fewer DMAs) it waits
// for all. The DMAs are inline asm so the compiler does not make LDS reads wait for them.
constexpr int TRB = 64;          // rows per tile
constexpr int NS = 5;            // ring slots
constexpr int DFP = 132;         // df staging row (elements; 66 dwords: conflict-free 8-B writes)
constexpr int GA_FLOATS = 512;   // gadd rows of a tile: samples n0 .. n0 + 4 (P >= 16)
constexpr int HB_D = 4, HB_S = 3;  // DMAs and df stores per wave and tile
template <typename E>
struct HeadSlot {
  E f[TRB * C];
  float dl[2][TRB];
  float ga[GA_FLOATS];
};
template <typename E>
struct HeadLds {
  HeadSlot<E> ring[NS];
  E w[NH * WP];     // W1 rows [c][k]
  E dh[TRB * NH];   // swizzled dh image; after the tile loop: the dw2 combine
  E dfs[TRB * DFP]; // df of the tile, [px][k]
  f32x4 w2v[NH / 4];
};
static_assert(sizeof(HeadLds<__bf16>) <= 160 * 1024, "k_heads_bwd LDS");

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)(p);
}
// one full-wave LDS-DMA: 16 B (x4) or 4 B (x1) a lane, lane-linear at LDS byte address m0v;
// from a 64-bit per-lane address, or (_s) a wave-uniform base plus a 32-bit per-lane offset
__device__ __forceinline__ void dma_x4(const void* src, uint32_t m0v) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0v) : "memory", "m0");
}
__device__ __forceinline__ void dma_x1(const void* src, uint32_t m0v) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(m0v) : "memory", "m0");
}
__device__ __forceinline__ void dma_x4_s(const void* base, uint32_t off, uint32_t m0v) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(off), "s"(base), "s"(m0v)
               : "memory", "m0");
}
__device__ __forceinline__ void dma_x1_s(const void* base, uint32_t off, uint32_t m0v) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1" ::"v"(off), "s"(base), "s"(m0v)
               : "memory", "m0");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 15) | ((N >> 4) << 14));
}
template <int I>
__device__ __forceinline__ void wait_tile(int i) {  // vmcnt of iteration i (I = min(i, NS - 1))
  if constexpr (I + 1 < NS) {
    if (i == I) return wait_vm<(NS - 1) * HB_D + I * HB_S>();
    return wait_tile<I + 1>(i);
  } else {
    wait_vm<(NS - 1) * (HB_D + HB_S)>();
  }
}

// wave WV's four DMAs of global tile t into ring slot s: f chunks 3 WV .. 3 WV + 2 (LDS order,
// so the source chunk carries the swizzle), plus dlp (wave 0), dlm (wave 1), gadd (waves 2, 3;
// samples n0 .. n0 + 4 of the tile's rows, clamped to the buffer); without dlm / gadd a wave
// re-loads a valid address into the unused space so that every wave issues four. A full tile
// addresses its rows from a wave-uniform base (SGPRs) plus this lane's fixed offset (foff);
// the last, partial tile clamps its rows to M - 1 with 64-bit per-lane addresses.
template <typename E, int WV, bool GDMA>
__device__ __forceinline__ void heads_issue(const HeadBwdParams<E>& p, HeadSlot<E>& S, int64_t t, int lane,
                                            const uint32_t (&foff)[3]) {
  const int64_t base = t * TRB, last = p.M - 1;
  const uint32_t fb = __builtin_amdgcn_readfirstlane(lds_addr(S.f));
  const uint32_t db = __builtin_amdgcn_readfirstlane(lds_addr(S.dl[WV & 1]));
  const uint32_t gb = __builtin_amdgcn_readfirstlane(lds_addr(S.ga) + (WV & 1) * 1024);
  if (base + TRB <= p.M) {
    const E* fbase = p.f + base * C;
#pragma unroll
    for (int j = 0; j < 3; ++j) dma_x4_s(fbase, foff[j], fb + (3 * WV + j) * 1024);
    if constexpr (WV < 2) {
      dma_x1_s((WV == 0 || !p.dlm ? p.dlp : p.dlm) + base, lane * 4, db);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int lc = (3 * WV + j) * 64 + lane, r = lc / 12, chs = lc - r * 12, ch = chs ^ ((r >> 2) & 3);
      const int64_t row = base + r < p.M ? base + r : last;
      dma_x4(p.f + row * C + ch * 8, fb + (3 * WV + j) * 1024);
    }
    if constexpr (WV < 2) {
      const int64_t rowl = base + lane < p.M ? base + lane : last;
      dma_x1((WV == 0 || !p.dlm ? p.dlp : p.dlm) + rowl, db);
    }
  }
  if constexpr (WV >= 2) {
    if (GDMA) {
      const int64_t nfl = (p.M / p.P) * C;  // gadd floats
      int64_t q = (base / p.P) * C + (WV - 2) * 256 + lane * 4;
      q = q + 4 <= nfl ? q : nfl - 4;
      dma_x4(p.gadd + q, gb);
    } else {  // a placeholder DMA keeps the per-wave count at four: 1 KiB of W1 (>= 18 KiB), always in bounds
      dma_x4_s(p.w1, lane * 16, gb);
    }
  }
}

template <typename E, int WV, bool GDMA>
__device__ __forceinline__ void heads_bwd_body(const HeadBwdParams<E>& p, HeadLds<E>& L) {
  typedef typename EV<E>::v8 E8;
  typedef typename EV<E>::v4 E4;
  constexpr int PT = WV & 1, HD = WV >> 1;
  constexpr int KT0 = WV < 2 ? 0 : 2, NKT = WV < 2 ? 2 : 1;  // df k-tiles
  constexpr int T0 = WV < 2 ? 4 * WV : 8 + 5 * (WV - 2), NTW = WV < 2 ? 4 : 5;  // dW1 tiles
  constexpr int CT0 = T0 / 3, CT1 = (T0 + NTW - 1) / 3;  // c-tiles of this wave's dW1 tiles
  // db1 c-tiles (each c-tile in exactly one wave, among its dW1 c-tiles): {0,1} {2} {3} {4,5}
  constexpr int B0 = WV == 0 ? 0 : (WV == 1 ? 2 : (WV == 2 ? 3 : 4)), NB = (WV == 0 || WV == 3) ? 2 : 1;
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hh = lane >> 5;
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  f32x16 dwacc[NTW], dbacc[NB];
#pragma unroll
  for (int t = 0; t < NTW; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) dwacc[t][i] = 0.f;
#pragma unroll
  for (int t = 0; t < NB; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) dbacc[t][i] = 0.f;
  float dw2a[3][16];  // channel (3 HD + j) * 32 + 8 (r >> 2) + 4 hh + (r & 3), this lane's pixels
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) dw2a[j][r] = 0.f;
  // b1 in the H accumulators' layout: the first MFMA of each chain starts from it (h = W1 f + b1)
  f32x16 b1i[3];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) b1i[j][r] = p.b1[(3 * HD + j) * 32 + 8 * (r >> 2) + 4 * hh + (r & 3)];
  E8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (E)1.0f;
  uint32_t foff[3];  // this lane's f chunks of a full tile: byte offsets from the tile's first row
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int lc = (3 * WV + j) * 64 + lane, r = lc / 12, chs = lc - r * 12, ch = chs ^ ((r >> 2) & 3);
    foff[j] = (uint32_t)((r * C + ch * 8) * 2);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): b1 is in registers before the ring's DMAs start

  const int64_t ntiles = (p.M + TRB - 1) / TRB;
  const int nloc = (int)((ntiles - blockIdx.x + gridDim.x - 1) / gridDim.x);  // tiles of this workgroup
#ifdef MC_DIAG
  unsigned long long dacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif
  for (int i = 0; i + 1 < NS && i < nloc; ++i)
    heads_issue<E, WV, GDMA>(p, L.ring[i], blockIdx.x + (int64_t)i * gridDim.x, lane, foff);
  const bool mine_dl = HD == 0 || p.dlm != nullptr;
  for (int i = 0; i < nloc; ++i) {
    const int64_t tile = blockIdx.x + (int64_t)i * gridDim.x, base = tile * TRB;
    HSTAMP(7);
    if (i + NS - 1 < nloc) {
      heads_issue<E, WV, GDMA>(p, L.ring[(i + NS - 1) % NS], tile + (int64_t)(NS - 1) * gridDim.x, lane, foff);
      HSTAMP(0);
      wait_tile<0>(i);
    } else {
      HSTAMP(0);
      wait_vm<0>();
    }
    HSTAMP(1);
    lds_barrier();  // every wave's share of tile i has landed
    HSTAMP(2);
    const HeadSlot<E>& S = L.ring[i % NS];
    const int zo = opaque0();

    // ---- H^T (+ b1) for this head's 96 channels and px-tile PT; dh -> LDS; dw2 in-lane ----
    {
      const int px = PT * 32 + l32;
      f32x4 w2r[3][4];  // w2 of this lane's channels, read before the MFMAs finish
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) w2r[j][g4] = L.w2v[((3 * HD + j) * 32 + 8 * g4 + 4 * hh) / 4 + zo];
      const float dl = (base + px < p.M && mine_dl) ? S.dl[HD][px] : 0.f;
      f32x16 acc[3];
      // operands double-buffered, order pinned: step ks+1's LDS reads before step ks's MFMAs
      E8 Af[2][3], Bf[2];
      auto ld = [&](int ks, E8 (&a)[3], E8& bb) {
        bb = *reinterpret_cast<const E8*>(&S.f[sf_off(px, ks * 16 + 8 * hh) + zo]);
#pragma unroll
        for (int j = 0; j < 3; ++j)
          a[j] = *reinterpret_cast<const E8*>(&L.w[((3 * HD + j) * 32 + l32) * WP + ks * 16 + 8 * hh + zo]);
      };
      ld(0, Af[0], Bf[0]);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int ks = 0; ks < 6; ++ks) {
        if (ks + 1 < 6) {
          ld(ks + 1, Af[(ks + 1) & 1], Bf[(ks + 1) & 1]);
          __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[j] = mfma32(Af[ks & 1][j], Bf[ks & 1], ks == 0 ? b1i[j] : acc[j]);
        __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
      }
      // h = max(acc, 0); dw2 += h dl = acc (dl if acc > 0 else 0); dh = (dl if acc > 0 else 0) w2
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int c0 = (3 * HD + j) * 32 + 8 * g4 + 4 * hh;
          E4 d4;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * g4 + e;
            const float t = acc[j][r] > 0.f ? dl : 0.f;
            dw2a[j][r] = __builtin_fmaf(acc[j][r], t, dw2a[j][r]);
            d4[e] = (E)(t * w2r[j][g4][e]);
          }
          *reinterpret_cast<E4*>(&L.dh[sd_off(px, c0)]) = d4;
        }
    }
    HSTAMP(3);
    lds_barrier();
    HSTAMP(2);
    // ---- df^T[k][px] = sum_c W1p[c][k] dh[px][c], k-tiles KT0 .., px-tile PT -> dfs ----
    {
      const int rb = PT * 32 + l32;
      f32x16 acc2[NKT];
      if (p.gadd) {  // (uniform) the accumulators start at gadd[row / P]
        const int64_t rowc = base + rb < p.M ? base + rb : p.M - 1;
        const float* ga;
        if constexpr (GDMA) ga = S.ga + (rowc / p.P - base / p.P) * C;
        else ga = p.gadd + (rowc / p.P) * C;
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
          for (int r = 0; r < 16; ++r) acc2[u][r] = 0.f;
      }
      // operands double-buffered, order pinned: step ks+1's LDS reads before step ks's MFMAs
      E8 A[2][NKT], Bv[2];
      auto ld = [&](int ks, E8 (&a)[NKT], E8& bb) {
        bb = *reinterpret_cast<const E8*>(&L.dh[sd_off(rb, ks * 16 + 8 * hh)]);
        const int r0 = ks * 16 + 8 * (g >> 1) + q;  // W1 rows (K = c), transposed read
#pragma unroll
        for (int u = 0; u < NKT; ++u) {  // (W1 is loop-invariant: the opaque zero keeps the reads in the loop)
          const int col = (KT0 + u) * 32 + 16 * (g & 1) + 4 * pp + zo;
          a[u] = cat8(lds_tr4(&L.w[r0 * WP + col]), lds_tr4(&L.w[(r0 + 4) * WP + col]));
        }
      };
      ld(0, A[0], Bv[0]);
      __builtin_amdgcn_sched_group_barrier(0x100, 1 + 2 * NKT, 0);
#pragma unroll
      for (int ks = 0; ks < 6; ++ks) {
        if (ks + 1 < 6) {
          ld(ks + 1, A[(ks + 1) & 1], Bv[(ks + 1) & 1]);
          __builtin_amdgcn_sched_group_barrier(0x100, 1 + 2 * NKT, 0);
        }
#pragma unroll
        for (int u = 0; u < NKT; ++u) acc2[u] = mfma32(A[ks & 1][u], Bv[ks & 1], acc2[u]);
        __builtin_amdgcn_sched_group_barrier(0x008, NKT, 0);
      }
      // acc2[u][r] = df[px = rb][k = (KT0 + u) * 32 + 8 (r >> 2) + 4 hh + (r & 3)]
#pragma unroll
      for (int u = 0; u < NKT; ++u)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg)
          *reinterpret_cast<E4*>(&L.dfs[rb * DFP + (KT0 + u) * 32 + 8 * gg + 4 * hh]) =
              E4{(E)acc2[u][4 * gg + 0], (E)acc2[u][4 * gg + 1], (E)acc2[u][4 * gg + 2], (E)acc2[u][4 * gg + 3]};
    }
    HSTAMP(4);
    // ---- dW1[c][k] += sum_px dh[px][c] f[px][k]; db1[c] += sum_px dh[px][c] (B = ones) ----
    {
      constexpr int NA = CT1 - CT0 + 1;
      E8 av[2][NA], bv[2][3];
      auto ld = [&](int kk, E8 (&a)[NA], E8 (&b)[3]) {
        // (no opaque zero here: the dh / f tiles are rewritten every tile, so nothing can be hoisted,
        // and with a compile-time row the swizzles fold into per-lane constants + immediate offsets)
        const int r0 = kk * 16 + 8 * (g >> 1) + q;
#pragma unroll
        for (int ct = CT0; ct <= CT1; ++ct) {
          const int col = ct * 32 + 16 * (g & 1) + 4 * pp;
          a[ct - CT0] = cat8(lds_tr4(&L.dh[sd_off(r0, col)]), lds_tr4(&L.dh[sd_off(r0 + 4, col)]));
        }
#pragma unroll
        for (int kt = 0; kt < 3; ++kt) {
          const int col = kt * 32 + 16 * (g & 1) + 4 * pp;
          b[kt] = cat8(lds_tr4(&S.f[sf_off(r0, col)]), lds_tr4(&S.f[sf_off(r0 + 4, col)]));
        }
      };
      ld(0, av[0], bv[0]);
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * (NA + 3), 0);
#pragma unroll
      for (int kk = 0; kk < TRB / 16; ++kk) {
        if (kk + 1 < TRB / 16) {
          ld(kk + 1, av[(kk + 1) & 1], bv[(kk + 1) & 1]);
          __builtin_amdgcn_sched_group_barrier(0x100, 2 * (NA + 3), 0);
        }
#pragma unroll
        for (int t = 0; t < NTW; ++t) {
          const int tt = T0 + t;
          dwacc[t] = mfma32(av[kk & 1][tt / 3 - CT0], bv[kk & 1][tt % 3], dwacc[t]);
        }
#pragma unroll
        for (int t = 0; t < NB; ++t) dbacc[t] = mfma32(av[kk & 1][B0 + t - CT0], ones, dbacc[t]);
        __builtin_amdgcn_sched_group_barrier(0x008, NTW + NB, 0);
      }
    }
    HSTAMP(5);
    lds_barrier();  // dfs complete; the slot, dh and dfs are free after the stores' reads below
    HSTAMP(2);
    // ---- df rows: 16-B chunks, whole 192-B rows (exactly HB_S stores a wave on a full tile) ----
    E* dft = p.df + base * C;
    const bool full = base + TRB <= p.M;
#pragma unroll
    for (int k = 0; k < HB_S; ++k) {
      const int c = tid + 256 * k, r = c / 12, ch = c - r * 12;
      const u32x4 v = *reinterpret_cast<const u32x4*>(&L.dfs[r * DFP + ch * 8]);
      if (full || base + r < p.M) *reinterpret_cast<u32x4*>(&dft[c * 8]) = v;  // row r, chunk ch: c * 8
    }
  }
#ifdef MC_DIAG
  if (p.diag && lane == 0)
    for (int k = 0; k < 8; ++k) p.diag[((size_t)blockIdx.x * 4 + WV) * 8 + k] = dacc[k];
#endif
  // ---- partials: dW1 tiles, db1 (column 0 of the ones products: lanes 0 and 32), dw2 summed
  // over the lanes (pixels); the two px-tile waves of a head combine dw2 in fixed order
  // through LDS (the dh region) in the caller ----
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
  if (l32 == 0) {
#pragma unroll
    for (int t = 0; t < NB; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) part[NH * C + NH + (B0 + t) * 32 + 8 * (r >> 2) + 4 * hh + (r & 3)] = dbacc[t][r];
  }
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) dw2a[j][r] += __shfl_xor(dw2a[j][r], o);
  lds_barrier();  // the dh region is free
  float* red = reinterpret_cast<float*>(L.dh);  // [2 pt][NH]
  if (l32 == 0) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[PT * NH + (3 * HD + j) * 32 + 8 * (r >> 2) + 4 * hh + (r & 3)] = dw2a[j][r];
  }
}

template <typename E, bool GDMA>
__global__ __launch_bounds__(256, 1) void k_heads_bwd(HeadBwdParams<E> p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  HeadLds<E>& L = *reinterpret_cast<HeadLds<E>*>(smem);
  const int tid = threadIdx.x;
  for (int i = tid; i < NH * 12; i += 256) {
    const int c = i / 12, k8 = i - c * 12;
    *reinterpret_cast<u32x4*>(&L.w[c * WP + k8 * 8]) = *reinterpret_cast<const u32x4*>(&p.w1[c * C + k8 * 8]);
  }
  for (int i = tid; i < NH / 4; i += 256) L.w2v[i] = reinterpret_cast<const f32x4*>(p.w2)[i];
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the staging loads are done before the DMAs start
  __syncthreads();
  switch (__builtin_amdgcn_readfirstlane(tid >> 6)) {
    case 0: heads_bwd_body<E, 0, GDMA>(p, L); break;
    case 1: heads_bwd_body<E, 1, GDMA>(p, L); break;
    case 2: heads_bwd_body<E, 2, GDMA>(p, L); break;
    default: heads_bwd_body<E, 3, GDMA>(p, L); break;
  }
  __syncthreads();
  const float* red = reinterpret_cast<const float*>(L.dh);
  float* part = p.part + (size_t)blockIdx.x * PART;
  for (int i = tid; i < NH; i += 256) part[NH * C + i] = red[i] + red[NH + i];
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

int bwd_grid(int64_t M) {  // one k_heads_bwd workgroup per CU
  const int64_t ntiles = (M + TRB - 1) / TRB;
  const int cap = num_cus();
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

#ifdef MC_DIAG
unsigned long long* g_heads_diag = nullptr;
#endif

template <typename E, bool GDMA>
int launch_heads_bwd(const HeadBwdParams<E>& p, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_heads_bwd<E, GDMA>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)sizeof(HeadLds<E>));
    attr = true;
  }
  hipLaunchKernelGGL((k_heads_bwd<E, GDMA>), dim3(grid), dim3(256), sizeof(HeadLds<E>), s, p);
  return check("k_heads_bwd");
}

template <typename E>
int run_heads_bwd(const uint16_t* f, const float* dlp, const float* dlm, const uint16_t* w1, const float* b1,
                  const float* w2, const float* gadd, int32_t P, uint16_t* df, float* dw1, float* db1, float* dw2,
                  float* work, int64_t M, int grid, hipStream_t s) {
  HeadBwdParams<E> p;
  p.f = reinterpret_cast<const E*>(f);
  p.dlp = dlp;
  p.dlm = dlm;
  p.w1 = reinterpret_cast<const E*>(w1);
  p.b1 = b1;
  p.w2 = w2;
  p.gadd = gadd;
  p.df = reinterpret_cast<E*>(df);
  p.part = work;
  p.M = M;
  p.P = P;
  p.diag = nullptr;
#ifdef MC_DIAG
  p.diag = g_heads_diag;
#endif
  // gadd rows by LDS-DMA need a tile to span at most 5 samples (P >= 16); smaller boards read
  // them with plain loads (correct, slower: the compiler's waits for them also wait for the ring);
  // without gadd the kernel without gadd DMAs (P is not used then)
  const int rc = (gadd && P >= 16) ? launch_heads_bwd<E, true>(p, grid, s) : launch_heads_bwd<E, false>(p, grid, s);
  if (rc) return rc;
  hipLaunchKernelGGL(k_heads_reduce, dim3((PART + HR_IB - 1) / HR_IB), dim3(256), 0, s, (const float*)work, grid, dw1,
                     dw2, db1);
  return check("k_heads_reduce");
}

}  // namespace

extern "C" {

#ifdef MC_DIAG
// diagnostics only (not in mscnn.h): per-wave phase cycle totals of the next heads backwards
void mc_set_heads_diag(unsigned long long* d) { g_heads_diag = d; }
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
  if (dtype == MC_DT_BF16) return run_heads_bwd<__bf16>(f, dlp, dlm, w1, b1, w2, gadd, P, df, dw1, db1, dw2, work, M, grid, s);
  if (dtype == MC_DT_F16)
    return run_heads_bwd<_Float16>(f, dlp, dlm, w1, b1, w2, gadd, P, df, dw1, db1, dw2, work, M, grid, s);
  snprintf(g_err, sizeof g_err, "mc_heads_bwd: dtype %d unsupported (0 bf16, 1 f16)", dtype);
  return MS_EINVAL;
}

}  // extern "C"
