// msenv.hip — MI355X (gfx950) vectorised Minesweeper board step + rollout kernels.
//
// Implements the C ABI of include/msenv.h. Reference behaviour followed
// (yakvrz/minesweeper-ppo, /root/reference):
//   MinesweeperEnv.step            minesweeper/env.py:103-152
//   _place_mines_safe              minesweeper/env.py:280-312 (numpy choice, Floyd)
//   _compute_adjacent_counts       minesweeper/env.py:314-335
//   flood_fill_reveal              minesweeper/env_numba.py:17-77
//   _build_obs / action mask / aux minesweeper/env.py:163-196
//   VecMinesweeper init/reset/step minesweeper/env.py:382-511
//   RolloutBuffer.compute_gae      minesweeper/buffers.py:78-94
//   masked Categorical sampling    train_rl.py:229-235
//
// Design: one board per 64-lane wavefront, one wavefront per
// workgroup. Lane r holds row r of the board as a W-bit mask (W <= 62,
// H <= 64). The zero-region flood-fill is a frontier dilation to fixpoint:
// horizontal dilation by shifts inside the lane, vertical by cross-lane
// shuffles, termination by a wave ballot. The numpy-compatible PCG64 stream
// of each env is wave-uniform, so mine placement (Floyd's algorithm + the
// discarded shuffle draws) runs on scalar registers and builds the per-lane
// mine rows directly (membership test = one ballot). The f32 one-hot
// observation, which is ~97% of the bytes a step moves, is emitted as
// coalesced 16-B stores (one 1 KiB wave-instruction per channel plane on
// 16x16) from a per-cell code computed from LDS-staged rows.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>
#include <type_traits>
#include <vector>

#include "../../include/msenv.h"
#include "../../include/msenv_debug.h"

namespace {

constexpr int kWave = 64;
constexpr int kMaxH = 64;
constexpr int kMaxW = 62;

// ---------------------------------------------------------------------------
// Per-env persistent state in HBM (array of structs, 48 B per env).
// ---------------------------------------------------------------------------
struct alignas(16) EnvMeta {
  uint64_t st_hi, st_lo, inc_hi, inc_lo;  // PCG64 state / increment
  uint32_t has32, uinteger;               // numpy next_uint32 half-word buffer
  int32_t step_count;
  uint32_t flags;                         // bit0: first_click_done
};
static_assert(sizeof(EnvMeta) == 48, "EnvMeta layout");

struct KParams {
  const void* actions;   // int64 or int32 [n]
  float* obs;            // [n,10,H,W]
  uint8_t* mask;         // [n,A]
  float* reward;
  uint8_t* done;
  int32_t* step;
  int32_t* last_new;
  double* frac;
  int8_t* outcome;
  EnvMeta* meta;
  uint64_t* mine_words;  // [n, NW] packed rows
  uint64_t* rev_words;   // [n, NW]
  int64_t n;
  int32_t H, W, K, guarantee;
  int32_t actions_i32;
  double win_reward, loss_reward, step_penalty;
  const uint64_t* jump;  // [64][4] PCG64 jump-ahead table {A_hi, A_lo, C_hi, C_lo}, k = 1..64
  uint64_t* diag;        // MS_DIAG builds only: per-env s_memtime stamps [n][8]
  uint32_t dbg_flags;    // MS_DBG_* (msenv_debug.h)
  uint8_t* codes;        // [n,A] cell codes (ms_step_codes: 0 hidden, 1 + k revealed with k), or NULL
};

// ---------------------------------------------------------------------------
// Wave helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
  return ((uint64_t)rfl((uint32_t)(x >> 32)) << 32) | rfl((uint32_t)x);
}

// DPP moves (gfx9 family): wave_shr:1 = lane r <- lane r-1, wave_shl:1 =
// lane r <- lane r+1, row_shr:n = lane r <- lane r-n inside a 16-lane row;
// bound_ctrl fills out-of-range sources with 0. One VALU op each, no LDS.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, true);
}
__device__ __forceinline__ uint64_t wave_shr1(uint64_t v) {  // lane r <- lane r-1 (lane 0 <- 0)
  return ((uint64_t)dpp32<0x138>((uint32_t)(v >> 32)) << 32) | dpp32<0x138>((uint32_t)v);
}
__device__ __forceinline__ uint64_t wave_shl1(uint64_t v) {  // lane r <- lane r+1 (lane 63 <- 0)
  return ((uint64_t)dpp32<0x130>((uint32_t)(v >> 32)) << 32) | dpp32<0x130>((uint32_t)v);
}
__device__ __forceinline__ uint32_t readlane32(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  return ((uint64_t)readlane32((uint32_t)(v >> 32), l) << 32) | readlane32((uint32_t)v, l);
}
// Wave-local LDS barrier. A workgroup of k_step / k_tape holds several boards,
// one per wave, each with its own LDS region, so a board's LDS exchanges only
// have to be ordered inside its wave: a wave's DS operations execute in issue
// order, so this is a compiler code-motion fence plus a wait for outstanding
// LDS results, not an s_barrier (waves of one workgroup never wait for each other).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// wave-wide sum: 4 DPP row-prefix adds + 4 readlanes (uniform result)
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  v += dpp32<0x111>(v);
  v += dpp32<0x112>(v);
  v += dpp32<0x114>(v);
  v += dpp32<0x118>(v);
  return readlane32(v, 15) + readlane32(v, 31) + readlane32(v, 47) + readlane32(v, 63);
}

// ---------------------------------------------------------------------------
// numpy PCG64 (setseq_128 XSL-RR) + bounded Lemire draw, wave-uniform.
// ---------------------------------------------------------------------------
struct Pcg {
  uint64_t hi, lo, ihi, ilo;
  uint32_t has32, uinteger;
};

__device__ __forceinline__ void pcg_step(Pcg& r) {
  constexpr uint64_t MH = 0x2360ED051FC65DA4ull, ML = 0x4385DF649FCCF645ull;
  const uint64_t lo = r.lo * ML;
  uint64_t hi = __umul64hi(r.lo, ML) + r.lo * MH + r.hi * ML;
  const uint64_t lo2 = lo + r.ilo;
  hi += r.ihi + (lo2 < lo ? 1ull : 0ull);
  r.lo = lo2;
  r.hi = hi;
}

__device__ __forceinline__ uint64_t pcg_next64(Pcg& r) {
  pcg_step(r);
  const uint64_t v = r.hi ^ r.lo;
  const unsigned rot = (unsigned)(r.hi >> 58);
  return (v >> rot) | (v << ((64u - rot) & 63u));
}

__device__ __forceinline__ uint32_t pcg_next32(Pcg& r) {
  if (r.has32) {
    r.has32 = 0;
    return r.uinteger;
  }
  const uint64_t x = pcg_next64(r);
  r.has32 = 1;
  r.uinteger = (uint32_t)(x >> 32);
  return (uint32_t)x;
}

// random_bounded_uint64(0, j) for j < 2^32-1: numpy's buffered Lemire.
__device__ __forceinline__ uint32_t pcg_bounded(Pcg& r, uint32_t j) {
  if (j == 0) return 0;
  const uint32_t excl = j + 1u;
  uint64_t m = (uint64_t)pcg_next32(r) * excl;
  uint32_t left = (uint32_t)m;
  if (left < excl) {
    const uint32_t thr = (0xffffffffu - j) % excl;
    while (left < thr) {
      m = (uint64_t)pcg_next32(r) * excl;
      left = (uint32_t)m;
    }
  }
  return (uint32_t)(m >> 32);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// ---------------------------------------------------------------------------
// Board geometry: compile-time for the benchmark shapes, runtime otherwise.
// Rows are packed RPW = floor(64/W) rows per u64 word (no row straddles a
// word): 16x16 -> 4 words (32 B/plane), 9x9 -> 2, 30x16 -> 8, 16x30 -> 8.
// ---------------------------------------------------------------------------
template <int H_, int W_>
struct Geo {
  int H, W;
  __device__ __forceinline__ Geo(int h, int w) : H(H_ ? H_ : h), W(W_ ? W_ : w) {}
  __device__ __forceinline__ int A() const { return H * W; }
  __device__ __forceinline__ int RPW() const { return 64 / W; }
  __device__ __forceinline__ int NW() const { return (H + RPW() - 1) / RPW(); }
  __device__ __forceinline__ uint64_t rowmask() const { return (1ull << W) - 1ull; }
};

template <int H_, int W_>
__device__ __forceinline__ uint64_t load_row(const uint64_t* words, const Geo<H_, W_>& g, int lane) {
  // no branch around the load: lanes past the board read a valid word (clamped index)
  // and are masked afterwards, so the compiler can issue every load of the kernel's
  // prologue back to back instead of waiting out each one inside a divergent branch
  const int rpw = g.RPW();
  const int w = lane / rpw;
  const int wc = w < g.NW() ? w : g.NW() - 1;
  const int sh = (lane - w * rpw) * g.W;
  const uint64_t v = words[wc];
  const uint64_t keep = 0ull - (uint64_t)(lane < g.H);  // a mask, not a select: a select
  return (v >> sh) & g.rowmask() & keep;                 // lets the load sink into a branch
}

// rows -> packed words. rows-per-word a power of two (W=16: 4, W=30: 2, W=8: 8,
// W>32: 1): OR the lane group's shifted rows with DPP (quad_perm xor1/xor2,
// row_half_mirror, row_mirror), no LDS. Otherwise (W=9: 7 rows/word) through
// LDS (srow: this wave's 64-entry row buffer).
template <int H_, int W_>
__device__ __forceinline__ void store_rows(uint64_t* words, uint64_t row, uint64_t* srow,
                                           const Geo<H_, W_>& g, int lane) {
  const int nw = g.NW(), rpw = g.RPW();
  if ((rpw & (rpw - 1)) == 0 && rpw <= 16) {
    uint64_t v = row << ((lane & (rpw - 1)) * g.W);
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    if (rpw >= 2) { lo |= dpp32<0xB1>(lo); hi |= dpp32<0xB1>(hi); }
    if (rpw >= 4) { lo |= dpp32<0x4E>(lo); hi |= dpp32<0x4E>(hi); }
    if (rpw >= 8) { lo |= dpp32<0x141>(lo); hi |= dpp32<0x141>(hi); }
    if (rpw >= 16) { lo |= dpp32<0x140>(lo); hi |= dpp32<0x140>(hi); }
    const int w = lane / rpw;
    if ((lane & (rpw - 1)) == 0 && w < nw) words[w] = ((uint64_t)hi << 32) | lo;
    return;
  }
  srow[lane] = row;
  wave_sync();
  if (lane < nw) {
    uint64_t acc = 0;
    for (int k = 0; k < rpw; ++k) {
      const int r = lane * rpw + k;
      if (r < g.H) acc |= srow[r] << (k * g.W);
    }
    words[lane] = acc;
  }
  wave_sync();
}

// allowed-index -> cell for the ascending forbidden list f[0..m) (numpy's
// flatnonzero(~forbidden) order, env.py:302).
__device__ __forceinline__ int map_allowed(int t, const int (&f)[9], int m) {
#pragma unroll
  for (int i = 0; i < 9; ++i)
    if (i < m && f[i] <= t) ++t;
  return t;
}

// ---------------------------------------------------------------------------
// Per-cell observation code: 0 hidden, 1+count revealed, 10 revealed with no
// count plane (first_click_done False; unreachable but exact).
// sM: padded mine rows shifted left by one (sM[r+1] = mine_r << 1).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t cell_code(const uint64_t* sR, const uint64_t* sM, int r, int c, bool fc) {
  const uint32_t rv = (uint32_t)(sR[r] >> c) & 1u;
  const uint64_t up = sM[r] >> c, mid = sM[r + 1] >> c, dn = sM[r + 2] >> c;
  const uint32_t cnt = (uint32_t)__popcll(up & 7ull) + (uint32_t)__popcll(dn & 7ull) +
                       (uint32_t)(mid & 1ull) + (uint32_t)((mid >> 2) & 1ull);
  return rv ? (fc ? 1u + cnt : 10u) : 0u;
}

// Writes obs [10,A] f32 and mask [A] u8 of one env from the LDS rows. (sCode: A bytes of
// this wave's LDS scratch, reserved for a code-staged emit; a flat 8-B stream of the
// env's 10*A floats measured slower on 9x9 than the per-cell stores below.)
// codes (may be NULL): the cell codes of the obs (1 + count where plane 1 + count is set; the
// unreachable code 10 -- revealed before the first click, plane 0 only -- becomes 0, as
// mc_obs_encode reads such an obs), 4-B aligned when A % 4 == 0.
template <int H_, int W_>
__device__ __forceinline__ void emit_obs(float* __restrict__ obs, uint8_t* __restrict__ mask,
                                         uint8_t* __restrict__ codes, const uint64_t* sR, const uint64_t* sM,
                                         bool fc, const Geo<H_, W_>& g, int lane, uint8_t* sCode) {
  const int A = g.A(), W = g.W;
  if ((A & 3) == 0) {
    const int nq = A >> 2;
    for (int q = lane; q < nq; q += kWave) {
      uint32_t code[4];
      if ((W & 3) == 0) {  // the quad lies in one row: 4 LDS reads for 4 cells
        const int r = (4 * q) / W, c0 = 4 * q - r * W;
        const uint32_t rv = (uint32_t)(sR[r] >> c0);
        const uint64_t up = sM[r] >> c0, mid = sM[r + 1] >> c0, dn = sM[r + 2] >> c0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t cnt = (uint32_t)__popcll((up >> k) & 7ull) + (uint32_t)__popcll((dn >> k) & 7ull) +
                               (uint32_t)((mid >> k) & 1ull) + (uint32_t)((mid >> (k + 2)) & 1ull);
          code[k] = ((rv >> k) & 1u) ? (fc ? 1u + cnt : 10u) : 0u;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int i = 4 * q + k;
          const int r = i / W, c = i - (i / W) * W;
          code[k] = cell_code(sR, sM, r, c, fc);
        }
      }
      if (obs) {
        float4* o4 = reinterpret_cast<float4*>(obs) + q;
        const int stride4 = A >> 2;
        float4 v;
        v.x = code[0] ? 1.f : 0.f;
        v.y = code[1] ? 1.f : 0.f;
        v.z = code[2] ? 1.f : 0.f;
        v.w = code[3] ? 1.f : 0.f;
        o4[0] = v;
#pragma unroll
        for (uint32_t ch = 1; ch < 10; ++ch) {
          v.x = code[0] == ch ? 1.f : 0.f;
          v.y = code[1] == ch ? 1.f : 0.f;
          v.z = code[2] == ch ? 1.f : 0.f;
          v.w = code[3] == ch ? 1.f : 0.f;
          o4[ch * stride4] = v;
        }
      }
      if (mask) {
        const uint32_t m = (code[0] ? 0u : 1u) | ((code[1] ? 0u : 1u) << 8) |
                           ((code[2] ? 0u : 1u) << 16) | ((code[3] ? 0u : 1u) << 24);
        reinterpret_cast<uint32_t*>(mask)[q] = m;
      }
      if (codes) {
        uint32_t cw = 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) cw |= (code[k] == 10u ? 0u : code[k]) << (8 * k);
        reinterpret_cast<uint32_t*>(codes)[q] = cw;
      }
    }
  } else {
    (void)sCode;
    for (int i = lane; i < A; i += kWave) {
      const int r = i / W, c = i - (i / W) * W;
      const uint32_t code = cell_code(sR, sM, r, c, fc);
      if (obs) {
        obs[i] = code ? 1.f : 0.f;
#pragma unroll
        for (uint32_t ch = 1; ch < 10; ++ch) obs[ch * A + i] = code == ch ? 1.f : 0.f;
      }
      if (mask) mask[i] = code ? 0 : 1;
      if (codes) codes[i] = (uint8_t)(code == 10u ? 0u : code);
    }
  }
}

template <int H_, int W_>
__device__ __forceinline__ void stage_rows(uint64_t* sR, uint64_t* sM, uint64_t rev, uint64_t mine,
                                           const Geo<H_, W_>& g, int lane) {
  sR[lane] = rev;
  sM[lane + 1] = mine << 1;
  if (lane == 0) {
    sM[0] = 0ull;
    sM[kWave + 1] = 0ull;
  }
  wave_sync();
}

// ---------------------------------------------------------------------------
// Mine placement (env.py:280-312): numpy's choice(allowed, K, replace=False)
// = Floyd over j in [pop-K, pop) + (K-1) discarded Fisher-Yates draws.
// ---------------------------------------------------------------------------
struct Forbid {  // ascending forbidden cells (the click's clipped 3x3 block, or the click)
  int f[9];
  int m;
  int pop;
};

template <int H_, int W_>
__device__ __forceinline__ Forbid make_forbid(int cell, int ar, int ac, int K, bool guarantee, const Geo<H_, W_>& g) {
  Forbid F;
  F.m = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) F.f[i] = 0;
  if (guarantee) {
#pragma unroll
    for (int dr = -1; dr <= 1; ++dr)
#pragma unroll
      for (int dc = -1; dc <= 1; ++dc) {
        const int rr = ar + dr, cc = ac + dc;
        if (rr >= 0 && rr < g.H && cc >= 0 && cc < g.W) {  // row-major scan = ascending cells
#pragma unroll
          for (int i = 0; i < 9; ++i)
            if (i == F.m) F.f[i] = rr * g.W + cc;
          ++F.m;
        }
      }
  } else {
    F.f[0] = cell;
    F.m = 1;
  }
  F.pop = g.A() - F.m;
  if (F.pop < K) {  // env.py:303-307: relax to the clicked cell only
    F.f[0] = cell;
    F.m = 1;
    F.pop = g.A() - 1;
  }
  return F;
}

// One Floyd insertion in cell space; `mine` holds row r in lane r.
template <int H_, int W_>
__device__ __forceinline__ void floyd_insert(uint64_t& mine, int c1, int j, const Forbid& F, const Geo<H_, W_>& g,
                                             int lane) {
  int r1 = c1 / g.W;
  int col = c1 - r1 * g.W;
  if ((readlane64(mine, r1) >> col) & 1ull) {  // t already chosen: take j instead
    c1 = map_allowed(j, F.f, F.m);
    r1 = c1 / g.W;
    col = c1 - r1 * g.W;
  }
  if (lane == r1) mine |= 1ull << col;
}

// The forbidden cells of a placement (env.py:280-307) as a block: nr rows of nc cells from
// cell base0 (the click's clipped 3x3 neighbourhood, or the click alone: nr = nc = 1).
struct Block {
  int base0, nr, nc, pop;
};
template <int H_, int W_>
__device__ __forceinline__ Block make_block(int cell, int ar, int ac, int K, bool guarantee) {
  Block B;
  if (guarantee) {
    const int r0 = ar > 0 ? ar - 1 : 0, r1 = ar < H_ - 1 ? ar + 1 : H_ - 1;
    const int c0 = ac > 0 ? ac - 1 : 0, c1 = ac < W_ - 1 ? ac + 1 : W_ - 1;
    B.base0 = r0 * W_ + c0;
    B.nr = r1 - r0 + 1;
    B.nc = c1 - c0 + 1;
  } else {
    B.base0 = cell;
    B.nr = B.nc = 1;
  }
  B.pop = H_ * W_ - B.nr * B.nc;
  if (B.pop < K) {  // env.py:303-307: relax to the clicked cell only
    B.base0 = cell;
    B.nr = B.nc = 1;
    B.pop = H_ * W_ - 1;
  }
  return B;
}
// allowed index t -> cell (numpy's flatnonzero(~forbidden)[t], env.py:302), closed form:
// past base0 the allowed cells come in gaps of W - nc between the block's row runs.
template <int W_>
__device__ __forceinline__ int map_block(int t, const Block& B) {
  static_assert(W_ > 3, "a 3-wide block must leave a gap in every row");
  if (t < B.base0) return t;
  const int tp = t - B.base0;
  const int q = B.nc == 3 ? tp / (W_ - 3) : (B.nc == 2 ? tp / (W_ - 2) : tp / (W_ - 1));
  return B.base0 + tp + B.nc * (1 + (q < B.nr - 1 ? q : B.nr - 1));
}

// Serial reference-order placement (also the fallback of the parallel one).
template <int H_, int W_>
__device__ void place_serial(Pcg& rng, uint64_t& mine, const Forbid& F, int K, const Geo<H_, W_>& g, int lane) {
  mine = 0ull;
  for (int j = F.pop - K; j < F.pop; ++j) {
    const int t = (int)pcg_bounded(rng, (uint32_t)j);
    floyd_insert(mine, map_allowed(t, F.f, F.m), j, F, g, lane);
  }
  for (int i = K - 1; i >= 1; --i) (void)pcg_bounded(rng, (uint32_t)i);  // shuffle draws
}

__device__ __forceinline__ bool lemire_rejects(uint32_t left, uint32_t bound) {
  // numpy buffered_bounded_lemire_uint32: redraw iff leftover < (2^32-1-rng) % (rng+1)
  const uint32_t excl = bound + 1u;
  if (left >= excl) return false;
  return left < (0xffffffffu - bound) % excl;
}

// Parallel placement: the PCG64 outputs the placement consumes are computed
// lane-parallel by jump-ahead (state after k steps = A_k*s + C_k*inc, table
// `jt` for k = 1..64), every draw's Floyd value / Lemire test is evaluated in
// its lane, and only the set-membership chain of Floyd stays serial (one
// readlane test per draw). Returns false, leaving rng/mine untouched, if any
// consumed draw would be rejected by Lemire (p ~ 1e-6): the caller then runs
// place_serial, so results are always the reference's.
template <int H_, int W_>
__device__ bool place_parallel(Pcg& rng, uint64_t& mine_out, const Forbid& F, int K, const uint64_t (&J)[4],
                               const Geo<H_, W_>& g, int lane) {
  if (K == 0) {
    mine_out = 0ull;
    return true;
  }
  const int pop = F.pop;
  const int z0 = (pop == K) ? 1 : 0;  // Floyd j = 0 consumes no draw
  const int nF = K - z0;               // Floyd draws
  const int D = nF + (K - 1);          // + shuffle draws
  const int h0 = rng.has32 ? 1 : 0;    // draw 0 comes from the buffered half-word
  const int rem = D - h0;              // draws taken from fresh outputs (>= 0: D >= 1 when h0)
  const int n_out = (rem + 1) >> 1;
  uint64_t mine = 0ull;
  // Floyd iterations without a draw (only j = 0)
  for (int i = 0; i < z0; ++i) floyd_insert(mine, map_allowed(0, F.f, F.m), pop - K + i, F, g, lane);
  if (h0 && D > 0) {
    const uint32_t bound = (nF > 0) ? (uint32_t)(pop - K + z0) : (uint32_t)(K - 1);
    const uint64_t m64 = (uint64_t)rng.uinteger * (bound + 1u);
    if (lemire_rejects((uint32_t)m64, bound)) return false;
    if (nF > 0) floyd_insert(mine, map_allowed((int)(m64 >> 32), F.f, F.m), pop - K + z0, F, g, lane);
  }
  uint64_t bhi = rng.hi, blo = rng.lo;  // base state of the current chunk
  uint64_t fin_hi = rng.hi, fin_lo = rng.lo;
  uint32_t fin_uint = rng.uinteger;
  const uint64_t Ah = J[0], Al = J[1], Ch = J[2], Cl = J[3];
  // C_k * inc is the same for every chunk
  const uint64_t ci_lo = Cl * rng.ilo;
  const uint64_t ci_hi = __umul64hi(Cl, rng.ilo) + Cl * rng.ihi + Ch * rng.ilo;
  for (int c = 0; 64 * c < n_out; ++c) {
    const int q = 64 * c + lane + 1;  // this lane's output index (1-based)
    const uint64_t l1 = Al * blo;
    const uint64_t h1 = __umul64hi(Al, blo) + Al * bhi + Ah * blo;
    const uint64_t sl = l1 + ci_lo;
    const uint64_t sh = h1 + ci_hi + (sl < l1 ? 1ull : 0ull);
    const uint64_t v = sh ^ sl;
    const unsigned rot = (unsigned)(sh >> 58);
    const uint64_t x = (v >> rot) | (v << ((64u - rot) & 63u));
    int tc[2];
    bool rej = false;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int pidx = h0 + 2 * (q - 1) + hf;
      const uint32_t d = hf ? (uint32_t)(x >> 32) : (uint32_t)x;
      const bool is_floyd = pidx < nF;
      const uint32_t bound = is_floyd ? (uint32_t)(pop - K + z0 + pidx) : (uint32_t)(K - 1 - (pidx - nF));
      const uint64_t m64 = (uint64_t)d * (bound + 1u);
      if (q <= n_out && pidx < D) rej |= lemire_rejects((uint32_t)m64, bound);
      tc[hf] = is_floyd ? map_allowed((int)(m64 >> 32), F.f, F.m) : 0;
    }
    if (__ballot(rej) != 0ull) return false;
    // serial Floyd chain over this chunk's draws
    const int pbeg = h0 + 128 * c;
    const int pend = min(h0 + 128 * c + 128, nF);
    for (int pidx = pbeg; pidx < pend; ++pidx) {
      const int rel = pidx - pbeg;
      const int ln = rel >> 1;
      const int c1 = (rel & 1) ? (int)readlane32((uint32_t)tc[1], ln) : (int)readlane32((uint32_t)tc[0], ln);
      floyd_insert(mine, c1, pop - K + z0 + pidx, F, g, lane);
    }
    const int last = min(n_out - 64 * c, 64) - 1;  // lane holding this chunk's last output
    fin_hi = readlane64(sh, last);
    fin_lo = readlane64(sl, last);
    fin_uint = readlane32((uint32_t)(x >> 32), last);
    bhi = readlane64(sh, 63);
    blo = readlane64(sl, 63);
  }
  rng.hi = fin_hi;
  rng.lo = fin_lo;
  if (D > 0) {
    rng.has32 = (uint32_t)(rem & 1);
    rng.uinteger = fin_uint;
  }
  mine_out = mine;
  return true;
}

// x = XSL-RR(state after k steps from (bhi,blo)), jump entry of this lane (k = lane+1)
struct Out {
  uint64_t sh, sl, x;
};
__device__ __forceinline__ Out jump_out(uint64_t bhi, uint64_t blo, uint64_t Ah, uint64_t Al, uint64_t ci_hi,
                                        uint64_t ci_lo) {
  Out o;
  const uint64_t l1 = Al * blo;
  const uint64_t h1 = __umul64hi(Al, blo) + Al * bhi + Ah * blo;
  o.sl = l1 + ci_lo;
  o.sh = h1 + ci_hi + (o.sl < l1 ? 1ull : 0ull);
  const uint64_t v = o.sh ^ o.sl;
  const unsigned rot = (unsigned)(o.sh >> 58);
  o.x = (v >> rot) | (v << ((64u - rot) & 63u));
  return o;
}

__device__ __forceinline__ uint32_t bperm(uint32_t v, int src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}

// Fully lane-parallel placement for 1 <= K <= 128 (every benchmark board): the <= 128
// PCG64 outputs come from two jump-ahead chunks, and lane i (and i+64) owns Floyd iteration
// i: j_i = pop-K+i, t_i = its bounded draw in [0, j_i]. Floyd inserts t_i unless it is
// already chosen, then j_i. The j are distinct and larger than every earlier choice, so "t_i
// already chosen" has a closed form: t_i equals an earlier t_k (chosen either way: as itself
// or because it already was), or t_i equals j_k for the one k = t_i - (pop-K) < i whose own
// t_k collided. The first term is one LDS atomicMin per iteration into a table indexed by t
// (t_i repeats an earlier draw iff the table's minimum is not i); the second follows k by
// ds_bpermute until nothing changes (chains are short: 1-2 rounds). Returns false on a
// Lemire rejection (the caller falls back to place_serial), leaving rng untouched.
__device__ __forceinline__ bool lemire_maybe(uint32_t left, uint32_t bound) {  // a rejection is possible
  return left < bound + 1u;
}
// MS_DIAG builds: sub-phase stamps of a placement (diag slots 8..13 of the env)
#ifdef MS_DIAG
#define PSTAMP(k)                                                  \
  do {                                                             \
    if (dg && lane == 0) dg[(k)] = __builtin_amdgcn_s_memtime();    \
  } while (0)
#else
#define PSTAMP(k) do { } while (0)
#endif

// NS = iteration slots per lane: 1 for K <= 64 (one jump-ahead chunk), 2 for K <= 128.
// Compile-time shapes with W > 3 map allowed indices to cells in closed form (map_block).
template <int H_, int W_, int NS>
__device__ bool place_fixpoint(Pcg& rng, uint64_t& mine_out, const Forbid& F, const Block& B, int K,
                               const uint64_t (&J)[4], uint32_t* tab, uint64_t* srow, const Geo<H_, W_>& g, int lane,
                               uint64_t* dg = nullptr) {
  (void)B;
  (void)dg;
  PSTAMP(8);
  const int A = g.A(), W = g.W;
  const int pop = F.pop;
  const int z0 = (pop == K) ? 1 : 0;
  const int nF = K - z0;
  const int D = nF + (K - 1);
  const int h0 = rng.has32 ? 1 : 0;
  const int rem = D - h0;
  const int n_out = (rem + 1) >> 1;  // <= 128
  const uint64_t ci_lo = J[3] * rng.ilo;
  const uint64_t ci_hi = __umul64hi(J[3], rng.ilo) + J[3] * rng.ihi + J[2] * rng.ilo;
  const Out o0 = jump_out(rng.hi, rng.lo, J[0], J[1], ci_hi, ci_lo);
  Out o1 = o0;
  if (NS == 2 && n_out > 64) o1 = jump_out(readlane64(o0.sh, 63), readlane64(o0.sl, 63), J[0], J[1], ci_hi, ci_lo);
  PSTAMP(9);
  // Lemire rejection test of every consumed draw (draw p of output q, half hf). A draw can
  // only be rejected if its leftover is below bound + 1, which almost never happens: the
  // exact test (a 32-bit remainder) runs only in a wave where some draw is that low.
  uint32_t lft[5], bnd[5];
  bool maybe = false;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    lft[k] = 0xffffffffu;
    bnd[k] = 0u;
  }
  if (h0 && D > 0) {
    bnd[4] = (nF > 0) ? (uint32_t)(pop - K + z0) : (uint32_t)(K - 1);
    lft[4] = (uint32_t)((uint64_t)rng.uinteger * (bnd[4] + 1u));
  }
#pragma unroll
  for (int ch = 0; ch < NS; ++ch) {
    const uint64_t x = ch ? o1.x : o0.x;
    const int q = 64 * ch + lane + 1;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int pidx = h0 + 2 * (q - 1) + hf;
      if (q <= n_out && pidx < D) {
        const uint32_t d = hf ? (uint32_t)(x >> 32) : (uint32_t)x;
        bnd[2 * ch + hf] = pidx < nF ? (uint32_t)(pop - K + z0 + pidx) : (uint32_t)(K - 1 - (pidx - nF));
        lft[2 * ch + hf] = (uint32_t)((uint64_t)d * (bnd[2 * ch + hf] + 1u));
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 5; ++k) maybe |= lemire_maybe(lft[k], bnd[k]);
  if (__ballot(maybe) != 0ull) {  // (uniform, rare) the exact test
    bool rej = false;
#pragma unroll
    for (int k = 0; k < 5; ++k) rej |= lemire_rejects(lft[k], bnd[k]);
    if (__ballot(rej) != 0ull) return false;
  }
  PSTAMP(10);
  // Floyd draws: lane owns iterations i = lane + 64 s
  int t[NS], jj[NS];
  bool valid[NS];
#pragma unroll
  for (int s2 = 0; s2 < NS; ++s2) {
    const int i = lane + 64 * s2;
    valid[s2] = i < K;
    jj[s2] = pop - K + i;
    const int pidx = i - z0;
    const int idx = pidx - h0;
    // ds_bpermute delivers the SOURCE lane's register: fetch both halves of both
    // chunks in converged control flow, then select by this lane's idx
    const int src = (idx >> 1) & 63;
    const uint32_t w0l = bperm((uint32_t)o0.x, src), w0h = bperm((uint32_t)(o0.x >> 32), src);
    uint32_t d = (idx & 1) ? w0h : w0l;
    if (NS == 2) {
      const uint32_t w1l = bperm((uint32_t)o1.x, src), w1h = bperm((uint32_t)(o1.x >> 32), src);
      if (idx >> 7) d = (idx & 1) ? w1h : w1l;
    }
    if (h0 && pidx == 0) d = rng.uinteger;
    t[s2] = (i >= z0) ? (int)(((uint64_t)d * (uint32_t)(jj[s2] + 1)) >> 32) : 0;
  }
  for (int c = lane; c < A; c += kWave) tab[c] = 0xffffffffu;
  wave_sync();
  PSTAMP(11);
#pragma unroll
  for (int s2 = 0; s2 < NS; ++s2)
    if (valid[s2]) atomicMin(&tab[t[s2]], (uint32_t)(lane + 64 * s2));
  wave_sync();
  bool dup[NS], col[NS], kv[NS];
  int ks[NS];
#pragma unroll
  for (int s2 = 0; s2 < NS; ++s2) {
    const int i = lane + 64 * s2;
    dup[s2] = valid[s2] && tab[t[s2]] != (uint32_t)i;
    ks[s2] = t[s2] - (pop - K);  // t_i == j_ks
    kv[s2] = valid[s2] && ks[s2] >= 0 && ks[s2] < i;
    col[s2] = dup[s2];
  }
  uint32_t rounds = 0;
  while (true) {
    ++rounds;
    bool changed = false;
    bool nc[NS];
#pragma unroll
    for (int s2 = 0; s2 < NS; ++s2) {
      // every lane takes part in the reads (ds_bpermute returns 0 from an EXEC-disabled lane)
      const int src = ks[s2] & 63;
      const uint32_t c0 = bperm(col[0] ? 1u : 0u, src);
      const uint32_t c1 = NS == 2 ? bperm(col[NS - 1] ? 1u : 0u, src) : 0u;
      nc[s2] = dup[s2] || (kv[s2] && ((ks[s2] >= 64 ? c1 : c0) != 0u));
      changed |= nc[s2] != col[s2];
    }
#pragma unroll
    for (int s2 = 0; s2 < NS; ++s2) col[s2] = nc[s2];
    if (__ballot(changed) == 0ull) break;
  }
#ifdef MS_DIAG
  if (dg && lane == 0) dg[14] = rounds;
#else
  (void)rounds;
#endif
  PSTAMP(12);
  srow[lane] = 0ull;
  wave_sync();
#pragma unroll
  for (int s2 = 0; s2 < NS; ++s2)
    if (valid[s2]) {
      int cell;
      if constexpr (W_ > 3) cell = map_block<W_>(col[s2] ? jj[s2] : t[s2], B);
      else cell = map_allowed(col[s2] ? jj[s2] : t[s2], F.f, F.m);
      const int r = cell / W;
      atomicOr((unsigned long long*)&srow[r], 1ull << (cell - r * W));
    }
  wave_sync();
  mine_out = lane < g.H ? srow[lane] : 0ull;
  wave_sync();
  // RNG state after the D draws
  if (n_out > 0) {
    const int lastq = n_out - 1;
    const Out& ol = (lastq >= 64) ? o1 : o0;
    rng.hi = readlane64(ol.sh, lastq & 63);
    rng.lo = readlane64(ol.sl, lastq & 63);
    rng.uinteger = readlane32((uint32_t)(ol.x >> 32), lastq & 63);
  }
  if (D > 0) rng.has32 = (uint32_t)(rem & 1);
  PSTAMP(13);
  return true;
}

// ---------------------------------------------------------------------------
// ms_step: one wave = one env.
// ---------------------------------------------------------------------------

#ifdef MS_DIAG
#define STAMP(k)                                                              \
  do {                                                                        \
    if (p.diag && lane == 0) {                                                \
      p.diag[env * 16 + (k)] = __builtin_amdgcn_s_memtime();                  \
      if ((k) == 0) p.diag[env * 16 + 6] = __builtin_amdgcn_s_memrealtime();  \
      if ((k) == 5) p.diag[env * 16 + 7] = __builtin_amdgcn_s_memrealtime();  \
    }                                                                         \
  } while (0)
#else
#define STAMP(k) do { } while (0)
#endif

// ---------------------------------------------------------------------------
// One reveal on one board (MinesweeperEnv.step env.py:103-137 minus the reward /
// step bookkeeping): first-click placement, mine hit, flood fill, win check.
// Wave-uniform results: done, outcome, newly revealed, total revealed.
// ---------------------------------------------------------------------------
template <int H_, int W_>
__device__ __forceinline__ void board_click(Pcg& rng, uint64_t& mine, uint64_t& rev, bool& fc, int cell,
                                            const KParams& p, const uint64_t (&J)[4], uint32_t* sTab,
                                            uint64_t* sR, const Geo<H_, W_>& g, int lane, bool& done,
                                            int& outcome, uint32_t& newly, uint32_t& total_rev,
                                            bool& mines_changed, int64_t env = -1) {
  const int H = g.H, W = g.W, A = g.A();
  const uint64_t rowmask = g.rowmask();
  const int ar = cell / W, ac = cell - (cell / W) * W;
  done = false;
  outcome = MS_OUTCOME_NONE;
  newly = 0;
  const bool cell_rev = (readlane64(rev, ar) >> ac) & 1ull;
  if (!cell_rev) {
    if (!fc) {
      const Forbid F = make_forbid(cell, ar, ac, p.K, p.guarantee != 0, g);
      bool ok = false;
      if (!(p.dbg_flags & MS_DBG_FORCE_SERIAL_PLACEMENT)) {
        if (p.K >= 1 && p.K <= 128 && !(p.dbg_flags & MS_DBG_FORCE_CHAIN_PLACEMENT)) {
          Block B{};
          if constexpr (W_ > 3) B = make_block<H_, W_>(cell, ar, ac, p.K, p.guarantee != 0);
#ifdef MS_DIAG
          uint64_t* dgp = (p.diag && env >= 0) ? p.diag + env * 16 : nullptr;
#else
          uint64_t* dgp = nullptr;
#endif
          ok = p.K <= 64 ? place_fixpoint<H_, W_, 1>(rng, mine, F, B, p.K, J, sTab, sR, g, lane, dgp)
                         : place_fixpoint<H_, W_, 2>(rng, mine, F, B, p.K, J, sTab, sR, g, lane, dgp);
        }
        else
          ok = place_parallel(rng, mine, F, p.K, J, g, lane);
      }
      if (!ok) place_serial(rng, mine, F, p.K, g, lane);
      fc = true;
      mines_changed = true;
    }
    if (env >= 0) STAMP(2);
    const bool hit = (readlane64(mine, ar) >> ac) & 1ull;
    if (hit) {
      if (lane == ar) rev |= 1ull << ac;
      done = true;
      outcome = MS_OUTCOME_LOSS;
    } else {
      // ---- flood_fill_reveal (env_numba.py:17-77) as dilation to fixpoint ----
      const uint64_t U = wave_shr1(mine) | wave_shl1(mine);
      const uint64_t nb = U | (U << 1) | (U >> 1) | (mine << 1) | (mine >> 1);
      const uint64_t zero = ~nb & rowmask;
      const uint64_t allow = ~mine & ~rev & (lane < H ? rowmask : 0ull);
      uint64_t Fr = (lane == ar) ? (1ull << ac) : 0ull;
      while (true) {
        const uint64_t S = Fr & zero;
        const uint64_t Dh = S | (S << 1) | (S >> 1);
        const uint64_t Dv = Dh | wave_shr1(Dh) | wave_shl1(Dh);
        const uint64_t Fn = Fr | (Dv & allow);
        const bool changed = __ballot(Fn != Fr) != 0ull;
        Fr = Fn;
        if (!changed) break;
      }
      rev |= Fr;
      newly = (uint32_t)__popcll(Fr);
    }
  }
  // one reduction for both counts: total revealed (hi 16) | newly revealed (lo 16)
  const uint32_t packed = wave_sum(((uint32_t)__popcll(rev) << 16) | newly);
  total_rev = packed >> 16;
  newly = packed & 0xffffu;
  if (!cell_rev && outcome != MS_OUTCOME_LOSS && (int)total_rev >= A - p.K) {
    done = true;
    outcome = MS_OUTCOME_WIN;
  }
}

// Step outputs of one env in three store instructions, one per element width: lanes
// 0..2 write the 4-byte fields (reward, step, last_new), lanes 0..1 the 1-byte fields
// (done, outcome), lane 0 revealed_frac. Reported before the auto-reset (env.py:492-505).
__device__ __forceinline__ void store_aux(const KParams& p, int64_t idx, int lane, double reward, bool done,
                                          int32_t step_count, uint32_t newly, uint32_t total_rev, int outcome, int A) {
  // The pointers become scalar values before the per-lane select: selecting between the
  // fields themselves compiles to a lane-indexed load from the kernel arguments, and its
  // vmcnt(0) waits for every store in flight (in k_run: the previous step's obs). Global
  // address space: a generic pointer would become a flat store, which also counts in
  // lgkmcnt and so holds up the LDS waits behind it.
  typedef __attribute__((address_space(1))) uint32_t gu32;
  typedef __attribute__((address_space(1))) uint8_t gu8;
  const uint64_t pr = rfl64((uint64_t)p.reward), ps = rfl64((uint64_t)p.step), pl = rfl64((uint64_t)p.last_new);
  const uint64_t pd = rfl64((uint64_t)p.done), po = rfl64((uint64_t)p.outcome);
  gu32* d4 = (gu32*)(lane == 0 ? pr : (lane == 1 ? ps : pl));
  const uint32_t v4 = lane == 0 ? __float_as_uint((float)reward) : (lane == 1 ? (uint32_t)step_count : newly);
  if (lane < 3 && d4) d4[idx] = v4;
  gu8* d1 = (gu8*)(lane == 0 ? pd : po);
  const uint8_t v1 = lane == 0 ? (uint8_t)(done ? 1 : 0) : (uint8_t)(int8_t)outcome;
  if (lane < 2 && d1) d1[idx] = v1;
  if (lane == 0 && p.frac) p.frac[idx] = (double)total_rev / (double)(A > 1 ? A : 1);
}

// EnvMeta write-back in two 16-B stores: {st_hi, st_lo} and {has32, uinteger, step_count, flags}
__device__ __forceinline__ void store_meta(EnvMeta* mp, const Pcg& rng, int32_t step_count, bool fc, int lane) {
  if (lane == 0) {
    *reinterpret_cast<ulonglong2*>(&mp->st_hi) = make_ulonglong2(rng.hi, rng.lo);
    *reinterpret_cast<uint4*>(&mp->has32) =
        make_uint4(rng.has32, rng.uinteger, (uint32_t)step_count, fc ? 1u : 0u);
  }
}

// EPW boards per workgroup, one per wave, each with its own LDS slice: fewer,
// larger workgroups halve the dispatch cost of a 4096-board launch, and no
// wave ever waits on another (board code syncs with wave_sync only).
template <int H_, int W_, int EPW>
__global__ __launch_bounds__(64 * EPW) void k_step(KParams p) {
  __shared__ uint64_t sR_all[EPW][kWave];
  __shared__ uint64_t sM_all[EPW][kWave + 2];
  __shared__ uint32_t sTab_all[EPW][(H_ && W_) ? H_ * W_ : kMaxH * kMaxW];
  const int lane = lane_id();
  const int wv = (EPW == 1) ? 0 : (int)rfl(threadIdx.x >> 6);
  // A wave past the last env (tail of the last workgroup) loads env n-1 and leaves
  // before any store: no early exit that would make every load wait for p.n.
  const int64_t env_raw = (int64_t)blockIdx.x * EPW + wv;
  const bool live = env_raw < p.n;
  const int64_t env = live ? env_raw : p.n - 1;
  uint64_t* sR = sR_all[wv];
  uint64_t* sM = sM_all[wv];
  uint32_t* sTab = sTab_all[wv];
  STAMP(0);
  const Geo<H_, W_> g(p.H, p.W);
  const int A = g.A(), NW = g.NW();

  EnvMeta* mp = p.meta + env;
  uint64_t* mwords = p.mine_words + env * NW;
  uint64_t* rwords = p.rev_words + env * NW;
  // issue every load up front
  uint64_t mine = load_row(mwords, g, lane);
  uint64_t rev = load_row(rwords, g, lane);
  // jump-ahead entry k = lane+1 (2 KiB shared by every wave, L2-resident). Only a board
  // whose next click is its first needs it, but every wave loads it here, right behind
  // its rows: gating it on first_click_done would put a second dependent round trip on
  // exactly the placement waves that end the launch. A placement consumes at most
  // 2K-1 draws = K outputs, so only lanes < K need their entry.
  uint64_t J[4] = {0ull, 0ull, 0ull, 0ull};
  if (lane < p.K) {
    const ulonglong2* e = reinterpret_cast<const ulonglong2*>(p.jump + 4 * lane);
    const ulonglong2 a0 = e[0], a1 = e[1];
    J[0] = a0.x;
    J[1] = a0.y;
    J[2] = a1.x;
    J[3] = a1.y;
  }
  Pcg rng;
  rng.hi = rfl64(mp->st_hi);
  rng.lo = rfl64(mp->st_lo);
  rng.ihi = rfl64(mp->inc_hi);
  rng.ilo = rfl64(mp->inc_lo);
  rng.has32 = rfl(mp->has32);
  rng.uinteger = rfl(mp->uinteger);
  int32_t step_count = (int32_t)rfl((uint32_t)mp->step_count);
  bool fc = (rfl(mp->flags) & 1u) != 0;
  // the action as two unconditional 4-B loads (int32: the element twice; int64: both
  // halves): no branch, so they issue right behind the meta loads
  const uint32_t* ap = reinterpret_cast<const uint32_t*>(p.actions);
  const int64_t aw = p.actions_i32 ? env : 2 * env;
  const uint32_t a_lo = ap[aw], a_hi = ap[p.actions_i32 ? aw : aw + 1];
  int64_t a = p.actions_i32 ? (int64_t)(int32_t)a_lo : (int64_t)(((uint64_t)a_hi << 32) | a_lo);
  a = (int64_t)rfl64((uint64_t)a);
  int64_t cell64 = a % A;  // Python modulo (env.py:106)
  if (cell64 < 0) cell64 += A;
  const int cell = (int)cell64;
  if (!live) return;
  STAMP(1);

  double reward = 0.0;
  bool done = false;
  int outcome = MS_OUTCOME_NONE;
  uint32_t newly = 0, total_rev = 0;
  bool mines_changed = false;
  board_click(rng, mine, rev, fc, cell, p, J, sTab, sR, g, lane, done, outcome, newly, total_rev, mines_changed,
              env);
  STAMP(3);
  if (outcome == MS_OUTCOME_LOSS) reward += p.loss_reward;
  if (outcome == MS_OUTCOME_WIN) reward += p.win_reward;
  reward -= p.step_penalty;
  step_count += 1;

  store_aux(p, env, lane, reward, done, step_count, newly, total_rev, outcome, A);
  if (done) {  // auto-reset (env.py:497-498 -> reset env.py:87-101); RNG continues
    mine = 0ull;
    rev = 0ull;
    fc = false;
    step_count = 0;
    mines_changed = true;
  }
  STAMP(4);

  // ---- observation + action mask (env.py:172-196), issued before the state write-back:
  // the obs stores are ~97 % of the bytes and the launch ends when they drain ----
  if (p.obs || p.mask || p.codes) {
    stage_rows(sR, sM, rev, mine, g, lane);
    emit_obs(p.obs ? p.obs + env * 10 * A : nullptr, p.mask ? p.mask + env * A : nullptr,
             p.codes ? p.codes + env * A : nullptr, sR, sM, fc, g, lane, reinterpret_cast<uint8_t*>(sTab));
  }
  // ---- persist state ----
  store_meta(mp, rng, step_count, fc, lane);
  if (mines_changed) store_rows(mwords, mine, sR, g, lane);
  store_rows(rwords, rev, sR, g, lane);
  STAMP(5);
}

// ---------------------------------------------------------------------------
// ms_step, lane-packed: four boards per wave for small boards (H <= 16, A <= 128,
// 1 <= K <= 16; the 9x9x10 and 8x8x10 benchmark shapes). Board b of the wave lives
// in DPP row b (lanes 16b..16b+15); lane 16b+r holds row r as a W-bit mask. Vertical
// neighbours are row_shr/row_shl:1 with bound_ctrl, which stop at the board edge;
// board sums are row_ror adds; a board-wide predicate is the board's 16 bits of a
// wave ballot; and every per-board scalar (PCG64 state, click, step count) is a VGPR
// that is uniform across the board's 16 lanes. The 4 boards' obs are one contiguous
// 40*A-float span, written as full 1 KiB float4 wave stores from a per-cell plane-bit
// table in this wave's LDS (wave-local: no workgroup barrier). A 9x9 board fills 9 of
// 64 lanes in k_step; here 36 of 64, with a quarter of the waves.
// ---------------------------------------------------------------------------

template <int B>
__device__ __forceinline__ float ub2f(uint32_t w) {  // byte B of w as f32 (one v_cvt_f32_ubyteB)
  return (float)((w >> (8 * B)) & 0xffu);
}

__device__ __forceinline__ uint32_t row_shr1(uint32_t v) { return dpp32<0x111>(v); }  // r <- r-1; r=0 <- 0
__device__ __forceinline__ uint32_t row_shl1(uint32_t v) { return dpp32<0x101>(v); }  // r <- r+1; r=15 <- 0
// LPB = lanes per board (16: four boards per wave, 32: two). A board's rows live in the first
// 16 lanes of its group, so the DPP row ops stay inside one DPP row either way.
template <int LPB>
__device__ __forceinline__ int board_base(int lane) { return lane & (64 - LPB); }
// sum over the board's lanes, result in each of them (row_ror:8,4,2,1; + the other row for 32)
template <int LPB>
__device__ __forceinline__ uint32_t board_sum(uint32_t v, int lane) {
  v += dpp32<0x128>(v);
  v += dpp32<0x124>(v);
  v += dpp32<0x122>(v);
  v += dpp32<0x121>(v);
  if (LPB == 32) v += bperm(v, lane ^ 16);
  return v;
}
template <int LPB>
__device__ __forceinline__ bool board_any(bool v, int lane) {
  constexpr uint64_t M = LPB == 64 ? ~0ull : ((1ull << LPB) - 1ull);
  return ((__ballot(v) >> board_base<LPB>(lane)) & M) != 0ull;
}
template <int LPB>
__device__ __forceinline__ uint32_t board_read(uint32_t v, int lane, int r) {  // v of the board's lane r
  return bperm(v, board_base<LPB>(lane) | (r & 15));
}
template <int LPB>
__device__ __forceinline__ uint64_t board_read64(uint64_t v, int lane, int r) {
  return ((uint64_t)board_read<LPB>((uint32_t)(v >> 32), lane, r) << 32) | board_read<LPB>((uint32_t)v, lane, r);
}

// row r (bits r*W .. r*W+W-1) of a 128-bit cell set
template <int H_, int W_>
__device__ __forceinline__ uint32_t set_row(uint64_t s0, uint64_t s1, int r, const Geo<H_, W_>& g) {
  if (r >= g.H) return 0u;
  const int s = r * g.W;
  const uint64_t v = s >= 64 ? (s1 >> (s - 64)) : ((s0 >> s) | (s ? (s1 << (64 - s)) : 0ull));
  return (uint32_t)(v & g.rowmask());
}
__device__ __forceinline__ bool set_has(uint64_t s0, uint64_t s1, uint32_t c) {
  return (((c < 64u) ? s0 : s1) >> (c & 63u)) & 1ull;
}
__device__ __forceinline__ void set_add(uint64_t& s0, uint64_t& s1, uint32_t c) {
  const uint64_t bit = 1ull << (c & 63u);
  if (c < 64u) s0 |= bit;
  else s1 |= bit;
}

// Placement of one packed board (same draws and result as place_fixpoint). The <= 16
// PCG64 outputs come from one jump-ahead per lane (lane r: output r+1), and lane r owns
// Floyd iteration r: j_r = pop-K+r, t_r = bounded draw in [0, j_r]. Floyd inserts t_r
// unless it is already chosen, then j_r. Because the j are distinct and exceed every
// earlier choice, "t_i already chosen" has a closed form: t_i equals an earlier t_k (which
// is chosen either way), or equals j_k for the one k = t_i - (pop-K) < i whose own t_k
// collided. Lane i gets the first from the board's 16 t values (one LDS broadcast read)
// and resolves the second by following k (a bpermute per link; chains are short).
// Mine rows are built with LDS ORs. Returns false on a Lemire rejection, leaving rng
// untouched (the caller then runs place_serial_packed).
template <int H_, int W_, int LPB>
__device__ bool place_packed(Pcg& rng, uint32_t& mine_out, const Block& B, int K, const uint64_t (&J)[4],
                             uint32_t* sBuf, int lane, uint64_t* dg = nullptr) {
  const int r = lane & (LPB - 1);
  (void)dg;
#ifdef MS_DIAG
#define QSTAMP(k)                                          \
  do {                                                     \
    if (dg && r == 0) dg[(k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define QSTAMP(k) do { } while (0)
#endif
  QSTAMP(15);
  const int pop = B.pop;
  const int z0 = (pop == K) ? 1 : 0;
  const int nF = K - z0;
  const int D = nF + (K - 1);
  const int h0 = rng.has32 ? 1 : 0;
  const int rem = D - h0;
  const int n_out = (rem + 1) >> 1;  // <= K <= 16
  const uint64_t ci_lo = J[3] * rng.ilo;
  const uint64_t ci_hi = __umul64hi(J[3], rng.ilo) + J[3] * rng.ihi + J[2] * rng.ilo;
  const Out o = jump_out(rng.hi, rng.lo, J[0], J[1], ci_hi, ci_lo);
  // Lemire rejection test of the board's draws; the exact test (a 32-bit remainder) runs only
  // in a wave where some leftover is below its bound + 1 (place_fixpoint)
  uint32_t lft[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, bnd[3] = {0u, 0u, 0u};
  if (h0 && D > 0) {
    bnd[2] = (nF > 0) ? (uint32_t)(pop - K + z0) : (uint32_t)(K - 1);
    lft[2] = (uint32_t)((uint64_t)rng.uinteger * (bnd[2] + 1u));
  }
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    const int pidx = h0 + 2 * r + hf;
    if (r < n_out && pidx < D) {
      const uint32_t d = hf ? (uint32_t)(o.x >> 32) : (uint32_t)o.x;
      bnd[hf] = pidx < nF ? (uint32_t)(pop - K + z0 + pidx) : (uint32_t)(K - 1 - (pidx - nF));
      lft[hf] = (uint32_t)((uint64_t)d * (bnd[hf] + 1u));
    }
  }
  const bool maybe = lemire_maybe(lft[0], bnd[0]) || lemire_maybe(lft[1], bnd[1]) || lemire_maybe(lft[2], bnd[2]);
  if (__ballot(maybe) != 0ull) {
    const bool rej = lemire_rejects(lft[0], bnd[0]) || lemire_rejects(lft[1], bnd[1]) || lemire_rejects(lft[2], bnd[2]);
    if (board_any<LPB>(rej, lane)) return false;
  }
  QSTAMP(10);
  // lane r: Floyd iteration i = r (draw pidx = i - z0, from output (pidx - h0) / 2)
  const int jr = pop - K + r;
  const int pidx = r - z0;
  const int idx = pidx - h0;
  const uint32_t wl = board_read<LPB>((uint32_t)o.x, lane, (idx >> 1) & 15);
  const uint32_t wh = board_read<LPB>((uint32_t)(o.x >> 32), lane, (idx >> 1) & 15);
  uint32_t d = (idx & 1) ? wh : wl;
  if (h0 && pidx == 0) d = rng.uinteger;
  const uint32_t t = r >= K ? 0xffffffffu : (r >= z0 ? (uint32_t)(((uint64_t)d * (uint32_t)(jr + 1)) >> 32) : 0u);
  sBuf[lane] = t;
  wave_sync();
  const uint4* tb = reinterpret_cast<const uint4*>(sBuf + board_base<LPB>(lane));
  const uint4 q0 = tb[0], q1 = tb[1], q2 = tb[2], q3 = tb[3];
  const uint32_t tk[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                           q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
  bool dup = false;
#pragma unroll
  for (int k = 0; k < 15; ++k) dup |= (k < r) && tk[k] == t;
  QSTAMP(11);
  const int ks = (int)t - (pop - K);  // t == j_ks
  const bool kv = r < K && ks >= 0 && ks < r;
  bool col = dup;
  while (true) {
    // every lane of the board takes part: ds_bpermute returns 0 from an EXEC-disabled source
    const uint32_t col_ks = board_read<LPB>(col ? 1u : 0u, lane, ks);
    const bool nc = dup || (kv && col_ks != 0u);
    const bool changed = __ballot(nc != col) != 0ull;
    col = nc;
    if (!changed) break;
  }
  QSTAMP(12);
  const int cell = map_block<W_>(col ? jr : (int)t, B);
  wave_sync();
  sBuf[lane] = 0u;
  wave_sync();
  if (r < K) atomicOr(&sBuf[board_base<LPB>(lane) + cell / W_], 1u << (cell % W_));
  wave_sync();
  mine_out = r < H_ ? sBuf[lane] : 0u;
  wave_sync();
  if (n_out > 0) {
    const int lq = n_out - 1;
    rng.hi = board_read64<LPB>(o.sh, lane, lq);
    rng.lo = board_read64<LPB>(o.sl, lane, lq);
    rng.uinteger = board_read<LPB>((uint32_t)(o.x >> 32), lane, lq);
  }
  if (D > 0) rng.has32 = (uint32_t)(rem & 1);
  QSTAMP(13);
  return true;
}

// Serial reference-order placement of one packed board: each lane of the board runs
// the same draws on its copy of the board's state (the Lemire-rejection fallback).
template <int H_, int W_>
__device__ void place_serial_packed(Pcg& rng, uint32_t& mine_out, const Block& B, int K, const Geo<H_, W_>& g,
                                    int r) {
  uint64_t s0 = 0ull, s1 = 0ull;
  for (int j = B.pop - K; j < B.pop; ++j) {
    uint32_t c = (uint32_t)map_block<W_>((int)pcg_bounded(rng, (uint32_t)j), B);
    if (set_has(s0, s1, c)) c = (uint32_t)map_block<W_>(j, B);
    set_add(s0, s1, c);
  }
  for (int i = K - 1; i >= 1; --i) (void)pcg_bounded(rng, (uint32_t)i);  // shuffle draws
  mine_out = set_row(s0, s1, r, g);
}

// Placement of one packed 16x16 board for K <= 48 (same draws and result as place_fixpoint):
// lane r of the board owns Floyd iterations r, r + 16, r + 32 and computes PCG64 outputs
// r + 1, r + 17, r + 33 from its one jump entry (k = r + 1) in three chunks of 16 (a chunk's
// base state is lane 15's state of the previous one). The outputs' words go to the board's LDS
// scratch, so iteration i reads its draw by index; "t_i repeats an earlier t" is an atomicMin
// into the board's 256-entry table, the collision chain follows k = t_i - (pop - K) by
// ds_bpermute (place_fixpoint's closed form), and the mine rows are LDS ORs. Returns false on a
// Lemire rejection, leaving rng untouched (the caller then runs place_serial_packed_w).
// scr: the wave's scratch, [4 boards][A] table | [4][96] output words | [4][16] rows.
template <int H_, int W_>
__device__ bool place_packed3(Pcg& rng, uint32_t& mine_out, const Block& B, int K, const uint64_t (&J)[4],
                              uint32_t* scr, int lane) {
  constexpr int A = H_ * W_;
  static_assert(H_ <= 16 && A <= 256, "16 rows, 8-bit cells");
  const int r = lane & 15, bb = lane >> 4;
  uint32_t* tab = scr + bb * A;
  uint32_t* xw = scr + 4 * A + bb * 96;
  uint32_t* rows = scr + 4 * A + 4 * 96 + bb * 16;
  const int pop = B.pop;
  const int z0 = (pop == K) ? 1 : 0;
  const int nF = K - z0;
  const int D = nF + (K - 1);
  const int h0 = rng.has32 ? 1 : 0;
  const int rem = D - h0;
  const int n_out = (rem + 1) >> 1;  // <= K <= 48
  const uint64_t ci_lo = J[3] * rng.ilo;
  const uint64_t ci_hi = __umul64hi(J[3], rng.ilo) + J[3] * rng.ihi + J[2] * rng.ilo;
  Out o[3];
  o[0] = jump_out(rng.hi, rng.lo, J[0], J[1], ci_hi, ci_lo);
#pragma unroll
  for (int c = 1; c < 3; ++c)
    o[c] = jump_out(board_read64<16>(o[c - 1].sh, lane, 15), board_read64<16>(o[c - 1].sl, lane, 15), J[0], J[1],
                    ci_hi, ci_lo);
  // Lemire rejection test of every consumed draw (exact test only where a leftover is low)
  uint32_t lft[7], bnd[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    lft[k] = 0xffffffffu;
    bnd[k] = 0u;
  }
  if (h0 && D > 0) {
    bnd[6] = (nF > 0) ? (uint32_t)(pop - K + z0) : (uint32_t)(K - 1);
    lft[6] = (uint32_t)((uint64_t)rng.uinteger * (bnd[6] + 1u));
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int q = 16 * c + r + 1;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int pidx = h0 + 2 * (q - 1) + hf;
      if (q <= n_out && pidx < D) {
        const uint32_t d = hf ? (uint32_t)(o[c].x >> 32) : (uint32_t)o[c].x;
        bnd[2 * c + hf] = pidx < nF ? (uint32_t)(pop - K + z0 + pidx) : (uint32_t)(K - 1 - (pidx - nF));
        lft[2 * c + hf] = (uint32_t)((uint64_t)d * (bnd[2 * c + hf] + 1u));
      }
    }
  }
  bool maybe = false;
#pragma unroll
  for (int k = 0; k < 7; ++k) maybe |= lemire_maybe(lft[k], bnd[k]);
  if (__ballot(maybe) != 0ull) {
    bool rej = false;
#pragma unroll
    for (int k = 0; k < 7; ++k) rej |= lemire_rejects(lft[k], bnd[k]);
    if (board_any<16>(rej, lane)) return false;
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    xw[32 * c + 2 * r] = (uint32_t)o[c].x;
    xw[32 * c + 2 * r + 1] = (uint32_t)(o[c].x >> 32);
  }
#pragma unroll
  for (int k = 0; k < A / 16; ++k) tab[16 * k + r] = 0xffffffffu;
  wave_sync();
  int t[3], jj[3];
  bool valid[3];
#pragma unroll
  for (int s2 = 0; s2 < 3; ++s2) {
    const int i = r + 16 * s2;
    valid[s2] = i < K;
    jj[s2] = pop - K + i;
    const int pidx = i - z0;
    const int idx = pidx - h0;  // word of the fresh outputs (output idx / 2, half idx & 1)
    uint32_t d = xw[idx < 0 ? 0 : (idx > 95 ? 95 : idx)];
    if (h0 && pidx == 0) d = rng.uinteger;
    t[s2] = (valid[s2] && i >= z0) ? (int)(((uint64_t)d * (uint32_t)(jj[s2] + 1)) >> 32) : 0;
    if (valid[s2]) atomicMin(&tab[t[s2]], (uint32_t)i);
  }
  wave_sync();
  bool dup[3], col[3], kv[3];
  int ks[3];
#pragma unroll
  for (int s2 = 0; s2 < 3; ++s2) {
    const int i = r + 16 * s2;
    dup[s2] = valid[s2] && tab[t[s2]] != (uint32_t)i;
    ks[s2] = t[s2] - (pop - K);  // t_i == j_ks
    kv[s2] = valid[s2] && ks[s2] >= 0 && ks[s2] < i;
    col[s2] = dup[s2];
  }
  while (true) {
    bool changed = false, nc[3];
#pragma unroll
    for (int s2 = 0; s2 < 3; ++s2) {
      // every lane of the board takes part: ds_bpermute returns 0 from an EXEC-disabled source
      const int src = ks[s2] & 15, sl = (ks[s2] >> 4) & 3;
      const uint32_t c0 = board_read<16>(col[0] ? 1u : 0u, lane, src);
      const uint32_t c1 = board_read<16>(col[1] ? 1u : 0u, lane, src);
      const uint32_t c2 = board_read<16>(col[2] ? 1u : 0u, lane, src);
      const uint32_t cs = sl == 0 ? c0 : (sl == 1 ? c1 : c2);
      nc[s2] = dup[s2] || (kv[s2] && cs != 0u);
      changed |= nc[s2] != col[s2];
    }
#pragma unroll
    for (int s2 = 0; s2 < 3; ++s2) col[s2] = nc[s2];
    if (__ballot(changed) == 0ull) break;
  }
  rows[r] = 0u;
  wave_sync();
#pragma unroll
  for (int s2 = 0; s2 < 3; ++s2)
    if (valid[s2]) {
      const int cell = map_block<W_>(col[s2] ? jj[s2] : t[s2], B);
      atomicOr(&rows[cell / W_], 1u << (cell % W_));
    }
  wave_sync();
  mine_out = r < H_ ? rows[r] : 0u;
  wave_sync();
  if (n_out > 0) {  // the state after the last consumed output (board-uniform chunk c, lane lr)
    const int lq = n_out - 1, c = lq >> 4, lr = lq & 15;
    const uint64_t sh = c == 0 ? o[0].sh : (c == 1 ? o[1].sh : o[2].sh);
    const uint64_t sl = c == 0 ? o[0].sl : (c == 1 ? o[1].sl : o[2].sl);
    const uint64_t x = c == 0 ? o[0].x : (c == 1 ? o[1].x : o[2].x);
    rng.hi = board_read64<16>(sh, lane, lr);
    rng.lo = board_read64<16>(sl, lane, lr);
    rng.uinteger = board_read<16>((uint32_t)(x >> 32), lane, lr);
  }
  if (D > 0) rng.has32 = (uint32_t)(rem & 1);
  return true;
}

// Serial reference-order placement of one packed board of up to 256 cells (the Lemire
// fallback of place_packed3): every lane of the board runs the same draws.
template <int H_, int W_>
__device__ void place_serial_packed_w(Pcg& rng, uint32_t& mine_out, const Block& B, int K, int r) {
  static_assert(64 % W_ == 0 && H_ * W_ <= 256, "rows inside one 64-bit word");
  uint64_t s0 = 0ull, s1 = 0ull, s2 = 0ull, s3 = 0ull;
  auto word = [&](uint32_t c) -> uint64_t& { return c < 64u ? s0 : (c < 128u ? s1 : (c < 192u ? s2 : s3)); };
  for (int j = B.pop - K; j < B.pop; ++j) {
    uint32_t c = (uint32_t)map_block<W_>((int)pcg_bounded(rng, (uint32_t)j), B);
    if ((word(c) >> (c & 63u)) & 1ull) c = (uint32_t)map_block<W_>(j, B);
    word(c) |= 1ull << (c & 63u);
  }
  for (int i = K - 1; i >= 1; --i) (void)pcg_bounded(rng, (uint32_t)i);  // shuffle draws
  const uint32_t c0 = (uint32_t)(r * W_);
  mine_out = r < H_ ? (uint32_t)((word(c0) >> (c0 & 63u)) & ((1ull << W_) - 1ull)) : 0u;
}

// 16x16 boards four to a wave (k_step_packed): 16 rows in a 16-lane DPP row, K <= 48
template <int H_, int W_>
constexpr bool packable16() {
  return H_ == 16 && W_ == 16;
}

template <int H_, int W_>
constexpr bool packable() {
  // W_ <= 30: pk_emit's neighbour count shifts a u32 row by up to W_ + 1 bits
  return H_ >= 1 && H_ <= 16 && W_ >= 1 && W_ <= 30 && H_ * W_ <= 128;
}

// MS_DIAG builds: per-board phase stamps into this env's diag row (lane r == 0 of the board)
#ifdef MS_DIAG
#define DSTAMP(k)                                                            \
  do {                                                                       \
    if (dgs && r == 0) {                                                     \
      dgs[(k)] = __builtin_amdgcn_s_memtime();                               \
      if ((k) == 0) dgs[6] = __builtin_amdgcn_s_memrealtime();               \
      if ((k) == 5) dgs[7] = __builtin_amdgcn_s_memrealtime();               \
    }                                                                        \
  } while (0)
#else
#define DSTAMP(k) do { } while (0)
#endif

// LDS of one wave of the packed kernels
template <int H_, int W_, int BPW>
struct PackedLds {
  static constexpr int A = H_ * W_;
  static constexpr int IMG16 = (BPW * 10 * A + 15) / 16;  // 16-B units of the obs byte image
  uint4 img[IMG16];                     // the wave's boards' obs as 0/1 bytes, in store order
  uint32_t mask[(BPW * A + 3) / 4];     // their action-mask bytes
  alignas(16) uint32_t row[kWave];      // placement scratch; mine rows for the word store
  uint32_t rev[kWave];                  // revealed rows for the word store
};

// LDS of one wave of the 16x16 packed kernel: no byte image (pk_emit16 stores straight from
// the rows), the placement scratch of place_packed3, rows for the word store
template <int H_, int W_, int BPW>
struct PackedLds16 {
  static constexpr int A = H_ * W_;
  uint32_t scr[4 * (A + 96 + 16)];
  alignas(16) uint32_t row[kWave];
  uint32_t rev[kWave];
};

// One reveal on each board of the wave (env.py:103-137 minus the reward / step bookkeeping):
// first-click placement, mine hit, flood fill, win check. Per-board results are uniform
// across the board's lanes.
template <int H_, int W_, int LPB>
__device__ __forceinline__ void pk_click(const KParams& p, Pcg& rng, uint32_t& mine, uint32_t& rev, bool& fc, int cell,
                                         const uint64_t (&J)[4], uint32_t* sRow, int lane, uint64_t* dgs,
                                         bool& done, int& outcome, uint32_t& newly, uint32_t& total_rev,
                                         bool& mines_changed, bool& cell_rev) {
  constexpr int A = H_ * W_;
  constexpr uint32_t ROWMASK = (1u << W_) - 1u;
  const int r = lane & (LPB - 1);
  const Geo<H_, W_> g(H_, W_);
  const int ar = cell / W_, ac = cell - (cell / W_) * W_;
  done = false;
  outcome = MS_OUTCOME_NONE;
  newly = 0;
  cell_rev = board_any<LPB>(r == ar && ((rev >> ac) & 1u), lane);
  if (!cell_rev) {
    if (!fc) {
      const Block B = make_block<H_, W_>(cell, ar, ac, p.K, p.guarantee != 0);
      bool ok = false;
      if constexpr (packable16<H_, W_>()) {
        if (!(p.dbg_flags & MS_DBG_FORCE_SERIAL_PLACEMENT)) ok = place_packed3<H_, W_>(rng, mine, B, p.K, J, sRow, lane);
        if (!ok) place_serial_packed_w<H_, W_>(rng, mine, B, p.K, r);
      } else {
        if (!(p.dbg_flags & MS_DBG_FORCE_SERIAL_PLACEMENT)) ok = place_packed<H_, W_, LPB>(rng, mine, B, p.K, J, sRow, lane, dgs);
        if (!ok) place_serial_packed(rng, mine, B, p.K, g, r);
      }
      fc = true;
      mines_changed = true;
    }
    DSTAMP(2);
    const bool hit = board_any<LPB>(r == ar && ((mine >> ac) & 1u), lane);
    if (hit) {
      if (r == ar) rev |= 1u << ac;
      done = true;
      outcome = MS_OUTCOME_LOSS;
    } else {  // flood_fill_reveal (env_numba.py:17-77): dilation to a fixpoint inside the board's row
      const uint32_t U = row_shr1(mine) | row_shl1(mine);
      const uint32_t nb = U | (U << 1) | (U >> 1) | (mine << 1) | (mine >> 1);
      const uint32_t zero = ~nb & ROWMASK;
      const uint32_t allow = ~mine & ~rev & (r < H_ ? ROWMASK : 0u);
      uint32_t Fr = (r == ar) ? (1u << ac) : 0u;
      while (true) {
        const uint32_t S = Fr & zero;
        const uint32_t Dh = S | (S << 1) | (S >> 1);
        const uint32_t Dv = Dh | row_shr1(Dh) | row_shl1(Dh);
        const uint32_t Fn = Fr | (Dv & allow);
        const bool changed = __ballot(Fn != Fr) != 0ull;
        Fr = Fn;
        if (!changed) break;
      }
      rev |= Fr;
      newly = (uint32_t)__popc(Fr);
    }
  }
  const uint32_t packed = board_sum<LPB>(((uint32_t)__popc(rev) << 16) | newly, lane);
  total_rev = packed >> 16;
  newly = packed & 0xffffu;
  if (!cell_rev && outcome != MS_OUTCOME_LOSS && (int)total_rev >= A - p.K) {
    done = true;
    outcome = MS_OUTCOME_WIN;
  }
}

// Observation + action mask (env.py:172-196) of the wave's nbl live boards, written to the
// contiguous chunks ob (nbl*10*A floats, 16-B aligned) and mb (nbl*A bytes, 4-B aligned for
// BPW = 4, 2-B for BPW = 2). The obs are one-hot, so the wave zero-fills a byte image of them
// in LDS, each lane sets the (at most two) 1 bytes of each revealed cell of its row, and the
// wave copies the image out as whole 1 KiB float4 stores (4 bytes -> 4 floats with
// v_cvt_f32_ubyte0..3).
template <int H_, int W_, int BPW, int LPB>
__device__ __forceinline__ void pk_emit(float* ob, uint8_t* mb, int nbl, uint32_t mine, uint32_t rev, bool fc,
                                        PackedLds<H_, W_, BPW>& S, int lane, uint64_t* dgs) {
  constexpr int A = H_ * W_;
  constexpr int IMG16 = PackedLds<H_, W_, BPW>::IMG16;
  const int r = lane & (LPB - 1);
  uint8_t* sImg = reinterpret_cast<uint8_t*>(S.img);
  uint8_t* sMask = reinterpret_cast<uint8_t*>(S.mask);
#pragma unroll
  for (int k = 0; k < (IMG16 + kWave - 1) / kWave; ++k)
    if (k * kWave + lane < IMG16) S.img[k * kWave + lane] = make_uint4(0u, 0u, 0u, 0u);
  const uint32_t m1 = mine << 1;
  const uint32_t up1 = row_shr1(m1), dn1 = row_shl1(m1);  // rows r-1, r+1 (0 past the edge)
  wave_sync();
  if (r < H_) {
    uint8_t* img = sImg + (lane / LPB) * (10 * A) + r * W_;
    uint8_t* mk = sMask + (lane / LPB) * A + r * W_;
#pragma unroll
    for (int c = 0; c < W_; ++c) {
      const uint32_t cnt = (uint32_t)__popc((up1 >> c) & 7u) + (uint32_t)__popc((dn1 >> c) & 7u) +
                           ((m1 >> c) & 1u) + ((m1 >> (c + 2)) & 1u);
      const uint32_t rv = (rev >> c) & 1u;
      mk[c] = (uint8_t)(rv ^ 1u);
      // unconditional byte stores, no branch per cell: channel 0 = revealed, channel 1 + count
      // = 1 for a revealed cell after the first click (env.py:183-190); a hidden cell writes a
      // 0 over the zero-filled byte of its channel 1 + count
      img[c] = (uint8_t)rv;
      img[(1 + cnt) * A + c] = (uint8_t)(fc ? rv : 0u);
    }
  }
  DSTAMP(8);
  wave_sync();
  if (ob) {
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(sImg);
    if (nbl == BPW) {
      constexpr int NQ = BPW * 10 * A / 4;
      float4* o4 = reinterpret_cast<float4*>(ob);
#pragma unroll
      for (int k = 0; k < (NQ + kWave - 1) / kWave; ++k) {
        const int q = k * kWave + lane;
        if (q < NQ) {
          const uint32_t w = s32[q];
          o4[q] = make_float4(ub2f<0>(w), ub2f<1>(w), ub2f<2>(w), ub2f<3>(w));
        }
      }
    } else {  // partial last wave: whole float4s, then the odd tail floats
      const int nf = nbl * 10 * A;
      for (int q = lane; q < (nf >> 2); q += kWave) {
        const uint32_t w = s32[q];
        reinterpret_cast<float4*>(ob)[q] = make_float4(ub2f<0>(w), ub2f<1>(w), ub2f<2>(w), ub2f<3>(w));
      }
      for (int f = (nf & ~3) + lane; f < nf; f += kWave) ob[f] = (float)sImg[f];
    }
  }
  DSTAMP(9);
  if (mb) {
    const int nbytes = nbl * A;
    if (BPW == 4) {
      for (int q = lane; q < (nbytes >> 2); q += kWave) reinterpret_cast<uint32_t*>(mb)[q] = S.mask[q];
      for (int i = (nbytes & ~3) + lane; i < nbytes; i += kWave) mb[i] = sMask[i];
    } else {
      const uint16_t* m16 = reinterpret_cast<const uint16_t*>(sMask);
      for (int q = lane; q < (nbytes >> 1); q += kWave) reinterpret_cast<uint16_t*>(mb)[q] = m16[q];
      if ((nbytes & 1) && lane == 0) mb[nbytes - 1] = sMask[nbytes - 1];
    }
  }
}

// Observation + action mask of the wave's nbl live 16x16 boards without an LDS image: per
// board, lane l covers row l / 4, cells 4 (l % 4) .. +3, fetching that row and its two
// neighbours from the board's lanes; each of the 10 channel planes is then one 1 KiB float4
// store of the wave and the mask one 256-B dword store. Same bytes as pk_emit (env.py:172-196).
template <int H_, int W_, int BPW>
__device__ __forceinline__ void pk_emit16(float* ob, uint8_t* mb, int nbl, uint32_t mine, uint32_t rev, bool fc,
                                          int lane) {
  static_assert(H_ == 16 && W_ == 16, "16x16 boards");
  constexpr int A = H_ * W_;
  const int row = lane >> 2, c0 = 4 * (lane & 3);
#pragma unroll
  for (int b = 0; b < BPW; ++b) {
    if (b >= nbl) break;  // (wave-uniform)
    const int src = 16 * b + row;
    const uint32_t m = bperm(mine, src), rv = bperm(rev, src);
    const uint32_t mu0 = bperm(mine, (src - 1) & 63), md0 = bperm(mine, (src + 1) & 63);
    const uint32_t mu = row > 0 ? mu0 : 0u, md = row < 15 ? md0 : 0u;
    const bool f = bperm(fc ? 1u : 0u, 16 * b) != 0u;
    const uint32_t m1 = m << 1, up1 = mu << 1, dn1 = md << 1;
    uint32_t cnt[4], rb[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = c0 + e;
      cnt[e] = (uint32_t)__popc((up1 >> c) & 7u) + (uint32_t)__popc((dn1 >> c) & 7u) + ((m1 >> c) & 1u) +
               ((m1 >> (c + 2)) & 1u);
      rb[e] = (rv >> c) & 1u;
    }
    if (ob) {
      float4* o4 = reinterpret_cast<float4*>(ob + (size_t)b * 10 * A) + lane;
#pragma unroll
      for (int ch = 0; ch < 10; ++ch) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[e] = ch == 0 ? (float)rb[e] : ((f && rb[e] && cnt[e] + 1u == (uint32_t)ch) ? 1.f : 0.f);
        o4[ch * (A / 4)] = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    if (mb)
      reinterpret_cast<uint32_t*>(mb + (size_t)b * A)[lane] =
          (rb[0] ^ 1u) | ((rb[1] ^ 1u) << 8) | ((rb[2] ^ 1u) << 16) | ((rb[3] ^ 1u) << 24);
  }
}

// EnvMeta and the row words of each live board (rows -> packed words through LDS)
template <int H_, int W_, int BPW, int LPB, class Lds>
__device__ __forceinline__ void pk_store_state(EnvMeta* mp, uint64_t* mwords, uint64_t* rwords, const Pcg& rng,
                                               int32_t step_count, bool fc, uint32_t mine, uint32_t rev,
                                               bool mines_changed, bool live, Lds& S, int lane) {
  constexpr int RPW = 64 / W_;
  constexpr int NW = (H_ + RPW - 1) / RPW;
  const int r = lane & (LPB - 1);
  store_meta(mp, rng, step_count, fc, live ? r : 1);
  const int rb = board_base<LPB>(lane);
  S.row[lane] = mine;
  S.rev[lane] = rev;
  wave_sync();
  if (live && r < NW) {
    uint64_t am = 0ull, ar_ = 0ull;
#pragma unroll
    for (int k = 0; k < RPW; ++k)
      if (r * RPW + k < H_) {
        am |= (uint64_t)S.row[rb + r * RPW + k] << (k * W_);
        ar_ |= (uint64_t)S.rev[rb + r * RPW + k] << (k * W_);
      }
    if (mines_changed) mwords[r] = am;
    rwords[r] = ar_;
  }
}

// Loads of one packed board: rows, this lane's jump entry (k = r+1: a placement uses outputs
// 1..K), and the meta (every lane of the board reads the same 48 B)
template <int H_, int W_>
__device__ __forceinline__ void pk_load(const KParams& p, int64_t env, int r, uint32_t& mine, uint32_t& rev,
                                        uint64_t (&J)[4], Pcg& rng, int32_t& step_count, bool& fc) {
  constexpr int RPW = 64 / W_;
  constexpr int NW = (H_ + RPW - 1) / RPW;
  const Geo<H_, W_> g(H_, W_);
  const EnvMeta* mp = p.meta + env;
  mine = (uint32_t)load_row(p.mine_words + env * NW, g, r);
  rev = (uint32_t)load_row(p.rev_words + env * NW, g, r);
  J[0] = J[1] = J[2] = J[3] = 0ull;
  if (r < p.K) {
    const ulonglong2* e = reinterpret_cast<const ulonglong2*>(p.jump + 4 * r);
    const ulonglong2 a0 = e[0], a1 = e[1];
    J[0] = a0.x;
    J[1] = a0.y;
    J[2] = a1.x;
    J[3] = a1.y;
  }
  const ulonglong2 st = *reinterpret_cast<const ulonglong2*>(&mp->st_hi);
  const ulonglong2 inc = *reinterpret_cast<const ulonglong2*>(&mp->inc_hi);
  const uint4 m4 = *reinterpret_cast<const uint4*>(&mp->has32);
  rng.hi = st.x;
  rng.lo = st.y;
  rng.ihi = inc.x;
  rng.ilo = inc.y;
  rng.has32 = m4.x;
  rng.uinteger = m4.y;
  step_count = (int32_t)m4.z;
  fc = (m4.w & 1u) != 0;
}

template <int H_, int W_, int WPG, int BPW>
__global__ __launch_bounds__(64 * WPG) void k_step_packed(KParams p) {
  constexpr int LPB = kWave / BPW;  // lanes per board (the board's rows: its first H)
  constexpr bool BIG = packable16<H_, W_>();  // 16x16: place_packed3 + pk_emit16
  static_assert(BPW == 2 || BPW == 4, "boards per wave");
  static_assert(packable<H_, W_>() || (BIG && BPW == 4), "packed board shape");
  constexpr int A = H_ * W_;
  constexpr int RPW = 64 / W_;
  constexpr int NW = (H_ + RPW - 1) / RPW;
  using Lds = std::conditional_t<BIG, PackedLds16<H_, W_, BPW>, PackedLds<H_, W_, BPW>>;
  __shared__ Lds S_all[WPG];
  const int lane = lane_id();
  const int r = lane & (LPB - 1);
  const int wv = (WPG == 1) ? 0 : (int)rfl(threadIdx.x >> 6);
  Lds& S = S_all[wv];
  const int64_t env0 = ((int64_t)blockIdx.x * WPG + wv) * BPW;
  const bool wave_live = env0 < p.n;
  const int64_t env_raw = env0 + (lane / LPB);
  const bool live = env_raw < p.n;
  const int64_t env = live ? env_raw : p.n - 1;  // a board past the end loads env n-1, stores nothing
  uint64_t* dgs = (p.diag && live) ? p.diag + env * 16 : nullptr;
  (void)dgs;
  DSTAMP(0);
  uint32_t mine, rev;
  uint64_t J[4];
  Pcg rng;
  int32_t step_count;
  bool fc;
  pk_load<H_, W_>(p, env, r, mine, rev, J, rng, step_count, fc);
  const uint32_t* ap = reinterpret_cast<const uint32_t*>(p.actions);
  const int64_t aw = p.actions_i32 ? env : 2 * env;
  const uint32_t a_lo = ap[aw], a_hi = ap[p.actions_i32 ? aw : aw + 1];
  if (!wave_live) return;
  const int64_t a = p.actions_i32 ? (int64_t)(int32_t)a_lo : (int64_t)(((uint64_t)a_hi << 32) | a_lo);
  int64_t cell64 = a % A;  // Python modulo (env.py:106)
  if (cell64 < 0) cell64 += A;
  DSTAMP(1);
  bool done, mines_changed = false, cell_rev;
  int outcome;
  uint32_t newly, total_rev;
  uint32_t* scr;
  if constexpr (BIG) scr = S.scr;
  else scr = S.row;
  pk_click<H_, W_, LPB>(p, rng, mine, rev, fc, (int)cell64, J, scr, lane, dgs, done, outcome, newly, total_rev,
                        mines_changed, cell_rev);
  DSTAMP(3);
  double reward = 0.0;
  if (outcome == MS_OUTCOME_LOSS) reward += p.loss_reward;
  if (outcome == MS_OUTCOME_WIN) reward += p.win_reward;
  reward -= p.step_penalty;
  step_count += 1;
  store_aux(p, env, live ? r : kWave, reward, done, step_count, newly, total_rev, outcome, A);
  if (done) {  // auto-reset (env.py:497-498 -> reset env.py:87-101); RNG continues
    mine = 0u;
    rev = 0u;
    fc = false;
    step_count = 0;
    mines_changed = true;
  }
  DSTAMP(4);
  const int nbl = (p.n - env0 < BPW) ? (int)(p.n - env0) : BPW;  // live boards of this wave
  if constexpr (BIG) {
    if (p.obs || p.mask)
      pk_emit16<H_, W_, BPW>(p.obs ? p.obs + env0 * 10 * A : nullptr, p.mask ? p.mask + env0 * A : nullptr, nbl, mine,
                             rev, fc, lane);
    DSTAMP(9);
  } else {
    if (p.obs || p.mask)
      pk_emit<H_, W_, BPW, LPB>(p.obs ? p.obs + env0 * 10 * A : nullptr, p.mask ? p.mask + env0 * A : nullptr, nbl,
                                mine, rev, fc, S, lane, dgs);
  }
  pk_store_state<H_, W_, BPW, LPB>(p.meta + env, p.mine_words + env * NW, p.rev_words + env * NW, rng, step_count, fc,
                                   mine, rev, mines_changed, live, S, lane);
  DSTAMP(5);
}

// ---------------------------------------------------------------------------
// ms_reset: clear boards (RNG continues) + obs zeros + mask ones.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_reset(EnvMeta* meta, uint64_t* mw, uint64_t* rw, int64_t n,
                                                int NW, float* obs, uint8_t* mask, int A) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = tid; e < n; e += nthreads) {
    meta[e].step_count = 0;
    meta[e].flags = 0;
  }
  for (int64_t i = tid; i < n * NW; i += nthreads) {
    mw[i] = 0;
    rw[i] = 0;
  }
  if (obs) {
    const int64_t tot = n * 10 * (int64_t)A;
    if ((tot & 3) == 0) {
      float4* o4 = reinterpret_cast<float4*>(obs);
      for (int64_t i = tid; i < tot / 4; i += nthreads) o4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      for (int64_t i = tid; i < tot; i += nthreads) obs[i] = 0.f;
    }
  }
  if (mask)
    for (int64_t i = tid; i < n * (int64_t)A; i += nthreads) mask[i] = 1;
}

// ---------------------------------------------------------------------------
// ms_labels / ms_snapshot: one wave per env, cell-parallel.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_labels(const EnvMeta* meta, const uint64_t* mw, const uint64_t* rw,
                                               int64_t n, int H, int W, float* labels, uint8_t* valid) {
  __shared__ uint64_t sMine[kWave], sRev[kWave];
  const int lane = lane_id();
  const int64_t env = blockIdx.x;
  if (env >= n) return;
  const Geo<0, 0> g(H, W);
  const int NW = g.NW(), A = g.A();
  sMine[lane] = load_row(mw + env * NW, g, lane);
  sRev[lane] = load_row(rw + env * NW, g, lane);
  const bool fc = (meta[env].flags & 1u) != 0;
  __syncthreads();
  for (int i = lane; i < A; i += kWave) {
    const int r = i / W, c = i - r * W;
    const uint32_t mb = (uint32_t)(sMine[r] >> c) & 1u, rb = (uint32_t)(sRev[r] >> c) & 1u;
    if (labels) labels[env * A + i] = fc ? (float)mb : 0.f;
    if (valid) valid[env * A + i] = fc ? (uint8_t)(rb ^ 1u) : 0;
  }
}

__global__ __launch_bounds__(64) void k_snapshot(const EnvMeta* meta, const uint64_t* mw, const uint64_t* rw,
                                                 int64_t n, int H, int W, uint8_t* mine, uint8_t* revealed,
                                                 uint8_t* counts, uint8_t* first_click, int32_t* step_count) {
  __shared__ uint64_t sMine[kWave + 2], sRev[kWave];
  const int lane = lane_id();
  const int64_t env = blockIdx.x;
  if (env >= n) return;
  const Geo<0, 0> g(H, W);
  const int NW = g.NW(), A = g.A();
  const uint64_t m = load_row(mw + env * NW, g, lane);
  sRev[lane] = load_row(rw + env * NW, g, lane);
  sMine[lane + 1] = m << 1;
  if (lane == 0) {
    sMine[0] = 0;
    sMine[kWave + 1] = 0;
    if (first_click) first_click[env] = (uint8_t)(meta[env].flags & 1u);
    if (step_count) step_count[env] = meta[env].step_count;
  }
  __syncthreads();
  for (int i = lane; i < A; i += kWave) {
    const int r = i / W, c = i - r * W;
    if (mine) mine[env * A + i] = (uint8_t)((sMine[r + 1] >> (c + 1)) & 1ull);
    if (revealed) revealed[env * A + i] = (uint8_t)((sRev[r] >> c) & 1ull);
    if (counts) {
      const uint64_t up = sMine[r] >> c, mid = sMine[r + 1] >> c, dn = sMine[r + 2] >> c;
      counts[env * A + i] = (uint8_t)(__popcll(up & 7ull) + __popcll(dn & 7ull) + (mid & 1ull) + ((mid >> 2) & 1ull));
    }
  }
}

__global__ __launch_bounds__(256) void k_rng_state(const EnvMeta* meta, int64_t n, uint64_t* out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const EnvMeta m = meta[e];
  out[6 * e + 0] = m.st_hi;
  out[6 * e + 1] = m.st_lo;
  out[6 * e + 2] = m.inc_hi;
  out[6 * e + 3] = m.inc_lo;
  out[6 * e + 4] = m.has32;
  out[6 * e + 5] = m.uinteger;
}

// ---------------------------------------------------------------------------
// ms_tape_actions: synthetic policy, one wave per env.
// ---------------------------------------------------------------------------


// exclusive prefix sum inside each 16-lane row (row_shr 1/2/4/8)
__device__ __forceinline__ uint32_t row_excl_scan16(uint32_t v) {
  uint32_t s = v;
  s += dpp32<0x111>(s);
  s += dpp32<0x112>(s);
  s += dpp32<0x114>(s);
  s += dpp32<0x118>(s);
  return s - v;
}

// exclusive prefix sum over the wave: Kogge-Stone inside 16-lane rows
// (row_shr 1/2/4/8), then row_bcast15 / row_bcast31 carry across rows (GFX9 DPP)
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v) {
  uint32_t s = v;
  s += dpp32<0x111>(s);
  s += dpp32<0x112>(s);
  s += dpp32<0x114>(s);
  s += dpp32<0x118>(s);
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x142, 0xa, 0xf, false);
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x143, 0xc, 0xf, false);
  return s - v;
}

// One lane per env: the packed row words of a board are its cells in row-major
// order (rows never straddle a word), so "k-th valid cell" is the k-th set bit
// across the NW words of ~revealed (& ~mine). A wave covers 64 boards with
// coalesced 16-B word loads, and the whole launch is a single load round trip
// plus ~100 lane-local instructions.
__device__ __forceinline__ int select_bit64(uint64_t x, uint32_t k) {  // k-th set bit, k < popc(x)
  int pos = 0;
#pragma unroll
  for (int half = 32; half >= 1; half >>= 1) {
    const uint64_t lowmask = (1ull << half) - 1ull;
    const uint32_t c = (uint32_t)__popcll(x & lowmask);
    if (k >= c) {
      k -= c;
      x >>= half;
      pos += half;
    }
  }
  return pos;
}

__device__ __forceinline__ int select_bit32(uint32_t x, uint32_t k) {  // k-th set bit, k < popc(x)
  int pos = 0;
#pragma unroll
  for (int half = 16; half >= 1; half >>= 1) {
    const uint32_t c = (uint32_t)__popc(x & ((1u << half) - 1u));
    if (k >= c) {
      k -= c;
      x >>= half;
      pos += half;
    }
  }
  return pos;
}

// x mod c for c <= 65535 in 32-bit arithmetic (a 64-bit remainder is a long
// software sequence on the GPU): x = hi * 2^32 + lo, 2^32 mod c = (2^32 - c) mod c
__device__ __forceinline__ uint32_t mod64_small(uint64_t x, uint32_t c) {
  const uint32_t hi = (uint32_t)(x >> 32), lo = (uint32_t)x;
  const uint32_t r = ((hi % c) * ((0u - c) % c)) % c;  // < c^2 < 2^32
  return (r + lo % c) % c;                              // < 2c
}

// The launch is one short dependency chain per lane (a load round trip, ~100 ALU
// instructions), so its time is latency: one-wave workgroups spread the waves over
// as many CUs as possible, the board words are loaded once (16-B loads) and kept in
// registers, and the remainder is 32-bit.
template <int H_, int W_>
__global__ __launch_bounds__(64) void k_tape(const uint64_t* mw, const uint64_t* rw, int64_t n, int H_rt, int W_rt,
                                             int64_t env_begin, uint64_t t, int mode, int64_t* actions) {
  const int64_t env = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (env >= n) return;
  const Geo<H_, W_> g(H_rt, W_rt);
  const int W = g.W, rpw = g.RPW(), NW = g.NW();
  constexpr int kNW = (H_ && W_) ? (H_ + (64 / W_) - 1) / (64 / W_) : 64;
  constexpr bool kStatic = H_ && W_;
  const bool safe_mode = mode == MS_TAPE_SAFE_BIASED;
  const uint64_t* rp = rw + env * NW;
  const uint64_t* mp = mw + env * NW;
  auto valid_mask = [&](int w) -> uint64_t {
    const int rows = min(rpw, g.H - w * rpw);
    const int bits = rows * W;
    return bits >= 64 ? ~0ull : ((1ull << bits) - 1ull);
  };
  uint64_t vw[kStatic ? kNW : 1], sw[kStatic ? kNW : 1];
  uint32_t n_valid = 0, n_safe = 0;
  if constexpr (kStatic) {
    // all loads first: the words of a board are contiguous (NW * 8 bytes)
    uint64_t rr[kNW], mm[kNW];
#pragma unroll
    for (int w = 0; w < kNW; ++w) rr[w] = rp[w];
    if (safe_mode) {
#pragma unroll
      for (int w = 0; w < kNW; ++w) mm[w] = mp[w];
    }
#pragma unroll
    for (int w = 0; w < kNW; ++w) {
      vw[w] = ~rr[w] & valid_mask(w);
      n_valid += (uint32_t)__popcll(vw[w]);
      sw[w] = safe_mode ? (vw[w] & ~mm[w]) : 0ull;
      n_safe += (uint32_t)__popcll(sw[w]);
    }
  } else {
    for (int w = 0; w < NW; ++w) {
      const uint64_t v = ~rp[w] & valid_mask(w);
      n_valid += (uint32_t)__popcll(v);
      if (safe_mode) n_safe += (uint32_t)__popcll(v & ~mp[w]);
    }
  }
  const uint64_t gidx = (uint64_t)(env_begin + env);
  const uint64_t x = splitmix64(0xC0FFEEull ^ (gidx << 32) ^ t);
  const bool want_safe = safe_mode && (x & 0xFFFFull) < 65208ull && n_safe > 0;
  const uint32_t cnt = want_safe ? n_safe : n_valid;
  const uint64_t sel = safe_mode ? (x >> 16) : x;
  int64_t act = 0;
  if (cnt > 0) {
    uint32_t target = mod64_small(sel, cnt);
    if constexpr (kStatic) {
#pragma unroll
      for (int w = 0; w < kNW; ++w) {
        if (target != 0xFFFFFFFFu) {
          const uint64_t b = want_safe ? sw[w] : vw[w];
          const uint32_t pc = (uint32_t)__popcll(b);
          if (target < pc) {
            const int pos = select_bit64(b, target);
            const int r = w * rpw + pos / W;
            act = (int64_t)r * W + (pos - (pos / W) * W);
            target = 0xFFFFFFFFu;  // found
          } else {
            target -= pc;
          }
        }
      }
    } else {
      for (int w = 0; w < NW && target != 0xFFFFFFFFu; ++w) {
        uint64_t b = ~rp[w] & valid_mask(w);
        if (want_safe) b &= ~mp[w];
        const uint32_t pc = (uint32_t)__popcll(b);
        if (target < pc) {
          const int pos = select_bit64(b, target);
          const int r = w * rpw + pos / W;
          act = (int64_t)r * W + (pos - (pos / W) * W);
          target = 0xFFFFFFFFu;
        } else {
          target -= pc;
        }
      }
    }
  }
  actions[env] = act;
}

// ---------------------------------------------------------------------------
// Late-start resets (VecMinesweeper._apply_late_start, env.py:416-466).
// The reference draws every late start from ONE generator shared by all envs, in
// env order, and each env consumes a data-dependent number of draws, so the envs
// form a sequential chain: one wave walks them in order (each board's clicks are
// still wave-parallel: placement + flood fill as in k_step). Only envs flagged in
// `need` (the step's dones; all envs on ms_reset) are visited.
// ---------------------------------------------------------------------------
struct LateCfg {
  double prob;
  int32_t min_hidden, max_hidden, max_attempts, max_extra_steps;
};

// The late-start generator of the keyed mode (MS_LATE_KEYED): a PCG64 state built from
// (late seed, GLOBAL env index, the env's own PCG64 state at the reset) by splitmix64.
// The env's own state advances every episode (each episode places its mines), so every
// reset of every env has its own stream, independent of the world size and of the order
// in which envs reset. oracle/ms_oracle.c (keyed_late_rng) restates it.
__device__ __forceinline__ Pcg keyed_late_pcg(uint64_t seed, uint64_t gidx, uint64_t st_hi, uint64_t st_lo) {
  Pcg L;
  L.hi = splitmix64(seed ^ splitmix64(gidx ^ 0x6C8E9CF570932BD5ull));
  L.lo = splitmix64(L.hi ^ st_lo);
  L.ihi = splitmix64(L.lo ^ st_hi);
  L.ilo = splitmix64(L.ihi ^ 0xA0761D6478BD642Full) | 1ull;
  L.has32 = 0u;
  L.uinteger = 0u;
  return L;
}

// An env's state as late_env reads it: its rows in lanes and its meta (wave-uniform). k_late
// loads the next env's state before running the current one, so the load round trip of a
// reset overlaps the previous reset's clicks instead of heading the serial chain.
struct LateState {
  uint64_t mine, rev;
  uint64_t st_hi, st_lo, inc_hi, inc_lo;
  uint32_t has32, uinteger, step_count, flags;
};

template <int H_, int W_>
__device__ __forceinline__ LateState late_load(const KParams& p, int64_t env, const Geo<H_, W_>& g, int lane) {
  const int NW = g.NW();
  const EnvMeta* mp = p.meta + env;
  LateState s;
  s.mine = load_row(p.mine_words + env * NW, g, lane);
  s.rev = load_row(p.rev_words + env * NW, g, lane);
  s.st_hi = rfl64(mp->st_hi);
  s.st_lo = rfl64(mp->st_lo);
  s.inc_hi = rfl64(mp->inc_hi);
  s.inc_lo = rfl64(mp->inc_lo);
  s.has32 = rfl(mp->has32);
  s.uinteger = rfl(mp->uinteger);
  s.step_count = rfl((uint32_t)mp->step_count);
  s.flags = rfl(mp->flags);
  return s;
}

// The late-start generator of the shared mode as a jump-ahead batch: lane i holds output i + 1 of
// the batch (and the state after it), computed from the batch's base state with the handle's
// jump table, so a draw is a readlane instead of a serial 128-bit PCG step (~45 scalar
// instructions) on the critical chain. The buffered half-word (has32 / uinteger) follows
// numpy's next_uint32 as in pcg_next32. lr_state() is the PCG64 state after the last consumed
// output. The keyed mode keeps a plain Pcg (one reset per wave: nothing to batch).
struct LateRng {
  Pcg base;           // state before the batch; inc, has32 / uinteger are the generator's own
  uint32_t xlo, xhi;  // lane i: output i + 1 of the batch
  uint64_t sh, sl;    // lane i: the state after it
  int used;           // outputs of the batch consumed (uniform)
};
__device__ __forceinline__ void lr_fill(LateRng& R, const uint64_t (&J)[4]) {
  const uint64_t ci_lo = J[3] * R.base.ilo;
  const uint64_t ci_hi = __umul64hi(J[3], R.base.ilo) + J[3] * R.base.ihi + J[2] * R.base.ilo;
  const Out o = jump_out(R.base.hi, R.base.lo, J[0], J[1], ci_hi, ci_lo);
  R.sh = o.sh;
  R.sl = o.sl;
  R.xlo = (uint32_t)o.x;
  R.xhi = (uint32_t)(o.x >> 32);
  R.used = 0;
}
__device__ __forceinline__ uint64_t lr_next64(LateRng& R, const uint64_t (&J)[4]) {
  if (R.used == kWave) {
    R.base.hi = readlane64(R.sh, kWave - 1);
    R.base.lo = readlane64(R.sl, kWave - 1);
    lr_fill(R, J);
  }
  const int u = R.used++;
  return ((uint64_t)readlane32(R.xhi, u) << 32) | readlane32(R.xlo, u);
}
__device__ __forceinline__ uint64_t lr_next64(Pcg& L, const uint64_t (&J)[4]) {
  (void)J;
  return pcg_next64(L);
}
__device__ __forceinline__ uint32_t lr_next32(LateRng& R, const uint64_t (&J)[4]) {
  if (R.base.has32) {
    R.base.has32 = 0;
    return R.base.uinteger;
  }
  const uint64_t x = lr_next64(R, J);
  R.base.has32 = 1;
  R.base.uinteger = (uint32_t)(x >> 32);
  return (uint32_t)x;
}
// random_bounded_uint64(0, j), numpy's buffered Lemire (as pcg_bounded)
__device__ __forceinline__ uint32_t lr_bounded(LateRng& R, const uint64_t (&J)[4], uint32_t j) {
  if (j == 0) return 0;
  const uint32_t excl = j + 1u;
  uint64_t m = (uint64_t)lr_next32(R, J) * excl;
  uint32_t left = (uint32_t)m;
  if (left < excl) {
    const uint32_t thr = (0xffffffffu - j) % excl;
    while (left < thr) {
      m = (uint64_t)lr_next32(R, J) * excl;
      left = (uint32_t)m;
    }
  }
  return (uint32_t)(m >> 32);
}
__device__ __forceinline__ uint32_t lr_bounded(Pcg& L, const uint64_t (&J)[4], uint32_t j) {
  (void)J;
  return pcg_bounded(L, j);
}
__device__ __forceinline__ Pcg lr_state(const LateRng& R) {
  Pcg P = R.base;
  if (R.used > 0) {
    P.hi = readlane64(R.sh, R.used - 1);
    P.lo = readlane64(R.sl, R.used - 1);
  }
  return P;
}

// MS_DIAG builds: k_late's cycle accounting (tools/late_diag.py), summed over the launch in dacc:
// [0] whole launch, [1] envs visited, [2] late starts, [3] envs without a late start (draw + stores
// + emit), [4] first clicks (placement included), [5] extra-click loops, [6] extra clicks,
// [7] of them flood fills, [8] flood iterations, [9] late envs' stores + emit, [10] attempts,
// [14] cycles of flood fills (dilation + list rebuild), [15] cycles of flood clicks before the fill
#ifdef MS_DIAG
#define LSTAMP(k)                                          \
  do {                                                     \
    if (dacc) {                                            \
      const uint64_t t_ = __builtin_amdgcn_s_memtime();    \
      dacc[(k)] += t_ - tl_;                               \
      tl_ = t_;                                            \
    }                                                      \
  } while (0)
#define LCOUNT(k, v)            \
  do {                          \
    if (dacc) dacc[(k)] += (v); \
  } while (0)
#else
#define LSTAMP(k) do { } while (0)
#define LCOUNT(k, v) do { } while (0)
#endif


template <int H_, int W_, class Rng>
__device__ __forceinline__ void late_env(const KParams& p, Rng& L, const LateCfg& lc, int64_t env,
                                         const LateState& st, const uint64_t (&J)[4], uint64_t* sR, uint64_t* sM,
                                         uint32_t* sTab, const Geo<H_, W_>& g, int lane, uint64_t* dacc = nullptr) {
  (void)dacc;
#ifdef MS_DIAG
  uint64_t tl_ = __builtin_amdgcn_s_memtime();
  LCOUNT(1, 1);
#endif
  bool late = false;
  const int H = g.H, A = g.A(), NW = g.NW();
  const uint64_t rowmask = g.rowmask();
  const int safe_total = A - p.K;
  EnvMeta* mp = p.meta + env;
  uint64_t* mwords = p.mine_words + env * NW;
  uint64_t* rwords = p.rev_words + env * NW;
  uint64_t mine = st.mine;
  uint64_t rev = st.rev;
  Pcg rng;
  rng.hi = st.st_hi;
  rng.lo = st.st_lo;
  rng.ihi = st.inc_hi;
  rng.ilo = st.inc_lo;
  rng.has32 = st.has32;
  rng.uinteger = st.uinteger;
  int32_t step_count = (int32_t)st.step_count;
  bool fc = (st.flags & 1u) != 0;
  // prob <= 0 short-circuits before the draw (env.py:421)
  if (lc.prob > 0.0 && (double)(lr_next64(L, J) >> 11) * 0x1.0p-53 < lc.prob) {
    late = true;
    LCOUNT(2, 1);
    bool success = false;
    for (int att = 0; att < lc.max_attempts && !success; ++att) {
      LCOUNT(10, 1);
      if (fc) {  // env.reset() (env.py:87-101): the env's own RNG continues
        mine = 0ull;
        rev = 0ull;
        fc = false;
        step_count = 0;
      }
      const int first = (int)lr_bounded(L, J, (uint32_t)(A - 1));
      bool done, mc = false;
      int oc;
      uint32_t nw, tr;
      board_click(rng, mine, rev, fc, first, p, J, sTab, sR, g, lane, done, oc, nw, tr, mc);
      step_count += 1;
      LSTAMP(4);
      if (done) continue;
      int target = lc.min_hidden + (int)lr_bounded(L, J, (uint32_t)(lc.max_hidden - lc.min_hidden));
      target = target < safe_total ? target : safe_total;
      target = target > 1 ? target : 1;
      int revealed = (int)tr;
      // The extra clicks hit safe unrevealed cells of a placed board (the candidates are
      // ~mine & ~revealed, flags are never set), so each is MinesweeperEnv.step's reveal branch
      // alone: the candidates number safe_total - revealed (no count reduction), a cell with
      // adjacent mines reveals just itself (no flood-fill fixpoint), and the step ends the
      // episode only by a win. The mines are fixed now: their zero-cell map is built once.
      const uint64_t Um = wave_shr1(mine) | wave_shl1(mine);
      const uint64_t zero = ~(Um | (Um << 1) | (Um >> 1) | (mine << 1) | (mine >> 1)) & rowmask;
      // Compile-time boards of <= 256 cells (<= 32 columns, <= 16 rows) keep the candidates
      // (np.flatnonzero order) as a list in lane registers, four cell indices per lane (byte j of
      // lane l = entry 4l + j): the k-th is one readlane, and a numbered cell leaves the list by a
      // one-entry shift; the list is rebuilt from the rows after a flood fill.
      constexpr bool kList = H_ && W_ && H_ <= 16 && W_ <= 32 && H_ * W_ <= 256;
      uint32_t lword = 0u;
      auto build_list = [&]() {
        uint8_t* lst = reinterpret_cast<uint8_t*>(sTab);
        const uint32_t b = (uint32_t)(~mine & ~rev & (lane < H ? rowmask : 0ull));
        const uint32_t i0 = row_excl_scan16((uint32_t)__popc(b));
        // every column at once (predicated byte stores; a clear-lowest-bit loop is a serial,
        // divergent chain of the lone wave): cell j of the row goes to i0 + (candidates before it)
#pragma unroll
        for (int j = 0; j < W_; ++j)
          if ((b >> j) & 1u) lst[i0 + (uint32_t)__popc(b & ((1u << j) - 1u))] = (uint8_t)(lane * W_ + j);
        wave_sync();
        lword = reinterpret_cast<const uint32_t*>(lst)[lane];
        wave_sync();
      };
      if constexpr (kList) build_list();
      for (int k = 0; k < lc.max_extra_steps; ++k) {
        if (safe_total - revealed <= target) {
          success = true;
          break;
        }
        const uint32_t cnt = (uint32_t)(safe_total - revealed);
#ifdef MS_DIAG
        const uint64_t ts_ = __builtin_amdgcn_s_memtime();
#endif
        const uint32_t kk = lr_bounded(L, J, cnt - 1u);  // rng.choice(flatnonzero(...)) (row-major)
        LCOUNT(6, 1);
        int src, col;
        if constexpr (kList) {
          const int cell = (int)((readlane32(lword, (int)(kk >> 2)) >> (8u * (kk & 3u))) & 0xffu);
          src = cell / W_;
          col = cell - src * W_;
        } else {
          const uint64_t cand = ~mine & ~rev & (lane < H ? rowmask : 0ull);
          const uint32_t pc = (uint32_t)__popcll(cand);
          const uint32_t before = wave_excl_scan(pc);
          const bool mine_lane = kk >= before && kk < before + pc;
          const uint64_t who = __ballot(mine_lane);
          src = __ffsll((unsigned long long)who) - 1;
          // the k-th candidate of the row by a popcount bisection (a clear-lowest-bit loop cost
          // ~2x the whole click: tools/late_diag.py)
          const int sel = (W_ && W_ <= 32) ? select_bit32((uint32_t)cand, kk - before) : select_bit64(cand, kk - before);
          col = (int)readlane32((uint32_t)(mine_lane ? sel : 0), src);
        }
        if (((readlane64(zero, src) >> col) & 1ull) == 0ull) {
          if (lane == src) rev |= 1ull << col;
          revealed += 1;
          if constexpr (kList) {  // entry kk leaves the list: the entries after it move down one
            const uint32_t nxt = dpp32<0x130>(lword);  // lane l <- lane l + 1 (wave_shl:1)
            const uint32_t shifted = (lword >> 8) | (nxt << 24);
            const int lk = (int)(kk >> 2);
            const uint32_t keep = lane < lk ? 0xffffffffu : (lane == lk ? (1u << (8u * (kk & 3u))) - 1u : 0u);
            lword = (lword & keep) | (shifted & ~keep);
          }
        } else {  // flood_fill_reveal (env_numba.py:17-77) from a zero cell, as board_click
#ifdef MS_DIAG
          const uint64_t tf_ = __builtin_amdgcn_s_memtime();
          LCOUNT(15, tf_ - ts_);
#endif
          const uint64_t allow = ~mine & ~rev & (lane < H ? rowmask : 0ull);
          uint64_t Fr = (lane == src) ? (1ull << col) : 0ull;
          LCOUNT(7, 1);
          while (true) {
            LCOUNT(8, 1);
            const uint64_t S = Fr & zero;
            const uint64_t Dh = S | (S << 1) | (S >> 1);
            const uint64_t Dv = Dh | wave_shr1(Dh) | wave_shl1(Dh);
            const uint64_t Fn = Fr | (Dv & allow);
            const bool changed = __ballot(Fn != Fr) != 0ull;
            Fr = Fn;
            if (!changed) break;
          }
          rev |= Fr;
          revealed += (int)wave_sum((uint32_t)__popcll(Fr));
          if constexpr (kList) build_list();
#ifdef MS_DIAG
          LCOUNT(14, __builtin_amdgcn_s_memtime() - tf_);
#endif
        }
        step_count += 1;
        done = revealed >= safe_total;  // a win (env.py:133-140)
        if (done) break;
      }
      if (!success && !done && safe_total - revealed <= target) success = true;
      LSTAMP(5);
    }
    if (!success) {  // fallback: leave the board fresh (env.py:465-466)
      mine = 0ull;
      rev = 0ull;
      fc = false;
      step_count = 0;
    }
  }
  if (!late) {  // no late start: board, meta and obs are what the step (or ms_reset) just wrote
    LSTAMP(3);
    return;
  }
  if (lane == 0) {
    mp->st_hi = rng.hi;
    mp->st_lo = rng.lo;
    mp->has32 = rng.has32;
    mp->uinteger = rng.uinteger;
    mp->step_count = step_count;
    mp->flags = fc ? 1u : 0u;
  }
  store_rows(mwords, mine, sR, g, lane);
  store_rows(rwords, rev, sR, g, lane);
  __syncthreads();
  if (p.obs || p.mask || p.codes) {
    stage_rows(sR, sM, rev, mine, g, lane);
    emit_obs(p.obs ? p.obs + env * 10 * A : nullptr, p.mask ? p.mask + env * A : nullptr,
             p.codes ? p.codes + env * A : nullptr, sR, sM, fc, g, lane, reinterpret_cast<uint8_t*>(sTab));
  }
  __syncthreads();
  LSTAMP(9);
}

__device__ __forceinline__ void load_jump(const uint64_t* jump, int lane, uint64_t (&J)[4]) {
  const ulonglong2* e = reinterpret_cast<const ulonglong2*>(jump + 4 * lane);
  const ulonglong2 a0 = e[0], a1 = e[1];
  J[0] = a0.x;
  J[1] = a0.y;
  J[2] = a1.x;
  J[3] = a1.y;
}

// MS_LATE_SHARED (the reference): one wave walks the envs in order with the shared generator.
template <int H_, int W_>
__global__ __launch_bounds__(64) void k_late(KParams p, Pcg* lstate, LateCfg lc, const uint8_t* need) {
  __shared__ uint64_t sR[kWave];
  __shared__ uint64_t sM[kWave + 2];
  __shared__ uint32_t sTab[(H_ && W_) ? H_ * W_ : kMaxH * kMaxW];
  const int lane = lane_id();
  const Geo<H_, W_> g(p.H, p.W);
  LateRng L;
  L.base.hi = lstate->hi;
  L.base.lo = lstate->lo;
  L.base.ihi = lstate->ihi;
  L.base.ilo = lstate->ilo;
  L.base.has32 = lstate->has32;
  L.base.uinteger = lstate->uinteger;
  uint64_t J[4];
  load_jump(p.jump, lane, J);
  lr_fill(L, J);
  // the flags of 64 envs per load and ballot (one dependent scalar load per env cost ~0.5 us each);
  // the next env's state is loaded before the current env runs
  int64_t base = -kWave;
  uint64_t todo = 0ull;
  auto next_env = [&]() -> int64_t {
    while (todo == 0ull) {
      base += kWave;
      if (base >= p.n) return -1;
      const int64_t e = base + lane;
      todo = __ballot(e < p.n && (!need || need[e]));
    }
    const int l = __ffsll((unsigned long long)todo) - 1;
    todo &= todo - 1ull;
    return base + l;
  };
  uint64_t* dacc = nullptr;
#ifdef MS_DIAG
  uint64_t dv[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (p.diag) dacc = dv;
  const uint64_t t_begin = __builtin_amdgcn_s_memtime();
#endif
  int64_t cur = next_env();
  LateState sc = {};
  if (cur >= 0) sc = late_load(p, cur, g, lane);
  while (cur >= 0) {
    const int64_t nxt = next_env();
    LateState sn = sc;
    if (nxt >= 0) sn = late_load(p, nxt, g, lane);
    late_env(p, L, lc, cur, sc, J, sR, sM, sTab, g, lane, dacc);
    cur = nxt;
    sc = sn;
  }
#ifdef MS_DIAG
  if (dacc) {
    dv[0] = __builtin_amdgcn_s_memtime() - t_begin;
    if (lane == 0)
      for (int k = 0; k < 16; ++k) p.diag[k] = dv[k];
  }
#endif
  const Pcg Lf = lr_state(L);
  if (lane == 0) {
    lstate->hi = Lf.hi;
    lstate->lo = Lf.lo;
    lstate->has32 = Lf.has32;
    lstate->uinteger = Lf.uinteger;
  }
}

// MS_LATE_KEYED: one wave per env, every resetting env at once, each with its own
// keyed generator (keyed_late_pcg).
template <int H_, int W_>
__global__ __launch_bounds__(64) void k_late_keyed(KParams p, LateCfg lc, uint64_t seed, int64_t env_begin,
                                                   const uint8_t* need) {
  __shared__ uint64_t sR[kWave];
  __shared__ uint64_t sM[kWave + 2];
  __shared__ uint32_t sTab[(H_ && W_) ? H_ * W_ : kMaxH * kMaxW];
  const int64_t env = blockIdx.x;
  if (need && !need[env]) return;  // (uniform: one wave per workgroup)
  const int lane = lane_id();
  const Geo<H_, W_> g(p.H, p.W);
  uint64_t J[4];
  load_jump(p.jump, lane, J);
  const EnvMeta* mp = p.meta + env;
  Pcg L = keyed_late_pcg(seed, (uint64_t)(env_begin + env), rfl64(mp->st_hi), rfl64(mp->st_lo));
  late_env(p, L, lc, env, late_load(p, env, g, lane), J, sR, sM, sTab, g, lane);
}

// ---------------------------------------------------------------------------
// ms_run_tape: T consecutive (ms_tape_actions, ms_step) pairs in ONE launch.
// A wave keeps its board in registers (rows in lanes, the PCG64 state in SGPRs)
// for all T steps: per step it picks the tape action from the current board (the
// rule of k_tape, evaluated wave-parallel: DPP sums, an exclusive scan and a
// k-th-set-bit select), applies board_click, writes every output of the step,
// auto-resets, and goes on. Meta and rows are read once and written once. With no
// launch boundary between steps the waves drift apart, so one wave's obs stores
// overlap another's flood fill. Bit-exact with the two-call sequence.
// ---------------------------------------------------------------------------
struct RunParams {
  uint64_t t0;
  int32_t T, mode, slots;
  int64_t env_begin;
  int64_t* actions;  // optional: the action of each step
};

template <int H_, int W_>
__device__ __forceinline__ int tape_cell(uint64_t mine, uint64_t rev, const Geo<H_, W_>& g, int lane,
                                         uint64_t gidx, uint64_t t, int mode) {
  const uint64_t valid = ~rev & g.rowmask() & (lane < g.H ? ~0ull : 0ull);
  const uint64_t x = splitmix64(0xC0FFEEull ^ (gidx << 32) ^ t);
  uint64_t bits = valid;
  uint32_t cnt = wave_sum((uint32_t)__popcll(valid));
  uint64_t sel = x;
  if (mode == MS_TAPE_SAFE_BIASED) {  // (uniform branch: mode is a kernel argument)
    const uint64_t safe = valid & ~mine;
    const uint32_t n_safe = wave_sum((uint32_t)__popcll(safe));
    sel = x >> 16;
    if ((x & 0xFFFFull) < 65208ull && n_safe > 0) {
      bits = safe;
      cnt = n_safe;
    }
  }
  if (cnt == 0) return 0;
  const uint32_t target = mod64_small(sel, cnt);
  const uint32_t pc = (uint32_t)__popcll(bits);
  const uint32_t before = wave_excl_scan(pc);
  const bool hit = target >= before && target < before + pc;
  const uint64_t who = __ballot(hit);
  const int src = __ffsll((unsigned long long)who) - 1;
  const int col = (int)readlane32((uint32_t)(hit ? select_bit64(bits, target - before) : 0), src);
  return src * g.W + col;
}

template <int H_, int W_, int EPW>
__global__ __launch_bounds__(64 * EPW) void k_run(KParams p, RunParams r) {
  __shared__ uint64_t sR_all[EPW][kWave];
  __shared__ uint64_t sM_all[EPW][kWave + 2];
  __shared__ uint32_t sTab_all[EPW][(H_ && W_) ? H_ * W_ : kMaxH * kMaxW];
  const int lane = lane_id();
  const int wv = (EPW == 1) ? 0 : (int)rfl(threadIdx.x >> 6);
  const int64_t env = (int64_t)blockIdx.x * EPW + wv;
  if (env >= p.n) return;
  uint64_t* sR = sR_all[wv];
  uint64_t* sM = sM_all[wv];
  uint32_t* sTab = sTab_all[wv];
  const Geo<H_, W_> g(p.H, p.W);
  const int A = g.A(), NW = g.NW();
  EnvMeta* mp = p.meta + env;
  uint64_t* mwords = p.mine_words + env * NW;
  uint64_t* rwords = p.rev_words + env * NW;
  uint64_t mine = load_row(mwords, g, lane);
  uint64_t rev = load_row(rwords, g, lane);
  uint64_t J[4] = {0ull, 0ull, 0ull, 0ull};
  if (lane < p.K) {
    const ulonglong2* e = reinterpret_cast<const ulonglong2*>(p.jump + 4 * lane);
    const ulonglong2 a0 = e[0], a1 = e[1];
    J[0] = a0.x;
    J[1] = a0.y;
    J[2] = a1.x;
    J[3] = a1.y;
  }
  Pcg rng;
  rng.hi = rfl64(mp->st_hi);
  rng.lo = rfl64(mp->st_lo);
  rng.ihi = rfl64(mp->inc_hi);
  rng.ilo = rfl64(mp->inc_lo);
  rng.has32 = rfl(mp->has32);
  rng.uinteger = rfl(mp->uinteger);
  int32_t step_count = (int32_t)rfl((uint32_t)mp->step_count);
  bool fc = (rfl(mp->flags) & 1u) != 0;
  const uint64_t gidx = (uint64_t)(r.env_begin + env);
  const int64_t n = p.n;
  for (int t = 0; t < r.T; ++t) {
    const int64_t slot = (r.slots ? (int64_t)t * n : 0) + env;
    const int cell = tape_cell(mine, rev, g, lane, gidx, r.t0 + (uint64_t)t, r.mode);
    double reward = 0.0;
    bool done = false;
    int outcome = MS_OUTCOME_NONE;
    uint32_t newly = 0, total_rev = 0;
    bool mines_changed = false;
    board_click(rng, mine, rev, fc, cell, p, J, sTab, sR, g, lane, done, outcome, newly, total_rev, mines_changed);
    if (outcome == MS_OUTCOME_LOSS) reward += p.loss_reward;
    if (outcome == MS_OUTCOME_WIN) reward += p.win_reward;
    reward -= p.step_penalty;
    step_count += 1;
    if (r.actions && lane == 0) r.actions[slot] = cell;
    store_aux(p, slot, lane, reward, done, step_count, newly, total_rev, outcome, A);
    if (done) {  // auto-reset; the RNG continues
      mine = 0ull;
      rev = 0ull;
      fc = false;
      step_count = 0;
    }
    if (p.obs || p.mask) {
      stage_rows(sR, sM, rev, mine, g, lane);
      emit_obs(p.obs ? p.obs + slot * 10 * A : nullptr, p.mask ? p.mask + slot * A : nullptr, nullptr, sR, sM, fc, g, lane,
               reinterpret_cast<uint8_t*>(sTab));
    }
    wave_sync();  // this step's LDS reads before the next step's placement / staging writes
  }
  store_meta(mp, rng, step_count, fc, lane);
  store_rows(mwords, mine, sR, g, lane);
  store_rows(rwords, rev, sR, g, lane);
}

// ms_run_tape on packed boards: k_run's T (tape, step) pairs per launch with k_step_packed's
// layout (four boards per wave). The synthetic policy's k-th valid cell is found per board:
// board sums and a DPP row scan over the board's 16 lanes, the board's bits of one ballot.
__device__ __forceinline__ uint32_t row_excl_scan(uint32_t v) {  // inside one 16-lane DPP row
  uint32_t s = v;
  s += dpp32<0x111>(s);
  s += dpp32<0x112>(s);
  s += dpp32<0x114>(s);
  s += dpp32<0x118>(s);
  return s - v;
}

template <int H_, int W_, int LPB>
__device__ __forceinline__ int pk_tape_cell(uint32_t mine, uint32_t rev, int lane, uint64_t gidx, uint64_t t, int mode) {
  constexpr uint32_t ROWMASK = (1u << W_) - 1u;
  constexpr uint64_t BM = (1ull << LPB) - 1ull;
  const int r = lane & (LPB - 1);
  const uint32_t valid = ~rev & ROWMASK & (r < H_ ? ~0u : 0u);
  const uint64_t x = splitmix64(0xC0FFEEull ^ (gidx << 32) ^ t);
  uint32_t bits = valid;
  uint32_t cnt = board_sum<LPB>((uint32_t)__popc(valid), lane);
  uint64_t sel = x;
  if (mode == MS_TAPE_SAFE_BIASED) {  // (uniform branch: mode is a kernel argument)
    const uint32_t safe = valid & ~mine;
    const uint32_t n_safe = board_sum<LPB>((uint32_t)__popc(safe), lane);
    sel = x >> 16;
    if ((x & 0xFFFFull) < 65208ull && n_safe > 0) {
      bits = safe;
      cnt = n_safe;
    }
  }
  const uint32_t target = mod64_small(sel, cnt ? cnt : 1u);
  const uint32_t pc = (uint32_t)__popc(bits);
  const uint32_t before = row_excl_scan(pc);
  const bool hit = target >= before && target < before + pc;
  const uint64_t who = (__ballot(hit) >> board_base<LPB>(lane)) & BM;
  const int src = who ? __ffsll((unsigned long long)who) - 1 : 0;
  const int col = (int)board_read<LPB>(hit ? (uint32_t)select_bit64(bits, target - before) : 0u, lane, src);
  return cnt ? src * W_ + col : 0;
}

template <int H_, int W_, int WPG, int BPW>
__global__ __launch_bounds__(64 * WPG) void k_run_packed(KParams p, RunParams rp) {
  constexpr int LPB = kWave / BPW;
  constexpr bool BIG = packable16<H_, W_>();  // 16x16: place_packed3 + pk_emit16
  static_assert(BPW == 2 || BPW == 4, "boards per wave");
  static_assert(packable<H_, W_>() || (BIG && BPW == 4), "packed board shape");
  constexpr int A = H_ * W_;
  constexpr int RPW = 64 / W_;
  constexpr int NW = (H_ + RPW - 1) / RPW;
  using Lds = std::conditional_t<BIG, PackedLds16<H_, W_, BPW>, PackedLds<H_, W_, BPW>>;
  __shared__ Lds S_all[WPG];
  const int lane = lane_id();
  const int r = lane & (LPB - 1);
  const int wv = (WPG == 1) ? 0 : (int)rfl(threadIdx.x >> 6);
  Lds& S = S_all[wv];
  uint32_t* scr;
  if constexpr (BIG) scr = S.scr;
  else scr = S.row;
  const int64_t env0 = ((int64_t)blockIdx.x * WPG + wv) * BPW;
  if (env0 >= p.n) return;  // (wave-uniform)
  const int64_t env_raw = env0 + (lane / LPB);
  const bool live = env_raw < p.n;
  const int64_t env = live ? env_raw : p.n - 1;
  uint32_t mine, rev;
  uint64_t J[4];
  Pcg rng;
  int32_t step_count;
  bool fc;
  pk_load<H_, W_>(p, env, r, mine, rev, J, rng, step_count, fc);
  const uint64_t gidx = (uint64_t)(rp.env_begin + env);
  const int64_t n = p.n;
  const int nbl = (n - env0 < BPW) ? (int)(n - env0) : BPW;
  for (int t = 0; t < rp.T; ++t) {
    const int64_t sbase = rp.slots ? (int64_t)t * n : 0;
    const int cell = pk_tape_cell<H_, W_, LPB>(mine, rev, lane, gidx, rp.t0 + (uint64_t)t, rp.mode);
    bool done, mines_changed = false, cell_rev;
    int outcome;
    uint32_t newly, total_rev;
    pk_click<H_, W_, LPB>(p, rng, mine, rev, fc, cell, J, scr, lane, nullptr, done, outcome, newly, total_rev,
                          mines_changed, cell_rev);
    double reward = 0.0;
    if (outcome == MS_OUTCOME_LOSS) reward += p.loss_reward;
    if (outcome == MS_OUTCOME_WIN) reward += p.win_reward;
    reward -= p.step_penalty;
    step_count += 1;
    if (rp.actions && live && r == 0) rp.actions[sbase + env] = cell;
    store_aux(p, sbase + env, live ? r : kWave, reward, done, step_count, newly, total_rev, outcome, A);
    if (done) {  // auto-reset; the RNG continues
      mine = 0u;
      rev = 0u;
      fc = false;
      step_count = 0;
    }
    if constexpr (BIG) {
      if (p.obs || p.mask)
        pk_emit16<H_, W_, BPW>(p.obs ? p.obs + (sbase + env0) * 10 * A : nullptr,
                               p.mask ? p.mask + (sbase + env0) * A : nullptr, nbl, mine, rev, fc, lane);
    } else {
      if (p.obs || p.mask)
        pk_emit<H_, W_, BPW, LPB>(p.obs ? p.obs + (sbase + env0) * 10 * A : nullptr,
                                  p.mask ? p.mask + (sbase + env0) * A : nullptr, nbl, mine, rev, fc, S, lane, nullptr);
    }
    wave_sync();  // this step's LDS reads before the next step's placement / image writes
  }
  pk_store_state<H_, W_, BPW, LPB>(p.meta + env, p.mine_words + env * NW, p.rev_words + env * NW, rng, step_count, fc,
                                   mine, rev, true, live, S, lane);
}

// ---------------------------------------------------------------------------
// ms_gae: thread per env, reverse scan over T, reference f32 op order
// (buffers.py:87-94) with explicit round-to-nearest ops (no contraction).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gae(const float* __restrict__ rewards, const float* __restrict__ values,
                                             const uint8_t* __restrict__ dones, const float* __restrict__ last_values,
                                             int T, int64_t N, float gamma, float gl, float* __restrict__ adv,
                                             float* __restrict__ ret) {
#pragma clang fp contract(off)
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float last_adv = 0.f;
  float nv = last_values[n];
  for (int t = T - 1; t >= 0; --t) {
    const int64_t i = (int64_t)t * N + n;
    const float v = values[i];
    // plain operators under `fp contract(off)`: each op rounds to f32 (the
    // __f*_rn helpers are header functions compiled with contraction on)
    const float nnt = 1.0f - (dones[i] ? 1.0f : 0.0f);
    const float t1 = gamma * nv;
    const float t2 = t1 * nnt;
    const float t3 = rewards[i] + t2;
    const float delta = t3 - v;
    const float t4 = gl * nnt;
    const float t5 = t4 * last_adv;
    last_adv = delta + t5;
    adv[i] = last_adv;
    ret[i] = last_adv + v;
    nv = v;
  }
}

// ---------------------------------------------------------------------------
// ms_sample_masked: one wave per row; Gumbel-max over valid cells.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t counter, uint64_t row, uint64_t col) {
  const uint64_t h = splitmix64(seed ^ splitmix64(counter ^ splitmix64(row * 0x100000001B3ull + col)));
  // 24 random bits -> (0, 1)
  return ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

// ---------------------------------------------------------------------------
// ms_dropout_masks: Dropout2d channel masks keyed by GLOBAL sample index.
// out[b][i][c] = (u(seed', counter, rows[i], b*C + c) >= p) / (1 - p), so a
// sample draws the same masks whichever rank (or minibatch position) holds it.
// One thread per 4 output channels (float4 store).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_dropout(const int64_t* __restrict__ rows, int64_t N, int nblk, int C,
                                                 uint64_t seed, uint64_t counter, float p, float scale,
                                                 float* __restrict__ out) {
  const int C4 = C >> 2;
  const int64_t total = (int64_t)nblk * N * C4;
  const uint64_t s = splitmix64(seed ^ 0xD1B54A32D192ED03ull);  // domain-separated from k_sample
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int c4 = (int)(q % C4);
    const int64_t bi = q / C4;
    const int64_t i = bi % N;
    const int b = (int)(bi / N);
    const uint64_t row = (uint64_t)rows[i];
    float4 v;
    float* vp = &v.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float u = uniform01(s, counter, row, (uint64_t)(b * C + 4 * c4 + j));
      vp[j] = u >= p ? scale : 0.f;
    }
    reinterpret_cast<float4*>(out)[q] = v;
  }
}

__global__ __launch_bounds__(256) void k_sample(const float* __restrict__ logits, const uint8_t* __restrict__ mask,
                                                int64_t N, int A, int64_t row_begin, uint64_t seed,
                                                uint64_t counter, int64_t* __restrict__ actions,
                                                float* __restrict__ logp) {
  const int lane = lane_id();
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
  if (row >= N) return;
  const float* lr = logits + row * A;
  const uint8_t* mr = mask + row * A;
  int any = 0;
  for (int i = lane; i < A; i += kWave) any |= mr[i] ? 1 : 0;
  const bool all_valid = __ballot(any) == 0ull;  // train_rl.py:166-168
  float mx = -INFINITY;
  for (int i = lane; i < A; i += kWave)
    if (all_valid || mr[i]) mx = fmaxf(mx, lr[i]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
  float se = 0.f;
  float best = -INFINITY;
  int best_i = 0x7fffffff;
  for (int i = lane; i < A; i += kWave) {
    if (all_valid || mr[i]) {
      const float l = lr[i];
      se += expf(l - mx);
      const float u = uniform01(seed, counter, (uint64_t)(row_begin + row), (uint64_t)i);
      const float gk = l - logf(-logf(u));
      if (gk > best || (gk == best && i < best_i)) {
        best = gk;
        best_i = i;
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    se += __shfl_xor(se, off);
    const float ob = __shfl_xor(best, off);
    const int oi = __shfl_xor(best_i, off);
    if (ob > best || (ob == best && oi < best_i)) {
      best = ob;
      best_i = oi;
    }
  }
  if (lane == 0) {
    actions[row] = best_i;
    logp[row] = (lr[best_i] - mx) - logf(se);
  }
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
thread_local char g_err[512] = "";

int fail(int code, const char* fmt, const char* a = "", const char* b = "") {
  snprintf(g_err, sizeof g_err, fmt, a, b);
  return code;
}

int hip_fail(hipError_t e, const char* where) {
  return fail(MS_EHIP, "%s: %s", where, hipGetErrorString(e));
}

// numpy SeedSequence -> PCG64 seeding, host side (bit_generator.pyx / pcg64.c).
struct HostPcg {
  unsigned __int128 state, inc;
  int has32;
  uint32_t uinteger;
};

void host_seed(HostPcg& r, uint64_t seed) {
  uint32_t ent[2];
  int ne = 0;
  if (seed == 0) ent[ne++] = 0;
  while (seed) {
    ent[ne++] = (uint32_t)seed;
    seed >>= 32;
  }
  uint32_t hc = 0x43b0d7e5u;
  auto hashmix = [&hc](uint32_t v) {
    v ^= hc;
    hc *= 0x931e8875u;
    v *= hc;
    return v ^ (v >> 16);
  };
  auto mix = [](uint32_t x, uint32_t y) {
    uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;
    return r ^ (r >> 16);
  };
  uint32_t pool[4];
  for (int i = 0; i < 4; ++i) pool[i] = hashmix(i < ne ? ent[i] : 0u);
  for (int s = 0; s < 4; ++s)
    for (int d = 0; d < 4; ++d)
      if (s != d) pool[d] = mix(pool[d], hashmix(pool[s]));
  uint32_t w32[8];
  uint32_t hb = 0x8b51f9ddu;
  for (int i = 0; i < 8; ++i) {
    uint32_t v = pool[i & 3] ^ hb;
    hb *= 0x58f38dedu;
    v *= hb;
    w32[i] = v ^ (v >> 16);
  }
  uint64_t w[4];
  for (int i = 0; i < 4; ++i) w[i] = (uint64_t)w32[2 * i] | ((uint64_t)w32[2 * i + 1] << 32);
  const unsigned __int128 M = ((unsigned __int128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;
  const unsigned __int128 initstate = ((unsigned __int128)w[0] << 64) | w[1];
  const unsigned __int128 initseq = ((unsigned __int128)w[2] << 64) | w[3];
  r.inc = (initseq << 1) | 1u;
  r.state = 0;
  r.state = r.state * M + r.inc;
  r.state += initstate;
  r.state = r.state * M + r.inc;
  r.has32 = 0;
  r.uinteger = 0;
}

uint32_t host_next32(HostPcg& r) {
  if (r.has32) {
    r.has32 = 0;
    return r.uinteger;
  }
  const unsigned __int128 M = ((unsigned __int128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;
  r.state = r.state * M + r.inc;
  const uint64_t hi = (uint64_t)(r.state >> 64), lo = (uint64_t)r.state;
  const unsigned rot = (unsigned)(hi >> 58);
  const uint64_t v = hi ^ lo;
  const uint64_t x = (v >> rot) | (v << ((64u - rot) & 63u));
  r.has32 = 1;
  r.uinteger = (uint32_t)(x >> 32);
  return (uint32_t)x;
}

uint32_t host_bounded(HostPcg& r, uint32_t j) {
  if (j == 0) return 0;
  const uint32_t excl = j + 1u;
  uint64_t m = (uint64_t)host_next32(r) * excl;
  uint32_t left = (uint32_t)m;
  if (left < excl) {
    const uint32_t thr = (0xffffffffu - j) % excl;
    while (left < thr) {
      m = (uint64_t)host_next32(r) * excl;
      left = (uint32_t)m;
    }
  }
  return (uint32_t)(m >> 32);
}

}  // namespace

struct ms_handle {
  ms_cfg cfg;
  int64_t n_total, env_begin, n;
  int H, W, A, NW;
  int device;
  EnvMeta* meta;
  uint64_t* mine_words;
  uint64_t* rev_words;
  uint64_t* jump;  // [64][4] PCG64 jump-ahead table (device)
  uint64_t* diag;  // optional stamp buffer (MS_DIAG builds)
  uint32_t dbg_flags;
  int epw;         // boards per workgroup of k_step (4; generic shapes use 1)
  int late_on;     // ms_set_late_start called with prob > 0
  hipEvent_t ev_start, ev_stop;  // ms_set_timing_events (measurement only): stamp k_step / k_run
  LateCfg late;
  Pcg* late_rng;   // device: the shared late-start generator
  int late_mode;   // MS_LATE_SHARED (the reference's one generator) | MS_LATE_KEYED
  uint64_t late_seed;
};

namespace {

bool shape_ok(const ms_cfg* c) {
  return c->H >= 1 && c->H <= kMaxH && c->W >= 1 && c->W <= kMaxW && c->mine_count >= 0 &&
         c->mine_count < c->H * c->W;
}

// ev0/ev1 non-null (ms_set_timing_events): the dispatch itself stamps the events, so their
// difference is the kernel's execution time as the profiler sees it (no launch gap)
// 16x16 boards four to a wave from this many envs on: measured 2-4 % faster than the one-board
// kernel at 65,536, within +-3 % at 8,192-32,768 and 10 % slower at 4,096 (both store-bound at
// 32k+, the one-board kernel's 4x more waves hide latency better at 4k; profiles/r04/
// packed16_step.txt); MS_DBG_FORCE_PACKED takes the packed kernel at any count
constexpr int64_t kPack16MinEnvs = 65536;
// the multistep form (ms_run_tape), whose boards stay in registers across the launch's steps: the
// packed kernel measured 3 % faster at 4,096 envs, 3-12 % at 32,768 and ~10 % at 65,536 (a wash at
// 8,192; profiles/r04/packed16_run.txt), so it is taken at every env count
constexpr int64_t kPack16RunMinEnvs = 0;

template <int H_, int W_>
void launch_step(const KParams& p, int epw, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  if constexpr (packable16<H_, W_>()) {
    if (p.K >= 1 && p.K <= 48 &&
        !(p.dbg_flags & (MS_DBG_ONE_BOARD_PER_WAVE | MS_DBG_FORCE_CHAIN_PLACEMENT | MS_DBG_TWO_BOARDS_PER_WAVE)) &&
        (p.n >= kPack16MinEnvs || (p.dbg_flags & MS_DBG_FORCE_PACKED)) && ((uintptr_t)p.obs & 15u) == 0 &&
        ((uintptr_t)p.mask & 3u) == 0 && !p.codes) {
      constexpr int WPG = 4;
      const unsigned grid = (unsigned)((p.n + 4 * WPG - 1) / (4 * WPG));
      hipExtLaunchKernelGGL((k_step_packed<H_, W_, WPG, 4>), dim3(grid), dim3(64 * WPG), 0, s, ev0, ev1, 0, p);
      return;
    }
  }
  if constexpr (packable<H_, W_>()) {
    // small boards: four per wave (k_step_packed); its float4 / dword stores need a
    // 16-B obs and 4-B mask base
    if (p.K >= 1 && p.K <= 16 && !(p.dbg_flags & (MS_DBG_ONE_BOARD_PER_WAVE | MS_DBG_FORCE_CHAIN_PLACEMENT)) &&
        ((uintptr_t)p.obs & 15u) == 0 && ((uintptr_t)p.mask & 3u) == 0 && !p.codes) {
      constexpr int WPG = 4;
      if (p.dbg_flags & MS_DBG_TWO_BOARDS_PER_WAVE) {
        const unsigned grid = (unsigned)((p.n + 2 * WPG - 1) / (2 * WPG));
        hipExtLaunchKernelGGL((k_step_packed<H_, W_, WPG, 2>), dim3(grid), dim3(64 * WPG), 0, s, ev0, ev1, 0, p);
      } else {
        const unsigned grid = (unsigned)((p.n + 4 * WPG - 1) / (4 * WPG));
        hipExtLaunchKernelGGL((k_step_packed<H_, W_, WPG, 4>), dim3(grid), dim3(64 * WPG), 0, s, ev0, ev1, 0, p);
      }
      return;
    }
  }
  // generic shapes keep one board per workgroup (their LDS table is sized for 64x62)
  if (H_ && W_ && epw == 4) {
    hipExtLaunchKernelGGL((k_step<H_, W_, 4>), dim3((unsigned)((p.n + 3) / 4)), dim3(256), 0, s, ev0, ev1, 0, p);
  } else {
    hipExtLaunchKernelGGL((k_step<H_, W_, 1>), dim3((unsigned)p.n), dim3(64), 0, s, ev0, ev1, 0, p);
  }
}

template <int H_, int W_>
void launch_run(const KParams& p, const RunParams& r, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  if constexpr (packable16<H_, W_>()) {  // (as launch_step; each step's 4-board chunk is 16-B aligned)
    if (p.K >= 1 && p.K <= 48 &&
        !(p.dbg_flags & (MS_DBG_ONE_BOARD_PER_WAVE | MS_DBG_FORCE_CHAIN_PLACEMENT | MS_DBG_TWO_BOARDS_PER_WAVE)) &&
        (p.n >= kPack16RunMinEnvs || (p.dbg_flags & MS_DBG_FORCE_PACKED)) && ((uintptr_t)p.obs & 15u) == 0 &&
        ((uintptr_t)p.mask & 3u) == 0) {
      constexpr int WPG = 4;
      const unsigned grid = (unsigned)((p.n + 4 * WPG - 1) / (4 * WPG));
      hipExtLaunchKernelGGL((k_run_packed<H_, W_, WPG, 4>), dim3(grid), dim3(64 * WPG), 0, s, ev0, ev1, 0, p, r);
      return;
    }
  }
  if constexpr (packable<H_, W_>()) {
    // small boards: four per wave (k_run_packed); each step's 4-board obs / mask chunk must
    // start 16-B / 4-B aligned, in every slot
    const bool slot_ok = !r.slots || ((p.n * H_ * W_) & 3) == 0;
    if (p.K >= 1 && p.K <= 16 && !(p.dbg_flags & (MS_DBG_ONE_BOARD_PER_WAVE | MS_DBG_FORCE_CHAIN_PLACEMENT)) &&
        ((uintptr_t)p.obs & 15u) == 0 && ((uintptr_t)p.mask & 3u) == 0 && slot_ok) {
      constexpr int WPG = 4;
      if (p.dbg_flags & MS_DBG_TWO_BOARDS_PER_WAVE) {
        const unsigned grid = (unsigned)((p.n + 2 * WPG - 1) / (2 * WPG));
        hipExtLaunchKernelGGL((k_run_packed<H_, W_, WPG, 2>), dim3(grid), dim3(64 * WPG), 0, s, ev0, ev1, 0, p, r);
      } else {
        const unsigned grid = (unsigned)((p.n + 4 * WPG - 1) / (4 * WPG));
        hipExtLaunchKernelGGL((k_run_packed<H_, W_, WPG, 4>), dim3(grid), dim3(64 * WPG), 0, s, ev0, ev1, 0, p, r);
      }
      return;
    }
  }
  if (H_ && W_)
    hipExtLaunchKernelGGL((k_run<H_, W_, 4>), dim3((unsigned)((p.n + 3) / 4)), dim3(256), 0, s, ev0, ev1, 0, p, r);
  else hipExtLaunchKernelGGL((k_run<H_, W_, 1>), dim3((unsigned)p.n), dim3(64), 0, s, ev0, ev1, 0, p, r);
}

template <int H_, int W_>
void launch_late_t(const KParams& p, Pcg* st, const LateCfg& c, const uint8_t* need, hipStream_t s) {
  hipLaunchKernelGGL((k_late<H_, W_>), dim3(1), dim3(64), 0, s, p, st, c, need);
}

void fill_params(const ms_handle* h, KParams& p) {
  p.meta = h->meta;
  p.mine_words = h->mine_words;
  p.rev_words = h->rev_words;
  p.n = h->n;
  p.H = h->H;
  p.W = h->W;
  p.K = h->cfg.mine_count;
  p.guarantee = h->cfg.guarantee_safe_neighborhood ? 1 : 0;
  p.win_reward = h->cfg.win_reward;
  p.loss_reward = h->cfg.loss_reward;
  p.step_penalty = h->cfg.step_penalty;
  p.jump = h->jump;
  p.diag = h->diag;
  p.dbg_flags = h->dbg_flags;
}

template <int H_, int W_>
void launch_late_keyed_t(const KParams& p, const ms_handle* h, const uint8_t* need, hipStream_t s) {
  hipLaunchKernelGGL((k_late_keyed<H_, W_>), dim3((unsigned)p.n), dim3(64), 0, s, p, h->late, h->late_seed,
                     h->env_begin, need);
}

int launch_late(const ms_handle* h, const KParams& p, const uint8_t* need, hipStream_t s) {
  if (h->late_mode == MS_LATE_KEYED) {
    if (h->H == 16 && h->W == 16) launch_late_keyed_t<16, 16>(p, h, need, s);
    else if (h->H == 9 && h->W == 9) launch_late_keyed_t<9, 9>(p, h, need, s);
    else launch_late_keyed_t<0, 0>(p, h, need, s);
  } else if (h->H == 16 && h->W == 16) launch_late_t<16, 16>(p, h->late_rng, h->late, need, s);
  else if (h->H == 9 && h->W == 9) launch_late_t<9, 9>(p, h->late_rng, h->late, need, s);
  else launch_late_t<0, 0>(p, h->late_rng, h->late, need, s);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? MS_OK : hip_fail(e, "late-start launch");
}

int do_step(ms_handle* h, const void* actions, int i32, float* obs, uint8_t* mask, float* reward,
            uint8_t* done, int32_t* step, int32_t* last_new, double* frac, int8_t* outcome, void* stream,
            uint8_t* codes = nullptr) {
  if (!h) return fail(MS_EINVAL, "ms_step: null handle");
  if (!actions) return fail(MS_EINVAL, "ms_step: null actions");
  if (codes && ((h->H * h->W) & 3) == 0 && ((uintptr_t)codes & 3u) != 0)
    return fail(MS_EINVAL, "ms_step_codes: codes must be 4-byte aligned");
  KParams p = {};
  p.actions = actions;
  p.codes = codes;
  p.obs = obs;
  p.mask = mask;
  p.reward = reward;
  p.done = done;
  p.step = step;
  p.last_new = last_new;
  p.frac = frac;
  p.outcome = outcome;
  fill_params(h, p);
  p.actions_i32 = i32;
  hipStream_t s = (hipStream_t)stream;
  if (h->late_on && !done) return fail(MS_EINVAL, "ms_step: late start needs the done output");
  if (h->H == 16 && h->W == 16) launch_step<16, 16>(p, h->epw, s, h->ev_start, h->ev_stop);
  else if (h->H == 9 && h->W == 9) launch_step<9, 9>(p, h->epw, s, h->ev_start, h->ev_stop);
  else if (h->H == 30 && h->W == 16) launch_step<30, 16>(p, h->epw, s, h->ev_start, h->ev_stop);
  else if (h->H == 16 && h->W == 30) launch_step<16, 30>(p, h->epw, s, h->ev_start, h->ev_stop);
  else if (h->H == 8 && h->W == 8) launch_step<8, 8>(p, h->epw, s, h->ev_start, h->ev_stop);
  else launch_step<0, 0>(p, h->epw, s, h->ev_start, h->ev_stop);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "ms_step launch");
  // auto-resets that draw a late start (env.py:497-498 -> 406-414), in env order
  if (h->late_on) return launch_late(h, p, done, s);
  return MS_OK;
}

}  // namespace

extern "C" {

const char* ms_last_error(void) { return g_err; }

int32_t ms_abi_version(void) { return MSENV_ABI_VERSION; }

int ms_create(const ms_cfg* cfg, int64_t n_total, uint64_t base_seed, int64_t env_begin, int64_t env_count,
              ms_handle** out) {
  if (!cfg || !out) return fail(MS_EINVAL, "ms_create: null argument");
  *out = nullptr;
  if (!shape_ok(cfg))
    return fail(MS_EINVAL, "ms_create: unsupported board (need 1<=H<=64, 1<=W<=62, 0<=mine_count<H*W)");
  if (n_total <= 0 || env_begin < 0 || env_count <= 0 || env_begin + env_count > n_total)
    return fail(MS_EINVAL, "ms_create: bad env range");
  if (n_total > (int64_t)1 << 31) return fail(MS_EINVAL, "ms_create: n_total too large");
  ms_handle* h = new (std::nothrow) ms_handle();
  if (!h) return fail(MS_ENOMEM, "ms_create: host allocation failed");
  h->cfg = *cfg;
  h->n_total = n_total;
  h->env_begin = env_begin;
  h->n = env_count;
  h->H = cfg->H;
  h->W = cfg->W;
  h->A = cfg->H * cfg->W;
  const int rpw = 64 / cfg->W;
  h->NW = (cfg->H + rpw - 1) / rpw;
  (void)hipGetDevice(&h->device);
  h->epw = 4;

  // env.py:393-395: base = default_rng(seed); seeds = base.integers(0, 2**31-1, N)
  std::vector<EnvMeta> meta((size_t)env_count);
  HostPcg base;
  host_seed(base, base_seed);
  for (int64_t i = 0; i < env_begin + env_count; ++i) {
    const uint32_t s = host_bounded(base, 2147483646u);
    if (i < env_begin) continue;
    HostPcg r;
    host_seed(r, s);
    EnvMeta& m = meta[(size_t)(i - env_begin)];
    m.st_hi = (uint64_t)(r.state >> 64);
    m.st_lo = (uint64_t)r.state;
    m.inc_hi = (uint64_t)(r.inc >> 64);
    m.inc_lo = (uint64_t)r.inc;
    m.has32 = 0;
    m.uinteger = 0;
    m.step_count = 0;
    m.flags = 0;
  }
  // PCG64 jump-ahead: state after k steps = M^k s + (sum_{i<k} M^i) inc, k = 1..64
  uint64_t jt[64 * 4];
  {
    const unsigned __int128 M = ((unsigned __int128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;
    unsigned __int128 Ak = 1, Ck = 0;
    for (int k = 1; k <= 64; ++k) {
      Ck = Ck + Ak;  // sum_{i<k} M^i
      Ak = Ak * M;   // M^k
      jt[4 * (k - 1) + 0] = (uint64_t)(Ak >> 64);
      jt[4 * (k - 1) + 1] = (uint64_t)Ak;
      jt[4 * (k - 1) + 2] = (uint64_t)(Ck >> 64);
      jt[4 * (k - 1) + 3] = (uint64_t)Ck;
    }
  }
  hipError_t e = hipMalloc((void**)&h->meta, sizeof(EnvMeta) * (size_t)env_count);
  if (e == hipSuccess) e = hipMalloc((void**)&h->jump, sizeof(jt));
  if (e == hipSuccess) e = hipMemcpy(h->jump, jt, sizeof(jt), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc((void**)&h->mine_words, sizeof(uint64_t) * (size_t)env_count * h->NW);
  if (e == hipSuccess) e = hipMalloc((void**)&h->rev_words, sizeof(uint64_t) * (size_t)env_count * h->NW);
  if (e == hipSuccess)
    e = hipMemcpy(h->meta, meta.data(), sizeof(EnvMeta) * (size_t)env_count, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(h->mine_words, 0, sizeof(uint64_t) * (size_t)env_count * h->NW);
  if (e == hipSuccess) e = hipMemset(h->rev_words, 0, sizeof(uint64_t) * (size_t)env_count * h->NW);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    const int rc = hip_fail(e, "ms_create");
    ms_destroy(h);
    return rc;
  }
  *out = h;
  return MS_OK;
}

int ms_destroy(ms_handle* h) {
  if (!h) return MS_OK;
  if (h->meta) (void)hipFree(h->meta);
  if (h->mine_words) (void)hipFree(h->mine_words);
  if (h->rev_words) (void)hipFree(h->rev_words);
  if (h->jump) (void)hipFree(h->jump);
  if (h->late_rng) (void)hipFree(h->late_rng);
  delete h;
  return MS_OK;
}

// Diagnostics (not part of msenv.h): per-env s_memtime stamps [env_count][8]
// are written by libmsenv_diag.so (built with -DMS_DIAG); NULL disables.
int ms_set_debug_flags(ms_handle* h, uint32_t flags) {
  if (!h) return fail(MS_EINVAL, "ms_set_debug_flags: null handle");
  h->dbg_flags = flags;
  return MS_OK;
}

int ms_set_timing_events(ms_handle* h, void* start_event, void* stop_event) {
  if (!h) return fail(MS_EINVAL, "ms_set_timing_events: null handle");
  h->ev_start = (hipEvent_t)start_event;
  h->ev_stop = (hipEvent_t)stop_event;
  return MS_OK;
}

int ms_event_create(void** event) {
  if (!event) return fail(MS_EINVAL, "ms_event_create: null argument");
  hipEvent_t e = nullptr;
  hipError_t r = hipEventCreate(&e);
  if (r != hipSuccess) return hip_fail(r, "hipEventCreate");
  *event = (void*)e;
  return MS_OK;
}

int ms_event_elapsed_ms(void* start_event, void* stop_event, float* ms) {
  if (!start_event || !stop_event || !ms) return fail(MS_EINVAL, "ms_event_elapsed_ms: null argument");
  hipError_t r = hipEventElapsedTime(ms, (hipEvent_t)start_event, (hipEvent_t)stop_event);
  return r == hipSuccess ? MS_OK : hip_fail(r, "hipEventElapsedTime");
}

int ms_event_destroy(void* event) {
  if (event) (void)hipEventDestroy((hipEvent_t)event);
  return MS_OK;
}

int ms_set_diag(ms_handle* h, uint64_t* stamps) {
  if (!h) return fail(MS_EINVAL, "ms_set_diag: null handle");
  h->diag = stamps;
  return MS_OK;
}

int ms_reset(ms_handle* h, float* obs, uint8_t* mask, void* stream) {
  if (!h) return fail(MS_EINVAL, "ms_reset: null handle");
  const int64_t work = h->n * 10 * (int64_t)h->A / 4 + 1;
  int blocks = (int)((work + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_reset, dim3(blocks), dim3(256), 0, (hipStream_t)stream, h->meta, h->mine_words,
                     h->rev_words, h->n, h->NW, obs, mask, h->A);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "ms_reset launch");
  if (h->late_on) {  // every env: _reset_env_state (env.py:406-414, 468-477)
    KParams p = {};
    fill_params(h, p);
    p.obs = obs;
    p.mask = mask;
    return launch_late(h, p, nullptr, (hipStream_t)stream);
  }
  return MS_OK;
}

int ms_set_late_start(ms_handle* h, double prob, int32_t min_hidden, int32_t max_hidden, int32_t max_attempts,
                      int32_t max_extra_steps, uint64_t late_seed) {
  if (!h) return fail(MS_EINVAL, "ms_set_late_start: null handle");
  // clamps of env.py:424-430
  LateCfg c;
  c.prob = prob;
  c.min_hidden = min_hidden < 1 ? 1 : min_hidden;
  c.max_hidden = max_hidden < c.min_hidden ? c.min_hidden : max_hidden;
  c.max_attempts = max_attempts < 1 ? 1 : max_attempts;
  c.max_extra_steps = max_extra_steps < 1 ? 1 : max_extra_steps;
  HostPcg r;
  host_seed(r, late_seed);
  Pcg d;
  d.hi = (uint64_t)(r.state >> 64);
  d.lo = (uint64_t)r.state;
  d.ihi = (uint64_t)(r.inc >> 64);
  d.ilo = (uint64_t)r.inc;
  d.has32 = (uint32_t)r.has32;
  d.uinteger = r.uinteger;
  if (!h->late_rng) {
    hipError_t e = hipMalloc(&h->late_rng, sizeof(Pcg));
    if (e != hipSuccess) return hip_fail(e, "ms_set_late_start alloc");
  }
  hipError_t e = hipMemcpy(h->late_rng, &d, sizeof(Pcg), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(e, "ms_set_late_start copy");
  h->late = c;
  h->late_on = 1;
  h->late_seed = late_seed;
  return MS_OK;
}

int ms_set_late_start_mode(ms_handle* h, int32_t mode) {
  if (!h) return fail(MS_EINVAL, "ms_set_late_start_mode: null handle");
  if (mode != MS_LATE_SHARED && mode != MS_LATE_KEYED) return fail(MS_EINVAL, "ms_set_late_start_mode: bad mode");
  h->late_mode = mode;
  return MS_OK;
}

int ms_late_rng_state(ms_handle* h, uint64_t* out) {
  if (!h || !out) return fail(MS_EINVAL, "ms_late_rng_state: bad argument");
  if (!h->late_rng) return fail(MS_EINVAL, "ms_late_rng_state: late start not configured");
  Pcg d;
  hipError_t e = hipMemcpy(&d, h->late_rng, sizeof(Pcg), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_fail(e, "ms_late_rng_state copy");
  out[0] = d.hi;
  out[1] = d.lo;
  out[2] = d.ihi;
  out[3] = d.ilo;
  out[4] = d.has32;
  out[5] = d.uinteger;
  return MS_OK;
}

int ms_step(ms_handle* h, const int64_t* actions, float* obs, uint8_t* mask, float* reward, uint8_t* done,
            int32_t* step, int32_t* last_new, double* revealed_frac, int8_t* outcome, void* stream) {
  return do_step(h, actions, 0, obs, mask, reward, done, step, last_new, revealed_frac, outcome, stream);
}

int ms_step_i32(ms_handle* h, const int32_t* actions, float* obs, uint8_t* mask, float* reward, uint8_t* done,
                int32_t* step, int32_t* last_new, double* revealed_frac, int8_t* outcome, void* stream) {
  return do_step(h, actions, 1, obs, mask, reward, done, step, last_new, revealed_frac, outcome, stream);
}

int ms_step_codes(ms_handle* h, const int64_t* actions, uint8_t* codes, uint8_t* mask, float* reward, uint8_t* done,
                  int32_t* step, int32_t* last_new, double* revealed_frac, int8_t* outcome, void* stream) {
  return do_step(h, actions, 0, nullptr, mask, reward, done, step, last_new, revealed_frac, outcome, stream, codes);
}

int ms_run_tape(ms_handle* h, uint64_t t0, int32_t T, int32_t mode, int32_t slots, int64_t* actions, float* obs,
                uint8_t* mask, float* reward, uint8_t* done, int32_t* step, int32_t* last_new, double* revealed_frac,
                int8_t* outcome, void* stream) {
  if (!h) return fail(MS_EINVAL, "ms_run_tape: null handle");
  if (T < 1) return fail(MS_EINVAL, "ms_run_tape: T must be >= 1");
  if (mode != MS_TAPE_UNIFORM && mode != MS_TAPE_SAFE_BIASED) return fail(MS_EINVAL, "ms_run_tape: bad mode");
  if (h->late_on) return fail(MS_EINVAL, "ms_run_tape: late-start resets are not supported");
  KParams p = {};
  fill_params(h, p);
  p.actions = nullptr;
  p.obs = obs;
  p.mask = mask;
  p.reward = reward;
  p.done = done;
  p.step = step;
  p.last_new = last_new;
  p.frac = revealed_frac;
  p.outcome = outcome;
  RunParams r;
  r.t0 = t0;
  r.T = T;
  r.mode = mode;
  r.slots = slots ? 1 : 0;
  r.env_begin = h->env_begin;
  r.actions = actions;
  const hipStream_t s = (hipStream_t)stream;
  if (h->H == 16 && h->W == 16) launch_run<16, 16>(p, r, s, h->ev_start, h->ev_stop);
  else if (h->H == 9 && h->W == 9) launch_run<9, 9>(p, r, s, h->ev_start, h->ev_stop);
  else if (h->H == 30 && h->W == 16) launch_run<30, 16>(p, r, s, h->ev_start, h->ev_stop);
  else if (h->H == 16 && h->W == 30) launch_run<16, 30>(p, r, s, h->ev_start, h->ev_stop);
  else if (h->H == 8 && h->W == 8) launch_run<8, 8>(p, r, s, h->ev_start, h->ev_stop);
  else launch_run<0, 0>(p, r, s, h->ev_start, h->ev_stop);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? MS_OK : hip_fail(e, "ms_run_tape launch");
}

int ms_labels(ms_handle* h, float* mine_labels, uint8_t* mine_valid, void* stream) {
  if (!h) return fail(MS_EINVAL, "ms_labels: null handle");
  hipLaunchKernelGGL(k_labels, dim3((unsigned)h->n), dim3(64), 0, (hipStream_t)stream, h->meta, h->mine_words,
                     h->rev_words, h->n, h->H, h->W, mine_labels, mine_valid);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? MS_OK : hip_fail(e, "ms_labels launch");
}

int ms_snapshot(ms_handle* h, uint8_t* mine, uint8_t* revealed, uint8_t* counts, uint8_t* first_click,
                int32_t* step_count, void* stream) {
  if (!h) return fail(MS_EINVAL, "ms_snapshot: null handle");
  hipLaunchKernelGGL(k_snapshot, dim3((unsigned)h->n), dim3(64), 0, (hipStream_t)stream, h->meta,
                     h->mine_words, h->rev_words, h->n, h->H, h->W, mine, revealed, counts, first_click,
                     step_count);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? MS_OK : hip_fail(e, "ms_snapshot launch");
}

int ms_rng_state(ms_handle* h, uint64_t* out, void* stream) {
  if (!h || !out) return fail(MS_EINVAL, "ms_rng_state: null argument");
  hipLaunchKernelGGL(k_rng_state, dim3((unsigned)((h->n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     h->meta, h->n, out);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? MS_OK : hip_fail(e, "ms_rng_state launch");
}

int ms_tape_actions(ms_handle* h, uint64_t t, int32_t mode, int64_t* actions, void* stream) {
  if (!h || !actions) return fail(MS_EINVAL, "ms_tape_actions: null argument");
  if (mode != MS_TAPE_UNIFORM && mode != MS_TAPE_SAFE_BIASED) return fail(MS_EINVAL, "ms_tape_actions: bad mode");
  const hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)((h->n + 63) / 64)), block(64);
  if (h->H == 16 && h->W == 16)
    hipLaunchKernelGGL((k_tape<16, 16>), grid, block, 0, s, h->mine_words, h->rev_words, h->n, h->H, h->W,
                       h->env_begin, t, mode, actions);
  else if (h->H == 9 && h->W == 9)
    hipLaunchKernelGGL((k_tape<9, 9>), grid, block, 0, s, h->mine_words, h->rev_words, h->n, h->H, h->W,
                       h->env_begin, t, mode, actions);
  else if (h->H == 30 && h->W == 16)
    hipLaunchKernelGGL((k_tape<30, 16>), grid, block, 0, s, h->mine_words, h->rev_words, h->n, h->H, h->W,
                       h->env_begin, t, mode, actions);
  else if (h->H == 16 && h->W == 30)
    hipLaunchKernelGGL((k_tape<16, 30>), grid, block, 0, s, h->mine_words, h->rev_words, h->n, h->H, h->W,
                       h->env_begin, t, mode, actions);
  else
    hipLaunchKernelGGL((k_tape<0, 0>), grid, block, 0, s, h->mine_words, h->rev_words, h->n, h->H, h->W,
                       h->env_begin, t, mode, actions);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? MS_OK : hip_fail(e, "ms_tape_actions launch");
}

int ms_gae(const float* rewards, const float* values, const uint8_t* dones, const float* last_values, int32_t T,
           int64_t N, float gamma, float gamma_lambda, float* adv, float* ret, void* stream) {
  if (!rewards || !values || !dones || !last_values || !adv || !ret || T <= 0 || N <= 0)
    return fail(MS_EINVAL, "ms_gae: bad argument");
  hipLaunchKernelGGL(k_gae, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, rewards, values,
                     dones, last_values, (int)T, N, gamma, gamma_lambda, adv, ret);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? MS_OK : hip_fail(e, "ms_gae launch");
}

int ms_sample_masked(const float* logits, const uint8_t* mask, int64_t N, int32_t A, int64_t row_begin,
                     uint64_t seed, uint64_t counter, int64_t* actions, float* logp, void* stream) {
  if (!logits || !mask || !actions || !logp || N <= 0 || A <= 0 || row_begin < 0)
    return fail(MS_EINVAL, "ms_sample_masked: bad argument");
  hipLaunchKernelGGL(k_sample, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, (hipStream_t)stream, logits, mask, N,
                     (int)A, row_begin, seed, counter, actions, logp);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? MS_OK : hip_fail(e, "ms_sample_masked launch");
}

int ms_dropout_masks(const int64_t* rows, int64_t N, int32_t nblk, int32_t C, uint64_t seed, uint64_t counter,
                     float p, float* out, void* stream) {
  if (!rows || !out || N <= 0 || nblk <= 0 || C <= 0 || (C & 3) || !(p > 0.f && p < 1.f))
    return fail(MS_EINVAL, "ms_dropout_masks: bad argument");
  const int64_t total = (int64_t)nblk * N * (C / 4);
  const unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(k_dropout, dim3(grid), dim3(256), 0, (hipStream_t)stream, rows, N, (int)nblk, (int)C, seed,
                     counter, p, 1.0f / (1.0f - p), out);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? MS_OK : hip_fail(e, "ms_dropout_masks launch");
}

}  // extern "C"
