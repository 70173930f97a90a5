// mscnn_common.h — types and wave helpers shared by the fused residual-CNN
// kernels (mscnn.hip forward, mscnn_bwd.hip backward).
#pragma once

#include <hip/hip_runtime.h>

#include <stdint.h>

namespace mc {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
// native vector: HIP's uint4 struct copies through memcpy and is left in scratch
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// 16-bit activation / weight element: __bf16 (bf16 autocast) or _Float16 (fp16 autocast,
// the reference's own training precision); all sums are f32 either way
template <typename E>
struct EV;
template <>
struct EV<__bf16> {
  typedef bf16x8 v8;
  typedef bf16x4 v4;
};
template <>
struct EV<_Float16> {
  typedef f16x8 v8;
  typedef f16x4 v4;
};

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

constexpr int COUT = 96;  // trunk width of the shipped configs (stem_channels)
constexpr int NGRP = 6;   // GroupNorm groups (96 / 16)
constexpr int WAVES = 4;  // 256-thread workgroups

extern thread_local char g_err[256];

int num_cus();

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, true));
}

// sum over each 16-lane row; the result is valid in lanes 15, 31, 47, 63
__device__ __forceinline__ float row_sum16(float v) {
  v += dppf<0x111>(v);
  v += dppf<0x112>(v);
  v += dppf<0x114>(v);
  v += dppf<0x118>(v);
  return v;
}

__device__ __forceinline__ float readlane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q / columns
// 4p..4p+3 of a 4x16 block of 16-bit elements; lane i receives column i.
template <typename E>
__device__ __forceinline__ typename EV<E>::v4 lds_tr4(const E* p) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
  return __builtin_bit_cast(typename EV<E>::v4, v);
}

// An SGPR zero the compiler cannot see through: indexing loop-invariant LDS data with
// it keeps the loads inside a persistent loop instead of hoisting them all into
// registers (which spills).
__device__ __forceinline__ int opaque0() {
  int z = 0;
  asm volatile("" : "+s"(z));
  return z;
}

// An f32 value the compiler must materialise: (E)(a * b) and (E)(a + b) otherwise may become one
// v_fma_mix*_f16 with a single rounding to 16 bits, chosen per call site, so two kernels
// computing the same expression could round differently. Pinned, every such site rounds to f32
// first and then to 16 bits, as PyTorch's f32-compute autocast does.
__device__ __forceinline__ float pin_f32(float v) {
  asm("" : "+v"(v));
  return v;
}

// fmaf(a, (float)h, c) for the low / high fp16 half h of a 32-bit word, as one v_fma_mix_f32:
// the f16 -> f32 conversion is exact, so it rounds once exactly as the v_cvt_f32_f16 + v_fma_f32
// pair it replaces (the compiler does not form it from a vector element extraction)
__device__ __forceinline__ float fmix_lo(float a, uint32_t h2, float c) {
  float r;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(r) : "v"(a), "v"(h2), "v"(c));
  return r;
}
__device__ __forceinline__ float fmix_hi(float a, uint32_t h2, float c) {
  float r;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(r) : "v"(a), "v"(h2), "v"(c));
  return r;
}

// (float)a + (float)b for the low / high fp16 halves of two words, as 1 * a + b in one v_fma_mix_f32
// (both widenings exact, one rounding: the f32 sum the cvt + cvt + add sequence gives)
__device__ __forceinline__ float fmix2_lo(uint32_t a2, uint32_t b2) {
  float r;
  asm("v_fma_mix_f32 %0, 1.0, %1, %2 op_sel_hi:[0,1,1]" : "=v"(r) : "v"(a2), "v"(b2));
  return r;
}
__device__ __forceinline__ float fmix2_hi(uint32_t a2, uint32_t b2) {
  float r;
  asm("v_fma_mix_f32 %0, 1.0, %1, %2 op_sel:[0,1,1] op_sel_hi:[0,1,1]" : "=v"(r) : "v"(a2), "v"(b2));
  return r;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations and
// meets the other waves, leaving global loads and stores in flight. __syncthreads()'s
// workgroup release fence turns into s_waitcnt vmcnt(0) as soon as global stores are
// outstanding (gfx9 counts stores on vmcnt), draining an epilogue's stores and any
// prefetched loads at every barrier. The memory clobber keeps the compiler from moving
// memory operations across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// sum over the whole wave, returned in every lane (row sums, then the four rows' last lanes)
__device__ __forceinline__ float wave_sum(float v) {
  v = row_sum16(v);
  return (readlane_f(v, 15) + readlane_f(v, 31)) + (readlane_f(v, 47) + readlane_f(v, 63));
}

// Barrier among the 4 waves of one role of a wave-specialised workgroup, through a monotonic LDS
// counter (s_barrier would hold the other role's waves too): each wave finishes its LDS work,
// adds 1, and waits until the counter reaches target = 4 * (barriers passed so far).
__device__ __forceinline__ void grp_bar(unsigned* cnt, unsigned target, int lane) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
  asm volatile("" ::: "memory");
}

// Kernel variants (msenv_debug.h mc_set_variant): 0 = the dispatcher's choice.
enum { MCV_FWD = 0, MCV_BWD = 1, MCV_WGRAD = 2, MCV_TRUNK_FWD = 3, MCV_COUNT = 4 };
extern int g_variant[MCV_COUNT];

__device__ __forceinline__ bf16x8 cat8(bf16x4 lo, bf16x4 hi) {
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
__device__ __forceinline__ f16x8 cat8(f16x4 lo, f16x4 hi) {
  return f16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// the dtype argument of the mscnn.h entry points
enum { MC_DT_BF16 = 0, MC_DT_F16 = 1 };

}  // namespace mc
