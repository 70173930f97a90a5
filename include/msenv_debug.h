/*
 * msenv_debug.h — test/diagnostic hooks of libmsenv.so (not part of the
 * drop-in boundary; bench.py and the GPU tests use them).
 */
#ifndef MSENV_DEBUG_H
#define MSENV_DEBUG_H

#include <stdint.h>

#include "msenv.h"

#ifdef __cplusplus
extern "C" {
#endif

/* debug flags */
#define MS_DBG_FORCE_SERIAL_PLACEMENT 1u /* serial reference-order PCG draws + Floyd chain */
#define MS_DBG_FORCE_CHAIN_PLACEMENT 2u  /* jump-ahead draws + serial Floyd chain (K > 128 path) */
#define MS_DBG_ONE_BOARD_PER_WAVE 4u     /* ms_step: k_step (one board per wave) even where the
                                            lane-packed k_step_packed applies (9x9, 8x8, K<=16) */
#define MS_DBG_TWO_BOARDS_PER_WAVE 8u    /* k_step_packed with two boards per wave (32-lane groups) */
#define MS_DBG_FORCE_PACKED 16u          /* 16x16: k_step_packed at any env count (default: >= 65536) */

int ms_set_debug_flags(ms_handle* h, uint32_t flags);

/* Kernel variants of the fused CNN layer (mscnn.h), for same-process A/B runs and for the
 * parity tests of every path. Kernel 0 = mc_conv_gn_fwd, 1 = mc_conv_gn_bwd's data backward:
 * variant 0 = the dispatcher's choice (default) = 1 = the per-sample kernel (two 256-thread
 * workgroups per CU). (Round 4's wave-specialised forms, variants 2-5, measured slower and were
 * removed from the library in round 5; DESIGN.md §5 keeps their record, git history the code.)
 * Kernel 2 = the weight gradient on 16x16 boards with 96 channels: variant 0 = default (= 3),
 * 1 = k_wgrad (three ci-slice workgroups a sample group, the compiler's LDS-read schedule),
 * 2 = k_wgrad with the next step's reads pinned between this step's MFMAs, 3 = k_wgrad_c96 (one
 * workgroup a CU owns all 81 tiles; dy by LDS-DMA). Kernel 3 = mc_trunk_fwd on boards of <= 256
 * cells: variant 0 = default (k_trunk_fwd_pp, the ping-pong forward, when nothing is saved --
 * the rollout's forward; k_trunk_fwd2 when y / stats / ReLU bits are saved -- the training
 * forward), 1 = k_trunk_fwd2 always, 2 = k_trunk_fwd_pp always. Any other (kernel, variant) is
 * MS_EINVAL. Process-wide, not thread-safe. */
#define MC_VAR_FWD 0
#define MC_VAR_BWD 1
#define MC_VAR_WGRAD 2
#define MC_VAR_TRUNK_FWD 3
int mc_set_variant(int32_t kernel, int32_t variant);

/* Measurement (bench.py): while set, every k_step / k_run launch of this handle is
 * dispatched with hipExtLaunchKernel(start_event, stop_event), so the events are stamped
 * by the dispatch itself and bracket exactly the kernel's execution (what rocprofv3's
 * kernel trace reports), without the launch gap a stream event would include.
 * NULL, NULL restores plain launches. Not for graph capture. */
int ms_set_timing_events(ms_handle* h, void* start_event, void* stop_event);
int ms_event_create(void** event);
int ms_event_elapsed_ms(void* start_event, void* stop_event, float* ms);
int ms_event_destroy(void* event);

/* libmsenv_diag.so only: per-env s_memtime/s_memrealtime stamps, device
 * u64[env_count][16] (slots 0-5 phases, 6-7 realtime, 8-14 placement sub-phases; NULL
 * disables). Ignored by the production build. */
int ms_set_diag(ms_handle* h, uint64_t* stamps);

#ifdef __cplusplus
}
#endif

#endif /* MSENV_DEBUG_H */
