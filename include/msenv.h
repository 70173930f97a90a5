/*
 * msenv.h — C ABI of the MI355X-native vectorised Minesweeper board step and
 * the on-device rollout kernels (GAE, masked categorical sampling).
 *
 * The reference (yakvrz/minesweeper-ppo) has no FFI: its hot path sits behind
 * the duck-typed Python class `VecMinesweeper` (minesweeper/env.py:379-517)
 * with an inner numba boundary `flood_fill_reveal` (minesweeper/env_numba.py:17-77).
 * Each entry point below names the reference interface it replaces.
 * INTEGRATION.md shows the ctypes binding a maintainer adds on the reference side.
 *
 * Conventions
 *   - Plain pointers and sizes only. Every array argument is a DEVICE pointer
 *     (e.g. a torch tensor's data_ptr()) unless the comment says "host".
 *   - `stream` is a hipStream_t passed as void* (NULL = the default stream).
 *     Calls are asynchronous on that stream; no host synchronisation happens
 *     inside ms_step / ms_reset / ms_labels / ms_tape_actions / ms_gae /
 *     ms_sample_masked, so they can be captured into a hipGraph.
 *   - Return value: 0 (MS_OK) on success, a nonzero MS_E* code otherwise;
 *     ms_last_error() returns a thread-local message for the last failure.
 *   - One handle per stream; calls on one handle are not re-entrant.
 *   - Boards up to H <= 64 rows and W <= 62 columns (A = H*W <= 3968 cells), the
 *     range in which numpy's choice(replace=False) uses Floyd's algorithm.
 */
#ifndef MSENV_H
#define MSENV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSENV_ABI_VERSION 3

enum {
  MS_OK = 0,
  MS_EINVAL = 1,   /* bad argument (shape, size, null handle) */
  MS_EHIP = 2,     /* HIP runtime error */
  MS_ENOMEM = 3    /* allocation failure */
};

/* outcome codes written by ms_step (reference: info["outcome"], env.py:113-145) */
enum { MS_OUTCOME_NONE = 0, MS_OUTCOME_WIN = 1, MS_OUTCOME_LOSS = 2 };

/* action-tape modes for ms_tape_actions (SURVEY.md §8d synthetic policy) */
enum { MS_TAPE_UNIFORM = 0, MS_TAPE_SAFE_BIASED = 1 };
/* Late-start generator modes (ms_set_late_start_mode). */
enum { MS_LATE_SHARED = 0, MS_LATE_KEYED = 1 };

/* Replaces EnvConfig (env.py:19-30). use_pair_constraints / solver_preset are
 * inert on the step path and therefore absent. Rewards are doubles: the
 * reference accumulates the reward in Python float and casts to f32 at
 * env.py:483/501. */
typedef struct ms_cfg {
  int32_t H;
  int32_t W;
  int32_t mine_count;
  int32_t guarantee_safe_neighborhood; /* bool */
  double win_reward;
  double loss_reward;
  double step_penalty;
} ms_cfg;

typedef struct ms_handle ms_handle;

/* Thread-local description of the last error (never NULL). */
const char* ms_last_error(void);

/* ABI version (MSENV_ABI_VERSION). */
int32_t ms_abi_version(void);

/* Replaces VecMinesweeper.__init__ (env.py:382-403) + MinesweeperEnv.__init__
 * (env.py:41-77). Per-env seeds are derived for all n_total envs exactly as
 * `default_rng(base_seed).integers(0, 2**31-1, size=n_total)` (env.py:393-394)
 * and this handle owns envs [env_begin, env_begin+env_count) of that list, each
 * with its own numpy-compatible PCG64 stream (env.py:49). A sharded run is
 * therefore trajectory-identical to a single-device run. Allocates HBM state
 * on the current HIP device. */
int ms_create(const ms_cfg* cfg, int64_t n_total, uint64_t base_seed,
              int64_t env_begin, int64_t env_count, ms_handle** out);

/* Frees the handle and its HBM state. NULL is a no-op. */
int ms_destroy(ms_handle* h);

/* Replaces VecMinesweeper.reset (env.py:468-477): clears every board (the RNG
 * streams continue, env.py:87-101) and writes obs f32[env_count,10,H,W] and
 * mask u8[env_count,H*W]. Either output may be NULL. */
int ms_reset(ms_handle* h, float* obs, uint8_t* mask, void* stream);

/* Replaces VecMinesweeper.step (env.py:479-511) and, inside it,
 * MinesweeperEnv.step (env.py:103-152), _place_mines_safe (env.py:280-312),
 * _compute_adjacent_counts (env.py:314-335) and flood_fill_reveal
 * (env_numba.py:17-77). actions: int64[env_count] (ms_step) or
 * int32[env_count] (ms_step_i32), wrapped with Python `%` semantics.
 * Done envs auto-reset; obs/mask then hold the reset observation while
 * reward/done/step/last_new/revealed_frac/outcome describe the finished step
 * (env.py:492-505). Output shapes: obs f32[env_count,10,H,W],
 * mask u8[env_count,H*W], reward f32, done u8, step i32, last_new i32,
 * revealed_frac f64, outcome i8 (all [env_count]). Any output may be NULL. */
int ms_step(ms_handle* h, const int64_t* actions, float* obs, uint8_t* mask,
            float* reward, uint8_t* done, int32_t* step, int32_t* last_new,
            double* revealed_frac, int8_t* outcome, void* stream);
int ms_step_i32(ms_handle* h, const int32_t* actions, float* obs, uint8_t* mask,
                float* reward, uint8_t* done, int32_t* step, int32_t* last_new,
                double* revealed_frac, int8_t* outcome, void* stream);

/* ms_step for the training rollout's buffer (no reference counterpart: the reference buffer
 * stores the f32 one-hot obs, buffers.py:24-36): instead of obs f32[env_count,10,H,W] it writes
 * the cell codes u8[env_count,H*W] -- 0 hidden, 1 + k revealed with k adjacent mines, the obs's
 * one-hot planes as one byte (mscnn.h mc_obs_encode reads an obs into the same codes) -- 40x
 * fewer bytes. codes must be 4-byte aligned when H*W % 4 == 0. Other outputs as ms_step. */
int ms_step_codes(ms_handle* h, const int64_t* actions, uint8_t* codes, uint8_t* mask,
                  float* reward, uint8_t* done, int32_t* step, int32_t* last_new,
                  double* revealed_frac, int8_t* outcome, void* stream);

/* Replaces the per-env label loop of collect_rollout (train_rl.py:203-219):
 * mine_labels f32[env_count,H,W] = mine_mask if first_click_done else 0;
 * mine_valid u8[env_count,H,W] = ~revealed & ~flags if first_click_done else 0.
 * Either output may be NULL. */
int ms_labels(ms_handle* h, float* mine_labels, uint8_t* mine_valid, void* stream);

/* Backs the `envs[i]` proxies (eval.py:350-398, train_rl.py:205-212):
 * mine/revealed/counts u8[env_count,H,W], first_click u8[env_count],
 * step_count i32[env_count]. Any output may be NULL. */
int ms_snapshot(ms_handle* h, uint8_t* mine, uint8_t* revealed, uint8_t* counts,
                uint8_t* first_click, int32_t* step_count, void* stream);

/* PCG64 state per env as u64[env_count,6] = {state_hi, state_lo, inc_hi,
 * inc_lo, has_uint32, uinteger} (numpy's bit_generator.state layout). */
int ms_rng_state(ms_handle* h, uint64_t* out, void* stream);

/* Late-start resets (VecMinesweeper late_start_cfg, env.py:397-403, 416-466):
 * from now on every reset (ms_reset: all envs; ms_step: the auto-reset of each
 * done env) applies _apply_late_start with ONE generator shared by the envs of
 * this handle, seeded like numpy default_rng(late_seed), consumed in env order.
 * Arguments as the reference's cfg keys (prob, min_hidden, max_hidden,
 * max_attempts, max_extra_steps; pass H*W for the default max_extra_steps), with
 * the reference's clamps. Bit-exact with the reference for an unsharded handle
 * (env_begin 0, env_count n_total); a shard gets its own stream. ms_step then
 * requires its `done` output. */
int ms_set_late_start(ms_handle* h, double prob, int32_t min_hidden, int32_t max_hidden,
                      int32_t max_attempts, int32_t max_extra_steps, uint64_t late_seed);

/* Which generator the late starts draw from.
 * MS_LATE_SHARED (default): the reference's ONE generator, consumed in env order
 *   (env.py:397-403, 416-466). Each reset consumes a data-dependent number of
 *   draws, so the resets of a step form one serial chain (one wave walks them).
 *   Bit-exact with the reference on one handle; a shard draws its own stream.
 * MS_LATE_KEYED: each reset draws from its own PCG64 stream keyed by (late_seed,
 *   GLOBAL env index, the env's own generator state at the reset), so all of a
 *   step's resets run at once (one wave per env) and a shard's resets are those of
 *   the unsharded run. Same procedure and distribution as the reference; not the
 *   reference's stream of draws (oracle: mso_set_late_start_mode). */
int ms_set_late_start_mode(ms_handle* h, int32_t mode);

/* The late-start generator's state as u64[6] (ms_rng_state layout); synchronous. */
int ms_late_rng_state(ms_handle* h, uint64_t* out);

/* Synthetic policy: for global env g and step t,
 * x = splitmix64(0xC0FFEE ^ (g << 32) ^ t); MS_TAPE_UNIFORM picks the
 * (x mod popcount(mask))-th valid cell; MS_TAPE_SAFE_BIASED picks a non-mine
 * valid cell when (x & 0xFFFF) < 65208 (p = 0.995), else any valid cell, with
 * index (x >> 16) mod count. Writes actions int64[env_count]. */
int ms_tape_actions(ms_handle* h, uint64_t t, int32_t mode, int64_t* actions,
                    void* stream);

/* Env-only synthetic rollout: T consecutive steps t0 .. t0+T-1 of every env, each
 * equal to ms_tape_actions(t) followed by ms_step, in ONE launch that keeps every
 * board in registers between steps (bit-exact with the two-call sequence; the
 * reference analogue is stepping VecMinesweeper in a loop with random valid
 * actions, scripts/profile_env.py:17-30). slots = 0: every output is
 * overwritten by each step (the shapes of ms_step); slots = 1: step k writes
 * slot k of [T][env_count, ...] outputs. actions (int64, optional) receives the
 * tape's actions. Any output may be NULL. Late-start handles are rejected. */
int ms_run_tape(ms_handle* h, uint64_t t0, int32_t T, int32_t mode, int32_t slots,
                int64_t* actions, float* obs, uint8_t* mask, float* reward, uint8_t* done,
                int32_t* step, int32_t* last_new, double* revealed_frac, int8_t* outcome,
                void* stream);

/* Replaces RolloutBuffer.compute_gae (buffers.py:78-94). rewards/values f32
 * [T,N], dones u8[T,N], last_values f32[N]; writes adv and ret f32[T,N]. The
 * f32 op order is the reference's (no contraction), so results are bitwise
 * those of the torch loop given gamma = f32(gamma) and
 * gamma_lambda = f32(gamma*lambda) computed in double. */
int ms_gae(const float* rewards, const float* values, const uint8_t* dones,
           const float* last_values, int32_t T, int64_t N, float gamma,
           float gamma_lambda, float* adv, float* ret, void* stream);

/* Replaces masked_fill + Categorical(logits).sample/log_prob
 * (train_rl.py:229-235). logits f32[N,A], mask u8[N,A] (rows with no valid
 * cell are treated as all-valid, train_rl.py:166-168). Gumbel-max sampling
 * from a counter-based hash of (seed, counter, row_begin + row, cell): with
 * row_begin = the shard's first GLOBAL env index, a sharded rollout draws the
 * same actions as an unsharded one. Writes actions int64[N] and logp f32[N]
 * (log_softmax of the masked row at the action). */
int ms_sample_masked(const float* logits, const uint8_t* mask, int64_t N,
                     int32_t A, int64_t row_begin, uint64_t seed,
                     uint64_t counter, int64_t* actions, float* logp,
                     void* stream);

/* Replaces nn.Dropout2d's torch-RNG channel masks in the training forward
 * (cnn_residual.py:14,22; train mode in collect_rollout train_rl.py:221 and in
 * ppo_update ppo.py:25-30). rows int64[N] = GLOBAL sample ids (buffer row
 * t*num_envs_total + global env). Writes out f32[nblk][N][C] = keep / (1-p),
 * keep = u(seed, counter, rows[i], b*C + c) >= p from a counter-based hash, so
 * a data-parallel rank draws exactly the masks its samples get in a one-GPU
 * run. C % 4 == 0, 0 < p < 1. */
int ms_dropout_masks(const int64_t* rows, int64_t N, int32_t nblk, int32_t C,
                     uint64_t seed, uint64_t counter, float p, float* out,
                     void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MSENV_H */
