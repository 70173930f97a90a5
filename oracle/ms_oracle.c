/*
 * ms_oracle.c — TEST INFRASTRUCTURE ONLY. CPU restatement of the reference's
 * hot path, used as the parity checker by tests/, __graft_entry__.smoke() and
 * as bench.py's cpu_baseline leg. The product (minesweeper-ppo_amd/) never
 * links, loads or calls this file.
 *
 * What it restates (reference = yakvrz/minesweeper-ppo under /root/reference):
 *   - numpy 2.2 SeedSequence / PCG64 / random_bounded_uint64 / Generator.choice
 *     (third-party arithmetic used at env.py:49, 309, 393-394). numpy's C
 *     sources are not vendored in the reference; the algorithm restated is
 *     numpy's published one (bit_generator.pyx SeedSequence, pcg64.h
 *     setseq_128 XSL-RR, distributions.c buffered_bounded_lemire_uint32,
 *     _generator.pyx choice -> Floyd + _shuffle_int). Pinned by
 *     tests/golden/ fixtures captured from numpy 2.2.6 + the reference here, and
 *     directly against numpy in tests/test_oracle.py.
 *   - MinesweeperEnv.step (env.py:103-152), _place_mines_safe (env.py:280-312),
 *     _compute_adjacent_counts (env.py:314-335), flood_fill_reveal
 *     (env_numba.py:17-77, the BFS with a `queued` array), _build_obs
 *     (env.py:172-192), _compute_action_mask (env.py:194-196), _build_aux
 *     (env.py:163-170), VecMinesweeper.__init__/reset/step (env.py:382-511),
 *     _apply_late_start (env.py:416-466).
 *   - RolloutBuffer.compute_gae (buffers.py:78-94) in f32 with torch's op order.
 *
 * The C ABI mirrors include/msenv.h with an `mso_` prefix and HOST pointers.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/msenv.h"

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------- */
/* numpy SeedSequence (bit_generator.pyx)                                     */
/* ------------------------------------------------------------------------- */
#define SS_INIT_A 0x43b0d7e5u
#define SS_MULT_A 0x931e8875u
#define SS_INIT_B 0x8b51f9ddu
#define SS_MULT_B 0x58f38dedu
#define SS_MIX_L 0xca01f9ddu
#define SS_MIX_R 0x4973f715u

static uint32_t ss_hashmix(uint32_t value, uint32_t* hc) {
  value ^= *hc;
  *hc *= SS_MULT_A;
  value *= *hc;
  value ^= value >> 16;
  return value;
}

static uint32_t ss_mix(uint32_t x, uint32_t y) {
  uint32_t r = SS_MIX_L * x - SS_MIX_R * y;
  r ^= r >> 16;
  return r;
}

/* entropy = python int `seed` -> little-endian u32 words (0 -> [0]). */
static void seed_sequence_state(uint64_t seed, uint64_t out[4]) {
  uint32_t ent[2];
  int n_ent = 0;
  if (seed == 0) {
    ent[n_ent++] = 0;
  } else {
    while (seed) {
      ent[n_ent++] = (uint32_t)(seed & 0xffffffffu);
      seed >>= 32;
    }
  }
  uint32_t pool[4];
  uint32_t hc = SS_INIT_A;
  for (int i = 0; i < 4; i++) pool[i] = ss_hashmix(i < n_ent ? ent[i] : 0u, &hc);
  for (int s = 0; s < 4; s++)
    for (int d = 0; d < 4; d++)
      if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], &hc));
  /* (n_ent <= 2 < pool size: no trailing entropy words) */
  uint32_t words[8];
  uint32_t hb = SS_INIT_B;
  for (int i = 0; i < 8; i++) {
    uint32_t v = pool[i & 3];
    v ^= hb;
    hb *= SS_MULT_B;
    v *= hb;
    v ^= v >> 16;
    words[i] = v;
  }
  for (int i = 0; i < 4; i++) out[i] = (uint64_t)words[2 * i] | ((uint64_t)words[2 * i + 1] << 32);
}

/* ------------------------------------------------------------------------- */
/* PCG64 (setseq 128, XSL-RR 64) + numpy's next_uint32 half-word buffer       */
/* ------------------------------------------------------------------------- */
typedef struct {
  u128 state, inc;
  int has32;
  uint32_t uinteger;
} pcg64_t;

static const u128 PCG_MULT =
    ((u128)0x2360ED051FC65DA4ULL << 64) | (u128)0x4385DF649FCCF645ULL;

static inline void pcg_step(pcg64_t* r) { r->state = r->state * PCG_MULT + r->inc; }

static inline uint64_t pcg_next64(pcg64_t* r) {
  pcg_step(r);
  uint64_t hi = (uint64_t)(r->state >> 64), lo = (uint64_t)r->state;
  unsigned rot = (unsigned)(hi >> 58);
  uint64_t v = hi ^ lo;
  return (v >> rot) | (v << ((64u - rot) & 63u));
}

static inline uint32_t pcg_next32(pcg64_t* r) {
  if (r->has32) {
    r->has32 = 0;
    return r->uinteger;
  }
  uint64_t n = pcg_next64(r);
  r->has32 = 1;
  r->uinteger = (uint32_t)(n >> 32);
  return (uint32_t)n;
}

static void pcg_seed(pcg64_t* r, uint64_t seed) {
  uint64_t w[4];
  seed_sequence_state(seed, w);
  u128 initstate = ((u128)w[0] << 64) | w[1];
  u128 initseq = ((u128)w[2] << 64) | w[3];
  r->state = 0;
  r->inc = (initseq << 1) | 1u;
  pcg_step(r);
  r->state += initstate;
  pcg_step(r);
  r->has32 = 0;
  r->uinteger = 0;
}

/* random_bounded_uint64(off=0, rng=j, mask=0, use_masked=false), j < 2^32-1 */
static inline uint64_t rng_bounded(pcg64_t* r, uint64_t j) {
  if (j == 0) return 0;
  const uint32_t excl = (uint32_t)j + 1u;
  uint64_t m = (uint64_t)pcg_next32(r) * excl;
  uint32_t left = (uint32_t)m;
  if (left < excl) {
    const uint32_t thr = (uint32_t)(0xffffffffu - (uint32_t)j) % excl;
    while (left < thr) {
      m = (uint64_t)pcg_next32(r) * excl;
      left = (uint32_t)m;
    }
  }
  return m >> 32;
}

static inline double rng_random(pcg64_t* r) {
  return (double)(pcg_next64(r) >> 11) * (1.0 / 9007199254740992.0);
}

/* ---- exported RNG probes (tests compare these against numpy itself) ---- */
static void pcg_export(const pcg64_t* r, uint64_t out[6]) {
  out[0] = (uint64_t)(r->state >> 64);
  out[1] = (uint64_t)r->state;
  out[2] = (uint64_t)(r->inc >> 64);
  out[3] = (uint64_t)r->inc;
  out[4] = (uint64_t)r->has32;
  out[5] = (uint64_t)r->uinteger;
}
static void pcg_import(pcg64_t* r, const uint64_t in[6]) {
  r->state = ((u128)in[0] << 64) | in[1];
  r->inc = ((u128)in[2] << 64) | in[3];
  r->has32 = (int)in[4];
  r->uinteger = (uint32_t)in[5];
}

void mso_seed_state(uint64_t seed, uint64_t out[6]) {
  pcg64_t r;
  pcg_seed(&r, seed);
  pcg_export(&r, out);
}

/* n draws of bounded(j) from `state` (updated in place). */
void mso_bounded_draws(uint64_t state[6], uint64_t j, int64_t n, uint64_t* out) {
  pcg64_t r;
  pcg_import(&r, state);
  for (int64_t i = 0; i < n; i++) out[i] = rng_bounded(&r, j);
  pcg_export(&r, state);
}

void mso_u64_draws(uint64_t state[6], int64_t n, uint64_t* out) {
  pcg64_t r;
  pcg_import(&r, state);
  for (int64_t i = 0; i < n; i++) out[i] = pcg_next64(&r);
  pcg_export(&r, state);
}

/* Generator.choice(pop, K, replace=False) index draws (Floyd + shuffle),
 * pop <= 10000 path of _generator.pyx. out[K] = selected values in numpy's
 * idx order (pre-shuffle values, post-shuffle order). */
void mso_choice_noreplace(uint64_t state[6], int64_t pop, int64_t K, int64_t* out) {
  pcg64_t r;
  pcg_import(&r, state);
  uint8_t* in_set = (uint8_t*)calloc((size_t)(pop > 0 ? pop : 1), 1);
  for (int64_t j = pop - K; j < pop; j++) {
    int64_t v = (int64_t)rng_bounded(&r, (uint64_t)j);
    if (!in_set[v]) {
      in_set[v] = 1;
      out[j - pop + K] = v;
    } else {
      in_set[j] = 1;
      out[j - pop + K] = j;
    }
  }
  for (int64_t i = K - 1; i >= 1; i--) {
    int64_t jj = (int64_t)rng_bounded(&r, (uint64_t)i);
    int64_t t = out[jj];
    out[jj] = out[i];
    out[i] = t;
  }
  free(in_set);
  pcg_export(&r, state);
}

/* default_rng(seed).integers(0, 2**31-1, size=n, dtype=int64) (env.py:393-394) */
void mso_env_seeds(uint64_t base_seed, int64_t n, int64_t* out, uint64_t state_after[6]) {
  pcg64_t r;
  pcg_seed(&r, base_seed);
  for (int64_t i = 0; i < n; i++) out[i] = (int64_t)rng_bounded(&r, 2147483646ULL);
  if (state_after) pcg_export(&r, state_after);
}

/* ------------------------------------------------------------------------- */
/* Environment                                                               */
/* ------------------------------------------------------------------------- */
typedef struct {
  uint8_t* mine;
  uint8_t* revealed;
  uint8_t* counts;
  int first_click;
  int32_t step_count;
  int32_t last_new;
  pcg64_t rng;
} env_t;

typedef struct {
  double prob;
  int32_t min_hidden, max_hidden, max_attempts, max_extra_steps;
} late_cfg_t;

struct mso_vec {
  ms_cfg cfg;
  int64_t n_total, env_begin, n;
  int A;
  env_t* envs;
  uint8_t* pool; /* backing store for the per-env planes */
  /* scratch per thread is allocated on the fly */
  int late_on;
  late_cfg_t late;
  pcg64_t late_rng;
  int late_mode; /* 0 shared generator (the reference), 1 keyed per reset */
  uint64_t late_seed;
};
typedef struct mso_vec mso_vec;

static __thread char g_err[256];
const char* mso_last_error(void) { return g_err; }

/* _compute_adjacent_counts (env.py:314-335): 8-neighbour count, mines incl. */
static void compute_counts(const mso_vec* v, env_t* e) {
  const int H = v->cfg.H, W = v->cfg.W;
  for (int r = 0; r < H; r++)
    for (int c = 0; c < W; c++) {
      int n = 0;
      for (int dr = -1; dr <= 1; dr++)
        for (int dc = -1; dc <= 1; dc++) {
          if (!dr && !dc) continue;
          int rr = r + dr, cc = c + dc;
          if (rr < 0 || rr >= H || cc < 0 || cc >= W) continue;
          n += e->mine[rr * W + cc];
        }
      e->counts[r * W + c] = (uint8_t)n;
    }
}

/* _place_mines_safe (env.py:280-312) */
static void place_mines(const mso_vec* v, env_t* e, int r0, int c0, int64_t* scratch_allowed,
                        int64_t* scratch_idx, uint8_t* scratch_set) {
  const int H = v->cfg.H, W = v->cfg.W, A = v->A, K = v->cfg.mine_count;
  uint8_t forb[4096];
  memset(forb, 0, (size_t)A);
  if (v->cfg.guarantee_safe_neighborhood) {
    for (int dr = -1; dr <= 1; dr++)
      for (int dc = -1; dc <= 1; dc++) {
        int rr = r0 + dr, cc = c0 + dc;
        if (rr >= 0 && rr < H && cc >= 0 && cc < W) forb[rr * W + cc] = 1;
      }
  }
  forb[r0 * W + c0] = 1;
  int pop = 0;
  for (int i = 0; i < A; i++)
    if (!forb[i]) scratch_allowed[pop++] = i;
  if (pop < K) { /* env.py:303-307 relax to the clicked cell only */
    pop = 0;
    for (int i = 0; i < A; i++)
      if (i != r0 * W + c0) scratch_allowed[pop++] = i;
  }
  /* rng.choice(allowed, size=K, replace=False): Floyd + K-1 shuffle draws */
  memset(scratch_set, 0, (size_t)(pop > 0 ? pop : 1));
  for (int j = pop - K; j < pop; j++) {
    int64_t t = (int64_t)rng_bounded(&e->rng, (uint64_t)j);
    if (!scratch_set[t]) {
      scratch_set[t] = 1;
      scratch_idx[j - pop + K] = t;
    } else {
      scratch_set[j] = 1;
      scratch_idx[j - pop + K] = j;
    }
  }
  for (int i = K - 1; i >= 1; i--) { /* consumed draws; the set is unchanged */
    int64_t jj = (int64_t)rng_bounded(&e->rng, (uint64_t)i);
    int64_t t = scratch_idx[jj];
    scratch_idx[jj] = scratch_idx[i];
    scratch_idx[i] = t;
  }
  memset(e->mine, 0, (size_t)A);
  for (int k = 0; k < K; k++) e->mine[scratch_allowed[scratch_idx[k]]] = 1;
  compute_counts(v, e);
}

/* flood_fill_reveal (env_numba.py:17-77). flags are all-False on every
 * reference path (their only writer, _apply_deductions env.py:246, has no
 * callers), so the flags tests are omitted. */
static int flood_fill(const mso_vec* v, env_t* e, int sr, int sc, int32_t* qbuf, uint8_t* queued) {
  const int H = v->cfg.H, W = v->cfg.W;
  if (e->revealed[sr * W + sc]) return 0;
  if (e->mine[sr * W + sc]) return 0;
  memset(queued, 0, (size_t)v->A);
  int head = 0, tail = 0;
  qbuf[tail++] = sr * W + sc;
  queued[sr * W + sc] = 1;
  int newly = 0;
  while (head < tail) {
    int idx = qbuf[head++];
    if (e->revealed[idx]) continue;
    if (e->mine[idx]) continue;
    e->revealed[idx] = 1;
    newly++;
    if (e->counts[idx] == 0) {
      int rr = idx / W, cc = idx % W;
      for (int dr = -1; dr <= 1; dr++)
        for (int dc = -1; dc <= 1; dc++) {
          if (!dr && !dc) continue;
          int nr = rr + dr, nc = cc + dc;
          if (nr < 0 || nr >= H || nc < 0 || nc >= W) continue;
          int n = nr * W + nc;
          if (queued[n]) continue;
          if (e->revealed[n] || e->mine[n]) continue;
          qbuf[tail++] = n;
          queued[n] = 1;
        }
    }
  }
  return newly;
}

static void env_reset(const mso_vec* v, env_t* e) { /* env.py:87-101 */
  memset(e->mine, 0, (size_t)v->A);
  memset(e->revealed, 0, (size_t)v->A);
  memset(e->counts, 0, (size_t)v->A);
  e->first_click = 0;
  e->step_count = 0;
  e->last_new = 0;
}

typedef struct {
  int64_t* allowed;
  int64_t* idx;
  uint8_t* set;
  int32_t* q;
  uint8_t* queued;
} scratch_t;

static void scratch_init(scratch_t* s, int A) {
  s->allowed = (int64_t*)malloc(sizeof(int64_t) * (size_t)A);
  s->idx = (int64_t*)malloc(sizeof(int64_t) * (size_t)A);
  s->set = (uint8_t*)malloc((size_t)A);
  s->q = (int32_t*)malloc(sizeof(int32_t) * (size_t)A);
  s->queued = (uint8_t*)malloc((size_t)A);
}
static void scratch_free(scratch_t* s) {
  free(s->allowed);
  free(s->idx);
  free(s->set);
  free(s->q);
  free(s->queued);
}

static int revealed_sum(const mso_vec* v, const env_t* e) {
  int s = 0;
  for (int i = 0; i < v->A; i++) s += e->revealed[i];
  return s;
}

/* MinesweeperEnv.step (env.py:103-152). Returns reward (double), sets done/outcome. */
static double env_step(const mso_vec* v, env_t* e, int64_t action, int* done, int* outcome,
                       scratch_t* s) {
  const int A = v->A, W = v->cfg.W;
  int64_t cell = action % A; /* python modulo: non-negative for A > 0 */
  if (cell < 0) cell += A;
  int r = (int)(cell / W), c = (int)(cell % W);
  double reward = 0.0;
  *done = 0;
  *outcome = MS_OUTCOME_NONE;
  e->last_new = 0;
  const int total_safe = A - v->cfg.mine_count;
  if (!e->revealed[cell]) {
    if (!e->first_click) {
      place_mines(v, e, r, c, s->allowed, s->idx, s->set);
      e->first_click = 1;
    }
    if (e->mine[cell]) {
      e->revealed[cell] = 1;
      *done = 1;
      *outcome = MS_OUTCOME_LOSS;
      reward += v->cfg.loss_reward;
    } else {
      int newly = flood_fill(v, e, r, c, s->q, s->queued);
      e->last_new = newly;
      if (revealed_sum(v, e) >= total_safe) {
        *done = 1;
        *outcome = MS_OUTCOME_WIN;
        reward += v->cfg.win_reward;
      }
    }
  }
  reward -= v->cfg.step_penalty;
  e->step_count += 1;
  return reward;
}

/* _build_obs (env.py:172-192) + _compute_action_mask (env.py:194-196) */
static void write_obs(const mso_vec* v, const env_t* e, float* obs, uint8_t* mask) {
  const int A = v->A;
  if (obs) {
    memset(obs, 0, sizeof(float) * 10 * (size_t)A);
    for (int i = 0; i < A; i++) {
      if (e->revealed[i]) {
        obs[i] = 1.0f;
        if (e->first_click) obs[(size_t)(1 + e->counts[i]) * A + i] = 1.0f;
      }
    }
  }
  if (mask)
    for (int i = 0; i < A; i++) mask[i] = (uint8_t)!e->revealed[i];
}

static inline uint64_t splitmix64(uint64_t x);

/* MS_LATE_KEYED (include/msenv.h): the reset's own generator, keyed by (late seed, GLOBAL
 * env index, the env's own PCG64 state at the reset) through splitmix64 (keyed_late_pcg in
 * csrc/msenv.hip). A raw PCG64 state (no SeedSequence), has_uint32 = 0. */
static pcg64_t keyed_late_rng(uint64_t seed, uint64_t gidx, const pcg64_t* env_rng) {
  const uint64_t st_hi = (uint64_t)(env_rng->state >> 64), st_lo = (uint64_t)env_rng->state;
  const uint64_t a = splitmix64(seed ^ splitmix64(gidx ^ 0x6C8E9CF570932BD5ULL));
  const uint64_t b = splitmix64(a ^ st_lo);
  const uint64_t c = splitmix64(b ^ st_hi);
  const uint64_t d = splitmix64(c ^ 0xA0761D6478BD642FULL) | 1ULL;
  pcg64_t r;
  r.state = ((u128)a << 64) | b;
  r.inc = ((u128)c << 64) | d;
  r.has32 = 0;
  r.uinteger = 0;
  return r;
}

/* _apply_late_start (env.py:416-466) */
static void apply_late_start(mso_vec* v, env_t* e, scratch_t* s) {
  pcg64_t keyed;
  pcg64_t* rng = &v->late_rng;
  if (v->late_mode == 1) {
    keyed = keyed_late_rng(v->late_seed, (uint64_t)(v->env_begin + (e - v->envs)), &e->rng);
    rng = &keyed;
  }
  const late_cfg_t* L = &v->late;
  if (L->prob <= 0.0 || rng_random(rng) >= L->prob) return;
  int min_h = L->min_hidden < 1 ? 1 : L->min_hidden;
  int max_h = L->max_hidden < min_h ? min_h : L->max_hidden;
  int attempts = L->max_attempts < 1 ? 1 : L->max_attempts;
  int extra = L->max_extra_steps < 1 ? 1 : L->max_extra_steps;
  const int A = v->A;
  const int safe_total = A - v->cfg.mine_count;
  int64_t* cand = s->allowed; /* reuse scratch */
  for (int a = 0; a < attempts; a++) {
    if (e->first_click) env_reset(v, e);
    int first_idx = (int)rng_bounded(rng, (uint64_t)(A - 1));
    int done = 0, oc = 0;
    env_step(v, e, first_idx, &done, &oc, s);
    if (done) continue;
    int target = min_h + (int)rng_bounded(rng, (uint64_t)(max_h - min_h));
    if (target > safe_total) target = safe_total;
    if (target < 1) target = 1;
    int ok = 0;
    for (int k = 0; k < extra; k++) {
      int remaining = safe_total - revealed_sum(v, e);
      if (remaining <= target) {
        ok = 1;
        break;
      }
      int nc = 0;
      for (int i = 0; i < A; i++)
        if (!e->mine[i] && !e->revealed[i]) cand[nc++] = i;
      if (nc == 0) break;
      int64_t idx = cand[rng_bounded(rng, (uint64_t)(nc - 1))];
      env_step(v, e, idx, &done, &oc, s);
      if (done) break;
    }
    if (ok) return;
    int remaining = safe_total - revealed_sum(v, e);
    if (!done && remaining <= target) return;
  }
  env_reset(v, e);
}

static void reset_env_state(mso_vec* v, env_t* e, scratch_t* s) { /* env.py:406-414 */
  env_reset(v, e);
  if (v->late_on) apply_late_start(v, e, s);
}

/* ------------------------------------------------------------------------- */
/* Vec API                                                                   */
/* ------------------------------------------------------------------------- */
int mso_create(const ms_cfg* cfg, int64_t n_total, uint64_t base_seed, int64_t env_begin,
               int64_t env_count, mso_vec** out) {
  if (!cfg || !out || n_total <= 0 || env_begin < 0 || env_count <= 0 ||
      env_begin + env_count > n_total || cfg->H <= 0 || cfg->W <= 0 || cfg->H * cfg->W > 4096 ||
      cfg->mine_count < 0 || cfg->mine_count >= cfg->H * cfg->W) {
    snprintf(g_err, sizeof g_err, "mso_create: invalid arguments");
    return MS_EINVAL;
  }
  mso_vec* v = (mso_vec*)calloc(1, sizeof(mso_vec));
  v->cfg = *cfg;
  v->n_total = n_total;
  v->env_begin = env_begin;
  v->n = env_count;
  v->A = cfg->H * cfg->W;
  v->envs = (env_t*)calloc((size_t)env_count, sizeof(env_t));
  v->pool = (uint8_t*)calloc((size_t)env_count * 3 * (size_t)v->A, 1);
  int64_t* seeds = (int64_t*)malloc(sizeof(int64_t) * (size_t)n_total);
  mso_env_seeds(base_seed, n_total, seeds, NULL);
  for (int64_t i = 0; i < env_count; i++) {
    env_t* e = &v->envs[i];
    e->mine = v->pool + (size_t)i * 3 * v->A;
    e->revealed = e->mine + v->A;
    e->counts = e->revealed + v->A;
    pcg_seed(&e->rng, (uint64_t)seeds[env_begin + i]);
  }
  free(seeds);
  *out = v;
  return MS_OK;
}

/* Late start (env.py:397-403; train_rl.py:350-361 passes seed+1). */
int mso_set_late_start(mso_vec* v, double prob, int32_t min_hidden, int32_t max_hidden,
                       int32_t max_attempts, int32_t max_extra_steps, uint64_t late_seed) {
  v->late_on = 1;
  v->late.prob = prob;
  v->late.min_hidden = min_hidden;
  v->late.max_hidden = max_hidden;
  v->late.max_attempts = max_attempts;
  v->late.max_extra_steps = max_extra_steps;
  pcg_seed(&v->late_rng, late_seed);
  v->late_seed = late_seed;
  return MS_OK;
}

int mso_set_late_start_mode(mso_vec* v, int32_t mode) {
  if (mode != 0 && mode != 1) {
    snprintf(g_err, sizeof g_err, "mso_set_late_start_mode: bad mode");
    return MS_EINVAL;
  }
  v->late_mode = mode;
  return MS_OK;
}

void mso_destroy(mso_vec* v) {
  if (!v) return;
  free(v->pool);
  free(v->envs);
  free(v);
}

int mso_reset(mso_vec* v, float* obs, uint8_t* mask) { /* env.py:468-477 */
  scratch_t s;
  scratch_init(&s, v->A);
  for (int64_t i = 0; i < v->n; i++) {
    reset_env_state(v, &v->envs[i], &s);
    write_obs(v, &v->envs[i], obs ? obs + (size_t)i * 10 * v->A : NULL,
              mask ? mask + (size_t)i * v->A : NULL);
  }
  scratch_free(&s);
  return MS_OK;
}

typedef struct {
  mso_vec* v;
  int64_t b, e;
  const int64_t* a64;
  const int32_t* a32;
  float* obs;
  uint8_t* mask;
  float* reward;
  uint8_t* done;
  int32_t* step;
  int32_t* last_new;
  double* frac;
  int8_t* outcome;
} step_job_t;

static void step_range(step_job_t* j) {
  mso_vec* v = j->v;
  scratch_t s;
  scratch_init(&s, v->A);
  const int A = v->A;
  for (int64_t i = j->b; i < j->e; i++) {
    env_t* e = &v->envs[i];
    int64_t a = j->a64 ? j->a64[i] : (int64_t)j->a32[i];
    int done, oc;
    double rew = env_step(v, e, a, &done, &oc, &s);
    /* aux is built before the auto-reset (env.py:492-505) */
    if (j->step) j->step[i] = e->step_count;
    if (j->last_new) j->last_new[i] = e->last_new;
    if (j->frac) j->frac[i] = (double)revealed_sum(v, e) / (double)(A > 1 ? A : 1);
    if (j->reward) j->reward[i] = (float)rew;
    if (j->done) j->done[i] = (uint8_t)done;
    if (j->outcome) j->outcome[i] = (int8_t)(done ? oc : MS_OUTCOME_NONE);
    if (done) reset_env_state(v, e, &s);
    write_obs(v, e, j->obs ? j->obs + (size_t)i * 10 * A : NULL,
              j->mask ? j->mask + (size_t)i * A : NULL);
  }
  scratch_free(&s);
}

static void* step_thread(void* p) {
  step_job_t* j = (step_job_t*)p;
  step_range(j);
  return NULL;
}

/* VecMinesweeper.step (env.py:479-511). nthreads > 1 splits the envs into
 * contiguous chunks (the CPU baseline); late start forces nthreads = 1 since
 * it shares one RNG stream across envs in env order. */
static int step_impl(mso_vec* v, const int64_t* a64, const int32_t* a32, float* obs,
                     uint8_t* mask, float* reward, uint8_t* done, int32_t* step,
                     int32_t* last_new, double* frac, int8_t* outcome, int nthreads) {
  if (!v || (!a64 && !a32)) {
    snprintf(g_err, sizeof g_err, "mso_step: null argument");
    return MS_EINVAL;
  }
  if (nthreads < 1 || (v->late_on && v->late_mode == 0)) nthreads = 1; /* the shared generator is a serial chain */
  if (nthreads > v->n) nthreads = (int)v->n;
  step_job_t jobs[256];
  pthread_t th[256];
  if (nthreads > 256) nthreads = 256;
  for (int t = 0; t < nthreads; t++) {
    step_job_t* j = &jobs[t];
    j->v = v;
    j->b = v->n * t / nthreads;
    j->e = v->n * (t + 1) / nthreads;
    j->a64 = a64;
    j->a32 = a32;
    j->obs = obs;
    j->mask = mask;
    j->reward = reward;
    j->done = done;
    j->step = step;
    j->last_new = last_new;
    j->frac = frac;
    j->outcome = outcome;
  }
  if (nthreads == 1) {
    step_range(&jobs[0]);
    return MS_OK;
  }
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, step_thread, &jobs[t]);
  step_range(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
  return MS_OK;
}

int mso_step(mso_vec* v, const int64_t* actions, float* obs, uint8_t* mask, float* reward,
             uint8_t* done, int32_t* step, int32_t* last_new, double* frac, int8_t* outcome,
             int32_t nthreads) {
  return step_impl(v, actions, NULL, obs, mask, reward, done, step, last_new, frac, outcome,
                   nthreads);
}

int mso_step_i32(mso_vec* v, const int32_t* actions, float* obs, uint8_t* mask, float* reward,
                 uint8_t* done, int32_t* step, int32_t* last_new, double* frac, int8_t* outcome,
                 int32_t nthreads) {
  return step_impl(v, NULL, actions, obs, mask, reward, done, step, last_new, frac, outcome,
                   nthreads);
}

/* collect_rollout label capture (train_rl.py:203-219) */
int mso_labels(mso_vec* v, float* labels, uint8_t* valid) {
  const int A = v->A;
  for (int64_t i = 0; i < v->n; i++) {
    const env_t* e = &v->envs[i];
    for (int k = 0; k < A; k++) {
      if (labels) labels[(size_t)i * A + k] = e->first_click ? (float)e->mine[k] : 0.0f;
      if (valid) valid[(size_t)i * A + k] = e->first_click ? (uint8_t)!e->revealed[k] : 0;
    }
  }
  return MS_OK;
}

int mso_snapshot(mso_vec* v, uint8_t* mine, uint8_t* revealed, uint8_t* counts,
                 uint8_t* first_click, int32_t* step_count) {
  const int A = v->A;
  for (int64_t i = 0; i < v->n; i++) {
    const env_t* e = &v->envs[i];
    if (mine) memcpy(mine + (size_t)i * A, e->mine, (size_t)A);
    if (revealed) memcpy(revealed + (size_t)i * A, e->revealed, (size_t)A);
    if (counts) memcpy(counts + (size_t)i * A, e->counts, (size_t)A);
    if (first_click) first_click[i] = (uint8_t)e->first_click;
    if (step_count) step_count[i] = e->step_count;
  }
  return MS_OK;
}

int mso_rng_state(mso_vec* v, uint64_t* out) {
  for (int64_t i = 0; i < v->n; i++) pcg_export(&v->envs[i].rng, out + 6 * i);
  return MS_OK;
}

/* ------------------------------------------------------------------------- */
/* Synthetic action tape                                      */
/* ------------------------------------------------------------------------- */
static inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

uint64_t mso_splitmix64(uint64_t x) { return splitmix64(x); }

/* SURVEY.md §8d action tape for env i at step t (same rule as ms_tape_actions) */
static int64_t tape_one(const mso_vec* v, int64_t i, uint64_t t, int32_t mode) {
  const int A = v->A;
  const env_t* e = &v->envs[i];
  uint64_t g = (uint64_t)(v->env_begin + i);
  uint64_t x = splitmix64(0xC0FFEEULL ^ (g << 32) ^ t);
  int n_valid = 0, n_safe = 0;
  for (int k = 0; k < A; k++) {
    n_valid += !e->revealed[k];
    n_safe += (!e->revealed[k] && !e->mine[k]);
  }
  int want_safe = (mode == MS_TAPE_SAFE_BIASED) && ((x & 0xFFFFu) < 65208u) && n_safe > 0;
  int64_t act = 0;
  if (want_safe) {
    int target = (int)((x >> 16) % (uint64_t)n_safe);
    for (int k = 0; k < A; k++)
      if (!e->revealed[k] && !e->mine[k] && target-- == 0) {
        act = k;
        break;
      }
  } else if (n_valid > 0) {
    uint64_t sel = (mode == MS_TAPE_SAFE_BIASED) ? (x >> 16) : x;
    int target = (int)(sel % (uint64_t)n_valid);
    for (int k = 0; k < A; k++)
      if (!e->revealed[k] && target-- == 0) {
        act = k;
        break;
      }
  }
  return act;
}

/* CPU baseline (bench.py cpu_baseline): `steps` consecutive (tape action, board step) pairs
 * for every env, on a pool of nthreads threads that each own a contiguous block of envs for
 * the whole run. Envs are independent (no shared RNG without late start), so the threads
 * never synchronise: the per-env sequential algorithm of env_numba / env.py, one env per
 * task, over every core given. Outputs go to caller buffers sized for all envs (each env's
 * slot is overwritten every step). */
typedef struct {
  step_job_t j;
  uint64_t t0;
  int64_t steps;
  int32_t mode;
} run_job_t;

static void* run_thread(void* p) {
  run_job_t* r = (run_job_t*)p;
  step_job_t* j = &r->j;
  int64_t* act = (int64_t*)malloc(sizeof(int64_t) * (size_t)(j->e > j->b ? j->e : 1));
  if (!act) return NULL;
  int64_t* a_full = act - j->b;  /* index by global env id within this handle */
  j->a64 = a_full;
  for (int64_t s = 0; s < r->steps; s++) {
    for (int64_t i = j->b; i < j->e; i++) a_full[i] = tape_one(j->v, i, r->t0 + (uint64_t)s, r->mode);
    step_range(j);
  }
  free(act);
  return NULL;
}

int mso_run_baseline(mso_vec* v, uint64_t t0, int64_t steps, int32_t mode, int32_t nthreads, float* obs,
                     uint8_t* mask, float* reward, uint8_t* done, int32_t* step, int32_t* last_new,
                     double* frac, int8_t* outcome) {
  if (!v || steps < 0) {
    snprintf(g_err, sizeof g_err, "mso_run_baseline: bad argument");
    return MS_EINVAL;
  }
  if (nthreads < 1 || (v->late_on && v->late_mode == 0)) nthreads = 1; /* the shared generator is a serial chain */
  if (nthreads > v->n) nthreads = (int)v->n;
  if (nthreads > 1024) nthreads = 1024;
  run_job_t* jobs = (run_job_t*)calloc((size_t)nthreads, sizeof(run_job_t));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  if (!jobs || !th) {
    free(jobs);
    free(th);
    snprintf(g_err, sizeof g_err, "mso_run_baseline: out of memory");
    return MS_EINVAL;
  }
  for (int t = 0; t < nthreads; t++) {
    step_job_t* j = &jobs[t].j;
    j->v = v;
    j->b = v->n * t / nthreads;
    j->e = v->n * (t + 1) / nthreads;
    j->obs = obs;
    j->mask = mask;
    j->reward = reward;
    j->done = done;
    j->step = step;
    j->last_new = last_new;
    j->frac = frac;
    j->outcome = outcome;
    jobs[t].t0 = t0;
    jobs[t].steps = steps;
    jobs[t].mode = mode;
  }
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, run_thread, &jobs[t]);
  run_thread(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
  free(jobs);
  free(th);
  return MS_OK;
}

int mso_tape_actions(mso_vec* v, uint64_t t, int32_t mode, int64_t* actions) {
  for (int64_t i = 0; i < v->n; i++) {
    actions[i] = tape_one(v, i, t, mode);
  }
  return MS_OK;
}

/* ------------------------------------------------------------------------- */
/* GAE (buffers.py:78-94), f32, torch op order, no FMA contraction            */
/* ------------------------------------------------------------------------- */
#pragma GCC push_options
#pragma GCC optimize("fp-contract=off")
void mso_gae(const float* rewards, const float* values, const uint8_t* dones,
             const float* last_values, int32_t T, int64_t N, float gamma, float gamma_lambda,
             float* adv, float* ret) {
  for (int64_t n = 0; n < N; n++) {
    volatile float last_adv = 0.0f;
    for (int t = T - 1; t >= 0; t--) {
      float nv = (t == T - 1) ? last_values[n] : values[(size_t)(t + 1) * N + n];
      float nnt = 1.0f - (float)dones[(size_t)t * N + n];
      volatile float t1 = gamma * nv;
      volatile float t2 = t1 * nnt;
      volatile float t3 = rewards[(size_t)t * N + n] + t2;
      volatile float delta = t3 - values[(size_t)t * N + n];
      volatile float t4 = gamma_lambda * nnt;
      volatile float t5 = t4 * last_adv;
      last_adv = delta + t5;
      adv[(size_t)t * N + n] = last_adv;
    }
  }
  for (int64_t i = 0; i < (int64_t)T * N; i++) ret[i] = adv[i] + values[i];
}
#pragma GCC pop_options

/* Probe: MinesweeperEnv(cfg, seed)._place_mines_safe((r, c)) on a fresh env
 * (env.py:41-77, 280-335). Writes mine/counts u8[A] and the RNG state after. */
int mso_place_probe(const ms_cfg* cfg, uint64_t seed, int32_t r, int32_t c, uint8_t* mine_out,
                    uint8_t* counts_out, uint64_t state_out[6]) {
  mso_vec v;
  memset(&v, 0, sizeof v);
  v.cfg = *cfg;
  v.A = cfg->H * cfg->W;
  v.n = 1;
  env_t e;
  memset(&e, 0, sizeof e);
  e.mine = mine_out;
  e.counts = counts_out;
  uint8_t rev[4096];
  memset(rev, 0, sizeof rev);
  e.revealed = rev;
  pcg_seed(&e.rng, seed);
  scratch_t s;
  scratch_init(&s, v.A);
  place_mines(&v, &e, r, c, s.allowed, s.idx, s.set);
  scratch_free(&s);
  pcg_export(&e.rng, state_out);
  return MS_OK;
}
