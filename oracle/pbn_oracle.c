/*
 * pbn_oracle.c -- CPU restatement of the batched PBN env step.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP path
 * in pbn_rl_amd/csrc: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product path never links or calls it.
 *
 * What it restates.  The reference's env step lives in the external package
 * gym_PBN (requirements.txt:11), which is absent from /root/reference and not
 * installed, so the transition itself is PARITY-UNPINNED by the reference; it
 * follows the frozen semantics of DESIGN.md "Step semantics" (SURVEY.md
 * Appendix C).  The parts that are pinned by the reference are cited inline:
 *   - action encoding 0 = no-op, a > 0 flips node a-1, duplicates removed
 *     (bdq_model/__init__.py:76-84,176);
 *   - per-node probabilistic rule selection among weighted functions
 *     (weights as passed at train_assa_BQN.py:109,121-124);
 *   - truncation at horizon (train_BDQ.py:50, counted at bdq_model/__init__.py:179-180);
 *   - termination = s' in the target attractor (model_tester.py:616 in_target);
 *   - wildcard '*' -> 0 in attractor states (model_tester.py:609), applied by
 *     the Python side before it builds the descriptor.
 * Philox4x32-R follows the Random123 definition (Salmon et al., SC'11); every
 * stream draws R = 7 rounds (DESIGN.md "RNG").  The round function is pinned by
 * rocRAND's philox4x32_10 engine (R = 10) and Random123's known-answer vectors
 * (R = 7 and 10) in tests/test_philox.py.
 *
 * Written for clarity: scalar per env, the group selection words recomputed
 * per group of 32 envs (the unit the semantics defines), OpenMP over groups.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/pbn_env.h"

enum { STREAM_SEL = 0, STREAM_ENV = 1, STREAM_PERT = 2, STREAM_RESET = 3, STREAM_SETTLE_SEL = 5, STREAM_SETTLE_ENV = 6 };

/* every stream draws Philox4x32-7 (DESIGN.md "RNG"); the KAT export runs any round count */
enum { PHILOX_ROUNDS = 7 };

static void philox4x32_r(const uint32_t ctr_in[4], uint32_t k0, uint32_t k1, uint32_t out[4], int rounds) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  for (int r = 0; r < rounds; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  philox4x32_r(ctr, key[0], key[1], out, 10);
}

void oracle_philox4x32_r(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4], int rounds) {
  philox4x32_r(ctr, key[0], key[1], out, rounds);
}

static void draw(uint64_t seed, uint64_t id, uint64_t step, uint32_t stream, uint32_t idx,
                 uint32_t out[4]) {
  uint32_t ctr[4];
  ctr[0] = (uint32_t)id;
  ctr[1] = (uint32_t)step;
  ctr[2] = (stream << 28) | (idx & 0x0FFFFFFFu);
  ctr[3] = (uint32_t)((id >> 32) & 0xFFFFu) | (uint32_t)(((step >> 32) & 0xFFFFu) << 16);
  philox4x32_r(ctr, (uint32_t)seed, (uint32_t)(seed >> 32), out, PHILOX_ROUNDS);
}

static int words_of(int n) { return (n + 31) / 32; }

static int gap_of(const pbn_net_desc* d, uint32_t u) {
  /* smallest m in 1..N with u < C[m]; N+1 if none */
  for (int m = 1; m <= d->n_nodes; ++m)
    if (u < d->perturb_cdf[m - 1]) return m;
  return d->n_nodes + 1;
}

/* plane reference r: node r of s (r < N), else the value of gate r - N (gv) */
static int plane_of(const pbn_net_desc* d, int r, const uint32_t* s, const uint8_t* gv) {
  return r < d->n_nodes ? (int)((s[r >> 5] >> (r & 31)) & 1u) : gv[r - d->n_nodes];
}

/* the combinational gates of the lowered wide functions, in order (gate g reads gates < g) */
static void eval_gates(const pbn_net_desc* d, const uint32_t* s, uint8_t* gv) {
  for (int g = 0; g < d->n_gates; ++g) {
    uint32_t m = 0;
    for (int j = 0; j < d->gate_arity[g]; ++j) m |= (uint32_t)plane_of(d, d->gate_inputs[4 * g + j], s, gv) << j;
    gv[g] = (uint8_t)((d->gate_table[g] >> m) & 1u);
  }
}

static int eval_func(const pbn_net_desc* d, int f, const uint32_t* s, const uint8_t* gv) {
  int k = d->func_arity[f];
  uint32_t m = 0;
  for (int j = 0; j < k; ++j) m |= (uint32_t)plane_of(d, d->func_inputs[4 * f + j], s, gv) << j;
  return (int)((d->func_table[f] >> m) & 1u);
}

/* attractor id of state s, or -1 */
static int attractor_of(const pbn_net_desc* d, const uint32_t* s, int W) {
  for (int a = 0; a < d->n_attractors; ++a) {
    for (int k = d->attractor_start[a]; k < d->attractor_start[a + 1]; ++k) {
      int eq = 1;
      for (int w = 0; w < W; ++w)
        if (d->attractor_states[(size_t)k * W + w] != s[w]) { eq = 0; break; }
      if (eq) return a;
    }
  }
  return -1;
}

static void valid_mask(int n, int W, uint32_t* m) {
  for (int w = 0; w < W; ++w) {
    int bits = n - 32 * w;
    m[w] = bits >= 32 ? 0xFFFFFFFFu : (bits <= 0 ? 0u : ((1u << bits) - 1u));
  }
}

/* one bounded draw from a 64-bit uniform X = (hi:lo), keeping the rest of X for the next:
 * v = floor(X * K / 2^64) in [0, K), X <- X * K mod 2^64 (multiply-shift "batched dice rolls",
 * Brackett-Rozinsky & Lemire 2024, without rejection): bias <= K / 2^64 per draw */
static uint32_t ext64(uint32_t* hi, uint32_t* lo, uint32_t K) {
  uint64_t a = (uint64_t)(*lo) * K;
  uint64_t b = (uint64_t)(*hi) * K + (a >> 32);
  *lo = (uint32_t)a;
  *hi = (uint32_t)b;
  return (uint32_t)(b >> 32);
}

/* the attractor draws of a reset from the 64-bit uniform X = (hi:lo), advancing X: start
 * attractor a_s and target a_t != a_s in one draw over the A(A-1) pairs (A >= 2), then the start
 * state uniformly within a_s; *sidx = its row in attractor_states (A >= 1) */
static void reset_draw(const pbn_net_desc* d, uint32_t* hi, uint32_t* lo, int* sidx, uint8_t* target) {
  int A = d->n_attractors;
  uint32_t as = 0, at = 0;
  if (A >= 2) {
    uint32_t c = ext64(hi, lo, (uint32_t)A * (uint32_t)(A - 1));
    as = c / (uint32_t)(A - 1);
    at = c % (uint32_t)(A - 1);
    at += (at >= as);
  }
  int start = d->attractor_start[as];
  uint32_t size = (uint32_t)(d->attractor_start[as + 1] - start);
  uint32_t idx = ext64(hi, lo, size);
  *sidx = start + (int)idx;
  *target = (uint8_t)at;
}

/* pbn_reset: the attractor draws from RESET call 0 words 1:0, or (no attractors) a uniform
 * random state from RESET call 1 */
static void reset_one(const pbn_net_desc* d, uint64_t seed, uint64_t e, uint64_t step, uint32_t hi, uint32_t lo,
                      uint32_t* state, uint8_t* target) {
  int N = d->n_nodes, W = words_of(N), A = d->n_attractors;
  uint32_t vm[4];
  valid_mask(N, W, vm);
  if (A >= 1) {
    int sidx;
    reset_draw(d, &hi, &lo, &sidx, target);
    for (int w = 0; w < W; ++w) state[w] = d->attractor_states[(size_t)sidx * W + w];
  } else {
    uint32_t r[4];
    draw(seed, e, step, STREAM_RESET, 1, r);
    for (int w = 0; w < W; ++w) state[w] = r[w] & vm[w];
    *target = PBN_NO_TARGET;
  }
}

int oracle_reset(const pbn_net_desc* d, uint64_t seed, uint64_t step, uint64_t env_offset,
                 int64_t n, uint32_t* state, uint8_t* target, uint8_t* t) {
  int W = words_of(d->n_nodes);
  for (int64_t i = 0; i < n; ++i) {
    uint64_t e = env_offset + (uint64_t)i;
    uint32_t r[4], s[4];
    draw(seed, e, step, STREAM_RESET, 0, r);
    reset_one(d, seed, e, step, r[1], r[0], s, &target[i]);
    for (int w = 0; w < W; ++w) state[(size_t)w * n + i] = s[w];
    t[i] = 0;
  }
  return 0;
}

/* the rule update of every node from state s1 and the nodes' B-bit selection uniforms U[i]
 * (function j = min{j : U[i] < c_ij}) */
static void rule_update(const pbn_net_desc* d, const uint32_t* s1, const uint32_t* U, uint32_t* sp) {
  const int N = d->n_nodes, W = words_of(N);
  uint8_t gv[PBN_MAX_GATES];
  eval_gates(d, s1, gv);
  for (int w = 0; w < W; ++w) sp[w] = 0;
  for (int i = 0; i < N; ++i) {
    int f0 = d->node_func_start[i], nf = d->node_func_start[i + 1] - f0, j = 0;
    while (j < nf - 1 && !(U[i] < d->func_threshold[f0 + j])) ++j;
    if (eval_func(d, f0 + j, s1, gv)) sp[i >> 5] |= 1u << (i & 31);
  }
}

/* one-update law: selection digit words of group G (SEL call 4i + c, word d & 3 = digit plane
 * 4c + d, digit 0 the MSB), and env bit b's uniforms U[i] from them */
static void group_digits(const pbn_net_desc* d, uint64_t seed, uint64_t G, uint64_t step, uint32_t D[][16]) {
  const int N = d->n_nodes, B = d->prob_bits;
  for (int i = 0; i < N; ++i) {
    int nf = d->node_func_start[i + 1] - d->node_func_start[i];
    if (nf < 2) continue;
    for (int c = 0; c < B / 4; ++c) draw(seed, G, step, STREAM_SEL, (uint32_t)(4 * i + c), &D[i][4 * c]);
  }
}

static void group_uniforms(const pbn_net_desc* d, uint32_t D[][16], int b, uint32_t* U) {
  const int N = d->n_nodes, B = d->prob_bits;
  for (int i = 0; i < N; ++i) {
    int nf = d->node_func_start[i + 1] - d->node_func_start[i];
    U[i] = 0;
    if (nf < 2) continue;
    for (int dd = 0; dd < B; ++dd) U[i] |= ((D[i][dd] >> b) & 1u) << (B - 1 - dd);
  }
}

/* settle law: env e's uniforms of update k of its step, keyed per env (DESIGN.md "Step law"):
 * node i's is the top B bits of 16-bit field i & 1 of word (i >> 1) & 3 of SETTLE_SEL call
 * (k << 8 | i >> 3) */
static void env_uniforms(const pbn_net_desc* d, uint64_t seed, uint64_t e, uint64_t step, int k, uint32_t* U) {
  const int N = d->n_nodes, B = d->prob_bits;
  uint32_t P[4];
  for (int i = 0; i < N; ++i) {
    if ((i & 7) == 0) draw(seed, e, step, STREAM_SETTLE_SEL, ((uint32_t)k << 8) | (uint32_t)(i >> 3), P);
    U[i] = ((P[(i >> 1) & 3] >> (16 * (i & 1))) & 0xFFFFu) >> (16 - B);
  }
}

/* settle law (settle_max >= 2): updates k = 1 .. settle_max-1 of env e from sp until sp is a
 * state of some attractor.  Update k: perturbation gaps j = 0, 1, ... from SETTLE_ENV call
 * ((k-1) << 8 | j >> 2), word j & 3; unperturbed, the rule update with env e's SETTLE_SEL
 * uniforms of update k.  Returns 1 if still outside every attractor after the last update;
 * *nupd counts the updates applied. */
static int settle(const pbn_net_desc* d, uint64_t seed, uint64_t e, uint64_t step, uint32_t* sp, int* perturbed,
                  int* nupd) {
  const int N = d->n_nodes, W = words_of(N);
  for (int k = 1; k < d->settle_max; ++k) {
    if (attractor_of(d, sp, W) >= 0) return 0;
    uint32_t gam[4] = {0, 0, 0, 0}, P[4];
    int pos = -1;
    for (int j = 0; pos < N - 1; ++j) {
      if ((j & 3) == 0) draw(seed, e, step, STREAM_SETTLE_ENV, ((uint32_t)(k - 1) << 8) | (uint32_t)(j >> 2), P);
      pos += gap_of(d, P[j & 3]);
      if (pos >= N) break;
      gam[pos >> 5] |= 1u << (pos & 31);
    }
    int pk = 0;
    for (int w = 0; w < W; ++w) pk |= gam[w] != 0;
    if (pk) {
      for (int w = 0; w < W; ++w) sp[w] ^= gam[w];
      *perturbed = 1;
    } else {
      uint32_t U[PBN_MAX_NODES], x[4];
      env_uniforms(d, seed, e, step, k, U);
      rule_update(d, sp, U, x);
      for (int w = 0; w < W; ++w) sp[w] = x[w];
    }
    ++*nupd;
  }
  return attractor_of(d, sp, W) < 0;
}

/* one env step of every env; updates (nullable) = the synchronous updates applied per env
 * (1, or the settle length under the settle law: pbn_rollout_ex's d_updates) */
int oracle_step_ex(const pbn_net_desc* d, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n,
                   uint32_t mode, const uint32_t* state, uint32_t* flipmask, uint8_t* target, uint8_t* t,
                   uint32_t* state_out, uint32_t* final_state, float* reward, uint8_t* flags, uint16_t* updates,
                   int n_threads) {
  const int N = d->n_nodes, W = words_of(N);
  if ((env_offset & 31u) || (n & 31)) return PBN_EINVAL;
  if (d->settle_max < 0 || d->settle_max > PBN_MAX_SETTLE) return PBN_EINVAL;
  const int64_t n_groups = n / 32;
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(static)
#endif
  for (int64_t g = 0; g < n_groups; ++g) {
    const uint64_t G = (env_offset >> 5) + (uint64_t)g;
    /* one-update law: the selection digit words of this group: D[i][d], digit d = 0 is the MSB
     * of u; the settle law keys every update's selection per env (env_uniforms) */
    const int settle_law = d->settle_max >= 2;
    uint32_t D[PBN_MAX_NODES][16];
    if (!settle_law) group_digits(d, seed, G, step, D);
    for (int b = 0; b < 32; ++b) {
      const int64_t li = g * 32 + b;
      const uint64_t e = env_offset + (uint64_t)li;
      uint32_t vm[4], s[4] = {0, 0, 0, 0}, m[4] = {0, 0, 0, 0}, s1[4], gam[4] = {0, 0, 0, 0},
               sp[4] = {0, 0, 0, 0};
      valid_mask(N, W, vm);
      /* one ENV call per env-step: words 0, 1 are the first two perturbation gaps; words 3:2
       * are a 64-bit uniform X from which, in this order, the action draw, the autoreset draws
       * and the third gap's uniform (the top word of what remains of X) are taken */
      uint32_t E[4];
      draw(seed, e, step, STREAM_ENV, 0, E);
      for (int w = 0; w < W; ++w) s[w] = state[(size_t)w * n + li] & vm[w];
      uint32_t hi = E[3], lo = E[2], n1 = (uint32_t)(N + 1);
      uint32_t c = ext64(&hi, &lo, n1 * n1 * n1);   /* drawn in every mode */
      int rs_idx = 0;
      uint8_t rs_tg = PBN_NO_TARGET;
      if (d->n_attractors >= 1) reset_draw(d, &hi, &lo, &rs_idx, &rs_tg);
      const uint32_t u2 = hi;
      /* 1-2. interventions: 0 = no-op, a > 0 flips node a-1, each distinct node once
       *      (bdq_model/__init__.py:76-84 explore branch, :176 action.unique()) */
      if (mode & PBN_MODE_RANDOM_ACTIONS) {
        /* three actions uniform on [0, N] (np.random.randint(0, N+1, 3), bdq_model/__init__.py:76):
         * the base-(N+1) digits of one draw over (N+1)^3 */
        for (int k = 0; k < 3; ++k) {
          uint32_t a = c % n1;
          c /= n1;
          if (a > 0) m[(a - 1) >> 5] |= 1u << ((a - 1) & 31);
        }
        for (int w = 0; w < W; ++w) flipmask[(size_t)w * n + li] = m[w];
      } else {
        for (int w = 0; w < W; ++w) m[w] = flipmask[(size_t)w * n + li] & vm[w];
      }
      for (int w = 0; w < W; ++w) s1[w] = s[w] ^ m[w];
      /* 3. perturbation: gaps between flipped nodes are geometric(p) draws; gaps 0, 1 are ENV
       *    words 0, 1, gap 2 is u2, gap k >= 3 is PERT call (k-3)>>2, word (k-3)&3 */
      {
        int pos = -1, k = 0;
        uint32_t P[4];
        while (pos < N - 1) {
          uint32_t u;
          if (k < 2) u = E[k];
          else if (k == 2) u = u2;
          else {
            if (((k - 3) & 3) == 0) draw(seed, e, step, STREAM_PERT, (uint32_t)((k - 3) >> 2), P);
            u = P[(k - 3) & 3];
          }
          ++k;
          pos += gap_of(d, u);
          if (pos >= N) break;
          gam[pos >> 5] |= 1u << (pos & 31);
        }
      }
      int perturbed = 0;
      for (int w = 0; w < W; ++w) perturbed |= gam[w] != 0;
      /* 4. transition */
      if (perturbed) {
        for (int w = 0; w < W; ++w) sp[w] = s1[w] ^ gam[w];
      } else {
        uint32_t U[PBN_MAX_NODES];
        if (settle_law) env_uniforms(d, seed, e, step, 0, U);
        else group_uniforms(d, D, b, U);
        rule_update(d, s1, U, sp);
      }
      int nupd = 1;
      int unsettled = settle_law ? settle(d, seed, e, step, sp, &perturbed, &nupd) : 0;
      if (updates) updates[li] = (uint16_t)nupd;
      /* 5. reward / termination */
      int a = attractor_of(d, sp, W);
      int in_attr = a >= 0;
      int term = in_attr && (uint32_t)a == target[li];
      int tt = t[li] + 1;
      if (tt > 255) tt = 255;
      int trunc = d->horizon > 0 && tt >= d->horizon;
      int wrong = in_attr && !term;
      int pc = 0;
      for (int w = 0; w < W; ++w) pc += __builtin_popcount(m[w]);
      reward[li] = d->reward_table[(2 * term + wrong) * (N + 1) + pc];
      uint8_t fl = (uint8_t)(term | (trunc << 1) | (in_attr << 2) | (perturbed << 3) | (unsettled << 5));
      if (final_state)
        for (int w = 0; w < W; ++w) final_state[(size_t)w * n + li] = sp[w];
      if ((mode & PBN_MODE_AUTORESET) && (term || trunc)) {
        if (d->n_attractors >= 1) {
          for (int w = 0; w < W; ++w) state_out[(size_t)w * n + li] = d->attractor_states[(size_t)rs_idx * W + w];
          target[li] = rs_tg;
        } else {
          uint32_t r[4];
          draw(seed, e, step, STREAM_RESET, 1, r);
          for (int w = 0; w < W; ++w) state_out[(size_t)w * n + li] = r[w] & vm[w];
          target[li] = PBN_NO_TARGET;
        }
        t[li] = 0;
        fl |= PBN_FLAG_RESET;
      } else {
        for (int w = 0; w < W; ++w) state_out[(size_t)w * n + li] = sp[w];
        t[li] = (uint8_t)tt;
      }
      flags[li] = fl;
    }
  }
  return 0;
}

int oracle_step(const pbn_net_desc* d, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n,
                uint32_t mode, const uint32_t* state, uint32_t* flipmask, uint8_t* target, uint8_t* t,
                uint32_t* state_out, uint32_t* final_state, float* reward, uint8_t* flags, int n_threads) {
  return oracle_step_ex(d, seed, step, env_offset, n, mode, state, flipmask, target, t, state_out, final_state,
                        reward, flags, NULL, n_threads);
}
