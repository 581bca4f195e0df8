// pbn_env.hip -- MI355X (gfx950) batched PBN environment: kernels + C-ABI.
//
// Replaces the per-env, per-node Python step of the external gym_PBN package
// that the reference calls once per frame (bdq_model/__init__.py:177); the ABI
// is include/pbn_env.h, the semantics DESIGN.md "Step semantics".
//
// Layout: one thread owns 32 consecutive envs ("a group") and works on them
// bit-sliced: after a 32x32 transpose, VGPR/LDS word i of the thread holds
// node i of all 32 envs, so one 32-bit VALU op evaluates one boolean
// operation for 32 envs.  A wave covers 2048 envs.  Per-env scalar work
// (interventions, perturbation, reward, reset) runs on the per-env words.
//
// Per node the S planes (current state, bit-sliced) are read from LDS by
// uniform input index; each function is a 4-level mux tree over its (<= 4)
// input planes with 16 precomputed leaf masks held in SGPRs; the selected
// function is chosen by comparing the prob_bits-bit uniform (bit-sliced digit
// planes straight out of Philox) against the node's cumulative thresholds.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/pbn_env.h"
#include "bitslice.h"
#include "philox.h"

using pbn::bfi;
using pbn::Word4;

namespace {

constexpr int kFuncRecWords = 24;  // in[4], leaf[16], thr, pad[3]
constexpr int kMaxHashBits = 12;

struct FuncRec {
  uint32_t in[4];      // input node index per mux level (padded with 0)
  uint32_t leaf[16];   // leaf[m] = d_m (x0 mask), leaf[8+m] = beta_m
  uint32_t thr;        // cumulative selection threshold c_f (prob_bits units)
  uint32_t pad[3];
};
static_assert(sizeof(FuncRec) == kFuncRecWords * 4, "FuncRec layout");

struct StepArgs {
  const FuncRec* funcs;
  const int32_t* node_fs;       // [N+1]
  const uint32_t* tab;          // packed LDS image (cdf | reward | hash)
  const int32_t* att_start;     // [A+1]
  const uint32_t* att_states;   // [S*W]
  const uint32_t* state;
  uint32_t* flipmask;
  uint8_t* target;
  uint8_t* t;
  uint32_t* state_out;
  uint32_t* final_state;
  float* reward;
  uint8_t* flags;
  uint64_t seed, step, env_offset;
  int64_t n_envs;
  int64_t n_groups;
  int n_nodes;
  int n_attr;
  int horizon;
  int mode;
  int cdf_len;       // power of two >= N (LDS cdf table length, padded with 0xFFFFFFFF)
  int hash_bits;     // 0 = no attractors
  int hash_probes;   // max probe count (>= 1 when attractors exist)
  int tab_words;     // words of the LDS table image
  int prob_bits;
  int n_funcs;
  uint32_t hash_mult[4];
};

// ---------------------------------------------------------------- helpers
__device__ __forceinline__ uint32_t valid_word_mask(int n, int w) {
  const int bits = n - 32 * w;
  return bits >= 32 ? 0xFFFFFFFFu : (bits <= 0 ? 0u : ((1u << bits) - 1u));
}

// gap(u) = min{m in 1..N : u < C[m-1]} (N+1 or more if none); C padded with 0xFFFFFFFF.
__device__ __forceinline__ int gap_of(const uint32_t* __restrict__ cdf, int len, uint32_t u) {
  int cnt = 0;
  for (int s = len >> 1; s >= 1; s >>= 1)
    if (cdf[cnt + s - 1] <= u) cnt += s;
  if (cdf[cnt] <= u) cnt += 1;
  return cnt + 1;
}

__device__ __forceinline__ uint32_t eval_func(const FuncRec* __restrict__ fr,
                                              const uint32_t* __restrict__ S) {
  const uint32_t x0 = S[fr->in[0] * 64];
  const uint32_t x1 = S[fr->in[1] * 64];
  const uint32_t x2 = S[fr->in[2] * 64];
  const uint32_t x3 = S[fr->in[3] * 64];
  uint32_t v[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) v[m] = (x0 & fr->leaf[m]) ^ fr->leaf[8 + m];
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) w[q] = bfi(x1, v[2 * q + 1], v[2 * q]);
  const uint32_t y0 = bfi(x2, w[1], w[0]);
  const uint32_t y1 = bfi(x2, w[3], w[2]);
  return bfi(x3, y1, y0);
}

// lanes-of-32-envs bit mask of (u < c), u = digits dig[0..B) MSB first (B = prob_bits).
__device__ __forceinline__ uint32_t less_than(const uint32_t (&dig)[16], uint32_t c, int B) {
  uint32_t lt = 0;
#pragma unroll
  for (int d = 15; d >= 0; --d) {
    if (d < B) {
      const uint32_t C = ((c >> (B - 1 - d)) & 1u) ? 0xFFFFFFFFu : 0u;
      const uint32_t m = dig[d] ^ ~C;
      lt = bfi(m, lt, C);
    }
  }
  return lt;
}

// ------------------------------------------------- step kernel, one thread per group
template <int W>
__global__ void __launch_bounds__(128) pbn_step_lane(StepArgs a) {
  extern __shared__ uint32_t smem[];
  for (int i = threadIdx.x; i < a.tab_words; i += blockDim.x) smem[i] = a.tab[i];
  __syncthreads();

  const int64_t grp = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (grp >= a.n_groups) return;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const uint32_t* cdf = smem;
  const float* rtab = reinterpret_cast<const float*>(smem + a.cdf_len);
  const uint32_t* htab = smem + a.cdf_len + 4 * (a.n_nodes + 1);
  uint32_t* S = smem + a.tab_words + wave * (2 * 32 * W * 64) + lane;  // plane p at S[p*64]
  uint32_t* R = S + 32 * W * 64;

  const int N = a.n_nodes;
  const int64_t n = a.n_envs;
  const int64_t e0 = grp * 32;                       // first local env of the group
  const uint64_t ge0 = a.env_offset + (uint64_t)e0;  // first global env id
  const uint64_t G = ge0 >> 5;                       // global group id
  const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
  const uint32_t st_lo = (uint32_t)a.step;
  const uint32_t st_hi = (uint32_t)((a.step >> 32) & 0xFFFFu) << 16;
  const bool random_actions = (a.mode & PBN_MODE_RANDOM_ACTIONS) != 0;

  // ---- A. load the group's state words, t, target
  uint32_t s1[W][32];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const uint4* p = reinterpret_cast<const uint4*>(a.state + (size_t)w * n + e0);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint4 v = p[q];
      s1[w][4 * q + 0] = v.x;
      s1[w][4 * q + 1] = v.y;
      s1[w][4 * q + 2] = v.z;
      s1[w][4 * q + 3] = v.w;
    }
  }
  uint32_t tpk[8], tgpk[8];
  {
    const uint4* pt = reinterpret_cast<const uint4*>(a.t + e0);
    const uint4* pg = reinterpret_cast<const uint4*>(a.target + e0);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const uint4 v = pt[q], g = pg[q];
      tpk[4 * q + 0] = v.x; tpk[4 * q + 1] = v.y; tpk[4 * q + 2] = v.z; tpk[4 * q + 3] = v.w;
      tgpk[4 * q + 0] = g.x; tgpk[4 * q + 1] = g.y; tgpk[4 * q + 2] = g.z; tgpk[4 * q + 3] = g.w;
    }
  }

  // ---- B. per env: interventions, perturbation gaps 0/1, reset word
  uint32_t gam[W][32];
  uint32_t rword[32];
  uint32_t pcpk[8];      // popcount(flipmask) per env, packed bytes
  uint32_t pmask = 0;    // bit b: env b perturbed
  uint32_t pend = 0;     // bit b: env b needs gap draws beyond E1
#pragma unroll
  for (int q = 0; q < 8; ++q) pcpk[q] = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    uint32_t mq[W][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = 4 * q + r;
      const uint64_t ge = ge0 + (uint64_t)b;
      const Word4 E = pbn::philox4x32_10((uint32_t)ge, st_lo, pbn::kStreamEnv << 28,
                                         (uint32_t)((ge >> 32) & 0xFFFFu) | st_hi, k0, k1);
      uint32_t m[W];
#pragma unroll
      for (int w = 0; w < W; ++w) m[w] = 0;
      if (random_actions) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const uint32_t act = (((E.w >> (10 * k)) & 1023u) * (uint32_t)(N + 1)) >> 10;
          if (act > 0) {
#pragma unroll
            for (int w = 0; w < W; ++w)
              if ((int)((act - 1) >> 5) == w) m[w] |= 1u << ((act - 1) & 31);
          }
        }
      } else {
#pragma unroll
        for (int w = 0; w < W; ++w)
          m[w] = a.flipmask[(size_t)w * n + e0 + b] & valid_word_mask(N, w);
      }
      uint32_t pc = 0;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        mq[w][r] = m[w];
        pc += __builtin_popcount(m[w]);
        s1[w][b] = (s1[w][b] & valid_word_mask(N, w)) ^ m[w];
        gam[w][b] = 0;
      }
      pcpk[q] |= pc << (8 * r);
      // perturbation: positions are partial sums of geometric gaps
      int pos = gap_of(cdf, a.cdf_len, E.x) - 1;
      if (pos < N) {
#pragma unroll
        for (int w = 0; w < W; ++w)
          if ((pos >> 5) == w) gam[w][b] |= 1u << (pos & 31);
        pmask |= 1u << b;
        if (pos < N - 1) {
          pos += gap_of(cdf, a.cdf_len, E.y);
          if (pos < N) {
#pragma unroll
            for (int w = 0; w < W; ++w)
              if ((pos >> 5) == w) gam[w][b] |= 1u << (pos & 31);
            if (pos < N - 1) pend |= 1u << b;
          }
        }
      }
      rword[b] = E.z;
    }
    if (random_actions) {
#pragma unroll
      for (int w = 0; w < W; ++w)
        reinterpret_cast<uint4*>(a.flipmask + (size_t)w * n + e0)[q] =
            make_uint4(mq[w][0], mq[w][1], mq[w][2], mq[w][3]);
    }
  }
  // rare: envs with >= 2 flips so far that may flip more nodes
  while (__any(pend != 0)) {
    if (pend) {
      const int b = __builtin_ctz(pend);
      pend &= pend - 1;
      uint32_t g[W];
      int pos = -1;
#pragma unroll
      for (int bb = 0; bb < 32; ++bb) {
        if (bb == b) {
#pragma unroll
          for (int w = 0; w < W; ++w) g[w] = gam[w][bb];
        }
      }
#pragma unroll
      for (int w = 0; w < W; ++w)
        if (g[w]) pos = 32 * w + 31 - __builtin_clz(g[w]);
      const uint64_t ge = ge0 + (uint64_t)b;
      uint32_t P[4] = {0, 0, 0, 0};
      for (int k = 0; pos < N - 1; ++k) {
        if ((k & 3) == 0) {
          const Word4 pw = pbn::philox4x32_10(
              (uint32_t)ge, st_lo, (pbn::kStreamPert << 28) | (uint32_t)(k >> 2),
              (uint32_t)((ge >> 32) & 0xFFFFu) | st_hi, k0, k1);
          P[0] = pw.x; P[1] = pw.y; P[2] = pw.z; P[3] = pw.w;
        }
        pos += gap_of(cdf, a.cdf_len, P[k & 3]);
        if (pos >= N) break;
#pragma unroll
        for (int w = 0; w < W; ++w)
          if ((pos >> 5) == w) g[w] |= 1u << (pos & 31);
      }
#pragma unroll
      for (int bb = 0; bb < 32; ++bb) {
        if (bb == b) {
#pragma unroll
          for (int w = 0; w < W; ++w) gam[w][bb] = g[w];
        }
      }
    }
  }

  // ---- C. bit-slice: S = planes of s1, R = planes of s1 ^ gamma
#pragma unroll
  for (int w = 0; w < W; ++w) {
    pbn::transpose32(s1[w]);
    pbn::transpose32(gam[w]);
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      S[(32 * w + k) * 64] = s1[w][k];
      R[(32 * w + k) * 64] = s1[w][k] ^ gam[w][k];
    }
  }

  // ---- D. node loop: selection digits, function evaluation, mux
  for (int i = 0; i < N; ++i) {
    const int f0 = a.node_fs[i];
    const int nf = a.node_fs[i + 1] - f0;
    uint32_t dig[16];
    if (nf > 1) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (4 * c >= a.prob_bits) break;
        const Word4 d = pbn::philox4x32_10((uint32_t)G, st_lo,
                                           (pbn::kStreamSel << 28) | (uint32_t)(4 * i + c),
                                           (uint32_t)((G >> 32) & 0xFFFFu) | st_hi, k0, k1);
        dig[4 * c + 0] = d.x;
        dig[4 * c + 1] = d.y;
        dig[4 * c + 2] = d.z;
        dig[4 * c + 3] = d.w;
      }
    }
    uint32_t x = eval_func(a.funcs + f0 + nf - 1, S);
    for (int j = nf - 2; j >= 0; --j) {
      const FuncRec* fr = a.funcs + f0 + j;
      const uint32_t fj = eval_func(fr, S);
      const uint32_t lt = less_than(dig, fr->thr, a.prob_bits);
      x = bfi(lt, fj, x);
    }
    R[i * 64] = bfi(pmask, R[i * 64], x);
  }

  // ---- E. back to per-env words
  uint32_t sp[W][32];
#pragma unroll
  for (int w = 0; w < W; ++w) {
#pragma unroll
    for (int k = 0; k < 32; ++k) sp[w][k] = R[(32 * w + k) * 64];
    pbn::transpose32(sp[w]);
  }
  if (a.final_state) {
#pragma unroll
    for (int w = 0; w < W; ++w) {
      uint4* p = reinterpret_cast<uint4*>(a.final_state + (size_t)w * n + e0);
#pragma unroll
      for (int q = 0; q < 8; ++q)
        p[q] = make_uint4(sp[w][4 * q], sp[w][4 * q + 1], sp[w][4 * q + 2], sp[w][4 * q + 3]);
    }
  }

  // ---- F. reward, termination, autoreset
  const int hmask = (1 << a.hash_bits) - 1;
  const uint32_t* hid = htab + (size_t)W * (hmask + 1);
  uint32_t flpk[8], topk[8];
  bool any_reset = false;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float rq[4];
    uint32_t fl4 = 0, t4 = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = 4 * q + r;
      const uint32_t tgt = (tgpk[q] >> (8 * r)) & 0xFFu;
      int att = -1;
      if (a.hash_bits > 0) {
        uint32_t h = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) h += sp[w][b] * a.hash_mult[w];
        h >>= (32 - a.hash_bits);
        for (int pr = 0; pr < a.hash_probes; ++pr) {
          const uint32_t slot = (h + pr) & hmask;
          bool eq = true;
#pragma unroll
          for (int w = 0; w < W; ++w) eq = eq && (htab[(size_t)w * (hmask + 1) + slot] == sp[w][b]);
          const uint32_t id = hid[slot];
          if (eq && id != 0xFFFFFFFFu) att = (int)id;
        }
      }
      const bool in_attr = att >= 0;
      const bool term = in_attr && (uint32_t)att == tgt;
      const bool wrong = in_attr && !term;
      int tt = (int)((tpk[q] >> (8 * r)) & 0xFFu) + 1;
      tt = tt > 255 ? 255 : tt;
      const bool trunc = a.horizon > 0 && tt >= a.horizon;
      const uint32_t pc = (pcpk[q] >> (8 * r)) & 0xFFu;
      rq[r] = reinterpret_cast<const float*>(rtab)[(2 * (int)term + (int)wrong) * (N + 1) + (int)pc];
      uint32_t fl = (uint32_t)term | ((uint32_t)trunc << 1) | ((uint32_t)in_attr << 2) |
                    (((pmask >> b) & 1u) << 3);
      uint32_t tnew = (uint32_t)tt;
      if ((a.mode & PBN_MODE_AUTORESET) && (term || trunc)) {
        const uint32_t Rw = rword[b];
        uint32_t ns[W];
        uint32_t nt;
        const uint64_t ge = ge0 + (uint64_t)b;
        if (a.n_attr >= 1) {
          const uint32_t A = (uint32_t)a.n_attr;
          const uint32_t as = ((Rw & 1023u) * A) >> 10;
          const int st0 = a.att_start[as];
          const uint32_t size = (uint32_t)(a.att_start[as + 1] - st0);
          const uint32_t idx = (((Rw >> 20) & 4095u) * size) >> 12;
#pragma unroll
          for (int w = 0; w < W; ++w) ns[w] = a.att_states[(size_t)(st0 + idx) * W + w];
          nt = as;
          if (A >= 2) {
            nt = (((Rw >> 10) & 1023u) * (A - 1)) >> 10;
            nt += (nt >= as) ? 1u : 0u;
          }
        } else {
          const Word4 rr = pbn::philox4x32_10((uint32_t)ge, st_lo, (pbn::kStreamReset << 28) | 1u,
                                              (uint32_t)((ge >> 32) & 0xFFFFu) | st_hi, k0, k1);
          const uint32_t rw[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
          for (int w = 0; w < W; ++w) ns[w] = rw[w] & valid_word_mask(N, w);
          nt = PBN_NO_TARGET;
        }
#pragma unroll
        for (int w = 0; w < W; ++w) sp[w][b] = ns[w];
        tgpk[q] = (tgpk[q] & ~(0xFFu << (8 * r))) | (nt << (8 * r));
        tnew = 0;
        fl |= PBN_FLAG_RESET;
        any_reset = true;
      }
      fl4 |= fl << (8 * r);
      t4 |= tnew << (8 * r);
    }
    reinterpret_cast<float4*>(a.reward + e0)[q] = make_float4(rq[0], rq[1], rq[2], rq[3]);
    flpk[q] = fl4;
    topk[q] = t4;
  }
#pragma unroll
  for (int w = 0; w < W; ++w) {
    uint4* p = reinterpret_cast<uint4*>(a.state_out + (size_t)w * n + e0);
#pragma unroll
    for (int q = 0; q < 8; ++q)
      p[q] = make_uint4(sp[w][4 * q], sp[w][4 * q + 1], sp[w][4 * q + 2], sp[w][4 * q + 3]);
  }
  {
    uint4* pf = reinterpret_cast<uint4*>(a.flags + e0);
    uint4* pt = reinterpret_cast<uint4*>(a.t + e0);
    pf[0] = make_uint4(flpk[0], flpk[1], flpk[2], flpk[3]);
    pf[1] = make_uint4(flpk[4], flpk[5], flpk[6], flpk[7]);
    pt[0] = make_uint4(topk[0], topk[1], topk[2], topk[3]);
    pt[1] = make_uint4(topk[4], topk[5], topk[6], topk[7]);
    if (any_reset) {
      uint4* pg = reinterpret_cast<uint4*>(a.target + e0);
      pg[0] = make_uint4(tgpk[0], tgpk[1], tgpk[2], tgpk[3]);
      pg[1] = make_uint4(tgpk[4], tgpk[5], tgpk[6], tgpk[7]);
    }
  }
}

// ------------------------------------------- step kernel, a team of T threads per group
//
// For batches too small to fill 256 CUs with one thread per 32-env group, T
// lanes of one wave share a group: each lane runs the per-env work of 32/T envs
// and the node loop of nodes i = j, j+T, ...; the group's state planes are
// exchanged through LDS.  Per-group LDS: S[32W] planes of s1, R[32W] planes of
// s1^gamma (then of s'), WS/WR[32][W] per-env words, P (perturbed mask).
// FuncRecs and node ranges are staged in LDS because each lane evaluates a
// different node.

// eval of a lane-varying function: record in LDS, planes in LDS
__device__ __forceinline__ uint32_t eval_func_lds(const uint32_t* __restrict__ fr,
                                                  const uint32_t* __restrict__ S) {
  const uint4 in = *reinterpret_cast<const uint4*>(fr);
  const uint32_t x0 = S[in.x], x1 = S[in.y], x2 = S[in.z], x3 = S[in.w];
  const uint4 d0 = *reinterpret_cast<const uint4*>(fr + 4);
  const uint4 d1 = *reinterpret_cast<const uint4*>(fr + 8);
  const uint4 b0 = *reinterpret_cast<const uint4*>(fr + 12);
  const uint4 b1 = *reinterpret_cast<const uint4*>(fr + 16);
  const uint32_t v0 = (x0 & d0.x) ^ b0.x, v1 = (x0 & d0.y) ^ b0.y, v2 = (x0 & d0.z) ^ b0.z,
                 v3 = (x0 & d0.w) ^ b0.w, v4 = (x0 & d1.x) ^ b1.x, v5 = (x0 & d1.y) ^ b1.y,
                 v6 = (x0 & d1.z) ^ b1.z, v7 = (x0 & d1.w) ^ b1.w;
  const uint32_t w0 = bfi(x1, v1, v0), w1 = bfi(x1, v3, v2), w2 = bfi(x1, v5, v4), w3 = bfi(x1, v7, v6);
  return bfi(x3, bfi(x2, w3, w2), bfi(x2, w1, w0));
}

template <int W, int T>
__global__ void __launch_bounds__(256) pbn_step_team(StepArgs a) {
  constexpr int GPB = 256 / T;        // groups per block
  constexpr int EPT = 32 / T;         // envs per thread
  constexpr int GW = 32 * W;          // planes per group
  constexpr int GSTRIDE = 4 * GW + 4; // LDS words per group
  extern __shared__ uint32_t smem[];
  const int N = a.n_nodes;
  const int fwords = a.n_funcs * kFuncRecWords;
  uint32_t* funcs_l = smem + a.tab_words;
  int32_t* nodefs_l = reinterpret_cast<int32_t*>(funcs_l + fwords);
  uint32_t* groups_l = funcs_l + fwords + ((N + 1 + 3) & ~3);
  for (int i = threadIdx.x; i < a.tab_words; i += 256) smem[i] = a.tab[i];
  for (int i = threadIdx.x; i < fwords; i += 256) funcs_l[i] = reinterpret_cast<const uint32_t*>(a.funcs)[i];
  for (int i = threadIdx.x; i <= N; i += 256) nodefs_l[i] = a.node_fs[i];
  const int team = threadIdx.x / T, j = threadIdx.x % T;
  uint32_t* S = groups_l + team * GSTRIDE;
  uint32_t* R = S + GW;
  uint32_t* WS = R + GW;
  uint32_t* WR = WS + GW;
  uint32_t* P = WR + GW;
  if (j == 0) *P = 0;
  __syncthreads();

  const uint32_t* cdf = smem;
  const float* rtab = reinterpret_cast<const float*>(smem + a.cdf_len);
  const uint32_t* htab = smem + a.cdf_len + 4 * (N + 1);
  const int64_t n = a.n_envs;
  int64_t g = (int64_t)blockIdx.x * GPB + team;
  const bool live = g < a.n_groups;
  if (!live) g = a.n_groups - 1;  // dead teams mirror the last group, store nothing
  const int64_t e0 = g * 32;
  const uint64_t ge0 = a.env_offset + (uint64_t)e0;
  const uint64_t G = ge0 >> 5;
  const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
  const uint32_t st_lo = (uint32_t)a.step;
  const uint32_t st_hi = (uint32_t)((a.step >> 32) & 0xFFFFu) << 16;
  const bool random_actions = (a.mode & PBN_MODE_RANDOM_ACTIONS) != 0;

  // ---- per env: interventions, perturbation, reset word
  uint32_t tt_[EPT], tg_[EPT], pc_[EPT], rw_[EPT];
  bool pert_[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int b = j + k * T;
    const int64_t le = e0 + b;
    const uint64_t ge = ge0 + (uint64_t)b;
    const uint32_t ghi = (uint32_t)((ge >> 32) & 0xFFFFu) | st_hi;
    const Word4 E = pbn::philox4x32_10((uint32_t)ge, st_lo, pbn::kStreamEnv << 28, ghi, k0, k1);
    uint32_t s1[W], m[W], gam[W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      s1[w] = a.state[(size_t)w * n + le] & valid_word_mask(N, w);
      m[w] = 0;
      gam[w] = 0;
    }
    tt_[k] = a.t[le];
    tg_[k] = a.target[le];
    if (random_actions) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const uint32_t act = (((E.w >> (10 * q)) & 1023u) * (uint32_t)(N + 1)) >> 10;
        if (act > 0) {
#pragma unroll
          for (int w = 0; w < W; ++w)
            if ((int)((act - 1) >> 5) == w) m[w] |= 1u << ((act - 1) & 31);
        }
      }
      if (live) {
#pragma unroll
        for (int w = 0; w < W; ++w) a.flipmask[(size_t)w * n + le] = m[w];
      }
    } else {
#pragma unroll
      for (int w = 0; w < W; ++w) m[w] = a.flipmask[(size_t)w * n + le] & valid_word_mask(N, w);
    }
    uint32_t pc = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      pc += __builtin_popcount(m[w]);
      s1[w] ^= m[w];
    }
    // perturbation: flip positions are partial sums of geometric gaps
    int pos = -1;
    uint32_t P4[4] = {0, 0, 0, 0};
    for (int kk = 0; pos < N - 1; ++kk) {
      uint32_t u;
      if (kk == 0) {
        u = E.x;
      } else if (kk == 1) {
        u = E.y;
      } else {
        if (((kk - 2) & 3) == 0) {
          const Word4 pw = pbn::philox4x32_10((uint32_t)ge, st_lo,
                                              (pbn::kStreamPert << 28) | (uint32_t)((kk - 2) >> 2), ghi, k0, k1);
          P4[0] = pw.x; P4[1] = pw.y; P4[2] = pw.z; P4[3] = pw.w;
        }
        u = P4[(kk - 2) & 3];
      }
      pos += gap_of(cdf, a.cdf_len, u);
      if (pos >= N) break;
#pragma unroll
      for (int w = 0; w < W; ++w)
        if ((pos >> 5) == w) gam[w] |= 1u << (pos & 31);
    }
    bool pert = false;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      pert = pert || gam[w] != 0;
      WS[b * W + w] = s1[w];
      WR[b * W + w] = s1[w] ^ gam[w];
    }
    if (pert) atomicOr(P, 1u << b);
    pc_[k] = pc;
    rw_[k] = E.z;
    pert_[k] = pert;
  }
  __syncthreads();

  // ---- bit-slice the group: plane p = bit p of every env word
  for (int p = j; p < GW; p += T) {
    const int w = p >> 5, c = p & 31;
    uint32_t sa = 0, ra = 0;
#pragma unroll
    for (int e = 0; e < 32; ++e) {
      sa |= ((WS[e * W + w] >> c) & 1u) << e;
      ra |= ((WR[e * W + w] >> c) & 1u) << e;
    }
    S[p] = sa;
    R[p] = ra;
  }
  __syncthreads();

  // ---- node loop: lane j owns nodes j, j+T, ...
  const uint32_t pmask = *P;
  for (int i = j; i < N; i += T) {
    const int f0 = nodefs_l[i];
    const int nf = nodefs_l[i + 1] - f0;
    uint32_t dig[16];
    if (nf > 1) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (4 * c >= a.prob_bits) break;
        const Word4 d = pbn::philox4x32_10((uint32_t)G, st_lo, (pbn::kStreamSel << 28) | (uint32_t)(4 * i + c),
                                           (uint32_t)((G >> 32) & 0xFFFFu) | st_hi, k0, k1);
        dig[4 * c + 0] = d.x;
        dig[4 * c + 1] = d.y;
        dig[4 * c + 2] = d.z;
        dig[4 * c + 3] = d.w;
      }
    }
    const uint32_t* fr = funcs_l + (size_t)(f0 + nf - 1) * kFuncRecWords;
    uint32_t x = eval_func_lds(fr, S);
    for (int jj = nf - 2; jj >= 0; --jj) {
      fr = funcs_l + (size_t)(f0 + jj) * kFuncRecWords;
      const uint32_t fj = eval_func_lds(fr, S);
      x = bfi(less_than(dig, fr[20], a.prob_bits), fj, x);
    }
    R[i] = bfi(pmask, R[i], x);
  }
  __syncthreads();

  // ---- per env: back to words, reward, termination, autoreset, stores
  const int hmask = (1 << a.hash_bits) - 1;
  const uint32_t* hid = htab + (size_t)W * (hmask + 1);
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int b = j + k * T;
    const int64_t le = e0 + b;
    const uint64_t ge = ge0 + (uint64_t)b;
    uint32_t sp[W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      uint32_t acc = 0;
#pragma unroll
      for (int c = 0; c < 32; ++c) acc |= ((R[32 * w + c] >> b) & 1u) << c;
      sp[w] = acc;
    }
    if (!live) continue;
    if (a.final_state) {
#pragma unroll
      for (int w = 0; w < W; ++w) a.final_state[(size_t)w * n + le] = sp[w];
    }
    int att = -1;
    if (a.hash_bits > 0) {
      uint32_t h = 0;
#pragma unroll
      for (int w = 0; w < W; ++w) h += sp[w] * a.hash_mult[w];
      h >>= (32 - a.hash_bits);
      for (int pr = 0; pr < a.hash_probes; ++pr) {
        const uint32_t slot = (h + pr) & hmask;
        bool eq = true;
#pragma unroll
        for (int w = 0; w < W; ++w) eq = eq && (htab[(size_t)w * (hmask + 1) + slot] == sp[w]);
        const uint32_t id = hid[slot];
        if (eq && id != 0xFFFFFFFFu) att = (int)id;
      }
    }
    const bool in_attr = att >= 0;
    const bool term = in_attr && (uint32_t)att == tg_[k];
    const bool wrong = in_attr && !term;
    int tt = (int)tt_[k] + 1;
    tt = tt > 255 ? 255 : tt;
    const bool trunc = a.horizon > 0 && tt >= a.horizon;
    a.reward[le] = rtab[(2 * (int)term + (int)wrong) * (N + 1) + (int)pc_[k]];
    uint32_t fl = (uint32_t)term | ((uint32_t)trunc << 1) | ((uint32_t)in_attr << 2) | ((uint32_t)pert_[k] << 3);
    if ((a.mode & PBN_MODE_AUTORESET) && (term || trunc)) {
      const uint32_t Rw = rw_[k];
      uint32_t nt;
      if (a.n_attr >= 1) {
        const uint32_t A = (uint32_t)a.n_attr;
        const uint32_t as = ((Rw & 1023u) * A) >> 10;
        const int st0 = a.att_start[as];
        const uint32_t size = (uint32_t)(a.att_start[as + 1] - st0);
        const uint32_t idx = (((Rw >> 20) & 4095u) * size) >> 12;
#pragma unroll
        for (int w = 0; w < W; ++w) sp[w] = a.att_states[(size_t)(st0 + idx) * W + w];
        nt = as;
        if (A >= 2) {
          nt = (((Rw >> 10) & 1023u) * (A - 1)) >> 10;
          nt += (nt >= as) ? 1u : 0u;
        }
      } else {
        const Word4 rr = pbn::philox4x32_10((uint32_t)ge, st_lo, (pbn::kStreamReset << 28) | 1u,
                                            (uint32_t)((ge >> 32) & 0xFFFFu) | st_hi, k0, k1);
        const uint32_t rw4[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
        for (int w = 0; w < W; ++w) sp[w] = rw4[w] & valid_word_mask(N, w);
        nt = PBN_NO_TARGET;
      }
      a.target[le] = (uint8_t)nt;
      tt = 0;
      fl |= PBN_FLAG_RESET;
    }
#pragma unroll
    for (int w = 0; w < W; ++w) a.state_out[(size_t)w * n + le] = sp[w];
    a.t[le] = (uint8_t)tt;
    a.flags[le] = (uint8_t)fl;
  }
}

// ---------------------------------------------------------------- reset kernel
template <int W>
__global__ void __launch_bounds__(256) pbn_reset_kernel(const int32_t* __restrict__ att_start,
                                                        const uint32_t* __restrict__ att_states,
                                                        int n_attr, int N, uint64_t seed, uint64_t step,
                                                        uint64_t env_offset, int64_t n, uint32_t* state,
                                                        uint8_t* target, uint8_t* t) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t ge = env_offset + (uint64_t)i;
  const Word4 r0 = pbn::draw(seed, ge, step, pbn::kStreamReset, 0);
  uint32_t ns[W];
  uint32_t nt;
  if (n_attr >= 1) {
    const uint32_t Rw = r0.x, A = (uint32_t)n_attr;
    const uint32_t as = ((Rw & 1023u) * A) >> 10;
    const int st0 = att_start[as];
    const uint32_t size = (uint32_t)(att_start[as + 1] - st0);
    const uint32_t idx = (((Rw >> 20) & 4095u) * size) >> 12;
#pragma unroll
    for (int w = 0; w < W; ++w) ns[w] = att_states[(size_t)(st0 + idx) * W + w];
    nt = as;
    if (A >= 2) {
      nt = (((Rw >> 10) & 1023u) * (A - 1)) >> 10;
      nt += (nt >= as) ? 1u : 0u;
    }
  } else {
    const Word4 r1 = pbn::draw(seed, ge, step, pbn::kStreamReset, 1);
    const uint32_t rw[4] = {r1.x, r1.y, r1.z, r1.w};
#pragma unroll
    for (int w = 0; w < W; ++w) ns[w] = rw[w] & valid_word_mask(N, w);
    nt = PBN_NO_TARGET;
  }
#pragma unroll
  for (int w = 0; w < W; ++w) state[(size_t)w * n + i] = ns[w];
  target[i] = (uint8_t)nt;
  t[i] = 0;
}

// ---------------------------------------------------------------- host side
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_OK(expr)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return fail(PBN_EDEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

using StepFn = void (*)(StepArgs);

constexpr int kTeamSizes[5] = {2, 4, 8, 16, 32};

StepFn pick_lane(int W) {
  switch (W) {
    case 1: return pbn_step_lane<1>;
    case 2: return pbn_step_lane<2>;
    case 3: return pbn_step_lane<3>;
    case 4: return pbn_step_lane<4>;
  }
  return nullptr;
}

template <int W>
StepFn pick_team_w(int T) {
  switch (T) {
    case 2: return pbn_step_team<W, 2>;
    case 4: return pbn_step_team<W, 4>;
    case 8: return pbn_step_team<W, 8>;
    case 16: return pbn_step_team<W, 16>;
    case 32: return pbn_step_team<W, 32>;
  }
  return nullptr;
}

StepFn pick_team(int W, int T) {
  switch (W) {
    case 1: return pick_team_w<1>(T);
    case 2: return pick_team_w<2>(T);
    case 3: return pick_team_w<3>(T);
    case 4: return pick_team_w<4>(T);
  }
  return nullptr;
}

using ResetFn = void (*)(const int32_t*, const uint32_t*, int, int, uint64_t, uint64_t, uint64_t, int64_t,
                         uint32_t*, uint8_t*, uint8_t*);
ResetFn pick_reset(int W) {
  switch (W) {
    case 1: return pbn_reset_kernel<1>;
    case 2: return pbn_reset_kernel<2>;
    case 3: return pbn_reset_kernel<3>;
    case 4: return pbn_reset_kernel<4>;
  }
  return nullptr;
}

}  // namespace

struct pbn_net {
  int device = 0;
  int n_nodes = 0, W = 0, B = 0, horizon = 0, n_attr = 0, n_states = 0;
  int cdf_len = 0, hash_bits = 0, hash_probes = 0, tab_words = 0;
  uint32_t hash_mult[4] = {0, 0, 0, 0};
  int n_funcs = 0;
  int waves_per_block = 1;   // lane kernel
  size_t lds_lane = 0;
  size_t lds_team[5] = {0, 0, 0, 0, 0};
  StepFn lane = nullptr;
  StepFn team[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  int force_team = -1;       // PBN_TEAM env override (1 = lane kernel)
  ResetFn reset = nullptr;
  FuncRec* d_funcs = nullptr;
  int32_t* d_node_fs = nullptr;
  uint32_t* d_tab = nullptr;
  int32_t* d_att_start = nullptr;
  uint32_t* d_att_states = nullptr;
};

namespace {

void free_net(pbn_net* net) {
  if (!net) return;
  (void)hipFree(net->d_funcs);
  (void)hipFree(net->d_node_fs);
  (void)hipFree(net->d_tab);
  (void)hipFree(net->d_att_start);
  (void)hipFree(net->d_att_states);
  delete net;
}

template <typename T>
int upload(T** dst, const T* src, size_t count) {
  if (count == 0) count = 1;
  HIP_OK(hipMalloc(reinterpret_cast<void**>(dst), count * sizeof(T)));
  if (src) HIP_OK(hipMemcpy(*dst, src, count * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

// open-addressing hash of the attractor states; deterministic multiplier search
bool build_hash(const std::vector<std::vector<uint32_t>>& states, const std::vector<uint32_t>& ids, int W,
                int* bits_out, int* probes_out, uint32_t mult_out[4], std::vector<uint32_t>* image) {
  const size_t S = states.size();
  int bits = 1;
  while ((size_t(1) << bits) < 2 * S) ++bits;
  uint64_t rng = 0x9E3779B97F4A7C15ull;
  auto next = [&rng]() {
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return (uint32_t)(rng >> 11) | 1u;
  };
  for (; bits <= kMaxHashBits; ++bits) {
    const uint32_t size = 1u << bits, mask = size - 1;
    int best_probes = 1 << 30;
    uint32_t best_mult[4] = {0, 0, 0, 0};
    for (int trial = 0; trial < 64; ++trial) {
      uint32_t mult[4];
      for (int w = 0; w < 4; ++w) mult[w] = next();
      std::vector<int> slot_used(size, 0);
      int probes = 1;
      for (size_t k = 0; k < S; ++k) {
        uint32_t h = 0;
        for (int w = 0; w < W; ++w) h += states[k][w] * mult[w];
        h >>= (32 - bits);
        int p = 0;
        while (slot_used[(h + p) & mask]) ++p;
        slot_used[(h + p) & mask] = 1;
        probes = std::max(probes, p + 1);
      }
      if (probes < best_probes) {
        best_probes = probes;
        std::copy(mult, mult + 4, best_mult);
      }
      if (best_probes == 1) break;
    }
    if (best_probes <= 4 || bits == kMaxHashBits) {
      image->assign((size_t)(W + 1) * size, 0u);
      std::vector<int> used(size, 0);
      for (uint32_t s = 0; s < size; ++s) (*image)[(size_t)W * size + s] = 0xFFFFFFFFu;
      for (size_t k = 0; k < S; ++k) {
        uint32_t h = 0;
        for (int w = 0; w < W; ++w) h += states[k][w] * best_mult[w];
        h >>= (32 - bits);
        int p = 0;
        while (used[(h + p) & mask]) ++p;
        const uint32_t slot = (h + p) & mask;
        used[slot] = 1;
        for (int w = 0; w < W; ++w) (*image)[(size_t)w * size + slot] = states[k][w];
        (*image)[(size_t)W * size + slot] = ids[k];
      }
      *bits_out = bits;
      *probes_out = best_probes;
      std::copy(best_mult, best_mult + 4, mult_out);
      return true;
    }
  }
  return false;
}

}  // namespace

extern "C" {

const char* pbn_last_error(void) { return g_err.c_str(); }
int pbn_abi_version(void) { return PBN_ABI_VERSION; }

int pbn_net_words(const pbn_net* net) { return net ? net->W : PBN_EINVAL; }

int pbn_net_create(const pbn_net_desc* d, pbn_net** out) {
  if (!d || !out) return fail(PBN_EINVAL, "null descriptor/out");
  *out = nullptr;
  const int N = d->n_nodes;
  if (N < 1 || N > PBN_MAX_NODES) return fail(PBN_EINVAL, "n_nodes out of range 1..128");
  if (!(d->prob_bits == 4 || d->prob_bits == 8 || d->prob_bits == 12 || d->prob_bits == 16))
    return fail(PBN_EINVAL, "prob_bits must be 4, 8, 12 or 16");
  if (d->horizon < 0 || d->horizon > 255) return fail(PBN_EINVAL, "horizon out of range 0..255");
  if (d->n_attractors < 0 || d->n_attractors > PBN_MAX_ATTRACTORS)
    return fail(PBN_EINVAL, "n_attractors out of range 0..254");
  if (!d->node_func_start || !d->func_arity || !d->func_inputs || !d->func_table || !d->func_threshold ||
      !d->perturb_cdf || !d->reward_table)
    return fail(PBN_EINVAL, "null table in descriptor");
  const int W = (N + 31) / 32;
  const uint32_t one = 1u << d->prob_bits;
  if (d->node_func_start[0] != 0 || d->node_func_start[N] != d->n_funcs)
    return fail(PBN_EINVAL, "node_func_start must span 0..n_funcs");
  std::vector<FuncRec> recs(d->n_funcs);
  for (int i = 0; i < N; ++i) {
    const int f0 = d->node_func_start[i], f1 = d->node_func_start[i + 1];
    if (f1 <= f0 || f1 - f0 > PBN_MAX_FUNCS_PER_NODE)
      return fail(PBN_EINVAL, "node " + std::to_string(i) + " needs 1..16 functions");
    uint32_t prev = 0;
    for (int f = f0; f < f1; ++f) {
      const int k = d->func_arity[f];
      if (k < 0 || k > PBN_MAX_ARITY) return fail(PBN_EINVAL, "function arity must be 0..4");
      const uint32_t c = d->func_threshold[f];
      if (c < prev || c > one) return fail(PBN_EINVAL, "thresholds must be non-decreasing and <= 2^prob_bits");
      if (f == f1 - 1 && c != one) return fail(PBN_EINVAL, "last threshold of a node must be 2^prob_bits");
      prev = c;
      FuncRec& r = recs[f];
      memset(&r, 0, sizeof r);
      for (int j = 0; j < 4; ++j) {
        int g = j < k ? d->func_inputs[4 * f + j] : 0;
        if (g < 0 || g >= N) return fail(PBN_EINVAL, "function input index out of range");
        r.in[j] = (uint32_t)g;
      }
      const uint32_t T = d->func_table[f];
      const uint32_t kmask = (k >= 5) ? 0xFFFFFFFFu : ((1u << k) - 1u);
      if (k < 5 && (T >> (1u << k)) != 0u && (1u << k) < 32)
        return fail(PBN_EINVAL, "truth table has bits beyond 2^arity");
      for (int m = 0; m < 8; ++m) {
        const uint32_t lo = (T >> ((2u * m) & kmask)) & 1u;        // x0 = 0
        const uint32_t hi = (T >> ((2u * m + 1u) & kmask)) & 1u;   // x0 = 1
        r.leaf[8 + m] = lo ? 0xFFFFFFFFu : 0u;
        r.leaf[m] = (lo ^ hi) ? 0xFFFFFFFFu : 0u;
      }
      r.thr = c;
    }
  }
  // attractors
  const int A = d->n_attractors;
  const int S = A ? d->n_attractor_states : 0;
  std::vector<std::vector<uint32_t>> states;
  std::vector<uint32_t> ids;
  if (A) {
    if (!d->attractor_start || !d->attractor_states) return fail(PBN_EINVAL, "null attractor tables");
    if (d->attractor_start[0] != 0 || d->attractor_start[A] != S) return fail(PBN_EINVAL, "bad attractor_start");
    for (int at = 0; at < A; ++at) {
      if (d->attractor_start[at + 1] <= d->attractor_start[at]) return fail(PBN_EINVAL, "empty attractor");
      for (int k = d->attractor_start[at]; k < d->attractor_start[at + 1]; ++k) {
        states.emplace_back(d->attractor_states + (size_t)k * W, d->attractor_states + (size_t)k * W + W);
        ids.push_back((uint32_t)at);
      }
    }
  }
  pbn_net* net = new pbn_net();
  net->n_nodes = N;
  net->W = W;
  net->B = d->prob_bits;
  net->horizon = d->horizon;
  net->n_attr = A;
  net->n_states = S;
  net->cdf_len = 32;
  while (net->cdf_len < N) net->cdf_len <<= 1;
  std::vector<uint32_t> hash_img;
  if (A) {
    if (!build_hash(states, ids, W, &net->hash_bits, &net->hash_probes, net->hash_mult, &hash_img)) {
      free_net(net);
      return fail(PBN_EINVAL, "too many attractor states for the LDS hash");
    }
  }
  // LDS table image: cdf[cdf_len] | reward[4(N+1)] | hash[(W+1) << bits]
  std::vector<uint32_t> tab(net->cdf_len, 0xFFFFFFFFu);
  for (int m = 0; m < N; ++m) tab[m] = d->perturb_cdf[m];
  for (int m = 1; m < N; ++m)
    if (tab[m] < tab[m - 1]) {
      free_net(net);
      return fail(PBN_EINVAL, "perturb_cdf must be non-decreasing");
    }
  for (int k = 0; k < 4 * (N + 1); ++k) {
    uint32_t u;
    memcpy(&u, &d->reward_table[k], 4);
    tab.push_back(u);
  }
  tab.insert(tab.end(), hash_img.begin(), hash_img.end());
  while (tab.size() & 3) tab.push_back(0u);  // keep the FuncRec image 16-byte aligned in LDS
  net->tab_words = (int)tab.size();
  net->n_funcs = d->n_funcs;
  net->waves_per_block = (W == 1) ? 2 : 1;
  net->lds_lane = (size_t)net->tab_words * 4 + (size_t)net->waves_per_block * 2 * 32 * W * 64 * 4;
  const size_t team_fixed =
      ((size_t)net->tab_words + (size_t)d->n_funcs * kFuncRecWords + (size_t)((N + 1 + 3) & ~3)) * 4;
  for (int ti = 0; ti < 5; ++ti) {
    const int T = kTeamSizes[ti];
    net->lds_team[ti] = team_fixed + (size_t)(256 / T) * (4 * 32 * W + 4) * 4;
    net->team[ti] = pick_team(W, T);
  }
  net->lane = pick_lane(W);
  net->reset = pick_reset(W);
  if (const char* env = getenv("PBN_TEAM")) net->force_team = atoi(env);
  int rc;
  if (hipGetDevice(&net->device) != hipSuccess) {
    free_net(net);
    return fail(PBN_EDEVICE, "no HIP device");
  }
  if ((rc = upload(&net->d_funcs, recs.data(), recs.size())) ||
      (rc = upload(&net->d_node_fs, d->node_func_start, (size_t)N + 1)) ||
      (rc = upload(&net->d_tab, tab.data(), tab.size())) ||
      (rc = upload(&net->d_att_start, A ? d->attractor_start : nullptr, (size_t)A + 1)) ||
      (rc = upload(&net->d_att_states, S ? d->attractor_states : nullptr, (size_t)S * W))) {
    free_net(net);
    return rc;
  }
  for (int ti = -1; ti < 5; ++ti) {
    const StepFn fn = ti < 0 ? net->lane : net->team[ti];
    const size_t bytes = ti < 0 ? net->lds_lane : net->lds_team[ti];
    if (bytes > 160 * 1024) continue;  // variant unusable for this net; never picked
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)bytes) != hipSuccess) {
      free_net(net);
      return fail(PBN_EDEVICE, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
    }
  }
  if (net->lds_lane > 160 * 1024 && net->lds_team[4] > 160 * 1024) {
    free_net(net);
    return fail(PBN_EINVAL, "LDS budget exceeded");
  }
  *out = net;
  return PBN_OK;
}

int pbn_net_destroy(pbn_net* net) {
  if (!net) return PBN_OK;
  free_net(net);
  return PBN_OK;
}

static int check_common(pbn_net* net, uint64_t env_offset, int64_t n_envs) {
  if (!net) return fail(PBN_EINVAL, "null net");
  if (n_envs < 0) return fail(PBN_EINVAL, "n_envs < 0");
  if ((n_envs & 31) || (env_offset & 31))
    return fail(PBN_EINVAL, "n_envs and env_offset must be multiples of 32");
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != net->device)
    return fail(PBN_EDEVICE, "current device differs from the net's device");
  return PBN_OK;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

int pbn_reset(pbn_net* net, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n_envs,
              uint32_t* d_state, uint8_t* d_target, uint8_t* d_t, void* stream) {
  int rc = check_common(net, env_offset, n_envs);
  if (rc) return rc;
  if (n_envs == 0) return PBN_OK;
  if (!d_state || !d_target || !d_t) return fail(PBN_EINVAL, "null buffer");
  const int threads = 256;
  const unsigned blocks = (unsigned)((n_envs + threads - 1) / threads);
  hipLaunchKernelGGL(net->reset, dim3(blocks), dim3(threads), 0, (hipStream_t)stream, net->d_att_start,
                     net->d_att_states, net->n_attr, net->n_nodes, seed, step, env_offset, n_envs, d_state,
                     d_target, d_t);
  HIP_OK(hipGetLastError());
  return PBN_OK;
}

int pbn_step(pbn_net* net, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n_envs, uint32_t mode,
             const uint32_t* d_state, uint32_t* d_flipmask, uint8_t* d_target, uint8_t* d_t,
             uint32_t* d_state_out, uint32_t* d_final_state, float* d_reward, uint8_t* d_flags,
             void* stream) {
  int rc = check_common(net, env_offset, n_envs);
  if (rc) return rc;
  if (n_envs == 0) return PBN_OK;
  if (mode & ~(PBN_MODE_AUTORESET | PBN_MODE_RANDOM_ACTIONS)) return fail(PBN_EINVAL, "unknown mode bits");
  if (!d_state || !d_flipmask || !d_target || !d_t || !d_state_out || !d_reward || !d_flags)
    return fail(PBN_EINVAL, "null buffer");
  if (d_state_out == d_state) return fail(PBN_EINVAL, "d_state_out must not alias d_state");
  if (!aligned16(d_state) || !aligned16(d_flipmask) || !aligned16(d_target) || !aligned16(d_t) ||
      !aligned16(d_state_out) || !aligned16(d_reward) || !aligned16(d_flags) ||
      (d_final_state && !aligned16(d_final_state)))
    return fail(PBN_EINVAL, "device buffers must be 16-byte aligned");
  StepArgs a;
  memset(&a, 0, sizeof a);
  a.funcs = net->d_funcs;
  a.node_fs = net->d_node_fs;
  a.tab = net->d_tab;
  a.att_start = net->d_att_start;
  a.att_states = net->d_att_states;
  a.state = d_state;
  a.flipmask = d_flipmask;
  a.target = d_target;
  a.t = d_t;
  a.state_out = d_state_out;
  a.final_state = d_final_state;
  a.reward = d_reward;
  a.flags = d_flags;
  a.seed = seed;
  a.step = step;
  a.env_offset = env_offset;
  a.n_envs = n_envs;
  a.n_groups = n_envs / 32;
  a.n_nodes = net->n_nodes;
  a.n_attr = net->n_attr;
  a.horizon = net->horizon;
  a.mode = (int)mode;
  a.cdf_len = net->cdf_len;
  a.hash_bits = net->n_attr ? net->hash_bits : 0;
  a.hash_probes = net->hash_probes;
  a.tab_words = net->tab_words;
  memcpy(a.hash_mult, net->hash_mult, sizeof a.hash_mult);
  a.prob_bits = net->B;
  a.n_funcs = net->n_funcs;
  // launch shape: one thread per 32-env group when that fills the chip, else a
  // team of T lanes per group (smallest T reaching ~4 waves per SIMD, max 32)
  int T = 1;
  const int64_t target_threads = 256 * 4 * 4 * 64;
  while (T < 32 && a.n_groups * T < target_threads) T <<= 1;
  if (net->force_team > 0) T = net->force_team;
  int ti = -1;
  for (int k = 0; k < 5; ++k)
    if (kTeamSizes[k] == T) ti = k;
  if (T != 1 && (ti < 0 || net->lds_team[ti] > 160 * 1024)) T = 1, ti = -1;
  if (T == 1 && net->lds_lane > 160 * 1024) ti = 4;
  if (ti < 0) {
    const int threads = 64 * net->waves_per_block;
    const unsigned blocks = (unsigned)((a.n_groups + threads - 1) / threads);
    hipLaunchKernelGGL(net->lane, dim3(blocks), dim3(threads), net->lds_lane, (hipStream_t)stream, a);
  } else {
    const int gpb = 256 / kTeamSizes[ti];
    const unsigned blocks = (unsigned)((a.n_groups + gpb - 1) / gpb);
    hipLaunchKernelGGL(net->team[ti], dim3(blocks), dim3(256), net->lds_team[ti], (hipStream_t)stream, a);
  }
  HIP_OK(hipGetLastError());
  return PBN_OK;
}

}  // extern "C"
