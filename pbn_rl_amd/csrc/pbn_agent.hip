// pbn_agent.hip -- the env<->agent edges of the batched BDQ frame loop.
//
// The reference's frame loop (bdq_model/__init__.py:172-177) builds the Q-network input on
// the host (np.stack((state, target)) -> float (2,1,N), :92-93), takes argmax over each of the
// 3 action branches (:95-96), and hands list(action.unique()) to env.step (:176-177), whose
// action a > 0 flips node a-1 (:81-84).  Batched on the GPU these become two HBM-bound kernels
// around the PyTorch Q-network forward:
//
//   pbn_obs_unpack        packed state words + target attractor id -> fp32 (2, n, N)
//   pbn_bilinear_targets  the Q-network's bilinear layer straight from the packed state (below)
//   pbn_q_to_flipmask     Q (n, K, N+1) -> epsilon-greedy actions -> flip mask words (W, n)
//
// None of them does arithmetic worth an MFMA; they are one pass over their bytes with
// coalesced accesses.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "../../include/pbn_env.h"
#include "net_view.h"
#include "philox.h"
#include "replay_draw.h"

namespace {

constexpr int kObsThreads = 256;
constexpr int kQEnvs = 64;          // envs per q_to_flipmask block (one wave, one env per lane)
constexpr int kMaxBranches = 7;     // random actions: branch k from EXPLORE word k + 1 (two calls)

// out[p][e][i], p = 0: bit i of env e's state, p = 1: bit i of the first state of env e's
// target attractor (all zeros without a target).  Four consecutive (e, i) elements per
// thread, written as one float4 per plane; n * N is a multiple of 4 because n is a
// multiple of 32.
__global__ void __launch_bounds__(kObsThreads) obs_unpack_kernel(const uint32_t* __restrict__ state,
                                                                 const uint8_t* __restrict__ target,
                                                                 const int32_t* __restrict__ att_start,
                                                                 const uint32_t* __restrict__ att_states,
                                                                 int n_attr, int N, int W, uint32_t n,
                                                                 float* __restrict__ out) {
  const uint32_t total4 = n * (uint32_t)N / 4u;
  float4* out_s = reinterpret_cast<float4*>(out);
  float4* out_t = reinterpret_cast<float4*>(out + (size_t)n * N);
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < total4; q += gridDim.x * blockDim.x) {
    const uint32_t f = 4u * q;
    uint32_t e = f / (uint32_t)N;
    int i = (int)(f - e * (uint32_t)N);
    float vs[4], vt[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t sw = state[(size_t)(i >> 5) * n + e];
      const uint32_t tg = target[e];
      const uint32_t tw = tg < (uint32_t)n_attr ? att_states[(size_t)att_start[tg] * W + (i >> 5)] : 0u;
      vs[r] = (float)((sw >> (i & 31)) & 1u);
      vt[r] = (float)((tw >> (i & 31)) & 1u);
      if (++i == N) {
        i = 0;
        ++e;
      }
    }
    out_s[q] = make_float4(vs[0], vs[1], vs[2], vs[3]);
    out_t[q] = make_float4(vt[0], vt[1], vt[2], vt[3]);
  }
}

// The first layer of BranchingQNetwork is bilinear in (state, target):
//   y[e][o] = bias[o] + sum_ij s_e[i] t_e[j] W[o][i][j]   (bdq_model/network.py:8-21).
// Both inputs are 0/1 and t_e is the first state of env e's target attractor, one of A.  With
// T[a][i][o] = sum_j t_a[j] W[o][i][j] precomputed (a (A, N) @ (N, N*O) GEMM), the layer is
//   y[e][o] = bias[o] + sum over the set bits i of s_e of T[target_e][i][o],
// i.e. |s_e| row reads of T (L2-resident: A * N * O floats) per env instead of the
// (n, N*N) outer product and its (n, N*N) @ (N*N, O) GEMM.  Rows are added in ascending i.
// One wave per env (four per block, kBilEnvs envs per block); lane l owns outputs 4l..4l+3
// (+ 256 k), read and written as float4.  The env's state words and target id are
// wave-uniform, so the bit loop is scalar; its row loads go out eight at a time and are then
// added in ascending i (the L2 round trip, not the adds, is the cost of a row).
constexpr int kBilThreads = 256;
constexpr int kBilEnvs = 16;
constexpr int kBilBatch = 8;

template <int W>
__global__ void __launch_bounds__(kBilThreads) bilinear_targets_kernel(const uint32_t* __restrict__ state,
                                                                       const uint8_t* __restrict__ target,
                                                                       const float* __restrict__ T,
                                                                       const float* __restrict__ bias, int N,
                                                                       int A, int O, uint32_t n, int leaky,
                                                                       float slope, float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int O4 = O >> 2;
  const uint32_t e0 = blockIdx.x * kBilEnvs;
  const float4* bias4 = reinterpret_cast<const float4*>(bias);
  for (int r = wv; r < kBilEnvs; r += kBilThreads / 64) {
    const uint32_t e = e0 + (uint32_t)r;
    if (e >= n) break;
    const uint32_t tg = __builtin_amdgcn_readfirstlane((uint32_t)target[e]);
    uint32_t words[W];
#pragma unroll
    for (int w = 0; w < W; ++w) words[w] = __builtin_amdgcn_readfirstlane(state[(size_t)w * n + e]);
    float4* y4 = reinterpret_cast<float4*>(y + (size_t)e * O);
    for (int o4 = lane; o4 < O4; o4 += 64) {
      float4 acc = bias4[o4];
      if (tg < (uint32_t)A) {
        const float4* Ta = reinterpret_cast<const float4*>(T + (size_t)tg * N * O) + o4;
#pragma unroll
        for (int w = 0; w < W; ++w) {
          uint32_t b = words[w];
          while (b) {
            int idx[kBilBatch];
#pragma unroll
            for (int k = 0; k < kBilBatch; ++k) {
              idx[k] = b ? 32 * w + __builtin_ctz(b) : -1;
              b = b ? (b & (b - 1u)) : 0u;
            }
            float4 v[kBilBatch];
#pragma unroll
            for (int k = 0; k < kBilBatch; ++k)
              v[k] = idx[k] >= 0 ? Ta[(size_t)idx[k] * O4] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int k = 0; k < kBilBatch; ++k) {
              if (idx[k] >= 0) {
                acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w;
              }
            }
          }
        }
      }
      if (leaky) {   // the LeakyReLU after the layer, as torch computes it: x > 0 ? x : x * slope
        acc.x = acc.x > 0.f ? acc.x : acc.x * slope;
        acc.y = acc.y > 0.f ? acc.y : acc.y * slope;
        acc.z = acc.z > 0.f ? acc.z : acc.z * slope;
        acc.w = acc.w > 0.f ? acc.w : acc.w * slope;
      }
      y4[o4] = acc;
    }
  }
}

// The same layer with the table staged in LDS.  The rows an env sums are T[target][i] for its
// set bits i, 1 KB each: read from L2 that is ~750 MB per 32,768 Bittner-28 envs, and the kernel
// above runs at two thirds of the L2 bandwidth.  A block of kBlEnvs envs instead walks the
// outputs in 32-wide tiles and stages tile p's slice of the whole table, T[.][.][32p, 32p + 32)
// (A N rows of 128 B, 50 KB for Bittner-28), in LDS once: L2 reads drop to A N x 1 KB per
// block, and the gathers hit LDS.  The slices are copied by LDS-DMA (global_load_lds_dwordx4: a
// wave-instruction fills 1 KB of LDS linearly, eight rows, with no VGPR round trip) and
// double-buffered, so the next slice lands while this tile is summed; the bias is staged once
// beside them (an ordinary global load in the loop would make the compiler drain the DMA).
// TPE threads per env, each owning 32 / TPE outputs of the tile; the sum order is the kernel
// above's (bias, then the rows in ascending i), so the two agree bit for bit.
constexpr int kBlEnvs = 128;
constexpr int kBlBatch = 4;   // set bits whose rows are read before they are added
constexpr int kBlTpe = 4;     // threads per env (2 measured 46 us against 29.6 us at 32,768 envs)

template <int W, int TPE>
__global__ void __launch_bounds__(kBlEnvs * TPE) bilinear_lds_kernel(const uint32_t* __restrict__ state,
                                                                      const uint8_t* __restrict__ target,
                                                                      const float* __restrict__ T,
                                                                      const float* __restrict__ bias, int N, int A,
                                                                      int O, uint32_t n, int leaky, float slope,
                                                                      float* __restrict__ y) {
  constexpr int kThreads = kBlEnvs * TPE;
  constexpr int Q = 8 / TPE;   // float4s of the tile per thread
  extern __shared__ __attribute__((aligned(16))) float sl[];   // [2][A N][32] | bias [O]
  const int rows = A * N;
  const int slice = rows * 32;
  float* sbias = sl + 2 * slice;
  const int t = (int)threadIdx.x;
  const int lane = t & 63;
  const int sub = t % TPE;
  const uint32_t e = blockIdx.x * kBlEnvs + (uint32_t)(t / TPE);
  const bool live = e < n;
  const uint32_t tg = live ? (uint32_t)target[e] : 0xFFu;
  const bool has_t = tg < (uint32_t)A;
  uint32_t words[W];
#pragma unroll
  for (int w = 0; w < W; ++w) words[w] = (live && has_t) ? state[(size_t)w * n + e] : 0u;
  for (int i = t; i < O; i += kThreads) sbias[i] = bias[i];
  // the state word has landed before any DMA is issued (its first use behind one would drain it)
#pragma unroll
  for (int w = 0; w < W; ++w) asm volatile("" ::"v"(words[w]));
  const int rowbase = has_t ? (int)tg * N : 0;
  const int n_items = rows * 8;   // float4s of one slice
  const float4* T4 = reinterpret_cast<const float4*>(T);
  // slice p into buffer b: LDS float4 P = 64 j' + lane of the wave's stripes holds row P >> 3,
  // columns 32p + 4 (P & 7) .. + 3
#define PBN_BL_STAGE(p_, b_)                                                                       \
  for (int base = t - lane; base < n_items; base += kThreads) {                                    \
    const int P = base + lane;                                                                     \
    if (P < n_items)                                                                               \
      __builtin_amdgcn_global_load_lds(                                                            \
          (__attribute__((address_space(1))) void*)(T4 + (size_t)(P >> 3) * (O >> 2) + 8 * (p_) + (P & 7)), \
          (__attribute__((address_space(3))) void*)(sl + (b_) * slice + 4 * base), 16, 0, 0);      \
  }
  const int n_tiles = O >> 5;
  PBN_BL_STAGE(0, 0)
  __syncthreads();
  for (int p = 0; p < n_tiles; ++p) {
    if (p + 1 < n_tiles) { PBN_BL_STAGE(p + 1, (p + 1) & 1) }
    const float* S = sl + (p & 1) * slice + 4 * Q * sub;
    float4 acc[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) acc[q] = *reinterpret_cast<const float4*>(sbias + 32 * p + 4 * (Q * sub + q));
#pragma unroll
    for (int w = 0; w < W; ++w) {
      uint32_t b = words[w];
      while (b) {
        int idx[kBlBatch];
#pragma unroll
        for (int k = 0; k < kBlBatch; ++k) {
          idx[k] = b ? 32 * w + __builtin_ctz(b) : -1;
          b = b ? (b & (b - 1u)) : 0u;
        }
        float4 v[kBlBatch][Q];
#pragma unroll
        for (int k = 0; k < kBlBatch; ++k) {
          const float4* r = reinterpret_cast<const float4*>(S + (rowbase + (idx[k] >= 0 ? idx[k] : 0)) * 32);
#pragma unroll
          for (int q = 0; q < Q; ++q) v[k][q] = r[q];
        }
#pragma unroll
        for (int k = 0; k < kBlBatch; ++k) {
          if (idx[k] >= 0) {
#pragma unroll
            for (int q = 0; q < Q; ++q) {
              acc[q].x += v[k][q].x; acc[q].y += v[k][q].y; acc[q].z += v[k][q].z; acc[q].w += v[k][q].w;
            }
          }
        }
      }
    }
    if (live) {
      float4* yo = reinterpret_cast<float4*>(y + (size_t)e * O) + 8 * p + Q * sub;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        float4 a = acc[q];
        if (leaky) {   // torch's LeakyReLU: x > 0 ? x : x * slope
          a.x = a.x > 0.f ? a.x : a.x * slope;
          a.y = a.y > 0.f ? a.y : a.y * slope;
          a.z = a.z > 0.f ? a.z : a.z * slope;
          a.w = a.w > 0.f ? a.w : a.w * slope;
        }
        yo[q] = a;
      }
    }
    __syncthreads();   // (waits for the next slice's DMA: vmcnt(0))
  }
#undef PBN_BL_STAGE
}

// torch.argmax semantics: the first maximal index; NaN counts as the maximum
__device__ __forceinline__ int argmax_row(const float* __restrict__ r, int A) {
  float best = r[0];
  int bi = 0;
  for (int j = 1; j < A; ++j) {
    const float v = r[j];
    const bool take = !isnan(best) && (isnan(v) || v > best);
    best = take ? v : best;
    bi = take ? j : bi;
  }
  return bi;
}

// One wave per 64 envs: the block's Q rows (contiguous, 64 * K * A floats) are staged through
// LDS with coalesced float4 loads, then lane e reduces its K rows.  Row stride K * A words:
// odd for the kaban networks' K = 3, so the per-lane row reads spread over the banks.
// heads = 1: q holds the raw head outputs (K+1, n, A) of BranchingQNetwork (head 0 = value,
// output 0) instead of Q; the dueling combination is done here, per env and branch, as
//   q_a = (v + adv_a) - mean,  mean = (adv_0 + adv_1 + ... + adv_{A-1}) / A   (left to right),
// the order of bdq_model/network.py:59-61 with the mean summed sequentially.
__global__ void __launch_bounds__(kQEnvs * kMaxBranches) q_to_flipmask_kernel(
    const float* __restrict__ q, int heads, int K, int A, int N, int W, int64_t n, uint64_t seed, uint64_t step,
    const uint64_t* __restrict__ d_step, uint64_t env_offset, uint64_t eps_u, const float* __restrict__ d_eps,
    uint32_t* __restrict__ flipmask, int32_t* __restrict__ actions) {
  // one wave per branch (K waves), lane = env of the block; the chosen actions meet in LDS
  extern __shared__ float sq[];
  const int64_t e0 = (int64_t)blockIdx.x * kQEnvs;
  const int row = K * A;
  const int n_blk = (int)((n - e0) < kQEnvs ? (n - e0) : kQEnvs);   // 32 or 64
  const int nthr = (int)blockDim.x;
  if (!heads) {
    const float4* src = reinterpret_cast<const float4*>(q + (size_t)e0 * row);
    const int words4 = n_blk * row / 4;
    for (int k = threadIdx.x; k < words4; k += nthr) reinterpret_cast<float4*>(sq)[k] = src[k];
  } else {   // K + 1 chunks of n_blk rows, one per head
    const int chunk4 = n_blk * A / 4;
    for (int h = 0; h <= K; ++h) {
      const float4* src = reinterpret_cast<const float4*>(q + ((size_t)h * n + e0) * A);
      float4* dst = reinterpret_cast<float4*>(sq + (size_t)h * n_blk * A);
      for (int k = threadIdx.x; k < chunk4; k += nthr) dst[k] = src[k];
    }
  }
  int* act_lds = reinterpret_cast<int*>(sq + (size_t)(heads ? K + 1 : K) * kQEnvs * A);   // [K][64]
  __syncthreads();
  const int k = (int)threadIdx.x >> 6;            // this wave's branch
  const int t = (int)threadIdx.x & 63;            // env of the block
  if (t < n_blk) {
    const int64_t e = e0 + t;
    const uint64_t ge = env_offset + (uint64_t)e;
    const uint64_t st = d_step ? *d_step : step;
    const pbn::Word4 r = pbn::draw(seed, ge, st, pbn::kStreamExplore, 0);
    if (d_eps) {   // device epsilon (graph replays): clamped to [0, 1], NaN -> 0
      const float ef = fminf(fmaxf(*d_eps, 0.f), 1.f);
      eps_u = (uint64_t)floor((double)ef * 4294967296.0);
    }
    const bool explore = (uint64_t)r.x < eps_u;
    int a;
    if (explore) {
      // branch k: EXPLORE word k + 1 (call (k + 1) >> 2), multiply-high onto [0, N]:
      // bias <= (N + 1) / 2^32 against np.random.randint (bdq_model/__init__.py:76)
      uint32_t rw = k == 0 ? r.y : (k == 1 ? r.z : r.w);
      if (k >= 3) {
        const pbn::Word4 r1 = pbn::draw(seed, ge, st, pbn::kStreamExplore, 1);
        rw = k == 3 ? r1.x : (k == 4 ? r1.y : (k == 5 ? r1.z : r1.w));
      }
      a = (int)__umulhi(rw, (uint32_t)(N + 1));
    } else if (!heads) {
      a = argmax_row(sq + (size_t)t * row + k * A, A);
    } else {
      const float v = sq[(size_t)t * A];
      const float* adv = sq + ((size_t)(k + 1) * n_blk + t) * A;
      float sum = 0.f;
      for (int j = 0; j < A; ++j) sum += adv[j];
      const float mean = sum / (float)A;
      float best = (v + adv[0]) - mean;
      int bi = 0;
      for (int j = 1; j < A; ++j) {   // torch.argmax: first maximum, NaN is the maximum
        const float qj = (v + adv[j]) - mean;
        const bool take = !isnan(best) && (isnan(qj) || qj > best);
        best = take ? qj : best;
        bi = take ? j : bi;
      }
      a = bi;
    }
    if (actions) actions[e * K + k] = a;
    act_lds[k * kQEnvs + t] = a;
  }
  __syncthreads();
  if (k == 0 && t < n_blk) {
    uint32_t m[4] = {0u, 0u, 0u, 0u};
    for (int kk = 0; kk < K; ++kk) {
      const int a = act_lds[kk * kQEnvs + t];
      if (a > 0 && a <= N) {   // a > 0 flips node a-1, once however often it repeats
        const int node = a - 1;
#pragma unroll
        for (int w = 0; w < 4; ++w)
          if (w == (node >> 5)) m[w] |= 1u << (node & 31);
      }
    }
    const int64_t e = e0 + t;
#pragma unroll
    for (int w = 0; w < 4; ++w)
      if (w < W) flipmask[(size_t)w * n + e] = m[w];
  }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

// ---- n transitions into the replay ring in one pass (pbn_replay_store): env e goes to slot
// (pos + e) mod capacity, pos read from device memory (graph replays advance it on the stream).
// Replaces the ring's six index_copy_ launches and the slot arithmetic.
__global__ void __launch_bounds__(kObsThreads) replay_store_kernel(
    int64_t n, const int64_t* __restrict__ pos, int64_t cap, int W, int K, const uint32_t* st,
    const uint32_t* __restrict__ nst, const uint8_t* tgt, const int32_t* __restrict__ act,
    const float* __restrict__ rew, const uint8_t* __restrict__ done, uint32_t done_mask, uint8_t* __restrict__ done_out,
    uint32_t* __restrict__ r_st, uint32_t* __restrict__ r_nst, uint8_t* __restrict__ r_tgt, int32_t* __restrict__ r_act,
    float* __restrict__ r_rew, uint8_t* __restrict__ r_done, uint32_t* st_dst, const uint32_t* __restrict__ st_src,
    uint8_t* tgt_dst, const uint8_t* __restrict__ tgt_src) {
  const int64_t p0 = *pos;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = (p0 + e) % cap;
    for (int w = 0; w < W; ++w) {
      const uint32_t sv = st[(size_t)w * n + e];
      r_st[(size_t)w * cap + j] = sv;
      r_nst[(size_t)w * cap + j] = nst[(size_t)w * n + e];
      // (st_dst may be st: each element is read above before this thread overwrites it)
      if (st_dst) st_dst[(size_t)w * n + e] = st_src[(size_t)w * n + e];
    }
    const uint8_t tv = tgt[e];
    r_tgt[j] = tv;
    if (tgt_dst) tgt_dst[e] = tgt_src[e];
    for (int k = 0; k < K; ++k) r_act[(size_t)j * K + k] = act[(size_t)e * K + k];
    r_rew[j] = rew[e];
    const uint8_t d = done_mask ? ((done[e] & done_mask) ? 1 : 0) : (done[e] ? 1 : 0);
    r_done[j] = d;
    if (done_out) done_out[e] = d;
  }
}

// ---- the learning frame's counters and the update's rows, one single-block launch
// (pbn_replay_advance): the env step index, the ring position and fill level after n_store
// transitions, epsilon's linear decay (decrement_epsilon, bdq_model/__init__.py:141-148, in fp64
// and its fp32 copy), then n_idx ring rows uniform over the new fill level: row b of draw c
// (*counter) is mulhi64(x << 32 | y, size) of Philox word pair (x, y) = REPLAY(seed, id = b,
// step = c) -- with replacement, as sample_indices; *counter then advances.  Replaces ~14
// one-element PyTorch launches of a captured frame.
__global__ void __launch_bounds__(256) replay_advance_kernel(int64_t n_store, int64_t cap, int64_t* __restrict__ pos,
                                                             int64_t* __restrict__ size, int64_t* __restrict__ step,
                                                             double* __restrict__ eps64, float* __restrict__ eps32,
                                                             double eps_final, double eps_step, int64_t n_idx,
                                                             uint64_t seed, int64_t* __restrict__ counter,
                                                             int64_t* __restrict__ idx) {
  pbn::frame_advance_block(n_store, cap, pos, size, step, eps64, eps32, eps_final, eps_step, n_idx, seed, counter,
                           idx, 0);
}

// ---- a replay batch in one pass (pbn_replay_batch): rows idx of the ring unpacked into the
// update's network input x = (2, 2B, N) (plane 0: the states in rows 0..B-1, the next states in
// rows B..2B-1; plane 1: the target attractor's first state for both), plus the actions as int64,
// the rewards and the done masks as float.  Replaces three index_selects, two obs unpacks, one
// concatenation and the five gathers and casts of the scalars.
__global__ void __launch_bounds__(kObsThreads) replay_batch_kernel(
    const int64_t* __restrict__ idx, int B, int64_t cap, const uint32_t* __restrict__ st,
    const uint32_t* __restrict__ nst, const uint8_t* __restrict__ tgt, const int32_t* __restrict__ act, int K,
    const float* __restrict__ rew, const uint8_t* __restrict__ done, const int32_t* __restrict__ att_start,
    const uint32_t* __restrict__ att_states, int n_attr, int N, int W, float* __restrict__ x,
    int64_t* __restrict__ act_out, float* __restrict__ rew_out, float* __restrict__ mask_out) {
  const int64_t rows = 2 * (int64_t)B;
  const int64_t total = rows * N;
  for (int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; f < total; f += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = f / N;
    const int i = (int)(f - r * N);
    const int b = (int)(r < B ? r : r - B);
    const int64_t j = idx[b];
    const uint32_t sw = (r < B ? st : nst)[(size_t)(i >> 5) * cap + j];
    const uint32_t tg = tgt[j];
    const uint32_t tw = tg < (uint32_t)n_attr ? att_states[(size_t)att_start[tg] * W + (i >> 5)] : 0u;
    x[f] = (float)((sw >> (i & 31)) & 1u);
    x[total + f] = (float)((tw >> (i & 31)) & 1u);
    if (i == 0 && r < B) {
      for (int k = 0; k < K; ++k) act_out[(size_t)b * K + k] = (int64_t)act[(size_t)j * K + k];
      rew_out[b] = rew[j];
      mask_out[b] = (float)done[j];
    }
  }
}

// ---- the learner's TD loss (bdq_model/__init__.py:111-126, bdq_update in pbn_rl_amd/replay.py)
// on raw head outputs: one pass where PyTorch runs both duelings, the online argmax, the two
// gathers, the target, the MSE and their backward (~25 launches at the update's batch).
// Per (row b, branch k), with heads [K+1][rows][A] (head 0 = value, output 0):
//   q(h, r, a)  = (v + adv_a) - mean(adv)            the dueling of row r (torch's expression)
//   current     = q(online, b, a_bk)
//   a*          = argmax_a q(online, B + b, a)      (first maximum, NaN maximal: torch.argmax)
//   expected    = r_b + (q(target, b, a*) * gamma) * m_b
//   loss        = sum (expected - current)^2 / (B K)
//   d loss / d online[k+1][b][j] = g (j == a_bk) - g / A,  d / d online[0][b][0] = sum_k g,
//   g = 2 (current - expected) / (B K); every other gradient entry (the rows B.. and the unused
//   value-head outputs) is 0.
// A block takes kTdRows rows: their head rows (online states, online next states, target) come
// into LDS with coalesced loads, one thread per (row, branch) pair does the arithmetic from LDS,
// and the block writes its gradient rows and one partial sum; a second one-block launch adds the
// partial sums in block order (fixed order: the loss is reproducible).
constexpr int kTdRows = 8;
constexpr int kTdThreads = 256;

__device__ __forceinline__ float td_mean(const float* __restrict__ adv, int A) {
  float s = 0.f;
  for (int j = 0; j < A; ++j) s += adv[j];
  return s / (float)A;
}

__global__ void __launch_bounds__(kTdThreads) td_loss_kernel(const float* __restrict__ on, const float* __restrict__ tg,
                                                             const int64_t* __restrict__ actions,
                                                             const float* __restrict__ rewards,
                                                             const float* __restrict__ masks, int B, int K, int A,
                                                             float gamma, float* __restrict__ partial,
                                                             float* __restrict__ grad) {
  extern __shared__ float sm[];
  const int H = K + 1;
  const int R = kTdRows;
  const int b0 = blockIdx.x * R;
  const int nr = min(R, B - b0);
  const int64_t rows = 2 * (int64_t)B;
  float* so = sm;                              // [H][2][R][A]: online rows b0.. and B + b0..
  float* st = so + (size_t)H * 2 * R * A;      // [H][R][A]: target rows b0..
  float* sg = st + (size_t)H * R * A;          // [R][K]: g per pair
  float* sd = sg + R * K;                      // [R][K]: (expected - current)^2 per pair
  const int t = threadIdx.x;
  const int per = nr * A;                      // floats of one head's block of rows
  for (int h = 0; h < H; ++h) {
    for (int i = t; i < per; i += kTdThreads) {
      so[((size_t)h * 2 + 0) * R * A + i] = on[((size_t)h * rows + b0) * A + i];
      so[((size_t)h * 2 + 1) * R * A + i] = on[((size_t)h * rows + B + b0) * A + i];
      st[(size_t)h * R * A + i] = tg[((size_t)h * B + b0) * A + i];
    }
  }
  __syncthreads();
  const float inv_bk = 1.f / (float)(B * K);
  if (t < nr * K) {
    const int r = t / K, k = t - r * K, b = b0 + r;
    const float* adv = so + ((size_t)(k + 1) * 2 + 0) * R * A + (size_t)r * A;
    const float v = so[(size_t)r * A];
    const int a = (int)actions[(size_t)b * K + k];
    const float current = (v + adv[a]) - td_mean(adv, A);
    const float* adv2 = so + ((size_t)(k + 1) * 2 + 1) * R * A + (size_t)r * A;
    const float v2 = so[(size_t)R * A + (size_t)r * A];
    const float m2 = td_mean(adv2, A);
    float best = (v2 + adv2[0]) - m2;
    int am = 0;
    for (int j = 1; j < A; ++j) {
      const float qj = (v2 + adv2[j]) - m2;
      const bool take = !isnan(best) && (isnan(qj) || qj > best);
      best = take ? qj : best;
      am = take ? j : am;
    }
    const float* tadv = st + (size_t)(k + 1) * R * A + (size_t)r * A;
    const float tnext = (st[(size_t)r * A] + tadv[am]) - td_mean(tadv, A);
    const float expected = rewards[b] + (tnext * gamma) * masks[b];
    const float d = expected - current;
    sd[t] = d * d;
    sg[t] = 2.f * (current - expected) * inv_bk;
  }
  __syncthreads();
  // gradient rows of this block, row-major and coalesced: head h, first-half row b0 + r, then the
  // second half's rows (zeros)
  for (int h = 0; h < H; ++h) {
    for (int i = t; i < per; i += kTdThreads) {
      const int r = i / A, j = i - r * A;
      float gv;
      if (h == 0) {
        float s = 0.f;
        for (int k = 0; k < K; ++k) s += sg[r * K + k];
        gv = j == 0 ? s : 0.f;
      } else {
        const float g = sg[r * K + h - 1];
        gv = (j == (int)actions[(size_t)(b0 + r) * K + h - 1] ? g : 0.f) - g / (float)A;
      }
      grad[((size_t)h * rows + b0) * A + i] = gv;
      grad[((size_t)h * rows + B + b0) * A + i] = 0.f;
    }
  }
  if (t == 0) {
    float s = 0.f;
    for (int p = 0; p < nr * K; ++p) s += sd[p];
    partial[blockIdx.x] = s;
  }
}

// the loss: the blocks' partial sums added in block order
__global__ void td_loss_sum_kernel(const float* __restrict__ partial, int n, float inv_bk, float* __restrict__ loss) {
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < n; ++i) s += partial[i];
    loss[0] = s * inv_bk;
  }
}

extern "C" {

int pbn_obs_unpack(const pbn_net* net, int64_t n_envs, const uint32_t* d_state, const uint8_t* d_target,
                   float* d_obs, void* stream) {
  pbn::NetView v;
  int rc = pbn::net_view(net, &v);
  if (rc) return rc;
  if ((rc = pbn::check_device(net))) return rc;
  if (n_envs < 0 || (n_envs & 31)) return pbn::set_error(PBN_EINVAL, "n_envs must be a non-negative multiple of 32");
  if ((int64_t)n_envs * v.n_nodes >= ((int64_t)1 << 31)) return pbn::set_error(PBN_EINVAL, "n_envs * n_nodes >= 2^31");
  if (n_envs == 0) return PBN_OK;
  if (!d_state || !d_target || !d_obs) return pbn::set_error(PBN_EINVAL, "null buffer");
  if (!aligned16(d_obs)) return pbn::set_error(PBN_EINVAL, "d_obs must be 16-byte aligned");
  const int64_t total4 = n_envs * v.n_nodes / 4;
  const unsigned blocks = (unsigned)std::min<int64_t>((total4 + kObsThreads - 1) / kObsThreads, 8192);
  hipLaunchKernelGGL(obs_unpack_kernel, dim3(blocks), dim3(kObsThreads), 0, (hipStream_t)stream, d_state, d_target,
                     v.att_start, v.att_states, v.n_attr, v.n_nodes, v.W, (uint32_t)n_envs, d_obs);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pbn::set_error(PBN_EDEVICE, hipGetErrorString(e));
  return PBN_OK;
}

int pbn_bilinear_targets(const pbn_net* net, int64_t n_envs, const uint32_t* d_state, const uint8_t* d_target,
                         const float* d_T, const float* d_bias, int32_t out_dim, int32_t leaky, float slope,
                         float* d_y, void* stream) {
  pbn::NetView v;
  int rc = pbn::net_view(net, &v);
  if (rc) return rc;
  if ((rc = pbn::check_device(net))) return rc;
  if (n_envs < 0 || (n_envs & 31)) return pbn::set_error(PBN_EINVAL, "n_envs must be a non-negative multiple of 32");
  if (n_envs >= ((int64_t)1 << 31) / 1024) return pbn::set_error(PBN_EINVAL, "n_envs too large");
  if (out_dim < 4 || out_dim > 1024 || (out_dim & 3)) return pbn::set_error(PBN_EINVAL, "out_dim must be a multiple of 4 in 4..1024");
  if (n_envs == 0) return PBN_OK;
  if (!d_state || !d_target || !d_bias || !d_y || (v.n_attr > 0 && !d_T)) return pbn::set_error(PBN_EINVAL, "null buffer");
  if (!aligned16(d_bias) || !aligned16(d_y) || (d_T && !aligned16(d_T)))
    return pbn::set_error(PBN_EINVAL, "d_T, d_bias and d_y must be 16-byte aligned");
  const uint32_t n = (uint32_t)n_envs;
  // the LDS-staged kernel when both table slices fit (A N <= 556 rows: Bittner-28's 14 x 28 and
  // pbn7's; not pbn70's 16 x 70) and the outputs come in 32-wide tiles; PBN_BILINEAR=l2 forces
  // the L2 kernel (tests compare the two)
  const size_t lds = (2 * (size_t)v.n_attr * v.n_nodes * 32 + (size_t)out_dim) * sizeof(float);
  const char* force = getenv("PBN_BILINEAR");
  if (v.n_attr > 0 && (out_dim & 31) == 0 && lds <= 140 * 1024 && !(force && !strcmp(force, "l2"))) {
    using K = void (*)(const uint32_t*, const uint8_t*, const float*, const float*, int, int, int, uint32_t, int,
                       float, float*);
    static const K kerns[4] = {bilinear_lds_kernel<1, kBlTpe>, bilinear_lds_kernel<2, kBlTpe>,
                               bilinear_lds_kernel<3, kBlTpe>, bilinear_lds_kernel<4, kBlTpe>};
    const K kern = kerns[v.W - 1];
    if (lds > 64 * 1024) {
      static bool raised[64] = {};
      const int dv = v.device >= 0 && v.device < 64 ? v.device : 0;
      if (!raised[dv]) {
        for (int w = 0; w < 4; ++w)
          if (hipFuncSetAttribute(reinterpret_cast<const void*>(kerns[w]), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024) != hipSuccess)
            return pbn::set_error(PBN_EDEVICE, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
        raised[dv] = true;
      }
    }
    const unsigned bl = (unsigned)((n_envs + kBlEnvs - 1) / kBlEnvs);
    hipLaunchKernelGGL(kern, dim3(bl), dim3(kBlEnvs * kBlTpe), lds, (hipStream_t)stream, d_state, d_target, d_T, d_bias,
                       v.n_nodes, v.n_attr, out_dim, n, leaky, slope, d_y);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return pbn::set_error(PBN_EDEVICE, hipGetErrorString(e));
    return PBN_OK;
  }
  const unsigned blocks = (unsigned)((n_envs + kBilEnvs - 1) / kBilEnvs);
  switch (v.W) {
    case 1: hipLaunchKernelGGL(bilinear_targets_kernel<1>, dim3(blocks), dim3(kBilThreads), 0, (hipStream_t)stream,
                               d_state, d_target, d_T, d_bias, v.n_nodes, v.n_attr, out_dim, n, leaky, slope, d_y); break;
    case 2: hipLaunchKernelGGL(bilinear_targets_kernel<2>, dim3(blocks), dim3(kBilThreads), 0, (hipStream_t)stream,
                               d_state, d_target, d_T, d_bias, v.n_nodes, v.n_attr, out_dim, n, leaky, slope, d_y); break;
    case 3: hipLaunchKernelGGL(bilinear_targets_kernel<3>, dim3(blocks), dim3(kBilThreads), 0, (hipStream_t)stream,
                               d_state, d_target, d_T, d_bias, v.n_nodes, v.n_attr, out_dim, n, leaky, slope, d_y); break;
    default: hipLaunchKernelGGL(bilinear_targets_kernel<4>, dim3(blocks), dim3(kBilThreads), 0, (hipStream_t)stream,
                                d_state, d_target, d_T, d_bias, v.n_nodes, v.n_attr, out_dim, n, leaky, slope, d_y); break;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pbn::set_error(PBN_EDEVICE, hipGetErrorString(e));
  return PBN_OK;
}

static int q_to_flipmask_impl(const pbn_net* net, uint64_t seed, uint64_t step, const uint64_t* d_step,
                              uint64_t env_offset, int64_t n_envs, int32_t n_branches, int32_t n_actions,
                              const float* d_q, float epsilon, const float* d_epsilon, uint32_t* d_flipmask,
                              int32_t* d_actions, void* stream, int heads = 0) {
  pbn::NetView v;
  int rc = pbn::net_view(net, &v);
  if (rc) return rc;
  if ((rc = pbn::check_device(net))) return rc;
  if (n_envs < 0 || (n_envs & 31) || (env_offset & 31))
    return pbn::set_error(PBN_EINVAL, "n_envs and env_offset must be multiples of 32");
  if (n_branches < 1 || n_branches > kMaxBranches) return pbn::set_error(PBN_EINVAL, "n_branches must be 1..7");
  if (n_actions != v.n_nodes + 1) return pbn::set_error(PBN_EINVAL, "n_actions must be n_nodes + 1");
  if (!(epsilon >= 0.f && epsilon <= 1.f)) return pbn::set_error(PBN_EINVAL, "epsilon must be in [0, 1]");
  if (n_envs == 0) return PBN_OK;
  if (!d_q || !d_flipmask) return pbn::set_error(PBN_EINVAL, "null buffer");
  if (!aligned16(d_q)) return pbn::set_error(PBN_EINVAL, "d_q must be 16-byte aligned");
  // explore iff word 0 < floor(epsilon * 2^32): epsilon = 1 always explores, 0 never
  const uint64_t eps_u = (uint64_t)floor((double)epsilon * 4294967296.0);
  const size_t lds = (size_t)kQEnvs * (n_branches + heads) * n_actions * sizeof(float) +
                    (size_t)kQEnvs * n_branches * sizeof(int);
  if (lds > 160 * 1024) return pbn::set_error(PBN_EINVAL, "n_branches * n_actions too large");
  if (lds > 64 * 1024) {   // beyond the default dynamic-LDS limit (e.g. heads of a 70-node network)
    static bool raised[64] = {};   // per device (a pbn_net is bound to one)
    const int dv = v.device >= 0 && v.device < 64 ? v.device : 0;
    if (!raised[dv]) {
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(q_to_flipmask_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
        return pbn::set_error(PBN_EDEVICE, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
      raised[dv] = true;
    }
  }
  const unsigned blocks = (unsigned)((n_envs + kQEnvs - 1) / kQEnvs);
  hipLaunchKernelGGL(q_to_flipmask_kernel, dim3(blocks), dim3(kQEnvs * n_branches), lds, (hipStream_t)stream, d_q, heads, n_branches,
                     n_actions, v.n_nodes, v.W, n_envs, seed, step, d_step, env_offset, eps_u, d_epsilon, d_flipmask, d_actions);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pbn::set_error(PBN_EDEVICE, hipGetErrorString(e));
  return PBN_OK;
}

int pbn_q_to_flipmask(const pbn_net* net, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n_envs,
                      int32_t n_branches, int32_t n_actions, const float* d_q, float epsilon, uint32_t* d_flipmask,
                      int32_t* d_actions, void* stream) {
  return q_to_flipmask_impl(net, seed, step, nullptr, env_offset, n_envs, n_branches, n_actions, d_q, epsilon,
                            nullptr, d_flipmask, d_actions, stream);
}

int pbn_q_to_flipmask_dev(const pbn_net* net, uint64_t seed, const uint64_t* d_step, uint64_t env_offset,
                          int64_t n_envs, int32_t n_branches, int32_t n_actions, const float* d_q, float epsilon,
                          const float* d_epsilon, uint32_t* d_flipmask, int32_t* d_actions, void* stream) {
  if (!d_step) return pbn::set_error(PBN_EINVAL, "null d_step");
  if (((uintptr_t)d_step & 7u) != 0) return pbn::set_error(PBN_EINVAL, "d_step must be 8-byte aligned");
  if (d_epsilon && ((uintptr_t)d_epsilon & 3u) != 0) return pbn::set_error(PBN_EINVAL, "d_epsilon misaligned");
  return q_to_flipmask_impl(net, seed, 0, d_step, env_offset, n_envs, n_branches, n_actions, d_q, epsilon,
                            d_epsilon, d_flipmask, d_actions, stream);
}

int pbn_heads_to_flipmask(const pbn_net* net, uint64_t seed, uint64_t step, const uint64_t* d_step,
                          uint64_t env_offset, int64_t n_envs, int32_t n_branches, int32_t n_actions,
                          const float* d_heads, float epsilon, const float* d_epsilon, uint32_t* d_flipmask,
                          int32_t* d_actions, void* stream) {
  if (d_step && ((uintptr_t)d_step & 7u) != 0) return pbn::set_error(PBN_EINVAL, "d_step must be 8-byte aligned");
  if (d_epsilon && ((uintptr_t)d_epsilon & 3u) != 0) return pbn::set_error(PBN_EINVAL, "d_epsilon misaligned");
  return q_to_flipmask_impl(net, seed, step, d_step, env_offset, n_envs, n_branches, n_actions, d_heads, epsilon,
                            d_epsilon, d_flipmask, d_actions, stream, 1);
}

int pbn_replay_store(int64_t n, const int64_t* d_pos, int64_t capacity, int32_t words, int32_t n_branches,
                     const uint32_t* d_state, const uint32_t* d_next_state, const uint8_t* d_target,
                     const int32_t* d_action, const float* d_reward, const uint8_t* d_done, uint32_t done_mask,
                     uint8_t* d_done_out, uint32_t* d_ring_state, uint32_t* d_ring_next_state, uint8_t* d_ring_target,
                     int32_t* d_ring_action, float* d_ring_reward, uint8_t* d_ring_done, uint32_t* d_state_dst,
                     const uint32_t* d_state_src, uint8_t* d_target_dst, const uint8_t* d_target_src, void* stream) {
  if ((d_state_dst != nullptr) != (d_state_src != nullptr) || (d_target_dst != nullptr) != (d_target_src != nullptr))
    return pbn::set_error(PBN_EINVAL, "state_dst / state_src and target_dst / target_src come in pairs");
  if (n < 1 || capacity < n || words < 1 || words > 4 || n_branches < 1)
    return pbn::set_error(PBN_EINVAL, "n >= 1, capacity >= n, words 1..4, n_branches >= 1");
  if (!d_pos || !d_state || !d_next_state || !d_target || !d_action || !d_reward || !d_done || !d_ring_state ||
      !d_ring_next_state || !d_ring_target || !d_ring_action || !d_ring_reward || !d_ring_done)
    return pbn::set_error(PBN_EINVAL, "null buffer");
  const unsigned blocks = (unsigned)std::min<int64_t>((n + kObsThreads - 1) / kObsThreads, 4096);
  hipLaunchKernelGGL(replay_store_kernel, dim3(blocks), dim3(kObsThreads), 0, (hipStream_t)stream, n, d_pos, capacity,
                     words, n_branches, d_state, d_next_state, d_target, d_action, d_reward, d_done, done_mask,
                     d_done_out, d_ring_state, d_ring_next_state, d_ring_target, d_ring_action, d_ring_reward,
                     d_ring_done, d_state_dst, d_state_src, d_target_dst, d_target_src);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pbn::set_error(PBN_EDEVICE, hipGetErrorString(e));
  return PBN_OK;
}

int pbn_replay_advance(int64_t n_store, int64_t capacity, int64_t* d_pos, int64_t* d_size, int64_t* d_step,
                       double* d_eps64, float* d_eps32, double eps_final, double eps_step, int64_t n_idx,
                       uint64_t seed, int64_t* d_counter, int64_t* d_idx, void* stream) {
  if (n_store < 0 || capacity < 1 || n_idx < 0) return pbn::set_error(PBN_EINVAL, "n_store >= 0, capacity >= 1, n_idx >= 0");
  if (!d_size || (n_store > 0 && !d_pos) || (n_idx > 0 && (!d_counter || !d_idx)))
    return pbn::set_error(PBN_EINVAL, "null buffer");
  hipLaunchKernelGGL(replay_advance_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, n_store, capacity, d_pos,
                     d_size, d_step, d_eps64, d_eps32, eps_final, eps_step, n_idx, seed, d_counter, d_idx);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pbn::set_error(PBN_EDEVICE, hipGetErrorString(e));
  return PBN_OK;
}

int pbn_replay_batch(const pbn_net* net, int64_t batch, const int64_t* d_idx, int64_t capacity,
                     const uint32_t* d_state, const uint32_t* d_next_state, const uint8_t* d_target,
                     const int32_t* d_action, int32_t n_branches, const float* d_reward, const uint8_t* d_done,
                     float* d_x, int64_t* d_actions, float* d_rewards, float* d_masks, void* stream) {
  pbn::NetView v;
  int rc = pbn::net_view(net, &v);
  if (rc) return rc;
  if ((rc = pbn::check_device(net))) return rc;
  if (batch < 1 || capacity < 1 || n_branches < 1) return pbn::set_error(PBN_EINVAL, "batch, capacity, n_branches >= 1");
  if (2 * batch * v.n_nodes >= ((int64_t)1 << 31)) return pbn::set_error(PBN_EINVAL, "batch too large");
  if (!d_idx || !d_state || !d_next_state || !d_target || !d_action || !d_reward || !d_done || !d_x || !d_actions ||
      !d_rewards || !d_masks)
    return pbn::set_error(PBN_EINVAL, "null buffer");
  const int64_t total = 2 * batch * v.n_nodes;
  const unsigned blocks = (unsigned)std::min<int64_t>((total + kObsThreads - 1) / kObsThreads, 4096);
  hipLaunchKernelGGL(replay_batch_kernel, dim3(blocks), dim3(kObsThreads), 0, (hipStream_t)stream, d_idx, (int)batch,
                     capacity, d_state, d_next_state, d_target, d_action, n_branches, d_reward, d_done, v.att_start,
                     v.att_states, v.n_attr, v.n_nodes, v.W, d_x, d_actions, d_rewards, d_masks);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pbn::set_error(PBN_EDEVICE, hipGetErrorString(e));
  return PBN_OK;
}

int pbn_bdq_td_loss(const float* d_online, const float* d_target, const int64_t* d_actions, const float* d_rewards,
                    const float* d_masks, int32_t batch, int32_t n_branches, int32_t n_actions, float gamma,
                    float* d_loss, float* d_grad, float* d_scratch, void* stream) {
  if (batch < 1 || n_branches < 1 || n_branches > 7 || n_actions < 1 || n_actions > 128)
    return pbn::set_error(PBN_EINVAL, "batch >= 1, n_branches 1..7, n_actions 1..128");
  if (!d_online || !d_target || !d_actions || !d_rewards || !d_masks || !d_loss || !d_grad || !d_scratch)
    return pbn::set_error(PBN_EINVAL, "null buffer");
  const int blocks = (batch + kTdRows - 1) / kTdRows;
  const int H = n_branches + 1;
  const size_t lds = ((size_t)H * 3 * kTdRows * n_actions + 2 * kTdRows * n_branches) * sizeof(float);
  if (lds > 64 * 1024 &&   // (up to 98 KB at 8 heads of 128 actions)
      hipFuncSetAttribute((const void*)td_loss_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return pbn::set_error(PBN_EDEVICE, "hipFuncSetAttribute failed");
  hipLaunchKernelGGL(td_loss_kernel, dim3(blocks), dim3(kTdThreads), lds, (hipStream_t)stream, d_online, d_target,
                     d_actions, d_rewards, d_masks, batch, n_branches, n_actions, gamma, d_scratch, d_grad);
  if (hipGetLastError() != hipSuccess) return pbn::set_error(PBN_EDEVICE, "td_loss_kernel launch failed");
  hipLaunchKernelGGL(td_loss_sum_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d_scratch, blocks,
                     1.f / (float)(batch * n_branches), d_loss);
  if (hipGetLastError() != hipSuccess) return pbn::set_error(PBN_EDEVICE, "td_loss_sum_kernel launch failed");
  return PBN_OK;
}

}  // extern "C"
