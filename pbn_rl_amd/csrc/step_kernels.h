// step_kernels.h -- the device side of libpbn_env.so: the step / rollout / reset / histogram
// kernels and their helpers (library-internal).  Included by pbn_env.hip (host side, the
// one-update instances) and pbn_settle.hip (the settle-law instances), so the two halves of
// the template instances compile in parallel.
#pragma once
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/pbn_env.h"
#include "bitslice.h"
#include "philox.h"

using pbn::bfi;
using pbn::Word4;

namespace {

constexpr int kFuncRecWords = 24;  // in[4], leaf[16], thr, pad[3]
constexpr int kNodeRecs = 4;       // compact records prefetched per node by the wave kernel
constexpr int kStatePrio = 2;      // s_setprio of the pipelined rollout's state wave

constexpr int kWavesPerBlock = 4;  // wave kernel: waves (32-env groups) per block, sharing one LDS table image
constexpr int kMaxHashBits = 12;

struct FuncRec {   // host-side function record (validation, leaf tables for the selectors)
  uint32_t in[4];      // input node index per mux level (padded with 0)
  uint32_t leaf[16];   // leaf[m] = d_m (x0 mask), leaf[8+m] = beta_m
  uint32_t thr;        // cumulative selection threshold c_f (prob_bits units)
  uint32_t pad[3];
};
static_assert(sizeof(FuncRec) == kFuncRecWords * 4, "FuncRec layout");

struct StepArgs {
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
  const uint64_t* step_ptr;     // single-step kernel: step index read from device memory (nullable)
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
  int wave_words;    // wave kernel: per-wave LDS words of S planes (after the shared table image)
  int gap_exact;     // 1: binary search for gaps (p == 0 or tiny); 0: log estimate + fix-up;
                     // 2: bucket table (gap_lut_off)
  int gap_lut_off;   // LDS image offset of the gap bucket table, uint2 [gap_nb + 1] {threshold, gap}
  int gap_shift;     // bucket of u = u >> gap_shift
  int gap_nb;        // buckets below C[N-1]; entry gap_nb is the sentinel {0xFFFFFFFF, N+1}
  float inv_log2q;   // 1 / log2(1 - p)
  const uint4* fcompact;   // [n_funcs] {inputs (4 x u8), truth table, threshold, 0}
  const uint4* nrec;       // [N * kNodeRecs] node-major copy of the first records (+ nf, f0 in .w)
  uint32_t hash_mult[4];
  unsigned long long* stamps;  // diagnostic builds (-DPBN_STAMPS) only: per-wave phase clocks
  int n_steps;       // steps per launch (wave kernel); outputs are [n_steps][...] arrays
  uint32_t* obs;     // [n_steps][W][n] observation before each step (nullable)
  int n_states;      // attractor states (bounds of att_states; checked builds)
  int att_off;       // LDS image offset of attractor start[A+1] | states[S][W] (wave kernel)
  int sel_off;       // LDS image offset of the leaf selectors, uint4 [kNodeRecs][2][32W] (wave kernel)
  int nrec_off;      // LDS image offset of the node records, record-major uint4 [kNodeRecs][32W]
  int cm_off;        // LDS image offset of pbn_rollout_pipe's threshold digit masks (W == 1),
                     // [32][sel_mask_stride(B)] lane-major
  int n_cls;         // 1..4: the first kNodeRecs thresholds of every node take one of n_cls values
                     // uthr[0..n_cls) (record .y = class index); 0: per-node thresholds
  uint32_t uthr[kNodeRecs];
  int max_nf;        // largest function count of a node
  int lq;            // pipelined rollout: selection masks per node in a slot (max(max_nf - 1, 1))
  int slot_words;    // pipelined rollout: words of one step slot
  int gate_off;      // wave kernel: LDS image offset of the gate records, uint4 [n_gates] by level
  int glayer_off;    // LDS image offset of the level starts, int32 [n_glayers + 1]
  int n_glayers;     // 0: no gates
  int att_single;    // every attractor is one state: the reset state is attractor a's state a
  uint32_t n1_magic; // ceil(2^32 / (N + 1)): random-action digits
  uint32_t am1_magic;  // ceil(2^32 / (A - 1)) for A >= 2: autoreset (start, target) split
  uint64_t x_mult;     // (N+1)^3 * A(A-1) (A >= 2) mod 2^64: what the ENV draws before gap 2 leave
                       // of X is X * x_mult (times the start attractor's size, multi-state nets)
  int sel_prio;        // pipelined rollout: raise the selection wave's priority (grids of at most
                       // four blocks per CU)
  int settle_max;      // step law: >= 2 = the settle law (wave kernel variants 3, 4,
                       // pbn_rollout_settle)
  uint16_t* updates;   // rollouts: [n_steps][n] synchronous updates applied per env-step (nullable)
  const uint32_t* sthr;  // settle law: thresholds scaled to 16 bits, [lq][32W] (65536 past a node's
                         // last function): the per-env selection compares (settle_lt_word)
  const uint32_t* sthr_pk;  // the same, node pairs packed biased for settle_lt_word_pk: [lq][W][16]
                            // {(C[2j+1] ^ 0x8000) << 16 | (C[2j] ^ 0x8000)}, C clamped to 65535
  int settle_pk;            // 1: every threshold a compare uses is below 65536 (sthr_pk is exact)
  // pbn_rollout_copy: cp_n16 16-byte vectors from cp_src to cp_dst ride along the launch (the
  // pipelined kernel's fourth wave, ride_copy_wave); 0: none.  cp_u: vectors per lane and step
  // iteration (paced: the block's share in n_steps + 1 portions, one per block barrier); 0: the
  // share in one burst
  const void* cp_src;
  void* cp_dst;
  int64_t cp_n16;
  int cp_u;
  // pbn_step_dev_store (ABI 11): the one-update wave kernel also writes the step's transitions into
  // a replay ring (pbn_replay_store's layout), env le at row (*r_pos + le) mod r_cap; r_state null:
  // none
  uint32_t* r_state;
  uint32_t* r_next;
  uint8_t* r_target;
  int32_t* r_action;
  float* r_reward;
  uint8_t* r_done;
  const int32_t* r_act_in;   // [n][r_k] the frame's branch actions
  uint8_t* r_done_out;       // nullable: [n]
  const int64_t* r_pos;
  int64_t r_cap;
  int r_k;
  uint32_t r_done_mask;
};

typedef unsigned int pbn_u32x4 __attribute__((ext_vector_type(4)));

constexpr int kRingMaxK = 8;   // pbn_step_dev_store: branch actions per env (BDQ: K + 1 <= kMaxHeads)

// In-kernel phase clocks (cdna_hip_programming.md section 7, "In-kernel stamps"):
// compiled only into the diagnostic library (-DPBN_STAMPS), never the product.
#ifdef PBN_STAMPS
#define PBN_STAMP(k)                                                                          \
  do {                                                                                        \
    unsigned long long t_;                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");               \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    if (a.stamps && (threadIdx.x & 63) == 0)                                                  \
      a.stamps[(size_t)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 32 + (k)] = t_; \
  } while (0)
// pipelined rollout: per role, clocks at the start of iteration 10, after its work, after the barrier;
// rows of 32 per block (tools/stamps.py): role r at 4r + {0, 1, 2}, HW_ID at 14 / 7 / 11, the
// segment clocks of the single-word fast paths at 15, 3, 12, 13 (state), 16, 17 (env), 18 (selection)
#define PBN_PSTAMP(k, slot_)                                                                  \
  do {                                                                                        \
    if ((k) == 10) {                                                                          \
      unsigned long long t_;                                                                  \
      __builtin_amdgcn_sched_barrier(0);                                                      \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");             \
      __builtin_amdgcn_sched_barrier(0);                                                      \
      if (a.stamps && (threadIdx.x & 63) == 0)                                                \
        a.stamps[(size_t)blockIdx.x * 32 + (threadIdx.x >> 6) * 4 + (slot_)] = t_;            \
    }                                                                                         \
  } while (0)
#define PBN_PSTAMP_AT(k, idx_)                                                                \
  do {                                                                                        \
    if ((k) == 10) {                                                                          \
      unsigned long long t_;                                                                  \
      __builtin_amdgcn_sched_barrier(0);                                                      \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");             \
      __builtin_amdgcn_sched_barrier(0);                                                      \
      if (a.stamps && (threadIdx.x & 63) == 0) a.stamps[(size_t)blockIdx.x * 32 + (idx_)] = t_; \
    }                                                                                         \
  } while (0)
// pipelined rollout, launch anatomy: the state wave's s_memrealtime (100 MHz, one clock for the
// whole chip) at kernel entry, after the table image, at the loop start, after iterations 0 and
// 1, after the loop and after its final stores have landed; row gridDim.x + block
#define PBN_RSTAMP(idx_)                                                                      \
  do {                                                                                        \
    unsigned long long t_;                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    if (a.stamps && threadIdx.x == 0) a.stamps[(size_t)(gridDim.x + blockIdx.x) * 32 + (idx_)] = t_; \
  } while (0)
#elif defined(PBN_ISA_MARKS)
// assembly listings only (tools/isa_budget.py compiles one instance with -S): each stamp site
// becomes a comment line in the listing, fenced so that no instruction crosses it; no code
#define PBN_ISA_MARK(txt)                                                                     \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    asm volatile(";@mark " txt);                                                              \
    __builtin_amdgcn_sched_barrier(0);                                                        \
  } while (0)
#define PBN_STAMP(k) do {} while (0)
#define PBN_PSTAMP(k, slot_) PBN_ISA_MARK("P" #slot_)
#define PBN_PSTAMP_AT(k, idx_) PBN_ISA_MARK("A" #idx_)
#define PBN_RSTAMP(idx_) PBN_ISA_MARK("R" #idx_)
// names the side of a runtime uniform branch it opens (tools/isa_budget.py --arms picks the live ones)
#define PBN_ISA_ARM(name_)                                                                    \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    asm volatile(";@arm " name_);                                                             \
    __builtin_amdgcn_sched_barrier(0);                                                        \
  } while (0)
// names the loop body it opens (role and compile-time variant) in the listing
#define PBN_ISA_LOOP(name_, v_)                                                               \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    asm volatile(";@loop " name_ " %0" ::"i"(v_));                                            \
    __builtin_amdgcn_sched_barrier(0);                                                        \
  } while (0)
#else
#define PBN_STAMP(k) do {} while (0)
#define PBN_PSTAMP(k, slot_) do {} while (0)
#define PBN_PSTAMP_AT(k, idx_) do {} while (0)
#define PBN_RSTAMP(idx_) do {} while (0)
#endif
#ifndef PBN_ISA_LOOP
#define PBN_ISA_LOOP(name_, v_) do {} while (0)
#define PBN_ISA_ARM(name_) do {} while (0)
#endif

// Bounds-checked global indexing for the diagnostic library (-DPBN_CHECKS): an
// out-of-range index is printed and redirected to element 0 instead of faulting.
#ifdef PBN_CHECKS
__device__ __noinline__ size_t pbn_ck(size_t i, size_t len, int site) {
  if (i < len) return i;
  printf("pbn OOB site %d idx %llu len %llu block %u thread %u\n", site, (unsigned long long)i,
         (unsigned long long)len, blockIdx.x, threadIdx.x);
  return 0;
}
#define CK(i, len, site) pbn_ck((size_t)(i), (size_t)(len), (site))
#else
#define CK(i, len, site) (i)
#endif

// ---------------------------------------------------------------- helpers
// Element (uniform base + lane element) of an output array addressed as a wave-uniform 64-bit
// base (SGPRs, advanced per step on the SALU) plus the lane's 32-bit byte offset: the
// global_store / global_load "saddr" form, with no 64-bit VGPR address pair and no per-step
// VALU address arithmetic (lane_elem * sizeof(T) < 2^32: n_envs < 2^30).  Checked builds keep
// the bounds-checked index.
template <typename T>
__device__ __forceinline__ T& lane_at(T* base, size_t uniform_elems, uint32_t lane_bytes) {
  // laundered so that loop strength reduction cannot turn the sum into a 64-bit VGPR
  // induction variable
  asm volatile("" : "+s"(uniform_elems));
  asm volatile("" : "+v"(lane_bytes));
  return *reinterpret_cast<T*>(reinterpret_cast<char*>(base + uniform_elems) + lane_bytes);
}
#ifdef PBN_CHECKS
#define LANE_AT(base, ubase, le_, len, site) (base)[CK((ubase) + (size_t)(le_), (len), (site))]
#else
#define LANE_AT(base, ubase, le_, len, site) lane_at((base), (ubase), (uint32_t)(le_) * (uint32_t)sizeof(*(base)))
#endif
// Streaming store of a rollout output (pbn_rollout_pipe): non-temporal, so that the per-step
// obs / flip-mask / reward / flags stream does not evict the table image from L2 between
// launches (every launch re-reads it)
#ifndef PBN_CHECKS
#define LANE_ST(base, ubase, le_, len, site, v) __builtin_nontemporal_store((v), &LANE_AT(base, ubase, le_, len, site))
#else
#define LANE_ST(base, ubase, le_, len, site, v) (LANE_AT(base, ubase, le_, len, site) = (v))
#endif
// LANE_ST with a per-lane element index (pbn_rollout_settle: every env is at its own step, so
// the step's base is not wave-uniform).  Write-back stores, not streaming ones: the few lanes
// that end a step in an iteration each write one element of a different output row, and a
// non-temporal partial-line write went to HBM as a whole write each time (WRITE_SIZE 21x the
// outputs' bytes, r05_t); through the L2 the lines fill up over the iterations before they are
// written back
// (r05_u: 495 -> 49 MB written per 20-step launch at config 2, +1 % on the settle line)
#define LANE_STV(base, idx, len, site, v) ((base)[CK((idx), (len), (site))] = (v))
__device__ __forceinline__ uint32_t valid_word_mask(int n, int w) {
  const int bits = n - 32 * w;
  return bits >= 32 ? 0xFFFFFFFFu : (bits <= 0 ? 0u : ((1u << bits) - 1u));
}

// One bounded draw from the 64-bit uniform X = (hi:lo), keeping the rest of X: v =
// floor(X * K / 2^64) in [0, K), X <- X * K mod 2^64 (two v_mad_u64_u32; bias <= K / 2^64;
// oracle/pbn_oracle.c ext64).
__device__ __forceinline__ uint32_t ext64(uint32_t& hi, uint32_t& lo, uint32_t K) {
  const uint64_t x = (uint64_t)lo * K;
  const uint64_t y = (uint64_t)hi * K + (x >> 32);
  lo = (uint32_t)x;
  hi = (uint32_t)y;
  return (uint32_t)(y >> 32);
}

// The LDS table image from global memory, all of a thread's loads issued before its stores
// (four loads in flight per thread, where a load-store loop waits once per element)
__device__ __forceinline__ void copy_image(uint32_t* L, const StepArgs& a) {
  // LDS-DMA (global_load_lds_dwordx4): every wave issues its share of the image at once, with no
  // VGPR round trip; the destination of a wave-instruction is base + 16 B x lane, so wave w
  // moves uint4s [base, base + 64) of each blockDim-wide stripe.  The caller's barrier waits for it.
  const int n4 = a.tab_words >> 2, lane = (int)threadIdx.x & 63;
  const uint4* src = reinterpret_cast<const uint4*>(a.tab);
  for (int base = (int)threadIdx.x - lane; base < n4; base += (int)blockDim.x) {
    if (base + lane < n4)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src + base + lane),
                                       (__attribute__((address_space(3))) void*)(L + 4 * base), 16, 0, 0);
  }
}

// LDS hash of the attractor states, slot-major: slot s holds its key words at [s * HS, s * HS +
// W) and the attractor id (0xFFFFFFFF: empty) at s * HS + W, HS = W + 1 rounded up to a power
// of two, so that one probe is one ds_read_b64 (W = 1) or ds_read_b128 (W = 2, 3)
template <int W>
struct HashStride {
  static constexpr int value = W == 1 ? 2 : (W <= 3 ? 4 : 8);
};

// attractor id of the state sp at slot s, or -1
template <int W>
__device__ __forceinline__ int hash_probe(const uint32_t* __restrict__ htab, uint32_t s, const uint32_t (&sp)[W]) {
  constexpr int HS = HashStride<W>::value;
  const uint32_t* e = htab + (size_t)s * HS;
  uint32_t ent[HS];
  if constexpr (HS == 2) {
    const uint2 v = *reinterpret_cast<const uint2*>(e);
    ent[0] = v.x; ent[1] = v.y;
  } else {
#pragma unroll
    for (int q = 0; q < HS / 4; ++q) {
      const uint4 v = reinterpret_cast<const uint4*>(e)[q];
      ent[4 * q] = v.x; ent[4 * q + 1] = v.y; ent[4 * q + 2] = v.z; ent[4 * q + 3] = v.w;
    }
  }
  bool eq = ent[W] != 0xFFFFFFFFu;
#pragma unroll
  for (int w = 0; w < W; ++w) eq = eq && ent[w] == sp[w];
  return eq ? (int)ent[W] : -1;
}

// Three actions uniform on [0, N]: the base-(N+1) digits of c, one draw over (N+1)^3.
// Division by N+1 is a multiply-high by magic = ceil(2^32 / (N+1)), exact for c * (N+1) < 2^32
// (c < (N+1)^3 <= 129^3).
template <int W>
__device__ __forceinline__ void actions_from_draw(uint32_t c, int N, uint32_t magic, uint32_t (&m)[W]) {
  const uint32_t n1 = (uint32_t)(N + 1);
#pragma unroll
  for (int q = 0; q < 3; ++q) {   // action a in [0, N]: 0 = no-op, else flip node a-1
    const uint32_t qt = __umulhi(c, magic);
    const int act = (int)(c - qt * n1);
    c = qt;
#pragma unroll
    for (int w = 0; w < W; ++w)
      if (act > 0 && ((act - 1) >> 5) == w) m[w] |= 1u << ((act - 1) & 31);
  }
}

// actions_from_draw for one word with N <= 31: action a sets bit a - 1 as 1 << (a - 1), where
// a = 0 shifts by 31 (the shift count's low five bits) onto a bit past the network that `vmask`
// (valid_word_mask(N, 0)) clears once for all three: no per-action guard
__device__ __forceinline__ uint32_t actions_mask31(uint32_t c, uint32_t n1, uint32_t magic, uint32_t vmask) {
  uint32_t m = 0;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const uint32_t qt = __umulhi(c, magic);
    m |= 1u << ((c - qt * n1 - 1u) & 31u);
    c = qt;
  }
  return m & vmask;
}

// gap(u) = min{m in 1..N : u < C[m-1]} (N+1 or more if none); C padded with 0xFFFFFFFF.
__device__ __forceinline__ int gap_of(const uint32_t* __restrict__ cdf, int len, uint32_t u) {
  int cnt = 0;
  for (int s = len >> 1; s >= 1; s >>= 1)
    if (cdf[cnt + s - 1] <= u) cnt += s;
  if (cdf[cnt] <= u) cnt += 1;
  return cnt + 1;
}

// lanes-of-32-envs bit mask of (u < c), u = digits dig[0..B) MSB first (B = prob_bits).
// From the least significant digit up: lt' = c_d ? (u_d ? lt : 1) : (u_d ? 0 : lt),
// one v_bitop3_b32 per digit over (u_d, lt, C_d) with LUT 0x8E.
__device__ __forceinline__ uint32_t less_than(const uint32_t (&dig)[16], uint32_t c, int B) {
  uint32_t lt = 0;
#pragma unroll
  for (int d = 15; d >= 0; --d) {
    if (d < B) {
      const uint32_t C = (uint32_t)__builtin_amdgcn_sbfe((int)c, B - 1 - d, 1);
      lt = __builtin_amdgcn_bitop3_b32(dig[d], lt, C, 0x8E);
    }
  }
  return lt;
}

// less_than with the threshold's digit masks read from LDS: cmq[d * stride] = ~0 if bit
// (B-1-d) of the threshold is set, else 0 (built once per block; saves a v_bfe per digit)
// pbn_rollout_pipe's threshold digit masks, lane-major: node i's masks of threshold q, digit d at
// cm[i * S + q * B + d], S = sel_mask_stride(B) words: four masks are one 16-byte ds_read_b128,
// and S = 4 x odd puts the 16 lanes of each read quarter on distinct 4-bank groups (conflict
// free; the node-major layout before it read two masks per ds_read2_b32, at twice the LDS-array
// cycles per mask)
__host__ __device__ constexpr int sel_mask_stride(int B) {
  return 4 * (((3 * B + 3) / 4) | 1);
}
template <int B>
__device__ __forceinline__ uint32_t less_than_cm4(const uint32_t (&dig)[16], const uint32_t* __restrict__ cmq) {
  const uint4* c4 = reinterpret_cast<const uint4*>(cmq);
  uint4 m[B / 4];
#pragma unroll
  for (int j = 0; j < B / 4; ++j) m[j] = c4[j];
  uint32_t lt = 0;
#pragma unroll
  for (int d = B - 1; d >= 0; --d) {
    const uint4 v = m[d >> 2];
    const uint32_t c = (d & 3) == 0 ? v.x : ((d & 3) == 1 ? v.y : ((d & 3) == 2 ? v.z : v.w));
    lt = __builtin_amdgcn_bitop3_b32(dig[d], lt, c, 0x8E);
  }
  return lt;
}

template <int B>
__device__ __forceinline__ uint32_t less_than_cm(const uint32_t (&dig)[16], const uint32_t* __restrict__ cmq,
                                                 int stride) {
  uint32_t lt = 0;
#pragma unroll
  for (int d = 15; d >= 0; --d) {
    if (d < B) lt = __builtin_amdgcn_bitop3_b32(dig[d], lt, cmq[d * stride], 0x8E);
  }
  return lt;
}

// ------------------------------------------- step kernel, one wave per 32-env group
//
// Lane j of the wave is env j (lanes 0-31) for the per-env work and node j (+32r) for
// the node work.  Blocks of kWavesPerBlock waves share one LDS copy of the tables; all
// global loads are issued before the Philox batch so their latency hides under it.
//   1. Philox: the lower half computes each env's ENV call and the first half of
//      its node's selection calls, the upper half the other selection calls plus
//      each env's first continuation-gap call; results meet via lane swaps;
//   2. per env (lower lanes): interventions, perturbation (gap = linear count
//      against the CDF in SGPRs for N <= 32), reset word;
//   3. 32x32 bit transposes as 5-stage cross-lane butterflies on DPP
//      (quad_perm, row_ror) and v_permlane16_swap: lane p ends up holding plane p;
//   4. lane i evaluates node i; selection digits stay in its registers;
//   5. butterfly back to per-env words, reward/termination/autoreset, stores.

// y = a of lane ^ J (J in 1, 2, 4, 8, 16), within 32-lane halves, without LDS
// ~0 on lanes with bit J of the lane index set, else 0 (a VGPR value: selecting with it
// needs no exec mask or SGPR pair, which the step loops cannot spare)
template <int J>
__device__ __forceinline__ uint32_t lane_bit_mask(int lane) {
  return 0u - (uint32_t)((lane & J) != 0);
}

// (every lane's DPP source is inside its row for these controls, so each lane is written and
// the "old" operand is never used: mov_dpp leaves it undefined, which saves the v_mov that
// update_dpp(0, ...) spends initialising the destination)
template <int J>
__device__ __forceinline__ uint32_t xor_lane(uint32_t a, int lane) {
  if constexpr (J == 1) {
    return __builtin_amdgcn_mov_dpp(a, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
  } else if constexpr (J == 2) {
    return __builtin_amdgcn_mov_dpp(a, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
  } else if constexpr (J == 4) {
    const uint32_t r4 = __builtin_amdgcn_mov_dpp(a, 0x124, 0xF, 0xF, true);   // row_ror:4
    const uint32_t r12 = __builtin_amdgcn_mov_dpp(a, 0x12C, 0xF, 0xF, true);  // row_ror:12
    return pbn::bfi3(lane_bit_mask<4>(lane), r4, r12);
  } else if constexpr (J == 8) {
    return __builtin_amdgcn_mov_dpp(a, 0x128, 0xF, 0xF, true);  // row_ror:8
  } else {
    const auto r = __builtin_amdgcn_permlane16_swap(a, a, false, false);
    return pbn::bfi3(lane_bit_mask<16>(lane), r[0], r[1]);
  }
}

// the ride-along copy of pbn_rollout_copy: a fourth wave per block (launched only when there is a
// copy) moves the block's contiguous share of the vectors and exits; s_barrier waits for the
// surviving waves only, so the three step roles run as without it.
//   burst (cp_u = 0): the share at once, kDepth 1-KB loads per lane in flight;
//   paced (cp_u = U): the share in n_steps + 1 portions of U vectors per lane, portion k stored
//   at iteration k's block barrier and requested A = 4 / U iterations ahead, so the copy's HBM
//   traffic spreads over the launch instead of competing with its first iterations (the burst:
//   0.65x of the bare launches' rate at 2,000 steps, paced 0.89x; r05_y, r05_za).
// (The copy folded into the env-draw waves' step loop held every iteration to the loads'
// latency: +48 us on a 100-step launch of 65,536 envs, r05_u, profiles/r05_u_ride_env_wave.patch.)
__device__ __forceinline__ void ride_copy_burst(const StepArgs& a, int lane) {
  constexpr int kDepth = 8;
  const int64_t per = ((a.cp_n16 + (int64_t)gridDim.x - 1) / (int64_t)gridDim.x + 63) & ~(int64_t)63;
  const int64_t i0 = (int64_t)blockIdx.x * per;
  const int64_t i1 = min(i0 + per, a.cp_n16);
  const pbn_u32x4* src = static_cast<const pbn_u32x4*>(a.cp_src);
  pbn_u32x4* dst = static_cast<pbn_u32x4*>(a.cp_dst);
  for (int64_t base = i0 + lane; base < i1; base += kDepth * 64) {
    pbn_u32x4 v[kDepth];
#pragma unroll
    for (int u = 0; u < kDepth; ++u)
      if (base + u * 64 < i1) v[u] = __builtin_nontemporal_load(src + base + u * 64);
#pragma unroll
    for (int u = 0; u < kDepth; ++u)
      if (base + u * 64 < i1) __builtin_nontemporal_store(v[u], dst + base + u * 64);
  }
}

// vectors per lane in flight in the paced copy: 4 measured 0.89x of the bare launches at 2,000
// steps, 2 0.69x, 8 0.81x, 16 (spills) 0.44x (profiles/r05_za_ab.json, r05_z)
constexpr int kRideVecs = 4;
template <int U>
__device__ __forceinline__ void ride_copy_paced(const StepArgs& a, int lane) {
  constexpr int A = kRideVecs / U > 0 ? kRideVecs / U : 1;   // portions in flight
  const int iters = a.n_steps + 1;
  const int64_t per = (int64_t)iters * U * 64;   // the host sized U so that the grid covers cp_n16
  const int64_t i0 = (int64_t)blockIdx.x * per + lane;
  const int64_t i1 = a.cp_n16;
  const pbn_u32x4* src = static_cast<const pbn_u32x4*>(a.cp_src);
  pbn_u32x4* dst = static_cast<pbn_u32x4*>(a.cp_dst);
  pbn_u32x4 v[A][U];
  auto load = [&](int k, pbn_u32x4 (&r)[U]) {
    if (k >= iters) return;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + ((int64_t)k * U + u) * 64;
      if (i < i1) r[u] = __builtin_nontemporal_load(src + i);   // (plain loads: equal, r05_z)
    }
  };
  auto store = [&](int k, const pbn_u32x4 (&r)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + ((int64_t)k * U + u) * 64;
      if (i < i1) __builtin_nontemporal_store(r[u], dst + i);
    }
  };
#pragma unroll
  for (int j = 0; j < A; ++j) load(j, v[j]);
  for (int k0 = 0; k0 < iters; k0 += A) {
#pragma unroll
    for (int j = 0; j < A; ++j) {
      const int k = k0 + j;
      if (k >= iters) return;
      store(k, v[j]);
      load(k + A, v[j]);
      __builtin_amdgcn_s_barrier();   // the block's barrier of iteration k (no LDS to fence)
    }
  }
}

__device__ __forceinline__ void ride_copy_wave(const StepArgs& a, int lane) {
  switch (a.cp_u) {
    case 1: ride_copy_paced<1>(a, lane); break;
    case 2: ride_copy_paced<2>(a, lane); break;
    case 4: ride_copy_paced<4>(a, lane); break;
    default: ride_copy_burst(a, lane); break;
  }
}

// one butterfly stage: lanes without bit J keep their M bits and take the partner's M bits
// shifted up by J; lanes with bit J take the partner's ~M bits shifted down.  Branch-free: the
// shift is a per-lane rotate (v_alignbit_b32; wrapped bits land outside the kept field) and
// the field a per-lane mask.
template <int J>
__device__ __forceinline__ uint32_t transpose_step(uint32_t a, int lane) {
  constexpr uint32_t M = J == 16 ? 0x0000FFFFu : (J == 8 ? 0x00FF00FFu : (J == 4 ? 0x0F0F0F0Fu : (J == 2 ? 0x33333333u : 0x55555555u)));
  const uint32_t y = xor_lane<J>(a, lane);
  const uint32_t up = lane_bit_mask<J>(lane);
  const uint32_t rot = __builtin_amdgcn_alignbit(y, y, (32u - J) ^ (up & ((32u - J) ^ (uint32_t)J)));
  return pbn::bfi3(M ^ ~up, rot, a);
}

// the partner value of lane ^ J within 32-lane halves through the LDS crossbar (ds_swizzle,
// bit mode: and 0x1F, xor J): no VALU issue slot, where DPP cannot cross rows of 16 lanes
template <int J>
__device__ __forceinline__ uint32_t swizzle_xor(uint32_t a) {
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)a, (J << 10) | 0x1F);
}

// byte-granular stages (J = 16, 8) as one v_perm_b32 with a per-lane selector: the shift and
// the field select of transpose_step in one instruction.  perm(y, a, sel): bytes 0-3 are a's,
// 4-7 the partner's.
//   J = 16: low lanes [a0 a1 y0 y1], high lanes [y2 y3 a2 a3]
//   J = 8:  low lanes [a0 y0 a2 y2], high lanes [y1 a1 y3 a3]
template <int J>
__device__ __forceinline__ uint32_t perm_sel(int lane) {
  if constexpr (J == 16) return (lane & 16) ? 0x03020706u : 0x05040100u;
  else return (lane & 8) ? 0x03070105u : 0x06020400u;
}

// lane k holds row k of a 32x32 bit matrix (per 32-lane half); afterwards lane c holds column c.
// 11 VALU (J = 16: swizzle + perm; 8: DPP + perm; 4: swizzle + alignbit + bitop3; 2, 1: DPP +
// alignbit + bitop3) where five transpose_step spend 20.
__device__ __forceinline__ uint32_t lane_transpose32(uint32_t a, int lane) {
  a = __builtin_amdgcn_perm(swizzle_xor<16>(a), a, perm_sel<16>(lane));
  a = __builtin_amdgcn_perm(xor_lane<8>(a, lane), a, perm_sel<8>(lane));
  {
    const uint32_t y = swizzle_xor<4>(a);
    const uint32_t up = lane_bit_mask<4>(lane);
    const uint32_t rot = __builtin_amdgcn_alignbit(y, y, 28u ^ (up & (28u ^ 4u)));
    a = pbn::bfi3(0x0F0F0F0Fu ^ ~up, rot, a);
  }
  a = transpose_step<2>(a, lane);
  a = transpose_step<1>(a, lane);
  return a;
}

// eval of a lane-varying function from its compact record: 4 input planes, 16-bit
// truth table T; leaf masks are sign-extended table bits (v_bfe_i32).
__device__ __forceinline__ uint32_t eval_compact(uint32_t ins, uint32_t T, const uint32_t* __restrict__ S) {
  const uint32_t x0 = S[ins & 0xFFu], x1 = S[(ins >> 8) & 0xFFu], x2 = S[(ins >> 16) & 0xFFu], x3 = S[ins >> 24];
  uint32_t v[8];
#pragma unroll
  for (int mm = 0; mm < 8; ++mm) {
    const uint32_t l0 = (uint32_t)__builtin_amdgcn_sbfe((int)T, 2 * mm, 1);
    const uint32_t l1 = (uint32_t)__builtin_amdgcn_sbfe((int)T, 2 * mm + 1, 1);
    v[mm] = bfi(x0, l1, l0);
  }
  const uint32_t w0 = bfi(x1, v[1], v[0]), w1 = bfi(x1, v[3], v[2]), w2 = bfi(x1, v[5], v[4]), w3 = bfi(x1, v[7], v[6]);
  return bfi(x3, bfi(x2, w3, w2), bfi(x2, w1, w0));
}

// eval from per-lane leaf selectors: leaf m = (T bit 2m, T bit 2m+1) = (value at x0 = 0,
// value at x0 = 1) is one of {0, x0, ~x0, ~0}, i.e. per byte one v_perm_b32 of {~x0 : x0}
// with selector byte j, 4 + j, 12 (0x00) or 13 (0xFF); the selectors are built on the host.
__device__ __forceinline__ uint32_t eval_sel(uint32_t ins, uint4 sa, uint4 sb, const uint32_t* __restrict__ S) {
  const uint32_t x0 = S[ins & 0xFFu], x1 = S[(ins >> 8) & 0xFFu], x2 = S[(ins >> 16) & 0xFFu], x3 = S[ins >> 24];
  const uint32_t nx0 = ~x0;
  const uint32_t v0 = __builtin_amdgcn_perm(nx0, x0, sa.x), v1 = __builtin_amdgcn_perm(nx0, x0, sa.y);
  const uint32_t v2 = __builtin_amdgcn_perm(nx0, x0, sa.z), v3 = __builtin_amdgcn_perm(nx0, x0, sa.w);
  const uint32_t v4 = __builtin_amdgcn_perm(nx0, x0, sb.x), v5 = __builtin_amdgcn_perm(nx0, x0, sb.y);
  const uint32_t v6 = __builtin_amdgcn_perm(nx0, x0, sb.z), v7 = __builtin_amdgcn_perm(nx0, x0, sb.w);
  const uint32_t w0 = bfi(x1, v1, v0), w1 = bfi(x1, v3, v2), w2 = bfi(x1, v5, v4), w3 = bfi(x1, v7, v6);
  return bfi(x3, bfi(x2, w3, w2), bfi(x2, w1, w0));
}

// eval_sel with the four input planes already read
__device__ __forceinline__ uint32_t eval_sel_in(const uint32_t (&x)[4], uint4 sa, uint4 sb) {
  const uint32_t x0 = x[0], nx0 = ~x0;
  const uint32_t v0 = __builtin_amdgcn_perm(nx0, x0, sa.x), v1 = __builtin_amdgcn_perm(nx0, x0, sa.y);
  const uint32_t v2 = __builtin_amdgcn_perm(nx0, x0, sa.z), v3 = __builtin_amdgcn_perm(nx0, x0, sa.w);
  const uint32_t v4 = __builtin_amdgcn_perm(nx0, x0, sb.x), v5 = __builtin_amdgcn_perm(nx0, x0, sb.y);
  const uint32_t v6 = __builtin_amdgcn_perm(nx0, x0, sb.z), v7 = __builtin_amdgcn_perm(nx0, x0, sb.w);
  const uint32_t w0 = bfi(x[1], v1, v0), w1 = bfi(x[1], v3, v2), w2 = bfi(x[1], v5, v4), w3 = bfi(x[1], v7, v6);
  return bfi(x[3], bfi(x[2], w3, w2), bfi(x[2], w1, w0));
}

// gap(u) = min{m : u < C[m-1]} from a float estimate of log(1-x)/log(1-p) corrected
// exactly (+-1) against the integer CDF in LDS; C padded with 0xFFFFFFFF.
__device__ __forceinline__ int gap_est(const uint32_t* __restrict__ cdf, int len, float inv_log2q, uint32_t u) {
  const float x = (float)u * 2.3283064365386963e-10f;   // u / 2^32
  const float l2 = __builtin_amdgcn_logf(1.0f - x);     // v_log_f32: log2
  float est = floorf(l2 * inv_log2q) + 1.0f;
  est = fminf(fmaxf(est, 1.0f), (float)len);
  int g = (int)est;
  // C[g-2] and C[g-1] as one pair of adjacent reads (no branch: g == 1 reads C[0], C[1])
  const int base = g >= 2 ? g - 2 : 0;
  const uint32_t c0 = cdf[base], c1 = cdf[base + 1];
  const uint32_t hi = g >= 2 ? c1 : c0;                 // C[g-1]
  const uint32_t lo = g >= 2 ? c0 : 0u;                 // C[g-2]
  g += (u >= hi) ? 1 : 0;
  g -= (g >= 2 && u < lo) ? 1 : 0;
  return g;
}

// gap(u) from the bucket table: within a bucket of u (its top bits) the gap takes at most two
// values, lo and lo + 1, split at threshold C[lo-1]; buckets from C[N-1] on share one sentinel
// entry (gap N+1, no flip).  One LDS read and two VALU ops, where gap_est spends ~22.
__device__ __forceinline__ int gap_lut(const uint2* __restrict__ lut, int shift, int nb, uint32_t u) {
  const uint32_t b = min(u >> shift, (uint32_t)nb);
  const uint2 e = lut[b];
  return (int)e.y + (u >= e.x ? 1 : 0);
}

// one gap by the net's method (mode: 0 estimate, 1 binary search, 2 bucket table)
__device__ __forceinline__ int gap_any(int mode, const uint32_t* __restrict__ L, const StepArgs& a, uint32_t u) {
  if (mode == 2) return gap_lut(reinterpret_cast<const uint2*>(L + a.gap_lut_off), a.gap_shift, a.gap_nb, u);
  return mode ? gap_of(L, a.cdf_len, u) : gap_est(L, a.cdf_len, a.inv_log2q, u);
}

// (u < c_q) for the wave-uniform threshold classes: one bit-sliced comparison per class with
// SGPR digit masks, then a per-lane pick by class index (record .y)
template <int B>
__device__ __forceinline__ void class_masks(const uint32_t (&dig)[16], const uint32_t (&uthr)[kNodeRecs], int n_cls,
                                            uint32_t (&ltc)[kNodeRecs]) {
#pragma unroll
  for (int v = 0; v < kNodeRecs; ++v) {
    ltc[v] = 0;
    if (v < n_cls) {
      uint32_t c = uthr[v];
      asm volatile("" : "+s"(c));   // digits re-extracted per step on the SALU (hoisted: SGPR spills)
      ltc[v] = less_than(dig, c, B);
    }
  }
}

__device__ __forceinline__ uint32_t pick_class(const uint32_t (&ltc)[kNodeRecs], uint32_t cls) {
  return cls == 0 ? ltc[0] : (cls == 1 ? ltc[1] : (cls == 2 ? ltc[2] : ltc[3]));
}

// Lower lanes receive the upper lanes' four words (upper lanes end with junk): per pair of
// words two v_permlane32_swap and no copies.  swap(X, Y) moves X's upper half into Y's
// lower half; swap(Y', X') then moves Y's upper half into X''s lower half.
__device__ __forceinline__ pbn::Word4 upper_to_lower(pbn::Word4 v) {
  const auto a1 = __builtin_amdgcn_permlane32_swap(v.x, v.y, false, false);
  const auto a2 = __builtin_amdgcn_permlane32_swap(a1[1], a1[0], false, false);
  const auto b1 = __builtin_amdgcn_permlane32_swap(v.z, v.w, false, false);
  const auto b2 = __builtin_amdgcn_permlane32_swap(b1[1], b1[0], false, false);
  return pbn::Word4{a2[0], a2[1], b2[0], b2[1]};
}

template <int W>
__device__ __forceinline__ void set_bit(uint32_t (&g)[W], int pos, int N) {
#pragma unroll
  for (int w = 0; w < W; ++w)
    if ((unsigned)pos < (unsigned)N && (pos >> 5) == w) g[w] |= 1u << (pos & 31);
}

// attractor id of the per-env state sp (open-addressing LDS hash; keys are unique, so the probe
// order does not matter: the first four probes are read side by side), or -1
template <int W>
__device__ __forceinline__ int attractor_lookup(const StepArgs& a, const uint32_t* __restrict__ htab,
                                                const uint32_t (&sp)[W]) {
  int att = -1;
  if (a.hash_bits > 0) {
    PBN_ISA_ARM("hash");
    const uint32_t hmask = (1u << a.hash_bits) - 1u;
    uint32_t h = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) h += sp[w] * a.hash_mult[w];
    h >>= (32 - a.hash_bits);
    // the first probe always (h < 2^bits needs no mask); the table is usually collision free
    // (hash_probes = 1: every bundled network), so the others sit behind a uniform branch
    att = hash_probe<W>(htab, h, sp);
    if (a.hash_probes > 1) {
      PBN_ISA_ARM("hash_more_probes");
      for (int pr = 1; pr < a.hash_probes; ++pr) {
        const int id = hash_probe<W>(htab, (h + pr) & hmask, sp);
        if (id >= 0) att = id;
      }
    }
  }
  return att;
}

// combinational gates of the lowered wide functions (lowering.py), level by level, all 64 lanes:
// gate record {input S indices, 16-bit table, output S index}; one wave's LDS operations execute
// in order, so level l + 1 reads what level l wrote
__device__ __forceinline__ void eval_gate_levels(const StepArgs& a, const uint32_t* __restrict__ L, uint32_t* S,
                                                 int lane) {
  const uint4* grec = reinterpret_cast<const uint4*>(L + a.gate_off);
  const int32_t* glev = reinterpret_cast<const int32_t*>(L + a.glayer_off);
  for (int lv = 0; lv < a.n_glayers; ++lv) {
    const int end = glev[lv + 1];
    for (int gi = glev[lv] + lane; gi < end; gi += 64) {
      const uint4 r = grec[gi];
      S[r.z] = eval_compact(r.x, r.y, S);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// The settle law's per-env selection (oracle/pbn_oracle.c env_uniforms): the 16 words of env
// ge's SETTLE_SEL calls 4r .. 4r+3 for update k; node 32r + b's 16-bit field is b & 1 of
// U[b >> 1].  Calls past the network's last node are not made (U = 0).
// XM: xor-ed into words 0 and 2 of every call (philox's last-round keys; settle_lt_word_pk's bias)
template <uint32_t XM = 0u>
__device__ __forceinline__ void settle_sel_words(uint32_t ge_lo, uint32_t ge_hi, uint32_t st_lo, uint32_t k, int r,
                                                 int N, uint32_t k0, uint32_t k1, uint32_t (&U)[16]) {
  const uint32_t c2 = (pbn::kStreamSettleSel << 28) | (k << 8) | (uint32_t)(4 * r);
  if (32 * r + 24 < N) {   // every call (a word of more than 24 nodes): in one block, interleaved
    PBN_ISA_ARM("sel_all_calls");
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const Word4 P = pbn::philox<pbn::kPhiloxRounds, XM>(ge_lo, st_lo, c2 | (uint32_t)c, ge_hi, k0, k1);
      U[4 * c + 0] = P.x; U[4 * c + 1] = P.y; U[4 * c + 2] = P.z; U[4 * c + 3] = P.w;
    }
  } else {
    PBN_ISA_ARM("sel_some_calls");
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      Word4 P = {0u, 0u, 0u, 0u};
      if (32 * r + 8 * c < N) P = pbn::philox<pbn::kPhiloxRounds, XM>(ge_lo, st_lo, c2 | (uint32_t)c, ge_hi, k0, k1);
      U[4 * c + 0] = P.x; U[4 * c + 1] = P.y; U[4 * c + 2] = P.z; U[4 * c + 3] = P.w;
    }
  }
}

// env-major selection word of one threshold: bit b = (field of node 32r + b < C[b]), C = the
// thresholds scaled to 16 bits (c << (16 - B); 65536 past a node's last function: sthr), most
// significant node first.  Per node one subtract (the field selected by SDWA) whose sign is the
// compare (both operands <= 2^16) and one v_alignbit_b32 that shifts it in: (lt:d) >> 31.  C is
// read through the constant address space, so the 32 thresholds of a row are scalar loads.
using ConstU32 = const __attribute__((address_space(4))) uint32_t;
__device__ __forceinline__ uint32_t settle_lt_word(const uint32_t (&U)[16], const uint32_t* C_) {
  ConstU32* C = (ConstU32*)C_;
  uint32_t lt = 0;
#pragma unroll
  for (int b = 31; b >= 0; --b) {
    const uint32_t u = (b & 1) ? (U[b >> 1] >> 16) : (U[b >> 1] & 0xFFFFu);
    lt = __builtin_amdgcn_alignbit(lt, u - C[b], 31);
  }
  return lt;
}

// settle_lt_word two nodes per instruction: U biased (^ 0x80008000) makes each 16-bit field a
// signed value whose order is the unsigned one, so the saturating v_pk_sub_i16 of the packed biased
// thresholds has the sign of (u < C) in bits 15 and 31 of each node pair's difference.  v_perm_b32's
// sign-replicating selectors (8-11: byte 1, 3, 5, 7's bit 7 as 0x00 / 0xFF) turn two pairs (four
// nodes) into four byte masks, and v_and_or_b32 drops four-node word m at bit offset m of every
// byte: bit 8c + m of the result = node 4m + c (pk_lane_node, the inverse, is applied at the
// planes' LDS write).  32 VALU per 32 nodes where settle_lt_word spends 64.
typedef short s16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t settle_lt_word_pk(const uint32_t (&Ub)[16], const uint32_t* Cpk_) {
  ConstU32* Cpk = (ConstU32*)Cpk_;
  uint32_t d[16];
#pragma unroll
  for (int j = 0; j < 16; ++j)
    d[j] = __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(s16x2_t, Ub[j]),
                                                                     __builtin_bit_cast(s16x2_t, Cpk[j])));
  uint32_t lt = 0;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    // byte masks: node 4m (d[2m] bit 15), 4m+1 (d[2m] bit 31), 4m+2 (d[2m+1] bit 15), 4m+3 (d[2m+1] bit 31)
    const uint32_t e = __builtin_amdgcn_perm(d[2 * m + 1], d[2 * m], 0x0B0A0908u);
    lt = (e & (0x01010101u << m)) | lt;
  }
  return lt;
}
// settle_lt_word_pk with the packed thresholds in registers (read from the kernel's LDS copy
// ahead of the iteration's Philox calls: as scalar loads next to their use, two s_waitcnt on the
// selection wave's chain)
__device__ __forceinline__ uint32_t settle_lt_word_pk_v(const uint32_t (&Ub)[16], const uint4 (&Cv)[4]) {
  uint32_t d[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint4 c4 = Cv[j >> 2];
    const uint32_t c = (j & 3) == 0 ? c4.x : ((j & 3) == 1 ? c4.y : ((j & 3) == 2 ? c4.z : c4.w));
    d[j] = __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(s16x2_t, Ub[j]),
                                                                     __builtin_bit_cast(s16x2_t, c)));
  }
  uint32_t lt = 0;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const uint32_t e = __builtin_amdgcn_perm(d[2 * m + 1], d[2 * m], 0x0B0A0908u);
    lt = (e & (0x01010101u << m)) | lt;
  }
  return lt;
}
// the node whose plane lane l32 holds after transposing a settle_lt_word_pk word
__device__ __forceinline__ int pk_lane_node(int l32) { return 4 * (l32 & 7) + (l32 >> 3); }

// node l32 + 32r on lane l32: the rule update of every env of the group from the bit-sliced
// planes S, the selection digit planes dig (perturbed envs are replaced by the caller)
template <int W, int B>
__device__ __forceinline__ void node_update(const StepArgs& a, const uint4 (&rec_)[W][kNodeRecs],
                                            const uint4* __restrict__ selq, const uint32_t* __restrict__ S,
                                            const uint32_t (&dig)[W][16], bool lo, int l32, uint32_t (&X)[W]) {
  const int N = a.n_nodes;
#pragma unroll
  for (int r = 0; r < W; ++r) {
    X[r] = 0;
    const int i = l32 + 32 * r;
    const int ii = lo && i < N ? i : 0;   // other lanes evaluate node 0 and discard it
    uint32_t x = 0;
    if (a.n_cls > 0 && a.max_nf <= kNodeRecs) {
      // thresholds from a few wave-uniform classes (all kaban networks: 1/3, 2/3)
      const int nf = (int)rec_[r][0].w;
      uint32_t ltc[kNodeRecs];
      class_masks<B>(dig[r], a.uthr, a.n_cls, ltc);
#pragma unroll
      for (int q = kNodeRecs - 1; q >= 0; --q) {
        if (q < a.max_nf) {
          const uint4 rc = rec_[r][q];
          const uint32_t fj = eval_sel(rc.x, selq[(2 * q) * 32 * W + ii], selq[(2 * q + 1) * 32 * W + ii], S);
          const uint32_t y = (q == nf - 1) ? fj : bfi(pick_class(ltc, rc.y), fj, x);
          x = (q < nf) ? y : x;
        }
      }
    } else {
      const int nf = (int)rec_[r][0].w;
      const int f0 = (int)rec_[r][1].w;
      // selection chain from the last function down: x = F_{nf-1}; x = lt_j ? F_j : x
      for (int j = nf - 1; j >= kNodeRecs; --j) {   // nodes with more than kNodeRecs functions (slow path)
        const uint4 rc = a.fcompact[CK(f0 + j, a.n_funcs, 9)];
        const uint32_t fj = eval_compact(rc.x, rc.y, S);
        x = (j == nf - 1) ? fj : bfi(less_than(dig[r], rc.z, B), fj, x);
      }
#pragma unroll
      for (int q = kNodeRecs - 1; q >= 0; --q) {
        if (q < nf) {
          const uint4 rc = rec_[r][q];
          const uint32_t fj = eval_sel(rc.x, selq[(2 * q) * 32 * W + ii], selq[(2 * q + 1) * 32 * W + ii], S);
          x = (q == nf - 1) ? fj : bfi(less_than(dig[r], rc.z, B), fj, x);
        }
      }
    }
    if (lo && i < N) X[r] = x;
  }
}

// settle law: node l32 + 32r's rule update on lane l32 (lower lanes) from the planes S, with env
// l32's per-env selection uniforms of update k (settle_sel_words; every lane computes its env's
// words, the upper half repeating the lower's: the settle variants are off the hot path).  The
// chain runs from the widest node's last function down (uniform q); threshold q's plane of every
// node is compared env-major and transposed once per q, so that only one word's uniforms are live.
template <int W, int B>
__device__ __forceinline__ void node_update_settle(const StepArgs& a, const uint4 (&rec_)[W][kNodeRecs],
                                                   const uint4* __restrict__ selq, const uint32_t* __restrict__ S,
                                                   uint32_t ge_lo, uint32_t ge_hi, uint32_t st_lo, uint32_t k,
                                                   int lane, uint32_t (&X)[W]) {
  const int N = a.n_nodes;
  const bool lo = lane < 32;
  const int l32 = lane & 31;
  const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
  const int mnf = a.max_nf;
#pragma unroll
  for (int r = 0; r < W; ++r) {
    X[r] = 0;
    const int i = l32 + 32 * r;
    const int ii = lo && i < N ? i : 0;   // other lanes evaluate node 0 and discard it
    uint32_t U[16];
    settle_sel_words(ge_lo, ge_hi, st_lo, k, r, N, k0, k1, U);
    const int nf = (int)rec_[r][0].w;
    const int f0 = (int)rec_[r][1].w;
    uint32_t x = 0;
    for (int q = mnf - 1; q >= 0; --q) {
      uint32_t pl = 0;
      if (q < mnf - 1) pl = lane_transpose32(settle_lt_word(U, a.sthr + (size_t)(q * W + r) * 32), lane);
      if (q < nf) {
        uint32_t fq;
        if (q < kNodeRecs) {
          const uint4 rc = q == 0 ? rec_[r][0] : (q == 1 ? rec_[r][1] : (q == 2 ? rec_[r][2] : rec_[r][3]));
          fq = eval_sel(rc.x, selq[(2 * q) * 32 * W + ii], selq[(2 * q + 1) * 32 * W + ii], S);
        } else {
          const uint4 rc = a.fcompact[CK(f0 + q, a.n_funcs, 9)];
          fq = eval_compact(rc.x, rc.y, S);
        }
        x = (q == nf - 1) ? fq : bfi(pl, fq, x);
      }
    }
    if (lo && i < N) X[r] = x;
  }
}

// The settle law (settle_max >= 2, include/pbn_env.h "Step law"): updates k = 1 ..
// settle_max - 1 of the envs (lower lanes) whose state sp is outside every attractor, until all
// of the wave's envs are in one.  Update k: perturbation gaps j = 0, 1, ... from SETTLE_ENV call
// ((k-1) << 8 | j >> 2), word j & 3 (per env); unperturbed envs take the rule update with their
// own SETTLE_SEL uniforms of update k (node_update_settle).  Returns true on lanes whose env is
// still outside after the last update (PBN_FLAG_UNSETTLED).
template <int W, int B>
__device__ __forceinline__ bool settle_updates(const StepArgs& a, const uint32_t* __restrict__ L, uint32_t* S,
                                            const uint4 (&rec_)[W][kNodeRecs], int lane, uint32_t ge_lo,
                                            uint32_t ge_hi, uint32_t st_lo, uint32_t (&sp)[W], int& att, bool& pert,
                                            uint32_t& nupd, bool live) {
  const bool lo = lane < 32;
  const int l32 = lane & 31;
  const int N = a.n_nodes;
  const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
  const uint4* selq = reinterpret_cast<const uint4*>(L + a.sel_off);
  const uint32_t* htab = L + a.cdf_len + 4 * (N + 1);
  bool open = live && att < 0;   // (envs past n_envs take part in the transposes only)
  for (int k = 1; k < a.settle_max; ++k) {
    if (__ballot(open) == 0) return false;
    const uint32_t sub = (uint32_t)(k - 1);
    uint32_t gam[W];
    bool pk = false;
#pragma unroll
    for (int w = 0; w < W; ++w) gam[w] = 0;
    if (open) {
      Word4 P = {0, 0, 0, 0};
      int pos = -1;
      for (int j = 0; pos < N - 1; ++j) {
        if ((j & 3) == 0)
          P = pbn::philox(ge_lo, st_lo, (pbn::kStreamSettleEnv << 28) | (sub << 8) | (uint32_t)(j >> 2), ge_hi, k0, k1);
        const int j4 = j & 3;
        const uint32_t u = j4 == 0 ? P.x : (j4 == 1 ? P.y : (j4 == 2 ? P.z : P.w));
        pos += gap_any(a.gap_exact, L, a, u);
        set_bit<W>(gam, pos, N);
      }
#pragma unroll
      for (int w = 0; w < W; ++w) pk = pk || gam[w] != 0;
    }
    // bit-slice sp (every lane takes part in the cross-lane transposes)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const uint32_t pl = lane_transpose32(sp[w], lane);
      if (lo) S[32 * w + l32] = pl;
    }
    __builtin_amdgcn_wave_barrier();
    if (a.n_glayers > 0) eval_gate_levels(a, L, S, lane);
    uint32_t X[W], x[W];
    node_update_settle<W, B>(a, rec_, selq, S, ge_lo, ge_hi, st_lo, (uint32_t)k, lane, X);
#pragma unroll
    for (int w = 0; w < W; ++w) x[w] = lane_transpose32(X[w], lane);
    if (open) {
#pragma unroll
      for (int w = 0; w < W; ++w) sp[w] = pk ? sp[w] ^ gam[w] : x[w];
      pert = pert || pk;
      ++nupd;
      att = attractor_lookup<W>(a, htab, sp);
      open = att < 0;
    }
  }
  return open;
}

// VARIANT 1: exactly one step (pbn_step; no loop, lowest VGPR count);
// 2: rollout with invariants recomputed per step (occupancy first; the rollout of networks
//    with gates, which the pipelined kernel does not run);
// 3, 4: 1 and 2 under the settle law (settle_max >= 2: settle_updates after the first update).
template <int W, int B, int VARIANT>
__global__ void __launch_bounds__(64 * kWavesPerBlock) pbn_step_wave(StepArgs a) {
  constexpr bool LEAN = VARIANT == 2 || VARIANT == 4;
  constexpr bool SINGLE = VARIANT == 1 || VARIANT == 3;
  constexpr bool SETTLE = VARIANT >= 3;
  constexpr int CPN = SETTLE ? 0 : B / 4;  // group selection calls per node (the settle law's are per env)
  constexpr int H = (CPN + 1) / 2;         // of which the lower half computes H
  constexpr int NLO = 1 + W * H;           // lower list: ENV, SEL(c < H)
  constexpr int NUP = W * (CPN - H);       // upper list: SEL(c >= H)
  constexpr int IT = NLO > NUP ? NLO : NUP;
  constexpr int UPC = (CPN - H) > 0 ? (CPN - H) : 1;  // divisor guard (B = 4: no upper calls)
  extern __shared__ uint32_t smem[];
  PBN_STAMP(0);
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t g = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  const int N = a.n_nodes;
  // LDS: the block's table image [cdf | reward | hash | attractors | leaf selectors], then
  // each wave's S planes
  uint32_t* L = smem;
  uint32_t* S = smem + a.tab_words + (size_t)wv * a.wave_words;
  const uint32_t* cdf = L;
  const float* rtab = reinterpret_cast<const float*>(L + a.cdf_len);
  const uint32_t* htab = L + a.cdf_len + 4 * (N + 1);
  const int64_t n = a.n_envs;
  const bool lo = lane < 32;
  const int l32 = lane & 31;
  const int64_t le = g * 32 + l32;
  const uint64_t ge = a.env_offset + (uint64_t)le;
  const uint64_t G = ge >> 5;
  const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
  const bool random_actions = (a.mode & PBN_MODE_RANDOM_ACTIONS) != 0;
  const size_t plane = (size_t)W * n;   // words per step of a [steps][W][n] output
  // env le exists (pbn_step takes any n_envs: the last group may be ragged; its other lanes
  // compute, take part in the cross-lane work, and load or store nothing)
  const bool live = lo && le < n;

  // ---- 0. issue the one-time global loads: env state, node records, tables
  uint32_t st[W];      // current observation s of env l32 (lower lanes), carried across steps
  uint32_t tt0 = 0, tg0 = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) st[w] = 0;
  if (live) {   // (waves past the end only help copy the tables; the bits past N are cleared after
                // the barrier: an AND here waited for the load ahead of the records and the image)
#pragma unroll
    for (int w = 0; w < W; ++w) st[w] = a.state[CK((size_t)w * n + le, plane, 1)];
    tt0 = a.t[CK(le, n, 2)];
    tg0 = a.target[CK(le, n, 3)];
  }
  // pbn_step_dev_store: the transition's row, and the env's branch actions requested now
  // (unguarded, clamped: a guarded load's select would wait for it here, ahead of the node records
  // and the table image); the row is written after the step (s, the target, the actions, s'
  // before an autoreset, the reward, done)
  // one-step launches: the step index (pbn_step_dev) and the env's flip mask requested here too
  // (after the barrier each was a round trip of its own before the Philox calls and the update)
  uint64_t step_pre = a.step;
  uint32_t mpre[W];
  if constexpr (SINGLE) {
    if (a.step_ptr) step_pre = *a.step_ptr;
    const int64_t lc = le < n ? le : n - 1;   // (unguarded; random-action launches ignore it)
#pragma unroll
    for (int w = 0; w < W; ++w) mpre[w] = a.flipmask[CK((size_t)w * n + lc, plane, 6)];
  }
  int64_t rj = 0;
  int32_t rav[kRingMaxK];
  if constexpr (!SETTLE) {
    if (a.r_state) {
      rj = (int64_t)(((uint64_t)*a.r_pos + (uint64_t)le) % (uint64_t)a.r_cap);
      const int64_t lc = le < n ? le : n - 1;
#pragma unroll
      for (int k = 0; k < kRingMaxK; ++k)
        rav[k] = a.r_act_in[CK((size_t)lc * a.r_k + (k < a.r_k ? k : a.r_k - 1), (size_t)n * a.r_k, 43)];
    }
  }
  // node l32 + 32r: its first kNodeRecs compact records {inputs, table, threshold, meta}
  // (node-major, fixed stride: no dependent load); meta of record 0 = nf, of record 1 = f0
  uint4 rec_[W][kNodeRecs];
#pragma unroll
  for (int r = 0; r < W; ++r) {
    const int i = l32 + 32 * r;
    const int ic = i < N ? i : 0;
#pragma unroll
    for (int q = 0; q < kNodeRecs; ++q) rec_[r][q] = a.nrec[CK((size_t)ic * kNodeRecs + q, N * kNodeRecs, 4)];
  }
  copy_image(L, a);
  __syncthreads();   // the kernel's only block barrier
  if (g >= a.n_groups) return;  // whole wave
#pragma unroll
  for (int w = 0; w < W; ++w) st[w] &= valid_word_mask(N, w);
  asm volatile("" : "+v"(tt0), "+v"(tg0));   // (their first uses here, not hoisted above the barrier)
  const uint4* selq = reinterpret_cast<const uint4*>(L + a.sel_off);

  const int n_steps = SINGLE ? 1 : a.n_steps;
  // Random-action mode issues no global load inside the step loop (attractor tables live in
  // LDS), so stores never have to drain (vmcnt retires in issue order).  A given flip mask
  // is loaded and consumed inside its own branch, so the wait for it stays on that path.
  for (int ks = 0; ks < n_steps; ++ks) {
  if constexpr (LEAN) {
    // keep loop-invariant expansions (leaf masks, threshold digits, key schedule, first-round
    // products) inside the loop so VGPRs stay low and occupancy high
#pragma unroll
    for (int r = 0; r < W; ++r) {
#pragma unroll
      for (int q = 0; q < kNodeRecs; ++q) {
        asm volatile("" : "+v"(rec_[r][q].x), "+v"(rec_[r][q].z));
      }
    }
  }
  const uint32_t kk0 = k0, kk1 = k1, ge_lo = (uint32_t)ge, G_lo = (uint32_t)G;
  uint64_t step = a.step + (uint64_t)ks;
  if constexpr (SINGLE) step = step_pre;   // (by value, or pbn_step_dev's device step index)
  const uint32_t st_lo = (uint32_t)step;
  const uint32_t st_hi = (uint32_t)((step >> 32) & 0xFFFFu) << 16;
  const uint32_t ge_hi = (uint32_t)((ge >> 32) & 0xFFFFu) | st_hi;
  const uint32_t G_hi = (uint32_t)((G >> 32) & 0xFFFFu) | st_hi;
  uint32_t m[W], s1[W];
#pragma unroll
  for (int w = 0; w < W; ++w) { m[w] = 0; s1[w] = st[w]; }
  if (live && a.obs) {
#pragma unroll
    for (int w = 0; w < W; ++w) a.obs[CK(ks * plane + (size_t)w * n + le, (size_t)n_steps * plane, 7)] = st[w];
  }

  // ---- 1. all Philox calls of the group, two half-wave work lists
  PBN_STAMP(1);
  Word4 out[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    uint32_t lc0, lc2, lc3, uc0, uc2, uc3;
    if (it == 0) {
      lc0 = ge_lo; lc2 = pbn::kStreamEnv << 28; lc3 = ge_hi;
    } else {
      constexpr int HD = H > 0 ? H : 1;   // (the settle variants have no group selection calls)
      const int idx = it - 1;
      const int r = (idx / HD) < W ? idx / HD : W - 1;
      const int c = idx % HD;
      lc0 = G_lo; lc2 = (pbn::kStreamSel << 28) | (uint32_t)(4 * (l32 + 32 * r) + c); lc3 = G_hi;
    }
    if (it < W * (CPN - H)) {
      const int r = it / UPC;
      const int c = H + it % UPC;
      uc0 = G_lo; uc2 = (pbn::kStreamSel << 28) | (uint32_t)(4 * (l32 + 32 * r) + c); uc3 = G_hi;
    } else {   // (upper list done: a discarded call)
      uc0 = ge_lo; uc2 = pbn::kStreamEnv << 28; uc3 = ge_hi;
    }
    out[it] = pbn::philox(lo ? lc0 : uc0, st_lo, lo ? lc2 : uc2, lo ? lc3 : uc3, kk0, kk1);
  }
  // digits of node l32 + 32r: calls c < H from this lane, c >= H from lane + 32
  uint32_t dig[W][16];
#pragma unroll
  for (int r = 0; r < W; ++r) {
#pragma unroll
    for (int c = 0; c < CPN; ++c) {
      const Word4 d = c < H ? out[(1 + r * H + c) < IT ? (1 + r * H + c) : 0]
                            : upper_to_lower(out[r * (CPN - H) + (c - H)]);
      dig[r][4 * c + 0] = d.x; dig[r][4 * c + 1] = d.y; dig[r][4 * c + 2] = d.z; dig[r][4 * c + 3] = d.w;
    }
  }
  const Word4 E = out[0];

  // ---- 2. per env (lower lanes): interventions, perturbation, reset word
  PBN_STAMP(2);
  uint32_t gam[W];
  uint32_t pc = 0;
  bool pert = false;
#pragma unroll
  for (int w = 0; w < W; ++w) gam[w] = 0;
  // ENV words 3:2 = a 64-bit uniform X: the action draw (every mode), the autoreset draws,
  // then gap 2's uniform u2 = what remains of X's top word (DESIGN.md "Step semantics")
  uint32_t r_row = 0, r_nt = 0, u2 = 0;
  if (lo) {
    uint32_t xhi = E.w, xlo = E.z;
    const uint32_t n1 = (uint32_t)(N + 1);
    const uint32_t c_act = ext64(xhi, xlo, n1 * n1 * n1);
    if (a.n_attr >= 1) {
      const int32_t* att_first = reinterpret_cast<const int32_t*>(L + a.att_off);
      const uint32_t A = (uint32_t)a.n_attr;
      uint32_t as = 0;
      if (A >= 2) {
        const uint32_t c = ext64(xhi, xlo, A * (A - 1));
        as = a.am1_magic ? __umulhi(c, a.am1_magic) : c;   // c / (A - 1)
        r_nt = c - as * (A - 1);
        r_nt += (r_nt >= as) ? 1u : 0u;
      }
      // (single-state attractors: the draw over one state is 0 and state a is attractor a's)
      const int st0 = a.att_single ? (int)as : att_first[as];
      r_row = (uint32_t)st0 + (a.att_single ? 0u : ext64(xhi, xlo, (uint32_t)(att_first[as + 1] - st0)));
    }
    u2 = xhi;
    if (random_actions) {
      actions_from_draw<W>(c_act, N, a.n1_magic, m);
      if (live) {
#pragma unroll
        for (int w = 0; w < W; ++w) a.flipmask[CK(ks * plane + (size_t)w * n + le, (size_t)n_steps * plane, 8)] = m[w];
      }
    } else if (live) {
#pragma unroll
      for (int w = 0; w < W; ++w)
        m[w] = (SINGLE ? mpre[w] : a.flipmask[CK(ks * plane + (size_t)w * n + le, (size_t)n_steps * plane, 6)]) &
               valid_word_mask(N, w);
    }
#pragma unroll
    for (int w = 0; w < W; ++w) {
      pc += __builtin_popcount(m[w]);
      s1[w] ^= m[w];
    }
    // perturbation positions are prefix sums of geometric gaps; the first three gaps
    // (u = E.x, E.y, u2) are independent, so they are computed side by side
    int g0, g1, g2;
    if (a.gap_exact == 2) {
      g0 = gap_any(2, L, a, E.x); g1 = gap_any(2, L, a, E.y); g2 = gap_any(2, L, a, u2);
    } else if (a.gap_exact) {
      g0 = gap_of(cdf, a.cdf_len, E.x); g1 = gap_of(cdf, a.cdf_len, E.y); g2 = gap_of(cdf, a.cdf_len, u2);
    } else {
      g0 = gap_est(cdf, a.cdf_len, a.inv_log2q, E.x);
      g1 = gap_est(cdf, a.cdf_len, a.inv_log2q, E.y);
      g2 = gap_est(cdf, a.cdf_len, a.inv_log2q, u2);
    }
    const int p0 = g0 - 1, p1 = p0 + g1, p2 = p1 + g2;
    set_bit<W>(gam, p0, N);
    set_bit<W>(gam, p1, N);
    set_bit<W>(gam, p2, N);
    if (p2 < N - 1) {   // rare: a fourth flip is possible (gap k >= 3: PERT call (k-3)>>2, word (k-3)&3)
      Word4 P = E;
      int pos = p2;
      for (int kk = 3; pos < N - 1; ++kk) {
        if (((kk - 3) & 3) == 0)
          P = pbn::philox(ge_lo, st_lo, (pbn::kStreamPert << 28) | (uint32_t)((kk - 3) >> 2), ge_hi, kk0, kk1);
        const int j4 = (kk - 3) & 3;
        const uint32_t u = j4 == 0 ? P.x : (j4 == 1 ? P.y : (j4 == 2 ? P.z : P.w));
        pos += gap_any(a.gap_exact, L, a, u);
        set_bit<W>(gam, pos, N);
      }
    }
#pragma unroll
    for (int w = 0; w < W; ++w) pert = pert || gam[w] != 0;
  }

  // ---- 3. bit-slice s1: lane p <- plane p (node p over the 32 envs), to LDS
  PBN_STAMP(3);
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const uint32_t sp = lane_transpose32(s1[w], lane);
    if (lo) S[32 * w + l32] = sp;
  }
  __builtin_amdgcn_wave_barrier();
  if (a.n_glayers > 0) eval_gate_levels(a, L, S, lane);

  // ---- 4. node l32 + 32r on lane l32: X = rule update of every env (perturbed envs are
  // replaced after the back-transpose)
  PBN_STAMP(4);
  uint32_t X[W];
  if constexpr (SETTLE) node_update_settle<W, B>(a, rec_, selq, S, ge_lo, ge_hi, st_lo, 0u, lane, X);
  else node_update<W, B>(a, rec_, selq, S, dig, lo, l32, X);

  // ---- 5. back to per-env words, reward, termination, autoreset, stores
  PBN_STAMP(5);
  uint32_t sp[W];
#pragma unroll
  for (int w = 0; w < W; ++w) sp[w] = lane_transpose32(X[w], lane);
  PBN_STAMP(6);
  if (lo && pert) {
#pragma unroll
    for (int w = 0; w < W; ++w) sp[w] = s1[w] ^ gam[w];
  }
  int att = lo ? attractor_lookup<W>(a, htab, sp) : 0;
  bool unsettled = false;
  uint32_t nupd = 1;   // synchronous updates applied this step
  if constexpr (SETTLE) {   // the whole wave (cross-lane transposes)
    unsettled = settle_updates<W, B>(a, L, S, rec_, lane, ge_lo, ge_hi, st_lo, sp, att, pert, nupd, live);
  }
  if (live) {
  if constexpr (!SINGLE) {
    if (a.updates) a.updates[CK(ks * n + le, n_steps * n, 23)] = (uint16_t)min(nupd, 0xFFFFu);
  }
  if (a.final_state) {
#pragma unroll
    for (int w = 0; w < W; ++w) a.final_state[CK(ks * plane + (size_t)w * n + le, (size_t)n_steps * plane, 10)] = sp[w];
  }
  if constexpr (!SETTLE) {
    if (a.r_state) {   // (st and tg0 are still the step's inputs here: the autoreset comes below)
#pragma unroll
      for (int w = 0; w < W; ++w) {
        a.r_state[CK((size_t)w * a.r_cap + rj, (size_t)W * a.r_cap, 40)] = st[w];
        a.r_next[CK((size_t)w * a.r_cap + rj, (size_t)W * a.r_cap, 44)] = sp[w];
      }
      a.r_target[CK(rj, a.r_cap, 41)] = (uint8_t)tg0;
#pragma unroll
      for (int k = 0; k < kRingMaxK; ++k)
        if (k < a.r_k) a.r_action[CK((size_t)rj * a.r_k + k, (size_t)a.r_cap * a.r_k, 42)] = rav[k];
    }
  }
  const bool in_attr = att >= 0;
  const bool term = in_attr && (uint32_t)att == tg0;
  const bool wrong = in_attr && !term;
  int tt = (int)tt0 + 1;
  tt = tt > 255 ? 255 : tt;
  const bool trunc = a.horizon > 0 && tt >= a.horizon;
  const float rwd = rtab[(int)pc * 4 + 2 * (int)term + (int)wrong];
  a.reward[CK(ks * n + le, n_steps * n, 11)] = rwd;
  uint32_t fl = (uint32_t)term | ((uint32_t)trunc << 1) | ((uint32_t)in_attr << 2) | ((uint32_t)pert << 3) |
                ((uint32_t)unsettled << 5);
  if ((a.mode & PBN_MODE_AUTORESET) && (term || trunc)) {
    uint32_t nt;
    if (a.n_attr >= 1) {   // the attractor draws of step 2 (attractor states from the LDS image)
      const uint32_t* att_words = L + a.att_off + a.n_attr + 1;
#pragma unroll
      for (int w = 0; w < W; ++w) sp[w] = att_words[(size_t)r_row * W + w];
      nt = r_nt;
    } else {
      const Word4 rr = pbn::philox(ge_lo, st_lo, (pbn::kStreamReset << 28) | 1u, ge_hi, kk0, kk1);
      const uint32_t rw4[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
      for (int w = 0; w < W; ++w) sp[w] = rw4[w] & valid_word_mask(N, w);
      nt = PBN_NO_TARGET;
    }
    tg0 = nt;
    tt = 0;
    fl |= PBN_FLAG_RESET;
  }
  a.flags[CK(ks * n + le, n_steps * n, 15)] = (uint8_t)fl;
  if constexpr (!SETTLE) {
    if (a.r_state) {   // done as pbn_replay_store derives it from the flags byte
      const uint8_t d = a.r_done_mask ? ((fl & a.r_done_mask) ? 1 : 0) : ((uint8_t)fl ? 1 : 0);
      a.r_reward[CK(rj, a.r_cap, 45)] = rwd;
      a.r_done[CK(rj, a.r_cap, 46)] = d;
      if (a.r_done_out) a.r_done_out[CK(le, n, 47)] = d;
    }
  }
  tt0 = (uint32_t)tt;
#pragma unroll
  for (int w = 0; w < W; ++w) st[w] = sp[w];
  }  // live
  PBN_STAMP(7);
  }  // steps

  if (live) {
#pragma unroll
    for (int w = 0; w < W; ++w) a.state_out[CK((size_t)w * n + le, plane, 16)] = st[w];
    a.t[CK(le, n, 17)] = (uint8_t)tt0;
    a.target[CK(le, n, 18)] = (uint8_t)tg0;
  }
}


// Block barrier ordering LDS only.  __syncthreads() is a workgroup fence on every address
// space, so each wave would first wait (s_waitcnt vmcnt(0)) for its global stores -- the
// per-step obs / reward / flags / flip-mask stores -- to complete.  The step loops
// communicate through LDS alone and never read back what they store to HBM in the loop.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ------------------------------- rollout kernel, three waves per pair of 32-env groups
// Block = two groups (64 envs; lanes 32h..32h+31 of every wave work on group 2*block + h).
// The step splits into work that depends only on the counter-based RNG and work that
// depends on the state, so different waves run different steps:
//   wave 1 (env draws): ENV + PERT call 0 of env `lane` -> actions / given flip mask,
//     perturbation mask, autoreset draw;
//   wave 2 (selection): SEL calls of node `lane & 31` -> the (u < c_j) masks of its thresholds;
//   wave 0 (state): s1 = s ^ m, bit-slice, node evaluation from the masks, back-transpose,
//     attractor lookup, reward, flags, autoreset, stores.
// Iteration k: waves 1 and 2 produce step k into slot k&1 while wave 0 consumes step k-1
// from the other slot; the block barrier ends the iteration.  Same results as pbn_step_wave.
// Each wave alone is latency-bound, so the split (three instruction streams per group pair)
// is what fills the SIMDs at small batches.

// input plane k of a record's input word: byte k is a plane index, or with BY (the pipelined
// kernel's LDS records for W <= 2) the plane's byte offset, so that the address is one add of
// a byte field (v_add_u32 with an SDWA byte select) instead of extract + shift-add
template <bool BY>
__device__ __forceinline__ uint32_t plane_in(const uint32_t* __restrict__ S, uint32_t ins, int k) {
  const uint32_t f = k == 3 ? ins >> 24 : (ins >> (8 * k)) & 0xFFu;
  if constexpr (BY) return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(S) + f);
  else return S[f];
}

// node chain from precomputed selection masks: x = F_{nf-1}; x = lt_j ? F_j : x, with every
// LDS read of the K records issued before any use (K = wave-uniform bound, nf per lane)
template <int K, bool BY>
__device__ __forceinline__ uint32_t chain_from_masks(const uint4 (&rec)[kNodeRecs], const uint4* __restrict__ sel,
                                                     int stride, const uint32_t* __restrict__ S,
                                                     const uint32_t* __restrict__ lt, int lt_stride, int nf,
                                                     bool tail, uint32_t x) {
  uint32_t xin[K][4], ltv[K];
  uint4 sa[K], sb[K];
#pragma unroll
  for (int q = 0; q < K; ++q) {
    const uint32_t ins = rec[q].x;
#pragma unroll
    for (int k = 0; k < 4; ++k) xin[q][k] = plane_in<BY>(S, ins, k);
    sa[q] = sel[(2 * q) * stride];
    sb[q] = sel[(2 * q + 1) * stride];
    // mask q exists for q < K - 1, and for q = K - 1 too when some node has more than K
    // (= kNodeRecs) functions
    ltv[q] = (q < K - 1 || tail) ? lt[q * lt_stride] : 0u;
  }
#pragma unroll
  for (int q = K - 1; q >= 0; --q) {
    const uint32_t x0 = xin[q][0], x1 = xin[q][1], x2 = xin[q][2], x3 = xin[q][3];
    const uint32_t nx0 = ~x0;
    const uint32_t v0 = __builtin_amdgcn_perm(nx0, x0, sa[q].x), v1 = __builtin_amdgcn_perm(nx0, x0, sa[q].y);
    const uint32_t v2 = __builtin_amdgcn_perm(nx0, x0, sa[q].z), v3 = __builtin_amdgcn_perm(nx0, x0, sa[q].w);
    const uint32_t v4 = __builtin_amdgcn_perm(nx0, x0, sb[q].x), v5 = __builtin_amdgcn_perm(nx0, x0, sb[q].y);
    const uint32_t v6 = __builtin_amdgcn_perm(nx0, x0, sb[q].z), v7 = __builtin_amdgcn_perm(nx0, x0, sb[q].w);
    const uint32_t w0 = bfi(x1, v1, v0), w1 = bfi(x1, v3, v2), w2 = bfi(x1, v5, v4), w3 = bfi(x1, v7, v6);
    const uint32_t fj = bfi(x3, bfi(x2, w3, w2), bfi(x2, w1, w0));
    const uint32_t y = (q == nf - 1) ? fj : bfi(ltv[q], fj, x);
    x = (q < nf) ? y : x;
  }
  return x;
}

// chain over padded records (every node has max_nf <= kNodeRecs records, the last function
// repeated; lanes past N have all-zero selectors and evaluate to 0): x = F_{K-1}; x = lt_q ? F_q
// : x, with no per-lane function count
template <int K, bool BY>
__device__ __forceinline__ uint32_t chain_padded(const uint4* __restrict__ rec, const uint4* __restrict__ sel,
                                                 int stride, const uint32_t* __restrict__ S,
                                                 const uint32_t* __restrict__ lt, int lt_stride) {
  uint32_t xin[K][4], ltv[K];
  uint4 sa[K], sb[K];
#pragma unroll
  for (int q = 0; q < K; ++q) {
    const uint32_t ins = rec[q * stride].x;
#pragma unroll
    for (int k = 0; k < 4; ++k) xin[q][k] = plane_in<BY>(S, ins, k);
    sa[q] = sel[(2 * q) * stride];
    sb[q] = sel[(2 * q + 1) * stride];
    ltv[q] = q < K - 1 ? lt[q * lt_stride] : 0u;
  }
  uint32_t x = 0;
#pragma unroll
  for (int q = K - 1; q >= 0; --q) {
    const uint32_t fj = eval_sel_in(xin[q], sa[q], sb[q]);
    x = (q == K - 1) ? fj : bfi(ltv[q], fj, x);
  }
  return x;
}

// MANY: some node has more than kNodeRecs functions.  Those chains read records past the LDS
// copy (global fcompact) and hold every record of a node in registers; compiled out of the
// common instances (every bundled network has at most 3 functions per node), they no longer set
// the register allocation of the whole kernel: 167 -> 88 VGPRs at three state words (pbn70),
// 121 -> 83 at two, 242 -> 93 at four.
// Waves per SIMD the register allocation must allow for single-word states: 6 (<= 80 VGPRs,
// no spill in the step loops) runs 1M envs 10 % faster than the unconstrained 86 VGPRs (5 waves);
// 7 and 8 spill to scratch in the state loop and lose (profiles/r02_ab_waves_per_eu.jsonl).
// Multi-word states: 5 waves without MANY; with MANY, three words are held to 3 waves (167 VGPRs,
// where the compiler's choice is 181: 2 waves) and two words fit 4 waves as they are.
#define PBN_PIPE_ATTR __attribute__((amdgpu_waves_per_eu(W == 1 ? 6 : (MANY ? (W == 3 ? 3 : 1) : 5), 8)))
template <int W, int B, bool MANY>
__global__ void __launch_bounds__(256) PBN_PIPE_ATTR pbn_rollout_pipe(StepArgs a) {
  constexpr int CPN = B / 4;              // selection calls per node
  extern __shared__ uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int role = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: scalar branches
  // the state wave bounds every iteration: let it win VALU issue against the RNG waves of
  // other blocks sharing its SIMD
  PBN_RSTAMP(0);
  if (role == 0) __builtin_amdgcn_s_setprio(kStatePrio);
  // with one block per SIMD triple (every SIMD holds one wave of each role) the selection wave,
  // the longest instruction stream, also goes ahead of the env-draw wave: -5 % per step at
  // 65,536 envs; with more blocks resident it loses 4-8 % (profiles/r02_ab_wave_priority.jsonl)
  if (role == 2 && a.sel_prio) __builtin_amdgcn_s_setprio(1);
#ifdef PBN_STAMPS
  // placement of this wave: HW_ID (wave, SIMD, CU, SH, SE) in the low word, XCC_ID above it
  if (a.stamps && lane == 0)
    a.stamps[(size_t)blockIdx.x * 32 + (role == 0 ? 14 : role * 4 + 3)] =
        (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
        ((unsigned long long)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32);
#endif
  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int64_t g = (int64_t)blockIdx.x * 2 + half;
  const bool valid = g < a.n_groups;
  const int N = a.n_nodes;
  const int64_t n = a.n_envs;
  const int64_t le = g * 32 + l32;
  const uint64_t ge = a.env_offset + (uint64_t)le;
  const uint64_t G = ge >> 5;
  const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
  const bool random_actions = (a.mode & PBN_MODE_RANDOM_ACTIONS) != 0;
  const size_t plane = (size_t)W * n;
  const int n_steps = a.n_steps;
  const int LQ = a.lq;
  // LDS: table image | S planes [2][32W] | two slots
  //   slot = m[W][64] | gam[W][64] | rs[W][64] | info[64] | lt[LQ][2][32W]
  uint32_t* L = smem;
  const uint32_t* cdf = L;
  const float* rtab = reinterpret_cast<const float*>(L + a.cdf_len);
  const uint32_t* htab = L + a.cdf_len + 4 * (N + 1);
  const uint4* selq = reinterpret_cast<const uint4*>(L + a.sel_off);
  uint32_t* Sg = smem + a.tab_words + half * 32 * W;   // this half's group
  uint32_t* slots = smem + a.tab_words + 2 * 32 * W;
  uint32_t st[W];
  uint32_t tt0 = 0, tg0 = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) st[w] = 0;
  if (role == 0 && valid) {   // issued first: their latency overlaps the image copy
#pragma unroll
    for (int w = 0; w < W; ++w) st[w] = a.state[CK((size_t)w * n + le, plane, 1)];
    tt0 = a.t[CK(le, n, 2)];
    tg0 = a.target[CK(le, n, 3)];
  }
  copy_image(L, a);
#pragma unroll
  for (int w = 0; w < W; ++w) st[w] &= valid_word_mask(N, w);
  // node records live in LDS (L + nrec_off), record-major [kNodeRecs][32W] so that a wave's
  // lanes (nodes) read consecutive 16-byte records without bank conflicts: each role reads
  // what it needs per step, so no record is carried in VGPRs across the step loop
  const uint4* recL = reinterpret_cast<const uint4*>(L + a.nrec_off);
  // wave-uniform parameters, re-defined (laundered) every iteration: hoisted out of the step
  // loop, the conditions built from them occupy SGPR pairs and spill to VGPR lanes
  uint32_t u_k0 = k0, u_k1 = k1;
  int u_gx = a.gap_exact, u_na = a.n_attr,  u_mnf = a.max_nf, u_hb = a.hash_bits,
      u_hp = a.hash_probes, u_hz = a.horizon;
  uint32_t u_fl = __builtin_amdgcn_readfirstlane((a.obs ? 1u : 0u) | (a.final_state ? 2u : 0u) |
                                                 (random_actions ? 4u : 0u) | ((a.mode & PBN_MODE_AUTORESET) ? 8u : 0u) |
                                                 (a.att_single ? 16u : 0u));
  // digit masks of the first kNodeRecs - 1 thresholds of every node, lane-major
  // [32][sel_mask_stride(B)], for the selection wave's compares: built on the host into the table
  // image (single-word states only: for W > 1 the extra LDS cost more occupancy than it saved,
  // measured -15 % on pbn70 x 1M).  Built here from the records, they took a second barrier.
  const uint32_t* cm = L + a.cm_off;
  __syncthreads();
  PBN_RSTAMP(1);
  if (role == 3) {   // (pbn_rollout_copy) past the block's last __syncthreads
    ride_copy_wave(a, lane);
    return;
  }
  // drain the initial state loads here: otherwise the loop-carried st / t / target copies at
  // the bottom of the loop wait on vmcnt(0), which also waits for every store of the step
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) expcnt(7) lgkmcnt(15)
  PBN_RSTAMP(2);

  // one loop per role: every wave passes the same n_steps + 1 block barriers, and each role's
  // loop-carried values (hoisted invariants) occupy registers only in that role's loop
  if (role == 1 && (u_fl & 4u) && u_gx == 2 && u_na >= 2 && (u_fl & 16u) && (W > 1 || N <= 31)) {
    // env draws, common configuration (random actions, gap bucket table, two or more
    // single-state attractors): the same draws as the general loop below, branch-free apart from
    // the rare fourth-flip tail and the guarded flip-mask store, so that the next step's ENV call
    // (computed here, one step ahead) interleaves with this step's dependent draws and LDS reads
    // instead of following them
    const uint32_t A = (uint32_t)u_na;
    const uint32_t n1 = (uint32_t)(N + 1);
    const uint32_t* att_words = L + a.att_off + u_na + 1;
    const uint2* lut = reinterpret_cast<const uint2*>(L + a.gap_lut_off);
    auto env_call = [&](int k) {
      const uint64_t step = a.step + (uint64_t)k;
      const uint32_t ge_hi = (uint32_t)((ge >> 32) & 0xFFFFu) | ((uint32_t)((step >> 32) & 0xFFFFu) << 16);
      return pbn::philox((uint32_t)ge, (uint32_t)step, pbn::kStreamEnv << 28, ge_hi, u_k0, u_k1);
    };
    // one step: this step's draws from E, the next step's ENV call into E_next
    auto env_step = [&](int k, const Word4& E, Word4& E_next) {
      asm volatile("" : "+s"(u_k0), "+s"(u_k1), "+s"(u_gx), "+s"(u_na), "+s"(u_mnf));
      asm volatile("" : "+s"(u_hb), "+s"(u_hp), "+s"(u_hz), "+s"(u_fl));
      PBN_ISA_LOOP("env_fast", W);
      PBN_PSTAMP(k, 0);
      if (k < n_steps) {
        uint32_t* slot = slots + (size_t)(k & 1) * a.slot_words;
        // part 1: the draws that feed LDS reads, and the reads themselves
        uint32_t xhi = E.w, xlo = E.z;
        const uint32_t c_act = ext64(xhi, xlo, n1 * n1 * n1);
        const uint32_t u2 = (uint32_t)((((((uint64_t)E.w) << 32) | E.z) * a.x_mult) >> 32);
        const uint32_t c = ext64(xhi, xlo, A * (A - 1));
        const uint32_t as = a.am1_magic ? __umulhi(c, a.am1_magic) : c;   // c / (A - 1)
        uint32_t rs[W];
#pragma unroll
        for (int w = 0; w < W; ++w) rs[w] = att_words[(size_t)as * W + w];
        const uint2 e0 = lut[min(E.x >> a.gap_shift, (uint32_t)a.gap_nb)];
        const uint2 e1 = lut[min(E.y >> a.gap_shift, (uint32_t)a.gap_nb)];
        const uint2 e2 = lut[min(u2 >> a.gap_shift, (uint32_t)a.gap_nb)];
        // part 2: the next step's ENV call runs while those reads are in flight (the scheduling
        // barriers keep the compiler from hoisting it above them or sinking it to the latch)
        asm volatile("" ::: "memory");   // the LDS reads above are issued here
        __builtin_amdgcn_sched_barrier(0);
        PBN_PSTAMP_AT(k, 16);
        E_next = env_call(k + 1);   // (one unused call per launch)
        asm volatile("" : "+v"(E_next.x), "+v"(E_next.y), "+v"(E_next.z), "+v"(E_next.w));
        __builtin_amdgcn_sched_barrier(0);
        PBN_PSTAMP_AT(k, 17);
        // part 3: the rest of step k's draws
        uint32_t rt = c - as * (A - 1);
        rt += (rt >= as) ? 1u : 0u;
        uint32_t m[W], gam[W];
#pragma unroll
        for (int w = 0; w < W; ++w) { m[w] = 0; gam[w] = 0; }
        if constexpr (W == 1) m[0] = actions_mask31(c_act, n1, a.n1_magic, valid_word_mask(N, 0));   // N <= 31
        else actions_from_draw<W>(c_act, N, a.n1_magic, m);
        uint32_t pc = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) pc += __builtin_popcount(m[w]);
        const int g0 = (int)e0.y + (E.x >= e0.x ? 1 : 0);   // gap_lut
        const int g1 = (int)e1.y + (E.y >= e1.x ? 1 : 0);
        const int g2 = (int)e2.y + (u2 >= e2.x ? 1 : 0);
        const int p0 = g0 - 1, p1 = p0 + g1, p2 = p1 + g2;
        if constexpr (W == 1) {
          // N <= 31: a position past the network lands on a bit >= N (bit 31 at most), cleared by
          // the word mask once
          gam[0] = ((1u << min((uint32_t)p0, 31u)) | (1u << min((uint32_t)p1, 31u)) |
                    (1u << min((uint32_t)p2, 31u))) & valid_word_mask(N, 0);
        } else {
          set_bit<W>(gam, p0, N);
          set_bit<W>(gam, p1, N);
          set_bit<W>(gam, p2, N);
        }
        bool pert = false;
#pragma unroll
        for (int w = 0; w < W; ++w) {
          pert = pert || gam[w] != 0;
          slot[w * 64 + lane] = m[w];
          slot[(W + w) * 64 + lane] = gam[w];
          slot[(2 * W + w) * 64 + lane] = rs[w];
        }
        slot[3 * W * 64 + lane] = rt | (pc << 8) | ((uint32_t)pert << 16);
        if (valid) {
#pragma unroll
          for (int w = 0; w < W; ++w) LANE_ST(a.flipmask, k * plane + (size_t)w * n, le, (size_t)n_steps * plane, 8, m[w]);
        }
        if (p2 < N - 1) {   // rare: a fourth flip is possible (gap k >= 3: PERT call (k-3)>>2, word (k-3)&3)
          const uint64_t step = a.step + (uint64_t)k;
          const uint32_t ge_hi = (uint32_t)((ge >> 32) & 0xFFFFu) | ((uint32_t)((step >> 32) & 0xFFFFu) << 16);
          Word4 P = E;
          int pos = p2;
          for (int kk = 3; pos < N - 1; ++kk) {
            if (((kk - 3) & 3) == 0)
              P = pbn::philox((uint32_t)ge, (uint32_t)step, (pbn::kStreamPert << 28) | (uint32_t)((kk - 3) >> 2), ge_hi, u_k0, u_k1);
            const int j4 = (kk - 3) & 3;
            const uint32_t u = j4 == 0 ? P.x : (j4 == 1 ? P.y : (j4 == 2 ? P.z : P.w));
            pos += gap_lut(lut, a.gap_shift, a.gap_nb, u);
            set_bit<W>(gam, pos, N);
          }
          pert = false;
#pragma unroll
          for (int w = 0; w < W; ++w) {
            pert = pert || gam[w] != 0;
            slot[(W + w) * 64 + lane] = gam[w];
          }
          slot[3 * W * 64 + lane] = rt | (pc << 8) | ((uint32_t)pert << 16);
        }
      }
      PBN_PSTAMP(k, 1);
      lds_barrier();
      PBN_PSTAMP(k, 2);
    };
    // two steps per trip with the ENV words alternating between EA and EB: no copies between steps
    Word4 EA = env_call(0), EB = EA;
    for (int k = 0; k <= n_steps; k += 2) {
      env_step(k, EA, EB);
      if (k + 1 <= n_steps) env_step(k + 1, EB, EA);
    }
  } else if (role == 1) {
    for (int k = 0; k <= n_steps; ++k) {
      asm volatile("" : "+s"(u_k0), "+s"(u_k1), "+s"(u_gx), "+s"(u_na), "+s"(u_mnf));
      asm volatile("" : "+s"(u_hb), "+s"(u_hp), "+s"(u_hz), "+s"(u_fl));
      PBN_PSTAMP(k, 0);
      if (k < n_steps) {
        // ---- env draws of step k, env `lane`
        uint32_t* slot = slots + (size_t)(k & 1) * a.slot_words;
        const uint64_t step = a.step + (uint64_t)k;
        const uint32_t st_lo = (uint32_t)step;
        const uint32_t ge_hi = (uint32_t)((ge >> 32) & 0xFFFFu) | ((uint32_t)((step >> 32) & 0xFFFFu) << 16);
        const uint32_t ge_lo = (uint32_t)ge;
        // one ENV call: words 0, 1 = gaps 0, 1; X = words 3:2 gives, in order, the action draw
        // (every mode), the autoreset draws and gap 2's uniform u2 (DESIGN.md "Step semantics")
        const Word4 E = pbn::philox(ge_lo, st_lo, pbn::kStreamEnv << 28, ge_hi, u_k0, u_k1);
        if (valid) {
          uint32_t m[W], gam[W], rs[W];
#pragma unroll
          for (int w = 0; w < W; ++w) { m[w] = 0; gam[w] = 0; rs[w] = 0; }
          uint32_t xhi = E.w, xlo = E.z;
          const uint32_t n1 = (uint32_t)(N + 1);
          const uint32_t c_act = ext64(xhi, xlo, n1 * n1 * n1);
          // X after the action and pair draws, X * x_mult mod 2^64, as one product off the
          // draws' dependency chain
          uint64_t xr = ((((uint64_t)E.w) << 32) | E.z) * a.x_mult;
          // autoreset draw (used by wave 0 only if the env's episode ends): (start, target) in
          // one draw over the A(A-1) pairs, then the state within the start attractor
          uint32_t rt;
          if (u_na >= 1) {
            const int32_t* att_first = reinterpret_cast<const int32_t*>(L + a.att_off);
            const uint32_t* att_words = L + a.att_off + u_na + 1;
            const uint32_t A = (uint32_t)u_na;
            uint32_t as = 0;
            rt = 0;
            if (A >= 2) {
              const uint32_t c = ext64(xhi, xlo, A * (A - 1));
              as = a.am1_magic ? __umulhi(c, a.am1_magic) : c;   // c / (A - 1)
              rt = c - as * (A - 1);
              rt += (rt >= as) ? 1u : 0u;
            }
            // (single-state attractors: the draw over one state is 0 and state a is attractor a's)
            const int st0 = (u_fl & 16u) ? (int)as : att_first[as];
            uint32_t idx = 0;
            if (!(u_fl & 16u)) {
              const uint32_t size = (uint32_t)(att_first[as + 1] - st0);
              idx = ext64(xhi, xlo, size);
              xr *= size;
            }
#pragma unroll
            for (int w = 0; w < W; ++w) rs[w] = att_words[(size_t)(st0 + idx) * W + w];
          } else {
            const Word4 rr = pbn::philox(ge_lo, st_lo, (pbn::kStreamReset << 28) | 1u, ge_hi, u_k0, u_k1);
            const uint32_t rw4[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
            for (int w = 0; w < W; ++w) rs[w] = rw4[w] & valid_word_mask(N, w);
            rt = PBN_NO_TARGET;
          }
          const uint32_t u2 = (uint32_t)(xr >> 32);   // = xhi
          if (u_fl & 4u) {
            actions_from_draw<W>(c_act, N, a.n1_magic, m);
#pragma unroll
            for (int w = 0; w < W; ++w) LANE_ST(a.flipmask, k * plane + (size_t)w * n, le, (size_t)n_steps * plane, 8, m[w]);
          } else {
#pragma unroll
            for (int w = 0; w < W; ++w)
              m[w] = LANE_AT(a.flipmask, k * plane + (size_t)w * n, le, (size_t)n_steps * plane, 6) & valid_word_mask(N, w);
          }
          uint32_t pc = 0;
#pragma unroll
          for (int w = 0; w < W; ++w) pc += __builtin_popcount(m[w]);
          int g0, g1, g2;
          if (u_gx == 2) {
            g0 = gap_any(2, L, a, E.x); g1 = gap_any(2, L, a, E.y); g2 = gap_any(2, L, a, u2);
          } else if (u_gx) {
            g0 = gap_of(cdf, a.cdf_len, E.x); g1 = gap_of(cdf, a.cdf_len, E.y); g2 = gap_of(cdf, a.cdf_len, u2);
          } else {
            g0 = gap_est(cdf, a.cdf_len, a.inv_log2q, E.x);
            g1 = gap_est(cdf, a.cdf_len, a.inv_log2q, E.y);
            g2 = gap_est(cdf, a.cdf_len, a.inv_log2q, u2);
          }
          const int p0 = g0 - 1, p1 = p0 + g1, p2 = p1 + g2;
          set_bit<W>(gam, p0, N);
          set_bit<W>(gam, p1, N);
          set_bit<W>(gam, p2, N);
          if (p2 < N - 1) {   // rare: a fourth flip is possible (gap k >= 3: PERT call (k-3)>>2, word (k-3)&3)
            Word4 P = E;
            int pos = p2;
            for (int kk = 3; pos < N - 1; ++kk) {
              if (((kk - 3) & 3) == 0)
                P = pbn::philox(ge_lo, st_lo, (pbn::kStreamPert << 28) | (uint32_t)((kk - 3) >> 2), ge_hi, u_k0, u_k1);
              const int j4 = (kk - 3) & 3;
              const uint32_t u = j4 == 0 ? P.x : (j4 == 1 ? P.y : (j4 == 2 ? P.z : P.w));
              pos += gap_any(u_gx, L, a, u);
              set_bit<W>(gam, pos, N);
            }
          }
          bool pert = false;
#pragma unroll
          for (int w = 0; w < W; ++w) pert = pert || gam[w] != 0;
#pragma unroll
          for (int w = 0; w < W; ++w) {
            slot[w * 64 + lane] = m[w];
            slot[(W + w) * 64 + lane] = gam[w];
            slot[(2 * W + w) * 64 + lane] = rs[w];
          }
          slot[3 * W * 64 + lane] = rt | (pc << 8) | ((uint32_t)pert << 16);
        }
      }
      PBN_PSTAMP(k, 1);
      lds_barrier();
    }
  } else if (role == 2 && W == 1 && u_mnf >= 2 && u_mnf <= kNodeRecs) {
    // selection, single-word states with at most kNodeRecs functions per node: branch-free over
    // the lanes (lanes past N, single-function nodes and thresholds past a node's last compute
    // values the padded chain ignores), one loop per threshold count, and the next step's
    // SEL calls computed in the same block as this step's compares
    auto sel_fast = [&](auto nq_c) {
      constexpr int NQ = decltype(nq_c)::value;   // thresholds per node: max_nf - 1
      const uint32_t* cmi = cm + l32 * sel_mask_stride(B);
      uint32_t* lt_base = slots + (3 * W + 1) * 64 + half * 32 * W + l32;
      auto sel_calls = [&](int k, uint32_t (&d)[16]) {
        const uint64_t step = a.step + (uint64_t)k;
        const uint32_t G_hi = (uint32_t)((G >> 32) & 0xFFFFu) | ((uint32_t)((step >> 32) & 0xFFFFu) << 16);
#pragma unroll
        for (int c = 0; c < CPN; ++c) {
          const Word4 o = pbn::philox((uint32_t)G, (uint32_t)step, (pbn::kStreamSel << 28) | (uint32_t)(4 * l32 + c),
                                             G_hi, u_k0, u_k1);
          d[4 * c + 0] = o.x; d[4 * c + 1] = o.y; d[4 * c + 2] = o.z; d[4 * c + 3] = o.w;
        }
      };
      // one step: this step's compares from `cur`, the next step's calls into `nxt`
      auto sel_step = [&](int k, const uint32_t (&cur)[16], uint32_t (&nxt)[16]) {
        asm volatile("" : "+s"(u_k0), "+s"(u_k1));
        PBN_ISA_LOOP("sel_fast", NQ);
        PBN_PSTAMP(k, 0);
        if (k < n_steps) {
          sel_calls(k + 1, nxt);   // (one unused set per launch)
#ifdef PBN_STAMPS
#pragma unroll
          for (int d = 0; d < 16; ++d) asm volatile("" : "+v"(nxt[d]));
#endif
          PBN_PSTAMP_AT(k, 18);
          uint32_t* lt_out = lt_base + (size_t)(k & 1) * a.slot_words;
#pragma unroll
          for (int q = 0; q < NQ; ++q)
            lt_out[q * 64] = less_than_cm4<B>(cur, cmi + q * B);
          // keeps the next calls in this block (LLVM would sink them to the loop latch)
#pragma unroll
          for (int d = 0; d < 16; ++d) asm volatile("" : "+v"(nxt[d]));
        }
        PBN_PSTAMP(k, 1);
        lds_barrier();
        PBN_PSTAMP(k, 2);
      };
      // two steps per trip with the digit arrays swapping roles: no copies between steps
      uint32_t dA[16], dB[16];
#pragma unroll
      for (int d = 0; d < 16; ++d) { dA[d] = 0; dB[d] = 0; }
      sel_calls(0, dA);
      for (int k = 0; k <= n_steps; k += 2) {
        sel_step(k, dA, dB);
        if (k + 1 <= n_steps) sel_step(k + 1, dB, dA);
      }
    };
    switch (u_mnf) {
      case 2: sel_fast(std::integral_constant<int, 1>{}); break;
      case 3: sel_fast(std::integral_constant<int, 2>{}); break;
      default: sel_fast(std::integral_constant<int, 3>{}); break;
    }
  } else if (role == 2) {
    for (int k = 0; k <= n_steps; ++k) {
      asm volatile("" : "+s"(u_k0), "+s"(u_k1), "+s"(u_gx), "+s"(u_na), "+s"(u_mnf));
      asm volatile("" : "+s"(u_hb), "+s"(u_hp), "+s"(u_hz), "+s"(u_fl));
      PBN_PSTAMP(k, 0);
      if (k < n_steps) {
        // ---- selection masks of step k: node l32 + 32r of group g
        uint32_t* lt_out = slots + (size_t)(k & 1) * a.slot_words + (3 * W + 1) * 64 + half * 32 * W;
        const uint64_t step = a.step + (uint64_t)k;
        const uint32_t st_lo = (uint32_t)step;
        const uint32_t G_hi = (uint32_t)((G >> 32) & 0xFFFFu) | ((uint32_t)((step >> 32) & 0xFFFFu) << 16);
        const uint32_t G_lo = (uint32_t)G;
#pragma unroll
        for (int r = 0; r < W; ++r) {
          const int i = l32 + 32 * r;
          const int ic = i < N ? i : 0;
          const uint4 r0 = recL[ic];
          if (valid && i < N && (int)r0.w > 1) {
            uint32_t dig[16];
#pragma unroll
            for (int c = 0; c < CPN; ++c) {
              const Word4 o = pbn::philox(G_lo, st_lo, (pbn::kStreamSel << 28) | (uint32_t)(4 * i + c), G_hi, u_k0, u_k1);
              dig[4 * c + 0] = o.x; dig[4 * c + 1] = o.y; dig[4 * c + 2] = o.z; dig[4 * c + 3] = o.w;
            }
            const int nf = (int)r0.w;
            {   // per-lane thresholds: the selection wave has slack, the SGPRs are scarce
#pragma unroll
              for (int q = 0; q < kNodeRecs - 1; ++q)
                if (q < nf - 1) {
                  if constexpr (W == 1)
                    lt_out[q * 64 * W + i] = less_than_cm<B>(dig, cm + i * sel_mask_stride(B) + q * B, 1);
                  else
                    lt_out[q * 64 * W + i] = less_than(dig, recL[q * 32 * W + ic].z, B);
                }
              if constexpr (MANY) {   // nodes with more than kNodeRecs functions
                const int f0 = (int)recL[32 * W + ic].w;
                for (int j = kNodeRecs - 1; j < nf - 1; ++j)
                  lt_out[j * 64 * W + i] = less_than(dig, a.fcompact[CK(f0 + j, a.n_funcs, 9)].z, B);
              }
            }
          }
        }
      }
      PBN_PSTAMP(k, 1);
      lds_barrier();
    }
  } else {
    // the epilogue of step t (after the back-transpose): perturbed envs, outputs, attractor
    // hash, reward, flags, autoreset
    auto finish = [&](int t, uint32_t (&sp)[W], const uint32_t (&s1)[W], const uint32_t (&gam)[W],
                      const uint32_t (&rs)[W], uint32_t info) {
      {
        // branch-free epilogue (this wave bounds the iteration): only the stores are guarded
        const bool pert = (info >> 16) & 1u;
        const uint32_t pc = (info >> 8) & 0xFFu;
#pragma unroll
        for (int w = 0; w < W; ++w) sp[w] = pert ? (s1[w] ^ gam[w]) : sp[w];
        if (valid && (u_fl & 2u)) {
#pragma unroll
          for (int w = 0; w < W; ++w) LANE_ST(a.final_state, t * plane + (size_t)w * n, le, (size_t)n_steps * plane, 10, sp[w]);
        }
        // reward candidates depend only on popcount(flipmask): one 16-byte row {none, wrong,
        // term, -} read beside the hash
        const float4 r4 = reinterpret_cast<const float4*>(rtab)[pc];
        const float r_none = r4.x, r_wrong = r4.y, r_term = r4.z;
        int att = -1;
        if (u_hb > 0) {
          const uint32_t hmask = (1u << u_hb) - 1u;
          uint32_t h = 0;
#pragma unroll
          for (int w = 0; w < W; ++w) h += sp[w] * a.hash_mult[w];
          h >>= (32 - u_hb);
          // the table is usually collision-free (one probe, h < 2^bits needs no mask); keys
          // are unique, so probe order does not matter
          att = hash_probe<W>(htab, h, sp);
          for (int pr = 1; pr < u_hp; ++pr) {
            const int id = hash_probe<W>(htab, (h + pr) & hmask, sp);
            if (id >= 0) att = id;
          }
        }
        const bool in_attr = att >= 0;
        const bool term = in_attr && (uint32_t)att == tg0;
        const bool wrong = in_attr && !term;
        int tt = (int)tt0 + 1;
        tt = tt > 255 ? 255 : tt;
        const bool trunc = u_hz > 0 && tt >= u_hz;
        const bool reset = (u_fl & 8u) && (term || trunc);
        const uint32_t fl = (uint32_t)term | ((uint32_t)trunc << 1) | ((uint32_t)in_attr << 2) |
                            ((uint32_t)pert << 3) | ((uint32_t)reset << 4);
        if (valid) {
          LANE_ST(a.reward, (size_t)t * n, le, (size_t)n_steps * n, 11, term ? r_term : (wrong ? r_wrong : r_none));
          LANE_ST(a.flags, (size_t)t * n, le, (size_t)n_steps * n, 15, (uint8_t)fl);
        }
        tg0 = reset ? (info & 0xFFu) : tg0;
        tt0 = reset ? 0u : (uint32_t)tt;
#pragma unroll
        for (int w = 0; w < W; ++w) st[w] = reset ? rs[w] : sp[w];
      }
    };
    if (W == 1 && u_mnf >= 1 && u_mnf <= kNodeRecs) {
      // single-word states with at most kNodeRecs functions per node: the loop-invariant record
      // inputs held in VGPRs, and this step's selection masks and selectors read before the
      // transpose, so that their LDS latency is off the chain slot -> transpose -> gathers ->
      // mux trees -> back-transpose
      auto state_fast = [&](auto k_c) {
        constexpr int K = decltype(k_c)::value;
        uint32_t ins[K];
#pragma unroll
        for (int q = 0; q < K; ++q) ins[q] = recL[q * 32 + l32].x;
        for (int k = 0; k <= n_steps; ++k) {
          asm volatile("" : "+s"(u_hb), "+s"(u_hp), "+s"(u_hz), "+s"(u_fl));
          // the 4K plane addresses of the gathers are re-derived from ins[] every step: hoisted
          // out of the loop they are 4K more live VGPRs, one was spilled, and its reload's
          // s_waitcnt vmcnt(0) waited on the step's streaming stores in the middle of the chain
#pragma unroll
          for (int q = 0; q < K; ++q) asm volatile("" : "+v"(ins[q]));
          PBN_ISA_LOOP("state_fast", K);
          PBN_PSTAMP(k, 0);
          if (k >= 1) {
            const int t = k - 1;
            const uint32_t* slot = slots + (size_t)(t & 1) * a.slot_words;
            const uint32_t* lt_in = slot + 4 * 64 + half * 32 + l32;
            uint32_t s1[W], gam[W], rs[W];
            s1[0] = st[0] ^ slot[lane];
            gam[0] = slot[64 + lane];
            rs[0] = slot[2 * 64 + lane];
            const uint32_t info = slot[3 * 64 + lane];
            uint32_t ltv[K];
            uint4 sa[K], sb[K];
#pragma unroll
            for (int q = 0; q < K; ++q) {
              ltv[q] = q < K - 1 ? lt_in[q * 64] : 0u;
              sa[q] = selq[(2 * q) * 32 + l32];
              sb[q] = selq[(2 * q + 1) * 32 + l32];
            }
            if (valid && (u_fl & 1u)) LANE_ST(a.obs, (size_t)t * plane, le, (size_t)n_steps * plane, 7, st[0]);
            PBN_PSTAMP_AT(k, 15);
            Sg[l32] = lane_transpose32(s1[0], lane);
            __builtin_amdgcn_wave_barrier();
            PBN_PSTAMP_AT(k, 3);
            uint32_t x = 0;
#pragma unroll
            for (int q = K - 1; q >= 0; --q) {
              uint32_t xin[4];
#pragma unroll
              for (int kk = 0; kk < 4; ++kk) xin[kk] = plane_in<true>(Sg, ins[q], kk);
              const uint32_t fj = eval_sel_in(xin, sa[q], sb[q]);
              x = (q == K - 1) ? fj : bfi(ltv[q], fj, x);
            }
            PBN_PSTAMP_AT(k, 12);
            uint32_t sp[W];
            sp[0] = lane_transpose32(x, lane);
            PBN_PSTAMP_AT(k, 13);
            finish(t, sp, s1, gam, rs, info);
          }
          PBN_PSTAMP(k, 1);
          lds_barrier();
          PBN_PSTAMP(k, 2);
          if (k <= 1) PBN_RSTAMP(3 + k);
        }
      };
      switch (u_mnf) {
        case 1: state_fast(std::integral_constant<int, 1>{}); break;
        case 2: state_fast(std::integral_constant<int, 2>{}); break;
        case 3: state_fast(std::integral_constant<int, 3>{}); break;
        default: state_fast(std::integral_constant<int, 4>{}); break;
      }
    } else
    for (int k = 0; k <= n_steps; ++k) {
      asm volatile("" : "+s"(u_k0), "+s"(u_k1), "+s"(u_gx), "+s"(u_na), "+s"(u_mnf));
      asm volatile("" : "+s"(u_hb), "+s"(u_hp), "+s"(u_hz), "+s"(u_fl));
      PBN_PSTAMP(k, 0);
      if (k >= 1) {
        // ---- state part of step t = k - 1
        const int t = k - 1;
        const uint32_t* slot = slots + (size_t)(t & 1) * a.slot_words;
        const uint32_t* lt_in = slot + (3 * W + 1) * 64 + half * 32 * W;
        uint32_t s1[W], gam[W], rs[W];
        uint32_t info = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
          s1[w] = st[w] ^ slot[w * 64 + lane];
          gam[w] = slot[(W + w) * 64 + lane];
          rs[w] = slot[(2 * W + w) * 64 + lane];
        }
        info = slot[3 * W * 64 + lane];
        if (valid && (u_fl & 1u)) {
#pragma unroll
          for (int w = 0; w < W; ++w) LANE_ST(a.obs, t * plane + (size_t)w * n, le, (size_t)n_steps * plane, 7, st[w]);
        }
#pragma unroll
        for (int w = 0; w < W; ++w) Sg[32 * w + l32] = lane_transpose32(s1[w], lane);
        __builtin_amdgcn_wave_barrier();
        PBN_PSTAMP_AT(k, 3);
        uint32_t X[W];
        if (!MANY || u_mnf <= kNodeRecs) {
#pragma unroll
          for (int r = 0; r < W; ++r) {
            int i = l32 + 32 * r;
            asm volatile("" : "+v"(i));   // selector and record reads stay in the step loop
            const uint4* rc = recL + i;
            const uint4* sel = selq + i;
            const uint32_t* lti = lt_in + i;
            switch (u_mnf) {
              case 1: X[r] = chain_padded<1, (W <= 2)>(rc, sel, 32 * W, Sg, lti, 64 * W); break;
              case 2: X[r] = chain_padded<2, (W <= 2)>(rc, sel, 32 * W, Sg, lti, 64 * W); break;
              case 3: X[r] = chain_padded<3, (W <= 2)>(rc, sel, 32 * W, Sg, lti, 64 * W); break;
              default: X[r] = chain_padded<4, (W <= 2)>(rc, sel, 32 * W, Sg, lti, 64 * W); break;
            }
          }
        } else
#pragma unroll
        for (int r = 0; r < W; ++r) {
          const int i = l32 + 32 * r;
          int ii = i < N ? i : 0;
          asm volatile("" : "+v"(ii));   // selector and record reads stay in the step loop
          uint4 rec_r[kNodeRecs];
#pragma unroll
          for (int q = 0; q < kNodeRecs; ++q) rec_r[q] = recL[q * 32 * W + ii];
          const int nf = (int)rec_r[0].w;
          uint32_t x = 0;
          if (u_mnf > kNodeRecs) {   // chain tail of nodes with more than kNodeRecs functions
            const int f0 = (int)rec_r[1].w;
            for (int j = nf - 1; j >= kNodeRecs; --j) {
              const uint4 rc = a.fcompact[CK(f0 + j, a.n_funcs, 9)];
              const uint32_t fj = eval_compact(rc.x, rc.y, Sg);
              x = (j == nf - 1) ? fj : bfi(lt_in[j * 64 * W + ii], fj, x);
            }
          }
          const uint4* sel = selq + ii;
          const uint32_t* lti = lt_in + ii;
          switch (u_mnf) {
            case 1: x = chain_from_masks<1, (W <= 2)>(rec_r, sel, 32 * W, Sg, lti, 64 * W, nf, u_mnf > kNodeRecs, x); break;
            case 2: x = chain_from_masks<2, (W <= 2)>(rec_r, sel, 32 * W, Sg, lti, 64 * W, nf, u_mnf > kNodeRecs, x); break;
            case 3: x = chain_from_masks<3, (W <= 2)>(rec_r, sel, 32 * W, Sg, lti, 64 * W, nf, u_mnf > kNodeRecs, x); break;
            default: x = chain_from_masks<4, (W <= 2)>(rec_r, sel, 32 * W, Sg, lti, 64 * W, nf, u_mnf > kNodeRecs, x); break;
          }
          X[r] = i < N ? x : 0u;
        }
        PBN_PSTAMP_AT(k, 12);
        uint32_t sp[W];
#pragma unroll
        for (int w = 0; w < W; ++w) sp[w] = lane_transpose32(X[w], lane);
        PBN_PSTAMP_AT(k, 13);
        finish(t, sp, s1, gam, rs, info);
      }
      PBN_PSTAMP(k, 1);
      lds_barrier();
      PBN_PSTAMP(k, 2);
    }
    PBN_RSTAMP(5);
    if (valid) {
#pragma unroll
      for (int w = 0; w < W; ++w) a.state_out[CK((size_t)w * n + le, plane, 16)] = st[w];
      a.t[CK(le, n, 17)] = (uint8_t)tt0;
      a.target[CK(le, n, 18)] = (uint8_t)tg0;
    }
#ifdef PBN_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
    PBN_RSTAMP(6);
#endif
  }
}

// ------------------------------- settle-law rollout, three waves per pair of 32-env groups
// pbn_rollout under the settle law (settle_max = K >= 2, include/pbn_env.h "Step law"): the
// intervention, then synchronous updates until the env's state is in an attractor or K updates
// have run.  The roles of pbn_rollout_pipe, but one iteration is one UPDATE (t, k) of a step t,
// and every env runs its own sequence of updates: the settle law keys each update's selection per
// env (SETTLE_SEL call (k << 8 | i >> 3) of env e; DESIGN.md "Step law"), so an env that settles
// starts its next step while the other envs of its 32-env word are still updating.
//   wave 1 (env draws, lane = env): the update's draws: k = 0 the ENV call (actions, the step's
//     autoreset draws, gaps 0-2), k >= 1 the SETTLE_ENV call (gaps), one call per lane with a
//     per-lane counter; flip mask, perturbation mask (and at k = 0 the reset state, target and
//     action count) to the slot, env-major;
//   wave 2 (selection, lane = env): the env's SETTLE_SEL words of its update, compared with the
//     thresholds env-major (a subtract and a v_alignbit per node and threshold), transposed to
//     the (u < c_j) bit planes of every node;
//   wave 0 (state): the update of every env whose update is valid (s1 = s ^ m, bit-slice, node
//     chains, back-transpose, perturbed envs s1 ^ gamma), the attractor lookup, the per-env
//     decision to continue or end the step, and the step's epilogue (reward, flags, s', update
//     count, autoreset, next obs) in the iteration that ends it.
// Iteration i: the RNG waves produce each env's update R(i) into slot i & 1 while the state wave
// applies R(i-1) (EnvPlan); the state wave publishes each env's decision C (next update) in LDS.
// Results are bit-identical to pbn_step_wave's settle variants and to oracle/pbn_oracle.c.
constexpr uint32_t kNoUpd = 0xFFFFFFFFu;

// pbn_rollout_settle's output rows in LDS: every env ends its steps in its
// own iterations, so the per-env stores of the round-5 kernel were a few lanes wide and went out
// as partial-line write-backs (2.1x the outputs' bytes at 20 steps, 12.6x at 100).  The block's
// 64 envs now put step t's outputs into row t mod R of a ring in LDS, and the env-draw wave (the
// role with the most barrier slack) stores a row with full-line non-temporal stores once every
// env of the block has ended step t.  An env at most R - 1 steps ahead of the block's slowest
// waits (its update is produced and not applied), so a row is never reused before it is stored.
// Row layout (words): final [W][64] | obs [W][64] | flip mask [W][64] | reward [64] | flags
// [64 bytes] | update counts [64 u16].
__host__ __device__ constexpr int settle_stage_rows(int W) { return W == 1 ? 16 : (W == 2 ? 8 : 4); }
__host__ __device__ constexpr int settle_row_words(int W) { return 3 * 64 * W + 64 + 16 + 32; }
struct StageOut {   // the output pointers the row stores use, copied to LDS at kernel start
  uint32_t* final_state;
  uint32_t* obs;
  uint32_t* flipmask;
  float* reward;
  uint8_t* flags;
  uint16_t* updates;
};
constexpr uint32_t kSettleStampIt = 300;   // stamps build: the iteration the settle kernel clocks

// The per-env update plan of pbn_rollout_settle, in that env's lane of every wave (VGPRs; the
// same values in all three waves).  P = R(i-1), the update the RNG waves produced in the previous
// iteration (kNoUpd: none); C = the next update the env needs, the state wave's decision in
// iteration i-1; R = R(i), the update produced in iteration i.  R(i-1) is applied in iteration i
// iff it equals C.  A valid R(i-1) = (t, k) continues speculatively as (t, k+1), or (t+1, 0) at
// the cap; when the state wave finds the env settled the speculation is dropped and C re-issued
// (one idle iteration per step that ends before the cap).
struct EnvPlan {
  uint32_t Pt = kNoUpd, Pk = 0, Rt = 0, Rk = 0;
  bool v = false;
  __device__ __forceinline__ void next(uint32_t Ct, uint32_t Ck, uint32_t K) {
    v = Pt == Ct && Pk == Ck;
    const bool cap = Pk + 1 >= K;
    Rt = v ? (cap ? Pt + 1 : Pt) : Ct;
    Rk = v ? (cap ? 0u : Pk + 1) : Ck;
  }
  __device__ __forceinline__ void done() { Pt = Rt; Pk = Rk; }
};

template <int W, int B>
__global__ void __launch_bounds__(192) __attribute__((amdgpu_waves_per_eu(4, 8)))
pbn_rollout_settle(StepArgs a) {
  extern __shared__ uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int role = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (role == 0) __builtin_amdgcn_s_setprio(kStatePrio);
  // the env-draw wave ahead of the selection wave (it was the iteration's pole at equal priority:
  // +5 % at the driver's shape, profiles/r05_k_ab.json)
  if (role == 1) __builtin_amdgcn_s_setprio(1);

  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int64_t g = (int64_t)blockIdx.x * 2 + half;
  const bool valid = g < a.n_groups;
  const int N = a.n_nodes;
  const int64_t n = a.n_envs;
  const int64_t le = g * 32 + l32;
  const uint64_t ge = a.env_offset + (uint64_t)le;
  const size_t plane = (size_t)W * n;
  const uint32_t n_steps = (uint32_t)a.n_steps;
  const uint32_t K = (uint32_t)a.settle_max;
  const int lq = a.lq;
  // iterations that always suffice (a step takes at most K updates and one dropped speculation):
  // a guard every wave reaches, never the exit
  const uint64_t max_it = (uint64_t)n_steps * (K + 1) + 1;
  // the first step's index: by value, or from device memory (pbn_step_dev's one-step launch)
  const uint64_t step0 = a.step_ptr ? *a.step_ptr : a.step;
  uint32_t* L = smem;
  const float* rtab = reinterpret_cast<const float*>(L + a.cdf_len);
  const uint32_t* htab = L + a.cdf_len + 4 * (N + 1);
  const uint4* selq = reinterpret_cast<const uint4*>(L + a.sel_off);
  const uint4* recL = reinterpret_cast<const uint4*>(L + a.nrec_off);
  uint32_t* Sg = smem + a.tab_words + half * 32 * W;
  // slot (per iteration parity), env-major [.][64]: flip mask [W] | perturbation mask [W] | k = 0:
  // reset state [W] | k = 0: {reset target, action count} | selection planes [lq][2][32W]
  uint32_t* slots = smem + a.tab_words + 2 * 32 * W;
  constexpr int kGP = 64 * W, kRS = 128 * W, kIN = 192 * W, kLT = 192 * W + 64;
  // [parity][64]{C.t, C.k, R.t, R.k}: per env the state wave's decision C and the plan R of the
  // next iteration (EnvPlan, derived once by the state wave for all three)
  uint4* ctl = reinterpret_cast<uint4*>(slots + 2 * (size_t)a.slot_words);
  if (threadIdx.x < 64) {   // C = R = (0, 0) before iteration 0:
    const uint32_t c0 = valid ? 0u : n_steps;
    ctl[64 + threadIdx.x] = make_uint4(c0, 0u, c0, 0u);
  }
  // the packed thresholds (settle_pk), [lq][W][16] words after ctl: the selection wave reads them
  // by broadcast LDS reads
  uint32_t* thr_l = reinterpret_cast<uint32_t*>(ctl + 128);
  if (a.settle_pk) {
    for (int i = (int)threadIdx.x; i < lq * W * 16; i += (int)blockDim.x) thr_l[i] = a.sthr_pk[i];
  }
  // the output rows [R][settle_row_words(W)] after the thresholds, then the lowest step not yet
  // stored, by iteration parity (written by the env-draw wave in iteration i, read by the state
  // wave in iteration i + 1)
  constexpr int R = settle_stage_rows(W), RW = settle_row_words(W);
  constexpr int kSF = 0, kSO = 64 * W, kSM = 128 * W, kSR = 192 * W, kSFL = 192 * W + 64, kSU = 192 * W + 80;
  uint32_t* stg = thr_l + ((lq * W * 16 + 3) & ~3);
  uint32_t* stg_base = stg + R * RW;
  uint64_t* stg_out = reinterpret_cast<uint64_t*>(stg_base + 2);   // the row stores' pointers (StageOut)
  if (threadIdx.x < 2) stg_base[threadIdx.x] = 0u;
  if (threadIdx.x == 0) {
    stg_out[0] = reinterpret_cast<uint64_t>(a.final_state);
    stg_out[1] = reinterpret_cast<uint64_t>(a.obs);
    stg_out[2] = reinterpret_cast<uint64_t>(a.flipmask);
    stg_out[3] = reinterpret_cast<uint64_t>(a.reward);
    stg_out[4] = reinterpret_cast<uint64_t>(a.flags);
    stg_out[5] = reinterpret_cast<uint64_t>(a.updates);
  }
                                                         // (0, 0); envs of groups past the end: finished
  uint32_t st[W];
  uint32_t tt0 = 0, tg0 = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) st[w] = 0;
  if (role == 0 && valid) {
#pragma unroll
    for (int w = 0; w < W; ++w) st[w] = a.state[CK((size_t)w * n + le, plane, 1)];
    tt0 = a.t[CK(le, n, 2)];
    tg0 = a.target[CK(le, n, 3)];
  }
  copy_image(L, a);
#pragma unroll
  for (int w = 0; w < W; ++w) st[w] &= valid_word_mask(N, w);
  uint32_t u_k0 = (uint32_t)a.seed, u_k1 = (uint32_t)(a.seed >> 32);
  const uint32_t u_fl = __builtin_amdgcn_readfirstlane((a.obs ? 1u : 0u) | (a.final_state ? 2u : 0u) |
                                                       ((a.mode & PBN_MODE_RANDOM_ACTIONS) ? 4u : 0u) |
                                                       ((a.mode & PBN_MODE_AUTORESET) ? 8u : 0u) |
                                                       (a.updates ? 32u : 0u));
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the initial state loads (see pbn_rollout_pipe)
  const int mnf = __builtin_amdgcn_readfirstlane(a.max_nf);
  const uint32_t ge_lo = (uint32_t)ge;

  // one loop per role; every role derives the same plans and loop exit from the same C values
  // (the env draws' fast path: random actions, the gap bucket table, two or more single-state
  // attractors and N <= 31 for single-word states -- every kaban network -- branch-free)
  const bool env_fast = __builtin_amdgcn_readfirstlane((u_fl & 4u) && a.gap_exact == 2 && a.n_attr >= 2 &&
                                                       a.att_single && (W > 1 || N <= 31) ? 1 : 0) != 0;
  // the env-draw wave's row stores: rows [base, t_lo) once every env of the block has ended those
  // steps (t_lo = the block's lowest current step, from the decisions C), full-line non-temporal
  // stores of 64 consecutive envs; at the loop's exit every remaining row
  uint32_t base = 0;
  const int nv = (int64_t)blockIdx.x * 2 + 1 < a.n_groups ? 64 : 32;   // envs of this block (an odd group
                                                                       // count leaves a phantom half)
  auto flush_rows = [&](uint32_t ct, uint32_t it) __attribute__((always_inline)) {
    while (base < n_steps && __ballot(valid && ct <= base) == 0) {
      // the output pointers from their LDS copy, read here on this rare path (taken from the
      // kernel arguments, the compiler hoisted them out of the step loops, where they held SGPRs
      // and spilled: 2 -> 25 SGPR spills); stores through VGPR addresses
      const StageOut* ap = reinterpret_cast<const StageOut*>(stg_out);
      const uint32_t* row = stg + (size_t)(base % R) * RW;
      const size_t er = (size_t)base * (size_t)n + (size_t)blockIdx.x * 64 + (size_t)lane;   // [t][n] element
      const size_t ep = (size_t)base * plane + (size_t)blockIdx.x * 64 + (size_t)lane;      // [t][W][n] element
      if (valid) {
        if (u_fl & 2u) {
#pragma unroll
          for (int w = 0; w < W; ++w) __builtin_nontemporal_store(row[kSF + w * 64 + lane], ap->final_state + CK(ep + (size_t)w * n, (size_t)n_steps * plane, 10));
        }
        if (u_fl & 1u) {
#pragma unroll
          for (int w = 0; w < W; ++w) __builtin_nontemporal_store(row[kSO + w * 64 + lane], ap->obs + CK(ep + (size_t)w * n, (size_t)n_steps * plane, 7));
        }
        if (u_fl & 4u) {
#pragma unroll
          for (int w = 0; w < W; ++w) __builtin_nontemporal_store(row[kSM + w * 64 + lane], ap->flipmask + CK(ep + (size_t)w * n, (size_t)n_steps * plane, 8));
        }
        __builtin_nontemporal_store(__uint_as_float(row[kSR + lane]), ap->reward + CK(er, (size_t)n_steps * n, 11));
      }
      const size_t eb = (size_t)base * (size_t)n + (size_t)blockIdx.x * 64;   // the row's first env
      if (lane < nv / 4)   // the flags, four envs per dword
        __builtin_nontemporal_store(row[kSFL + lane], reinterpret_cast<uint32_t*>(ap->flags) + CK(eb / 4 + lane, (size_t)n_steps * n / 4, 15));
      if ((u_fl & 32u) && lane < nv / 2)   // the update counts, two envs per dword
        __builtin_nontemporal_store(row[kSU + lane], reinterpret_cast<uint32_t*>(ap->updates) + CK(eb / 2 + lane, (size_t)n_steps * n / 2, 23));
      ++base;
    }
    if (lane == 0) stg_base[it & 1] = base;
  };
  if (role == 1 && env_fast) {
    // ---- the draws of each env's update R(i), env `lane`: one Philox call (ENV at k = 0,
    // SETTLE_ENV at k >= 1); the step's draws are computed on every lane and kept where k = 0
    const uint2* lut = reinterpret_cast<const uint2*>(L + a.gap_lut_off);
    const uint32_t* att_words = L + a.att_off + a.n_attr + 1;
    const uint32_t A = (uint32_t)a.n_attr, n1 = (uint32_t)(N + 1);
    for (uint32_t it = 0;; ++it) {
      asm volatile("" : "+s"(u_k0), "+s"(u_k1));
      PBN_ISA_LOOP("settle_env_fast", W);
      PBN_PSTAMP(it - kSettleStampIt + 10, 0);
      uint4 C = ctl[((it + 1) & 1) * 64 + lane];   // {C(i), R(i)}
      // all four words from one read, ahead of the exit test (split, R came in a second round trip)
      asm volatile("" : "+v"(C.x), "+v"(C.y), "+v"(C.z), "+v"(C.w));
      flush_rows(C.x, it);
      if (__ballot(C.x < n_steps) == 0 || (uint64_t)it > max_it) break;
      const uint32_t t = C.z, k = C.w;
      uint32_t* slot = slots + (size_t)(it & 1) * a.slot_words;
      PBN_PSTAMP_AT(it - kSettleStampIt + 10, 16);
      const bool live = valid && t < n_steps, first = k == 0;
      const uint64_t step = step0 + (uint64_t)t;
      const uint32_t st_lo = (uint32_t)step;
      const uint32_t ge_hi = (uint32_t)((ge >> 32) & 0xFFFFu) | ((uint32_t)((step >> 32) & 0xFFFFu) << 16);
      const uint32_t c2 = first ? (pbn::kStreamEnv << 28) : ((pbn::kStreamSettleEnv << 28) | ((k - 1) << 8));
      const Word4 E = pbn::philox(ge_lo, st_lo, c2, ge_hi, u_k0, u_k1);
      // the step's draws from X = ENV words 3:2 (used where k = 0): actions, the autoreset pair,
      // gap 2's uniform (X * x_mult, off the draws' chain)
      uint32_t xhi = E.w, xlo = E.z;
      const uint32_t c_act = ext64(xhi, xlo, n1 * n1 * n1);
      const uint32_t c = ext64(xhi, xlo, A * (A - 1));
      const uint32_t as = a.am1_magic ? __umulhi(c, a.am1_magic) : c;   // c / (A - 1)
      const uint32_t u2 = first ? (uint32_t)((((((uint64_t)E.w) << 32) | E.z) * a.x_mult) >> 32) : E.z;
      uint32_t rs[W];
#pragma unroll
      for (int w = 0; w < W; ++w) rs[w] = att_words[(size_t)as * W + w];
      const uint2 e0 = lut[min(E.x >> a.gap_shift, (uint32_t)a.gap_nb)];
      const uint2 e1 = lut[min(E.y >> a.gap_shift, (uint32_t)a.gap_nb)];
      const uint2 e2 = lut[min(u2 >> a.gap_shift, (uint32_t)a.gap_nb)];
      uint32_t rt = c - as * (A - 1);
      rt += (rt >= as) ? 1u : 0u;
      uint32_t m[W], gam[W];
#pragma unroll
      for (int w = 0; w < W; ++w) { m[w] = 0; gam[w] = 0; }
      if constexpr (W == 1) m[0] = actions_mask31(c_act, n1, a.n1_magic, valid_word_mask(N, 0));   // N <= 31
      else actions_from_draw<W>(c_act, N, a.n1_magic, m);
      uint32_t pcv = 0;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        m[w] = live && first ? m[w] : 0u;
        pcv += __builtin_popcount(m[w]);
      }
      const int g0 = (int)e0.y + (E.x >= e0.x ? 1 : 0);   // gap_lut
      const int g1 = (int)e1.y + (E.y >= e1.x ? 1 : 0);
      const int g2 = (int)e2.y + (u2 >= e2.x ? 1 : 0);
      const int p0 = g0 - 1, p1 = p0 + g1, p2 = p1 + g2;
      if constexpr (W == 1) {
        // N <= 31: a position past the network lands on a bit >= N (bit 31 at most), cleared by
        // the word mask once
        gam[0] = ((1u << min((uint32_t)p0, 31u)) | (1u << min((uint32_t)p1, 31u)) |
                  (1u << min((uint32_t)p2, 31u))) & valid_word_mask(N, 0);
      } else {
        set_bit<W>(gam, p0, N);
        set_bit<W>(gam, p1, N);
        set_bit<W>(gam, p2, N);
      }
      if (live && p2 < N - 1) {   // rare: more gaps (k = 0: PERT call (j-3) >> 2, word (j-3) & 3;
                                  // k >= 1: gap 3 is word 3, gap j >= 4 SETTLE_ENV call (k-1) << 8 | j >> 2)
        Word4 P = E;
        int pos = p2;
        for (int j = 3; pos < N - 1; ++j) {
          const int jj = first ? j - 3 : j;
          if ((jj & 3) == 0)
            P = pbn::philox(ge_lo, st_lo,
                            first ? ((pbn::kStreamPert << 28) | (uint32_t)(jj >> 2))
                                  : ((pbn::kStreamSettleEnv << 28) | ((k - 1) << 8) | (uint32_t)(jj >> 2)),
                            ge_hi, u_k0, u_k1);
          const int j4 = jj & 3;
          const uint32_t u = j4 == 0 ? P.x : (j4 == 1 ? P.y : (j4 == 2 ? P.z : P.w));
          pos += gap_lut(lut, a.gap_shift, a.gap_nb, u);
          set_bit<W>(gam, pos, N);
        }
      }
      if (live && first && t < base + R) {   // (an update past the ring is not applied: no row)
        uint32_t* row = stg + (size_t)(t % R) * RW;
#pragma unroll
        for (int w = 0; w < W; ++w) row[kSM + w * 64 + lane] = m[w];
      }
      PBN_PSTAMP_AT(it - kSettleStampIt + 10, 17);
#pragma unroll
      for (int w = 0; w < W; ++w) {
        slot[w * 64 + lane] = m[w];
        slot[kGP + w * 64 + lane] = live ? gam[w] : 0u;
        slot[kRS + w * 64 + lane] = rs[w];
      }
      slot[kIN + lane] = rt | (pcv << 8);
      PBN_PSTAMP(it - kSettleStampIt + 10, 1);
      lds_barrier();
      PBN_PSTAMP(it - kSettleStampIt + 10, 2);
    }
  } else if (role == 1) {
    // ---- the draws of each env's update R(i), env `lane` (general networks and modes)
    for (uint32_t it = 0;; ++it) {
      asm volatile("" : "+s"(u_k0), "+s"(u_k1));
      PBN_PSTAMP(it - kSettleStampIt + 10, 0);
      uint4 C = ctl[((it + 1) & 1) * 64 + lane];   // {C(i), R(i)}
      // all four words from one read, ahead of the exit test (split, R came in a second round trip)
      asm volatile("" : "+v"(C.x), "+v"(C.y), "+v"(C.z), "+v"(C.w));
      flush_rows(C.x, it);
      if (__ballot(C.x < n_steps) == 0 || (uint64_t)it > max_it) break;
      const uint32_t t = C.z, k = C.w;
      uint32_t* slot = slots + (size_t)(it & 1) * a.slot_words;
      PBN_PSTAMP_AT(it - kSettleStampIt + 10, 16);
      uint32_t m[W], gam[W];
#pragma unroll
      for (int w = 0; w < W; ++w) { m[w] = 0; gam[w] = 0; }
      if (valid && t < n_steps) {
        const uint64_t step = step0 + (uint64_t)t;
        const uint32_t st_lo = (uint32_t)step;
        const uint32_t ge_hi = (uint32_t)((ge >> 32) & 0xFFFFu) | ((uint32_t)((step >> 32) & 0xFFFFu) << 16);
        const bool first = k == 0;
        // one call per update: ENV at k = 0, SETTLE_ENV call (k-1) << 8 at k >= 1
        const uint32_t c2 = first ? (pbn::kStreamEnv << 28) : ((pbn::kStreamSettleEnv << 28) | ((k - 1) << 8));
        const Word4 E = pbn::philox(ge_lo, st_lo, c2, ge_hi, u_k0, u_k1);
        uint32_t u2 = E.z;
        if (first) {
          // the step's draws from X = ENV words 3:2: actions, the autoreset draws, gap 2's uniform
          uint32_t xhi = E.w, xlo = E.z;
          const uint32_t n1 = (uint32_t)(N + 1);
          const uint32_t c_act = ext64(xhi, xlo, n1 * n1 * n1);
          uint64_t xr = ((((uint64_t)E.w) << 32) | E.z) * a.x_mult;
          uint32_t rs[W], rtv;
          if (a.n_attr >= 1) {
            const int32_t* att_first = reinterpret_cast<const int32_t*>(L + a.att_off);
            const uint32_t* att_words = L + a.att_off + a.n_attr + 1;
            const uint32_t A = (uint32_t)a.n_attr;
            uint32_t as = 0;
            rtv = 0;
            if (A >= 2) {
              const uint32_t c = ext64(xhi, xlo, A * (A - 1));
              as = a.am1_magic ? __umulhi(c, a.am1_magic) : c;
              rtv = c - as * (A - 1);
              rtv += (rtv >= as) ? 1u : 0u;
            }
            const int st0 = a.att_single ? (int)as : att_first[as];
            uint32_t idx = 0;
            if (!a.att_single) {
              const uint32_t size = (uint32_t)(att_first[as + 1] - st0);
              idx = ext64(xhi, xlo, size);
              xr *= size;
            }
#pragma unroll
            for (int w = 0; w < W; ++w) rs[w] = att_words[(size_t)(st0 + idx) * W + w];
          } else {
            const Word4 rr = pbn::philox(ge_lo, st_lo, (pbn::kStreamReset << 28) | 1u, ge_hi, u_k0, u_k1);
            const uint32_t rw4[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
            for (int w = 0; w < W; ++w) rs[w] = rw4[w] & valid_word_mask(N, w);
            rtv = PBN_NO_TARGET;
          }
          u2 = (uint32_t)(xr >> 32);
          if (u_fl & 4u) {
            actions_from_draw<W>(c_act, N, a.n1_magic, m);
            if (t < base + R) {   // (an update past the ring is not applied: no row)
              uint32_t* row = stg + (size_t)(t % R) * RW;
#pragma unroll
              for (int w = 0; w < W; ++w) row[kSM + w * 64 + lane] = m[w];
            }
          } else {
#pragma unroll
            for (int w = 0; w < W; ++w)
              m[w] = a.flipmask[CK(((size_t)t * plane + (size_t)w * n) + (size_t)le, (size_t)n_steps * plane, 6)] & valid_word_mask(N, w);
          }
          uint32_t pcv = 0;
#pragma unroll
          for (int w = 0; w < W; ++w) {
            pcv += __builtin_popcount(m[w]);
            slot[kRS + w * 64 + lane] = rs[w];
          }
          slot[kIN + lane] = rtv | (pcv << 8);
        }
        // gaps 0, 1 = words 0, 1; gap 2 = u2 (k = 0) or word 2 (k >= 1); then, rarely, more
        int g0, g1, g2;
        if (a.gap_exact == 2) {   // the bucket table (every kaban network): three reads side by side
          const uint2* lut = reinterpret_cast<const uint2*>(L + a.gap_lut_off);
          g0 = gap_lut(lut, a.gap_shift, a.gap_nb, E.x);
          g1 = gap_lut(lut, a.gap_shift, a.gap_nb, E.y);
          g2 = gap_lut(lut, a.gap_shift, a.gap_nb, u2);
        } else {
          g0 = gap_any(a.gap_exact, L, a, E.x);
          g1 = gap_any(a.gap_exact, L, a, E.y);
          g2 = gap_any(a.gap_exact, L, a, u2);
        }
        const int p0 = g0 - 1, p1 = p0 + g1, p2 = p1 + g2;
        set_bit<W>(gam, p0, N);
        set_bit<W>(gam, p1, N);
        set_bit<W>(gam, p2, N);
        if (p2 < N - 1) {   // k = 0: gap j >= 3 is PERT call (j-3) >> 2, word (j-3) & 3;
                            // k >= 1: gap 3 is word 3, gap j >= 4 SETTLE_ENV call (k-1) << 8 | j >> 2
          Word4 P = E;
          int pos = p2;
          for (int j = 3; pos < N - 1; ++j) {
            const int jj = first ? j - 3 : j;
            if ((jj & 3) == 0)
              P = pbn::philox(ge_lo, st_lo,
                              first ? ((pbn::kStreamPert << 28) | (uint32_t)(jj >> 2))
                                    : ((pbn::kStreamSettleEnv << 28) | ((k - 1) << 8) | (uint32_t)(jj >> 2)),
                              ge_hi, u_k0, u_k1);
            const int j4 = jj & 3;
            const uint32_t u = j4 == 0 ? P.x : (j4 == 1 ? P.y : (j4 == 2 ? P.z : P.w));
            pos += gap_any(a.gap_exact, L, a, u);
            set_bit<W>(gam, pos, N);
          }
        }
      }
      PBN_PSTAMP_AT(it - kSettleStampIt + 10, 17);
#pragma unroll
      for (int w = 0; w < W; ++w) {
        slot[w * 64 + lane] = m[w];
        slot[kGP + w * 64 + lane] = gam[w];
      }
      PBN_PSTAMP(it - kSettleStampIt + 10, 1);
      lds_barrier();
      PBN_PSTAMP(it - kSettleStampIt + 10, 2);
    }
  } else if (role == 2) {
    // ---- selection planes of each env's update R(i), env `lane`; one loop per threshold count
    // NQ (= mnf - 1) and compare form PK, so that neither is a branch inside the loop (NQ = 0: every
    // node has one function, no draws are needed)
    const int pk_node = pk_lane_node(l32);
    // (the key by value: captured by reference it left the env role's laundered copy in VGPRs)
    auto sel_loop = [&, s_k0 = u_k0, s_k1 = u_k1](auto nq_c, auto pk_c) __attribute__((always_inline)) {
    constexpr int NQ = decltype(nq_c)::value;
    constexpr bool PK = decltype(pk_c)::value;
    for (uint32_t it = 0;; ++it) {
      PBN_ISA_LOOP("settle_sel", 2 * NQ + (PK ? 1 : 0));
      PBN_PSTAMP(it - kSettleStampIt + 10, 0);
      uint4 C = ctl[((it + 1) & 1) * 64 + lane];   // {C(i), R(i)}
      // all four words from one read, ahead of the exit test (split, R came in a second round trip)
      asm volatile("" : "+v"(C.x), "+v"(C.y), "+v"(C.z), "+v"(C.w));
      if (__ballot(C.x < n_steps) == 0 || (uint64_t)it > max_it) break;
      const uint32_t t = C.z, k = C.w;   // (no update: the words are computed and discarded)
      // PK: this iteration's packed thresholds, requested now (used after the Philox calls)
      uint4 thv[W][NQ > 0 ? NQ : 1][4];
      if constexpr (PK) {
#pragma unroll
        for (int r = 0; r < W; ++r)
#pragma unroll
          for (int q = 0; q < NQ; ++q)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              thv[r][q][c] = reinterpret_cast<const uint4*>(thr_l + (size_t)(q * W + r) * 16)[c];
            }
      }
      uint32_t* lt_out = slots + (size_t)(it & 1) * a.slot_words + kLT + half * 32 * W;
      const uint64_t step = step0 + (uint64_t)t;
      const uint32_t st_lo = (uint32_t)step;
      const uint32_t ge_hi = (uint32_t)((ge >> 32) & 0xFFFFu) | ((uint32_t)((step >> 32) & 0xFFFFu) << 16);
      const uint32_t* th = a.sthr;
      asm volatile("" : "+s"(th));   // the thresholds are read per iteration (hoisted: SGPR spills)
#pragma unroll
      for (int r = 0; r < W; ++r) {
        if constexpr (NQ > 0) {
          uint32_t U[16];
          // PK: the compares' bias (^ 0x80008000) folded into words 0 and 2 of every call
          settle_sel_words<PK ? 0x80008000u : 0u>(ge_lo, ge_hi, st_lo, k, r, N, s_k0, s_k1, U);
          PBN_PSTAMP_AT(it - kSettleStampIt + 10, 18);
          if constexpr (PK) {
#pragma unroll
            for (int j = 0; j < 16; ++j)
              if (j & 1) U[j] ^= 0x80008000u;   // words 1 and 3 (the low products) are not
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
              const uint32_t lt = settle_lt_word_pk_v(U, thv[r][q]);
              lt_out[q * 64 * W + 32 * r + pk_node] = lane_transpose32(lt, lane);
            }
          } else {
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
              const uint32_t lt = settle_lt_word(U, th + (size_t)(q * W + r) * 32);
              lt_out[q * 64 * W + 32 * r + l32] = lane_transpose32(lt, lane);
            }
          }
        }
      }
      PBN_PSTAMP(it - kSettleStampIt + 10, 1);
      lds_barrier();
      PBN_PSTAMP(it - kSettleStampIt + 10, 2);
    }
    };
    const bool pk = __builtin_amdgcn_readfirstlane(a.settle_pk) != 0;
    using T_ = std::true_type;
    using F_ = std::false_type;
    switch (min(mnf - 1, kNodeRecs - 1)) {   // (lq >= 1 in the slot layout; one function per node needs no draws)
      case 0: sel_loop(std::integral_constant<int, 0>{}, F_{}); break;
      case 1: pk ? sel_loop(std::integral_constant<int, 1>{}, T_{}) : sel_loop(std::integral_constant<int, 1>{}, F_{}); break;
      case 2: pk ? sel_loop(std::integral_constant<int, 2>{}, T_{}) : sel_loop(std::integral_constant<int, 2>{}, F_{}); break;
      default: pk ? sel_loop(std::integral_constant<int, 3>{}, T_{}) : sel_loop(std::integral_constant<int, 3>{}, F_{}); break;
    }
  } else {
    // ---- state of env `lane` (env-major), bit-sliced per update for the node chains
    uint32_t rs[W];           // the autoreset state drawn at the current step's first update
    uint32_t rtv = 0, pcv = 0;
    uint32_t Ct = valid ? 0u : n_steps, Ck = 0;
    bool pacc = false;
#pragma unroll
    for (int w = 0; w < W; ++w) rs[w] = 0;
    // one loop per function count KF (mnf, at most kNodeRecs): no switch inside the loop
    auto state_loop = [&](auto kf_c) __attribute__((always_inline)) {
    constexpr int KF = decltype(kf_c)::value;
    // single-word states: the node records' input indices held in VGPRs, and each update's
    // selection planes and selectors read before the transpose (as pbn_rollout_pipe's state_fast),
    // so that their LDS latency is off the chain slot -> transpose -> gathers -> back-transpose
    uint32_t ins[KF];
#pragma unroll
    for (int q = 0; q < KF; ++q) ins[q] = W == 1 ? recL[q * 32 + l32].x : 0u;
    EnvPlan p;
    p.next(Ct, Ck, K);   // iteration 0's plan (then each iteration's, at the end of the one before)
    for (uint32_t it = 0;; ++it) {
      PBN_ISA_LOOP("settle_state", KF);
      PBN_PSTAMP(it - kSettleStampIt + 10, 0);
      if (__ballot(Ct < n_steps) == 0 || (uint64_t)it > max_it) break;
      // the lowest step whose row is not stored yet, as the env-draw wave left it in the iteration
      // that produced this update: an update R - 1 or more steps past it waits (no row to write)
      const uint32_t sbase = stg_base[(it + 1) & 1];
      const bool proc = p.v && p.Pt < n_steps && p.Pt < sbase + R;
      const uint32_t t = p.Pt, k = p.Pk;
      uint32_t* row = stg + (size_t)(t % R) * RW;
      const uint32_t* slot = slots + (size_t)((it + 1) & 1) * a.slot_words;
      const uint32_t* lt_in = slot + kLT + half * 32 * W;
      uint32_t s1[W], gam[W];
      bool pk = false;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        s1[w] = st[w] ^ slot[w * 64 + lane];   // (the flip mask is 0 past an update's first)
        gam[w] = slot[kGP + w * 64 + lane];
        pk = pk || gam[w] != 0;
      }
      if (proc && k == 0) {   // the step's reset draw and action count; the step's observation
#pragma unroll
        for (int w = 0; w < W; ++w) row[kSO + w * 64 + lane] = st[w];
#pragma unroll
        for (int w = 0; w < W; ++w) rs[w] = slot[kRS + w * 64 + lane];
        const uint32_t info = slot[kIN + lane];
        rtv = info & 0xFFu;
        pcv = (info >> 8) & 0xFFu;
        pacc = false;
      }
      uint32_t X[W];
      if constexpr (W == 1) {
        uint32_t ltv[KF];
        uint4 sa[KF], sb[KF];
#pragma unroll
        for (int q = 0; q < KF; ++q) {
          ltv[q] = q < KF - 1 ? lt_in[q * 64 + l32] : 0u;
          sa[q] = selq[(2 * q) * 32 + l32];
          sb[q] = selq[(2 * q + 1) * 32 + l32];
        }
        Sg[l32] = lane_transpose32(s1[0], lane);
        PBN_PSTAMP_AT(it - kSettleStampIt + 10, 15);
        __builtin_amdgcn_wave_barrier();
        uint32_t x = 0;
#pragma unroll
        for (int q = KF - 1; q >= 0; --q) {
          uint32_t xin[4];
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) xin[kk] = plane_in<true>(Sg, ins[q], kk);
          const uint32_t fj = eval_sel_in(xin, sa[q], sb[q]);
          x = (q == KF - 1) ? fj : bfi(ltv[q], fj, x);
        }
        X[0] = x;
      } else {
#pragma unroll
        for (int w = 0; w < W; ++w) Sg[32 * w + l32] = lane_transpose32(s1[w], lane);
        PBN_PSTAMP_AT(it - kSettleStampIt + 10, 15);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < W; ++r) {
          int i = l32 + 32 * r;
          asm volatile("" : "+v"(i));   // selector and record reads stay in the loop
          const uint4* rc = recL + i;
          const uint4* sel = selq + i;
          const uint32_t* lti = lt_in + i;
          X[r] = chain_padded<KF, (W <= 2)>(rc, sel, 32 * W, Sg, lti, 64 * W);
        }
      }
      PBN_PSTAMP_AT(it - kSettleStampIt + 10, 3);
      uint32_t cur[W];
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const uint32_t x = lane_transpose32(X[w], lane);
        cur[w] = proc ? (pk ? s1[w] ^ gam[w] : x) : st[w];
      }
      PBN_PSTAMP_AT(it - kSettleStampIt + 10, 12);
      const int att = attractor_lookup<W>(a, htab, cur);
      const bool open = att < 0;
      const bool end = proc && (!open || k + 1 >= K);
      if (proc) {
        pacc = pacc || pk;
        Ct = end ? t + 1 : t;
        Ck = end ? 0u : k + 1;
      }
      // the next iteration's plan, published with the decision (the RNG waves read it)
      p.done();
      p.next(Ct, Ck, K);
      ctl[(it & 1) * 64 + lane] = make_uint4(Ct, Ck, p.Rt, p.Rk);
#pragma unroll
      for (int w = 0; w < W; ++w) st[w] = cur[w];
      if (end) {
        // the epilogue of step t, into the block's row of step t (stored by the env-draw wave)
#pragma unroll
        for (int w = 0; w < W; ++w) row[kSF + w * 64 + lane] = cur[w];
        reinterpret_cast<uint16_t*>(row + kSU)[lane] = (uint16_t)min(k + 1, 0xFFFFu);
        const bool in_attr = att >= 0;
        const bool term = in_attr && (uint32_t)att == tg0;
        const bool wrong = in_attr && !term;
        int tt = (int)tt0 + 1;
        tt = tt > 255 ? 255 : tt;
        const bool trunc = a.horizon > 0 && tt >= a.horizon;
        const bool rst = (u_fl & 8u) && (term || trunc);
        const uint32_t fl = (uint32_t)term | ((uint32_t)trunc << 1) | ((uint32_t)in_attr << 2) |
                            ((uint32_t)pacc << 3) | ((uint32_t)rst << 4) | ((uint32_t)open << 5);
        // the reward row as one 16-byte read (split by the compiler into reads under the term /
        // wrong branches, it cost two round trips in the epilogue)
        float4 r4 = reinterpret_cast<const float4*>(rtab)[pcv];
        asm volatile("" : "+v"(r4.x), "+v"(r4.y), "+v"(r4.z));
        row[kSR + lane] = __float_as_uint(term ? r4.z : (wrong ? r4.y : r4.x));
        reinterpret_cast<uint8_t*>(row + kSFL)[lane] = (uint8_t)fl;
        tg0 = rst ? rtv : tg0;
        tt0 = rst ? 0u : (uint32_t)tt;
#pragma unroll
        for (int w = 0; w < W; ++w) st[w] = rst ? rs[w] : cur[w];
      }
      PBN_PSTAMP(it - kSettleStampIt + 10, 1);
      lds_barrier();
      PBN_PSTAMP(it - kSettleStampIt + 10, 2);
    }
    };
    switch (mnf) {
      case 1: state_loop(std::integral_constant<int, 1>{}); break;
      case 2: state_loop(std::integral_constant<int, 2>{}); break;
      case 3: state_loop(std::integral_constant<int, 3>{}); break;
      default: state_loop(std::integral_constant<int, 4>{}); break;
    }
    if (valid) {
#pragma unroll
      for (int w = 0; w < W; ++w) a.state_out[CK((size_t)w * n + le, plane, 16)] = st[w];
      a.t[CK(le, n, 17)] = (uint8_t)tt0;
      a.target[CK(le, n, 18)] = (uint8_t)tg0;
    }
  }
}

// ------------------------------------------------------------- state histogram
// Visits per state for the steady-state distribution.  States of a steady-state chain
// concentrate on a few attractor basins, so a wave first merges equal values (a few
// ballot rounds: the leader adds the count of its value) before per-lane atomics.
__global__ void __launch_bounds__(256) pbn_hist_kernel(const uint32_t* __restrict__ states, int64_t n_rows,
                                                       int64_t n_cols, int64_t row_stride, uint32_t mask,
                                                       uint32_t* __restrict__ hist) {
  const int64_t total = n_rows * n_cols;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < total; base += stride) {
    const int64_t i = base + threadIdx.x;
    const bool have = i < total;
    uint32_t v = 0;
    if (have) {
      const int64_t r = i / n_cols, c = i - r * n_cols;
      v = states[r * row_stride + c] & mask;
    }
    bool pending = have;
#pragma unroll
    for (int round = 0; round < 4; ++round) {
      const uint64_t act = __ballot(pending);
      if (act == 0) break;
      const int leader = __builtin_ctzll(act);
      const uint32_t lv = __shfl(v, leader);
      const uint64_t same = __ballot(pending && v == lv);
      if ((threadIdx.x & 63) == leader) atomicAdd(&hist[lv], (uint32_t)__popcll(same));
      if (pending && v == lv) pending = false;
    }
    if (pending) atomicAdd(&hist[v], 1u);
  }
}

// ---------------------------------------------------------------- reset kernel
template <int W>
__global__ void __launch_bounds__(256) pbn_reset_kernel(const int32_t* __restrict__ att_start,
                                                        const uint32_t* __restrict__ att_states,
                                                        int n_attr, int n_states, int N, uint64_t seed, uint64_t step,
                                                        uint64_t env_offset, int64_t n, uint32_t* state,
                                                        uint8_t* target, uint8_t* t) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t ge = env_offset + (uint64_t)i;
  const Word4 r0 = pbn::draw(seed, ge, step, pbn::kStreamReset, 0);
  uint32_t ns[W];
  uint32_t nt;
  if (n_attr >= 1) {
    // (start, target != start) in one draw over the A(A-1) pairs, then the start state
    // uniformly within the start attractor, from the 64-bit value (word 1 : word 0)
    uint32_t hi = r0.y, lo = r0.x;
    const uint32_t A = (uint32_t)n_attr;
    uint32_t as = 0;
    nt = 0;
    if (A >= 2) {
      const uint32_t c = ext64(hi, lo, A * (A - 1));
      as = c / (A - 1);
      nt = c - as * (A - 1);
      nt += (nt >= as) ? 1u : 0u;
    }
    const int st0 = att_start[CK(as, n_attr + 1, 20)];
    const uint32_t size = (uint32_t)(att_start[CK(as + 1, n_attr + 1, 21)] - st0);
    const uint32_t idx = ext64(hi, lo, size);
#pragma unroll
    for (int w = 0; w < W; ++w) ns[w] = att_states[CK((size_t)(st0 + idx) * W + w, (size_t)n_states * W, 22)];
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

}  // namespace
