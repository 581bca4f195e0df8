// pbn_learn.hip -- the BDQ learner's update_policy step (bdq_model/__init__.py:100-139) as three
// HIP launches over one flat parameter buffer (SURVEY.md 8(f) #3, config 5's training frame).
//
// The reference's update is a PyTorch program: np.stack of 256 sampled transitions, two forwards
// of the online network and one of the target network, the double-DQN target, the MSE, autograd,
// a per-tensor gradient clamp and Adam (:100-131).  On the GPU that is ~100 kernels of a few
// microseconds each, and the frame waits on their launch latency, not on arithmetic (the whole
// update is ~0.3 GFLOP).  Here it is three launches:
//
//   learn_fwd    3 B/16 blocks.  Block = 16 transitions of one of three row sets (online network
//                on s, online on s', target network on s').  The bilinear layer is a sum of
//                target-table rows (T[t][i][:] = sum_j target_t[j] W[:, i, j], the table the acting
//                kernel reads) over the state's set bits; the trunk and the heads run on
//                v_mfma_f32_16x16x4_f32 with the 16 transitions as the MFMA's columns and the
//                activations in LDS.  Stores the raw head outputs of all three sets and, for the
//                online s rows, every layer's activation (the backward's operands).
//   learn_bwd    B/16 blocks.  The TD error of bdq_update per (transition, branch): both duelings,
//                the online argmax over s', the target network's value there, the MSE's partial
//                sum, and the gradient at the head outputs; then the backward through the heads
//                and the trunk (transposed MFMA tiles, LeakyReLU derivative from the stored
//                activation), storing every layer's delta.
//   learn_apply  one wave per 16 x 16 gradient tile (K = the batch: dW = delta . act^T), the
//                bilinear layer's weight gradient from the packed state and target bits
//                (dW[o][i][j] = sum_r g[o][r] s_i[r] t_j[r]); each wave clamps its tile to
//                [-c, c] (:129-130), takes the Adam step on it, and, for the bilinear layer,
//                recomputes the target-table rows of the weights it just wrote.  Block 0 adds
//                the MSE's partial sums in block order (the loss is reproducible).
//
// Parameters, Adam's moments and the gradient share one layout (pbn_bdq_layout): the module's
// nn.Parameters are views into it (pbn_rl_amd/replay.py FusedBDQUpdate), so the acting kernel,
// the checkpoint and the PyTorch forward all see the same weights.  Row sets and activations
// are [feature][batch] in the workspace: both MFMA operands of a gradient tile are float4 loads
// along the batch.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "../../include/pbn_env.h"
#include "net_view.h"
#include "replay_draw.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kRows = 16;              // transitions per tile: the MFMA's 16 columns
constexpr int kWaves = 8;              // waves per forward / backward block
constexpr int kThreads = 64 * kWaves;
constexpr int kApplyWaves = 4;
constexpr int kD0 = 256, kD1 = 128, kD2 = 64, kD3 = 32, kDH = 64;   // bdq_model/network.py:29-36,46
constexpr int kMaxNT = 8;              // 16-column tiles of the bilinear layer's j (N <= 127)

enum Seg { BIL_W, BIL_B, L2_W, L2_B, L3_W, L3_B, L4_W, L4_B, H1_W, H1_B, H2_W, H2_B, TOTAL };

__host__ __device__ inline int64_t al16(int64_t x) { return (x + 15) & ~int64_t(15); }

void make_layout(int N, int H, int64_t* off) {
  const int64_t A = N + 1;
  const int64_t sz[TOTAL] = {256LL * N * N, kD0, (int64_t)kD1 * kD0, kD1, (int64_t)kD2 * kD1, kD2,
                             (int64_t)kD3 * kD2, kD3, (int64_t)H * kDH * kD3, (int64_t)H * kDH, H * A * kDH, H * A};
  int64_t o = 0;
  for (int s = 0; s < TOTAL; ++s) {
    off[s] = o;
    o += al16(sz[s]);
  }
  off[TOTAL] = o;
}

// ---- the network image (pbn_bdq_pack; the online one rewritten by learn_apply): the bilinear
// target table [n_attr][N][256] (the acting kernels' operand), then the dense layers' weights as
// 16 x 16 tiles in MFMA-fragment order, so that a wave's fragment of a tile is one 1 KB contiguous
// load (as 16-row x 64-byte fragment loads of the row-major weights they cost learn_fwd 3.7 of its
// 22.8 us, profiles/r06_l_learn_fwd_probes.json).  Layer matrix M (rows R, columns C; the second
// head layers stacked as H x Apad rows, zero past each head's A), tile (ot, kt) at float
// (ot * C/16 + kt) * 256, twice:
//   fwd: lane g*16 + r holds M[16 ot + r][16 kt + 4g + v], v = 0..3 (learn_fwd's A operand)
//   bwd: lane g*16 + r holds M[16 ot + 4g + v][16 kt + r]            (learn_bwd's transposed one)
enum Lay { LY2, LY3, LY4, LYH1, LYH2, NLAY };

struct ImageLayout {
  int64_t fwd[NLAY], bwd[NLAY], total;   // float offsets from the image's start
  int rows[NLAY], cols[NLAY];
};

void make_image(int N, int H, int n_attr, ImageLayout* im) {
  const int Apad = 16 * ((N + 1 + 15) / 16);
  const int R[NLAY] = {kD1, kD2, kD3, H * kDH, H * Apad}, C[NLAY] = {kD0, kD1, kD2, kD3, kDH};
  int64_t o = (int64_t)n_attr * N * 256;
  for (int l = 0; l < NLAY; ++l) {
    im->rows[l] = R[l];
    im->cols[l] = C[l];
    im->fwd[l] = o;
    o += (int64_t)R[l] * C[l];
    im->bwd[l] = o;
    o += (int64_t)R[l] * C[l];
  }
  im->total = o;
}

struct LearnArgs {
  // the replay ring and the sampled rows
  const int64_t* idx;
  int B;
  int64_t cap;
  const uint32_t* st;
  const uint32_t* nst;
  const uint8_t* tgt;
  const int32_t* act;
  const float* rew;
  const uint8_t* done;
  // the network's attractor table (first state of attractor t: the target half of the input)
  const uint32_t* att_first;   // [n_attr][W]
  int n_attr, N, W, K, H, A, Apad;
  // parameters (online, updated in place; target, read), their target tables, Adam's state
  float* P;
  float* Tq;          // the online network's image (its table, then the weight tiles: make_image)
  const float* PT;
  const float* TqT;   // the target network's
  int64_t ifw[NLAY], ibw[NLAY];   // the weight tiles' offsets in the images
  float* m;
  float* v;
  float* step;
  int64_t off[TOTAL + 1];
  float lr, b1, b2, eps, gamma, clampv, slope;
  // workspace: [feature][B] planes
  float* heads;   // [3][H][B][Apad]: a row's outputs contiguous (the TD pass reads them by rows)
  float* y1;      // [256][B]  online s rows, after the activation
  float* h2;      // [128][B]
  float* h3;      // [64][B]
  float* h4;      // [32][B]
  float* hh;      // [64 H][B]
  float* dheads;  // [H][Apad][B]
  float* dhh;     // [64 H][B]
  float* dh4;     // [32][B]
  float* dh3;     // [64][B]
  float* dh2;     // [128][B]
  float* g1;      // [256][B]
  uint32_t* srow; // [W][B] state words of the sampled rows
  uint32_t* trow; // [W][B] their target attractors' first-state words
  float* partial; // [B / 16]
  float* loss;
  float* grad;    // optional: the clamped gradient, parameter layout
  unsigned long long* stamps;   // diagnostic builds (PBN_STAMPS): [kernel][block][wave][32] s_memtime
  // the frame's counters and the next frame's rows (pbn_frame_advance): learn_apply's extra last
  // block, when adv_on
  int adv_on;
  pbn_frame_advance adv;
};

// Diagnostic phase clocks (tools/learn_stamps.py): lane 0 of every wave of the first 1,024 blocks
// stores s_memtime at numbered points of each kernel (below), and s_memrealtime at entry (31)
constexpr int kLStampRow = 32;
#ifdef PBN_STAMPS
#define PBN_LSTAMP(k, i)                                                                                      \
  do {                                                                                                      \
    if (a.stamps && (threadIdx.x & 63) == 0 && blockIdx.x < 1024)                                           \
      a.stamps[(((size_t)(k) * 1024 + blockIdx.x) * 8 + (threadIdx.x >> 6)) * kLStampRow + (i)] =           \
          (i) == 31 ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();                      \
  } while (0)
#else
#define PBN_LSTAMP(k, i) do {} while (0)
#endif

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float leaky(float x, float slope) { return x > 0.f ? x : x * slope; }

// A block barrier that orders LDS only: the waves of learn_fwd / learn_bwd exchange nothing
// through global memory, so a barrier need not wait for their global stores (on CDNA they count
// in vmcnt with the loads) or for the weight fragments requested ahead.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ int64_t row_index(const LearnArgs& a, int b) {
  const int64_t j = a.idx[b];
  return j < 0 ? 0 : (j >= a.cap ? a.cap - 1 : j);   // (sample_indices keeps 0 <= j < size)
}

// ---- forward tiles.  Activations in LDS are blocked [K/16][16 rows][16]: the float4 at
// (kb, r, 4g) holds features 16 kb + 4g .. +3 of row r, the B operand of four k-steps of lane
// (g = lane >> 4, r = lane & 15).  D[o][r] = sum_k W[o][k] X[k][r] for the 16 outputs o0..o0+15:
// lane l supplies A[o0 + (l & 15)][k] = one float4 of weight row o0 + (l & 15); its accumulator
// holds D[o0 + 4g + v][r], v = 0..3.
// The weight fragments come in registers, loaded by wfrag before the layer's inputs are ready
// (every layer's fragments are requested at kernel entry: one L2 round trip, not one per layer):
// output tile ot of a layer with K inputs, from its fwd tiles in the image (zero past n_ot tiles)
template <int K>
__device__ __forceinline__ void wfrag(float4 (&w)[K / 16], const float* __restrict__ tiles, int ot, int n_ot, int lane) {
  const bool ok = ot < n_ot;
  const float4* t = reinterpret_cast<const float4*>(tiles) + (size_t)(ok ? ot : 0) * (K / 16) * 64 + lane;
#pragma unroll
  for (int kb = 0; kb < K / 16; ++kb) {
    w[kb] = t[kb * 64];
    if (!ok) w[kb] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int K>
__device__ __forceinline__ f32x4 fwd_tile(const float4 (&wf)[K / 16], const float* __restrict__ Xs, int lane) {
  const int g = lane >> 4, rr = lane & 15;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kb = 0; kb < K / 16; ++kb) {
    const float4 w = wf[kb];
    const float4 x = *reinterpret_cast<const float4*>(Xs + (kb * 16 + rr) * 16 + 4 * g);
    acc = mfma(w.x, x.x, acc);
    acc = mfma(w.y, x.y, acc);
    acc = mfma(w.z, x.z, acc);
    acc = mfma(w.w, x.w, acc);
  }
  return acc;
}

// bias + LeakyReLU, into the blocked LDS plane (tile o0) and, when `out` is set, the [O][B] plane
__device__ __forceinline__ void fwd_store(f32x4 acc, const float* __restrict__ bias, int o0, float slope,
                                          float* __restrict__ Ys, float* __restrict__ out, int B, int b0, int lane) {
  const int g = lane >> 4, rr = lane & 15;
  float4 y;
  float* yp = &y.x;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int o = o0 + 4 * g + v;
    yp[v] = leaky(acc[v] + bias[o], slope);
    if (out) out[(size_t)o * B + b0 + rr] = yp[v];
  }
  *reinterpret_cast<float4*>(Ys + ((o0 >> 4) * 16 + rr) * 16 + 4 * g) = y;
}

// learn_fwd's biases in LDS: [bilinear 256 | 128 | 64 | 32 | H x 64 | H x A] (the layer epilogues
// read them there: a global load of the bias put its round trip on every layer's path)
__host__ __device__ inline int fwd_bias_floats(int H, int A) { return kD0 + kD1 + kD2 + kD3 + kDH * H + H * A; }
__device__ __forceinline__ int64_t fwd_bias_src(const LearnArgs& a, int idx) {
  if (idx < kD0) return a.off[BIL_B] + idx;
  idx -= kD0;
  if (idx < kD1) return a.off[L2_B] + idx;
  idx -= kD1;
  if (idx < kD2) return a.off[L3_B] + idx;
  idx -= kD2;
  if (idx < kD3) return a.off[L4_B] + idx;
  idx -= kD3;
  if (idx < kDH * a.H) return a.off[H1_B] + idx;
  return a.off[H2_B] + idx - kDH * a.H;
}

__global__ void __launch_bounds__(kThreads) learn_fwd_kernel(LearnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Y1 = lds;                    // [256/16][16][16]
  float* X2 = Y1 + kD0 * kRows;       // [128/16][16][16]
  float* X3 = X2 + kD1 * kRows;
  float* X4 = X3 + kD2 * kRows;
  float* XH = X4 + kD3 * kRows;       // [64 H / 16][16][16]
  uint32_t* sw = reinterpret_cast<uint32_t*>(XH + kDH * a.H * kRows);   // [4][16]
  int* stg = reinterpret_cast<int*>(sw + 4 * kRows);                  // [16]
  int* scnt = stg + kRows;                                            // [16]: set bits per row
  uint8_t* slist = reinterpret_cast<uint8_t*>(scnt + kRows);          // [16][128]: their indices, ascending
  float* sbias = reinterpret_cast<float*>(slist + kRows * 128);       // fwd_bias_floats
  const int tiles = a.B / kRows;
  const int set = blockIdx.x / tiles;
  const int b0 = (blockIdx.x - set * tiles) * kRows;
  const float* P = set == 2 ? a.PT : a.P;
  const float* Tq = set == 2 ? a.TqT : a.Tq;
  PBN_LSTAMP(0, 31);
  PBN_LSTAMP(0, 0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // the biases, requested first (unguarded: a clamped index) and stored to LDS before the first
  // barrier
  const int nbias = fwd_bias_floats(a.H, a.A);
  float bv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) bv[k] = P[fwd_bias_src(a, min(tid + kThreads * k, nbias - 1))];
  const int B = a.B;
  float* keep = nullptr;   // the online s rows keep their activations for the backward
  // every layer's weight fragments of this wave, requested at entry (they arrive during the row
  // and bilinear phases: no barrier waits for them)
  const int at16 = a.Apad / 16;
  float4 w2[kD0 / 16], w3[kD1 / 16], w4[kD2 / 16], wh1[2][kD3 / 16], wh2[kDH / 16];
  auto fetch_weights = [&]() {
    wfrag<kD0>(w2, Tq + a.ifw[LY2], wave, kD1 / 16, lane);
    if (wave < kD2 / 16) wfrag<kD1>(w3, Tq + a.ifw[LY3], wave, kD2 / 16, lane);   // (only these waves
    if (wave < kD3 / 16) wfrag<kD2>(w4, Tq + a.ifw[LY4], wave, kD3 / 16, lane);   // compute the layers)
#pragma unroll
    for (int u = 0; u < 2; ++u) wfrag<kD3>(wh1[u], Tq + a.ifw[LYH1], wave + kWaves * u, a.H * kDH / 16, lane);
    wfrag<kDH>(wh2, Tq + a.ifw[LYH2], wave < a.H * at16 ? wave : 0, a.H * at16, lane);
  };
  if (wave != 0) fetch_weights();   // (wave 0 loads the rows first: the load counter is in order)
  if (tid < kRows) {   // the rows' targets, state words and the list of their set bits
    const int64_t j = row_index(a, b0 + tid);
    stg[tid] = a.tgt[j];
    int c = 0;
    for (int w = 0; w < a.W; ++w) {
      uint32_t x = (set == 0 ? a.st : a.nst)[(size_t)w * a.cap + j];
      if (w == a.W - 1 && (a.N & 31)) x &= (1u << (a.N & 31)) - 1u;
      sw[w * kRows + tid] = x;
      while (x) {
        slist[tid * 128 + c++] = (uint8_t)(32 * w + __builtin_ctz(x));
        x &= x - 1u;
      }
    }
    scnt[tid] = c;
  }
  if (wave == 0) fetch_weights();
  // (unconditional: past the biases into a spare slot; a branch here made the wait counter's merge
  // hold the first barrier for every weight fragment)
#pragma unroll
  for (int k = 0; k < 4; ++k) sbias[min(tid + kThreads * k, nbias)] = bv[k];
  lds_barrier();
  PBN_LSTAMP(0, 1);
  // bilinear layer: y[o] = bias[o] + sum over the set bits i of T[t][i][o] (t = the row's target;
  // a row without a target has an all-zero second input: bias only).  Wave w takes rows 2w, 2w+1;
  // lane p reads Tq positions 4p..4p+3 ([t][i][j][q] = T[t][i][16 q + j]: o = 16 q + j): only the
  // table rows of set bits, eight of each row per round trip.
  {
    const float* bias = sbias;
    const int r0 = 2 * wave;
    const int t0 = stg[r0], t1 = stg[r0 + 1];
    const int c0 = t0 < a.n_attr ? scnt[r0] : 0, c1 = t1 < a.n_attr ? scnt[r0 + 1] : 0;
    float4 acc[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
    const int cm = max(c0, c1);
    if (cm > 0) {
      const uint8_t* l0 = slist + r0 * 128;
      const uint8_t* l1 = l0 + 128;
      // buffer loads: a lane past its row's count gets an out-of-range offset, whose load returns
      // zeros without memory traffic (it read table row 0 before: ~35 % of the reads at 14-17 bits)
      const int tb0 = __builtin_amdgcn_readfirstlane(c0 ? t0 : 0), tb1 = __builtin_amdgcn_readfirstlane(c1 ? t1 : 0);
      const int nrec = a.N * 256 * 4;
      __amdgpu_buffer_rsrc_t R0 = __builtin_amdgcn_make_buffer_rsrc((void*)(Tq + (size_t)tb0 * a.N * 256), (short)0, nrec, 0x00020000);
      __amdgpu_buffer_rsrc_t R1 = __builtin_amdgcn_make_buffer_rsrc((void*)(Tq + (size_t)tb1 * a.N * 256), (short)0, nrec, 0x00020000);
      for (int p0 = 0; p0 < cm; p0 += 8) {
        float4 x0[8], x1[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int p = p0 + u;
          const int i0 = l0[min(p, 127)], i1 = l1[min(p, 127)];
          const int o0 = p < c0 ? (i0 * 256 + 4 * lane) * 4 : 0x40000000;
          const int o1 = p < c1 ? (i1 * 256 + 4 * lane) * 4 : 0x40000000;
          auto v0 = __builtin_amdgcn_raw_buffer_load_b128(R0, o0, 0, 0);
          auto v1 = __builtin_amdgcn_raw_buffer_load_b128(R1, o1, 0, 0);
          x0[u] = *reinterpret_cast<float4*>(&v0);
          x1[u] = *reinterpret_cast<float4*>(&v1);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const bool on0 = p0 + u < c0, on1 = p0 + u < c1;
          acc[0].x += on0 ? x0[u].x : 0.f;
          acc[0].y += on0 ? x0[u].y : 0.f;
          acc[0].z += on0 ? x0[u].z : 0.f;
          acc[0].w += on0 ? x0[u].w : 0.f;
          acc[1].x += on1 ? x1[u].x : 0.f;
          acc[1].y += on1 ? x1[u].y : 0.f;
          acc[1].z += on1 ? x1[u].z : 0.f;
          acc[1].w += on1 ? x1[u].w : 0.f;
        }
      }
    }
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int r = r0 + rr;
      const float* ap = &acc[rr].x;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int o = 16 * (4 * (lane & 3) + c) + (lane >> 2);
        const float y = leaky(ap[c] + bias[o], a.slope);
        Y1[((o >> 4) * 16 + r) * 16 + (o & 15)] = y;
        if (set == 0) a.y1[(size_t)o * B + b0 + r] = y;
      }
    }
  }
  PBN_LSTAMP(0, 2);
  lds_barrier();
  PBN_LSTAMP(0, 3);
  if (set == 0) keep = a.h2;
  {   // 256 -> 128: one output tile per wave
    const f32x4 acc = fwd_tile<kD0>(w2, Y1, lane);
    fwd_store(acc, sbias + kD0, 16 * wave, a.slope, X2, keep, B, b0, lane);
  }
  PBN_LSTAMP(0, 4);
  lds_barrier();
  PBN_LSTAMP(0, 5);
  if (wave < kD2 / 16) {   // 128 -> 64
    const f32x4 acc = fwd_tile<kD1>(w3, X2, lane);
    fwd_store(acc, sbias + kD0 + kD1, 16 * wave, a.slope, X3, set == 0 ? a.h3 : nullptr, B, b0, lane);
  }
  lds_barrier();
  PBN_LSTAMP(0, 6);
  if (wave < kD3 / 16) {   // 64 -> 32
    const f32x4 acc = fwd_tile<kD2>(w4, X3, lane);
    fwd_store(acc, sbias + kD0 + kD1 + kD2, 16 * wave, a.slope, X4, set == 0 ? a.h4 : nullptr, B, b0, lane);
  }
  lds_barrier();
  PBN_LSTAMP(0, 7);
  {   // the H first head layers: 32 -> 64 H
    const int n1 = a.H * kDH / 16;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int tt = wave + kWaves * u;
      if (tt < n1) {
        const f32x4 acc = fwd_tile<kD3>(wh1[u], X4, lane);
        fwd_store(acc, sbias + kD0 + kD1 + kD2 + kD3, 16 * tt, a.slope, XH, set == 0 ? a.hh : nullptr, B, b0, lane);
      }
    }
    for (int tt = wave + 2 * kWaves; tt < n1; tt += kWaves) {
      float4 wl[kD3 / 16];
      wfrag<kD3>(wl, Tq + a.ifw[LYH1], tt, n1, lane);
      const f32x4 acc = fwd_tile<kD3>(wl, X4, lane);
      fwd_store(acc, sbias + kD0 + kD1 + kD2 + kD3, 16 * tt, a.slope, XH, set == 0 ? a.hh : nullptr, B, b0, lane);
    }
  }
  lds_barrier();
  PBN_LSTAMP(0, 8);
  // second head layers: head h, outputs 16 at .. (A of them, no activation) -> heads[set][h][b][a]
  auto head_out = [&](const float4 (&wl)[kDH / 16], int tt) {
    const int h = tt / at16, o0 = 16 * (tt - h * at16);
    const f32x4 acc = fwd_tile<kDH>(wl, XH + h * kDH * kRows, lane);
    const int g = lane >> 4, rr = lane & 15;
    const float* b2 = sbias + kD0 + kD1 + kD2 + kD3 + kDH * a.H + h * a.A;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int o = o0 + 4 * g + v;
      if (o < a.A) a.heads[(((size_t)set * a.H + h) * B + b0 + rr) * a.Apad + o] = acc[v] + b2[o];
    }
  };
  if (wave < a.H * at16) head_out(wh2, wave);
  for (int tt = wave + kWaves; tt < a.H * at16; tt += kWaves) {
    float4 wl[kDH / 16];
    wfrag<kDH>(wl, Tq + a.ifw[LYH2], tt, a.H * at16, lane);
    head_out(wl, tt);
  }
  PBN_LSTAMP(0, 9);
}

// ---- backward tiles: dX[k][r] = sum_o W[o][k] dY[o][r] for the 16 inputs k0..k0+15 (A operand
// lane l: W[o][k0 + (l & 15)] for the k-step's o = 16 ob + 4g + v; B operand: the blocked dY
// plane, as the forward's X).  The accumulator holds dX[k0 + 4g + v][r].  Fragments (bwd_frag)
// are loaded ahead of the layer that uses them (bwd_mma).
// times LeakyReLU' (from the stored activation: y > 0 exactly when its input was), into the
// blocked LDS plane (rows kk0..) when Ys is set and the [K][B] plane
// the stored activations a backward tile's derivative needs (loaded ahead, like the weights)
__device__ __forceinline__ f32x4 act_frag(const float* __restrict__ act, int kk0, int B, int b0, int lane) {
  const int g = lane >> 4, rr = lane & 15;
  f32x4 y;
#pragma unroll
  for (int v = 0; v < 4; ++v) y[v] = act[(size_t)(kk0 + 4 * g + v) * B + b0 + rr];
  return y;
}

__device__ __forceinline__ void bwd_store(f32x4 acc, f32x4 yv, int kk0, float slope, float* __restrict__ Ys,
                                          float* __restrict__ out, int B, int b0, int lane) {
  const int g = lane >> 4, rr = lane & 15;
  float4 d;
  float* dp = &d.x;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int k = kk0 + 4 * g + v;
    const float y = yv[v];
    dp[v] = y > 0.f ? acc[v] : acc[v] * slope;
    out[(size_t)k * B + b0 + rr] = dp[v];
  }
  if (Ys) *reinterpret_cast<float4*>(Ys + ((kk0 >> 4) * 16 + rr) * 16 + 4 * g) = d;
}

// a layer's weight fragments for bwd_mma: input tile kt of a layer with KT input tiles, NOB
// output blocks from ob0, from its bwd tiles in the image (0 past n_ob)
template <int NOB>
__device__ __forceinline__ void bwd_frag(float (&w)[NOB][4], const float* __restrict__ tiles, int KT, int kt, int ob0,
                                         int n_ob, int lane) {
#pragma unroll
  for (int u = 0; u < NOB; ++u) {
    const bool ok = ob0 + u < n_ob;
    const float4 x = reinterpret_cast<const float4*>(tiles)[((size_t)(ok ? ob0 + u : 0) * KT + kt) * 64 + lane];
    w[u][0] = ok ? x.x : 0.f;
    w[u][1] = ok ? x.y : 0.f;
    w[u][2] = ok ? x.z : 0.f;
    w[u][3] = ok ? x.w : 0.f;
  }
}

template <int NOB>
__device__ __forceinline__ f32x4 bwd_mma(f32x4 acc, const float (&w)[NOB][4], int ob0, int n_ob,
                                         const float* __restrict__ dYs, int lane) {
  const int g = lane >> 4, rr = lane & 15;
#pragma unroll
  for (int u = 0; u < NOB; ++u) {
    if (ob0 + u < n_ob) {
      const float4 y = *reinterpret_cast<const float4*>(dYs + ((ob0 + u) * 16 + rr) * 16 + 4 * g);
      acc = mfma(w[u][0], y.x, acc);
      acc = mfma(w[u][1], y.y, acc);
      acc = mfma(w[u][2], y.z, acc);
      acc = mfma(w[u][3], y.w, acc);
    }
  }
  return acc;
}

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m);
  return x;
}

__global__ void __launch_bounds__(kThreads) learn_bwd_kernel(LearnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int H = a.H, A = a.A, Ap = a.Apad, K = a.K, B = a.B;
  float* DH = lds;                        // per head [Apad/16][16][16]
  float* DHH = DH + H * Ap * kRows;       // [64 H / 16][16][16]
  float* DH4 = DHH + H * kDH * kRows;
  float* DH3 = DH4 + kD3 * kRows;
  float* DH2 = DH3 + kD2 * kRows;
  float* part = DH2 + kD1 * kRows;        // [8 waves][64 lanes][4]: the split first-head-layer tiles
  const int planes = (H * Ap + H * kDH + kD3 + kD2 + kD1) * kRows + kWaves * 64 * 4;
  float* sg = lds + max(planes, 3 * H * kRows * (Ap + 4));   // [16][K] (past the TD pass's staged heads)
  float* sd = sg + kRows * K;                          // [16][K]
  int* sact = reinterpret_cast<int*>(sd + kRows * K);  // [16][K]
  const int tile = blockIdx.x, b0 = tile * kRows;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, rr = lane & 15;
  const float* Tw = a.Tq;   // the online network's weight tiles
  PBN_LSTAMP(1, 31);
  PBN_LSTAMP(1, 0);
  // Issue order (vmcnt retires in order: a wait for a load waits for every load issued before
  // it): the TD pass's operands first -- the sampled rows' indices, the block's head rows, then
  // the rows' actions, rewards and done flags -- and only then the weight fragments and stored
  // activations the backward layers need after the pass, so that the pass waits for its own loads
  // alone (it waited for all of them; profiles/r06_ad_bwd_issue_order_ab.json)
  // [set][h][16][Apad + 4]: the row pitch Apad + 4 puts the 16 rows' lanes on distinct banks
  float* SH = lds;
  const int pitch = Ap + 4;
  const int per4 = kRows * Ap / 4;   // float4s of one (set, head) block of rows
  const int n4 = 3 * H * per4;
  // the TD pass: four lanes per (row r, branch k) pair p = tid >> 2 (r = p & 15, k = p >> 4)
  const bool tdl = tid < 4 * kRows * K;
  const int tp = tid >> 2, tq = tid & 3;
  int64_t jrow = 0;
  if (tdl) jrow = row_index(a, b0 + (tp & 15));
  int64_t jw = 0;   // wave 7: the rows' words for learn_apply
  const bool wrow = tid >= 64 * (kWaves - 1) && tid - 64 * (kWaves - 1) < kRows;
  if (wrow) jw = row_index(a, b0 + tid - 64 * (kWaves - 1));
  constexpr int kHeadPre = 4;   // head float4s per thread issued ahead (n4 <= 2048: every K <= 3 shape
                                // with N <= 31; more in the loop below)
  float4 hv[kHeadPre];
  auto head_src = [&](int e) __attribute__((always_inline)) {
    const int sh = e / per4, f = e - sh * per4;   // sh = set * H + h
    return reinterpret_cast<const float4*>(a.heads + ((size_t)sh * B + b0) * Ap)[f];
  };
  auto head_dst = [&](int e) __attribute__((always_inline)) {
    const int sh = e / per4, f = e - sh * per4;
    const int r = f / (Ap / 4), c = f - r * (Ap / 4);
    return reinterpret_cast<float4*>(SH + ((size_t)sh * kRows + r) * pitch + 4 * c);
  };
#pragma unroll
  for (int k = 0; k < kHeadPre; ++k) hv[k] = head_src(min(tid + kThreads * k, n4 - 1));
  int ak = 0;
  float rwj = 0.f, dnj = 0.f;
  if (tdl) {
    ak = a.act[(size_t)jrow * K + (tp >> 4)];
    rwj = a.rew[jrow];
    dnj = (float)a.done[jrow];
  }
  if (wrow) {
    const int b = b0 + tid - 64 * (kWaves - 1);
    const int tg = a.tgt[jw];
    for (int w = 0; w < a.W; ++w) {
      a.srow[(size_t)w * B + b] = a.st[(size_t)w * a.cap + jw];
      a.trow[(size_t)w * B + b] = tg < a.n_attr ? a.att_first[(size_t)tg * a.W + w] : 0u;
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  // the weight fragments of the first four backward layers: second head layers (tiles wave, wave
  // + 8 of H x 4), the first head layers split four ways per output tile (wave & 1 = tile, wave >> 1
  // = quarter of the 4 H blocks), 32 -> 64 (waves < 4) and 64 -> 128
  const int at16 = Ap / 16;
  float wh2[2][2][4], wh1[8][4], w4[2][4], w3[4][4];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int tt = min(wave + kWaves * u, H * (kDH / 16) - 1), h = tt >> 2;
    bwd_frag<2>(wh2[u], Tw + a.ibw[LYH2] + (size_t)h * at16 * (kDH / 16) * 256, kDH / 16, tt & 3, 0, at16, lane);
  }
  const int q1 = wave >> 1;   // quarter of the first head layers' 4 H output blocks: [q H, q H + H)
  bwd_frag<8>(wh1, Tw + a.ibw[LYH1], kD3 / 16, wave & 1, q1 * H, q1 * H + H, lane);
  bwd_frag<2>(w4, Tw + a.ibw[LY4], kD2 / 16, wave & 3, 0, kD3 / 16, lane);
  bwd_frag<4>(w3, Tw + a.ibw[LY3], kD1 / 16, wave, 0, kD2 / 16, lane);
  // and the stored activations of the same tiles (the LeakyReLU derivative)
  f32x4 yh2[2], y4 = act_frag(a.h4, 16 * (wave & 1), B, b0, lane), y3 = act_frag(a.h3, 16 * (wave & 3), B, b0, lane),
        y2 = act_frag(a.h2, 16 * wave, B, b0, lane), y1v[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int tt = min(wave + kWaves * u, H * (kDH / 16) - 1);
    yh2[u] = act_frag(a.hh, (tt >> 2) * kDH + 16 * (tt & 3), B, b0, lane);
    y1v[u] = act_frag(a.y1, 16 * (wave + kWaves * u), B, b0, lane);
  }
  __builtin_amdgcn_sched_barrier(0);
  PBN_LSTAMP(1, 1);

  // the TD error per (row, branch): bdq_update / update_policy (:111-126) on the raw heads.  The
  // block's head rows of the three sets come into LDS (coalesced; the staging area is the delta
  // planes', written only after this pass), then thread (row r, branch k) runs the duelings and
  // the online argmax over s' as sequential sums (the order of pbn_bdq_td_loss).
#pragma unroll
  for (int k = 0; k < kHeadPre; ++k)
    if (tid + kThreads * k < n4) *head_dst(tid + kThreads * k) = hv[k];
  for (int e = tid + kThreads * kHeadPre; e < n4; e += kThreads) *head_dst(e) = head_src(e);
  ak = ak < 0 ? 0 : (ak >= A ? A - 1 : ak);
  lds_barrier();
  PBN_LSTAMP(1, 2);
  if (tdl) {
    const int r = tp & 15, k = tp >> 4;
    auto hrow = [&](int set, int h) { return SH + ((size_t)(set * H + h) * kRows + r) * pitch; };
    const float* adv0 = hrow(0, k + 1);
    const float* adv1 = hrow(1, k + 1);
    const float* adv2 = hrow(2, k + 1);
    // the three duelings' means: lane tq < 3 sums set tq's row in order (eight LDS reads in
    // flight, the next eight requested before these are added); the means to every lane of the pair
    const float* mine = tq == 0 ? adv0 : (tq == 1 ? adv1 : adv2);
    float ssum = 0.f;
    float xc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) xc[u] = mine[min(u, A - 1)];
    for (int o0 = 0; o0 < A; o0 += 8) {
      float xn[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) xn[u] = mine[min(o0 + 8 + u, A - 1)];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (o0 + u < A) ssum += xc[u];
#pragma unroll
      for (int u = 0; u < 8; ++u) xc[u] = xn[u];
    }
    const float mq = ssum / (float)A;   // (lane 3: a fourth copy of set 2's, unused)
    const int l0 = lane & ~3;
    const float m0 = __shfl(mq, l0), m1 = __shfl(mq, l0 + 1), m2 = __shfl(mq, l0 + 2);
    // the online argmax over s' (torch.argmax: first maximum, NaN is the maximum): each lane scans
    // a quarter of actions 1 .. A-1 with the sequential rule, then the quarters are combined in
    // order with the same rule (which makes the combination the sequential scan's result)
    const float v1 = hrow(1, 0)[0];
    const int seg = (A - 1 + 3) / 4, lo = 1 + tq * seg, hi = min(lo + seg, A);
    bool have = lo < hi;
    float best = 0.f;
    int am = 0;
    if (have) {
      best = (v1 + adv1[lo]) - m1;
      am = lo;
      for (int o = lo + 1; o < hi; ++o) {
        const float qo = (v1 + adv1[o]) - m1;
        const bool take = !isnan(best) && (isnan(qo) || qo > best);
        best = take ? qo : best;
        am = take ? o : am;
      }
    }
    float gbest = (v1 + adv1[0]) - m1;
    int gam = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float b = __shfl(best, l0 + q);
      const int ai = __shfl(am, l0 + q);
      const bool h = __shfl((int)have, l0 + q) != 0;
      const bool take = h && !isnan(gbest) && (isnan(b) || b > gbest);
      gbest = take ? b : gbest;
      gam = take ? ai : gam;
    }
    if (tq == 0) {
      const float current = (hrow(0, 0)[0] + adv0[ak]) - m0;
      const float tnext = (hrow(2, 0)[0] + adv2[gam]) - m2;
      const float expected = rwj + (tnext * a.gamma) * dnj;
      const float d = expected - current;
      sd[r * K + k] = d * d;
      sg[r * K + k] = 2.f * (current - expected) / (float)(B * K);
      sact[r * K + k] = ak;
    }
  }
  PBN_LSTAMP(1, 3);
  lds_barrier();
  PBN_LSTAMP(1, 4);
  // the gradient at the head outputs: d/d adv[k][o] = g_k ([o == a_k] - 1/A), d/d v = sum_k g_k
  // (0 for the value head's other outputs and the padding)
  for (int e = tid; e < H * Ap * kRows; e += kThreads) {
    const int oi = e & 15, r = (e >> 4) & 15, hb = e >> 8;   // hb = h * Apad/16 + o/16
    const int h = hb / at16, o = 16 * (hb - h * at16) + oi;
    float val = 0.f;
    if (o < A) {
      if (h == 0) {
        if (o == 0)
          for (int k = 0; k < K; ++k) val += sg[r * K + k];
      } else {
        const float gk = sg[r * K + h - 1];
        val = (o == sact[r * K + h - 1] ? gk : 0.f) - gk / (float)A;
      }
    }
    DH[e] = val;
    a.dheads[((size_t)h * Ap + o) * B + b0 + r] = val;
  }
  if (wave == 0) {   // the block's squared TD errors, a fixed-order reduction
    float sacc = 0.f;
    for (int p = lane; p < kRows * K; p += 64) sacc += sd[p];
    sacc = wave_sum(sacc);
    if (lane == 0) {
      a.partial[tile] = sacc;
      if (tile == 0) a.step[0] += 1.f;   // Adam's step count, read by learn_apply
    }
  }
  lds_barrier();
  // the last layer's fragments (256 inputs: tiles wave, wave + 8), requested now for the end
  float w2[2][8][4];
#pragma unroll
  for (int u = 0; u < 2; ++u) bwd_frag<8>(w2[u], Tw + a.ibw[LY2], kD0 / 16, wave + kWaves * u, 0, kD1 / 16, lane);
  // second head layers: Apad -> 64 per head
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int tt = wave + kWaves * u;
    if (tt < H * (kDH / 16)) {
      const int h = tt >> 2, c0 = 16 * (tt & 3);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      acc = bwd_mma<2>(acc, wh2[u], 0, at16, DH + h * Ap * kRows, lane);
      for (int ob0 = 2; ob0 < at16; ob0 += 2) {   // (A > 32)
        float wl[2][4];
        bwd_frag<2>(wl, Tw + a.ibw[LYH2] + (size_t)h * at16 * (kDH / 16) * 256, kDH / 16, c0 / 16, ob0, at16, lane);
        acc = bwd_mma<2>(acc, wl, ob0, at16, DH + h * Ap * kRows, lane);
      }
      bwd_store(acc, yh2[u], h * kDH + c0, a.slope, DHH, a.dhh, B, b0, lane);
    }
  }
  for (int tt = wave + 2 * kWaves; tt < H * (kDH / 16); tt += kWaves) {   // (H > 4)
    const int h = tt >> 2, c0 = 16 * (tt & 3);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int ob0 = 0; ob0 < at16; ob0 += 2) {
      float wl[2][4];
      bwd_frag<2>(wl, Tw + a.ibw[LYH2] + (size_t)h * at16 * (kDH / 16) * 256, kDH / 16, c0 / 16, ob0, at16, lane);
      acc = bwd_mma<2>(acc, wl, ob0, at16, DH + h * Ap * kRows, lane);
    }
    bwd_store(acc, act_frag(a.hh, h * kDH + c0, B, b0, lane), h * kDH + c0, a.slope, DHH, a.dhh, B, b0, lane);
  }
  PBN_LSTAMP(1, 5);
  lds_barrier();
  PBN_LSTAMP(1, 6);
  {   // first head layers: 64 H -> 32, each output tile split over four waves (H blocks each)
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = bwd_mma<8>(acc, wh1, q1 * H, q1 * H + H, DHH, lane);
    *reinterpret_cast<f32x4*>(part + (wave * 64 + lane) * 4) = acc;
  }
  lds_barrier();
  if (wave < kD3 / 16) {   // the four quarters added in order
    f32x4 acc = *reinterpret_cast<const f32x4*>(part + (wave * 64 + lane) * 4);
#pragma unroll
    for (int qq = 1; qq < 4; ++qq) acc += *reinterpret_cast<const f32x4*>(part + ((wave + 2 * qq) * 64 + lane) * 4);
    bwd_store(acc, y4, 16 * wave, a.slope, DH4, a.dh4, B, b0, lane);
  }
  lds_barrier();
  PBN_LSTAMP(1, 7);
  if (wave < kD2 / 16) {   // 32 -> 64
    const f32x4 acc = bwd_mma<2>(f32x4{0.f, 0.f, 0.f, 0.f}, w4, 0, kD3 / 16, DH4, lane);
    bwd_store(acc, y3, 16 * wave, a.slope, DH3, a.dh3, B, b0, lane);
  }
  lds_barrier();
  {   // 64 -> 128
    const f32x4 acc = bwd_mma<4>(f32x4{0.f, 0.f, 0.f, 0.f}, w3, 0, kD2 / 16, DH3, lane);
    bwd_store(acc, y2, 16 * wave, a.slope, DH2, a.dh2, B, b0, lane);
  }
  lds_barrier();
  PBN_LSTAMP(1, 8);
#pragma unroll
  for (int u = 0; u < 2; ++u) {   // 128 -> 256: the bilinear layer's output gradient
    const f32x4 acc = bwd_mma<8>(f32x4{0.f, 0.f, 0.f, 0.f}, w2[u], 0, kD1 / 16, DH2, lane);
    bwd_store(acc, y1v[u], 16 * (wave + kWaves * u), a.slope, nullptr, a.g1, B, b0, lane);
  }
  PBN_LSTAMP(1, 9);
  (void)g;
  (void)rr;
}

// ---- Adam (torch.optim.Adam, fused, defaults but lr: bdq_model/__init__.py:34) on one element,
// after clamping its gradient to [-c, c] (torch.clamp: NaN stays NaN)
// The element's parameter and moments are loaded ahead (adam_load, at the task's start: the
// round trip overlaps the gradient loop), adam_apply writes the step and returns the new value.
struct AdamIn {
  float p, m, v;
};

__device__ __forceinline__ AdamIn adam_load(const LearnArgs& a, int64_t i, bool ok) {
  return ok ? AdamIn{a.P[i], a.m[i], a.v[i]} : AdamIn{0.f, 0.f, 0.f};
}

__device__ __forceinline__ float adam_apply(const LearnArgs& a, int64_t i, AdamIn in, float g, float bc1, float bc2s) {
  g = isnan(g) ? g : fminf(fmaxf(g, -a.clampv), a.clampv);
  if (a.grad) a.grad[i] = g;
  const float m = a.b1 * in.m + (1.f - a.b1) * g;
  const float v = a.b2 * in.v + (1.f - a.b2) * g * g;
  a.m[i] = m;
  a.v[i] = v;
  const float denom = sqrtf(v) / bc2s + a.eps;
  const float p = in.p - (a.lr / bc1) * m / denom;
  a.P[i] = p;
  return p;
}

__device__ __forceinline__ uint4 target_words(const LearnArgs& a, int t) {
  uint32_t tw[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) tw[w] = (t < a.n_attr && w < a.W) ? a.att_first[(size_t)t * a.W + w] : 0u;
  return make_uint4(tw[0], tw[1], tw[2], tw[3]);
}

// Loads issued ahead of their use in straight-line code, without a branch or a select at the
// load: a guarded load puts its select right behind the load, and that select's s_waitcnt waits
// out every load issued before it (vmcnt retires in order: learn_apply's ISA had a vmcnt(0)
// behind each of its 16 target-word loads, and its gradient operands queued behind the Adam
// state).  Clamped to a valid element; the callers use only the valid lanes' values.
__device__ __forceinline__ uint4 target_words_ahead(const LearnArgs& a, int t) {
  const uint32_t* af = a.n_attr > 0 ? a.att_first : reinterpret_cast<const uint32_t*>(a.P);   // (no attractors: unused)
  const uint32_t* row = af + (size_t)(t < a.n_attr ? t : (a.n_attr > 0 ? a.n_attr - 1 : 0)) * a.W;
  return make_uint4(row[0], row[a.W > 1 ? 1 : 0], row[a.W > 2 ? 2 : 0], row[a.W > 3 ? 3 : 0]);
}
__device__ __forceinline__ AdamIn adam_load_ahead(const LearnArgs& a, int64_t i) {
  return AdamIn{a.P[i], a.m[i], a.v[i]};
}

struct Dense {
  const float* dY;
  const float* X;
  int64_t w_off, b_off;
  int ldw, o_valid, k_tiles;
  int lay, ot0;   // the layer's tiles in the image; its first output tile there (head h: h Apad/16)
};

template <int NT>
__global__ void __launch_bounds__(64 * kApplyWaves) learn_apply_kernel(LearnArgs a) {
  __shared__ float wsc[kApplyWaves][16][kMaxNT * 16 + 1];   // a bilinear tile's new weights, per wave
  if (a.adv_on && blockIdx.x == gridDim.x - 1) {   // the frame's counters and the next frame's rows
    const pbn_frame_advance& f = a.adv;             // (this launch reads neither; the earlier ones
    pbn::frame_advance_block(f.n_store, f.capacity, f.d_pos, f.d_size, f.d_step, f.d_eps64, f.d_eps32,   // of
                             f.eps_final, f.eps_step, f.n_idx, f.seed, f.d_counter, f.d_idx, f.n_store);   // the
    return;                                                                                              // call
  }                                                                                                      // did)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, rr = lane & 15;
  const int B = a.B;
  PBN_LSTAMP(2, 31);
  PBN_LSTAMP(2, 0);
  if (blockIdx.x == 0 && wave == 0) {   // the loss: the backward blocks' partial sums, a fixed-order reduction
    float s = 0.f;
    for (int p = lane; p < B / kRows; p += 64) s += a.partial[p];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
    if (lane == 0) a.loss[0] = s / (float)(B * a.K);
  }
  const float stepc = a.step[0];
  const float bc1 = 1.f - powf(a.b1, stepc);
  const float bc2s = sqrtf(1.f - powf(a.b2, stepc));
  int task = blockIdx.x * kApplyWaves + wave;
  const int n_bil = 16 * a.N;
  if (task < n_bil) {
    // bilinear weight tile: outputs o0..o0+15 of input i, all j: D[o][j] = sum_r g1[o][r] s_i[r] t_j[r]
    const int ot = task / a.N, i = task - ot * a.N, o0 = 16 * ot;
    const int64_t NN = (int64_t)a.N * a.N;
    const uint32_t* si = a.srow + (size_t)(i >> 5) * B;
    const float* grow = a.g1 + (size_t)(o0 + rr) * B;
    f32x4 acc[NT];
#pragma unroll
    for (int jt = 0; jt < NT; ++jt) acc[jt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bsum = 0.f;
    constexpr int RC = NT <= 2 ? 8 : 4;   // 16-row steps per round of loads
    const uint32_t sh = i & 31;
    float4 y[RC];
    uint4 sv[RC], tv[RC][NT];
    auto round_loads = [&](int r0) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < RC; ++u) {
        const int rb = min(r0 + 16 * u, B - 16) + 4 * g;
        y[u] = *reinterpret_cast<const float4*>(grow + rb);
        sv[u] = *reinterpret_cast<const uint4*>(si + rb);
#pragma unroll
        for (int jt = 0; jt < NT; ++jt)
          tv[u][jt] = *reinterpret_cast<const uint4*>(a.trow + (size_t)((16 * jt + rr) >> 5) * B + rb);
      }
    };
    // the first round's gradient operands, then the tile's Adam state and the first four target
    // rows' words of this lane (t = g + 4u) behind them (used after the loop), then the rounds
    round_loads(0);
    __builtin_amdgcn_sched_barrier(0);
    AdamIn pre[NT][4];
#pragma unroll
    for (int jt = 0; jt < NT; ++jt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int jj = min(16 * jt + rr, a.N - 1);   // (lanes past N: never applied)
        pre[jt][v] = adam_load_ahead(a, a.off[BIL_W] + (o0 + 4 * g + v) * NN + (int64_t)i * a.N + jj);
      }
    const AdamIn preb = adam_load_ahead(a, a.off[BIL_B] + o0 + rr);   // (applied by i == 0, g == 0)
    const uint4 tw0 = target_words_ahead(a, rr);   // target rr's words: the first table tile (t < n_attr)
    __builtin_amdgcn_sched_barrier(0);
    for (int r0 = 0; r0 < B; r0 += 16 * RC) {
      if (r0 > 0) round_loads(r0);
#pragma unroll
      for (int u = 0; u < RC; ++u) {
        if (r0 + 16 * u < B) {
          float4 yy = y[u];
          bsum += (yy.x + yy.y) + (yy.z + yy.w);
          yy.x = (sv[u].x >> sh) & 1u ? yy.x : 0.f;
          yy.y = (sv[u].y >> sh) & 1u ? yy.y : 0.f;
          yy.z = (sv[u].z >> sh) & 1u ? yy.z : 0.f;
          yy.w = (sv[u].w >> sh) & 1u ? yy.w : 0.f;
#pragma unroll
          for (int jt = 0; jt < NT; ++jt) {
            const uint32_t tsh = (16 * jt + rr) & 31;
            acc[jt] = mfma(yy.x, (float)((tv[u][jt].x >> tsh) & 1u), acc[jt]);
            acc[jt] = mfma(yy.y, (float)((tv[u][jt].y >> tsh) & 1u), acc[jt]);
            acc[jt] = mfma(yy.z, (float)((tv[u][jt].z >> tsh) & 1u), acc[jt]);
            acc[jt] = mfma(yy.w, (float)((tv[u][jt].w >> tsh) & 1u), acc[jt]);
          }
        }
      }
    }
    PBN_LSTAMP(2, 1);
#pragma unroll
    for (int jt = 0; jt < NT; ++jt) {
      const int jj = 16 * jt + rr;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int o = o0 + 4 * g + v;
        float nw = 0.f;
        if (jj < a.N) nw = adam_apply(a, a.off[BIL_W] + o * NN + (int64_t)i * a.N + jj, pre[jt][v], acc[jt][v], bc1, bc2s);
        wsc[wave][4 * g + v][jj] = nw;
      }
    }
    if (i == 0) {   // the bilinear bias: sum over the batch of g1 (lane groups added in a fixed order)
      bsum += __shfl_xor(bsum, 16);
      bsum += __shfl_xor(bsum, 32);
      if (g == 0) adam_apply(a, a.off[BIL_B] + o0 + rr, preb, bsum, bc1, bc2s);
    }
    PBN_LSTAMP(2, 2);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the target-table rows of input i for these 16 outputs, from the weights just written, 16
    // targets per MFMA tile: D[o][t] = sum_j W[o][i][j] x_t[j], j ascending through the k-steps
    // (the f32 MFMA is an fmaf chain, and x_t[j] is 0 or 1: pack_kernel's sequential sums bit for
    // bit).  A operand lane (g, r): W[o = r][j = s + g] from this wave's LDS rows; B: x_{t0 + r}[s + g]
    for (int t0 = 0; t0 < a.n_attr; t0 += 16) {
      const int t = t0 + rr;
      const uint4 tw = t0 == 0 ? tw0 : target_words(a, t);
      f32x4 d = {0.f, 0.f, 0.f, 0.f};
      for (int s4 = 0; s4 < a.N; s4 += 4) {
        const int j = s4 + g;
        const uint32_t word = (j >> 5) == 0 ? tw.x : (j >> 5) == 1 ? tw.y : (j >> 5) == 2 ? tw.z : tw.w;
        const bool in = j < a.N;
        d = mfma(in ? wsc[wave][rr][j] : 0.f, (in && t < a.n_attr && ((word >> (j & 31)) & 1u)) ? 1.f : 0.f, d);
      }
      if (t < a.n_attr) {
#pragma unroll
        for (int v = 0; v < 4; ++v) a.Tq[((size_t)t * a.N + i) * 256 + (4 * g + v) * 16 + ot] = d[v];
      }
    }
    PBN_LSTAMP(2, 3);
    return;
  }
  task -= n_bil;
  // dense layers: (layer, output tile, input tile) -> dW[o][k] = sum_r dY[o][r] X[k][r]
  const int H = a.H, at16 = a.Apad / 16;
  Dense L;
  int ot, kt;
  const int n0 = (kD1 / 16) * (kD0 / 16), n1 = (kD2 / 16) * (kD1 / 16), n2 = (kD3 / 16) * (kD2 / 16),
            n3 = (H * kDH / 16) * (kD3 / 16), n4 = H * at16 * (kDH / 16);
  if (task < n0) {
    L = Dense{a.dh2, a.y1, a.off[L2_W], a.off[L2_B], kD0, kD1, kD0 / 16, LY2, 0};
  } else if ((task -= n0) < n1) {
    L = Dense{a.dh3, a.h2, a.off[L3_W], a.off[L3_B], kD1, kD2, kD1 / 16, LY3, 0};
  } else if ((task -= n1) < n2) {
    L = Dense{a.dh4, a.h3, a.off[L4_W], a.off[L4_B], kD2, kD3, kD2 / 16, LY4, 0};
  } else if ((task -= n2) < n3) {
    L = Dense{a.dhh, a.h4, a.off[H1_W], a.off[H1_B], kD3, H * kDH, kD3 / 16, LYH1, 0};
  } else if ((task -= n3) < n4) {
    const int per = at16 * (kDH / 16);
    const int h = task / per;
    task -= h * per;
    // head h's second layer: rows are its A outputs (the value head has one real output)
    L = Dense{a.dheads + (size_t)h * a.Apad * B, a.hh + (size_t)h * kDH * B, a.off[H2_W] + (int64_t)h * a.A * kDH,
              a.off[H2_B] + (int64_t)h * a.A, kDH, h == 0 ? 1 : a.A, kDH / 16, LYH2, h * at16};
  } else {
    return;
  }
  ot = task / L.k_tiles;
  kt = task - ot * L.k_tiles;
  const int o0 = 16 * ot, k0 = 16 * kt;
  const float* yrow = L.dY + (size_t)(o0 + rr) * B;
  const float* xrow = L.X + (size_t)(k0 + rr) * B;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  float4 y[8], x[8];
  auto round_loads = [&](int r0) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int rb = min(r0 + 16 * u, B - 16) + 4 * g;
      y[u] = *reinterpret_cast<const float4*>(yrow + rb);
      x[u] = *reinterpret_cast<const float4*>(xrow + rb);
    }
  };
  round_loads(0);   // then the Adam state behind the first round's operands (the bilinear tiles' order)
  __builtin_amdgcn_sched_barrier(0);
  AdamIn pre[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int o = o0 + 4 * g + v;
    pre[v] = adam_load_ahead(a, L.w_off + (int64_t)(o < L.o_valid ? o : 0) * L.ldw + k0 + rr);   // (o < o_valid only)
  }
  const AdamIn preb = adam_load_ahead(a, L.b_off + (o0 + rr < L.o_valid ? o0 + rr : 0));   // (kt, g == 0, valid rows)
  __builtin_amdgcn_sched_barrier(0);
  for (int r0 = 0; r0 < B; r0 += 128) {   // eight 16-row steps per round of loads
    if (r0 > 0) round_loads(r0);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (r0 + 16 * u < B) {
        bsum += (y[u].x + y[u].y) + (y[u].z + y[u].w);
        acc = mfma(y[u].x, x[u].x, acc);
        acc = mfma(y[u].y, x[u].y, acc);
        acc = mfma(y[u].z, x[u].z, acc);
        acc = mfma(y[u].w, x[u].w, acc);
      }
    }
  }
  PBN_LSTAMP(2, 4);
  float nw[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int o = o0 + 4 * g + v;
    nw[v] = o < L.o_valid ? adam_apply(a, L.w_off + (int64_t)o * L.ldw + k0 + rr, pre[v], acc[v], bc1, bc2s) : 0.f;
  }
  {   // the tile's new weights into the online image (the learn_fwd / learn_bwd operands of the
      // next update and pbn_bdq_pack's values; rows past o_valid: the flat buffer's zero padding)
    const size_t tix = ((size_t)(L.ot0 + ot) * L.k_tiles + kt) * 64 + lane;
    reinterpret_cast<float4*>(a.Tq + a.ibw[L.lay])[tix] = make_float4(nw[0], nw[1], nw[2], nw[3]);
    float* sc = &wsc[wave][0][0];   // the fwd order is the tile transposed: through this wave's LDS
#pragma unroll
    for (int v = 0; v < 4; ++v) sc[(4 * g + v) * 17 + rr] = nw[v];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    reinterpret_cast<float4*>(a.Tq + a.ifw[L.lay])[tix] =
        make_float4(sc[rr * 17 + 4 * g], sc[rr * 17 + 4 * g + 1], sc[rr * 17 + 4 * g + 2], sc[rr * 17 + 4 * g + 3]);
  }
  if (kt == 0) {
    bsum += __shfl_xor(bsum, 16);
    bsum += __shfl_xor(bsum, 32);
    if (g == 0 && o0 + rr < L.o_valid) adam_apply(a, L.b_off + o0 + rr, preb, bsum, bc1, bc2s);
  }
  PBN_LSTAMP(2, 5);
}

// the target table of the bilinear layer, [t][i][j][q] = T[t][i][16 q + j] (the layout the
// acting kernel reads); block (t, i), thread o
__global__ void __launch_bounds__(256) pack_kernel(const float* __restrict__ P, int64_t w_off, int N, int W,
                                                   const uint32_t* __restrict__ att_first, float* __restrict__ Tq) {
  const int t = blockIdx.x / N, i = blockIdx.x - t * N, o = threadIdx.x;
  const uint32_t* ts = att_first + (size_t)t * W;
  const float* wrow = P + w_off + (int64_t)o * N * N + (int64_t)i * N;
  float s = 0.f;
  for (int j = 0; j < N; ++j) {
    const bool on = (ts[j >> 5] >> (j & 31)) & 1u;
    s += on ? wrow[j] : 0.f;
  }
  Tq[((size_t)t * N + i) * 256 + (o & 15) * 16 + (o >> 4)] = s;
}

// the weight tiles of one network's image from its flat parameters (make_image's layout): thread =
// one lane's float4 of one tile of one order
__global__ void __launch_bounds__(256) pack_tiles_kernel(const float* __restrict__ P, LearnArgs a, int64_t n4) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n4) return;
  // (layer, order, tile, lane) from the flat float4 index over the tiles region
  int64_t r = e;
  int l = 0, bwd = 0;
  int64_t per = 0;
  for (l = 0; l < NLAY; ++l) {
    const int R = l == LY2 ? kD1 : l == LY3 ? kD2 : l == LY4 ? kD3 : l == LYH1 ? a.H * kDH : a.H * a.Apad;
    const int C = l == LY2 ? kD0 : l == LY3 ? kD1 : l == LY4 ? kD2 : l == LYH1 ? kD3 : kDH;
    per = (int64_t)R * C / 4;   // float4s of one order of this layer
    if (r < 2 * per) break;
    r -= 2 * per;
  }
  bwd = r >= per;
  if (bwd) r -= per;
  const int C = l == LY2 ? kD0 : l == LY3 ? kD1 : l == LY4 ? kD2 : l == LYH1 ? kD3 : kDH;
  const int64_t tile = r >> 6;
  const int lane = (int)(r & 63), g = lane >> 4, rr = lane & 15;
  const int ot = (int)(tile / (C / 16)), kt = (int)(tile - (int64_t)ot * (C / 16));
  float x[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int row = bwd ? 16 * ot + 4 * g + v : 16 * ot + rr;
    const int col = bwd ? 16 * kt + rr : 16 * kt + 4 * g + v;
    float val;
    if (l == LYH2) {
      const int h = row / a.Apad, o = row - h * a.Apad;
      val = o < a.A ? P[a.off[H2_W] + ((int64_t)h * a.A + o) * kDH + col] : 0.f;
    } else {
      const int64_t w_off = l == LY2 ? a.off[L2_W] : l == LY3 ? a.off[L3_W] : l == LY4 ? a.off[L4_W] : a.off[H1_W];
      val = P[w_off + (int64_t)row * C + col];
    }
    x[v] = val;
  }
  reinterpret_cast<float4*>(a.Tq + (bwd ? a.ibw[l] : a.ifw[l]))[tile * 64 + lane] = make_float4(x[0], x[1], x[2], x[3]);
}

struct Work {
  int64_t heads, y1, h2, h3, h4, hh, dheads, dhh, dh4, dh3, dh2, g1, srow, trow, partial, total;   // float offsets
};

Work make_work(int N, int H, int64_t B) {
  const int A = N + 1, Ap = 16 * ((A + 15) / 16), W = (N + 31) / 32;
  Work w;
  int64_t o = 0;
  auto take = [&](int64_t n) { const int64_t at = o; o += al16(n); return at; };
  w.heads = take(3LL * H * Ap * B);
  w.y1 = take(kD0 * B);
  w.h2 = take(kD1 * B);
  w.h3 = take(kD2 * B);
  w.h4 = take(kD3 * B);
  w.hh = take((int64_t)H * kDH * B);
  w.dheads = take((int64_t)H * Ap * B);
  w.dhh = take((int64_t)H * kDH * B);
  w.dh4 = take(kD3 * B);
  w.dh3 = take(kD2 * B);
  w.dh2 = take(kD1 * B);
  w.g1 = take(kD0 * B);
  w.srow = take((int64_t)W * B);
  w.trow = take((int64_t)W * B);
  w.partial = take(B / kRows);
  w.total = o;
  return w;
}

#ifdef PBN_STAMPS
unsigned long long* g_lstamps = nullptr;   // pbn_debug_set_learn_stamps
#endif

// learn_bwd's LDS: the delta planes and the split tiles, or the TD pass's staged head rows (the
// same space), then the per-(row, branch) TD values
size_t learn_bwd_lds(int H, int Apad, int K) {
  const size_t planes = (size_t)(H * Apad + H * kDH + kD3 + kD2 + kD1) * kRows + kWaves * 64 * 4;
  const size_t staged = (size_t)3 * H * kRows * (Apad + 4);
  return (std::max(planes, staged) + 3 * kRows * K) * sizeof(float);
}

int check_shape(int N, int n_branches) {
  if (N < 1 || N > 127) return pbn::set_error(PBN_EINVAL, "fused BDQ update: 1 <= n_nodes <= 127");
  if (n_branches < 1 || n_branches > 7) return pbn::set_error(PBN_EINVAL, "fused BDQ update: n_branches 1..7");
  return PBN_OK;
}

}  // namespace

extern "C" {

#ifdef PBN_STAMPS
// diagnostic builds: the learner kernels' phase clocks go to d_buf (uint64 [3][1024][8][32]), or
// nowhere when null
int pbn_debug_set_learn_stamps(unsigned long long* d_buf) {
  g_lstamps = d_buf;
  return PBN_OK;
}
#endif

int pbn_bdq_layout(int32_t n_nodes, int32_t n_branches, int64_t* offsets) {
  int rc = check_shape(n_nodes, n_branches);
  if (rc) return rc;
  if (!offsets) return pbn::set_error(PBN_EINVAL, "null offsets");
  make_layout(n_nodes, n_branches + 1, offsets);
  return PBN_OK;
}

int pbn_bdq_learn_workspace(int32_t n_nodes, int32_t n_branches, int64_t batch, int64_t* bytes) {
  int rc = check_shape(n_nodes, n_branches);
  if (rc) return rc;
  if (!bytes) return pbn::set_error(PBN_EINVAL, "null bytes");
  if (batch < kRows || batch % kRows || batch > (1 << 20))
    return pbn::set_error(PBN_EINVAL, "fused BDQ update: batch a multiple of 16, 16..2^20");
  if (learn_bwd_lds(n_branches + 1, 16 * ((n_nodes + 16) / 16), n_branches) > 160 * 1024)
    return pbn::set_error(PBN_EINVAL, "fused BDQ update: (n_branches + 1) x (n_nodes + 1) too large for one block's LDS");
  *bytes = make_work(n_nodes, n_branches + 1, batch).total * (int64_t)sizeof(float);
  return PBN_OK;
}

int pbn_bdq_image_floats(const pbn_net* net, int32_t n_branches, int64_t* floats) {
  pbn::NetView v;
  int rc = pbn::net_view(net, &v);
  if (rc) return rc;
  if ((rc = check_shape(v.n_nodes, n_branches))) return rc;
  if (!floats) return pbn::set_error(PBN_EINVAL, "null floats");
  ImageLayout im;
  make_image(v.n_nodes, n_branches + 1, v.n_attr, &im);
  *floats = im.total;
  return PBN_OK;
}

int pbn_bdq_pack(const pbn_net* net, int32_t n_branches, const float* d_params, float* d_Tq, void* stream) {
  pbn::NetView v;
  int rc = pbn::net_view(net, &v);
  if (rc) return rc;
  if ((rc = pbn::check_device(net))) return rc;
  if ((rc = check_shape(v.n_nodes, n_branches))) return rc;
  if (!d_params || !d_Tq) return pbn::set_error(PBN_EINVAL, "null buffer");
  if (((uintptr_t)d_params | (uintptr_t)d_Tq) & 15u) return pbn::set_error(PBN_EINVAL, "buffers: 16-byte aligned");
  const int N = v.n_nodes, H = n_branches + 1;
  LearnArgs a;
  memset(&a, 0, sizeof a);
  a.N = N;
  a.H = H;
  a.A = N + 1;
  a.Apad = 16 * ((N + 16) / 16);
  make_layout(N, H, a.off);
  ImageLayout im;
  make_image(N, H, v.n_attr, &im);
  for (int l = 0; l < NLAY; ++l) {
    a.ifw[l] = im.fwd[l];
    a.ibw[l] = im.bwd[l];
  }
  a.Tq = d_Tq;
  const hipStream_t s = (hipStream_t)stream;
  if (v.n_attr > 0) {
    hipLaunchKernelGGL(pack_kernel, dim3(v.n_attr * N), dim3(256), 0, s, d_params, a.off[BIL_W], N, v.W, v.att_first,
                       d_Tq);
    if (hipGetLastError() != hipSuccess) return pbn::set_error(PBN_EDEVICE, "pack_kernel launch failed");
  }
  const int64_t n4 = (im.total - im.fwd[0]) / 4;
  hipLaunchKernelGGL(pack_tiles_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, d_params, a, n4);
  if (hipGetLastError() != hipSuccess) return pbn::set_error(PBN_EDEVICE, "pack_tiles_kernel launch failed");
  return PBN_OK;
}

int pbn_bdq_learn(const pbn_net* net, int64_t batch, const int64_t* d_idx, int64_t capacity, const uint32_t* d_state,
                  const uint32_t* d_next_state, const uint8_t* d_target, const int32_t* d_action, int32_t n_branches,
                  const float* d_reward, const uint8_t* d_done, float* d_params, float* d_Tq,
                  const float* d_target_params, const float* d_target_Tq, float* d_adam_m, float* d_adam_v,
                  float* d_adam_step, float lr, float beta1, float beta2, float eps, float gamma, float grad_clamp,
                  float slope, void* d_workspace, int64_t workspace_bytes, float* d_loss, float* d_grad,
                  const pbn_frame_advance* advance, void* stream) {
  pbn::NetView nv;
  int rc = pbn::net_view(net, &nv);
  if (rc) return rc;
  if ((rc = pbn::check_device(net))) return rc;
  const int N = nv.n_nodes;
  if ((rc = check_shape(N, n_branches))) return rc;
  int64_t need = 0;
  if ((rc = pbn_bdq_learn_workspace(N, n_branches, batch, &need))) return rc;
  if (capacity < 1) return pbn::set_error(PBN_EINVAL, "capacity >= 1");
  if (workspace_bytes < need) return pbn::set_error(PBN_EINVAL, "workspace too small (pbn_bdq_learn_workspace)");
  if (!d_idx || !d_state || !d_next_state || !d_target || !d_action || !d_reward || !d_done || !d_params ||
      !d_target_params || !d_adam_m || !d_adam_v || !d_adam_step || !d_workspace || !d_loss)
    return pbn::set_error(PBN_EINVAL, "null buffer");
  if (!d_Tq || !d_target_Tq) return pbn::set_error(PBN_EINVAL, "null network image");
  for (const void* p : {(const void*)d_params, (const void*)d_target_params, (const void*)d_adam_m,
                        (const void*)d_adam_v, (const void*)d_workspace, (const void*)d_Tq, (const void*)d_target_Tq})
    if ((uintptr_t)p & 15u) return pbn::set_error(PBN_EINVAL, "parameter, table and workspace buffers: 16-byte aligned");
  const int H = n_branches + 1, A = N + 1;
  LearnArgs a;
  a.idx = d_idx;
  a.B = (int)batch;
  a.cap = capacity;
  a.st = d_state;
  a.nst = d_next_state;
  a.tgt = d_target;
  a.act = d_action;
  a.rew = d_reward;
  a.done = d_done;
  a.att_first = nv.att_first;
  a.n_attr = nv.n_attr;
  a.N = N;
  a.W = nv.W;
  a.K = n_branches;
  a.H = H;
  a.A = A;
  a.Apad = 16 * ((A + 15) / 16);
  a.P = d_params;
  a.Tq = d_Tq;
  a.PT = d_target_params;
  a.TqT = d_target_Tq;
  a.m = d_adam_m;
  a.v = d_adam_v;
  a.step = d_adam_step;
  make_layout(N, H, a.off);
  ImageLayout im;
  make_image(N, H, nv.n_attr, &im);
  for (int l = 0; l < NLAY; ++l) {
    a.ifw[l] = im.fwd[l];
    a.ibw[l] = im.bwd[l];
  }
  a.lr = lr;
  a.b1 = beta1;
  a.b2 = beta2;
  a.eps = eps;
  a.gamma = gamma;
  a.clampv = grad_clamp;
  a.slope = slope;
  const Work w = make_work(N, H, batch);
  float* ws = static_cast<float*>(d_workspace);
  a.heads = ws + w.heads;
  a.y1 = ws + w.y1;
  a.h2 = ws + w.h2;
  a.h3 = ws + w.h3;
  a.h4 = ws + w.h4;
  a.hh = ws + w.hh;
  a.dheads = ws + w.dheads;
  a.dhh = ws + w.dhh;
  a.dh4 = ws + w.dh4;
  a.dh3 = ws + w.dh3;
  a.dh2 = ws + w.dh2;
  a.g1 = ws + w.g1;
  a.srow = reinterpret_cast<uint32_t*>(ws + w.srow);
  a.trow = reinterpret_cast<uint32_t*>(ws + w.trow);
  a.partial = ws + w.partial;
  a.loss = d_loss;
  a.grad = d_grad;
  a.stamps = nullptr;
#ifdef PBN_STAMPS
  a.stamps = g_lstamps;
#endif
  a.adv_on = 0;
  memset(&a.adv, 0, sizeof a.adv);
  if (advance) {
    const pbn_frame_advance& f = *advance;
    if (f.n_store < 0 || f.capacity < 1 || f.n_idx < 0 || !f.d_size || (f.n_store > 0 && !f.d_pos) ||
        (f.n_idx > 0 && (!f.d_counter || !f.d_idx)))
      return pbn::set_error(PBN_EINVAL, "pbn_frame_advance: n_store, n_idx >= 0, capacity >= 1, buffers");
    if (f.d_idx == d_idx && f.n_idx < batch)
      return pbn::set_error(PBN_EINVAL, "pbn_frame_advance: d_idx draws fewer rows than the batch");
    a.adv_on = 1;
    a.adv = f;
  }
  const hipStream_t s = (hipStream_t)stream;
  const int tiles = (int)(batch / kRows);
  const size_t lds_f = ((size_t)(kD0 + kD1 + kD2 + kD3 + kDH * H) * kRows + 4 * kRows + 2 * kRows) * sizeof(float) +
                       kRows * 128 + (size_t)(fwd_bias_floats(H, A) + 1) * sizeof(float);
  if (lds_f > 64 * 1024 && hipFuncSetAttribute((const void*)learn_fwd_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_f) != hipSuccess)
    return pbn::set_error(PBN_EDEVICE, "hipFuncSetAttribute failed");
  hipLaunchKernelGGL(learn_fwd_kernel, dim3(3 * tiles), dim3(kThreads), lds_f, s, a);
  if (hipGetLastError() != hipSuccess) return pbn::set_error(PBN_EDEVICE, "learn_fwd_kernel launch failed");
  const size_t lds_b = learn_bwd_lds(H, a.Apad, n_branches);
  if (lds_b > 64 * 1024 && hipFuncSetAttribute((const void*)learn_bwd_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_b) != hipSuccess)
    return pbn::set_error(PBN_EDEVICE, "hipFuncSetAttribute failed");
  hipLaunchKernelGGL(learn_bwd_kernel, dim3(tiles), dim3(kThreads), lds_b, s, a);
  if (hipGetLastError() != hipSuccess) return pbn::set_error(PBN_EDEVICE, "learn_bwd_kernel launch failed");
  const int ntasks = 16 * N + (kD1 / 16) * (kD0 / 16) + (kD2 / 16) * (kD1 / 16) + (kD3 / 16) * (kD2 / 16) +
                     (H * kDH / 16) * (kD3 / 16) + H * (a.Apad / 16) * (kDH / 16);
  const dim3 grid((ntasks + kApplyWaves - 1) / kApplyWaves + (a.adv_on ? 1 : 0)), blk(64 * kApplyWaves);
  switch ((N + 15) / 16) {
    case 1: hipLaunchKernelGGL(learn_apply_kernel<1>, grid, blk, 0, s, a); break;
    case 2: hipLaunchKernelGGL(learn_apply_kernel<2>, grid, blk, 0, s, a); break;
    case 3: hipLaunchKernelGGL(learn_apply_kernel<3>, grid, blk, 0, s, a); break;
    case 4: hipLaunchKernelGGL(learn_apply_kernel<4>, grid, blk, 0, s, a); break;
    case 5: hipLaunchKernelGGL(learn_apply_kernel<5>, grid, blk, 0, s, a); break;
    case 6: hipLaunchKernelGGL(learn_apply_kernel<6>, grid, blk, 0, s, a); break;
    case 7: hipLaunchKernelGGL(learn_apply_kernel<7>, grid, blk, 0, s, a); break;
    default: hipLaunchKernelGGL(learn_apply_kernel<8>, grid, blk, 0, s, a); break;
  }
  if (hipGetLastError() != hipSuccess) return pbn::set_error(PBN_EDEVICE, "learn_apply_kernel launch failed");
  return PBN_OK;
}

}  // extern "C"
