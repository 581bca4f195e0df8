// pbn_qnet.hip -- the layers of BranchingQNetwork after the bilinear one, fused into one MFMA
// kernel (config 5's acting frame).
//
// bdq_model/network.py:35-61: model = Bilinear(N, N, 256), LeakyReLU, Linear(256, 128),
// LeakyReLU, Linear(128, 64), LeakyReLU, Linear(64, 32), LeakyReLU; value head Linear(32, 64),
// LeakyReLU, Linear(64, 1); K advantage heads Linear(32, 64), LeakyReLU, Linear(64, A).  The
// bilinear layer (+ its LeakyReLU) comes from pbn_bilinear_targets; this kernel takes its
// output y (n, 256) and writes the raw head outputs (K+1, n, A) that pbn_heads_to_flipmask
// combines (dueling) and argmaxes -- in one launch where PyTorch spends four GEMMs and three
// elementwise launches.
//
// Layout: one wave per 16 envs, feature-major.  Every layer is out^T = W . in^T on
// v_mfma_f32_16x16x4_f32 (exact f32): the envs are the 16 MFMA columns (lane & 15), the output
// features the rows, so an accumulator tile of one layer is the B operand of the next with no
// data movement: register i of a 16-feature tile holds feature 4 g + i on lane group g = lane >> 4,
// and k-step (tile p, register i) of the next layer takes group g's element from there, i.e.
// inputs 16 p + 4 g + i.  The A operand (weights) is then W[out][16 p + 4 g + i] for i = 0..3:
// one float4 of the weight row per four MFMAs (from LDS: the weight stream below).  Sixteen envs
// per wave make 2,048 waves at config 5's 32,768 envs, two per SIMD: one wave's barriers, LDS
// reads and epilogue run under the other's MFMAs (with 32 envs per wave on the 32x32x2 form, one
// wave per SIMD, the kernel took 51 us against 28 us of MFMA issue).
// Biases initialise the accumulators; LeakyReLU (x > 0 ? x : x * slope, torch's form) is
// applied in registers between layers.  y is read in the same feature order (one float4 per lane
// per 16-feature tile).
#include <hip/hip_runtime.h>

#include <limits.h>
#include <stdint.h>

#include "../../include/pbn_env.h"
#include "net_view.h"
#include "philox.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kD0 = 256, kD1 = 128, kD2 = 64, kD3 = 32, kDH = 64;   // BranchingQNetwork widths
constexpr int kMaxHeads = 8;                                         // value + up to 7 branches
constexpr int kMaxActTiles = 4;                                      // A <= 128 (pbn70: 71), 32 per tile
constexpr int kEnvs = 16;                                            // envs per wave
constexpr int kWaves = 8;                                            // waves per block (128 envs)
static_assert(kWaves == 8, "stage loads: 512 threads = 64 rows x 8 float4 columns per pass");
constexpr int kBiasFloats = kD1 + kD2 + kD3 + (kDH + 32 * kMaxActTiles) * kMaxHeads;

struct QnetArgs {
  const float* y;                  // [n][256]
  const float *w1, *b1, *w2, *b2, *w3, *b3;
  const float *wh1, *bh1;          // [64 H][32], [64 H]
  const float *wh2, *bh2;          // [H][A][64], [H][A]
  float* heads;                    // [H][n][A] (FLIP = false)
  int64_t n;
  int n_heads, n_act;
  float slope;
  // FLIP = true: the acting epilogue of pbn_heads_to_flipmask in place of the head outputs
  uint64_t seed, step, env_offset, eps_u;
  const uint64_t* d_step;          // step index in device memory (graph replays), or null
  const float* d_eps;              // epsilon in device memory, or null
  uint32_t* flipmask;              // [W][n]
  int32_t* actions;                // [n][H - 1], or null
  int n_nodes, W;
  // BIL = true: the bilinear layer (+ LeakyReLU) computed here from the packed state, in place of y
  const uint32_t* state;           // [W][n]
  const uint8_t* target;           // [n]
  const float* T;                  // [n_attr][n_nodes][256]: the layer's weight contracted with each
                                   // attractor's first state (MyBilinear.target_table)
  const float* b0;                 // [256]
  int n_attr;
  unsigned long long* stamps;      // diagnostic builds (PBN_STAMPS): [block][wave][kQStampRow] s_memtime
};

// Diagnostic phase clocks (tools/qnet_stamps.py): lane 0 of every wave stores s_memtime at
// 0 entry, 1 after the block's target sort, 2 after the bilinear layer, 3 stage 0 in LDS, and for
// stage s at 4 + 3 s (its MFMA body starts), 5 + 3 s (body done), 6 + 3 s (past its barrier);
// inside the sort 57 keys stored, 58 past the barrier, 59 ranked, 60 past the barrier, 61 chunk
// prefixes, 62 key prefix
constexpr int kQStampRow = 64;
#ifdef PBN_STAMPS
#define PBN_QSTAMP(i)                                                                                       \
  do {                                                                                                    \
    if (a.stamps && (threadIdx.x & 63) == 0)                                                              \
      a.stamps[((size_t)blockIdx.x * kWaves + (threadIdx.x >> 6)) * kQStampRow + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define PBN_QSTAMP(i) do {} while (0)
#endif

constexpr int kPitch = 36;                   // weight row pitch in LDS (floats): conflict-free float4 reads
constexpr int kBufFloats = 5 * 64 * kPitch;  // one stage buffer: 320 rows (the largest stage, below)
constexpr int kMaxPieces = 5;

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// acc = bias of the output features 16 m + 4 g + i (0 past n_out; b in LDS)
__device__ __forceinline__ f32x4 bias_tile(const float* __restrict__ b, int m, int g, int n_out) {
  f32x4 acc;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int o = 16 * m + 4 * g + i;
    acc[i] = o < n_out ? b[o] : 0.f;
  }
  return acc;
}

__device__ __forceinline__ f32x4 leaky(f32x4 x, float slope) {
#pragma unroll
  for (int i = 0; i < 4; ++i) x[i] = x[i] > 0.f ? x[i] : x[i] * slope;
  return x;
}

// acc[m] += W[16 m .., chunk] . X over the 8 k-steps of one 32-column chunk (input tiles X0,
// X1), m < MT.  The A operand of tile p's k-steps is one float4 of weight row 16 m + (lane & 15)
// at column 16 p + 4 g; tile 1's float4s are read while tile 0's MFMAs run, and the MT
// accumulators interleave.
template <int MT>
__device__ __forceinline__ void mfma_chunk(f32x4 (&acc)[MT], const float* __restrict__ buf, int lane,
                                           const f32x4& X0, const f32x4& X1) {
  const float* r = buf + (lane & 15) * kPitch + 4 * (lane >> 4);
  float4 w[MT], wn[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) w[m] = *reinterpret_cast<const float4*>(r + 16 * m * kPitch);
#pragma unroll
  for (int m = 0; m < MT; ++m) wn[m] = *reinterpret_cast<const float4*>(r + 16 * m * kPitch + 16);
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = mfma(w[m].x, X0[0], acc[m]);
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = mfma(w[m].y, X0[1], acc[m]);
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = mfma(w[m].z, X0[2], acc[m]);
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = mfma(w[m].w, X0[3], acc[m]);
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = mfma(wn[m].x, X1[0], acc[m]);
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = mfma(wn[m].y, X1[1], acc[m]);
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = mfma(wn[m].z, X1[2], acc[m]);
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = mfma(wn[m].w, X1[3], acc[m]);
}

// The weights reach the MFMAs through LDS as a stream of STAGES, double-buffered: while the
// block's waves run one stage's MFMAs from one buffer, every thread holds the next stage's global
// loads in registers and stores them into the other buffer after the MFMAs; one block barrier per
// stage.  A stage is a few 32-column pieces of weight matrices (up to 320 rows), each row padded to
// 36 floats (the 16 rows one quarter-wave reads start on 16 distinct 4-bank groups):
//   stages 0-3   Linear(256, 128), 64 input columns each (two 128-row pieces)
//   stage 4      Linear(128, 64), all of it (four 64-row pieces)
//   stage 5      Linear(64, 32) (two 32-row pieces), and the first heads that fit beside it
//   then         the other heads, as many per stage as fit: per head Linear(32, 64) (64 rows) and
//                Linear(64, A) (two pieces of 32 AT rows, rows past A read as 0)
// Round 3 streamed 32-column chunks only (26 stages and barriers at Bittner-28); round 4 began with
// 13 stages, whose LDS stores, barrier and first LDS reads cost ≈ 1,300 cycles each
// (tools/qnet_stamps.py); Bittner-28 now runs 7.
// Stage kinds; row r of a stage occupies rows r of its buffer (float offset r * kPitch), so only
// the source of a row depends on the kind.
enum StageKind { kL1 = 0, kL2 = 1, kS9 = 2, kHead = 3 };
constexpr int kRows = kBufFloats / kPitch;   // rows per stage buffer (320)
constexpr int kL1Cols = 64;                  // layer-1 input columns per stage
constexpr int kL1Stages = kD0 / kL1Cols;

template <int AT>
struct StagePlan {
  static constexpr int kHeadRows = 64 + 64 * AT;        // Linear(32, 64), then Linear(64, A) as two
                                                        // pieces of 32 AT rows (32 input columns each)
  static constexpr int kHPS = kRows / kHeadRows;        // heads per head stage
  static constexpr int kS9Heads = (kRows - 64) / kHeadRows < kHPS ? (kRows - 64) / kHeadRows : kHPS;
  static constexpr int kS9Rows = 64 + kS9Heads * kHeadRows;
  static constexpr int kS9Passes = kS9Rows / 64;
  static constexpr int kHeadPasses = kHPS * kHeadRows / 64;
  static constexpr int kL2Stage = kL1Stages, kS9Stage = kL1Stages + 1, kFirstHeadStage = kL1Stages + 2;
  static_assert(kHPS >= 1 && kS9Rows % 64 == 0 && (kHPS * kHeadRows) % 64 == 0, "stage rows");
  static_assert(kS9Passes <= kMaxPieces && kHeadPasses <= kMaxPieces && 2 * 128 / 64 <= kMaxPieces, "passes");
};

// row r of head k's stage rows: its source and whether it is a row of the matrix (rows past A
// load row A - 1 and are stored as 0)
__device__ __forceinline__ const float* head_row(const QnetArgs& a, int k, int r, int at32, bool& real) {
  if (r < 64) {
    real = true;
    return a.wh1 + (size_t)kDH * kD3 * k + (size_t)r * kD3;
  }
  const int r2 = r - 64, j = r2 >= at32 ? 1 : 0, row = r2 - j * at32;
  real = row < a.n_act;
  return a.wh2 + (size_t)a.n_act * kDH * k + 32 * j + (size_t)min(row, a.n_act - 1) * kDH;
}

// row r of a stage of kind KIND (idx = the layer-1 stage, or the stage's first head); heads past
// the last (the last head stage's unused slots) read head H - 1's rows and are stored as 0
template <int AT, int KIND>
__device__ __forceinline__ const float* stage_row(const QnetArgs& a, int idx, int r, bool& real) {
  constexpr int HR = StagePlan<AT>::kHeadRows;
  if constexpr (KIND == kL1) {
    real = true;
    return a.w1 + kL1Cols * idx + 32 * (r >> 7) + (size_t)(r & 127) * kD0;
  } else if constexpr (KIND == kL2) {
    real = true;
    return a.w2 + 32 * (r >> 6) + (size_t)(r & 63) * kD1;
  } else if constexpr (KIND == kS9) {
    if (r < 64) {
      real = true;
      return a.w3 + 32 * (r >> 5) + (size_t)(r & 31) * kD2;
    }
    const int j = (r - 64) / HR;
    const float* p = head_row(a, min(j, a.n_heads - 1), r - 64 - j * HR, 32 * AT, real);
    real = real && j < a.n_heads;
    return p;
  } else {
    const int j = r / HR, k = idx + j;
    const float* p = head_row(a, min(k, a.n_heads - 1), r - j * HR, 32 * AT, real);
    real = real && k < a.n_heads;
    return p;
  }
}

// thread t's share of a stage: rows (t >> 3) + 64 j, columns 4 (t & 7) .. + 3 (PASSES x 64 rows)
template <int AT, int KIND, int PASSES>
__device__ __forceinline__ void fetch_stage(const QnetArgs& a, int idx, int t, f32x4 (&sv)[kMaxPieces]) {
  const int srow = t >> 3, scol = 4 * (t & 7);
#pragma unroll
  for (int j = 0; j < PASSES; ++j) {
    bool real;
    sv[j] = *reinterpret_cast<const f32x4*>(stage_row<AT, KIND>(a, idx, srow + 64 * j, real) + scol);
  }
}

template <int AT, int KIND, int PASSES>
__device__ __forceinline__ void put_stage(const QnetArgs& a, int idx, int t, float* buf, f32x4 (&sv)[kMaxPieces]) {
  const int srow = t >> 3, scol = 4 * (t & 7);
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};   // masked here, not at the load (a select on
                                           // the loaded value would wait for it)
#pragma unroll
  for (int j = 0; j < PASSES; ++j) {
    bool real;
    (void)stage_row<AT, KIND>(a, idx, srow + 64 * j, real);
    *reinterpret_cast<f32x4*>(buf + (srow + 64 * j) * kPitch + scol) = real ? sv[j] : z;
  }
}

// The dueling combination and argmax of one advantage head, as pbn_heads_to_flipmask computes
// them (pbn_agent.hip, q_to_flipmask_kernel): q_a = (v + adv_a) - mean, mean = the left-to-right
// float32 sum of adv_0 .. adv_{A-1} over A, torch.argmax's first maximum with NaN maximal.
// Action a = 16 m + 4 g + i of the env sits in register i of tile m on lane group g.  Branch-free
// over A: vm (this lane group's bit 4 m + i = action 16 m + 4 g + i < A) pads the actions past A
// with -0.0 for the sum (x + -0.0 == x for every x, so the walk over all 16 T16 entries is the
// walk over the first A) and with -inf for the argmax (below every number; a tie goes to the lower,
// real, index).
// The sum: every lane gathers its env's row from the four groups and walks it in order, through
// the wave's LDS scratch row block [16 envs][16 T16 actions] (SCR: T16 + 4 T16 LDS operations) or
// by __shfl (heads too wide for a scratch block).
// The argmax: each lane group walks its own actions in ascending order in registers, then the four
// groups' candidates meet in two xor butterflies.  The rule -- a NaN before any number, the lower
// index among NaNs, else the larger value, the lower index on a tie -- picks what the left-to-right
// walk picks and is associative, so the split is exact.
__device__ __forceinline__ float pad_if(uint32_t vm, int bit, float x, uint32_t pad) {
  const uint32_t mk = (uint32_t)__builtin_amdgcn_sbfe((int)vm, bit, 1);
  return __builtin_bit_cast(float, (__builtin_bit_cast(uint32_t, x) & mk) | (pad & ~mk));
}

template <int T16, int NB, bool SCR>
__device__ __forceinline__ void dueling_argmax(const f32x4 (&o)[NB][T16], int lane, int A, uint32_t vm, float v,
                                               float* scr, int (&act)[NB]) {
  // NB heads at once, head b innermost in every loop: their dependent chains (the sums, the
  // walks) interleave instead of running one after the other
  f32x4 op[NB][T16];   // -0.0 past A
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int m = 0; m < T16; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) op[b][m][i] = pad_if(vm, 4 * m + i, o[b][m][i], 0x80000000u);
  float row[NB][T16][4][4];   // [b][m][g][i]
  if constexpr (SCR) {
    // [b][16 envs][kScrPitch]: rows 16 T16 + 4 floats apart, so the 16 rows of a 16-byte access
    // start on 16 distinct 4-bank groups (a 16 T16-float pitch put them on one or two: 8-way conflicts)
    constexpr int P = 16 * T16 + 4;
    float* mine = scr + (lane & 15) * P;
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int m = 0; m < T16; ++m)
        *reinterpret_cast<f32x4*>(mine + b * 16 * P + 16 * m + 4 * (lane >> 4)) = op[b][m];
    __builtin_amdgcn_wave_barrier();   // one wave's LDS operations execute in order
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int m = 0; m < T16; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 q = *reinterpret_cast<const f32x4*>(mine + b * 16 * P + 16 * m + 4 * g);
#pragma unroll
          for (int i = 0; i < 4; ++i) row[b][m][g][i] = q[i];
        }
    __builtin_amdgcn_wave_barrier();   // (the next heads' writes follow these reads)
  } else {
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int m = 0; m < T16; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int i = 0; i < 4; ++i) row[b][m][g][i] = __shfl(op[b][m][i], (lane & 15) + 16 * g);
  }
  float sum[NB], mean[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) sum[b] = 0.f;
#pragma unroll
  for (int m = 0; m < T16; ++m)
#pragma unroll
    for (int f = 0; f < 16; ++f)
#pragma unroll
      for (int b = 0; b < NB; ++b) sum[b] += row[b][m][f >> 2][f & 3];
#pragma unroll
  for (int b = 0; b < NB; ++b) mean[b] = sum[b] / (float)A;
  const int g = lane >> 4;
  float best[NB];
  int bi[NB];
#pragma unroll
  for (int m = 0; m < T16; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const float qa = pad_if(vm, 4 * m + i, (v + o[b][m][i]) - mean[b], 0xFF800000u);   // -inf past A
        // (bitwise & and |: the short-circuit forms compile to exec-mask branches)
        const bool take = (m == 0 && i == 0) || ((!isnan(best[b])) & (isnan(qa) | (qa > best[b])));
        best[b] = take ? qa : best[b];
        bi[b] = take ? 16 * m + 4 * g + i : bi[b];
      }
#pragma unroll
  for (int x = 16; x <= 32; x <<= 1)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const float ob = __shfl_xor(best[b], x);
      const int oi = __shfl_xor(bi[b], x);
      const bool nm = isnan(best[b]), no = isnan(ob);
      const bool take = (nm & no) ? oi < bi[b]
                                  : (no ? true : (nm ? false : ((ob > best[b]) | ((ob == best[b]) & (oi < bi[b])))));
      best[b] = take ? ob : best[b];
      bi[b] = take ? oi : bi[b];
    }
#pragma unroll
  for (int b = 0; b < NB; ++b) act[b] = bi[b];
}

template <int AT, bool FLIP, bool BIL>   // AT: the second head layers' outputs in 32-row units, A <= 32 AT
__global__ void __launch_bounds__(64 * kWaves) qnet_tail_kernel(QnetArgs a) {
  constexpr int T16 = 2 * AT;   // 16-feature output tiles of the second head layers
  using Plan = StagePlan<AT>;
  __shared__ __attribute__((aligned(16))) float wbuf[2 * kBufFloats];
  // FLIP: per-wave scratch rows of the dueling epilogue (AT <= 2: 16 KB or 32 KB per block)
  // branch heads of stage S9 wait for the first head stage and are dueled with its heads
  constexpr int kPend = Plan::kS9Heads > 1 ? Plan::kS9Heads - 1 : 0;
  constexpr int kNB = kPend + Plan::kHPS;   // heads dueled together at most
  constexpr int kScrWave = kNB * 16 * (16 * T16 + 4);   // one wave's scratch rows (dueling_argmax)
  constexpr int kScr = (FLIP && AT <= 2) ? kWaves * kScrWave : 1;
  __shared__ __attribute__((aligned(16))) float escr[kScr];
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;
  const int A = a.n_act;
  const int H = a.n_heads;
  // heads kS9Heads + kHPS j .. in head stage kFirstHeadStage + j
  const int n_stages = Plan::kFirstHeadStage + (H - Plan::kS9Heads + Plan::kHPS - 1) / Plan::kHPS;
  PBN_QSTAMP(0);
  // this lane's env: the wave's 16 envs in order (y input), or (BIL) the wave's 16 of the block's
  // slice of its sort domain's envs stably sorted by target, so that a wave's envs share one target's
  // table (sometimes two)
  int64_t e;
  bool live;
  int key = 0;   // BIL: target id, n_attr = none, 255 = past the end
  if constexpr (!BIL) {
    const int64_t e0 = ((int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6)) * kEnvs;
    live = e0 < a.n;   // (a wave past the end still stages weights and meets the barriers)
    e = live ? e0 + (lane & 15) : 0;
  } else {
    // Sort domain: the kDom envs of kDom / 128 consecutive blocks.  Every block of a domain sorts
    // the domain's keys (stable counting sort) and takes its own 128-env slice of the order: a
    // target's run is then ~kDom / A envs long (73 at Bittner-28's 14 targets), so most waves hold
    // one target (1.2 bilinear passes per wave on average, against 2.75 when each block sorted its
    // own 128).  The sort's LDS is the second weight buffer's, first written by stage 1's loads.
    constexpr int kDom = 1024, kChunks = kDom / 64, kSlices = kDom / (kWaves * kEnvs);
    static_assert(kWaves * 64 * 2 == kDom, "two keys per thread");
    static_assert(kDom + 2 * kDom + 2 * kChunks * 256 + 2 * 256 <= 4 * kBufFloats, "sort LDS");
    uint8_t* const skey = reinterpret_cast<uint8_t*>(wbuf + kBufFloats);   // [kDom]
    uint16_t* const sperm = reinterpret_cast<uint16_t*>(skey + kDom);        // [kDom]
    uint16_t* const wcnt = sperm + kDom;     // [256][kChunks]: keys per 64-key chunk, then their prefix
    uint16_t* const kbase = wcnt + kChunks * 256;   // [256]: key totals, then keys below
    const int64_t d0 = (int64_t)(blockIdx.x / kSlices) * kDom;
    const int slice = (int)(blockIdx.x % kSlices);
    const int tt = threadIdx.x;
    const int wv = tt >> 6;
    for (int i = tt; i < kChunks * 128; i += 64 * kWaves) reinterpret_cast<uint32_t*>(wcnt)[i] = 0u;
    int kq[2], rank[2] = {0, 0};
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // keys tt and 512 + tt: chunks wv and kWaves + wv
      const int i = h * 64 * kWaves + tt;
      const bool lv = d0 + i < a.n;
      const uint32_t tg = lv ? (uint32_t)a.target[d0 + i] : 255u;
      kq[h] = lv ? (int)(tg < (uint32_t)a.n_attr ? tg : (uint32_t)a.n_attr) : 255;
      skey[i] = (uint8_t)kq[h];
    }
    PBN_QSTAMP(57);
    __syncthreads();
    PBN_QSTAMP(58);
    // rank among equal keys of the chunk and the chunk's counts: the lanes with an equal key are the
    // AND over the 8 key bits of ballot(bit) or its complement (8 ballots per key, where one ballot
    // per distinct key took a serial scalar loop: 4,500 cycles at 15 keys)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = kq[h], c = h * kWaves + wv;
      uint64_t eq = ~0ull;
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const bool bit = (k >> b) & 1;
        const uint64_t bl = __ballot(bit);
        eq &= bit ? bl : ~bl;
      }
      rank[h] = __builtin_popcountll(eq & ((1ull << lane) - 1ull));
      if ((eq & ~((2ull << lane) - 1ull)) == 0ull)   // the last lane of its key
        wcnt[k * kChunks + c] = (uint16_t)__builtin_popcountll(eq);
    }
    PBN_QSTAMP(59);
    __syncthreads();
    PBN_QSTAMP(60);
    if (tt < 256) {   // per key: exclusive prefix over the chunks, in place (its 16 counts are two
                      // 16-byte words); the key's total
      static_assert(kChunks == 16, "two uint4 of uint16 counts per key");
      uint4* const row = reinterpret_cast<uint4*>(wcnt + tt * kChunks);
      const uint4 q0 = row[0], q1 = row[1];
      const uint32_t in[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
      uint32_t outw[8];
      uint32_t run = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t lo = in[j] & 0xFFFFu, hi = in[j] >> 16;
        outw[j] = run | ((run + lo) << 16);
        run += lo + hi;
      }
      row[0] = make_uint4(outw[0], outw[1], outw[2], outw[3]);
      row[1] = make_uint4(outw[4], outw[5], outw[6], outw[7]);
      kbase[tt] = (uint16_t)run;
    }
    __syncthreads();
    PBN_QSTAMP(61);
    if (wv == 0) {   // exclusive prefix over the 256 keys: four per lane, then across lanes
      int c4[4], tot = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c4[j] = tot;
        tot += (int)kbase[4 * lane + j];
      }
      int inc = tot;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(inc, d);
        inc += lane >= d ? y : 0;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) kbase[4 * lane + j] = (uint16_t)(inc - tot + c4[j]);
    }
    __syncthreads();
    PBN_QSTAMP(62);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = kq[h], c = h * kWaves + wv;
      sperm[(int)kbase[k] + (int)wcnt[k * kChunks + c] + rank[h]] = (uint16_t)(h * 64 * kWaves + tt);
    }
    __syncthreads();
    PBN_QSTAMP(1);
    const int li = sperm[slice * kWaves * kEnvs + (threadIdx.x >> 6) * kEnvs + (lane & 15)];
    key = skey[li];
    live = key != 255;
    e = live ? d0 + li : 0;
  }

  const int t = threadIdx.x;
  f32x4 sv[kMaxPieces];   // the next stage's loads in flight
  // one stage step: the next stage's loads (kept above the MFMAs by the scheduling barriers: LLVM
  // would sink them to their LDS stores and expose their L2 round trip), this stage's MFMAs (BODY
  // reads `buf`; waves past the end compute on env 0 and store nothing), the next stage into the
  // other buffer (the waves left it at the previous barrier), barrier.  NEXT_PASSES = 0: the last
  // stage, nothing to fetch.
#define PBN_STAGE(s_, NEXT_KIND, NEXT_IDX, NEXT_PASSES, BODY)                                      \
  do {                                                                                             \
    const int ss_ = (s_);                                                                          \
    if constexpr ((NEXT_PASSES) > 0) fetch_stage<AT, (NEXT_KIND), (NEXT_PASSES)>(a, (NEXT_IDX), t, sv); \
    __builtin_amdgcn_sched_barrier(0);                                                             \
    PBN_QSTAMP(4 + 3 * ss_);                                                                       \
    const float* buf = wbuf + (ss_ & 1) * kBufFloats;                                              \
    BODY                                                                                           \
    __builtin_amdgcn_sched_barrier(0);                                                             \
    PBN_QSTAMP(5 + 3 * ss_);                                                                       \
    if constexpr ((NEXT_PASSES) > 0) {                                                             \
      put_stage<AT, (NEXT_KIND), (NEXT_PASSES)>(a, (NEXT_IDX), t, wbuf + ((ss_ + 1) & 1) * kBufFloats, sv); \
      __syncthreads();                                                                             \
    }                                                                                              \
    PBN_QSTAMP(6 + 3 * ss_);                                                                       \
  } while (0)

  // every bias, staged once in LDS (a per-head bias load from L2 sat in front of the head's
  // first MFMA): b1 | b2 | b3 | bh1 [64 H] | bh2 [H][A]
  __shared__ float bias[kBiasFloats];
  float* const bs1 = bias;
  float* const bs2 = bs1 + kD1;
  float* const bs3 = bs2 + kD2;
  float* const bsh1 = bs3 + kD3;
  float* const bsh2 = bsh1 + kDH * kMaxHeads;
  for (int i = t; i < kD1; i += 64 * kWaves) bs1[i] = a.b1[i];
  for (int i = t; i < kD2; i += 64 * kWaves) bs2[i] = a.b2[i];
  for (int i = t; i < kD3; i += 64 * kWaves) bs3[i] = a.b3[i];
  for (int i = t; i < kDH * H; i += 64 * kWaves) bsh1[i] = a.bh1[i];
  // bh2 as [H][32 AT], zero past A: the head's bias tiles read it with no per-element test
  for (int i = t; i < 32 * AT * H; i += 64 * kWaves) {
    const int kk = i / (32 * AT), aa = i - kk * 32 * AT;
    bsh2[i] = aa < A ? a.bh2[kk * A + aa] : 0.f;
  }

  fetch_stage<AT, kL1, 4>(a, 0, t, sv);
  put_stage<AT, kL1, 4>(a, 0, t, wbuf, sv);

  // ---- Linear(256, 128): input tiles from y, features 16 p + 4 g .. + 3 (one float4 per tile);
  // a stage is two tiles, whose loads fly one stage ahead
  f32x4 x1[kD1 / 16];
  if constexpr (!BIL) {
    const float* yrow = a.y + (size_t)e * kD0 + 4 * g;
    f32x4 yv[4], yn[4];   // a stage's four input tiles: columns 64 p + 16 j + 4 g .. + 3
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 u = *reinterpret_cast<const float4*>(yrow + 16 * j);
      yv[j] = f32x4{u.x, u.y, u.z, u.w};
    }
    __syncthreads();   // stage 0 and the biases are in LDS
#pragma unroll
    for (int m = 0; m < kD1 / 16; ++m) x1[m] = bias_tile(bs1, m, g, kD1);
#pragma unroll
    for (int p = 0; p < kL1Stages; ++p) {
      if (p + 1 < kL1Stages) {   // the next stage's y tiles fly under this stage's MFMAs
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 u = *reinterpret_cast<const float4*>(yrow + kL1Cols * (p + 1) + 16 * j);
          yn[j] = f32x4{u.x, u.y, u.z, u.w};
        }
      }
      if (p + 1 < kL1Stages)
        PBN_STAGE(p, kL1, p + 1, 4, { mfma_chunk<kD1 / 16>(x1, buf, lane, yv[0], yv[1]);
                                      mfma_chunk<kD1 / 16>(x1, buf + 128 * kPitch, lane, yv[2], yv[3]); });
      else
        PBN_STAGE(p, kL2, 0, 4, { mfma_chunk<kD1 / 16>(x1, buf, lane, yv[0], yv[1]);
                                  mfma_chunk<kD1 / 16>(x1, buf + 128 * kPitch, lane, yv[2], yv[3]); });
#pragma unroll
      for (int j = 0; j < 4; ++j) yv[j] = yn[j];
    }
  } else {
    // the bilinear layer of the wave's 16 envs, all 256 outputs, in registers: y^T = b0 +
    // sum over the targets a present of T[a]^T . S_a, S_a[i][j] = bit i of env j's state if env
    // j's target is a, else 0 (on v_mfma_f32_16x16x4_f32: k = node, A = T[a][node][out], B = the
    // 0/1 bits); then LeakyReLU.  Register tile q = outputs 16 q + 4 g + i: layer 1's B operand.
    const int N = a.n_nodes;
    uint32_t sw[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int w = 0; w < 4; ++w)
      if (w < a.W && live) sw[w] = a.state[(size_t)w * a.n + e];
    f32x4 yt[kD0 / 16];
#pragma unroll
    for (int q = 0; q < kD0 / 16; ++q) {
      const float4 b4 = *reinterpret_cast<const float4*>(a.b0 + 16 * q + 4 * g);
      yt[q] = f32x4{b4.x, b4.y, b4.z, b4.w};
    }
    const int klo = __shfl(key, 0), khi = __shfl(key, 15);   // the wave's keys are sorted
    const int kend = khi < a.n_attr ? khi : a.n_attr - 1;
    for (int ta = klo; ta <= kend; ++ta) {
      if (!__any(key == ta)) continue;
      // T in the from_state layout [a][node][j][q] = T[a][node][16 q + j]: lane j's 16 A operands
      // of a k-step (outputs 16 q + j, q = 0..15) are 64 contiguous bytes, four 16-byte loads
      const float* Ta = a.T + (size_t)ta * N * kD0 + 16 * (lane & 15);
      const bool mine = key == ta;
      // k-step s4: nodes s4 .. s4 + 3, this lane's s4 + g; the next step's 4 table loads are
      // issued before this step's 16 MFMAs (rows past N load row N - 1 and meet a 0 operand)
      f32x4 av[4], an[4];
      {
        const float* Tn = Ta + (size_t)min(g, N - 1) * kD0;
#pragma unroll
        for (int u = 0; u < 4; ++u) av[u] = *reinterpret_cast<const f32x4*>(Tn + 4 * u);
      }
      for (int s4 = 0; s4 < N; s4 += 4) {
        const float* Tn = Ta + (size_t)min(s4 + 4 + g, N - 1) * kD0;
#pragma unroll
        for (int u = 0; u < 4; ++u) an[u] = *reinterpret_cast<const f32x4*>(Tn + 4 * u);
        __builtin_amdgcn_sched_barrier(0);
        const int node = s4 + g;
        uint32_t wsel = sw[0];
#pragma unroll
        for (int w = 1; w < 4; ++w) wsel = (node >> 5) == w ? sw[w] : wsel;
        const float bv = (mine && node < N && ((wsel >> (node & 31)) & 1u)) ? 1.f : 0.f;
#pragma unroll
        for (int q = 0; q < kD0 / 16; ++q) yt[q] = mfma(av[q >> 2][q & 3], bv, yt[q]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 4; ++u) av[u] = an[u];
      }
    }
#pragma unroll
    for (int q = 0; q < kD0 / 16; ++q) yt[q] = leaky(yt[q], a.slope);
    PBN_QSTAMP(2);
    __syncthreads();   // stage 0 and the biases are in LDS
    PBN_QSTAMP(3);
#pragma unroll
    for (int m = 0; m < kD1 / 16; ++m) x1[m] = bias_tile(bs1, m, g, kD1);
#pragma unroll
    for (int p = 0; p < kL1Stages; ++p) {
      if (p + 1 < kL1Stages)
        PBN_STAGE(p, kL1, p + 1, 4, { mfma_chunk<kD1 / 16>(x1, buf, lane, yt[4 * p], yt[4 * p + 1]);
                                      mfma_chunk<kD1 / 16>(x1, buf + 128 * kPitch, lane, yt[4 * p + 2], yt[4 * p + 3]); });
      else
        PBN_STAGE(p, kL2, 0, 4, { mfma_chunk<kD1 / 16>(x1, buf, lane, yt[4 * p], yt[4 * p + 1]);
                                  mfma_chunk<kD1 / 16>(x1, buf + 128 * kPitch, lane, yt[4 * p + 2], yt[4 * p + 3]); });
    }
  }
#pragma unroll
  for (int m = 0; m < kD1 / 16; ++m) x1[m] = leaky(x1[m], a.slope);

  // ---- Linear(128, 64): stage 8, its four 64-row pieces of 32 input columns
  f32x4 x2[kD2 / 16];
#pragma unroll
  for (int m = 0; m < kD2 / 16; ++m) x2[m] = bias_tile(bs2, m, g, kD2);
  auto layer2 = [&](const float* buf) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < kD1 / 32; ++p) mfma_chunk<kD2 / 16>(x2, buf + p * 64 * kPitch, lane, x1[2 * p], x1[2 * p + 1]);
  };
  PBN_STAGE(Plan::kL2Stage, kS9, 0, Plan::kS9Passes, { layer2(buf); });
#pragma unroll
  for (int m = 0; m < kD2 / 16; ++m) x2[m] = leaky(x2[m], a.slope);

  // ---- heads: Linear(32, 64) + LeakyReLU per head (stacked rows 64 k .. 64 k + 63), then
  // Linear(64, A) of that head's 64 features; raw outputs to heads[k][e][a], or (FLIP) the
  // value, then each branch's action into the flip mask
  float v = 0.f;
  bool explore = false;
  pbn::Word4 r0{0u, 0u, 0u, 0u}, r1{0u, 0u, 0u, 0u};
  u32x4 mk = {0u, 0u, 0u, 0u};   // flip-mask words (a vector: no per-thread array in memory)
  uint32_t vm = 0;                // bit 4 m + i: this lane group's action 16 m + 4 g + i < A
#pragma unroll
  for (int m = 0; m < T16; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) vm |= (16 * m + 4 * g + i < A ? 1u : 0u) << (4 * m + i);
  if constexpr (FLIP) {   // the EXPLORE draws of env e (the four lane groups draw the same)
    const uint64_t ge = a.env_offset + (uint64_t)e;
    const uint64_t st = a.d_step ? *a.d_step : a.step;
    uint64_t eps_u = a.eps_u;
    if (a.d_eps) {   // device epsilon (graph replays): clamped to [0, 1], NaN -> 0
      const float ef = fminf(fmaxf(*a.d_eps, 0.f), 1.f);
      eps_u = (uint64_t)floor((double)ef * 4294967296.0);
    }
    r0 = pbn::draw(a.seed, ge, st, pbn::kStreamExplore, 0);
    if (H > 4) r1 = pbn::draw(a.seed, ge, st, pbn::kStreamExplore, 1);
    explore = (uint64_t)r0.x < eps_u;
  }
  // head k from its stage buffer: the Linear(32, 64) piece at h1, the Linear(64, A) pieces at h2
  // and h2 + 32 AT rows, into o (raw outputs)
  f32x4 x3[kD3 / 16];
  auto head = [&](int k, const float* h1, const float* h2, f32x4 (&o)[T16]) __attribute__((always_inline)) {
    f32x4 z[kDH / 16];
#pragma unroll
    for (int m = 0; m < kDH / 16; ++m) z[m] = bias_tile(bsh1 + kDH * k, m, g, kDH);
    mfma_chunk<kDH / 16>(z, h1, lane, x3[0], x3[1]);
#pragma unroll
    for (int m = 0; m < kDH / 16; ++m) z[m] = leaky(z[m], a.slope);
#pragma unroll
    for (int m = 0; m < T16; ++m) o[m] = bias_tile(bsh2 + 32 * AT * k, m, g, 32 * AT);
    mfma_chunk<T16>(o, h2, lane, z[0], z[1]);
    mfma_chunk<T16>(o, h2 + 32 * AT * kPitch, lane, z[2], z[3]);
  };
  // !FLIP: head k's raw outputs to heads[k][e][a]
  auto store_head = [&](int k, const f32x4 (&o)[T16]) __attribute__((always_inline)) {
    if (!live) return;
    float* out = a.heads + ((size_t)k * a.n + e) * A;
#pragma unroll
    for (int m = 0; m < T16; ++m) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int act = 16 * m + 4 * g + i;
        if (act < A) out[act] = o[m][i];
      }
    }
  };
  // FLIP: the actions of branch heads kk[b] (those >= H skipped) into the flip mask: epsilon-greedy,
  // EXPLORE word b + 1 across calls 0 and 1 onto [0, N] for an exploring env, else the dueling argmax
  auto act_heads = [&](auto nb_c, const f32x4 (&o)[decltype(nb_c)::value][T16], const int (&kk)[decltype(nb_c)::value])
      __attribute__((always_inline)) {
    constexpr int NB = decltype(nb_c)::value;
    uint32_t vmk = vm;
    asm volatile("" : "+v"(vmk));   // (hoisted, its selects were SGPR pairs that spilled)
    int act[NB];
    dueling_argmax<T16, NB, (AT <= 2)>(o, lane, A, vmk, v, (AT <= 2) ? escr + (threadIdx.x >> 6) * kScrWave : nullptr,
                                       act);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (kk[b] >= H) continue;
      const int br = kk[b] - 1;   // branch
      const uint32_t rw = br == 0 ? r0.y : br == 1 ? r0.z : br == 2 ? r0.w : br == 3 ? r1.x
                        : br == 4 ? r1.y : br == 5 ? r1.z : r1.w;
      const int ac = explore ? (int)__umulhi(rw, (uint32_t)(a.n_nodes + 1)) : act[b];
      if (ac > 0 && ac <= a.n_nodes) {   // a > 0 flips node a - 1, once however often
#pragma unroll
        for (int w = 0; w < 4; ++w)
          if (w == ((ac - 1) >> 5)) mk[w] |= 1u << ((ac - 1) & 31);
      }
      if (a.actions && live && g == 0) a.actions[e * (H - 1) + br] = ac;
    }
  };
  f32x4 pend[kPend > 0 ? kPend : 1][T16];   // FLIP: stage S9's branch heads, dueled later

  // ---- Linear(64, 32) (stage S9, with the heads that fit beside it)
#pragma unroll
  for (int m = 0; m < kD3 / 16; ++m) x3[m] = bias_tile(bs3, m, g, kD3);
  auto stage9 = [&](const float* buf, bool last) __attribute__((always_inline)) {
    mfma_chunk<kD3 / 16>(x3, buf, lane, x2[0], x2[1]);
    mfma_chunk<kD3 / 16>(x3, buf + 32 * kPitch, lane, x2[2], x2[3]);
#pragma unroll
    for (int m = 0; m < kD3 / 16; ++m) x3[m] = leaky(x3[m], a.slope);
#pragma unroll
    for (int j = 0; j < Plan::kS9Heads; ++j) {
      if (j >= H) continue;
      f32x4 o[T16];
      head(j, buf + (64 + j * Plan::kHeadRows) * kPitch, buf + (128 + j * Plan::kHeadRows) * kPitch, o);
      if constexpr (!FLIP) {
        store_head(j, o);
      } else if (j == 0) {
        v = __shfl(o[0][0], lane & 15);   // value head output 0: register 0 of lane group 0
      } else {
#pragma unroll
        for (int m = 0; m < T16; ++m) pend[j - 1][m] = o[m];
      }
    }
    if constexpr (FLIP && kPend > 0) {
      if (last) {   // no head stage follows
        int kk[kPend];
#pragma unroll
        for (int b = 0; b < kPend; ++b) kk[b] = 1 + b;
        act_heads(std::integral_constant<int, kPend>{}, pend, kk);
      }
    }
  };
  // the heads of one head stage (those past H, in the last stage's unused slots, are skipped);
  // FLIP: dueled together, with stage S9's pending heads in the first head stage
  auto heads = [&](int k0, const float* buf, bool first) __attribute__((always_inline)) {
    f32x4 oc[Plan::kHPS][T16];
#pragma unroll
    for (int j = 0; j < Plan::kHPS; ++j) {
      if (k0 + j < H) head(k0 + j, buf + j * Plan::kHeadRows * kPitch, buf + (64 + j * Plan::kHeadRows) * kPitch, oc[j]);
      if constexpr (!FLIP) {
        if (k0 + j < H) store_head(k0 + j, oc[j]);
      }
    }
    if constexpr (FLIP) {
      if (kPend > 0 && first) {
        f32x4 ob[kNB][T16];
        int kk[kNB];
#pragma unroll
        for (int b = 0; b < kNB; ++b) {
#pragma unroll
          for (int m = 0; m < T16; ++m) ob[b][m] = b < kPend ? pend[b < kPend ? b : 0][m] : oc[b < kPend ? 0 : b - kPend][m];
          kk[b] = b < kPend ? 1 + b : k0 + b - kPend;
        }
        act_heads(std::integral_constant<int, kNB>{}, ob, kk);
      } else {
        int kk[Plan::kHPS];
#pragma unroll
        for (int j = 0; j < Plan::kHPS; ++j) kk[j] = k0 + j;
        act_heads(std::integral_constant<int, Plan::kHPS>{}, oc, kk);
      }
    }
  };
  if (n_stages > Plan::kFirstHeadStage)
    PBN_STAGE(Plan::kS9Stage, kHead, Plan::kS9Heads, Plan::kHeadPasses, { stage9(buf, false); });
  else
    PBN_STAGE(Plan::kS9Stage, kHead, 0, 0, { stage9(buf, true); });
  for (int s = Plan::kFirstHeadStage; s < n_stages; ++s) {
    const int k0 = Plan::kS9Heads + (s - Plan::kFirstHeadStage) * Plan::kHPS;
    const bool first = s == Plan::kFirstHeadStage;
    if (s + 1 < n_stages) PBN_STAGE(s, kHead, k0 + Plan::kHPS, Plan::kHeadPasses, { heads(k0, buf, first); });
    else PBN_STAGE(s, kHead, 0, 0, { heads(k0, buf, first); });
  }
  if constexpr (FLIP) {
    if (live && g == 0) {
#pragma unroll
      for (int w = 0; w < 4; ++w)
        if (w < a.W) a.flipmask[(size_t)w * a.n + e] = mk[w];
    }
  }
#undef PBN_STAGE
}

bool al16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

int qnet_check(const pbn_net* net, int64_t n_envs, const float* d_y, const float* d_w1, const float* d_b1,
                      const float* d_w2, const float* d_b2, const float* d_w3, const float* d_b3, const float* d_wh1,
                      const float* d_bh1, const float* d_wh2, const float* d_bh2, int32_t n_heads, int32_t n_actions) {
  int rc = pbn::check_device(net);
  if (rc) return rc;
  if (n_envs < 0 || (n_envs & 31)) return pbn::set_error(PBN_EINVAL, "n_envs must be a non-negative multiple of 32");
  if (n_heads < 1 || n_heads > kMaxHeads) return pbn::set_error(PBN_EINVAL, "n_heads must be 1..8");
  if (n_actions < 1 || n_actions > 32 * kMaxActTiles) return pbn::set_error(PBN_EINVAL, "n_actions must be 1..128");
  if (n_envs == 0) return PBN_OK;
  if (!d_y || !d_w1 || !d_b1 || !d_w2 || !d_b2 || !d_w3 || !d_b3 || !d_wh1 || !d_bh1 || !d_wh2 || !d_bh2)
    return pbn::set_error(PBN_EINVAL, "null buffer");
  // float4 weight-row and y loads: rows of 256 / 128 / 64 / 32 floats start 16-byte aligned
  // when the base is; the second head layer's rows are 64 floats
  if (!al16(d_y) || !al16(d_w1) || !al16(d_w2) || !al16(d_w3) || !al16(d_wh1) || !al16(d_wh2))
    return pbn::set_error(PBN_EINVAL, "y and weight buffers must be 16-byte aligned");
  return PBN_OK;
}

#ifdef PBN_STAMPS
unsigned long long* g_qstamps = nullptr;   // pbn_debug_set_qnet_stamps
#endif

template <bool FLIP, bool BIL>
int qnet_launch(const QnetArgs& a_in, void* stream) {
  QnetArgs a = a_in;
#ifdef PBN_STAMPS
  a.stamps = g_qstamps;
#endif
  const int64_t waves = a.n / kEnvs;
  const unsigned blocks = (unsigned)((waves + kWaves - 1) / kWaves);
  void (*kernels[kMaxActTiles])(QnetArgs) = {qnet_tail_kernel<1, FLIP, BIL>, qnet_tail_kernel<2, FLIP, BIL>,
                                              qnet_tail_kernel<3, FLIP, BIL>, qnet_tail_kernel<4, FLIP, BIL>};
  hipLaunchKernelGGL(kernels[(a.n_act + 31) / 32 - 1], dim3(blocks), dim3(64 * kWaves), 0, (hipStream_t)stream, a);
  if (hipGetLastError() != hipSuccess) return pbn::set_error(PBN_EDEVICE, "qnet_tail_kernel launch failed");
  return PBN_OK;
}

// the bilinear layer's inputs of the _from_state forms; on success fills a's BIL fields
int bil_check(const pbn_net* net, const uint32_t* d_state, const uint8_t* d_target, const float* d_T,
              const float* d_b0, QnetArgs& a) {
  pbn::NetView v;
  int rc = pbn::net_view(net, &v);
  if (rc) return rc;
  if (!d_state || !d_target || !d_b0 || (v.n_attr > 0 && !d_T)) return pbn::set_error(PBN_EINVAL, "null buffer");
  if (!al16(d_b0) || !al16(d_T)) return pbn::set_error(PBN_EINVAL, "d_b0 and d_T must be 16-byte aligned");
  a.state = d_state; a.target = d_target; a.T = d_T; a.b0 = d_b0;
  a.n_attr = v.n_attr; a.n_nodes = v.n_nodes; a.W = v.W;
  return PBN_OK;
}

}  // namespace

extern "C" {

#ifdef PBN_STAMPS
int pbn_debug_set_qnet_stamps(unsigned long long* d_buf) {
  g_qstamps = d_buf;
  return 0;
}
#endif

int pbn_qnet_heads(const pbn_net* net, int64_t n_envs, const float* d_y, const float* d_w1, const float* d_b1,
                   const float* d_w2, const float* d_b2, const float* d_w3, const float* d_b3, const float* d_wh1,
                   const float* d_bh1, const float* d_wh2, const float* d_bh2, int32_t n_heads, int32_t n_actions,
                   float slope, float* d_heads, void* stream) {
  int rc = qnet_check(net, n_envs, d_y, d_w1, d_b1, d_w2, d_b2, d_w3, d_b3, d_wh1, d_bh1, d_wh2, d_bh2, n_heads,
                      n_actions);
  if (rc || n_envs == 0) return rc;
  if (!d_heads) return pbn::set_error(PBN_EINVAL, "null buffer");
  QnetArgs a{};
  a.y = d_y; a.w1 = d_w1; a.b1 = d_b1; a.w2 = d_w2; a.b2 = d_b2; a.w3 = d_w3; a.b3 = d_b3;
  a.wh1 = d_wh1; a.bh1 = d_bh1; a.wh2 = d_wh2; a.bh2 = d_bh2; a.heads = d_heads;
  a.n = n_envs; a.n_heads = n_heads; a.n_act = n_actions; a.slope = slope;
  return qnet_launch<false, false>(a, stream);
}

int pbn_qnet_flipmask(const pbn_net* net, uint64_t seed, uint64_t step, const uint64_t* d_step, uint64_t env_offset,
                      int64_t n_envs, const float* d_y, const float* d_w1, const float* d_b1, const float* d_w2,
                      const float* d_b2, const float* d_w3, const float* d_b3, const float* d_wh1, const float* d_bh1,
                      const float* d_wh2, const float* d_bh2, int32_t n_branches, int32_t n_actions, float slope,
                      float epsilon, const float* d_epsilon, uint32_t* d_flipmask, int32_t* d_actions,
                      void* stream) {
  pbn::NetView v;
  int rc = pbn::net_view(net, &v);
  if (rc) return rc;
  if (n_branches < 1 || n_branches > kMaxHeads - 1) return pbn::set_error(PBN_EINVAL, "n_branches must be 1..7");
  if ((rc = qnet_check(net, n_envs, d_y, d_w1, d_b1, d_w2, d_b2, d_w3, d_b3, d_wh1, d_bh1, d_wh2, d_bh2,
                       n_branches + 1, n_actions)))
    return rc;
  if (env_offset & 31) return pbn::set_error(PBN_EINVAL, "env_offset must be a multiple of 32");
  if (n_actions != v.n_nodes + 1) return pbn::set_error(PBN_EINVAL, "n_actions must be n_nodes + 1");
  if (!(epsilon >= 0.f && epsilon <= 1.f)) return pbn::set_error(PBN_EINVAL, "epsilon must be in [0, 1]");
  if (d_step && ((uintptr_t)d_step & 7u) != 0) return pbn::set_error(PBN_EINVAL, "d_step must be 8-byte aligned");
  if (d_epsilon && ((uintptr_t)d_epsilon & 3u) != 0) return pbn::set_error(PBN_EINVAL, "d_epsilon misaligned");
  if (n_envs == 0) return PBN_OK;
  if (!d_flipmask) return pbn::set_error(PBN_EINVAL, "null buffer");
  QnetArgs a{};
  a.y = d_y; a.w1 = d_w1; a.b1 = d_b1; a.w2 = d_w2; a.b2 = d_b2; a.w3 = d_w3; a.b3 = d_b3;
  a.wh1 = d_wh1; a.bh1 = d_bh1; a.wh2 = d_wh2; a.bh2 = d_bh2;
  a.n = n_envs; a.n_heads = n_branches + 1; a.n_act = n_actions; a.slope = slope;
  // explore iff EXPLORE word 0 < floor(epsilon * 2^32), as pbn_q_to_flipmask
  a.seed = seed; a.step = step; a.env_offset = env_offset; a.eps_u = (uint64_t)floor((double)epsilon * 4294967296.0);
  a.d_step = d_step; a.d_eps = d_epsilon; a.flipmask = d_flipmask; a.actions = d_actions;
  a.n_nodes = v.n_nodes; a.W = v.W;
  return qnet_launch<true, false>(a, stream);
}

int pbn_qnet_heads_from_state(const pbn_net* net, int64_t n_envs, const uint32_t* d_state, const uint8_t* d_target,
                              const float* d_T, const float* d_b0, const float* d_w1, const float* d_b1,
                              const float* d_w2, const float* d_b2, const float* d_w3, const float* d_b3,
                              const float* d_wh1, const float* d_bh1, const float* d_wh2, const float* d_bh2,
                              int32_t n_heads, int32_t n_actions, float slope, float* d_heads, void* stream) {
  QnetArgs a{};
  int rc = qnet_check(net, n_envs, d_b0, d_w1, d_b1, d_w2, d_b2, d_w3, d_b3, d_wh1, d_bh1, d_wh2, d_bh2, n_heads,
                      n_actions);
  if (rc || n_envs == 0) return rc;
  if ((rc = bil_check(net, d_state, d_target, d_T, d_b0, a))) return rc;
  if (!d_heads) return pbn::set_error(PBN_EINVAL, "null buffer");
  a.w1 = d_w1; a.b1 = d_b1; a.w2 = d_w2; a.b2 = d_b2; a.w3 = d_w3; a.b3 = d_b3;
  a.wh1 = d_wh1; a.bh1 = d_bh1; a.wh2 = d_wh2; a.bh2 = d_bh2; a.heads = d_heads;
  a.n = n_envs; a.n_heads = n_heads; a.n_act = n_actions; a.slope = slope;
  return qnet_launch<false, true>(a, stream);
}

int pbn_qnet_flipmask_from_state(const pbn_net* net, uint64_t seed, uint64_t step, const uint64_t* d_step,
                                 uint64_t env_offset, int64_t n_envs, const uint32_t* d_state,
                                 const uint8_t* d_target, const float* d_T, const float* d_b0, const float* d_w1,
                                 const float* d_b1, const float* d_w2, const float* d_b2, const float* d_w3,
                                 const float* d_b3, const float* d_wh1, const float* d_bh1, const float* d_wh2,
                                 const float* d_bh2, int32_t n_branches, int32_t n_actions, float slope,
                                 float epsilon, const float* d_epsilon, uint32_t* d_flipmask, int32_t* d_actions,
                                 void* stream) {
  pbn::NetView v;
  int rc = pbn::net_view(net, &v);
  if (rc) return rc;
  if (n_branches < 1 || n_branches > kMaxHeads - 1) return pbn::set_error(PBN_EINVAL, "n_branches must be 1..7");
  if ((rc = qnet_check(net, n_envs, d_b0, d_w1, d_b1, d_w2, d_b2, d_w3, d_b3, d_wh1, d_bh1, d_wh2, d_bh2,
                       n_branches + 1, n_actions)))
    return rc;
  if (env_offset & 31) return pbn::set_error(PBN_EINVAL, "env_offset must be a multiple of 32");
  if (n_actions != v.n_nodes + 1) return pbn::set_error(PBN_EINVAL, "n_actions must be n_nodes + 1");
  if (!(epsilon >= 0.f && epsilon <= 1.f)) return pbn::set_error(PBN_EINVAL, "epsilon must be in [0, 1]");
  if (d_step && ((uintptr_t)d_step & 7u) != 0) return pbn::set_error(PBN_EINVAL, "d_step must be 8-byte aligned");
  if (d_epsilon && ((uintptr_t)d_epsilon & 3u) != 0) return pbn::set_error(PBN_EINVAL, "d_epsilon misaligned");
  if (n_envs == 0) return PBN_OK;
  QnetArgs a{};
  if ((rc = bil_check(net, d_state, d_target, d_T, d_b0, a))) return rc;
  if (!d_flipmask) return pbn::set_error(PBN_EINVAL, "null buffer");
  a.w1 = d_w1; a.b1 = d_b1; a.w2 = d_w2; a.b2 = d_b2; a.w3 = d_w3; a.b3 = d_b3;
  a.wh1 = d_wh1; a.bh1 = d_bh1; a.wh2 = d_wh2; a.bh2 = d_bh2;
  a.n = n_envs; a.n_heads = n_branches + 1; a.n_act = n_actions; a.slope = slope;
  a.seed = seed; a.step = step; a.env_offset = env_offset; a.eps_u = (uint64_t)floor((double)epsilon * 4294967296.0);
  a.d_step = d_step; a.d_eps = d_epsilon; a.flipmask = d_flipmask; a.actions = d_actions;
  return qnet_launch<true, true>(a, stream);
}

}  // extern "C"
