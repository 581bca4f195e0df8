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
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>
#include <string>
#include <vector>

#include "../../include/pbn_env.h"
#include "bitslice.h"
#include "net_view.h"
#include "philox.h"

#include "step_kernels.h"

namespace pbn {
// pbn_settle.hip: pbn_step_wave<W, B, 3> (lean = 0, pbn_step) or <W, B, 4> (lean = 1,
// pbn_rollout) under the settle law, as an untyped host stub pointer (nullptr: no such W, B)
void* settle_kernel(int W, int B, int lean);
// pbn_settle.hip: pbn_rollout_settle<W, B> (pbn_rollout under the settle law, pipelined)
void* settle_pipe_kernel(int W, int B);
}  // namespace pbn

namespace {

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


template <int W, int V>
StepFn pick_wave_w(int B) {
  switch (B) {
    case 4: return pbn_step_wave<W, 4, V>;
    case 8: return pbn_step_wave<W, 8, V>;
    case 12: return pbn_step_wave<W, 12, V>;
    case 16: return pbn_step_wave<W, 16, V>;
  }
  return nullptr;
}

template <int V>
StepFn pick_wave(int W, int B) {
  switch (W) {
    case 1: return pick_wave_w<1, V>(B);
    case 2: return pick_wave_w<2, V>(B);
    case 3: return pick_wave_w<3, V>(B);
    case 4: return pick_wave_w<4, V>(B);
  }
  return nullptr;
}

template <int W, bool MANY>
StepFn pick_pipe_w(int B) {
  switch (B) {
    case 4: return pbn_rollout_pipe<W, 4, MANY>;
    case 8: return pbn_rollout_pipe<W, 8, MANY>;
    case 12: return pbn_rollout_pipe<W, 12, MANY>;
    case 16: return pbn_rollout_pipe<W, 16, MANY>;
  }
  return nullptr;
}

// many: some node has more than kNodeRecs functions (the instance that carries those chains)
StepFn pick_pipe(int W, int B, bool many) {
  switch (W) {
    case 1: return many ? pick_pipe_w<1, true>(B) : pick_pipe_w<1, false>(B);
    case 2: return many ? pick_pipe_w<2, true>(B) : pick_pipe_w<2, false>(B);
    case 3: return many ? pick_pipe_w<3, true>(B) : pick_pipe_w<3, false>(B);
    case 4: return many ? pick_pipe_w<4, true>(B) : pick_pipe_w<4, false>(B);
  }
  return nullptr;
}

using ResetFn = void (*)(const int32_t*, const uint32_t*, int, int, int, uint64_t, uint64_t, uint64_t, int64_t,
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
  int n_cus = 256;   // compute units of the device (the pipelined rollout's priority choice)
  int n_nodes = 0, W = 0, B = 0, horizon = 0, n_attr = 0, n_states = 0;
  int cdf_len = 0, hash_bits = 0, hash_probes = 0, tab_words = 0;
  uint32_t hash_mult[4] = {0, 0, 0, 0};
  int wave_words = 0;
  int att_off = 0;
  int sel_off = 0;
  int nrec_off = 0;
  int cm_off = 0;   // the pipelined kernel's threshold digit masks in the image (W == 1)
  int n_cls = 0;
  uint32_t uthr[kNodeRecs] = {0, 0, 0, 0};
  int gap_exact = 1;
  int gap_lut_off = 0, gap_shift = 0, gap_nb = 0;
  float inv_log2q = 0.f;
  uint4* d_fcompact = nullptr;
  uint4* d_nrec = nullptr;
  uint32_t* d_sthr = nullptr;   // settle law: thresholds scaled to 16 bits [lq][32W] (StepArgs::sthr)
  uint32_t* d_sthr_pk = nullptr;   // the same, packed biased node pairs [lq][W][16] (StepArgs::sthr_pk)
  int settle_pk = 0;
  int n_funcs = 0;
  size_t lds_wave = 0;
  StepFn wave1 = nullptr;       // single step (pbn_step)
  StepFn wave_lean = nullptr;   // rollout, one wave per group (networks with gates)
  StepFn wave_settle = nullptr;       // pbn_step under the settle law (settle_max >= 2)
  StepFn wave_settle_lean = nullptr;  // pbn_rollout under the settle law (networks with gates)
  StepFn pipe_settle = nullptr;       // pbn_rollout under the settle law, three waves per group pair
  size_t lds_settle = 0;
  int settle_max = 0;
  StepFn pipe = nullptr;        // rollout, three waves per group pair (every other network)
  size_t lds_pipe = 0;
  int n_gates = 0, n_glayers = 0, gate_off = 0, glayer_off = 0;   // lowered wide functions
  int max_nf = 0, lq = 1, slot_words = 0, slot_words_settle = 0;
  uint32_t n1_magic = 0, am1_magic = 0;   // ceil(2^32 / (N + 1)), ceil(2^32 / (A - 1))
  uint64_t x_mult = 0;
  int att_single = 0;                     // every attractor is a single state
  int force_roll = 0;        // PBN_ROLL env override: 2 = lean (wave kernel), 3 = pipe
  ResetFn reset = nullptr;
  uint32_t* d_tab = nullptr;
  int32_t* d_att_start = nullptr;
  uint32_t* d_att_states = nullptr;
  uint32_t* d_att_first = nullptr;        // [n_attr][W]: each attractor's first state
};

namespace pbn {

int set_error(int code, const char* msg) { return fail(code, msg); }

int net_view(const pbn_net* net, NetView* v) {
  if (!net || !v) return fail(PBN_EINVAL, "null net");
  v->device = net->device;
  v->n_nodes = net->n_nodes;
  v->W = net->W;
  v->n_attr = net->n_attr;
  v->n_states = net->n_states;
  v->att_start = net->d_att_start;
  v->att_states = net->d_att_states;
  v->att_first = net->d_att_first;
  return PBN_OK;
}

int check_device(const pbn_net* net) {
  if (!net) return fail(PBN_EINVAL, "null net");
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != net->device)
    return fail(PBN_EDEVICE, "current device differs from the net's device");
  return PBN_OK;
}

}  // namespace pbn

namespace {

void free_net(pbn_net* net) {
  if (!net) return;
  (void)hipFree(net->d_fcompact);
  (void)hipFree(net->d_nrec);
  (void)hipFree(net->d_sthr);
  (void)hipFree(net->d_sthr_pk);
  (void)hipFree(net->d_tab);
  (void)hipFree(net->d_att_start);
  (void)hipFree(net->d_att_states);
  (void)hipFree(net->d_att_first);
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
  // prefer a collision-free table (one probe per lookup) up to 16x the minimal size
  const int min_bits = bits;
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
    const bool accept = best_probes == 1 || (best_probes <= 4 && bits >= std::min(min_bits + 4, kMaxHashBits));
    if (accept || bits == kMaxHashBits) {
      const int HS = W == 1 ? 2 : (W <= 3 ? 4 : 8);   // HashStride<W>
      image->assign((size_t)HS * size, 0u);
      std::vector<int> used(size, 0);
      for (uint32_t s = 0; s < size; ++s) (*image)[(size_t)s * HS + W] = 0xFFFFFFFFu;
      for (size_t k = 0; k < S; ++k) {
        uint32_t h = 0;
        for (int w = 0; w < W; ++w) h += states[k][w] * best_mult[w];
        h >>= (32 - bits);
        int p = 0;
        while (used[(h + p) & mask]) ++p;
        const uint32_t slot = (h + p) & mask;
        used[slot] = 1;
        for (int w = 0; w < W; ++w) (*image)[(size_t)slot * HS + w] = states[k][w];
        (*image)[(size_t)slot * HS + W] = ids[k];
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

int pbn_state_histogram(const uint32_t* d_states, int64_t n_rows, int64_t n_cols, int64_t row_stride,
                        int32_t n_bits, uint32_t* d_hist, void* stream) {
  if (n_rows < 0 || n_cols < 0 || row_stride < n_cols) return fail(PBN_EINVAL, "bad histogram shape");
  if (n_bits < 1 || n_bits > 32) return fail(PBN_EINVAL, "n_bits must be 1..32");
  if (n_rows == 0 || n_cols == 0) return PBN_OK;
  if (!d_states || !d_hist) return fail(PBN_EINVAL, "null buffer");
  const uint32_t mask = n_bits == 32 ? 0xFFFFFFFFu : ((1u << n_bits) - 1u);
  const int64_t total = n_rows * n_cols;
  const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(pbn_hist_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, d_states, n_rows, n_cols,
                     row_stride, mask, d_hist);
  HIP_OK(hipGetLastError());
  return PBN_OK;
}
int pbn_abi_version(void) { return PBN_ABI_VERSION; }

int pbn_host_buffer(int64_t bytes, void** h_ptr, void** d_ptr) {
  if (bytes <= 0 || !h_ptr || !d_ptr) return fail(PBN_EINVAL, "bytes <= 0 or null out pointer");
  *h_ptr = nullptr;
  *d_ptr = nullptr;
  void* h = nullptr;
  if (hipHostMalloc(&h, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess || !h)
    return fail(PBN_ENOMEM, "hipHostMalloc failed");
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) {
    (void)hipHostFree(h);
    return fail(PBN_EDEVICE, "hipHostGetDevicePointer failed");
  }
  memset(h, 0, (size_t)bytes);
  *h_ptr = h;
  *d_ptr = d;
  return PBN_OK;
}

int pbn_host_buffer_free(void* h_ptr) {
  if (!h_ptr) return PBN_OK;
  HIP_OK(hipHostFree(h_ptr));
  return PBN_OK;
}

int pbn_stream_sync(void* stream) {
  HIP_OK(hipStreamSynchronize((hipStream_t)stream));
  return PBN_OK;
}

// pbn_copy_async: a grid-stride copy in 16-byte non-temporal vectors (the records are read once and
// go to the learner: neither side should displace the rollout's table image from L2), four
// independent vectors in flight per thread
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) pbn_copy_kernel(u32x4* __restrict__ dst, const u32x4* __restrict__ src,
                                                       int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
    for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(v[u], dst + i + u * stride);
  }
  for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

int pbn_copy_async(void* d_dst, const void* d_src, int64_t bytes, void* stream) {
  if (bytes < 0) return fail(PBN_EINVAL, "bytes < 0");
  if (bytes == 0) return PBN_OK;
  if (!d_dst || !d_src) return fail(PBN_EINVAL, "null buffer");
  if ((bytes & 15) || ((uintptr_t)d_dst & 15u) || ((uintptr_t)d_src & 15u))
    return fail(PBN_EINVAL, "pointers and bytes must be 16-byte aligned");
  const char* d = static_cast<const char*>(d_dst);
  const char* s = static_cast<const char*>(d_src);
  if (d < s + bytes && s < d + bytes) return fail(PBN_EINVAL, "overlapping ranges");
  const int64_t n16 = bytes / 16;
  int dev = 0, n_cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n_cus, hipDeviceAttributeMultiprocessorCount, dev);
  // 8 blocks per CU at most, each thread moving 4 vectors per trip (the last hand-off of a run, on
  // the launch stream: the most blocks that still stream full 1-KB rows per wave)
  constexpr int64_t kCopyBlocksPerCu = 8;
  const int64_t want = (n16 + 4 * 256 - 1) / (4 * 256);
  const unsigned blocks =
      (unsigned)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)n_cus * kCopyBlocksPerCu));
  hipLaunchKernelGGL(pbn_copy_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, static_cast<u32x4*>(d_dst),
                     static_cast<const u32x4*>(d_src), n16);
  HIP_OK(hipGetLastError());
  return PBN_OK;
}

int pbn_net_words(const pbn_net* net) { return net ? net->W : PBN_EINVAL; }

int pbn_net_create(const pbn_net_desc* d, pbn_net** out) {
  if (!d || !out) return fail(PBN_EINVAL, "null descriptor/out");
  *out = nullptr;
  const int N = d->n_nodes;
  if (N < 1 || N > PBN_MAX_NODES) return fail(PBN_EINVAL, "n_nodes out of range 1..128");
  if (!(d->prob_bits == 4 || d->prob_bits == 8 || d->prob_bits == 12 || d->prob_bits == 16))
    return fail(PBN_EINVAL, "prob_bits must be 4, 8, 12 or 16");
  if (d->horizon < 0 || d->horizon > 255) return fail(PBN_EINVAL, "horizon out of range 0..255");
  if (d->settle_max < 0 || d->settle_max > PBN_MAX_SETTLE) return fail(PBN_EINVAL, "settle_max out of range 0..4096");
  if (d->n_attractors < 0 || d->n_attractors > PBN_MAX_ATTRACTORS)
    return fail(PBN_EINVAL, "n_attractors out of range 0..254");
  if (!d->node_func_start || !d->func_arity || !d->func_inputs || !d->func_table || !d->func_threshold ||
      !d->perturb_cdf || !d->reward_table)
    return fail(PBN_EINVAL, "null table in descriptor");
  const int W = (N + 31) / 32;
  const uint32_t one = 1u << d->prob_bits;
  const int n_gates = d->n_gates;
  if (n_gates < 0 || n_gates > PBN_MAX_GATES || 32 * W + n_gates > 256)
    return fail(PBN_EINVAL, "n_gates out of range (32 * W + n_gates must be <= 256)");
  if (n_gates && (!d->gate_arity || !d->gate_inputs || !d->gate_table)) return fail(PBN_EINVAL, "null gate table");
  // gate levels: 1 + the deepest gate input (nodes are level 0)
  std::vector<int> glevel(n_gates, 1);
  for (int g = 0; g < n_gates; ++g) {
    const int k = d->gate_arity[g];
    if (k < 0 || k > PBN_MAX_ARITY) return fail(PBN_EINVAL, "gate arity must be 0..4");
    if (k < 5 && (1u << k) < 32 && (d->gate_table[g] >> (1u << k)) != 0u)
      return fail(PBN_EINVAL, "gate truth table has bits beyond 2^arity");
    for (int j = 0; j < k; ++j) {
      const int r = d->gate_inputs[4 * g + j];
      if (r < 0 || r >= N + g) return fail(PBN_EINVAL, "gate input must be a node or an earlier gate");
      if (r >= N) glevel[g] = std::max(glevel[g], glevel[r - N] + 1);
    }
  }
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
        if (g < 0 || g >= N + n_gates) return fail(PBN_EINVAL, "function input reference out of range");
        r.in[j] = (uint32_t)(g < N ? g : 32 * W + (g - N));   // LDS plane index
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
  // LDS table image: cdf[cdf_len] | reward[N+1][4] | hash[1 << bits][HashStride<W>]
  std::vector<uint32_t> tab(net->cdf_len, 0xFFFFFFFFu);
  for (int m = 0; m < N; ++m) tab[m] = d->perturb_cdf[m];
  for (int m = 1; m < N; ++m)
    if (tab[m] < tab[m - 1]) {
      free_net(net);
      return fail(PBN_EINVAL, "perturb_cdf must be non-decreasing");
    }
  // reward rows by popcount(flipmask): {none, wrong attractor, target, 0} (one 16-byte read)
  for (int pc = 0; pc <= N; ++pc)
    for (int c = 0; c < 4; ++c) {
      uint32_t u = 0;
      if (c < 3) memcpy(&u, &d->reward_table[c * (N + 1) + pc], 4);
      tab.push_back(u);
    }
  tab.insert(tab.end(), hash_img.begin(), hash_img.end());
  // attractor start[A+1] | states[S][W], read by autoreset in the wave kernel
  net->att_off = (int)tab.size();
  if (A) {
    for (int k = 0; k <= A; ++k) tab.push_back((uint32_t)d->attractor_start[k]);
    tab.insert(tab.end(), d->attractor_states, d->attractor_states + (size_t)S * W);
  }
  while (tab.size() & 3) tab.push_back(0u);  // 16-byte aligned uint4 selectors
  for (int i = 0; i < N; ++i)
    net->max_nf = std::max(net->max_nf, d->node_func_start[i + 1] - d->node_func_start[i]);
  // records per node in the LDS image: no kernel reads record q >= max_nf (the chains stop at a
  // node's function count, the padded ones at max_nf), so the image holds min(max_nf, kNodeRecs)
  // of them at the [kNodeRecs]-layout's strides (pbn70: 4.6 KB less LDS per block)
  const int Q = std::min(std::max(net->max_nf, 1), kNodeRecs);
  // leaf selectors of the first Q functions of every node, uint4 [Q][2][32W]
  // (lane-consecutive 16-byte reads); see eval_sel
  net->sel_off = (int)tab.size();
  {
    std::vector<uint32_t> sel((size_t)Q * 2 * 32 * W * 4, 0x0C0C0C0Cu);
    for (int i = 0; i < N; ++i) {
      const int f0 = d->node_func_start[i], nf = d->node_func_start[i + 1] - f0;
      // records beyond a node's last function (up to Q) repeat the last one: the
      // pipelined kernel's chain then needs no per-lane function count (x = lt ? f : x with
      // f == x is x)
      for (int q = 0; q < Q; ++q) {
        const int qf = std::min(q, nf - 1);
        const uint32_t T = d->func_table[f0 + qf];
        const int k = d->func_arity[f0 + qf];
        for (int mm = 0; mm < 8; ++mm) {
          // table bit of input index m (missing inputs read plane 0 but do not matter)
          auto bit = [&](uint32_t m) { return (T >> (k >= 5 ? m : (m & ((1u << k) - 1u)))) & 1u; };
          const uint32_t l0 = bit(2u * mm), l1 = bit(2u * mm + 1u);
          uint32_t word = 0;
          for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t b = (!l0 && !l1) ? 12u : (l0 && l1) ? 13u : (l1 ? j : 4u + j);
            word |= b << (8 * j);
          }
          const int h = mm >> 2;
          sel[(((size_t)q * 2 + h) * 32 * W + i) * 4 + (mm & 3)] = word;
        }
      }
    }
    tab.insert(tab.end(), sel.begin(), sel.end());
  }
  // threshold classes: the distinct values among the first kNodeRecs thresholds of all nodes;
  // with at most kNodeRecs of them the kernels compare against wave-uniform digits
  std::vector<uint32_t> cls_of((size_t)d->n_funcs, 0u);
  {
    std::vector<uint32_t> vals;
    bool ok = true;
    for (int i = 0; i < N && ok; ++i) {
      const int f0 = d->node_func_start[i], nf = d->node_func_start[i + 1] - f0;
      for (int q = 0; q < kNodeRecs && q < nf - 1; ++q) {
        const uint32_t c = d->func_threshold[f0 + q];
        auto it = std::find(vals.begin(), vals.end(), c);
        if (it == vals.end()) {
          if ((int)vals.size() == kNodeRecs) { ok = false; break; }
          vals.push_back(c);
          it = vals.end() - 1;
        }
        cls_of[f0 + q] = (uint32_t)(it - vals.begin());
      }
    }
    net->n_cls = ok ? (int)vals.size() : 0;
    for (int q = 0; q < kNodeRecs; ++q) net->uthr[q] = (ok && q < (int)vals.size()) ? vals[q] : 0u;
    net->lq = std::max(net->max_nf - 1, 1);
  }
  std::vector<uint4> fcomp(d->n_funcs);
  for (int f = 0; f < d->n_funcs; ++f) {
    const FuncRec& r = recs[f];
    uint32_t T4 = 0;
    for (int mm = 0; mm < 8; ++mm) {
      const uint32_t b0 = r.leaf[8 + mm] & 1u;               // value at x0 = 0
      const uint32_t b1 = (r.leaf[8 + mm] ^ r.leaf[mm]) & 1u; // value at x0 = 1
      T4 |= (b0 << (2 * mm)) | (b1 << (2 * mm + 1));
    }
    fcomp[f] = make_uint4(r.in[0] | (r.in[1] << 8) | (r.in[2] << 16) | (r.in[3] << 24), T4, r.thr, 0u);
  }
  std::vector<uint4> nrec((size_t)N * kNodeRecs, make_uint4(0, 0, 0, 0));
  for (int i = 0; i < N; ++i) {
    const int f0 = d->node_func_start[i], nf = d->node_func_start[i + 1] - f0;
    for (int q = 0; q < kNodeRecs && q < nf; ++q) {
      nrec[(size_t)i * kNodeRecs + q] = fcomp[f0 + q];
      nrec[(size_t)i * kNodeRecs + q].y = cls_of[f0 + q];   // threshold class (the table lives in the selectors)
    }
    nrec[(size_t)i * kNodeRecs + 0].w = (uint32_t)nf;
    nrec[(size_t)i * kNodeRecs + 1].w = (uint32_t)f0;
  }
  // the records in the LDS image too, record-major uint4 [Q][32W] (the pipelined
  // kernel reads them per step instead of keeping them in VGPRs across its loop; lane = node,
  // so consecutive lanes read consecutive 16-byte records: no LDS bank conflicts, where the
  // node-major layout's 64-byte lane stride conflicted 4 ways)
  net->nrec_off = (int)tab.size();
  for (int q = 0; q < Q; ++q)
    for (int i = 0; i < 32 * W; ++i) {
      uint4 r4 = i < N ? nrec[(size_t)i * kNodeRecs + q] : make_uint4(0, 0, 0, 0);
      if (i < N) {   // padded inputs as the selectors above (the .w metadata stays)
        const int nf = d->node_func_start[i + 1] - d->node_func_start[i];
        if (q >= nf) r4.x = nrec[(size_t)i * kNodeRecs + nf - 1].x;
      }
      if (W <= 2) r4.x *= 4u;   // plane byte offsets (every index < 64: no carry between bytes)
      tab.push_back(r4.x); tab.push_back(r4.y); tab.push_back(r4.z); tab.push_back(r4.w);
    }
  // gate records by level: {input plane indices as bytes, 16-bit table (unused inputs
  // replicated), output plane index 32W + g, 0}, then the level starts
  net->n_gates = n_gates;
  if (n_gates) {
    int n_lv = 0;
    for (int g = 0; g < n_gates; ++g) n_lv = std::max(n_lv, glevel[g]);
    std::vector<int> order(n_gates);
    for (int g = 0; g < n_gates; ++g) order[g] = g;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return glevel[x] < glevel[y]; });
    net->gate_off = (int)tab.size();
    std::vector<int> starts(n_lv + 1, 0);
    for (int idx = 0; idx < n_gates; ++idx) {
      const int g = order[idx], k = d->gate_arity[g];
      uint32_t ins = 0;
      for (int j = 0; j < k; ++j) {
        const int r = d->gate_inputs[4 * g + j];
        ins |= (uint32_t)(r < N ? r : 32 * W + (r - N)) << (8 * j);
      }
      const uint32_t T = d->gate_table[g];
      const uint32_t kmask = (1u << k) - 1u;
      uint32_t T16 = 0;
      for (uint32_t m = 0; m < 16; ++m) T16 |= ((T >> (m & kmask)) & 1u) << m;
      tab.push_back(ins); tab.push_back(T16); tab.push_back((uint32_t)(32 * W + g)); tab.push_back(0u);
      starts[glevel[g]] = idx + 1;   // running end of each level (levels are contiguous)
    }
    net->glayer_off = (int)tab.size();
    tab.push_back(0u);
    for (int lv = 1; lv <= n_lv; ++lv) {
      if (starts[lv] == 0) starts[lv] = starts[lv - 1];
      tab.push_back((uint32_t)starts[lv]);
    }
    net->n_glayers = n_lv;
  }
  // gap bucket table (gap_lut): the smallest bucket width 2^shift, shift = 32 - k with
  // k = 6..10, under which every bucket below C[N-1] holds at most one CDF threshold;
  // none found (p tiny) -> the estimate / binary search paths
  {
    const double p = (double)d->perturb_cdf[0] / 4294967296.0;
    const bool exact = p < 1e-6 || p > 0.5;
    auto gap_at = [&](uint64_t u) {   // min{m : u < C[m-1]}, N+1 if none
      int m = 1;
      while (m <= N && (uint64_t)d->perturb_cdf[m - 1] <= u) ++m;
      return m;
    };
    if (!exact) {
      for (int k = 6; k <= 10 && !net->gap_nb; ++k) {
        const int shift = 32 - k;
        const uint64_t w = 1ull << shift;
        const uint32_t nb = (uint32_t)(((uint64_t)d->perturb_cdf[N - 1]) >> shift) + 1u;   // buckets that can see a flip
        bool ok = true;
        std::vector<uint32_t> lut;
        for (uint32_t b = 0; b < nb && ok; ++b) {
          const int lo = gap_at((uint64_t)b * w), hi = gap_at((uint64_t)b * w + w - 1);
          ok = hi - lo <= 1;
          lut.push_back(lo <= N ? d->perturb_cdf[lo - 1] : 0xFFFFFFFFu);
          lut.push_back((uint32_t)lo);
        }
        if (!ok) continue;
        lut.push_back(0xFFFFFFFFu);   // sentinel: u >= C[N-1] -> gap N+1 (u = 2^32-1 gives N+2, also no flip)
        lut.push_back((uint32_t)(N + 1));
        while (tab.size() & 1) tab.push_back(0u);
        net->gap_lut_off = (int)tab.size();
        tab.insert(tab.end(), lut.begin(), lut.end());
        net->gap_shift = shift;
        net->gap_nb = (int)nb;
      }
    }
  }
  // the pipelined one-update kernel's threshold digit masks (single-word states), lane-major
  // [32][sel_mask_stride(B)]: mask (i, q, d) = ~0 if bit B-1-d of node i's threshold q is set.  In
  // the image, they arrive with the table copy; built by each block from the LDS records, they
  // cost a second prologue barrier (0.48 us of a 20-step launch, DESIGN.md "Launch anatomy")
  net->cm_off = 0;
  if (W == 1) {
    while (tab.size() & 3) tab.push_back(0u);
    net->cm_off = (int)tab.size();
    const int B = d->prob_bits, S = sel_mask_stride(B);
    std::vector<uint32_t> cmv((size_t)32 * S, 0u);
    for (int i = 0; i < N; ++i) {
      const int f0 = d->node_func_start[i], nf = d->node_func_start[i + 1] - f0;
      for (int q = 0; q < kNodeRecs - 1 && q < nf - 1; ++q) {
        const uint32_t c = recs[f0 + q].thr;
        for (int dd = 0; dd < B; ++dd) cmv[(size_t)i * S + q * B + dd] = ((c >> (B - 1 - dd)) & 1u) ? ~0u : 0u;
      }
    }
    tab.insert(tab.end(), cmv.begin(), cmv.end());
  }
  while (tab.size() & 3) tab.push_back(0u);   // the kernels copy the image as uint4
  net->tab_words = (int)tab.size();
  net->n_funcs = d->n_funcs;
  net->wave_words = (32 * W + n_gates + 3) & ~3;   // S planes (+ gate planes) per wave
  {
    const double p = (double)d->perturb_cdf[0] / 4294967296.0;
    net->gap_exact = (p < 1e-6 || p > 0.5) ? 1 : (net->gap_nb ? 2 : 0);
    net->inv_log2q = net->gap_exact ? 0.f : (float)(1.0 / log2(1.0 - p));
  }
  net->lds_wave = ((size_t)net->tab_words + (size_t)kWavesPerBlock * net->wave_words) * 4;
  net->slot_words = (3 * W + 1) * 64 + net->lq * 64 * W;
  // (the selection wave's threshold digit masks are part of the image: cm_off)
  net->lds_pipe = ((size_t)net->tab_words + 64 * (size_t)W + 2 * (size_t)net->slot_words) * 4;
  // compact records for the wave kernel: {inputs as bytes, 4-input truth table, threshold, 0}
  net->wave1 = pick_wave<1>(W, d->prob_bits);
  net->wave_lean = pick_wave<2>(W, d->prob_bits);
  net->wave_settle = reinterpret_cast<StepFn>(pbn::settle_kernel(W, d->prob_bits, 0));
  net->wave_settle_lean = reinterpret_cast<StepFn>(pbn::settle_kernel(W, d->prob_bits, 1));
  net->settle_max = d->settle_max;
  net->pipe_settle = net->max_nf <= kNodeRecs ? reinterpret_cast<StepFn>(pbn::settle_pipe_kernel(W, d->prob_bits))
                                              : nullptr;
  // pbn_rollout_settle: S planes [64W] | 2 slots {flip mask, perturbation mask, reset state [3W][64],
  // reset target and action count [64], selection planes [lq][64W]} | C [parity][64]{t, k}
  net->slot_words_settle = 192 * W + 64 + net->lq * 64 * W;
  // + ctl [2][64] uint4 + the packed thresholds [lq][W][16]
  // + the output rows [settle_stage_rows(W)][settle_row_words(W)], the stored-row counter [2] and
  // the rows' output pointers (6 x 8 bytes)
  net->lds_settle = ((size_t)net->tab_words + 64 * (size_t)W + 2 * (size_t)net->slot_words_settle + 512 +
                     (((size_t)net->lq * W * 16 + 3) & ~(size_t)3) +
                     (size_t)settle_stage_rows(W) * settle_row_words(W) + 2 + 12 + 2) * 4;
  net->pipe = pick_pipe(W, d->prob_bits, net->max_nf > kNodeRecs);
  net->reset = pick_reset(W);
  // multiply-high divisors (exact for the operand ranges used: see actions_from_draw, autoreset)
  net->n1_magic = (uint32_t)(((1ull << 32) + (uint64_t)N) / (uint64_t)(N + 1));
  net->att_single = A >= 1 && S == A ? 1 : 0;
  net->am1_magic = A >= 3 ? (uint32_t)(((1ull << 32) + (uint64_t)(A - 2)) / (uint64_t)(A - 1)) : 0u;   // 0: A - 1 == 1
  net->x_mult = (uint64_t)(N + 1) * (uint64_t)(N + 1) * (uint64_t)(N + 1) * (A >= 2 ? (uint64_t)A * (uint64_t)(A - 1) : 1ull);
  if (const char* env = getenv("PBN_ROLL")) {
    if (!strcmp(env, "lean")) net->force_roll = 2;
    if (!strcmp(env, "pipe")) net->force_roll = 3;
  }
  // the settle law's per-env selection thresholds (settle_lt_word): node i, threshold q <
  // nf_i - 1 as c << (16 - B), 65536 (always) past a node's last function and past the network
  std::vector<uint32_t> sthr((size_t)net->lq * 32 * W, 65536u);
  for (int i = 0; i < N; ++i) {
    const int f0 = d->node_func_start[i], nf = d->node_func_start[i + 1] - f0;
    for (int q = 0; q < nf - 1 && q < net->lq; ++q)
      sthr[(size_t)q * 32 * W + i] = d->func_threshold[f0 + q] << (16 - d->prob_bits);
  }
  // packed biased node pairs for settle_lt_word_pk, exact when no compared threshold is 65536
  std::vector<uint32_t> sthr_pk((size_t)net->lq * W * 16);
  net->settle_pk = 1;
  for (int q = 0; q < net->lq; ++q)
    for (int i = 0; i < 32 * W; i += 2) {
      uint32_t c[2];
      for (int h = 0; h < 2; ++h) {
        const int ii = i + h;
        const bool real = ii < N && q < d->node_func_start[ii + 1] - d->node_func_start[ii] - 1;
        const uint32_t v = sthr[(size_t)q * 32 * W + ii];
        if (real && v > 65535u) net->settle_pk = 0;
        c[h] = std::min(v, 65535u) ^ 0x8000u;
      }
      sthr_pk[((size_t)q * W + i / 32) * 16 + (i % 32) / 2] = c[0] | (c[1] << 16);
    }
  std::vector<uint32_t> att_first((size_t)A * W);
  for (int t = 0; t < A; ++t)
    for (int w = 0; w < W; ++w) att_first[(size_t)t * W + w] = d->attractor_states[(size_t)d->attractor_start[t] * W + w];
  int rc;
  if (hipGetDevice(&net->device) != hipSuccess) {
    free_net(net);
    return fail(PBN_EDEVICE, "no HIP device");
  }
  if (hipDeviceGetAttribute(&net->n_cus, hipDeviceAttributeMultiprocessorCount, net->device) != hipSuccess ||
      net->n_cus <= 0)
    net->n_cus = 256;
  if ((rc = upload(&net->d_fcompact, fcomp.data(), fcomp.size())) ||
      (rc = upload(&net->d_nrec, nrec.data(), nrec.size())) ||
      (rc = upload(&net->d_sthr, sthr.data(), sthr.size())) ||
      (rc = upload(&net->d_sthr_pk, sthr_pk.data(), sthr_pk.size())) ||
      (rc = upload(&net->d_tab, tab.data(), tab.size())) ||
      (rc = upload(&net->d_att_start, A ? d->attractor_start : nullptr, (size_t)A + 1)) ||
      (rc = upload(&net->d_att_states, S ? d->attractor_states : nullptr, (size_t)S * W)) ||
      (rc = upload(&net->d_att_first, A ? att_first.data() : nullptr, (size_t)A * W))) {
    free_net(net);
    return rc;
  }
  for (int ti = 0; ti < 6; ++ti) {
    const StepFn fns[6] = {net->wave_settle, net->wave_settle_lean, net->wave_lean, net->wave1, net->pipe,
                           net->pipe_settle};
    const StepFn fn = fns[ti];
    const size_t bytes = ti == 5 ? net->lds_settle : (ti == 4 ? net->lds_pipe : net->lds_wave);
    if (!fn || bytes > 160 * 1024) continue;  // variant unusable for this net; never picked
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)bytes) != hipSuccess) {
      free_net(net);
      return fail(PBN_EDEVICE, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
    }
  }
  if (net->lds_wave > 160 * 1024) {
    free_net(net);
    return fail(PBN_EINVAL, "LDS budget exceeded");
  }
  *out = net;
  return PBN_OK;
}

#ifdef PBN_STAMPS
static unsigned long long* g_stamps = nullptr;
int pbn_debug_set_stamps(unsigned long long* d_buf) {
  g_stamps = d_buf;
  return 0;
}
#endif

int pbn_net_destroy(pbn_net* net) {
  if (!net) return PBN_OK;
  free_net(net);
  return PBN_OK;
}

// ragged: n_envs may be any count (pbn_step: the last 32-env group is partial); env_offset is
// always a multiple of 32 (the groups' RNG keys)
static int check_common(pbn_net* net, uint64_t env_offset, int64_t n_envs, bool ragged = false) {
  if (!net) return fail(PBN_EINVAL, "null net");
  if (n_envs < 0) return fail(PBN_EINVAL, "n_envs < 0");
  if (ragged ? (env_offset & 31) != 0 : ((n_envs & 31) || (env_offset & 31)))
    return fail(PBN_EINVAL, ragged ? "env_offset must be a multiple of 32"
                                   : "n_envs and env_offset must be multiples of 32");
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != net->device)
    return fail(PBN_EDEVICE, "current device differs from the net's device");
  return PBN_OK;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// The launch arguments every step kernel shares: the net's tables and encodings, the key and
// the env range (the caller adds its buffers, mode and step count)
static void fill_args(const pbn_net* net, StepArgs* p, uint64_t seed, uint64_t step, uint64_t env_offset,
                      int64_t n_envs) {
  StepArgs& a = *p;
  memset(&a, 0, sizeof a);
  a.tab = net->d_tab;
  a.att_start = net->d_att_start;
  a.att_states = net->d_att_states;
  a.seed = seed;
  a.step = step;
  a.env_offset = env_offset;
  a.n_envs = n_envs;
  a.n_groups = (n_envs + 31) / 32;
  a.n_steps = 1;
  a.n_nodes = net->n_nodes;
  a.n_attr = net->n_attr;
  a.horizon = net->horizon;
  a.cdf_len = net->cdf_len;
  a.hash_bits = net->n_attr ? net->hash_bits : 0;
  a.hash_probes = net->hash_probes;
  a.tab_words = net->tab_words;
  a.n_states = net->n_states;
  a.att_off = net->att_off;
  a.sel_off = net->sel_off;
  a.nrec_off = net->nrec_off;
  a.cm_off = net->cm_off;
  a.n_cls = net->n_cls;
  a.max_nf = net->max_nf;
  a.lq = net->lq;
  a.slot_words = net->slot_words;
  a.gate_off = net->gate_off;
  a.glayer_off = net->glayer_off;
  a.n_glayers = net->n_glayers;
  memcpy(a.uthr, net->uthr, sizeof a.uthr);
  memcpy(a.hash_mult, net->hash_mult, sizeof a.hash_mult);
  a.prob_bits = net->B;
  a.n_funcs = net->n_funcs;
  a.wave_words = net->wave_words;
  a.gap_exact = net->gap_exact;
  a.gap_lut_off = net->gap_lut_off;
  a.gap_shift = net->gap_shift;
  a.gap_nb = net->gap_nb;
  a.inv_log2q = net->inv_log2q;
  a.fcompact = net->d_fcompact;
  a.nrec = net->d_nrec;
  a.sthr = net->d_sthr;
  a.sthr_pk = net->d_sthr_pk;
  a.settle_pk = net->settle_pk;
  a.n1_magic = net->n1_magic;
  a.att_single = net->att_single;
  a.am1_magic = net->am1_magic;
  a.x_mult = net->x_mult;
  a.settle_max = net->settle_max;
#ifdef PBN_STAMPS
  a.stamps = g_stamps;
#endif
}

int pbn_reset(pbn_net* net, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n_envs,
              uint32_t* d_state, uint8_t* d_target, uint8_t* d_t, void* stream) {
  int rc = check_common(net, env_offset, n_envs, true);
  if (rc) return rc;
  if (n_envs == 0) return PBN_OK;
  if (!d_state || !d_target || !d_t) return fail(PBN_EINVAL, "null buffer");
  const int threads = 256;
  const unsigned blocks = (unsigned)((n_envs + threads - 1) / threads);
  hipLaunchKernelGGL(net->reset, dim3(blocks), dim3(threads), 0, (hipStream_t)stream, net->d_att_start,
                     net->d_att_states, net->n_attr, net->n_states, net->n_nodes, seed, step, env_offset, n_envs, d_state,
                     d_target, d_t);
  HIP_OK(hipGetLastError());
  return PBN_OK;
}

static int step_impl(pbn_net* net, uint64_t seed, uint64_t step, const uint64_t* d_step, uint64_t env_offset,
                     int64_t n_envs, uint32_t mode, const uint32_t* d_state, uint32_t* d_flipmask,
                     uint8_t* d_target, uint8_t* d_t, uint32_t* d_state_out, uint32_t* d_final_state,
                     float* d_reward, uint8_t* d_flags, void* stream, const pbn_ring_store* ring = nullptr) {
  int rc = check_common(net, env_offset, n_envs, true);
  if (rc) return rc;
  if (n_envs == 0) return PBN_OK;
  if (mode & ~(PBN_MODE_AUTORESET | PBN_MODE_RANDOM_ACTIONS)) return fail(PBN_EINVAL, "unknown mode bits");
  if (!d_state || !d_flipmask || !d_target || !d_t || !d_state_out || !d_reward || !d_flags)
    return fail(PBN_EINVAL, "null buffer");
  // (the ring form steps in place: the wave kernel's lane reads its env's state once, at entry)
  if (d_state_out == d_state && !ring) return fail(PBN_EINVAL, "d_state_out must not alias d_state");
  if (!aligned16(d_state) || !aligned16(d_flipmask) || !aligned16(d_target) || !aligned16(d_t) ||
      !aligned16(d_state_out) || !aligned16(d_reward) || !aligned16(d_flags) ||
      (d_final_state && !aligned16(d_final_state)))
    return fail(PBN_EINVAL, "device buffers must be 16-byte aligned");
  StepArgs a;
  fill_args(net, &a, seed, step, env_offset, n_envs);
  a.step_ptr = d_step;
  a.state = d_state;
  a.state_out = d_state_out;
  a.flipmask = d_flipmask;
  a.target = d_target;
  a.t = d_t;
  a.final_state = d_final_state;
  a.reward = d_reward;
  a.flags = d_flags;
  a.mode = (int)mode;
  if (net->lds_wave > 160 * 1024) return fail(PBN_EINVAL, "network too large for the step kernel's LDS");
  if (ring) {
    const pbn_ring_store& r = *ring;
    if (net->settle_max >= 2) return fail(PBN_EINVAL, "pbn_step_dev_store: the one-update law only (settle_max < 2)");
    if (r.capacity < n_envs) return fail(PBN_EINVAL, "pbn_ring_store: capacity < n_envs");
    if (r.n_branches < 1 || r.n_branches > kRingMaxK) return fail(PBN_EINVAL, "pbn_ring_store: n_branches 1..8");
    if (!r.d_pos || ((uintptr_t)r.d_pos & 7u) || !r.d_state || !r.d_next_state || !r.d_target || !r.d_reward ||
        !r.d_done || !r.d_action || !r.d_actions_in)
      return fail(PBN_EINVAL, "pbn_ring_store: null or misaligned buffer");
    a.r_state = r.d_state;
    a.r_next = r.d_next_state;
    a.r_target = r.d_target;
    a.r_action = r.d_action;
    a.r_reward = r.d_reward;
    a.r_done = r.d_done;
    a.r_act_in = r.d_actions_in;
    a.r_done_out = r.d_done_out;
    a.r_pos = r.d_pos;
    a.r_cap = r.capacity;
    a.r_k = r.n_branches;
    a.r_done_mask = r.done_mask;
  }
  // the settle law on whole groups: a one-step launch of the pipelined settle kernel
  // (pbn_rollout_settle; its env-major outputs of one step are pbn_step's), where every env runs
  // its own update sequence and an update is one pipeline iteration, against the wave kernel's
  // variant 3, whose wave runs every update of its slowest env as a serial chain (VERDICT r05
  // next 2).  Ragged env counts, gates, PBN_ROLL=lean: the wave kernel.
  if (net->settle_max >= 2 && !(n_envs & 31) && net->pipe_settle && !net->n_gates &&
      net->lds_settle <= 64 * 1024 && net->force_roll != 2) {
    a.slot_words = net->slot_words_settle;
    const int64_t pblocks = (a.n_groups + 1) / 2;
    hipLaunchKernelGGL(net->pipe_settle, dim3((unsigned)pblocks), dim3(192), net->lds_settle, (hipStream_t)stream, a);
    HIP_OK(hipGetLastError());
    return PBN_OK;
  }
  const unsigned blocks = (unsigned)((a.n_groups + kWavesPerBlock - 1) / kWavesPerBlock);  // one wave per group
  const StepFn fn = net->settle_max >= 2 ? net->wave_settle : net->wave1;
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(64 * kWavesPerBlock), net->lds_wave, (hipStream_t)stream, a);
  HIP_OK(hipGetLastError());
  return PBN_OK;
}

int pbn_step(pbn_net* net, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n_envs, uint32_t mode,
             const uint32_t* d_state, uint32_t* d_flipmask, uint8_t* d_target, uint8_t* d_t,
             uint32_t* d_state_out, uint32_t* d_final_state, float* d_reward, uint8_t* d_flags,
             void* stream) {
  return step_impl(net, seed, step, nullptr, env_offset, n_envs, mode, d_state, d_flipmask, d_target, d_t,
                   d_state_out, d_final_state, d_reward, d_flags, stream);
}

int pbn_step_dev(pbn_net* net, uint64_t seed, const uint64_t* d_step, uint64_t env_offset, int64_t n_envs,
                 uint32_t mode, const uint32_t* d_state, uint32_t* d_flipmask, uint8_t* d_target, uint8_t* d_t,
                 uint32_t* d_state_out, uint32_t* d_final_state, float* d_reward, uint8_t* d_flags,
                 void* stream) {
  if (!d_step) return fail(PBN_EINVAL, "null d_step");
  if (((uintptr_t)d_step & 7u) != 0) return fail(PBN_EINVAL, "d_step must be 8-byte aligned");
  return step_impl(net, seed, 0, d_step, env_offset, n_envs, mode, d_state, d_flipmask, d_target, d_t,
                   d_state_out, d_final_state, d_reward, d_flags, stream);
}

int pbn_step_dev_store(pbn_net* net, uint64_t seed, const uint64_t* d_step, uint64_t env_offset, int64_t n_envs,
                       uint32_t mode, uint32_t* d_state, uint32_t* d_flipmask, uint8_t* d_target, uint8_t* d_t,
                       uint32_t* d_final_state, float* d_reward, uint8_t* d_flags, const pbn_ring_store* ring,
                       void* stream) {
  if (!d_step) return fail(PBN_EINVAL, "null d_step");
  if (((uintptr_t)d_step & 7u) != 0) return fail(PBN_EINVAL, "d_step must be 8-byte aligned");
  if (!ring) return fail(PBN_EINVAL, "null ring");
  return step_impl(net, seed, 0, d_step, env_offset, n_envs, mode, d_state, d_flipmask, d_target, d_t, d_state,
                   d_final_state, d_reward, d_flags, stream, ring);
}

int pbn_rollout(pbn_net* net, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n_envs,
                int32_t n_steps, uint32_t mode, uint32_t* d_state, uint32_t* d_flipmask, uint8_t* d_target,
                uint8_t* d_t, uint32_t* d_obs, uint32_t* d_final_state, float* d_reward, uint8_t* d_flags,
                void* stream) {
  return pbn_rollout_ex(net, seed, step, env_offset, n_envs, n_steps, mode, d_state, d_flipmask, d_target, d_t,
                        d_obs, d_final_state, d_reward, d_flags, nullptr, stream);
}

}  // extern "C"


// pbn_rollout_ex, with (cp_bytes > 0) a copy riding along (pbn_rollout_copy): a fourth wave per
// block of the pipelined one-update kernel, else pbn_copy_async right after the launch on the
// same stream
static int rollout_impl(pbn_net* net, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n_envs,
                        int32_t n_steps, uint32_t mode, uint32_t* d_state, uint32_t* d_flipmask, uint8_t* d_target,
                        uint8_t* d_t, uint32_t* d_obs, uint32_t* d_final_state, float* d_reward, uint8_t* d_flags,
                        uint16_t* d_updates, void* cp_dst, const void* cp_src, int64_t cp_bytes, void* stream) {
  int rc = check_common(net, env_offset, n_envs);
  if (rc) return rc;
  if (n_steps < 0) return fail(PBN_EINVAL, "n_steps < 0");
  bool copy_after = cp_bytes > 0;   // cleared when the copy rides along the launch
  struct After {   // the standalone copy, if it is still owed when the launch has been issued
    bool& owed;
    void *dst, *stream;
    const void* src;
    int64_t bytes;
    int finish(int r) { return (r == PBN_OK && owed) ? pbn_copy_async(dst, src, bytes, stream) : r; }
  } after{copy_after, cp_dst, stream, cp_src, cp_bytes};
  if (n_envs == 0 || n_steps == 0) return after.finish(PBN_OK);
  if (mode & ~(PBN_MODE_AUTORESET | PBN_MODE_RANDOM_ACTIONS)) return fail(PBN_EINVAL, "unknown mode bits");
  if (!d_state || !d_flipmask || !d_target || !d_t || !d_reward || !d_flags) return fail(PBN_EINVAL, "null buffer");
  if (net->lds_wave > 160 * 1024) return fail(PBN_EINVAL, "network too large for the rollout kernel's LDS");
  StepArgs a;
  fill_args(net, &a, seed, step, env_offset, n_envs);
  a.state = d_state;
  a.state_out = d_state;   // in place: every env is read and written by one lane only
  a.flipmask = d_flipmask;
  a.target = d_target;
  a.t = d_t;
  a.final_state = d_final_state;
  a.obs = d_obs;
  a.reward = d_reward;
  a.flags = d_flags;
  a.n_steps = n_steps;
  a.mode = (int)mode;
  a.updates = d_updates;
  // the pipelined kernels for every network they support (they beat the one-wave-per-group
  // rollout at every measured size: profiles/r01_sweep_pbn28_variants_v4.jsonl); networks
  // with gates (lowered wide functions) run the wave kernel.  PBN_ROLL=lean|pipe forces one.
  const bool settle = net->settle_max >= 2;
  bool pipe = (settle ? net->lds_settle : net->lds_pipe) <= 64 * 1024 && !net->n_gates && (!settle || net->pipe_settle);
  if (net->force_roll) pipe = net->force_roll == 3 && !net->n_gates && (!settle || net->pipe_settle);
  if (pipe) {   // one block of three waves per pair of groups
    const int64_t pblocks = (a.n_groups + 1) / 2;
    if (settle) {
      a.slot_words = net->slot_words_settle;
      hipLaunchKernelGGL(net->pipe_settle, dim3((unsigned)pblocks), dim3(192), net->lds_settle,
                         (hipStream_t)stream, a);
      HIP_OK(hipGetLastError());
      return after.finish(PBN_OK);
    }
    // the one-update law applies exactly one synchronous update per env-step
    if (d_updates) HIP_OK(hipMemsetD16Async(d_updates, 1, (size_t)n_steps * (size_t)n_envs, (hipStream_t)stream));
    a.sel_prio = pblocks <= 4 * (int64_t)net->n_cus ? 1 : 0;
    if (cp_bytes > 0) {   // the ride-along copy: a fourth wave per block
      a.cp_src = cp_src;
      a.cp_dst = cp_dst;
      a.cp_n16 = cp_bytes / 16;
      // paced at U vectors per lane and iteration when the grid's barriers cover the copy with
      // U <= 4 (one hand-off of this launch's own records: 12 W + 5 bytes per env-step, 64 envs
      // per block, U = 2 for single-word states), else one burst
      const int64_t slots = (int64_t)(n_steps + 1) * pblocks * 64;
      const int64_t u = (a.cp_n16 + slots - 1) / slots;
      a.cp_u = u <= 1 ? 1 : (u <= 2 ? 2 : (u <= 4 ? 4 : 0));
      // a grid of more blocks than run at once: the burst, whose wave exits early, where the paced
      // wave held a block slot for the whole launch (1M envs: 0.69 -> 0.74x of the bare launches'
      // rate, pbn70 x 1M: 0.65 -> 0.73x; profiles/r05_zj_ab.json)
      if (pblocks > 4 * (int64_t)net->n_cus) a.cp_u = 0;
      copy_after = false;
    }
    hipLaunchKernelGGL(net->pipe, dim3((unsigned)pblocks), dim3(a.cp_n16 ? 256 : 192), net->lds_pipe,
                       (hipStream_t)stream, a);
    HIP_OK(hipGetLastError());
    return after.finish(PBN_OK);
  }
  const unsigned blocks = (unsigned)((a.n_groups + kWavesPerBlock - 1) / kWavesPerBlock);  // one wave per group
  hipLaunchKernelGGL(net->settle_max >= 2 ? net->wave_settle_lean : net->wave_lean, dim3(blocks),
                     dim3(64 * kWavesPerBlock), net->lds_wave, (hipStream_t)stream, a);
  HIP_OK(hipGetLastError());
  return after.finish(PBN_OK);
}

extern "C" {

int pbn_rollout_ex(pbn_net* net, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n_envs,
                   int32_t n_steps, uint32_t mode, uint32_t* d_state, uint32_t* d_flipmask, uint8_t* d_target,
                   uint8_t* d_t, uint32_t* d_obs, uint32_t* d_final_state, float* d_reward, uint8_t* d_flags,
                   uint16_t* d_updates, void* stream) {
  return rollout_impl(net, seed, step, env_offset, n_envs, n_steps, mode, d_state, d_flipmask, d_target, d_t, d_obs,
                      d_final_state, d_reward, d_flags, d_updates, nullptr, nullptr, 0, stream);
}

int pbn_rollout_copy(pbn_net* net, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n_envs,
                     int32_t n_steps, uint32_t mode, uint32_t* d_state, uint32_t* d_flipmask, uint8_t* d_target,
                     uint8_t* d_t, uint32_t* d_obs, uint32_t* d_final_state, float* d_reward, uint8_t* d_flags,
                     uint16_t* d_updates, void* d_copy_dst, const void* d_copy_src, int64_t copy_bytes,
                     void* stream) {
  if (copy_bytes < 0) return fail(PBN_EINVAL, "copy_bytes < 0");
  if (copy_bytes > 0) {
    if (!d_copy_dst || !d_copy_src) return fail(PBN_EINVAL, "null copy buffer");
    if ((copy_bytes & 15) || ((uintptr_t)d_copy_dst & 15u) || ((uintptr_t)d_copy_src & 15u))
      return fail(PBN_EINVAL, "copy pointers and bytes must be 16-byte aligned");
    const char* d = static_cast<const char*>(d_copy_dst);
    const char* s = static_cast<const char*>(d_copy_src);
    if (d < s + copy_bytes && s < d + copy_bytes) return fail(PBN_EINVAL, "overlapping copy ranges");
  }
  return rollout_impl(net, seed, step, env_offset, n_envs, n_steps, mode, d_state, d_flipmask, d_target, d_t, d_obs,
                      d_final_state, d_reward, d_flags, d_updates, d_copy_dst, d_copy_src, copy_bytes, stream);
}

}  // extern "C"
