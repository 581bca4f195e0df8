// VALU issue rate of gfx950 per SIMD, by instruction and by waves per SIMD (VERDICT r02 "What's
// weak" 2: calibrate the rollout kernel's VALU ceiling).  Each lane runs 8 independent chains of
// one instruction with VGPR-only operands (no literal, no SGPR: the VOP encodings the kernel
// issues), kIters x 8 instructions per wave.  Every wave reads the shader clock (s_memtime, one
// tick = one shader cycle) and the 100 MHz real-time clock (s_memrealtime) around its loop.
// Two rates per line:
//   simd_cycles_per_inst   = the chip-wide span of the loops (first start to last end, real
//                            time x the median shader clock) x SIMDs / wave-instructions issued:
//                            the SIMD issue cost, whatever the waves' co-residency;
//   cycles_per_wave_inst   = one wave's own loop cycles per instruction (its issue interval).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_valu_issue tools/ubench_valu_issue.hip
//   tools/ubench_valu_issue > profiles/r03_ubench_valu_issue.jsonl
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

constexpr int kIters = 2048;
constexpr int kChains = 8;

enum Op { kBitop3, kXor, kAdd, kFma, kPkFma, kPerm, kMadU64, kAlignbit, kNumOps };
const char* kNames[kNumOps] = {"v_bitop3_b32", "v_xor_b32", "v_add_u32", "v_fma_f32", "v_pk_fma_f32",
                               "v_perm_b32", "v_mad_u64_u32", "v_alignbit_b32"};

__device__ __forceinline__ unsigned long long clk() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
__device__ __forceinline__ unsigned long long rtc() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <int OP>
__global__ void __launch_bounds__(256) issue_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                    unsigned long long* __restrict__ stamps) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a[kChains], b[kChains], c[kChains];
  for (int k = 0; k < kChains; ++k) {   // VGPR operands from memory: nothing folds to a constant
    a[k] = in[(tid * 3 + k) & 1023];
    b[k] = in[(tid * 5 + k + 7) & 1023] | 1u;
    c[k] = in[(tid * 7 + k + 13) & 1023];
  }
  __syncthreads();
  const unsigned long long t0 = clk(), r0 = rtc();
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int k = 0; k < kChains; ++k) {
      if constexpr (OP == kBitop3) {
        a[k] = __builtin_amdgcn_bitop3_b32(a[k], b[k], c[k], 0x96);
      } else if constexpr (OP == kXor) {   // (asm: a plain ^= chain folds to one xor)
        asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[k]) : "v"(b[k]));
      } else if constexpr (OP == kAdd) {
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b[k]));
      } else if constexpr (OP == kFma) {
        float x = __uint_as_float(a[k]);
        x = __builtin_fmaf(x, __uint_as_float(b[k]), __uint_as_float(c[k]));
        a[k] = __float_as_uint(x);
      } else if constexpr (OP == kPkFma) {
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 x = {__uint_as_float(a[k]), __uint_as_float(c[k])};
        const f2 y = {__uint_as_float(b[k]), __uint_as_float(b[k])};
        x = __builtin_elementwise_fma(x, y, y);
        a[k] = __float_as_uint(x.x);
        c[k] = __float_as_uint(x.y);
      } else if constexpr (OP == kPerm) {
        a[k] = __builtin_amdgcn_perm(a[k], b[k], c[k]);
      } else if constexpr (OP == kMadU64) {
        const uint64_t p = (uint64_t)a[k] * b[k] + c[k];
        a[k] = (uint32_t)(p >> 32) ^ (uint32_t)p;
      } else {
        a[k] = __builtin_amdgcn_alignbit(a[k], b[k], c[k]);
      }
    }
  }
  const unsigned long long t1 = clk(), r1 = rtc();
  uint32_t r = 0;
  for (int k = 0; k < kChains; ++k) r ^= a[k] ^ c[k];
  out[tid] = r;
  if ((threadIdx.x & 63) == 0) {
    const int w = tid >> 6;
    stamps[4 * w] = t1 - t0;
    stamps[4 * w + 1] = r1 - r0;
    stamps[4 * w + 2] = r0;
    stamps[4 * w + 3] = r1;
  }
}

// instructions issued per inner element (kMadU64: the product plus the xor of its halves)
constexpr int kInstPer[kNumOps] = {1, 1, 1, 1, 1, 1, 2, 1};

template <int OP>
void run(int cus, int waves_per_simd, const uint32_t* d_in, uint32_t* d_out, unsigned long long* d_st) {
  const int blocks = cus * waves_per_simd;   // 4 waves per block: one per SIMD
  const int n_waves = blocks * 4;
  hipLaunchKernelGGL(issue_kernel<OP>, dim3(blocks), dim3(256), 0, 0, d_in, d_out, d_st);   // warm
  hipLaunchKernelGGL(issue_kernel<OP>, dim3(blocks), dim3(256), 0, 0, d_in, d_out, d_st);
  hipDeviceSynchronize();
  std::vector<unsigned long long> st(4 * (size_t)n_waves);
  hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> cyc(n_waves), mhz(n_waves);
  unsigned long long first = ~0ull, last = 0;
  for (int w = 0; w < n_waves; ++w) {
    cyc[w] = (double)st[4 * w];
    mhz[w] = (double)st[4 * w] / ((double)st[4 * w + 1] / 100.0);   // real-time clock: 100 MHz
    first = std::min(first, st[4 * w + 2]);
    last = std::max(last, st[4 * w + 3]);
  }
  std::sort(cyc.begin(), cyc.end());
  std::sort(mhz.begin(), mhz.end());
  const double inst = (double)kIters * kChains * kInstPer[OP];
  const double med = cyc[n_waves / 2];
  const double span_cycles = (double)(last - first) / 100.0 * mhz[n_waves / 2];   // 100 MHz ticks x MHz
  const double simd_rate = span_cycles * (4.0 * cus) / (inst * n_waves);
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"wave_loop_cycles_median\": %.0f, "
         "\"cycles_per_wave_inst\": %.3f, \"span_cycles\": %.0f, \"simd_cycles_per_inst\": %.3f, "
         "\"shader_mhz_median\": %.0f}\n",
         kNames[OP], waves_per_simd, med, med / inst, span_cycles, simd_rate, mhz[n_waves / 2]);
}

template <int OP>
void sweep(int cus, const uint32_t* d_in, uint32_t* d_out, unsigned long long* d_st) {
  for (int w : {1, 2, 3, 4, 6, 8}) run<OP>(cus, w, d_in, d_out, d_st);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t *d_in, *d_out;
  unsigned long long* d_st;
  std::vector<uint32_t> h(1024);
  for (int i = 0; i < 1024; ++i) h[i] = 0x3F800000u ^ (uint32_t)(i * 2654435761u >> 9);   // floats near 1
  hipMalloc(&d_in, 1024 * 4);
  hipMemcpy(d_in, h.data(), 1024 * 4, hipMemcpyHostToDevice);
  hipMalloc(&d_out, (size_t)cus * 8 * 256 * 4);
  hipMalloc(&d_st, (size_t)cus * 8 * 4 * 32);
  sweep<kBitop3>(cus, d_in, d_out, d_st);
  sweep<kXor>(cus, d_in, d_out, d_st);
  sweep<kAdd>(cus, d_in, d_out, d_st);
  sweep<kFma>(cus, d_in, d_out, d_st);
  sweep<kPkFma>(cus, d_in, d_out, d_st);
  sweep<kPerm>(cus, d_in, d_out, d_st);
  sweep<kMadU64>(cus, d_in, d_out, d_st);
  sweep<kAlignbit>(cus, d_in, d_out, d_st);
  hipFree(d_in);
  hipFree(d_out);
  hipFree(d_st);
  return 0;
}
