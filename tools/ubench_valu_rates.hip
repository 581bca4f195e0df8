// Relative issue cost of the rollout kernel's VALU mix on gfx950: 8 independent chains per lane
// of v_mad_u64_u32 (Philox products, bounded draws), v_bitop3_b32 (xor3, transposes, compares),
// v_perm_b32 (mux-tree leaves) and v_mul_hi_u32, at full occupancy (8 waves per SIMD), timed with
// HIP events.  Prints ns per wave-instruction per SIMD for each: the ratio to bitop3 is the cost
// of one instruction in units of a full-rate op.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kIters = 4096;

template <int OP>
__global__ void __launch_bounds__(256) rate_kernel(uint32_t* out, uint32_t seed) {
  uint32_t a[8], b[8];
  for (int k = 0; k < 8; ++k) { a[k] = seed * (threadIdx.x + 7 * k + 1); b[k] = a[k] ^ 0x9E3779B9u; }
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if constexpr (OP == 0) {
        const uint64_t p = (uint64_t)a[k] * 0xD2511F53u + b[k];
        a[k] = (uint32_t)(p >> 32); b[k] = (uint32_t)p;
      } else if constexpr (OP == 1) {
        a[k] = __builtin_amdgcn_bitop3_b32(a[k], b[k], 0x1234567u, 0x96);
      } else if constexpr (OP == 2) {
        a[k] = __builtin_amdgcn_perm(a[k], b[k], 0x05040100u + it);
      } else {
        a[k] = __umulhi(a[k], 0xCD9E8D57u) + b[k];
      }
    }
  }
  uint32_t r = 0;
  for (int k = 0; k < 8; ++k) r ^= a[k] ^ b[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int OP>
float run(uint32_t* d, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(rate_kernel<OP>, dim3(blocks), dim3(256), 0, 0, d, 3u);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(rate_kernel<OP>, dim3(blocks), dim3(256), 0, 0, d, 3u + r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  int dev = 0, cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int blocks = cus * 8;   // 8 blocks of 4 waves per CU: 8 waves per SIMD
  uint32_t* d;
  hipMalloc(&d, sizeof(uint32_t) * blocks * 256);
  const double insts_per_simd = (double)blocks * 4 / (cus * 4) * kIters * 8;   // wave-instructions per SIMD
  const char* names[4] = {"v_mad_u64_u32", "v_bitop3_b32", "v_perm_b32", "v_mul_hi_u32 + v_add"};
  float ms[4] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks)};
  for (int k = 0; k < 4; ++k)
    printf("{\"op\": \"%s\", \"ms\": %.4f, \"ns_per_wave_inst_per_simd\": %.4f, \"vs_bitop3\": %.2f}\n", names[k], ms[k],
           ms[k] * 1e6 / insts_per_simd, ms[k] / ms[1]);
  hipFree(d);
  return 0;
}
