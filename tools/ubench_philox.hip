// Philox4x32-10 throughput microbenchmark on gfx950.
// Each thread runs CALLS calls with ILP independent streams interleaved; the xor of
// all outputs is stored so nothing is dead.  Reports calls/s for the chip.
//   hipcc --offload-arch=gfx950 -O3 -o ubench_philox tools/ubench_philox.hip && ./ubench_philox
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ void round_mad(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                          uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
  const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
  const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
  c1 = (uint32_t)p1;
  c3 = (uint32_t)p0;
  c0 = n0;
  c2 = n2;
}

__device__ __forceinline__ void round_hilo(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                           uint32_t k1) {
  const uint32_t h0 = __umulhi(0xD2511F53u, c0), l0 = 0xD2511F53u * c0;
  const uint32_t h1 = __umulhi(0xCD9E8D57u, c2), l1 = 0xCD9E8D57u * c2;
  const uint32_t n0 = h1 ^ c1 ^ k0;
  const uint32_t n2 = h0 ^ c3 ^ k1;
  c1 = l1;
  c3 = l0;
  c0 = n0;
  c2 = n2;
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

__device__ __forceinline__ void round_x3(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                         uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
  const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, k0);
  const uint32_t n2 = xor3((uint32_t)(p0 >> 32), c3, k1);
  c1 = (uint32_t)p1;
  c3 = (uint32_t)p0;
  c0 = n0;
  c2 = n2;
}

template <int ILP, int MAD>
__global__ void __launch_bounds__(256) k_philox(uint32_t* out, int calls, uint32_t seed) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (int c = 0; c < calls; c += ILP) {
    uint32_t a[ILP][4];
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
      a[i][0] = tid;
      a[i][1] = (uint32_t)(c + i);
      a[i][2] = 0x12345u;
      a[i][3] = 7u;
    }
    uint32_t k0 = seed, k1 = seed ^ 0xABCDu;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
#pragma unroll
      for (int i = 0; i < ILP; ++i) {
        if (MAD == 1) round_mad(a[i][0], a[i][1], a[i][2], a[i][3], k0, k1);
        else if (MAD == 2) round_x3(a[i][0], a[i][1], a[i][2], a[i][3], k0, k1);
        else round_hilo(a[i][0], a[i][1], a[i][2], a[i][3], k0, k1);
      }
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
#pragma unroll
    for (int i = 0; i < ILP; ++i) acc ^= a[i][0] ^ a[i][1] ^ a[i][2] ^ a[i][3];
  }
  out[tid] = acc;
}

template <int ILP, int MAD>
void run(const char* name, int blocks, int calls) {
  uint32_t* d;
  (void)hipMalloc(&d, (size_t)blocks * 256 * 4);
  hipEvent_t s, e;
  (void)hipEventCreate(&s);
  (void)hipEventCreate(&e);
  k_philox<ILP, MAD><<<blocks, 256>>>(d, calls, 1);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(s);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) k_philox<ILP, MAD><<<blocks, 256>>>(d, calls, r);
  (void)hipEventRecord(e);
  (void)hipEventSynchronize(e);
  float ms;
  (void)hipEventElapsedTime(&ms, s, e);
  const double total = (double)blocks * 256 * calls * reps;
  printf("{\"variant\": \"%s\", \"ilp\": %d, \"blocks\": %d, \"calls_per_thread\": %d, \"ms\": %.3f, "
         "\"philox_calls_per_s\": %.4e}\n", name, ILP, blocks, calls, ms / reps, total / (ms * 1e-3));
  (void)hipFree(d);
}

int main() {
  for (int blocks : {1024, 4096, 16384}) {
    run<1, 1>("mad", blocks, 256);
    run<2, 1>("mad", blocks, 256);
    run<4, 1>("mad", blocks, 256);
    run<8, 1>("mad", blocks, 256);
    run<4, 0>("hilo", blocks, 256);
    run<1, 2>("mad_xor3", blocks, 256);
    run<4, 2>("mad_xor3", blocks, 256);
    run<8, 2>("mad_xor3", blocks, 256);
  }
  return 0;
}
