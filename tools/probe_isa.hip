// Probes gfx950 semantics the kernels rely on: v_bitop3_b32 LUT bit order and
// v_permlane16_swap / v_permlane32_swap lane movement.  Prints JSON.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k(unsigned* o) {
  const unsigned l = threadIdx.x;
  auto p16 = __builtin_amdgcn_permlane16_swap(l, l + 100u, false, false);
  auto p32 = __builtin_amdgcn_permlane32_swap(l, l + 100u, false, false);
  o[l * 4 + 0] = p16[0];
  o[l * 4 + 1] = p16[1];
  o[l * 4 + 2] = p32[0];
  o[l * 4 + 3] = p32[1];
  if (l == 0) {
    o[256] = __builtin_amdgcn_bitop3_b32(0xF0F0F0F0u, 0xCCCCCCCCu, 0xAAAAAAAAu, 0xCA);
    o[257] = __builtin_amdgcn_bitop3_b32(0xF0F0F0F0u, 0xCCCCCCCCu, 0xAAAAAAAAu, 0x80);
    o[258] = __builtin_amdgcn_bitop3_b32(0xF0F0F0F0u, 0xCCCCCCCCu, 0xAAAAAAAAu, 0x01);
  }
}

int main() {
  unsigned* d;
  unsigned h[260];
  (void)hipMalloc(&d, sizeof h);
  k<<<1, 64>>>(d);
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  printf("{\"bitop3_0xCA\": \"%08x\", \"bitop3_0x80\": \"%08x\", \"bitop3_0x01\": \"%08x\",\n", h[256], h[257], h[258]);
  printf(" \"permlane16_swap\": [");
  for (int l = 0; l < 64; ++l) printf("[%u,%u]%s", h[l * 4], h[l * 4 + 1], l < 63 ? "," : "");
  printf("],\n \"permlane32_swap\": [");
  for (int l = 0; l < 64; ++l) printf("[%u,%u]%s", h[l * 4 + 2], h[l * 4 + 3], l < 63 ? "," : "");
  printf("]}\n");
  return 0;
}
