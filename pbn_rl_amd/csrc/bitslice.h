// bitslice.h -- 32x32 bit-matrix transpose between per-env words and node planes.
//
// a[k] bit c  <->  a[c] bit k   (LSB-first on both axes).
// Five butterfly stages; the 16- and 8-bit stages are single byte permutes
// (v_perm_b32), the 4/2/1-bit stages two shifts + two v_bfi_b32 per pair.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pbn {

__host__ __device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
  return (m & a) | (~m & b);
}

// bfi as one v_bitop3_b32 (LUT 0xCA) on the device: for per-lane masks, where the compiler
// splits the and/or form into v_and + v_and_or (the transpose stages)
__host__ __device__ __forceinline__ uint32_t bfi3(uint32_t m, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);
#else
  return (m & a) | (~m & b);
#endif
}

// byte permute: result byte i = byte sel_i of {hi:lo} (lo = bytes 0-3, hi = bytes 4-7)
__host__ __device__ __forceinline__ uint32_t perm_bytes(uint32_t hi, uint32_t lo, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(hi, lo, sel);
#else
  const uint64_t v = ((uint64_t)hi << 32) | lo;
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) r |= (uint32_t)((v >> (8 * ((sel >> (8 * i)) & 7))) & 0xFF) << (8 * i);
  return r;
#endif
}

template <int J>
__host__ __device__ __forceinline__ void transpose_stage(uint32_t (&a)[32]) {
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    if (k & J) continue;
    const uint32_t x = a[k], y = a[k + J];
    if (J == 16) {
      // a[k] = x.lo16 | y.lo16 << 16 ; a[k+16] = x.hi16 | y.hi16 << 16
      a[k] = perm_bytes(y, x, 0x05040100u);
      a[k + J] = perm_bytes(y, x, 0x07060302u);
    } else if (J == 8) {
      // a[k] = [x.b0, y.b0, x.b2, y.b2] ; a[k+8] = [x.b1, y.b1, x.b3, y.b3]
      a[k] = perm_bytes(y, x, 0x06020400u);
      a[k + J] = perm_bytes(y, x, 0x07030501u);
    } else {
      constexpr uint32_t M = J == 4 ? 0x0F0F0F0Fu : (J == 2 ? 0x33333333u : 0x55555555u);
      a[k] = bfi(M, x, y << J);
      a[k + J] = bfi(M, x >> J, y);
    }
  }
}

__host__ __device__ __forceinline__ void transpose32(uint32_t (&a)[32]) {
  transpose_stage<16>(a);
  transpose_stage<8>(a);
  transpose_stage<4>(a);
  transpose_stage<2>(a);
  transpose_stage<1>(a);
}

}  // namespace pbn
