// philox.h -- Philox4x32-R (Salmon et al., SC'11 / Random123) for gfx950.  Every stream draws
// Philox4x32-7 (kPhiloxRounds, DESIGN.md "RNG"): seven rounds is the smallest round count of
// Philox4x32 with no TestU01 BigCrush failure in the paper (Random123 defaults to 10 for a
// three-round safety margin).  The round function is pinned at 10 rounds by rocRAND's engine and
// at 7 and 10 by Random123's published known-answer vectors (tests/test_philox.py).
//
// One round: two 32x32->64 products (v_mad_u64_u32), two 3-input xors
// (v_xor3_b32); the key schedule is wave-uniform and lives in SGPRs.
// Counter map (DESIGN.md "RNG stream map"):
//   ctr = (lo32(id), lo32(step), stream << 28 | idx, hi16(id) | hi16(step) << 16)
//   key = (lo32(seed), hi32(seed))
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pbn {

// EXPLORE = 4: epsilon-greedy draws of pbn_q_to_flipmask (per env; word 0 = explore test,
// word k + 1 = branch k's random action, by multiply-high); SETTLE_SEL = 5 (per env: node i's
// selection uniform of update k is 16-bit field i & 7 of call (k << 8) | (i >> 3)) and
// SETTLE_ENV = 6 (per env): updates k >= 1 of a step under the settle law (settle_updates);
// REPLAY = 7: the learner's replay rows (pbn_replay_advance: id = row of the batch, step = draw)
enum : uint32_t {
  kStreamSel = 0, kStreamEnv = 1, kStreamPert = 2, kStreamReset = 3, kStreamExplore = 4,
  kStreamSettleSel = 5, kStreamSettleEnv = 6, kStreamReplay = 7
};

struct Word4 {
  uint32_t x, y, z, w;
};

// a ^ b ^ c in one v_bitop3_b32 (gfx950; LUT 0x96 = 3-input xor)
__host__ __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

constexpr int kPhiloxRounds = 7;

// ctr = (c0, c1, c2, c3), key = (k0, k1); one round: two 32x32->64 products, two 3-input xors,
// the Weyl key bump (SALU: the key is wave-uniform).  XM (default 0) is xor-ed into output words
// 0 and 2 for free, through the last round's keys (the settle law's packed compares bias them).
template <int R = kPhiloxRounds, uint32_t XM = 0u>
__host__ __device__ __forceinline__ Word4 philox(uint32_t c0, uint32_t c1, uint32_t c2,
                                                  uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, r == R - 1 ? (k0 ^ XM) : k0);
    const uint32_t n2 = xor3((uint32_t)(p0 >> 32), c3, r == R - 1 ? (k1 ^ XM) : k1);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return Word4{c0, c1, c2, c3};
}

__host__ __device__ __forceinline__ Word4 draw(uint64_t seed, uint64_t id, uint64_t step,
                                                uint32_t stream, uint32_t idx) {
  return philox((uint32_t)id, (uint32_t)step, (stream << 28) | (idx & 0x0FFFFFFFu),
                       (uint32_t)((id >> 32) & 0xFFFFu) | ((uint32_t)((step >> 32) & 0xFFFFu) << 16),
                       (uint32_t)seed, (uint32_t)(seed >> 32));
}

}  // namespace pbn
