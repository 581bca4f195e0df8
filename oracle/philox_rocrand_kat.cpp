// Prints rocRAND philox4x32_10 outputs (engine.ten_rounds) for fixed and
// seeded-random counters/keys, one "c0 c1 c2 c3 k0 k1 -> o0 o1 o2 o3" line each.
// TEST INFRASTRUCTURE: used once by tools/gen_golden.py to pin oracle/pbn_oracle.c.
#include <cstdio>
#include <cstdint>
#include <rocrand/rocrand_philox4x32_10.h>

struct Probe : rocrand_device::philox4x32_10_engine {
  uint4 run(uint4 c, uint2 k) { return ten_rounds(c, k); }
};

static uint64_t sm = 0x243F6A8885A308D3ull;
static uint32_t next32() {  // splitmix64
  uint64_t z = (sm += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)(z ^ (z >> 31));
}

int main() {
  Probe p;
  const uint32_t fixed[3][6] = {
      {0, 0, 0, 0, 0, 0},
      {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu},
      {0x243f6a88u, 0x85a308d3u, 0x13198a2eu, 0x03707344u, 0xa4093822u, 0x299f31d0u}};
  for (int i = 0; i < 3 + 64; ++i) {
    uint32_t v[6];
    for (int j = 0; j < 6; ++j) v[j] = i < 3 ? fixed[i][j] : next32();
    uint4 c = {v[0], v[1], v[2], v[3]};
    uint2 k = {v[4], v[5]};
    uint4 o = p.run(c, k);
    std::printf("%08x %08x %08x %08x %08x %08x -> %08x %08x %08x %08x\n", v[0], v[1], v[2], v[3],
                v[4], v[5], o.x, o.y, o.z, o.w);
  }
  return 0;
}
