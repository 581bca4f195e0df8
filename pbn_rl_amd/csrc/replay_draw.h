// replay_draw.h -- the learning frame's counter advance and replay-row draw (library-internal),
// shared by pbn_replay_advance's single-block kernel (pbn_agent.hip) and the fused update's
// extra apply block (pbn_learn.hip, pbn_frame_advance).  One 256-thread block:
//   *pos = (*pos + n_store) mod cap, *size = min(*size + n_store, cap)      (n_store > 0)
//   *step += 1; *eps64 = max(eps_final, *eps64 - eps_step), *eps32 its fp32 copy
//   idx[b] = mulhi64(x << 32 | y, draw_size) for the REPLAY Philox pair (x, y) of (seed, id = b,
//   step = *counter), b < n_idx; *counter += 1.  draw_size = the new size plus draw_ahead stored
//   rows (min capacity): 0 for the frame being stored, n_store for the next frame's store (the
//   fused update draws the next frame's rows in advance).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "philox.h"

namespace pbn {

__device__ __forceinline__ void frame_advance_block(int64_t n_store, int64_t cap, int64_t* pos, int64_t* size,
                                                    int64_t* step, double* eps64, float* eps32, double eps_final,
                                                    double eps_step, int64_t n_idx, uint64_t seed, int64_t* counter,
                                                    int64_t* idx, int64_t draw_ahead) {
  __shared__ int64_t s_size;
  if (threadIdx.x == 0) {
    int64_t sz = *size;
    if (n_store > 0) {
      *pos = (*pos + n_store) % cap;
      sz = sz + n_store < cap ? sz + n_store : cap;
      *size = sz;
    }
    if (step) *step += 1;
    if (eps64) {
      const double e = *eps64 - eps_step;
      const double v = isnan(e) ? e : (e > eps_final ? e : eps_final);   // torch.maximum(final, e)
      *eps64 = v;
      if (eps32) *eps32 = (float)v;
    }
    s_size = sz + draw_ahead < cap ? sz + draw_ahead : cap;
  }
  __syncthreads();
  if (n_idx > 0) {
    const uint64_t sz = (uint64_t)(s_size > 0 ? s_size : 1);
    const uint64_t c = (uint64_t)*counter;
    for (int64_t b = threadIdx.x; b < n_idx; b += blockDim.x) {
      const Word4 r = draw(seed, (uint64_t)b, c, kStreamReplay, 0);
      idx[b] = (int64_t)__umul64hi(((uint64_t)r.x << 32) | r.y, sz);
    }
    __syncthreads();
    if (threadIdx.x == 0) *counter = (int64_t)(c + 1);
  }
}

}  // namespace pbn
