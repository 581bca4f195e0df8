// pbn_settle.hip -- the settle-law kernel instances (include/pbn_env.h "Step law"): the wave
// step kernel's variants 3 and 4 (pbn_step; the rollout of networks with gates) and the
// pipelined settle rollout pbn_rollout_settle, compiled beside pbn_env.hip so that the kernel
// instances build in parallel.
#include "step_kernels.h"

namespace {

template <int V>
void* pick_settle(int W, int B) {
#define PBN_SETTLE_CASE(w, b) \
  if (W == w && B == b) return reinterpret_cast<void*>(&pbn_step_wave<w, b, V>);
#define PBN_SETTLE_W(w) PBN_SETTLE_CASE(w, 4) PBN_SETTLE_CASE(w, 8) PBN_SETTLE_CASE(w, 12) PBN_SETTLE_CASE(w, 16)
  PBN_SETTLE_W(1) PBN_SETTLE_W(2) PBN_SETTLE_W(3) PBN_SETTLE_W(4)
#undef PBN_SETTLE_W
#undef PBN_SETTLE_CASE
  return nullptr;
}

void* pick_settle_pipe(int W, int B) {
#define PBN_SETTLE_CASE(w, b) \
  if (W == w && B == b) return reinterpret_cast<void*>(&pbn_rollout_settle<w, b>);
#define PBN_SETTLE_W(w) PBN_SETTLE_CASE(w, 4) PBN_SETTLE_CASE(w, 8) PBN_SETTLE_CASE(w, 12) PBN_SETTLE_CASE(w, 16)
  PBN_SETTLE_W(1) PBN_SETTLE_W(2) PBN_SETTLE_W(3) PBN_SETTLE_W(4)
#undef PBN_SETTLE_W
#undef PBN_SETTLE_CASE
  return nullptr;
}

}  // namespace

namespace pbn {

void* settle_kernel(int W, int B, int lean) { return lean ? pick_settle<4>(W, B) : pick_settle<3>(W, B); }

void* settle_pipe_kernel(int W, int B) { return pick_settle_pipe(W, B); }

}  // namespace pbn
