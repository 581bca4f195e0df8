// net_view.h -- read-only view of a pbn_net for the kernels outside pbn_env.hip
// (library-internal; not part of the C-ABI).
#pragma once
#include <stdint.h>

struct pbn_net;

namespace pbn {

struct NetView {
  int device;
  int n_nodes;
  int W;                        // state words per env
  int n_attr;
  int n_states;
  const int32_t* att_start;     // device [n_attr + 1]
  const uint32_t* att_states;   // device [n_states * W]
  const uint32_t* att_first;    // device [n_attr * W]: attractor t's first state (the BDQ target input)
};

// 0 on success, else a PBN_E* code with pbn_last_error() set
int net_view(const pbn_net* net, NetView* v);
// records `msg` for pbn_last_error() on this thread and returns `code`
int set_error(int code, const char* msg);
// checks that `net` is bound to the current device; 0 or PBN_EDEVICE/PBN_EINVAL
int check_device(const pbn_net* net);

}  // namespace pbn
